"""Debug aid (GPU box): run one Stage2_compute problem through the engine and the oracle and compare
the chaining state (minactive / maxactive and the per-hit link arrays) -- s2_scratch's layout."""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gmap-2024_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import gmapdp  # noqa: E402
from dpbind import Oracle  # noqa: E402


def a16(x):
    return (x + 15) & ~15


def layout(ql, T, nd):
    Q, D, H = ql + 1, max(nd, 1), max(T, 1)
    s = {"diff": 0}
    s["run"] = a16(4 * Q)
    s["off"] = a16(s["run"] + 8 * Q)
    s["minact"] = a16(s["off"] + 4 * Q)
    s["maxact"] = a16(s["minact"] + 4 * Q)
    s["first"] = a16(s["maxact"] + 4 * Q)
    s["proc"] = a16(s["first"] + 4 * Q)
    s["diags"] = a16(s["proc"] + 4 * Q)
    s["ord"] = a16(s["diags"] + 32 * D)
    s["tmp"] = a16(s["ord"] + 4 * D)
    s["hits"] = a16(s["tmp"] + 4 * D)
    s["maps"] = a16(s["hits"] + 32 * H)  # S2Hit {map_ (unused), consec, root, fpos, fhit, tracei, score, q}
    s["sc"] = a16(s["maps"] + 4 * H)
    s["end"] = a16(s["sc"] + 4 * H)
    return s


def main(k=0):
    import importlib.util
    spec = importlib.util.spec_from_file_location("mg", os.path.join(ROOT, "tests", "golden", "make_golden.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    g, probs, exp = m.load_stage2(os.path.join(ROOT, "tests", "golden", "stage2_golden.npz"))
    p = probs[k]
    orc = Oracle()
    orc.set_genome(g)
    sc = orc.oligo_mappings(dict(p, minor=0))[0]
    T, nd, ql = sc[0], sc[3], len(p["quc"])
    buf = (C.c_int * (2 * ql + 8 * T + 16))()
    orc.lib.orc_stage2_debug(buf)
    o = orc.stage2_compute(p)
    ob = np.frombuffer(buf, dtype=np.int32)
    eng = gmapdp.Engine(0)
    eng.set_genome(g)
    got = eng.stage2_batch([p])[0]
    L = layout(ql, T, nd)
    raw = np.zeros(L["end"], dtype=np.uint8)
    eng.lib.gmapdp_debug_stage2_scratch(eng.h, raw.ctypes.data, C.c_size_t(L["end"]))
    minact = raw[L["minact"]:L["minact"] + 4 * ql].view(np.uint32).astype(np.int64)
    maxact = raw[L["maxact"]:L["maxact"] + 4 * ql].view(np.uint32).astype(np.int64)
    rec = raw[L["hits"]:L["hits"] + 32 * T].view(np.int32).reshape(T, 8)
    maps = raw[L["maps"]:L["maps"] + 4 * T].view(np.int32)
    scs = raw[L["sc"]:L["sc"] + 4 * T].view(np.int32)
    # the oracle's field order {map, consec, root, fpos, fhit, tracei, score, active} (+ q): records are
    # written only for the hits the sweep scores, so compare those (score > 0)
    hits = np.zeros((T, 9), dtype=np.int32)
    hits[:, 0] = maps
    hits[:, 1:7] = rec[:, 1:7]
    hits[:, 6] = scs
    hits[:, 8] = rec[:, 7]
    print("problem", k, "T", T, "nd", nd, "ql", ql, "equal results:", got == o, "exp==orc:", exp[k] == o)
    omin = ob[:ql].view(np.uint32).astype(np.int64)
    omax = ob[ql:2 * ql].view(np.uint32).astype(np.int64)
    bad = np.nonzero(omin != minact)[0]
    print("minactive differs at", bad[:10], [(int(omin[i]), int(minact[i])) for i in bad[:5]])
    bad = np.nonzero(omax != maxact)[0]
    print("maxactive differs at", bad[:10], [(int(omax[i]), int(maxact[i])) for i in bad[:5]])
    oh = ob[2 * ql:2 * ql + 8 * T].reshape(T, 8)
    names = ["map", "consec", "root", "fpos", "fhit", "tracei", "score", "active"]
    scored = oh[:, 6] > 0
    for f in range(7):
        bad = np.nonzero((oh[:, f] != hits[:, f]) & (scored | (f in (0, 6))))[0]
        if len(bad):
            i = bad[0]
            print("hit field %s differs at %d hits, first hit %d (q %d): oracle %s gpu %s" % (
                names[f], len(bad), i, hits[i, 8], oh[i].tolist(), hits[i, :8].tolist()))


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 0)
