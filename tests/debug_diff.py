"""Debug helper (not a test): run seeded problems on the GPU, dump the first
differing problems vs the oracle to gpurun_out/fail.json."""
import json, os, random, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gmap-2024_amd")); sys.path.insert(0, os.path.join(ROOT, "tests"))
import gmapdp
from dpbind import Oracle, call_single, random_genome, single_gap_problem, edge_single_gap_problem

def main(n_typ=2000, n_edge=2000, seed=123):
    rng = random.Random(seed)
    g = random_genome(rng, 20000)
    probs = [single_gap_problem(rng, g) for _ in range(200)] + [edge_single_gap_problem(rng, g) for _ in range(56)]
    probs += [single_gap_problem(rng, g) for _ in range(n_typ)] + [edge_single_gap_problem(rng, g) for _ in range(n_edge)]
    eng = gmapdp.Engine(0); eng.set_genome(g)
    got = eng.single_gap_batch(probs)
    orc = Oracle(); orc.set_genome(g)
    fails = []
    for i, p in enumerate(probs):
        e = call_single(orc, p)
        if got[i] != e:
            fails.append(dict(i=i, p={k: (v.decode() if isinstance(v, bytes) else v) for k, v in p.items()},
                              gpu_scal=got[i][0], orc_scal=e[0],
                              gpu=[[str(x) for x in t] for t in (got[i][1] or [])],
                              orc=[[str(x) for x in t] for t in (e[1] or [])]))
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    json.dump(dict(nfail=len(fails), n=len(probs), fails=fails[:30]), open(os.path.join(ROOT, "gpurun_out", "fail.json"), "w"))
    print("fails", len(fails), "of", len(probs))

if __name__ == "__main__":
    main()
