#!/usr/bin/env python3
"""Regenerate the MaxEnt splice-site model tables the engine's device Maxent_hr_*_prob reads.

GMAP's splice-site models (maxent_hr.c:25-24660) are constant tables: per model a 7-mer/9-mer score table of
16 384 doubles and a 16-entry dinucleotide table (the acceptor models have five score tables).  This script
reads them from the reference's source where it lies (default /root/reference/src/maxent_hr.c), converts
every decimal literal the way a C compiler does (correctly rounded to the nearest double; Python's float() is
correctly rounded too) and writes them as one little-endian binary that libgmapdp.so loads
(gmap-2024_amd/lib/maxent_hr_tables.bin, next to the library; git-ignored, built by __graft_entry__.build()
and `make -C gmap-2024_amd`, travels to the GPU box with the built library).

Layout (include/gmapdp.h "Device MaxEnt"): 8-byte magic "GMDPMXT1", uint32 table count (16), uint32 0,
then per table in TABLES order: 32-byte NUL-padded name, uint32 entries, uint32 0, entries x float64.

  python3 tools/make_maxent_tables.py [--src maxent_hr.c] [--out gmap-2024_amd/lib/maxent_hr_tables.bin]
"""
import argparse
import os
import re
import struct
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# the order the engine uploads them in (gmapdp_engine.cpp kMaxentTables)
TABLES = [("donor_score_plus", 16384), ("donor_discore_plus", 16),
          ("acc_score1_plus", 16384), ("acc_score2_plus", 16384), ("acc_score3_plus", 16384),
          ("acc_discore_plus", 16), ("acc_score467_plus", 16384), ("acc_score589_plus", 16384),
          ("donor_score_minus", 16384), ("donor_discore_minus", 16),
          ("acc_score1_minus", 16384), ("acc_score2_minus", 16384), ("acc_score3_minus", 16384),
          ("acc_discore_minus", 16), ("acc_score467_minus", 16384), ("acc_score589_minus", 16384)]
MAGIC = b"GMDPMXT1"


def parse(src):
    text = open(src).read()
    out = {}
    for name, n in TABLES:
        m = re.search(r"static const double %s\[(\d+)\]\s*=\s*\{(.*?)\};" % name, text, re.S)
        if not m:
            raise SystemExit("make_maxent_tables: table %s not found in %s" % (name, src))
        if int(m.group(1)) != n:
            raise SystemExit("make_maxent_tables: %s has %s entries, expected %d" % (name, m.group(1), n))
        vals = [float(x) for x in m.group(2).replace("\n", " ").split(",") if x.strip()]
        if len(vals) != n:
            raise SystemExit("make_maxent_tables: %s: %d initialisers, expected %d" % (name, len(vals), n))
        out[name] = vals
    return out


def write(tables, path):
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    tmp = path + ".tmp"
    with open(tmp, "wb") as f:
        f.write(MAGIC + struct.pack("<II", len(TABLES), 0))
        for name, n in TABLES:
            f.write(name.encode().ljust(32, b"\0") + struct.pack("<II", n, 0))
            f.write(struct.pack("<%dd" % n, *tables[name]))
    os.replace(tmp, path)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--src", default="/root/reference/src/maxent_hr.c")
    ap.add_argument("--out", default=os.path.join(ROOT, "gmap-2024_amd", "lib", "maxent_hr_tables.bin"))
    a = ap.parse_args()
    if not os.path.exists(a.src):
        if os.path.exists(a.out):
            print("make_maxent_tables: %s absent, keeping %s" % (a.src, a.out))
            return 0
        raise SystemExit("make_maxent_tables: %s not found and no %s" % (a.src, a.out))
    write(parse(a.src), a.out)
    print("wrote %s (%d bytes)" % (a.out, os.path.getsize(a.out)))
    return 0


if __name__ == "__main__":
    sys.exit(main())
