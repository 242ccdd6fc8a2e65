"""Generate the end-to-end fixtures: seeded synthetic cDNA reads + genomic segment, and the reference
`gmap` program's own outputs on them (nosimd and AVX2 builds).

Run in the development container after `make -C oracle ref` (needs oracle/_ref/gmap_{nosimd,avx2},
the unmodified reference program compiled from /root/reference/src):

    python tests/golden/make_e2e.py

Inputs (SURVEY.md §8d read shape, restated): an i.i.d. uniform ACGT genomic segment (seed 38) and
2,000-nt reads of 5 exons x 400 nt cut from it, introns log-uniform in [80, 20000] nt with GT...AG
forced at every junction, 2 % uniform substitutions, 50 % reverse-complemented; read i uses
seed * 10**6 + i.  GMAP runs them in user-segment mode (`-g`, gmap.c:1468 stage3_skip_stage1:
stage 2 + stage 3 + every Dynprog_* entry point over the whole segment, both strands).

Outputs (data only):
  e2e_genome.fa          the genomic segment
  e2e_reads.fa           the reads
  e2e_nosimd.sam         `gmap_nosimd -g e2e_genome.fa -f samse --no-sam-headers e2e_reads.fa`
  e2e_avx2.sam           the same with the AVX2 build (SIMD-build DP semantics)
  cdna2_genetest2_*.txt  `gmap -g genetest2.fa cdna2.fa` (BASELINE configs[0] inputs; the bundled
                         cdna.fa is empty) in default output format, both builds
  e2e_short_genome.fa, e2e_short_reads.fa, e2e_short_{nosimd,avx2}.sam
                         reads whose stage 3 makes Oligoindex_get_mappings calls on 8-nt queries
                         (SHORT_OLIGO_READS, found with oracle/_ref/gmap_callmix), and the reference
                         program's outputs on them
  e2e_s8_reads.fa, e2e_s8_{nosimd,avx2}.sam
                         two reads of e2e_reads.fa with 8-nt reads after each (pieces of the read
                         before them and random 8-mers): GMAP calls Stage2_compute on each 8-nt read,
                         whose tally runs against the previous longer query's 8-mer flags
                         (oligoindex_hr.c:33478); against e2e_genome.fa, single worker (-t 1)
"""
import math
import os
import random
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
REF = os.path.join(ROOT, "oracle", "_ref")

GENOME_SEED = 38
READ_SEED = 38
GENOME_LEN = 300000
NREADS = 200
COMP = {"A": "T", "C": "G", "G": "C", "T": "A"}


def revcomp(s):
    return "".join(COMP[c] for c in reversed(s))


def synth_genome(n=GENOME_LEN, seed=GENOME_SEED):
    rng = random.Random(seed)
    return "".join(rng.choice("ACGT") for _ in range(n))


def synth_read(genome, i, seed=READ_SEED, nexons=5, exonlen=400, sub=0.02, intron_lo=80, intron_hi=20000):
    """One spliced read: returns (name, sequence).  The genome's junction dinucleotides are
    overwritten with GT...AG (the genome string is a list, modified in place)."""
    rng = random.Random(seed * 10**6 + i)
    introns = [int(round(math.exp(rng.uniform(math.log(intron_lo), math.log(intron_hi))))) for _ in range(nexons - 1)]
    span = nexons * exonlen + sum(introns)
    start = rng.randrange(1000, len(genome) - span - 1000)
    exons = []
    pos = start
    for e in range(nexons):
        exons.append((pos, pos + exonlen))
        if e < nexons - 1:
            il = introns[e]
            genome[pos + exonlen] = "G"
            genome[pos + exonlen + 1] = "T"
            genome[pos + exonlen + il - 2] = "A"
            genome[pos + exonlen + il - 1] = "G"
            pos += exonlen + il
    seq = list("".join("".join(genome[a:b]) for a, b in exons))
    for k in range(len(seq)):
        if rng.random() < sub:
            seq[k] = rng.choice([c for c in "ACGT" if c != seq[k]])
    seq = "".join(seq)
    rc = rng.random() < 0.5
    if rc:
        seq = revcomp(seq)
    name = "r%d_%d_%s" % (i, start + 1, "-" if rc else "+")
    return name, seq


def write_fasta(path, records, width=60):
    with open(path, "w") as f:
        for name, seq in records:
            f.write(">%s\n" % name)
            for k in range(0, len(seq), width):
                f.write(seq[k:k + width] + "\n")


# reads of the 30 000-read stream (tools/e2e_inputs.py /dir 30000: the segment with all 30 000 reads'
# junctions planted) whose stage 3 queries an oligoindex with 8 nt -- the reference answers from the
# previous longer query's 8-mer flags (Oligoindex_set_inquery :33478); read 15135 makes two such calls
SHORT_OLIGO_READS = (15135,)
SHORT_STREAM = 30000


def make_inputs():
    g = list(synth_genome())
    reads = [synth_read(g, i) for i in range(NREADS)]
    write_fasta(os.path.join(HERE, "e2e_genome.fa"), [("synseg", "".join(g))])
    write_fasta(os.path.join(HERE, "e2e_reads.fa"), reads)
    g2 = list(synth_genome())
    short = [r for i, r in ((i, synth_read(g2, i)) for i in range(SHORT_STREAM)) if i in SHORT_OLIGO_READS]
    write_fasta(os.path.join(HERE, "e2e_short_genome.fa"), [("synseg", "".join(g2))])
    write_fasta(os.path.join(HERE, "e2e_short_reads.fa"), short)
    rng = random.Random(8)
    s8 = []
    for name, seq in reads[:2]:
        s8.append((name, seq))
        for k in range(6):
            i = rng.randrange(0, len(seq) - 8)
            s8.append(("%s_in%d" % (name, k), seq[i:i + 8]))
            s8.append(("%s_rand%d" % (name, k), "".join(rng.choice("ACGT") for _ in range(8))))
    write_fasta(os.path.join(HERE, "e2e_s8_reads.fa"), s8)


def run_gmap(binary, args, out):
    with open(out, "w") as f:
        subprocess.run([binary] + args, stdout=f, stderr=subprocess.DEVNULL, check=True, cwd=HERE)


def main():
    make_inputs()
    for v in ("nosimd", "avx2"):
        exe = os.path.join(REF, "gmap_" + v)
        run_gmap(exe, ["-g", "e2e_genome.fa", "-f", "samse", "--no-sam-headers", "e2e_reads.fa"],
                 os.path.join(HERE, "e2e_%s.sam" % v))
        run_gmap(exe, ["-g", "genetest2.fa", "cdna2.fa"], os.path.join(HERE, "cdna2_genetest2_%s.txt" % v))
        run_gmap(exe, ["-g", "e2e_short_genome.fa", "-f", "samse", "--no-sam-headers", "e2e_short_reads.fa"],
                 os.path.join(HERE, "e2e_short_%s.sam" % v))
        run_gmap(exe, ["-t", "1", "-g", "e2e_genome.fa", "-f", "samse", "--no-sam-headers", "e2e_s8_reads.fa"],
                 os.path.join(HERE, "e2e_s8_%s.sam" % v))
    print("wrote e2e fixtures in", HERE)


if __name__ == "__main__":
    sys.exit(main())
