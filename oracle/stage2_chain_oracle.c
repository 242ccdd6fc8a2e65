/* oracle/stage2_chain_oracle.c -- TEST INFRASTRUCTURE ONLY (never shipped, never on the product path).
 *
 * CPU restatement of GMAP's stage-2 chaining: everything Stage2_compute
 * (stage2.c:6325) does after the seeding that stage2_oracle.c restates, with GMAP's arguments
 * (gmap.c:1208-1215: localp, skip_repetitive_p, proceed_pctcoverage 0.3, favor_right_p false,
 * max_nalignments 10; Stage2_setup gmap.c:6544: use_canonical_middle_p = cross_species_p = false,
 * mode STANDARD, snps_p false; MOVE_TO_STAGE3 and SEPARATE_FWD_REV undefined):
 *
 *   Diag_update_coverage        diag.c:216   covered query positions of the diagonals
 *   the proceed test            stage2.c:6521-6531
 *   Diag_compute_bounds         diag.c:597   assign_scores :521, compute_dominance :427,
 *                                            keep_center_diagonal :493, minactive / maxactive
 *   align_compute_lookback      stage2.c:4402
 *     align_compute_scores_lookback :3667   the querypos sweep, repetitive-position skipping,
 *                                            the grand lookback
 *     score_querypos_lookback_one   :1073   adjacent link, then ranges 0-4 over the processed
 *     score_querypos_lookback_mult  :1470   query positions (frontiers carried across hits)
 *     revise_active_lookback        :2956
 *     get_cells_fwd                 :3437   best cells per root position, score order
 *     traceback_one                 :4140
 *   convert_to_nucleotides      stage2.c:5334 (mode STANDARD, gap holders included)
 *   Stage2_filter_unique        stage2.c:6013
 *
 * The reference sorts with glibc qsort, which is a stable merge sort on this image (glibc 2.35:
 * msort for arrays that fit in memory); the ties of Cell_score_cmp, nconsecutive_cmp, diagonal_cmp
 * and stage2_cmp therefore keep input order, and so does stable_sort below.  Chrpos_T arithmetic is
 * unsigned 32-bit as in the reference.  Pinned against the reference's own Stage2_compute through
 * refh_stage2_compute (oracle/refharness.c) by tests/test_oracle.py.
 */
#include <stdlib.h>
#include <string.h>

#include "gmapdp_oracle.h"

#define INDEXSIZE 8                 /* the GMAP major oligoindex (oligoindex_hr.c:8606) */
#define EQUAL_DISTANCE_NOT_SPLICING 9
#define EQUAL_DISTANCE_FOR_CONSECUTIVE 0
#define ENOUGH_CONSECUTIVE 32
#define GREEDY_NCONSECUTIVE 100
#define EXON_DEFN 30
#define MIN_TERMINAL_NCONSECUTIVE 8
#define MAX_NACTIVE 100
#define MAX_SKIPPED 3
#define SCORE_FOR_RESTRICT 10
#define TEN_THOUSAND 8192
#define FINAL_SCORE_TOLERANCE 20
#define MAX_NALIGNMENTS 10          /* gmap.c:142 */
#define SUFF_NCOVERED 200
#define PROCEED_PCTCOVERAGE 0.3
#define DIAG_MIN_SCORE 10.0         /* diag.c:12-17 */
#define DOMINANCE_END_EQUIV 20
#define EXTRA_BOUNDS 20

/* stable sort of n pointers by cmp (glibc 2.35 qsort semantics: merge sort) */
static void
stable_sort (void **a, int n, int (*cmp) (const void *, const void *)) {
  void **tmp;
  int width, i, l, m, r, x, y, k;
  if (n < 2) return;
  tmp = (void **) malloc((size_t) n * sizeof(void *));
  for (width = 1; width < n; width *= 2) {
    for (i = 0; i < n; i += 2 * width) {
      l = i; m = i + width < n ? i + width : n; r = i + 2 * width < n ? i + 2 * width : n;
      x = l; y = m; k = l;
      while (x < m && y < r) tmp[k++] = (cmp(&a[y], &a[x]) < 0) ? a[y++] : a[x++];
      while (x < m) tmp[k++] = a[x++];
      while (y < r) tmp[k++] = a[y++];
    }
    memcpy(a, tmp, (size_t) n * sizeof(void *));
  }
  free(tmp);
}

/* ---------------------------------------------------------------- diag.c */

typedef struct {
  unsigned int diagonal;
  int querystart, queryend, nconsecutive, dominatedp;
  double score;
} ODiag;

static int
nconsecutive_desc (const void *x, const void *y) {
  const ODiag *a = *(ODiag * const *) x, *b = *(ODiag * const *) y;
  return (a->nconsecutive > b->nconsecutive) ? -1 : (b->nconsecutive > a->nconsecutive) ? 1 : 0;
}

static int
diagonal_asc (const void *x, const void *y) {
  const ODiag *a = *(ODiag * const *) x, *b = *(ODiag * const *) y;
  return (a->diagonal < b->diagonal) ? -1 : (b->diagonal < a->diagonal) ? 1 : 0;
}

/* compute_dominance (diag.c:427): array sorted by nconsecutive, dominated diagonals dropped */
static int
dominance (ODiag **arr, int n) {
  int nunique = n, i, j, k, start, end, expected, threshold;
  stable_sort((void **) arr, n, nconsecutive_desc);
  for (i = 0; i < nunique; i++) {
    ODiag *sup = arr[i];
    start = sup->querystart;
    end = sup->queryend;
    expected = end + 1 - start;
    if (expected < 100 && sup->nconsecutive > expected - 10) {
      threshold = sup->nconsecutive - DOMINANCE_END_EQUIV;
    } else if (expected >= 100 && sup->nconsecutive > expected * 0.90) {
      threshold = (int) (sup->nconsecutive * 0.80);
    } else {
      continue;
    }
    for (j = i + 1; j < nunique; j++)
      if (arr[j]->querystart >= start && arr[j]->queryend <= end && arr[j]->nconsecutive < threshold)
        arr[j]->dominatedp = 1;
    for (k = i + 1, j = i + 1; j < nunique; j++)
      if (!arr[j]->dominatedp) arr[k++] = arr[j];
    nunique = k;
  }
  return nunique;
}

/* Diag_compute_bounds (diag.c:597); diags in list order */
static void
compute_bounds (int *qstart, int *qend, unsigned int *minactive, unsigned int *maxactive, ODiag *diags,
                int nd, int querylength, unsigned int chrstart, unsigned int chrend, unsigned int chroffset,
                unsigned int chrhigh, int plusp) {
  unsigned int genomiclength = chrend - chrstart, chrinit, chrterm, diagonal = 0, position, center = 0;
  unsigned int mind, maxd;
  ODiag **arr;
  double *cum, count, run;
  int q, i, j, nunique, ngood, nbins, *bins, maxcount, activestart, activeend;

  chrinit = plusp ? chrstart : (chrhigh - chroffset) - chrend;
  chrterm = plusp ? chrend : (chrhigh - chroffset) - chrstart;
  if (nd == 0) {
    for (q = 0; q < querylength; q++) { minactive[q] = chrinit; maxactive[q] = chrterm; }
    *qstart = 0;
    *qend = querylength - 1;
    return;
  }

  /* assign_scores (diag.c:521): 1/depth per covered position, summed left to right */
  cum = (double *) calloc((size_t) querylength, sizeof(double));
  for (i = 0; i < nd; i++) {
    cum[diags[i].querystart] += 1.0;
    cum[diags[i].queryend] -= 1.0;
  }
  count = 0.0;
  for (q = 0; q < querylength; q++) {
    count += cum[q];
    cum[q] = (count > 0.0) ? 1.0 / (double) count : 0.0;
  }
  run = 0.0;
  for (q = 0; q < querylength; q++) {
    run += cum[q];
    cum[q] = run;
  }
  for (i = 0; i < nd; i++) diags[i].score = cum[diags[i].queryend] - cum[diags[i].querystart];
  free(cum);

  /* gooddiagonals: List_push (reverse list order) of those scoring MIN_SCORE */
  arr = (ODiag **) malloc((size_t) (nd > 0 ? nd : 1) * sizeof(ODiag *));
  for (ngood = 0, i = nd - 1; i >= 0; i--)
    if (diags[i].score >= DIAG_MIN_SCORE) arr[ngood++] = &diags[i];
  if (ngood == 0) {
    for (i = 0; i < nd; i++) arr[i] = &diags[i];
    ngood = nd;
  }
  nunique = dominance(arr, ngood);
  stable_sort((void **) arr, nunique, diagonal_asc);

  if (nunique > 100) {  /* keep_center_diagonal (diag.c:493) around the densest 10-kb bin */
    mind = arr[0]->diagonal;
    maxd = arr[nunique - 1]->diagonal;
    nbins = (int) ((maxd - mind) / 10000) + 1;
    bins = (int *) calloc((size_t) nbins, sizeof(int));
    for (i = 0; i < nunique; i++) bins[(arr[i]->diagonal - mind) / 10000] += 1;
    maxcount = 0;
    diagonal = mind;
    for (i = 0; i < nbins; i++) {
      if (bins[i] > maxcount) { maxcount = bins[i]; center = diagonal; }
      diagonal += 10000;
    }
    center += 5000;
    for (j = 0, i = 0; i < nunique; i++)
      if (!(arr[i]->diagonal + 10000 < center || arr[i]->diagonal > center + 10000)) arr[j++] = arr[i];
    nunique = j;
    free(bins);
  }

  activestart = arr[0]->querystart;
  activeend = arr[nunique - 1]->queryend;
  *qstart = querylength - 1;
  *qend = 0;
  for (i = 0; i < nunique; i++) {
    if (arr[i]->querystart < *qstart) *qstart = arr[i]->querystart;
    if (arr[i]->queryend > *qend) *qend = arr[i]->queryend;
  }

  /* minactive: 0 before the first diagonal, then each diagonal's line minus EXTRA_BOUNDS */
  for (q = 0; q < activestart; q++) minactive[q] = 0U;
  diagonal = arr[0]->diagonal;
  for (; q <= arr[0]->queryend; q++)
    minactive[q] = (diagonal + q < EXTRA_BOUNDS) ? chrinit : chrinit + diagonal + q - EXTRA_BOUNDS;
  for (i = 0; i < nunique; i = j) {
    for (j = i + 1; j < nunique && arr[j]->queryend <= arr[i]->queryend; j++) ;
    if (j < nunique) {
      diagonal = arr[i]->diagonal;
      for (; q <= arr[j]->queryend; q++)
        minactive[q] = (diagonal + q < EXTRA_BOUNDS) ? chrinit : chrinit + diagonal + q - EXTRA_BOUNDS;
    }
  }
  for (; q < querylength; q++)   /* the reference drops the diagonal here (diag.c:808) */
    minactive[q] = (diagonal + q < EXTRA_BOUNDS) ? chrinit : chrinit + q - EXTRA_BOUNDS;

  /* maxactive: mirror image from the 3' end */
  for (q = querylength - 1; q > activeend; q--) maxactive[q] = chrterm;
  diagonal = arr[nunique - 1]->diagonal;
  for (; q >= arr[nunique - 1]->querystart; q--) {
    position = diagonal + q + EXTRA_BOUNDS;
    maxactive[q] = (position > genomiclength) ? chrterm : chrinit + position;
  }
  for (i = nunique - 1; i >= 0; i = j) {
    for (j = i - 1; j >= 0 && arr[j]->querystart > arr[i]->querystart; j--) ;
    if (j >= 0) {
      diagonal = arr[i]->diagonal;
      for (; q >= arr[j]->querystart; q--) {
        position = diagonal + q + EXTRA_BOUNDS;
        maxactive[q] = (position > genomiclength) ? chrterm : chrinit + position;
      }
    }
  }
  for (; q >= 0; q--) {
    position = diagonal + q + EXTRA_BOUNDS;
    maxactive[q] = (position > genomiclength) ? chrterm : chrinit + position;
  }
  free(arr);
}

/* ------------------------------------------------------------- stage2.c links */

typedef struct {
  const unsigned int *map;    /* mappings, hit gi = off[q] + hit */
  const int *npos, *off;
  int *consec, *root, *fpos, *fhit, *tracei, *score, *active, *firstactive;
  int tracectr, splicingp, sufflookback, nsufflookback;
  unsigned int maxintronlen;
} Chain;

#define MAP(C, q, h) ((C)->map[(C)->off[q] + (h)])
#define LNK(C, f, q, h) ((C)->f[(C)->off[q] + (h)])

typedef struct {
  int consec, root, pp, ph, score, tracei;
} Best;

static void
finish_link (Chain *C, int q, int hit, const Best *b) {
  int gi = C->off[q] + hit;
  C->consec[gi] = b->consec;
  C->root[gi] = b->root;
  C->fpos[gi] = b->pp;
  C->fhit[gi] = b->ph;
  if (b->pp >= 0) {
    C->tracei[gi] = b->tracei;
    C->score[gi] = b->score;
  } else {                       /* localp (gmap.c:1213) */
    C->tracei[gi] = ++C->tracectr;
    C->score[gi] = INDEXSIZE;
  }
}

/* ranges 0-4 of score_querypos_lookback_one / _mult against one processed query position pq,
   starting at active hit ph; returns the hit where the range-1 skip stopped (the _mult frontier) */
static int
score_ranges (Chain *C, Best *b, int q, unsigned int position, int pq, int ph, int *last_tr, int range1) {
  int qd = q - pq, credit = -qd / INDEXSIZE, gendist, diff, fs, frontier;
  unsigned int pp;
  while (ph != -1 && LNK(C, tracei, pq, ph) == *last_tr) ph = LNK(C, active, pq, ph);   /* range 0 */
  if (ph != -1) *last_tr = LNK(C, tracei, pq, ph);
  if (range1)
    while (ph != -1 && MAP(C, pq, ph) + C->maxintronlen + (unsigned int) qd <= position) ph = LNK(C, active, pq, ph);
  frontier = ph;
  while (ph != -1 && (pp = MAP(C, pq, ph)) + EQUAL_DISTANCE_NOT_SPLICING + (unsigned int) qd < position) {
    gendist = (int) (position - pp);                           /* range 2: > 9 nt of genome skip */
    diff = gendist - qd;
    fs = LNK(C, score, pq, ph) + credit - (C->splicingp ? (diff / TEN_THOUSAND + 1) : (diff + 1));
    if (fs > b->score) {
      b->consec = (diff <= EQUAL_DISTANCE_FOR_CONSECUTIVE) ? LNK(C, consec, pq, ph) + qd : 0;
      b->root = LNK(C, root, pq, ph);
      b->score = fs;
      b->pp = pq;
      b->ph = ph;
      b->tracei = ++C->tracectr;
    }
    ph = LNK(C, active, pq, ph);
  }
  while (ph != -1 && (pp = MAP(C, pq, ph)) + INDEXSIZE <= position) {   /* ranges 3-4 */
    gendist = (int) (position - pp);
    diff = gendist > qd ? gendist - qd : qd - gendist;
    fs = LNK(C, score, pq, ph) + 1;
    if (fs > b->score) {
      b->consec = (diff <= EQUAL_DISTANCE_FOR_CONSECUTIVE) ? LNK(C, consec, pq, ph) + qd : 0;
      b->root = LNK(C, root, pq, ph);
      b->score = fs;
      b->pp = pq;
      b->ph = ph;
      b->tracei = LNK(C, tracei, pq, ph);
    }
    ph = LNK(C, active, pq, ph);
  }
  return frontier;
}

/* the adjacent link (section A): the active hit of pq at position - qd */
static int
adjacent (Chain *C, int pq, int *ph_io, int qd, unsigned int position) {
  int ph = *ph_io;
  unsigned int pp = position;
  while (ph != -1 && (pp = MAP(C, pq, ph)) + (unsigned int) qd < position) ph = LNK(C, active, pq, ph);
  *ph_io = ph;
  return pp + (unsigned int) qd == position;
}

/* score_querypos_lookback_one (stage2.c:1073); proc[0..np) oldest first */
static void
score_one (Chain *C, int q, int hit, const int *proc, int np) {
  unsigned int position = MAP(C, q, hit);
  Best b = {INDEXSIZE, (int) position, -1, -1, 0, 0};
  int nlookback = C->nsufflookback, lookback = C->sufflookback, k, nseen, donep, last_tr, pq, qd, ph;
  if (np > 0) {
    pq = proc[np - 1];
    qd = q - pq;
    ph = C->firstactive[pq];
    if (adjacent(C, pq, &ph, qd, position)) {
      b.consec = LNK(C, consec, pq, ph) + qd;
      b.root = LNK(C, root, pq, ph);
      b.score = LNK(C, score, pq, ph) + qd;
      b.pp = pq;
      b.ph = ph;
      b.tracei = LNK(C, tracei, pq, ph);
      nlookback = 1;
      lookback = C->sufflookback / 2;
    }
  }
  donep = 0;
  last_tr = -1;
  for (k = np - 1, nseen = 0; k >= 0 && b.consec < ENOUGH_CONSECUTIVE && !donep; k--, nseen++) {
    pq = proc[k];
    qd = q - pq;
    if (nseen > nlookback && qd - INDEXSIZE > lookback) donep = 1;
    if ((ph = C->firstactive[pq]) != -1) score_ranges(C, &b, q, position, pq, ph, &last_tr, C->splicingp);
  }
  finish_link(C, q, hit, &b);
}

/* score_querypos_lookback_mult (stage2.c:1470) over hits [low, high) */
static void
score_mult (Chain *C, int q, int low, int high, const int *proc, int np) {
  int nhits = high - low, hiti, adj, adq, n, maxadj = 0, maxnon = 0, overall = 0, adjf, ph, maxseen, nseen, k,
      last_tr, pq, qd;
  int *frontier;
  unsigned int position;
  Best b;
  if (np == 0) {
    for (hiti = 0; hiti < nhits; hiti++) {
      int gi = C->off[q] + low + hiti;
      C->consec[gi] = INDEXSIZE;
      C->root[gi] = (int) MAP(C, q, low + hiti);
      C->fpos[gi] = C->fhit[gi] = -1;
      C->tracei[gi] = ++C->tracectr;
      C->score[gi] = INDEXSIZE;
    }
    return;
  }
  adj = proc[np - 1];
  adq = q - adj;
  frontier = (int *) malloc((size_t) np * sizeof(int));
  for (n = 0; n < np; n++) {
    qd = q - proc[np - 1 - n];
    if (n <= 1 || qd - INDEXSIZE <= C->sufflookback / 2) maxadj = n;
    if (n <= C->nsufflookback || qd - INDEXSIZE <= C->sufflookback) maxnon = n;
    frontier[n] = C->firstactive[proc[np - 1 - n]];
  }
  adjf = C->firstactive[adj];
  for (hiti = 0; hiti < nhits; hiti++) {   /* can the hits be greedy? */
    position = MAP(C, q, low + hiti);
    ph = adjf;
    if (adjacent(C, adj, &ph, adq, position) && LNK(C, consec, adj, ph) + adq > overall)
      overall = LNK(C, consec, adj, ph) + adq;
    adjf = ph;
  }
  adjf = C->firstactive[adj];
  for (hiti = 0; hiti < nhits; hiti++) {
    position = MAP(C, q, low + hiti);
    ph = adjf;
    if (adjacent(C, adj, &ph, adq, position)) {
      b.consec = LNK(C, consec, adj, ph) + adq;
      b.root = LNK(C, root, adj, ph);
      b.pp = adj;
      b.ph = ph;
      b.score = LNK(C, score, adj, ph) + adq;
      b.tracei = LNK(C, tracei, adj, ph);
      maxseen = maxadj;
    } else {
      b.consec = INDEXSIZE;
      b.root = (int) position;
      b.pp = b.ph = -1;
      b.score = 0;
      b.tracei = -1;
      maxseen = maxnon;
    }
    adjf = ph;
    if (overall < GREEDY_NCONSECUTIVE) {
      last_tr = -1;
      for (k = np - 1, nseen = 0; k >= 0 && b.consec < ENOUGH_CONSECUTIVE && nseen <= maxseen; k--, nseen++) {
        if ((ph = frontier[nseen]) != -1) {
          pq = proc[k];
          frontier[nseen] = score_ranges(C, &b, q, position, pq, ph, &last_tr, 1);
        }
      }
    }
    finish_link(C, q, low + hiti, &b);
  }
  free(frontier);
}

/* revise_active_lookback (stage2.c:2956) */
static void
revise_active (Chain *C, int q, int low, int high) {
  int best, threshold, hit, *ptr;
  if (low >= high) {
    C->firstactive[q] = -1;
    return;
  }
  best = LNK(C, score, q, low);
  for (hit = low + 1; hit < high; hit++)
    if (LNK(C, score, q, hit) > best) best = LNK(C, score, q, hit);
  threshold = best - SCORE_FOR_RESTRICT;
  if (threshold < 0) threshold = 0;
  C->firstactive[q] = -1;
  ptr = &C->firstactive[q];
  hit = low;
  while (hit < high) {
    while (hit < high && LNK(C, score, q, hit) <= threshold) hit++;
    *ptr = hit;
    if (hit < high) {
      ptr = &LNK(C, active, q, hit);
      hit++;
    }
  }
  *ptr = -1;
}

typedef struct {
  int root, endpos, querypos, hit, score;
} OCell;

static int
cell_root_cmp (const void *x, const void *y) {   /* Cell_rootposition_left_cmp (stage2.c:3230) */
  const OCell *a = *(OCell * const *) x, *b = *(OCell * const *) y;
  if (a->root != b->root) return a->root < b->root ? -1 : 1;
  if (a->score != b->score) return a->score > b->score ? -1 : 1;
  if (a->querypos != b->querypos) return a->querypos > b->querypos ? -1 : 1;
  if (a->hit != b->hit) return a->hit < b->hit ? -1 : 1;
  return 0;
}

static int
cell_score_cmp (const void *x, const void *y) {  /* Cell_score_cmp (stage2.c:3323) */
  const OCell *a = *(OCell * const *) x, *b = *(OCell * const *) y;
  return (a->score > b->score) ? -1 : (b->score > a->score) ? 1 : 0;
}

typedef struct {
  OrcPair *p;
  int n, cap, overflow;
} Sink;

static void
push (Sink *s, int querypos, int genomepos, char cdna, char comp, char g, char galt) {
  if (querypos < 0 || genomepos < 0) return;  /* Pairpool_push (pairpool.c:190) */
  if (s->n >= s->cap) { s->overflow = 1; return; }
  OrcPair *r = &s->p[s->n++];
  memset(r, 0, sizeof(*r));
  r->querypos = querypos;
  r->genomepos = genomepos;
  r->cdna = cdna;
  r->comp = comp;
  r->genome = g;
  r->genomealt = galt;
}

static void
gapholder (Sink *s, int queryjump, int genomejump) {  /* Pairpool_push_gapholder (pairpool.c:375) */
  if (s->n >= s->cap) { s->overflow = 1; return; }
  OrcPair *r = &s->p[s->n++];
  memset(r, 0, sizeof(*r));
  r->querypos = r->genomepos = -1;
  r->queryjump = queryjump;
  r->genomejump = genomejump;
  r->cdna = r->comp = r->genome = r->genomealt = ' ';
  r->gapp = 1;
}

static const char complement_lc[128] =
  "???????????????????????????????? ??#$%&')(*+,-./0123456789:;>=<??TVGHEFCDIJMLKNOPQYSAABWXRZ]?[^_`tvghefcdijmlknopqysaabwxrz}|{~?";

/* get_genomic_nt (stage2.c:4124): no chromosome-bound check */
static char
genomic_nt (char *alt, unsigned int chrpos, unsigned int chroffset, unsigned int chrhigh, int plusp) {
  unsigned int length;
  const char *g = orc_genome_seq(&length);
  unsigned int pos = plusp ? chroffset + chrpos : chrhigh - chrpos;
  char c = (pos < length) ? g[pos] : 'N';
  if (c != 'A' && c != 'C' && c != 'G' && c != 'T') c = 'N';  /* flagged blocks read 'N' */
  if (!plusp) c = complement_lc[(int) c];
  *alt = c;
  return c;
}

/* traceback_one (stage2.c:4140) + List_reverse + convert_to_nucleotides (stage2.c:5334): the path
   from cell (q, hit) back to its root, as the ascending-querypos pair list Stage2_compute keeps as
   `middle`.  Returns the number of records appended to s. */
static int
emit_path (Chain *C, Sink *s, int q, int hit, const char *queryseq, const char *queryuc, unsigned int chroffset,
           unsigned int chrhigh, int plusp, int *pathq, int *pathh) {
  int n = 0, pq, i, start = s->n, lastq, lastg, qj, gj, fill, querypos, genomepos;
  char c, calt;
  while (q >= 0 && LNK(C, consec, q, hit) < MIN_TERMINAL_NCONSECUTIVE) {   /* prune the 3' end */
    pq = q;
    q = LNK(C, fpos, pq, hit);
    hit = LNK(C, fhit, pq, hit);
  }
  while (q >= 0) {   /* the path, 3' end first (= List_reverse of traceback_one's list) */
    if ((int) MAP(C, q, hit) >= 0) { pathq[n] = q; pathh[n] = hit; n++; }  /* Pairpool_push drops < 0 */
    pq = q;
    q = LNK(C, fpos, pq, hit);
    hit = LNK(C, fhit, pq, hit);
  }
  if (n == 0) return 0;
  /* convert_to_nucleotides prepends, walking 3' to 5'; build the list in reverse and flip it */
  querypos = pathq[0];
  genomepos = (int) MAP(C, pathq[0], pathh[0]);
  for (lastq = querypos + INDEXSIZE - 1, lastg = genomepos + INDEXSIZE - 1; lastq > querypos; lastq--, lastg--) {
    c = genomic_nt(&calt, (unsigned int) lastg, chroffset, chrhigh, plusp);
    push(s, lastq, lastg, queryseq[lastq], '|', c, calt);
  }
  push(s, querypos, genomepos, queryseq[querypos], '|', queryuc[querypos], queryuc[querypos]);
  lastq = querypos;
  lastg = genomepos;
  for (i = 1; i < n; i++) {
    querypos = pathq[i];
    genomepos = (int) MAP(C, pathq[i], pathh[i]);
    qj = lastq - 1 - querypos;
    gj = lastg - 1 - genomepos;
    if (qj != 0 || gj != 0) {
      if (querypos + INDEXSIZE - 1 >= lastq || genomepos + INDEXSIZE - 1 >= lastg)
        fill = (lastq - querypos < lastg - genomepos) ? lastq - querypos - 1 : lastg - genomepos - 1;
      else
        fill = INDEXSIZE - 1;
      qj -= fill;
      gj -= fill;
      if (gj > 0 || qj > 0) gapholder(s, qj, gj);
      for (lastq = querypos + fill, lastg = genomepos + fill; lastq > querypos; lastq--, lastg--) {
        c = genomic_nt(&calt, (unsigned int) lastg, chroffset, chrhigh, plusp);
        push(s, lastq, lastg, queryseq[lastq], '|', c, calt);
      }
    }
    push(s, querypos, genomepos, queryseq[querypos], '|', queryuc[querypos], queryuc[querypos]);
    lastq = querypos;
    lastg = genomepos;
  }
  /* records were appended in prepend order: reverse to the list order */
  for (i = start, n = s->n - 1; i < n; i++, n--) {
    OrcPair t = s->p[i];
    s->p[i] = s->p[n];
    s->p[n] = t;
  }
  return s->n - start;
}

typedef struct {
  int offset, npairs;
  unsigned int start, end;    /* genomepos of the first and last pair */
} OPath;

static int
path_cmp (const void *x, const void *y) {   /* stage2_cmp (stage2.c:5740) */
  const OPath *a = *(OPath * const *) x, *b = *(OPath * const *) y;
  if (a->start != b->start) return a->start < b->start ? -1 : 1;
  if (a->end != b->end) return a->end < b->end ? -1 : 1;
  return 0;
}

/* stage2pairs_overlap_p (stage2.c:5925) */
static int
overlap_p (const OPath *x, const OPath *y) {
  unsigned int overlap;
  double fraction;
  if (y->start > x->end || x->start > y->end) return 0;
  if (y->start < x->start) {
    if (y->end < x->end) {
      overlap = y->end - x->start;
      fraction = (y->end - y->start < x->end - x->start) ? (double) overlap / (double) (y->end - y->start)
                                                         : (double) overlap / (double) (x->end - x->start);
      return fraction > 0.5;
    }
    return 1;
  }
  if (y->end < x->end) return 1;
  overlap = x->end - y->start;
  fraction = (y->end - y->start < x->end - x->start) ? (double) overlap / (double) (y->end - y->start)
                                                     : (double) overlap / (double) (x->end - x->start);
  return fraction > 0.5;
}

/* Test instrumentation: when set, the next orc_stage2_compute writes its minactive, maxactive
   (querylength each) and per hit {map, consec, root, fpos, fhit, tracei, score, active} (8 ints, hits
   in querypos order) here. */
static int *S_debug = NULL;
int
orc_stage2_debug (int *buf) {
  S_debug = buf;
  return 0;
}

int
orc_stage2_compute (const char *queryseq, const char *queryuc, int querylength, unsigned int chrstart,
                    unsigned int chrend, unsigned int chroffset, unsigned int chrhigh, int plusp, int splicingp,
                    int maxintronlen, int *scalars, int *paths, int path_cap, OrcPair *pairs, int pair_cap) {
  int *npos, sc[4], *dg, nd, npositions_total, i, q, hit, ncovered, count, *cover, qstart, qend, low, high,
      nskipped, min_hits, specific_q, specific_low = 0, specific_high = 0, next_q, best_hit, best_score,
      grand_score, grand_q, grand_hit, *proc, np, ncells, k, bestscore, npaths, nkept, *pathq, *pathh, *elim,
      status = 0, rc;
  unsigned int *positions, *minactive, *maxactive, position, prevposition;
  ODiag *diags;
  Chain Cst, *C = &Cst;
  OCell *cellv, **cells, **sorted;
  OPath *pv, **parr;
  Sink sink = {pairs, 0, pair_cap, 0};
  double pct;
  int pos_cap = 1 << 22, diag_cap = 1 << 16;

  for (i = 0; i < 6; i++) scalars[i] = 0;
  npos = (int *) calloc((size_t) querylength + 1, sizeof(int));
  positions = (unsigned int *) malloc((size_t) pos_cap * sizeof(unsigned int));
  dg = (int *) malloc((size_t) diag_cap * 4 * sizeof(int));
  rc = orc_oligo_mappings(queryuc, querylength, chrstart, chrend, chroffset, chrhigh, plusp, /*minor*/0, npos,
                          positions, pos_cap, sc, dg, diag_cap);
  if (rc < 0) {
    free(npos); free(positions); free(dg);
    return rc;
  }
  npositions_total = sc[0];
  nd = sc[3];
  diags = (ODiag *) calloc((size_t) (nd > 0 ? nd : 1), sizeof(ODiag));
  for (i = 0; i < nd; i++) {
    diags[i].diagonal = (unsigned int) dg[4 * i];
    diags[i].querystart = dg[4 * i + 1];
    diags[i].queryend = dg[4 * i + 2];
    diags[i].nconsecutive = dg[4 * i + 3];
  }
  free(dg);

  /* Diag_update_coverage (diag.c:216) */
  cover = (int *) calloc((size_t) querylength + 1, sizeof(int));
  for (i = 0; i < nd; i++) {
    cover[diags[i].querystart] += 1;
    cover[diags[i].queryend] -= 1;
  }
  for (q = 0, count = 0, ncovered = 0; q < querylength; q++) {
    count += cover[q];
    if (count > 0) ncovered++;
  }
  free(cover);
  pct = (double) ncovered / (double) querylength;
  scalars[2] = ncovered;

  if (npositions_total == 0) {
    status = 0;
  } else if (querylength > 150 && pct < PROCEED_PCTCOVERAGE && ncovered < SUFF_NCOVERED) {
    status = 1;
  } else {
    status = 2;
  }
  scalars[3] = status;
  if (status != 2) {
    free(npos); free(positions); free(diags);
    return 0;
  }

  minactive = (unsigned int *) malloc((size_t) querylength * sizeof(unsigned int));
  maxactive = (unsigned int *) malloc((size_t) querylength * sizeof(unsigned int));
  compute_bounds(&qstart, &qend, minactive, maxactive, diags, nd, querylength, chrstart, chrend, chroffset,
                 chrhigh, plusp);
  scalars[4] = qstart;
  scalars[5] = qend;

  /* Linkmatrix_1d_new / intmatrix_1d_new: one CALLOC'ed row per query position */
  memset(C, 0, sizeof(*C));
  C->npos = npos;
  C->map = positions;
  {
    int *off = (int *) malloc(((size_t) querylength + 1) * sizeof(int));
    for (q = 0, off[0] = 0; q < querylength; q++) off[q + 1] = off[q] + npos[q];
    C->off = off;
  }
  C->consec = (int *) calloc((size_t) npositions_total + 1, sizeof(int));
  C->root = (int *) calloc((size_t) npositions_total + 1, sizeof(int));
  C->fpos = (int *) calloc((size_t) npositions_total + 1, sizeof(int));
  C->fhit = (int *) calloc((size_t) npositions_total + 1, sizeof(int));
  C->tracei = (int *) calloc((size_t) npositions_total + 1, sizeof(int));
  C->score = (int *) calloc((size_t) npositions_total + 1, sizeof(int));
  C->active = (int *) calloc((size_t) npositions_total + 1, sizeof(int));
  C->firstactive = (int *) malloc((size_t) querylength * sizeof(int));
  C->splicingp = splicingp;
  C->maxintronlen = (unsigned int) maxintronlen;
  C->sufflookback = 60;            /* gmap.c:269-270 */
  C->nsufflookback = 5;
  C->tracectr = 0;
  proc = (int *) malloc((size_t) querylength * sizeof(int));
  np = 0;

  /* align_compute_scores_lookback (stage2.c:3746-3816) */
  for (q = 0; q < qstart; q++) C->firstactive[q] = -1;
  while (q <= qend && npos[q] <= 0) C->firstactive[q++] = -1;
  if (q <= qend) {
    for (hit = 0; hit < npos[q]; hit++) {
      LNK(C, fpos, q, hit) = LNK(C, fhit, q, hit) = -1;
      LNK(C, consec, q, hit) = INDEXSIZE;
      LNK(C, tracei, q, hit) = -1;
      LNK(C, score, q, hit) = INDEXSIZE;
    }
    revise_active(C, q, 0, npos[q]);
  }
  grand_score = 0;
  grand_q = grand_hit = -1;
  nskipped = 0;
  min_hits = 1000000;
  specific_q = -1;
  while (q <= qend) {
    best_score = 0;
    best_hit = -1;
    for (hit = 0; hit < npos[q] && MAP(C, q, hit) < minactive[q]; hit++) ;
    low = hit;
    for (; hit < npos[q] && MAP(C, q, hit) <= maxactive[q]; hit++) ;
    high = hit;
    if (high - low >= MAX_NACTIVE && nskipped <= MAX_SKIPPED) {   /* skip_repetitive_p */
      C->firstactive[q] = -1;
      nskipped++;
      if (high - low < min_hits) {
        min_hits = high - low;
        specific_q = q;
        specific_low = low;
        specific_high = high;
      }
      q++;
      continue;
    }
    if (nskipped > MAX_SKIPPED) {   /* back to the most specific skipped position */
      next_q = q;
      q = specific_q;
      low = specific_low;
      high = specific_high;
    } else {
      next_q = q + 1;
    }
    if (high - low > 0) {
      if (high - low == 1) {
        score_one(C, q, low, proc, np);
        if (LNK(C, score, q, low) > 0) {
          best_score = LNK(C, score, q, low);
          best_hit = low;
        }
      } else {
        score_mult(C, q, low, high, proc, np);
        for (hit = low; hit < high; hit++)
          if (LNK(C, score, q, hit) > best_score) {
            best_score = LNK(C, score, q, hit);
            best_hit = hit;
          }
      }
      nskipped = 0;
      min_hits = 1000000;
      specific_q = -1;
      /* grand lookback (stage2.c:3983-4009) */
      if (splicingp && best_hit >= 0 && LNK(C, fhit, q, best_hit) < 0 && grand_q >= 0 && q >= grand_q + INDEXSIZE) {
        if ((best_score = LNK(C, score, grand_q, grand_hit) - (q - grand_q)) > 0) {
          prevposition = MAP(C, grand_q, grand_hit);
          for (hit = low; hit < high; hit++) {
            position = MAP(C, q, hit);
            if (position > prevposition + C->maxintronlen) {
              /* too long */
            } else if (position >= prevposition + INDEXSIZE) {
              LNK(C, consec, q, hit) = INDEXSIZE;
              LNK(C, fpos, q, hit) = grand_q;
              LNK(C, fhit, q, hit) = grand_hit;
              LNK(C, tracei, q, hit) = ++C->tracectr;
              LNK(C, score, q, hit) = best_score;
            }
          }
        }
      }
      if (best_hit >= 0 && best_score >= grand_score && LNK(C, consec, q, best_hit) > EXON_DEFN) {
        grand_score = best_score;
        grand_q = q;
        grand_hit = best_hit;
      }
    }
    revise_active(C, q, low, high);
    if (npos[q] > 0) proc[np++] = q;
    q = next_q;
  }

  if (S_debug) {
    int *d = S_debug;
    memcpy(d, minactive, (size_t) querylength * 4);
    memcpy(d + querylength, maxactive, (size_t) querylength * 4);
    d += 2 * querylength;
    for (i = 0; i < npositions_total; i++, d += 8) {
      d[0] = (int) positions[i]; d[1] = C->consec[i]; d[2] = C->root[i]; d[3] = C->fpos[i]; d[4] = C->fhit[i];
      d[5] = C->tracei[i]; d[6] = C->score[i]; d[7] = C->active[i];
    }
    S_debug = NULL;
  }

  /* get_cells_fwd (stage2.c:3437) */
  cellv = (OCell *) malloc(((size_t) npositions_total + 1) * sizeof(OCell));
  cells = (OCell **) malloc(((size_t) npositions_total + 1) * sizeof(OCell *));
  sorted = (OCell **) malloc(((size_t) npositions_total + 1) * sizeof(OCell *));
  ncells = 0;
  for (q = qstart; q <= qend; q++)
    for (hit = 0; hit < npos[q]; hit++)
      if (LNK(C, score, q, hit) > 0) {
        OCell *c = &cellv[ncells];
        c->root = LNK(C, root, q, hit);
        c->endpos = (int) MAP(C, q, hit);
        c->querypos = q;
        c->hit = hit;
        c->score = LNK(C, score, q, hit);
        cells[ncells] = c;
        ncells++;
      }
  /* Cellpool_push prepends and List_to_array keeps list order: newest cell first */
  for (i = 0; i < ncells / 2; i++) {
    OCell *t = cells[i];
    cells[i] = cells[ncells - 1 - i];
    cells[ncells - 1 - i] = t;
  }
  stable_sort((void **) cells, ncells, cell_root_cmp);
  {
    int last_root = -1, best_for_root = -1;
    for (k = 0, i = 0; i < ncells; i++) {
      if (cells[i]->root != last_root) {
        sorted[k++] = cells[i];
        last_root = cells[i]->root;
        best_for_root = cells[i]->score;
      } else if (cells[i]->score == best_for_root) {
        sorted[k++] = cells[i];
      }
    }
  }
  ncells = k;
  stable_sort((void **) sorted, ncells, cell_score_cmp);

  /* align_compute_lookback (stage2.c:4465-4515): paths of the best cells */
  pathq = (int *) malloc(((size_t) querylength + 1) * sizeof(int));
  pathh = (int *) malloc(((size_t) querylength + 1) * sizeof(int));
  pv = (OPath *) malloc((size_t) (ncells + 1) * sizeof(OPath));
  npaths = 0;
  if (ncells > 0) {
    bestscore = sorted[0]->score;
    for (i = 0; i < ncells && (i < MAX_NALIGNMENTS || sorted[i]->score == bestscore) &&
                sorted[i]->score > bestscore - FINAL_SCORE_TOLERANCE; i++) {
      int off0 = sink.n, n = emit_path(C, &sink, sorted[i]->querypos, sorted[i]->hit, queryseq, queryuc, chroffset,
                                        chrhigh, plusp, pathq, pathh);
      pv[npaths].offset = off0;
      pv[npaths].npairs = n;
      if (n > 0 && !sink.overflow) {
        pv[npaths].start = (unsigned int) sink.p[off0].genomepos;
        pv[npaths].end = (unsigned int) sink.p[off0 + n - 1].genomepos;
      } else {
        pv[npaths].start = pv[npaths].end = 0;
      }
      npaths++;
    }
  }
  scalars[1] = npaths;

  /* Stage2_filter_unique (stage2.c:6013): all_stage2results lists the paths in cell order */
  parr = (OPath **) malloc((size_t) (npaths + 1) * sizeof(OPath *));
  elim = (int *) calloc((size_t) npaths + 1, sizeof(int));
  for (i = 0; i < npaths; i++) parr[i] = &pv[i];
  stable_sort((void **) parr, npaths, path_cmp);
  for (i = 0; i < npaths; i++)
    for (k = i + 1; k < npaths; k++)
      if (overlap_p(parr[i], parr[k])) elim[k] = 1;
  for (nkept = 0, i = 0; i < npaths; i++) {
    if (elim[i]) continue;
    if (nkept < path_cap) {
      paths[2 * nkept] = parr[i]->offset;
      paths[2 * nkept + 1] = parr[i]->npairs;
    }
    nkept++;
  }
  scalars[0] = nkept;

  free(elim); free(parr); free(pv); free(pathq); free(pathh);
  free(cellv); free(cells); free(sorted); free(proc);
  free(C->consec); free(C->root); free(C->fpos); free(C->fhit); free(C->tracei); free(C->score);
  free(C->active); free(C->firstactive); free((void *) C->off);
  free(minactive); free(maxactive); free(diags); free(npos); free(positions);
  if (sink.overflow || nkept > path_cap) return -1;
  return nkept;
}

/* Test instrumentation (whole-block parity, tests/test_gpu_stage2_plan.py): n orc_stage2_compute calls
   on the current genome over `nthreads` threads (the restatement keeps no state between calls but the
   genome, which is only read).  Call i reads qseq / quc at qoff[i]; it writes scalars[8 i ...] = {its
   return value (nkept, or < 0), npaths, ncovered, status, diag_querystart, diag_queryend, 0, 0},
   paths[2 (path_cap i + k) ...] = {first record, records} of kept path k, and its pair records from
   pairs[pair_off[i]] on, pair_off[i + 1] - pair_off[i] at most (else scalars[8 i] = -9), in the engine's
   gmapdp_path_pair layout
   (20 B: querypos, genomepos, queryjump, genomejump, cdna, comp, genome, genomealt). */
#include <pthread.h>

typedef struct {
  int querypos, genomepos, queryjump, genomejump;
  char cdna, comp, genome, genomealt;
} OrcPathPair;

typedef struct {
  int n;
  const char *qseq, *quc;
  const int *qoff, *qlen, *plusp, *splicingp, *maxintronlen;
  const unsigned int *chrstart, *chrend, *chroffset, *chrhigh;
  int *scalars, *paths, path_cap;
  OrcPathPair *pairs;
  const long *pair_off;
  int next;
  pthread_mutex_t lock;
} S2Batch;

static void *
s2batch_worker (void *arg) {
  S2Batch *B = (S2Batch *) arg;
  int *kp = (int *) malloc(2 * (size_t) B->path_cap * sizeof(int));
  for (;;) {
    int i, k, j, r, cap;
    OrcPair *tmp;
    pthread_mutex_lock(&B->lock);
    i = B->next++;
    pthread_mutex_unlock(&B->lock);
    if (i >= B->n) break;
    cap = 64 * B->qlen[i] > (1 << 18) ? 64 * B->qlen[i] : (1 << 18);  /* every traced path's records */
    tmp = (OrcPair *) malloc((size_t) cap * sizeof(OrcPair));
    r = orc_stage2_compute(B->qseq + B->qoff[i], B->quc + B->qoff[i], B->qlen[i], B->chrstart[i], B->chrend[i],
                           B->chroffset[i], B->chrhigh[i], B->plusp[i], B->splicingp[i], B->maxintronlen[i],
                           B->scalars + 8 * (size_t) i, kp, B->path_cap, tmp, cap);
    B->scalars[8 * (size_t) i] = r;
    /* kept paths, their records packed from the call's first pair slot on */
    {
      long o = B->pair_off[i];
      int *pp = B->paths + 2 * (size_t) B->path_cap * i;
      for (k = 0; r > 0 && k < r; k++) {
        if (o + kp[2 * k + 1] > B->pair_off[i + 1]) {  /* the call's output slot is too small */
          B->scalars[8 * (size_t) i] = -9;
          break;
        }
        pp[2 * k] = (int) (o - B->pair_off[i]);
        pp[2 * k + 1] = kp[2 * k + 1];
        for (j = 0; j < kp[2 * k + 1]; j++, o++) {
          const OrcPair *x = &tmp[kp[2 * k] + j];
          OrcPathPair *y = &B->pairs[o];
          y->querypos = x->querypos;
          y->genomepos = x->genomepos;
          y->queryjump = x->queryjump;
          y->genomejump = x->genomejump;
          y->cdna = x->cdna;
          y->comp = x->comp;
          y->genome = x->genome;
          y->genomealt = x->genomealt;
        }
      }
    }
    free(tmp);
  }
  free(kp);
  return NULL;
}

int
orc_stage2_batch (int n, const char *qseq, const char *quc, const int *qoff, const int *qlen,
                  const unsigned int *chrstart, const unsigned int *chrend, const unsigned int *chroffset,
                  const unsigned int *chrhigh, const int *plusp, const int *splicingp, const int *maxintronlen,
                  int *scalars, int *paths, int path_cap, void *pairs, const long *pair_off, int nthreads) {
  S2Batch B;
  pthread_t th[64];
  int t;
  if (nthreads < 1) nthreads = 1;
  if (nthreads > 64) nthreads = 64;
  B.n = n; B.qseq = qseq; B.quc = quc; B.qoff = qoff; B.qlen = qlen; B.plusp = plusp; B.splicingp = splicingp;
  B.maxintronlen = maxintronlen; B.chrstart = chrstart; B.chrend = chrend; B.chroffset = chroffset;
  B.chrhigh = chrhigh; B.scalars = scalars; B.paths = paths; B.path_cap = path_cap;
  B.pairs = (OrcPathPair *) pairs; B.pair_off = pair_off; B.next = 0;
  pthread_mutex_init(&B.lock, NULL);
  for (t = 0; t < nthreads; t++) pthread_create(&th[t], NULL, s2batch_worker, &B);
  for (t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
  pthread_mutex_destroy(&B.lock);
  return 0;
}
