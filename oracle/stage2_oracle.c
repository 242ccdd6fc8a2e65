/* oracle/stage2_oracle.c -- TEST INFRASTRUCTURE ONLY (never shipped, never on the product path).
 *
 * CPU restatement of GMAP's stage-2 seeding, as Stage2_compute runs it for GMAP
 * (stage2.c:6413-6501: one oligoindex source, coveredp all false):
 *   Oligoindex_set_inquery     oligoindex_hr.c:33454 (trimp false: the query's 8-mers)
 *   Oligoindex_hr_tally        :33849 -> count_positions_fwd/rev_std :19260/:30761 (8-mers starting
 *                              in [mappingstart, mappingend - 8], only when that range has more than
 *                              one start; Count_T is unsigned char, so counts wrap mod 256),
 *                              Oligoindex_allocate_positions :32520 (counts masked by inquery, table
 *                              slices in oligo order), store_positions_fwd/rev_std :20426/:31741
 *                              (walking from the chrpos origin's far end, each oligo keeps its
 *                              `count` occurrences nearest that end, stored in ascending chrpos)
 *   Oligoindex_get_mappings    :34127 (per querypos the table slice of its 8-mer; cum_nohits; the
 *                              Genomicdiag_T consecutive-run tracking with diag_lookback and
 *                              suffnconsecutive; good diagonals in the order they reach
 *                              suffnconsecutive, else the best one; Diagpool_push of each)
 * with the oligoindex parameters of Oligoindex_array_new_major / _minor for GMAP
 * (oligoindex_hr.c:8606-8616: indexsize 8, diag_lookback 120 / 60, suffnconsecutive 20 / 10).
 * Genome words are read as .genomecomp codes: A C G T = 0 1 2 3, 'X' and the padding past the
 * genome 3, any other byte (N) 0 -- the 2-bit field Compress_create_blocks_comp stores.
 * Pinned against the reference objects by tests/test_oracle.py.
 */
#include <stdlib.h>
#include <string.h>

#include "gmapdp_oracle.h"

#define K 8
#define OLIGOSPACE 65536

static const char *S_genome;
static unsigned int S_length;

static int
gcode (unsigned long long pos) {
  if (pos >= S_length) return 3;  /* 'X' padding (compress-write.c:640-643) */
  switch (S_genome[pos]) {
  case 'A': case 'a': return 0;
  case 'C': case 'c': return 1;
  case 'G': case 'g': return 2;
  case 'T': case 't': case 'X': case 'x': return 3;
  default: return 0;
  }
}

/* forward 8-mer starting at genome position p, first base most significant */
static unsigned int
kmer_fwd (unsigned long long p) {
  unsigned int m = 0;
  int i;
  for (i = 0; i < K; i++) m = (m << 2) | (unsigned int) gcode(p + i);
  return m;
}

/* its reverse complement: the complemented base at p + 7 most significant */
static unsigned int
kmer_rev (unsigned long long p) {
  unsigned int m = 0;
  int i;
  for (i = K - 1; i >= 0; i--) m = (m << 2) | (unsigned int) (3 - gcode(p + i));
  return m;
}

struct Gdiag {  /* struct Genomicdiag_T (oligoindex_hr.c:106) */
  int i, querypos, best_nconsecutive, nconsecutive, best_consecutive_start, consecutive_start,
      best_consecutive_end;
};

int
orc_oligo_mappings (const char *queryuc, int querylength, unsigned int chrstart, unsigned int chrend,
                    unsigned int chroffset, unsigned int chrhigh, int plusp, int minor, int *npositions,
                    unsigned int *positions, int pos_cap, int *scalars, int *diags, int diag_cap) {
  const int diag_lookback = minor ? 60 : 120, suffn = minor ? 10 : 20;
  unsigned char *inquery, *counts, *work;
  unsigned int *offs, *table = NULL, oligo = 0, m, chrpos0, chrinit, genomiclength;
  unsigned long long left, lpl, p;
  int in_counter, i, q, hit, nhits, total = 0, totalpositions = 0, maxn = 0, n = 0, nd = 0, ngood = 0;
  int *cum_alloc, *cum, *good, best = -1;
  char *init_p;
  struct Gdiag *gd, *ptr;
  unsigned int *mapoff;

  /* oned_matrix_p is only written past get_mappings' chrend <= chrstart return (:34159); the
     harness starts it false */
  scalars[0] = scalars[1] = scalars[2] = scalars[3] = 0;
  memset(npositions, 0, (size_t) querylength * sizeof(int));
  S_genome = orc_genome_seq(&S_length);
  if (querylength <= K) return -3;  /* set_inquery returns before clearing inquery (:33478): stale state */
  inquery = (unsigned char *) calloc(OLIGOSPACE, 1);
  counts = (unsigned char *) calloc(OLIGOSPACE, 1);
  work = (unsigned char *) malloc(OLIGOSPACE);
  offs = (unsigned int *) calloc(OLIGOSPACE, sizeof(unsigned int));
  mapoff = (unsigned int *) calloc((size_t) querylength + 1, sizeof(unsigned int));

  /* Oligoindex_set_inquery (:33490-33515) */
  for (i = 0, in_counter = 0; i < querylength; i++) {
    in_counter++;
    switch (queryuc[i]) {
    case 'A': oligo = oligo << 2; break;
    case 'C': oligo = (oligo << 2) | 1; break;
    case 'G': oligo = (oligo << 2) | 2; break;
    case 'T': oligo = (oligo << 2) | 3; break;
    default: oligo = 0; in_counter = 0; break;
    }
    if (in_counter == K) {
      inquery[oligo & 0xFFFF] = 1;
      in_counter--;
    }
  }

  /* Oligoindex_hr_tally: count, allocate, store */
  left = (unsigned long long) chroffset + chrstart;
  lpl = (unsigned long long) chroffset + chrend + (plusp ? 0 : 1);
  lpl = lpl < K ? 0 : lpl - K;
  chrpos0 = plusp ? chrstart : (chrhigh - chroffset) - chrend;
  /* (the 8-mers rolled along the window: kmer_fwd(p + 1) / kmer_rev(p + 1) from p's -- the same values) */
  if (lpl > left) {
    m = plusp ? kmer_fwd(left) : kmer_rev(left);
    for (p = left;; p++) {
      counts[m] += 1;  /* wraps mod 256 */
      if (p == lpl) break;
      m = plusp ? (((m << 2) | (unsigned int) gcode(p + K)) & 0xFFFFu)
                : ((m >> 2) | ((unsigned int) (3 - gcode(p + K)) << (2 * K - 2)));
    }
  }
  for (m = 0; m < OLIGOSPACE; m++) {
    if (!inquery[m]) counts[m] = 0;
    offs[m] = (unsigned int) total;
    total += counts[m];
  }
  if (total > 0) {
    table = (unsigned int *) malloc((size_t) total * sizeof(unsigned int));
    memcpy(work, counts, OLIGOSPACE);
    if (plusp) {
      m = kmer_fwd(lpl);
      for (p = lpl + 1; p-- > left;) {  /* right to left, chrpos descending */
        if (p < lpl) m = (m >> 2) | ((unsigned int) gcode(p) << (2 * K - 2));  /* kmer_fwd(p) */
        if (work[m]) table[offs[m] + (--work[m])] = chrpos0 + (unsigned int) (p - left);
      }
    } else {
      m = kmer_rev(left);
      for (p = left; p <= lpl; p++) {   /* left to right, chrpos descending */
        if (p > left) m = (m >> 2) | ((unsigned int) (3 - gcode(p + K - 1)) << (2 * K - 2));  /* kmer_rev(p) */
        if (work[m]) table[offs[m] + (--work[m])] = chrpos0 + (unsigned int) (lpl - p);
      }
    }
  }

  /* Oligoindex_get_mappings (:34159-34346) */
  if (chrend > chrstart) {
    scalars[2] = 1;
    genomiclength = chrend - chrstart;
    chrinit = plusp ? chrstart : (chrhigh - chroffset) - chrend;
    init_p = (char *) calloc((size_t) querylength + genomiclength + 1, 1);
    gd = (struct Gdiag *) calloc((size_t) querylength + genomiclength + 1, sizeof(struct Gdiag));
    cum_alloc = (int *) calloc((size_t) querylength + K + 1, sizeof(int));
    cum = cum_alloc + K + 1;
    good = (int *) malloc(((size_t) querylength + genomiclength + 1) * sizeof(int));
    oligo = 0;
    q = -K;
    for (i = 0, in_counter = 0; i < querylength; i++) {
      in_counter++;
      q++;
      switch (queryuc[i]) {
      case 'A': oligo = oligo << 2; break;
      case 'C': oligo = (oligo << 2) | 1; break;
      case 'G': oligo = (oligo << 2) | 2; break;
      case 'T': oligo = (oligo << 2) | 3; break;
      default: oligo = 0; in_counter = 0; break;
      }
      cum[q] = cum[q - 1];
      if (in_counter == K) {
        m = oligo & 0xFFFF;
        nhits = counts[m];  /* lookup (:34069) */
        npositions[q] = nhits;
        mapoff[q] = offs[m];
        if (nhits <= 0) {
          cum[q] += 1;
        } else {
          totalpositions += nhits;
          for (hit = 0; hit < nhits; hit++) {
            unsigned int diagi = table[offs[m] + hit] + (unsigned int) (querylength - q) - chrinit;
            if (diagi > (unsigned int) querylength + genomiclength) {
              n = -4;  /* the reference asserts (:34255) */
              continue;
            }
            ptr = &gd[diagi];
            if (!init_p[diagi]) {
              init_p[diagi] = 1;
              ptr->i = (int) diagi;
              ptr->querypos = -diag_lookback;
              ptr->best_nconsecutive = 0;
              ptr->nconsecutive = 0;
              ptr->consecutive_start = 0;
            }
            if (ptr->querypos < 0) {  /* querystart 0 */
              ptr->nconsecutive = 0;
              ptr->consecutive_start = q;
            } else if (q - ptr->querypos >= diag_lookback + cum[q] - cum[ptr->querypos]) {
              ptr->nconsecutive = 0;
              ptr->consecutive_start = q;
            } else if (++ptr->nconsecutive > ptr->best_nconsecutive) {
              ptr->best_consecutive_start = ptr->consecutive_start;
              ptr->best_consecutive_end = q;
              ptr->best_nconsecutive = ptr->nconsecutive;
              if (ptr->best_nconsecutive == suffn) good[ngood++] = (int) diagi;
              if (ptr->best_nconsecutive > maxn) {
                best = (int) diagi;
                maxn = ptr->best_nconsecutive;
              }
            }
            ptr->querypos = q;
          }
        }
        in_counter--;
      }
    }
    if (ngood == 0 && maxn > 0) good[ngood++] = best;
    /* List_push then pop-and-Diagpool_push: the returned list runs in the order the diagonals
       reached suffnconsecutive */
    for (i = 0; i < ngood; i++) {
      ptr = &gd[good[i]];
      if (nd < diag_cap) {
        diags[4 * nd + 0] = ptr->i >= querylength ? ptr->i - querylength : querylength - ptr->i;
        diags[4 * nd + 1] = ptr->best_consecutive_start;
        diags[4 * nd + 2] = ptr->best_consecutive_end;
        diags[4 * nd + 3] = ptr->best_nconsecutive + 1;
      }
      nd++;
    }
    free(init_p);
    free(gd);
    free(cum_alloc);
    free(good);
  }
  if (n == 0) {
    for (q = 0; q < querylength; q++) {
      if (npositions[q] <= 0) continue;
      if (n + npositions[q] > pos_cap) { n = -1; break; }
      memcpy(positions + n, table + mapoff[q], (size_t) npositions[q] * sizeof(unsigned int));
      n += npositions[q];
    }
  }
  scalars[0] = totalpositions;
  scalars[1] = maxn;
  scalars[3] = nd;
  free(inquery); free(counts); free(work); free(offs); free(mapoff); free(table);
  return (n >= 0 && nd > diag_cap) ? -1 : n;
}
