/* oracle/microexon_oracle.c -- TEST INFRASTRUCTURE ONLY (see gmapdp_oracle.h).
 *
 * CPU restatement of Dynprog_microexon_int (dynprog_single.c:900-1182), the microexon search GMAP's
 * stage 3 runs inside an intron (stage3.c:9664), written from a reading of the reference:
 *   - the two mismatch-bounded starts (leftbound, rightbound: :1001-1047);
 *   - for every cL with the intron's 5' dinucleotide and every cR with its 3' dinucleotide
 *     (:1053-1085), the middle piece searched exactly in the intron (BoyerMoore_nt,
 *     boyer-moore.c:356: every occurrence j in [0, textlen - querylen], listed by Intlist_push, i.e.
 *     in descending j; no occurrence when the piece holds anything but A/C/G/T, query_okay :263);
 *   - each occurrence flanked by the 3' and 5' dinucleotides is a candidate (:1109-1116) scored by
 *     two MaxEnt probabilities (:1120-1144), kept when (float) prob2 + (float) prob3 beats the best
 *     so far (:1147, float arithmetic);
 *   - the winner becomes make_microexon_pairs_double (:683): left piece, gap holder, microexon, gap
 *     holder, right piece, the gap holders' comp set to the intron direction's character.
 * The MaxEnt probabilities are an input (the host's Maxent_hr_*_prob at the positions
 * orc_microexon_candidates lists), as for orc_genome_gap.
 */
#include <float.h>
#include <limits.h>
#include <stdlib.h>
#include <string.h>

#include "gmapdp_oracle.h"

#define MIN_MICROEXON_LENGTH 3    /* dynprog_single.c:83 */
#define MAX_MICROEXON_LENGTH 12   /* :87 (GMAP, not PMAP) */
#define MICROINTRON_LENGTH 9      /* :89 */
#define GTAG_FWD 0x20             /* intron.h:27 */
#define GTAG_REV 0x04             /* intron.h:31 */
#define NONINTRON 0x00            /* intron.h:35 */
#define FWD_CANONICAL_INTRON_COMP '>'  /* comp.h:15 */
#define REV_CANONICAL_INTRON_COMP '<'  /* comp.h:18 */
#define DYNPROG_MATCH_COMP '*'
#define AMBIGUOUS_COMP ':'
#define MISMATCH_COMP ' '
enum { M_DONOR = 0, M_ACCEPTOR = 1, M_ANTIDONOR = 2, M_ANTIACCEPTOR = 3 };

static const char compl_code[128] = {
  ['A'] = 'T', ['C'] = 'G', ['G'] = 'C', ['T'] = 'A', ['N'] = 'N', ['*'] = '*', ['X'] = 'X',
  ['a'] = 't', ['c'] = 'g', ['g'] = 'c', ['t'] = 'a', ['n'] = 'n', [' '] = ' ', ['-'] = '-'};

/* get_genomic_nt (dynprog_single.c:116) over the oracle genome (no alternate genome) */
static char
genomic_nt (int genomicpos, unsigned int chroffset, unsigned int chrhigh, int watsonp) {
  unsigned int len, pos;
  const char *g = orc_genome_seq(&len);
  if (watsonp) {
    pos = chroffset + (unsigned int) genomicpos;
    if (pos < chroffset || pos >= chrhigh) return '*';
    return g[pos];
  }
  pos = chrhigh - (unsigned int) genomicpos;
  if (pos < chroffset || pos >= chrhigh) return '*';
  return compl_code[(int) g[pos]];
}

static int
query_okay (const char *q, int n) {
  int i;
  for (i = 0; i < n; i++)
    if (q[i] != 'A' && q[i] != 'C' && q[i] != 'G' && q[i] != 'T') return 0;
  return 1;
}

/* BoyerMoore_nt's hit list, head first (descending j).  Returns the number of hits. */
static int
exact_hits (const char *query, int querylen, int textoffset, int textlen, unsigned int chroffset,
            unsigned int chrhigh, int watsonp, int **hits, int *hcap) {
  char *text, *alt;
  int j, n = 0, len = textlen + querylen;
  if (!query_okay(query, querylen)) return 0;
  text = (char *) malloc((size_t) len + 1);
  alt = (char *) malloc((size_t) len + 1);
  if (watsonp) orc_get_segment(1, chroffset + (unsigned int) textoffset, len, chrhigh, 0, text, alt);
  else orc_get_segment(0, chrhigh - (unsigned int) textoffset + 1u, len, chroffset, 1, text, alt);
  if (text[0] != '\0') {
    for (j = textlen - querylen; j >= 0; j--) {
      if (memcmp(query, text + j, (size_t) querylen) == 0) {
        if (n >= *hcap) {
          *hcap = 2 * *hcap + 16;
          *hits = (int *) realloc(*hits, sizeof(int) * (size_t) *hcap);
        }
        (*hits)[n++] = j;
      }
    }
  }
  free(text);
  free(alt);
  return n;
}

typedef struct {
  int cL, cR, candidate, middlelength;
  unsigned int pos2, pos3;
  int model2, model3;
} Cand;

/* The candidates in the reference's loop order.  Returns their number, or -2 for cdna_direction 0
   (the reference returns NULL with NONINTRON before searching). */
static int
search (const char *rsequence, const char *rsequenceuc, int rlength, int goffsetL, int rev_goffsetR,
        int cdna_direction, unsigned int chroffset, unsigned int chrhigh, int watsonp, Cand **out, int *ocap) {
  char intron1, intron2, intron3, intron4, c;
  int leftbound, rightbound, nmismatches, i, cL, cR, mincR, maxcR, middlelength, textleft, textright, k, nh, n = 0;
  int *hits = NULL, hcap = 0;
  if (cdna_direction > 0) {
    intron1 = 'G'; intron2 = 'T'; intron3 = 'A'; intron4 = 'G';
  } else if (cdna_direction < 0) {
    intron1 = 'C'; intron2 = 'T'; intron3 = 'A'; intron4 = 'C';
  } else {
    return -2;
  }
  leftbound = 0;
  nmismatches = 0;
  while (leftbound < rlength - 1 && nmismatches <= 1) {
    c = genomic_nt(goffsetL + leftbound, chroffset, chrhigh, watsonp);
    if (rsequenceuc[leftbound] != c) nmismatches++;
    leftbound++;
  }
  leftbound--;
  rightbound = 0;
  i = rlength - 1;
  nmismatches = 0;
  while (i >= 0 && nmismatches <= 1) {
    c = genomic_nt(rev_goffsetR - rightbound, chroffset, chrhigh, watsonp);
    if (rsequenceuc[i] != c) nmismatches++;
    rightbound++;
    i--;
  }
  rightbound--;
  for (cL = 1; cL <= leftbound; cL++) {
    if (genomic_nt(goffsetL + cL, chroffset, chrhigh, watsonp) != intron1 ||
        genomic_nt(goffsetL + cL + 1, chroffset, chrhigh, watsonp) != intron2)
      continue;
    mincR = rlength - MAX_MICROEXON_LENGTH - cL;
    if (mincR < 1) mincR = 1;
    maxcR = rlength - MIN_MICROEXON_LENGTH - cL;
    if (maxcR > rightbound) maxcR = rightbound;
    for (cR = mincR; cR <= maxcR; cR++) {
      if (genomic_nt(rev_goffsetR - cR - 1, chroffset, chrhigh, watsonp) != intron3 ||
          genomic_nt(rev_goffsetR - cR, chroffset, chrhigh, watsonp) != intron4)
        continue;
      middlelength = rlength - cL - cR;
      textleft = goffsetL + cL + MICROINTRON_LENGTH;
      textright = rev_goffsetR - cR - MICROINTRON_LENGTH;
      if (textright < textleft + middlelength) continue;
      nh = exact_hits(rsequence + cL, middlelength, textleft, textright - textleft, chroffset, chrhigh, watsonp,
                      &hits, &hcap);
      for (k = 0; k < nh; k++) {
        const int cand = textleft + hits[k];
        Cand *e;
        if (genomic_nt(cand - 2, chroffset, chrhigh, watsonp) != intron3 ||
            genomic_nt(cand - 1, chroffset, chrhigh, watsonp) != intron4 ||
            genomic_nt(cand + middlelength, chroffset, chrhigh, watsonp) != intron1 ||
            genomic_nt(cand + middlelength + 1, chroffset, chrhigh, watsonp) != intron2)
          continue;
        if (n >= *ocap) {
          *ocap = 2 * *ocap + 16;
          *out = (Cand *) realloc(*out, sizeof(Cand) * (size_t) *ocap);
        }
        e = &(*out)[n++];
        e->cL = cL; e->cR = cR; e->candidate = cand; e->middlelength = middlelength;
        if (watsonp) {
          e->pos2 = chroffset + (unsigned int) (cand - 1) + 1u;
          e->pos3 = chroffset + (unsigned int) (cand + middlelength);
          e->model2 = cdna_direction > 0 ? M_ACCEPTOR : M_ANTIDONOR;
          e->model3 = cdna_direction > 0 ? M_DONOR : M_ANTIACCEPTOR;
        } else {
          e->pos2 = chrhigh - (unsigned int) (cand - 1);
          e->pos3 = chrhigh - (unsigned int) (cand + middlelength) + 1u;
          e->model2 = cdna_direction > 0 ? M_ANTIACCEPTOR : M_DONOR;
          e->model3 = cdna_direction > 0 ? M_ANTIDONOR : M_ACCEPTOR;
        }
      }
    }
  }
  free(hits);
  return n;
}

int
orc_microexon_candidates (const char *rsequence, const char *rsequenceuc, int rlength, int goffsetL,
                          int rev_goffsetR, int cdna_direction, unsigned int chroffset, unsigned int chrhigh,
                          int watsonp, int *cands, unsigned int *positions, int *models, int cap) {
  Cand *c = NULL;
  int ocap = 0, k, n = search(rsequence, rsequenceuc, rlength, goffsetL, rev_goffsetR, cdna_direction, chroffset,
                              chrhigh, watsonp, &c, &ocap);
  if (n > cap) n = -1;
  for (k = 0; k < n; k++) {
    cands[4 * k] = c[k].cL; cands[4 * k + 1] = c[k].cR;
    cands[4 * k + 2] = c[k].candidate; cands[4 * k + 3] = c[k].middlelength;
    positions[2 * k] = c[k].pos2; positions[2 * k + 1] = c[k].pos3;
    models[2 * k] = c[k].model2; models[2 * k + 1] = c[k].model3;
  }
  free(c);
  return n;
}

/* one of make_microexon_pairs_double's three pieces (:696-714): query rsequence[r0 + i] (querypos
   roffset + r0 + i) against genome position goffset + i */
static void
piece (OrcPair *out, int *n, int max_pairs, const char *rsequence, const char *rsequenceuc, int r0, int roffset,
       int goffset, int length, unsigned int chroffset, unsigned int chrhigh, int watsonp, int genestrand, int dpi) {
  int i;
  unsigned char cons[128 * 128];
  orc_consistent(genestrand, cons);
  for (i = 0; i < length; i++) {
    const char c1 = rsequence[r0 + i], c1_uc = rsequenceuc[r0 + i];
    const char c2 = genomic_nt(goffset + i, chroffset, chrhigh, watsonp);
    char comp;
    if (roffset + r0 + i < 0 || goffset + i < 0) continue;  /* Pairpool_push drops them (pairpool.c:188) */
    if (c1_uc == c2) comp = DYNPROG_MATCH_COMP;
    else if (cons[(unsigned char) c1_uc * 128 + (unsigned char) c2]) comp = AMBIGUOUS_COMP;
    else comp = MISMATCH_COMP;
    if (*n < max_pairs) {
      OrcPair *p = &out[*n];
      p->querypos = roffset + r0 + i; p->genomepos = goffset + i; p->queryjump = 0; p->genomejump = 0;
      p->dynprogindex = dpi; p->cdna = c1; p->comp = comp; p->genome = c2; p->genomealt = c2; p->gapp = 0;
    }
    (*n)++;
  }
}

static void
gapholder (OrcPair *out, int *n, int max_pairs, int genomejump, char gapchar) {
  if (*n < max_pairs) {
    OrcPair *p = &out[*n];
    p->querypos = -1; p->genomepos = -1; p->queryjump = 0; p->genomejump = genomejump;
    p->dynprogindex = 0; p->cdna = ' '; p->comp = gapchar; p->genome = ' '; p->genomealt = ' '; p->gapp = 1;
  }
  (*n)++;
}

int
orc_microexon_int (const char *rsequence, const char *rsequenceuc, int rlength, int roffset, int goffsetL,
                   int rev_goffsetR, int cdna_direction, unsigned int chroffset, unsigned int chrhigh, int watsonp,
                   int genestrand, int dynprogindex, const double *cand_probs, int *scalars, double *dscalars,
                   OrcPair *out, int max_pairs) {
  Cand *c = NULL;
  int ocap = 0, k, best = -1, n = 0, i, j;
  float bestprob = 0.0f, prob2, prob3;
  char gapchar;
  const int nc = search(rsequence, rsequenceuc, rlength, goffsetL, rev_goffsetR, cdna_direction, chroffset, chrhigh,
                        watsonp, &c, &ocap);
  dscalars[0] = dscalars[1] = 0.0;
  scalars[0] = dynprogindex;
  if (nc == -2) {
    scalars[1] = NONINTRON;
    return -1;
  }
  scalars[1] = cdna_direction > 0 ? GTAG_FWD : GTAG_REV;
  gapchar = cdna_direction > 0 ? FWD_CANONICAL_INTRON_COMP : REV_CANONICAL_INTRON_COMP;
  for (k = 0; k < nc; k++) {
    prob2 = (float) cand_probs[2 * k];
    prob3 = (float) cand_probs[2 * k + 1];
    if (prob2 + prob3 > bestprob) {
      best = k;
      dscalars[0] = prob2;
      dscalars[1] = prob3;
      bestprob = prob2 + prob3;
    }
  }
  if (best < 0) {
    free(c);
    scalars[1] = NONINTRON;
    return -1;
  }
  {
    const Cand *b = &c[best];
    const int lengthL = b->cL, lengthM = b->middlelength, lengthR = b->cR;
    const int goffsetM = b->candidate, goffsetR = rev_goffsetR - b->cR + 1;
    /* push order: left piece, gap, microexon, gap, right piece */
    piece(out, &n, max_pairs, rsequence, rsequenceuc, 0, roffset, goffsetL, lengthL, chroffset, chrhigh, watsonp,
          genestrand, dynprogindex);
    gapholder(out, &n, max_pairs, goffsetM - (goffsetL + lengthL), gapchar);
    piece(out, &n, max_pairs, rsequence, rsequenceuc, lengthL, roffset, goffsetM, lengthM, chroffset, chrhigh,
          watsonp, genestrand, dynprogindex);
    gapholder(out, &n, max_pairs, goffsetR - (goffsetM + lengthM), gapchar);
    piece(out, &n, max_pairs, rsequence, rsequenceuc, lengthL + lengthM, roffset, goffsetR, lengthR, chroffset,
          chrhigh, watsonp, genestrand, dynprogindex);
  }
  free(c);
  scalars[0] = dynprogindex + (dynprogindex > 0 ? +1 : -1);
  if (n > max_pairs) return -2;
  for (i = 0, j = n - 1; i < j; i++, j--) {  /* push order -> list order */
    OrcPair t = out[i];
    out[i] = out[j];
    out[j] = t;
  }
  return n;
}
