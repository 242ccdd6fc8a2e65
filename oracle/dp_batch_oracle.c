/* oracle/dp_batch_oracle.c -- TEST INFRASTRUCTURE ONLY (see gmapdp_oracle.h).
 *
 * orc_dp_batch: the oracle's Dynprog_single_gap / _end5_gap / _end3_gap / _genome_gap /
 * _microexon_int over a whole batch of engine descriptors (include/gmapdp.h layouts) on a pthread
 * pool, so that a GPU test can compare EVERY call of a bench block with the restatement (VERDICT r5
 * item 2) instead of a sample -- the DP families' counterpart of orc_stage2_batch.  The genome is
 * the one orc_set_genome installed; the caller groups problems by chromosome and rebases them
 * (chroffset 0), as the per-call tests do.  Splice probabilities are the oracle's MaxEnt
 * restatement (maxent_oracle.c; orc_maxent_load first), exactly as tests/dpbind.py's
 * oracle_splice_probs and microexon_probs compute them per call:
 *   genome gaps: zeros outside the size guard (rlength <= 1 or > 660, glengths > 2000), else
 *     Maxent_hr_*_prob at orc_genome_splice_sites' positions;
 *   microexons: the candidates' two sites (orc_microexon_candidates).
 *
 * Outputs, per problem i (kind: 0 single, 1 end, 2 genome gap, 3 microexon):
 *   scal[16 i + ...]: 0 npairs (-1: NULL list), 1.. the call's scalars (single / end: dynprogindex,
 *     score, nmatches, nmismatches, nopens, nindels; genome gap: the 10 of orc_genome_gap;
 *     microexon: dynprogindex, microintrontype), 12 index of the gap holder with a nonzero
 *     queryjump (-1: none), 13 that queryjump, 14 how many holders have one, 15 nonzero when a
 *     non-holder record carries a jump or another dynprogindex than the call's (the engine's
 *     records cannot express that, so the comparison must know);
 *   dscal[2 i + ...]: genome gap left_prob, right_prob; microexon bestprob2, bestprob3;
 *   pairs: the list as the engine's 16-B gmapdp_pair records at pair_off[i] (holders: querypos =
 *     genomepos = -1, jump = genomejump), at most pair_off[i + 1] - pair_off[i] (scal[0] = -9 when
 *     the slot is too small). */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "gmapdp_oracle.h"
#include "../include/gmapdp.h"

typedef struct {
  int kind, n;
  const void *probs;
  const char *q, *quc;
  int *scal;
  double *dscal;
  gmapdp_pair *pairs;
  const long *pair_off;
  int next;
  pthread_mutex_t lock;
} DpBatch;

static void
emit (DpBatch *B, int i, int npairs, const OrcPair *tmp, int dpi) {
  int *s = B->scal + 16 * (size_t) i;
  const long o = B->pair_off[i], cap = B->pair_off[i + 1] - o;
  int k;
  s[0] = npairs;
  s[12] = -1;
  s[13] = 0;
  s[14] = 0;
  s[15] = 0;
  if (npairs > cap) {
    s[0] = -9;
    return;
  }
  for (k = 0; k < npairs; k++) {
    const OrcPair *x = &tmp[k];
    gmapdp_pair *y = &B->pairs[o + k];
    if (x->gapp) {
      y->querypos = -1;
      y->genomepos = -1;
      y->jump = x->genomejump;
      if (x->queryjump != 0) {
        s[12] = k;
        s[13] = x->queryjump;
        s[14]++;
      }
    } else {
      y->querypos = x->querypos;
      y->genomepos = x->genomepos;
      y->jump = 0;
      if (x->queryjump != 0 || x->genomejump != 0 || x->dynprogindex != dpi) s[15] = 1;
    }
    y->cdna = x->cdna;
    y->comp = x->comp;
    y->genome = x->genome;
    y->genomealt = x->genomealt;
  }
}

static void *
dpbatch_worker (void *arg) {
  DpBatch *B = (DpBatch *) arg;
  long cap = 1 << 16;
  OrcPair *tmp = (OrcPair *) malloc((size_t) cap * sizeof(OrcPair));
  double *probs = (double *) malloc(2 * 4096 * sizeof(double));
  unsigned int *pos = (unsigned int *) malloc(2 * 4096 * sizeof(unsigned int));
  int *mod = (int *) malloc(2 * 4096 * sizeof(int));
  for (;;) {
    int i, r, k;
    int sc[16];
    double ds[2] = {0.0, 0.0};
    pthread_mutex_lock(&B->lock);
    i = B->next++;
    pthread_mutex_unlock(&B->lock);
    if (i >= B->n) break;
    memset(sc, 0, sizeof(sc));
    if (B->kind == 0) {
      const gmapdp_single_problem *p = (const gmapdp_single_problem *) B->probs + i;
      r = orc_single_gap(B->q + p->qoff, B->quc + p->qoff, p->rlength, p->glength, p->roffset, p->goffset,
                         (unsigned int) p->chroffset, (unsigned int) p->chrhigh, p->flags & 1, p->genestrand,
                         (p->flags >> 1) & 1, p->extraband, (p->flags >> 2) & 1, p->defect_rate, p->dynprogindex, sc,
                         tmp, (int) cap);
      emit(B, i, r, tmp, p->dynprogindex);
      memcpy(B->scal + 16 * (size_t) i + 1, sc, 6 * sizeof(int));
    } else if (B->kind == 1) {
      const gmapdp_end_problem *p = (const gmapdp_end_problem *) B->probs + i;
      const int qpos = p->end3p ? 0 : (p->rlength > 0 ? p->rlength - 1 : 0);
      r = orc_end_gap(p->end3p, B->q + p->qoff, B->quc + p->qoff, qpos, p->rlength, p->glength, p->roffset, p->goffset,
                      (unsigned int) p->chroffset, (unsigned int) p->chrhigh, p->flags & 1, p->genestrand,
                      (p->flags >> 1) & 1, p->extraband, p->defect_rate, p->endalign, p->require_pos_score_p,
                      p->dynprogindex, sc, tmp, (int) cap);
      emit(B, i, r, tmp, p->dynprogindex);
      memcpy(B->scal + 16 * (size_t) i + 1, sc, 6 * sizeof(int));
    } else if (B->kind == 2) {
      const gmapdp_genome_problem *p = (const gmapdp_genome_problem *) B->probs + i;
      const int gL = p->glengthL > 0 ? p->glengthL : 0, gR = p->glengthR > 0 ? p->glengthR : 0;
      double *lp = probs, *rp = probs + 4096;
      for (k = 0; k < gL && k < 4096; k++) lp[k] = 0.0;
      for (k = 0; k < gR && k < 4096; k++) rp[k] = 0.0;
      if (!(p->rlength <= 1 || p->rlength > 660 || p->glengthL > 2000 || p->glengthR > 2000)) {
        orc_genome_splice_sites(gL, gR, p->goffsetL, p->rev_goffsetR, (unsigned int) p->chroffset,
                                (unsigned int) p->chrhigh, p->cdna_direction, p->flags & 1, pos, mod, pos + 4096,
                                mod + 4096);
        for (k = 0; k < gL; k++) lp[k] = orc_maxent(mod[k], pos[k], (unsigned long long) p->chroffset);
        for (k = 0; k < gR; k++) rp[k] = orc_maxent(mod[4096 + k], pos[4096 + k], (unsigned long long) p->chroffset);
      }
      r = orc_genome_gap(B->q + p->qoff, B->quc + p->qoff, p->rlength, p->glengthL, p->glengthR, p->roffset,
                         p->goffsetL, p->rev_goffsetR, (unsigned int) p->chroffset, (unsigned int) p->chrhigh,
                         p->cdna_direction, p->flags, p->genestrand, p->extraband, p->defect_rate, p->maxpeelback,
                         p->dynprogindex, lp, rp, sc, ds, tmp, (int) cap);
      emit(B, i, r, tmp, p->dynprogindex);
      memcpy(B->scal + 16 * (size_t) i + 1, sc, 10 * sizeof(int));
    } else {
      const gmapdp_microexon_problem *p = (const gmapdp_microexon_problem *) B->probs + i;
      int cands[4 * 4096];
      int nc = orc_microexon_candidates(B->q + p->qoff, B->quc + p->qoff, p->rlength, p->goffsetL, p->rev_goffsetR,
                                        p->cdna_direction, (unsigned int) p->chroffset, (unsigned int) p->chrhigh,
                                        p->watsonp, cands, pos, mod, 4096);
      if (nc == -1) {
        B->scal[16 * (size_t) i] = -8;  /* more candidates than this runner holds */
        continue;
      }
      if (nc < 0) nc = 0;
      for (k = 0; k < 2 * nc; k++) probs[k] = orc_maxent(mod[k], pos[k], (unsigned long long) p->chroffset);
      r = orc_microexon_int(B->q + p->qoff, B->quc + p->qoff, p->rlength, p->roffset, p->goffsetL, p->rev_goffsetR,
                            p->cdna_direction, (unsigned int) p->chroffset, (unsigned int) p->chrhigh, p->watsonp,
                            p->genestrand, p->dynprogindex, probs, sc, ds, tmp, (int) cap);
      emit(B, i, r, tmp, p->dynprogindex);
      memcpy(B->scal + 16 * (size_t) i + 1, sc, 2 * sizeof(int));
    }
    B->dscal[2 * (size_t) i] = ds[0];
    B->dscal[2 * (size_t) i + 1] = ds[1];
  }
  free(tmp);
  free(probs);
  free(pos);
  free(mod);
  return NULL;
}

int
orc_dp_batch (int kind, int n, const void *probs, const char *q, const char *quc, int *scal, double *dscal,
              void *pairs, const long *pair_off, int nthreads) {
  DpBatch B;
  pthread_t th[64];
  int t;
  if (kind < 0 || kind > 3) return -1;
  if (nthreads < 1) nthreads = 1;
  if (nthreads > 64) nthreads = 64;
  B.kind = kind;
  B.n = n;
  B.probs = probs;
  B.q = q;
  B.quc = quc;
  B.scal = scal;
  B.dscal = dscal;
  B.pairs = (gmapdp_pair *) pairs;
  B.pair_off = pair_off;
  B.next = 0;
  pthread_mutex_init(&B.lock, NULL);
  for (t = 0; t < nthreads; t++) pthread_create(&th[t], NULL, dpbatch_worker, &B);
  for (t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
  pthread_mutex_destroy(&B.lock);
  return 0;
}
