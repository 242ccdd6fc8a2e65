/* oracle/refharness.c -- TEST INFRASTRUCTURE ONLY (never shipped, never on the
 * product path).
 *
 * A flat, plain-C API over the *reference's own* compiled Dynprog_* objects
 * (built by oracle/ref.mk into oracle/_ref/librefdp_<variant>.so).  Tests and
 * tests/golden/make_golden.py call it through ctypes to (1) pin the CPU
 * restatement in oracle/gmapdp_oracle.c and (2) generate golden vectors.
 *
 * Everything below only *calls* reference functions; the algorithm lives in the
 * reference objects.  Interfaces used (all /root/reference/src):
 *   Dynprog_init            dynprog.c:1008
 *   Dynprog_new             dynprog.c:631 (sizes as gmap.c:4898-4903)
 *   Dynprog_single_gap      dynprog_single.c:429
 *   Dynprog_end5_gap        dynprog_end.c:1294
 *   Dynprog_end3_gap        dynprog_end.c:1924
 *   Genome_from_sequence    genome.c:307
 *   Pairpool_new/reset      pairpool.c
 *   Oligoindex_hr_setup / _array_new_major / _minor / _hr_tally / _get_mappings / _untally
 *                           oligoindex_hr.c:8672/8808/33849/34127/33994 (stage-2 seeding)
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "bool.h"
#include "mem.h"
#include "list.h"
#include "pair.h"
#include "pairdef.h"
#include "pairpool.h"
#include "sequence.h"
#include "genome.h"
#include "compress-write.h"
#include "dynprog.h"
#include "dynprog_single.h"
#include "dynprog_end.h"
#include "dynprog_genome.h"
#include "dynprog_cdna.h"
#include "maxent_hr.h"
#include "oligoindex_hr.h"
#include "diag.h"
#include "diagpool.h"
#include "cellpool.h"
#include "stage2.h"

/* Flat pair record (matches oracle/gmapdp_oracle.h RefPair / GmapdpPair
 * semantics: one record per Pair_T in list order). */
typedef struct {
  int querypos;
  int genomepos;
  int queryjump;
  int genomejump;
  int dynprogindex;
  char cdna, comp, genome, genomealt;
  int gapp;
} RefPair;

static Dynprog_T dynprogM = NULL, dynprogL = NULL, dynprogR = NULL;
static Pairpool_T pairpool = NULL;
static Genome_T genome = NULL;
static Sequence_T genome_seq = NULL;
static int initialized = 0;

/* gmap.c:259,275-277 and stage3.h:36 defaults */
#define NULLGAP 600
#define EXTRAQUERYGAP 20
#define MAXPEELBACK 60
#define EXTRAMATERIAL_END 10
#define EXTRAMATERIAL_PAIRED 8

int
refh_init (int user_open, int user_extend, int user_dynprog_p) {
  if (initialized) return 0;
  Dynprog_init(STANDARD);
  Dynprog_single_setup(user_open, user_extend, user_dynprog_p ? true : false, /*homopolymerp*/false);
  Dynprog_end_setup(/*splicesites*/NULL, /*splicetypes*/NULL, /*splicedists*/NULL, /*nsplicesites*/0,
                    /*trieoffsets_obs*/NULL, /*triecontents_obs*/NULL,
                    /*trieoffsets_max*/NULL, /*triecontents_max*/NULL,
                    user_open, user_extend, user_dynprog_p ? true : false);
  /* gmap.c:6548 with no splicing IIT (-s not given); novelsplicingp defaults to true (gmap.c:465) */
  Dynprog_genome_setup(/*novelsplicingp*/true, /*splicing_iit*/NULL, /*splicing_divint_crosstable*/NULL,
                       /*donor_typeint*/-1, /*acceptor_typeint*/-1,
                       user_open, user_extend, user_dynprog_p ? true : false);
  dynprogM = Dynprog_new(NULLGAP, EXTRAQUERYGAP, MAXPEELBACK, EXTRAMATERIAL_END, EXTRAMATERIAL_PAIRED, false);
  dynprogL = Dynprog_new(NULLGAP, EXTRAQUERYGAP, MAXPEELBACK, EXTRAMATERIAL_END, EXTRAMATERIAL_PAIRED, true);
  dynprogR = Dynprog_new(NULLGAP, EXTRAQUERYGAP, MAXPEELBACK, EXTRAMATERIAL_END, EXTRAMATERIAL_PAIRED, true);
  pairpool = Pairpool_new();
  initialized = 1;
  return 0;
}

/* Fill the SIMD builds' score and direction arenas (Dynprog_new, dynprog.c:686-731: posix_memalign'd, never
   cleared) with one byte value.  Test instrumentation: Dynprog_simd_{8,16}[_upper/_lower] read
   matrix cells outside the row block they computed (e.g. dynprog_simd.c:3290
   matrix[c-1][rlo-1]), so their output can depend on what earlier calls left there; the tests
   call this to measure that dependence.  A no-op for the nosimd build. */
int
refh_poison_arenas (int byte, int what) {
#ifdef HAVE_SSE2
  size_t one = (size_t)(dynprogM->max_glength + 1) * (dynprogM->max_rlength + SIMD_NCHARS + SIMD_NCHARS) * 2;
  size_t up = (size_t)(dynprogL->max_glength + 1) * (dynprogL->max_rlength + SIMD_NCHARS + SIMD_NCHARS) * 2;
  size_t lo = (size_t)(dynprogL->max_rlength + 1) * (dynprogL->max_glength + SIMD_NCHARS + SIMD_NCHARS) * 2;
  Dynprog_T two[2];
  int k;
  if (what & 1) memset(dynprogM->aligned.one.matrix_space, byte, one);
  if (what & 2) {
    memset(dynprogM->aligned.one.directions_space_0, byte, one);
    memset(dynprogM->aligned.one.directions_space_1, byte, one);
    memset(dynprogM->aligned.one.directions_space_2, byte, one);
  }
  two[0] = dynprogL;
  two[1] = dynprogR;
  for (k = 0; k < 2; k++) {
    if (what & 1) {
      memset(two[k]->aligned.two.upper_matrix_space, byte, up);
      memset(two[k]->aligned.two.lower_matrix_space, byte, lo);
    }
    if (what & 2) {
      memset(two[k]->aligned.two.upper_directions_space_0, byte, up);
      memset(two[k]->aligned.two.upper_directions_space_1, byte, up);
      memset(two[k]->aligned.two.lower_directions_space_0, byte, lo);
      memset(two[k]->aligned.two.lower_directions_space_1, byte, lo);
    }
  }
  return 1;
#else
  (void) byte;
  (void) what;
  return 0;
#endif
}

int
refh_max_lengths (int *max_rlength, int *max_glength) {
  *max_rlength = dynprogM->max_rlength;
  *max_glength = dynprogM->max_glength;
  return 0;
}

/* The genome is wrapped the way GMAP wraps a user-supplied segment (-g):
   Genome_from_sequence (genome.c:307) packs it into .genomecomp blocks. */
int
refh_set_genome (const char *seq, int length) {
  char *copy = (char *) malloc(length + 1);
  memcpy(copy, seq, length);
  copy[length] = '\0';
  genome_seq = Sequence_genomic_new(copy, length, /*copyp*/true);
  genome = Genome_from_sequence(genome_seq);
  free(copy);
  return 0;
}

static int
flatten (List_T pairs, RefPair *out, int max_pairs) {
  int n = 0;
  List_T p;
  Pair_T pair;
  for (p = pairs; p != NULL; p = List_next(p)) {
    pair = (Pair_T) List_head(p);
    if (n < max_pairs) {
      out[n].querypos = pair->querypos;
      out[n].genomepos = (int) pair->genomepos;
      out[n].queryjump = pair->queryjump;
      out[n].genomejump = pair->genomejump;
      out[n].dynprogindex = pair->dynprogindex;
      out[n].cdna = pair->cdna;
      out[n].comp = pair->comp;
      out[n].genome = pair->genome;
      out[n].genomealt = pair->genomealt;
      out[n].gapp = pair->gapp ? 1 : 0;
    }
    n++;
  }
  return n;
}

/* scalars[0..5] = dynprogindex(after), finalscore, nmatches, nmismatches, nopens, nindels.
   Returns number of pairs, or -1 when the reference returned NULL. */
int
refh_single_gap (const char *rsequence, const char *rsequenceuc, int rlength, int glength,
                 int roffset, int goffset, unsigned int chroffset, unsigned int chrhigh,
                 int watsonp, int genestrand, int jump_late_p, int extraband_single, int widebandp,
                 double defect_rate, int dynprogindex, int *scalars, RefPair *out, int max_pairs) {
  List_T pairs;
  int finalscore = 0, nmatches = 0, nmismatches = 0, nopens = 0, nindels = 0, n;

  Pairpool_reset(pairpool);
  pairs = Dynprog_single_gap(&dynprogindex, &finalscore, &nmatches, &nmismatches, &nopens, &nindels,
                             dynprogM, (char *) rsequence, (char *) rsequenceuc, rlength, glength,
                             roffset, goffset, (Univcoord_T) chroffset, (Univcoord_T) chrhigh,
                             watsonp ? true : false, genestrand, jump_late_p ? true : false,
                             genome, genome, pairpool, extraband_single, widebandp ? true : false,
                             defect_rate);
  scalars[0] = dynprogindex; scalars[1] = finalscore; scalars[2] = nmatches;
  scalars[3] = nmismatches; scalars[4] = nopens; scalars[5] = nindels;
  if (pairs == NULL) return -1;
  n = flatten(pairs, out, max_pairs);
  return n;
}

/* CPU baseline loop for bench.py: the reference's Dynprog_single_gap over a
   batch laid out like include/gmapdp.h's gmapdp_single_problem array (the
   struct is restated here; bench.py passes the same bytes to both).  Returns
   the total number of pairs produced. */
typedef struct {
  int qoff, rlength, glength, roffset, goffset;
  unsigned int chroffset, chrhigh;
  int flags, genestrand, extraband;
  double defect_rate;
  int dynprogindex, pad_;
} RefSingleProblem;

long
refh_single_gap_batch (const RefSingleProblem *probs, int n, const char *qseq, const char *qseq_uc) {
  long total = 0;
  int i, dpi, finalscore, nmatches, nmismatches, nopens, nindels;
  List_T pairs;
  for (i = 0; i < n; i++) {
    const RefSingleProblem *p = &probs[i];
    Pairpool_reset(pairpool);
    dpi = p->dynprogindex;
    pairs = Dynprog_single_gap(&dpi, &finalscore, &nmatches, &nmismatches, &nopens, &nindels, dynprogM,
                               (char *) qseq + p->qoff, (char *) qseq_uc + p->qoff, p->rlength, p->glength,
                               p->roffset, p->goffset, (Univcoord_T) p->chroffset, (Univcoord_T) p->chrhigh,
                               (p->flags & 1) ? true : false, p->genestrand, (p->flags & 2) ? true : false,
                               genome, genome, pairpool, p->extraband, (p->flags & 4) ? true : false,
                               p->defect_rate);
    total += List_length(pairs);
  }
  return total;
}

/* Same for Dynprog_end5_gap / Dynprog_end3_gap over include/gmapdp.h's
   gmapdp_end_problem layout (restated). */
typedef struct {
  int qoff, rlength, glength, roffset, goffset;
  unsigned int chroffset, chrhigh;
  int flags, genestrand, extraband, end3p, endalign, require_pos_score_p, dynprogindex;
  double defect_rate;
} RefEndProblem;

long
refh_end_gap_batch (const RefEndProblem *probs, int n, const char *qseq, const char *qseq_uc) {
  long total = 0;
  int i, dpi, score, nmatches, nmismatches, nopens, nindels;
  List_T pairs;
  for (i = 0; i < n; i++) {
    const RefEndProblem *p = &probs[i];
    Pairpool_reset(pairpool);
    dpi = p->dynprogindex;
    if (p->end3p) {
      pairs = Dynprog_end3_gap(&dpi, &score, &nmatches, &nmismatches, &nopens, &nindels, dynprogR,
                               (char *) qseq + p->qoff, (char *) qseq_uc + p->qoff, p->rlength, p->glength,
                               p->roffset, p->goffset, (Univcoord_T) p->chroffset, (Univcoord_T) p->chrhigh,
                               (p->flags & 1) ? true : false, p->genestrand, (p->flags & 2) ? true : false,
                               genome, genome, pairpool, p->extraband, p->defect_rate,
                               (Endalign_T) p->endalign, p->require_pos_score_p ? true : false);
    } else {
      pairs = Dynprog_end5_gap(&dpi, &score, &nmatches, &nmismatches, &nopens, &nindels, dynprogL,
                               (char *) qseq + p->qoff + p->rlength - 1, (char *) qseq_uc + p->qoff + p->rlength - 1,
                               p->rlength, p->glength, p->roffset, p->goffset,
                               (Univcoord_T) p->chroffset, (Univcoord_T) p->chrhigh,
                               (p->flags & 1) ? true : false, p->genestrand, (p->flags & 2) ? true : false,
                               genome, genome, pairpool, p->extraband, p->defect_rate,
                               (Endalign_T) p->endalign, p->require_pos_score_p ? true : false);
    }
    total += List_length(pairs);
  }
  return total;
}

/* endalign: 0 QUERYEND_GAP, 1 QUERYEND_INDELS, 2 QUERYEND_NOGAPS, 3 BEST_LOCAL (dynprog.h:23) */
int
refh_end_gap (int end3p, const char *qbuf, const char *qucbuf, int qpos, int rlength, int glength,
              int roffset, int goffset, unsigned int chroffset, unsigned int chrhigh,
              int watsonp, int genestrand, int jump_late_p, int extraband_end,
              double defect_rate, int endalign, int require_pos_score_p, int dynprogindex,
              int *scalars, RefPair *out, int max_pairs) {
  List_T pairs;
  int finalscore = 0, nmatches = 0, nmismatches = 0, nopens = 0, nindels = 0, n;
  const char *rsequence = qbuf + qpos, *rsequenceuc = qucbuf + qpos;

  Pairpool_reset(pairpool);
  if (end3p) {
    pairs = Dynprog_end3_gap(&dynprogindex, &finalscore, &nmatches, &nmismatches, &nopens, &nindels,
                             dynprogR, (char *) rsequence, (char *) rsequenceuc, rlength, glength,
                             roffset, goffset, (Univcoord_T) chroffset, (Univcoord_T) chrhigh,
                             watsonp ? true : false, genestrand, jump_late_p ? true : false,
                             genome, genome, pairpool, extraband_end, defect_rate,
                             (Endalign_T) endalign, require_pos_score_p ? true : false);
  } else {
    pairs = Dynprog_end5_gap(&dynprogindex, &finalscore, &nmatches, &nmismatches, &nopens, &nindels,
                             dynprogL, (char *) rsequence, (char *) rsequenceuc, rlength, glength,
                             roffset, goffset, (Univcoord_T) chroffset, (Univcoord_T) chrhigh,
                             watsonp ? true : false, genestrand, jump_late_p ? true : false,
                             genome, genome, pairpool, extraband_end, defect_rate,
                             (Endalign_T) endalign, require_pos_score_p ? true : false);
  }
  scalars[0] = dynprogindex; scalars[1] = finalscore; scalars[2] = nmatches;
  scalars[3] = nmismatches; scalars[4] = nopens; scalars[5] = nindels;
  if (pairs == NULL) return -1;
  n = flatten(pairs, out, max_pairs);
  return n;
}

/* Dynprog_end5_splicejunction / Dynprog_end3_splicejunction (dynprog_end.c:1653/2249) with the
   junction string (rev_)gsequence = jbuf + jpos passed as both gsequence and gsequence_alt.
   scalars[0..7] = dynprogindex(after), traceback_score, missscore, nmatches, nmismatches, nopens,
   nindels, list index of the Pair_T with knowngapp (-1 none); the out-parameters start at INT_MIN so
   that unwritten ones show.  chroffset/chrhigh/watsonp only feed the reference's debug paths. */
int
refh_end_splicejunction (int end3p, const char *qbuf, const char *qucbuf, int qpos, const char *jbuf, int jpos,
                         int rlength, int glength, int roffset, int goffset_anchor, int goffset_far, int genestrand,
                         int jump_late_p, int extraband_end, double defect_rate, int contlength, int dynprogindex,
                         int *scalars, RefPair *out, int max_pairs) {
  List_T pairs, p;
  int score = -2147483647 - 1, missscore = score, nmatches = score, nmismatches = score, nopens = score;
  int nindels = score, n, known = -1;
  char *rsequence = (char *) qbuf + qpos, *rsequenceuc = (char *) qucbuf + qpos, *gseq = (char *) jbuf + jpos;

  Pairpool_reset(pairpool);
  if (end3p) {
    pairs = Dynprog_end3_splicejunction(&dynprogindex, &score, &missscore, &nmatches, &nmismatches, &nopens, &nindels,
                                        dynprogR, rsequence, rsequenceuc, gseq, gseq, rlength, glength, roffset,
                                        goffset_anchor, goffset_far, /*chroffset*/0, /*chrhigh*/0, /*watsonp*/true,
                                        genestrand, jump_late_p ? true : false, genome, genome, pairpool,
                                        extraband_end, defect_rate, contlength);
  } else {
    pairs = Dynprog_end5_splicejunction(&dynprogindex, &score, &missscore, &nmatches, &nmismatches, &nopens, &nindels,
                                        dynprogL, rsequence, rsequenceuc, gseq, gseq, rlength, glength, roffset,
                                        goffset_anchor, goffset_far, /*chroffset*/0, /*chrhigh*/0, /*watsonp*/true,
                                        genestrand, jump_late_p ? true : false, genome, genome, pairpool,
                                        extraband_end, defect_rate, contlength);
  }
  scalars[0] = dynprogindex; scalars[1] = score; scalars[2] = missscore; scalars[3] = nmatches;
  scalars[4] = nmismatches; scalars[5] = nopens; scalars[6] = nindels;
  for (n = 0, p = pairs; p != NULL; p = List_next(p), n++)
    if (((Pair_T) List_head(p))->knowngapp && known < 0) known = n;
  scalars[7] = known;
  if (pairs == NULL) return -1;
  return flatten(pairs, out, max_pairs);
}

/* Dynprog_end5_known / Dynprog_end3_known (dynprog_end.c:2748/3009) over a known-site list given here
   (Dynprog_end_setup with the sites and types, no splice tries: trieoffsets NULL, as gmap.c sets them
   up when the tries are empty), then the list reset to none.  types: Splicetype_T values (types.h:130).
   scalars[0..8] = dynprogindex(after), finalscore, ambig_end_length, ambig_splicetype, nmatches,
   nmismatches, nopens, nindels, knownsplicep; unwritten ones stay INT_MIN. */
int
refh_end_known (int end3p, const unsigned int *sites, const int *types, int nsites, const char *qbuf,
                const char *qucbuf, int qpos, int rlength, int glength, int roffset, int goffset, int querylength,
                unsigned int chroffset, unsigned int chrhigh, unsigned int limit_low, unsigned int limit_high,
                int cdna_direction, int watsonp, int genestrand, int jump_late_p, int extraband_end,
                double defect_rate, int dynprogindex, int *scalars, RefPair *out, int max_pairs) {
  List_T pairs;
  Univcoord_T *usites = (Univcoord_T *) calloc(nsites + 1, sizeof(Univcoord_T));
  Splicetype_T *utypes = (Splicetype_T *) calloc(nsites + 1, sizeof(Splicetype_T));
  int score = -2147483647 - 1, ambig_end_length = score, nmatches = score, nmismatches = score, nopens = score;
  int nindels = score, i;
  Splicetype_T ambig_splicetype = (Splicetype_T) score;
  bool knownsplicep = false;
  char *rsequence = (char *) qbuf + qpos, *rsequenceuc = (char *) qucbuf + qpos;

  for (i = 0; i < nsites; i++) {
    usites[i] = (Univcoord_T) sites[i];
    utypes[i] = (Splicetype_T) types[i];
  }
  Dynprog_end_setup(usites, utypes, /*splicedists*/NULL, nsites, NULL, NULL, NULL, NULL, 0, 0, false);
  Pairpool_reset(pairpool);
  if (end3p) {
    pairs = Dynprog_end3_known(&knownsplicep, &dynprogindex, &score, &ambig_end_length, &ambig_splicetype, &nmatches,
                               &nmismatches, &nopens, &nindels, dynprogR, rsequence, rsequenceuc, rlength, glength,
                               roffset, goffset, querylength, chroffset, chrhigh, limit_low, limit_high,
                               cdna_direction, watsonp ? true : false, genestrand, jump_late_p ? true : false,
                               genome, genome, pairpool, extraband_end, defect_rate);
  } else {
    pairs = Dynprog_end5_known(&knownsplicep, &dynprogindex, &score, &ambig_end_length, &ambig_splicetype, &nmatches,
                               &nmismatches, &nopens, &nindels, dynprogL, rsequence, rsequenceuc, rlength, glength,
                               roffset, goffset, chroffset, chrhigh, limit_low, limit_high, cdna_direction,
                               watsonp ? true : false, genestrand, jump_late_p ? true : false, genome, genome,
                               pairpool, extraband_end, defect_rate);
  }
  Dynprog_end_setup(NULL, NULL, NULL, 0, NULL, NULL, NULL, NULL, 0, 0, false);
  free(usites);
  free(utypes);
  scalars[0] = dynprogindex; scalars[1] = score; scalars[2] = ambig_end_length; scalars[3] = (int) ambig_splicetype;
  scalars[4] = nmatches; scalars[5] = nmismatches; scalars[6] = nopens; scalars[7] = nindels;
  scalars[8] = knownsplicep ? 1 : 0;
  if (pairs == NULL) return -1;
  return flatten(pairs, out, max_pairs);
}

/* Dynprog_genome_gap (dynprog_genome.c:3288).  flags: 1 watsonp, 2 jump_late_p,
   8 halfp, 16 finalp.  scalars[0..9] = dynprogindex(after), traceback_score,
   nmatches, nmismatches, nopens, nindels, new_leftgenomepos,
   new_rightgenomepos, exonhead, introntype; out-parameters the reference does
   not write on the path taken keep the sentinel -2147483648.  dscalars[0..1] =
   left_prob, right_prob.  Returns the number of pairs or -1 for NULL. */
#define REFH_UNSET (-2147483647 - 1)

int
refh_genome_gap (const char *rsequence, const char *rsequenceuc, int rlength, int glengthL, int glengthR,
                 int roffset, int goffsetL, int rev_goffsetR, unsigned int chroffset, unsigned int chrhigh,
                 int cdna_direction, int flags, int genestrand, int extraband_paired, double defect_rate,
                 int maxpeelback, int dynprogindex, int *scalars, double *dscalars, RefPair *out, int max_pairs) {
  List_T pairs;
  int new_left = REFH_UNSET, new_right = REFH_UNSET, exonhead = REFH_UNSET, introntype = REFH_UNSET;
  int score = REFH_UNSET, nmatches = REFH_UNSET, nmismatches = REFH_UNSET, nopens = REFH_UNSET, nindels = REFH_UNSET;
  double left_prob = -1.0, right_prob = -1.0;

  Pairpool_reset(pairpool);
  pairs = Dynprog_genome_gap(&dynprogindex, &new_left, &new_right, &left_prob, &right_prob,
                             &score, &nmatches, &nmismatches, &nopens, &nindels, &exonhead, &introntype,
                             dynprogL, dynprogR, (char *) rsequence, (char *) rsequenceuc, rlength, glengthL, glengthR,
                             roffset, goffsetL, rev_goffsetR, /*chrnum*/1, (Univcoord_T) chroffset,
                             (Univcoord_T) chrhigh, cdna_direction, (flags & 1) ? true : false, genestrand,
                             (flags & 2) ? true : false, genome, genome, pairpool, extraband_paired, defect_rate,
                             maxpeelback, (flags & 8) ? true : false, (flags & 16) ? true : false);
  scalars[0] = dynprogindex; scalars[1] = score; scalars[2] = nmatches; scalars[3] = nmismatches;
  scalars[4] = nopens; scalars[5] = nindels; scalars[6] = new_left; scalars[7] = new_right;
  scalars[8] = exonhead; scalars[9] = introntype;
  dscalars[0] = left_prob; dscalars[1] = right_prob;
  if (pairs == NULL) return -1;
  return flatten(pairs, out, max_pairs);
}

/* Dynprog_microexon_int (dynprog_single.c:900) as stage3.c:9664 calls it: rsequence is the query slice
   (queryseq + roffset), the MaxEnt probabilities are the reference's own.  scalars[0..1] =
   dynprogindex(after), microintrontype; dscalars[0..1] = bestprob2, bestprob3.  Returns the number of
   pairs (list order) or -1 for NULL. */
int
refh_microexon_int (const char *rsequence, const char *rsequenceuc, int rlength, int roffset, int goffsetL,
                    int rev_goffsetR, int cdna_direction, unsigned int chroffset, unsigned int chrhigh, int watsonp,
                    int genestrand, int dynprogindex, int *scalars, double *dscalars, RefPair *out, int max_pairs) {
  List_T pairs;
  int microintrontype = REFH_UNSET;
  double prob2 = -1.0, prob3 = -1.0;
  Pairpool_reset(pairpool);
  pairs = Dynprog_microexon_int(&prob2, &prob3, &dynprogindex, &microintrontype, (char *) rsequence,
                                (char *) rsequenceuc, rlength, roffset, goffsetL, rev_goffsetR, cdna_direction,
                                (char *) rsequence - roffset, (char *) rsequenceuc - roffset, (Univcoord_T) chroffset,
                                (Univcoord_T) chrhigh, watsonp ? true : false, genestrand, genome, genome, pairpool);
  scalars[0] = dynprogindex;
  scalars[1] = microintrontype;
  dscalars[0] = prob2;
  dscalars[1] = prob3;
  if (pairs == NULL) return -1;
  return flatten(pairs, out, max_pairs);
}

/* Dynprog_cdna_gap (dynprog_cdna.c:787).  The query is one buffer: rsequenceL = qbuf + qposL,
   rev_rsequenceR = qbuf + qposR (the R piece's LAST character).  scalars[0..2] =
   dynprogindex(after), traceback_score (REFH_UNSET where the reference leaves it unwritten),
   incompletep (starts 0).  Returns the number of pairs or -1 for NULL. */
int
refh_cdna_gap (const char *qbuf, const char *qucbuf, int qposL, int qposR, int rlengthL, int rlengthR,
               int glength, int roffsetL, int rev_roffsetR, int goffset, unsigned int chroffset,
               unsigned int chrhigh, int watsonp, int genestrand, int jump_late_p, int extraband_paired,
               double defect_rate, int dynprogindex, int *scalars, RefPair *out, int max_pairs) {
  List_T pairs;
  int score = REFH_UNSET;
  bool incompletep = false;

  Pairpool_reset(pairpool);
  pairs = Dynprog_cdna_gap(&dynprogindex, &score, &incompletep, dynprogL, dynprogR,
                           (char *) qbuf + qposL, (char *) qucbuf + qposL, (char *) qbuf + qposR,
                           (char *) qucbuf + qposR, rlengthL, rlengthR, glength, roffsetL, rev_roffsetR, goffset,
                           (Univcoord_T) chroffset, (Univcoord_T) chrhigh, watsonp ? true : false, genestrand,
                           jump_late_p ? true : false, genome, genome, pairpool, extraband_paired, defect_rate);
  scalars[0] = dynprogindex; scalars[1] = score; scalars[2] = incompletep ? 1 : 0;
  if (pairs == NULL) return -1;
  return flatten(pairs, out, max_pairs);
}

/* The reference's splice-site models (maxent_hr.c:27357-27600):
   model 0 donor, 1 acceptor, 2 antidonor, 3 antiacceptor. */
double
refh_maxent (int model, unsigned int splicesitepos, unsigned int chroffset) {
  switch (model) {
  case 0: return Maxent_hr_donor_prob(genome, genome, (Univcoord_T) splicesitepos, (Univcoord_T) chroffset);
  case 1: return Maxent_hr_acceptor_prob(genome, genome, (Univcoord_T) splicesitepos, (Univcoord_T) chroffset);
  case 2: return Maxent_hr_antidonor_prob(genome, genome, (Univcoord_T) splicesitepos, (Univcoord_T) chroffset);
  case 3: return Maxent_hr_antiacceptor_prob(genome, genome, (Univcoord_T) splicesitepos, (Univcoord_T) chroffset);
  default: return -1.0;
  }
}

/* n evaluations in one call (measurement: the host MaxEnt work the GMAP drop-in does per genome gap,
   timed without a foreign-call transition per position) */
void
refh_maxent_batch (const int *models, const unsigned int *positions, unsigned int chroffset, int n, double *out) {
  int i;
  for (i = 0; i < n; i++) out[i] = refh_maxent(models[i], positions[i], chroffset);
}

/* CPU baseline loop over include/gmapdp.h's gmapdp_genome_problem layout
   (restated). */
typedef struct {
  int qoff, rlength, glengthL, glengthR, roffset, goffsetL, rev_goffsetR;
  unsigned int chroffset, chrhigh;
  int flags, cdna_direction, genestrand, extraband, maxpeelback, dynprogindex, pad_;
  double defect_rate;
  long prob_offset;
} RefGenomeProblem;

long
refh_genome_gap_batch (const RefGenomeProblem *probs, int n, const char *qseq, const char *qseq_uc) {
  long total = 0;
  int i, dpi, new_left, new_right, exonhead, introntype, score, nmatches, nmismatches, nopens, nindels;
  double left_prob, right_prob;
  List_T pairs;
  for (i = 0; i < n; i++) {
    const RefGenomeProblem *p = &probs[i];
    Pairpool_reset(pairpool);
    dpi = p->dynprogindex;
    pairs = Dynprog_genome_gap(&dpi, &new_left, &new_right, &left_prob, &right_prob, &score, &nmatches,
                               &nmismatches, &nopens, &nindels, &exonhead, &introntype, dynprogL, dynprogR,
                               (char *) qseq + p->qoff, (char *) qseq_uc + p->qoff, p->rlength, p->glengthL,
                               p->glengthR, p->roffset, p->goffsetL, p->rev_goffsetR, /*chrnum*/1,
                               (Univcoord_T) p->chroffset, (Univcoord_T) p->chrhigh, p->cdna_direction,
                               (p->flags & 1) ? true : false, p->genestrand, (p->flags & 2) ? true : false,
                               genome, genome, pairpool, p->extraband, p->defect_rate, p->maxpeelback,
                               (p->flags & 8) ? true : false, (p->flags & 16) ? true : false);
    total += List_length(pairs);
  }
  return total;
}

/* Reference genome-segment extraction (genome.c:11023/11079), for the oracle's
   unpacking to be checked against. */
int
refh_get_segment (int rightp, unsigned int pos, int length, unsigned int chrbound, int revcomp,
                  char *segment, char *segmentalt) {
  if (rightp) {
    Genome_get_segment_right(segment, segmentalt, genome, genome, (Univcoord_T) pos, (Chrpos_T) length,
                             (Univcoord_T) chrbound, revcomp ? true : false);
  } else {
    Genome_get_segment_left(segment, segmentalt, genome, genome, (Univcoord_T) pos, (Chrpos_T) length,
                            (Univcoord_T) chrbound, revcomp ? true : false);
  }
  return 0;
}

/* Copy of the mismatch-type score table the reference builds (dynprog.c:1008). */
int
refh_pairdistance (int mismatchtype, short *out128x128) {
  int i, j;
  for (i = 0; i < 128; i++) for (j = 0; j < 128; j++) out128x128[i * 128 + j] = pairdistance_array[mismatchtype][i][j];
  return 0;
}

int
refh_consistent (int genestrand, unsigned char *out128x128) {
  int i, j;
  for (i = 0; i < 128; i++) for (j = 0; j < 128; j++) out128x128[i * 128 + j] = consistent_array[genestrand][i][j] ? 1 : 0;
  return 0;
}

/* The reference's .genomecomp packing of a user segment
   (Compress_create_blocks_comp, compress-write.c:754): nwords = (len+31)/32*3 + 4. */
int
refh_pack_genome (const char *seq, unsigned int length, unsigned int *out) {
  Genomecomp_T *blocks;
  char *copy = (char *) malloc(length + 1);
  size_t nw = ((size_t) (length + 31) / 32) * 3 + 4, i;
  memcpy(copy, seq, length);
  copy[length] = '\0';
  blocks = Compress_create_blocks_comp(copy, (Univcoord_T) length);
  for (i = 0; i < nw; i++) out[i] = blocks[i];
  FREE(blocks);
  free(copy);
  return (int) nw;
}

int
refh_use8p_size (int *out4) {
  int i;
  for (i = 0; i < 4; i++) out4[i] = use8p_size[i];
  return 0;
}


/* Stage-2 seeding as GMAP's Stage2_compute runs it (stage2.c:6413-6501, one oligoindex source):
   Oligoindex_hr_tally (oligoindex_hr.c:33849) over the genomic window, then
   Oligoindex_get_mappings (:34127) with coveredp all false.  major: the 8-mer index with
   diag_lookback 120 / suffnconsecutive 20 (Oligoindex_array_new_major, :8606-8610), else the
   minor one (60 / 10).  Outputs: npositions[querylength] (0 where the query has no full 8-mer),
   positions: the mapping list of every querypos with npositions > 0, concatenated in querypos
   order; scalars = {totalpositions, maxnconsecutive, oned_matrix_p, ndiagonals}; diags: per
   diagonal in list order {diagonal, querystart, queryend, nconsecutive}.  Returns the number of
   positions written, -1 if pos_cap / diag_cap is too small. */
static Oligoindex_array_T oligo_major = NULL, oligo_minor = NULL;
static Diagpool_T diagpool = NULL;

int
refh_oligo_mappings (const char *queryuc, int querylength, unsigned int chrstart, unsigned int chrend,
                     unsigned int chroffset, unsigned int chrhigh, int plusp, int minor, int *npositions,
                     unsigned int *positions, int pos_cap, int *scalars, int *diags, int diag_cap) {
  Oligoindex_array_T array;
  Oligoindex_T oligoindex;
  Chrpos_T **mappings;
  bool *coveredp, oned_matrix_p = false;
  int totalpositions = 0, maxnconsecutive = 0, q, k, n = 0, nd = 0;
  List_T diagonals = NULL, p;
  char *quc;
  if (oligo_major == NULL) {
    Oligoindex_hr_setup(STANDARD);
    oligo_major = Oligoindex_array_new_major(100000, 1000000);  /* gmap.c:113-114, 4739-4740 */
    oligo_minor = Oligoindex_array_new_minor(100000, 1000000);
    diagpool = Diagpool_new();
  }
  array = minor ? oligo_minor : oligo_major;
  oligoindex = Oligoindex_array_elt(array, 0);
  quc = (char *) malloc(querylength + 1);
  memcpy(quc, queryuc, querylength);
  quc[querylength] = '\0';
  coveredp = (bool *) calloc(querylength + 1, sizeof(bool));
  mappings = (Chrpos_T **) calloc(querylength + 1, sizeof(Chrpos_T *));
  memset(npositions, 0, querylength * sizeof(int));
  Diagpool_reset(diagpool);
  if (plusp) {
    Oligoindex_hr_tally(oligoindex, (Univcoord_T) chroffset + chrstart, (Univcoord_T) chroffset + chrend, true,
                        quc, 0, querylength, chrstart, genome, 0);
  } else {
    Oligoindex_hr_tally(oligoindex, (Univcoord_T) chroffset + chrstart, (Univcoord_T) chroffset + chrend + 1, false,
                        quc, 0, querylength, (chrhigh - chroffset) - chrend, genome, 0);
  }
  diagonals = Oligoindex_get_mappings(diagonals, coveredp, mappings, npositions, &totalpositions, &oned_matrix_p,
                                      &maxnconsecutive, array, oligoindex, quc, 0, querylength, querylength,
                                      chrstart, chrend, chroffset, chrhigh, plusp ? true : false, diagpool);
  for (q = 0; q < querylength && n >= 0; q++) {
    if (npositions[q] <= 0) continue;
    if (n + npositions[q] > pos_cap) { n = -1; break; }
    for (k = 0; k < npositions[q]; k++) positions[n++] = mappings[q][k];
  }
  for (p = diagonals; p != NULL; p = List_next(p)) {
    Diag_T d = (Diag_T) List_head(p);
    if (nd < diag_cap) {
      diags[4 * nd + 0] = (int) Diag_diagonal(d);
      diags[4 * nd + 1] = Diag_querystart(d);
      diags[4 * nd + 2] = Diag_queryend(d);
      diags[4 * nd + 3] = Diag_nconsecutive(d);
    }
    nd++;
  }
  scalars[0] = totalpositions;
  scalars[1] = maxnconsecutive;
  scalars[2] = oned_matrix_p ? 1 : 0;
  scalars[3] = nd;
  Oligoindex_untally(oligoindex);
  free(mappings);
  free(coveredp);
  free(quc);
  return nd > diag_cap ? -1 : n;
}


/* Stage2_compute (stage2.c:6325) itself, with GMAP's arguments (gmap.c:1208-1215: query_offset 0,
   genestrand 0, proceed_pctcoverage 0.3, the major oligoindex array, genomealt = genome, localp,
   skip_repetitive_p, favor_right_p false, max_nalignments MAX_NALIGNMENTS = 10, no stopwatch) after
   Stage2_setup (gmap.c:6544: cross_species_p false, suboptimal_score_start -1 / _end 3,
   sufflookback 60, nsufflookback 5, STANDARD mode, no SNPs).  Each returned Stage2_T's middle list
   is flattened into `pairs` (list order); paths[2 i] / paths[2 i + 1] = its first record / count.
   scalars[0] = number of results; scalars[1] = 1 if any result has start or end lists (they stay
   NULL without MOVE_TO_STAGE3).  Returns the number of results, -1 when a capacity is too small. */
static Stage2_alloc_T stage2_alloc = NULL;
static Cellpool_T cellpool = NULL;
static int stage2_splicingp = -1, stage2_maxintronlen = -1;

int
refh_stage2_compute (const char *queryseq, const char *queryuc, int querylength, unsigned int chrstart,
                     unsigned int chrend, unsigned int chroffset, unsigned int chrhigh, int plusp, int splicingp,
                     int maxintronlen, int *scalars, int *paths, int path_cap, RefPair *pairs, int pair_cap) {
  List_T results, p, q;
  char *qs, *quc;
  int nres = 0, n = 0, k;
  if (oligo_major == NULL) {
    Oligoindex_hr_setup(STANDARD);
    oligo_major = Oligoindex_array_new_major(100000, 1000000);  /* gmap.c:113-114, 4739-4740 */
    oligo_minor = Oligoindex_array_new_minor(100000, 1000000);
    diagpool = Diagpool_new();
  }
  if (stage2_alloc == NULL) {
    stage2_alloc = Stage2_alloc_new(100000);  /* MAX_QUERYLENGTH_FOR_ALLOC, gmap.c:113 */
    cellpool = Cellpool_new();
  }
  if (splicingp != stage2_splicingp || maxintronlen != stage2_maxintronlen) {
    Stage2_setup(splicingp ? true : false, /*cross_species_p*/false, /*suboptimal_score_start*/-1,
                 /*suboptimal_score_end*/3, /*sufflookback*/60, /*nsufflookback*/5, maxintronlen, STANDARD,
                 /*snps_p*/false);
    stage2_splicingp = splicingp;
    stage2_maxintronlen = maxintronlen;
  }
  qs = (char *) malloc(querylength + 1);
  quc = (char *) malloc(querylength + 1);
  memcpy(qs, queryseq, querylength);
  memcpy(quc, queryuc, querylength);
  qs[querylength] = quc[querylength] = '\0';
  Pairpool_reset(pairpool);
  results = Stage2_compute(qs, quc, querylength, /*query_offset*/0, chrstart, chrend, chroffset, chrhigh,
                           plusp ? true : false, /*genestrand*/0, stage2_alloc, /*proceed_pctcoverage*/0.3,
                           oligo_major, genome, genome, pairpool, diagpool, cellpool, /*localp*/true,
                           /*skip_repetitive_p*/true, /*favor_right_p*/false, /*max_nalignments*/10,
                           /*stopwatch*/NULL, /*diag_debug*/false);
  scalars[0] = scalars[1] = 0;
  for (p = results; p != NULL; p = List_next(p)) {
    Stage2_T s2 = (Stage2_T) List_head(p);
    if (Stage2_all_starts(s2) != NULL || Stage2_all_ends(s2) != NULL) scalars[1] = 1;
    if (nres < path_cap) paths[2 * nres] = n;
    k = 0;
    for (q = Stage2_middle(s2); q != NULL; q = List_next(q), k++) {
      Pair_T pr = (Pair_T) List_head(q);
      if (n < pair_cap) {
        RefPair *r = &pairs[n];
        r->querypos = pr->querypos;
        r->genomepos = pr->genomepos;
        r->queryjump = pr->gapp ? pr->queryjump : 0;
        r->genomejump = pr->gapp ? pr->genomejump : 0;
        r->dynprogindex = pr->dynprogindex;
        r->cdna = pr->cdna;
        r->comp = pr->comp;
        r->genome = pr->genome;
        r->genomealt = pr->genomealt;
        r->gapp = pr->gapp ? 1 : 0;
      }
      n++;
    }
    if (nres < path_cap) paths[2 * nres + 1] = k;
    nres++;
    Stage2_free(&s2);
  }
  List_free(&results);
  scalars[0] = nres;
  free(qs);
  free(quc);
  return (nres > path_cap || n > pair_cap) ? -1 : nres;
}
