/* gmapdp_gmap_shim.c -- drop-in for GMAP's Dynprog_* entry points on the MI355X engine.
 *
 * Compiled INSIDE a GMAP build (against GMAP's own headers, -DHAVE_CONFIG_H)
 * and linked with
 *
 *   -Wl,--wrap=Dynprog_init,--wrap=Dynprog_single_setup,--wrap=Dynprog_end_setup,
 *   -Wl,--wrap=Dynprog_genome_setup,--wrap=Dynprog_single_gap,--wrap=Dynprog_end5_gap,
 *   -Wl,--wrap=Dynprog_end3_gap,--wrap=Dynprog_genome_gap,--wrap=Dynprog_cdna_gap
 *   -Wl,--wrap=Oligoindex_hr_tally,--wrap=Oligoindex_get_mappings  -lgmapdp
 *
 * so that every call GMAP's stage 3 makes to these functions (stage3.c:9081,
 * 9275, 9510, 9531, 10244-10600, ...) lands here with the reference's own signature
 * (dynprog_single.h:22, dynprog_end.h:25/47, dynprog_genome.h:24, dynprog_cdna.h:12) and returns
 * the reference's List_T of Pair_T built in the caller's Pairpool
 * (Pairpool_push / Pairpool_push_gapholder, pairpool.c:180/375).  The setup
 * functions are wrapped only to learn Mode_T and the user gap penalties; the
 * reference's own setup still runs.  See INTEGRATION.md.
 *
 * Semantics follow the GMAP build the shim is compiled into: a SIMD build
 * (HAVE_SSE2: gmap.sse42 / .avx2 / .avx512, dynprog_simd.c) gets GMAPDP_SIMD on
 * every call, a nosimd build the Dynprog_standard semantics.
 *
 * Scope (the engine's, include/gmapdp.h): no alternate-
 * allele genome (genomealt must equal genome); Dynprog_T created with
 * gmap.c's defaults (max_rlength 660, max_glength 2000); homopolymer mode
 * off; no splicing IIT in Dynprog_genome_gap.  Anything else is refused with
 * a message and abort() -- there is no silent CPU fallback.
 *
 * This file is one call per launch (a correctness drop-in).  Throughput comes
 * from batching many calls per launch (gmapdp_*_batch / gmapdp_plan_*), which
 * needs the caller to issue sub-problems of many reads together
 * (INTEGRATION.md "Batching").
 */
#ifdef HAVE_CONFIG_H
#include "config.h"
#endif
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <pthread.h>

#include "bool.h"
#include "list.h"
#include "pair.h"
#include "pairdef.h"
#include "pairpool.h"
#include "genome.h"
#include "maxent_hr.h"
#include "dynprog.h"
#include "dynprog_single.h"
#include "dynprog_end.h"
#include "dynprog_genome.h"
#include "dynprog_cdna.h"
#include "oligoindex_hr.h"
#include "diagpool.h"

#include "gmapdp.h"
#include "gmapdp_dynprog.h"

/* ---- the wrapped reference functions ---- */
extern void __real_Dynprog_init (Mode_T mode);
extern void __real_Dynprog_single_setup (int user_open_in, int user_extend_in, bool user_dynprog_p_in,
                                         bool homopolymerp_in);
extern void __real_Dynprog_end_setup (Univcoord_T *splicesites_in, Splicetype_T *splicetypes_in,
                                      Chrpos_T *splicedists_in, int nsplicesites_in,
                                      Trieoffset_T *trieoffsets_obs_in, Triecontent_T *triecontents_obs_in,
                                      Trieoffset_T *trieoffsets_max_in, Triecontent_T *triecontents_max_in,
                                      int user_open_in, int user_extend_in, bool user_dynprog_p_in);
extern void __real_Dynprog_genome_setup (bool novelsplicingp_in, IIT_T splicing_iit_in,
                                         int *splicing_divint_crosstable_in, int donor_typeint_in,
                                         int acceptor_typeint_in, int user_open_in, int user_extend_in,
                                         bool user_dynprog_p_in);

/* the semantics of the GMAP build this file is compiled into */
#ifdef HAVE_SSE2
#define SHIM_SIMD GMAPDP_SIMD
#else
#define SHIM_SIMD 0
#endif

static pthread_mutex_t shim_lock = PTHREAD_MUTEX_INITIALIZER;
static gmapdp_ctx *shim_ctx = NULL;
static Genome_T shim_genome = NULL;
static int shim_mode = 0, shim_user_open = 0, shim_user_extend = 0, shim_user_dynprog_p = 0;
static int shim_homopolymerp = 0, shim_splicing_iit = 0;

/* Calls that reached the engine, per wrapped entry point (printed at exit with GMAPDP_SHIM_STATS=1;
   tests use it to prove the pipeline really ran on the GPU). */
enum { ST_SINGLE, ST_END5, ST_END3, ST_GENOME, ST_CDNA, ST_OLIGO, ST_N };
static const char *const shim_stat_name[ST_N] = {"Dynprog_single_gap", "Dynprog_end5_gap", "Dynprog_end3_gap",
                                                 "Dynprog_genome_gap", "Dynprog_cdna_gap",
                                                 "Oligoindex_get_mappings"};
static unsigned long shim_stats[ST_N];

static void
shim_print_stats (void) {
  int i;
  fprintf(stderr, "gmapdp shim calls:");
  for (i = 0; i < ST_N; i++) fprintf(stderr, " %s=%lu", shim_stat_name[i], __atomic_load_n(&shim_stats[i], __ATOMIC_RELAXED));
  fprintf(stderr, "\n");
}

static void
shim_count (int which) {
  __atomic_fetch_add(&shim_stats[which], 1UL, __ATOMIC_RELAXED);
}

static void
shim_refuse (const char *what) {
  fprintf(stderr, "gmapdp shim: %s is not supported by the MI355X Dynprog engine\n", what);
  abort();
}

/* The engine's descriptors carry 32-bit genome coordinates (gmap's Univcoord_T, univcoord.h:9-11).
   A gmapl build (LARGE_GENOMES, 64-bit Univcoord_T) or any coordinate at or above 2^32 is refused
   instead of being truncated. */
#ifdef LARGE_GENOMES
#error "gmapdp shim: LARGE_GENOMES (gmapl, 64-bit Univcoord_T) is not supported by this engine build"
#endif
static uint32_t
shim_coord (Univcoord_T x) {
  if ((uint64_t) x > 0xFFFFFFFFu) shim_refuse("a genome coordinate at or above 2^32 (gmapl genomes)");
  return (uint32_t) x;
}

static void
shim_check (int rc, const char *what) {
  if (rc != GMAPDP_OK) {
    fprintf(stderr, "gmapdp shim: %s failed (%d): %s\n", what, rc, gmapdp_last_error(shim_ctx));
    abort();
  }
}

void
__wrap_Dynprog_init (Mode_T mode) {
  __real_Dynprog_init(mode);
  shim_mode = (int) mode;
}

void
__wrap_Dynprog_single_setup (int user_open_in, int user_extend_in, bool user_dynprog_p_in, bool homopolymerp_in) {
  __real_Dynprog_single_setup(user_open_in, user_extend_in, user_dynprog_p_in, homopolymerp_in);
  shim_user_open = user_open_in;
  shim_user_extend = user_extend_in;
  shim_user_dynprog_p = user_dynprog_p_in ? 1 : 0;
  shim_homopolymerp = homopolymerp_in ? 1 : 0;
}

void
__wrap_Dynprog_end_setup (Univcoord_T *splicesites_in, Splicetype_T *splicetypes_in, Chrpos_T *splicedists_in,
                          int nsplicesites_in, Trieoffset_T *trieoffsets_obs_in, Triecontent_T *triecontents_obs_in,
                          Trieoffset_T *trieoffsets_max_in, Triecontent_T *triecontents_max_in,
                          int user_open_in, int user_extend_in, bool user_dynprog_p_in) {
  __real_Dynprog_end_setup(splicesites_in, splicetypes_in, splicedists_in, nsplicesites_in, trieoffsets_obs_in,
                           triecontents_obs_in, trieoffsets_max_in, triecontents_max_in, user_open_in,
                           user_extend_in, user_dynprog_p_in);
}

void
__wrap_Dynprog_genome_setup (bool novelsplicingp_in, IIT_T splicing_iit_in, int *splicing_divint_crosstable_in,
                             int donor_typeint_in, int acceptor_typeint_in, int user_open_in, int user_extend_in,
                             bool user_dynprog_p_in) {
  __real_Dynprog_genome_setup(novelsplicingp_in, splicing_iit_in, splicing_divint_crosstable_in, donor_typeint_in,
                              acceptor_typeint_in, user_open_in, user_extend_in, user_dynprog_p_in);
  shim_splicing_iit = splicing_iit_in != NULL;
}

/* The engine context (one per process, calls serialised) with `genome` resident in HBM. */
static gmapdp_ctx *
shim_context (Genome_T genome, Genome_T genomealt, Dynprog_T dynprog) {
  const char *dev;
  uint64_t length;
  size_t nwords;
  if (genomealt != NULL && genomealt != genome) shim_refuse("an alternate-allele genome (genomealt)");
  if (dynprog != NULL && (dynprog->max_rlength != GMAPDP_MAX_RLENGTH || dynprog->max_glength != GMAPDP_MAX_GLENGTH))
    shim_refuse("a Dynprog_T with non-default maximum lengths");
  if (shim_ctx == NULL) {
    dev = getenv("GMAPDP_SHIM_STATS");
    if (dev != NULL && dev[0] == '1') atexit(shim_print_stats);
    dev = getenv("GMAPDP_DEVICE");
    shim_check(gmapdp_create(&shim_ctx, dev ? atoi(dev) : 0, shim_mode, shim_user_open, shim_user_extend,
                             shim_user_dynprog_p), "gmapdp_create");
  }
  if (genome != shim_genome) {
    length = (uint64_t) Genome_genomelength(genome);
    if (length > 0xFFFFFFFFull) shim_refuse("a genome of 2^32 nt or more (gmapl genomes)");
    nwords = gmapdp_genome_words(length);
    shim_check(gmapdp_set_genome(shim_ctx, (const uint32_t *) Genome_blocks(genome), nwords, length),
               "gmapdp_set_genome");
    shim_genome = genome;
  }
  return shim_ctx;
}

/* The engine's records in list order -> the reference's List_T (each push prepends).  The gap
   holder at gap_index carries gap_queryjump and, for introntype >= 0, the intron's type and
   splice probabilities (Dynprog_genome_gap); other gap holders carry queryjump 0. */
static List_T
shim_list (const gmapdp_pair *pairs, int n, int dynprogindex, int gap_index, int gap_queryjump, int introntype,
           double donor_prob, double acceptor_prob, Pairpool_T pairpool) {
  List_T list = NULL;
  Pair_T gappair;
  int i;
  for (i = n - 1; i >= 0; i--) {
    const gmapdp_pair *p = &pairs[i];
    if (p->querypos == -1 && p->genomepos == -1) {
      list = Pairpool_push_gapholder(list, pairpool, i == gap_index ? gap_queryjump : 0, p->jump,
                                     /*leftpair*/NULL, /*rightpair*/NULL, /*knownp*/false);
      if (i == gap_index && introntype >= 0) {
        gappair = (Pair_T) list->first;
        gappair->introntype = introntype;
        gappair->donor_prob = donor_prob;
        gappair->acceptor_prob = acceptor_prob;
      }
    } else {
      list = Pairpool_push(list, pairpool, p->querypos, p->genomepos, p->cdna, p->comp, p->genome, p->genomealt,
                           dynprogindex);
    }
  }
  return list;
}

List_T
__wrap_Dynprog_single_gap (int *dynprogindex, int *finalscore, int *nmatches, int *nmismatches, int *nopens,
                           int *nindels, Dynprog_T dynprog, char *sequence1, char *sequenceuc1, int length1,
                           int length2, int offset1, int offset2, Univcoord_T chroffset, Univcoord_T chrhigh,
                           bool watsonp, int genestrand, bool jump_late_p, Genome_T genome, Genome_T genomealt,
                           Pairpool_T pairpool, int extraband_single, bool widebandp, double defect_rate) {
  gmapdp_single_problem p;
  gmapdp_result res;
  gmapdp_pair *pairs;
  size_t cap;
  List_T list;
  if (shim_homopolymerp) shim_refuse("homopolymer mode (Dynprog_single_setup homopolymerp)");
  pthread_mutex_lock(&shim_lock);
  shim_context(genome, genomealt, dynprog);
  memset(&p, 0, sizeof(p));
  p.qoff = 0;
  p.rlength = length1;
  p.glength = length2;
  p.roffset = offset1;
  p.goffset = offset2;
  p.chroffset = shim_coord(chroffset);
  p.chrhigh = shim_coord(chrhigh);
  p.flags = (watsonp ? GMAPDP_WATSON : 0) | (jump_late_p ? GMAPDP_JUMP_LATE : 0) | (widebandp ? GMAPDP_WIDEBAND : 0) |
            SHIM_SIMD;
  p.genestrand = genestrand;
  p.extraband = extraband_single;
  p.defect_rate = defect_rate;
  p.dynprogindex = *dynprogindex;
  cap = gmapdp_single_pair_capacity(&p, 1);
  pairs = (gmapdp_pair *) malloc((cap ? cap : 1) * sizeof(gmapdp_pair));
  shim_check(gmapdp_single_gap_batch(shim_ctx, &p, 1, sequence1, sequenceuc1, length1 > 0 ? (size_t) length1 : 0,
                                     &res, pairs, cap), "gmapdp_single_gap_batch");
  shim_count(ST_SINGLE);
  pthread_mutex_unlock(&shim_lock);
  list = shim_list(pairs + res.pair_offset, res.npairs, p.dynprogindex, -1, 0, 0, 0.0, 0.0, pairpool);
  free(pairs);
  *dynprogindex = res.dynprogindex;
  *finalscore = res.traceback_score;
  *nmatches = res.nmatches;
  *nmismatches = res.nmismatches;
  *nopens = res.nopens;
  *nindels = res.nindels;
  return list;
}

static List_T
shim_end_gap (int end3p, int *dynprogindex, int *finalscore, int *nmatches, int *nmismatches, int *nopens,
              int *nindels, Dynprog_T dynprog, char *seq, char *sequc, int length1, int length2, int offset1,
              int offset2, Univcoord_T chroffset, Univcoord_T chrhigh, bool watsonp, int genestrand,
              bool jump_late_p, Genome_T genome, Genome_T genomealt, Pairpool_T pairpool, int extraband_end,
              double defect_rate, Endalign_T endalign, bool require_pos_score_p) {
  gmapdp_end_problem p;
  gmapdp_result res;
  gmapdp_pair *pairs;
  size_t cap;
  List_T list;
  const char *q, *quc;
  pthread_mutex_lock(&shim_lock);
  shim_context(genome, genomealt, dynprog);
  memset(&p, 0, sizeof(p));
  p.rlength = length1;
  p.glength = length2;
  p.roffset = offset1;
  p.goffset = offset2;
  p.chroffset = shim_coord(chroffset);
  p.chrhigh = shim_coord(chrhigh);
  p.flags = (watsonp ? GMAPDP_WATSON : 0) | (jump_late_p ? GMAPDP_JUMP_LATE : 0) | SHIM_SIMD;
  p.genestrand = genestrand;
  p.extraband = extraband_end;
  p.end3p = end3p;
  p.endalign = (int32_t) endalign;
  p.require_pos_score_p = require_pos_score_p ? 1 : 0;
  p.dynprogindex = *dynprogindex;
  p.defect_rate = defect_rate;
  /* end5's revsequence points at the LAST character of the slice (dynprog_end.c:1294) */
  q = (end3p || length1 <= 0) ? seq : seq - (length1 - 1);
  quc = (end3p || length1 <= 0) ? sequc : sequc - (length1 - 1);
  cap = gmapdp_end_pair_capacity(&p, 1);
  pairs = (gmapdp_pair *) malloc((cap ? cap : 1) * sizeof(gmapdp_pair));
  shim_check(gmapdp_end_gap_batch(shim_ctx, &p, 1, q, quc, length1 > 0 ? (size_t) length1 : 0, &res, pairs, cap),
             "gmapdp_end_gap_batch");
  shim_count(end3p ? ST_END3 : ST_END5);
  pthread_mutex_unlock(&shim_lock);
  list = shim_list(pairs + res.pair_offset, res.npairs, p.dynprogindex, -1, 0, 0, 0.0, 0.0, pairpool);
  free(pairs);
  *dynprogindex = res.dynprogindex;
  *finalscore = res.traceback_score;
  *nmatches = res.nmatches;
  *nmismatches = res.nmismatches;
  *nopens = res.nopens;
  *nindels = res.nindels;
  return list;
}

List_T
__wrap_Dynprog_end5_gap (int *dynprogindex, int *finalscore, int *nmatches, int *nmismatches, int *nopens,
                         int *nindels, Dynprog_T dynprog, char *revsequence1, char *revsequenceuc1, int length1,
                         int length2, int revoffset1, int revoffset2, Univcoord_T chroffset, Univcoord_T chrhigh,
                         bool watsonp, int genestrand, bool jump_late_p, Genome_T genome, Genome_T genomealt,
                         Pairpool_T pairpool, int extraband_end, double defect_rate, Endalign_T endalign,
                         bool require_pos_score_p) {
  return shim_end_gap(0, dynprogindex, finalscore, nmatches, nmismatches, nopens, nindels, dynprog, revsequence1,
                      revsequenceuc1, length1, length2, revoffset1, revoffset2, chroffset, chrhigh, watsonp,
                      genestrand, jump_late_p, genome, genomealt, pairpool, extraband_end, defect_rate, endalign,
                      require_pos_score_p);
}

List_T
__wrap_Dynprog_end3_gap (int *dynprogindex, int *finalscore, int *nmatches, int *nmismatches, int *nopens,
                         int *nindels, Dynprog_T dynprog, char *sequence1, char *sequenceuc1, int length1,
                         int length2, int offset1, int offset2, Univcoord_T chroffset, Univcoord_T chrhigh,
                         bool watsonp, int genestrand, bool jump_late_p, Genome_T genome, Genome_T genomealt,
                         Pairpool_T pairpool, int extraband_end, double defect_rate, Endalign_T endalign,
                         bool require_pos_score_p) {
  return shim_end_gap(1, dynprogindex, finalscore, nmatches, nmismatches, nopens, nindels, dynprog, sequence1,
                      sequenceuc1, length1, length2, offset1, offset2, chroffset, chrhigh, watsonp, genestrand,
                      jump_late_p, genome, genomealt, pairpool, extraband_end, defect_rate, endalign,
                      require_pos_score_p);
}

/* Maxent_hr_*_prob of one splice-site entry (the host's MaxEnt models, maxent_hr.c) */
static double
shim_maxent (Genome_T genome, Genome_T genomealt, uint8_t model, uint32_t pos, Univcoord_T chroffset) {
  switch (model) {
  case GMAPDP_MAXENT_DONOR: return Maxent_hr_donor_prob(genome, genomealt, (Univcoord_T) pos, chroffset);
  case GMAPDP_MAXENT_ACCEPTOR: return Maxent_hr_acceptor_prob(genome, genomealt, (Univcoord_T) pos, chroffset);
  case GMAPDP_MAXENT_ANTIDONOR: return Maxent_hr_antidonor_prob(genome, genomealt, (Univcoord_T) pos, chroffset);
  default: return Maxent_hr_antiacceptor_prob(genome, genomealt, (Univcoord_T) pos, chroffset);
  }
}

List_T
__wrap_Dynprog_genome_gap (int *dynprogindex, int *new_leftgenomepos, int *new_rightgenomepos, double *left_prob,
                           double *right_prob, int *traceback_score, int *nmatches, int *nmismatches, int *nopens,
                           int *nindels, int *exonhead, int *introntype, Dynprog_T dynprogL, Dynprog_T dynprogR,
                           char *rsequence, char *rsequenceuc, int rlength, int glengthL, int glengthR, int roffset,
                           int goffsetL, int rev_goffsetR, Chrnum_T chrnum, Univcoord_T chroffset,
                           Univcoord_T chrhigh, int cdna_direction, bool watsonp, int genestrand, bool jump_late_p,
                           Genome_T genome, Genome_T genomealt, Pairpool_T pairpool, int extraband_paired,
                           double defect_rate, int maxpeelback, bool halfp, bool finalp) {
  gmapdp_genome_problem p;
  gmapdp_genome_result res;
  gmapdp_pair *pairs;
  size_t cap, m, i;
  uint32_t *pos;
  uint8_t *model;
  double *probs;
  List_T list;
  (void) chrnum;
  if (shim_splicing_iit) shim_refuse("known splice sites (a splicing IIT) in Dynprog_genome_gap");
  pthread_mutex_lock(&shim_lock);
  shim_context(genome, genomealt, dynprogL);
  shim_context(genome, genomealt, dynprogR);
  memset(&p, 0, sizeof(p));
  p.rlength = rlength;
  p.glengthL = glengthL;
  p.glengthR = glengthR;
  p.roffset = roffset;
  p.goffsetL = goffsetL;
  p.rev_goffsetR = rev_goffsetR;
  p.chroffset = shim_coord(chroffset);
  p.chrhigh = shim_coord(chrhigh);
  p.flags = (watsonp ? GMAPDP_WATSON : 0) | (jump_late_p ? GMAPDP_JUMP_LATE : 0) | (halfp ? GMAPDP_HALFP : 0) |
            (finalp ? GMAPDP_FINALP : 0) | SHIM_SIMD;
  p.cdna_direction = cdna_direction;
  p.genestrand = genestrand;
  p.extraband = extraband_paired;
  p.maxpeelback = maxpeelback;
  p.dynprogindex = *dynprogindex;
  p.defect_rate = defect_rate;
  p.prob_offset = 0;
  /* the MaxEnt probabilities the bridge reads, computed by the host as the reference does;
     skipped where the engine resolves the call before reading them (rlength <= 1, size guard) */
  m = 0;
  if (rlength > 1 && rlength <= GMAPDP_MAX_RLENGTH && glengthL <= GMAPDP_MAX_GLENGTH &&
      glengthR <= GMAPDP_MAX_GLENGTH && glengthL > 0 && glengthR > 0)
    m = gmapdp_genome_prob_entries(&p, 1);
  probs = (double *) calloc(m ? m : 1, sizeof(double));
  if (m) {
    pos = (uint32_t *) malloc(m * sizeof(uint32_t));
    model = (uint8_t *) malloc(m);
    shim_check(gmapdp_genome_splice_sites(&p, 1, pos, model, m), "gmapdp_genome_splice_sites");
    /* the last entry of each side is never read (the reference leaves it unset too, :2575-2660) */
    for (i = 0; i < m; i++)
      if (i != (size_t) glengthL - 1 && i != m - 1)
        probs[i] = shim_maxent(genome, genomealt, model[i], pos[i], chroffset);
    free(pos);
    free(model);
  }
  cap = gmapdp_genome_pair_capacity(&p, 1);
  pairs = (gmapdp_pair *) malloc((cap ? cap : 1) * sizeof(gmapdp_pair));
  shim_check(gmapdp_genome_gap_batch(shim_ctx, &p, 1, rsequence, rsequenceuc, rlength > 0 ? (size_t) rlength : 0,
                                     probs, m, &res, pairs, cap), "gmapdp_genome_gap_batch");
  shim_count(ST_GENOME);
  pthread_mutex_unlock(&shim_lock);
  list = shim_list(pairs + res.pair_offset, res.npairs, p.dynprogindex, res.gap_index, res.gap_queryjump,
                   res.introntype, res.left_prob, res.right_prob, pairpool);
  free(pairs);
  free(probs);
  *dynprogindex = res.dynprogindex;
  *traceback_score = res.traceback_score;
  *nmatches = res.nmatches;
  *nmismatches = res.nmismatches;
  *nopens = res.nopens;
  *nindels = res.nindels;
  *introntype = res.introntype;
  *left_prob = res.left_prob;
  *right_prob = res.right_prob;
  if (res.new_leftgenomepos != GMAPDP_UNSET) *new_leftgenomepos = res.new_leftgenomepos;
  if (res.new_rightgenomepos != GMAPDP_UNSET) *new_rightgenomepos = res.new_rightgenomepos;
  if (res.exonhead != GMAPDP_UNSET) *exonhead = res.exonhead;
  return list;
}

List_T
__wrap_Dynprog_cdna_gap (int *dynprogindex, int *traceback_score, bool *incompletep, Dynprog_T dynprogL,
                         Dynprog_T dynprogR, char *rsequenceL, char *rsequence_ucL, char *rev_rsequenceR,
                         char *rev_rsequence_ucR, int rlengthL, int rlengthR, int glength, int roffsetL,
                         int rev_roffsetR, int goffset, Univcoord_T chroffset, Univcoord_T chrhigh, bool watsonp,
                         int genestrand, bool jump_late_p, Genome_T genome, Genome_T genomealt,
                         Pairpool_T pairpool, int extraband_paired, double defect_rate) {
  gmapdp_cdna_problem p;
  gmapdp_cdna_result res;
  gmapdp_pair *pairs;
  size_t cap;
  List_T list;
  const char *lo, *hi, *lo_uc;
  long span;
  /* one arena holds both query pieces (stage3.c passes two pointers into the same query,
     :9275-9285) and the stretch between them, which the SHORTGAP block reads */
  span = (long) rev_roffsetR - roffsetL + 1;
  if (span < rlengthL) span = rlengthL;
  lo = rsequenceL;
  if (rlengthR > 0 && rev_rsequenceR - (rlengthR - 1) < lo) lo = rev_rsequenceR - (rlengthR - 1);
  hi = rsequenceL + span;
  if (rev_rsequenceR + 1 > hi) hi = rev_rsequenceR + 1;
  lo_uc = rsequence_ucL - (rsequenceL - lo);
  if (rev_rsequence_ucR - lo_uc != rev_rsequenceR - lo) shim_refuse("query pieces from two different buffers");
  pthread_mutex_lock(&shim_lock);
  shim_context(genome, genomealt, dynprogL);
  shim_context(genome, genomealt, dynprogR);
  memset(&p, 0, sizeof(p));
  p.qoffL = (int32_t) (rsequenceL - lo);
  p.qoffR = (int32_t) (rev_rsequenceR - lo);
  p.rlengthL = rlengthL;
  p.rlengthR = rlengthR;
  p.glength = glength;
  p.roffsetL = roffsetL;
  p.rev_roffsetR = rev_roffsetR;
  p.goffset = goffset;
  p.chroffset = shim_coord(chroffset);
  p.chrhigh = shim_coord(chrhigh);
  p.flags = (watsonp ? GMAPDP_WATSON : 0) | (jump_late_p ? GMAPDP_JUMP_LATE : 0) | SHIM_SIMD;
  p.genestrand = genestrand;
  p.extraband = extraband_paired;
  p.dynprogindex = *dynprogindex;
  p.defect_rate = defect_rate;
  cap = gmapdp_cdna_pair_capacity(&p, 1);
  pairs = (gmapdp_pair *) malloc((cap ? cap : 1) * sizeof(gmapdp_pair));
  shim_check(gmapdp_cdna_gap_batch(shim_ctx, &p, 1, lo, lo_uc, (size_t) (hi - lo), &res, pairs, cap),
             "gmapdp_cdna_gap_batch");
  shim_count(ST_CDNA);
  pthread_mutex_unlock(&shim_lock);
  list = shim_list(pairs + res.pair_offset, res.npairs, p.dynprogindex, res.gap_index, res.gap_queryjump, -1, 0.0,
                   0.0, pairpool);
  free(pairs);
  *dynprogindex = res.dynprogindex;
  if (res.traceback_score != GMAPDP_UNSET) *traceback_score = res.traceback_score;
  if (res.incompletep) *incompletep = true;
  return list;
}

/* ---- stage-2 seeding: Oligoindex_hr_tally + Oligoindex_get_mappings (oligoindex_hr.c:33849/34127) ----
   Stage2_compute (stage2.c:6480-6495) calls the tally and then get_mappings for the same window; the
   tally only records its arguments here and the GPU runs both in get_mappings.  The table is allocated
   with GMAP's own MALLOC as this->table, so Oligoindex_untally frees it as usual. */
/* Thread-local: each GMAP worker runs Stage2_compute on its own oligoindices (gmap.c:4896), so the
   tally record of one thread must not be seen by another's get_mappings. */
static __thread struct {
  Oligoindex_T oligoindex;
  Univcoord_T mappingstart, mappingend;
  Chrpos_T chrpos;
  bool plusp;
  int querystart, queryend;
  Genome_T genome;
} shim_tally;

void
__wrap_Oligoindex_hr_tally (Oligoindex_T this, Univcoord_T mappingstart, Univcoord_T mappingend, bool plusp,
                            char *queryuc_ptr, int querystart, int queryend, Chrpos_T chrpos, Genome_T genome,
                            int genestrand) {
  (void) queryuc_ptr;
  (void) genestrand;
  if (shim_mode != 0) shim_refuse("stage-2 seeding outside STANDARD mode (cmet / atoi / ttoc reductions)");
  if (this->indexsize != 8) shim_refuse("an oligoindex with indexsize other than 8");
  shim_tally.oligoindex = this;
  shim_tally.mappingstart = mappingstart;
  shim_tally.mappingend = mappingend;
  shim_tally.plusp = plusp;
  shim_tally.chrpos = chrpos;
  shim_tally.querystart = querystart;
  shim_tally.queryend = queryend;
  shim_tally.genome = genome;
  this->table = NULL;
}

List_T
__wrap_Oligoindex_get_mappings (List_T diagonals, bool *coveredp, Chrpos_T **mappings, int *npositions,
                                int *totalpositions, bool *oned_matrix_p, int *maxnconsecutive,
                                Oligoindex_array_T array, Oligoindex_T this, char *queryuc_ptr, int querystart,
                                int queryend, int querylength, Chrpos_T chrstart, Chrpos_T chrend,
                                Univcoord_T chroffset, Univcoord_T chrhigh, bool plusp, Diagpool_T diagpool) {
  gmapdp_oligo_problem p;
  gmapdp_oligo_result res;
  int32_t *np, *mp, *dg;
  uint32_t *pos;
  size_t pc, dc;
  int q, k;
  (void) array;
  if (this != shim_tally.oligoindex || plusp != shim_tally.plusp || querystart != 0 || queryend != querylength ||
      shim_tally.querystart != 0 || shim_tally.queryend != querylength ||
      shim_tally.mappingstart != chroffset + chrstart ||
      shim_tally.mappingend != chroffset + chrend + (plusp ? 0 : 1) ||
      shim_tally.chrpos != (plusp ? chrstart : (Chrpos_T) (chrhigh - chroffset) - chrend))
    shim_refuse("Oligoindex_get_mappings on another window than Stage2_compute's tally");
  if (*totalpositions != 0 || *maxnconsecutive != 0) shim_refuse("a second oligoindex source (coverage loop)");
  for (q = 0; q < querylength; q++)
    if (coveredp[q]) shim_refuse("stage-2 seeding with covered query positions");
  memset(&p, 0, sizeof(p));
  p.qoff = 0;
  p.querylength = querylength;
  p.chrstart = chrstart;
  p.chrend = chrend;
  p.chroffset = shim_coord(chroffset);
  p.chrhigh = shim_coord(chrhigh);
  p.plusp = plusp ? 1 : 0;
  p.minor = this->diag_lookback == 60 ? 1 : 0;  /* Oligoindex_array_new_minor's index (oligoindex_hr.c:8612) */
  pthread_mutex_lock(&shim_lock);
  shim_context(shim_tally.genome, NULL, NULL);
  pc = gmapdp_oligo_positions_capacity(&p, 1);
  dc = gmapdp_oligo_diagonal_capacity(&p, 1);
  np = (int32_t *) malloc((querylength + 1) * sizeof(int32_t));
  mp = (int32_t *) malloc((querylength + 1) * sizeof(int32_t));
  pos = (uint32_t *) malloc((pc ? pc : 1) * sizeof(uint32_t));
  dg = (int32_t *) malloc(4 * (dc ? dc : 1) * sizeof(int32_t));
  shim_check(gmapdp_oligo_mappings_batch(shim_ctx, &p, 1, queryuc_ptr, (size_t) querylength, &res, np, mp, pos, pc,
                                         dg, dc), "gmapdp_oligo_mappings_batch");
  shim_count(ST_OLIGO);
  pthread_mutex_unlock(&shim_lock);
  /* the table, owned by the oligoindex (freed by Oligoindex_untally) */
  this->table = NULL;
  if (pc > 0) {
    this->table = (Chrpos_T *) MALLOC(pc * sizeof(Chrpos_T));
    memcpy(this->table, pos, pc * sizeof(Chrpos_T));
  }
  for (q = 0; q < querylength; q++) {
    if (np[q] > 0) {
      npositions[q] = np[q];
      mappings[q] = &this->table[mp[q]];
    } else if (q <= querylength - 8 && strspn(queryuc_ptr + q, "ACGT") >= 8) {
      /* lookup (:34069) on a full 8-mer without hits: nhits 0, mappings NULL; others stay as given */
      npositions[q] = 0;
      mappings[q] = NULL;
    }
  }
  *totalpositions = res.totalpositions;
  *maxnconsecutive = res.maxnconsecutive;
  if (chrend > chrstart) *oned_matrix_p = res.oned_matrix_p ? true : false;
  for (k = res.ndiagonals - 1; k >= 0; k--) {
    const int32_t *d = dg + 4 * (res.diag_offset + k);
    diagonals = Diagpool_push(diagonals, diagpool, d[0], d[1], d[2], d[3]);
  }
  free(np);
  free(mp);
  free(pos);
  free(dg);
  return diagonals;
}
