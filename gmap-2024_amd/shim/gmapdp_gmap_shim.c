/* gmapdp_gmap_shim.c -- drop-in for GMAP's Dynprog_* entry points on the MI355X engine.
 *
 * Compiled INSIDE a GMAP build (against GMAP's own headers, -DHAVE_CONFIG_H)
 * and linked with
 *
 *   -Wl,--wrap=Dynprog_init,--wrap=Dynprog_single_setup,--wrap=Dynprog_end_setup,
 *   -Wl,--wrap=Dynprog_genome_setup,--wrap=Dynprog_single_gap,--wrap=Dynprog_end5_gap,
 *   -Wl,--wrap=Dynprog_end3_gap,--wrap=Dynprog_genome_gap,--wrap=Dynprog_cdna_gap
 *   -Wl,--wrap=Oligoindex_hr_tally,--wrap=Oligoindex_get_mappings
 *   -Wl,--wrap=Stage2_setup,--wrap=Stage2_compute
 *   -Wl,--wrap=Dynprog_end5_splicejunction,--wrap=Dynprog_end3_splicejunction
 *   -Wl,--wrap=Dynprog_end5_known,--wrap=Dynprog_end3_known  -lgmapdp
 *
 * so that every call GMAP's stage 3 makes to these functions (stage3.c:9081,
 * 9275, 9510, 9531, 10244-10600, ...), and GMAP's per-read Stage2_compute (gmap.c:1208, 1323: seeding
 * and chaining, one call per genomic region), lands here with the reference's own signature
 * (dynprog_single.h:22, dynprog_end.h:25/47, dynprog_genome.h:24, dynprog_cdna.h:12) and returns
 * the reference's List_T of Pair_T built in the caller's Pairpool
 * (Pairpool_push / Pairpool_push_gapholder, pairpool.c:180/375).  The setup
 * functions are wrapped only to learn Mode_T, the user gap penalties and, with known splice sites
 * (-s), the site list, the splice tries and the splicing IIT; the reference's own setup still runs.
 * With -s, Dynprog_end5/3_known are restated here over the engine (the reference's
 * Splicetrie_solve_end5/3 walks the tries and its splice-junction calls land on the engine too), and
 * the genome gaps carry their windows' known sites.  See INTEGRATION.md.
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
 * Batching.  GMAP's worker threads (gmap.c:4867) each issue their calls one at a time and wait for
 * the answer (the API is synchronous).  Here a call becomes a request on one of three process-wide queues
 * and the calling thread sleeps on its own request.  Dispatcher threads each own an engine context with
 * one stream (the genome is uploaded to HBM once and shared): GMAPDP_SHIM_DISPATCHERS (default 2) on
 * queue 0, the short Dynprog_* calls (high-priority streams); GMAPDP_SHIM_LONG_DISPATCHERS (default 1) on
 * queue 2, the long fills and stage 3's oligoindex calls; GMAPDP_SHIM_STAGE2_DISPATCHERS (default 2) on
 * queue 1, Stage2_compute (low-priority streams).  That is five streams on HIP's default four hardware
 * queues (GPU_MAX_HW_QUEUES), so two of them share a queue; end to end, four dispatchers (one stage-2)
 * or more hardware queues measured slower (tools/e2e_timing.py --configs, profiles/r03_e2e).  A free
 * dispatcher takes every request queued meanwhile and runs them together: single / end / genome gaps and
 * microexon calls in one gmapdp_mixed_batch (one round trip), cDNA gaps, splice-junction ends and
 * stage-2 seeding in their own batches.  The callers then build their List_T from their own results in
 * their own Pairpool.  With many worker threads per GPU (gmap -t N, N well above the core count: the
 * workers mostly wait) one launch set carries many reads' calls.  GMAPDP_SHIM_STATS=1 prints the call
 * counts and the mean batch size.
 *
 * MaxEnt.  The genome gaps' splice probabilities and the microexon candidates' are evaluated by the
 * engine on the device (Maxent_hr_*_prob restated over the HBM genome, bit-identical doubles), so a
 * microexon call is one request; GMAPDP_SHIM_HOST_MAXENT=1 keeps the host's maxent_hr.c instead.
 */
#ifndef _GNU_SOURCE
#define _GNU_SOURCE
#endif
#ifdef HAVE_CONFIG_H
#include "config.h"
#endif
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <pthread.h>
#include <sys/prctl.h>

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
#include "cellpool.h"
#include "stopwatch.h"
#include "stage2.h"
#include "splicetrie.h"
#include "iit-read.h"
#include "complement.h"
#include "mem.h"

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

static __thread gmapdp_ctx *shim_ctx = NULL;   /* each dispatcher thread owns one engine context */
static __thread Genome_T shim_genome = NULL;  /* the genome resident in that context's HBM */
static int shim_mode = 0, shim_user_open = 0, shim_user_extend = 0, shim_user_dynprog_p = 0;
static int shim_homopolymerp = 0, shim_splicing_iit = 0;

/* Calls that reached the engine, per wrapped entry point (printed at exit with GMAPDP_SHIM_STATS=1;
   tests use it to prove the pipeline really ran on the GPU). */
enum { ST_SINGLE, ST_END5, ST_END3, ST_GENOME, ST_CDNA, ST_OLIGO, ST_STAGE2, ST_MICROEXON, ST_SJ5, ST_SJ3,
       ST_KNOWN5, ST_KNOWN3, ST_N };
static const char *const shim_stat_name[ST_N] = {"Dynprog_single_gap", "Dynprog_end5_gap", "Dynprog_end3_gap",
                                                 "Dynprog_genome_gap", "Dynprog_cdna_gap",
                                                 "Oligoindex_get_mappings", "Stage2_compute",
                                                 "Dynprog_microexon_int", "Dynprog_end5_splicejunction",
                                                 "Dynprog_end3_splicejunction", "Dynprog_end5_known",
                                                 "Dynprog_end3_known"};
static unsigned long shim_stats[ST_N];

static unsigned long shim_batches, shim_batched;
static FILE *shim_trace = NULL;  /* GMAPDP_SHIM_TRACE: per-batch record (diagnostics) */
static double shim_secs[4];  /* dispatcher wall time in the DP, cDNA, seeding and Stage2_compute batches */

#include <time.h>
static double
shim_now (void) {
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return (double) ts.tv_sec + 1e-9 * (double) ts.tv_nsec;
}

static void
shim_print_stats (void) {
  int i;
  fprintf(stderr, "gmapdp shim calls:");
  for (i = 0; i < ST_N; i++) fprintf(stderr, " %s=%lu", shim_stat_name[i], __atomic_load_n(&shim_stats[i], __ATOMIC_RELAXED));
  fprintf(stderr, " batches=%lu mean_batch=%.2f dp_s=%.3f cdna_s=%.3f stage2_s=%.3f chain_s=%.3f\n", shim_batches,
          shim_batches ? (double) shim_batched / (double) shim_batches : 0.0, shim_secs[0], shim_secs[1], shim_secs[2],
          shim_secs[3]);
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

/* Universal coordinates travel as 64-bit gmapdp_coord_t, so the same shim serves gmap (32-bit
   Univcoord_T) and gmapl (LARGE_GENOMES, 64-bit Univcoord_T, univcoord.h:9-11). */
static gmapdp_coord_t
shim_coord (Univcoord_T x) {
  return (gmapdp_coord_t) x;
}

static void
shim_check (int rc, const char *what) {
  if (rc != GMAPDP_OK) {
    fprintf(stderr, "gmapdp shim: %s failed (%d): %s\n", what, rc, gmapdp_last_error(shim_ctx));
    abort();
  }
}

#ifdef GMAPDP_SHIM_OWN
/* ---- the rest of the Dynprog_* interface, owned here (GMAP links without the six dynprog*.o) ---- */

/* consistent_array (dynprog.c:890) as Dynprog_init fills it (permute_cases / permute_cases_oneway,
   :904-1004, with PREUC, dynprog.h:165: every case combination of a pair): the (query, genome) characters
   that count as consistent, per genestrand -- [0] for STANDARD and the stranded modes, [+1] / [+2] for the
   nonstranded ones.  Only Dynprog_consistent_p reads it; the engine has its own device tables. */
static bool shim_consistent[3][128][128];

static void
shim_consistent_mark (int gs, int a, int b) {
  const int as[2] = {a, a - 'A' + 'a'}, bs[2] = {b, b - 'A' + 'a'};
  int i, j;
  for (i = 0; i < 2; i++)
    for (j = 0; j < 2; j++) shim_consistent[gs][as[i]][bs[j]] = true;
}

static void
shim_consistent_pair (int a, int b, Mode_T mode) {  /* permute_cases: both orders */
  if (mode == STANDARD || mode == CMET_STRANDED || mode == ATOI_STRANDED || mode == TTOC_STRANDED) {
    shim_consistent_mark(0, a, b);
    shim_consistent_mark(0, b, a);
  } else {
    shim_consistent_mark(1, a, b);
    shim_consistent_mark(2, a, b);
    shim_consistent_mark(1, b, a);
    shim_consistent_mark(2, b, a);
  }
}

static void
shim_init_tables (Mode_T mode) {
  /* FULLMATCH 'U'/'T', HALFMATCH and AMBIGUOUS IUPAC pairs, and N/N, X/X (dynprog.c:1094-1141) */
  static const char pairs[][2] = {{'U', 'T'}, {'R', 'A'}, {'R', 'G'}, {'Y', 'T'}, {'Y', 'C'}, {'W', 'A'}, {'W', 'T'},
                                  {'S', 'G'}, {'S', 'C'}, {'M', 'A'}, {'M', 'C'}, {'K', 'G'}, {'K', 'T'}, {'H', 'A'},
                                  {'H', 'T'}, {'H', 'C'}, {'B', 'G'}, {'B', 'C'}, {'B', 'T'}, {'V', 'G'}, {'V', 'A'},
                                  {'V', 'C'}, {'D', 'G'}, {'D', 'A'}, {'D', 'T'}, {'N', 'T'}, {'N', 'C'}, {'N', 'A'},
                                  {'N', 'G'}, {'X', 'T'}, {'X', 'C'}, {'X', 'A'}, {'X', 'G'}, {'N', 'N'}, {'X', 'X'}};
  int c;
  size_t i;
  memset(shim_consistent, 0, sizeof(shim_consistent));
  for (c = 'A'; c < 'Z'; c++) shim_consistent_pair(c, c, mode);  /* 'A'..'Y', as :1089 */
  for (i = 0; i < sizeof(pairs) / sizeof(pairs[0]); i++) shim_consistent_pair(pairs[i][0], pairs[i][1], mode);
  switch (mode) {  /* the one-way pairs of the bisulfite / RNA-editing modes (:1145-1173) */
  case STANDARD: break;
  case CMET_STRANDED: shim_consistent_mark(0, 'T', 'C'); break;
  case CMET_NONSTRANDED: shim_consistent_mark(1, 'T', 'C'); shim_consistent_mark(2, 'A', 'G'); break;
  case ATOI_STRANDED: shim_consistent_mark(0, 'G', 'A'); break;
  case ATOI_NONSTRANDED: shim_consistent_mark(1, 'G', 'A'); shim_consistent_mark(2, 'C', 'T'); break;
  case TTOC_STRANDED: shim_consistent_mark(0, 'C', 'T'); break;
  case TTOC_NONSTRANDED: shim_consistent_mark(1, 'C', 'T'); shim_consistent_mark(2, 'G', 'A'); break;
  default:
    fprintf(stderr, "Mode %d not recognized\n", mode);
    exit(9);
  }
}

bool
Dynprog_consistent_p (int c, int g, int g_alt, int genestrand) {  /* dynprog.c:895 */
  return shim_consistent[genestrand][c][g] || shim_consistent[genestrand][c][g_alt];
}

void
Dynprog_term (Mode_T mode) {  /* dynprog.c:1203: the tables are static here */
  (void) mode;
}

int
Dynprog_score (int matches, int mismatches, int qopens, int qindels, int topens, int tindels, double defect_rate,
               int user_open, int user_extend, bool user_dynprog_p) {  /* dynprog.c:126 */
  int mismatch, open, extend;
  if (user_dynprog_p == true) {
    mismatch = MISMATCH_HIGHQ;
    open = user_open;
    extend = user_extend;
  } else if (defect_rate < DEFECT_HIGHQ) {
    mismatch = MISMATCH_HIGHQ;
    open = SINGLE_OPEN_HIGHQ;
    extend = SINGLE_EXTEND_HIGHQ;
  } else if (defect_rate < DEFECT_MEDQ) {
    mismatch = MISMATCH_MEDQ;
    open = SINGLE_OPEN_MEDQ;
    extend = SINGLE_EXTEND_MEDQ;
  } else {
    mismatch = MISMATCH_LOWQ;
    open = SINGLE_OPEN_LOWQ;
    extend = SINGLE_EXTEND_LOWQ;
  }
  return FULLMATCH * matches + mismatch * mismatches + open * qopens + extend * qindels + open * topens +
         extend * tindels;
}

/* Dynprog_new (dynprog.c:631) as a limits-only handle: compute_maxlengths (:606) sets the two limits the
   engine checks (shim_check_call); the score and direction arenas the reference allocates per worker
   (12-17 MB each, three per worker thread) are never touched by the engine, so none are made. */
Dynprog_T
Dynprog_new (int maxlookback, int extraquerygap, int maxpeelback, int extramaterial_end, int extramaterial_paired,
             bool doublep) {
  Dynprog_T d = (Dynprog_T) calloc(1, sizeof(*d));
  int max_rlength = maxlookback + maxpeelback, max_glength;
  (void) doublep;
  if (d == NULL) {
    fprintf(stderr, "gmapdp shim: out of memory in Dynprog_new\n");
    abort();
  }
  if (max_rlength < 500) max_rlength = 500;  /* QUERY_MAXLENGTH */
  max_glength = max_rlength + extraquerygap +
                (extramaterial_end > extramaterial_paired ? extramaterial_end : extramaterial_paired);
  if (max_glength < 2000) max_glength = 2000;  /* GENOMIC_MAXLENGTH */
  d->max_rlength = max_rlength;
  d->max_glength = max_glength;
  return d;
}

void
Dynprog_free (Dynprog_T *old) {  /* dynprog.c:777 */
  if (*old) {
    free(*old);
    *old = NULL;
  }
}

static void shim_revcomp_inplace (char *s, int length);

/* The far piece of a splice junction (Dynprog_make_splicejunction_5 / _3, dynprog_end.c:2569 / 2670):
   splicelength genome characters that end at the far site (donor / antiacceptor) or start there
   (acceptor / antidonor), reverse-complemented on the minus strand.  False when the piece would start
   before the genome. */
static bool
shim_splicejunction_far (char *distal, char *distal_alt, Univcoord_T splicecoord, int splicelength,
                         Splicetype_T far_splicetype, Genome_T genome, Genome_T genomealt, bool watsonp) {
  if (far_splicetype == ACCEPTOR || far_splicetype == ANTIDONOR) {
    Genome_fill_buffer_blocks_noterm(genome, genomealt, splicecoord, (Chrpos_T) splicelength, distal, distal_alt);
  } else if (splicecoord <= (Univcoord_T) splicelength) {
    return false;
  } else if (far_splicetype == ANTIACCEPTOR || far_splicetype == DONOR) {
    Genome_fill_buffer_blocks_noterm(genome, genomealt, splicecoord - splicelength, (Chrpos_T) splicelength, distal,
                                     distal_alt);
  } else {
    fprintf(stderr, "Unexpected far_splicetype value %d\n", far_splicetype);
    abort();
  }
  if (watsonp == false) {
    shim_revcomp_inplace(distal, splicelength);
    shim_revcomp_inplace(distal_alt, splicelength);
  }
  return true;
}

bool
Dynprog_make_splicejunction_5 (char *splicejunction, char *splicejunction_alt, Univcoord_T splicecoord,
                               int splicelength, int contlength, Splicetype_T far_splicetype, Genome_T genome,
                               Genome_T genomealt, bool watsonp) {
  (void) contlength;  /* the far piece leads the 5' junction */
  return shim_splicejunction_far(splicejunction, splicejunction_alt, splicecoord, splicelength, far_splicetype,
                                 genome, genomealt, watsonp);
}

bool
Dynprog_make_splicejunction_3 (char *splicejunction, char *splicejunction_alt, Univcoord_T splicecoord,
                               int splicelength, int contlength, Splicetype_T far_splicetype, Genome_T genome,
                               Genome_T genomealt, bool watsonp) {
  return shim_splicejunction_far(&splicejunction[contlength], &splicejunction_alt[contlength], splicecoord,
                                 splicelength, far_splicetype, genome, genomealt, watsonp);
}
#endif

void
GMAPDP_DYNPROG_ENTRY(Dynprog_init) (Mode_T mode) {
#ifdef GMAPDP_SHIM_OWN
  shim_init_tables(mode);
#else
  __real_Dynprog_init(mode);
#endif
  shim_mode = (int) mode;
}

void
GMAPDP_DYNPROG_ENTRY(Dynprog_single_setup) (int user_open_in, int user_extend_in, bool user_dynprog_p_in, bool homopolymerp_in) {
#ifndef GMAPDP_SHIM_OWN
  __real_Dynprog_single_setup(user_open_in, user_extend_in, user_dynprog_p_in, homopolymerp_in);
#endif
  shim_user_open = user_open_in;
  shim_user_extend = user_extend_in;
  shim_user_dynprog_p = user_dynprog_p_in ? 1 : 0;
  shim_homopolymerp = homopolymerp_in ? 1 : 0;
}

/* Known splice sites (-s), as Dynprog_end_setup records them (dynprog_end.c:119-141): the sites sorted by
   position with their types, and the observed / max-distance splice tries that Splicetrie_solve_end5/3
   (splicetrie.c) walk.  Dynprog_end5/3_known below restate their orchestration over these. */
static Univcoord_T *shim_splicesites = NULL;
static Splicetype_T *shim_splicetypes = NULL;
static int shim_nsplicesites = 0;
static Trieoffset_T *shim_trieoffsets_obs = NULL, *shim_trieoffsets_max = NULL;
static Triecontent_T *shim_triecontents_obs = NULL, *shim_triecontents_max = NULL;

void
GMAPDP_DYNPROG_ENTRY(Dynprog_end_setup) (Univcoord_T *splicesites_in, Splicetype_T *splicetypes_in, Chrpos_T *splicedists_in,
                          int nsplicesites_in, Trieoffset_T *trieoffsets_obs_in, Triecontent_T *triecontents_obs_in,
                          Trieoffset_T *trieoffsets_max_in, Triecontent_T *triecontents_max_in,
                          int user_open_in, int user_extend_in, bool user_dynprog_p_in) {
  shim_splicesites = splicesites_in;
  shim_splicetypes = splicetypes_in;
  shim_nsplicesites = nsplicesites_in;
  shim_trieoffsets_obs = trieoffsets_obs_in;
  shim_triecontents_obs = triecontents_obs_in;
  shim_trieoffsets_max = trieoffsets_max_in;
  shim_triecontents_max = triecontents_max_in;
#ifdef GMAPDP_SHIM_OWN
  (void) splicedists_in;
  (void) user_open_in;
  (void) user_extend_in;
  (void) user_dynprog_p_in;
#else
  __real_Dynprog_end_setup(splicesites_in, splicetypes_in, splicedists_in, nsplicesites_in, trieoffsets_obs_in,
                           triecontents_obs_in, trieoffsets_max_in, triecontents_max_in, user_open_in,
                           user_extend_in, user_dynprog_p_in);
#endif
}

/* The splicing IIT of -s as Dynprog_genome_setup records it (dynprog_genome.c:192-214): the genome
   gaps look their window's known sites up in it (get_known_splicesites, :405, restated below). */
static IIT_T shim_siit = NULL;
static int *shim_siit_cross = NULL;
static int shim_donor_typeint = -1, shim_acceptor_typeint = -1;

void
GMAPDP_DYNPROG_ENTRY(Dynprog_genome_setup) (bool novelsplicingp_in, IIT_T splicing_iit_in, int *splicing_divint_crosstable_in,
                             int donor_typeint_in, int acceptor_typeint_in, int user_open_in, int user_extend_in,
                             bool user_dynprog_p_in) {
  if (splicing_iit_in != NULL) {
    /* an introns file (no donor/acceptor types: intron-level bridging, dynprog_genome.c:2944) and
       known-only splicing (novel splicing off: genome_gap_simple then requires known sites, :3157) are
       not built */
    if (donor_typeint_in < 0 || acceptor_typeint_in < 0)
      shim_refuse("a known-introns file (-s without donor/acceptor tags: intron-level bridging)");
    if (!novelsplicingp_in) shim_refuse("known splice sites with novel splicing off");
  }
#ifndef GMAPDP_SHIM_OWN
  __real_Dynprog_genome_setup(novelsplicingp_in, splicing_iit_in, splicing_divint_crosstable_in, donor_typeint_in,
                              acceptor_typeint_in, user_open_in, user_extend_in, user_dynprog_p_in);
#endif
  shim_splicing_iit = splicing_iit_in != NULL;
  shim_siit = splicing_iit_in;
  shim_siit_cross = splicing_divint_crosstable_in;
  shim_donor_typeint = donor_typeint_in;
  shim_acceptor_typeint = acceptor_typeint_in;
}

/* get_known_splicesites (dynprog_genome.c:405-510), splice-site level: flags (1 = known) at the
   positions of left_known[0, glengthL] / right_known[0, glengthR] that the reference sets to
   KNOWN_SPLICESITE_REWARD.  The same IIT queries over the same (Chrpos_T) ranges. */
static void
shim_mark_sites (uint8_t *known, int index_sign, int index_base, Chrpos_T x, Chrpos_T y, int typeint, int sign,
                 Chrnum_T chrnum) {
  int *matches, nmatches, i;
  matches = IIT_get_typed_signed_with_divno(&nmatches, shim_siit, shim_siit_cross[chrnum], x, y, typeint, sign,
                                            /*sortp*/false);
  for (i = 0; i < nmatches; i++) {
    const int pos = (int) IIT_interval_low(shim_siit, matches[i]);
    known[index_sign > 0 ? pos - index_base : index_base - pos] = 1;
  }
  FREE(matches);
}

static void
shim_known_sites (uint8_t *left_known, uint8_t *right_known, int glengthL, int glengthR, int leftoffset,
                  int rightoffset, int cdna_direction, bool watsonp, Chrnum_T chrnum, Univcoord_T chroffset,
                  Univcoord_T chrhigh) {
  const int span = (int) (chrhigh - chroffset);
  const int ldonor = cdna_direction > 0 ? shim_donor_typeint : shim_acceptor_typeint;
  const int racceptor = cdna_direction > 0 ? shim_acceptor_typeint : shim_donor_typeint;
  if (watsonp) {
    const int sign = cdna_direction > 0 ? +1 : -1;
    /* left: splicesitepos = leftoffset + cL; right: splicesitepos = rightoffset - cR + 1 */
    shim_mark_sites(left_known, +1, leftoffset, leftoffset + 1, leftoffset + glengthL - 2, ldonor, sign, chrnum);
    shim_mark_sites(right_known, -1, rightoffset + 1, rightoffset - glengthR + 4, rightoffset + 1, racceptor, sign,
                    chrnum);
  } else {
    const int sign = cdna_direction > 0 ? -1 : +1;
    /* left: splicesitepos = span - leftoffset - cL + 1; right: splicesitepos = span - rightoffset + cR */
    shim_mark_sites(left_known, -1, span - leftoffset + 1, span - leftoffset - glengthL + 4, span - leftoffset + 1,
                    ldonor, sign, chrnum);
    shim_mark_sites(right_known, +1, span - rightoffset, span - rightoffset + 1, span - rightoffset + glengthR - 2,
                    racceptor, sign, chrnum);
  }
}

/* Refusals that depend on the caller's Dynprog_T / genomes (checked on the calling thread). */
static void
shim_check_call (Genome_T genome, Genome_T genomealt, Dynprog_T dynprog) {
  if (genomealt != NULL && genomealt != genome) shim_refuse("an alternate-allele genome (genomealt)");
  if (dynprog != NULL && (dynprog->max_rlength != GMAPDP_MAX_RLENGTH || dynprog->max_glength != GMAPDP_MAX_GLENGTH))
    shim_refuse("a Dynprog_T with non-default maximum lengths");
}

/* The engine context with `genome` resident in HBM (dispatcher thread only).  Every dispatcher owns a
   context with a single stream -- DP dispatchers at the device's highest stream priority, stage-2
   dispatchers at its lowest -- so that the dispatchers' streams fit the process's hardware queues
   (GPU_MAX_HW_QUEUES) and a DP batch never queues behind a stage-2 sweep.  Each GMAP genome (a Genome_T;
   a -g run over a multi-sequence file has several) is uploaded to HBM once, as a device genome every
   dispatcher context reads (gmapdp_dgenome_create / gmapdp_use_dgenome). */
static __thread int shim_reserved = 0;
static int shim_oligo_queue = 2;            /* the queue of stage 3's oligoindex calls (GMAPDP_SHIM_OLIGO_QUEUE) */
static __thread int shim_qi = 0;            /* the dispatcher's queue: 0 Dynprog_*, 1 stage 2, 2 long fills */
typedef struct shim_dgenome {
  Genome_T genome;
  gmapdp_dgenome *dg;
  struct shim_dgenome *next;
} shim_dgenome;
static pthread_mutex_t g_lock = PTHREAD_MUTEX_INITIALIZER;
static shim_dgenome *g_genomes = NULL;

static int
shim_device (void) {
  const char *dev = getenv("GMAPDP_DEVICE");
  return dev ? atoi(dev) : 0;
}

static gmapdp_ctx *
shim_context (Genome_T genome) {
  shim_dgenome *e;
  uint64_t length;
  size_t nwords;
  if (shim_ctx == NULL) {
    /* How a dispatcher waits for its batch: by default it polls the batch's completion every
       GMAPDP_POLL_US (10) microseconds and sleeps in between (GMAPDP_CTX_POLL_SYNC), which leaves the
       cores to GMAP's workers; GMAPDP_SHIM_POLL=0 spins in HIP's wait, GMAPDP_SHIM_BLOCKING=1 sleeps on
       a blocking-sync event (both measured slower end to end, profiles/r03_e2e). */
    const char *blk = getenv("GMAPDP_SHIM_BLOCKING"), *poll = getenv("GMAPDP_SHIM_POLL");
    const int wait = blk != NULL && blk[0] == '1' ? GMAPDP_CTX_BLOCKING_SYNC
                     : (poll != NULL && poll[0] == '0' ? 0 : GMAPDP_CTX_POLL_SYNC);
    /* GMAPDP_SHIM_MULTI_STREAM=1 (experiments): the short-call dispatchers' contexts keep their side streams,
       so a batch's launch classes can run side by side (with GMAPDP_SMALL_BATCH_STREAMS=1 in the engine) */
    const char *ms = getenv("GMAPDP_SHIM_MULTI_STREAM");
    const int one = (ms != NULL && ms[0] == '1' && shim_qi == 0) ? 0 : GMAPDP_CTX_ONE_STREAM;
    shim_check(gmapdp_create_ex(&shim_ctx, shim_device(), shim_mode, shim_user_open, shim_user_extend,
                                shim_user_dynprog_p, one | wait |
                                    (shim_qi != 1 ? GMAPDP_CTX_PRIO_HIGH : GMAPDP_CTX_PRIO_LOW)),
               "gmapdp_create_ex");
  }
  if (!shim_reserved) {  /* staging and scratch sized up front: growing them later stalls the device */
    shim_check(gmapdp_reserve(shim_ctx, shim_qi == 1 ? (size_t) 64 << 20 : (size_t) 16 << 20,
                              shim_qi == 1 ? GMAPDP_RESERVE_STAGE2
                                           : GMAPDP_RESERVE_DP | GMAPDP_RESERVE_AUX |
                                                 (shim_qi == shim_oligo_queue ? GMAPDP_RESERVE_STAGE2 : 0)),
               "gmapdp_reserve");
    shim_reserved = 1;
  }
  if (genome != shim_genome) {
    pthread_mutex_lock(&g_lock);
    for (e = g_genomes; e != NULL && e->genome != genome; e = e->next) ;
    if (e == NULL) {
      e = (shim_dgenome *) calloc(1, sizeof(shim_dgenome));
      if (e == NULL) shim_refuse("host memory for a genome record (out of memory)");
      length = (uint64_t) Genome_genomelength(genome);
      nwords = gmapdp_genome_words(length);
      shim_check(gmapdp_dgenome_create(shim_device(), (const uint32_t *) Genome_blocks(genome), nwords, length,
                                       &e->dg), "gmapdp_dgenome_create");
      e->genome = genome;
      e->next = g_genomes;
      g_genomes = e;
    }
    pthread_mutex_unlock(&g_lock);
    shim_check(gmapdp_use_dgenome(shim_ctx, e->dg), "gmapdp_use_dgenome");
    shim_genome = genome;
  }
  return shim_ctx;
}

/* ---- requests and the dispatcher ---- */
enum { K_SINGLE, K_END, K_GENOME, K_CDNA, K_MXS, K_MXF, K_OLIGO, K_STAGE2, K_SJ, K_MXW };  /* K_MXS / K_MXF: microexon
                                                                   search / finish; K_MXW: the whole call */

/* MaxEnt splice-site probabilities: on the device (the engine's Maxent_hr_*_prob restatement over its HBM
   genome, bit-identical doubles; include/gmapdp.h "Device MaxEnt") unless GMAPDP_SHIM_HOST_MAXENT=1, which
   keeps the host's own maxent_hr.c on the calling thread (two round trips per microexon call). */
static int shim_host_maxent = -1;
static int
shim_use_host_maxent (void) {
  if (shim_host_maxent < 0) {
    const char *st = getenv("GMAPDP_SHIM_HOST_MAXENT");
    shim_host_maxent = st != NULL && st[0] == '1';
  }
  return shim_host_maxent;
}

typedef struct shim_req {
  int kind;
  Genome_T genome;
  union {
    gmapdp_single_problem s;
    gmapdp_end_problem e;
    gmapdp_genome_problem g;
    gmapdp_cdna_problem c;
    gmapdp_oligo_problem o;
    gmapdp_stage2_problem s2;
    gmapdp_microexon_problem mx;
    gmapdp_sj_problem sj;
  } p;                          /* qoff / prob_offset relative to q and probs below */
  const char *q, *quc;          /* the query slice (borrowed: the caller waits) */
  char q9[16], quc9[16];        /* an 8-nt query as the 8-mer + 'N' (owned by the request across the
                                   caller's yield: another fiber of the same host may make such a call) */
  size_t qlen;
  const char *j;                /* splice-junction end gaps: the junction string (borrowed) */
  size_t jlen;
  uint8_t *known;               /* genome gaps with known splice sites: the flags (gmapdp_genome_known_bytes) */
  size_t nknown, knowncap;
  const double *probs;          /* genome gaps: the splice probabilities */
  size_t nprobs;
  /* outputs, filled by the dispatcher (pair_offset / table_offset / diag_offset rebased to 0) */
  gmapdp_result r;
  gmapdp_genome_result gr;
  gmapdp_cdna_result cr;
  gmapdp_sj_result sjr;
  gmapdp_oligo_result orr;
  gmapdp_stage2_result s2r;     /* path_offset rebased to 0, pair_offset of each path to the request's pairs */
  /* per-thread buffers (grown by the caller before submitting) */
  gmapdp_pair *pairs;
  size_t pcap;
  double *pbuf;
  size_t pbufcap;
  int32_t *np, *mp, *dg;
  uint32_t *pos;
  size_t npcap, mpcap, poscap, dgcap;
  size_t tabn;                  /* stage-2 seeding: the problem's table capacity */
  gmapdp_path *s2paths;         /* Stage2_compute: the results' path records and pairs */
  gmapdp_path_pair *s2pairs;
  size_t s2pathcap, s2paircap;
  gmapdp_microexon_result mxr;  /* microexon: cand_offset rebased to 0, pair_offset to 0 */
  gmapdp_microexon_candidate *mxc;
  double *mxp;                  /* the caller's MaxEnt probabilities of its candidates (2 per candidate) */
  size_t mxccap, mxpcap;
  int done;
  struct shim_fiber *fiber;     /* the calling fiber (GMAPDP_SHIM_FIBERS), else NULL: the caller sleeps on cv */
  int longp;                    /* a long fill: queue 2 */
  long cost;                    /* shim_cost of the fill (diagnostics) */
  pthread_mutex_t mtx;          /* guards done (the calling thread sleeps on cv) */
  pthread_cond_t cv;
  struct shim_req *next;
} shim_req;

/* Three queues: 0 for the short Dynprog_* calls (~250 per read), 1 for Stage2_compute (two ~10-ms
   batches per read), 2 for the long fills and stage 3's oligoindex calls, so that no call waits
   behind a batch far longer than its own work. */
static pthread_mutex_t q_lock = PTHREAD_MUTEX_INITIALIZER;
static pthread_cond_t q_cond[3] = {PTHREAD_COND_INITIALIZER, PTHREAD_COND_INITIALIZER, PTHREAD_COND_INITIALIZER};
static shim_req *q_head[3] = {NULL, NULL, NULL}, *q_tail[3] = {NULL, NULL, NULL};
/* Queue 2: Dynprog_* calls whose fill is long (shim_cost above GMAPDP_SHIM_LONG_COST, default 400 band-word
   columns: end gaps against up to 2000 genome columns, wide bands).  A batch lasts as long as its longest
   fill, so these get their own dispatcher and never hold back the short calls that are most of a read. */
static long shim_long_cost = 400;

/* band-word columns of a banded fill: columns x ceil(band width / 64) (Dynprog_compute_bands, wide band) */
static long
shim_cost (int rlength, int glength, int extraband) {
  long g = glength > 2000 ? 2000 : glength, w = (long) abs(glength - rlength) + 2L * extraband + 1L;
  return g < 0 ? 0 : g * ((w + 63) / 64);
}
static int dispatcher_started = 0;
static __thread shim_req *tl_req = NULL;

/* ---- fibers: GMAP's worker threads as user-level contexts (the owned link, GMAPDP_SHIM_OWN) ----
   GMAP runs one OS thread per worker (gmap.c:6639, worker_thread :4867), and each worker's read makes
   ~270 serially dependent engine calls; with hundreds of workers per GPU every call was a futex sleep and
   a scheduler wake-up of one of 512-2 048 threads.  Linked with --wrap=pthread_create,pthread_join,
   pthread_getspecific,pthread_setspecific, the workers become fibers: GMAPDP_SHIM_FIBER_HOSTS (default 16)
   OS threads each run their share round-robin, and a fiber's engine call queues its request and switches
   to the next runnable fiber of its host (swapcontext) instead of sleeping; a dispatcher that finishes a
   batch makes the callers' fibers runnable again, one wake-up per idle host.  GMAP keeps its per-thread
   state in pthread keys only (except.c:34-132 exception stacks, gmap.c:4920 the request), which become
   per-fiber; the output thread (Outbuffer_thread_*) stays an OS thread.  GMAPDP_SHIM_FIBERS=0 turns it
   off (one OS thread per worker, as before). */
#ifdef GMAPDP_SHIM_OWN
#include <ucontext.h>
#include <sys/mman.h>
#include "outbuffer.h"

extern int __real_pthread_create (pthread_t *th, const pthread_attr_t *attr, void *(*fn)(void *), void *arg);
extern int __real_pthread_join (pthread_t th, void **ret);
extern void *__real_pthread_getspecific (pthread_key_t key);
extern int __real_pthread_setspecific (pthread_key_t key, const void *value);

#define SHIM_NKEYS 64
#define SHIM_MAXHOSTS 256
#define SHIM_FIBER_STACK (8UL << 20)  /* glibc's default thread stack (reserved, touched pages only) */

typedef struct shim_fiber {
  ucontext_t ctx;
  struct shim_host *host;
  void *(*fn) (void *);
  void *arg, *ret;
  int finished;                /* 1: returned, 2: its host has left its stack (joinable) */
  shim_req *req;               /* the fiber's request (tl_req of an OS thread) */
  void *keys[SHIM_NKEYS];      /* pthread_getspecific / _setspecific values */
  void *stack;
  pthread_mutex_t jm;
  pthread_cond_t jc;
  struct shim_fiber *next, *all_next;
} shim_fiber;

typedef struct shim_host {
  ucontext_t ctx;              /* the scheduler loop's context */
  pthread_mutex_t mu;
  pthread_cond_t cv;
  shim_fiber *head, *tail;     /* runnable fibers */
} shim_host;

static shim_host shim_hosts[SHIM_MAXHOSTS];
static int shim_nhosts = 0, shim_nfibers = 0, shim_fiber_mode = -1, shim_fiber_hosts = 16;
static pthread_mutex_t shim_fiber_lock = PTHREAD_MUTEX_INITIALIZER;
static shim_fiber *shim_all_fibers = NULL;
static __thread shim_fiber *cur_fiber = NULL;

static int
shim_fibers_on (void) {
  if (shim_fiber_mode < 0) {
    const char *st = getenv("GMAPDP_SHIM_FIBERS");
    shim_fiber_mode = !(st != NULL && st[0] == '0');
    st = getenv("GMAPDP_SHIM_FIBER_HOSTS");
    if (st != NULL && atoi(st) > 0) shim_fiber_hosts = atoi(st) < SHIM_MAXHOSTS ? atoi(st) : SHIM_MAXHOSTS;
  }
  return shim_fiber_mode;
}

static void
shim_host_ready (shim_host *h, shim_fiber *f) {
  pthread_mutex_lock(&h->mu);
  f->next = NULL;
  if (h->tail != NULL) h->tail->next = f;
  else h->head = f;
  h->tail = f;
  pthread_cond_signal(&h->cv);
  pthread_mutex_unlock(&h->mu);
}

static void *
shim_host_main (void *arg) {
  shim_host *h = (shim_host *) arg;
  shim_fiber *f;
  pthread_setname_np(pthread_self(), "gmapdp-fibers");
  for (;;) {
    pthread_mutex_lock(&h->mu);
    while (h->head == NULL) pthread_cond_wait(&h->cv, &h->mu);
    f = h->head;
    h->head = f->next;
    if (h->head == NULL) h->tail = NULL;
    pthread_mutex_unlock(&h->mu);
    cur_fiber = f;
    swapcontext(&h->ctx, &f->ctx);  /* runs f until it waits for the engine or returns */
    cur_fiber = NULL;
    if (f->finished) {
      munmap(f->stack, SHIM_FIBER_STACK);
      pthread_mutex_lock(&f->jm);
      f->finished = 2;
      pthread_cond_broadcast(&f->jc);
      pthread_mutex_unlock(&f->jm);
    }
  }
  return NULL;
}

static void
shim_fiber_main (unsigned int lo, unsigned int hi) {
  shim_fiber *f = (shim_fiber *) (((uintptr_t) hi << 32) | (uintptr_t) lo);
  f->ret = f->fn(f->arg);
  f->finished = 1;  /* returning resumes the host (uc_link) */
}

int
__wrap_pthread_create (pthread_t *th, const pthread_attr_t *attr, void *(*fn) (void *), void *arg) {
  shim_fiber *f;
  pthread_attr_t da;
  int k;
  if (!shim_fibers_on() || fn == Outbuffer_thread_ordered || fn == Outbuffer_thread_anyorder)
    return __real_pthread_create(th, attr, fn, arg);
  f = (shim_fiber *) calloc(1, sizeof(shim_fiber));
  if (f == NULL) shim_refuse("host memory for a worker fiber (out of memory)");
  f->stack = mmap(NULL, SHIM_FIBER_STACK, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS | MAP_NORESERVE | MAP_STACK,
                  -1, 0);
  if (f->stack == MAP_FAILED) shim_refuse("a worker fiber's stack (mmap)");
  f->fn = fn;
  f->arg = arg;
  pthread_mutex_init(&f->jm, NULL);
  pthread_cond_init(&f->jc, NULL);
  pthread_mutex_lock(&shim_fiber_lock);
  k = shim_nfibers++ % shim_fiber_hosts;
  if (k >= shim_nhosts) {  /* hosts start with their first fiber */
    pthread_t tid;
    pthread_mutex_init(&shim_hosts[k].mu, NULL);
    pthread_cond_init(&shim_hosts[k].cv, NULL);
    pthread_attr_init(&da);
    pthread_attr_setdetachstate(&da, PTHREAD_CREATE_DETACHED);
    if (__real_pthread_create(&tid, &da, shim_host_main, &shim_hosts[k]) != 0)
      shim_refuse("a fiber host thread (pthread_create)");
    pthread_attr_destroy(&da);
    shim_nhosts = k + 1;
  }
  f->host = &shim_hosts[k];
  f->all_next = shim_all_fibers;
  shim_all_fibers = f;
  pthread_mutex_unlock(&shim_fiber_lock);
  getcontext(&f->ctx);
  f->ctx.uc_stack.ss_sp = f->stack;
  f->ctx.uc_stack.ss_size = SHIM_FIBER_STACK;
  f->ctx.uc_link = &f->host->ctx;
  makecontext(&f->ctx, (void (*)(void)) shim_fiber_main, 2, (unsigned int) (uintptr_t) f,
              (unsigned int) ((uintptr_t) f >> 32));
  *th = (pthread_t) f;
  shim_host_ready(f->host, f);
  return 0;
}

int
__wrap_pthread_join (pthread_t th, void **ret) {
  shim_fiber *f;
  pthread_mutex_lock(&shim_fiber_lock);
  for (f = shim_all_fibers; f != NULL && (pthread_t) f != th; f = f->all_next) ;
  pthread_mutex_unlock(&shim_fiber_lock);
  if (f == NULL) return __real_pthread_join(th, ret);
  pthread_mutex_lock(&f->jm);
  while (f->finished != 2) pthread_cond_wait(&f->jc, &f->jm);
  pthread_mutex_unlock(&f->jm);
  if (ret != NULL) *ret = f->ret;
  return 0;
}

/* GMAP's per-thread state (except.c exception stacks, gmap.c's request key) becomes per fiber.  A key past
   the table would fall back to the host thread's slot, which every fiber of that host shares: refused
   instead of mixing the fibers' state silently. */
void *
__wrap_pthread_getspecific (pthread_key_t key) {
  if (cur_fiber != NULL) {
    if (key >= SHIM_NKEYS) shim_refuse("a pthread key past the fibers' key table (GMAPDP_SHIM_FIBERS=0 runs it)");
    return cur_fiber->keys[key];
  }
  return __real_pthread_getspecific(key);
}

int
__wrap_pthread_setspecific (pthread_key_t key, const void *value) {
  if (cur_fiber != NULL) {
    if (key >= SHIM_NKEYS) shim_refuse("a pthread key past the fibers' key table (GMAPDP_SHIM_FIBERS=0 runs it)");
    cur_fiber->keys[key] = (void *) value;
    return 0;
  }
  return __real_pthread_setspecific(key, value);
}

static shim_req **
shim_req_slot (void) {
  return cur_fiber != NULL ? &cur_fiber->req : &tl_req;
}
#define SHIM_OS_THREAD_CREATE __real_pthread_create
#else
static shim_req **
shim_req_slot (void) {
  return &tl_req;
}
#define SHIM_OS_THREAD_CREATE pthread_create
#endif

static void *
shim_grow (void *p, size_t *cap, size_t want, size_t elt) {
  if (want <= *cap && p != NULL) return p;
  want = want < 64 ? 64 : want;
  p = realloc(p, want * elt);
  if (p == NULL) shim_refuse("host memory for a request (out of memory)");
  *cap = want;
  return p;
}

/* the calling thread's request (one outstanding call per thread) */
static shim_req *
shim_request (int kind) {
  shim_req **slot = shim_req_slot();
  shim_req *r = *slot;
  if (r == NULL) {
    r = (shim_req *) calloc(1, sizeof(shim_req));
    if (r == NULL) shim_refuse("host memory for a request (out of memory)");
    pthread_cond_init(&r->cv, NULL);
    pthread_mutex_init(&r->mtx, NULL);
    *slot = r;
  }
  r->kind = kind;
  r->longp = 0;
  r->cost = 0;
  r->q = r->quc = NULL;
  r->qlen = 0;
  r->probs = NULL;
  r->nprobs = 0;
  r->j = NULL;
  r->jlen = 0;
  r->nknown = 0;
  memset(&r->p, 0, sizeof(r->p));
  return r;
}

static void shim_run (shim_req *batch);

static void *
shim_dispatch (void *arg) {
  shim_req *batch, *r, *next;
  const int qi = (int) (intptr_t) arg;
  char name[16];
  shim_qi = qi;
  snprintf(name, sizeof(name), "gmapdp-q%d", qi);
  pthread_setname_np(pthread_self(), name);  /* per-thread CPU accounting (tools/thread_cpu.py) */
  prctl(PR_SET_TIMERSLACK, 2000UL, 0, 0, 0);  /* GMAPDP_SHIM_POLL: short sleeps between completion polls */
  for (;;) {
    pthread_mutex_lock(&q_lock);
    while (q_head[qi] == NULL) pthread_cond_wait(&q_cond[qi], &q_lock);
    batch = q_head[qi];
    q_head[qi] = q_tail[qi] = NULL;
    pthread_mutex_unlock(&q_lock);
    /* one engine batch per genome (requests keep their queue order within a genome) */
    while (batch != NULL) {
      shim_req *same = NULL, **st = &same, *rest = NULL, **rt = &rest;
      Genome_T g = batch->genome;
      for (r = batch; r != NULL; r = next) {
        next = r->next;
        r->next = NULL;
        if (r->genome == g) { *st = r; st = &r->next; }
        else { *rt = r; rt = &r->next; }
      }
      shim_run(same);
      /* wake each caller under its own request's lock: no herd on the queue lock */
      for (r = same; r != NULL; r = next) {
        next = r->next;
#ifdef GMAPDP_SHIM_OWN
        if (r->fiber != NULL) {  /* the caller's fiber runs again (r is its own from here on) */
          r->done = 1;
          shim_host_ready(r->fiber->host, r->fiber);
          continue;
        }
#endif
        pthread_mutex_lock(&r->mtx);
        r->done = 1;
        pthread_cond_signal(&r->cv);
        pthread_mutex_unlock(&r->mtx);
      }
      batch = rest;
    }
  }
  return NULL;
}

/* queue the calling thread's request and sleep until the dispatcher has run it */
static void
shim_submit (shim_req *r) {
  pthread_t th;
  pthread_attr_t attr;
  const char *st;
  int nd, nd2, nl, k;
  int qi;
  pthread_mutex_lock(&q_lock);
  if (!dispatcher_started) {
    st = getenv("GMAPDP_SHIM_STATS");
    if (st != NULL && st[0] == '1') atexit(shim_print_stats);
    st = getenv("GMAPDP_SHIM_TRACE");
    if (st != NULL && st[0] != '\0') shim_trace = fopen(st, "w");
    /* 2 short + 1 long + 2 stage-2 dispatchers, one stream each, on HIP's default 4 hardware queues
       (GPU_MAX_HW_QUEUES): measured end to end, more queues or dispatchers made every batch slower
       (tools/e2e_timing.py --configs, profiles/r03_e2e). */
    st = getenv("GMAPDP_SHIM_DISPATCHERS");
    nd = st != NULL ? atoi(st) : 2;
    if (nd < 1) nd = 1;
    st = getenv("GMAPDP_SHIM_LONG_DISPATCHERS");
    nl = st != NULL ? atoi(st) : 1;
    if (nl < 1) nl = 1;
    st = getenv("GMAPDP_SHIM_STAGE2_DISPATCHERS");
    nd2 = st != NULL ? atoi(st) : 2;
    if (nd2 < 1) nd2 = 1;
    st = getenv("GMAPDP_SHIM_OLIGO_QUEUE");
    if (st != NULL && atoi(st) >= 0 && atoi(st) <= 2) shim_oligo_queue = atoi(st);
    st = getenv("GMAPDP_SHIM_LONG_COST");
    if (st != NULL) shim_long_cost = atol(st);
    pthread_attr_init(&attr);
    pthread_attr_setdetachstate(&attr, PTHREAD_CREATE_DETACHED);
    for (k = 0; k < nd + nl + nd2; k++)
      if (SHIM_OS_THREAD_CREATE(&th, &attr, shim_dispatch, (void *) (intptr_t) (k < nd ? 0 : (k < nd + nl ? 2 : 1))) != 0)
        shim_refuse("a dispatcher thread (pthread_create)");
    pthread_attr_destroy(&attr);
    dispatcher_started = 1;
  }
  qi = r->kind == K_STAGE2 ? 1 : (r->kind == K_OLIGO ? shim_oligo_queue : (r->longp ? 2 : 0));
  r->done = 0;
  r->next = NULL;
#ifdef GMAPDP_SHIM_OWN
  r->fiber = cur_fiber;
#else
  r->fiber = NULL;
#endif
  if (q_tail[qi] != NULL) q_tail[qi]->next = r;
  else q_head[qi] = r;
  q_tail[qi] = r;
  pthread_cond_signal(&q_cond[qi]);
  pthread_mutex_unlock(&q_lock);
#ifdef GMAPDP_SHIM_OWN
  if (r->fiber != NULL) {  /* run the host's next fiber; the dispatcher makes this one runnable again */
    shim_fiber *f = r->fiber;
    swapcontext(&f->ctx, &f->host->ctx);
    return;
  }
#endif
  pthread_mutex_lock(&r->mtx);
  while (!r->done) pthread_cond_wait(&r->cv, &r->mtx);
  pthread_mutex_unlock(&r->mtx);
}

/* dispatcher-owned staging, grown as needed */
typedef struct {
  gmapdp_single_problem *s;
  gmapdp_end_problem *e;
  gmapdp_genome_problem *g;
  gmapdp_cdna_problem *c;
  gmapdp_oligo_problem *o;
  gmapdp_stage2_problem *s2;
  gmapdp_sj_problem *sj;
  gmapdp_sj_result *sjres;
  char *jq;
  size_t sjcap, sjrescap, jqcap;
  uint8_t *kn;
  size_t kncap;
  shim_req **rs, **re, **rg, **rc, **ro, **r2, **rxs, **rxf, **rsj, **rxw;
  size_t scap, ecap, gcap, ccap, ocap, s2cap, rscap, recap, rgcap, rccap, rocap, r2cap, rxscap, rxfcap, rsjcap, rxwcap;
  gmapdp_microexon_problem *mxw;             /* whole calls */
  gmapdp_microexon_result *mxwres;
  gmapdp_pair *mxwpairs;
  size_t mxwcap, mxwrescap, mxwpaircap;
  gmapdp_microexon_problem *mx, *mxf;        /* searches, finishes */
  gmapdp_microexon_result *mxres, *mxfres;
  gmapdp_microexon_candidate *mxc, *mxsc;     /* the finishes' candidates, the searches' candidates */
  double *mxp;
  gmapdp_pair *mxpairs;
  size_t mxcap, mxfcap, mxrescap, mxfrescap, mxccap, mxsccap, mxpcap, mxpaircap;
  char *q, *quc;
  size_t qcap, quccap;
  double *pr;
  size_t prcap;
  gmapdp_result *res;
  gmapdp_genome_result *gres;
  gmapdp_cdna_result *cres;
  gmapdp_oligo_result *ores;
  size_t rescap, grescap, crescap, orescap;
  gmapdp_pair *pairs;
  size_t paircap;
  int32_t *np, *mp, *dg;
  uint32_t *pos;
  size_t npcap, mpcap, poscap, dgcap;
  gmapdp_stage2_result *s2res;
  gmapdp_path *paths;
  gmapdp_path_pair *ppairs;
  size_t s2rescap, pathcap, ppaircap;
} shim_staging;
static __thread shim_staging D;  /* per dispatcher thread */

#define GROW(ptr, cap, want) ((ptr) = shim_grow((ptr), &(cap), (want), sizeof(*(ptr))))

static void
shim_copy_pairs (shim_req *r, const gmapdp_pair *src, int n) {
  if (n > 0) memcpy(r->pairs, src, (size_t) n * sizeof(gmapdp_pair));
}

static void
shim_run (shim_req *batch) {
  shim_req *r;
  size_t ns = 0, ne = 0, ng = 0, nc = 0, no = 0, n2 = 0, nxs = 0, nxf = 0, nsj = 0, nxw = 0, n = 0, qb = 0, pb = 0, cap, i;
  double t0, t1, td[4];
  Genome_T genome = NULL;
  for (r = batch; r != NULL; r = r->next) {
    n++;
    if (genome == NULL) genome = r->genome;  /* shim_dispatch hands over one genome's requests */
    switch (r->kind) {
    case K_SINGLE: GROW(D.rs, D.rscap, ns + 1); D.rs[ns++] = r; break;
    case K_END: GROW(D.re, D.recap, ne + 1); D.re[ne++] = r; break;
    case K_GENOME: GROW(D.rg, D.rgcap, ng + 1); D.rg[ng++] = r; break;
    case K_CDNA: GROW(D.rc, D.rccap, nc + 1); D.rc[nc++] = r; break;
    case K_STAGE2: GROW(D.r2, D.r2cap, n2 + 1); D.r2[n2++] = r; break;
    case K_MXS: GROW(D.rxs, D.rxscap, nxs + 1); D.rxs[nxs++] = r; break;
    case K_MXF: GROW(D.rxf, D.rxfcap, nxf + 1); D.rxf[nxf++] = r; break;
    case K_SJ: GROW(D.rsj, D.rsjcap, nsj + 1); D.rsj[nsj++] = r; break;
    case K_MXW: GROW(D.rxw, D.rxwcap, nxw + 1); D.rxw[nxw++] = r; break;
    default: GROW(D.ro, D.rocap, no + 1); D.ro[no++] = r; break;
    }
  }
  shim_context(genome);
  pthread_mutex_lock(&q_lock);
  shim_batches++;
  shim_batched += n;
  pthread_mutex_unlock(&q_lock);

  /* single, end and genome gaps and the microexon searches / finishes: one round trip over one query
     arena (gmapdp_mixed_batch) */
  t0 = shim_now();
  if (ns + ne + ng + nxs + nxf + nxw > 0) {
    gmapdp_mixed M;
    size_t nct = 0, xcap, wcap;
    int dev_probs = 0;
    int rc;
    memset(&M, 0, sizeof(M));
    qb = 0;
    pb = 0;
    GROW(D.s, D.scap, ns + 1);
    GROW(D.e, D.ecap, ne + 1);
    GROW(D.g, D.gcap, ng + 1);
    GROW(D.mx, D.mxcap, nxs + 1);
    GROW(D.mxf, D.mxfcap, nxf + 1);
    GROW(D.mxres, D.mxrescap, nxs + 1);
    GROW(D.mxfres, D.mxfrescap, nxf + 1);
    for (i = 0; i < ns; i++) qb += D.rs[i]->qlen;
    for (i = 0; i < ne; i++) qb += D.re[i]->qlen;
    size_t kb = 0;
    for (i = 0; i < ng; i++) {
      qb += D.rg[i]->qlen;
      pb += D.rg[i]->nprobs;
      kb += D.rg[i]->nknown;
      dev_probs |= D.rg[i]->probs == NULL;  /* device MaxEnt (every request of a process alike) */
    }
    GROW(D.mxw, D.mxwcap, nxw + 1);
    GROW(D.mxwres, D.mxwrescap, nxw + 1);
    for (i = 0; i < nxw; i++) qb += D.rxw[i]->qlen;
    GROW(D.kn, D.kncap, kb + 1);
    kb = 0;
    for (i = 0; i < nxs; i++) qb += D.rxs[i]->qlen;
    for (i = 0; i < nxf; i++) {
      qb += D.rxf[i]->qlen;
      nct += (size_t) D.rxf[i]->mxr.ncandidates;
    }
    GROW(D.q, D.qcap, qb + 1);
    GROW(D.quc, D.quccap, qb + 1);
    GROW(D.pr, D.prcap, pb + 1);
    GROW(D.mxc, D.mxccap, nct + 1);
    GROW(D.mxp, D.mxpcap, 2 * nct + 2);
    qb = 0;
    pb = 0;
#define STAGE(R, P)                                            \
    do {                                                        \
      (P).qoff = (int32_t) qb;                                  \
      if ((R)->qlen) {                                          \
        memcpy(D.q + qb, (R)->q, (R)->qlen);                    \
        memcpy(D.quc + qb, (R)->quc, (R)->qlen);                \
      }                                                         \
      qb += (R)->qlen;                                          \
    } while (0)
    for (i = 0; i < ns; i++) {
      D.s[i] = D.rs[i]->p.s;
      STAGE(D.rs[i], D.s[i]);
    }
    for (i = 0; i < ne; i++) {
      D.e[i] = D.re[i]->p.e;
      STAGE(D.re[i], D.e[i]);
    }
    for (i = 0; i < ng; i++) {
      D.g[i] = D.rg[i]->p.g;
      STAGE(D.rg[i], D.g[i]);
      D.g[i].prob_offset = (int64_t) pb;
      if (D.rg[i]->nprobs && D.rg[i]->probs) memcpy(D.pr + pb, D.rg[i]->probs, D.rg[i]->nprobs * sizeof(double));
      pb += D.rg[i]->nprobs;
      if (D.rg[i]->nknown) {
        D.g[i].known_offset = (int32_t) kb;
        memcpy(D.kn + kb, D.rg[i]->known, D.rg[i]->nknown);
        kb += D.rg[i]->nknown;
      }
    }
    for (i = 0; i < nxs; i++) {
      D.mx[i] = D.rxs[i]->p.mx;
      STAGE(D.rxs[i], D.mx[i]);
    }
    for (i = 0; i < nxw; i++) {
      D.mxw[i] = D.rxw[i]->p.mx;
      STAGE(D.rxw[i], D.mxw[i]);
    }
    nct = 0;
    for (i = 0; i < nxf; i++) {
      r = D.rxf[i];
      D.mxf[i] = r->p.mx;
      STAGE(r, D.mxf[i]);
      D.mxfres[i] = r->mxr;
      D.mxfres[i].cand_offset = (int64_t) nct;
      if (r->mxr.ncandidates > 0) {
        memcpy(D.mxc + nct, r->mxc, (size_t) r->mxr.ncandidates * sizeof(gmapdp_microexon_candidate));
        memcpy(D.mxp + 2 * nct, r->mxp, 2 * (size_t) r->mxr.ncandidates * sizeof(double));
      }
      nct += (size_t) r->mxr.ncandidates;
    }
#undef STAGE
    cap = gmapdp_single_pair_capacity(D.s, (int) ns) + gmapdp_end_pair_capacity(D.e, (int) ne) +
          gmapdp_genome_pair_capacity(D.g, (int) ng);
    GROW(D.pairs, D.paircap, cap + 1);
    GROW(D.res, D.rescap, ns + ne + 1);
    GROW(D.gres, D.grescap, ng + 1);
    xcap = gmapdp_microexon_pair_capacity(D.mxf, (int) nxf);
    GROW(D.mxpairs, D.mxpaircap, xcap + 1);
    GROW(D.mxsc, D.mxsccap, 8 * nxs + 64);
    wcap = gmapdp_microexon_pair_capacity(D.mxw, (int) nxw);
    GROW(D.mxwpairs, D.mxwpaircap, wcap + 1);
    M.singles = D.s;
    M.nsingle = (int) ns;
    M.ends = D.e;
    M.nend = (int) ne;
    M.genomes = D.g;
    M.ngenome = (int) ng;
    M.splice_probs = dev_probs ? NULL : D.pr;
    M.nprobs = pb;
    M.results = D.res;
    M.genome_results = D.gres;
    M.pairs = D.pairs;
    M.pair_capacity = cap;
    M.searches = D.mx;
    M.nsearch = (int) nxs;
    M.search_results = D.mxres;
    M.finishes = D.mxf;
    M.nfinish = (int) nxf;
    M.finish_candidates = D.mxc;
    M.finish_probs = D.mxp;
    M.nfinish_candidates = nct;
    M.finish_results = D.mxfres;
    M.finish_pairs = D.mxpairs;
    M.finish_pair_capacity = xcap;
    M.candidates = D.mxsc;
    M.candidate_capacity = D.mxsccap;
    M.known_sites = kb ? D.kn : NULL;
    M.nknown = kb;
    M.wholes = D.mxw;
    M.nwhole = (int) nxw;
    M.whole_results = D.mxwres;
    M.whole_pairs = D.mxwpairs;
    M.whole_pair_capacity = wcap;
    rc = gmapdp_mixed_batch(shim_ctx, D.q, D.quc, qb, &M);
    while (rc == GMAPDP_ESPACE) {  /* (rare) the searches found more candidates than D.mxsc holds */
      size_t need = M.candidates_needed;
      GROW(D.mxsc, D.mxsccap, need + 64);
      rc = gmapdp_microexon_search(shim_ctx, D.mx, (int) nxs, D.q, D.quc, qb, D.mxres, D.mxsc, D.mxsccap, &need);
      M.candidates_needed = need;
    }
    shim_check(rc, "gmapdp_mixed_batch");
    for (i = 0; i < ns; i++) {
      r = D.rs[i];
      r->r = D.res[i];
      shim_copy_pairs(r, D.pairs + r->r.pair_offset, r->r.npairs);
      r->r.pair_offset = 0;
    }
    for (i = 0; i < ne; i++) {
      r = D.re[i];
      r->r = D.res[ns + i];
      shim_copy_pairs(r, D.pairs + r->r.pair_offset, r->r.npairs);
      r->r.pair_offset = 0;
    }
    for (i = 0; i < ng; i++) {
      r = D.rg[i];
      r->gr = D.gres[i];
      shim_copy_pairs(r, D.pairs + r->gr.pair_offset, r->gr.npairs);
      r->gr.pair_offset = 0;
    }
    for (i = 0; i < nxs; i++) {
      r = D.rxs[i];
      r->mxr = D.mxres[i];
      GROW(r->mxc, r->mxccap, (size_t) r->mxr.ncandidates + 1);
      if (r->mxr.ncandidates > 0)
        memcpy(r->mxc, D.mxsc + r->mxr.cand_offset, (size_t) r->mxr.ncandidates * sizeof(gmapdp_microexon_candidate));
      r->mxr.cand_offset = 0;
    }
    for (i = 0; i < nxf; i++) {
      r = D.rxf[i];
      r->mxr = D.mxfres[i];
      if (r->mxr.npairs > 0) shim_copy_pairs(r, D.mxpairs + r->mxr.pair_offset, r->mxr.npairs);
      r->mxr.pair_offset = 0;
    }
    for (i = 0; i < nxw; i++) {
      r = D.rxw[i];
      r->mxr = D.mxwres[i];
      if (r->mxr.npairs > 0) shim_copy_pairs(r, D.mxwpairs + r->mxr.pair_offset, r->mxr.npairs);
      r->mxr.pair_offset = 0;
    }
  }
  t1 = shim_now();
  td[0] = t1 - t0;
  /* cDNA gaps (rare): their own batch, each problem's arena span copied whole */
  if (nc > 0) {
    GROW(D.c, D.ccap, nc + 1);
    qb = 0;
    for (i = 0; i < nc; i++) qb += D.rc[i]->qlen;
    GROW(D.q, D.qcap, qb + 1);
    GROW(D.quc, D.quccap, qb + 1);
    qb = 0;
    for (i = 0; i < nc; i++) {
      r = D.rc[i];
      D.c[i] = r->p.c;
      D.c[i].qoffL += (int32_t) qb;
      D.c[i].qoffR += (int32_t) qb;
      memcpy(D.q + qb, r->q, r->qlen);
      memcpy(D.quc + qb, r->quc, r->qlen);
      qb += r->qlen;
    }
    cap = gmapdp_cdna_pair_capacity(D.c, (int) nc);
    GROW(D.pairs, D.paircap, cap + 1);
    GROW(D.cres, D.crescap, nc + 1);
    shim_check(gmapdp_cdna_gap_batch(shim_ctx, D.c, (int) nc, D.q, D.quc, qb, D.cres, D.pairs, cap),
               "gmapdp_cdna_gap_batch");
    for (i = 0; i < nc; i++) {
      r = D.rc[i];
      r->cr = D.cres[i];
      shim_copy_pairs(r, D.pairs + r->cr.pair_offset, r->cr.npairs);
      r->cr.pair_offset = 0;
    }
  }
  /* splice-junction end gaps (known splice sites, -s): their own batch over a query and a junction arena */
  if (nsj > 0) {
    size_t jb = 0;
    GROW(D.sj, D.sjcap, nsj + 1);
    qb = 0;
    for (i = 0; i < nsj; i++) {
      qb += D.rsj[i]->qlen;
      jb += D.rsj[i]->jlen;
    }
    GROW(D.q, D.qcap, qb + 1);
    GROW(D.quc, D.quccap, qb + 1);
    GROW(D.jq, D.jqcap, jb + 1);
    qb = jb = 0;
    for (i = 0; i < nsj; i++) {
      r = D.rsj[i];
      D.sj[i] = r->p.sj;
      D.sj[i].qoff = (int32_t) qb;
      D.sj[i].joff = (int32_t) jb;
      if (r->qlen) {
        memcpy(D.q + qb, r->q, r->qlen);
        memcpy(D.quc + qb, r->quc, r->qlen);
      }
      if (r->jlen) memcpy(D.jq + jb, r->j, r->jlen);
      qb += r->qlen;
      jb += r->jlen;
    }
    cap = gmapdp_sj_pair_capacity(D.sj, (int) nsj);
    GROW(D.pairs, D.paircap, cap + 1);
    GROW(D.sjres, D.sjrescap, nsj + 1);
    shim_check(gmapdp_end_splicejunction_batch(shim_ctx, D.sj, (int) nsj, D.q, D.quc, qb, D.jq, jb, D.sjres,
                                               D.pairs, cap), "gmapdp_end_splicejunction_batch");
    for (i = 0; i < nsj; i++) {
      r = D.rsj[i];
      r->sjr = D.sjres[i];
      shim_copy_pairs(r, D.pairs + r->sjr.pair_offset, r->sjr.npairs);
      r->sjr.pair_offset = 0;
    }
  }

  t0 = shim_now();
  td[1] = t0 - t1;
  /* stage-2 seeding */
  if (no > 0) {
    size_t pc, dc;
    GROW(D.o, D.ocap, no + 1);
    qb = 0;
    for (i = 0; i < no; i++) qb += D.ro[i]->qlen;
    GROW(D.quc, D.quccap, qb + 1);
    qb = 0;
    for (i = 0; i < no; i++) {
      r = D.ro[i];
      D.o[i] = r->p.o;
      D.o[i].qoff = (int32_t) qb;
      memcpy(D.quc + qb, r->quc, r->qlen);
      qb += r->qlen;
    }
    pc = gmapdp_oligo_positions_capacity(D.o, (int) no);
    dc = gmapdp_oligo_diagonal_capacity(D.o, (int) no);
    GROW(D.np, D.npcap, qb + 1);
    GROW(D.mp, D.mpcap, qb + 1);
    GROW(D.pos, D.poscap, pc + 1);
    GROW(D.dg, D.dgcap, 4 * dc + 4);
    GROW(D.ores, D.orescap, no + 1);
    shim_check(gmapdp_oligo_mappings_batch(shim_ctx, D.o, (int) no, D.quc, qb, D.ores, D.np, D.mp, D.pos, pc, D.dg,
                                           dc), "gmapdp_oligo_mappings_batch");
    for (i = 0; i < no; i++) {
      size_t q, ql;
      r = D.ro[i];
      r->orr = D.ores[i];
      ql = r->qlen;
      for (q = 0; q < ql; q++) {
        r->np[q] = D.np[D.o[i].qoff + q];
        r->mp[q] = r->np[q] > 0 ? D.mp[D.o[i].qoff + q] - (int32_t) r->orr.table_offset : -1;
      }
      if (r->tabn) memcpy(r->pos, D.pos + r->orr.table_offset, r->tabn * sizeof(uint32_t));
      if (r->orr.ndiagonals > 0)
        memcpy(r->dg, D.dg + 4 * r->orr.diag_offset, 4 * (size_t) r->orr.ndiagonals * sizeof(int32_t));
      r->orr.table_offset = 0;
      r->orr.diag_offset = 0;
    }
  }
  t1 = shim_now();
  td[2] = t1 - t0;
  /* Stage2_compute: seeding and chaining in one batch */
  if (n2 > 0) {
    size_t pneed = 0, qneed = 0, k;
    int rc;
    GROW(D.s2, D.s2cap, n2 + 1);
    qb = 0;
    for (i = 0; i < n2; i++) qb += D.r2[i]->qlen;
    GROW(D.q, D.qcap, qb + 1);
    GROW(D.quc, D.quccap, qb + 1);
    qb = 0;
    for (i = 0; i < n2; i++) {
      r = D.r2[i];
      D.s2[i] = r->p.s2;
      D.s2[i].qoff = (int32_t) qb;
      memcpy(D.q + qb, r->q, r->qlen);
      memcpy(D.quc + qb, r->quc, r->qlen);
      qb += r->qlen;
    }
    GROW(D.s2res, D.s2rescap, n2 + 1);
    GROW(D.paths, D.pathcap, 4 * n2 + 16);
    GROW(D.ppairs, D.ppaircap, 3 * qb + 64);
    for (;;) {
      rc = gmapdp_stage2_batch(shim_ctx, D.s2, (int) n2, D.q, D.quc, qb, D.s2res, D.paths, D.pathcap, D.ppairs,
                               D.ppaircap, &pneed, &qneed);
      if (rc != GMAPDP_ESPACE) break;
      GROW(D.paths, D.pathcap, pneed + 16);
      GROW(D.ppairs, D.ppaircap, qneed + 64);
    }
    shim_check(rc, "gmapdp_stage2_batch");
    for (i = 0; i < n2; i++) {
      gmapdp_stage2_result *res = &D.s2res[i];
      size_t npairs = 0;
      r = D.r2[i];
      r->s2r = *res;
      GROW(r->s2paths, r->s2pathcap, (size_t) res->nresults + 1);
      GROW(r->s2pairs, r->s2paircap, (size_t) res->npairs + 1);
      for (k = 0; k < (size_t) res->nresults; k++) {
        const gmapdp_path *pa = &D.paths[res->path_offset + k];
        memcpy(r->s2pairs + npairs, D.ppairs + pa->pair_offset, (size_t) pa->npairs * sizeof(gmapdp_path_pair));
        r->s2paths[k] = *pa;
        r->s2paths[k].pair_offset = (int64_t) npairs;
        npairs += (size_t) pa->npairs;
      }
      r->s2r.path_offset = 0;
    }
  }
  td[3] = shim_now() - t1;
  pthread_mutex_lock(&q_lock);
  for (i = 0; i < 4; i++) shim_secs[i] += td[i];
  if (shim_trace != NULL) {  /* GMAPDP_SHIM_TRACE=<file>: one line per dispatcher batch */
    int gmax = 0, mk = -1, mr = 0, mg = 0;
    long mc = -1;
    for (i = 0; i < ns; i++) gmax = D.s[i].glength > gmax ? D.s[i].glength : gmax;
    for (i = 0; i < ne; i++) gmax = D.e[i].glength > gmax ? D.e[i].glength : gmax;
    for (i = 0; i < ng; i++) gmax = D.g[i].glengthL > gmax ? D.g[i].glengthL : gmax;
    for (r = batch; r != NULL; r = r->next)  /* the costliest fill: kind, rlength, glength, cost */
      if (r->cost > mc && r->kind <= K_GENOME) {
        mc = r->cost;
        mk = r->kind;
        mr = r->kind == K_SINGLE ? r->p.s.rlength : (r->kind == K_END ? r->p.e.rlength : r->p.g.rlength);
        mg = r->kind == K_SINGLE ? r->p.s.glength : (r->kind == K_END ? r->p.e.glength : r->p.g.glengthL);
      }
    fprintf(shim_trace, "%d %.6f %zu %zu %zu %zu %zu %zu %zu %d %.6f %.6f %.6f %.6f %d %d %d %ld\n", shim_qi, shim_now(),
            ns, ne, ng, nc, nxs, nxf, n2, gmax, td[0], td[1], td[2], td[3], mk, mr, mg, mc);
  }
  pthread_mutex_unlock(&q_lock);
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
GMAPDP_DYNPROG_ENTRY(Dynprog_single_gap) (int *dynprogindex, int *finalscore, int *nmatches, int *nmismatches, int *nopens,
                           int *nindels, Dynprog_T dynprog, char *sequence1, char *sequenceuc1, int length1,
                           int length2, int offset1, int offset2, Univcoord_T chroffset, Univcoord_T chrhigh,
                           bool watsonp, int genestrand, bool jump_late_p, Genome_T genome, Genome_T genomealt,
                           Pairpool_T pairpool, int extraband_single, bool widebandp, double defect_rate) {
  shim_req *r;
  gmapdp_single_problem *p;
  List_T list;
  if (shim_homopolymerp) shim_refuse("homopolymer mode (Dynprog_single_setup homopolymerp)");
  shim_check_call(genome, genomealt, dynprog);
  r = shim_request(K_SINGLE);
  p = &r->p.s;
  p->rlength = length1;
  p->glength = length2;
  p->roffset = offset1;
  p->goffset = offset2;
  p->chroffset = shim_coord(chroffset);
  p->chrhigh = shim_coord(chrhigh);
  p->flags = (watsonp ? GMAPDP_WATSON : 0) | (jump_late_p ? GMAPDP_JUMP_LATE : 0) | (widebandp ? GMAPDP_WIDEBAND : 0) |
             SHIM_SIMD;
  p->genestrand = genestrand;
  p->extraband = extraband_single;
  p->defect_rate = defect_rate;
  p->dynprogindex = *dynprogindex;
  r->genome = genome;
  r->q = sequence1;
  r->quc = sequenceuc1;
  r->qlen = length1 > 0 ? (size_t) length1 : 0;
  /* a call past the size guard (dynprog_single.c:509-521) is answered without a fill */
  r->cost = length1 > GMAPDP_MAX_RLENGTH || length2 > GMAPDP_MAX_GLENGTH ? 0 : shim_cost(length1, length2, extraband_single);
  r->longp = r->cost > shim_long_cost;
  GROW(r->pairs, r->pcap, gmapdp_single_pair_capacity(p, 1) + 1);
  shim_submit(r);
  shim_count(ST_SINGLE);
  list = shim_list(r->pairs, r->r.npairs, p->dynprogindex, -1, 0, 0, 0.0, 0.0, pairpool);
  *dynprogindex = r->r.dynprogindex;
  *finalscore = r->r.traceback_score;
  *nmatches = r->r.nmatches;
  *nmismatches = r->r.nmismatches;
  *nopens = r->r.nopens;
  *nindels = r->r.nindels;
  return list;
}

static List_T
shim_end_gap (int end3p, int *dynprogindex, int *finalscore, int *nmatches, int *nmismatches, int *nopens,
              int *nindels, Dynprog_T dynprog, char *seq, char *sequc, int length1, int length2, int offset1,
              int offset2, Univcoord_T chroffset, Univcoord_T chrhigh, bool watsonp, int genestrand,
              bool jump_late_p, Genome_T genome, Genome_T genomealt, Pairpool_T pairpool, int extraband_end,
              double defect_rate, Endalign_T endalign, bool require_pos_score_p) {
  shim_req *r;
  gmapdp_end_problem *p;
  List_T list;
  shim_check_call(genome, genomealt, dynprog);
  r = shim_request(K_END);
  p = &r->p.e;
  p->rlength = length1;
  p->glength = length2;
  p->roffset = offset1;
  p->goffset = offset2;
  p->chroffset = shim_coord(chroffset);
  p->chrhigh = shim_coord(chrhigh);
  p->flags = (watsonp ? GMAPDP_WATSON : 0) | (jump_late_p ? GMAPDP_JUMP_LATE : 0) | SHIM_SIMD;
  p->genestrand = genestrand;
  p->extraband = extraband_end;
  p->end3p = end3p;
  p->endalign = (int32_t) endalign;
  p->require_pos_score_p = require_pos_score_p ? 1 : 0;
  p->dynprogindex = *dynprogindex;
  p->defect_rate = defect_rate;
  /* end5's revsequence points at the LAST character of the slice (dynprog_end.c:1294) */
  r->genome = genome;
  r->q = (end3p || length1 <= 0) ? seq : seq - (length1 - 1);
  r->quc = (end3p || length1 <= 0) ? sequc : sequc - (length1 - 1);
  r->qlen = length1 > 0 ? (size_t) length1 : 0;
  r->cost = shim_cost(length1 > 660 ? 660 : length1, length2, extraband_end);
  r->longp = r->cost > shim_long_cost;
  GROW(r->pairs, r->pcap, gmapdp_end_pair_capacity(p, 1) + 1);
  shim_submit(r);
  shim_count(end3p ? ST_END3 : ST_END5);
  list = shim_list(r->pairs, r->r.npairs, p->dynprogindex, -1, 0, 0, 0.0, 0.0, pairpool);
  *dynprogindex = r->r.dynprogindex;
  *finalscore = r->r.traceback_score;
  *nmatches = r->r.nmatches;
  *nmismatches = r->r.nmismatches;
  *nopens = r->r.nopens;
  *nindels = r->r.nindels;
  return list;
}

List_T
GMAPDP_DYNPROG_ENTRY(Dynprog_end5_gap) (int *dynprogindex, int *finalscore, int *nmatches, int *nmismatches, int *nopens,
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
GMAPDP_DYNPROG_ENTRY(Dynprog_end3_gap) (int *dynprogindex, int *finalscore, int *nmatches, int *nmismatches, int *nopens,
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

/* ---- known splice sites (-s): Dynprog_end5/3_splicejunction, Dynprog_end5/3_known ---- */

/* The engine's records -> the reference's List_T; the gap holder at known_index is the known splice
   (Pairpool_push_gapholder with knownp, dynprog_end.c:1888/2484), other gap holders are not. */
static List_T
shim_list_known (const gmapdp_pair *pairs, int n, int dynprogindex, int known_index, Pairpool_T pairpool) {
  List_T list = NULL;
  int i;
  for (i = n - 1; i >= 0; i--) {
    const gmapdp_pair *p = &pairs[i];
    if (p->querypos == -1 && p->genomepos == -1)
      list = Pairpool_push_gapholder(list, pairpool, /*queryjump*/0, p->jump, /*leftpair*/NULL, /*rightpair*/NULL,
                                     /*knownp*/i == known_index);
    else
      list = Pairpool_push(list, pairpool, p->querypos, p->genomepos, p->cdna, p->comp, p->genome, p->genomealt,
                           dynprogindex);
  }
  return list;
}

/* Dynprog_end5_splicejunction (end3p 0) / Dynprog_end3_splicejunction (end3p 1): one request on the DP
   queue; the junction string travels with the query (gmapdp_end_splicejunction_batch). */
static List_T
shim_splicejunction (int end3p, int *dynprogindex, int *finalscore, int *missscore, int *nmatches, int *nmismatches,
                     int *nopens, int *nindels, Dynprog_T dynprog, char *seq, char *sequc, char *gseq, char *gseq_alt,
                     int length1, int length2, int offset1, int offset2_anchor, int offset2_far, int genestrand,
                     bool jump_late_p, Genome_T genome, Genome_T genomealt, Pairpool_T pairpool, int extraband_end,
                     double defect_rate, int contlength) {
  shim_req *r;
  gmapdp_sj_problem *p;
  List_T list;
  const int inside = length1 > 0 && length1 <= GMAPDP_MAX_RLENGTH && length2 > 0 && length2 <= GMAPDP_MAX_GLENGTH;
  shim_check_call(genome, genomealt, dynprog);
  /* end5's rev pointers are the slices' LAST characters (dynprog_end.c:1653) */
  const char *q = (end3p || !inside) ? seq : seq - (length1 - 1);
  const char *quc = (end3p || !inside) ? sequc : sequc - (length1 - 1);
  const char *j = (end3p || !inside) ? gseq : gseq - (length2 - 1);
  const char *j_alt = (end3p || !inside) ? gseq_alt : gseq_alt - (length2 - 1);
  if (inside && gseq_alt != NULL && j_alt != j && memcmp(j_alt, j, (size_t) length2) != 0)
    shim_refuse("a splice junction whose alternate-allele string differs (genomealt)");
  r = shim_request(K_SJ);
  p = &r->p.sj;
  p->rlength = length1;
  p->glength = length2;
  p->roffset = offset1;
  p->goffset_anchor = offset2_anchor;
  p->goffset_far = offset2_far;
  p->contlength = contlength;
  p->flags = (jump_late_p ? GMAPDP_JUMP_LATE : 0) | SHIM_SIMD;
  p->genestrand = genestrand;
  p->extraband = extraband_end;
  p->end3p = end3p;
  p->dynprogindex = *dynprogindex;
  p->defect_rate = defect_rate;
  r->genome = genome;
  r->q = q;
  r->quc = quc;
  r->qlen = inside ? (size_t) length1 : 0;
  r->j = j;
  r->jlen = inside ? (size_t) length2 : 0;
  r->cost = inside ? shim_cost(length1, length2, extraband_end) : 0;
  r->longp = r->cost > shim_long_cost;
  GROW(r->pairs, r->pcap, gmapdp_sj_pair_capacity(p, 1) + 1);
  shim_submit(r);
  shim_count(end3p ? ST_SJ3 : ST_SJ5);
  list = shim_list_known(r->pairs, r->sjr.npairs, p->dynprogindex, r->sjr.known_index, pairpool);
  /* a negative best endpoint leaves every out-parameter as it was (dynprog_end.c:1798-1800) */
  *dynprogindex = r->sjr.dynprogindex;
  if (r->sjr.traceback_score != GMAPDP_UNSET) *finalscore = r->sjr.traceback_score;
  if (r->sjr.missscore != GMAPDP_UNSET) *missscore = r->sjr.missscore;
  if (r->sjr.nmatches != GMAPDP_UNSET) *nmatches = r->sjr.nmatches;
  if (r->sjr.nmismatches != GMAPDP_UNSET) *nmismatches = r->sjr.nmismatches;
  if (r->sjr.nopens != GMAPDP_UNSET) *nopens = r->sjr.nopens;
  if (r->sjr.nindels != GMAPDP_UNSET) *nindels = r->sjr.nindels;
  return list;
}

List_T
GMAPDP_DYNPROG_ENTRY(Dynprog_end5_splicejunction) (int *dynprogindex, int *finalscore, int *missscore, int *nmatches,
                                    int *nmismatches, int *nopens, int *nindels, Dynprog_T dynprog,
                                    char *rev_rsequence, char *rev_rsequenceuc, char *rev_gsequence,
                                    char *rev_gsequence_alt, int length1, int length2, int revoffset1,
                                    int revoffset2_anchor, int revoffset2_far, Univcoord_T chroffset,
                                    Univcoord_T chrhigh, bool watsonp, int genestrand, bool jump_late_p,
                                    Genome_T genome, Genome_T genomealt, Pairpool_T pairpool, int extraband_end,
                                    double defect_rate, int contlength) {
  (void) chroffset;  /* genome skips take their characters from the junction string */
  (void) chrhigh;
  (void) watsonp;
  return shim_splicejunction(0, dynprogindex, finalscore, missscore, nmatches, nmismatches, nopens, nindels, dynprog,
                             rev_rsequence, rev_rsequenceuc, rev_gsequence, rev_gsequence_alt, length1, length2,
                             revoffset1, revoffset2_anchor, revoffset2_far, genestrand, jump_late_p, genome, genomealt,
                             pairpool, extraband_end, defect_rate, contlength);
}

List_T
GMAPDP_DYNPROG_ENTRY(Dynprog_end3_splicejunction) (int *dynprogindex, int *finalscore, int *missscore, int *nmatches,
                                    int *nmismatches, int *nopens, int *nindels, Dynprog_T dynprog, char *rsequence,
                                    char *rsequenceuc, char *gsequence, char *gsequence_alt, int length1,
                                    int length2, int offset1, int offset2_anchor, int offset2_far,
                                    Univcoord_T chroffset, Univcoord_T chrhigh, bool watsonp, int genestrand,
                                    bool jump_late_p, Genome_T genome, Genome_T genomealt, Pairpool_T pairpool,
                                    int extraband_end, double defect_rate, int contlength) {
  (void) chroffset;
  (void) chrhigh;
  (void) watsonp;
  return shim_splicejunction(1, dynprogindex, finalscore, missscore, nmatches, nmismatches, nopens, nindels, dynprog,
                             rsequence, rsequenceuc, gsequence, gsequence_alt, length1, length2, offset1,
                             offset2_anchor, offset2_far, genestrand, jump_late_p, genome, genomealt, pairpool,
                             extraband_end, defect_rate, contlength);
}

/* binary_search (dynprog_end.c:2722): the first site at or above goal in positions[lowi, highi) */
static int
shim_site_search (int lowi, int highi, const Univcoord_T *positions, Univcoord_T goal) {
  int middlei;
  while (lowi < highi) {
    middlei = lowi + ((highi - lowi) / 2);
    if (goal < positions[middlei]) highi = middlei;
    else if (goal > positions[middlei]) lowi = middlei + 1;
    else return middlei;
  }
  return highi;
}

static const char shim_compl[128] = COMPLEMENT_LC;

/* make_complement_inplace (dynprog_end.c:2501) */
static void
shim_revcomp_inplace (char *s, int length) {
  int i, k;
  char t;
  for (i = 0, k = length - 1; i < k; i++, k--) {
    t = shim_compl[(int) s[i]];
    s[i] = shim_compl[(int) s[k]];
    s[k] = t;
  }
  if (i == k) s[i] = shim_compl[(int) s[i]];
}

/* make_contjunction_5 / _3 (dynprog_end.c:2519 / 2620): the contlength characters next to the anchor
   site, at the junction's end (5') or start (3'), reverse-complemented on the minus strand */
static void
shim_contjunction (int end3p, char *sj, char *sj_alt, Univcoord_T splicecoord, int splicelength, int contlength,
                   Splicetype_T anchor_splicetype, Genome_T genome, Genome_T genomealt, bool watsonp) {
  char *prox = end3p ? sj : sj + splicelength, *prox_alt = end3p ? sj_alt : sj_alt + splicelength;
  int before;  /* the piece ends at the site (else starts there) */
  if (anchor_splicetype == ACCEPTOR || anchor_splicetype == ANTIDONOR) before = 0;
  else if (anchor_splicetype == ANTIACCEPTOR || anchor_splicetype == DONOR) before = 1;
  else shim_refuse("an unexpected anchor splice type");
  Genome_fill_buffer_blocks_noterm(genome, genomealt, before ? splicecoord - contlength : splicecoord,
                                   (Chrpos_T) contlength, prox, prox_alt);
  if (watsonp == false) {
    shim_revcomp_inplace(prox, contlength);
    shim_revcomp_inplace(prox_alt, contlength);
  }
}

/* Dynprog_end5_known (end3p 0, dynprog_end.c:2748-3005) / Dynprog_end3_known (end3p 1, :3009-3266):
   restated over the engine.  The straight end gap (QUERYEND_NOGAPS, then BEST_LOCAL when no splice wins)
   runs through the engine's Dynprog_end5/3_gap; every anchor site of the right type in the read end's
   span builds its half of the junction and hands it to the reference's Splicetrie_solve_end5/3
   (splicetrie.c, the trie walk over the far sites), whose Dynprog_end5/3_splicejunction calls land on
   the engine through the wraps above. */
static List_T
shim_known (int end3p, bool *knownsplicep, int *dynprogindex, int *finalscore, int *ambig_end_length,
            Splicetype_T *ambig_splicetype, int *nmatches, int *nmismatches, int *nopens, int *nindels,
            Dynprog_T dynprog, char *seq, char *sequc, int rlength, int glength, int roffset, int goffset,
            int querylength, Univcoord_T chroffset, Univcoord_T chrhigh, Univcoord_T knownsplice_limit_low,
            Univcoord_T knownsplice_limit_high, int cdna_direction, bool watsonp, int genestrand, bool jump_late_p,
            Genome_T genome, Genome_T genomealt, Pairpool_T pairpool, int extraband_end, double defect_rate) {
  List_T best_pairs = NULL, orig_pairs;
  Pair_T pair;
  Univcoord_T low, high, far_limit_low, far_limit_high;
  Splicetype_T anchor_splicetype = DONOR, far_splicetype = DONOR;
  int contlength, splicelength, j, orig_score, threshold_miss_score, perfect_score, obsmax_penalty;
  char *sj, *sj_alt;

  shim_count(end3p ? ST_KNOWN3 : ST_KNOWN5);
  *ambig_end_length = 0;
  if (rlength <= 0 || glength <= 0) {
    *finalscore = 0;
    *knownsplicep = false;
    return (List_T) NULL;
  }
  perfect_score = rlength * FULLMATCH;

  /* without splicing, all the way to the query end */
  best_pairs = end3p ? GMAPDP_DYNPROG_ENTRY(Dynprog_end3_gap)(dynprogindex, finalscore, nmatches, nmismatches, nopens, nindels,
                                               dynprog, seq, sequc, rlength, glength, roffset, goffset, chroffset,
                                               chrhigh, watsonp, genestrand, jump_late_p, genome, genomealt,
                                               pairpool, extraband_end, defect_rate, QUERYEND_NOGAPS, true)
                     : GMAPDP_DYNPROG_ENTRY(Dynprog_end5_gap)(dynprogindex, finalscore, nmatches, nmismatches, nopens, nindels,
                                               dynprog, seq, sequc, rlength, glength, roffset, goffset, chroffset,
                                               chrhigh, watsonp, genestrand, jump_late_p, genome, genomealt,
                                               pairpool, extraband_end, defect_rate, QUERYEND_NOGAPS, true);
  if (*finalscore <= 0) {
    orig_score = 0;
    orig_pairs = best_pairs = (List_T) NULL;
  } else {
    orig_score = *finalscore;
    orig_pairs = best_pairs;
  }
  threshold_miss_score = orig_score - perfect_score;
  if (threshold_miss_score < -2 * FULLMATCH) threshold_miss_score = -2 * FULLMATCH;  /* <= 2 mismatches */
  *knownsplicep = false;

  if (threshold_miss_score < 0 && glength > 0) {
    sj = (char *) malloc((size_t) glength + 1);
    sj_alt = (char *) malloc((size_t) glength + 1);
    if (sj == NULL || sj_alt == NULL) shim_refuse("host memory for a splice junction (out of memory)");
    if (!end3p) {
      if (watsonp == true) {
        low = chroffset + goffset - rlength + 2;
        high = chroffset + goffset + 1;
        anchor_splicetype = cdna_direction > 0 ? ACCEPTOR : ANTIDONOR;
        far_splicetype = cdna_direction > 0 ? DONOR : ANTIACCEPTOR;
      } else {
        low = chrhigh - goffset;
        high = chrhigh - (goffset - rlength) - 1;
        anchor_splicetype = cdna_direction > 0 ? ANTIACCEPTOR : DONOR;
        far_splicetype = cdna_direction > 0 ? ANTIDONOR : ACCEPTOR;
      }
    } else {
      if (watsonp == true) {
        low = chroffset + goffset;
        high = chroffset + goffset + rlength - 1;
        anchor_splicetype = cdna_direction > 0 ? DONOR : ANTIACCEPTOR;
        far_splicetype = cdna_direction > 0 ? ACCEPTOR : ANTIDONOR;
      } else {
        low = chrhigh - (goffset + rlength) + 2;
        high = chrhigh - goffset + 1;
        anchor_splicetype = cdna_direction > 0 ? ANTIDONOR : ACCEPTOR;
        far_splicetype = cdna_direction > 0 ? ANTIACCEPTOR : DONOR;
      }
    }
    far_limit_low = knownsplice_limit_low;
    far_limit_high = knownsplice_limit_high;
    j = shim_site_search(0, shim_nsplicesites, shim_splicesites, low);
    while (j < shim_nsplicesites && shim_splicesites[j] <= high) {
      if (shim_splicetypes[j] == anchor_splicetype) {
        /* 5': the anchor piece runs from the site to the read end's genomic end; 3': from its start */
        if (!end3p) contlength = watsonp ? (int) (high - shim_splicesites[j]) : (int) (shim_splicesites[j] - low);
        else contlength = watsonp ? (int) (shim_splicesites[j] - low) : (int) (high - shim_splicesites[j]);
        splicelength = glength - contlength;
        shim_contjunction(end3p, sj, sj_alt, shim_splicesites[j], splicelength, contlength, anchor_splicetype, genome,
                          genomealt, watsonp);
        if (watsonp == (end3p ? true : false)) far_limit_low = shim_splicesites[j];  /* 3' watson / 5' crick */
        else far_limit_high = shim_splicesites[j];                                  /* 5' watson / 3' crick */
        obsmax_penalty = 0;
        if (shim_trieoffsets_obs != NULL) {
          best_pairs = end3p
              ? Splicetrie_solve_end3(best_pairs, shim_triecontents_obs, shim_trieoffsets_obs, j, far_limit_low,
                                      far_limit_high, finalscore, nmatches, nmismatches, nopens, nindels, knownsplicep,
                                      ambig_end_length, &threshold_miss_score, /*obsmax_penalty*/0, perfect_score,
                                      shim_splicesites[j], sj, sj_alt, splicelength, contlength, far_splicetype,
                                      chroffset, chrhigh, dynprogindex, dynprog, seq, sequc, rlength, glength, roffset,
                                      goffset, cdna_direction, watsonp, genestrand, jump_late_p, genome, genomealt,
                                      pairpool, extraband_end, defect_rate)
              : Splicetrie_solve_end5(best_pairs, shim_triecontents_obs, shim_trieoffsets_obs, j, far_limit_low,
                                      far_limit_high, finalscore, nmatches, nmismatches, nopens, nindels, knownsplicep,
                                      ambig_end_length, &threshold_miss_score, /*obsmax_penalty*/0, perfect_score,
                                      shim_splicesites[j], sj, sj_alt, splicelength, contlength, far_splicetype,
                                      chroffset, chrhigh, dynprogindex, dynprog, seq, sequc, rlength, glength, roffset,
                                      goffset, cdna_direction, watsonp, genestrand, jump_late_p, genome, genomealt,
                                      pairpool, extraband_end, defect_rate);
          obsmax_penalty += FULLMATCH;
        }
        if (threshold_miss_score + obsmax_penalty < 0 && shim_trieoffsets_max != NULL) {
          best_pairs = end3p
              ? Splicetrie_solve_end3(best_pairs, shim_triecontents_max, shim_trieoffsets_max, j, far_limit_low,
                                      far_limit_high, finalscore, nmatches, nmismatches, nopens, nindels, knownsplicep,
                                      ambig_end_length, &threshold_miss_score, obsmax_penalty, perfect_score,
                                      shim_splicesites[j], sj, sj_alt, splicelength, contlength, far_splicetype,
                                      chroffset, chrhigh, dynprogindex, dynprog, seq, sequc, rlength, glength, roffset,
                                      goffset, cdna_direction, watsonp, genestrand, jump_late_p, genome, genomealt,
                                      pairpool, extraband_end, defect_rate)
              : Splicetrie_solve_end5(best_pairs, shim_triecontents_max, shim_trieoffsets_max, j, far_limit_low,
                                      far_limit_high, finalscore, nmatches, nmismatches, nopens, nindels, knownsplicep,
                                      ambig_end_length, &threshold_miss_score, obsmax_penalty, perfect_score,
                                      shim_splicesites[j], sj, sj_alt, splicelength, contlength, far_splicetype,
                                      chroffset, chrhigh, dynprogindex, dynprog, seq, sequc, rlength, glength, roffset,
                                      goffset, cdna_direction, watsonp, genestrand, jump_late_p, genome, genomealt,
                                      pairpool, extraband_end, defect_rate);
        }
      }
      j++;
    }
    free(sj_alt);
    free(sj);
  }

  if (best_pairs == NULL) {
    if (*ambig_end_length == 0) {
      /* not to the query end this time: the best local end (chopped to the Dynprog_T's limits) */
      if (rlength > dynprog->max_rlength) rlength = dynprog->max_rlength;
      if (glength > dynprog->max_glength) glength = dynprog->max_glength;
      orig_pairs = end3p ? GMAPDP_DYNPROG_ENTRY(Dynprog_end3_gap)(dynprogindex, finalscore, nmatches, nmismatches, nopens, nindels,
                                                   dynprog, seq, sequc, rlength, glength, roffset, goffset, chroffset,
                                                   chrhigh, watsonp, genestrand, jump_late_p, genome, genomealt,
                                                   pairpool, extraband_end, defect_rate, BEST_LOCAL, false)
                         : GMAPDP_DYNPROG_ENTRY(Dynprog_end5_gap)(dynprogindex, finalscore, nmatches, nmismatches, nopens, nindels,
                                                   dynprog, seq, sequc, rlength, glength, roffset, goffset, chroffset,
                                                   chrhigh, watsonp, genestrand, jump_late_p, genome, genomealt,
                                                   pairpool, extraband_end, defect_rate, BEST_LOCAL, false);
      *knownsplicep = false;
      return orig_pairs;
    }
    /* an ambiguous splice: the straight alignment truncated before the ambiguous part */
    *ambig_splicetype = anchor_splicetype;
    if (!end3p) {
      orig_pairs = List_reverse(orig_pairs);  /* querypos is decreasing */
      while (orig_pairs != NULL && ((Pair_T) orig_pairs->first)->querypos < *ambig_end_length)
        orig_pairs = Pairpool_pop(orig_pairs, &pair);
      orig_pairs = List_reverse(orig_pairs);
    } else {
      while (orig_pairs != NULL && ((Pair_T) orig_pairs->first)->querypos >= querylength - *ambig_end_length)
        orig_pairs = Pairpool_pop(orig_pairs, &pair);
    }
    *knownsplicep = false;
    *finalscore = orig_score;
    return orig_pairs;
  }
  *ambig_end_length = 0;
  if (*knownsplicep == true) return end3p ? Pair_protect_end3(best_pairs) : Pair_protect_end5(best_pairs);
  return best_pairs;
}

List_T
GMAPDP_DYNPROG_ENTRY(Dynprog_end5_known) (bool *knownsplicep, int *dynprogindex, int *finalscore, int *ambig_end_length,
                           Splicetype_T *ambig_splicetype, int *nmatches, int *nmismatches, int *nopens, int *nindels,
                           Dynprog_T dynprog, char *revsequence1, char *revsequenceuc1, int length1, int length2,
                           int revoffset1, int revoffset2, Univcoord_T chroffset, Univcoord_T chrhigh,
                           Univcoord_T knownsplice_limit_low, Univcoord_T knownsplice_limit_high, int cdna_direction,
                           bool watsonp, int genestrand, bool jump_late_p, Genome_T genome, Genome_T genomealt,
                           Pairpool_T pairpool, int extraband_end, double defect_rate) {
  return shim_known(0, knownsplicep, dynprogindex, finalscore, ambig_end_length, ambig_splicetype, nmatches,
                    nmismatches, nopens, nindels, dynprog, revsequence1, revsequenceuc1, length1, length2, revoffset1,
                    revoffset2, /*querylength*/0, chroffset, chrhigh, knownsplice_limit_low, knownsplice_limit_high,
                    cdna_direction, watsonp, genestrand, jump_late_p, genome, genomealt, pairpool, extraband_end,
                    defect_rate);
}

List_T
GMAPDP_DYNPROG_ENTRY(Dynprog_end3_known) (bool *knownsplicep, int *dynprogindex, int *finalscore, int *ambig_end_length,
                           Splicetype_T *ambig_splicetype, int *nmatches, int *nmismatches, int *nopens, int *nindels,
                           Dynprog_T dynprog, char *sequence1, char *sequenceuc1, int length1, int length2, int offset1,
                           int offset2, int querylength, Univcoord_T chroffset, Univcoord_T chrhigh,
                           Univcoord_T knownsplice_limit_low, Univcoord_T knownsplice_limit_high, int cdna_direction,
                           bool watsonp, int genestrand, bool jump_late_p, Genome_T genome, Genome_T genomealt,
                           Pairpool_T pairpool, int extraband_end, double defect_rate) {
  return shim_known(1, knownsplicep, dynprogindex, finalscore, ambig_end_length, ambig_splicetype, nmatches,
                    nmismatches, nopens, nindels, dynprog, sequence1, sequenceuc1, length1, length2, offset1, offset2,
                    querylength, chroffset, chrhigh, knownsplice_limit_low, knownsplice_limit_high, cdna_direction,
                    watsonp, genestrand, jump_late_p, genome, genomealt, pairpool, extraband_end, defect_rate);
}

/* Maxent_hr_*_prob of one splice-site entry (the host's MaxEnt models, maxent_hr.c) */
static double
shim_maxent (Genome_T genome, Genome_T genomealt, uint8_t model, gmapdp_coord_t pos, Univcoord_T chroffset) {
  switch (model) {
  case GMAPDP_MAXENT_DONOR: return Maxent_hr_donor_prob(genome, genomealt, (Univcoord_T) pos, chroffset);
  case GMAPDP_MAXENT_ACCEPTOR: return Maxent_hr_acceptor_prob(genome, genomealt, (Univcoord_T) pos, chroffset);
  case GMAPDP_MAXENT_ANTIDONOR: return Maxent_hr_antidonor_prob(genome, genomealt, (Univcoord_T) pos, chroffset);
  default: return Maxent_hr_antiacceptor_prob(genome, genomealt, (Univcoord_T) pos, chroffset);
  }
}

List_T
GMAPDP_DYNPROG_ENTRY(Dynprog_genome_gap) (int *dynprogindex, int *new_leftgenomepos, int *new_rightgenomepos, double *left_prob,
                           double *right_prob, int *traceback_score, int *nmatches, int *nmismatches, int *nopens,
                           int *nindels, int *exonhead, int *introntype, Dynprog_T dynprogL, Dynprog_T dynprogR,
                           char *rsequence, char *rsequenceuc, int rlength, int glengthL, int glengthR, int roffset,
                           int goffsetL, int rev_goffsetR, Chrnum_T chrnum, Univcoord_T chroffset,
                           Univcoord_T chrhigh, int cdna_direction, bool watsonp, int genestrand, bool jump_late_p,
                           Genome_T genome, Genome_T genomealt, Pairpool_T pairpool, int extraband_paired,
                           double defect_rate, int maxpeelback, bool halfp, bool finalp) {
  shim_req *r;
  gmapdp_genome_problem *p;
  gmapdp_genome_result *res;
  size_t m, i;
  static __thread gmapdp_coord_t *pos = NULL;
  static __thread uint8_t *model = NULL;
  static __thread size_t poscap = 0, modelcap = 0;
  List_T list;
  shim_check_call(genome, genomealt, dynprogL);
  shim_check_call(genome, genomealt, dynprogR);
  r = shim_request(K_GENOME);
  p = &r->p.g;
  p->rlength = rlength;
  p->glengthL = glengthL;
  p->glengthR = glengthR;
  p->roffset = roffset;
  p->goffsetL = goffsetL;
  p->rev_goffsetR = rev_goffsetR;
  p->chroffset = shim_coord(chroffset);
  p->chrhigh = shim_coord(chrhigh);
  p->flags = (watsonp ? GMAPDP_WATSON : 0) | (jump_late_p ? GMAPDP_JUMP_LATE : 0) | (halfp ? GMAPDP_HALFP : 0) |
             (finalp ? GMAPDP_FINALP : 0) | SHIM_SIMD;
  p->cdna_direction = cdna_direction;
  p->genestrand = genestrand;
  p->extraband = extraband_paired;
  p->maxpeelback = maxpeelback;
  p->dynprogindex = *dynprogindex;
  p->defect_rate = defect_rate;
  p->prob_offset = 0;
  /* the MaxEnt probabilities the bridge reads, computed on this thread with the host's own
     Maxent_hr_*_prob as the reference does; skipped where the engine resolves the call before
     reading them (rlength <= 1, size guard) */
  m = 0;
  if (rlength > 1 && rlength <= GMAPDP_MAX_RLENGTH && glengthL <= GMAPDP_MAX_GLENGTH &&
      glengthR <= GMAPDP_MAX_GLENGTH && glengthL > 0 && glengthR > 0)
    m = gmapdp_genome_prob_entries(p, 1);
  GROW(r->pbuf, r->pbufcap, m + 1);
  if (m && shim_use_host_maxent()) {
    memset(r->pbuf, 0, (m + 1) * sizeof(double));
    GROW(pos, poscap, m);
    GROW(model, modelcap, m);
    shim_check(gmapdp_genome_splice_sites(p, 1, pos, model, m), "gmapdp_genome_splice_sites");
    /* the last entry of each side is never read (the reference leaves it unset too, :2575-2660) */
    for (i = 0; i < m; i++)
      if (i != (size_t) glengthL - 1 && i != m - 1)
        r->pbuf[i] = shim_maxent(genome, genomealt, model[i], pos[i], chroffset);
  }
  if (m) {
    if (shim_siit != NULL) {
      /* known splice sites: the bridge's flags over the two windows and genome_gap_simple's over
         rlength (dynprog_genome.c:2938-2942, 3045-3049); the probabilities stay MaxEnt's */
      const size_t nk = gmapdp_genome_known_bytes(p);
      GROW(r->known, r->knowncap, nk);
      memset(r->known, 0, nk);
      shim_known_sites(r->known, r->known + glengthL, glengthL, glengthR, goffsetL, rev_goffsetR, cdna_direction,
                       watsonp, chrnum, chroffset, chrhigh);
      shim_known_sites(r->known + glengthL + glengthR, r->known + glengthL + glengthR + rlength + 1, rlength, rlength,
                       goffsetL, rev_goffsetR, cdna_direction, watsonp, chrnum, chroffset, chrhigh);
      p->flags |= GMAPDP_KNOWN_SITES;
      p->known_offset = 0;
      r->nknown = nk;
    }
  }
  r->genome = genome;
  r->q = rsequence;
  r->quc = rsequenceuc;
  r->qlen = rlength > 0 ? (size_t) rlength : 0;
  r->probs = shim_use_host_maxent() ? r->pbuf : NULL;  /* NULL: the engine evaluates them on the device */
  r->nprobs = m;
  r->cost = m == 0 ? 0 : 2 * shim_cost(rlength, glengthL > glengthR ? glengthL : glengthR, extraband_paired);
  r->longp = r->cost > shim_long_cost;
  GROW(r->pairs, r->pcap, gmapdp_genome_pair_capacity(p, 1) + 1);
  shim_submit(r);
  shim_count(ST_GENOME);
  res = &r->gr;
  list = shim_list(r->pairs, res->npairs, p->dynprogindex, res->gap_index, res->gap_queryjump, res->introntype,
                   res->left_prob, res->right_prob, pairpool);
  *dynprogindex = res->dynprogindex;
  *traceback_score = res->traceback_score;
  *nmatches = res->nmatches;
  *nmismatches = res->nmismatches;
  *nopens = res->nopens;
  *nindels = res->nindels;
  *introntype = res->introntype;
  *left_prob = res->left_prob;
  *right_prob = res->right_prob;
  if (res->new_leftgenomepos != GMAPDP_UNSET) *new_leftgenomepos = res->new_leftgenomepos;
  if (res->new_rightgenomepos != GMAPDP_UNSET) *new_rightgenomepos = res->new_rightgenomepos;
  if (res->exonhead != GMAPDP_UNSET) *exonhead = res->exonhead;
  return list;
}

List_T
GMAPDP_DYNPROG_ENTRY(Dynprog_cdna_gap) (int *dynprogindex, int *traceback_score, bool *incompletep, Dynprog_T dynprogL,
                         Dynprog_T dynprogR, char *rsequenceL, char *rsequence_ucL, char *rev_rsequenceR,
                         char *rev_rsequence_ucR, int rlengthL, int rlengthR, int glength, int roffsetL,
                         int rev_roffsetR, int goffset, Univcoord_T chroffset, Univcoord_T chrhigh, bool watsonp,
                         int genestrand, bool jump_late_p, Genome_T genome, Genome_T genomealt,
                         Pairpool_T pairpool, int extraband_paired, double defect_rate) {
  shim_req *r;
  gmapdp_cdna_problem *p;
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
  shim_check_call(genome, genomealt, dynprogL);
  shim_check_call(genome, genomealt, dynprogR);
  r = shim_request(K_CDNA);
  p = &r->p.c;
  p->qoffL = (int32_t) (rsequenceL - lo);
  p->qoffR = (int32_t) (rev_rsequenceR - lo);
  p->rlengthL = rlengthL;
  p->rlengthR = rlengthR;
  p->glength = glength;
  p->roffsetL = roffsetL;
  p->rev_roffsetR = rev_roffsetR;
  p->goffset = goffset;
  p->chroffset = shim_coord(chroffset);
  p->chrhigh = shim_coord(chrhigh);
  p->flags = (watsonp ? GMAPDP_WATSON : 0) | (jump_late_p ? GMAPDP_JUMP_LATE : 0) | SHIM_SIMD;
  p->genestrand = genestrand;
  p->extraband = extraband_paired;
  p->dynprogindex = *dynprogindex;
  p->defect_rate = defect_rate;
  r->genome = genome;
  r->q = lo;
  r->quc = lo_uc;
  r->qlen = (size_t) (hi - lo);
  GROW(r->pairs, r->pcap, gmapdp_cdna_pair_capacity(p, 1) + 1);
  shim_submit(r);
  shim_count(ST_CDNA);
  list = shim_list(r->pairs, r->cr.npairs, p->dynprogindex, r->cr.gap_index, r->cr.gap_queryjump, -1, 0.0, 0.0,
                   pairpool);
  *dynprogindex = r->cr.dynprogindex;
  if (r->cr.traceback_score != GMAPDP_UNSET) *traceback_score = r->cr.traceback_score;
  if (r->cr.incompletep) *incompletep = true;
  return list;
}

/* ---- Dynprog_microexon_int (dynprog_single.c:900, called at stage3.c:9664) ----
   One request (K_MXW): the GPU lists the candidates, scores their splice sites with its MaxEnt models,
   picks the winner and builds make_microexon_pairs_double's list, which is rebuilt here in the caller's
   Pairpool with the gap holders' comp set.  With GMAPDP_SHIM_HOST_MAXENT=1: two requests, the candidates
   scored on this thread with the host's maxent_hr.c in between. */
List_T
GMAPDP_DYNPROG_ENTRY(Dynprog_microexon_int) (double *bestprob2, double *bestprob3, int *dynprogindex, int *microintrontype,
                              char *rsequence, char *rsequenceuc, int rlength, int roffset, int goffsetL,
                              int rev_goffsetR, int cdna_direction, char *queryseq, char *queryuc,
                              Univcoord_T chroffset, Univcoord_T chrhigh, bool watsonp, int genestrand,
                              Genome_T genome, Genome_T genomealt, Pairpool_T pairpool) {
  shim_req *r;
  gmapdp_microexon_problem *p;
  List_T list = NULL;
  Pair_T gappair;
  int k;
  shim_check_call(genome, genomealt, NULL);
  /* make_microexon_pairs_double reads queryseq[roffset + i]; the engine reads the slice */
  if (rsequence != queryseq + roffset || rsequenceuc != queryuc + roffset)
    shim_refuse("Dynprog_microexon_int with rsequence other than queryseq + roffset");
  r = shim_request(shim_use_host_maxent() ? K_MXS : K_MXW);
  p = &r->p.mx;
  p->qoff = 0;
  p->rlength = rlength;
  p->roffset = roffset;
  p->goffsetL = goffsetL;
  p->rev_goffsetR = rev_goffsetR;
  p->cdna_direction = cdna_direction;
  p->chroffset = shim_coord(chroffset);
  p->chrhigh = shim_coord(chrhigh);
  p->watsonp = watsonp ? 1 : 0;
  p->genestrand = genestrand;
  p->dynprogindex = *dynprogindex;
  r->genome = genome;
  r->q = rsequence;
  r->quc = rsequenceuc;
  r->qlen = (size_t) (rlength > 0 ? rlength : 0);
  GROW(r->pairs, r->pcap, gmapdp_microexon_pair_capacity(p, 1) + 1);
  if (r->kind == K_MXS) {
    shim_submit(r);
    GROW(r->mxp, r->mxpcap, 2 * (size_t) r->mxr.ncandidates + 2);
    for (k = 0; k < r->mxr.ncandidates; k++) {
      const gmapdp_microexon_candidate *c = &r->mxc[k];
      r->mxp[2 * k] = shim_maxent(genome, genomealt, c->model2, c->pos2, chroffset);
      r->mxp[2 * k + 1] = shim_maxent(genome, genomealt, c->model3, c->pos3, chroffset);
    }
    r->kind = K_MXF;
  }
  shim_submit(r);
  shim_count(ST_MICROEXON);
  for (k = r->mxr.npairs - 1; k >= 0; k--) {
    const gmapdp_pair *e = &r->pairs[k];
    if (e->querypos == -1 && e->genomepos == -1) {
      list = Pairpool_push_gapholder(list, pairpool, /*queryjump*/0, e->jump, /*leftpair*/NULL, /*rightpair*/NULL,
                                     /*knownp*/false);
      gappair = (Pair_T) list->first;
      gappair->comp = e->comp;
    } else {
      list = Pairpool_push(list, pairpool, e->querypos, e->genomepos, e->cdna, e->comp, e->genome, e->genomealt,
                           p->dynprogindex);
    }
  }
  *bestprob2 = r->mxr.bestprob2;
  *bestprob3 = r->mxr.bestprob3;
  *microintrontype = r->mxr.microintrontype;
  *dynprogindex = r->mxr.dynprogindex;
  return r->mxr.npairs < 0 ? NULL : list;
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

/* Oligoindex_set_inquery (oligoindex_hr.c:33454) resets an oligoindex's inquery flags and marks the
   query's 8-mers only for queries longer than 8 nt; a shorter query's tally and lookups run against the
   flags of the last longer query on that oligoindex (they are never cleared between queries,
   Oligoindex_untally :33994).  The shim keeps that set per oligoindex (each GMAP worker thread owns
   its oligoindices) so that an 8-nt lookup answers as the reference's does. */
typedef struct {
  const void *oligoindex;
  uint32_t bits[2048];  /* 65536 8-mers */
} shim_inquery;
static __thread shim_inquery *shim_inq = NULL;
static __thread int shim_ninq = 0;

static shim_inquery *
shim_inquery_of (const void *oligoindex, int create) {
  int i;
  for (i = 0; i < shim_ninq; i++)
    if (shim_inq[i].oligoindex == oligoindex) return &shim_inq[i];
  if (!create) return NULL;
  shim_inq = (shim_inquery *) realloc(shim_inq, (size_t) (shim_ninq + 1) * sizeof(shim_inquery));
  if (shim_inq == NULL) shim_refuse("host memory for oligoindex state (out of memory)");
  memset(&shim_inq[shim_ninq], 0, sizeof(shim_inquery));
  shim_inq[shim_ninq].oligoindex = oligoindex;
  return &shim_inq[shim_ninq++];
}

/* the 8-mer following the encoding of set_inquery (A C G T = 0 1 2 3; other characters restart) */
static void
shim_set_inquery (const void *oligoindex, const char *queryuc, int querystart, int queryend) {
  shim_inquery *e;
  uint32_t oligo = 0;
  int i, in_counter = 0, c;
  if (queryend - querystart <= 8) return;  /* the flags stay as the last longer query left them */
  e = shim_inquery_of(oligoindex, 1);
  memset(e->bits, 0, sizeof(e->bits));
  for (i = querystart; i < queryend; i++) {
    in_counter++;
    switch (queryuc[i]) {
    case 'A': c = 0; break;
    case 'C': c = 1; break;
    case 'G': c = 2; break;
    case 'T': c = 3; break;
    default: c = -1; break;
    }
    if (c < 0) {
      oligo = 0;
      in_counter = 0;
      continue;
    }
    oligo = (oligo << 2) | (uint32_t) c;
    if (in_counter == 8) {
      const uint32_t m = oligo & 0xFFFFu;
      e->bits[m >> 5] |= 1u << (m & 31);
      in_counter--;
    }
  }
}

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
  shim_set_inquery(this, queryuc_ptr, querystart, queryend);
  this->table = NULL;
}

List_T
__wrap_Oligoindex_get_mappings (List_T diagonals, bool *coveredp, Chrpos_T **mappings, int *npositions,
                                int *totalpositions, bool *oned_matrix_p, int *maxnconsecutive,
                                Oligoindex_array_T array, Oligoindex_T this, char *queryuc_ptr, int querystart,
                                int queryend, int querylength, Chrpos_T chrstart, Chrpos_T chrend,
                                Univcoord_T chroffset, Univcoord_T chrhigh, bool plusp, Diagpool_T diagpool) {
  shim_req *r;
  gmapdp_oligo_problem *p;
  size_t dc;
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
  if (chrend <= chrstart) return diagonals;  /* :34157, before anything is written */
  if (querylength <= 8) {
    /* At most one 8-mer (querypos 0): lookups answer from the table that the tally built over the
       last longer query's 8-mers (shim_set_inquery).  Below 8 nt, or an 8-mer outside that set, there
       is no hit and nothing but oned_matrix_p is written (:34208-34305). */
    shim_inquery *e = shim_inquery_of(this, 0);
    uint32_t x = 0;
    int full = querylength == 8;
    for (q = 0; q < querylength && full; q++) {
      switch (queryuc_ptr[q]) {
      case 'A': x = x << 2; break;
      case 'C': x = (x << 2) | 1u; break;
      case 'G': x = (x << 2) | 2u; break;
      case 'T': x = (x << 2) | 3u; break;
      default: full = 0; break;
      }
    }
    *oned_matrix_p = true;
    if (!full) return diagonals;
    if (e == NULL || !((e->bits[x >> 5] >> (x & 31)) & 1u)) {  /* lookup: nhits 0 */
      npositions[0] = 0;
      mappings[0] = NULL;
      return diagonals;
    }
    /* the 8-mer is in the table: its positions in the window are the engine's answer for the query
       "8-mer" + 'N' (one distinct 8-mer; a single query position makes no consecutive run, so no
       diagonal and maxnconsecutive 0) */
    {
      r = shim_request(K_OLIGO);
      memcpy(r->quc9, queryuc_ptr, 8);
      r->quc9[8] = 'N';
      p = &r->p.o;
      p->querylength = 9;
      p->chrstart = chrstart;
      p->chrend = chrend;
      p->chroffset = shim_coord(chroffset);
      p->chrhigh = shim_coord(chrhigh);
      p->plusp = plusp ? 1 : 0;
      p->minor = this->diag_lookback == 60 ? 1 : 0;
      r->genome = shim_tally.genome;
      r->q = r->quc = r->quc9;
      r->qlen = 9;
      r->tabn = gmapdp_oligo_positions_capacity(p, 1);
      dc = gmapdp_oligo_diagonal_capacity(p, 1);
      GROW(r->np, r->npcap, r->qlen + 1);
      GROW(r->mp, r->mpcap, r->qlen + 1);
      GROW(r->pos, r->poscap, r->tabn + 1);
      GROW(r->dg, r->dgcap, 4 * dc + 4);
      shim_submit(r);
      shim_count(ST_OLIGO);
      if (r->orr.oned_matrix_p < 0) shim_refuse("Oligoindex_get_mappings: the engine reported a layout overflow");
      this->table = NULL;
      if (r->tabn > 0) {
        this->table = (Chrpos_T *) MALLOC(r->tabn * sizeof(Chrpos_T));
        memcpy(this->table, r->pos, r->tabn * sizeof(Chrpos_T));
      }
      npositions[0] = r->np[0];
      mappings[0] = r->np[0] > 0 ? &this->table[r->mp[0]] : NULL;
      *totalpositions = r->orr.totalpositions;
      return diagonals;
    }
  }
  r = shim_request(K_OLIGO);
  p = &r->p.o;
  p->querylength = querylength;
  p->chrstart = chrstart;
  p->chrend = chrend;
  p->chroffset = shim_coord(chroffset);
  p->chrhigh = shim_coord(chrhigh);
  p->plusp = plusp ? 1 : 0;
  p->minor = this->diag_lookback == 60 ? 1 : 0;  /* Oligoindex_array_new_minor's index (oligoindex_hr.c:8612) */
  r->genome = shim_tally.genome;
  r->q = r->quc = queryuc_ptr;
  r->qlen = querylength > 0 ? (size_t) querylength : 0;
  r->tabn = gmapdp_oligo_positions_capacity(p, 1);
  dc = gmapdp_oligo_diagonal_capacity(p, 1);
  GROW(r->np, r->npcap, r->qlen + 1);
  GROW(r->mp, r->mpcap, r->qlen + 1);
  GROW(r->pos, r->poscap, r->tabn + 1);
  GROW(r->dg, r->dgcap, 4 * dc + 4);
  shim_submit(r);
  shim_count(ST_OLIGO);
  /* oned_matrix_p -1: the engine's layout overflowed (nothing usable was written).  The request was sized
     with the worst-case capacities, so this cannot happen; never hand GMAP an empty "valid" answer. */
  if (r->orr.oned_matrix_p < 0) shim_refuse("Oligoindex_get_mappings: the engine reported a layout overflow");
  /* the table, owned by the oligoindex (freed by Oligoindex_untally) */
  this->table = NULL;
  if (r->tabn > 0) {
    this->table = (Chrpos_T *) MALLOC(r->tabn * sizeof(Chrpos_T));
    memcpy(this->table, r->pos, r->tabn * sizeof(Chrpos_T));
  }
  for (q = 0; q < querylength; q++) {
    if (r->np[q] > 0) {
      npositions[q] = r->np[q];
      mappings[q] = &this->table[r->mp[q]];
    } else if (q <= querylength - 8 && strspn(queryuc_ptr + q, "ACGT") >= 8) {
      /* lookup (:34069) on a full 8-mer without hits: nhits 0, mappings NULL; others stay as given */
      npositions[q] = 0;
      mappings[q] = NULL;
    }
  }
  *totalpositions = r->orr.totalpositions;
  *maxnconsecutive = r->orr.maxnconsecutive;
  if (chrend > chrstart) *oned_matrix_p = r->orr.oned_matrix_p ? true : false;
  for (k = r->orr.ndiagonals - 1; k >= 0; k--) {
    const int32_t *d = r->dg + 4 * k;
    diagonals = Diagpool_push(diagonals, diagpool, d[0], d[1], d[2], d[3]);
  }
  return diagonals;
}

/* ---- Stage2_compute (stage2.c:6325): seeding + chaining on the engine ----
   gmap.c's calls (update_stage3middle_list / update_stage3list, gmap.c:1208 / 1323) pass the major
   oligoindex array, localp, skip_repetitive_p, favor_right_p false and max_nalignments 10; the engine
   restates exactly that configuration and the shim refuses any other.  Each returned Stage2_T holds
   the middle path's pairs, pushed into the caller's Pairpool in list order; its all_starts / all_ends
   stay NULL as in the reference (MOVE_TO_STAGE3 undefined). */
extern void __real_Stage2_setup (bool splicingp_in, bool cross_species_p, int suboptimal_score_start_in,
                                 int suboptimal_score_end_in, int sufflookback_in, int nsufflookback_in,
                                 int maxintronlen_in, Mode_T mode_in, bool snps_p_in);
static int s2_splicingp = 1, s2_cross_species_p = 0, s2_sufflookback = 60, s2_nsufflookback = 5,
           s2_maxintronlen = 500000, s2_mode = 0, s2_snps_p = 0;

void
__wrap_Stage2_setup (bool splicingp_in, bool cross_species_p, int suboptimal_score_start_in,
                     int suboptimal_score_end_in, int sufflookback_in, int nsufflookback_in, int maxintronlen_in,
                     Mode_T mode_in, bool snps_p_in) {
  __real_Stage2_setup(splicingp_in, cross_species_p, suboptimal_score_start_in, suboptimal_score_end_in,
                      sufflookback_in, nsufflookback_in, maxintronlen_in, mode_in, snps_p_in);
  s2_splicingp = splicingp_in ? 1 : 0;
  s2_cross_species_p = cross_species_p ? 1 : 0;
  s2_sufflookback = sufflookback_in;
  s2_nsufflookback = nsufflookback_in;
  s2_maxintronlen = maxintronlen_in;
  s2_mode = (int) mode_in;
  s2_snps_p = snps_p_in ? 1 : 0;
}

/* struct Stage2_T (stage2.c:302): Stage2_free (FREE) and Stage2_middle read it */
struct shim_stage2 {
  List_T middle;
  List_T all_starts;
  List_T all_ends;
};

List_T
__wrap_Stage2_compute (char *queryseq_ptr, char *queryuc_ptr, int querylength, int query_offset, Chrpos_T chrstart,
                       Chrpos_T chrend, Univcoord_T chroffset, Univcoord_T chrhigh, bool plusp, int genestrand,
                       Stage2_alloc_T stage2_alloc, double proceed_pctcoverage, Oligoindex_array_T oligoindices,
                       Genome_T genome, Genome_T genomealt, Pairpool_T pairpool, Diagpool_T diagpool,
                       Cellpool_T cellpool, bool localp, bool skip_repetitive_p, bool favor_right_p,
                       int max_nalignments, Stopwatch_T stopwatch, bool diag_debug) {
  shim_req *r;
  gmapdp_stage2_problem *p;
  Oligoindex_T major;
  List_T results = NULL, middle;
  struct shim_stage2 *s2;
  int k, i;
  (void) stage2_alloc;
  (void) diagpool;
  (void) cellpool;
  (void) stopwatch;
  (void) genestrand;
  if (s2_mode != 0 || shim_mode != 0) shim_refuse("Stage2_compute outside STANDARD mode (cmet / atoi / ttoc)");
  if (s2_cross_species_p) shim_refuse("Stage2_compute with cross-species canonical scoring");
  if (s2_snps_p || (genomealt != NULL && genomealt != genome)) shim_refuse("Stage2_compute with an SNP genome");
  if (s2_sufflookback != 60 || s2_nsufflookback != 5) shim_refuse("Stage2_compute with non-default lookback");
  if (diag_debug) shim_refuse("Stage2_compute diagnostics (diag_debug)");
  if (query_offset != 0 || !localp || !skip_repetitive_p || favor_right_p || max_nalignments != 10 ||
      proceed_pctcoverage != 0.3)
    shim_refuse("a Stage2_compute call other than gmap.c's (localp, 0.3 coverage, 10 alignments)");
  if (Oligoindex_array_length(oligoindices) != 1) shim_refuse("more than one stage-2 oligoindex source");
  major = Oligoindex_array_elt(oligoindices, 0);
  if (major->indexsize != 8 || major->diag_lookback != 120 || major->suffnconsecutive != 20)
    shim_refuse("an oligoindex other than GMAP's major 8-mer index");
  /* Below 8 nt the query holds no 8-mer: Oligoindex_get_mappings finds no position, totalpositions is 0
     and the reference returns NULL (stage2.c:6524).  At exactly 8 nt the tally runs against the previous
     longer query's inquery flags (Oligoindex_set_inquery returns early, oligoindex_hr.c:33478; the shim
     keeps them per oligoindex): a full 8-mer outside them has no hit (NULL again); one inside them has
     the window positions of that 8-mer alone, which is what the engine computes for the query
     "8-mer" + 'N' -- one query position with hits, no diagonal, the same chaining and pairs (querypos
     0..7).  The 9th position never has a hit and lies past every pair. */
  if (querylength < 8) return NULL;
  if (querylength == 8) {
    shim_inquery *e = shim_inquery_of(major, 0);
    uint32_t x = 0;
    for (i = 0; i < 8; i++) {
      switch (queryuc_ptr[i]) {
      case 'A': x = x << 2; break;
      case 'C': x = (x << 2) | 1u; break;
      case 'G': x = (x << 2) | 2u; break;
      case 'T': x = (x << 2) | 3u; break;
      default: return NULL;  /* no full 8-mer: no lookup, totalpositions 0 */
      }
    }
    if (e == NULL || !((e->bits[x >> 5] >> (x & 31)) & 1u)) return NULL;  /* not in the stale flags */
  } else {
    shim_set_inquery(major, queryuc_ptr, 0, querylength);  /* the tally inside Stage2_compute sets them */
  }
  /* the chaining kernels keep Chrpos_T differences in 32-bit registers: checked here, on the calling
     thread, so that a refusal names its own call and never fails another thread's batch */
  if (chrend >= 0x80000000U || chrstart >= 0x80000000U)
    shim_refuse("Stage2_compute at chromosome positions past 2^31");
  r = shim_request(K_STAGE2);
  p = &r->p.s2;
  p->querylength = querylength;
  p->chrstart = chrstart;
  p->chrend = chrend;
  p->chroffset = shim_coord(chroffset);
  p->chrhigh = shim_coord(chrhigh);
  p->plusp = plusp ? 1 : 0;
  p->splicingp = s2_splicingp;
  p->maxintronlen = s2_maxintronlen;
  r->genome = genome;
  r->q = queryseq_ptr;
  r->quc = queryuc_ptr;
  r->qlen = (size_t) querylength;
  if (querylength == 8) {
    memcpy(r->q9, queryseq_ptr, 8);
    memcpy(r->quc9, queryuc_ptr, 8);
    r->q9[8] = r->quc9[8] = 'N';
    r->q = r->q9;
    r->quc = r->quc9;
    r->qlen = 9;
    p->querylength = 9;
  }
  shim_submit(r);
  shim_count(ST_STAGE2);
  /* the results in list order: build from the last (each List_push prepends) */
  for (k = r->s2r.nresults - 1; k >= 0; k--) {
    const gmapdp_path *pa = &r->s2paths[k];
    const gmapdp_path_pair *pr = r->s2pairs + pa->pair_offset;
    middle = NULL;
    for (i = pa->npairs - 1; i >= 0; i--) {
      if (pr[i].querypos == -1 && pr[i].genomepos == -1)
        middle = Pairpool_push_gapholder(middle, pairpool, pr[i].queryjump, pr[i].genomejump, /*leftpair*/NULL,
                                         /*rightpair*/NULL, /*knownp*/false);
      else
        middle = Pairpool_push(middle, pairpool, pr[i].querypos, pr[i].genomepos, pr[i].cdna, pr[i].comp,
                               pr[i].genome, pr[i].genomealt, /*dynprogindex*/0);
    }
    s2 = (struct shim_stage2 *) MALLOC(sizeof(struct shim_stage2));
    s2->middle = middle;
    s2->all_starts = NULL;
    s2->all_ends = NULL;
    results = List_push(results, (void *) s2);
  }
  return results;
}
