/* include/gmapdp.h -- C ABI of the MI355X GMAP Dynprog engine (libgmapdp.so).
 *
 * This is the drop-in boundary for GMAP's Dynprog_* hot path.  It is a
 * batched, plain-pointer restatement of the reference entry points; the
 * reference-signature wrappers (Dynprog_single_gap(...) etc., which take
 * GMAP's Dynprog_T / Genome_T / Pairpool_T and return List_T of Pair_T) are
 * declared in include/gmapdp_dynprog.h and documented in INTEGRATION.md.
 *
 * Entry point -> reference interface it replaces (paths under the reference
 * tree's src/):
 *   gmapdp_create            Dynprog_init (dynprog.c:1008) + Dynprog_single_setup
 *                            (dynprog_single.c:101) + Dynprog_end_setup (dynprog_end.c)
 *   gmapdp_destroy           Dynprog_term (dynprog.c:1203)
 *   gmapdp_pack_genome       Compress_create_blocks_comp (compress-write.c:754): the
 *                            .genomecomp block format that GMAP mmaps (genome.c:208)
 *   gmapdp_set_genome        Genome_new / Genome_from_sequence (genome.c:208/307):
 *                            the packed genome is made resident in HBM
 *   gmapdp_single_gap_batch  Dynprog_single_gap (dynprog_single.c:429), one call per
 *                            problem, many problems per launch
 *   gmapdp_end_gap_batch     Dynprog_end5_gap / Dynprog_end3_gap (dynprog_end.c:1294/1924)
 *   gmapdp_genome_gap_batch  Dynprog_genome_gap (dynprog_genome.c:3288) + Dynprog_genome_setup
 *                            (:192, no splicing IIT); gmapdp_genome_splice_sites lists the
 *                            Maxent_hr_*_prob calls (maxent_hr.c:27357-27600) whose values it takes
 *   gmapdp_plan_*            the same calls, planned once and replayed on device-resident
 *                            inputs (mixed single + end batches)
 *   gmapdp_compute_bands     Dynprog_compute_bands (dynprog.c:1247)
 *   gmapdp_cdna_gap_batch    Dynprog_cdna_gap (dynprog_cdna.c:787)
 *   gmapdp_end_splicejunction_batch  Dynprog_end5/3_splicejunction (dynprog_end.c:1653/2249), the
 *                            known-splice-site end alignments of Dynprog_end5/3_known (:2748/3009)
 *   gmapdp_oligo_mappings_batch  stage-2 seeding: Oligoindex_hr_tally + Oligoindex_get_mappings
 *                            (oligoindex_hr.c:33849/34127) as Stage2_compute calls them (stage2.c:6480-6495)
 *   gmapdp_stage2_batch      Stage2_compute (stage2.c:6325) as GMAP calls it (gmap.c:1208): the
 *                            seeding above, then Diag_compute_bounds (diag.c:597),
 *                            align_compute_lookback (stage2.c:4402), convert_to_nucleotides (:5334)
 *                            and Stage2_filter_unique (:6013)
 *
 * Semantics: every result is bit-identical to the reference's nosimd build
 * (Dynprog_standard + Dynprog_traceback_std), or with GMAPDP_SIMD to its SIMD builds
 * (dynprog_simd.c); stage-2 seeding has one semantics (both builds agree); see DESIGN.md "Parity".
 *
 * Errors: functions return 0 on success and a negative GMAPDP_E* code on
 * failure (no errno).  A per-problem NULL result (the reference returning a
 * NULL List_T) is reported as npairs == 0 with the reference's score
 * convention in traceback_score (NEG_INFINITY_32 = -32768 for the size
 * guard).
 *
 * Threading: a gmapdp_ctx and its plans are NOT thread-safe.  A context (its
 * scratch buffers, fork/join events and side streams) and every plan created on
 * it must be used by one host thread at a time, and a plan must not run on two
 * streams at once (its pool counter and the context scratch are shared).  Use
 * one context per thread, or serialise.  The GMAP shim gives each of its
 * dispatcher threads its own context (gmapdp_create_ex: one stream each, DP
 * dispatchers at high priority, stage-2 dispatchers at low priority) and
 * uploads the genome to HBM once: the other contexts share that copy
 * (gmapdp_share_genome), so GRCh38 costs 1.16 GB of HBM and a 17-Gnt genome
 * 6.4 GB whatever the number of dispatchers.
 */
#ifndef GMAPDP_H
#define GMAPDP_H

#include <stddef.h>
#include <stdint.h>

/* A universal genome coordinate (GMAP's Univcoord_T, univcoord.h:9-11): 64 bits so that one ABI
 * serves gmap (32-bit Univcoord_T) and gmapl (LARGE_GENOMES, genomes past 2^32 nt).  Chromosome
 * positions (Chrpos_T) stay 32-bit, as in both GMAP builds. */
typedef uint64_t gmapdp_coord_t;

#ifdef __cplusplus
extern "C" {
#endif

#define GMAPDP_OK 0
#define GMAPDP_EINVAL (-1)
#define GMAPDP_ENODEV (-2)
#define GMAPDP_ENOMEM (-3)
#define GMAPDP_ELAUNCH (-4)
#define GMAPDP_ENOGENOME (-5)

/* Reference limits (Dynprog_new with gmap.c defaults, dynprog.c:602-627). */
#define GMAPDP_MAX_RLENGTH 660
#define GMAPDP_MAX_GLENGTH 2000
#define GMAPDP_NEG_INFINITY_32 (-32768)

typedef struct gmapdp_ctx gmapdp_ctx;

/* One Pair_T (pairdef.h:8-42) as the engine emits it, in the order of the
 * List_T the reference returns.  A gap holder (Pairpool_push_gapholder,
 * pairpool.c:375) has querypos == genomepos == -1 and jump == genomejump;
 * ordinary pairs have jump == 0.  dynprogindex is per problem (all pairs of
 * one call carry the caller's *dynprogindex, gap holders carry 0). */
typedef struct {
  int32_t querypos;
  int32_t genomepos;
  int32_t jump;
  char cdna;
  char comp;
  char genome;
  char genomealt;
} gmapdp_pair;

/* Problem flags */
#define GMAPDP_WATSON     0x1  /* watsonp */
#define GMAPDP_JUMP_LATE  0x2  /* jump_late_p */
#define GMAPDP_WIDEBAND   0x4  /* widebandp */
/* Reproduce the reference's SIMD builds (gmap.sse42/.avx2/.avx512, dynprog_simd.c) instead of
 * the nosimd build (Dynprog_standard): Dynprog_simd_8/16 for single gaps, the
 * Dynprog_simd_8/16_upper/_lower triangles with their endpoint scans, bridge and tracebacks for
 * end and genome gaps.  Valid in every problem family (genome gaps: in `flags` as well).  The
 * SIMD fills read arena cells the call never wrote; the engine defines those as zero (a fresh
 * arena).  End gaps with rlength > glength + 1 (chopped lengths, QUERYEND_NOGAPS excepted) are
 * GMAPDP_EINVAL: the reference's lower-triangle scan reads uninitialised scores there. */
#define GMAPDP_SIMD       0x40

/* One Dynprog_single_gap call (dynprog_single.c:429 argument list).  The
 * query slice is qseq[qoff .. qoff+rlength) (rsequence, case as given) and
 * qseq_uc[...] (rsequenceuc) in the batch's query arena. */
typedef struct {
  int32_t qoff;
  int32_t rlength;
  int32_t glength;
  int32_t roffset;
  int32_t goffset;
  gmapdp_coord_t chroffset;
  gmapdp_coord_t chrhigh;
  int32_t flags;          /* GMAPDP_WATSON | GMAPDP_JUMP_LATE | GMAPDP_WIDEBAND */
  int32_t genestrand;     /* 0, +1, +2 */
  int32_t extraband;      /* extraband_single */
  double defect_rate;
  int32_t dynprogindex;   /* *dynprogindex on entry */
  int32_t pad_;
} gmapdp_single_problem;

/* Endalign_T (dynprog.h:25) */
#define GMAPDP_QUERYEND_GAP     0
#define GMAPDP_QUERYEND_INDELS  1
#define GMAPDP_QUERYEND_NOGAPS  2
#define GMAPDP_BEST_LOCAL       3

/* One Dynprog_end5_gap (end3p = 0, dynprog_end.c:1294) or Dynprog_end3_gap
 * (end3p = 1, dynprog_end.c:1924) call.  The query slice is
 * qseq[qoff .. qoff+rlength): for end3 the reference's rsequence points at its
 * first character, for end5 rev_rsequence points at its LAST character (the
 * DP walks away from the anchor).  roffset/goffset are the reference's
 * (rev_)roffset/(rev_)goffset.  The engine applies the reference's chopping
 * to 660 x 2000 (except QUERYEND_NOGAPS). */
typedef struct {
  int32_t qoff;
  int32_t rlength;
  int32_t glength;
  int32_t roffset;
  int32_t goffset;
  gmapdp_coord_t chroffset;
  gmapdp_coord_t chrhigh;
  int32_t flags;          /* GMAPDP_WATSON | GMAPDP_JUMP_LATE */
  int32_t genestrand;
  int32_t extraband;      /* extraband_end */
  int32_t end3p;
  int32_t endalign;       /* GMAPDP_QUERYEND_* / GMAPDP_BEST_LOCAL */
  int32_t require_pos_score_p;
  int32_t dynprogindex;
  double defect_rate;
} gmapdp_end_problem;

/* Per-problem outputs (the reference's out-parameters). */
typedef struct {
  int32_t npairs;          /* 0 <=> NULL List_T */
  int32_t pair_offset;     /* first pair in the batch's pair arena */
  int32_t traceback_score; /* *finalscore / *traceback_score */
  int32_t nmatches;
  int32_t nmismatches;
  int32_t nopens;
  int32_t nindels;
  int32_t dynprogindex;    /* *dynprogindex on exit */
} gmapdp_result;

/* Dynprog_genome_gap flags (in addition to GMAPDP_WATSON / GMAPDP_JUMP_LATE) */
#define GMAPDP_HALFP   0x8
#define GMAPDP_FINALP  0x10
/* Known splice sites (gmap -s with a splice-site file: Dynprog_genome_setup with a splicing IIT and
 * donor/acceptor types, novel splicing on; get_known_splicesites, dynprog_genome.c:405).  The problem's
 * flags per position are in the batch's known-site arena at known_offset (one byte each, 0 or 1):
 *   [0, glengthL)                        the bridge's left_known (dynprog_genome.c:2938-2942)
 *   [glengthL, glengthL + glengthR)      its right_known
 *   then rlength + 1 bytes, then rlength + 1 bytes: genome_gap_simple's left_known / right_known
 *   (:3045-3049, queried with glength = rlength)
 * A known position scores KNOWN_SPLICESITE_REWARD in genome_gap_simple and has probability 1.0; the
 * probability arena then holds the MaxEnt values at every position (known or not).  Both builds'
 * semantics (with GMAPDP_SIMD the SIMD bridge reads the same flags). */
#define GMAPDP_KNOWN_SITES 0x80

/* One Dynprog_genome_gap call (dynprog_genome.c:3288 argument list).  The
 * query slice is qseq[qoff .. qoff+rlength) (rsequence / rsequenceuc).
 * chrnum is not needed (it only serves known-splice-site IIT lookups, which
 * the engine does not perform: see splice probabilities below).
 * Domain: glengthL and glengthR must exceed rlength (every stage3.c call
 * passes queryjump + extramaterial_paired); outside it the reference reads
 * uninitialised probabilities (dynprog_genome.c:2575-2660 leave the last
 * entry unset), so the engine rejects such a batch with GMAPDP_EINVAL.
 *
 * Splice probabilities.  The reference's bridge (dynprog_genome.c:2569-2660)
 * and genome_gap_simple (:3171) read MaxEnt splice-site probabilities
 * (Maxent_hr_*_prob, maxent_hr.c, a host symbol the Dynprog objects import).
 * The caller supplies them in a double arena: problem i's left
 * probabilities at [prob_offset, prob_offset + glengthL) and its right ones
 * at [prob_offset + glengthL, prob_offset + glengthL + glengthR);
 * gmapdp_genome_splice_sites lists the (position, model) of every entry. */
typedef struct {
  int32_t qoff;
  int32_t rlength;
  int32_t glengthL;
  int32_t glengthR;
  int32_t roffset;
  int32_t goffsetL;
  int32_t rev_goffsetR;
  gmapdp_coord_t chroffset;
  gmapdp_coord_t chrhigh;
  int32_t flags;          /* GMAPDP_WATSON | GMAPDP_JUMP_LATE | GMAPDP_HALFP | GMAPDP_FINALP */
  int32_t cdna_direction;
  int32_t genestrand;
  int32_t extraband;      /* extraband_paired (+ peeled indels, stage3.c:9538) */
  int32_t maxpeelback;
  int32_t dynprogindex;
  int32_t known_offset;   /* with GMAPDP_KNOWN_SITES: the problem's first byte in the known-site arena */
  double defect_rate;
  int64_t prob_offset;
} gmapdp_genome_problem;

/* Out-parameters of Dynprog_genome_gap.  new_leftgenomepos,
 * new_rightgenomepos and exonhead are GMAPDP_UNSET where the reference does
 * not write them.  The intron gap holder (Pairpool_push_gapholder with
 * queryjump, genomejump, introntype, donor_prob = left_prob, acceptor_prob =
 * right_prob; dynprog_genome.c:3227-3232 / 3859-3865) is pairs[gap_index]
 * (gap_index -1 for a NULL result); its record carries jump = genomejump. */
#define GMAPDP_UNSET ((int32_t)0x80000000)
typedef struct {
  int32_t npairs;          /* 0 <=> NULL List_T */
  int32_t pair_offset;
  int32_t traceback_score;
  int32_t nmatches;
  int32_t nmismatches;
  int32_t nopens;
  int32_t nindels;
  int32_t dynprogindex;
  int32_t new_leftgenomepos;
  int32_t new_rightgenomepos;
  int32_t exonhead;
  int32_t introntype;
  int32_t gap_index;
  int32_t gap_queryjump;
  double left_prob;
  double right_prob;
} gmapdp_genome_result;

/* Splice-site model of a probability-array entry */
#define GMAPDP_MAXENT_DONOR        0  /* Maxent_hr_donor_prob */
#define GMAPDP_MAXENT_ACCEPTOR     1  /* Maxent_hr_acceptor_prob */
#define GMAPDP_MAXENT_ANTIDONOR    2  /* Maxent_hr_antidonor_prob */
#define GMAPDP_MAXENT_ANTIACCEPTOR 3  /* Maxent_hr_antiacceptor_prob */

/* Device MaxEnt.  The engine evaluates Maxent_hr_{donor,acceptor,antidonor,antiacceptor}_prob
 * (maxent_hr.c:27357 / 27433 / 27512 / 27586) itself, on the HBM-resident genome, bit-identical doubles
 * (genomealt == genome, the engine's scope).  The model tables are the reference's constants
 * (maxent_hr.c:25-24660) as tools/make_maxent_tables.py writes them: maxent_hr_tables.bin next to
 * libgmapdp.so, or the file GMAPDP_MAXENT_TABLES names; loaded on first use, once per device.
 *   - genome gaps: pass splice_probs = NULL (gmapdp_genome_gap_batch[_known], gmapdp_dynprog_batch,
 *     gmapdp_mixed.splice_probs) and the probability entries are computed on the device in the batch's
 *     stream (nprobs / nsplice_probs still give the arena size, gmapdp_genome_prob_entries);
 *   - microexons: gmapdp_microexon_finish with cand_probs = NULL (gmapdp_mixed.finish_probs = NULL)
 *     evaluates the candidates' two sites in the finish kernel; gmapdp_mixed's "whole microexon" section
 *     runs search and finish in the one round trip;
 *   - plans: gmapdp_plan_bind_genome_maxent; gmapdp_microexon_plan_run with d_cand_probs = NULL.
 * Missing tables make these calls fail with GMAPDP_EINVAL ("maxent tables: ...") -- never a host
 * fallback. */
/* 1 when the tables load (host only, no device needed), else 0; path: the file used or looked for. */
int gmapdp_maxent_available (char *path, size_t path_bytes);
/* out[i] = Maxent_hr_<models[i]>_prob(splice_pos = positions[i], chroffset = chroffsets[i]) on ctx's genome
 * (synchronous). */
int gmapdp_maxent_sites (gmapdp_ctx *ctx, const gmapdp_coord_t *positions, const uint8_t *models,
                         const gmapdp_coord_t *chroffsets, size_t n, double *out);

/* For each problem, write glengthL + glengthR (splicesitepos, model) pairs
 * at the problem's prob_offset: the arguments of the Maxent_hr_*_prob call
 * (with the problem's chroffset) whose result belongs at that entry
 * (dynprog_genome.c:2573-2660).  Host-only; no device needed. */
int gmapdp_genome_splice_sites (const gmapdp_genome_problem *problems, int n, gmapdp_coord_t *positions,
                                uint8_t *models, size_t nentries);
/* Entries of the probability arena needed by the batch (max prob_offset + glengthL + glengthR). */
size_t gmapdp_genome_prob_entries (const gmapdp_genome_problem *problems, int n);

/* Run n Dynprog_genome_gap problems (same conventions as the other batches).
 * splice_probs: host arena of gmapdp_genome_prob_entries doubles. */
int gmapdp_genome_gap_batch (gmapdp_ctx *ctx, const gmapdp_genome_problem *problems, int n,
                             const char *qseq, const char *qseq_uc, size_t qbytes,
                             const double *splice_probs, size_t nprobs,
                             gmapdp_genome_result *results, gmapdp_pair *pairs, size_t pair_capacity);
/* The same with the known-site arena (nknown bytes) of GMAPDP_KNOWN_SITES problems. */
int gmapdp_genome_gap_batch_known (gmapdp_ctx *ctx, const gmapdp_genome_problem *problems, int n,
                                   const char *qseq, const char *qseq_uc, size_t qbytes,
                                   const double *splice_probs, size_t nprobs, const uint8_t *known_sites,
                                   size_t nknown, gmapdp_genome_result *results, gmapdp_pair *pairs,
                                   size_t pair_capacity);
/* Bytes of the problem's region of the known-site arena: glengthL + glengthR + 2 * (rlength + 1). */
size_t gmapdp_genome_known_bytes (const gmapdp_genome_problem *problem);
size_t gmapdp_genome_pair_capacity (const gmapdp_genome_problem *problems, int n);

/* Dynprog_single_gap + Dynprog_end5/3_gap + Dynprog_genome_gap calls of many callers in one
 * synchronous batch (the drop-in's dispatcher: one launch set for whatever GMAP's worker threads have
 * issued meanwhile).  One query arena (all qoff index qseq / qseq_uc), one splice-probability arena;
 * results has nsingle + nend entries (singles first), genome_results ngenome; pair_capacity at least
 * gmapdp_single_pair_capacity + gmapdp_end_pair_capacity + gmapdp_genome_pair_capacity. */
int gmapdp_dynprog_batch (gmapdp_ctx *ctx, const gmapdp_single_problem *singles, int nsingle,
                          const gmapdp_end_problem *ends, int nend, const gmapdp_genome_problem *genomes, int ngenome,
                          const char *qseq, const char *qseq_uc, size_t qbytes, const double *splice_probs,
                          size_t nprobs, gmapdp_result *results, gmapdp_genome_result *genome_results,
                          gmapdp_pair *pairs, size_t pair_capacity);

/* One Dynprog_cdna_gap call (dynprog_cdna.c:787 argument list): a cDNA insertion between two
 * anchors.  rsequenceL / rsequence_ucL = qseq / qseq_uc + qoffL (the L piece's first character),
 * rev_rsequenceR / rev_rsequence_ucR = qseq / qseq_uc + qoffR (the R piece's LAST character).  The
 * SHORTGAP block pushed when the bridge leaves a 9 x 9 gap reads rsequenceL up to
 * rev_roffsetR - roffsetL, so the arena must hold qseq[qoffL .. qoffL + rev_roffsetR - roffsetL].
 * Penalties are CDNA_OPEN/CDNA_EXTEND (dynprog_cdna.c:32-38) whatever the mode.
 * Domain: rlengthL == rlengthR >= glength, as stage3.c passes (both pieces queryjump' = genomejump +
 * extramaterial_paired, stage3.c:9275); outside it the reference's bridge reads cells no fill wrote,
 * and the engine rejects the batch with GMAPDP_EINVAL. */
typedef struct {
  int32_t qoffL;
  int32_t qoffR;
  int32_t rlengthL;
  int32_t rlengthR;
  int32_t glength;
  int32_t roffsetL;
  int32_t rev_roffsetR;
  int32_t goffset;
  gmapdp_coord_t chroffset;
  gmapdp_coord_t chrhigh;
  int32_t flags;          /* GMAPDP_WATSON | GMAPDP_JUMP_LATE | GMAPDP_SIMD */
  int32_t genestrand;
  int32_t extraband;      /* extraband_paired */
  int32_t dynprogindex;
  double defect_rate;
} gmapdp_cdna_problem;

/* Out-parameters of Dynprog_cdna_gap.  traceback_score is GMAPDP_UNSET where the reference leaves
 * it unwritten (the glength <= 1 and size-guard NULL returns).  When the bridge leaves anything but
 * a 9 x 9 block, the list carries a gap holder (Pairpool_push_gapholder, dynprog_cdna.c:1270) at
 * pairs[gap_index] with jump = genomejump and incompletep = 1. */
typedef struct {
  int32_t npairs;          /* 0 <=> NULL List_T */
  int32_t pair_offset;
  int32_t traceback_score;
  int32_t dynprogindex;
  int32_t incompletep;
  int32_t gap_index;       /* -1: no gap holder */
  int32_t gap_queryjump;
  int32_t pad_;
} gmapdp_cdna_result;

int gmapdp_cdna_gap_batch (gmapdp_ctx *ctx, const gmapdp_cdna_problem *problems, int n,
                           const char *qseq, const char *qseq_uc, size_t qbytes,
                           gmapdp_cdna_result *results, gmapdp_pair *pairs, size_t pair_capacity);
size_t gmapdp_cdna_pair_capacity (const gmapdp_cdna_problem *problems, int n);

/* One Dynprog_end5_splicejunction (end3p = 0, dynprog_end.c:1653) or Dynprog_end3_splicejunction
 * (end3p = 1, dynprog_end.c:2249) call: the known-splice-site end alignment Splicetrie_solve_end5/3
 * (splicetrie.c) run for each candidate far exon.  The query slice is qseq[qoff .. qoff+rlength) as
 * for an end-gap problem: end5's rev_rsequence points at its LAST character.  The junction string
 * (the caller's splicejunction buffer, built by Dynprog_make_splicejunction_5/3) is
 * jseq[joff .. joff+glength) in string order: end5's rev_gsequence points at its last character,
 * end3's gsequence at its first.  Junction characters must be A C G T or N.  Nosimd semantics
 * (Dynprog_standard + traceback_local_std), or with GMAPDP_SIMD the SIMD builds' (the
 * Dynprog_simd_8/16_upper/_lower triangles + traceback_local_8/16_upper/_lower; rlength > glength + 1
 * is then GMAPDP_EINVAL, as for the SIMD end gaps). */
typedef struct {
  int32_t qoff;
  int32_t joff;
  int32_t rlength;
  int32_t glength;
  int32_t roffset;          /* (rev_)roffset */
  int32_t goffset_anchor;   /* (rev_)goffset_anchor */
  int32_t goffset_far;      /* (rev_)goffset_far */
  int32_t contlength;
  int32_t flags;            /* GMAPDP_JUMP_LATE */
  int32_t genestrand;
  int32_t extraband;        /* extraband_end */
  int32_t end3p;
  int32_t dynprogindex;
  int32_t pad_;
  double defect_rate;
} gmapdp_sj_problem;

/* Out-parameters of the splice-junction end gaps.  NULL (npairs 0) with the size guard's values
 * (traceback_score 0, missscore -100, counters 0) for lengths outside 1..660 x 1..2000; NULL with
 * everything but dynprogindex GMAPDP_UNSET when the best endpoint scores below 0 (the reference
 * writes nothing then).  Otherwise the list's pairs[known_index] is the known-splice gap holder
 * (Pairpool_push_gapholder with knownp = true, jump = its genomejump). */
typedef struct {
  int32_t npairs;
  int32_t pair_offset;
  int32_t traceback_score;
  int32_t missscore;
  int32_t nmatches;
  int32_t nmismatches;
  int32_t nopens;
  int32_t nindels;
  int32_t dynprogindex;
  int32_t known_index;      /* -1 for NULL */
} gmapdp_sj_result;

int gmapdp_end_splicejunction_batch (gmapdp_ctx *ctx, const gmapdp_sj_problem *problems, int n,
                                     const char *qseq, const char *qseq_uc, size_t qbytes,
                                     const char *jseq, size_t jbytes,
                                     gmapdp_sj_result *results, gmapdp_pair *pairs, size_t pair_capacity);
size_t gmapdp_sj_pair_capacity (const gmapdp_sj_problem *problems, int n);

/* Dynprog_microexon_int (dynprog_single.c:900, replaced at stage3.c:9664): the
 * microexon search inside an intron, in two steps because the reference scores each candidate with the
 * host's MaxEnt model (Maxent_hr_*_prob, maxent_hr.c:27357-27600) between finding and choosing:
 *   1. gmapdp_microexon_search lists each problem's candidates in the reference's loop order (cL
 *      ascending, cR ascending, occurrences as BoyerMoore_nt lists them: descending), with the two
 *      splice sites (position, GMAPDP_MAXENT_* model) whose probabilities prob2 / prob3 it needs;
 *   2. the caller evaluates them (candidate k's prob2 at cand_probs[2 (cand_offset + k)], prob3 next);
 *   3. gmapdp_microexon_finish keeps the first candidate whose (float) prob2 + prob3 beats the best so
 *      far and emits make_microexon_pairs_double's list (dynprog_single.c:683): left piece, gap holder,
 *      microexon, gap holder, right piece.  The gap holders carry comp = '>' (cdna_direction > 0) or
 *      '<' and jump = genomejump; queryjump is 0.
 * rsequence = qseq + qoff (queryseq + roffset as stage3.c passes it); results[i].pair_offset is
 * problem i's slot in the pair arena (rlength + 2 records, gmapdp_microexon_pair_capacity). */
typedef struct {
  int32_t qoff;
  int32_t rlength;
  int32_t roffset;
  int32_t goffsetL;
  int32_t rev_goffsetR;
  int32_t cdna_direction;
  gmapdp_coord_t chroffset;
  gmapdp_coord_t chrhigh;
  int32_t watsonp;
  int32_t genestrand;
  int32_t dynprogindex;
  int32_t pad_;
} gmapdp_microexon_problem;

typedef struct {
  int32_t cL, cR;          /* lengths of the left and right pieces */
  int32_t candidate;       /* genomic offset of the microexon (goffsetM) */
  int32_t middlelength;
  gmapdp_coord_t pos2, pos3;  /* splice_pos of prob2 and prob3 (universal coordinates) */
  int32_t model2, model3;  /* GMAPDP_MAXENT_* */
} gmapdp_microexon_candidate;

typedef struct {
  int32_t ncandidates;
  int32_t dynprogindex;    /* after the call */
  int32_t microintrontype; /* intron.h: GTAG_FWD 0x20, GTAG_REV 0x04, NONINTRON 0 */
  int32_t npairs;          /* -1: NULL List_T */
  int64_t cand_offset;     /* first candidate in the candidate array */
  int64_t pair_offset;
  double bestprob2, bestprob3;
} gmapdp_microexon_result;

/* Step 1.  On GMAPDP_ESPACE (cand_capacity too small) *cands_needed holds the size required. */
int gmapdp_microexon_search (gmapdp_ctx *ctx, const gmapdp_microexon_problem *problems, int n,
                             const char *qseq, const char *qseq_uc, size_t qbytes, gmapdp_microexon_result *results,
                             gmapdp_microexon_candidate *candidates, size_t cand_capacity, size_t *cands_needed);
/* Step 3: results and candidates as step 1 left them; cand_probs as above. */
int gmapdp_microexon_finish (gmapdp_ctx *ctx, const gmapdp_microexon_problem *problems, int n,
                             const char *qseq, const char *qseq_uc, size_t qbytes,
                             const gmapdp_microexon_candidate *candidates, const double *cand_probs, size_t ncands,
                             gmapdp_microexon_result *results, gmapdp_pair *pairs, size_t pair_capacity);
size_t gmapdp_microexon_pair_capacity (const gmapdp_microexon_problem *problems, int n);

/* The GMAP drop-in's dispatcher batch in ONE round trip: gmapdp_dynprog_batch's calls,
 * gmapdp_microexon_search's calls and gmapdp_microexon_finish's calls (of other, earlier searches)
 * over one query arena -- one host-to-device copy, the kernels on the context's stream, one
 * device-to-host copy, one wait.  Each section means what the separate entry point's arguments
 * mean; a section with n = 0 is skipped.  The rare search that overflows the candidate pool is
 * rerun as gmapdp_microexon_search would (extra round trips).  GMAPDP_ESPACE: candidate_capacity too
 * small (*candidates_needed holds the size required); everything else is then still filled in.  Pair
 * arenas (pair_capacity, finish_pair_capacity, whole_pair_capacity) are checked up front against
 * gmapdp_*_pair_capacity of their calls: too small is GMAPDP_EINVAL, nothing run.  splice_probs = NULL / finish_probs = NULL: device MaxEnt (see "Device MaxEnt"). */
typedef struct {
  const gmapdp_single_problem *singles; int nsingle;
  const gmapdp_end_problem *ends; int nend;
  const gmapdp_genome_problem *genomes; int ngenome;
  const double *splice_probs; size_t nprobs;
  gmapdp_result *results;                    /* nsingle + nend */
  gmapdp_genome_result *genome_results;      /* ngenome */
  gmapdp_pair *pairs; size_t pair_capacity;
  const gmapdp_microexon_problem *searches; int nsearch;
  gmapdp_microexon_result *search_results;   /* nsearch */
  gmapdp_microexon_candidate *candidates; size_t candidate_capacity; size_t candidates_needed;
  const gmapdp_microexon_problem *finishes; int nfinish;
  const gmapdp_microexon_candidate *finish_candidates; const double *finish_probs; size_t nfinish_candidates;
  gmapdp_microexon_result *finish_results;   /* in: the searches' results; out: the choices */
  gmapdp_pair *finish_pairs; size_t finish_pair_capacity;
  const uint8_t *known_sites; size_t nknown; /* GMAPDP_KNOWN_SITES genome gaps' arena (else NULL, 0) */
  /* whole Dynprog_microexon_int calls: the search, the candidates' MaxEnt on the device and the choice,
   * all in this batch (the candidates stay on the device); whole_results as gmapdp_microexon_finish
   * leaves them, call i's pairs at the prefix sum of the earlier calls' rlength + 2
   * (gmapdp_microexon_pair_capacity) */
  const gmapdp_microexon_problem *wholes; int nwhole;
  gmapdp_microexon_result *whole_results;
  gmapdp_pair *whole_pairs; size_t whole_pair_capacity;
} gmapdp_mixed;
int gmapdp_mixed_batch (gmapdp_ctx *ctx, const char *qseq, const char *qseq_uc, size_t qbytes, gmapdp_mixed *m);

/* Device-resident microexon plan (the bench's path): descriptors uploaded once; the search is run at
 * plan time to size each call's candidate region, so gmapdp_microexon_plan_run writes candidates to
 * fixed regions (call i's at the prefix sum of the earlier calls' counts, device array
 * gmapdp_microexon_plan_device_candidates) and d_cand_probs (2 doubles per candidate, that order)
 * lines up with them.  what: 1 search, 2 finish, 3 both; qoff index the device arenas d_qseq /
 * d_qseq_uc; d_results (n records) and d_pairs (gmapdp_microexon_plan_pair_capacity records, call i's
 * at the prefix sum of rlength + 2) are the caller's device buffers. */
typedef struct gmapdp_microexon_plan gmapdp_microexon_plan;
int gmapdp_microexon_plan_create (gmapdp_ctx *ctx, const gmapdp_microexon_problem *problems, int n,
                                  const char *qseq, const char *qseq_uc, size_t qbytes,
                                  gmapdp_microexon_plan **plan);
size_t gmapdp_microexon_plan_candidates (const gmapdp_microexon_plan *plan);
size_t gmapdp_microexon_plan_pair_capacity (const gmapdp_microexon_plan *plan);
const gmapdp_microexon_candidate *gmapdp_microexon_plan_device_candidates (const gmapdp_microexon_plan *plan);
int gmapdp_microexon_plan_run (gmapdp_ctx *ctx, const gmapdp_microexon_plan *plan, const char *d_qseq,
                               const char *d_qseq_uc, const double *d_cand_probs, gmapdp_microexon_result *d_results,
                               gmapdp_pair *d_pairs, int what, void *stream);
void gmapdp_microexon_plan_destroy (gmapdp_microexon_plan *plan);

/* Stage-2 seeding: Oligoindex_hr_tally + Oligoindex_get_mappings
 * (oligoindex_hr.c:33849/34127) as Stage2_compute runs them for GMAP (stage2.c:6413-6501: one
 * 8-mer oligoindex, coveredp all false).  One problem = one (query, genomic window) pair:
 * queryuc_ptr = qseq_uc + qoff (upper-case query), the window [chrstart, chrend) of the chromosome
 * at chroffset..chrhigh on the plus (plusp) or minus strand.  minor selects
 * Oligoindex_array_new_minor's index (diag_lookback 60, suffnconsecutive 10) instead of the major
 * one (120, 20).  Domain: querylength > 8 (Oligoindex_set_inquery leaves stale state below that)
 * and at most 16384 distinct query 8-mers. */
typedef struct {
  int32_t qoff;
  int32_t querylength;
  uint32_t chrstart;
  uint32_t chrend;
  gmapdp_coord_t chroffset;
  gmapdp_coord_t chrhigh;
  int32_t plusp;
  int32_t minor;
} gmapdp_oligo_problem;

/* Per problem: *totalpositions, *maxnconsecutive, *oned_matrix_p (0 where the reference leaves it
 * unwritten: chrend <= chrstart) and the diagonals list (Diagpool_push records, list order) at
 * diagonals[4 * diag_offset ...]: {diagonal, querystart, queryend, nconsecutive} each.  Per query
 * position q: npositions[qoff + q] (0 without a full 8-mer or without hits) and
 * mappings[qoff + q], the index in `positions` of mappings[q][0] (-1 without hits); the problem's
 * table occupies positions[table_offset ...].  The batch's table arena stays below 2^31 entries
 * (GMAPDP_EINVAL otherwise; split the batch). */
typedef struct {
  int32_t totalpositions;
  int32_t maxnconsecutive;
  int32_t oned_matrix_p;
  int32_t ndiagonals;
  int64_t table_offset;
  int64_t diag_offset;
} gmapdp_oligo_result;

/* npositions, mappings: qbytes entries each (indexed like the query arena); mappings are absolute
 * indexes into `positions`.  Each problem writes its own query slice [qoff, qoff + querylength), so the
 * problems' slices must be disjoint (GMAPDP_EINVAL otherwise). */
int gmapdp_oligo_mappings_batch (gmapdp_ctx *ctx, const gmapdp_oligo_problem *problems, int n,
                                 const char *qseq_uc, size_t qbytes, gmapdp_oligo_result *results,
                                 int32_t *npositions, int32_t *mappings, uint32_t *positions,
                                 size_t positions_capacity, int32_t *diagonals, size_t diagonal_capacity);
/* Table entries / diagonal records (4 x int32) a batch may need. */
size_t gmapdp_oligo_positions_capacity (const gmapdp_oligo_problem *problems, int n);
size_t gmapdp_oligo_diagonal_capacity (const gmapdp_oligo_problem *problems, int n);
/* Device-resident path (bench / pipelined callers): plan once (distinct 8-mers, launch classes,
 * table / diagonal / scratch offsets; the descriptors are uploaded), then run asynchronously on
 * `stream` (hipStream_t; NULL = the context's stream) against a device-resident upper-case query
 * arena.  d_results has n entries in problem order; d_npositions / d_mappings are indexed like the
 * query arena, and a device mapping is relative to its problem's table: mappings[q][0] is
 * d_positions[table_offset + d_mappings[qoff + q]] (so the table arena may pass 2^31 entries);
 * d_positions / d_diagonals hold the plan's capacities.  A problem that needs more hit-list, table or
 * diagonal room than the layout gave it reports oned_matrix_p = -1 and writes nothing else. */
typedef struct gmapdp_oligo_plan gmapdp_oligo_plan;
int gmapdp_oligo_plan_create (gmapdp_ctx *ctx, const gmapdp_oligo_problem *problems, int n, const char *qseq_uc,
                              size_t qbytes, gmapdp_oligo_plan **plan);
size_t gmapdp_oligo_plan_positions_capacity (const gmapdp_oligo_plan *plan);
size_t gmapdp_oligo_plan_diagonal_capacity (const gmapdp_oligo_plan *plan);
int gmapdp_oligo_plan_nlaunches (const gmapdp_oligo_plan *plan);
int gmapdp_oligo_plan_run (gmapdp_ctx *ctx, const gmapdp_oligo_plan *plan, const char *d_qseq_uc,
                           gmapdp_oligo_result *d_results, int32_t *d_npositions, int32_t *d_mappings,
                           uint32_t *d_positions, int32_t *d_diagonals, void *stream);
void gmapdp_oligo_plan_destroy (gmapdp_oligo_plan *plan);

/* Stage2_compute (stage2.c:6325) as GMAP's update_stage3middle_list calls it (gmap.c:1208-1215):
 * query_offset 0, genestrand 0, proceed_pctcoverage 0.3, the major oligoindex array (8-mers,
 * diag_lookback 120, suffnconsecutive 20), localp, skip_repetitive_p, favor_right_p false,
 * max_nalignments 10; Stage2_setup (gmap.c:6544) without cross-species canonical scoring, without SNPs,
 * STANDARD mode, sufflookback 60, nsufflookback 5.  queryseq_ptr = qseq + qoff (case as given, the
 * Pair cdna), queryuc_ptr = qseq_uc + qoff.  Domain as for gmapdp_oligo_problem: querylength > 8, and
 * genomic positions below 2^31 (Pairpool_push drops negative ones; the engine does not model that). */
typedef struct {
  int32_t qoff;
  int32_t querylength;
  uint32_t chrstart;
  uint32_t chrend;
  gmapdp_coord_t chroffset;
  gmapdp_coord_t chrhigh;
  int32_t plusp;
  int32_t splicingp;       /* Stage2_setup's splicingp_in (novelsplicingp || knownsplicingp) */
  int32_t maxintronlen;    /* Stage2_setup's maxintronlen_in */
  int32_t pad_;
} gmapdp_stage2_problem;

/* Per call: the returned List_T of Stage2_T, in list order, as nresults path records starting at
 * paths[path_offset]; each record's pairs are its Stage2_middle list (all_starts / all_ends are NULL
 * in this build of the reference).  status: 0 no positions, 1 the coverage filter declined
 * (stage2.c:6526), 2 chained; negative: GMAPDP internal (never returned by gmapdp_stage2_batch). */
typedef struct {
  int32_t nresults;
  int32_t npaths;          /* paths traced before Stage2_filter_unique */
  int32_t ncovered;        /* Diag_update_coverage's ncovered */
  int32_t status;
  int32_t diag_querystart; /* Diag_compute_bounds' query bounds (status 2) */
  int32_t diag_queryend;
  int32_t path_offset;
  int32_t npairs;          /* pair records of all nresults paths */
} gmapdp_stage2_result;

typedef struct {
  int64_t pair_offset;     /* first record in the pair arena */
  int32_t npairs;
  int32_t pad_;
} gmapdp_path;

/* One Pair_T of a stage-2 path (convert_to_nucleotides): querypos, genomepos, cdna, comp ('|'),
 * genome, genomealt; a gap holder (Pairpool_push_gapholder) has querypos = genomepos = -1, its
 * queryjump / genomejump, and blanks; ordinary pairs carry queryjump = genomejump = 0. */
typedef struct {
  int32_t querypos;
  int32_t genomepos;
  int32_t queryjump;
  int32_t genomejump;
  char cdna;
  char comp;
  char genome;
  char genomealt;
} gmapdp_path_pair;

#define GMAPDP_ESPACE (-6)  /* an output arena is too small: *_needed say how large it must be */

/* n Stage2_compute calls.  results: n entries.  paths / pairs: caller arenas of path_cap / pair_cap
 * records; on GMAPDP_ESPACE nothing else is valid and *paths_needed / *pairs_needed hold the sizes the
 * call needs (call again with larger arenas).  On success they hold the records used. */
int gmapdp_stage2_batch (gmapdp_ctx *ctx, const gmapdp_stage2_problem *problems, int n, const char *qseq,
                         const char *qseq_uc, size_t qbytes, gmapdp_stage2_result *results, gmapdp_path *paths,
                         size_t path_cap, gmapdp_path_pair *pairs, size_t pair_cap, size_t *paths_needed,
                         size_t *pairs_needed);

/* Device-resident Stage2_compute (bench / pipelined callers): plan once (the seeding plan, the
 * chaining scratch sized from one seeding run at plan time, output pools), then run asynchronously on
 * `stream` against device-resident query arenas.  what: 1 seeding only, 2 chaining only (after a
 * seeding run), 3 both.  d_results: n entries in problem order; paths and pairs stay in the plan's
 * pools (gmapdp_stage2_plan_outputs: device pointers and the counters {scratch, paths, pairs} bytes /
 * records used); a result with status -2 did not fit them.  Profiling: what = 4, 8 or 16 re-runs one
 * chaining kernel alone (s2a, the s2b sweep, s2c) over the scratch of a previous full run. */
typedef struct gmapdp_stage2_plan gmapdp_stage2_plan;
int gmapdp_stage2_plan_create (gmapdp_ctx *ctx, const gmapdp_stage2_problem *problems, int n, const char *qseq,
                               const char *qseq_uc, size_t qbytes, gmapdp_stage2_plan **plan);
int gmapdp_stage2_plan_run (gmapdp_ctx *ctx, const gmapdp_stage2_plan *plan, const char *d_qseq,
                            const char *d_qseq_uc, gmapdp_stage2_result *d_results, int what, void *stream);
int gmapdp_stage2_plan_outputs (const gmapdp_stage2_plan *plan, gmapdp_path **d_paths, gmapdp_path_pair **d_pairs,
                                unsigned long long **d_counters, size_t *scratch_bytes);
/* The outputs of a finished gmapdp_stage2_plan_run (chaining) on `stream` (NULL = the context's stream;
 * synchronised here), in gmapdp_stage2_batch's format: n results copied from d_results, and the path
 * and pair records into host arenas of path_cap / pair_cap records (GMAPDP_ESPACE with *_needed when
 * they are too small).  A result with status -2 overflowed the plan's pools or its seeding layout. */
int gmapdp_stage2_plan_fetch (gmapdp_ctx *ctx, const gmapdp_stage2_plan *plan, const gmapdp_stage2_result *d_results,
                              void *stream, gmapdp_stage2_result *results, gmapdp_path *paths, size_t path_cap,
                              gmapdp_path_pair *pairs, size_t pair_cap, size_t *paths_needed, size_t *pairs_needed);
/* The seeding results of the plan's last run (n, problem order; table_offset / diag_offset index the plan's
 * own arenas), synchronising `stream` (NULL = the context's). */
int gmapdp_stage2_plan_seeding_results (gmapdp_ctx *ctx, const gmapdp_stage2_plan *plan, void *stream,
                                        gmapdp_oligo_result *out);
/* How many of the plan's calls seed with 16-bit and with 32-bit counters (after the plan's sizing run
 * moved every call with fewer than 2^16 hits to the 16-bit class). */
int gmapdp_stage2_plan_seeding_classes (const gmapdp_stage2_plan *plan, int *n16, int *n32);
/* The compact stream of a finished chaining run's path pairs (gmapdp_plan_compact_pairs' format, 21-B RAW
 * ops: gmapdp_path_pair records with a jump or a negative position): one list per record of the plan's path
 * pool (*path_cap of them; records past the pool's count are empty lists).  d_offsets: path_cap + 1 uint64
 * (device), exclusive offsets and the total; d_out NULL sizes only, else at least
 * gmapdp_stage2_plan_compact_bound bytes.  gmapdp_expand_path_pairs restores the records on the host, each
 * path's npairs at its pair_offset (the path records as gmapdp_stage2_plan_fetch returns them). */
size_t gmapdp_stage2_plan_compact_bound (const gmapdp_stage2_plan *plan, size_t *path_cap);
int gmapdp_stage2_plan_compact_pairs (gmapdp_ctx *ctx, const gmapdp_stage2_plan *plan, uint8_t *d_out,
                                      uint64_t *d_offsets, void *stream);
int gmapdp_expand_path_pairs (const uint8_t *stream, const uint64_t *offsets, int npaths, const gmapdp_path *paths,
                              gmapdp_path_pair *out, int nthreads);
void gmapdp_stage2_plan_destroy (gmapdp_stage2_plan *plan);

/* Create a context on HIP device `device`.  mode = Mode_T (mode.h:5;
 * 0 = STANDARD).  user_* mirror Dynprog_single_setup. */
int gmapdp_create (gmapdp_ctx **ctx, int device, int mode,
                   int user_open, int user_extend, int user_dynprog_p);
void gmapdp_destroy (gmapdp_ctx *ctx);
/* gmapdp_create with flags, for callers that run several contexts at once (the GMAP drop-in's
 * dispatcher threads): GMAPDP_CTX_ONE_STREAM creates no side streams (a process has few hardware
 * queues, GPU_MAX_HW_QUEUES, and streams beyond them share one and serialise); GMAPDP_CTX_PRIO_HIGH /
 * _LOW create the context's stream at the device's highest / lowest priority; GMAPDP_CTX_BLOCKING_SYNC
 * makes the synchronous batch calls wait without spinning; GMAPDP_CTX_POLL_SYNC makes them poll the
 * batch's completion every GMAPDP_POLL_US microseconds (default 10) and sleep in between. */
#define GMAPDP_CTX_ONE_STREAM 0x1
#define GMAPDP_CTX_PRIO_HIGH  0x2
#define GMAPDP_CTX_PRIO_LOW   0x4
#define GMAPDP_CTX_BLOCKING_SYNC 0x8  /* batch calls sleep on a blocking-sync event instead of spinning */
#define GMAPDP_CTX_POLL_SYNC 0x10     /* batch calls poll their completion, sleeping between polls */
/* Plans spread their launch classes (longest-processing-time first) over the caller's stream and two
 * side streams instead of three: for a caller that keeps the process's fourth hardware queue for other
 * work of its own, e.g. Stage2_compute on its own stream beside the plan (bench.py), so that no stream
 * receives two of the plan's lists. */
#define GMAPDP_CTX_TWO_SIDES 0x20
int gmapdp_create_ex (gmapdp_ctx **ctx, int device, int mode, int user_open, int user_extend, int user_dynprog_p,
                      int flags);
/* Use `owner`'s HBM-resident genome in `ctx` (no copy; same device).  `owner` must outlive every
 * context sharing its genome and keep that genome until they are done. */
int gmapdp_share_genome (gmapdp_ctx *ctx, const gmapdp_ctx *owner);
/* A packed genome resident in one device's HBM, independent of any context: upload once, then let any
 * number of contexts read it (gmapdp_use_dgenome; no copy).  The drop-in keeps one per GMAP Genome_T
 * (a -g run over a multi-sequence file has several).  Destroy it only after every context using it is
 * done with it. */
/* Grow the context's staging and scratch buffers to `bytes` each (4x for the direction and chaining
 * scratch) now, so that a long-running caller does not grow them later: a buffer's growth frees the old
 * one, and hipFree waits for the whole device, stalling every context's streams.  what: GMAPDP_RESERVE_DP
 * (single / end / genome-gap batches), _AUX (microexon and cDNA-gap batches), _STAGE2 (Stage2_compute and
 * seeding batches). */
#define GMAPDP_RESERVE_DP     0x1
#define GMAPDP_RESERVE_AUX    0x2
#define GMAPDP_RESERVE_STAGE2 0x4
int gmapdp_reserve (gmapdp_ctx *ctx, size_t bytes, int what);
typedef struct gmapdp_dgenome gmapdp_dgenome;
int gmapdp_dgenome_create (int device, const uint32_t *blocks, size_t nwords, uint64_t length, gmapdp_dgenome **g);
void gmapdp_dgenome_destroy (gmapdp_dgenome *g);
int gmapdp_use_dgenome (gmapdp_ctx *ctx, const gmapdp_dgenome *g);

/* Words needed for a packed genome of `length` nt ((len+31)/32*3 + 4). */
size_t gmapdp_genome_words (uint64_t length);
/* Pack characters into .genomecomp blocks (A=0 C=1 G=2 T=3, 32 nt per
 * {high, low, flags} triple, non-ACGT flagged).  `blocks` must hold
 * gmapdp_genome_words(length) words. */
int gmapdp_pack_genome (const char *seq, uint64_t length, uint32_t *blocks);
/* Upload packed blocks (e.g. Genome_blocks(genome) of a loaded GMAP
 * genome) to HBM.  nwords as returned by gmapdp_genome_words.  Genomes of
 * 2^32 nt or more (gmapl, 64-bit Univcoord_T) are GMAPDP_EINVAL. */
int gmapdp_set_genome (gmapdp_ctx *ctx, const uint32_t *blocks, size_t nwords, uint64_t length);

/* Run n Dynprog_single_gap problems.  Host arrays in, host arrays out
 * (the engine stages them through pinned device buffers).  `pairs` must
 * have room for gmapdp_single_pair_capacity(problems, n) records; result
 * i's pairs are pairs[results[i].pair_offset .. +npairs). */
int gmapdp_single_gap_batch (gmapdp_ctx *ctx, const gmapdp_single_problem *problems, int n,
                             const char *qseq, const char *qseq_uc, size_t qbytes,
                             gmapdp_result *results, gmapdp_pair *pairs, size_t pair_capacity);
size_t gmapdp_single_pair_capacity (const gmapdp_single_problem *problems, int n);

/* Run n Dynprog_end5_gap / Dynprog_end3_gap problems (same conventions).
 * NULL results follow dynprog_end.c: traceback_score 0; dynprogindex is left
 * unchanged on the early returns (rlength <= 0, end5 goffset < 0,
 * glength <= 0) and advanced otherwise. */
int gmapdp_end_gap_batch (gmapdp_ctx *ctx, const gmapdp_end_problem *problems, int n,
                          const char *qseq, const char *qseq_uc, size_t qbytes,
                          gmapdp_result *results, gmapdp_pair *pairs, size_t pair_capacity);
size_t gmapdp_end_pair_capacity (const gmapdp_end_problem *problems, int n);

/* Device-resident path for pipelined callers and throughput measurement.
 * gmapdp_plan_single resolves penalties, bands and launch classes once on
 * the host (problems resolved on the host -- the size guard -- are written
 * to host_results immediately) and uploads the descriptors.  The upload
 * may still be in flight when the create call returns (the host goes on to
 * its next work); the plan's first run waits for it, so nothing changes for
 * the caller.  gmapdp_plan_run then launches asynchronously on `stream` (a hipStream_t;
 * NULL = the context's stream) against device-resident query arenas; GPU
 * results land in d_results[gmapdp_plan_dev_index(plan, i)] and pairs in
 * d_pairs (capacity gmapdp_plan_pair_capacity). */
typedef struct gmapdp_plan gmapdp_plan;
/* Mixed batch: host_results has nsingle + nend entries (singles first). */
int gmapdp_plan_create (gmapdp_ctx *ctx, const gmapdp_single_problem *singles, int nsingle,
                        const gmapdp_end_problem *ends, int nend, gmapdp_result *host_results,
                        gmapdp_plan **plan);
int gmapdp_plan_single (gmapdp_ctx *ctx, const gmapdp_single_problem *problems, int n,
                        gmapdp_result *host_results, gmapdp_plan **plan);
/* All three families: host_results has nsingle + nend entries, host_genome_results
 * ngenome entries.  Launch members number the problems singles, ends, genome gaps. */
int gmapdp_plan_create_all (gmapdp_ctx *ctx, const gmapdp_single_problem *singles, int nsingle,
                            const gmapdp_end_problem *ends, int nend, const gmapdp_genome_problem *genomes,
                            int ngenome, gmapdp_result *host_results, gmapdp_genome_result *host_genome_results,
                            gmapdp_plan **plan);
/* Device buffers of the genome-gap problems: the splice-probability arena and the
 * results (indexed by gmapdp_plan_genome_dev_index).  Required before running a plan
 * that has genome-gap problems on the GPU. */
int gmapdp_plan_bind_genome (gmapdp_plan *plan, const double *d_splice_probs, gmapdp_genome_result *d_genome_results);
/* The same with device MaxEnt: d_splice_probs (gmapdp_genome_prob_entries doubles) is scratch that each
 * genome-gap launch class fills for its own problems on its own stream before its fill kernel. */
int gmapdp_plan_bind_genome_maxent (gmapdp_ctx *ctx, gmapdp_plan *plan, double *d_splice_probs,
                                    gmapdp_genome_result *d_genome_results);
int gmapdp_plan_genome_gpu_problems (const gmapdp_plan *plan);
int gmapdp_plan_genome_dev_index (const gmapdp_plan *plan, int j);
/* 0: Dynprog_single_gap / end-gap kernel (one problem per wave), 1: Dynprog_genome_gap
 * kernel, 2: packed single/end-gap kernel (64/S narrow-band problems per wave; for these
 * gmapdp_plan_launch_info reports R = S and lds = the per-problem LDS slot), 3: SIMD-build
 * single gaps (sx), 4: SIMD-build end gaps (uxe), 5: SIMD-build genome gaps (uxg),
 * 7: single/end gaps whose band is wider than the query (lanes over query rows) */
int gmapdp_plan_launch_kind (const gmapdp_plan *plan, int li);
size_t gmapdp_plan_pair_capacity (const gmapdp_plan *plan);
int gmapdp_plan_gpu_problems (const gmapdp_plan *plan);
int gmapdp_plan_dev_index (const gmapdp_plan *plan, int i);
int gmapdp_plan_nlaunches (const gmapdp_plan *plan);
int gmapdp_plan_run (gmapdp_ctx *ctx, const gmapdp_plan *plan, const char *d_qseq, const char *d_qseq_uc,
                     gmapdp_result *d_results, gmapdp_pair *d_pairs, void *stream);
/* The compact pair stream (run-length ops plus one character code per record; the host expands
 * it into the same records -- Pair_T lists -- with gmapdp_expand_pairs).  After gmapdp_plan_run on `stream`:
 * each GPU problem's list (dev slots 0..gmapdp_plan_gpu_problems - 1, then the genome gaps' slots) becomes a
 * byte stream; d_offsets (gpu problems + genome gpu problems + 1 uint64, device) receives the exclusive
 * offsets and the total.  d_out NULL: the offsets only (to size a copy); else at least
 * gmapdp_plan_compact_bound bytes.  Stream format: pc_kernel.hip. */
size_t gmapdp_plan_compact_bound (const gmapdp_plan *plan);
int gmapdp_plan_compact_pairs (gmapdp_ctx *ctx, const gmapdp_plan *plan, const gmapdp_result *d_results,
                               const gmapdp_pair *d_pairs, uint8_t *d_out, uint64_t *d_offsets, void *stream);
/* Host: problem i's ops (stream[offsets[i], offsets[i + 1])) back to its npairs[i] records at
 * out[pair_offsets[i]], on nthreads host threads (0: the plan builders' default).  GMAPDP_EINVAL when a
 * problem's ops do not decode to exactly its records. */
int gmapdp_expand_pairs (const uint8_t *stream, const uint64_t *offsets, int n, const int32_t *npairs,
                         const int64_t *pair_offsets, gmapdp_pair *out, int nthreads);
/* Per-launch-class access (one kernel launch per class; for profiling). */
int gmapdp_plan_launch_info (const gmapdp_plan *plan, int li, int *R, int *dirs_lds, int *count, size_t *lds);
/* Launch classes are spread over the caller's stream (0) and three side streams (1..3),
 * longest-processing-time first; launches are numbered in issue order.  is_tail: 1 if the
 * launch runs on a side stream. */
int gmapdp_plan_launch_stream (const gmapdp_plan *plan, int li);
int gmapdp_plan_launch_is_tail (const gmapdp_plan *plan, int li);
/* Original problem indices of launch li (count entries, launch order). */
int gmapdp_plan_launch_members (const gmapdp_plan *plan, int li, int *problem_indices);
int gmapdp_plan_run_launch (gmapdp_ctx *ctx, const gmapdp_plan *plan, int li, const char *d_qseq,
                            const char *d_qseq_uc, gmapdp_result *d_results, gmapdp_pair *d_pairs, void *stream);
/* The same launch's kernel alone: a genome-gap class's device-MaxEnt prologue is not re-run (the splice
 * probabilities a previous full run computed stay in the bound arena).  For timing one kernel's launches. */
int gmapdp_plan_run_launch_kernel (gmapdp_ctx *ctx, const gmapdp_plan *plan, int li, const char *d_qseq,
                                   const char *d_qseq_uc, gmapdp_result *d_results, gmapdp_pair *d_pairs,
                                   void *stream);
void gmapdp_plan_destroy (gmapdp_plan *plan);
/* The context's HIP stream (hipStream_t). */
void *gmapdp_stream (gmapdp_ctx *ctx);

void gmapdp_compute_bands (int *lband, int *uband, int rlength, int glength, int extraband, int widebandp);

/* Last error message for this context (static storage). */
const char *gmapdp_last_error (gmapdp_ctx *ctx);

#ifdef __cplusplus
}
#endif
#endif
