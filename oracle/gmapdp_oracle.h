/* oracle/gmapdp_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the reference GMAP 2024-02-22 Dynprog_* path, written in
 * plain C from a reading of /root/reference/src (never copied).  It is the
 * checker for the HIP engine: only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load it.  The product (libgmapdp.so) never
 * links or calls it.
 *
 * Parity pinning: tests/test_oracle_vs_ref.py compares every entry point
 * against the reference's own objects (oracle/_ref/librefdp_*.so, built by
 * oracle/ref.mk) on seeded random problems, and against the committed golden
 * vectors in tests/golden/ (generated from those objects by
 * tests/golden/make_golden.py).
 */
#ifndef GMAPDP_ORACLE_H
#define GMAPDP_ORACLE_H

#ifdef __cplusplus
extern "C" {
#endif

/* One Pair_T of the reference (pairdef.h:8-42), flattened: the fields a
   Dynprog_* call sets.  Same layout as refharness.c RefPair. */
typedef struct {
  int querypos;
  int genomepos;
  int queryjump;
  int genomejump;
  int dynprogindex;
  char cdna, comp, genome, genomealt;
  int gapp;
} OrcPair;

/* mode: Mode_T of mode.h:5 (0 = STANDARD). */
int orc_init (int mode, int user_open, int user_extend, int user_dynprog_p);

/* The genome as unpacked characters (A,C,G,T,N), i.e. what
   Genome_get_char / uncompress_mmap return for each position. */
int orc_set_genome (const char *genome, unsigned int length);

/* Dynprog_single_gap (dynprog_single.c:429), nosimd semantics.
   scalars[0..5] = dynprogindex(after), finalscore, nmatches, nmismatches,
   nopens, nindels.  Returns npairs (list order), or -1 for a NULL list. */
int orc_set_simd (int simd);
int orc_single_gap (const char *rsequence, const char *rsequenceuc, int rlength, int glength,
                    int roffset, int goffset, unsigned int chroffset, unsigned int chrhigh,
                    int watsonp, int genestrand, int jump_late_p, int extraband_single, int widebandp,
                    double defect_rate, int dynprogindex, int *scalars, OrcPair *out, int max_pairs);

/* Dynprog_end5_gap (end3p = 0) / Dynprog_end3_gap (end3p = 1)
   (dynprog_end.c:1294/1924), nosimd semantics.  The reference's
   (rev_)rsequence pointer is qbuf + qpos (end5: the LAST query character).
   endalign: 0 QUERYEND_GAP, 1 QUERYEND_INDELS, 2 QUERYEND_NOGAPS, 3 BEST_LOCAL. */
int orc_end_gap (int end3p, const char *qbuf, const char *qucbuf, int qpos, int rlength, int glength,
                 int roffset, int goffset, unsigned int chroffset, unsigned int chrhigh,
                 int watsonp, int genestrand, int jump_late_p, int extraband_end, double defect_rate,
                 int endalign, int require_pos_score_p, int dynprogindex, int *scalars, OrcPair *out,
                 int max_pairs);

/* Dynprog_end5_splicejunction (end3p = 0) / Dynprog_end3_splicejunction (end3p = 1)
   (dynprog_end.c:1653/2249), nosimd semantics.  (rev_)rsequence = qbuf + qpos as for orc_end_gap;
   the junction string (rev_)gsequence = jbuf + jpos (end5: its LAST character).
   scalars[0..7] = dynprogindex(after), traceback_score, missscore, nmatches, nmismatches, nopens,
   nindels, list index of the known-splice gap holder (-1 none); unwritten ones are INT_MIN.
   Returns npairs or -1 for NULL. */
int orc_end_splicejunction (int end3p, const char *qbuf, const char *qucbuf, int qpos, const char *jbuf, int jpos,
                            int rlength, int glength, int roffset, int goffset_anchor, int goffset_far,
                            int genestrand, int jump_late_p, int extraband_end, double defect_rate, int contlength,
                            int dynprogindex, int *scalars, OrcPair *out, int max_pairs);

/* Genome_get_segment_right / _left (genome.c:11023/11079) over the oracle
   genome (no alternate genome: segmentalt = segment). */
int orc_get_segment (int rightp, unsigned int pos, int length, unsigned int chrbound, int revcomp,
                     char *segment, char *segmentalt);

/* Dynprog_standard (dynprog.c:1268) on explicit segments; exported so the
   fill can be checked cell by cell.  matrix: (glength+1)*(rlength+1) int32,
   dirs: 3 planes of the same size (nogap, Egap, Fgap), [c][r] layout. */
int orc_standard_fill (const char *rsequence, const char *gsequence, const char *gsequence_alt,
                       int rlength, int glength, int mismatchtype, int open, int extend,
                       int lband, int uband, int jump_late_p, int revp, int saturation,
                       int upperp, int lowerp, int *matrix, signed char *dirs);

/* Dynprog_genome_gap (dynprog_genome.c:3288), nosimd semantics, no splicing
   IIT.  flags: 1 watsonp, 2 jump_late_p, 8 halfp, 16 finalp.  left_probs /
   right_probs: glengthL / glengthR MaxEnt probabilities at the positions of
   orc_genome_splice_sites (the host's Maxent_hr_*_prob values).
   scalars[0..9] = dynprogindex(after), traceback_score, nmatches,
   nmismatches, nopens, nindels, new_leftgenomepos, new_rightgenomepos,
   exonhead, introntype (INT_MIN where the reference leaves an out-parameter
   unwritten); dscalars[0..1] = left_prob, right_prob. */
/* Known-site flags (GMAPDP_KNOWN_SITES layout) for the following orc_genome_gap calls; NULL: none. */
void orc_set_known (const unsigned char *known);

int orc_genome_gap (const char *rsequence, const char *rsequenceuc, int rlength, int glengthL, int glengthR,
                    int roffset, int goffsetL, int rev_goffsetR, unsigned int chroffset, unsigned int chrhigh,
                    int cdna_direction, int flags, int genestrand, int extraband_paired, double defect_rate,
                    int maxpeelback, int dynprogindex, const double *left_probs, const double *right_probs,
                    int *scalars, double *dscalars, OrcPair *out, int max_pairs);
/* splice-site position + model (0 donor, 1 acceptor, 2 antidonor, 3
   antiacceptor) of each probability-array entry */
int orc_genome_splice_sites (int glengthL, int glengthR, int goffsetL, int rev_goffsetR, unsigned int chroffset,
                             unsigned int chrhigh, int cdna_direction, int watsonp, unsigned int *posL, int *modelL,
                             unsigned int *posR, int *modelR);
/* intron_score_setup's six arrays: [sense, antisense, either][prelim, final][64] */
int orc_intron_scores (int *out3x2x64);

int orc_pairdistance (int mismatchtype, short *out128x128);
int orc_consistent (int genestrand, unsigned char *out128x128);

/* Dynprog_cdna_gap (dynprog_cdna.c:787), nosimd or SIMD semantics (orc_set_simd).
   rsequenceL = qbuf + qposL, rev_rsequenceR = qbuf + qposR (the R piece's last character).
   scalars[0..2] = dynprogindex(after), traceback_score (INT_MIN when unwritten), incompletep.
   Returns npairs, -1 for NULL, -3 outside the domain (rlengthL == rlengthR >= glength). */
int orc_cdna_gap (const char *qbuf, const char *qucbuf, int qposL, int qposR, int rlengthL, int rlengthR,
                  int glength, int roffsetL, int rev_roffsetR, int goffset, unsigned int chroffset,
                  unsigned int chrhigh, int watsonp, int genestrand, int jump_late_p, int extraband_paired,
                  double defect_rate, int dynprogindex, int *scalars, OrcPair *out, int max_pairs);

/* Dynprog_microexon_int (dynprog_single.c:900; microexon_oracle.c).  rsequence / rsequenceuc: the
   query slice (stage3.c:9664 passes queryseq + querydp5 and roffset = querydp5).
   orc_microexon_candidates lists the candidates in the reference's loop order: cands[4 k..] = cL, cR,
   candidate, middlelength; positions / models [2 k..] = the splice sites of prob2 and prob3 (models
   as orc_genome_splice_sites).  Returns their number, -1 when cap is too small, -2 for cdna_direction 0.
   orc_microexon_int takes those probabilities (cand_probs[2 k], [2 k + 1], the host's
   Maxent_hr_*_prob values).  scalars[0..1] = dynprogindex(after), microintrontype; dscalars[0..1] =
   bestprob2, bestprob3.  Returns npairs (list order) or -1 for NULL. */
int orc_microexon_candidates (const char *rsequence, const char *rsequenceuc, int rlength, int goffsetL,
                              int rev_goffsetR, int cdna_direction, unsigned int chroffset, unsigned int chrhigh,
                              int watsonp, int *cands, unsigned int *positions, int *models, int cap);
int orc_microexon_int (const char *rsequence, const char *rsequenceuc, int rlength, int roffset, int goffsetL,
                       int rev_goffsetR, int cdna_direction, unsigned int chroffset, unsigned int chrhigh,
                       int watsonp, int genestrand, int dynprogindex, const double *cand_probs, int *scalars,
                       double *dscalars, OrcPair *out, int max_pairs);

/* The genome set by orc_set_genome. */
const char *orc_genome_seq (unsigned int *length);

/* maxent_oracle.c: Maxent_hr_*_prob (model GMAPDP_MAXENT_*, maxent_hr.c:27357-27652) over the genome of
   orc_set_genome, from the tables tools/make_maxent_tables.py wrote (orc_maxent_load: 0 on success). */
int orc_maxent_load (const char *path);
double orc_maxent (int model, unsigned long long splice_pos, unsigned long long chroffset);
void orc_maxent_batch (const int *models, const unsigned long long *positions, unsigned long long chroffset, int n,
                       double *out);

/* Stage-2 seeding (stage2_oracle.c): Oligoindex_hr_tally + Oligoindex_get_mappings as
   Stage2_compute runs them for GMAP; same arguments and outputs as refh_oligo_mappings
   (oracle/refharness.c).  Returns the positions written, -1 when a capacity is too small, -3 for
   querylength <= 8 (outside the reference's defined behaviour), -4 for a diagonal past the
   genomicdiag array (the reference asserts). */
int orc_oligo_mappings (const char *queryuc, int querylength, unsigned int chrstart, unsigned int chrend,
                        unsigned int chroffset, unsigned int chrhigh, int plusp, int minor, int *npositions,
                        unsigned int *positions, int pos_cap, int *scalars, int *diags, int diag_cap);

/* Stage2_compute (stage2.c:6325) as GMAP calls it (stage2_chain_oracle.c): the seeding above, then
   Diag_update_coverage, the proceed test, Diag_compute_bounds, align_compute_lookback,
   convert_to_nucleotides and Stage2_filter_unique.  Same arguments and outputs as
   refh_stage2_compute (oracle/refharness.c): the kept results' middle lists in `pairs`, result i at
   pairs[paths[2 i]] with paths[2 i + 1] records.  scalars[0..5] = results kept, paths traced,
   ncovered, exit (0 no positions, 1 coverage filter, 2 chained), diag_querystart, diag_queryend.
   Returns the number of results, -1 when a capacity is too small, the seeding's codes below 0. */
int orc_stage2_compute (const char *queryseq, const char *queryuc, int querylength, unsigned int chrstart,
                        unsigned int chrend, unsigned int chroffset, unsigned int chrhigh, int plusp, int splicingp,
                        int maxintronlen, int *scalars, int *paths, int path_cap, OrcPair *pairs, int pair_cap);

#ifdef __cplusplus
}
#endif
#endif
