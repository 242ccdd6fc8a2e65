/* include/gmapdp_dynprog.h -- reference-signature drop-in for GMAP's Dynprog_* entry points.
 *
 * For a GMAP build only: include it with GMAP's src/ on the include path
 * (it needs GMAP's List_T, Pair_T, Pairpool_T, Genome_T, Dynprog_T types).
 * The implementation is gmap-2024_amd/shim/gmapdp_gmap_shim.c; INTEGRATION.md
 * gives the build recipe.  Linking GMAP with
 *
 *   -Wl,--wrap=Dynprog_init -Wl,--wrap=Dynprog_single_setup -Wl,--wrap=Dynprog_end_setup
 *   -Wl,--wrap=Dynprog_genome_setup -Wl,--wrap=Dynprog_single_gap -Wl,--wrap=Dynprog_end5_gap
 *   -Wl,--wrap=Dynprog_end3_gap -Wl,--wrap=Dynprog_genome_gap -Wl,--wrap=Dynprog_cdna_gap
 *   -Wl,--wrap=Dynprog_microexon_int -Wl,--wrap=Oligoindex_hr_tally -Wl,--wrap=Oligoindex_get_mappings
 *   -Wl,--wrap=Stage2_setup -Wl,--wrap=Stage2_compute  gmapdp_gmap_shim.o -lgmapdp
 *
 * makes every existing call site (stage3.c) resolve to the __wrap_ functions
 * below, which have exactly the reference's prototypes:
 *
 *   __wrap_Dynprog_single_gap   replaces Dynprog_single_gap   (dynprog_single.h:22, dynprog_single.c:429)
 *   __wrap_Dynprog_end5_gap     replaces Dynprog_end5_gap     (dynprog_end.h:25,    dynprog_end.c:1294)
 *   __wrap_Dynprog_end3_gap     replaces Dynprog_end3_gap     (dynprog_end.h:47,    dynprog_end.c:1924)
 *   __wrap_Dynprog_genome_gap   replaces Dynprog_genome_gap   (dynprog_genome.h:24, dynprog_genome.c:3288)
 *   __wrap_Dynprog_cdna_gap     replaces Dynprog_cdna_gap     (dynprog_cdna.h:18,   dynprog_cdna.c:787)
 *   __wrap_Dynprog_microexon_int replaces Dynprog_microexon_int (dynprog_single.h:33, dynprog_single.c:900)
 *   __wrap_Stage2_compute       replaces Stage2_compute       (stage2.h:58,         stage2.c:6325)
 *   __wrap_Stage2_setup         observes Stage2_setup         (stage2.h:42,         stage2.c:129) and forwards it
 *   __wrap_Oligoindex_hr_tally + __wrap_Oligoindex_get_mappings replace the stage-2 seeding pair
 *                               (oligoindex_hr.h:106/117) for callers other than Stage2_compute
 *   __wrap_Dynprog_init / _single_setup / _end_setup / _genome_setup observe the
 *                               reference's setup calls (dynprog.c:1008, dynprog_single.c:101,
 *                               dynprog_end.c, dynprog_genome.c:192) and forward them
 *
 * Owning the whole Dynprog_* interface (SURVEY §8b's unit of replacement): compiled with
 * -DGMAPDP_SHIM_OWN, the shim defines the reference's 21 exported Dynprog_* symbols under their own
 * names and GMAP links WITHOUT the six dynprog*.o objects (oracle/ref.mk gmap_gpu_*); only the
 * stage-2 pair (Stage2_setup / Stage2_compute, Oligoindex_hr_tally / Oligoindex_get_mappings) is still
 * routed with --wrap, since stage2.o / oligoindex_hr.o stay linked for their other entry points.  The
 * 21 are the entry points above plus
 *   Dynprog_new / Dynprog_free  (dynprog.c:631/777)   a limits-only handle: no score/direction arenas
 *   Dynprog_term                (dynprog.c:1203)
 *   Dynprog_score               (dynprog.c:126)
 *   Dynprog_consistent_p        (dynprog.c:895)       over the shim's own consistent table (Dynprog_init)
 *   Dynprog_end5/3_splicejunction, Dynprog_end5/3_known (dynprog_end.c:1653/2249/2748/3009)
 *   Dynprog_make_splicejunction_5/3 (dynprog_end.c:2569/2670)
 * Without GMAPDP_SHIM_OWN the entry points are the __wrap_ names (the link above keeps the reference's
 * dynprog objects for Dynprog_new/_free/_term/_score/_consistent_p/_make_splicejunction_5/3).
 *
 * Results are returned as the reference does: a List_T of Pair_T allocated in
 * the caller's Pairpool_T (same order, same fields), the same out-parameters.
 * GMAPDP_DEVICE selects the HIP device (default 0).
 */
#ifndef GMAPDP_DYNPROG_H
#define GMAPDP_DYNPROG_H

#include "bool.h"
#include "list.h"
#include "pairpool.h"
#include "genome.h"
#include "iit-read.h"
#include "dynprog.h"
#include "dynprog_end.h"
#include "diagpool.h"
#include "cellpool.h"
#include "stopwatch.h"
#include "oligoindex_hr.h"
#include "stage2.h"

#ifdef GMAPDP_SHIM_OWN
#define GMAPDP_DYNPROG_ENTRY(name) name
#else
#define GMAPDP_DYNPROG_ENTRY(name) __wrap_##name
#endif

extern void GMAPDP_DYNPROG_ENTRY(Dynprog_init) (Mode_T mode);
extern void GMAPDP_DYNPROG_ENTRY(Dynprog_single_setup) (int user_open_in, int user_extend_in, bool user_dynprog_p_in,
                                         bool homopolymerp_in);
extern void GMAPDP_DYNPROG_ENTRY(Dynprog_end_setup) (Univcoord_T *splicesites_in, Splicetype_T *splicetypes_in,
                                      Chrpos_T *splicedists_in, int nsplicesites_in,
                                      Trieoffset_T *trieoffsets_obs_in, Triecontent_T *triecontents_obs_in,
                                      Trieoffset_T *trieoffsets_max_in, Triecontent_T *triecontents_max_in,
                                      int user_open_in, int user_extend_in, bool user_dynprog_p_in);
extern void GMAPDP_DYNPROG_ENTRY(Dynprog_genome_setup) (bool novelsplicingp_in, IIT_T splicing_iit_in,
                                         int *splicing_divint_crosstable_in, int donor_typeint_in,
                                         int acceptor_typeint_in, int user_open_in, int user_extend_in,
                                         bool user_dynprog_p_in);

extern List_T
GMAPDP_DYNPROG_ENTRY(Dynprog_single_gap) (int *dynprogindex, int *finalscore, int *nmatches, int *nmismatches, int *nopens,
                           int *nindels, Dynprog_T dynprog, char *sequence1, char *sequenceuc1, int length1,
                           int length2, int offset1, int offset2, Univcoord_T chroffset, Univcoord_T chrhigh,
                           bool watsonp, int genestrand, bool jump_late_p, Genome_T genome, Genome_T genomealt,
                           Pairpool_T pairpool, int extraband_single, bool widebandp, double defect_rate);

extern List_T
GMAPDP_DYNPROG_ENTRY(Dynprog_end5_gap) (int *dynprogindex, int *finalscore, int *nmatches, int *nmismatches, int *nopens,
                         int *nindels, Dynprog_T dynprog, char *revsequence1, char *revsequenceuc1, int length1,
                         int length2, int revoffset1, int revoffset2, Univcoord_T chroffset, Univcoord_T chrhigh,
                         bool watsonp, int genestrand, bool jump_late_p, Genome_T genome, Genome_T genomealt,
                         Pairpool_T pairpool, int extraband_end, double defect_rate, Endalign_T endalign,
                         bool require_pos_score_p);

extern List_T
GMAPDP_DYNPROG_ENTRY(Dynprog_end3_gap) (int *dynprogindex, int *finalscore, int *nmatches, int *nmismatches, int *nopens,
                         int *nindels, Dynprog_T dynprog, char *sequence1, char *sequenceuc1, int length1,
                         int length2, int offset1, int offset2, Univcoord_T chroffset, Univcoord_T chrhigh,
                         bool watsonp, int genestrand, bool jump_late_p, Genome_T genome, Genome_T genomealt,
                         Pairpool_T pairpool, int extraband_end, double defect_rate, Endalign_T endalign,
                         bool require_pos_score_p);

extern List_T
GMAPDP_DYNPROG_ENTRY(Dynprog_genome_gap) (int *dynprogindex, int *new_leftgenomepos, int *new_rightgenomepos, double *left_prob,
                           double *right_prob, int *traceback_score, int *nmatches, int *nmismatches, int *nopens,
                           int *nindels, int *exonhead, int *introntype, Dynprog_T dynprogL, Dynprog_T dynprogR,
                           char *rsequence, char *rsequenceuc, int rlength, int glengthL, int glengthR, int roffset,
                           int goffsetL, int rev_goffsetR, Chrnum_T chrnum, Univcoord_T chroffset,
                           Univcoord_T chrhigh, int cdna_direction, bool watsonp, int genestrand, bool jump_late_p,
                           Genome_T genome, Genome_T genomealt, Pairpool_T pairpool, int extraband_paired,
                           double defect_rate, int maxpeelback, bool halfp, bool finalp);

extern List_T
GMAPDP_DYNPROG_ENTRY(Dynprog_cdna_gap) (int *dynprogindex, int *traceback_score, bool *incompletep, Dynprog_T dynprogL,
                         Dynprog_T dynprogR, char *rsequenceL, char *rsequence_ucL, char *rev_rsequenceR,
                         char *rev_rsequence_ucR, int rlengthL, int rlengthR, int glength, int roffsetL,
                         int rev_roffsetR, int goffset, Univcoord_T chroffset, Univcoord_T chrhigh, bool watsonp,
                         int genestrand, bool jump_late_p, Genome_T genome, Genome_T genomealt,
                         Pairpool_T pairpool, int extraband_paired, double defect_rate);

extern List_T
GMAPDP_DYNPROG_ENTRY(Dynprog_microexon_int) (double *bestprob2, double *bestprob3, int *dynprogindex, int *microintrontype,
                              char *rsequence, char *rsequenceuc, int rlength, int roffset, int goffsetL,
                              int rev_goffsetR, int cdna_direction, char *queryseq, char *queryuc,
                              Univcoord_T chroffset, Univcoord_T chrhigh, bool watsonp, int genestrand,
                              Genome_T genome, Genome_T genomealt, Pairpool_T pairpool);

extern void
__wrap_Oligoindex_hr_tally (Oligoindex_T this, Univcoord_T mappingstart, Univcoord_T mappingend, bool plusp,
                            char *queryuc_ptr, int querystart, int queryend, Chrpos_T chrpos, Genome_T genome,
                            int genestrand);

extern List_T
__wrap_Oligoindex_get_mappings (List_T diagonals, bool *coveredp, Chrpos_T **mappings, int *npositions,
                                int *totalpositions, bool *oned_matrix_p, int *maxnconsecutive,
                                Oligoindex_array_T array, Oligoindex_T this, char *queryuc_ptr, int querystart,
                                int queryend, int querylength, Chrpos_T chrstart, Chrpos_T chrend,
                                Univcoord_T chroffset, Univcoord_T chrhigh, bool plusp, Diagpool_T diagpool);

extern void
__wrap_Stage2_setup (bool splicingp_in, bool cross_species_p, int suboptimal_score_start_in,
                     int suboptimal_score_end_in, int sufflookback_in, int nsufflookback_in, int maxintronlen_in,
                     Mode_T mode_in, bool snps_p_in);

extern List_T
__wrap_Stage2_compute (char *queryseq_ptr, char *queryuc_ptr, int querylength, int query_offset, Chrpos_T chrstart,
                       Chrpos_T chrend, Univcoord_T chroffset, Univcoord_T chrhigh, bool plusp, int genestrand,
                       Stage2_alloc_T stage2_alloc, double proceed_pctcoverage, Oligoindex_array_T oligoindices,
                       Genome_T genome, Genome_T genomealt, Pairpool_T pairpool, Diagpool_T diagpool,
                       Cellpool_T cellpool, bool localp, bool skip_repetitive_p, bool favor_right_p,
                       int max_nalignments, Stopwatch_T stopwatch, bool diag_debug);

#endif
