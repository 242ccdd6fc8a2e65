/* include/gmapdp_dynprog.h -- reference-signature drop-in for GMAP's Dynprog_* entry points.
 *
 * For a GMAP build only: include it with GMAP's src/ on the include path
 * (it needs GMAP's List_T, Pair_T, Pairpool_T, Genome_T, Dynprog_T types).
 * The implementation is gmap-2024_amd/shim/gmapdp_gmap_shim.c; INTEGRATION.md
 * gives the build recipe.  Linking GMAP with
 *
 *   -Wl,--wrap=Dynprog_init -Wl,--wrap=Dynprog_single_setup -Wl,--wrap=Dynprog_end_setup
 *   -Wl,--wrap=Dynprog_genome_setup -Wl,--wrap=Dynprog_single_gap -Wl,--wrap=Dynprog_end5_gap
 *   -Wl,--wrap=Dynprog_end3_gap -Wl,--wrap=Dynprog_genome_gap  gmapdp_gmap_shim.o -lgmapdp
 *
 * makes every existing call site (stage3.c) resolve to the __wrap_ functions
 * below, which have exactly the reference's prototypes:
 *
 *   __wrap_Dynprog_single_gap   replaces Dynprog_single_gap   (dynprog_single.h:22, dynprog_single.c:429)
 *   __wrap_Dynprog_end5_gap     replaces Dynprog_end5_gap     (dynprog_end.h:25,    dynprog_end.c:1294)
 *   __wrap_Dynprog_end3_gap     replaces Dynprog_end3_gap     (dynprog_end.h:47,    dynprog_end.c:1924)
 *   __wrap_Dynprog_genome_gap   replaces Dynprog_genome_gap   (dynprog_genome.h:24, dynprog_genome.c:3288)
 *   __wrap_Dynprog_init / _single_setup / _end_setup / _genome_setup observe the
 *                               reference's setup calls (dynprog.c:1008, dynprog_single.c:101,
 *                               dynprog_end.c, dynprog_genome.c:192) and forward them
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

extern void __wrap_Dynprog_init (Mode_T mode);
extern void __wrap_Dynprog_single_setup (int user_open_in, int user_extend_in, bool user_dynprog_p_in,
                                         bool homopolymerp_in);
extern void __wrap_Dynprog_end_setup (Univcoord_T *splicesites_in, Splicetype_T *splicetypes_in,
                                      Chrpos_T *splicedists_in, int nsplicesites_in,
                                      Trieoffset_T *trieoffsets_obs_in, Triecontent_T *triecontents_obs_in,
                                      Trieoffset_T *trieoffsets_max_in, Triecontent_T *triecontents_max_in,
                                      int user_open_in, int user_extend_in, bool user_dynprog_p_in);
extern void __wrap_Dynprog_genome_setup (bool novelsplicingp_in, IIT_T splicing_iit_in,
                                         int *splicing_divint_crosstable_in, int donor_typeint_in,
                                         int acceptor_typeint_in, int user_open_in, int user_extend_in,
                                         bool user_dynprog_p_in);

extern List_T
__wrap_Dynprog_single_gap (int *dynprogindex, int *finalscore, int *nmatches, int *nmismatches, int *nopens,
                           int *nindels, Dynprog_T dynprog, char *sequence1, char *sequenceuc1, int length1,
                           int length2, int offset1, int offset2, Univcoord_T chroffset, Univcoord_T chrhigh,
                           bool watsonp, int genestrand, bool jump_late_p, Genome_T genome, Genome_T genomealt,
                           Pairpool_T pairpool, int extraband_single, bool widebandp, double defect_rate);

extern List_T
__wrap_Dynprog_end5_gap (int *dynprogindex, int *finalscore, int *nmatches, int *nmismatches, int *nopens,
                         int *nindels, Dynprog_T dynprog, char *revsequence1, char *revsequenceuc1, int length1,
                         int length2, int revoffset1, int revoffset2, Univcoord_T chroffset, Univcoord_T chrhigh,
                         bool watsonp, int genestrand, bool jump_late_p, Genome_T genome, Genome_T genomealt,
                         Pairpool_T pairpool, int extraband_end, double defect_rate, Endalign_T endalign,
                         bool require_pos_score_p);

extern List_T
__wrap_Dynprog_end3_gap (int *dynprogindex, int *finalscore, int *nmatches, int *nmismatches, int *nopens,
                         int *nindels, Dynprog_T dynprog, char *sequence1, char *sequenceuc1, int length1,
                         int length2, int offset1, int offset2, Univcoord_T chroffset, Univcoord_T chrhigh,
                         bool watsonp, int genestrand, bool jump_late_p, Genome_T genome, Genome_T genomealt,
                         Pairpool_T pairpool, int extraband_end, double defect_rate, Endalign_T endalign,
                         bool require_pos_score_p);

extern List_T
__wrap_Dynprog_genome_gap (int *dynprogindex, int *new_leftgenomepos, int *new_rightgenomepos, double *left_prob,
                           double *right_prob, int *traceback_score, int *nmatches, int *nmismatches, int *nopens,
                           int *nindels, int *exonhead, int *introntype, Dynprog_T dynprogL, Dynprog_T dynprogR,
                           char *rsequence, char *rsequenceuc, int rlength, int glengthL, int glengthR, int roffset,
                           int goffsetL, int rev_goffsetR, Chrnum_T chrnum, Univcoord_T chroffset,
                           Univcoord_T chrhigh, int cdna_direction, bool watsonp, int genestrand, bool jump_late_p,
                           Genome_T genome, Genome_T genomealt, Pairpool_T pairpool, int extraband_paired,
                           double defect_rate, int maxpeelback, bool halfp, bool finalp);

#endif
