// gmapdp_internal.h -- shared host/device definitions of libgmapdp (not part of the C ABI).
#pragma once
#include <stdint.h>

namespace gmapdp {

// Reference constants (dynprog.h:44-119, dynprog.c:104, scores.h, comp.h, pairpool.c).
constexpr int kNegInf32 = -32768;       // NEG_INFINITY_32 / NEG_INFINITY_INT
constexpr int kMatch = 1, kMismatch = -3, kQopen = -3, kQindel = -1, kTopen = -3, kTindel = -1;
constexpr int kMicrointronLength = 9;   // genome skips >= 9 become a gap holder (pairpool.c:1090)
constexpr int kMaxR = 64;               // band up to 64*64 = 4096 cells wide

// Genome character classes used for scoring: the packed genome only ever
// yields A C G T N, their complements, and '*' beyond the chromosome.
enum GClass : uint8_t { kA = 0, kC = 1, kG = 2, kT = 3, kN = 4, kStar = 5 };
constexpr int kNClass = 8;              // padded to 8 bytes per score row

// Problem kinds (one kernel serves all Dynprog_* fills with a traceback).
enum Kind : int32_t { kSingle = 0, kEnd5 = 1, kEnd3 = 2 };
// Endalign_T (dynprog.h:25)
enum Endalign : int32_t { kQueryendGap = 0, kQueryendIndels = 1, kQueryendNogaps = 2, kBestLocal = 3 };

// DevProblem.flags
constexpr int32_t kFWatson = 0x1;     // watsonp
constexpr int32_t kFLate = 0x2;       // tie rule of the fill/endpoint search: >= (jump late) instead of >
constexpr int32_t kFRequirePos = 0x4; // require_pos_score_p (end gaps)
constexpr int32_t kFSegLeft = 0x8;    // genome segment via Genome_get_segment_left (else _right)
constexpr int32_t kFSegRevcomp = 0x10;
constexpr int32_t kFRev = 0x20;       // revp: DP runs away from the anchor (end5)
constexpr int32_t kFScoreUC = 0x40;   // the fill scores rsequenceuc (Dynprog_end3_gap) instead of rsequence
constexpr int32_t kFSimd = 0x80;      // SIMD-build semantics (Dynprog_simd_8/16, sx_kernel)

// Device-side problem descriptor derived on the host (penalties, bands,
// orientation and the launch class are resolved once, in the plan).
struct DevProblem {
  int32_t qbase;          // arena index of the query character of DP row 1
  int32_t rlength;        // DP rows (after the reference's chopping)
  int32_t glength;        // DP columns
  int32_t roffset;        // querypos of row r = roffset + sgn*(r-1)
  int32_t goffset;        // genomepos of column c = goffset + sgn*(c-1)
  uint64_t chroffset;
  uint64_t chrhigh;
  uint64_t segpos;        // left (right variant) or right (left variant) coordinate of the segment
  uint64_t segbound;      // chrhigh (right variant) or chroffset (left variant)
  int32_t lband;
  int32_t uband;
  int32_t open;
  int32_t extend;
  int32_t mismatchtype;
  int32_t flags;
  int32_t genestrand;
  int32_t dynprogindex;
  int32_t pair_offset;
  int32_t kind;
  int32_t endalign;
  int64_t dirs_offset;    // byte offset into the global direction scratch (global-dirs classes)
};

// DevGenomeProblem.flags (kFWatson / kFLate as above; kFLate is jump_late_p as given)
constexpr int32_t kGHalf = 0x100;       // halfp
constexpr int32_t kGFinal = 0x200;      // finalp
constexpr int32_t kGSimple = 0x400;     // genome_gap_simple is tried first (!finalp && defect_rate < DEFECT_MEDQ)
constexpr int32_t kGSegLLeft = 0x800;   // gsequenceL via Genome_get_segment_left (minus strand)
constexpr int32_t kGSegLRc = 0x1000;
constexpr int32_t kGSegRLeft = 0x2000;  // rev_gsequenceR via Genome_get_segment_left (plus strand)
constexpr int32_t kGSegRRc = 0x4000;
constexpr int32_t kGSimd = 0x8000;      // SIMD-build semantics (triangle fills, uxg_kernel)
constexpr int32_t kGKnown = 0x10000;    // known splice sites: flags at known_offset (GMAPDP_KNOWN_SITES)
constexpr int kKnownReward = 20;        // KNOWN_SPLICESITE_REWARD (dynprog_genome.c:118)
constexpr int32_t kUnset = (int32_t)0x80000000;  // out-parameter the reference leaves unwritten

// Dynprog_genome_gap descriptor (dynprog_genome.c:3288): two fills share the
// query; the R fill runs on the reversed query against rev_gsequenceR.
struct DevGenomeProblem {
  int32_t qbase;          // arena index of rsequence[0]
  int32_t rlength;
  int32_t glengthL;
  int32_t glengthR;
  int32_t roffset;
  int32_t goffsetL;
  int32_t rev_goffsetR;
  uint64_t chroffset;
  uint64_t chrhigh;
  uint64_t segposL, segboundL;  // gsequenceL segment (see DevProblem.segpos)
  uint64_t segposR, segboundR;  // rev_gsequenceR segment
  int32_t lbandL;         // both fills (the R fill is called with lbandL, dynprog_genome.c:3813)
  int32_t ubandL;
  int32_t ubandR;
  int32_t open;
  int32_t extend;
  int32_t mismatchtype;
  int32_t flags;
  int32_t iclass;         // intron score array: 0 sense, 1 antisense, 2 either
  int32_t genestrand;
  int32_t dynprogindex;
  int32_t pair_offset;
  int32_t known_offset;   // kGKnown: bridge flags at [known_offset, +glengthL+glengthR), simple's follow
  int64_t prob_offset;    // left probabilities at [prob_offset, +glengthL), right ones follow
  int64_t dirs_offset;    // byte offset into the global scratch (global-dirs classes)
  int64_t reserved_;      // keeps the descriptor at 128 B
};

// DevCdnaProblem.flags (kFWatson / kFLate as above)
constexpr int32_t kCSegLeft = 0x100;    // gsequence via Genome_get_segment_left (minus strand)
constexpr int32_t kCSegRc = 0x200;
constexpr int32_t kCRSegLeft = 0x400;   // rev_gsequence via Genome_get_segment_left (plus strand)
constexpr int32_t kCRSegRc = 0x800;
constexpr int32_t kCSimd = 0x1000;      // SIMD-build semantics (triangle fills, uxc_kernel)

// Dynprog_cdna_gap descriptor (dynprog_cdna.c:787).  The L fill runs rsequenceL forward against
// gsequence, the R fill rev_rsequenceR backwards against rev_gsequence (the same genome interval).
// Inside the engine's domain (rlengthL == rlengthR >= glength) the fills' and both bridges' bands
// coincide: lband = rlength - glength + extraband_paired, uband = extraband_paired.
struct DevCdnaProblem {
  int32_t qbaseL;         // arena index of rsequenceL[0]
  int32_t qbaseR;         // arena index of rev_rsequenceR[0] (the R piece's last character)
  int32_t rlength;        // rlengthL = rlengthR
  int32_t glength;
  int32_t roffsetL;
  int32_t rev_roffsetR;
  int32_t goffset;
  int32_t lband;
  int32_t uband;
  uint64_t chroffset;
  uint64_t chrhigh;
  uint64_t segpos, segbound;    // gsequence segment (see DevProblem.segpos)
  uint64_t rsegpos, rsegbound;  // rev_gsequence segment
  int32_t open;
  int32_t extend;
  int32_t mismatchtype;
  int32_t flags;
  int32_t genestrand;
  int32_t dynprogindex;
  int32_t pair_offset;
  int64_t scratch_offset; // byte offset of the problem's region of the global scratch
};

// Dynprog_end5/3_splicejunction descriptor (dynprog_end.c:1653/2249).  Columns come from the batch's
// junction arena: column c is jseq[jbase + sgn*(c-1)] (sgn -1 for end5, whose rev_gsequence points at
// the junction's last character).
constexpr int kMismatchEndQ = 3;        // Mismatchtype_T ENDQ: the score-table slice of the end gaps
constexpr int kFullMatch = 3;           // FULLMATCH (dynprog.h:43)
struct DevSjProblem {
  int32_t qbase;          // arena index of the query character of DP row 1
  int32_t jbase;          // junction-arena index of the character of DP column 1
  int32_t rlength;
  int32_t glength;
  int32_t roffset;        // (rev_)roffset
  int32_t goffset_anchor; // (rev_)goffset_anchor: genome positions of the anchor piece
  int32_t goffset_far;    // (rev_)goffset_far: genome positions of the far exon's piece
  int32_t known_jump;     // genomejump of the known-splice gap holder
  int32_t contlength;     // endc of the far piece's traceback
  int32_t lband;
  int32_t uband;
  int32_t open;
  int32_t extend;
  int32_t late;           // tie rule of the fill and the endpoint scan (end5: !jump_late_p)
  int32_t end3p;
  int32_t genestrand;
  int32_t dynprogindex;
  int32_t pair_offset;
  int32_t simd;           // SIMD-build semantics (usj_kernel)
  int64_t dirs_offset;    // byte offset into the global direction scratch (!DIRS_LDS / usj classes)
};

// Stage-2 seeding descriptor (Oligoindex_hr_tally + Oligoindex_get_mappings, oligoindex_hr.c:33849/34127)
struct DevOligoProblem {
  int32_t qoff;           // arena index of queryuc_ptr[0]
  int32_t querylength;
  uint32_t chrstart, chrend;
  uint64_t chroffset, chrhigh;
  int32_t plusp;
  int32_t minor;          // oligoindices_minor (diag_lookback 60, suffnconsecutive 10), else major (120, 20)
  int32_t umax;           // LDS slots for the query's distinct 8-mers (>= their number)
  int32_t index;          // the problem's index in the batch (its result slot)
  int64_t table_offset;   // first entry of the problem's table in the positions arena (the mappings the
                          // kernels write are relative to it, so the arena may pass 2^31 entries)
  int64_t diag_offset;    // first diagonal record (4 x int32)
  int64_t scratch_offset; // byte offset of the problem's region of the global scratch (its launch chunk's)
  int64_t fallback_offset; // the sequential walk's region in the same scratch, or -1: none (exact pool)
  // What the layout gave the problem: hit-list entries, table entries, diagonal records.  A run that
  // needs more (a plan re-laid out from a measured run and then run on another query) reports overflow
  // (oned_matrix_p -1, Stage2_compute status -2) instead of writing past its slices.
  uint32_t hit_cap, table_cap, diag_cap;
  int32_t pad_;
};

// Stage2_compute descriptor (stage2.c:6325): the seeding problem's results slot plus the chaining
// parameters (Stage2_setup)
struct DevStage2Problem {
  int32_t qoff;           // arena index of queryseq_ptr[0] / queryuc_ptr[0]
  int32_t querylength;
  uint32_t chrstart, chrend;
  uint64_t chroffset, chrhigh;
  int32_t plusp;
  int32_t splicingp;
  uint32_t maxintronlen;
  int32_t index;          // the problem's index in the batch (seeding result and stage-2 result slot)
  int64_t scratch_offset; // byte offset of the problem's chaining scratch (s2_scratch, sized from the seeding)
};

}  // namespace gmapdp
