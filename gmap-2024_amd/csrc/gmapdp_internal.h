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

// Device-side problem descriptor derived on the host from gmapdp_single_problem
// (penalties, bands and the launch class are resolved once, in the plan).
struct DevSingle {
  int32_t qoff;
  int32_t rlength;
  int32_t glength;
  int32_t roffset;
  int32_t goffset;
  uint32_t chroffset;
  uint32_t chrhigh;
  int32_t lband;
  int32_t uband;
  int32_t open;
  int32_t extend;
  int32_t mismatchtype;
  int32_t flags;          // bit0 watson, bit1 jump_late
  int32_t genestrand;
  int32_t dynprogindex;
  int32_t pair_offset;
  int64_t dirs_offset;    // byte offset into the global direction scratch (global-dirs classes)
};

}  // namespace gmapdp
