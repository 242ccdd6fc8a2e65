// me_device.h -- device restatement of GMAP's MaxEnt splice-site models:
// Maxent_hr_donor_prob / _acceptor_prob / _antidonor_prob / _antiacceptor_prob (maxent_hr.c:27357 / 27433 /
// 27512 / 27586).
//
// The reference dispatches on the window start's shift within its 32-nt .genomecomp block to one of 32
// handlers per model, each pulling the model's k-mers out of the block words low / high / nextlow /
// nexthigh.  All 32 handlers compute the same thing: the 2-bit codes of the window's nucleotides (the one
// at startpos + k in bits 2k) indexed into the model's tables.  Here the window is one 64-bit funnel of
// the two blocks' words, and the lookups and multiplies follow the reference's order exactly (each a
// double multiply, then odds / (1 + odds), IEEE division), so the doubles are bit-identical.  The
// tables are the reference's constants (maxent_hr.c:25-24660), regenerated as a binary by
// tools/make_maxent_tables.py and resident in HBM (1.5 MB, L2-resident in use).
#pragma once
#include <stdint.h>

#include "gmapdp_internal.h"

namespace gmapdp {

// entries of the 16 tables, in tools/make_maxent_tables.py's TABLES order
constexpr int kMeEntries[16] = {16384, 16, 16384, 16384, 16384, 16, 16384, 16384,
                                16384, 16, 16384, 16384, 16384, 16, 16384, 16384};
__host__ __device__ constexpr int me_offset(int t) {
  int o = 0;
  for (int i = 0; i < t; i++) o += kMeEntries[i];
  return o;
}
constexpr int kMeTotal = me_offset(16);
constexpr int kMeDonorMargin = 3, kMeAcceptorMargin = 20, kMeAntidonorMargin = 6, kMeAntiacceptorMargin = 3;

#ifdef __HIPCC__
__device__ __forceinline__ uint32_t me_word(const uint32_t* __restrict__ blocks, uint64_t nwords, uint64_t i) {
  return i < nwords ? blocks[i] : 0xFFFFFFFFu;  // past the allocation: 'X' padding, as the trailing words
}

// model: GMAPDP_MAXENT_DONOR 0, _ACCEPTOR 1, _ANTIDONOR 2, _ANTIACCEPTOR 3
__device__ __forceinline__ double maxent_prob(const uint32_t* __restrict__ blocks, uint64_t nwords,
                                              const double* __restrict__ T, int model, uint64_t splice_pos,
                                              uint64_t chroffset) {
  const int margin = model == 0 ? kMeDonorMargin : model == 1 ? kMeAcceptorMargin
                   : model == 2 ? kMeAntidonorMargin : kMeAntiacceptorMargin;
  if (splice_pos < chroffset + (uint64_t)margin) return 0.0;
  const uint64_t start = splice_pos - (uint64_t)margin;
  const uint64_t ptr = start / 32u * 3u;
  const unsigned shift = (unsigned)(start % 32u);
  const uint64_t w0 = (uint64_t)me_word(blocks, nwords, ptr + 1) | ((uint64_t)me_word(blocks, nwords, ptr) << 32);
  const uint64_t w1 =
      (uint64_t)me_word(blocks, nwords, ptr + 4) | ((uint64_t)me_word(blocks, nwords, ptr + 3) << 32);
  const uint64_t W = shift ? (w0 >> (2u * shift)) | (w1 << (64u - 2u * shift)) : w0;
  double odds;
  if (model == 0) {  // donor_plus_XX
    odds = T[me_offset(0) + ((W & 0x3F) | ((W >> 4) & 0x3FC0))] * T[me_offset(1) + ((W >> 6) & 0xF)];
  } else if (model == 2) {  // donor_minus_XX
    odds = T[me_offset(8) + ((W & 0xFF) | ((W >> 4) & 0x3F00))] * T[me_offset(9) + ((W >> 8) & 0xF)];
  } else if (model == 1) {  // acceptor_plus_XX
    const uint64_t s = W >> 28;
    odds = T[me_offset(2) + (W & 0x3FFF)];
    odds *= T[me_offset(3) + ((W >> 14) & 0x3FFF)];
    odds *= T[me_offset(4) + ((s & 0xFF) | ((s >> 4) & 0x3F00))];
    odds *= T[me_offset(5) + ((s >> 8) & 0xF)];
    odds *= T[me_offset(6) + ((W >> 8) & 0x3FFF)];
    odds *= T[me_offset(7) + ((W >> 22) & 0x3FFF)];
  } else {  // acceptor_minus_XX
    odds = T[me_offset(10) + ((W >> 32) & 0x3FFF)];
    odds *= T[me_offset(11) + ((W >> 18) & 0x3FFF)];
    odds *= T[me_offset(12) + ((W & 0x3F) | ((W >> 4) & 0x3FC0))];
    odds *= T[me_offset(13) + ((W >> 6) & 0xF)];
    odds *= T[me_offset(14) + ((W >> 24) & 0x3FFF)];
    odds *= T[me_offset(15) + ((W >> 10) & 0x3FFF)];
  }
  return odds / (1.0 + odds);
}

// The probability bridge_intron_gap_site_level reads for genome-gap entry jj (dynprog_genome.c:2573-2660;
// me_gap_kernel's layout): left entries cL = jj < glengthL at chroffset + goffsetL + cL (plus strand) or
// chrhigh - goffsetL - cL + 1, right entries cR = jj - glengthL at chroffset + rev_goffsetR - cR + 1 or
// chrhigh - rev_goffsetR + cR; donor / acceptor models for cdna_direction > 0 (iclass 0), antiacceptor /
// antidonor otherwise, mirrored on the minus strand.
__device__ __forceinline__ double gg_site_prob(const DevGenomeProblem& P, const uint32_t* __restrict__ blocks,
                                               uint64_t nwords, const double* __restrict__ T, int jj) {
  const bool watson = P.flags & kFWatson;
  const bool sense = P.iclass == 0;
  const uint64_t lo = (uint64_t)(int64_t)P.goffsetL, ro = (uint64_t)(int64_t)P.rev_goffsetR;
  uint64_t pos;
  int model;
  if (jj < P.glengthL) {
    const uint64_t c = (uint64_t)jj;
    pos = watson ? P.chroffset + lo + c : P.chrhigh - lo - c + 1u;
    model = watson ? (sense ? 0 : 3) : (sense ? 2 : 1);
  } else {
    const uint64_t c = (uint64_t)(jj - P.glengthL);
    pos = watson ? P.chroffset + ro - c + 1u : P.chrhigh - ro + c;
    model = watson ? (sense ? 1 : 2) : (sense ? 3 : 0);
  }
  return maxent_prob(blocks, nwords, T, model, pos, P.chroffset);
}
#endif

}  // namespace gmapdp
