// cg_kernel.hip -- CDNA4 (gfx950) kernels for GMAP's Dynprog_cdna_gap: cg_kernel<R> as the nosimd
// build computes it (Dynprog_standard fills, bridge_cdna_gap), uxc_kernel<B> as the SIMD builds do
// (Dynprog_simd_{8,16}_upper/_lower triangles, bridge_cdna_gap_{8,16}_ud).
//
// Reference semantics restated (paths under the reference tree's src/):
//   Dynprog_cdna_gap              dynprog_cdna.c:787-1300: NULL for glength <= 1 (:830) and at the
//                                 size guard (:869/882, dynprogindex advanced), CDNA_OPEN/EXTEND
//                                 penalties (:852-867), use8p (:909), the R fill on the reversed
//                                 query against rev_gsequence with !jump_late_p (nosimd: with
//                                 lbandL, :1217), the R traceback and List_reverse, the 9 x 9
//                                 SHORTGAP block (:1241-1263) or the gap holder (:1270), the L
//                                 traceback, NULL when only the gap holder is left (:1282)
//   bridge_cdna_gap               dynprog_cdna.c:652-779 (its own bands :667-670)
//   bridge_cdna_gap_8_ud / _16_ud dynprog_cdna.c:124 / 387 (the fill bands; upper cells r < c,
//                                 lower cells r >= c)
//
// The bridge scans every column pair (cL, cR), cR from glength - cL down to 0 -- penalty 0 for the
// first cR and CDNA open for the others (the reference's "pen += extend" never accumulates: the
// loop body resets pen to open - extend) -- and inside a pair every (rL, rR) with
// rR < rightoffset - leftoffset - rL; ties keep the first candidate (>) or the last (>=, jump late).
// Sequentially that is O(g^2 b^2).  Here the rR loop collapses into a prefix maximum: PM[cR][j] is
// the best matrixR[cR][rR] over rR in [rloR, rloR + j] with its row (first maximum for >, last for
// >=), so a candidate (cL, cR, rL) is one lookup of PM at its rR bound.  The wave takes the
// (cR, rL) pairs of one column cL in parallel; each lane keeps the winner of its candidates by a
// (score, scan position) key and one wave reduction picks the reference's choice.  Matrices, PM and
// the direction words live in an L2-resident global scratch: cDNA gaps are rare,
// so one wave per problem and simple layouts are enough.
#include "ux_device.h"

namespace gmapdp {

constexpr int kInsertPairs = 9;  // INSERT_PAIRS (dynprog_cdna.c:40)

// nosimd: matrix[c][r] of a stored band fill; column 0 is the boundary column (dynprog.c:1331-1338)
struct BandCells {
  const int* m;
  int W, uband, open, ext;
  __device__ int operator()(int r, int c) const {
    if (c == 0) return open + r * ext;  // read only for 1 <= r <= lband
    return m[(size_t)c * W + (r - c + uband)];
  }
};
// SIMD: upper[c][r] for r < c, lower[r][c] otherwise (bridge_cdna_gap_*_ud)
struct UdCells {
  UxView u, l;
  __device__ int operator()(int r, int c) const { return r < c ? u.cell(r, c) : l.cell(r, c); }
};

struct CgBest {
  int cL, cR, rL, rR;
};

// The bridge over one problem (whole wave).  neg: the initial bestscore (NEG_INFINITY_32/_8/_16).
template <typename CL, typename CR>
__device__ CgBest cdna_bridge(int lane, const CL& cellL, const CR& cellR, int g, int rl, int lband, int uband,
                              int open, int late, int neg, int lim, int2* __restrict__ pm, int W) {
  // 1. prefix maxima of the R columns, one column per lane
  for (int cR = lane; cR <= g; cR += 64) {
    const int lo = max(1, cR - uband), hi = min(cR + lband, rl - 1);
    int bv = 0, ba = -1;
    for (int r = lo; r <= hi; r++) {
      const int v = cellR(r, cR);
      if (ba < 0 || v > bv - late) {
        bv = v;
        ba = r;
      }
      pm[(size_t)cR * W + (r - lo)] = make_int2(bv, ba);
    }
  }
  __threadfence_block();
  // 2. candidates (cL, cR, rL) in parallel; scan position (cL, a = glength - cL - cR, rL, rR)
  int bs = kSent;
  uint64_t bk = 0;
  for (int cL = 1; cL < g; cL++) {
    const int loL = max(1, cL - uband), hiL = min(cL + lband, rl - 1);
    const int nL = hiL - loL + 1;
    if (nL <= 0) continue;
    const int n = (g - cL + 1) * nL;
    for (int j = lane; j < n; j += 64) {
      const int a = j / nL, rL = loL + (j - a * nL);
      const int cR = g - cL - a;
      const int loR = max(1, cR - uband), hiR = min(cR + lband, rl - 1);
      const int top = min(hiR, lim - rL - 1);
      if (top < loR) continue;
      const int2 pv = pm[(size_t)cR * W + (top - loR)];
      const int s = cellL(rL, cL) + pv.x + (a == 0 ? 0 : open);
      if (s <= neg - late) continue;  // never beats the initial bestscore
      const uint64_t pos = ((uint64_t)cL << 31) | ((uint64_t)a << 20) | ((uint64_t)rL << 10) | (uint64_t)pv.y;
      const uint64_t k = late ? pos : ~pos;  // >= keeps the last in scan order, > the first
      if (s > bs || (s == bs && k > bk)) {
        bs = s;
        bk = k;
      }
    }
  }
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {
    const int s2 = __shfl_xor(bs, off, 64);
    const uint64_t k2 = __shfl_xor(bk, off, 64);
    if (s2 > bs || (s2 == bs && k2 > bk)) {
      bs = s2;
      bk = k2;
    }
  }
  CgBest b = {0, 0, 0, 0};  // no candidate: the oracle's zero-initialised coordinates
  if (bs != kSent) {
    const uint64_t pos = late ? bk : ~bk;
    b.cL = (int)(pos >> 31);
    b.cR = g - b.cL - (int)((pos >> 20) & 2047u);
    b.rL = (int)((pos >> 10) & 1023u);
    b.rR = (int)(pos & 1023u);
  }
  return b;
}

// The tail of Dynprog_cdna_gap: R traceback, List_reverse, the SHORTGAP block or the gap holder,
// L traceback, the NULL rule and the out-parameters.
template <typename TBR, typename TBL>
__device__ void cdna_finish(int lane, const DevCdnaProblem& P, int pid, const CgBest& b, const TBR& traceR,
                            const TBL& traceL, const char* __restrict__ qseq, const uint32_t* __restrict__ blocks,
                            uint64_t nwords, gmapdp_cdna_result* __restrict__ results, gmapdp_pair* out) {
  const bool watson = P.flags & kFWatson;
  const int rev_goffset = P.goffset + P.glength - 1;
  Tally t = {0, 0, 0, 0, 0, 0, 0, false};
  traceR(t);
  const int nR = t.count;
  reverse_records(lane, out, nR);
  const int queryjump = (P.rev_roffsetR - b.rR) - (P.roffsetL + b.rL) + 1;
  const int genomejump = (rev_goffset - b.cR) - (P.goffset + b.cL) + 1;
  int gap_index = -1;
  if (queryjump == kInsertPairs && genomejump == kInsertPairs) {
    {  // cDNA insertion: querypos rev_roffsetR - bestrR down to roffsetL + bestrL (:1243-1247)
      const int k = P.rev_roffsetR - b.rR - lane, gp = rev_goffset - b.cR + 1;
      const bool good = lane < kInsertPairs && k >= 0 && gp >= 0;
      const uint64_t m = ballot(good);
      if (good) put_pair(out, t.count + lanes_below(m, lane), k, gp, 0, qseq[P.qbaseL + k - P.roffsetL], '~', ' ', ' ');
      t.count += __popcll(m);
    }
    {  // genome insertion: genomepos rev_goffset - bestcR down to goffset + bestcL (:1252-1261)
      const int k = rev_goffset - b.cR - lane, qp = P.roffsetL + b.rL;
      const bool good = lane < kInsertPairs && qp >= 0 && k >= 0;
      const uint64_t m = ballot(good);
      if (good) {
        const char c2 = genomic_nt(blocks, nwords, k, P.chroffset, P.chrhigh, watson);
        put_pair(out, t.count + lanes_below(m, lane), qp, k, 0, ' ', '~', c2, c2);
      }
      t.count += __popcll(m);
    }
  } else {
    if (lane == 0) put_pair(out, t.count, -1, -1, genomejump, ' ', ' ', ' ', ' ');
    gap_index = t.count;
    t.count += 1;
  }
  traceL(t);
  int npairs = t.count;
  if (npairs == 1) {  // only a gap added (:1282)
    npairs = 0;
    gap_index = -1;
  }
  if (lane == 0) {
    gmapdp_cdna_result res;
    res.npairs = npairs;
    res.pair_offset = P.pair_offset;
    res.traceback_score = t.score + t.nmatches * kMatch + t.nmismatches * kMismatch;
    res.dynprogindex = P.dynprogindex + (P.dynprogindex > 0 ? 1 : -1);
    res.incompletep = (queryjump == kInsertPairs && genomejump == kInsertPairs) ? 0 : 1;
    res.gap_index = gap_index;
    res.gap_queryjump = queryjump;
    res.pad_ = 0;
    results[pid] = res;
  }
}

// Genome classes of both segments: gsequence column c = segment[c - 1]; rev_gsequence, walked
// backwards by the R fill, column c = segment[glength - c].
__device__ __forceinline__ void cdna_stage_genome(int lane, const DevCdnaProblem& P, const uint32_t* blocks,
                                                  uint64_t nwords, uint8_t* gclL, uint8_t* gclR) {
  const int g = P.glength, flags = P.flags;
  for (int i = lane; i < g; i += 64) {
    gclL[i + 1] = gclass(segment_nt(blocks, nwords, (uint32_t)i, (uint32_t)g, P.segpos, P.segbound,
                                    flags & kCSegLeft, flags & kCSegRc));
    gclR[g - i] = gclass(segment_nt(blocks, nwords, (uint32_t)i, (uint32_t)g, P.rsegpos, P.rsegbound,
                                    flags & kCRSegLeft, flags & kCRSegRc));
  }
}

// ---- scratch and LDS of one problem (must match the host's sizes) ----
struct ScratchCg {
  size_t dL, dR, mL, mR, pm, total;
};
__host__ __device__ inline ScratchCg scratch_cg(int g, int W, int R) {
  ScratchCg s;
  const size_t dirs = (size_t)(g + 1) * 4u * (size_t)R * 8u, mat = align16((size_t)(g + 1) * (size_t)W * 4u);
  size_t off = 0;
  s.dL = off; off += dirs;
  s.dR = off; off += dirs;
  s.mL = off; off += mat;
  s.mR = off; off += mat;
  s.pm = off; off += (size_t)(g + 1) * (size_t)W * 8u;
  s.total = align16(off);
  return s;
}
struct CarveCg {
  size_t scL, scR, gclL, gclR, total;
};
__host__ __device__ inline CarveCg carve_cg(int rl, int g) {
  CarveCg cv;
  const size_t srow = (size_t)(rl + 2);
  size_t off = 0;
  cv.scL = off;  off = align16(off + (size_t)kNClass * srow);
  cv.scR = off;  off = align16(off + (size_t)kNClass * srow);
  cv.gclL = off; off = align16(off + (size_t)(g + 2));
  cv.gclR = off; off = align16(off + (size_t)(g + 2));
  cv.total = off;
  return cv;
}
// SIMD: wave steps of the four triangles (4 x 16-lane segments, or 2 x 32 with L then R in each)
template <int B>
__host__ __device__ inline int uxc_tmax(int rl, int g, int lband, int uband) {
  const int su = ux_steps(rl, uband, B), sl = ux_steps(g, lband, B);
  return B == 16 ? max(su, sl) : 2 * max(su, sl);
}

// ===========================================================================
// cg_kernel<R>: nosimd.  One wave per problem: L fill, R fill (band-lane fills storing their
// scores), the bridge, the tracebacks.
// ===========================================================================
template <int R>
__global__ __launch_bounds__(64) void cg_kernel(
    const DevCdnaProblem* __restrict__ probs, const int* __restrict__ order, unsigned char* __restrict__ gscratch,
    const uint32_t* __restrict__ blocks, uint64_t nwords, const char* __restrict__ qseq,
    const char* __restrict__ qseq_uc, const int8_t* __restrict__ sctab, const uint8_t* __restrict__ constab,
    gmapdp_cdna_result* __restrict__ results, gmapdp_pair* __restrict__ pairs) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int lane = threadIdx.x;
  const int pid = order[blockIdx.x];
  const DevCdnaProblem P = probs[pid];
  const int rl = P.rlength, g = P.glength, lband = P.lband, uband = P.uband;
  const int W = lband + uband + 1;
  const int late = (P.flags & kFLate) ? 1 : 0;
  const bool watson = P.flags & kFWatson;
  const CarveCg cv = carve_cg(rl, g);
  int8_t* scL = reinterpret_cast<int8_t*>(smem + cv.scL);
  int8_t* scR = reinterpret_cast<int8_t*>(smem + cv.scR);
  uint8_t* gclL = smem + cv.gclL;
  uint8_t* gclR = smem + cv.gclR;
  const ScratchCg sg = scratch_cg(g, W, R);
  unsigned char* base = gscratch + P.scratch_offset;
  uint64_t* dL = reinterpret_cast<uint64_t*>(base + sg.dL);
  uint64_t* dR = reinterpret_cast<uint64_t*>(base + sg.dR);
  int* mL = reinterpret_cast<int*>(base + sg.mL);
  int* mR = reinterpret_cast<int*>(base + sg.mR);
  int2* pm = reinterpret_cast<int2*>(base + sg.pm);
  const int8_t* sct = sctab + (size_t)P.mismatchtype * 128 * kNClass;
  const uint8_t* cons = constab + (size_t)P.genestrand * 128 * kNClass;
  const int srow = rl + 2;

  // ---- stage: per-class score rows of both query pieces (the fills score rsequence), genome classes ----
  for (int i = lane; i < rl; i += 64) {
    const uint64_t ra = *reinterpret_cast<const uint64_t*>(sct + (uint8_t)(qseq[P.qbaseL + i] & 127) * kNClass);
    const uint64_t rb = *reinterpret_cast<const uint64_t*>(sct + (uint8_t)(qseq[P.qbaseR - i] & 127) * kNClass);
#pragma unroll
    for (int c = 0; c < 6; c++) {
      scL[c * srow + i + 1] = (int8_t)(ra >> (8 * c));
      scR[c * srow + i + 1] = (int8_t)(rb >> (8 * c));
    }
  }
  if (lane < 6) {  // rows 0 and rlength+1 are never scored but keep the clamped reads defined
    scL[lane * srow] = scL[lane * srow + rl + 1] = 0;
    scR[lane * srow] = scR[lane * srow + rl + 1] = 0;
  }
  cdna_stage_genome(lane, P, blocks, nwords, gclL, gclR);
  __syncthreads();

  // ---- the two fills (dynprog_cdna.c:1205-1219) ----
  int br, bc;
  fill_band<R, false, 64, false, true>(lane, rl, g, lband, uband, P.open, P.extend, late, 0, scL, srow, gclL, dL,
                                       nullptr, br, bc, 0, mL);
  fill_band<R, false, 64, false, true>(lane, rl, g, lband, uband, P.open, P.extend, 1 - late, 0, scR, srow, gclR,
                                       dR, nullptr, br, bc, 0, mR);
  __threadfence_block();

  // ---- bridge_cdna_gap (:652), its own bands equal the fills' inside the domain ----
  const BandCells cL{mL, W, uband, P.open, P.extend}, cR{mR, W, uband, P.open, P.extend};
  const CgBest b = cdna_bridge(lane, cL, cR, g, rl, lband, uband, P.open, late, kNegInf32,
                               P.rev_roffsetR - P.roffsetL, pm, W);

  // ---- tracebacks (Dynprog_traceback_std) ----
  const int rev_goffset = P.goffset + g - 1;
  const Geo GL{P.roffsetL, P.goffset, 1}, GR{P.rev_roffsetR, rev_goffset, -1};
  const QView qL{qseq + P.qbaseL, 1}, qucL{qseq_uc + P.qbaseL, 1};
  const QView qR{qseq + P.qbaseR, -1}, qucR{qseq_uc + P.qbaseR, -1};
  const GClassView gchL{gclL}, gchR{gclR};
  gmapdp_pair* out = pairs + P.pair_offset;
  auto traceR = [&](Tally& t) {
    traceback_band<R, uint64_t, QView, GClassView>(lane, dR, W, uband, b.rR, b.cR, GR, qR, qucR, gchR, cons, watson,
                                                   P.chroffset, P.chrhigh, blocks, nwords, out, t);
  };
  auto traceL = [&](Tally& t) {
    traceback_band<R, uint64_t, QView, GClassView>(lane, dL, W, uband, b.rL, b.cL, GL, qL, qucL, gchL, cons, watson,
                                                   P.chroffset, P.chrhigh, blocks, nwords, out, t);
  };
  cdna_finish(lane, P, pid, b, traceR, traceL, qseq, blocks, nwords, results, out);
}

// ===========================================================================
// uxc_kernel<B>: SIMD builds.  One wave per problem: the four triangles (L upper, L lower, R upper,
// R lower) concurrently in the wave's segments, the bridge, the upper/lower tracebacks.
// ===========================================================================
template <int B>
__global__ __launch_bounds__(64) void uxc_kernel(
    const DevCdnaProblem* __restrict__ probs, const int* __restrict__ order, unsigned char* __restrict__ gscratch,
    const uint32_t* __restrict__ blocks, uint64_t nwords, const char* __restrict__ qseq,
    const char* __restrict__ qseq_uc, const int8_t* __restrict__ sctab, const uint8_t* __restrict__ constab,
    gmapdp_cdna_result* __restrict__ results, gmapdp_pair* __restrict__ pairs) {
  constexpr int NEG = (B == 32) ? -128 : -32768;
  constexpr int NSEG = 64 / B;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int lane = threadIdx.x;
  const int pid = order[blockIdx.x];
  const DevCdnaProblem P = probs[pid];
  const int rl = P.rlength, g = P.glength, lband = P.lband, uband = P.uband;
  const int W = lband + uband + 1;
  const int late = (P.flags & kFLate) ? 1 : 0;
  const bool watson = P.flags & kFWatson;
  const CarveUx cvL = carve_ux(rl, g, B, 0), cvR = carve_ux(rl, g, B, cvL.total);
  uint8_t* gclL = smem + cvL.gcl;
  uint8_t* gclR = smem + cvR.gcl;
  const int8_t* sct = sctab + (size_t)P.mismatchtype * 128 * kNClass;
  const uint8_t* cons = constab + (size_t)P.genestrand * 128 * kNClass;
  const int tmax = uxc_tmax<B>(rl, g, lband, uband);
  unsigned char* base = gscratch + P.scratch_offset;
  uint64_t* wd = reinterpret_cast<uint64_t*>(base);
  int16_t* ws = reinterpret_cast<int16_t*>(base + 16 * (size_t)tmax);
  int2* pm = reinterpret_cast<int2*>(base + 144 * (size_t)tmax);

  cdna_stage_genome(lane, P, blocks, nwords, gclL, gclR);
  __syncthreads();
  ux_stage<B>(lane, smem, cvL, rl, g, qseq + P.qbaseL, 1, sct);
  ux_stage<B>(lane, smem, cvR, rl, g, qseq + P.qbaseR, -1, sct);
  __syncthreads();

  // ---- the four triangles (dynprog_cdna.c:944-975 / 1075-1105); R with !jump_late_p ----
  UxFill F[4];
  const int su = ux_steps(rl, uband, B), sl = ux_steps(g, lband, B);
  F[0] = ux_fill<B>(smem, cvL, true, rl, g, uband, late, P.open, P.extend, 0);
  F[1] = ux_fill<B>(smem, cvL, false, rl, g, lband, late, P.open, P.extend, 0);
  F[2] = ux_fill<B>(smem, cvR, true, rl, g, uband, 1 - late, P.open, P.extend, B == 32 ? su : 0);
  F[3] = ux_fill<B>(smem, cvR, false, rl, g, lband, 1 - late, P.open, P.extend, B == 32 ? sl : 0);
  ux_run_fills<B>(lane, F, 4, tmax, wd, ws);
  __threadfence_block();
  __syncthreads();
  const UxView VLu = ux_view(wd, ws, 0 % NSEG, B, F[0], true), VLl = ux_view(wd, ws, 1 % NSEG, B, F[1], false);
  const UxView VRu = ux_view(wd, ws, 2 % NSEG, B, F[2], true), VRl = ux_view(wd, ws, 3 % NSEG, B, F[3], false);

  // ---- bridge_cdna_gap_{8,16}_ud (:124/:387) over the fill bands ----
  const UdCells cL{VLu, VLl}, cR{VRu, VRl};
  const CgBest b = cdna_bridge(lane, cL, cR, g, rl, lband, uband, P.open, late, NEG, P.rev_roffsetR - P.roffsetL,
                               pm, W);

  // ---- tracebacks: Dynprog_traceback_{8,16}_upper when bestc >= bestr, else _lower ----
  const int rev_goffset = P.goffset + g - 1;
  const Geo GL{P.roffsetL, P.goffset, 1}, GR{P.rev_roffsetR, rev_goffset, -1};
  const QView qL{qseq + P.qbaseL, 1}, qucL{qseq_uc + P.qbaseL, 1};
  const QView qR{qseq + P.qbaseR, -1}, qucR{qseq_uc + P.qbaseR, -1};
  const GClassView gchL{gclL}, gchR{gclR};
  gmapdp_pair* out = pairs + P.pair_offset;
  const bool upR = b.cR >= b.rR, upL = b.cL >= b.rL;
  auto traceR = [&](Tally& t) {
    traceback_walk(lane, upR ? VRu : VRl, b.rR, b.cR, GR, qR, qucR, gchR, cons, watson, P.chroffset, P.chrhigh,
                   blocks, nwords, out, t, upR ? 1 : 2);
  };
  auto traceL = [&](Tally& t) {
    traceback_walk(lane, upL ? VLu : VLl, b.rL, b.cL, GL, qL, qucL, gchL, cons, watson, P.chroffset, P.chrhigh,
                   blocks, nwords, out, t, upL ? 1 : 2);
  };
  cdna_finish(lane, P, pid, b, traceR, traceL, qseq, blocks, nwords, results, out);
}

// ---- host-side sizes and launches ----
// RB: band words per lane R (nosimd) or the fill width B (SIMD, 16 / 32)
size_t lds_bytes_cg(int rlength, int glength, bool simd, int RB) {
  if (!simd) return carve_cg(rlength, glength).total;
  const CarveUx a = carve_ux(rlength, glength, RB, 0);
  return carve_ux(rlength, glength, RB, a.total).total;
}
size_t scratch_bytes_cg(int rlength, int glength, int lband, int uband, bool simd, int RB) {
  const int W = lband + uband + 1;
  if (!simd) return scratch_cg(glength, W, RB).total;
  const int tmax = RB == 32 ? uxc_tmax<32>(rlength, glength, lband, uband) : uxc_tmax<16>(rlength, glength, lband, uband);
  return align16(144u * (size_t)tmax + (size_t)(glength + 1) * (size_t)W * 8u);
}

hipError_t launch_cg(bool simd, int RB, int nproblems, size_t lds, hipStream_t stream, const DevCdnaProblem* probs,
                     const int* order, unsigned char* gscratch, const uint32_t* blocks, uint64_t nwords,
                     const char* qseq, const char* qseq_uc, const int8_t* sctab, const uint8_t* constab,
                     gmapdp_cdna_result* results, gmapdp_pair* pairs) {
  void* fn = nullptr;
  if (simd) {
    if (RB == 16) fn = reinterpret_cast<void*>(&uxc_kernel<16>);
    else if (RB == 32) fn = reinterpret_cast<void*>(&uxc_kernel<32>);
  } else {
    switch (RB) {
      case 1: fn = reinterpret_cast<void*>(&cg_kernel<1>); break;
      case 2: fn = reinterpret_cast<void*>(&cg_kernel<2>); break;
      case 4: fn = reinterpret_cast<void*>(&cg_kernel<4>); break;
      case 8: fn = reinterpret_cast<void*>(&cg_kernel<8>); break;
      case 16: fn = reinterpret_cast<void*>(&cg_kernel<16>); break;
      case 32: fn = reinterpret_cast<void*>(&cg_kernel<32>); break;
      case 64: fn = reinterpret_cast<void*>(&cg_kernel<64>); break;
      default: break;
    }
  }
  if (!fn) return hipErrorInvalidValue;
  if (lds > 64 * 1024) {
    hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
  }
  void* args[] = {(void*)&probs, (void*)&order, (void*)&gscratch, (void*)&blocks, (void*)&nwords, (void*)&qseq,
                  (void*)&qseq_uc, (void*)&sctab, (void*)&constab, (void*)&results, (void*)&pairs};
  return hipLaunchKernel(fn, dim3(nproblems), dim3(64), args, lds, stream);
}

}  // namespace gmapdp
