// ux_kernel.hip -- CDNA4 (gfx950) kernels for Dynprog_end5_gap / Dynprog_end3_gap and
// Dynprog_genome_gap as GMAP's SIMD builds compute them (gmap.sse42 / .avx2 / .avx512 link
// dynprog_simd.c; SURVEY §8 "S" semantics, selected per problem with GMAPDP_SIMD).
//
// Reference semantics restated (paths under the reference tree's src/):
//   Dynprog_simd_8_upper / _16_upper   dynprog_simd.c:4304 / 7714  (c >= r, horizontal gaps only)
//   Dynprog_simd_8_lower / _16_lower   dynprog_simd.c:5340 / 8586  (r >= c, vertical gaps only)
//   Dynprog_traceback_{8,16}_upper/_lower  dynprog_simd.c:9319/9439, 9716/9836
//   find_best_endpoint_8/_16, ..._to_queryend_indels_8/_16   dynprog_end.c:144/220, 359/437
//   Dynprog_end5_gap / _end3_gap SIMD branches   dynprog_end.c:1406-1610 / 2027-2220
//   Dynprog_genome_gap SIMD branch     dynprog_genome.c:3501-3795
//   bridge_intron_gap_8_ud/_16_ud -> _site_level   dynprog_genome.c:1388/2263 -> 867/1742
//
// The triangle fills have no intra-column recurrence: a cell takes its diagonal from
// (r-1, c-1) and its one gap type from the previous step (upper: (r, c-1), lower: (r-1, c)).
// They are emulated block by block exactly as the reference's vectors run them -- one B-lane
// DPP segment per fill (B = 32 for the 8-bit fills, 16 for the 16-bit ones, the AVX2 widths,
// dynprog.h:128-133), lane = query row (upper) / genome column (lower) inside the block, one
// wave step per column (upper) / row (lower) -- with int8/int16 saturating arithmetic, the
// E_mask that pins a lane's gap to NEG until the lane leaves the diagonal, the diagonal
// forced DIAG, the row above a block read from the previous block's last lane (two LDS
// buffers by block parity), and cells no block wrote reading 0 / DIAG (a zeroed Dynprog_T
// arena; the reference never clears it -- DESIGN.md "Parity").  All fills of a problem run
// concurrently in the segments of one wave (4 x 16 lanes, or 2 x 32 lanes with two fills
// each); per step the wave stores two ballots (nogap, gap) and each lane its score (int16)
// in an L2-resident scratch.  The endpoint scan (end gaps) or the bridge (genome gaps) and
// the upper/lower tracebacks then run with the whole wave.
#include "ux_device.h"

namespace gmapdp {

// ===========================================================================
// uxe_kernel<B>: Dynprog_end5_gap / Dynprog_end3_gap, SIMD builds.  One wave per problem:
// segment 0 the upper triangle, segment 1 the lower one.
// ===========================================================================
template <int B>
__global__ __launch_bounds__(64) void uxe_kernel(
    const DevProblem* __restrict__ probs, const int* __restrict__ order, unsigned char* __restrict__ gscratch,
    const uint32_t* __restrict__ blocks, uint64_t nwords, const char* __restrict__ qseq,
    const char* __restrict__ qseq_uc, const int8_t* __restrict__ sctab, const uint8_t* __restrict__ constab,
    gmapdp_result* __restrict__ results, gmapdp_pair* __restrict__ pairs) {
  constexpr int NEG = (B == 32) ? -128 : -32768;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int lane = threadIdx.x;
  const int pid = order[blockIdx.x];
  const DevProblem P = probs[pid];
  const int rlen = P.rlength, glen = P.glength, flags = P.flags;
  const int late = (flags & kFLate) ? 1 : 0;
  const bool rev = flags & kFRev;
  const int qstep = rev ? -1 : 1;
  const int8_t* sct = sctab + (size_t)P.mismatchtype * 128 * kNClass;
  const CarveUx cv = carve_ux(rlen, glen, B, 0);
  uint8_t* gcl = smem + cv.gcl;

  // ---- stage: genome classes (end5 walks the segment from its right end), lane words ----
  const bool segleft = flags & kFSegLeft, segrc = flags & kFSegRevcomp;
  for (int i = lane; i < glen; i += 64) {
    const char c2 = segment_nt(blocks, nwords, (uint32_t)i, (uint32_t)glen, P.segpos, P.segbound, segleft, segrc);
    gcl[rev ? glen - i : i + 1] = gclass(c2);
  }
  __syncthreads();
  const char* qfill = ((flags & kFScoreUC) ? qseq_uc : qseq) + P.qbase;  // end3 fills on rsequenceuc
  ux_stage<B>(lane, smem, cv, rlen, glen, qfill, qstep, sct);
  __syncthreads();

  // ---- the two triangles, concurrently ----
  UxFill F[2];
  F[0] = ux_fill<B>(smem, cv, true, rlen, glen, P.uband, late, P.open, P.extend, 0);
  F[1] = ux_fill<B>(smem, cv, false, rlen, glen, P.lband, late, P.open, P.extend, 0);
  const int tmax = max(ux_steps(rlen, P.uband, B), ux_steps(glen, P.lband, B));
  uint64_t* wd = reinterpret_cast<uint64_t*>(gscratch + P.dirs_offset);
  int16_t* ws = reinterpret_cast<int16_t*>(gscratch + P.dirs_offset + 16 * (size_t)tmax);
  ux_run_fills<B>(lane, F, 2, tmax, wd, ws);
  __threadfence_block();
  __syncthreads();
  const UxView VU = ux_view(wd, ws, 0, B, F[0], true), VL = ux_view(wd, ws, 1, B, F[1], false);

  // ---- find_best_endpoint_8/16 or _to_queryend_indels_8/16: lower[r][c] for c < r (bounded by r,
  //      not chigh), then upper[c][r] up to chigh; > keeps the first cell, >= the last ----
  const bool indels = P.endalign == kQueryendIndels;
  const int init = indels ? NEG : 0;
  uint64_t key = 0;
  auto take = [&](int r, int c, int s) {
    if (late ? (s >= init) : (s > init)) {
      const uint32_t ord = ((uint32_t)r << 12) | (uint32_t)c;
      const uint64_t kk = ((uint64_t)(uint32_t)(s + (1 << 30)) << 24) | (late ? ord : 0xffffffu - ord);
      key = kk > key ? kk : key;
    }
  };
  if (indels) {  // one row
    const int r = rlen, clo = max(1, r - P.lband), cend = max(r - 1, min(r + P.uband, glen));
    for (int c = clo + lane; c <= cend; c += 64) take(r, c, (c < r) ? VL.cell(r, c) : VU.cell(r, c));
  } else {
    // the key is a total order, so the cells go in any order: the lower cells (c < r) by column
    // blocks of the lower fill, the upper ones by row blocks of the upper fill, lane = (row or
    // column in the block, group), B consecutive lanes of one step per load
    constexpr int NSEG = 64 / B;
    const int i = lane & (B - 1), g = lane / B;
    for (int lo = 0; lo < rlen; lo += B) {  // lower cells by column blocks: c = lo + i, rows r = x
      const int c = lo + i;
      const int xend = min(lo + B - 1 + P.lband, rlen);
      for (int x0 = lo + 1; x0 <= xend; x0 += NSEG) {
        const int r = x0 + g;
        if (c >= 1 && r <= rlen && c < r && c >= r - P.lband) take(r, c, VL.cell(r, c));
      }
    }
    for (int lo = 0; lo <= rlen; lo += B) {
      const int r = lo + i;
      const bool row = r >= 1 && r <= rlen;
      const int cu = row ? max(max(1, r - P.lband), r) : 1, ce = row ? max(r - 1, min(r + P.uband, glen)) : 0;
      const int xend = min(lo + B - 1 + P.uband, glen);
      for (int x0 = lo; x0 <= xend; x0 += NSEG) {
        const int c = x0 + g;
        if (c >= cu && c <= ce) take(r, c, VU.cell(r, c));
      }
    }
  }
  key = wave_max_u64(key);
  int bestr, bestc;
  if (key == 0) {
    bestr = indels ? rlen : 0;
    bestc = 0;
  } else {
    const uint32_t ord = late ? (uint32_t)(key & 0xffffffu) : 0xffffffu - (uint32_t)(key & 0xffffffu);
    bestr = (int)(ord >> 12);
    bestc = (int)(ord & 4095u);
  }
  // Dynprog_traceback_{8,16}_upper when bestc >= bestr, else _lower (dynprog_end.c:1574-1610)
  const bool up = bestc >= bestr;
  finish_dp(lane, P, pid, false, bestr, bestc, up ? VU : VL, QView{qseq + P.qbase, qstep},
            QView{qseq_uc + P.qbase, qstep}, GClassView{gcl}, constab, blocks, nwords, results, pairs, up ? 1 : 2);
}

// ===========================================================================
// uxg_kernel<B>: Dynprog_genome_gap, SIMD builds.  One wave per problem: genome_gap_simple
// first (as the nosimd kernel), then the four triangles (L upper, L lower, R upper, R lower)
// concurrently, the bridge (bridge_intron_gap_*_site_level over the triangles), the R and L
// tracebacks around the intron gap holder and Pair_maxnegscore.
// ===========================================================================
struct CarveUxg {
  CarveUx L, R;
  size_t pL, pR, ldi, rdi, isc, total;
};
template <int B>
__host__ __device__ inline CarveUxg carve_uxg(int rlength, int glengthL, int glengthR) {
  CarveUxg cv;
  size_t off = 0;
  cv.pL = off;  off = align16(off + 8u * (size_t)glengthL);
  cv.pR = off;  off = align16(off + 8u * (size_t)glengthR);
  cv.ldi = off; off = align16(off + (size_t)(glengthL + 2));
  cv.rdi = off; off = align16(off + (size_t)(glengthR + 2));
  cv.isc = off; off = align16(off + 64);
  cv.L = carve_ux(rlength, glengthL, B, off);
  cv.R = carve_ux(rlength, glengthR, B, cv.L.total);
  cv.total = cv.R.total;
  return cv;
}
// wave steps of the genome-gap fills: 4 x 16-lane segments, or 2 x 32 with L then R in each
template <int B>
__host__ __device__ inline int uxg_tmax(int rlength, int glengthL, int glengthR, int extraband) {
  const int uL = glengthL - rlength + extraband, uR = glengthR - rlength + extraband, l = extraband;
  const int a = ux_steps(rlength, uL, B), b = ux_steps(glengthL, l, B);
  const int c = ux_steps(rlength, uR, B), d = ux_steps(glengthR, l, B);
  if (B == 16) return max(max(a, b), max(c, d));
  return max(a + c, b + d);
}

template <int B>
__global__ __launch_bounds__(64) void uxg_kernel(
    const DevGenomeProblem* __restrict__ probs, const int* __restrict__ order, unsigned char* __restrict__ gscratch,
    const uint32_t* __restrict__ blocks, uint64_t nwords, const char* __restrict__ qseq,
    const char* __restrict__ qseq_uc, const double* __restrict__ sprob, const int8_t* __restrict__ sctab,
    const uint8_t* __restrict__ constab, const int8_t* __restrict__ isctab,
    gmapdp_genome_result* __restrict__ results, gmapdp_pair* __restrict__ pairs, const uint8_t* __restrict__ known) {
  constexpr int NEG = (B == 32) ? -128 : -32768;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int lane = threadIdx.x;
  const int pid = order[blockIdx.x];
  const DevGenomeProblem P = probs[pid];
  const int rlen = P.rlength, gL = P.glengthL, gR = P.glengthR, flags = P.flags;
  const int late = (flags & kFLate) ? 1 : 0;
  const bool watson = flags & kFWatson;
  const int eb = P.lbandL;  // extraband_paired: lbandL = lbandR (Dynprog_compute_bands, glength > rlength)
  const int ubandL = P.ubandL, ubandR = P.ubandR;
  const uint8_t* kb = (flags & kGKnown) ? known + P.known_offset : nullptr;  // known splice sites
  const CarveUxg cv = carve_uxg<B>(rlen, gL, gR);
  double* pL = reinterpret_cast<double*>(smem + cv.pL);
  double* pR = reinterpret_cast<double*>(smem + cv.pR);
  uint8_t* ldi = smem + cv.ldi;
  uint8_t* rdi = smem + cv.rdi;
  int8_t* isc = reinterpret_cast<int8_t*>(smem + cv.isc);
  uint8_t* gclL = smem + cv.L.gcl;
  uint8_t* gclR = smem + cv.R.gcl;
  const int8_t* sct = sctab + (size_t)P.mismatchtype * 128 * kNClass;
  const uint8_t* cons = constab + (size_t)P.genestrand * 128 * kNClass;
  const QView qL{qseq + P.qbase, 1}, qucL{qseq_uc + P.qbase, 1};
  const QView qR{qseq + P.qbase + rlen - 1, -1}, qucR{qseq_uc + P.qbase + rlen - 1, -1};
  const GClassView gchL{gclL}, gchR{gclR};
  gmapdp_pair* out = pairs + P.pair_offset;
  const int rev_roffset = P.roffset + rlen - 1;
  const Geo GL{P.roffset, P.goffsetL, 1};
  const Geo GR{rev_roffset, P.rev_goffsetR, -1};
  const int tmax = uxg_tmax<B>(rlen, gL, gR, eb);
  uint64_t* wd = reinterpret_cast<uint64_t*>(gscratch + P.dirs_offset);
  int16_t* ws = reinterpret_cast<int16_t*>(gscratch + P.dirs_offset + 16 * (size_t)tmax);
  int* diagL = reinterpret_cast<int*>(gscratch + P.dirs_offset + 144 * (size_t)tmax);
  int* diagR = diagL + (rlen + 1);

  // ---- stage: genome classes of both segments, splice probabilities, dinucleotides, lane words ----
  for (int i = lane; i < gL; i += 64) {
    const char c2 = segment_nt(blocks, nwords, (uint32_t)i, (uint32_t)gL, P.segposL, P.segboundL,
                               flags & kGSegLLeft, flags & kGSegLRc);
    gclL[i + 1] = gclass(c2);
    pL[i] = (kb && kb[i]) ? 1.0 : sprob[P.prob_offset + i];  // known sites: 1.0 (dynprog_genome.c:978)
  }
  for (int i = lane; i < gR; i += 64) {
    const char c2 = segment_nt(blocks, nwords, (uint32_t)i, (uint32_t)gR, P.segposR, P.segboundR,
                               flags & kGSegRLeft, flags & kGSegRRc);
    gclR[gR - i] = gclass(c2);  // rev_gsequenceR[1-c] = segment[glengthR-c]
    pR[i] = (kb && kb[gL + i]) ? 1.0 : sprob[P.prob_offset + gL + i];
  }
  isc[lane] = isctab[(size_t)P.iclass * 128 + ((flags & kGFinal) ? 64 : 0) + lane];
  __syncthreads();
  for (int c = lane; c <= gL; c += 64) ldi[c] = (c < gL - 1) ? left_dinucl(gchL[c + 1], gchL[c + 2]) : 0;
  for (int c = lane; c <= gR; c += 64) rdi[c] = (c < gR - 1) ? right_dinucl(gchR[c + 2], gchR[c + 1]) : 0;
  ux_stage<B>(lane, smem, cv.L, rlen, gL, qseq + P.qbase, 1, sct);
  ux_stage<B>(lane, smem, cv.R, rlen, gR, qseq + P.qbase + rlen - 1, -1, sct);
  __syncthreads();

  gmapdp_genome_result res;
  res.npairs = 0;
  res.pair_offset = P.pair_offset;
  res.traceback_score = 0;
  res.nmatches = res.nmismatches = res.nopens = res.nindels = 0;
  res.dynprogindex = P.dynprogindex;
  res.new_leftgenomepos = res.new_rightgenomepos = res.exonhead = kUnset;
  res.introntype = 0;
  res.gap_index = -1;
  res.gap_queryjump = 0;
  res.left_prob = res.right_prob = 0.0;
  const int dpi_next = P.dynprogindex + (P.dynprogindex > 0 ? 1 : -1);

  // ---- 1. genome_gap_simple (dynprog_genome.c:3479-3498), before the SIMD branch ----
  if ((flags & kGSimple) && gg_simple_wave(lane, P, pid, sctab, isctab, cons, qL, qucL, qR, qucR, gclL, gclR, gchL,
                                           gchR, ldi, rdi, pL, pR, diagL, diagR, out, res, results,
                                           kb ? kb + gL + gR : nullptr, sprob + P.prob_offset))
    return;

  // ---- 2. the four triangles (:3510-3547 / :3655-3689); the R side runs with !jump_late_p ----
  UxFill F[4];
  const int sLu = ux_steps(rlen, ubandL, B), sLl = ux_steps(gL, eb, B);
  F[0] = ux_fill<B>(smem, cv.L, true, rlen, gL, ubandL, late, P.open, P.extend, 0);
  F[1] = ux_fill<B>(smem, cv.L, false, rlen, gL, eb, late, P.open, P.extend, 0);
  F[2] = ux_fill<B>(smem, cv.R, true, rlen, gR, ubandR, 1 - late, P.open, P.extend, B == 32 ? sLu : 0);
  F[3] = ux_fill<B>(smem, cv.R, false, rlen, gR, eb, 1 - late, P.open, P.extend, B == 32 ? sLl : 0);
  ux_run_fills<B>(lane, F, 4, tmax, wd, ws);
  __threadfence_block();
  __syncthreads();
  constexpr int NSEG = 64 / B;
  const UxView VLu = ux_view(wd, ws, 0 % NSEG, B, F[0], true), VLl = ux_view(wd, ws, 1 % NSEG, B, F[1], false);
  const UxView VRu = ux_view(wd, ws, 2 % NSEG, B, F[2], true), VRl = ux_view(wd, ws, 3 % NSEG, B, F[3], false);

  // ---- 3. bridge_intron_gap_{8,16}_site_level (:867-1384): per row rL the candidates A; B over
  //      R lower then (diagonal skipped) R upper; C over L lower then L upper.  The sequential
  //      rule ("> score, or = score and > prob") keeps the lexicographic max of (score, probL +
  //      probR) that comes first in scan order; lanes take the candidates of a row in parallel and
  //      keep their own best, merged at the end.  bestscore starts at NEG_INFINITY_8/16. ----
  const int rdist = P.rev_goffsetR - P.goffsetL;  // "cR < rightoffset - leftoffset - cL"
  int ws_ = NEG, wrL = -1, wcL = 0, wcR = 0, word = -1;  // the initial state wins ties with it
  double wp = 0.0;
  int ds = NEG, drL = 0x7fffffff;  // best dinucleotide (A) candidate: max prob, earliest
  double dp = 0.0;
  // The candidates go in any order: the rule is a total order on (score, prob, scan order), and
  // the A candidates' dinucleotide first-max rule holds per lane (a lane's rows ascend) and in the
  // merge (earliest row wins ties).  Every cell is read where its fill stored it side by side:
  // the upper-triangle cells by row blocks of the upper fill (lane = row in the block, column
  // group), the lower-triangle cells by column blocks of the lower fill (lane = column in the
  // block, row group), so one load reads B consecutive lanes of one step (32-64 B).  The
  // diagonal cells, one per row and side, are staged in LDS first (the fills' block-row buffers
  // are free by now).
  auto take = [&](int s, double pr, int ordv, int rL, int cL, int cR) {
    if (s > ws_ || (s == ws_ && (pr > wp || (pr == wp && ordv < word)))) {
      ws_ = s; wp = pr; wrL = rL; wcL = cL; wcR = cR; word = ordv;
    }
  };
  int* dgL = reinterpret_cast<int*>(smem + cv.L.bufU);  // 4 (gL + 1) >= 4 (rlen + 1) bytes
  int* dgR = reinterpret_cast<int*>(smem + cv.R.bufU);
  for (int r = lane; r <= rlen; r += 64) {
    dgL[r] = VLu.cell(r, r);
    dgR[r] = VRu.cell(r, r);
  }
  __syncthreads();
  // A: cL = rL, cR = rR
  for (int rL = 1 + lane; rL < rlen; rL += 64) {
    const int rR = rlen - rL;
    const int sI = isc[ldi[rL] & rdi[rR]];
    const int s = dgL[rL] + sI + dgR[rR];
    const double pr = pL[rL] + pR[rR];
    take(s, pr, (rL << 14) | rL, rL, rL, rR);
    if (sI > 0 && pr > dp) {  // first max of this lane's rows
      dp = pr;
      ds = s;
      drL = rL;
    }
  }
  {
    const int i = lane & (B - 1), g = lane / B;
    // B lower: cL = rL, cR in [cloR, eB) (cR < rR): column blocks of VRl, rows rR = x
    for (int lo = 0; lo < rlen; lo += B) {
      const int cR = lo + i;
      const int xend = min(lo + B - 1 + eb, rlen - 1);
      for (int x0 = lo + 1; x0 <= xend; x0 += NSEG) {
        const int rR = x0 + g, rL = rlen - rR;
        if (cR < 1 || rR > rlen - 1) continue;
        const int cloR = max(1, rR - eb), eB = max(cloR, min(rR, rdist - rL));
        if (cR >= cloR && cR < eB) {
          const int sI = isc[ldi[rL] & rdi[cR]];
          take(dgL[rL] + sI + VRl.cell(rR, cR), pL[rL] + pR[cR], (rL << 14) | (1 << 12) | cR, rL, rL, cR);
        }
      }
    }
    // C lower: cR = rR, cL in [cloL, eC) (cL < rL): column blocks of VLl, rows rL = x
    for (int lo = 0; lo < rlen; lo += B) {
      const int cL = lo + i;
      const int xend = min(lo + B - 1 + eb, rlen - 1);
      for (int x0 = lo + 1; x0 <= xend; x0 += NSEG) {
        const int rL = x0 + g, rR = rlen - rL;
        if (cL < 1 || rL > rlen - 1) continue;
        const int cloL = max(1, rL - eb), eC = max(cloL, min(rL, rdist - rR));
        if (cL >= cloL && cL < eC) {
          const int sI = isc[ldi[cL] & rdi[rR]];
          take(VLl.cell(rL, cL) + sI + dgR[rR], pL[cL] + pR[rR], (rL << 14) | (2 << 12) | cL, rL, cL, rR);
        }
      }
    }
    // C upper: cR = rR, cL in [eC + 1, min(chighL, rdist - rR)): row blocks of VLu
    for (int lo = 0; lo < rlen; lo += B) {
      const int rL = lo + i, rR = rlen - rL;
      int cu = 0, ce = 0;
      if (rL >= 1 && rL < rlen) {
        const int limC = rdist - rR;
        cu = max(max(1, rL - eb), min(rL, limC)) + 1;
        ce = min(min(rL + ubandL, gL - 1), limC);
      }
      const int xend = min(lo + B - 1 + ubandL, gL - 1);
      for (int x0 = lo + 1; x0 < xend; x0 += NSEG) {
        const int cL = x0 + g;
        if (cL >= cu && cL < ce) {
          const int sI = isc[ldi[cL] & rdi[rR]];
          take(VLu.cell(rL, cL) + sI + dgR[rR], pL[cL] + pR[rR], (rL << 14) | (2 << 12) | cL, rL, cL, rR);
        }
      }
    }
    // B upper: cL = rL, cR in [eB + 1, min(chighR, rdist - rL)): row blocks of VRu
    for (int lo = 0; lo < rlen; lo += B) {
      const int rR = lo + i, rL = rlen - rR;
      int cu = 0, ce = 0;
      if (rR >= 1 && rR < rlen) {
        const int limB = rdist - rL;
        cu = max(max(1, rR - eb), min(rR, limB)) + 1;
        ce = min(min(rR + ubandR, gR - 1), limB);
      }
      const int xend = min(lo + B - 1 + ubandR, gR - 1);
      for (int x0 = lo + 1; x0 < xend; x0 += NSEG) {
        const int cR = x0 + g;
        if (cR >= cu && cR < ce) {
          const int sI = isc[ldi[rL] & rdi[cR]];
          take(dgL[rL] + sI + VRu.cell(rR, cR), pL[rL] + pR[cR], (rL << 14) | (1 << 12) | cR, rL, rL, cR);
        }
      }
    }
  }
  // merge the lanes: (score desc, prob desc, scan order asc); the untouched initial state
  // (NEG, 0.0) only wins when no candidate beat it, as in the reference
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {
    const int s2 = __shfl_xor(ws_, off, 64);
    const double p2 = __shfl_xor(wp, off, 64);
    const int o2 = __shfl_xor(word, off, 64);
    const int r2 = __shfl_xor(wrL, off, 64);
    const int cl2 = __shfl_xor(wcL, off, 64);
    const int cr2 = __shfl_xor(wcR, off, 64);
    const int ds2 = __shfl_xor(ds, off, 64);
    const double dp2 = __shfl_xor(dp, off, 64);
    const int dr2 = __shfl_xor(drL, off, 64);
    if (s2 > ws_ || (s2 == ws_ && (p2 > wp || (p2 == wp && o2 < word)))) {
      ws_ = s2; wp = p2; word = o2; wrL = r2; wcL = cl2; wcR = cr2;
    }
    if (dp2 > dp || (dp2 == dp && dr2 < drL)) {
      dp = dp2;
      ds = ds2;
      drL = dr2;
    }
  }
  ws_ = __builtin_amdgcn_readfirstlane(ws_);
  wrL = __builtin_amdgcn_readfirstlane(wrL);
  wcL = __builtin_amdgcn_readfirstlane(wcL);
  wcR = __builtin_amdgcn_readfirstlane(wcR);
  wp = __shfl(wp, 0, 64);
  ds = __builtin_amdgcn_readfirstlane(ds);
  drL = __builtin_amdgcn_readfirstlane(drL);
  dp = __shfl(dp, 0, 64);

  // a candidate that only ties the initial (NEG, 0.0) state never replaced it: the reference's
  // best is then still its initial (bestrL = -1) and bestscore = NEG < 0 rejects below
  int bestscore = ws_, bestrL = wrL, bestrR = rlen - wrL, bestcL = wcL, bestcR = wcR;
  bool use_dinucl;
  if (wp > 2 * 0.85) use_dinucl = false;  // bestprob_with_score > 2*PROB_CEILING
  else if (dp == 0.0) use_dinucl = false;
  else if (ds < 0 || ds < bestscore - 9) use_dinucl = false;
  else use_dinucl = true;
  if (use_dinucl) {
    bestscore = ds;
    bestrL = bestcL = drL;
    bestrR = bestcR = rlen - drL;
  }
  int finalscore = bestscore;
  if (bestscore >= 0 && (flags & kGHalf)) finalscore = bestscore - isc[ldi[bestcL] & rdi[bestcR]] / 2;
  if (finalscore < 0) {
    if (lane == 0) {
      res.traceback_score = -100;
      results[pid] = res;
    }
    return;
  }

  // ---- 4. tracebacks (upper when bestc >= bestr, else lower) around the intron gap holder ----
  res.left_prob = pL[bestcL];
  res.right_prob = pR[bestcR];
  const int new_left = P.goffsetL + (bestcL - 1);
  const int new_right = P.rev_goffsetR - (bestcR - 1);
  Tally t = {0, 0, 0, 0, 0, 0, 0, false};
  const bool upR = bestcR >= bestrR, upL = bestcL >= bestrL;
  traceback_walk(lane, upR ? VRu : VRl, bestrR, bestcR, GR, qR, qucR, gchR, cons, watson, P.chroffset, P.chrhigh,
                 blocks, nwords, out, t, upR ? 1 : 2);
  const int nR = t.count;
  reverse_records(lane, out, nR);
  const int queryjump = (rev_roffset - bestrR) - (P.roffset + bestrL) + 1;
  if (lane == 0) put_pair(out, nR, -1, -1, new_right - new_left - 1, ' ', ' ', ' ', ' ');
  t.count += 1;
  traceback_walk(lane, upL ? VLu : VLl, bestrL, bestcL, GL, qL, qucL, gchL, cons, watson, P.chroffset, P.chrhigh,
                 blocks, nwords, out, t, upL ? 1 : 2);
  int npairs = t.count;
  int score = t.score + t.nmatches * kMatch + t.nmismatches * kMismatch;
  if (npairs == 1) {
    npairs = 0;  // only the gap holder: NULL (:3629-3632)
  } else {
    __threadfence_block();
    if (wave_maxnegscore(lane, out, npairs) < -10) {
      npairs = 0;
      score = -100;
    }
  }
  if (lane == 0) {
    res.npairs = npairs;
    res.traceback_score = score;
    res.nmatches = t.nmatches;
    res.nmismatches = t.nmismatches;
    res.nopens = t.nopens;
    res.nindels = t.nindels;
    res.dynprogindex = dpi_next;
    res.new_leftgenomepos = new_left;
    res.new_rightgenomepos = new_right;
    res.exonhead = rev_roffset - (bestrR - 1);
    res.gap_index = npairs ? nR : -1;
    res.gap_queryjump = queryjump;
    results[pid] = res;
  }
}

// ---- host-side sizes and launches ----
size_t lds_bytes_uxe(int rlength, int glength, int B) { return carve_ux(rlength, glength, B, 0).total; }
size_t scratch_bytes_uxe(int rlength, int glength, int lband, int uband, int B) {
  const int tmax = max(ux_steps(rlength, uband, B), ux_steps(glength, lband, B));
  return 144u * (size_t)tmax;
}
size_t lds_bytes_uxg(int rlength, int glengthL, int glengthR, int B) {
  return B == 32 ? carve_uxg<32>(rlength, glengthL, glengthR).total : carve_uxg<16>(rlength, glengthL, glengthR).total;
}
size_t scratch_bytes_uxg(int rlength, int glengthL, int glengthR, int extraband, int B) {
  const int tmax = B == 32 ? uxg_tmax<32>(rlength, glengthL, glengthR, extraband)
                           : uxg_tmax<16>(rlength, glengthL, glengthR, extraband);
  return 144u * (size_t)tmax + 8u * (size_t)(rlength + 1);
}

hipError_t launch_uxe(int B, int nproblems, size_t lds, hipStream_t stream, const DevProblem* probs, const int* order,
                      unsigned char* gscratch, const uint32_t* blocks, uint64_t nwords, const char* qseq,
                      const char* qseq_uc, const int8_t* sctab, const uint8_t* constab, gmapdp_result* results,
                      gmapdp_pair* pairs) {
  if (B != 16 && B != 32) return hipErrorInvalidValue;
  void* fn = (B == 16) ? reinterpret_cast<void*>(&uxe_kernel<16>) : reinterpret_cast<void*>(&uxe_kernel<32>);
  if (lds > 64 * 1024) {
    hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
  }
  void* args[] = {(void*)&probs, (void*)&order, (void*)&gscratch, (void*)&blocks, (void*)&nwords, (void*)&qseq,
                  (void*)&qseq_uc, (void*)&sctab, (void*)&constab, (void*)&results, (void*)&pairs};
  return hipLaunchKernel(fn, dim3(nproblems), dim3(64), args, lds, stream);
}

hipError_t launch_uxg(int B, int nproblems, size_t lds, hipStream_t stream, const DevGenomeProblem* probs,
                      const int* order, unsigned char* gscratch, const uint32_t* blocks, uint64_t nwords,
                      const char* qseq, const char* qseq_uc, const double* sprob, const int8_t* sctab,
                      const uint8_t* constab, const int8_t* isctab, gmapdp_genome_result* results,
                      gmapdp_pair* pairs, const uint8_t* known) {
  if (B != 16 && B != 32) return hipErrorInvalidValue;
  void* fn = (B == 16) ? reinterpret_cast<void*>(&uxg_kernel<16>) : reinterpret_cast<void*>(&uxg_kernel<32>);
  if (lds > 64 * 1024) {
    hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
  }
  void* args[] = {(void*)&probs, (void*)&order, (void*)&gscratch, (void*)&blocks, (void*)&nwords, (void*)&qseq,
                  (void*)&qseq_uc, (void*)&sprob, (void*)&sctab, (void*)&constab, (void*)&isctab, (void*)&results,
                  (void*)&pairs, (void*)&known};
  return hipLaunchKernel(fn, dim3(nproblems), dim3(64), args, lds, stream);
}

}  // namespace gmapdp
