// gg2_kernel.hip -- Dynprog_genome_gap (dynprog_genome.c:3288-3901), nosimd semantics, for bands up
// to 64 cells wide (every genome gap stage3.c makes at extraband_paired 14 and glength = rlength + 8;
// wider bands take gg_kernel<R>, dp_kernel.hip).  The algorithm and the wave split are gg_kernel's:
//   1. genome_gap_simple (:3006) on wave 0 when !finalp && defect_rate < DEFECT_MEDQ;
//   2. the two fills concurrently, wave 0 the R fill (reversed query vs rev_gsequenceR, lbandL,
//      !jump_late_p, :3810), wave 1 the L fill (:3801), each carrying its side's
//      bridge_intron_gap_site_level candidates along the band rows (:2736-2844);
//   3. the bridge on wave 0 (one lane per row rL, then a wave reduction);
//   4. traceback R, List_reverse, the intron gap holder, traceback L, Pair_maxnegscore.
//
// What changes is where the fill's operands live.  Lane k holds band offset k (row r = c - uband + k)
// of column c; every operand a column needs is fetched one column ahead, so no LDS read sits on the
// column's dependency chain:
//   * per fill row r, one 8-byte record {4-bit score word of the query row, the row's five possible
//     intron scores isc[rowdi & code] packed 6 bits each}; the column's dinucleotide code (one of four,
//     or none) selects the field, so the bridge's intron-score lookup is a bit-field extract;
//   * per column one byte {genome class, dinucleotide selector} and the column's splice probability,
//     read at a wave-uniform address;
//   * the row's own probability (the other side's, indexed by rlength - r).
// Direction bits are accumulated per lane, 4 bits per column (nogap=HORIZ, nogap=VERT, Egap=HORIZ,
// Fgap=VERT), and one 32-bit word per lane is written every 8 columns: in LDS for the common sizes,
// in the global scratch above a size threshold.  Bridge candidates per row are kept as (score, column)
// in LDS; their probability probL + probR is recomputed in the bridge from the same two doubles in the
// same order, so it is bit-identical to the one the fill compared.
#include "dp_device.h"

namespace gmapdp {

struct Gg2Row {
  int32_t sw;    // 4-bit score word of the fill's query row (one field per genome class)
  uint32_t isc;  // isc[rowdi[other] & code_j] in bits 6j..6j+5, j = 0..3 the side's codes, j = 4 code 0
};

__host__ __device__ inline size_t gg2_dirs_words(int glength, int W) { return (size_t)((glength + 7) / 8) * (size_t)W; }

struct CarveGG2 {
  size_t rowL, rowR, pL, pR, codeL, codeR, gclL, gclR, ldi, rdi, isc, partB, partC, diagL, diagR, flag, dirsL, dirsR,
      total;
};

__host__ __device__ inline CarveGG2 carve_gg2(int rlength, int gL, int gR, int WL, int WR, bool dirs_lds) {
  CarveGG2 cv;
  size_t off = 0;
  cv.rowL = off;  off = align16(off + 8u * (size_t)(rlength + 2));
  cv.rowR = off;  off = align16(off + 8u * (size_t)(rlength + 2));
  cv.pL = off;    off = align16(off + 8u * (size_t)(gL + 1));
  cv.pR = off;    off = align16(off + 8u * (size_t)(gR + 1));
  cv.partB = off; off = align16(off + 8u * (size_t)(rlength + 1));
  cv.partC = off; off = align16(off + 8u * (size_t)(rlength + 1));
  cv.diagL = off; off = align16(off + 4u * (size_t)(rlength + 1));
  cv.diagR = off; off = align16(off + 4u * (size_t)(rlength + 1));
  cv.codeL = off; off = align16(off + (size_t)(gL + 2));
  cv.codeR = off; off = align16(off + (size_t)(gR + 2));
  cv.gclL = off;  off = align16(off + (size_t)(gL + 3));
  cv.gclR = off;  off = align16(off + (size_t)(gR + 3));
  cv.ldi = off;   off = align16(off + (size_t)(gL + 2));
  cv.rdi = off;   off = align16(off + (size_t)(gR + 2));
  cv.isc = off;   off = align16(off + 64);
  cv.flag = off;  off = align16(off + 4);
  cv.dirsL = cv.dirsR = 0;
  if (dirs_lds) {
    cv.dirsL = off; off = align16(off + 4u * gg2_dirs_words(gL, WL));
    cv.dirsR = off; off = align16(off + 4u * gg2_dirs_words(gR, WR));
  }
  cv.total = off;
  return cv;
}

__host__ __device__ inline size_t scratch_gg2_bytes(int gL, int gR, int WL, int WR, bool dirs_lds) {
  return dirs_lds ? 0 : align16(4u * gg2_dirs_words(gL, WL)) + align16(4u * gg2_dirs_words(gR, WR));
}

// dinucleotide selector of a column (the field of Gg2Row.isc): left codes of the L fill's columns,
// right codes of the R fill's
__device__ __forceinline__ uint32_t sel_left(uint8_t d) {
  return d == 0x21 ? 0u : d == 0x10 ? 1u : d == 0x08 ? 2u : d == 0x06 ? 3u : 4u;
}
__device__ __forceinline__ uint32_t sel_right(uint8_t d) {
  return d == 0x30 ? 0u : d == 0x0C ? 1u : d == 0x02 ? 2u : d == 0x01 ? 3u : 4u;
}
__device__ __forceinline__ uint32_t isc_pack(const int8_t* isc, uint8_t rowdi, bool left_cols) {
  const uint8_t lc[4] = {0x21, 0x10, 0x08, 0x06}, rc[4] = {0x30, 0x0C, 0x02, 0x01};
  uint32_t w = 0;
#pragma unroll
  for (int j = 0; j < 4; j++) w |= ((uint32_t)(uint8_t)isc[rowdi & (left_cols ? lc[j] : rc[j])] & 63u) << (6 * j);
  return w | (((uint32_t)(uint8_t)isc[0] & 63u) << 24);
}

// Direction bits of the packed layout: word ((c-1)/8)*W + k holds band offset k of columns c..c+7,
// 4 bits per column (bit t of nibble (c-1)%8: t = 0 nogap=HORIZ, 1 nogap=VERT, 2 Egap=HORIZ, 3 Fgap=VERT);
// offsets outside the band read DIAG, as the reference's cleared arrays (dynprog.c:498).
struct Gg2Dirs {
  const uint32_t* d;
  int W, uband;
  __device__ uint32_t operator()(int c, int t, int r) const {
    const int k = r - c + uband;
    if (k < 0 || k >= W) return 0u;
    return (d[(size_t)((c - 1) >> 3) * W + k] >> ((((c - 1) & 7) << 2) + t)) & 1u;
  }
};

// One fill of Dynprog_genome_gap (Dynprog_standard, dynprog.c:1268-1786, upperp = lowerp = true,
// saturation NEG_INFINITY_INT) with the bridge candidates carried along the band rows.  Restates
// fill_band<1, true> (dp_device.h) -- recurrence, boundary row/column, last_nogap entering rlo, the
// unclamped band-top diagonal, `a > b - late` ties, the F max-plus scan -- with the operand layout
// described at the top of this file.  colp: this side's probabilities by column; rowp: the other
// side's, indexed by rlength - r.
template <bool DIRS_LDS>
__device__ __forceinline__ void fill_gg2(int lane, int rlen, int glen, int lband, int uband, int open, int ext,
                                         int late, const Gg2Row* rows, const uint8_t* code, const double* colp,
                                         const double* rowp, uint32_t* dirs, int2* part, int* diag, int rdist) {
  const int W = lband + uband + 1;
  const int k = lane;
  int Hs = kNegInf32, E = kNegInf32;
  {  // column 0 (dynprog.c:1331-1369)
    const int r = k - uband;
    if (k < W && r >= 0 && r <= rlen) Hs = (r == 0) ? 0 : (r <= lband ? open + r * ext : kNegInf32);
  }
  const int kext = k * ext;
  int cs = 0, cc = -1;
  double cp = 0.0;
  int rtop_ext = -uband * ext;
  int oce = open;
  uint32_t acc = 0;
  // operands of column 1, fetched ahead
  int rr = min(max(1 - uband + k, 0), rlen + 1);
  Gg2Row nrow = rows[rr];
  double nrp = rowp[min(max(rlen - (1 - uband + k), 0), rlen)];
  int ncode = code[1];
  double ncp = colp[1];
  for (int c = 1; c <= glen; c++) {
    const Gg2Row row = nrow;
    const double rp = nrp;
    const int cd = __builtin_amdgcn_readfirstlane(ncode);
    const double cpc = ncp;
    if (c < glen) {  // the next column's operands, off this column's chain
      rr = min(max(c + 1 - uband + k, 0), rlen + 1);
      nrow = rows[rr];
      nrp = rowp[min(max(rlen - (c + 1 - uband + k), 0), rlen)];
      ncode = code[c + 1];
      ncp = colp[c + 1];
    }
    const int gi4 = (cd & 7) << 2;
    const int sel6 = (cd >> 3) * 6;
    const int rtop = c - uband;
    const int rlo = rtop < 1 ? 1 : rtop;
    const int rhigh = (c + lband) < rlen ? (c + lband) : rlen;
    rtop_ext += ext;
    oce += ext;
    const int L0 = (c == 1) ? (kNegInf32 - open + 1) : (c <= uband ? oce : kNegInf32);  // last_nogap into rlo
    const int row0 = (c <= uband) ? oce : kNegInf32;                                  // row 0 of this column
    const int Ein = dpp_wave_shl1(E, kNegInf32);
    const int Hin = dpp_wave_shl1(Hs, kNegInf32);
    const int r = rtop + k;
    const bool valid = (k < W) & (r >= rlo) & (r <= rhigh);
    const int s = __builtin_amdgcn_sbfe(row.sw, gi4, 4);
    // Egap (dynprog.c:1518-1524), nogap
    const int es = Hin + open;
    const bool eb = Ein > es - late;
    const int En = max(Ein, es) + ext;
    const int dg = Hs + s;
    const bool hb = En > dg - late;
    const int Hp = max(En, dg);
    // F chain: F(r) = r*ext + max(init, max_{rlo<=j<r} (H'(j) + open - j*ext))
    const int A = valid ? Hp + open - rtop_ext - kext : kSent;
    const int X = dpp_wave_shr1(wave_scan_max(A), kSent);
    const int init = max(kNegInf32, L0 + open) - ((rtop > 1) ? rtop_ext - ext : 0);
    const int F = rtop_ext + kext + max(init, X);
    const bool vb = F > Hp - late;
    const int Hun = max(F, Hp);
    // Fgap direction from F(r-1), H(r-1) of this column (dynprog.c:1486-1492)
    const int Fup = dpp_wave_shr1(F, kNegInf32);
    const int Hup = dpp_wave_shr1(Hun, kNegInf32);
    const bool top = r == rlo;
    const int fprev = top ? kNegInf32 : Fup;
    const int hprev = top ? L0 : Hup;
    const bool fb = fprev > hprev + open - late;
    const uint32_t nib = valid ? ((vb ? 2u : (hb ? 1u : 0u)) | (eb ? 4u : 0u) | (fb ? 8u : 0u)) : 0u;
    acc |= nib << (((c - 1) & 7) << 2);
    const int Hc = max(Hun, kNegInf32);
    Hs = valid ? ((k == 0) ? Hun : Hc) : ((r == 0) ? row0 : kNegInf32);
    E = valid ? En : kNegInf32;
    // bridge candidates: arrive from band offset k+1 of the previous column
    const int ics = dpp_wave_shl1(cs, 0);
    const int icc = dpp_wave_shl1(cc, -1);
    double icp;
    {
      const int2 v = *reinterpret_cast<const int2*>(&cp);
      int2 w;
      w.x = dpp_wave_shl1(v.x, 0);
      w.y = dpp_wave_shl1(v.y, 0);
      icp = *reinterpret_cast<const double*>(&w);
    }
    const int other = rlen - r;
    const bool inrow = (r >= 1) & (r <= rlen - 1) & (k < W);
    const bool cand = inrow & (k >= 1) & valid & (c <= glen - 2) & (c < rdist - other);
    const int s2 = (int)__builtin_amdgcn_ubfe(row.isc, sel6, 6) + Hc;
    const double p = rp + cpc;
    const bool take = cand & ((icc < 0) | (s2 > ics) | ((s2 == ics) & (p > icp)));
    cs = take ? s2 : ics;
    cc = take ? c : icc;
    cp = take ? p : icp;
    if (inrow && k == uband) diag[r] = Hc;                 // matrix[r][r]
    if (inrow && k == 0) part[r] = make_int2(cs, cc);      // the row leaves the band: its candidate is final
    if (((c - 1) & 7) == 7 || c == glen) {
      if (k < W) dirs[(size_t)((c - 1) >> 3) * W + k] = acc;
      acc = 0;
    }
  }
  {  // rows still inside the band after the last column
    const int r = glen - uband + k;
    if (k < W && r >= 1 && r <= rlen - 1) part[r] = make_int2(cs, cc);
  }
}

template <bool DIRS_LDS>
__global__ __launch_bounds__(128) void gg2_kernel(
    const DevGenomeProblem* __restrict__ probs, const int* __restrict__ order,
    const uint32_t* __restrict__ blocks, uint64_t nwords,
    const char* __restrict__ qseq, const char* __restrict__ qseq_uc, const double* __restrict__ sprob,
    const int8_t* __restrict__ sctab, const uint8_t* __restrict__ constab, const int8_t* __restrict__ isctab,
    gmapdp_genome_result* __restrict__ results, gmapdp_pair* __restrict__ pairs,
    unsigned char* __restrict__ gscratch) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int pid = order[blockIdx.x];
  const DevGenomeProblem P = probs[pid];
  const int rlen = P.rlength, gL = P.glengthL, gR = P.glengthR;
  const int flags = P.flags;
  const bool watson = flags & kFWatson;
  const int late = (flags & kFLate) ? 1 : 0;
  const int lband = P.lbandL, ubandL = P.ubandL, ubandR = P.ubandR;
  const int WL = lband + ubandL + 1, WR = lband + ubandR + 1;
  const CarveGG2 cv = carve_gg2(rlen, gL, gR, WL, WR, DIRS_LDS);
  Gg2Row* rowL = reinterpret_cast<Gg2Row*>(smem + cv.rowL);
  Gg2Row* rowR = reinterpret_cast<Gg2Row*>(smem + cv.rowR);
  double* pL = reinterpret_cast<double*>(smem + cv.pL);
  double* pR = reinterpret_cast<double*>(smem + cv.pR);
  int2* partB = reinterpret_cast<int2*>(smem + cv.partB);  // indexed by rR
  int2* partC = reinterpret_cast<int2*>(smem + cv.partC);  // indexed by rL
  int* diagL = reinterpret_cast<int*>(smem + cv.diagL);
  int* diagR = reinterpret_cast<int*>(smem + cv.diagR);
  uint8_t* codeL = reinterpret_cast<uint8_t*>(smem + cv.codeL);
  uint8_t* codeR = reinterpret_cast<uint8_t*>(smem + cv.codeR);
  uint8_t* gclL = reinterpret_cast<uint8_t*>(smem + cv.gclL);
  uint8_t* gclR = reinterpret_cast<uint8_t*>(smem + cv.gclR);
  uint8_t* ldi = reinterpret_cast<uint8_t*>(smem + cv.ldi);
  uint8_t* rdi = reinterpret_cast<uint8_t*>(smem + cv.rdi);
  int8_t* isc = reinterpret_cast<int8_t*>(smem + cv.isc);
  int* done = reinterpret_cast<int*>(smem + cv.flag);
  uint32_t* dirsL;
  uint32_t* dirsR;
  if constexpr (DIRS_LDS) {
    dirsL = reinterpret_cast<uint32_t*>(smem + cv.dirsL);
    dirsR = reinterpret_cast<uint32_t*>(smem + cv.dirsR);
  } else {
    dirsL = reinterpret_cast<uint32_t*>(gscratch + P.dirs_offset);
    dirsR = dirsL + align16(4u * gg2_dirs_words(gL, WL)) / 4u;
  }
  // query rows in both DP orders straight from HBM: qL[r] = rsequence[r-1], qR[r] = rsequence[rlength-r]
  const QView qL{qseq + P.qbase, 1}, qucL{qseq_uc + P.qbase, 1};
  const QView qR{qseq + P.qbase + rlen - 1, -1}, qucR{qseq_uc + P.qbase + rlen - 1, -1};
  const GClassView gchL{gclL}, gchR{gclR};
  const int8_t* sct = sctab + (size_t)P.mismatchtype * 128 * kNClass;
  const uint8_t* cons = constab + (size_t)P.genestrand * 128 * kNClass;
  gmapdp_pair* out = pairs + P.pair_offset;
  const int rev_roffset = P.roffset + rlen - 1;
  const Geo GL{P.roffset, P.goffsetL, 1};
  const Geo GR{rev_roffset, P.rev_goffsetR, -1};
  const bool halfp = flags & kGHalf;

  // ---- stage 1: score words in both DP orders, both genome segments as classes, probabilities ----
  for (int i = tid; i < rlen; i += 128) {
    const char c1 = qseq[P.qbase + i];
    const uint64_t row = *reinterpret_cast<const uint64_t*>(sct + (uint8_t)(c1 & 127) * kNClass);
    uint32_t w = 0;
#pragma unroll
    for (int g = 0; g < 6; g++) w |= (uint32_t)((row >> (8 * g)) & 0xfu) << (4 * g);
    rowL[i + 1].sw = (int32_t)w;
    rowR[rlen - i].sw = (int32_t)w;
  }
  if (tid < 2) {
    const int r = tid ? rlen + 1 : 0;
    rowL[r].sw = rowR[r].sw = 0;
    rowL[r].isc = rowR[r].isc = 0;
  }
  for (int i = tid; i < gL; i += 128) {
    const char c2 = segment_nt(blocks, nwords, (uint32_t)i, (uint32_t)gL, P.segposL, P.segboundL,
                               flags & kGSegLLeft, flags & kGSegLRc);
    gclL[i + 1] = gclass(c2);
    pL[i] = sprob[P.prob_offset + i];
  }
  for (int i = tid; i < gR; i += 128) {
    const char c2 = segment_nt(blocks, nwords, (uint32_t)i, (uint32_t)gR, P.segposR, P.segboundR,
                               flags & kGSegRLeft, flags & kGSegRRc);
    gclR[gR - i] = gclass(c2);  // rev_gsequenceR[1-c] = segment[glengthR-c]
    pR[i] = sprob[P.prob_offset + gL + i];
  }
  if (tid < 64) isc[tid] = isctab[(size_t)P.iclass * 128 + ((flags & kGFinal) ? 64 : 0) + tid];
  if (tid == 0) {
    *done = 0;
    pL[gL] = 0.0;
    pR[gR] = 0.0;
    gclL[0] = gclR[0] = kN;
  }
  __syncthreads();
  // leftdi[cL] from gsequenceL[cL], [cL+1]; rightdi[cR] from rev_gsequenceR[-cR-1], [-cR] (:2518-2566)
  for (int c = tid; c <= gL; c += 128) ldi[c] = (c < gL - 1) ? left_dinucl(gchL[c + 1], gchL[c + 2]) : 0;
  for (int c = tid; c <= gR; c += 128) rdi[c] = (c < gR - 1) ? right_dinucl(gchR[c + 2], gchR[c + 1]) : 0;
  __syncthreads();
  // ---- stage 2: per fill row the intron scores by column code, per column {class, selector} ----
  for (int r = tid + 1; r <= rlen; r += 128) {
    const int other = rlen - r;
    rowL[r].isc = isc_pack(isc, rdi[other], true);   // L fill: row rL, other = rR, columns carry leftdi
    rowR[r].isc = isc_pack(isc, ldi[other], false);  // R fill: row rR, other = rL, columns carry rightdi
  }
  for (int c = tid; c <= gL; c += 128) codeL[c] = (uint8_t)(gclL[c] | (sel_left(ldi[c]) << 3));
  for (int c = tid; c <= gR; c += 128) codeR[c] = (uint8_t)(gclR[c] | (sel_right(rdi[c]) << 3));
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

  // ---- 1. genome_gap_simple (dynprog_genome.c:3006-3280), wave 0 ----
  if (flags & kGSimple) {
    if (wave == 0) {
      const bool ok = gg_simple_wave(lane, P, pid, sctab, isctab, cons, qL, qucL, qR, qucR, gclL, gclR, gchL, gchR,
                                     ldi, rdi, pL, pR, diagL, diagR, out, res, results);
      if (lane == 0) *done = ok ? 1 : 0;
    }
    __syncthreads();
    if (*done) return;
  }

  // ---- 2. fills, concurrently: wave 0 R (feeds the B candidates), wave 1 L (the C candidates) ----
  const int rdist = P.rev_goffsetR - P.goffsetL;  // "cR < rightoffset - leftoffset - cL"
  if (wave == 0)
    fill_gg2<DIRS_LDS>(lane, rlen, gR, lband, ubandR, P.open, P.extend, 1 - late, rowR, codeR, pR, pL, dirsR, partB,
                       diagR, rdist);
  else
    fill_gg2<DIRS_LDS>(lane, rlen, gL, lband, ubandL, P.open, P.extend, late, rowL, codeL, pL, pR, dirsL, partC,
                       diagL, rdist);
  __threadfence_block();
  __syncthreads();
  if (wave != 0) return;

  // ---- 3. bridge: per-lane scan of rows rL = lane+1, lane+65, ... (A, B, C per row) ----
  int ws = kNegInf32, wrL = -1, wcL = 0, wcR = 0;  // (NEG_INFINITY_32, 0.0) is the reference's initial state
  double wp = 0.0;
  int ds = 0, drL = 0x7fffffff;                    // best dinucleotide (A) candidate: max prob, earliest
  double dp = 0.0;
  for (int rL = lane + 1; rL <= rlen - 1; rL += 64) {
    const int rR = rlen - rL;
    const int dL = diagL[rL], dR = diagR[rR];
    // A: cL = rL, cR = rR
    const int sI = isc[ldi[rL] & rdi[rR]];
    int rs = dL + sI + dR, rcL = rL, rcR = rR;
    double rp = pL[rL] + pR[rR];
    if (sI > 0 && rp > dp) {
      dp = rp;
      ds = rs;
      drL = rL;
    }
    // B: cL = rL, best cR of R row rR (+ matrixL[rL][rL]); its probability probL[rL] + probR[cR]
    const int2 b = partB[rR];
    if (b.y >= 0) {
      const double bp = pL[rL] + pR[b.y];
      if (lex_better(dL + b.x, bp, rs, rp)) {
        rs = dL + b.x;
        rp = bp;
        rcL = rL;
        rcR = b.y;
      }
    }
    // C: cR = rR, best cL of L row rL (+ matrixR[rR][rR]); its probability probR[rR] + probL[cL]
    const int2 cpart = partC[rL];
    if (cpart.y >= 0) {
      const double cpp = pR[rR] + pL[cpart.y];
      if (lex_better(dR + cpart.x, cpp, rs, rp)) {
        rs = dR + cpart.x;
        rp = cpp;
        rcL = cpart.y;
        rcR = rR;
      }
    }
    if (lex_better(rs, rp, ws, wp)) {  // later rows replace only when strictly better
      ws = rs;
      wp = rp;
      wrL = rL;
      wcL = rcL;
      wcR = rcR;
    }
  }
  // merge rows across lanes: (score desc, prob desc, rL asc)
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {
    const int s2 = __shfl_xor(ws, off, 64);
    const double p2 = __shfl_xor(wp, off, 64);
    const int r2 = __shfl_xor(wrL, off, 64);
    const int cl2 = __shfl_xor(wcL, off, 64);
    const int cr2 = __shfl_xor(wcR, off, 64);
    const int ds2 = __shfl_xor(ds, off, 64);
    const double dp2 = __shfl_xor(dp, off, 64);
    const int dr2 = __shfl_xor(drL, off, 64);
    if (lex_better(s2, p2, ws, wp) || (s2 == ws && p2 == wp && r2 < wrL)) {
      ws = s2;
      wp = p2;
      wrL = r2;
      wcL = cl2;
      wcR = cr2;
    }
    if (dp2 > dp || (dp2 == dp && dr2 < drL)) {
      dp = dp2;
      ds = ds2;
      drL = dr2;
    }
  }
  ws = __builtin_amdgcn_readfirstlane(ws);
  wrL = __builtin_amdgcn_readfirstlane(wrL);
  wcL = __builtin_amdgcn_readfirstlane(wcL);
  wcR = __builtin_amdgcn_readfirstlane(wcR);
  wp = __shfl(wp, 0, 64);
  ds = __builtin_amdgcn_readfirstlane(ds);
  drL = __builtin_amdgcn_readfirstlane(drL);
  dp = __shfl(dp, 0, 64);

  int bestscore = ws, bestrL = wrL, bestrR = rlen - wrL, bestcL = wcL, bestcR = wcR;
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
  if (bestscore >= 0 && halfp) finalscore = bestscore - isc[ldi[bestcL] & rdi[bestcR]] / 2;
  if (finalscore < 0) {
    if (lane == 0) {
      res.traceback_score = -100;
      results[pid] = res;
    }
    return;
  }

  // ---- 4. tracebacks around the intron gap holder ----
  res.left_prob = pL[bestcL];
  res.right_prob = pR[bestcR];
  const int new_left = P.goffsetL + (bestcL - 1);
  const int new_right = P.rev_goffsetR - (bestcR - 1);
  Tally t = {0, 0, 0, 0, 0, 0, 0, false};
  traceback_walk(lane, Gg2Dirs{dirsR, WR, ubandR}, bestrR, bestcR, GR, qR, qucR, gchR, cons, watson, P.chroffset,
                 P.chrhigh, blocks, nwords, out, t);
  const int nR = t.count;
  reverse_records(lane, out, nR);
  const int queryjump = (rev_roffset - bestrR) - (P.roffset + bestrL) + 1;
  if (lane == 0) put_pair(out, nR, -1, -1, new_right - new_left - 1, ' ', ' ', ' ', ' ');
  t.count += 1;
  traceback_walk(lane, Gg2Dirs{dirsL, WL, ubandL}, bestrL, bestcL, GL, qL, qucL, gchL, cons, watson, P.chroffset,
                 P.chrhigh, blocks, nwords, out, t);
  int npairs = t.count;
  int score = t.score + t.nmatches * kMatch + t.nmismatches * kMismatch;
  if (npairs == 1) {
    npairs = 0;  // only the gap holder: NULL (:3877-3880)
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

// ---- host-side entry points ----
size_t lds_bytes_gg2(int rlength, int glengthL, int glengthR, int WL, int WR, bool dirs_lds) {
  return carve_gg2(rlength, glengthL, glengthR, WL, WR, dirs_lds).total;
}
size_t scratch_bytes_gg2(int glengthL, int glengthR, int WL, int WR, bool dirs_lds) {
  return scratch_gg2_bytes(glengthL, glengthR, WL, WR, dirs_lds);
}

hipError_t launch_gg2(bool dirs_lds, int nblocks, size_t lds, hipStream_t stream, const DevGenomeProblem* probs,
                      const int* order, const uint32_t* blocks, uint64_t nwords, const char* qseq,
                      const char* qseq_uc, const double* sprob, const int8_t* sctab, const uint8_t* constab,
                      const int8_t* isctab, gmapdp_genome_result* results, gmapdp_pair* pairs,
                      unsigned char* gscratch) {
  void* fn = dirs_lds ? reinterpret_cast<void*>(&gg2_kernel<true>) : reinterpret_cast<void*>(&gg2_kernel<false>);
  if (lds > 64 * 1024) {
    hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
  }
  void* args[] = {(void*)&probs, (void*)&order, (void*)&blocks, (void*)&nwords, (void*)&qseq, (void*)&qseq_uc,
                  (void*)&sprob, (void*)&sctab, (void*)&constab, (void*)&isctab, (void*)&results, (void*)&pairs,
                  (void*)&gscratch};
  return hipLaunchKernel(fn, dim3(nblocks), dim3(128), args, lds, stream);
}

}  // namespace gmapdp
