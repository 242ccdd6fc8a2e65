// ggp_kernel.hip -- Dynprog_genome_gap (dynprog_genome.c:3288-3901, nosimd semantics) packed
// 64/S problems per wave.
//
// gg_kernel (dp_kernel.hip) spends one 64-lane wave per fill on a band of ~37 cells: 40 % of the
// lanes idle and ~470 instructions of per-column overhead (the cross-lane F scan, ballots, the
// bridge-candidate bookkeeping) for 37 cells, which makes it VALU-issue bound.  Here an S-lane
// group holds one problem and each lane R consecutive band offsets (W <= S*R), so one wave
// instruction advances 64/S problems and the cross-lane work per column is a 2-3 step group scan.
// The work is split by resource profile into three launches over one launch class:
//
//   ggp_prep_kernel  (one wave per problem, few registers, latency-bound):
//       stages the problem into its global scratch (4-bit score word per query row in both DP
//       orders, genome classes and dinucleotide codes of both segments) and tries
//       genome_gap_simple (:3006) exactly as gg_kernel; a problem it settles is done, the others
//       are flagged for the full path;
//   ggp_fill_kernel<S, R>  (64/S problems per wave, register-heavy, VALU-bound):
//       the R fill (reversed query vs rev_gsequenceR, lband = lbandL, !jump_late_p, :3810) and
//       the L fill (:3801) of every flagged problem in its group, each carrying its side's
//       bridge candidates along the band rows (BridgeCarry, as gg_kernel), direction nibbles per
//       lane to scratch; then bridge_intron_gap_site_level's row scan (:2469) across the group
//       and the group's reduction, recorded per problem;
//   ggp_tail_kernel  (one wave per problem, latency-bound):
//       the dinucleotide / halfp decision, the two tracebacks around the intron gap holder,
//       Pair_maxnegscore and the result (gg_kernel's tail, reading the group fill's directions).
//
// Bit-exact with gg_kernel, the oracle and the reference (tests/test_gpu_genome_gap.py).
#include "dp_device.h"

namespace gmapdp {

// ---- S-lane group primitives (S = 4 or 8; the group is lanes [S*g, S*g+S)) ----
// lane <- lane+1 of its group; the group's last lane <- fill
template <int S>
__device__ __forceinline__ int grp_shl1(int x, int fill, int lk) {
  static_assert(S == 4 || S == 8 || S == 16, "group width");
  if constexpr (S == 16) return __builtin_amdgcn_update_dpp(fill, x, 0x101, 0xf, 0xf, false);  // row_shl:1
  int v;
  if constexpr (S == 4) v = __builtin_amdgcn_update_dpp(0, x, 0xF9, 0xf, 0xf, false);  // quad_perm:[1,2,3,3]
  else v = __builtin_amdgcn_update_dpp(0, x, 0x101, 0xf, 0xf, false);                  // row_shl:1
  return (lk == S - 1) ? fill : v;
}
// lane <- lane-1 of its group; the group's first lane <- fill
template <int S>
__device__ __forceinline__ int grp_shr1(int x, int fill, int lk) {
  if constexpr (S == 16) return __builtin_amdgcn_update_dpp(fill, x, 0x111, 0xf, 0xf, false);  // row_shr:1
  int v;
  if constexpr (S == 4) v = __builtin_amdgcn_update_dpp(0, x, 0x90, 0xf, 0xf, false);  // quad_perm:[0,0,1,2]
  else v = __builtin_amdgcn_update_dpp(0, x, 0x111, 0xf, 0xf, false);                  // row_shr:1
  return (lk == 0) ? fill : v;
}
// inclusive max-scan within the group (lane order); kSent is the identity
template <int S>
__device__ __forceinline__ int grp_scan_max(int x, int lk) {
  if constexpr (S == 4) {
    int y = __builtin_amdgcn_update_dpp(0, x, 0x90, 0xf, 0xf, false);  // lane-1
    x = max(x, lk >= 1 ? y : kSent);
    y = __builtin_amdgcn_update_dpp(0, x, 0x40, 0xf, 0xf, false);      // quad_perm:[0,0,0,1]: lane-2
    x = max(x, lk >= 2 ? y : kSent);
  } else if constexpr (S == 16) {  // lanes without a source read the identity
    x = max(x, __builtin_amdgcn_update_dpp(kSent, x, 0x111, 0xf, 0xf, false));  // row_shr:1
    x = max(x, __builtin_amdgcn_update_dpp(kSent, x, 0x112, 0xf, 0xf, false));  // row_shr:2
    x = max(x, __builtin_amdgcn_update_dpp(kSent, x, 0x114, 0xf, 0xf, false));  // row_shr:4
    x = max(x, __builtin_amdgcn_update_dpp(kSent, x, 0x118, 0xf, 0xf, false));  // row_shr:8
  } else {
    int y = __builtin_amdgcn_update_dpp(0, x, 0x111, 0xf, 0xf, false);  // row_shr:1
    x = max(x, lk >= 1 ? y : kSent);
    y = __builtin_amdgcn_update_dpp(0, x, 0x112, 0xf, 0xf, false);      // row_shr:2
    x = max(x, lk >= 2 ? y : kSent);
    y = __builtin_amdgcn_update_dpp(0, x, 0x114, 0xf, 0xf, false);      // row_shr:4
    x = max(x, lk >= 4 ? y : kSent);
  }
  return x;
}
template <int S>
__device__ __forceinline__ double grp_shl1_d(double x, int lk) {
  // a double's two halves through grp_shl1 (fill 0.0)
  const int2 v = *reinterpret_cast<const int2*>(&x);
  int2 w;
  w.x = grp_shl1<S>(v.x, 0, lk);
  w.y = grp_shl1<S>(v.y, 0, lk);
  return *reinterpret_cast<const double*>(&w);
}

// Per-problem global scratch of the packed genome-gap path (DevGenomeProblem.dirs_offset).
struct ScratchGGP {
  size_t scL, scR, gclL, gclR, ldi, rdi, partB, partC, diagL, diagR, sum, total;
};
// Bridge outcome of one problem (written by the fill kernel's group, read by the tail), where its
// direction ballots are, and the result fields genome_gap_simple leaked when it declined (prep).
struct GGPSummary {
  int ws, wrL, wcL, wcR, ds, drL, full, lane0;
  double wp, dp;
  int64_t dirsR, dirsL;  // byte offsets of the fills' ballot words in the scratch
  gmapdp_genome_result res;
};

__host__ __device__ inline ScratchGGP scratch_ggp(int rlength, int glengthL, int glengthR) {
  ScratchGGP sv;
  size_t off = 0;
  sv.sum = off;   off = align16(off + sizeof(GGPSummary));
  sv.scL = off;   off = align16(off + 4u * (size_t)(rlength + 2));
  sv.scR = off;   off = align16(off + 4u * (size_t)(rlength + 2));
  sv.gclL = off;  off = align16(off + (size_t)(glengthL + 2));
  sv.gclR = off;  off = align16(off + (size_t)(glengthR + 2));
  sv.ldi = off;   off = align16(off + (size_t)(glengthL + 2));
  sv.rdi = off;   off = align16(off + (size_t)(glengthR + 2));
  sv.partB = off; off = align16(off + 16u * (size_t)(rlength + 1));
  sv.partC = off; off = align16(off + 16u * (size_t)(rlength + 1));
  sv.diagL = off; off = align16(off + 4u * (size_t)(rlength + 1));
  sv.diagR = off; off = align16(off + 4u * (size_t)(rlength + 1));
  sv.total = off;
  return sv;
}

// Direction bits of a group fill: whole-wave ballots, per column c the words [c][t][i] (t: nogap=HORIZ,
// nogap=VERT, Egap=HORIZ, Fgap=VERT; i: the cell of a lane), bit lane0 + j for the group's lane j, which
// holds band offsets k = j*R + i.
template <int R>
struct BallotDirs {
  const uint64_t* dirs;
  int W, uband, lane0;
  __device__ uint32_t operator()(int c, int t, int r) const {
    const int k = r - c + uband;
    if (k < 0 || k >= W) return 0u;  // outside the band: cleared to DIAG (dynprog.c:498)
    const int j = k / R, i = k - j * R;
    return (uint32_t)(dirs[((size_t)c * 4 + t) * R + i] >> (lane0 + j)) & 1u;
  }
};

// One fill of Dynprog_genome_gap by an S-lane group (Dynprog_standard, dynprog.c:1268-1786, with
// bridge candidates carried along the band rows: gg_kernel's fill_band<R, true> restated for a group;
// see the BridgeCarry comment in dp_device.h).  Lane lk owns band offsets k = lk*R + i; row
// r = c - uband + k.  The per-row values -- the 4-bit score word (bits 0-23) with the other side's
// dinucleotide code (bits 24-31), the other side's probability, the carried candidate -- move one
// band offset up per column with their row, so each column only the row entering at the group's
// last offset is loaded.  Everything that moves is shifted in place in ascending i (cell i takes
// cell i+1's old value, the last cell the next lane's first), which keeps one copy per cell in
// registers.  The band tests of a cell are ranges of i, set once per column.  The four direction
// bits of every cell are the compare masks themselves (ballots), stored per column as 4R words
// for the whole wave (dirs).  cend: the wave's longest fill; a group past its own glen idles.
template <int S, int R>
__device__ __forceinline__ void fill_grp(int lane, int lk, bool act, int rlen, int glen, int cend, int lband,
                                         int uband, int open, int ext, int late, const int32_t* __restrict__ sc,
                                         const uint8_t* __restrict__ gcl, const uint8_t* __restrict__ rowdi,
                                         const uint8_t* __restrict__ coldi, const double* __restrict__ rowp,
                                         const double* __restrict__ colp, const int8_t* isc, int rdist, Part* part,
                                         int* diag, uint64_t* __restrict__ dirs) {
  const int W = lband + uband + 1;
  const int sat = kNegInf32;
  const int k0 = lk * R;
  int Hs[R], E[R], qw[R], cs[R], cc[R];
  double cp[R], rp[R];
  // the per-row values of band offset k at column c (row r = c - uband + k)
  auto rowval = [&](int c, int k, int& w, double& p) {
    const int r = c - uband + k;
    const int rr = min(max(r, 0), rlen + 1);
    const int other = rlen - r;
    const bool inrow = (r >= 1) & (r <= rlen - 1);
    w = (sc[rr] & 0xffffff) | (inrow ? ((int)rowdi[other] << 24) : 0);
    p = inrow ? rowp[other] : 0.0;
  };
#pragma unroll
  for (int i = 0; i < R; i++) {  // column 0 (dynprog.c:1331-1369)
    const int k = k0 + i;
    const int r = k - uband;
    int v = kNegInf32;
    if (k < W && r >= 0 && r <= rlen) v = (r == 0) ? 0 : (r <= lband ? open + r * ext : kNegInf32);
    Hs[i] = v;
    E[i] = kNegInf32;
    cs[i] = 0;
    cc[i] = -1;
    cp[i] = 0.0;
    if (act) rowval(1, k, qw[i], rp[i]);
    else { qw[i] = 0; rp[i] = 0.0; }
  }
  int rtop_ext = -uband * ext;
  int oce = open;
  int gi_next = act ? gcl[1] : 0;
  int di_next = act ? coldi[1] : 0;
  double p_next = act ? colp[1] : 0.0;
  for (int c = 1; c <= cend; c++) {
    // the first lane of an active group stores the column's ballot words (inside the divergent
    // body, where the ballots are wave values); a column no group fills keeps zero words
    const uint64_t mact = ballot(act && c <= glen);
    const int src = (int)__ffsll((long long)mact) - 1;
    if (!mact && lane < 4 * R) dirs[(size_t)c * 4 * R + lane] = 0;
    if (act && c <= glen) {  // the group is uniform: all its lanes take the same branch
      uint64_t mH[R], mV[R], mE[R], mF[R];
      const int gi = gi_next, cdi = di_next;
      const double cpc = p_next;
      if (c < glen) {  // next column's genome class, dinucleotide, probability, off the dependency chain
        gi_next = gcl[c + 1];
        di_next = coldi[c + 1];
        p_next = (c + 1 < glen) ? colp[c + 1] : 0.0;  // colp has glen entries; column glen is never a candidate
      }
      const int rtop = c - uband;
      const int rlo = rtop < 1 ? 1 : rtop;
      const int rhigh = (c + lband) < rlen ? (c + lband) : rlen;
      rtop_ext += ext;
      oce += ext;
      const int L0 = (c == 1) ? (kNegInf32 - open + 1) : (c <= uband ? oce : kNegInf32);
      const int row0 = (c <= uband) ? oce : kNegInf32;
      const int gi4 = gi << 2;
      const int rext0 = rtop_ext + k0 * ext;  // r*ext of cell 0
      // this lane's cells i as ranges: valid [vlo, vhi], the band-top row itop, row 0 at i0,
      // bridge candidates [clo, chi] (1 <= k, r <= rlength-1, c <= glength-2, c < rdist - other)
      const int vlo = (rlo - rtop) - k0;
      const int vhi = min(W - 1, rhigh - rtop) - k0;
      const int itop = vlo;
      const int i0 = -rtop - k0;
      const int clo = max(max(vlo, 1 - k0), c - rdist + rlen - rtop - k0 + 1);
      const int chi = (c <= glen - 2) ? min(vhi, (rlen - 1 - rtop) - k0) : -1;

      // pass 1: E and the pre-F score H' of every cell; E moves in place (cell i reads cell i+1)
      const int Elast = grp_shl1<S>(E[0], kNegInf32, lk);
      const int Hlast = grp_shl1<S>(Hs[0], kNegInf32, lk);
      int Hp[R], pre[R];
#pragma unroll
      for (int i = 0; i < R; i++) {
        const bool valid = (i >= vlo) & (i <= vhi);
        const int Ein = (i < R - 1) ? E[i + 1] : Elast;
        const int Hin = (i < R - 1) ? Hs[i + 1] : Hlast;
        const int s = __builtin_amdgcn_sbfe(qw[i], gi4, 4);
        const int es = Hin + open;
        const bool eb = Ein > es - late;
        const int En = max(Ein, es) + ext;
        const int dg = Hs[i] + s;
        const bool hb = En > dg - late;
        Hp[i] = max(En, dg);
        const int A = valid ? Hp[i] + open - (rext0 + i * ext) : kSent;
        pre[i] = (i == 0) ? A : max(pre[i - 1], A);
        E[i] = valid ? En : kNegInf32;
        const uint64_t mv = ballot(valid);
        mE[i] = ballot(eb) & mv;
        mH[i] = ballot(hb) & mv;  // & ~mV below
      }
      // F chain: F(r) = r*ext + max(init, max_{rlo<=j<r} (H'(j) + open - j*ext)), exclusive across lanes
      const int X = grp_shr1<S>(grp_scan_max<S>(pre[R - 1], lk), kSent, lk);
      const int init = max(kNegInf32, L0 + open) - ((rtop > 1) ? rtop_ext - ext : 0);
      // the last cell of the previous lane: F and H of row r-1 for the Fgap direction
      int Flane, Hlane;
      {
        const int ex = (R == 1) ? X : max(X, pre[R - 2]);
        Flane = rext0 + (R - 1) * ext + max(init, ex);
        Hlane = max(Flane, Hp[R - 1]);
      }
      const int Fup = grp_shr1<S>(Flane, kNegInf32, lk);
      const int Hup = grp_shr1<S>(Hlane, kNegInf32, lk);
      // values moving in from the next lane (its cell 0) into this lane's last cell
      // (every DPP runs with the whole group active: a source lane masked off would read as 0)
      int qw_new = grp_shl1<S>(qw[0], 0, lk);
      double rp_new = grp_shl1_d<S>(rp[0], lk);
      const int cs_in = grp_shl1<S>(cs[0], 0, lk);
      const int cc_in = grp_shl1<S>(cc[0], -1, lk);
      const double cp_in = grp_shl1_d<S>(cp[0], lk);
      if (lk == S - 1) rowval(c + 1, S * R - 1, qw_new, rp_new);  // the row entering the group
      // pass 2: F, H, directions, bridge candidates; the moving values shift in place
      int dval = 0;
      int Fprev = Fup, Hprev = Hup;
#pragma unroll
      for (int i = 0; i < R; i++) {
        const bool v = (i >= vlo) & (i <= vhi);
        const int ex = (i == 0) ? X : max(X, pre[i - 1]);
        const int F = rext0 + i * ext + max(init, ex);
        const bool vb = F > Hp[i] - late;
        const int Hun = max(F, Hp[i]);
        const bool top = i == itop;
        const int fprev = top ? kNegInf32 : Fprev;
        const int hprev = top ? L0 : Hprev;
        const bool fb = fprev > hprev + open - late;
        Fprev = F;
        Hprev = Hun;
        const uint64_t mv = ballot(v);
        mV[i] = ballot(vb) & mv;
        mH[i] &= ~mV[i];
        mF[i] = ballot(fb) & mv;
        const int Hc = max(Hun, sat);
        const bool kzero = (lk == 0) && (i == 0);
        Hs[i] = v ? (kzero ? Hun : Hc) : ((i == i0) ? row0 : kNegInf32);
        // bridge candidate of this cell (dynprog_genome.c:2736-2844); the row's carried candidate
        // comes from band offset k+1 of the previous column
        const bool cand = (i >= clo) & (i <= chi);
        const int s = isc[((qw[i] >> 24) & 0xff) & cdi] + Hc;
        const double p = rp[i] + cpc;
        const int ics = (i < R - 1) ? cs[i + 1] : cs_in;
        const int icc = (i < R - 1) ? cc[i + 1] : cc_in;
        const double icp = (i < R - 1) ? cp[i + 1] : cp_in;
        const bool take = cand & ((icc < 0) | (s > ics) | ((s == ics) & (p > icp)));
        cs[i] = take ? s : ics;
        cc[i] = take ? c : icc;
        cp[i] = take ? p : icp;
        dval = (k0 + i == uband) ? Hc : dval;  // matrix[r][r]
        qw[i] = (i < R - 1) ? qw[i + 1] : qw_new;
        rp[i] = (i < R - 1) ? rp[i + 1] : rp_new;
      }
      if (lane == src) {
        uint64_t* dcol = dirs + (size_t)c * 4 * R;
#pragma unroll
        for (int i = 0; i < R; i++) {
          dcol[0 * R + i] = mH[i];
          dcol[1 * R + i] = mV[i];
          dcol[2 * R + i] = mE[i];
          dcol[3 * R + i] = mF[i];
        }
      }
      if (c <= rlen - 1 && lk == uband / R) diag[c] = dval;  // the cell (c, c) at band offset uband
      if (lk == 0) {  // the row at offset 0 leaves the band: its candidate is final
        const int r = rtop;
        if (r >= 1 && r <= rlen - 1) {
          part[r].s = cs[0];
          part[r].c = cc[0];
          part[r].p = cp[0];
        }
      }
      if (c == glen) {  // rows still inside the band after the last column
#pragma unroll
        for (int i = 0; i < R; i++) {
          const int k = k0 + i;
          const int r = glen - uband + k;
          if (k >= 1 && k < W && r >= 1 && r <= rlen - 1) {
            part[r].s = cs[i];
            part[r].c = cc[i];
            part[r].p = cp[i];
          }
        }
      }
    }
  }
}

// ---------------------------------------------------------------------------
// 1. prep: stage into scratch, genome_gap_simple (one wave per problem)
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(64) void ggp_prep_kernel(
    const DevGenomeProblem* __restrict__ probs, const int* __restrict__ order, const uint32_t* __restrict__ blocks,
    uint64_t nwords, const char* __restrict__ qseq, const char* __restrict__ qseq_uc,
    const double* __restrict__ sprob, const int8_t* __restrict__ sctab, const uint8_t* __restrict__ constab,
    const int8_t* __restrict__ isctab, gmapdp_genome_result* __restrict__ results, gmapdp_pair* __restrict__ pairs,
    unsigned char* __restrict__ gscratch) {
  const int lane = threadIdx.x;
  const int pid = order[blockIdx.x];
  const DevGenomeProblem P = probs[pid];
  const int rlen = P.rlength, gL = P.glengthL, gR = P.glengthR;
  const int flags = P.flags;
  const ScratchGGP sv = scratch_ggp(rlen, gL, gR);
  unsigned char* gb = gscratch + P.dirs_offset;
  int32_t* scL = reinterpret_cast<int32_t*>(gb + sv.scL);
  int32_t* scR = reinterpret_cast<int32_t*>(gb + sv.scR);
  uint8_t* gclL = gb + sv.gclL;
  uint8_t* gclR = gb + sv.gclR;
  uint8_t* ldi = gb + sv.ldi;
  uint8_t* rdi = gb + sv.rdi;
  GGPSummary* sum = reinterpret_cast<GGPSummary*>(gb + sv.sum);
  const int8_t* sct = sctab + (size_t)P.mismatchtype * 128 * kNClass;
  for (int i = lane; i < rlen; i += 64) {
    const char c1 = qseq[P.qbase + i];
    const uint64_t row = *reinterpret_cast<const uint64_t*>(sct + (uint8_t)(c1 & 127) * kNClass);
    uint32_t w = 0;
#pragma unroll
    for (int g = 0; g < 6; g++) w |= (uint32_t)((row >> (8 * g)) & 0xfu) << (4 * g);
    scL[i + 1] = (int32_t)w;
    scR[rlen - i] = (int32_t)w;
  }
  if (lane < 2) {
    scL[lane ? rlen + 1 : 0] = 0;
    scR[lane ? rlen + 1 : 0] = 0;
  }
  for (int i = lane; i < gL; i += 64) {
    const char c2 = segment_nt(blocks, nwords, (uint32_t)i, (uint32_t)gL, P.segposL, P.segboundL, flags & kGSegLLeft,
                               flags & kGSegLRc);
    gclL[i + 1] = gclass(c2);
  }
  for (int i = lane; i < gR; i += 64) {
    const char c2 = segment_nt(blocks, nwords, (uint32_t)i, (uint32_t)gR, P.segposR, P.segboundR, flags & kGSegRLeft,
                               flags & kGSegRRc);
    gclR[gR - i] = gclass(c2);  // rev_gsequenceR[1-c] = segment[glengthR-c]
  }
  __threadfence_block();
  const GClassView gchL{gclL}, gchR{gclR};
  // leftdi[cL] from gsequenceL[cL], [cL+1]; rightdi[cR] from rev_gsequenceR[-cR-1], [-cR] (:2518-2566)
  for (int c = lane; c <= gL; c += 64) ldi[c] = (c < gL - 1) ? left_dinucl(gchL[c + 1], gchL[c + 2]) : 0;
  for (int c = lane; c <= gR; c += 64) rdi[c] = (c < gR - 1) ? right_dinucl(gchR[c + 2], gchR[c + 1]) : 0;
  __threadfence_block();

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
  bool done = false;
  if (flags & kGSimple) {
    const QView qL{qseq + P.qbase, 1}, qucL{qseq_uc + P.qbase, 1};
    const QView qR{qseq + P.qbase + rlen - 1, -1}, qucR{qseq_uc + P.qbase + rlen - 1, -1};
    const uint8_t* cons = constab + (size_t)P.genestrand * 128 * kNClass;
    int* diagL = reinterpret_cast<int*>(gb + sv.diagL);
    int* diagR = reinterpret_cast<int*>(gb + sv.diagR);
    done = gg_simple_wave(lane, P, pid, sctab, isctab, cons, qL, qucL, qR, qucR, gclL, gclR, gchL, gchR, ldi, rdi,
                          sprob + P.prob_offset, sprob + P.prob_offset + gL, diagL, diagR, pairs + P.pair_offset, res,
                          results);
  }
  if (lane == 0) {
    sum->full = done ? 0 : 1;
    sum->res = res;
  }
}

// ---------------------------------------------------------------------------
// 2. fills + bridge: one wave per chunk of kGgpChunk class members; the members genome_gap_simple
//    left are compacted in order and filled 64/S at a time (rounds)
// ---------------------------------------------------------------------------
// Ballot words of one round: both fills, (gmax + 1) columns x 4R words each.
__host__ __device__ inline size_t ggp_round_bytes(int gmax, int R) { return 2u * (size_t)(gmax + 1) * 4u * (size_t)R * 8u; }

template <int S, int R>
__global__ __launch_bounds__(64) void ggp_fill_kernel(const DevGenomeProblem* __restrict__ probs,
                                                      const int* __restrict__ order, int count,
                                                      const double* __restrict__ sprob,
                                                      const int8_t* __restrict__ isctab,
                                                      unsigned char* __restrict__ gscratch) {
  constexpr int NP = 64 / S;
  static_assert(kGgpChunk <= 64, "one flag per lane");
  __shared__ int8_t isc_lds[NP][64];
  __shared__ int members[kGgpChunk];
  const int lane = threadIdx.x;
  const int grp = lane / S, lk = lane & (S - 1);
  const int first = blockIdx.x * kGgpChunk;
  const int n = min(kGgpChunk, count - first);
  // the chunk's members that need the full path, in class order
  bool full = false;
  int gmax = 0;
  if (lane < n) {
    const DevGenomeProblem Q = probs[order[first + lane]];
    const ScratchGGP q = scratch_ggp(Q.rlength, Q.glengthL, Q.glengthR);
    full = reinterpret_cast<const GGPSummary*>(gscratch + Q.dirs_offset + q.sum)->full != 0;
    gmax = max(Q.glengthL, Q.glengthR);
  }
  const uint64_t mfull = ballot(full);
  if (full) members[lanes_below(mfull, lane)] = first + lane;
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) gmax = max(gmax, __shfl_xor(gmax, off, 64));
  const int nfull = __popcll(mfull);
  const int64_t region = probs[order[first]].aux_offset;  // the chunk's ballot words
  __syncthreads();

  for (int round = 0; round * NP < nfull; round++) {
    const int m = round * NP + grp;
    const bool act = m < nfull;
    const int pid = order[act ? members[m] : members[round * NP]];
    const DevGenomeProblem P = probs[pid];
    const int rlen = P.rlength, gL = P.glengthL, gR = P.glengthR;
    const ScratchGGP sv = scratch_ggp(rlen, gL, gR);
    unsigned char* gb = gscratch + P.dirs_offset;
    GGPSummary* sum = reinterpret_cast<GGPSummary*>(gb + sv.sum);
    // the group's intron score array (64 entries)
    for (int i = lk; i < 64; i += S)
      isc_lds[grp][i] = isctab[(size_t)P.iclass * 128 + ((P.flags & kGFinal) ? 64 : 0) + i];
    __syncthreads();
    const int8_t* isc = isc_lds[grp];
    const int late = (P.flags & kFLate) ? 1 : 0;
    const int lband = P.lbandL;
    const int32_t* scL = reinterpret_cast<const int32_t*>(gb + sv.scL);
    const int32_t* scR = reinterpret_cast<const int32_t*>(gb + sv.scR);
    const uint8_t* gclL = gb + sv.gclL;
    const uint8_t* gclR = gb + sv.gclR;
    const uint8_t* ldi = gb + sv.ldi;
    const uint8_t* rdi = gb + sv.rdi;
    const double* pL = sprob + P.prob_offset;
    const double* pR = sprob + P.prob_offset + gL;
    Part* partB = reinterpret_cast<Part*>(gb + sv.partB);  // indexed by rR
    Part* partC = reinterpret_cast<Part*>(gb + sv.partC);  // indexed by rL
    int* diagL = reinterpret_cast<int*>(gb + sv.diagL);
    int* diagR = reinterpret_cast<int*>(gb + sv.diagR);
    const int64_t rbase = region + (int64_t)round * (int64_t)ggp_round_bytes(gmax, R);
    uint64_t* dirsR = reinterpret_cast<uint64_t*>(gscratch + rbase);
    uint64_t* dirsL = dirsR + (size_t)(gmax + 1) * 4 * R;
    const int rdist = P.rev_goffsetR - P.goffsetL;  // "cR < rightoffset - leftoffset - cL"
    // the round's longest fill of each side
    int gmR = act ? gR : 0, gmL = act ? gL : 0;
#pragma unroll
    for (int off = S; off < 64; off <<= 1) {
      gmR = max(gmR, __shfl_xor(gmR, off, 64));
      gmL = max(gmL, __shfl_xor(gmL, off, 64));
    }
    // R fill: reversed query vs rev_gsequenceR, lband = lbandL, !jump_late_p (:3810); B candidates
    fill_grp<S, R>(lane, lk, act, rlen, gR, gmR, lband, P.ubandR, P.open, P.extend, 1 - late, scR, gclR, ldi, rdi, pL,
                   pR, isc, rdist, partB, diagR, dirsR);
    // L fill (:3801); C candidates
    fill_grp<S, R>(lane, lk, act, rlen, gL, gmL, lband, P.ubandL, P.open, P.extend, late, scL, gclL, rdi, ldi, pR,
                   pL, isc, rdist, partC, diagL, dirsL);
    __threadfence_block();

    // bridge: the group's lanes scan rows rL = lk+1, lk+1+S, ... (A, B, C per row), then reduce
    int ws = kNegInf32, wrL = -1, wcL = 0, wcR = 0;
    double wp = 0.0;
    int ds = 0, drL = 0x7fffffff;
    double dp = 0.0;
    if (act) {
      for (int rL = lk + 1; rL <= rlen - 1; rL += S) {
        const int rR = rlen - rL;
        const int dL = diagL[rL], dR = diagR[rR];
        const int sI = isc[ldi[rL] & rdi[rR]];
        int rs = dL + sI + dR, rcL = rL, rcR = rR;
        double rp = pL[rL] + pR[rR];
        if (sI > 0 && rp > dp) {
          dp = rp;
          ds = rs;
          drL = rL;
        }
        const Part b = partB[rR];
        if (b.c >= 0 && lex_better(dL + b.s, b.p, rs, rp)) {
          rs = dL + b.s;
          rp = b.p;
          rcL = rL;
          rcR = b.c;
        }
        const Part cpart = partC[rL];
        if (cpart.c >= 0 && lex_better(dR + cpart.s, cpart.p, rs, rp)) {
          rs = dR + cpart.s;
          rp = cpart.p;
          rcL = cpart.c;
          rcR = rR;
        }
        if (lex_better(rs, rp, ws, wp)) {
          ws = rs;
          wp = rp;
          wrL = rL;
          wcL = rcL;
          wcR = rcR;
        }
      }
    }
#pragma unroll
    for (int off = S / 2; off >= 1; off >>= 1) {  // merge rows across the group: (score desc, prob desc, rL asc)
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
    if (act && lk == 0) {
      sum->ws = ws;
      sum->wrL = wrL;
      sum->wcL = wcL;
      sum->wcR = wcR;
      sum->ds = ds;
      sum->drL = drL;
      sum->wp = wp;
      sum->dp = dp;
      sum->lane0 = grp * S;
      sum->dirsR = rbase;
      sum->dirsL = rbase + (int64_t)(gmax + 1) * 4 * R * 8;
    }
    __syncthreads();  // isc_lds is rewritten by the next round
  }
}

// ---------------------------------------------------------------------------
// 3. tail: decision, tracebacks, gap holder, Pair_maxnegscore, result (one wave per problem)
// ---------------------------------------------------------------------------
template <int S, int R>
__global__ __launch_bounds__(64) void ggp_tail_kernel(
    const DevGenomeProblem* __restrict__ probs, const int* __restrict__ order, const uint32_t* __restrict__ blocks,
    uint64_t nwords, const char* __restrict__ qseq, const char* __restrict__ qseq_uc,
    const double* __restrict__ sprob, const uint8_t* __restrict__ constab, const int8_t* __restrict__ isctab,
    gmapdp_genome_result* __restrict__ results, gmapdp_pair* __restrict__ pairs,
    unsigned char* __restrict__ gscratch) {
  const int lane = threadIdx.x;
  const int pid = order[blockIdx.x];
  const DevGenomeProblem P = probs[pid];
  const int rlen = P.rlength, gL = P.glengthL, gR = P.glengthR;
  const ScratchGGP sv = scratch_ggp(rlen, gL, gR);
  unsigned char* gb = gscratch + P.dirs_offset;
  const GGPSummary* sum = reinterpret_cast<const GGPSummary*>(gb + sv.sum);
  if (!sum->full) return;
  gmapdp_genome_result res = sum->res;
  const int flags = P.flags;
  const bool watson = flags & kFWatson;
  const int lband = P.lbandL, ubandL = P.ubandL, ubandR = P.ubandR;
  const int WL = lband + ubandL + 1, WR = lband + ubandR + 1;
  const int8_t* isc = isctab + (size_t)P.iclass * 128 + ((flags & kGFinal) ? 64 : 0);
  const uint8_t* ldi = gb + sv.ldi;
  const uint8_t* rdi = gb + sv.rdi;
  const double* pL = sprob + P.prob_offset;
  const double* pR = sprob + P.prob_offset + gL;
  const bool halfp = flags & kGHalf;
  const int ws = sum->ws, wrL = sum->wrL, wcL = sum->wcL, wcR = sum->wcR, ds = sum->ds, drL = sum->drL;
  const double wp = sum->wp, dp = sum->dp;

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

  const uint8_t* gclL = gb + sv.gclL;
  const uint8_t* gclR = gb + sv.gclR;
  const QView qL{qseq + P.qbase, 1}, qucL{qseq_uc + P.qbase, 1};
  const QView qR{qseq + P.qbase + rlen - 1, -1}, qucR{qseq_uc + P.qbase + rlen - 1, -1};
  const GClassView gchL{gclL}, gchR{gclR};
  const uint8_t* cons = constab + (size_t)P.genestrand * 128 * kNClass;
  gmapdp_pair* out = pairs + P.pair_offset;
  const int rev_roffset = P.roffset + rlen - 1;
  const Geo GL{P.roffset, P.goffsetL, 1};
  const Geo GR{rev_roffset, P.rev_goffsetR, -1};
  const BallotDirs<R> dR{reinterpret_cast<const uint64_t*>(gscratch + sum->dirsR), WR, ubandR, sum->lane0};
  const BallotDirs<R> dLd{reinterpret_cast<const uint64_t*>(gscratch + sum->dirsL), WL, ubandL, sum->lane0};
  const int dpi_next = P.dynprogindex + (P.dynprogindex > 0 ? 1 : -1);

  res.left_prob = pL[bestcL];
  res.right_prob = pR[bestcR];
  const int new_left = P.goffsetL + (bestcL - 1);
  const int new_right = P.rev_goffsetR - (bestcR - 1);
  Tally t = {0, 0, 0, 0, 0, 0, 0, false};
  traceback_walk(lane, dR, bestrR, bestcR, GR, qR, qucR, gchR, cons, watson, P.chroffset, P.chrhigh, blocks, nwords,
                 out, t);
  const int nR = t.count;
  reverse_records(lane, out, nR);
  const int queryjump = (rev_roffset - bestrR) - (P.roffset + bestrL) + 1;
  if (lane == 0) put_pair(out, nR, -1, -1, new_right - new_left - 1, ' ', ' ', ' ', ' ');
  t.count += 1;
  traceback_walk(lane, dLd, bestrL, bestcL, GL, qL, qucL, gchL, cons, watson, P.chroffset, P.chrhigh, blocks, nwords,
                 out, t);
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

// ---- host-side launch ----
size_t scratch_bytes_ggp(int rlength, int glengthL, int glengthR) {
  return scratch_ggp(rlength, glengthL, glengthR).total;
}
// ballot words of one fill chunk whose longest segment is gmax (every round of the chunk)
size_t chunk_bytes_ggp(int gmax, int S, int R) {
  return (size_t)((kGgpChunk + 64 / S - 1) / (64 / S)) * ggp_round_bytes(gmax, R);
}

template <int S, int R>
static hipError_t launch_ggp_t(int count, hipStream_t stream, const DevGenomeProblem* probs, const int* order,
                               const uint32_t* blocks, uint64_t nwords, const char* qseq, const char* qseq_uc,
                               const double* sprob, const int8_t* sctab, const uint8_t* constab, const int8_t* isctab,
                               gmapdp_genome_result* results, gmapdp_pair* pairs, unsigned char* gscratch) {
  hipLaunchKernelGGL(ggp_prep_kernel, dim3(count), dim3(64), 0, stream, probs, order, blocks, nwords, qseq, qseq_uc,
                     sprob, sctab, constab, isctab, results, pairs, gscratch);
  hipLaunchKernelGGL((ggp_fill_kernel<S, R>), dim3((count + kGgpChunk - 1) / kGgpChunk), dim3(64), 0, stream, probs,
                     order, count, sprob, isctab, gscratch);
  hipLaunchKernelGGL((ggp_tail_kernel<S, R>), dim3(count), dim3(64), 0, stream, probs, order, blocks, nwords, qseq,
                     qseq_uc, sprob, constab, isctab, results, pairs, gscratch);
  return hipGetLastError();
}

// (S, R) in {(8, 5), (8, 6), (16, 4)}: band width W <= S*R
hipError_t launch_ggp(int S, int R, int count, hipStream_t stream, const DevGenomeProblem* probs, const int* order,
                      const uint32_t* blocks, uint64_t nwords, const char* qseq, const char* qseq_uc,
                      const double* sprob, const int8_t* sctab, const uint8_t* constab, const int8_t* isctab,
                      gmapdp_genome_result* results, gmapdp_pair* pairs, unsigned char* gscratch) {
  if (count <= 0) return hipSuccess;
#define GMAPDP_GGP_CASE(SS, RR)                                                                                   \
  if (S == SS && R == RR)                                                                                      \
    return launch_ggp_t<SS, RR>(count, stream, probs, order, blocks, nwords, qseq, qseq_uc, sprob, sctab, constab, \
                                isctab, results, pairs, gscratch);
  GMAPDP_GGP_CASE(8, 5)
  GMAPDP_GGP_CASE(8, 6)
  GMAPDP_GGP_CASE(16, 3)
  GMAPDP_GGP_CASE(16, 4)
#undef GMAPDP_GGP_CASE
  return hipErrorInvalidValue;
}

}  // namespace gmapdp
