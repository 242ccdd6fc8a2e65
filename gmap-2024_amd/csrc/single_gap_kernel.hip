// single_gap_kernel.hip -- CDNA4 (gfx950) kernel for GMAP's Dynprog_single_gap.
//
// One 64-lane wavefront (= one workgroup) owns one DP sub-problem.  Reference
// semantics restated (paths under the reference tree's src/):
//   Dynprog_single_gap      dynprog_single.c:429-676 (simple path :346-425)
//   Dynprog_standard        dynprog.c:1268-1786 (nosimd fill; recurrence, band,
//                           boundary rows/columns, >= vs > tie rule, clamp)
//   Dynprog_traceback_std   dynprog.c:1796-1948
//   Pairpool_add_queryskip / _add_genomeskip / _push_gapholder  pairpool.c:981/1068/375
//   Genome_get_segment_right/_left, get_genomic_nt   genome.c:11023/11079, dynprog_single.c:116
//
// Design (not a translation of the reference's column loop):
//  * Band-major lanes: lane L holds band offsets k = L*R .. L*R+R-1 of the
//    current genome column c (row r = c - uband + k).  The diagonal input of a
//    cell is the same band offset one column back (a register), the E
//    (horizontal) input is band offset k+1 one column back (one DPP
//    wave_shl:1), and the vertical F chain -- the only intra-column
//    dependence -- is resolved with a max-plus prefix scan across the wave
//    (DPP row_shr/row_bcast), using F(r) = ext + max(F(r-1), H'(r-1)+open),
//    valid because open <= 0 (H' = max(diag+pair, E), the H value before F).
//  * Direction bits never leave the CU: per column four 64-bit ballots
//    (nogap=HORIZ, nogap=VERT, Egap=HORIZ, Fgap=VERT) go to LDS (or, for the
//    rare very long / very wide problems, to an L2-resident scratch).
//  * Traceback is wave-cooperative: each run (diagonal run, E chain, F chain)
//    is found with one ballot over 64 candidate cells, and its Pair records
//    are expanded by all 64 lanes and stream-compacted straight to HBM in the
//    reference's List_T order.
//  * The genome segment is decoded in-kernel from the HBM-resident packed
//    .genomecomp blocks (3 x u32 per 32 nt).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "gmapdp_internal.h"
#include "../../include/gmapdp.h"

namespace gmapdp {

constexpr int kSent = -(1 << 28);  // scan identity, far below any reachable score

__device__ __forceinline__ int dpp_wave_shl1(int x, int fill) {
  // lane i <- lane i+1; lane 63 <- fill
  return __builtin_amdgcn_update_dpp(fill, x, 0x130, 0xf, 0xf, false);
}
__device__ __forceinline__ int dpp_wave_shr1(int x, int fill) {
  // lane i <- lane i-1; lane 0 <- fill
  return __builtin_amdgcn_update_dpp(fill, x, 0x138, 0xf, 0xf, false);
}

// Inclusive max-scan over the 64 lanes (lane order), identity kSent.
__device__ __forceinline__ int wave_scan_max(int x) {
  x = max(x, __builtin_amdgcn_update_dpp(kSent, x, 0x111, 0xf, 0xf, false));  // row_shr:1
  x = max(x, __builtin_amdgcn_update_dpp(kSent, x, 0x112, 0xf, 0xf, false));  // row_shr:2
  x = max(x, __builtin_amdgcn_update_dpp(kSent, x, 0x114, 0xf, 0xf, false));  // row_shr:4
  x = max(x, __builtin_amdgcn_update_dpp(kSent, x, 0x118, 0xf, 0xf, false));  // row_shr:8
  x = max(x, __builtin_amdgcn_update_dpp(kSent, x, 0x142, 0xa, 0xf, false));  // row_bcast:15
  x = max(x, __builtin_amdgcn_update_dpp(kSent, x, 0x143, 0xc, 0xf, false));  // row_bcast:31
  return x;
}

__device__ __forceinline__ uint64_t ballot(bool p) { return __ballot(p); }
__device__ __forceinline__ int lanes_below(uint64_t m, int lane) {
  return __popcll(m & ((lane == 0) ? 0ull : (~0ull >> (64 - lane))));
}

// ---- genome access (.genomecomp: {high nt16-31, low nt0-15, flags} per 32 nt) ----
__device__ __forceinline__ char decode_nt(const uint32_t* __restrict__ blocks, uint64_t nwords, uint32_t pos) {
  const uint64_t ptr = (uint64_t)(pos >> 5) * 3u;
  if (ptr + 2 >= nwords) return 'N';  // beyond the allocation (reference: undefined)
  const uint32_t bit = pos & 31u;
  if ((blocks[ptr + 2] >> bit) & 1u) return 'N';
  const uint32_t w = (bit < 16) ? blocks[ptr + 1] : blocks[ptr];
  const uint32_t x = (w >> (2u * (bit & 15u))) & 3u;
  return (char)((0x54474341u >> (8u * x)) & 0xffu);  // "ACGT"
}
__device__ __forceinline__ char compl_nt(char c) {
  switch (c) { case 'A': return 'T'; case 'C': return 'G'; case 'G': return 'C'; case 'T': return 'A'; default: return c; }
}
__device__ __forceinline__ uint8_t gclass(char c) {
  switch (c) { case 'A': return kA; case 'C': return kC; case 'G': return kG; case 'T': return kT; case '*': return kStar; default: return kN; }
}
// get_genomic_nt (dynprog_single.c:116; Univcoord_T is 32-bit)
__device__ __forceinline__ char genomic_nt(const uint32_t* __restrict__ blocks, uint64_t nwords, int genomicpos,
                                           uint32_t chroffset, uint32_t chrhigh, bool watson) {
  if (watson) {
    const uint32_t pos = chroffset + (uint32_t)genomicpos;
    if (pos < chroffset || pos >= chrhigh) return '*';
    return decode_nt(blocks, nwords, pos);
  } else {
    const uint32_t pos = chrhigh - (uint32_t)genomicpos;
    if (pos < chroffset || pos >= chrhigh) return '*';
    return compl_nt(decode_nt(blocks, nwords, pos));
  }
}
// Character i of the segment Dynprog_single_gap extracts (dynprog_single.c:565-571 ->
// Genome_get_segment_right / Genome_get_segment_left + revcomp).
__device__ __forceinline__ char segment_nt(const uint32_t* __restrict__ blocks, uint64_t nwords, uint32_t i,
                                           uint32_t length, int goffset, uint32_t chroffset, uint32_t chrhigh,
                                           bool watson) {
  if (watson) {
    const uint32_t left = chroffset + (uint32_t)goffset;
    if (left >= chrhigh) return '*';
    if (left + length >= chrhigh) {
      const uint32_t oob = left + length - chrhigh;
      if (i + oob >= length) return '*';
    }
    return decode_nt(blocks, nwords, left + i);
  } else {
    const uint32_t right = chrhigh - (uint32_t)goffset + 1u;
    const uint32_t j = length - 1u - i;  // position in the forward (pre-revcomp) segment
    if (right < chroffset) return '*';
    if (right < chroffset + length) {
      const uint32_t oob = chroffset + length - right;
      if (j < oob) return '*';
    }
    return compl_nt(decode_nt(blocks, nwords, right - length + j));
  }
}

// ---- LDS carve (must match lds_bytes_single on the host) ----
__host__ __device__ constexpr size_t align16(size_t x) { return (x + 15) & ~size_t(15); }
struct Carve {
  size_t sc, q, quc, gch, gcls, dirs, total;
};
__host__ __device__ inline Carve carve_single(int rlength, int glength, int R, bool dirs_lds) {
  Carve cv;
  size_t off = 0;
  cv.sc = off;   off = align16(off + 8 * (size_t)(rlength + 1));
  cv.q = off;    off = align16(off + (size_t)(rlength + 1));
  cv.quc = off;  off = align16(off + (size_t)(rlength + 1));
  cv.gch = off;  off = align16(off + (size_t)(glength + 1));
  cv.gcls = off; off = align16(off + (size_t)(glength + 1));
  cv.dirs = off;
  if (dirs_lds) off = align16(off + (size_t)(glength + 1) * 4u * (size_t)R * 8u);
  cv.total = off;
  return cv;
}

// direction planes: [c][t][i] 64-bit masks; t: 0 nogap=HORIZ, 1 nogap=VERT, 2 Egap=HORIZ, 3 Fgap=VERT;
// band offset k lives in word i = k % R at bit k / R.
template <int R>
__device__ __forceinline__ uint32_t dir_bit(const uint64_t* dirs, int c, int t, int k, int W) {
  if (k < 0 || k >= W) return 0u;  // outside the band: cleared to DIAG (dynprog.c:498)
  const uint64_t m = dirs[((size_t)c * 4 + t) * R + (k % R)];
  return (uint32_t)(m >> (k / R)) & 1u;
}

struct Tally {
  int score, nmatches, nmismatches, nopens, nindels, count;
};

// Pair record writer with wave stream compaction.
__device__ __forceinline__ void put_pair(gmapdp_pair* __restrict__ out, int idx, int querypos, int genomepos, int jump,
                                         char cdna, char comp, char genome, char genomealt) {
  int4 v;
  v.x = querypos;
  v.y = genomepos;
  v.z = jump;
  v.w = (int)((uint32_t)(uint8_t)cdna | ((uint32_t)(uint8_t)comp << 8) | ((uint32_t)(uint8_t)genome << 16) |
              ((uint32_t)(uint8_t)genomealt << 24));
  reinterpret_cast<int4*>(out)[idx] = v;
}

// Diagonal run: cells (r-j, c-j), j in [0, n)  (dynprog.c:1861-1915)
__device__ __forceinline__ void emit_diag(int lane, int r, int c, int n, const DevSingle& P, const char* q, const char* quc,
                          const char* gch, const uint8_t* __restrict__ cons, gmapdp_pair* out, Tally& t) {
  for (int base = 0; base < n; base += 64) {
    const int j = base + lane;
    const bool active = j < n;
    bool notstar = false, good = false, matchish = false, amb = false;
    int qp = 0, gp = 0;
    char c1 = 0, c2 = 0;
    if (active) {
      const int qc = r - 1 - j, gc = c - 1 - j;
      c1 = q[qc + 1];
      const char c1u = quc[qc + 1];
      c2 = gch[gc + 1];
      notstar = c2 != '*';
      if (c1u == c2) {
        matchish = true;
      } else if (cons[(uint8_t)(c1u & 127) * kNClass + gclass(c2)]) {
        matchish = true;
        amb = true;
      }
      qp = P.roffset + qc;
      gp = P.goffset + gc;
      good = notstar && qp >= 0 && gp >= 0;
    }
    const uint64_t mgood = ballot(good);
    t.nmatches += __popcll(ballot(active && notstar && matchish));
    t.nmismatches += __popcll(ballot(active && notstar && !matchish));
    if (good) {
      put_pair(out, t.count + lanes_below(mgood, lane), qp, gp, 0, c1, matchish ? (amb ? ':' : '*') : ' ', c2, c2);
    }
    t.count += __popcll(mgood);
  }
}

// Query skip: Pairpool_add_queryskip(pairs, rs, c, dist, ...) (pairpool.c:981), revp false
__device__ __forceinline__ void emit_queryskip(int lane, int rs, int c, int dist, const DevSingle& P, const char* q, gmapdp_pair* out,
                               Tally& t) {
  const int gp = P.goffset + c - 1;
  for (int base = 0; base < dist; base += 64) {
    const int j = base + lane;
    const bool active = j < dist;
    const int qc = rs - 1 - j;
    const int qp = P.roffset + qc;
    const bool good = active && qp >= 0 && gp >= 0;
    const uint64_t mgood = ballot(good);
    if (good) put_pair(out, t.count + lanes_below(mgood, lane), qp, gp, 0, q[qc + 1], '-', ' ', ' ');
    t.count += __popcll(mgood);
  }
  t.score += kQopen + dist * kQindel;
  t.nopens += 1;
  t.nindels += dist;
}

// Genome skip: Pairpool_add_genomeskip(&add_dashes_p, pairs, r, cs, dist, NULL, ...) (pairpool.c:1068)
__device__ __forceinline__ void emit_genomeskip(int lane, int r, int cs, int dist, const DevSingle& P, const uint32_t* blocks,
                                uint64_t nwords, gmapdp_pair* out, Tally& t) {
  if (dist >= kMicrointronLength) {
    if (lane == 0) put_pair(out, t.count, -1, -1, dist, ' ', ' ', ' ', ' ');
    t.count += 1;
    return;
  }
  const bool watson = P.flags & GMAPDP_WATSON;
  const int qp = P.roffset + r - 1;
  for (int base = 0; base < dist; base += 64) {
    const int j = base + lane;
    const bool active = j < dist;
    const int gc = cs - 1 - j;
    const int gp = P.goffset + gc;
    const bool good = active && qp >= 0 && gp >= 0;
    const uint64_t mgood = ballot(good);
    if (good) {
      const char c2 = genomic_nt(blocks, nwords, gp, P.chroffset, P.chrhigh, watson);
      put_pair(out, t.count + lanes_below(mgood, lane), qp, gp, 0, ' ', '-', c2, c2);
    }
    t.count += __popcll(mgood);
  }
  t.score += kTopen + dist * kTindel;
  t.nopens += 1;
  t.nindels += dist;
}

template <int R, bool DIRS_LDS>
__global__ __launch_bounds__(64) void single_gap_kernel(
    const DevSingle* __restrict__ probs, const int* __restrict__ order,
    const uint32_t* __restrict__ blocks, uint64_t nwords,
    const char* __restrict__ qseq, const char* __restrict__ qseq_uc,
    const int8_t* __restrict__ sctab, const uint8_t* __restrict__ constab,
    gmapdp_result* __restrict__ results, gmapdp_pair* __restrict__ pairs,
    uint64_t* __restrict__ gdirs) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int lane = threadIdx.x;
  const int pid = order[blockIdx.x];
  const DevSingle P = probs[pid];
  const int rlen = P.rlength, glen = P.glength;
  const bool watson = P.flags & GMAPDP_WATSON;
  const bool late = P.flags & GMAPDP_JUMP_LATE;
  const Carve cv = carve_single(rlen, glen, R, DIRS_LDS);
  uint64_t* scrow = reinterpret_cast<uint64_t*>(smem + cv.sc);
  char* q = reinterpret_cast<char*>(smem + cv.q);
  char* quc = reinterpret_cast<char*>(smem + cv.quc);
  char* gch = reinterpret_cast<char*>(smem + cv.gch);
  uint8_t* gcl = reinterpret_cast<uint8_t*>(smem + cv.gcls);
  uint64_t* dirs = DIRS_LDS ? reinterpret_cast<uint64_t*>(smem + cv.dirs)
                            : reinterpret_cast<uint64_t*>(reinterpret_cast<unsigned char*>(gdirs) + P.dirs_offset);
  const int8_t* sct = sctab + (size_t)P.mismatchtype * 128 * kNClass;
  const uint8_t* cons = constab + (size_t)P.genestrand * 128 * kNClass;
  gmapdp_pair* out = pairs + P.pair_offset;

  // ---- stage query, score rows and genome segment in LDS ----
  for (int i = lane; i < rlen; i += 64) {
    const char c1 = qseq[P.qoff + i];
    q[i + 1] = c1;
    quc[i + 1] = qseq_uc[P.qoff + i];
    scrow[i + 1] = *reinterpret_cast<const uint64_t*>(sct + (uint8_t)(c1 & 127) * kNClass);
  }
  for (int i = lane; i < glen; i += 64) {
    const char c2 = segment_nt(blocks, nwords, (uint32_t)i, (uint32_t)glen, P.goffset, P.chroffset, P.chrhigh, watson);
    gch[i + 1] = c2;
    gcl[i + 1] = gclass(c2);
  }
  __syncthreads();

  Tally t = {0, 0, 0, 0, 0, 0};
  const int dpi_next = P.dynprogindex + (P.dynprogindex > 0 ? 1 : -1);

  // ---- single_gap_simple (dynprog_single.c:346, taken when glength == rlength) ----
  if (glen == rlen) {
    int nmism = 0;
    for (int base = 0; base < rlen; base += 64) {
      const int qc = base + lane;
      bool mism = false;
      if (qc < rlen) {
        const char c1u = quc[qc + 1], c2 = gch[qc + 1];
        mism = (c2 != '*') && (c1u != c2) && !cons[(uint8_t)(c1u & 127) * kNClass + gclass(c2)];
      }
      nmism += __popcll(ballot(mism));
    }
    if (nmism <= 1) {
      // pushes r = 1..rlength, no List_reverse: list order is descending
      for (int base = 0; base < rlen; base += 64) {
        const int j = base + lane;
        const bool active = j < rlen;
        const int qc = rlen - 1 - j;
        bool notstar = false, matchish = false, amb = false, good = false;
        char c1 = 0, c2 = 0;
        int qp = 0, gp = 0;
        if (active) {
          c1 = q[qc + 1];
          const char c1u = quc[qc + 1];
          c2 = gch[qc + 1];
          notstar = c2 != '*';
          if (c1u == c2) matchish = true;
          else if (cons[(uint8_t)(c1u & 127) * kNClass + gclass(c2)]) { matchish = true; amb = true; }
          qp = P.roffset + qc;
          gp = P.goffset + qc;
          good = notstar && qp >= 0 && gp >= 0;
        }
        const uint64_t mgood = ballot(good);
        t.nmatches += __popcll(ballot(active && notstar && matchish));
        t.nmismatches += __popcll(ballot(active && notstar && !matchish));
        if (good) put_pair(out, t.count + lanes_below(mgood, lane), qp, gp, 0, c1, matchish ? (amb ? ':' : '*') : ' ', c2, c2);
        t.count += __popcll(mgood);
      }
      if (lane == 0) {
        gmapdp_result res;
        res.npairs = t.count;
        res.pair_offset = P.pair_offset;
        res.traceback_score = t.nmatches * kMatch + t.nmismatches * kMismatch;
        res.nmatches = t.nmatches;
        res.nmismatches = t.nmismatches;
        res.nopens = 0;
        res.nindels = 0;
        res.dynprogindex = dpi_next;
        results[pid] = res;
      }
      return;
    }
  }

  // ---- banded fill (Dynprog_standard, upperp = lowerp = true) ----
  const int lband = P.lband, uband = P.uband, open = P.open, ext = P.extend;
  const int W = lband + uband + 1;
  const int sat = kNegInf32;  // saturation NEG_INFINITY_INT (dynprog_single.c:638)

  int Hc[R], Hu[R], E[R];
#pragma unroll
  for (int i = 0; i < R; i++) {  // column 0 (dynprog.c:1331-1369)
    const int k = lane * R + i;
    const int r = k - uband;
    int v = kNegInf32;
    if (k < W && r >= 0 && r <= rlen) v = (r == 0) ? 0 : (r <= lband ? open + r * ext : kNegInf32);
    Hc[i] = v;
    Hu[i] = v;
    E[i] = kNegInf32;
  }

  for (int c = 1; c <= glen; c++) {
    const int gi = gcl[c];
    const int rtop = c - uband;
    const int rlo = rtop < 1 ? 1 : rtop;
    const int rhigh = (c + lband) < rlen ? (c + lband) : rlen;
    // last_nogap entering row rlo (dynprog.c:1411-1449)
    const int L0 = (c == 1) ? (kNegInf32 - open + 1) : (c <= uband ? open + c * ext : kNegInf32);

    int Ein[R], Hin[R];
#pragma unroll
    for (int i = 0; i < R - 1; i++) { Ein[i] = E[i + 1]; Hin[i] = Hc[i + 1]; }
    Ein[R - 1] = dpp_wave_shl1(E[0], kNegInf32);
    Hin[R - 1] = dpp_wave_shl1(Hc[0], kNegInf32);

    int Hp[R], En[R], A[R], rr[R];
    bool valid[R], eb[R], hb[R];
#pragma unroll
    for (int i = 0; i < R; i++) {
      const int k = lane * R + i;
      const int r = rtop + k;
      rr[i] = r;
      valid[i] = (k < W) && (r >= rlo) && (r <= rhigh);
      const int diag = (r == rlo && rlo > 1) ? Hu[i] : Hc[i];  // first_nogap is unclamped (dynprog.c:1579)
      const int s = valid[i] ? (int)(int8_t)(scrow[r] >> (8 * gi)) : 0;
      // Egap (dynprog.c:1518-1524)
      const int es = Hin[i] + open;
      eb[i] = late ? (Ein[i] >= es) : (Ein[i] > es);
      En[i] = eb[i] ? Ein[i] + ext : es + ext;
      int hp = diag + s;
      hb[i] = late ? (En[i] >= hp) : (En[i] > hp);
      if (hb[i]) hp = En[i];
      Hp[i] = hp;
      A[i] = valid[i] ? hp + open - r * ext : kSent;
    }
    // F chain: F(r) = r*ext + max(init, max_{rlo<=j<r} (H'(j) + open - j*ext))
    int pre[R];
    pre[0] = A[0];
#pragma unroll
    for (int i = 1; i < R; i++) pre[i] = max(pre[i - 1], A[i]);
    const int X = dpp_wave_shr1(wave_scan_max(pre[R - 1]), kSent);
    const int init = max(kNegInf32, L0 + open) - (rlo - 1) * ext;
    int F[R], Hun[R];
    bool vb[R];
#pragma unroll
    for (int i = 0; i < R; i++) {
      const int ex = (i == 0) ? X : max(X, pre[i - 1]);
      F[i] = rr[i] * ext + max(init, ex);
      vb[i] = late ? (F[i] >= Hp[i]) : (F[i] > Hp[i]);
      Hun[i] = vb[i] ? F[i] : Hp[i];
    }
    // Fgap direction needs F(r-1), H(r-1) of this column (dynprog.c:1486-1492)
    const int Fup = dpp_wave_shr1(F[R - 1], kNegInf32);
    const int Hup = dpp_wave_shr1(Hun[R - 1], kNegInf32);
    uint64_t mH[R], mV[R], mE[R], mF[R];
#pragma unroll
    for (int i = 0; i < R; i++) {
      int fprev = (i == 0) ? Fup : F[i - 1];
      int hprev = (i == 0) ? Hup : Hun[i - 1];
      if (rr[i] == rlo) { fprev = kNegInf32; hprev = L0; }
      const int fs = hprev + open;
      const bool fb = late ? (fprev >= fs) : (fprev > fs);
      mV[i] = ballot(valid[i] && vb[i]);
      mH[i] = ballot(valid[i] && hb[i] && !vb[i]);
      mE[i] = ballot(valid[i] && eb[i]);
      mF[i] = ballot(valid[i] && fb);
      // state for the next column
      if (valid[i]) {
        Hu[i] = Hun[i];
        Hc[i] = Hun[i] < sat ? sat : Hun[i];
        E[i] = En[i];
      } else {
        const int v = (rr[i] == 0 && c <= uband) ? open + c * ext : kNegInf32;  // row 0 (dynprog.c:1318-1325)
        Hu[i] = v;
        Hc[i] = v;
        E[i] = kNegInf32;
      }
    }
#pragma unroll
    for (int w0 = 0; w0 < 4 * R; w0 += 64) {  // 4R words per column, 64 lanes per pass
      const int w = w0 + lane;
      if (w < 4 * R) {
        const int t = w / R, i = w % R;
        uint64_t m = 0;
#pragma unroll
        for (int ii = 0; ii < R; ii++) {
          if (ii == i) m = (t == 0) ? mH[ii] : (t == 1) ? mV[ii] : (t == 2) ? mE[ii] : mF[ii];
        }
        dirs[((size_t)c * 4 + t) * R + i] = m;
      }
    }
  }
  if (DIRS_LDS) __syncthreads();
  else __threadfence_block();

  // ---- wave-cooperative traceback (Dynprog_traceback_std, dynprog.c:1796-1948) ----
  int r = rlen, c = glen;
  while (r > 0 && c > 0) {
    const int k = r - c + uband;
    const uint32_t isV = dir_bit<R>(dirs, c, 1, k, W);
    const uint32_t isH = dir_bit<R>(dirs, c, 0, k, W);
    if (!isV && isH) {
      // E chain along row r: columns c, c-1, ... while Egap == HORIZ
      int n = 0;
      for (int base = 0;; base += 64) {
        const int j = base + lane;
        const bool cont = (c - j >= 1) && dir_bit<R>(dirs, c - j, 2, k + j, W);
        const uint64_t stop = ~ballot(cont);
        if (stop) { n = base + __ffsll((long long)stop) - 1; break; }
      }
      const int dist = n + 1;
      const int c_end = (c - n - 1) > 0 ? (c - n - 1) : 0;
      emit_genomeskip(lane, r, c_end + dist, dist, P, blocks, nwords, out, t);
      c = c_end;
    } else if (isV) {
      // F chain up column c: rows r, r-1, ... while Fgap == VERT
      int n = 0;
      for (int base = 0;; base += 64) {
        const int j = base + lane;
        const bool cont = (r - j >= 1) && dir_bit<R>(dirs, c, 3, k - j, W);
        const uint64_t stop = ~ballot(cont);
        if (stop) { n = base + __ffsll((long long)stop) - 1; break; }
      }
      const int dist = n + 1;
      const int r_end = (r - n - 1) > 0 ? (r - n - 1) : 0;
      emit_queryskip(lane, r_end + dist, c, dist, P, q, out, t);
      r = r_end;
    } else {
      // diagonal run at fixed band offset k
      int n = 0;
      for (int base = 0;; base += 64) {
        const int j = base + lane;
        const bool cont = (j == 0) || ((c - j >= 1) && (r - j >= 1) && !dir_bit<R>(dirs, c - j, 0, k, W) &&
                                       !dir_bit<R>(dirs, c - j, 1, k, W));
        const bool inrange = (c - j >= 1) && (r - j >= 1);
        const uint64_t stop = ~ballot(cont && inrange);
        if (stop) { n = base + __ffsll((long long)stop) - 1; break; }
      }
      emit_diag(lane, r, c, n, P, q, quc, gch, cons, out, t);
      r -= n;
      c -= n;
    }
  }
  if (r == 0 && c == 0) {
  } else if (c == 0) {
    emit_queryskip(lane, r, 1, r, P, q, out, t);  // LAZY_INDEL
  } else {
    emit_genomeskip(lane, 1, c, c, P, blocks, nwords, out, t);
  }

  if (lane == 0) {
    gmapdp_result res;
    res.npairs = t.count;
    res.pair_offset = P.pair_offset;
    res.traceback_score = t.score + t.nmatches * kMatch + t.nmismatches * kMismatch;
    res.nmatches = t.nmatches;
    res.nmismatches = t.nmismatches;
    res.nopens = t.nopens;
    res.nindels = t.nindels;
    res.dynprogindex = dpi_next;
    results[pid] = res;
  }
}

// ---- host-side launch table ----
typedef void (*SingleKernelFn)(const DevSingle*, const int*, const uint32_t*, uint64_t, const char*, const char*,
                               const int8_t*, const uint8_t*, gmapdp_result*, gmapdp_pair*, uint64_t*);

template <int R, bool D>
static void* kptr() { return reinterpret_cast<void*>(&single_gap_kernel<R, D>); }

size_t lds_bytes_single(int rlength, int glength, int R, bool dirs_lds) {
  return carve_single(rlength, glength, R, dirs_lds).total;
}

hipError_t launch_single(int R, bool dirs_lds, int nblocks, size_t lds, hipStream_t stream, const DevSingle* probs,
                         const int* order, const uint32_t* blocks, uint64_t nwords, const char* qseq,
                         const char* qseq_uc, const int8_t* sctab, const uint8_t* constab, gmapdp_result* results,
                         gmapdp_pair* pairs, uint64_t* gdirs) {
  void* fn = nullptr;
#define GMAPDP_CASE(RR)                                          \
  case RR:                                                       \
    fn = dirs_lds ? kptr<RR, true>() : kptr<RR, false>();        \
    break;
  switch (R) {
    GMAPDP_CASE(1)
    GMAPDP_CASE(2)
    GMAPDP_CASE(4)
    GMAPDP_CASE(8)
    GMAPDP_CASE(16)
    GMAPDP_CASE(32)
    GMAPDP_CASE(64)
    default: return hipErrorInvalidValue;
  }
#undef GMAPDP_CASE
  if (lds > 64 * 1024) {
    hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
  }
  void* args[] = {(void*)&probs, (void*)&order, (void*)&blocks, (void*)&nwords, (void*)&qseq, (void*)&qseq_uc,
                  (void*)&sctab, (void*)&constab, (void*)&results, (void*)&pairs, (void*)&gdirs};
  return hipLaunchKernel(fn, dim3(nblocks), dim3(64), args, lds, stream);
}

}  // namespace gmapdp
