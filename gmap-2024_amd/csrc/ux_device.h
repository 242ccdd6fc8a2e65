// ux_device.h -- device helpers of the SIMD-build triangle fills (Dynprog_simd_{8,16}_upper /
// _lower, dynprog_simd.c:4304/7714, 5340/8586), shared by ux_kernel.hip (end and genome gaps) and
// cg_kernel.hip (cDNA gaps).  See ux_kernel.hip for the emulation scheme.
#pragma once
#include "dp_device.h"

namespace gmapdp {

// One triangle fill, as one segment runs it.  Lanes index query rows (upper) or genome columns
// (lower); steps walk genome columns (upper) or query rows (lower).
struct UxFill {
  int nrow, ncol;       // lane extent (upper: rlength, lower: glength), step extent (the other)
  int band;             // uband (upper) / lband (lower)
  int late, open, ext;
  int t0;               // wave step of the fill's first step
  const uint32_t* lw;   // LDS: per lane index a word of 4-bit pair scores by step class
  const uint8_t* sx;    // LDS: per step index its class (genome class, or nt_to_int of the query)
  int16_t* buf;         // LDS: 2 x (ncol + 1): last lane of the previous block, by block parity
};

__host__ __device__ inline int ux_steps(int nrow, int band, int B) { return (nrow / B + 1) * (B + band); }

// Cells of one fill as the segment `seg` stored them: wd[2 t + {0 nogap, 1 gap}] ballots,
// ws[64 t + lane] scores.
struct UxView {
  const uint64_t* wd;
  const int16_t* ws;
  int seg, B, t0, nrow, ncol, band, upper;
  int lgB;  // log2(B): B is 16 or 32, so blocks are shifts, not divisions
  __device__ int step(int i, int x) const {  // -1 where no block of the fill wrote
    if (i < 0 || i > nrow || x < 0) return -1;
    const int k = i >> lgB, lo = k << lgB, hi = min(lo + B - 1, nrow);
    if (x < lo || x > min(hi + band, ncol)) return -1;
    return t0 + k * (B + band) + (x - lo);
  }
  __device__ uint32_t bit(int i, int x, int plane) const {
    const int s = step(i, x);
    if (s < 0) return 0u;
    return (uint32_t)(wd[2 * (size_t)s + plane] >> (seg * B + (i & (B - 1)))) & 1u;
  }
  __device__ int score(int i, int x) const {
    const int s = step(i, x);
    return s < 0 ? 0 : (int)ws[(size_t)s * 64 + seg * B + (i & (B - 1))];
  }
  __device__ int cell(int r, int c) const { return upper ? score(r, c) : score(c, r); }
  // traceback_walk's view: t 0 nogap=HORIZ, 1 nogap=VERT, 2 Egap=HORIZ, 3 Fgap=VERT
  __device__ uint32_t operator()(int c, int t, int r) const {
    if (upper) return t == 0 ? bit(r, c, 0) : (t == 2 ? bit(r, c, 1) : 0u);
    return t == 1 ? bit(c, r, 0) : (t == 3 ? bit(c, r, 1) : 0u);
  }
};

// All fills of one problem, fill f on segment f % NSEG, a segment's fills back to back.
template <int B>
__device__ void ux_run_fills(int lane, const UxFill* F, int nfill, int tmax, uint64_t* __restrict__ wd,
                             int16_t* __restrict__ ws) {
  constexpr int NSEG = 64 / B;
  constexpr int NEG = (B == 32) ? -128 : -32768;  // NEG_INFINITY_8 / NEG_INFINITY_16
  constexpr int POS = (B == 32) ? 127 : 32767;
  const int seg = lane / B, sl = lane & (B - 1);
  int fi = seg;
  bool live = fi < nfill;
  UxFill f = F[live ? fi : 0];
  int nblk = f.nrow / B + 1, stride = B + f.band;
  int k = 0, o = 0, H = 0, E = 0;
  for (int t = 0; t < tmax; t++) {
    const int lo = k * B, hi = min(lo + B - 1, f.nrow), x = lo + o;
    const bool act = live && x <= min(hi + f.band, f.ncol);
    if (o == 0) {  // block start (dynprog_simd.c:4479-4483): "compensate for T1 = H + open"
      E = f.late ? NEG : NEG + 1;
      H = NEG - f.open;
    }
    int X = 0;  // H of the row above the block, previous step (lane 0's diagonal input)
    if (act && x > 0) {
      if (lo == 0) X = NEG;
      else if (x - lo <= f.band) X = f.buf[((k - 1) & 1) * (f.ncol + 1) + x - 1];
    }
    const int cls = (!act || x == 0) ? 4 : min((int)f.sx[x], 4);
    const int p = act ? __builtin_amdgcn_sbfe((int)f.lw[lo + sl], 4 * cls, 4) : 0;
    const bool m = sl >= o;  // E_mask: lanes still on or below the diagonal
    if (m) E = NEG;
    const int T1 = sat_add(H, f.open, NEG, POS);
    bool dE = f.late ? (E >= T1) : (E > T1);
    E = sat_add(max(E, T1), f.ext, NEG, POS);
    if (m) E = NEG;
    const int Hs = seg_shr1<B>(H, X, sl);
    const int Hd = sat_add(Hs, p, NEG, POS);
    bool dN = f.late ? (E >= Hd) : (E > Hd);
    const int Hn = max(Hd, E);
    if (x <= hi && lo + sl == x) {  // the diagonal cell's directions are forced DIAG (:4614-4618)
      dE = false;
      dN = false;
    }
    const uint64_t mN = ballot(act && dN), mE = ballot(act && dE);
    if (lane == 0) {
      wd[2 * (size_t)t] = mN;
      wd[2 * (size_t)t + 1] = mE;
    }
    if (act) {
      H = Hn;
      ws[(size_t)t * 64 + lane] = (int16_t)Hn;
      if (sl == B - 1) f.buf[(k & 1) * (f.ncol + 1) + x] = (int16_t)Hn;
    }
    if (live && ++o == stride) {
      o = 0;
      if (++k == nblk) {
        fi += NSEG;
        live = fi < nfill;
        if (live) {
          f = F[fi];
          nblk = f.nrow / B + 1;
          stride = B + f.band;
          k = 0;
        }
      }
    }
  }
}

__device__ __forceinline__ int nt_class(char c) {  // nt_to_int_array (dynprog.c:1012-1019)
  switch (c) {
    case 'A': case 'a': return 0;
    case 'C': case 'c': return 1;
    case 'G': case 'g': return 2;
    case 'T': case 't': return 3;
    default: return 4;
  }
}

// 4-bit scores of one query byte against the genome classes A C G T N (upper pair scores)
__device__ __forceinline__ uint32_t row_word(const int8_t* sct, char c1) {
  const uint64_t row = *reinterpret_cast<const uint64_t*>(sct + (uint8_t)(c1 & 127) * kNClass);
  uint32_t w = 0;
#pragma unroll
  for (int g = 0; g < 5; g++) w |= (uint32_t)((row >> (8 * g)) & 0xfu) << (4 * g);
  return w;
}
// 4-bit scores of query classes A C G T N against one genome class (lower pair scores)
__device__ __forceinline__ uint32_t col_word(const int8_t* sct, int gcls) {
  uint32_t w = 0;
#pragma unroll
  for (int k = 0; k < 5; k++) {
    const char a = (char)((0x4E54474341ull >> (8 * k)) & 0xff);  // "ACGTN"
    w |= (uint32_t)(sct[(uint8_t)a * kNClass + gcls] & 0xf) << (4 * k);
  }
  return w;
}

// Per-side LDS of the triangle fills: upper lane words (query rows), lower lane words (genome
// columns), query classes, genome classes, the two block-row buffers of each fill.
struct CarveUx {
  size_t qw, cw, qc, gcl, bufU, bufL, total;
};
__host__ __device__ inline int ux_ceil(int n, int B) { return ((n + B) / B) * B; }
__host__ __device__ inline CarveUx carve_ux(int rlength, int glength, int B, size_t off) {
  CarveUx cv;
  cv.qw = off;   off = align16(off + 4u * (size_t)ux_ceil(rlength, B));
  cv.cw = off;   off = align16(off + 4u * (size_t)ux_ceil(glength, B));
  cv.qc = off;   off = align16(off + (size_t)(rlength + 2));
  cv.gcl = off;  off = align16(off + (size_t)(glength + 2));
  cv.bufU = off; off = align16(off + 4u * (size_t)(glength + 1));
  cv.bufL = off; off = align16(off + 4u * (size_t)(rlength + 1));
  cv.total = off;
  return cv;
}

// Stage one side: the fill's query (row r = qp[qstep * (r - 1)]), its genome classes, lane words.
template <int B>
__device__ void ux_stage(int lane, unsigned char* smem, const CarveUx& cv, int rlen, int glen, const char* qp,
                         int qstep, const int8_t* sct) {
  uint32_t* qw = reinterpret_cast<uint32_t*>(smem + cv.qw);
  uint32_t* cw = reinterpret_cast<uint32_t*>(smem + cv.cw);
  uint8_t* qc = smem + cv.qc;
  const uint8_t* gcl = smem + cv.gcl;
  const int cr = ux_ceil(rlen, B), cg = ux_ceil(glen, B);
  for (int i = lane; i < cr; i += 64) {  // row 0 scores 'N' (:4424); rows past rlength 0
    uint32_t w = 0;
    if (i == 0) w = row_word(sct, 'N');
    else if (i <= rlen) {
      const char c1 = qp[qstep * (i - 1)];
      w = row_word(sct, c1);
      qc[i] = (uint8_t)nt_class(c1);
    }
    qw[i] = w;
  }
  for (int i = lane; i < cg; i += 64) {  // column 0: byte 4 (8-bit, :5459) / 'N' (16-bit, :8690)
    uint32_t w = 0;
    if (i == 0) w = (B == 32) ? 0u : col_word(sct, kN);
    else if (i <= glen) w = col_word(sct, gcl[i]);
    cw[i] = w;
  }
}

template <int B>
__device__ __forceinline__ UxFill ux_fill(unsigned char* smem, const CarveUx& cv, bool upper, int rlen, int glen,
                                          int band, int late, int open, int ext, int t0) {
  UxFill f;
  f.nrow = upper ? rlen : glen;
  f.ncol = upper ? glen : rlen;
  f.band = band;
  f.late = late;
  f.open = open;
  f.ext = ext;
  f.t0 = t0;
  f.lw = reinterpret_cast<const uint32_t*>(smem + (upper ? cv.qw : cv.cw));
  f.sx = smem + (upper ? cv.gcl : cv.qc);
  f.buf = reinterpret_cast<int16_t*>(smem + (upper ? cv.bufU : cv.bufL));
  return f;
}

__device__ __forceinline__ UxView ux_view(const uint64_t* wd, const int16_t* ws, int seg, int B, const UxFill& f,
                                          bool upper) {
  return UxView{wd, ws, seg, B, f.t0, f.nrow, f.ncol, f.band, upper ? 1 : 0, B == 32 ? 5 : 4};
}

}  // namespace gmapdp
