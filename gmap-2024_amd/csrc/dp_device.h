// dp_device.h -- device helpers shared by the Dynprog_* kernels (dp_kernel.hip, ux_kernel.hip):
// genome decoding, DPP scans, the band fill, the wave-cooperative traceback and Pair emission,
// the genome-gap simple path and Pair_maxnegscore.  Not part of the C ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>


#include "gmapdp_internal.h"
#include "../../include/gmapdp.h"
#include "me_device.h"

namespace gmapdp {


constexpr int kSent = (int)0x80000000;  // max-scan identity (INT_MIN); only ever max'ed, never added to

__device__ __forceinline__ int dpp_wave_shl1(int x, int fill) {
  // lane i <- lane i+1; lane 63 <- fill
  return __builtin_amdgcn_update_dpp(fill, x, 0x130, 0xf, 0xf, false);
}
// lane i <- lane i+1; lane 63 <- 0 (bound_ctrl: one DPP move, no default copied in first)
__device__ __forceinline__ int dpp_wave_shl1_zero(int x) {
  return __builtin_amdgcn_update_dpp(0, x, 0x130, 0xf, 0xf, true);
}
__device__ __forceinline__ int dpp_wave_shr1(int x, int fill) {
  // lane i <- lane i-1; lane 0 <- fill
  return __builtin_amdgcn_update_dpp(fill, x, 0x138, 0xf, 0xf, false);
}
// lane i <- lane i-1; lane 0 <- 0 (for values lane 0 never reads)
__device__ __forceinline__ int dpp_wave_shr1_zero(int x) {
  return __builtin_amdgcn_update_dpp(0, x, 0x138, 0xf, 0xf, true);
}

// Inclusive max-scan over the 64 lanes (lane order).  Lanes without a source
// read the identity INT_MIN, so the DPP move folds into v_max_i32_dpp.
__device__ __forceinline__ int wave_scan_max(int x) {
  x = max(x, __builtin_amdgcn_update_dpp(kSent, x, 0x111, 0xf, 0xf, false));  // row_shr:1
  x = max(x, __builtin_amdgcn_update_dpp(kSent, x, 0x112, 0xf, 0xf, false));  // row_shr:2
  x = max(x, __builtin_amdgcn_update_dpp(kSent, x, 0x114, 0xf, 0xf, false));  // row_shr:4
  x = max(x, __builtin_amdgcn_update_dpp(kSent, x, 0x118, 0xf, 0xf, false));  // row_shr:8
  x = max(x, __builtin_amdgcn_update_dpp(kSent, x, 0x142, 0xa, 0xf, false));  // row_bcast:15
  x = max(x, __builtin_amdgcn_update_dpp(kSent, x, 0x143, 0xc, 0xf, false));  // row_bcast:31
  return x;
}

// ---- segmented variants: a wave split into 64/S segments of S lanes, one DP problem each ----
// lane i <- lane i+1 of its segment; the segment's last lane <- fill
template <int S>
__device__ __forceinline__ int seg_shl1(int x, int fill, int sl) {
  if constexpr (S == 64) {
    return dpp_wave_shl1(x, fill);
  } else if constexpr (S == 16) {
    return __builtin_amdgcn_update_dpp(fill, x, 0x101, 0xf, 0xf, false);  // row_shl:1
  } else {
    const int v = dpp_wave_shl1(x, fill);
    return (sl == S - 1) ? fill : v;
  }
}
// lane i <- lane i-1 of its segment; the segment's first lane <- fill
template <int S>
__device__ __forceinline__ int seg_shr1(int x, int fill, int sl) {
  if constexpr (S == 64) {
    return dpp_wave_shr1(x, fill);
  } else if constexpr (S == 16) {
    return __builtin_amdgcn_update_dpp(fill, x, 0x111, 0xf, 0xf, false);  // row_shr:1
  } else {
    const int v = dpp_wave_shr1(x, fill);
    return (sl == 0) ? fill : v;
  }
}
// inclusive max-scan within each segment
template <int S>
__device__ __forceinline__ int seg_scan_max(int x) {
  if constexpr (S == 64) return wave_scan_max(x);
  x = max(x, __builtin_amdgcn_update_dpp(kSent, x, 0x111, 0xf, 0xf, false));  // row_shr:1
  x = max(x, __builtin_amdgcn_update_dpp(kSent, x, 0x112, 0xf, 0xf, false));  // row_shr:2
  x = max(x, __builtin_amdgcn_update_dpp(kSent, x, 0x114, 0xf, 0xf, false));  // row_shr:4
  x = max(x, __builtin_amdgcn_update_dpp(kSent, x, 0x118, 0xf, 0xf, false));  // row_shr:8
  if constexpr (S == 32)
    x = max(x, __builtin_amdgcn_update_dpp(kSent, x, 0x142, 0xa, 0xf, false));  // row_bcast:15 (rows 1, 3)
  return x;
}

// wave64 ballot straight from the compare mask (no bool materialisation)
__device__ __forceinline__ uint64_t ballot(bool p) { return __builtin_amdgcn_ballot_w64(p); }
__device__ __forceinline__ int lanes_below(uint64_t m, int lane) {
  return __popcll(m & ((1ull << lane) - 1ull));
}

// ---- genome access (.genomecomp: {high nt16-31, low nt0-15, flags} per 32 nt) ----
__device__ __forceinline__ char decode_nt(const uint32_t* __restrict__ blocks, uint64_t nwords, uint64_t pos) {
  const uint64_t ptr = (pos >> 5) * 3u;
  if (ptr + 2 >= nwords) return 'N';  // beyond the allocation (reference: undefined)
  const uint32_t bit = pos & 31u;
  if ((blocks[ptr + 2] >> bit) & 1u) return 'N';
  const uint32_t w = (bit < 16) ? blocks[ptr + 1] : blocks[ptr];
  const uint32_t x = (w >> (2u * (bit & 15u))) & 3u;
  return (char)((0x54474341u >> (8u * x)) & 0xffu);  // "ACGT"
}
__device__ __forceinline__ char compl_nt(char c) {
  // only A C G T N * occur: complement of ACGT via a 4-entry table, N and * unchanged
  return (c == 'A') ? 'T' : (c == 'C') ? 'G' : (c == 'G') ? 'C' : (c == 'T') ? 'A' : c;
}
__device__ __forceinline__ uint8_t gclass(char c) {
  return (c == 'A') ? kA : (c == 'C') ? kC : (c == 'G') ? kG : (c == 'T') ? kT : (c == '*') ? kStar : kN;
}
// get_genomic_nt (dynprog_single.c:116): Univcoord_T arithmetic, the int position sign-extended
__device__ __forceinline__ char genomic_nt(const uint32_t* __restrict__ blocks, uint64_t nwords, int genomicpos,
                                           uint64_t chroffset, uint64_t chrhigh, bool watson) {
  const uint64_t g = (uint64_t)(int64_t)genomicpos;
  const uint64_t pos = watson ? chroffset + g : chrhigh - g;
  if (pos < chroffset || pos >= chrhigh) return '*';
  const char c = decode_nt(blocks, nwords, pos);
  return watson ? c : compl_nt(c);
}
// Character i of Genome_get_segment_right(left=pos, L, chrhigh=bound) or
// Genome_get_segment_left(right=pos, L, chroffset=bound), optionally
// reverse-complemented (genome.c:11023-11135).
__device__ __forceinline__ char segment_nt(const uint32_t* __restrict__ blocks, uint64_t nwords, uint32_t i,
                                           uint32_t L, uint64_t pos, uint64_t bound, bool leftvariant,
                                           bool revcomp) {
  const uint64_t j = revcomp ? L - 1u - i : i;  // index into the forward segment
  char c;
  if (!leftvariant) {
    const uint64_t left = pos, chrhigh = bound;
    if (left >= chrhigh) return '*';
    if (left + L >= chrhigh && j + (left + L - chrhigh) >= L) return '*';
    c = decode_nt(blocks, nwords, left + j);
  } else {
    const uint64_t right = pos, chroffset = bound;
    if (right < chroffset) return '*';
    if (right < chroffset + L && j < chroffset + L - right) return '*';
    c = decode_nt(blocks, nwords, right - L + j);
  }
  return revcomp ? compl_nt(c) : c;
}

// ---- LDS carve (must match lds_bytes_dp on the host) ----
__host__ __device__ constexpr size_t align16(size_t x) { return (x + 15) & ~size_t(15); }
struct Carve {
  size_t sc, q, quc, gch, gcls, dirs, total;
};
__host__ __device__ inline Carve carve_dp(int rlength, int glength, int R, bool dirs_lds) {
  Carve cv;
  size_t off = 0;
  const size_t srow = (size_t)(rlength + 2);
  cv.sc = off;   off = align16(off + (size_t)kNClass * srow);  // int8 sc[class][row], rows 0..rlength+1
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
// bitoff: first bit of the problem's segment when a packed wave stores whole-wave ballots
template <int R, typename WORD = uint64_t>
__device__ __forceinline__ uint32_t dir_bit(const WORD* dirs, int c, int t, int k, int W, int bitoff = 0) {
  if (k < 0 || k >= W) return 0u;  // outside the band: cleared to DIAG (dynprog.c:498)
  const WORD m = dirs[((size_t)c * 4 + t) * R + (k % R)];
  return (uint32_t)(m >> (k / R + bitoff)) & 1u;
}

struct Tally {
  int score, nmatches, nmismatches, nopens, nindels, count;
  int lead;        // leading INDEL records (dropped by the end gaps)
  bool seen;       // a non-INDEL record has been emitted
};

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

struct Geo {  // coordinate transform of a problem (revp flips both axes)
  int roffset, goffset, sgn;
  __device__ int qpos(int r) const { return roffset + sgn * (r - 1); }
  __device__ int gpos(int c) const { return goffset + sgn * (c - 1); }
};

// Views of a problem's characters by DP row / column.  The kernels that stage them in LDS pass
// plain `const char*` arrays (row r at q[r]); the packed kernel reads the query from the HBM arena
// and derives genome characters from their classes, which keeps its LDS slot small.
struct QView {  // character of DP row r: p[step * (r - 1)]
  const char* p;
  int step;
  __device__ char operator[](int r) const { return p[step * (r - 1)]; }
};
struct GClassView {  // genome character of column c from its class (A C G T N *)
  const uint8_t* cls;
  __device__ char operator[](int c) const { return (char)((0x2A4E54474341ull >> (8u * cls[c])) & 0xffu); }
};

// Diagonal run: cells (r-j, c-j), j in [0, n)  (dynprog.c:1861-1915, traceback_nogaps)
template <typename QV, typename GV>
__device__ __forceinline__ void emit_diag(int lane, int r, int c, int n, const Geo& G, const QV& q, const QV& quc,
                                          const GV& gch, const uint8_t* __restrict__ cons, gmapdp_pair* out,
                                          Tally& t) {
  for (int base = 0; base < n; base += 64) {
    const int j = base + lane;
    const bool active = j < n;
    bool notstar = false, good = false, matchish = false, amb = false;
    int qp = 0, gp = 0;
    char c1 = 0, c2 = 0;
    if (active) {
      const int rr = r - j, cc = c - j;
      c1 = q[rr];
      const char c1u = quc[rr];
      c2 = gch[cc];
      notstar = c2 != '*';
      if (c1u == c2) {
        matchish = true;
      } else if (cons[(uint8_t)(c1u & 127) * kNClass + gclass(c2)]) {
        matchish = true;
        amb = true;
      }
      qp = G.qpos(rr);
      gp = G.gpos(cc);
      good = notstar && qp >= 0 && gp >= 0;
    }
    const uint64_t mgood = ballot(good);
    t.nmatches += __popcll(ballot(active && notstar && matchish));
    t.nmismatches += __popcll(ballot(active && notstar && !matchish));
    if (good) {
      put_pair(out, t.count + lanes_below(mgood, lane), qp, gp, 0, c1, matchish ? (amb ? ':' : '*') : ' ', c2, c2);
    }
    t.count += __popcll(mgood);
    if (mgood) t.seen = true;
  }
}

// Query skip: Pairpool_add_queryskip(pairs, rs, c, dist, ...) (pairpool.c:981): rows rs, rs-1, ...
template <typename QV>
__device__ __forceinline__ void emit_queryskip(int lane, int rs, int c, int dist, const Geo& G, const QV& q,
                                               gmapdp_pair* out, Tally& t) {
  const int gp = G.gpos(c);
  for (int base = 0; base < dist; base += 64) {
    const int j = base + lane;
    const bool active = j < dist;
    const int rr = rs - j;
    const int qp = G.qpos(rr);
    const bool good = active && qp >= 0 && gp >= 0;
    const uint64_t mgood = ballot(good);
    if (good) put_pair(out, t.count + lanes_below(mgood, lane), qp, gp, 0, q[rr], '-', ' ', ' ');
    const int nw = __popcll(mgood);
    t.count += nw;
    if (!t.seen) t.lead += nw;
  }
  t.score += kQopen + dist * kQindel;
  t.nopens += 1;
  t.nindels += dist;
}

// Genome skip: Pairpool_add_genomeskip(&add_dashes_p, pairs, r, cs, dist, NULL, ...) (pairpool.c:1068):
// columns cs, cs-1, ...; dist >= 9 gives one gap holder
__device__ __forceinline__ void emit_genomeskip(int lane, int r, int cs, int dist, const Geo& G, bool watson,
                                                uint64_t chroffset, uint64_t chrhigh, const uint32_t* blocks,
                                                uint64_t nwords, gmapdp_pair* out, Tally& t) {
  if (dist >= kMicrointronLength) {
    if (lane == 0) put_pair(out, t.count, -1, -1, dist, ' ', ' ', ' ', ' ');
    t.count += 1;
    t.seen = true;
    return;
  }
  const int qp = G.qpos(r);
  for (int base = 0; base < dist; base += 64) {
    const int j = base + lane;
    const bool active = j < dist;
    const int gp = G.gpos(cs - j);
    const bool good = active && qp >= 0 && gp >= 0;
    const uint64_t mgood = ballot(good);
    if (good) {
      const char c2 = genomic_nt(blocks, nwords, gp, chroffset, chrhigh, watson);
      put_pair(out, t.count + lanes_below(mgood, lane), qp, gp, 0, ' ', '-', c2, c2);
    }
    const int nw = __popcll(mgood);
    t.count += nw;
    if (!t.seen) t.lead += nw;
  }
  t.score += kTopen + dist * kTindel;
  t.nopens += 1;
  t.nindels += dist;
}

// 64-bit max across the wave (used once per problem for the best endpoint).
__device__ __forceinline__ uint64_t wave_max_u64(uint64_t x) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {
    const uint64_t y = __shfl_xor(x, off, 64);
    x = y > x ? y : x;
  }
  return x;
}
template <int S>
__device__ __forceinline__ uint64_t seg_max_u64(uint64_t x) {
#pragma unroll
  for (int off = S / 2; off >= 1; off >>= 1) {
    const uint64_t y = __shfl_xor(x, off, 64);
    x = y > x ? y : x;
  }
  return x;
}

// ---- banded fill (Dynprog_standard, upperp = lowerp = true, saturation NEG_INFINITY_INT) ----
// Rows r = c - uband + k, k = lane*R + i.  Writes the four direction ballots of every column to
// `dirs`; with CARRY also the Dynprog_genome_gap bridge candidates (BridgeCarry).  track: 0 none, 1 best endpoint over
// the whole band (find_best_endpoint_std), 2 best endpoint on row rlength (_to_queryend_indels_std).
// Bridge candidates of Dynprog_genome_gap carried along band rows during a fill
// (bridge_intron_gap_site_level, dynprog_genome.c:2736-2844).  A row's cells
// arrive column by column, and a row moves one band offset down per column --
// the path the E input already takes -- so each row's best candidate so far
// travels with it (DPP wave_shl:1) and is final when the row leaves the band.
// R fill ("B", indel on the right): row rR, other = rL = rlength - rR, candidate
//   cR: isc[leftdi[rL] & rightdi[cR]] + matrixR[cR][rR], probL[rL] + probR[cR].
// L fill ("C", indel on the left): row rL, other = rR, candidate cL:
//   matrixL[cL][rL] + isc[leftdi[cL] & rightdi[rR]], probL[cL] + probR[rR].
// A cell is a candidate when 1 <= r <= rlength-1, band offset k >= 1
// (c < r + uband), c <= glength-2 and c < (rev_goffsetR - goffsetL) - other;
// c >= r - lband holds inside the band.  Ties keep the earlier column.
struct BridgeCarry {
  const uint8_t* rowdi;   // dinucleotide code of the other side, indexed by `other`
  const uint8_t* coldi;   // dinucleotide code of this side, indexed by column
  const double* rowp;     // probability of the other side, indexed by `other`
  const double* colp;     // probability of this side, indexed by column
  const int8_t* isc;      // intron score array (64 entries)
  int rdist;              // rev_goffsetR - goffsetL
  struct Part* part;      // best candidate per row of this fill
  int* diag;              // matrix[r][r] per row
};
struct Part {
  double p;
  int s;
  int c;  // -1: no candidate
};

// S < 64: the wave holds 64/S problems, one per S-lane segment (R must be 1); every argument
// is then per segment, `gmax` is the wave's largest glength, the score rows are transposed
// (sc[r*8 + class], no per-column multiply) and lane 0 stores the whole-wave ballots (segment j
// owns bits [j*S, j*S+S) of each word).
// STORE: also write the stored score of every band cell, smat[c * W + k] (the `matrix` that
// Dynprog_cdna_gap's bridge reads at arbitrary cells).
// Direction words packed for a band of W <= 64 lanes (DPK, the genome-gap kernel's LDS planes): per column
// the low 32 bits of the four ballots (one 16-byte record, dirs[4c + t]) and, in a second region after all
// columns (hi = dirs + 4 (glen + 1)), the ballots' bits 32.. W-1: gg_dir_nhigh(W) words per column, plane t's
// bits from bit t * 8 * nhigh.  16 + 4 nhigh bytes per column instead of 32.
__host__ __device__ inline int gg_dir_nhigh(int W) { return W <= 32 ? 0 : W <= 40 ? 1 : W <= 48 ? 2 : 4; }
struct PackedDirs {
  const uint32_t* lo;
  const uint32_t* hi;
  int W, uband, nhigh;
  __device__ uint32_t operator()(int c, int t, int r) const {
    const int k = r - c + uband;
    if (k < 0 || k >= W) return 0u;  // outside the band: cleared to DIAG (dynprog.c:498)
    if (k < 32) return (lo[4 * c + t] >> k) & 1u;
    const int b = t * 8 * nhigh + (k - 32);
    return (hi[c * nhigh + (b >> 5)] >> (b & 31)) & 1u;
  }
};

// NB (whole-wave fills only): the band is narrower than the wave's 64 R elements, so the last lane's last
// element is never a valid cell and the E / H values shifted into it need no -infinity default.
template <int R, bool CARRY, int S = 64, bool PK = (S < 64), bool STORE = false, bool DPK = false, bool NB = false>
__device__ __forceinline__ void fill_band(int lane, int rlen, int glen, int lband, int uband, int open, int ext,
                                          int late, int track, const int8_t* sc, int srow, const uint8_t* gcl,
                                          uint64_t* dirs, const BridgeCarry* bc_, int& bestr, int& bestc,
                                          int gmax = 0, int* smat = nullptr, int* best_score = nullptr) {
  static_assert(S == 64 || (R == 1 && !CARRY), "segmented fills are single-word, no bridge carry");
  static_assert(!STORE || S == 64, "score matrices are stored by whole-wave fills only");
  static_assert(!DPK || (R == 1 && S == 64), "packed direction words: one-word bands");
  static_assert(!NB || S == 64, "narrow-band shifts: whole-wave fills");
  const int lk = (S == 64) ? lane : (lane & (S - 1));  // lane within the segment
  const int cend = (S == 64) ? glen : gmax;
  const int sat = kNegInf32;
  const int W = lband + uband + 1;
  const int binit = (track == 2) ? kNegInf32 : 0;
  int Hs[R], E[R], bv[R], bcol[R];
#pragma unroll
  for (int i = 0; i < R; i++) {  // column 0 (dynprog.c:1331-1369)
    const int k = lk * R + i;
    const int r = k - uband;
    int v = kNegInf32;
    if (k < W && r >= 0 && r <= rlen) v = (r == 0) ? 0 : (r <= lband ? open + r * ext : kNegInf32);
    Hs[i] = v;
    E[i] = kNegInf32;
    bv[i] = binit;
    bcol[i] = 0;
  }
  // Hs holds the stored nogap value (clamped at `sat`) except on band offset 0, whose only reader is
  // itself as the diagonal of the band-top row, which the reference takes unclamped (first_nogap).
  int kext[R];  // k*ext per element: r*ext = rtop*ext + k*ext without a per-column multiply
#pragma unroll
  for (int i = 0; i < R; i++) kext[i] = (lk * R + i) * ext;
  // carried bridge candidate per band row: score, column + 1 (0: none), probability -- zero-filled shifts
  int cs[R], cc[R];
  double cp[R];
#pragma unroll
  for (int i = 0; i < R; i++) {
    cs[i] = 0;
    cc[i] = 0;
    cp[i] = 0.0;
  }
  // The genome-gap fills (CARRY: packed score rows in LDS) keep the row clamp and the table's LDS address in
  // VGPRs: as scalars they were among the kernel's spilled SGPRs, reloaded by v_readlane every column.
  int rlen1 = rlen + 1;
  uint32_t scb = 0;
  if constexpr (CARRY && PK) {
    scb = (uint32_t)(size_t)(const __attribute__((address_space(3))) int32_t*)reinterpret_cast<const int32_t*>(sc);
    asm volatile("" : "+v"(rlen1), "+v"(scb));
  }
  int rtop_ext = -uband * ext;  // (c - uband) * ext, advanced by ext per column
  int oce = open;               // open + c * ext
  int gi_next = (S == 64) ? 0 : gcl[min(1, glen)];
  for (int c = 1; c <= cend; c++) {
    const bool colact = (S == 64) || (c <= glen);
    // genome class: wave-uniform (SGPR) for one problem per wave; per segment otherwise, read one
    // column ahead so the LDS latency is off the column's dependency chain
    int gi;
    if constexpr (S == 64) {
      gi = __builtin_amdgcn_readfirstlane(gcl[c]);
    } else {
      gi = gi_next;
      gi_next = gcl[min(c + 1, glen)];
    }
    const int rtop = c - uband;
    const int rlo = rtop < 1 ? 1 : rtop;
    const int rhigh = (c + lband) < rlen ? (c + lband) : rlen;
    rtop_ext += ext;
    oce += ext;
    // last_nogap entering row rlo (dynprog.c:1411-1449)
    const int L0 = (c == 1) ? (kNegInf32 - open + 1) : (c <= uband ? oce : kNegInf32);
    const int row0 = (c <= uband) ? oce : kNegInf32;  // row 0 of this column (dynprog.c:1318-1325)
    const int8_t* scg = PK ? sc : sc + gi * srow;
    const int gi4 = gi << 2;  // packed: bit offset of the class in the row's score word

    int Ein[R], Hin[R];
#pragma unroll
    for (int i = 0; i < R - 1; i++) { Ein[i] = E[i + 1]; Hin[i] = Hs[i + 1]; }
    if constexpr (NB) {  // (lane 63's element R-1 lies outside the band: whatever arrives there is unread)
      Ein[R - 1] = dpp_wave_shl1_zero(E[0]);
      Hin[R - 1] = dpp_wave_shl1_zero(Hs[0]);
    } else {
      Ein[R - 1] = seg_shl1<S>(E[0], kNegInf32, lk);
      Hin[R - 1] = seg_shl1<S>(Hs[0], kNegInf32, lk);
    }

    int Hp[R], En[R], A[R];
    bool valid[R], eb[R], hb[R];
#pragma unroll
    for (int i = 0; i < R; i++) {
      const int k = lk * R + i;
      const int r = rtop + k;
      valid[i] = (k < W) & (r >= rlo) & (r <= rhigh) & colact;
      // (rows outside [0, rlen + 1] are invalid cells: unsigned, a negative row clamps to rlen + 1)
      const int rr = (int)min((unsigned)r, (unsigned)rlen1);
      int s;
      if constexpr (!PK) s = scg[rr];
      else if constexpr (CARRY)
        s = __builtin_amdgcn_sbfe(*(const __attribute__((address_space(3))) int32_t*)(size_t)(scb + 4u * (uint32_t)rr),
                                  gi4, 4);
      else s = __builtin_amdgcn_sbfe(reinterpret_cast<const int32_t*>(sc)[rr], gi4, 4);
      // Egap (dynprog.c:1518-1524)
      const int es = Hin[i] + open;
      eb[i] = Ein[i] > es - late;
      En[i] = max(Ein[i], es) + ext;
      const int dg = Hs[i] + s;
      hb[i] = En[i] > dg - late;
      Hp[i] = max(En[i], dg);
      A[i] = valid[i] ? Hp[i] + open - rtop_ext - kext[i] : kSent;
    }
    // F chain: F(r) = r*ext + max(init, max_{rlo<=j<r} (H'(j) + open - j*ext))
    int pre[R];
    pre[0] = A[0];
#pragma unroll
    for (int i = 1; i < R; i++) pre[i] = max(pre[i - 1], A[i]);
    const int X = seg_shr1<S>(seg_scan_max<S>(pre[R - 1]), kSent, lk);
    const int init = max(kNegInf32, L0 + open) - ((rtop > 1) ? rtop_ext - ext : 0);  // (rlo - 1) * ext
    int F[R], Hun[R];
    bool vb[R];
#pragma unroll
    for (int i = 0; i < R; i++) {
      const int ex = (i == 0) ? X : max(X, pre[i - 1]);
      F[i] = rtop_ext + kext[i] + max(init, ex);
      vb[i] = F[i] > Hp[i] - late;
      Hun[i] = max(F[i], Hp[i]);
    }
    // Fgap direction needs F(r-1), H(r-1) of this column (dynprog.c:1486-1492).  Lane 0's element 0 reads
    // them only when valid, and then it is the column's top row (r = rtop = rlo), which takes the constants
    // below instead: a whole-wave fill shifts in zeros there (one DPP move, no default copied in first).
    int Fup, Hup;
    if constexpr (S == 64) {
      Fup = dpp_wave_shr1_zero(F[R - 1]);
      Hup = dpp_wave_shr1_zero(Hun[R - 1]);
    } else {
      Fup = seg_shr1<S>(F[R - 1], kNegInf32, lk);
      Hup = seg_shr1<S>(Hun[R - 1], kNegInf32, lk);
    }
    uint64_t mH[R], mV[R], mE[R], mF[R];
#pragma unroll
    for (int i = 0; i < R; i++) {
      const int k = lk * R + i;
      const int r = rtop + k;
      const bool top = r == rlo;
      const int fprev = top ? kNegInf32 : ((i == 0) ? Fup : F[i - 1]);
      const int hprev = top ? L0 : ((i == 0) ? Hup : Hun[i - 1]);
      const bool fb = fprev > hprev + open - late;
      const uint64_t mvalid = ballot(valid[i]);
      mV[i] = ballot(vb[i]) & mvalid;
      mH[i] = ballot(hb[i]) & ~mV[i] & mvalid;
      mE[i] = ballot(eb[i]) & mvalid;
      mF[i] = ballot(fb) & mvalid;
      const int Hc = max(Hun[i], sat);
      if (STORE && valid[i]) smat[(size_t)c * W + k] = Hc;
      // branch-free state update for the next column
      Hs[i] = valid[i] ? ((k == 0) ? Hun[i] : Hc) : ((r == 0) ? row0 : kNegInf32);
      E[i] = valid[i] ? En[i] : kNegInf32;
      // best endpoint (find_best_endpoint_std / _to_queryend_indels_std): scan-order first/last max
      const bool cand = valid[i] & ((track == 1) | ((track == 2) & (r == rlen))) & (Hc > bv[i] - late);
      bv[i] = cand ? Hc : bv[i];
      bcol[i] = cand ? c : bcol[i];
    }
    if (CARRY) {
      const BridgeCarry& B = *bc_;
      const int cdi = __builtin_amdgcn_readfirstlane(B.coldi[c]);
      const double cpc = B.colp[c];
      // carried values arrive from band offset k+1 of the previous column
      int ics[R], icc[R];
      double icp[R];
#pragma unroll
      for (int i = 0; i < R - 1; i++) { ics[i] = cs[i + 1]; icc[i] = cc[i + 1]; icp[i] = cp[i + 1]; }
      ics[R - 1] = dpp_wave_shl1_zero(cs[0]);
      icc[R - 1] = dpp_wave_shl1_zero(cc[0]);
      {
        const int2 v = *reinterpret_cast<const int2*>(&cp[0]);
        int2 w;
        w.x = dpp_wave_shl1_zero(v.x);
        w.y = dpp_wave_shl1_zero(v.y);
        icp[R - 1] = *reinterpret_cast<const double*>(&w);
      }
#pragma unroll
      for (int i = 0; i < R; i++) {
        const int k = lk * R + i;
        const int r = rtop + k;
        const int other = rlen - r;
        const bool inrow = (r >= 1) & (r <= rlen - 1) & (k < W);
        const bool cand = inrow & (k >= 1) & valid[i] & (c <= glen - 2) & (c < B.rdist - other);
        const int Hc = max(Hun[i], sat);
        int s = 0;
        double p = 0.0;
        if (cand) {
          s = B.isc[B.rowdi[other] & cdi] + Hc;
          p = B.rowp[other] + cpc;
        }
        const bool take = cand & ((icc[i] == 0) | (s > ics[i]) | ((s == ics[i]) & (p > icp[i])));
        cs[i] = take ? s : ics[i];
        cc[i] = take ? c + 1 : icc[i];
        cp[i] = take ? p : icp[i];
        if (inrow && k == uband) B.diag[r] = Hc;  // matrix[r][r]
        if (inrow && k == 0) {                    // the row leaves the band: its candidate is final
          B.part[r].s = cs[i];
          B.part[r].c = cc[i] - 1;
          B.part[r].p = cp[i];
        }
      }
    }
#ifdef GMAPDP_GGX_NODIRS
    if (!CARRY)  // timing experiment only (make variant): the genome-gap fills store no directions
#endif
    if constexpr (DPK) {
      if (lane == 0) {
        uint32_t* lo = reinterpret_cast<uint32_t*>(dirs);
        *reinterpret_cast<uint4*>(lo + 4 * c) = make_uint4((uint32_t)mH[0], (uint32_t)mV[0], (uint32_t)mE[0], (uint32_t)mF[0]);
        const int nh = gg_dir_nhigh(W);
        uint32_t* hi = lo + 4 * (glen + 1) + nh * c;
        const uint32_t h0 = (uint32_t)(mH[0] >> 32), h1 = (uint32_t)(mV[0] >> 32), h2 = (uint32_t)(mE[0] >> 32),
                       h3 = (uint32_t)(mF[0] >> 32);
        if (nh == 1) {
          hi[0] = (h0 & 0xffu) | ((h1 & 0xffu) << 8) | ((h2 & 0xffu) << 16) | (h3 << 24);
        } else if (nh == 2) {
          *reinterpret_cast<uint2*>(hi) = make_uint2((h0 & 0xffffu) | (h1 << 16), (h2 & 0xffffu) | (h3 << 16));
        } else if (nh == 4) {
          *reinterpret_cast<uint4*>(hi) = make_uint4(h0, h1, h2, h3);
        }
      }
    } else
    if (lane == 0) {  // one lane stores the column's 4R direction words
      uint64_t* dcol = dirs + (size_t)c * 4 * R;
#pragma unroll
      for (int i = 0; i < R; i++) {
        dcol[0 * R + i] = mH[i];
        dcol[1 * R + i] = mV[i];
        dcol[2 * R + i] = mE[i];
        dcol[3 * R + i] = mF[i];
      }
    }
  }
  if (CARRY) {  // rows still inside the band after the last column
    const BridgeCarry& B = *bc_;
#pragma unroll
    for (int i = 0; i < R; i++) {
      const int k = lk * R + i;
      const int r = glen - uband + k;
      if (k < W && r >= 1 && r <= rlen - 1) {
        B.part[r].s = cs[i];
        B.part[r].c = cc[i] - 1;
        B.part[r].p = cp[i];
      }
    }
  }
  if (track) {
    // reduce the endpoint over the wave: key orders (score, r, c) so that the max key is the
    // reference's choice (> keeps the first in r-major scan order, >= the last)
    uint64_t key = 0;
#pragma unroll
    for (int i = 0; i < R; i++) {
      if (bcol[i] > 0) {
        const int r = bcol[i] - uband + lk * R + i;
        const uint32_t rk = late ? (uint32_t)r : 4095u - (uint32_t)r;
        const uint32_t ck = late ? (uint32_t)bcol[i] : 4095u - (uint32_t)bcol[i];
        const uint64_t kk = ((uint64_t)(uint32_t)(bv[i] + (1 << 30)) << 24) | ((uint64_t)rk << 12) | ck;
        key = kk > key ? kk : key;
      }
    }
    key = seg_max_u64<S>(key);
    // the endpoint's score (find_best_endpoint_to_queryend_indels_std's *finalscore; NEG_INFINITY_32
    // when no cell of the scanned row beat the initial value)
    if (best_score) *best_score = key ? (int)(uint32_t)(key >> 24) - (1 << 30) : kNegInf32;
    if (key == 0) {
      bestr = (track == 2) ? rlen : 0;
      bestc = 0;
    } else {
      const uint32_t rk = (uint32_t)(key >> 12) & 4095u, ck = (uint32_t)key & 4095u;
      bestr = late ? (int)rk : 4095 - (int)rk;
      bestc = late ? (int)ck : 4095 - (int)ck;
    }
  } else {
    bestr = rlen;
    bestc = glen;
  }
}

// ---- row-major fill: the same recurrence with lanes over query rows ----
// For a band much wider than the query (a short query against a long genome segment: the stage-3
// single gaps across ~2000-nt genomic gaps), the band layout above spends R = W/64 words per lane on
// a column that holds at most rlength + 1 live cells.  Here lane L owns rows r = L*R + i
// (64*R >= rlength + 1), so a column costs R words however wide the band is.  The inputs swap
// places: the horizontal (E) input is the same register one column back, the diagonal one is row
// r - 1 (the register below, or DPP wave_shr:1 from the previous lane); the F chain is the same
// max-plus scan.  Cells outside the band (k = r - c + uband outside [0, W)) are not computed and
// read back as NEG_INFINITY, exactly as the band layout's edges.  Direction words: bit r / R of
// word r % R (RowDirs).  No bridge carry, no stored scores (single and end gaps only).
template <int R>
__device__ __forceinline__ void fill_rows(int lane, int rlen, int glen, int lband, int uband, int open, int ext,
                                          int late, int track, const int8_t* sc, int srow, const uint8_t* gcl,
                                          uint64_t* dirs, int& bestr, int& bestc) {
  const int sat = kNegInf32;
  const int binit = (track == 2) ? kNegInf32 : 0;
  int Hs[R], E[R], bv[R], bcol[R], rext[R];
#pragma unroll
  for (int i = 0; i < R; i++) {  // column 0 (dynprog.c:1331-1369)
    const int r = lane * R + i;
    int v = kNegInf32;
    if (r <= rlen) v = (r == 0) ? 0 : (r <= lband ? open + r * ext : kNegInf32);
    Hs[i] = v;
    E[i] = kNegInf32;
    bv[i] = binit;
    bcol[i] = 0;
    rext[i] = r * ext;
  }
  int rtop_ext = -uband * ext;  // (c - uband) * ext
  int oce = open;               // open + c * ext
  for (int c = 1; c <= glen; c++) {
    const int gi = __builtin_amdgcn_readfirstlane(gcl[c]);
    const int rtop = c - uband;
    const int rlo = rtop < 1 ? 1 : rtop;
    const int rhigh = (c + lband) < rlen ? (c + lband) : rlen;
    rtop_ext += ext;
    oce += ext;
    const int L0 = (c == 1) ? (kNegInf32 - open + 1) : (c <= uband ? oce : kNegInf32);
    const int row0 = (c <= uband) ? oce : kNegInf32;
    const int8_t* scg = sc + gi * srow;
    // diagonal input: row r - 1, previous column
    int Hd[R];
    Hd[0] = dpp_wave_shr1(Hs[R - 1], kNegInf32);
#pragma unroll
    for (int i = 1; i < R; i++) Hd[i] = Hs[i - 1];
    int Hp[R], En[R], A[R];
    bool valid[R], eb[R], hb[R];
#pragma unroll
    for (int i = 0; i < R; i++) {
      const int r = lane * R + i;
      valid[i] = (r >= rlo) & (r <= rhigh);
      const int s = scg[min(r, rlen + 1)];
      const int es = Hs[i] + open;  // Egap from the same row (dynprog.c:1518-1524)
      eb[i] = E[i] > es - late;
      En[i] = max(E[i], es) + ext;
      const int dg = Hd[i] + s;
      hb[i] = En[i] > dg - late;
      Hp[i] = max(En[i], dg);
      A[i] = valid[i] ? Hp[i] + open - rext[i] : kSent;
    }
    int pre[R];
    pre[0] = A[0];
#pragma unroll
    for (int i = 1; i < R; i++) pre[i] = max(pre[i - 1], A[i]);
    const int X = dpp_wave_shr1(wave_scan_max(pre[R - 1]), kSent);
    const int init = max(kNegInf32, L0 + open) - ((rtop > 1) ? rtop_ext - ext : 0);  // (rlo - 1) * ext
    int F[R], Hun[R];
    bool vb[R];
#pragma unroll
    for (int i = 0; i < R; i++) {
      const int ex = (i == 0) ? X : max(X, pre[i - 1]);
      F[i] = rext[i] + max(init, ex);
      vb[i] = F[i] > Hp[i] - late;
      Hun[i] = max(F[i], Hp[i]);
    }
    const int Fup = dpp_wave_shr1(F[R - 1], kNegInf32);
    const int Hup = dpp_wave_shr1(Hun[R - 1], kNegInf32);
    uint64_t mH[R], mV[R], mE[R], mF[R];
#pragma unroll
    for (int i = 0; i < R; i++) {
      const int r = lane * R + i;
      const bool top = r == rlo;
      const int fprev = top ? kNegInf32 : ((i == 0) ? Fup : F[i - 1]);
      const int hprev = top ? L0 : ((i == 0) ? Hup : Hun[i - 1]);
      const bool fb = fprev > hprev + open - late;
      const uint64_t mvalid = ballot(valid[i]);
      mV[i] = ballot(vb[i]) & mvalid;
      mH[i] = ballot(hb[i]) & ~mV[i] & mvalid;
      mE[i] = ballot(eb[i]) & mvalid;
      mF[i] = ballot(fb) & mvalid;
      const int Hc = max(Hun[i], sat);
      // band offset 0 keeps its unclamped value: its only reader is the next band-top cell's diagonal
      Hs[i] = valid[i] ? ((r == rtop) ? Hun[i] : Hc) : ((r == 0) ? row0 : kNegInf32);
      E[i] = valid[i] ? En[i] : kNegInf32;
      const bool cand = valid[i] & ((track == 1) | ((track == 2) & (r == rlen))) & (Hc > bv[i] - late);
      bv[i] = cand ? Hc : bv[i];
      bcol[i] = cand ? c : bcol[i];
    }
    if (lane == 0) {
      uint64_t* dcol = dirs + (size_t)c * 4 * R;
#pragma unroll
      for (int i = 0; i < R; i++) {
        dcol[0 * R + i] = mH[i];
        dcol[1 * R + i] = mV[i];
        dcol[2 * R + i] = mE[i];
        dcol[3 * R + i] = mF[i];
      }
    }
  }
  if (track) {  // as fill_band: the max (score, r, c) key is the reference's scan-order choice
    uint64_t key = 0;
#pragma unroll
    for (int i = 0; i < R; i++) {
      if (bcol[i] > 0) {
        const int r = lane * R + i;
        const uint32_t rk = late ? (uint32_t)r : 4095u - (uint32_t)r;
        const uint32_t ck = late ? (uint32_t)bcol[i] : 4095u - (uint32_t)bcol[i];
        const uint64_t kk = ((uint64_t)(uint32_t)(bv[i] + (1 << 30)) << 24) | ((uint64_t)rk << 12) | ck;
        key = kk > key ? kk : key;
      }
    }
    key = wave_max_u64(key);
    if (key == 0) {
      bestr = (track == 2) ? rlen : 0;
      bestc = 0;
    } else {
      const uint32_t rk = (uint32_t)(key >> 12) & 4095u, ck = (uint32_t)key & 4095u;
      bestr = late ? (int)rk : 4095 - (int)rk;
      bestc = late ? (int)ck : 4095 - (int)ck;
    }
  } else {
    bestr = rlen;
    bestc = glen;
  }
}

// direction bits of fill_rows: row r in word r % R at bit r / R; cells outside the band read DIAG
template <int R>
struct RowDirs {
  const uint64_t* dirs;
  int W, uband;
  __device__ uint32_t operator()(int c, int t, int r) const {
    const int k = r - c + uband;
    if (k < 0 || k >= W || r < 0) return 0u;
    return (uint32_t)(dirs[((size_t)c * 4 + t) * R + (r % R)] >> (r / R)) & 1u;
  }
};

// ---- wave-cooperative traceback (Dynprog_traceback_std, dynprog.c:1796-1948) ----
// Emits the reference's push order into out[t.count ...].  `dir(c, t, r)` is the direction bit
// t (0 nogap=HORIZ, 1 nogap=VERT, 2 Egap=HORIZ, 3 Fgap=VERT) of cell (r, c), 0 (DIAG) for
// cells the fill did not write.  Dynprog_traceback_8/_16 (dynprog_simd.c:9154/9553) walk the
// same way, so the SIMD-semantics kernel shares this with its own direction layout.
template <typename DA, typename QV, typename GV>
__device__ __forceinline__ void traceback_walk(int lane, const DA& dir, int r, int c, const Geo& G, const QV& q,
                                               const QV& quc, const GV& gch, const uint8_t* __restrict__ cons,
                                               bool watson, uint64_t chroffset, uint64_t chrhigh,
                                               const uint32_t* __restrict__ blocks, uint64_t nwords,
                                               gmapdp_pair* out, Tally& t, int mode = 0) {
  while (r > 0 && c > 0) {
    const uint32_t isV = dir(c, 1, r);
    const uint32_t isH = dir(c, 0, r);
    if (!isV && isH) {
      // E chain along row r: columns c, c-1, ... while Egap == HORIZ
      int n = 0;
      for (int base = 0;; base += 64) {
        const int j = base + lane;
        const bool cont = (c - j >= 1) && dir(c - j, 2, r);
        const uint64_t stop = ~ballot(cont);
        if (stop) { n = base + __ffsll((long long)stop) - 1; break; }
      }
      const int dist = n + 1;
      const int c_end = (c - n - 1) > 0 ? (c - n - 1) : 0;
      emit_genomeskip(lane, r, c_end + dist, dist, G, watson, chroffset, chrhigh, blocks, nwords, out, t);
      c = c_end;
    } else if (isV) {
      // F chain up column c: rows r, r-1, ... while Fgap == VERT
      int n = 0;
      for (int base = 0;; base += 64) {
        const int j = base + lane;
        const bool cont = (r - j >= 1) && dir(c, 3, r - j);
        const uint64_t stop = ~ballot(cont);
        if (stop) { n = base + __ffsll((long long)stop) - 1; break; }
      }
      const int dist = n + 1;
      const int r_end = (r - n - 1) > 0 ? (r - n - 1) : 0;
      emit_queryskip(lane, r_end + dist, c, dist, G, q, out, t);
      r = r_end;
    } else {
      // diagonal run
      int n = 0;
      for (int base = 0;; base += 64) {
        const int j = base + lane;
        const bool inrange = (c - j >= 1) && (r - j >= 1);
        const bool cont = (j == 0) || (inrange && !dir(c - j, 0, r - j) && !dir(c - j, 1, r - j));
        const uint64_t stop = ~ballot(cont && inrange);
        if (stop) { n = base + __ffsll((long long)stop) - 1; break; }
      }
      emit_diag(lane, r, c, n, G, q, quc, gch, cons, out, t);
      r -= n;
      c -= n;
    }
  }
  // mode 1/2: Dynprog_traceback_{8,16}_upper / _lower (dynprog_simd.c:9415-9433 / 9530-9546) end
  // with a genome skip of c (upper) or a query skip of r (lower) whatever the other coordinate
  if ((r == 0 && c == 0) || (mode == 1 && c == 0) || (mode == 2 && r == 0)) {
  } else if (mode == 2 || (mode == 0 && c == 0)) {
    emit_queryskip(lane, r, 1, r, G, q, out, t);  // LAZY_INDEL
  } else {
    emit_genomeskip(lane, 1, c, c, G, watson, chroffset, chrhigh, blocks, nwords, out, t);
  }
}

// direction bits of the banded fills: band offset k = r - c + uband (dir_bit)
template <int R, typename WORD>
struct BandDirs {
  const WORD* dirs;
  int W, uband, bitoff;
  __device__ uint32_t operator()(int c, int t, int r) const {
    return dir_bit<R, WORD>(dirs, c, t, r - c + uband, W, bitoff);
  }
};

template <int R, typename WORD = uint64_t, typename QV = const char*, typename GV = const char*>
__device__ __forceinline__ void traceback_band(int lane, const WORD* dirs, int W, int uband, int r, int c,
                                               const Geo& G, const QV& q, const QV& quc, const GV& gch,
                                               const uint8_t* __restrict__ cons, bool watson, uint64_t chroffset,
                                               uint64_t chrhigh, const uint32_t* __restrict__ blocks,
                                               uint64_t nwords, gmapdp_pair* out, Tally& t, int bitoff = 0) {
  const BandDirs<R, WORD> d{dirs, W, uband, bitoff};
  traceback_walk(lane, d, r, c, G, q, quc, gch, cons, watson, chroffset, chrhigh, blocks, nwords, out, t);
}

// Genome skip whose characters come from the problem's own genome string (Pairpool_add_genomeskip with a
// genomesequence, pairpool.c:1145-1154): column cc's character is gch[cc].
template <typename GV>
__device__ __forceinline__ void emit_genomeskip_seq(int lane, int r, int cs, int dist, const Geo& G, const GV& gch,
                                                    gmapdp_pair* out, Tally& t) {
  if (dist >= kMicrointronLength) {
    if (lane == 0) put_pair(out, t.count, -1, -1, dist, ' ', ' ', ' ', ' ');
    t.count += 1;
    t.seen = true;
    return;
  }
  const int qp = G.qpos(r);
  for (int base = 0; base < dist; base += 64) {
    const int j = base + lane;
    const bool active = j < dist;
    const int gp = G.gpos(cs - j);
    const bool good = active && qp >= 0 && gp >= 0;
    const uint64_t mgood = ballot(good);
    if (good) {
      const char c2 = gch[cs - j];
      put_pair(out, t.count + lanes_below(mgood, lane), qp, gp, 0, ' ', '-', c2, c2);
    }
    const int nw = __popcll(mgood);
    t.count += nw;
    if (!t.seen) t.lead += nw;
  }
  t.score += kTopen + dist * kTindel;
  t.nopens += 1;
  t.nindels += dist;
}

// ---- traceback_local_std (dynprog_end.c:1138-1289) ----
// The splice-junction end gaps trace back in two pieces: from the endpoint until the column reaches
// `endc` (the far exon's piece of the junction string), then -- after the caller's gap holder -- on
// to column 0.  Differences from Dynprog_traceback_std that this restates:
//  * a gap step is taken at the start cell and after every diagonal step, whatever `endc` is (so an
//    E chain may cross `endc`), and the walk continues only while r > 0 and c > endc;
//  * the boundary cells are walked too: row 0 (nogap = HORIZ for c <= uband, dynprog.c:1304-1309)
//    is a genome skip to column 0, column 0 (nogap = VERT for r <= lband) a query skip to row 0;
//    outside the band they are DIAG (Directions32_alloc clears them, dynprog.c:497);
//  * genome skips take their characters from the genome string.
// Every walk here is wave-cooperative as in traceback_walk: a run is found with one ballot over 64
// candidate cells.
template <typename DA, typename QV, typename GV>
__device__ __forceinline__ void traceback_local(int lane, const DA& dir, int& r, int& c, int endc, int lband,
                                                int uband, const Geo& G, const QV& q, const QV& quc, const GV& gch,
                                                const uint8_t* __restrict__ cons, gmapdp_pair* out, Tally& t) {
  auto gap = [&]() {
    if (r == 0) {
      if (c <= uband) {
        emit_genomeskip_seq(lane, 0, c, c, G, gch, out, t);
        c = 0;
      }
      return;
    }
    if (c == 0) {
      if (r <= lband) {
        emit_queryskip(lane, r, 0, r, G, q, out, t);
        r = 0;
      }
      return;
    }
    const uint32_t isV = dir(c, 1, r);
    const uint32_t isH = dir(c, 0, r);
    if (!isV && isH) {
      int n = 0;
      for (int base = 0;; base += 64) {
        const int j = base + lane;
        const bool cont = (c - j >= 1) && dir(c - j, 2, r);
        const uint64_t stop = ~ballot(cont);
        if (stop) { n = base + __ffsll((long long)stop) - 1; break; }
      }
      const int dist = n + 1;
      const int c_end = (c - n - 1) > 0 ? (c - n - 1) : 0;
      emit_genomeskip_seq(lane, r, c_end + dist, dist, G, gch, out, t);
      c = c_end;
    } else if (isV) {
      int n = 0;
      for (int base = 0;; base += 64) {
        const int j = base + lane;
        const bool cont = (r - j >= 1) && dir(c, 3, r - j);
        const uint64_t stop = ~ballot(cont);
        if (stop) { n = base + __ffsll((long long)stop) - 1; break; }
      }
      const int dist = n + 1;
      const int r_end = (r - n - 1) > 0 ? (r - n - 1) : 0;
      emit_queryskip(lane, r_end + dist, c, dist, G, q, out, t);
      r = r_end;
    }
  };
  if (c > endc) gap();
  while (r > 0 && c > endc) {
    // diagonal run: the walk goes on from cell j >= 1 while it is inside (r > 0, c > endc) and DIAG
    int n = 0;
    for (int base = 0;; base += 64) {
      const int j = base + lane;
      const bool cont = (j == 0) || ((r - j >= 1) && (c - j > endc) && !dir(c - j, 0, r - j) && !dir(c - j, 1, r - j));
      const uint64_t stop = ~ballot(cont);
      if (stop) { n = base + __ffsll((long long)stop) - 1; break; }
    }
    emit_diag(lane, r, c, n, G, q, quc, gch, cons, out, t);
    r -= n;
    c -= n;
    if (!(r == 0 && c == 0)) gap();
  }
}

// reverse out[0..n) in place (List_reverse of an already emitted run)
__device__ __forceinline__ void reverse_records(int lane, gmapdp_pair* out, int n) {
  __threadfence_block();
  int4* recs = reinterpret_cast<int4*>(out);
  for (int a = lane; a < n / 2; a += 64) {
    const int b = n - 1 - a;
    const int4 x = recs[a], y = recs[b];
    recs[a] = y;
    recs[b] = x;
  }
  __threadfence_block();
}


// Pair emission of one problem after its fill (the tail of dp_kernel): traceback or the
// simple/no-gap diagonal, end-gap INDEL trimming and end5 reversal, the result record.
template <typename DA, typename QV, typename GV>
__device__ __forceinline__ void finish_dp(int lane, const DevProblem& P, int pid, bool simple, int bestr, int bestc,
                                          const DA& dir, const QV& q, const QV& quc, const GV& gch,
                                          const uint8_t* __restrict__ constab, const uint32_t* __restrict__ blocks,
                                          uint64_t nwords, gmapdp_result* __restrict__ results,
                                          gmapdp_pair* __restrict__ pairs, int mode = 0) {
  const int rlen = P.rlength, flags = P.flags, kind = P.kind, endalign = P.endalign;
  const bool rev = flags & kFRev;
  const bool is_end = kind != kSingle;
  const uint8_t* cons = constab + (size_t)P.genestrand * 128 * kNClass;
  gmapdp_pair* out = pairs + P.pair_offset;
  const Geo G{P.roffset, P.goffset, rev ? -1 : 1};
  const int dpi_next = P.dynprogindex + (P.dynprogindex > 0 ? 1 : -1);
  Tally t = {0, 0, 0, 0, 0, 0, 0, false};
#ifdef GMAPDP_EXPERIMENT_NO_EMIT
  if (lane == 0) results[pid].npairs = 0;  // timing experiment only: fills without the emission phase
  return;
#endif
  if (simple) {
    // single_gap_simple: pushes r = 1..rlength without List_reverse: list order r = rlength .. 1
    emit_diag(lane, rlen, rlen, rlen, G, q, quc, gch, cons, out, t);
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
  const bool skip = is_end && endalign != kQueryendNogaps && (flags & kFRequirePos);
  if (is_end && endalign == kQueryendNogaps) {
    emit_diag(lane, bestr, bestc, bestr, G, q, quc, gch, cons, out, t);  // traceback_nogaps
  } else if (!skip) {
    traceback_walk(lane, dir, bestr, bestc, G, q, quc, gch, cons, flags & kFWatson, P.chroffset, P.chrhigh, blocks,
                   nwords, out, t, mode);
  }
  int score = t.score + t.nmatches * kMatch + t.nmismatches * kMismatch;
  int first = 0, npairs = t.count;
  if (is_end) {
    if ((endalign == kQueryendGap || endalign == kBestLocal) && (t.nmatches + 1) < t.nmismatches) {
      score = 0;  // dynprog_end.c:1623-1626: list dropped, counters kept
      npairs = 0;
    } else {
      first = t.lead;  // INDEL pairs at the far end removed (dynprog_end.c:1629-1632)
      npairs = t.count - t.lead;
      if (kind == kEnd5 && npairs > 1) reverse_records(lane, out + first, npairs);  // dynprog_end.c:1646
    }
  }
  if (lane == 0) {
    gmapdp_result res;
    res.npairs = npairs;
    res.pair_offset = P.pair_offset + first;
    res.traceback_score = score;
    res.nmatches = t.nmatches;
    res.nmismatches = t.nmismatches;
    res.nopens = t.nopens;
    res.nindels = t.nindels;
    res.dynprogindex = dpi_next;
    results[pid] = res;
  }
}


__device__ __forceinline__ int sat_add(int a, int b, int lo, int hi) { return min(max(a + b, lo), hi); }

// intron.h dinucleotide codes; the engine's genome has no alternate alleles (alt == ref)
__device__ __forceinline__ uint8_t left_dinucl(char a, char b) {
  if (a == 'G' && b == 'T') return 0x21;  // LEFT_GT
  if (a == 'G' && b == 'C') return 0x10;  // LEFT_GC
  if (a == 'A' && b == 'T') return 0x08;  // LEFT_AT
  if (a == 'C' && b == 'T') return 0x06;  // LEFT_CT
  return 0;
}
__device__ __forceinline__ uint8_t right_dinucl(char right2, char right1) {
  if (right2 == 'A' && right1 == 'G') return 0x30;  // RIGHT_AG
  if (right2 == 'A' && right1 == 'C') return 0x0C;  // RIGHT_AC
  if (right2 == 'G' && right1 == 'C') return 0x02;  // RIGHT_GC
  if (right2 == 'A' && right1 == 'T') return 0x01;  // RIGHT_AT
  return 0;
}

// inclusive prefix sum / max across the wave
__device__ __forceinline__ int wave_scan_add(int lane, int x) {
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const int y = __shfl_up(x, off, 64);
    if (lane >= off) x += y;
  }
  return x;
}
__device__ __forceinline__ int wave_scan_maxi(int lane, int x) {
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const int y = __shfl_up(x, off, 64);
    if (lane >= off) x = max(x, y);
  }
  return x;
}
__device__ __forceinline__ int wave_min_i(int x) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) x = min(x, __shfl_xor(x, off, 64));
  return x;
}

// Pair_maxnegscore (pair.c:8528) of the list held in out[0..n) in REVERSE order (it is evaluated
// before Dynprog_genome_gap's final List_reverse).  Running score: match +1, mismatch -3, an
// INDEL run -3 -1 per record; prevhigh = max(0, running max); minimum of score - prevhigh after
// every mismatch and INDEL record.
__device__ inline int wave_maxnegscore(int lane, const gmapdp_pair* out, int n) {
  int carry = 0, high = 0, worst = 0;
  bool prev_indel = false;
  const int4* recs = reinterpret_cast<const int4*>(out);
  for (int base = 0; base < n; base += 64) {
    const int p = base + lane;
    int delta = 0;
    bool eval = false, indel = false;
    if (p < n) {
      const int4 rec = recs[n - 1 - p];
      const bool gap = rec.x == -1 && rec.y == -1;
      const char comp = (char)((rec.w >> 8) & 0xff);
      if (gap) {
      } else if (comp == ' ') {
        delta = kMismatch;
        eval = true;
      } else if (comp == '-') {
        indel = true;
        eval = true;
      } else {
        delta = kMatch;
      }
    }
    const int up = __shfl_up((int)indel, 1, 64);  // all lanes take part in the shuffle
    const bool before = (lane == 0) ? prev_indel : (up != 0);
    if (indel) delta = before ? kQindel : kQopen + kQindel;
    const int score = carry + wave_scan_add(lane, delta);
    const int hi = max(high, wave_scan_maxi(lane, score));
    if (eval) worst = min(worst, score - hi);
    carry = __shfl(score, 63, 64);
    high = __shfl(hi, 63, 64);
    prev_indel = __shfl((int)indel, 63, 64) != 0;
  }
  return wave_min_i(worst);
}

__device__ __forceinline__ bool lex_better(int s1, double p1, int s2, double p2) {
  return s1 > s2 || (s1 == s2 && p1 > p2);
}

// genome_gap_simple (dynprog_genome.c:3006-3280) with one wave: prefix sums of the two
// diagonals (in diagL / diagR, global scratch), then one (score, rL) max-reduction.  Writes the
// result and returns true when the simple path is taken.  When it declines, `res` keeps the
// introntype and probabilities it looked at (the reference leaks them into its out-parameters).
__device__ inline bool gg_simple_wave(int lane, const DevGenomeProblem& P, int pid, const int8_t* __restrict__ sctab,
                               const int8_t* __restrict__ isctab, const uint8_t* __restrict__ cons, const QView& qL,
                               const QView& qucL, const QView& qR, const QView& qucR, const uint8_t* gclL,
                               const uint8_t* gclR, const GClassView& gchL, const GClassView& gchR,
                               const uint8_t* ldi, const uint8_t* rdi, const double* pL, const double* pR,
                               int* diagL, int* diagR, gmapdp_pair* out, gmapdp_genome_result& res,
                               gmapdp_genome_result* __restrict__ results, const uint8_t* __restrict__ ks = nullptr,
                               const double* __restrict__ raw = nullptr, const uint32_t* __restrict__ blocks = nullptr,
                               uint64_t nwords = 0, const double* __restrict__ metab = nullptr) {
  // ks: genome_gap_simple's own known-site flags (left [0, rlength], right after them; nullptr: none),
  // raw: the MaxEnt probabilities (left [0, glengthL), right after them) that get_splicesite_probs
  // returns for an unknown site (dynprog_genome.c:3045-3049, 3118-3119, 3171); raw NULL: evaluated
  // here from the models (metab) on the genome (blocks)
  const int rlen = P.rlength;
  const int8_t* sct = sctab + (size_t)P.mismatchtype * 128 * kNClass;
  const int8_t* iscp = isctab + (size_t)P.iclass * 128;  // prelim array (:3032)
  const bool halfp = P.flags & kGHalf;
  const Geo GL{P.roffset, P.goffsetL, 1};
  const Geo GR{P.roffset + rlen - 1, P.rev_goffsetR, -1};
  // diagL[r] / diagR[r] hold the prefix sums scoreL(r) / scoreR(r) of the two diagonals
  int carryL = 0, carryR = 0;
  for (int base = 0; base < rlen; base += 64) {
    const int r = base + lane + 1;
    int vL = 0, vR = 0;
    if (r <= rlen - 1) {
      vL = sct[(uint8_t)(qucL[r] & 127) * kNClass + gclL[r]];
      vR = sct[(uint8_t)(qucR[r] & 127) * kNClass + gclR[r]];
    }
    const int sL = carryL + wave_scan_add(lane, vL), sR = carryR + wave_scan_add(lane, vR);
    if (r <= rlen - 1) {
      diagL[r] = sL;
      diagR[r] = sR;
    }
    carryL = __shfl(sL, 63, 64);
    carryR = __shfl(sR, 63, 64);
  }
  __threadfence_block();
  // best: max score >= 0 among intron-type sites, ties -> largest rL ("Use >= for jump late")
  uint64_t key = 0;
  for (int rL = lane + 1; rL <= rlen - 1; rL += 64) {
    const int rR = rlen - rL;
    const int it = ldi[rL] & rdi[rR];
    const int kl = (ks && ks[rL]) ? kKnownReward : 0, kr = (ks && ks[rlen + 1 + rR]) ? kKnownReward : 0;
    const int score = diagL[rL] + kl + iscp[it] + kr + diagR[rR];
    if ((it != 0 || kl != 0 || kr != 0) && score >= 0) {
      const uint64_t kk = ((uint64_t)(uint32_t)score << 32) | (uint32_t)rL;
      key = kk > key ? kk : key;
    }
  }
  key = wave_max_u64(key);
  if (key == 0) return false;
  const int bestrL = (int)(key & 0xffffffffu), bestscore = (int)(key >> 32), bestrR = rlen - bestrL;
  const int it = ldi[bestrL] & rdi[bestrR];
  const int scoreI = iscp[it];
  res.introntype = it;
  const int finalscore = halfp ? bestscore - scoreI / 2 : bestscore;
  if (finalscore <= 0) return false;
  if (ks) {
    res.left_prob = ks[bestrL] ? 1.0 : raw ? raw[bestrL] : gg_site_prob(P, blocks, nwords, metab, bestrL);
    res.right_prob = ks[rlen + 1 + bestrR] ? 1.0
                   : raw ? raw[P.glengthL + bestrR] : gg_site_prob(P, blocks, nwords, metab, P.glengthL + bestrR);
  } else {
    res.left_prob = pL[bestrL];
    res.right_prob = pR[bestrR];
  }
  if (!(res.left_prob >= 0.90 && res.right_prob >= 0.90)) return false;
  Tally t = {0, 0, 0, 0, 0, 0, 0, false};
  // list = reverse of the push order (no List_reverse): R diagonal r = 1..bestrR, gap, L r = bestrL..1
  emit_diag(lane, bestrR, bestrR, bestrR, GR, qR, qucR, gchR, cons, out, t);
  const int nR = t.count;
  reverse_records(lane, out, nR);
  const int new_left = P.goffsetL + (bestrL - 1);
  const int new_right = P.rev_goffsetR - (bestrR - 1);
  if (lane == 0) put_pair(out, nR, -1, -1, new_right - new_left - 1, ' ', ' ', ' ', ' ');
  t.count += 1;
  emit_diag(lane, bestrL, bestrL, bestrL, GL, qL, qucL, gchL, cons, out, t);
  if (lane == 0) {
    res.npairs = t.count;
    res.traceback_score = t.nmatches * kMatch + t.nmismatches * kMismatch;
    res.nmatches = t.nmatches;
    res.nmismatches = t.nmismatches;
    res.dynprogindex = P.dynprogindex + (P.dynprogindex > 0 ? 1 : -1);
    res.new_leftgenomepos = new_left;
    res.new_rightgenomepos = res.exonhead = new_right;
    res.gap_index = nR;
    res.gap_queryjump = 0;
    results[pid] = res;
  }
  return true;
}


}  // namespace gmapdp
