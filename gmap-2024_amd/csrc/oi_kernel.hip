// oi_kernel.hip -- CDNA4 (gfx950) kernel for GMAP's stage-2 seeding:
// Oligoindex_hr_tally + Oligoindex_get_mappings as Stage2_compute runs them for GMAP
// (stage2.c:6413-6501; one oligoindex source, indexsize 8, coveredp all false).
//
// Reference semantics restated (paths under the reference tree's src/):
//   Oligoindex_set_inquery         oligoindex_hr.c:33454 (the query's 8-mers; trimp false)
//   count_positions_fwd/rev_std    :19260 / :30761 (8-mers starting in [mappingstart, mappingend-8],
//                                  none unless that range has two starts; Count_T wraps mod 256)
//   Oligoindex_allocate_positions  :32520 (counts masked by inquery; one table slice per oligo)
//   store_positions_fwd/rev_std    :20426 / :31741 (walking from the far end of the chrpos origin,
//                                  an oligo keeps its `count` occurrences nearest that end, stored
//                                  in ascending chrpos)
//   Oligoindex_get_mappings        :34127 (mappings/npositions per querypos, cum_nohits, the
//                                  Genomicdiag_T consecutive-run state per diagonal, the good
//                                  diagonals in the order they reach suffnconsecutive, else the best)
//
// Design.  Two kernels, one wave per (read, genomic window) each.  oi_kernel: the query's distinct
// 8-mers are a 64-K-bit bitmap in LDS; the bitmap's per-word prefix popcounts give every query 8-mer
// a dense id in oligo order, so membership and the id of a window 8-mer are two LDS reads and a
// popcount -- no 64-K count table, no hash.  A window 8-mer is one 64-bit funnel of two 16-nt genome
// half-words (one half-word per lane and step): the reverse complement is its bitwise complement,
// the forward oligo its 2-bit reversal.  Pass 1 counts per id (LDS atomics) and appends the hits to a
// hit list; an exclusive scan lays out the table; pass 2 walks the hit list in descending chrpos and
// places 64 hits at a time, each hit's rank among the step's hits of its oligo coming from a ballot
// match on the id bits, which reproduces the reference's keep-the-nearest-`count` rule exactly.
// oi_map_kernel (1 KB of LDS, so many waves per CU) sorts the hits by diagonal and evaluates each
// diagonal's state machine with segmented scans (oi_mappings_sorted); a problem that does not fit the
// batch's event pool walks the query sequentially instead.
#include <cstdlib>

#include "dp_device.h"

namespace gmapdp {

constexpr int kOiK = 8;

// Phase timing (tools_oi_timing.py; built only into the GMAPDP_OI_TIMING variant of the library):
// every wave adds its wall-clock timestamp at each mark, so mark k - mark k-1 summed over the waves
// is the time spent in phase k.
#ifdef GMAPDP_OI_TIMING
__device__ unsigned long long g_oi_marks[2][16];
// per call (index < 16384): oi_kernel wave 0's and oi_map_kernel's durations (ticks), the events E
__device__ unsigned int g_oi_wave[3][16384];
#define OI_MARK(k)                                                 \
  do {                                                             \
    if (threadIdx.x == 0) {                                        \
      atomicAdd(&g_oi_marks[0][k], (unsigned long long)wall_clock64()); \
      atomicAdd(&g_oi_marks[1][k], 1ull);                          \
    }                                                              \
  } while (0)
#else
#define OI_MARK(k) \
  do {             \
  } while (0)
#endif
constexpr int kOiWords = 65536 / 32;  // bitmap words

// 16-nt half-word h of the packed genome (.genomecomp: {high nt 16-31, low nt 0-15, flags})
__device__ __forceinline__ uint32_t half_word(const uint32_t* __restrict__ blocks, uint64_t h) {
  return blocks[3 * (h >> 1) + ((h & 1) ? 0 : 1)];
}
// forward oligo: first nt most significant (reverse the 2-bit groups)
__device__ __forceinline__ uint32_t oligo_fwd(uint32_t x) {
  x = ((x & 0x3333u) << 2) | ((x >> 2) & 0x3333u);
  x = ((x & 0x0F0Fu) << 4) | ((x >> 4) & 0x0F0Fu);
  x = ((x & 0x00FFu) << 8) | ((x >> 8) & 0x00FFu);
  return x & 0xFFFFu;
}

struct OiState {  // struct Genomicdiag_T (oligoindex_hr.c:106); i is the array index
  int querypos, best_n, n, cstart, best_start, best_end;
};

__device__ __forceinline__ int nt_code(char c) {  // -1 resets the 8-mer (oligoindex_hr.c:34213-34223)
  return c == 'A' ? 0 : c == 'C' ? 1 : c == 'G' ? 2 : c == 'T' ? 3 : -1;
}

__device__ __forceinline__ int oligo_id(const uint32_t* bitmap, const uint16_t* wrank, uint32_t m, bool& in) {
  const uint32_t wbits = bitmap[m >> 5];
  in = (wbits >> (m & 31)) & 1u;
  return wrank[m >> 5] + __popc(wbits & ((1u << (m & 31)) - 1u));
}

// per-problem scratch: cum_nohits (querylength + 1 ints), the event-pool offset and the split kernels'
// hand-over (OiMeta), the window's hit list
struct ScratchOi {
  size_t poolbase, hits, total;
};
struct OiMeta {                 // at poolbase
  unsigned long long poolbase;  // the problem's event-pool offset (or ~0)
  int n0, nhits, U, pad;        // oi_scan_kernel -> oi_build_kernel: wave 0's hits, all hits, distinct 8-mers
};
__host__ __device__ inline ScratchOi scratch_oi(int querylength, uint32_t genomiclength) {
  ScratchOi s;
  s.poolbase = align16(4 * (size_t)(querylength + 1));
  s.hits = align16(s.poolbase + sizeof(OiMeta));
  s.total = align16(s.hits + 8 * ((size_t)genomiclength + 2));
  return s;
}
// the sequential walk's region (only when the event pool cannot take the problem): the genomicdiag init
// flags and states, one per diagonal (querylength + window + 1); DevOligoProblem.fallback_offset
struct ScratchOiFb {
  size_t initp, states, total;
};
__host__ __device__ inline ScratchOiFb scratch_oi_fb(int querylength, uint32_t genomiclength) {
  const size_t nd = (size_t)querylength + genomiclength + 1;
  ScratchOiFb s;
  s.initp = 0;
  s.states = align16(nd);
  s.total = align16(s.states + nd * sizeof(OiState));
  return s;
}

// ---- get_mappings over events sorted by diagonal ----
// The reference visits the hits query position by query position; a diagonal's state only ever sees
// its own hits, in ascending querypos.  So the events (diagi, querypos), generated in query order and
// stably sorted by diagi, put every diagonal's hits in one contiguous segment in the order the
// reference visits them, and its consecutive-run state becomes segmented scans:
//   a run starts at the diagonal's first hit and wherever q - q_prev >= diag_lookback + cum[q] - cum[q_prev];
//   n after a hit = its distance from the run start; best_nconsecutive = the segment's maximum n,
//   reached first at the first hit carrying it (best_end; best_start = its run's first querypos);
//   a diagonal is good when n reaches suffnconsecutive, at the first such hit; the reference appends
//   it there, so the good list is ordered by (querypos, diagi) of that hit (hits of one querypos are
//   visited in ascending chrpos = ascending diagi); maxnconsecutive = the largest n, and the fallback
//   best diagonal the one owning the first (querypos, diagi) hit with that n.

// inclusive max-scan within segments [segstart, e] of consecutive lanes (64-bit values)
__device__ __forceinline__ uint64_t seg_scan_max64(int lane, uint64_t x, int e, int segstart) {
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const uint64_t y = __shfl_up(x, off, 64);
    if (lane >= off && e - off >= segstart && y > x) x = y;
  }
  return x;
}
__device__ __forceinline__ int seg_scan_min(int lane, int x, int e, int segstart) {
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const int y = __shfl_up(x, off, 64);
    if (lane >= off && e - off >= segstart) x = min(x, y);
  }
  return x;
}

constexpr int kOiHist = 4 * 256;  // = 2 x 512

// Event keys, ordered by diagi (the sort's digits) then by generation order (query order).  The run test
// of the reference, q - q_prev >= diag_lookback + cum[q] - cum[q_prev], is (q - cum[q]) - (q_prev -
// cum[q_prev]) >= diag_lookback: with t = q - cum_nohits[q] in the key the sweep compares two keys and
// reads no cum_nohits (two scattered loads per event otherwise).  t rises by one at every query position
// that has hits (cum_nohits only counts positions without), so on the positions events come from t is
// strictly increasing in q: (t, diagi) orders events as (q, diagi) does, and q is recovered, for the few
// events whose querypos the records need, as the first position with q - cum[q] >= t (binary search).
// So a 2-kb read's 214-kb window takes 32-bit keys (diagi < 2^20 - 1, t < 4096: half the bytes of every
// event pass and radix scatter, the kernel being bound by that traffic); longer queries or windows keep
// 64 bits with q (and t below 2^16) inside.
__device__ __forceinline__ uint64_t readlane64(uint64_t k, int l) {
  return ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(k >> 32), l) << 32) |
         (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)k, l);
}
// first query position whose q - cum[q] reaches t (q - cum[q] is non-decreasing)
__device__ __forceinline__ uint32_t oi_q_of_t(int t, const int* __restrict__ cum, int nq) {
  int lo = 0, hi = nq - 1;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (mid - cum[mid] >= t) hi = mid;
    else lo = mid + 1;
  }
  return (uint32_t)lo;
}
struct OiKeyT32 {  // diagi << 12 | t
  using K = uint32_t;
  static constexpr uint32_t kMax = ~0u;
  __device__ static uint32_t make(uint32_t di, uint32_t, uint32_t t) { return (di << 12) | t; }
  __device__ static uint32_t di(uint32_t k) { return k >> 12; }
  __device__ static int t(uint32_t k, const int* __restrict__) { return (int)(k & 0xFFFu); }
  __device__ static uint32_t ord(uint32_t k) { return k & 0xFFFu; }  // orders events as q does
  __device__ static uint32_t q(uint32_t k, const int* __restrict__ cum, int nq) {
    return oi_q_of_t((int)(k & 0xFFFu), cum, nq);
  }
  __device__ static uint32_t readlane(uint32_t k, int l) { return (uint32_t)__builtin_amdgcn_readlane((int)k, l); }
};
struct OiKeyQT {  // diagi << 32 | q << 16 | t
  using K = uint64_t;
  static constexpr uint64_t kMax = ~0ull;
  __device__ static uint64_t make(uint32_t di, uint32_t q, uint32_t t) {
    return ((uint64_t)di << 32) | (q << 16) | t;
  }
  __device__ static uint32_t di(uint64_t k) { return (uint32_t)(k >> 32); }
  __device__ static int t(uint64_t k, const int* __restrict__) { return (int)((uint32_t)k & 0xFFFFu); }
  __device__ static uint32_t ord(uint64_t k) { return (uint32_t)k >> 16; }
  __device__ static uint32_t q(uint64_t k, const int* __restrict__, int) { return (uint32_t)k >> 16; }
  __device__ static uint64_t readlane(uint64_t k, int l) { return readlane64(k, l); }
};
struct OiKeyQ {  // diagi << 32 | q
  using K = uint64_t;
  static constexpr uint64_t kMax = ~0ull;
  __device__ static uint64_t make(uint32_t di, uint32_t q, uint32_t) { return ((uint64_t)di << 32) | q; }
  __device__ static uint32_t di(uint64_t k) { return (uint32_t)(k >> 32); }
  __device__ static int t(uint64_t k, const int* __restrict__ cum) { return (int)(uint32_t)k - cum[(uint32_t)k]; }
  __device__ static uint32_t ord(uint64_t k) { return (uint32_t)k; }
  __device__ static uint32_t q(uint64_t k, const int* __restrict__, int) { return (uint32_t)k; }
  __device__ static uint64_t readlane(uint64_t k, int l) { return readlane64(k, l); }
};

// The get_mappings pieces below run on ONE wave (oi_map_kernel's, or wave 0 of oi_build_kernel while its
// other waves have finished): a wave's LDS operations complete in order, so a fence at wavefront scope
// (the compiler's lgkmcnt waits) is the only synchronisation they need between their phases.
__device__ __forceinline__ void oi_wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

// ---- the pieces of get_mappings over sorted events (shared by the global-pool and the LDS paths) ----

// One problem's events in query order, hits of one querypos in table (ascending chrpos) order, 256 query
// positions per step (their nhits / table offsets loaded a step ahead).  The step's exclusive event
// offsets and table offsets go to LDS (evq: 3 x 256 ints); each event finds its query position there by
// binary search, 256 events at a time, so their table loads all issue together.  f(e, v, di, key) is
// called once per group of 64 events (wave-uniform call; per lane: the event's index in query order, valid,
// its diagonal, its key).
// (sb0, sbstep: the steps this wave takes -- all of them by default; the event index e counts only those)
template <typename KT, typename F>
__device__ __forceinline__ void oi_for_events(int lane, int qlen, int nq, uint32_t chrinit,
                                              const int32_t* __restrict__ npq, const int32_t* __restrict__ mpq,
                                              const int* __restrict__ cum, const uint32_t* __restrict__ table_all,
                                              int* evq, F&& f, int sb0 = 0, int sbstep = 4 * 64) {
  int* exo = evq;          // [256] exclusive event offset of each query position of the step
  int* mos = evq + 256;    // [256] its table offset
  int* cus = evq + 512;    // [256] its cum_nohits
  int eoff = 0;
  int nh_n[4], mo_n[4], cu_n[4];
#pragma unroll
  for (int r = 0; r < 4; r++) {
    const int q = sb0 + 64 * r + lane;
    nh_n[r] = q < nq ? npq[q] : 0;
    mo_n[r] = q < nq ? mpq[q] : 0;
    cu_n[r] = q < nq ? cum[q] : 0;
  }
  for (int sb = sb0; sb < nq; sb += sbstep) {
    int nh[4], mo[4], cu[4];
#pragma unroll
    for (int r = 0; r < 4; r++) {
      nh[r] = max(nh_n[r], 0);
      mo[r] = mo_n[r];
      cu[r] = cu_n[r];
      const int q = sb + sbstep + 64 * r + lane;
      nh_n[r] = q < nq ? npq[q] : 0;
      mo_n[r] = q < nq ? mpq[q] : 0;
      cu_n[r] = q < nq ? cum[q] : 0;
    }
    int run = 0;
#pragma unroll
    for (int r = 0; r < 4; r++) {
      const int incl = wave_scan_add(lane, nh[r]);
      exo[64 * r + lane] = run + incl - nh[r];
      mos[64 * r + lane] = mo[r];
      cus[64 * r + lane] = cu[r];
      run += __builtin_amdgcn_readlane(incl, 63);
    }
    const int T = run;
    oi_wave_sync();
    for (int g0 = 0; g0 < T; g0 += 4 * 64) {
      uint32_t tv[4];
      int qv[4], cv[4];
#pragma unroll
      for (int gi = 0; gi < 4; gi++) {
        const int j = g0 + 64 * gi + lane;
        int l = 0;  // the last position whose events start at or before j
#pragma unroll
        for (int step = 128; step >= 1; step >>= 1)
          if (exo[l + step] <= j) l += step;
        qv[gi] = sb + l;
        cv[gi] = cus[l];
        tv[gi] = j < T ? table_all[mos[l] + (j - exo[l])] : 0u;
      }
#pragma unroll
      for (int gi = 0; gi < 4; gi++) {
        const int j = g0 + 64 * gi + lane;
        const uint32_t di = tv[gi] + (uint32_t)(qlen - qv[gi]) - chrinit;
        f(eoff + j, j < T, di, KT::make(di, (uint32_t)qv[gi], (uint32_t)(qv[gi] - cv[gi])));
      }
    }
    eoff += T;
    oi_wave_sync();
  }
}

// Radix digits: 9 bits wide when maxdiag < 2^18 (2 passes of 512 buckets: a 214-kb window), else 8 bits
// (at most 4 passes of 256); hist holds kOiHist counters.
struct OiDigits {
  int db, npass;
  uint32_t dmask;
};
__device__ __forceinline__ OiDigits oi_digits(uint32_t maxdiag) {
  OiDigits d;
  d.db = maxdiag < (1u << 18) ? 9 : 8;
  d.dmask = (1u << d.db) - 1u;
  d.npass = 0;  // digits of the largest possible diagi
  while (d.npass < 4 && (maxdiag >> (d.db * d.npass)) != 0) d.npass++;
  return d;
}
// every radix pass's digit histogram, counted as the keys are generated (the sort never re-reads the keys
// to count them): one LDS atomic per distinct digit of the group (the hits of a group mostly share a few
// diagonals, and same-address atomics serialise)
__device__ __forceinline__ void oi_hist_add(int lane, bool v, uint32_t di, const OiDigits& D, uint32_t* hist) {
  for (int p = 0; p < D.npass; p++) {
    const uint32_t dg = (di >> (D.db * p)) & D.dmask;
    uint64_t eq = ballot(v);
#pragma unroll
    for (int b = 0; b < 9; b++) {  // (bit 8 of an 8-bit digit is 0 in every lane)
      const uint64_t m = ballot((dg >> b) & 1u);
      eq &= ((dg >> b) & 1u) ? m : ~m;
    }
    if (v && lanes_below(eq, lane) == 0) atomicAdd(&hist[(D.dmask + 1) * p + dg], (uint32_t)__popcll(eq));
  }
}

// Stable LSD radix sort of E keys on diagi, src and dst ping-pong (global pool or LDS); returns the sorted
// buffer.  256 keys per step: their 4 loads and 4 stores each go out together; the ranks are taken chunk
// by chunk in order, which keeps the sort stable.
template <typename KT>
__device__ __forceinline__ typename KT::K* oi_radix(int lane, typename KT::K* src, typename KT::K* dst, int E,
                                                    const OiDigits& D, uint32_t* hist) {
  using K = typename KT::K;
  for (int p = 0; p < D.npass; p++) {
    uint32_t* hp = hist + (D.dmask + 1) * p;
    const int shift = D.db * p;
    const int cpl = (int)(D.dmask + 1) / 64;  // buckets per lane: 8 or 4
    uint32_t h8[8], hs = 0;
#pragma unroll
    for (int k = 0; k < 8; k++) {
      h8[k] = k < cpl ? hp[cpl * lane + k] : 0u;
      hs += h8[k];
    }
    uint32_t at = (uint32_t)wave_scan_add(lane, (int)hs) - hs;
#pragma unroll
    for (int k = 0; k < 8; k++) {
      if (k < cpl) hp[cpl * lane + k] = at;
      at += h8[k];
    }
    oi_wave_sync();
    for (int e0 = 0; e0 < E; e0 += 4 * 64) {
      K key[4];
      uint32_t dpos[4];
#pragma unroll
      for (int r = 0; r < 4; r++) {
        const int e = e0 + 64 * r + lane;
        key[r] = e < E ? src[e] : (K)0;
      }
#pragma unroll
      for (int r = 0; r < 4; r++) {
        const bool v = e0 + 64 * r + lane < E;
        const uint32_t d = (KT::di(key[r]) >> shift) & D.dmask;
        uint64_t eq = ballot(v);
#pragma unroll
        for (int b = 0; b < 9; b++) {
          const uint64_t m = ballot((d >> b) & 1u);
          eq &= ((d >> b) & 1u) ? m : ~m;
        }
        const int rank = lanes_below(eq, lane);
        const uint32_t pos = v ? hp[d] : 0u;  // every lane reads before any lane bumps
        oi_wave_sync();
        dpos[r] = pos + (uint32_t)rank;
        if (v && rank == 0) hp[d] = pos + (uint32_t)__popcll(eq);
        oi_wave_sync();
      }
#pragma unroll
      for (int r = 0; r < 4; r++)
        if (e0 + 64 * r + lane < E) dst[dpos[r]] = key[r];
    }
    __threadfence_block();
    K* t = src;
    src = dst;
    dst = t;
  }
  __threadfence_block();
  return src;
}

// Sweep over the E sorted events S: runs, each diagonal's maximum and its first event, the first event
// reaching suffn; a diagonal's last event appends its record (grec) when it is good.  Per lane, the largest
// n seen and the smallest (querypos, diagi) event carrying it (the fallback best).  Then the records in the
// reference's order into `good` (gkey: ngood 64-bit scratch keys).  Returns ngood (-1: more than gcap).
template <typename KT>
__device__ __forceinline__ int oi_sweep(int lane, const typename KT::K* S, int E, int qlen, int nq, int lookback,
                                        int suffn, const int* __restrict__ cum, int4* grec, uint64_t* gkey,
                                        int32_t* __restrict__ good, int gcap, int& maxn_out) {
  using K = typename KT::K;
  constexpr K kMax = KT::kMax;
  int c_rs = -1, c_ds = -1, c_fs = 0x7fffffff, ngood = 0;
  uint64_t c_mk = 0;
  K c_key = 0;
  int bm = -1, be = -1;
  uint64_t bkey = ~0ull;
  // 256 events per step: their key loads go out together; the 4 chunks are then scanned in order with the
  // carries
  for (int s0 = 0; s0 < E; s0 += 4 * 64) {
    K key[4];
#pragma unroll
    for (int r = 0; r < 4; r++) {
      const int e = s0 + 64 * r + lane;
      key[r] = e < E ? S[e] : kMax;
    }
    const K after = s0 + 4 * 64 < E ? S[s0 + 4 * 64] : kMax;  // the event after this step
    K pkey[4];
    int tq[4], tpq[4];
#pragma unroll
    for (int r = 0; r < 4; r++) {
      K pk = __shfl_up(key[r], 1, 64);
      if (lane == 0) pk = r == 0 ? c_key : KT::readlane(key[r - 1], 63);
      pkey[r] = pk;
      const bool v = s0 + 64 * r + lane < E;
      tq[r] = v ? KT::t(key[r], cum) : 0;
      tpq[r] = v && s0 + 64 * r + lane > 0 ? KT::t(pk, cum) : 0;
    }
#pragma unroll
    for (int r = 0; r < 4; r++) {
      const int e0 = s0 + 64 * r;
      const int e = e0 + lane;
      const bool v = e < E;
      const K key_r = key[r], pk = pkey[r];
      const uint32_t d = KT::di(key_r), q = KT::ord(key_r);  // (q or t: the same order)
      const bool newdiag = v && (e == 0 || KT::di(pk) != d);
      bool newrun = newdiag;
      if (v && !newdiag) newrun = tq[r] - tpq[r] >= lookback;
      const int rs = max(wave_scan_max(newrun ? e : -1), c_rs);
      const int ds = max(wave_scan_max(newdiag ? e : -1), c_ds);
      const int n = e - rs;
      uint64_t mk = v ? (((uint64_t)(uint32_t)n << 32) | (uint64_t)(~(uint32_t)e)) : 0ull;
      mk = seg_scan_max64(lane, mk, e, ds);
      if (ds < e0 && c_mk > mk) mk = c_mk;
      int fs = (v && n == suffn) ? e : 0x7fffffff;
      fs = seg_scan_min(lane, fs, e, ds);
      if (ds < e0) fs = min(fs, c_fs);
      K nk = __shfl_down(key_r, 1, 64);
      if (lane == 63) nk = r < 3 ? KT::readlane(key[r + 1], 0) : after;
      const bool dend = v && (e + 1 == E || KT::di(nk) != d);
      const bool isgood = dend && fs != 0x7fffffff;
      const uint64_t gm = ballot(isgood);
      if (isgood)  // {first event with n == suffn, first event with the maximum, the maximum, diagi}
        grec[ngood + lanes_below(gm, lane)] = make_int4(fs, (int)~(uint32_t)mk, (int)(mk >> 32), (int)d);
      ngood += __popcll(gm);
      if (v) {
        const uint64_t k2 = ((uint64_t)q << 32) | d;
        if (n > bm || (n == bm && k2 < bkey)) {
          bm = n;
          bkey = k2;
          be = e;
        }
      }
      c_rs = __builtin_amdgcn_readlane(rs, 63);
      c_ds = __builtin_amdgcn_readlane(ds, 63);
      c_fs = __builtin_amdgcn_readlane(fs, 63);
      c_mk = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(mk >> 32), 63) << 32) |
             (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)mk, 63);
      c_key = KT::readlane(key_r, 63);
    }
  }
  // the global maximum and the first (querypos, diagi) event carrying it
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {
    const int om = __shfl_xor(bm, off, 64);
    const uint64_t ok = __shfl_xor(bkey, off, 64);
    const int oe = __shfl_xor(be, off, 64);
    if (om > bm || (om == bm && ok < bkey)) {
      bm = om;
      bkey = ok;
      be = oe;
    }
  }
  const int M = max(bm, 0);
  __threadfence_block();
  if (ngood == 0 && M > 0) {
    if (lane == 0) grec[0] = make_int4(-1, be, M, (int)(uint32_t)bkey);
    ngood = 1;
  }
  __threadfence_block();
  // records and their (querypos, diagi) keys; then the reference's order
  for (int g = lane; g < ngood; g += 64) {
    const int4 r = grec[g];
    const uint32_t di = (uint32_t)r.w;
    const int eb = r.y, bn = r.z;
    const uint32_t qreach = r.x >= 0 ? KT::q(S[r.x], cum, nq) : 0u;
    gkey[g] = ((uint64_t)qreach << 32) | di;
    grec[g] = make_int4(di >= (uint32_t)qlen ? (int)(di - (uint32_t)qlen) : (int)((uint32_t)qlen - di),
                        (int)KT::q(S[eb - bn], cum, nq), (int)KT::q(S[eb], cum, nq), bn + 1);
  }
  __threadfence_block();
  if (ngood > gcap) ngood = -1;  // more good diagonals than the layout gave the problem: overflow
  for (int g = lane; g < ngood; g += 64) {
    const uint64_t k = gkey[g];
    int rank = 0;
    for (int h = 0; h < ngood; h++) rank += gkey[h] < k ? 1 : 0;
    reinterpret_cast<int4*>(good)[rank] = grec[g];
  }
  maxn_out = M;
  return ngood;
}

// get_mappings over the shared global event pool.  Returns false (nothing written) when the pool could not
// hold this problem's 3 E slots (`base` == ~0).
// With `slots` (kOimSlots 16-bit LDS counters) the events are first counted per diagonal slot (a hash of the
// diagonal) and only those of slots holding at least suffn + 1 events are sorted and swept: a good diagonal
// holds that many, so every event of every good diagonal is kept, and when some diagonal is good the good list
// and maxnconsecutive are exactly the full event set's (oi_mappings_lds gives the argument).  On a 214-kb
// window that is the read's locus, ~2 000 of ~8 300 events: a quarter of the keys written and scattered by
// the radix passes.  With no good diagonal the full event set is sorted and swept after all.
constexpr int kOimSlots = 1024;
__device__ __forceinline__ uint32_t oim_slot(uint32_t di) { return (di * 2654435761u) >> 22; }

template <typename KT, bool kSlots>
__device__ bool oi_mappings_sorted(int lane, int qlen, int nq, int E, uint32_t maxdiag, uint32_t chrinit,
                                   int lookback, int suffn, const int32_t* __restrict__ npq,
                                   const int32_t* __restrict__ mpq, const int* __restrict__ cum,
                                   const uint32_t* __restrict__ table_all, uint64_t* __restrict__ pool,
                                   unsigned long long base, uint32_t* hist,
                                   int* evq, int32_t* __restrict__ good, int gcap, int& ngood_out, int& maxn_out,
                                   uint32_t* slots = nullptr) {
  OI_MARK(9);
  if (base == ~0ull) return false;
  using K = typename KT::K;
  K* evA = reinterpret_cast<K*>(pool + base);       // events (OiKeyT32 / OiKeyQT / OiKeyQ)
  K* evB = evA + E;                                 // radix-sort ping-pong
  int4* grec = reinterpret_cast<int4*>(pool + base + 2 * (size_t)E);  // good records (at most E / 2)
  const OiDigits D = oi_digits(maxdiag);
  // the good diagonals' query-order keys: the free sort buffer (64-bit events), or the pool's second E words
  // (32-bit events: both sort buffers sit in the first)
  const uint32_t need = (uint32_t)suffn + 1u;
  bool filtered = kSlots && E < 65536;
  if (filtered) {
    for (int i = lane; i < kOimSlots / 2; i += 64) slots[i] = 0u;
    oi_wave_sync();
    oi_for_events<KT>(lane, qlen, nq, chrinit, npq, mpq, cum, table_all, evq, [&](int, bool v, uint32_t di, K) {
      if (v) {
        const uint32_t h = oim_slot(di);
        atomicAdd(&slots[h >> 1], 1u << (16 * (h & 1)));
      }
    });
    oi_wave_sync();
  }
  for (;;) {
    for (int i = lane; i < kOiHist; i += 64) hist[i] = 0u;
    oi_wave_sync();
    int C = 0;
    oi_for_events<KT>(lane, qlen, nq, chrinit, npq, mpq, cum, table_all, evq,
                      [&](int, bool v, uint32_t di, K key) {
                        bool c = v;
                        if (filtered) {
                          const uint32_t h = oim_slot(di);
                          c = v && ((slots[h >> 1] >> (16 * (h & 1))) & 0xFFFFu) >= need;
                        }
                        const uint64_t cm = ballot(c);
                        if (c) evA[C + lanes_below(cm, lane)] = key;
                        oi_hist_add(lane, c, di, D, hist);
                        C += __popcll(cm);
                      });
    __threadfence_block();
    oi_wave_sync();
    OI_MARK(5);
    const K* S = oi_radix<KT>(lane, evA, evB, C, D, hist);
    OI_MARK(6);
    uint64_t* gkey = sizeof(K) == 8 ? reinterpret_cast<uint64_t*>(S == evA ? evB : evA) : pool + base + E;
    int maxn = 0;
    const int ngood = oi_sweep<KT>(lane, S, C, qlen, nq, lookback, suffn, cum, grec, gkey, good, gcap, maxn);
    if (filtered && ngood != -1 && (ngood == 0 || maxn < suffn)) {  // no good diagonal: the full event set
      filtered = false;
      continue;
    }
    ngood_out = ngood;
    maxn_out = maxn;
    return true;
  }
}

// Per-id counters: 16-bit when the window has fewer than 65536 8-mer starts (no count or table
// offset can reach 2^16, and the 28-KB LDS of a 2-kb read drops to 20 KB: 8 waves per CU, not 5),
// 32-bit otherwise.  Pass 1 increments a 16-bit counter through its 32-bit word.
template <typename CT>
__device__ __forceinline__ void count_inc(CT* cnt, int u) {
  if constexpr (sizeof(CT) == 4) {
    atomicAdd(reinterpret_cast<uint32_t*>(cnt) + u, 1u);
  } else {
    atomicAdd(reinterpret_cast<uint32_t*>(cnt) + (u >> 1), 1u << (16 * (u & 1)));
  }
}

// A problem that outgrew its layout: no hits, oned_matrix_p -1 (Stage2_compute status -2), the event pool
// slot marked empty, nothing written past the problem's slices.  Block-uniform: every thread calls it.
__device__ void oi_report_overflow(const DevOligoProblem& P, int tid, int nthreads, int qlen, int32_t* npq,
                                   int32_t* mpq, gmapdp_oligo_result* results, unsigned char* poolslot) {
  for (int i = tid; i < qlen; i += nthreads) {
    npq[i] = 0;
    mpq[i] = -1;
  }
  if (tid == 0) {
    gmapdp_oligo_result res;
    res.totalpositions = 0;
    res.maxnconsecutive = 0;
    res.oned_matrix_p = -1;
    res.ndiagonals = 0;
    res.table_offset = P.table_offset;
    res.diag_offset = P.diag_offset;
    results[P.index] = res;
    *reinterpret_cast<unsigned long long*>(poolslot) = ~0ull;
  }
}

// Two waves per problem: both take half of the query's 8-mers and half of the window's pass-1 scan (the
// long phase: ~200 steps on a 214-kb window) over the same LDS tables; the phases that carry a running
// value in order (the id ranks, the table layout, pass 2's placement, the per-position mappings) stay
// on wave 0 between workgroup barriers.  Wave 1 appends its hits from the far end of the hit list (so
// the two lists meet only when the layout's capacity is exceeded, which is reported as overflow).
constexpr int kOiWaves = 2;
// Pass 2's table through LDS images (GMAPDP_OI_STAGE builds, experiments): ~5x fewer bytes written, but the
// seeding measured 0.3 ms slower per 10 k-read block in the bench step (6.89 vs 6.61 ms alone,
// profiles/r06_seed), so the product keeps the direct scattered stores.
#ifdef GMAPDP_OI_STAGE
constexpr bool kOiStage = true;
#else
constexpr bool kOiStage = false;
#endif

#define OI_PASS_ARGS                                                                                          \
  const DevOligoProblem *__restrict__ probs, const uint32_t *__restrict__ blocks, const char *__restrict__ quc_all, \
      unsigned char *__restrict__ scratch, gmapdp_oligo_result *__restrict__ results,                             \
      int32_t *__restrict__ npos_out, int32_t *__restrict__ map_out, uint32_t *__restrict__ table_all,            \
      unsigned long long *__restrict__ pool_counter, unsigned long long pool_cap, int32_t *__restrict__ nhits_out
template <typename CT>
__device__ __forceinline__ void oi_pass(OI_PASS_ARGS) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  __shared__ int nh_wave[kOiWaves];  // each wave's pass-1 hits
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const DevOligoProblem P = probs[blockIdx.x];
  uint32_t* bitmap = reinterpret_cast<uint32_t*>(smem);                  // 2048 words
  uint16_t* wrank = reinterpret_cast<uint16_t*>(smem + 4 * kOiWords);     // set bits before word w
  CT* cnt = reinterpret_cast<CT*>(smem + 6 * kOiWords);                   // per id: count, then remaining
  CT* offs = cnt + P.umax;                                                // per id: table offset
  const char* quc = quc_all + P.qoff;
  const int qlen = P.querylength;
  OI_MARK(0);
#ifdef GMAPDP_OI_TIMING
  const unsigned long long oi_t0 = wall_clock64();
#endif
  const int nq = qlen - kOiK + 1;  // query positions with a full 8-mer

  // ---- the query's 8-mers (Oligoindex_set_inquery) ----
  for (int w = tid; w < kOiWords; w += 64 * kOiWaves) bitmap[w] = 0u;
  __syncthreads();
  int32_t* npq = npos_out + P.qoff;
  int32_t* mpq = map_out + P.qoff;  // holds each querypos's 8-mer (or -1) until get_mappings
  // 256 query positions per step: one coalesced character load per lane and chunk (5 chunks: the
  // last supplies the 7-character overlap), all issued together; the 8-mer at i takes the codes of
  // lanes i..i+7 of its chunk and the next (ds_bpermute)
  for (int sb = 4 * 64 * wave; sb < qlen; sb += 4 * 64 * kOiWaves) {
    int ch[5];
#pragma unroll
    for (int r = 0; r < 5; r++) {
      const int i = sb + 64 * r + lane;
      ch[r] = i < qlen ? nt_code(quc[i]) : -1;
    }
#pragma unroll
    for (int r = 0; r < 4; r++) {
      const int i = sb + 64 * r + lane;
      uint32_t m = 0;
      bool ok = i < nq;
#pragma unroll
      for (int j = 0; j < kOiK; j++) {
        const int src = (lane + j) & 63;
        const int a = __shfl(ch[r], src, 64), b = __shfl(ch[r + 1], src, 64);
        const int cj = lane + j < 64 ? a : b;
        ok = ok && cj >= 0;
        m = (m << 2) | ((uint32_t)cj & 3u);
      }
      if (i < qlen) {
        mpq[i] = ok ? (int)m : -1;
        npq[i] = 0;
      }
      if (ok) atomicOr(&bitmap[m >> 5], 1u << (m & 31));
    }
  }
  __syncthreads();
  int run = 0;  // ids in oligo order: prefix popcounts over the bitmap words (every wave: U below)
  for (int base = 0; base < kOiWords; base += 64) {
    const int c = __popc(bitmap[base + lane]);
    const int incl = wave_scan_add(lane, c);
    if (wave == 0) wrank[base + lane] = (uint16_t)(run + incl - c);
    run += __builtin_amdgcn_readlane(incl, 63);
  }
  const int U = run;
  OI_MARK(1);
  unsigned char* base_s = scratch + P.scratch_offset;
  const ScratchOi so = scratch_oi(qlen, P.chrend > P.chrstart ? P.chrend - P.chrstart : 0);
  // More distinct 8-mers than the LDS bucket the plan gave the problem (a plan laid out from one query and
  // run on another): cnt / offs would run past the dynamic LDS, so report overflow before writing them.
  if (U > P.umax) {
    oi_report_overflow(P, tid, 64 * kOiWaves, qlen, npq, mpq, results, base_s + so.poolbase);
    return;
  }
  for (int u = tid; u < U; u += 64 * kOiWaves) cnt[u] = 0;
  __syncthreads();

  // ---- pass 1: counts of the window's query 8-mers ----
  const uint64_t left = (uint64_t)P.chroffset + P.chrstart;
  uint64_t lpl = (uint64_t)P.chroffset + P.chrend + (P.plusp ? 0 : 1);
  lpl = lpl < (uint64_t)kOiK ? 0 : lpl - kOiK;
  const uint64_t npos = lpl > left ? lpl - left + 1 : 0;
  // Each lane takes one 16-nt genome half-word (its 16 8-mer starts, from the half-word and the
  // next); the next step's two loads are issued before this step's LDS work.  Every hit is appended
  // to the problem's hit list {window index, id} in ascending position, so pass 2 never re-reads the
  // window.
  uint2* hitlist = reinterpret_cast<uint2*>(base_s + so.hits);
  uint32_t* hitlist32 = reinterpret_cast<uint32_t*>(base_s + so.hits);
  // hits as (window index << 14 | id) when the window has at most 2^18 starts (ids are below 2^14): half the
  // bytes the list writes and pass 2 reads back
  const bool compact = npos <= (1ull << 18);
  int nhits = 0;
  if (npos > 0) {
    // this wave's steps of 64 half-words: wave 0 the first half of the window's, wave 1 the rest
    const uint64_t hlo0 = left >> 4, hhi0 = lpl >> 4;
    const uint64_t nsteps = (hhi0 - hlo0) / 64 + 1, half = (nsteps + 1) / 2;
    const uint64_t hlo = hlo0 + (wave ? 64 * half : 0);
    const uint64_t hhi = wave ? hhi0 : (hlo0 + 64 * half - 1 < hhi0 ? hlo0 + 64 * half - 1 : hhi0);
    // a window of ~200 kb is ~200 steps: the half-words of the next kOiAhead steps are in flight, so a
    // step waits on an L2 / HBM round trip only at the start (one step ahead left every step waiting)
    constexpr int kOiAhead = 4;
    uint32_t pw0[kOiAhead], pw1[kOiAhead];
#pragma unroll
    for (int a = 0; a < kOiAhead; a++) {
      const uint64_t hh = hlo + 64 * a + lane;
      pw0[a] = hh <= hhi ? half_word(blocks, hh) : 0u;
      pw1[a] = hh <= hhi ? half_word(blocks, hh + 1) : 0u;
    }
    // one step: the lane's 16 8-mer starts of half-word h (v = half-words h, h + 1)
    auto step = [&](uint64_t hb, uint64_t v) {
      const uint64_t h = hb + lane;
      // the 8-mer at window offset j as its oligo: plus strand, first nt most significant (the 2-bit groups
      // of the 32 nt reversed once, then m_j = bits 2 (24 - j) ..); minus strand, the complement as read
      uint64_t vv;
      if (P.plusp) {
        vv = ((v >> 2) & 0x3333333333333333ull) | ((v & 0x3333333333333333ull) << 2);
        vv = ((vv >> 4) & 0x0F0F0F0F0F0F0F0Full) | ((vv & 0x0F0F0F0F0F0F0F0Full) << 4);
        vv = __builtin_bswap64(vv);
      } else {
        vv = ~v;
      }
      auto oligo_at = [&](int j) -> uint32_t {
        return (uint32_t)(vv >> (P.plusp ? 2 * (24 - j) : 2 * j)) & 0xFFFFu;
      };
      // the starts of this half-word inside [left, lpl]: bits jlo .. jhi
      uint32_t vmask = 0;
      if (h <= hhi) {
        const uint64_t p0 = 16 * h;
        const int jlo = left > p0 ? (int)(left - p0) : 0;
        const int jhi = lpl < p0 + 15 ? (int)(lpl - p0) : 15;
        if (jlo <= jhi) vmask = (0xFFFFu >> (15 - jhi)) & (0xFFFFu << jlo);
      }
      // membership first (one bitmap word each); the id (rank within the bitmap) only for the ~3 % of
      // 8-mers that hit, so the rank table is read by the hit lanes alone
      uint32_t hm = 0;
#pragma unroll
      for (int j = 0; j < 16; j++) {
        const uint32_t m = oligo_at(j);
        hm |= ((bitmap[m >> 5] >> (m & 31)) & 1u) << j;
      }
      hm &= vmask;
      const int c = __popc(hm);
      const int incl = wave_scan_add(lane, c);
      int o = nhits + incl - c;
      for (uint32_t r = hm; r; r &= r - 1) {
        const int j = __ffs(r) - 1;
        const uint32_t m = oligo_at(j);
        bool in;
        const int id = oligo_id(bitmap, wrank, m, in);
        count_inc(cnt, id);
        // wave 0 from the start of the list, wave 1 from its end (its k-th hit at hit_cap - 1 - k)
        if ((uint32_t)o < P.hit_cap) {
          const uint32_t at = wave ? P.hit_cap - 1 - (uint32_t)o : (uint32_t)o;
          const uint32_t k = (uint32_t)(16 * h + j - left);
          if (compact) hitlist32[at] = (k << 14) | (uint32_t)id;
          else hitlist[at] = make_uint2(k, (uint32_t)id);
        }
        o++;
      }
      nhits += __builtin_amdgcn_readlane(incl, 63);
    };
    // unrolled by kOiAhead so each slot is a fixed register pair and a step waits for its own loads only
    for (uint64_t hb0 = hlo; hlo <= hhi && hb0 <= hhi; hb0 += 64 * kOiAhead) {
#pragma unroll
      for (int a = 0; a < kOiAhead; a++) {
        const uint64_t hb = hb0 + 64 * a;
        if (hb > hhi) break;
        const uint64_t v = (uint64_t)pw0[a] | ((uint64_t)pw1[a] << 32);
        const uint64_t hh = hb + 64 * kOiAhead + lane;  // refill the slot with the step kOiAhead ahead
        pw0[a] = hh <= hhi ? half_word(blocks, hh) : 0u;
        pw1[a] = hh <= hhi ? half_word(blocks, hh + 1) : 0u;
        step(hb, v);
      }
    }
  }
  if (lane == 0) nh_wave[wave] = nhits;
  __syncthreads();
  const int n0 = nh_wave[0], n1 = nh_wave[1];
  nhits = n0 + n1;
  if (nhits_out && tid == 0) nhits_out[P.index] = nhits;  // the hit list's length (a plan's sizing run)
  // Count_T wraps; the table slices follow oligo order (wave 0; the total to both waves)
  __shared__ uint32_t tot_s;
  if (wave == 0) {
    uint32_t tot = 0;
    for (int base = 0; base < U; base += 64) {
      const int u = base + lane;
      const uint32_t c = u < U ? ((uint32_t)cnt[u] & 255u) : 0u;
      const uint32_t incl = (uint32_t)wave_scan_add(lane, (int)c);
      if (u < U) {
        offs[u] = (CT)(tot + incl - c);
        cnt[u] = (CT)c;
      }
      tot += (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
    }
    if (lane == 0) tot_s = tot;
  }
  // each query position's 8-mer as its id (get_mappings' lookups), so that the bitmap and its ranks are free
  // for pass 2's table staging
  for (int i = tid; i < nq; i += 64 * kOiWaves) {
    const int m = mpq[i];
    if (m >= 0) {
      bool in;
      mpq[i] = oligo_id(bitmap, wrank, (uint32_t)m, in);
    }
  }
  __syncthreads();
  const uint32_t tot = tot_s;
  OI_MARK(2);
  // More hits or table entries than the layout gave the problem (a plan re-laid out from a measured run,
  // then run on another query), or a 16-bit counter that could wrap: report overflow, as an exhausted
  // event pool does, with no hits and nothing written past the problem's slices.
  if ((uint32_t)nhits > P.hit_cap || tot > P.table_cap || (sizeof(CT) == 2 && nhits > 65535)) {
    oi_report_overflow(P, tid, 64 * kOiWaves, qlen, npq, mpq, results, base_s + so.poolbase);
    return;
  }

  // ---- pass 2: store in descending chrpos (plus: right to left; minus: left to right) ----
  // kOiStage (compact lists): each hit's table slot goes beside its entry (the hit region's second half,
  // unused by 4-B entries), then both waves place the hits into LDS images of the table, 3 072 slots at a
  // time, each written out coalesced -- instead of one scattered 4-B store per hit.
  uint32_t* table = table_all + P.table_offset;
  uint32_t* slotarr = hitlist32 + P.hit_cap;
  const uint32_t chrpos0 = P.plusp ? P.chrstart : (P.chrhigh - P.chroffset) - P.chrend;
  const int idbits = U > 1 ? 32 - __clz(U - 1) : 1;
  __threadfence_block();
  for (int c = 0; wave == 0 && c < nhits; c += 64) {
    const int sl = c + lane;  // sl-th hit in store order: plus walks the list backwards
    int id = -1;
    uint32_t k = 0, at = 0;
    if (sl < nhits) {
      // ascending position: wave 0's list, then wave 1's from the list's end backwards
      const int a = P.plusp ? nhits - 1 - sl : sl;
      at = a < n0 ? (uint32_t)a : P.hit_cap - 1 - (uint32_t)(a - n0);
      if (compact) {
        const uint32_t e = hitlist32[at];
        k = e >> 14;
        id = (int)(e & 0x3FFFu);
      } else {
        const uint2 hv = hitlist[at];
        k = hv.x;
        id = (int)hv.y;
      }
    }
    const uint64_t hits = ballot(id >= 0);
    // lane order = store order: a hit's rank among the chunk's hits of its oligo (ballot match on the
    // id bits) is how many of that oligo's remaining slots the lower lanes take first
    uint64_t eq = hits;
    for (int b = 0; b < idbits; b++) {
      const uint64_t m = ballot((id >> b) & 1);
      eq &= ((id >> b) & 1) ? m : ~m;
    }
    if (id >= 0) {
      const int rank = lanes_below(eq, lane);
      const int same = __popcll(eq);
      const int r0 = (int)cnt[id];  // every lane reads before the first lane of each oligo writes
      const uint32_t slot = (uint32_t)offs[id] + (uint32_t)(r0 - rank - 1);
      if (kOiStage && compact)
        slotarr[at] = r0 - rank > 0 ? slot : 0xFFFFFFFFu;
      else if (r0 - rank > 0)
        table[slot] = chrpos0 + (P.plusp ? k : (uint32_t)(npos - 1) - k);
      if (rank == 0) cnt[id] = (CT)max(r0 - same, 0);
    }
  }
  __threadfence_block();
  __syncthreads();
  if (kOiStage && compact) {  // every slot of [0, tot) is some hit's (a wrapped count keeps its first count & 255 hits)
    uint32_t* stage = reinterpret_cast<uint32_t*>(smem);  // the bitmap and ranks (12 KB)
    constexpr uint32_t kStage = 6 * kOiWords / 4;
    for (uint32_t b0 = 0; b0 < tot; b0 += kStage) {
      for (int a = tid; a < nhits; a += 64 * kOiWaves) {
        const uint32_t at = a < n0 ? (uint32_t)a : P.hit_cap - 1 - (uint32_t)(a - n0);
        const uint32_t sd = slotarr[at] - b0;
        if (sd < kStage) {
          const uint32_t k = hitlist32[at] >> 14;
          stage[sd] = chrpos0 + (P.plusp ? k : (uint32_t)(npos - 1) - k);
        }
      }
      __syncthreads();
      const uint32_t nb = min(kStage, tot - b0);
      for (uint32_t j = tid; j < nb; j += 64 * kOiWaves) table[b0 + j] = stage[j];
      __syncthreads();
    }
  }
  // the per-id counts again (nhits of lookup, :34074)
  OI_MARK(3);
  for (int u = tid; u < U; u += 64 * kOiWaves)
    cnt[u] = (CT)((u + 1 < U ? (uint32_t)offs[u + 1] : tot) - (uint32_t)offs[u]);
  __threadfence_block();
  __syncthreads();
  if (wave) return;  // the rest runs in query order on wave 0

  // ---- Oligoindex_get_mappings ----
  gmapdp_oligo_result res;
  res.totalpositions = 0;
  res.maxnconsecutive = 0;
  res.oned_matrix_p = 0;
  res.ndiagonals = 0;
  res.table_offset = P.table_offset;
  res.diag_offset = P.diag_offset;
  __threadfence_block();
  // per querypos: nhits and table offset; cum_nohits as an inclusive prefix count of the positions
  // whose 8-mer has no hit (a position without a full 8-mer carries it forward)
  int* cum = reinterpret_cast<int*>(base_s);
  int totalpositions = 0, cumrun = 0;
  for (int sb = 0; sb < nq; sb += 4 * 64) {  // 256 query positions per step, loads issued together
    int mm[4];
#pragma unroll
    for (int r = 0; r < 4; r++) {
      const int i = sb + 64 * r + lane;
      mm[r] = i < nq ? mpq[i] : -1;
    }
#pragma unroll
    for (int r = 0; r < 4; r++) {
      const int i = sb + 64 * r + lane;
      const int m = mm[r];
      int nh = -1;
      if (i < nq) {
        int mo = -1;
        if (m >= 0) {
          const int u = m;  // (the id, converted after pass 1)
          nh = (int)cnt[u];
          npq[i] = nh;
          if (nh > 0) mo = (int32_t)(uint32_t)offs[u];  // relative to the problem's table
        }
        mpq[i] = mo;
      }
      const int incl = wave_scan_add(lane, nh == 0 ? 1 : 0);
      if (i < nq) cum[i] = cumrun + incl;
      cumrun += __builtin_amdgcn_readlane(incl, 63);
      totalpositions += __builtin_amdgcn_readlane(wave_scan_add(lane, nh > 0 ? nh : 0), 63);
    }
  }
  __threadfence_block();
  res.totalpositions = totalpositions;
  if (lane == 0) {
    results[P.index] = res;
    // get_mappings' event pool: taken here, as the waves finish at scattered times, rather than by
    // every oi_map_kernel wave at once on one address
    unsigned long long b = ~0ull;
    if (P.chrend > P.chrstart) {
      const unsigned long long need = 3ull * (unsigned long long)totalpositions;
      b = atomicAdd(pool_counter, need);
      if (b + need > pool_cap) b = ~0ull;
    }
    *reinterpret_cast<unsigned long long*>(base_s + so.poolbase) = b;
  }
  OI_MARK(4);
#ifdef GMAPDP_OI_TIMING
  if (lane == 0 && P.index < 16384) g_oi_wave[0][P.index] = (unsigned int)(wall_clock64() - oi_t0);
#endif
}

// get_mappings by the reference's sequential walk, for a problem the event pool could not take: per-diagonal
// states in the problem's fallback region (DevOligoProblem.fallback_offset), hits of one query position in
// parallel lanes.  Returns false when the problem has no such region (a plan sized from a measured run has
// an exact pool and none: the caller reports the overflow).  ngood -1: more good diagonals than diag_cap.
__device__ bool oi_mappings_walk(int lane, const DevOligoProblem& P, unsigned char* __restrict__ scratch, int qlen,
                                 int nq, const int32_t* __restrict__ npq, const int32_t* __restrict__ mpq,
                                 const int* __restrict__ cum, const uint32_t* __restrict__ table, uint32_t chrinit,
                                 int diag_lookback, int suffn, int32_t* __restrict__ good, int& ngood_out,
                                 int& maxn_out) {
  if (P.fallback_offset < 0) return false;
  const ScratchOiFb fb = scratch_oi_fb(qlen, P.chrend - P.chrstart);
  unsigned char* initp = scratch + P.fallback_offset + fb.initp;
  OiState* st = reinterpret_cast<OiState*>(scratch + P.fallback_offset + fb.states);
  for (size_t b = 16 * (size_t)lane; b < fb.states - fb.initp; b += 16 * 64)
    *reinterpret_cast<uint4*>(initp + b) = make_uint4(0u, 0u, 0u, 0u);
  __threadfence_block();
  int best = -1;  // diagi of each good diagonal goes in field 0 of its record first
  int ngood = 0, maxn = 0;
  // query positions in chunks of 64: one coalesced load of their nhits, table offsets, cum_nohits
  // and first hits, then the sequential walk takes them by readlane (off the latency chain)
  for (int cb = 0; cb < nq; cb += 64) {
    const int qi = cb + lane;
    int c_nh = 0, c_mo = 0, c_cum = 0;
    uint32_t c_h0 = 0;
    if (qi < nq) {
      c_nh = npq[qi];
      c_mo = mpq[qi];
      c_cum = cum[qi];
      if (c_nh > 0) c_h0 = table[c_mo];
    }
    const int cend = min(64, nq - cb);
    for (int j = 0; j < cend; j++) {
      const int nh = __builtin_amdgcn_readlane(c_nh, j);
      if (nh <= 0) continue;
      const int q = cb + j;
      const int mo = __builtin_amdgcn_readlane(c_mo, j);
      const int cq = __builtin_amdgcn_readlane(c_cum, j);
      const uint32_t h0 = (uint32_t)__builtin_amdgcn_readlane((int)c_h0, j);
      for (int base = 0; base < nh; base += 64) {
        const int h = base + lane;
        int reached = 0, nb = 0;
        uint32_t diagi = 0;
        if (h < nh) {
          diagi = (h == 0 ? h0 : table[mo + h]) + (uint32_t)(qlen - q) - chrinit;
          const unsigned char ini = initp[diagi];
          OiState s = st[diagi];  // loaded with the flag; ignored when the flag is clear
          if (!ini) {
            initp[diagi] = 1;
            s.querypos = -diag_lookback;  // the first check is never consecutive
            s.best_n = s.n = s.cstart = s.best_start = s.best_end = 0;
          }
          if (s.querypos < 0) {
            s.n = 0;
            s.cstart = q;
          } else if (q - s.querypos >= diag_lookback + cq - cum[s.querypos]) {
            s.n = 0;
            s.cstart = q;
          } else if (++s.n > s.best_n) {
            s.best_start = s.cstart;
            s.best_end = q;
            s.best_n = s.n;
            reached = (s.best_n == suffn);
            nb = s.best_n;
          }
          s.querypos = q;
          st[diagi] = s;
        }
        // the good list in lane order; the global best: the first lane reaching the new maximum
        const uint64_t rm = ballot(reached);
        if (reached && ngood + lanes_below(rm, lane) < (int)min(P.diag_cap, 0x7fffffffu))
          good[4 * (ngood + lanes_below(rm, lane))] = (int32_t)diagi;
        ngood += __popcll(rm);
        int mx = nb;
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) mx = max(mx, __shfl_xor(mx, off, 64));
        if (mx > maxn) {
          const int l = __ffsll((long long)ballot(nb == mx)) - 1;
          best = __builtin_amdgcn_readlane((int)diagi, l);
          maxn = mx;
        }
      }
    }
  }
  if (ngood == 0 && maxn > 0) {
    if (lane == 0 && P.diag_cap > 0) good[0] = best;
    ngood = 1;
  }
  __threadfence_block();
  if ((uint32_t)ngood > P.diag_cap) ngood = -1;  // more diagonals than the layout gave: overflow
  for (int g = lane; g < ngood; g += 64) {
    const int di = good[4 * g];
    const OiState s = st[di];
    good[4 * g + 0] = di >= qlen ? di - qlen : qlen - di;
    good[4 * g + 1] = s.best_start;
    good[4 * g + 2] = s.best_end;
    good[4 * g + 3] = s.best_n + 1;
  }
  ngood_out = ngood;
  maxn_out = maxn;
  return true;
}

// get_mappings over the global event pool (oi_mappings_sorted with the key format the problem's shape
// allows), else the sequential walk; writes the result's maxnconsecutive / oned_matrix_p / ndiagonals.
// kSlots: the slot filter over `slots` (oi_map_kernel; oi_build_kernel's fallback goes without, which keeps
// that kernel's registers within its occupancy bound)
template <bool kSlots>
__device__ void oi_mappings_global(int lane, const DevOligoProblem& P, unsigned char* __restrict__ scratch, int qlen,
                                   int nq, int E, const int32_t* __restrict__ npq, const int32_t* __restrict__ mpq,
                                   const int* __restrict__ cum, const uint32_t* __restrict__ table,
                                   uint64_t* __restrict__ pool, unsigned long long pbase, uint32_t* hist, int* evq,
                                   int32_t* __restrict__ good, gmapdp_oligo_result* __restrict__ results,
                                   uint32_t* slots = nullptr) {
  const int diag_lookback = P.minor ? 60 : 120, suffn = P.minor ? 10 : 20;
  const uint32_t chrinit = P.plusp ? P.chrstart : (P.chrhigh - P.chroffset) - P.chrend;
  int ngood = 0, maxn = 0;
  const uint32_t maxdiag = (uint32_t)qlen + (P.chrend - P.chrstart);
  const int gcap = (int)min(P.diag_cap, 0x7fffffffu);
  const bool sorted =
      maxdiag < (1u << 20) - 1 && nq <= 4096
          ? oi_mappings_sorted<OiKeyT32, kSlots>(lane, qlen, nq, E, maxdiag, chrinit, diag_lookback, suffn, npq, mpq, cum,
                                         table, pool, pbase, hist, evq, good, gcap, ngood, maxn, slots)
      : nq < 65536
          ? oi_mappings_sorted<OiKeyQT, kSlots>(lane, qlen, nq, E, maxdiag, chrinit, diag_lookback, suffn, npq, mpq, cum,
                                        table, pool, pbase, hist, evq, good, gcap, ngood, maxn, slots)
          : oi_mappings_sorted<OiKeyQ, kSlots>(lane, qlen, nq, E, maxdiag, chrinit, diag_lookback, suffn, npq, mpq, cum,
                                       table, pool, pbase, hist, evq, good, gcap, ngood, maxn, slots);
  if (!sorted && !oi_mappings_walk(lane, P, scratch, qlen, nq, npq, mpq, cum, table, chrinit, diag_lookback, suffn,
                                   good, ngood, maxn))
    ngood = -1;  // no pool slot and no fallback region: Stage2_compute answers GMAPDP overflow (status -2)
  if (lane == 0) {
    results[P.index].maxnconsecutive = ngood < 0 ? 0 : maxn;
    results[P.index].oned_matrix_p = ngood < 0 ? -1 : 1;
    results[P.index].ndiagonals = max(ngood, 0);
  }
}

// The plan runs' kernel, and the same code under another name for a stage-2 plan's sizing run (nhits_out
// set), so that a profile of the bench tells the plan's one-time sizing dispatches from its step's.
template <typename CT>
__global__ __launch_bounds__(64 * kOiWaves) void oi_kernel(OI_PASS_ARGS) {
  oi_pass<CT>(probs, blocks, quc_all, scratch, results, npos_out, map_out, table_all, pool_counter, pool_cap,
              nhits_out);
}
template <typename CT>
__global__ __launch_bounds__(64 * kOiWaves) void oi_size_kernel(OI_PASS_ARGS) {
  oi_pass<CT>(probs, blocks, quc_all, scratch, results, npos_out, map_out, table_all, pool_counter, pool_cap,
              nhits_out);
}

// ---- Oligoindex_get_mappings' diagonal state machine, one wave per problem, after oi_kernel ----
// A kernel of its own: its only LDS is the radix histogram and the event step's offsets, so many more
// waves share a CU and hide the L2 latency of the event passes than oi_kernel's query tables would allow.
#define OI_MAP_ARGS                                                                                           \
  const DevOligoProblem *__restrict__ probs, unsigned char *__restrict__ scratch,                                 \
      gmapdp_oligo_result *__restrict__ results, const int32_t *__restrict__ npos_out,                            \
      const int32_t *__restrict__ map_out, const uint32_t *__restrict__ table_all, int32_t *__restrict__ diag_all, \
      uint64_t *__restrict__ pool
__device__ __forceinline__ void oi_map_pass(OI_MAP_ARGS) {
  __shared__ uint32_t hist[kOiHist];
  __shared__ int evq[3 * 256];
  __shared__ uint32_t slots[kOimSlots / 2];
  const int lane = threadIdx.x;
  const DevOligoProblem P = probs[blockIdx.x];
  if (P.chrend <= P.chrstart) return;  // oned_matrix_p stays 0 (oi_kernel wrote the record)
  if (results[P.index].oned_matrix_p < 0) return;  // oi_kernel reported overflow
  OI_MARK(8);
#ifdef GMAPDP_OI_TIMING
  const unsigned long long om_t0 = wall_clock64();
#endif
  const int qlen = P.querylength;
  const int nq = qlen - kOiK + 1;
  unsigned char* base_s = scratch + P.scratch_offset;
  const ScratchOi so = scratch_oi(qlen, P.chrend - P.chrstart);
  const int totalpositions = results[P.index].totalpositions;
  oi_mappings_global<true>(lane, P, scratch, qlen, nq, totalpositions, npos_out + P.qoff, map_out + P.qoff,
                     reinterpret_cast<const int*>(base_s), table_all + P.table_offset, pool,
                     *reinterpret_cast<const unsigned long long*>(base_s + so.poolbase), hist, evq,
                     diag_all + 4 * P.diag_offset, results, slots);
  OI_MARK(7);
#ifdef GMAPDP_OI_TIMING
  if (lane == 0 && P.index < 16384) {
    g_oi_wave[1][P.index] = (unsigned int)(wall_clock64() - om_t0);
    g_oi_wave[2][P.index] = (unsigned int)totalpositions;
  }
#endif
}

__global__ __launch_bounds__(64) void oi_map_kernel(OI_MAP_ARGS) {
  oi_map_pass(probs, scratch, results, npos_out, map_out, table_all, diag_all, pool);
}
__global__ __launch_bounds__(64) void oi_size_map_kernel(OI_MAP_ARGS) {  // a sizing run's (see oi_size_kernel)
  oi_map_pass(probs, scratch, results, npos_out, map_out, table_all, diag_all, pool);
}

// ---- the split seeding: oi_scan_kernel (the query's 8-mers, the window scan) + oi_build_kernel ----
// oi_kernel above writes each table entry with a scattered 4-B store (pass 2) and oi_map_kernel radix-sorts
// every event through the global pool (two scattered passes): partial cache lines, ~8x the seeding's
// algorithmic write bytes.  The split path keeps both scatters in LDS:
//   oi_scan_kernel (2 waves, 12 KB LDS: the bitmap and its ranks only) -- Oligoindex_set_inquery, each query
//     position's 8-mer id, and pass 1's hit list (4 B per hit when the window has at most 2^18 starts);
//   oi_build_kernel (4 waves) -- counts from the hit list, the table layout, pass 2's placement into an LDS
//     image of the table (written out coalesced), npositions / mappings / cum_nohits, then get_mappings:
//     the events counted per diagonal slot (a hash of the diagonal) in LDS; a good diagonal has at least
//     suffn + 1 events, so only the events of slots that reach that count are candidates (the answer is
//     exact when the sweep finds a good diagonal with n >= suffn; otherwise the call is swept again over
//     every event); they are emitted in query order into LDS, radix-sorted there and swept as
//     oi_mappings_sorted does.  A problem whose table or candidates do not fit its LDS falls back to the
//     global paths above.
// The synchronous batch APIs take this path; the device-resident plans (bench.py's step) keep oi_kernel +
// oi_map_kernel, which share the CUs with the DP launches better; oi_map_kernel applies the
// same slot filter to its global event sort.

// the query's 8-mers 256 positions at a time (one coalesced character load per lane and chunk, 5 chunks:
// the last supplies the 7-character overlap; the 8-mer at i takes the codes of lanes i..i+7): f(i, ok, m)
template <typename F>
__device__ __forceinline__ void oi_query_oligos(int lane, const char* __restrict__ quc, int qlen, int nq, int sb,
                                                F&& f) {
  int ch[5];
#pragma unroll
  for (int r = 0; r < 5; r++) {
    const int i = sb + 64 * r + lane;
    ch[r] = i < qlen ? nt_code(quc[i]) : -1;
  }
#pragma unroll
  for (int r = 0; r < 4; r++) {
    const int i = sb + 64 * r + lane;
    uint32_t m = 0;
    bool ok = i < nq;
#pragma unroll
    for (int j = 0; j < kOiK; j++) {
      const int src = (lane + j) & 63;
      const int a = __shfl(ch[r], src, 64), b = __shfl(ch[r + 1], src, 64);
      const int cj = lane + j < 64 ? a : b;
      ok = ok && cj >= 0;
      m = (m << 2) | ((uint32_t)cj & 3u);
    }
    f(i, ok, m);
  }
}

struct OiWindow {
  uint64_t left, lpl, npos;
  bool compact;  // hit-list entries as (window index << 14 | id): at most 2^18 starts, ids < 2^14
};
__device__ __forceinline__ OiWindow oi_window(const DevOligoProblem& P) {
  OiWindow w;
  w.left = (uint64_t)P.chroffset + P.chrstart;
  uint64_t lpl = (uint64_t)P.chroffset + P.chrend + (P.plusp ? 0 : 1);
  w.lpl = lpl < (uint64_t)kOiK ? 0 : lpl - kOiK;
  w.npos = w.lpl > w.left ? w.lpl - w.left + 1 : 0;
  w.compact = w.npos <= (1ull << 18);
  return w;
}

__global__ __launch_bounds__(64 * kOiWaves) void oi_scan_kernel(
    const DevOligoProblem* __restrict__ probs, const uint32_t* __restrict__ blocks, const char* __restrict__ quc_all,
    unsigned char* __restrict__ scratch, int32_t* __restrict__ npos_out, int32_t* __restrict__ map_out) {
  __shared__ uint32_t bitmap[kOiWords];
  __shared__ uint16_t wrank[kOiWords];  // set bits before word w
  __shared__ int nh_wave[kOiWaves];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const DevOligoProblem P = probs[blockIdx.x];
  const char* quc = quc_all + P.qoff;
  const int qlen = P.querylength;
  const int nq = qlen - kOiK + 1;
  OI_MARK(10);
  for (int w = tid; w < kOiWords; w += 64 * kOiWaves) bitmap[w] = 0u;
  __syncthreads();
  for (int sb = 4 * 64 * wave; sb < qlen; sb += 4 * 64 * kOiWaves)
    oi_query_oligos(lane, quc, qlen, nq, sb, [&](int, bool ok, uint32_t m) {
      if (ok) atomicOr(&bitmap[m >> 5], 1u << (m & 31));
    });
  __syncthreads();
  int run = 0;  // ids in oligo order: prefix popcounts over the bitmap words
  for (int base = 0; base < kOiWords; base += 64) {
    const int c = __popc(bitmap[base + lane]);
    const int incl = wave_scan_add(lane, c);
    if (wave == 0) wrank[base + lane] = (uint16_t)(run + incl - c);
    run += __builtin_amdgcn_readlane(incl, 63);
  }
  const int U = run;
  __syncthreads();
  // each query position's 8-mer id (-1: none), npositions 0 (oi_build_kernel turns the ids into mappings)
  int32_t* npq = npos_out + P.qoff;
  int32_t* mpq = map_out + P.qoff;
  for (int sb = 4 * 64 * wave; sb < qlen; sb += 4 * 64 * kOiWaves)
    oi_query_oligos(lane, quc, qlen, nq, sb, [&](int i, bool ok, uint32_t m) {
      if (i < qlen) {
        bool in;
        mpq[i] = ok ? oligo_id(bitmap, wrank, m, in) : -1;
        npq[i] = 0;
      }
    });

  // ---- pass 1: the window's hits in ascending position (no counts: oi_build_kernel counts the list) ----
  const OiWindow W = oi_window(P);
  const uint64_t left = W.left, lpl = W.lpl;
  unsigned char* base_s = scratch + P.scratch_offset;
  const ScratchOi so = scratch_oi(qlen, P.chrend > P.chrstart ? P.chrend - P.chrstart : 0);
  uint32_t* hl32 = reinterpret_cast<uint32_t*>(base_s + so.hits);
  uint2* hl64 = reinterpret_cast<uint2*>(base_s + so.hits);
  int nhits = 0;
  if (W.npos > 0) {
    // this wave's steps of 64 half-words: wave 0 the first half of the window's, wave 1 the rest
    const uint64_t hlo0 = left >> 4, hhi0 = lpl >> 4;
    const uint64_t nsteps = (hhi0 - hlo0) / 64 + 1, half = (nsteps + 1) / 2;
    const uint64_t hlo = hlo0 + (wave ? 64 * half : 0);
    const uint64_t hhi = wave ? hhi0 : (hlo0 + 64 * half - 1 < hhi0 ? hlo0 + 64 * half - 1 : hhi0);
    constexpr int kOiAhead = 4;  // half-words of the next steps in flight
    uint32_t pw0[kOiAhead], pw1[kOiAhead];
#pragma unroll
    for (int a = 0; a < kOiAhead; a++) {
      const uint64_t hh = hlo + 64 * a + lane;
      pw0[a] = hh <= hhi ? half_word(blocks, hh) : 0u;
      pw1[a] = hh <= hhi ? half_word(blocks, hh + 1) : 0u;
    }
    auto step = [&](uint64_t hb, uint64_t v) {
      const uint64_t h = hb + lane;
      uint64_t vv;  // plus strand: the 2-bit groups of the 32 nt reversed once; minus: the complement as read
      if (P.plusp) {
        vv = ((v >> 2) & 0x3333333333333333ull) | ((v & 0x3333333333333333ull) << 2);
        vv = ((vv >> 4) & 0x0F0F0F0F0F0F0F0Full) | ((vv & 0x0F0F0F0F0F0F0F0Full) << 4);
        vv = __builtin_bswap64(vv);
      } else {
        vv = ~v;
      }
      auto oligo_at = [&](int j) -> uint32_t {
        return (uint32_t)(vv >> (P.plusp ? 2 * (24 - j) : 2 * j)) & 0xFFFFu;
      };
      uint32_t vmask = 0;  // the starts of this half-word inside [left, lpl]
      if (h <= hhi) {
        const uint64_t p0 = 16 * h;
        const int jlo = left > p0 ? (int)(left - p0) : 0;
        const int jhi = lpl < p0 + 15 ? (int)(lpl - p0) : 15;
        if (jlo <= jhi) vmask = (0xFFFFu >> (15 - jhi)) & (0xFFFFu << jlo);
      }
      uint32_t hm = 0;
#pragma unroll
      for (int j = 0; j < 16; j++) {
        const uint32_t m = oligo_at(j);
        hm |= ((bitmap[m >> 5] >> (m & 31)) & 1u) << j;
      }
      hm &= vmask;
      const int c = __popc(hm);
      const int incl = wave_scan_add(lane, c);
      int o = nhits + incl - c;
      for (uint32_t r = hm; r; r &= r - 1) {
        const int j = __ffs(r) - 1;
        bool in;
        const int id = oligo_id(bitmap, wrank, oligo_at(j), in);
        const uint32_t k = (uint32_t)(16 * h + j - left);
        // wave 0 from the start of the list, wave 1 from its end (its k-th hit at hit_cap - 1 - k)
        if ((uint32_t)o < P.hit_cap) {
          const uint32_t at = wave ? P.hit_cap - 1 - (uint32_t)o : (uint32_t)o;
          if (W.compact) hl32[at] = (k << 14) | (uint32_t)id;
          else hl64[at] = make_uint2(k, (uint32_t)id);
        }
        o++;
      }
      nhits += __builtin_amdgcn_readlane(incl, 63);
    };
    for (uint64_t hb0 = hlo; hlo <= hhi && hb0 <= hhi; hb0 += 64 * kOiAhead) {
#pragma unroll
      for (int a = 0; a < kOiAhead; a++) {
        const uint64_t hb = hb0 + 64 * a;
        if (hb > hhi) break;
        const uint64_t v = (uint64_t)pw0[a] | ((uint64_t)pw1[a] << 32);
        const uint64_t hh = hb + 64 * kOiAhead + lane;
        pw0[a] = hh <= hhi ? half_word(blocks, hh) : 0u;
        pw1[a] = hh <= hhi ? half_word(blocks, hh + 1) : 0u;
        step(hb, v);
      }
    }
  }
  if (lane == 0) nh_wave[wave] = nhits;
  __syncthreads();
  if (tid == 0) {
    OiMeta* meta = reinterpret_cast<OiMeta*>(base_s + so.poolbase);
    meta->n0 = nh_wave[0];
    meta->nhits = nh_wave[0] + nh_wave[1];
    meta->U = U;
  }
  OI_MARK(11);
}

// oi_build_kernel: kOibWaves waves per problem.  Its LDS: R2 (the per-id table offsets and counters; later
// the diagonal-slot counters and the radix histograms; last the good records) then the table image (tcap
// entries; later each wave's event step, and the two candidate buffers).
constexpr int kOibWaves = 4;
__host__ __device__ inline int oib_r2_bytes(int umax) { return 8 * umax > 16384 ? 8 * umax : 16384; }
constexpr int kOibSlots = 2048;  // 16-bit event counters per diagonal slot (4 KB)
__device__ __forceinline__ uint32_t oib_slot(uint32_t di) {
  return (di * 2654435761u) >> 21;  // Fibonacci hashing: the top 11 bits
}

// get_mappings on candidate events in LDS, the event passes on every wave of the workgroup, the sort and
// the sweep on wave 0.  Returns (to every wave) false when the candidates do not fit or no diagonal is good:
// the caller's wave 0 then takes the global path (what this wrote to `good` is rewritten there).
// A good diagonal holds at least suffn + 1 events.  Every event's diagonal is counted in a slot (a hash of
// the diagonal; no counter wraps below 2^16 events); an event whose slot holds fewer than suffn + 1 events
// cannot be on a good diagonal, so the candidates -- the events of well-filled slots, in query order --
// contain every event of every good diagonal.  When at least one diagonal is good, maxnconsecutive is
// reached on a good diagonal (n >= suffn there), and the good list, its records and that maximum are
// exactly what the full event set gives.  With no good diagonal the answer is the best of all diagonals,
// which the candidates may not hold: the global path answers it.  On a 214-kb window the candidates are
// the read's locus diagonals (~2 000 of ~8 300 events).
template <typename KT>
__device__ bool oi_mappings_lds(int tid, int qlen, int nq, int E, uint32_t maxdiag, uint32_t chrinit, int lookback,
                                int suffn, const int32_t* __restrict__ npq, const int32_t* __restrict__ mpq,
                                const int* __restrict__ cum, const uint32_t* __restrict__ table,
                                unsigned char* r2, int r2_bytes, unsigned char* rt, int rt_bytes,
                                int32_t* __restrict__ good, int gcap, int& ngood_out, int& maxn_out) {
  using K = typename KT::K;
  __shared__ int wc[kOibWaves + 1];
  const int lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  if (E >= 65536) return false;  // (a slot counter could wrap)
  int* evq = reinterpret_cast<int*>(rt) + 3 * 256 * wave;  // each wave's event step
  const int cmax = (rt_bytes - 4 * 3 * 256 * kOibWaves) / (2 * (int)sizeof(K));
  if (cmax < 64) return false;
  uint32_t* slots = reinterpret_cast<uint32_t*>(r2);  // two 16-bit counters per word
  uint32_t* hist = slots + kOibSlots / 2;
  K* A = reinterpret_cast<K*>(rt + 4 * 3 * 256 * kOibWaves);
  K* Bf = A + cmax;
  for (int i = tid; i < kOibSlots / 2 + kOiHist; i += 64 * kOibWaves) slots[i] = 0u;
  __syncthreads();
  // every event's slot (order-free: each wave takes every kOibWaves-th step of 256 query positions)
  oi_for_events<KT>(lane, qlen, nq, chrinit, npq, mpq, cum, table, evq, [&](int, bool v, uint32_t di, K) {
    if (v) {
      const uint32_t h = oib_slot(di);
      atomicAdd(&slots[h >> 1], 1u << (16 * (h & 1)));
    }
  }, 4 * 64 * wave, 4 * 64 * kOibWaves);
  __syncthreads();
  OI_MARK(13);
  // the candidates in query order: per round each wave counts its step's, then writes them after the
  // earlier steps' (and counts their radix digits)
  const OiDigits D = oi_digits(maxdiag);
  const uint32_t need = (uint32_t)suffn + 1u;
  int C = 0;
  for (int r0 = 0; r0 < nq; r0 += 4 * 64 * kOibWaves) {
    const int sb = r0 + 4 * 64 * wave;
    int mine = 0;
    if (sb < nq)
      oi_for_events<KT>(lane, qlen, nq, chrinit, npq, mpq, cum, table, evq, [&](int, bool v, uint32_t di, K) {
        const uint32_t h = oib_slot(di);
        mine += __popcll(ballot(v && ((slots[h >> 1] >> (16 * (h & 1))) & 0xFFFFu) >= need));
      }, sb, 1 << 30);
    if (lane == 0) wc[wave] = mine;
    __syncthreads();
    int at = C;
    for (int w = 0; w < wave; w++) at += wc[w];
    for (int w = 0; w < kOibWaves; w++) C += wc[w];
    const bool fits = C <= cmax;  // (block-uniform)
    if (sb < nq && mine && fits)
      oi_for_events<KT>(lane, qlen, nq, chrinit, npq, mpq, cum, table, evq, [&](int, bool v, uint32_t di, K key) {
        const uint32_t h = oib_slot(di);
        const bool c = v && ((slots[h >> 1] >> (16 * (h & 1))) & 0xFFFFu) >= need;
        const uint64_t cm = ballot(c);
        if (c) A[at + lanes_below(cm, lane)] = key;
        oi_hist_add(lane, c, di, D, hist);
        at += __popcll(cm);
      }, sb, 1 << 30);
    __syncthreads();
  }
  OI_MARK(14);
  if (C > cmax) return false;
  // the sort and the sweep on wave 0; the good records and their keys over R2 (the slot counters are dead;
  // a good diagonal holds suffn + 1 events, so at most C / (suffn + 1) + 1 records)
  const int gmax = C / (suffn + 1) + 1;
  if (24 * gmax + 4 * kOiHist + 4 * kOibSlots / 2 > r2_bytes) return false;
  if (wave == 0) {
    const K* S = oi_radix<KT>(lane, A, Bf, C, D, hist);
    int4* grec = reinterpret_cast<int4*>(r2 + 4 * kOiHist + 4 * kOibSlots / 2);
    uint64_t* gkey = reinterpret_cast<uint64_t*>(reinterpret_cast<unsigned char*>(grec) + 16 * (size_t)gmax);
    // (a candidate list with no good diagonal ends with the fallback record: not exact here)
    int maxn = 0;
    const int ngood = oi_sweep<KT>(lane, S, C, qlen, nq, lookback, suffn, cum, grec, gkey, good, gcap, maxn);
    if (lane == 0) {
      wc[0] = ngood;
      wc[1] = maxn;
    }
  }
  __syncthreads();
  OI_MARK(15);
  const int ngood = wc[0], maxn = wc[1];
  if (ngood != -1 && (ngood == 0 || maxn < suffn)) return false;
  ngood_out = ngood;
  maxn_out = maxn;
  return true;
}

__global__ __launch_bounds__(64 * kOibWaves, 3) void oi_build_kernel(
    const DevOligoProblem* __restrict__ probs, unsigned char* __restrict__ scratch,
    gmapdp_oligo_result* __restrict__ results, int32_t* __restrict__ npos_out, int32_t* __restrict__ map_out,
    uint32_t* __restrict__ table_all, int32_t* __restrict__ diag_all, uint64_t* __restrict__ pool,
    unsigned long long* __restrict__ pool_counter, unsigned long long pool_cap, int r2_bytes, int tcap) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  __shared__ uint32_t tot_s;
  __shared__ int flag_s, wn_s[kOibWaves], wt_s[kOibWaves];
  constexpr int NT = 64 * kOibWaves;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const DevOligoProblem P = probs[blockIdx.x];
  const int qlen = P.querylength;
  const int nq = qlen - kOiK + 1;
  int32_t* npq = npos_out + P.qoff;
  int32_t* mpq = map_out + P.qoff;
  unsigned char* base_s = scratch + P.scratch_offset;
  const ScratchOi so = scratch_oi(qlen, P.chrend > P.chrstart ? P.chrend - P.chrstart : 0);
  OiMeta* meta = reinterpret_cast<OiMeta*>(base_s + so.poolbase);
  const int n0 = __builtin_amdgcn_readfirstlane(meta->n0), nhits = __builtin_amdgcn_readfirstlane(meta->nhits);
  const int U = __builtin_amdgcn_readfirstlane(meta->U);
  OI_MARK(12);
  // more hits or distinct 8-mers than the layout gave the problem (a plan laid out from one query and run
  // on another): overflow, nothing written past the problem's slices
  if ((uint32_t)nhits > P.hit_cap || U > P.umax) {
    oi_report_overflow(P, tid, NT, qlen, npq, mpq, results, base_s + so.poolbase);
    return;
  }
  const OiWindow W = oi_window(P);
  const uint32_t* hl32 = reinterpret_cast<const uint32_t*>(base_s + so.hits);
  const uint2* hl64 = reinterpret_cast<const uint2*>(base_s + so.hits);
  // the a-th hit in ascending window position: wave 0's list, then wave 1's from the list's end backwards;
  // {window index, id}
  auto hit_at = [&](int a) __attribute__((always_inline)) -> uint2 {
    const uint32_t at = a < n0 ? (uint32_t)a : P.hit_cap - 1 - (uint32_t)(a - n0);
    if (W.compact) {
      const uint32_t e = hl32[at];
      return make_uint2(e >> 14, e & 0x3FFFu);
    }
    return hl64[at];
  };
  uint32_t* cnt = reinterpret_cast<uint32_t*>(smem);  // per id: count, then fill / remaining, then kept count
  uint32_t* offs = cnt + P.umax;                      // per id: table offset
  uint32_t* tl = reinterpret_cast<uint32_t*>(smem + r2_bytes);
  for (int u = tid; u < U; u += NT) cnt[u] = 0u;
  __syncthreads();
  for (int a0 = 0; a0 < nhits; a0 += 4 * NT) {  // the counts (Count_T: mod 256 below), 4 hits per thread a step
    int id[4];
#pragma unroll
    for (int r = 0; r < 4; r++) id[r] = a0 + NT * r + tid < nhits ? (int)hit_at(a0 + NT * r + tid).y : -1;
#pragma unroll
    for (int r = 0; r < 4; r++)
      if (id[r] >= 0) atomicAdd(&cnt[id[r]], 1u);
  }
  __syncthreads();
  OI_MARK(2);
  if (wave == 0) {  // the table layout in oligo order (Count_T wraps); any oligo past 255 hits?
    uint32_t tot = 0;
    bool wrapped = false;
    for (int base = 0; base < U; base += 64) {
      const int u = base + lane;
      const uint32_t full = u < U ? cnt[u] : 0u;
      const uint32_t c = full & 255u;
      wrapped = wrapped || full > 255u;
      const uint32_t incl = (uint32_t)wave_scan_add(lane, (int)c);
      if (u < U) {
        offs[u] = tot + incl - c;
        cnt[u] = c;
      }
      tot += (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
    }
    const bool any_wrap = ballot(wrapped) != 0;
    if (lane == 0) {
      tot_s = tot;
      flag_s = any_wrap ? 1 : 0;
    }
  }
  __syncthreads();
  const uint32_t tot = tot_s;
  if (tot > P.table_cap) {
    oi_report_overflow(P, tid, NT, qlen, npq, mpq, results, base_s + so.poolbase);
    return;
  }
  OI_MARK(3);
  // ---- pass 2: the table.  Each oligo keeps the K = count mod 256 occurrences nearest the store walk's
  // start (descending chrpos), stored in ascending chrpos.  With no count past 255 every occurrence is
  // kept: the hits go to their oligo's slice in any order (one LDS atomic each) and each slice is sorted
  // (slices hold a few entries).  Otherwise wave 0 walks the hits in store order (the reference's rule). ----
  uint32_t* table = table_all + P.table_offset;
  const uint32_t chrpos0 = P.plusp ? P.chrstart : (P.chrhigh - P.chroffset) - P.chrend;
  const bool in_lds = tot <= (uint32_t)tcap;
  const bool wrapped = flag_s != 0;
  auto chrpos_of = [&](uint32_t k) __attribute__((always_inline)) {
    return chrpos0 + (P.plusp ? k : (uint32_t)(W.npos - 1) - k);
  };
  if (in_lds && !wrapped) {
    for (int u = tid; u < U; u += NT) cnt[u] = 0u;  // fill counters
    __syncthreads();
    for (int a0 = 0; a0 < nhits; a0 += 4 * NT) {
      uint2 hv[4];
#pragma unroll
      for (int r = 0; r < 4; r++) hv[r] = a0 + NT * r + tid < nhits ? hit_at(a0 + NT * r + tid) : make_uint2(0u, ~0u);
#pragma unroll
      for (int r = 0; r < 4; r++)
        if (hv[r].y != ~0u) tl[offs[hv[r].y] + atomicAdd(&cnt[hv[r].y], 1u)] = chrpos_of(hv[r].x);
    }
    __syncthreads();
    for (int u = tid; u < U; u += NT) {  // insertion sort of each oligo's slice
      const uint32_t b = offs[u], n = cnt[u];
      for (uint32_t i = 1; i < n; i++) {
        const uint32_t x = tl[b + i];
        uint32_t j = i;
        while (j > 0 && tl[b + j - 1] > x) {
          tl[b + j] = tl[b + j - 1];
          j--;
        }
        tl[b + j] = x;
      }
    }
  } else if (wave == 0) {
    uint32_t* dst = in_lds ? tl : table;
    const int idbits = U > 1 ? 32 - __clz(U - 1) : 1;
    for (int c = 0; c < nhits; c += 64) {
      const int sl = c + lane;  // sl-th hit in store order: plus walks the list backwards
      int id = -1;
      uint32_t k = 0;
      if (sl < nhits) {
        const uint2 hv = hit_at(P.plusp ? nhits - 1 - sl : sl);
        k = hv.x;
        id = (int)hv.y;
      }
      // lane order = store order: a hit's rank among the chunk's hits of its oligo (ballot match on the id
      // bits) is how many of that oligo's remaining slots the lower lanes take first
      uint64_t eq = ballot(id >= 0);
      for (int b = 0; b < idbits; b++) {
        const uint64_t m = ballot((id >> b) & 1);
        eq &= ((id >> b) & 1) ? m : ~m;
      }
      if (id >= 0) {
        const int rank = lanes_below(eq, lane);
        const int same = __popcll(eq);
        const int r0 = (int)cnt[id];  // every lane reads before the first lane of each oligo writes
        if (r0 - rank > 0) dst[offs[id] + r0 - rank - 1] = chrpos_of(k);
        if (rank == 0) cnt[id] = (uint32_t)max(r0 - same, 0);
      }
    }
  }
  __syncthreads();
  if (in_lds)
    for (uint32_t t = tid; t < tot; t += NT) table[t] = tl[t];  // written out coalesced
  // the per-id counts again (nhits of lookup, :34074)
  for (int u = tid; u < U; u += NT) cnt[u] = (u + 1 < U ? offs[u + 1] : tot) - offs[u];
  __syncthreads();
  OI_MARK(4);

  // ---- Oligoindex_get_mappings: per querypos nhits and table offset, cum_nohits (an inclusive prefix
  // count of the positions whose 8-mer has no hit).  Each wave takes a quarter of the positions: their
  // totals first, then the writes after the earlier quarters' counts ----
  int* cum = reinterpret_cast<int*>(base_s);
  const int qper = ((nq + kOibWaves - 1) / kOibWaves + 63) & ~63;
  const int qlo = min(nq, qper * wave), qhi = min(nq, qlo + qper);
  auto nh_of = [&](int i, int& mo) __attribute__((always_inline)) {
    const int u = mpq[i];
    mo = -1;
    if (u < 0) return -1;
    const int nh = (int)cnt[u];
    if (nh > 0) mo = (int32_t)offs[u];  // relative to the problem's table
    return nh;
  };
  int nohit = 0, tp = 0;
  for (int i0 = qlo; i0 < qhi; i0 += 64) {
    int mo;
    const int nh = i0 + lane < qhi ? nh_of(i0 + lane, mo) : -1;
    nohit += __popcll(ballot(nh == 0));
    tp += __builtin_amdgcn_readlane(wave_scan_add(lane, nh > 0 ? nh : 0), 63);
  }
  if (lane == 0) {
    wn_s[wave] = nohit;
    wt_s[wave] = tp;
  }
  __syncthreads();
  int cumrun = 0, totalpositions = 0;
  for (int w = 0; w < kOibWaves; w++) {
    if (w < wave) cumrun += wn_s[w];
    totalpositions += wt_s[w];
  }
  for (int i0 = qlo; i0 < qhi; i0 += 64) {
    const int i = i0 + lane;
    int mo = -1, nh = -1;
    if (i < qhi) {
      nh = nh_of(i, mo);
      if (nh >= 0) npq[i] = nh;
    }
    const int incl = wave_scan_add(lane, nh == 0 ? 1 : 0);
    if (i < qhi) {  // (each lane reads and then rewrites its own position's slot)
      mpq[i] = mo;
      cum[i] = cumrun + incl;
    }
    cumrun += __builtin_amdgcn_readlane(incl, 63);
  }
  __threadfence_block();
  if (tid == 0) {
    gmapdp_oligo_result res;
    res.totalpositions = totalpositions;
    res.maxnconsecutive = 0;
    res.oned_matrix_p = 0;
    res.ndiagonals = 0;
    res.table_offset = P.table_offset;
    res.diag_offset = P.diag_offset;
    results[P.index] = res;
  }
  OI_MARK(5);
  if (P.chrend <= P.chrstart) return;  // oned_matrix_p stays 0 (:34157)
  const int E = totalpositions;
  const int diag_lookback = P.minor ? 60 : 120, suffn = P.minor ? 10 : 20;
  const uint32_t maxdiag = (uint32_t)qlen + (P.chrend - P.chrstart);
  int32_t* good = diag_all + 4 * P.diag_offset;
  const int gcap = (int)min(P.diag_cap, 0x7fffffffu);
  int ngood = 0, maxn = 0;
  bool done = false;
  __syncthreads();
  if (maxdiag < (1u << 20) - 1 && nq <= 4096)
    done = oi_mappings_lds<OiKeyT32>(tid, qlen, nq, E, maxdiag, chrpos0, diag_lookback, suffn, npq, mpq, cum, table,
                                     smem, r2_bytes, smem + r2_bytes, 4 * tcap, good, gcap, ngood, maxn);
  else if (nq < 65536)
    done = oi_mappings_lds<OiKeyQT>(tid, qlen, nq, E, maxdiag, chrpos0, diag_lookback, suffn, npq, mpq, cum, table,
                                    smem, r2_bytes, smem + r2_bytes, 4 * tcap, good, gcap, ngood, maxn);
  if (wave) return;  // the rest is wave 0's
  if (done) {
    if (lane == 0) {
      results[P.index].maxnconsecutive = ngood < 0 ? 0 : maxn;
      results[P.index].oned_matrix_p = ngood < 0 ? -1 : 1;
      results[P.index].ndiagonals = max(ngood, 0);
    }
    return;
  }
  // the candidates did not fit the LDS: the global event pool (3 E slots), else the sequential walk
  unsigned long long b = ~0ull;
  if (lane == 0) {
    const unsigned long long need = 3ull * (unsigned long long)E;
    b = atomicAdd(pool_counter, need);
    if (b + need > pool_cap) b = ~0ull;
  }
  b = ((unsigned long long)(uint32_t)__builtin_amdgcn_readfirstlane((int)(b >> 32)) << 32) |
      (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)b);
  oi_wave_sync();
  uint32_t* hist = reinterpret_cast<uint32_t*>(smem);
  int* evq = reinterpret_cast<int*>(smem + 4 * kOiHist);
  oi_mappings_global<false>(lane, P, scratch, qlen, nq, E, npq, mpq, cum, table, pool, b, hist, evq, good, results);
}

size_t lds_bytes_oib(int umax, int* tcap) {
  const int r2 = oib_r2_bytes(umax);
  // the table image: 9 472 entries keeps r2 + image within a third of the CU's LDS for 2-kb reads (3
  // workgroups per CU) and holds a 214-kb window's ~8 300 hits.  GMAPDP_OI_LDS_TABLE (tests) caps it: 0 sends
  // every table and every non-empty candidate list to the global paths.
  int t = (163840 - r2) / 4;
  int lim = 9472;
  if (const char* ev = std::getenv("GMAPDP_OI_LDS_TABLE")) lim = std::atoi(ev);
  if (t > lim) t = lim;
  *tcap = t < 0 ? 0 : t & ~63;
  return (size_t)r2 + 4 * (size_t)*tcap;
}

hipError_t launch_oi_split(int nproblems, int umax, hipStream_t stream, const DevOligoProblem* probs,
                           const uint32_t* blocks, const char* quc, unsigned char* scratch,
                           gmapdp_oligo_result* results, int32_t* npos, int32_t* map, uint32_t* table, int32_t* diags,
                           uint64_t* pool, unsigned long long* pool_counter, unsigned long long pool_cap) {
  int tcap = 0;
  const size_t lds = lds_bytes_oib(umax, &tcap);
  const int r2 = oib_r2_bytes(umax);
  if (lds > 64 * 1024) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<void*>(&oi_build_kernel),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
  }
  void* args[] = {(void*)&probs, (void*)&blocks, (void*)&quc, (void*)&scratch, (void*)&npos, (void*)&map};
  hipError_t e = hipLaunchKernel(reinterpret_cast<void*>(&oi_scan_kernel), dim3(nproblems), dim3(64 * kOiWaves), args,
                                 0, stream);
  if (e != hipSuccess) return e;
  void* bargs[] = {(void*)&probs, (void*)&scratch, (void*)&results, (void*)&npos, (void*)&map, (void*)&table,
                   (void*)&diags, (void*)&pool, (void*)&pool_counter, (void*)&pool_cap, (void*)&r2, (void*)&tcap};
  return hipLaunchKernel(reinterpret_cast<void*>(&oi_build_kernel), dim3(nproblems), dim3(64 * kOibWaves), bargs, lds,
                         stream);
}

#ifdef GMAPDP_OI_TIMING
extern "C" int gmapdp_debug_oi_waves(unsigned int* out) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_oi_wave), sizeof(g_oi_wave)) != hipSuccess;
}
// copies out and clears the marks: [0..15] timestamp sums (100 MHz), [16..31] wave counts
extern "C" int gmapdp_debug_oi_marks(unsigned long long* out) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_oi_marks), sizeof(g_oi_marks)) != hipSuccess) return 1;
  static const unsigned long long zero[2][16] = {};
  return hipMemcpyToSymbol(HIP_SYMBOL(g_oi_marks), zero, sizeof(zero)) != hipSuccess;
}
#endif

size_t lds_bytes_oi(int umax, bool wide) { return 6 * (size_t)kOiWords + (wide ? 8 : 4) * (size_t)umax; }
size_t scratch_bytes_oi(int querylength, uint32_t genomiclength) {
  return scratch_oi(querylength, genomiclength).total;
}
size_t scratch_bytes_oi_hits(int querylength, size_t hitcap) {  // a measured hit count instead of the window
  return align16(scratch_oi(querylength, 0).hits + 8 * (hitcap + 2));
}
size_t scratch_bytes_oi_fallback(int querylength, uint32_t genomiclength) {
  return scratch_oi_fb(querylength, genomiclength).total;
}

hipError_t launch_oi(bool wide, int nproblems, size_t lds, hipStream_t stream, const DevOligoProblem* probs,
                     const uint32_t* blocks, const char* quc, unsigned char* scratch, gmapdp_oligo_result* results,
                     int32_t* npos, int32_t* map, uint32_t* table, int32_t* diags, uint64_t* pool,
                     unsigned long long* pool_counter, unsigned long long pool_cap, int32_t* nhits_out) {
  const bool sizing = nhits_out != nullptr;  // a stage-2 plan's sizing run: the same code, its own names
  void* fn = sizing ? (wide ? reinterpret_cast<void*>(&oi_size_kernel<uint32_t>)
                            : reinterpret_cast<void*>(&oi_size_kernel<uint16_t>))
                    : (wide ? reinterpret_cast<void*>(&oi_kernel<uint32_t>)
                            : reinterpret_cast<void*>(&oi_kernel<uint16_t>));
  if (lds > 64 * 1024) {
    hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
  }
  void* args[] = {(void*)&probs, (void*)&blocks, (void*)&quc, (void*)&scratch, (void*)&results, (void*)&npos,
                  (void*)&map, (void*)&table, (void*)&pool_counter, (void*)&pool_cap, (void*)&nhits_out};
  hipError_t e = hipLaunchKernel(fn, dim3(nproblems), dim3(64 * kOiWaves), args, lds, stream);
  if (e != hipSuccess) return e;
  void* margs[] = {(void*)&probs, (void*)&scratch, (void*)&results, (void*)&npos, (void*)&map, (void*)&table,
                   (void*)&diags, (void*)&pool};
  return hipLaunchKernel(sizing ? reinterpret_cast<void*>(&oi_size_map_kernel) : reinterpret_cast<void*>(&oi_map_kernel),
                         dim3(nproblems), dim3(64), margs, 0, stream);
}

}  // namespace gmapdp
