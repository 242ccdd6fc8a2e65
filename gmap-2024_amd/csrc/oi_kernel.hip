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

// per-problem scratch: cum_nohits (querylength + 1 ints), the event-pool offset, the window's hit list
struct ScratchOi {
  size_t poolbase, hits, total;
};
__host__ __device__ inline ScratchOi scratch_oi(int querylength, uint32_t genomiclength) {
  ScratchOi s;
  s.poolbase = align16(4 * (size_t)(querylength + 1));  // the problem's event-pool offset (or ~0)
  s.hits = align16(s.poolbase + 8);
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

// Returns false (nothing written) when the shared event pool could not hold this problem's 3 E slots
// (oi_kernel took them, `base`, with one atomic as it finished).
// maxdiag bounds every diagi (querylength + genomiclength); hist holds kOiHist LDS counters: the digits
// are 9 bits wide when maxdiag < 2^18 (2 passes of 512 buckets: a 214-kb window), else 8 bits (at most 4
// passes of 256).  (More LDS would cost oi_map_kernel a wave per SIMD.)
template <typename KT>
__device__ bool oi_mappings_sorted(int lane, int qlen, int nq, int E, uint32_t maxdiag, uint32_t chrinit,
                                   int lookback, int suffn, const int32_t* __restrict__ npq,
                                   const int32_t* __restrict__ mpq, const int* __restrict__ cum,
                                   const uint32_t* __restrict__ table_all, uint64_t* __restrict__ pool,
                                   unsigned long long base, uint32_t* hist,
                                   int* evq, int32_t* __restrict__ good, int gcap, int& ngood_out, int& maxn_out) {
  OI_MARK(9);
  if (base == ~0ull) return false;
  using K = typename KT::K;
  constexpr K kMax = KT::kMax;
  K* evA = reinterpret_cast<K*>(pool + base);       // events (OiKeyT32 / OiKeyQT / OiKeyQ)
  K* evB = evA + E;                                 // radix-sort ping-pong
  int4* grec = reinterpret_cast<int4*>(pool + base + 2 * (size_t)E);  // good records (at most E / 2)
  const int db = maxdiag < (1u << 18) ? 9 : 8;       // digit bits
  const uint32_t dmask = (1u << db) - 1u;
  int npass = 0;                                    // digits of the largest possible diagi
  while (npass < 4 && (maxdiag >> (db * npass)) != 0) npass++;
  for (int i = lane; i < kOiHist; i += 64) hist[i] = 0u;
  __syncthreads();

  // Events in query order, hits of one querypos in table (ascending chrpos) order, 256 query
  // positions per step (their nhits / table offsets loaded a step ahead).  The step's exclusive event
  // offsets and table offsets go to LDS; each event finds its query position there by binary search,
  // 256 events at a time, so their table loads all issue together.  The digit histograms of every
  // radix pass are counted here, so the sort never re-reads the keys to count them.
  int* exo = evq;          // [256] exclusive event offset of each query position of the step
  int* mos = evq + 256;    // [256] its table offset
  int* cus = evq + 512;    // [256] its cum_nohits
  int eoff = 0;
  int nh_n[4], mo_n[4], cu_n[4];
#pragma unroll
  for (int r = 0; r < 4; r++) {
    const int q = 64 * r + lane;
    nh_n[r] = q < nq ? npq[q] : 0;
    mo_n[r] = q < nq ? mpq[q] : 0;
    cu_n[r] = q < nq ? cum[q] : 0;
  }
  for (int sb = 0; sb < nq; sb += 4 * 64) {
    int nh[4], mo[4], cu[4];
#pragma unroll
    for (int r = 0; r < 4; r++) {
      nh[r] = max(nh_n[r], 0);
      mo[r] = mo_n[r];
      cu[r] = cu_n[r];
      const int q = sb + 4 * 64 + 64 * r + lane;
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
    __syncthreads();
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
        const bool v = j < T;
        const uint32_t di = tv[gi] + (uint32_t)(qlen - qv[gi]) - chrinit;
        if (v) evA[eoff + j] = KT::make(di, (uint32_t)qv[gi], (uint32_t)(qv[gi] - cv[gi]));
        // one LDS atomic per distinct digit: the hits of a group mostly share a few diagonals, and
        // same-address atomics serialise
        for (int p = 0; p < npass; p++) {
          const uint32_t dg = (di >> (db * p)) & dmask;
          uint64_t eq = ballot(v);
#pragma unroll
          for (int b = 0; b < 9; b++) {  // (bit 8 of an 8-bit digit is 0 in every lane)
            const uint64_t m = ballot((dg >> b) & 1u);
            eq &= ((dg >> b) & 1u) ? m : ~m;
          }
          if (v && lanes_below(eq, lane) == 0) atomicAdd(&hist[(dmask + 1) * p + dg], (uint32_t)__popcll(eq));
        }
      }
    }
    eoff += T;
    __syncthreads();
  }
  __threadfence_block();
  __syncthreads();
  OI_MARK(5);

  // stable LSD radix sort on diagi
  K* src = evA;
  K* dst = evB;
  for (int p = 0; p < npass; p++) {
    uint32_t* hp = hist + (dmask + 1) * p;
    const int shift = db * p;
    const int cpl = (int)(dmask + 1) / 64;  // buckets per lane: 8 or 4
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
    __syncthreads();
    // 256 keys per step: their 4 loads and 4 stores each go out together (one memory round trip per
    // step); the ranks are taken chunk by chunk in order, which keeps the sort stable
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
        const uint32_t d = (KT::di(key[r]) >> shift) & dmask;
        uint64_t eq = ballot(v);
#pragma unroll
        for (int b = 0; b < 9; b++) {
          const uint64_t m = ballot((d >> b) & 1u);
          eq &= ((d >> b) & 1u) ? m : ~m;
        }
        const int rank = lanes_below(eq, lane);
        const uint32_t pos = v ? hp[d] : 0u;  // every lane reads before any lane bumps
        __syncthreads();
        dpos[r] = pos + (uint32_t)rank;
        if (v && rank == 0) hp[d] = pos + (uint32_t)__popcll(eq);
        __syncthreads();
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
  const K* S = src;
  __threadfence_block();
  OI_MARK(6);

  // Sweep: runs, each diagonal's maximum and its first event, the first event reaching suffn; a
  // diagonal's last event appends its record when it is good.  Per lane, the largest n seen and the
  // smallest (querypos, diagi) event carrying it (the fallback best).  Nothing is stored per event.
  int c_rs = -1, c_ds = -1, c_fs = 0x7fffffff, ngood = 0;
  uint64_t c_mk = 0;
  K c_key = 0;
  int bm = -1, be = -1;
  uint64_t bkey = ~0ull;
  // 256 events per step: their key loads, then their cum_nohits loads, go out together (two memory
  // round trips per step); the 4 chunks are then scanned in order with the carries
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
  // the good diagonals' query-order keys: the free sort buffer (64-bit events), or the pool's second E
  // words (32-bit events: both sort buffers sit in the first)
  uint64_t* gkey = sizeof(K) == 8 ? reinterpret_cast<uint64_t*>(S == evA ? evB : evA) : pool + base + E;
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
  ngood_out = ngood;
  maxn_out = M;
  return true;
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

template <typename CT>
__global__ __launch_bounds__(64 * kOiWaves) void oi_kernel(
    const DevOligoProblem* __restrict__ probs, const uint32_t* __restrict__ blocks, const char* __restrict__ quc_all,
    unsigned char* __restrict__ scratch, gmapdp_oligo_result* __restrict__ results, int32_t* __restrict__ npos_out,
    int32_t* __restrict__ map_out, uint32_t* __restrict__ table_all, unsigned long long* __restrict__ pool_counter,
    unsigned long long pool_cap, int32_t* __restrict__ nhits_out) {
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
        if ((uint32_t)o < P.hit_cap)
          hitlist[wave ? P.hit_cap - 1 - (uint32_t)o : (uint32_t)o] =
              make_uint2((uint32_t)(16 * h + j - left), (uint32_t)id);
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
  uint32_t* table = table_all + P.table_offset;
  const uint32_t chrpos0 = P.plusp ? P.chrstart : (P.chrhigh - P.chroffset) - P.chrend;
  const int idbits = U > 1 ? 32 - __clz(U - 1) : 1;
  __threadfence_block();
  for (int c = 0; wave == 0 && c < nhits; c += 64) {
    const int sl = c + lane;  // sl-th hit in store order: plus walks the list backwards
    int id = -1;
    uint32_t k = 0;
    if (sl < nhits) {
      // ascending position: wave 0's list, then wave 1's from the list's end backwards
      const int a = P.plusp ? nhits - 1 - sl : sl;
      const uint2 hv = hitlist[a < n0 ? (uint32_t)a : P.hit_cap - 1 - (uint32_t)(a - n0)];
      k = hv.x;
      id = (int)hv.y;
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
      if (r0 - rank > 0)
        table[offs[id] + r0 - rank - 1] = chrpos0 + (P.plusp ? k : (uint32_t)(npos - 1) - k);
      if (rank == 0) cnt[id] = (CT)max(r0 - same, 0);
    }
  }
  __syncthreads();
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
          bool in;
          const int u = oligo_id(bitmap, wrank, (uint32_t)m, in);
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

// ---- Oligoindex_get_mappings' diagonal state machine, one wave per problem, after oi_kernel ----
// A kernel of its own: its only LDS is the radix histogram and the event step's offsets, so many more
// waves share a CU and hide the L2 latency of the event passes than oi_kernel's query tables would allow.
__global__ __launch_bounds__(64) void oi_map_kernel(
    const DevOligoProblem* __restrict__ probs, unsigned char* __restrict__ scratch,
    gmapdp_oligo_result* __restrict__ results, const int32_t* __restrict__ npos_out,
    const int32_t* __restrict__ map_out, const uint32_t* __restrict__ table_all, int32_t* __restrict__ diag_all,
    uint64_t* __restrict__ pool) {
  __shared__ uint32_t hist[kOiHist];
  __shared__ int evq[3 * 256];
  const int lane = threadIdx.x;
  const DevOligoProblem P = probs[blockIdx.x];
  if (P.chrend <= P.chrstart) return;  // oned_matrix_p stays 0 (oi_kernel wrote the record)
  if (results[P.index].oned_matrix_p < 0) return;  // oi_kernel reported overflow
  OI_MARK(8);
#ifdef GMAPDP_OI_TIMING
  const unsigned long long om_t0 = wall_clock64();
#endif
  const uint32_t* table = table_all + P.table_offset;  // the mappings are relative to it
  const int qlen = P.querylength;
  const int nq = qlen - kOiK + 1;
  const int32_t* npq = npos_out + P.qoff;
  const int32_t* mpq = map_out + P.qoff;
  unsigned char* base_s = scratch + P.scratch_offset;
  const int* cum = reinterpret_cast<const int*>(base_s);
  const ScratchOi so = scratch_oi(qlen, P.chrend - P.chrstart);
  const int totalpositions = results[P.index].totalpositions;
  {
    const int diag_lookback = P.minor ? 60 : 120, suffn = P.minor ? 10 : 20;
    const uint32_t chrinit = P.plusp ? P.chrstart : (P.chrhigh - P.chroffset) - P.chrend;
    int32_t* good = diag_all + 4 * P.diag_offset;  // records {diag, best_start, best_end, best_n + 1}
    int ngood = 0, maxn = 0;
    const uint32_t maxdiag = (uint32_t)qlen + (P.chrend - P.chrstart);
    const unsigned long long pbase = *reinterpret_cast<const unsigned long long*>(base_s + so.poolbase);
    const int gcap = (int)min(P.diag_cap, 0x7fffffffu);
    const bool sorted =
        maxdiag < (1u << 20) - 1 && nq <= 4096
            ? oi_mappings_sorted<OiKeyT32>(lane, qlen, nq, totalpositions, maxdiag, chrinit, diag_lookback, suffn,
                                           npq, mpq, cum, table, pool, pbase, hist, evq, good, gcap, ngood, maxn)
        : nq < 65536
            ? oi_mappings_sorted<OiKeyQT>(lane, qlen, nq, totalpositions, maxdiag, chrinit, diag_lookback, suffn,
                                           npq, mpq, cum, table, pool, pbase, hist, evq, good, gcap, ngood, maxn)
            : oi_mappings_sorted<OiKeyQ>(lane, qlen, nq, totalpositions, maxdiag, chrinit, diag_lookback, suffn,
                                           npq, mpq, cum, table, pool, pbase, hist, evq, good, gcap, ngood, maxn);
    if (!sorted) {
      // the event pool is full: the sequential walk (per-diagonal states in the problem's fallback region;
      // a plan sized from a measured run has an exact pool and none: report the overflow instead)
      if (P.fallback_offset < 0) {
        if (lane == 0) {
          results[P.index].maxnconsecutive = 0;
          results[P.index].ndiagonals = 0;
          results[P.index].oned_matrix_p = -1;  // Stage2_compute answers GMAPDP overflow (status -2)
        }
        return;
      }
      const ScratchOiFb fb = scratch_oi_fb(qlen, P.chrend - P.chrstart);
      unsigned char* initp = scratch + P.fallback_offset + fb.initp;
      OiState* st = reinterpret_cast<OiState*>(scratch + P.fallback_offset + fb.states);
      for (size_t b = 16 * (size_t)lane; b < fb.states - fb.initp; b += 16 * 64)
        *reinterpret_cast<uint4*>(initp + b) = make_uint4(0u, 0u, 0u, 0u);
      __threadfence_block();
      int best = -1;  // diagi of each good diagonal goes in field 0 of its record first
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
    }
    if (lane == 0) {
      results[P.index].maxnconsecutive = ngood < 0 ? 0 : maxn;
      results[P.index].oned_matrix_p = ngood < 0 ? -1 : 1;
      results[P.index].ndiagonals = max(ngood, 0);
    }
  }
  OI_MARK(7);
#ifdef GMAPDP_OI_TIMING
  if (lane == 0 && P.index < 16384) {
    g_oi_wave[1][P.index] = (unsigned int)(wall_clock64() - om_t0);
    g_oi_wave[2][P.index] = (unsigned int)totalpositions;
  }
#endif
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
  void* fn = wide ? reinterpret_cast<void*>(&oi_kernel<uint32_t>) : reinterpret_cast<void*>(&oi_kernel<uint16_t>);
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
  return hipLaunchKernel(reinterpret_cast<void*>(&oi_map_kernel), dim3(nproblems), dim3(64), margs, 0, stream);
}

}  // namespace gmapdp
