// dp_kernel.hip -- CDNA4 (gfx950) kernel for GMAP's Dynprog_single_gap,
// Dynprog_end5_gap and Dynprog_end3_gap (nosimd semantics).
//
// One 64-lane wavefront (= one workgroup) owns one DP sub-problem.  Reference
// semantics restated (paths under the reference tree's src/):
//   Dynprog_single_gap      dynprog_single.c:429-676 (simple path :346-425)
//   Dynprog_end5/3_gap      dynprog_end.c:1294-1647 / 1924-2247
//   find_best_endpoint_*    dynprog_end.c:297-587, traceback_nogaps :649
//   Dynprog_standard        dynprog.c:1268-1786 (fill: recurrence, band, boundary
//                           rows/columns, >= vs > tie rule, clamp, revp)
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
//  * Ties: "a wins over b" is `a > b - late` with late in {0,1} (>= for jump
//    late, > otherwise), one compare per decision.
//  * Direction bits never leave the CU: per column four 64-bit ballots
//    (nogap=HORIZ, nogap=VERT, Egap=HORIZ, Fgap=VERT) go to LDS (or, for the
//    rare very long / very wide problems, to an L2-resident scratch).
//  * End gaps track the best endpoint per lane during the fill and reduce it
//    across the wave with the reference's scan-order tie rule.
//  * Traceback is wave-cooperative: each run (diagonal run, E chain, F chain)
//    is found with one ballot over 64 candidate cells, and its Pair records
//    are expanded by all 64 lanes and stream-compacted straight to HBM in the
//    reference's List_T order.
//  * The genome segment is decoded in-kernel from the HBM-resident packed
//    .genomecomp blocks (3 x u32 per 32 nt).
#include "dp_device.h"

namespace gmapdp {

// Phase timing of gg_kernel (tools_oi_timing.py gg; GMAPDP_OI_TIMING variant of the library only):
// wave 0 of every block adds its wall-clock timestamp at each mark; blocks that finish early add
// the remaining marks at once.
#ifdef GMAPDP_OI_TIMING
__device__ unsigned long long g_gg_marks[2][16];
#define GG_MARK(k)                                                          \
  do {                                                                      \
    if (threadIdx.x == 0) {                                                 \
      atomicAdd(&g_gg_marks[0][k], (unsigned long long)wall_clock64());     \
      atomicAdd(&g_gg_marks[1][k], 1ull);                                   \
    }                                                                       \
  } while (0)
#define GG_MARK_TO(a, b) \
  do {                   \
    for (int gk_ = (a); gk_ <= (b); gk_++) GG_MARK(gk_); \
  } while (0)
extern "C" int gmapdp_debug_gg_marks(unsigned long long* out) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_gg_marks), sizeof(g_gg_marks)) != hipSuccess) return 1;
  static const unsigned long long zero[2][16] = {};
  return hipMemcpyToSymbol(HIP_SYMBOL(g_gg_marks), zero, sizeof(zero)) != hipSuccess;
}
#else
#define GG_MARK(k) \
  do {             \
  } while (0)
#define GG_MARK_TO(a, b) \
  do {                   \
  } while (0)
#endif

// ROWS: lanes over query rows (fill_rows, R = row words) instead of band offsets, for bands much
// wider than the query; dpr_kernel below.
template <int R, bool DIRS_LDS, bool ROWS>
__device__ __forceinline__ void dp_body(
    const DevProblem* __restrict__ probs, const int* __restrict__ order,
    const uint32_t* __restrict__ blocks, uint64_t nwords,
    const char* __restrict__ qseq, const char* __restrict__ qseq_uc,
    const int8_t* __restrict__ sctab, const uint8_t* __restrict__ constab,
    gmapdp_result* __restrict__ results, gmapdp_pair* __restrict__ pairs,
    uint64_t* __restrict__ gdirs) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int lane = threadIdx.x;
  const int pid = order[blockIdx.x];
  const DevProblem P = probs[pid];
  const int rlen = P.rlength, glen = P.glength;
  const int flags = P.flags;
  const bool watson = flags & kFWatson;
  const int late = (flags & kFLate) ? 1 : 0;
  const bool rev = flags & kFRev;
  const int kind = P.kind;
  const Carve cv = carve_dp(rlen, glen, R, DIRS_LDS);
  int8_t* sc = reinterpret_cast<int8_t*>(smem + cv.sc);
  char* q = reinterpret_cast<char*>(smem + cv.q);
  char* quc = reinterpret_cast<char*>(smem + cv.quc);
  char* gch = reinterpret_cast<char*>(smem + cv.gch);
  uint8_t* gcl = reinterpret_cast<uint8_t*>(smem + cv.gcls);
  uint64_t* dirs = DIRS_LDS ? reinterpret_cast<uint64_t*>(smem + cv.dirs)
                            : reinterpret_cast<uint64_t*>(reinterpret_cast<unsigned char*>(gdirs) + P.dirs_offset);
  const int8_t* sct = sctab + (size_t)P.mismatchtype * 128 * kNClass;
  const uint8_t* cons = constab + (size_t)P.genestrand * 128 * kNClass;
  gmapdp_pair* out = pairs + P.pair_offset;
  const Geo G{P.roffset, P.goffset, rev ? -1 : 1};
  const int srow = rlen + 2;

  // ---- stage query (DP row order), per-class score rows and the genome segment in LDS ----
  const int qstep = rev ? -1 : 1;
  const bool score_uc = flags & kFScoreUC;
  for (int i = lane; i < rlen; i += 64) {
    const char c1 = qseq[P.qbase + qstep * i];
    const char c1u = qseq_uc[P.qbase + qstep * i];
    q[i + 1] = c1;
    quc[i + 1] = c1u;
    const uint64_t row = *reinterpret_cast<const uint64_t*>(sct + (uint8_t)((score_uc ? c1u : c1) & 127) * kNClass);
#pragma unroll
    for (int g = 0; g < 6; g++) sc[g * srow + i + 1] = (int8_t)(row >> (8 * g));
  }
  if (lane < 6) {  // rows 0 and rlength+1 are never scored but keep the clamped reads defined
    sc[lane * srow] = 0;
    sc[lane * srow + rlen + 1] = 0;
  }
  const bool segleft = flags & kFSegLeft, segrc = flags & kFSegRevcomp;
  for (int i = lane; i < glen; i += 64) {
    const char c2 = segment_nt(blocks, nwords, (uint32_t)i, (uint32_t)glen, P.segpos, P.segbound, segleft, segrc);
    const int c = rev ? glen - i : i + 1;  // end5 walks the segment from its right end
    gch[c] = c2;
    gcl[c] = gclass(c2);
  }
  __syncthreads();

  Tally t = {0, 0, 0, 0, 0, 0, 0, false};
  const int dpi_next = P.dynprogindex + (P.dynprogindex > 0 ? 1 : -1);
  const int endalign = P.endalign;
  const bool is_end = kind != kSingle;

  // ---- single_gap_simple (dynprog_single.c:346, taken when glength == rlength) ----
  if (kind == kSingle && glen == rlen) {
    int nmism = 0;
    for (int base = 0; base < rlen; base += 64) {
      const int r = base + lane + 1;
      bool mism = false;
      if (r <= rlen) {
        const char c1u = quc[r], c2 = gch[r];
        mism = (c2 != '*') && (c1u != c2) && !cons[(uint8_t)(c1u & 127) * kNClass + gclass(c2)];
      }
      nmism += __popcll(ballot(mism));
    }
    if (nmism <= 1) {
      // pushes r = 1..rlength without List_reverse: list order is r = rlength .. 1, a diagonal run
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
  }

  const int lband = P.lband, uband = P.uband;
  const int W = lband + uband + 1;
  int bestr = 0, bestc = 0;

  if (!(is_end && endalign == kQueryendNogaps)) {
    const int track = !is_end ? 0 : ((endalign == kQueryendIndels) ? 2 : 1);
    if constexpr (ROWS)
      fill_rows<R>(lane, rlen, glen, lband, uband, P.open, P.extend, late, track, sc, srow, gcl, dirs, bestr, bestc);
    else
      fill_band<R, false>(lane, rlen, glen, lband, uband, P.open, P.extend, late, track, sc, srow, gcl, dirs,
                          nullptr, bestr, bestc);
    if (DIRS_LDS) __syncthreads();
    else __threadfence_block();
  } else {
    bestr = bestc = glen < rlen ? glen : rlen;  // find_best_endpoint_to_queryend_nogaps
  }

  const bool skip = is_end && endalign != kQueryendNogaps && (flags & kFRequirePos);
  if (is_end && endalign == kQueryendNogaps) {
    emit_diag(lane, bestr, bestc, bestr, G, q, quc, gch, cons, out, t);  // traceback_nogaps
  } else if (!skip) {
    if constexpr (ROWS)
      traceback_walk(lane, RowDirs<R>{dirs, W, uband}, bestr, bestc, G, q, quc, gch, cons, watson, P.chroffset,
                     P.chrhigh, blocks, nwords, out, t);
    else
      traceback_band<R>(lane, dirs, W, uband, bestr, bestc, G, q, quc, gch, cons, watson, P.chroffset, P.chrhigh,
                        blocks, nwords, out, t);
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
      // Dynprog_end5_gap returns List_reverse of that list (dynprog_end.c:1646)
      if (kind == kEnd5 && npairs > 1) reverse_records(lane, out + first, npairs);
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

#define GMAPDP_DP_ARGS                                                                                  \
  const DevProblem *__restrict__ probs, const int *__restrict__ order, const uint32_t *__restrict__ blocks, \
      uint64_t nwords, const char *__restrict__ qseq, const char *__restrict__ qseq_uc,                  \
      const int8_t *__restrict__ sctab, const uint8_t *__restrict__ constab,                             \
      gmapdp_result *__restrict__ results, gmapdp_pair *__restrict__ pairs, uint64_t *__restrict__ gdirs
template <int R, bool DIRS_LDS>
__global__ __launch_bounds__(64) void dp_kernel(GMAPDP_DP_ARGS) {
  dp_body<R, DIRS_LDS, false>(probs, order, blocks, nwords, qseq, qseq_uc, sctab, constab, results, pairs, gdirs);
}
template <int R, bool DIRS_LDS>
__global__ __launch_bounds__(64) void dpr_kernel(GMAPDP_DP_ARGS) {
  dp_body<R, DIRS_LDS, true>(probs, order, blocks, nwords, qseq, qseq_uc, sctab, constab, results, pairs, gdirs);
}
#undef GMAPDP_DP_ARGS

// ===========================================================================
// dpx_kernel<S>: Dynprog_single_gap / Dynprog_end{5,3}_gap for narrow bands,
// 64/S problems per wave.  Most sub-problems have band width <= 16
// (extraband 6 around a near-square gap) or <= 32, so a whole 64-lane wave per
// problem would leave 50-80 % of the lanes idle in the fill.  Here each S-lane
// segment fills its own problem (fill_band<1, false, S>: row_shl/row_shr DPP
// confined to the segment, segment-local F scan, S-bit direction words), and
// the tracebacks -- short next to the fills -- then run one problem at a time
// with the whole wave.  Semantics are those of dp_kernel.
// ===========================================================================
// Per-problem LDS slot of the packed kernel: one 32-bit score word per query row (rows
// 0..rlength+1; 4-bit score per genome class -- every pairdistance value lies in [-5, 3]) and the
// genome classes.  The query stays in HBM and genome characters derive from the classes.  The
// direction words of the whole wave (4 x u64 per column) precede the slots.
__host__ __device__ inline Carve carve_dpx(int rlength, int glength) {
  Carve cv;
  size_t off = 0;
  cv.sc = off;   off = align16(off + 4u * (size_t)(rlength + 2));
  cv.gcls = off; off = align16(off + (size_t)(glength + 2));
  cv.q = cv.quc = cv.gch = cv.dirs = 0;
  cv.total = off;
  return cv;
}

// GD: the whole-wave direction words live in an L2-resident global scratch (one region of
// dirs_bytes per workgroup) instead of LDS, for classes whose LDS footprint would limit occupancy.
template <int S, bool GD>
__global__ __launch_bounds__(64) void dpx_kernel(
    const DevProblem* __restrict__ probs, const int* __restrict__ order, int count, int slot, int dirs_bytes,
    unsigned char* __restrict__ gdirs,
    const uint32_t* __restrict__ blocks, uint64_t nwords,
    const char* __restrict__ qseq, const char* __restrict__ qseq_uc,
    const int8_t* __restrict__ sctab, const uint8_t* __restrict__ constab,
    gmapdp_result* __restrict__ results, gmapdp_pair* __restrict__ pairs) {
  constexpr int NP = 64 / S;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int lane = threadIdx.x;
  const int seg = lane / S, sl = lane & (S - 1);
  const int idx = blockIdx.x * NP + seg;
  const bool live = idx < count;
  const int pid = order[live ? idx : blockIdx.x * NP];
  const DevProblem P = probs[pid];
  const int rlen = live ? P.rlength : 0, glen = live ? P.glength : 0;
  const int flags = P.flags;
  const bool rev = flags & kFRev;
  const int kind = P.kind, endalign = P.endalign;
  const bool is_end = kind != kSingle;
  uint64_t* wdirs = GD ? reinterpret_cast<uint64_t*>(gdirs + (size_t)blockIdx.x * (size_t)dirs_bytes)
                       : reinterpret_cast<uint64_t*>(smem);
  const int lds_dirs = GD ? 0 : dirs_bytes;
  unsigned char* base = smem + lds_dirs + (size_t)seg * (size_t)slot;
  const Carve cv = carve_dpx(rlen, glen);
  int32_t* sc4 = reinterpret_cast<int32_t*>(base + cv.sc);
  uint8_t* gcl = reinterpret_cast<uint8_t*>(base + cv.gcls);
  const int8_t* sct = sctab + (size_t)P.mismatchtype * 128 * kNClass;
  const uint8_t* cons = constab + (size_t)P.genestrand * 128 * kNClass;
  const int qstep = rev ? -1 : 1;
  const QView qucv{qseq_uc + P.qbase, qstep};
  const GClassView gv{gcl};

  // ---- stage each segment's problem: per query row one word of 4-bit scores (by genome class) ----
  const bool score_uc = flags & kFScoreUC;
  for (int i = sl; i < rlen; i += S) {
    const char c1 = score_uc ? qseq_uc[P.qbase + qstep * i] : qseq[P.qbase + qstep * i];
    const uint64_t row = *reinterpret_cast<const uint64_t*>(sct + (uint8_t)(c1 & 127) * kNClass);
    uint32_t w = 0;
#pragma unroll
    for (int g = 0; g < 6; g++) w |= (uint32_t)((row >> (8 * g)) & 0xfu) << (4 * g);
    sc4[i + 1] = (int32_t)w;
  }
  if (live && sl < 2) sc4[sl ? rlen + 1 : 0] = 0;  // rows 0, rlength+1
  const bool segleft = flags & kFSegLeft, segrc = flags & kFSegRevcomp;
  for (int i = sl; i < glen; i += S) {
    const char c2 = segment_nt(blocks, nwords, (uint32_t)i, (uint32_t)glen, P.segpos, P.segbound, segleft, segrc);
    gcl[rev ? glen - i : i + 1] = gclass(c2);
  }
  __syncthreads();

  // ---- single_gap_simple test per segment (glength == rlength, <= 1 mismatch) ----
  const bool try_simple = live && kind == kSingle && glen == rlen;
  int rmax = rlen;
#pragma unroll
  for (int off = S; off < 64; off <<= 1) rmax = max(rmax, __shfl_xor(rmax, off, 64));
  int nmism = 0;
  const uint64_t segmask = ((1ull << S) - 1ull) << (seg * S);
  for (int base0 = 0; base0 < rmax; base0 += S) {
    const int r = base0 + sl + 1;
    bool mism = false;
    if (try_simple && r <= rlen) {
      const char c1u = qucv[r], c2 = gv[r];
      mism = (c2 != '*') && (c1u != c2) && !cons[(uint8_t)(c1u & 127) * kNClass + gcl[r]];
    }
    nmism += __popcll(ballot(mism) & segmask);
  }
  const bool simple = try_simple && nmism <= 1;

  // ---- the segments' fills, side by side ----
  const bool nogaps = is_end && endalign == kQueryendNogaps;
  const bool fills = live && !simple && !nogaps;
  const int gfill = fills ? glen : 0;
  int gmax = gfill;
#pragma unroll
  for (int off = S; off < 64; off <<= 1) gmax = max(gmax, __shfl_xor(gmax, off, 64));
  int bestr = 0, bestc = 0;
  {
    const int track = !is_end ? 0 : ((endalign == kQueryendIndels) ? 2 : 1);
    fill_band<1, false, S>(lane, fills ? rlen : 0, gfill, P.lband, P.uband, P.open, P.extend,
                           (flags & kFLate) ? 1 : 0, fills ? track : 0, reinterpret_cast<const int8_t*>(sc4), 0,
                           gcl, wdirs, nullptr, bestr, bestc, gmax);
  }
  if (nogaps) bestr = bestc = glen < rlen ? glen : rlen;  // find_best_endpoint_to_queryend_nogaps
  if (GD) __threadfence_block();
  __syncthreads();

  // ---- emission, one problem at a time with the whole wave ----
  for (int j = 0; j < NP; j++) {
    const int src = j * S;
    if (!__builtin_amdgcn_readlane((int)live, src)) continue;
    const int pj = __builtin_amdgcn_readlane(pid, src);
    const DevProblem Pj = probs[pj];
    const Carve cj = carve_dpx(Pj.rlength, Pj.glength);
    unsigned char* bj = smem + lds_dirs + (size_t)j * (size_t)slot;
    const int sj = (Pj.flags & kFRev) ? -1 : 1;
    const BandDirs<1, uint64_t> dj{wdirs, Pj.lband + Pj.uband + 1, Pj.uband, src};
    finish_dp(lane, Pj, pj, __builtin_amdgcn_readlane((int)simple, src) != 0,
              __builtin_amdgcn_readlane(bestr, src), __builtin_amdgcn_readlane(bestc, src), dj,
              QView{qseq + Pj.qbase, sj}, QView{qseq_uc + Pj.qbase, sj},
              GClassView{reinterpret_cast<const uint8_t*>(bj + cj.gcls)}, constab, blocks, nwords, results,
              pairs);
  }
}

// ===========================================================================
// sx_kernel<B>: Dynprog_single_gap as the SIMD builds compute it
// (gmap.sse42/.avx2/.avx512 link dynprog_simd.c, SURVEY §8 "S" semantics):
// Dynprog_simd_8 (dynprog_simd.c:2987, B = 32 rows per block, int8
// saturating) when rlength and glength are both below use8p_size, else
// Dynprog_simd_16 (:6562, B = 16, int16 saturating), both in the AVX2 layout
// (dynprog.h:128; AVX-512 builds use the same code), then
// Dynprog_traceback_8/_16 (:9154/:9553), whose walk is traceback_std's.
//
// The reference fills block by block: block rlo covers every column in
// [max(0, rlo-lband), min(rhigh+uband, glength)] for all B rows, in band or
// not, then a scalar loop adds vertical gaps inside the band and the band's
// bottom row is forced diagonal (:3391-3478).  Here one B-lane segment holds
// one block (lane = row), 64/B problems per wave step side by side, each
// segment through its own (block, column) sequence; the scalar F loop
// becomes a segmented max-plus scan.  The row above a block and the F carry
// live in LDS (two row buffers, one FF row); the direction words of a step go
// to an L2-resident scratch (4 whole-wave u64 per step).
//
// Cells no block writes read as zero / DIAG: the reference reads whatever its
// Dynprog_T arena held there (it is never cleared, dynprog.c:686-731), i.e. a
// fresh arena's zeros; DESIGN.md "Parity" has the measured dependence.
// ===========================================================================
struct CarveSx {
  size_t sc, gcls, pb0, pb1, ff, total;
};
__host__ __device__ inline int sx_ceil(int rlength, int B) { return ((rlength + B) / B) * B; }  // rlength_ceil
__host__ __device__ inline CarveSx carve_sx(int rlength, int glength, int B) {
  CarveSx cv;
  size_t off = 0;
  cv.sc = off;   off = align16(off + 4u * (size_t)sx_ceil(rlength, B));  // 4-bit scores by class, rows 0..ceil-1
  cv.gcls = off; off = align16(off + (size_t)(glength + 2));
  cv.pb0 = off;  off = align16(off + 2u * (size_t)(glength + 1));       // matrix row above the block (even k)
  cv.pb1 = off;  off = align16(off + 2u * (size_t)(glength + 1));       // (odd k)
  cv.ff = off;   off = align16(off + 4u * (size_t)(glength + 1));       // FF[c]: c_gap after the block's last row
  cv.total = off;
  return cv;
}
// fill steps of one problem: (rlength/B + 1) blocks, each at most B + lband + uband columns wide
__host__ __device__ inline int sx_stride(int lband, int uband, int B) { return B + lband + uband; }
__host__ __device__ inline int sx_steps(int rlength, int lband, int uband, int B) {
  return (rlength / B + 1) * sx_stride(lband, uband, B);
}

// direction bit t of cell (r, c): block k = r / B holds it at step k*stride + (c - cs_k)
template <int B>
struct SxDirs {
  const uint64_t* dirs;
  int lband, uband, rlength, glength, bitoff;
  __device__ uint32_t operator()(int c, int t, int r) const {
    const int k = r / B, lk = r - k * B;
    const int cs = max(0, k * B - lband);
    const int ce = min(min(k * B + B - 1, rlength) + uband, glength);
    if (c < cs || c > ce) return 0u;
    const size_t step = (size_t)k * (size_t)sx_stride(lband, uband, B) + (size_t)(c - cs);
    return (uint32_t)(dirs[step * 4 + t] >> (bitoff + lk)) & 1u;
  }
};


template <int B>
__global__ __launch_bounds__(64) void sx_kernel(
    const DevProblem* __restrict__ probs, const int* __restrict__ order, int count, int slot,
    long long wave_dirs_bytes, unsigned char* __restrict__ gdirs,
    const uint32_t* __restrict__ blocks, uint64_t nwords,
    const char* __restrict__ qseq, const char* __restrict__ qseq_uc,
    const int8_t* __restrict__ sctab, const uint8_t* __restrict__ constab,
    gmapdp_result* __restrict__ results, gmapdp_pair* __restrict__ pairs) {
  constexpr int NP = 64 / B;
  constexpr int NEG = (B == 32) ? -128 : -32768;  // NEG_INFINITY_8 / NEG_INFINITY_16
  constexpr int POS = (B == 32) ? 127 : 32767;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int lane = threadIdx.x;
  const int seg = lane / B, sl = lane & (B - 1);
  const int idx = blockIdx.x * NP + seg;
  const bool live = idx < count;
  const int pid = order[live ? idx : blockIdx.x * NP];
  const DevProblem P = probs[pid];
  const int rlen = live ? P.rlength : 0, glen = live ? P.glength : 0;
  const int flags = P.flags;
  const int lband = P.lband, uband = P.uband, open = P.open, ext = P.extend;
  const int late = (flags & kFLate) ? 1 : 0;
  uint64_t* wdirs = reinterpret_cast<uint64_t*>(gdirs + (size_t)blockIdx.x * (size_t)wave_dirs_bytes);
  unsigned char* base = smem + (size_t)seg * (size_t)slot;
  const CarveSx cv = carve_sx(rlen, glen, B);
  int32_t* sc4 = reinterpret_cast<int32_t*>(base + cv.sc);
  uint8_t* gcl = reinterpret_cast<uint8_t*>(base + cv.gcls);
  int16_t* pb0 = reinterpret_cast<int16_t*>(base + cv.pb0);
  int16_t* pb1 = reinterpret_cast<int16_t*>(base + cv.pb1);
  int* FF = reinterpret_cast<int*>(base + cv.ff);
  const int8_t* sct = sctab + (size_t)P.mismatchtype * 128 * kNClass;
  const uint8_t* cons = constab + (size_t)P.genestrand * 128 * kNClass;
  const int ceil_r = sx_ceil(rlen, B);

  // ---- stage: pairscores[5][rlength_ceil] as one word of 4-bit scores per row (row 0 scores
  //      'N', rows past rlength never reach rows <= rlength), the genome classes, zeroed rows ----
  const bool score_uc = flags & kFScoreUC;
  for (int i = sl; i < ceil_r; i += B) {
    uint32_t w = 0;
    if (live && i <= rlen) {
      const char c1 = (i == 0) ? 'N' : (score_uc ? qseq_uc[P.qbase + i - 1] : qseq[P.qbase + i - 1]);
      const uint64_t row = *reinterpret_cast<const uint64_t*>(sct + (uint8_t)(c1 & 127) * kNClass);
#pragma unroll
      for (int g = 0; g < 5; g++) w |= (uint32_t)((row >> (8 * g)) & 0xfu) << (4 * g);
    }
    if (live) sc4[i] = (int32_t)w;
  }
  const bool segleft = flags & kFSegLeft, segrc = flags & kFSegRevcomp;
  for (int i = sl; i < glen; i += B)
    gcl[i + 1] = gclass(segment_nt(blocks, nwords, (uint32_t)i, (uint32_t)glen, P.segpos, P.segbound, segleft, segrc));
  for (int i = sl; i <= glen; i += B) {
    pb0[i] = 0;
    pb1[i] = 0;
  }
  __syncthreads();

  // ---- single_gap_simple test per segment (glength == rlength, <= 1 mismatch) ----
  const QView qucv{qseq_uc + P.qbase, 1};
  const GClassView gv{gcl};
  const bool try_simple = live && P.kind == kSingle && glen == rlen;
  int rmax = rlen;
#pragma unroll
  for (int off = B; off < 64; off <<= 1) rmax = max(rmax, __shfl_xor(rmax, off, 64));
  int nmism = 0;
  const uint64_t segmask = ((B == 64) ? ~0ull : ((1ull << B) - 1ull)) << (seg * B);
  for (int b0 = 0; b0 < rmax; b0 += B) {
    const int r = b0 + sl + 1;
    bool mism = false;
    if (try_simple && r <= rlen) {
      const char c1u = qucv[r], c2 = gv[r];
      mism = (c2 != '*') && (c1u != c2) && !cons[(uint8_t)(c1u & 127) * kNClass + gcl[r]];
    }
    nmism += __popcll(ballot(mism) & segmask);
  }
  const bool simple = try_simple && nmism <= 1;

  // ---- the block fills, segments side by side ----
  const bool fills = live && !simple;
  const int nblk = fills ? rlen / B + 1 : 0;
  const int stride = sx_stride(lband, uband, B);
  int tmax = nblk * stride;
#pragma unroll
  for (int off = B; off < 64; off <<= 1) tmax = max(tmax, __shfl_xor(tmax, off, 64));
  int k = 0, o = 0;        // block, column step within the block
  int H = 0, E = 0;        // this lane's row: stored score / horizontal gap of the previous column
  for (int t = 0; t < tmax; t++) {
    const int rlo = k * B;
    const int rhigh = min(rlo + B - 1, rlen);
    const int cs = max(0, rlo - lband);
    const int ce = min(rhigh + uband, glen);
    const int c = cs + o;
    const bool act = (k < nblk) && (c <= ce);
    const int r = rlo + sl;
    const int16_t* pin = (k & 1) ? pb0 : pb1;  // block k reads the row block k-1 wrote
    int16_t* pout = (k & 1) ? pb1 : pb0;
    if (o == 0) {  // INFINITE_INITIAL_GAP_PENALTY block start: "compensate for T1 = H + open"
      E = late ? NEG : NEG + 1;
      H = NEG - open;
    }
    int X = NEG, G0 = kNegInf32, Lv = kNegInf32, cls = 0;
    if (act) {
      X = (c == 0) ? (rlo == 0 ? 0 : NEG) : (rlo == 0 ? NEG : (int)pin[c - 1]);
      cls = (c == 0) ? 0 : min((int)gcl[c], (int)kN);  // nt_to_int_array: '*' scores as 'N'
      if (rlo > 0 && c < rlo + uband) {
        G0 = FF[c];
        Lv = pin[c];
      }
    }
    // EGAP (horizontal): T1 = H + open, E >= T1 (late) / E > T1
    const int T1 = sat_add(H, open, NEG, POS);
    bool dE = late ? (E >= T1) : (E > T1);
    const int En = sat_add(max(E, T1), ext, NEG, POS);
    // NOGAP: H shifted down one row (row rlo from the row above), plus the pair score
    const int Hs = seg_shr1<B>(H, X, sl);
    int p;
    if (c == 0) p = (r == 0) ? 0 : NEG;  // pairscores_col0
    else p = __builtin_amdgcn_sbfe(sc4[min(r, ceil_r - 1)], cls * 4, 4);
    const int Hd = sat_add(Hs, p, NEG, POS);
    bool dN = late ? (En >= Hd) : (En > Hd);
    int Hn = max(Hd, En);
    int rhc = rhigh;
    if (rhigh >= c + lband) {
      rhc = c + lband;
      if (c > 0 && r == rhc) {  // bottom of the band: diagonal only
        Hn = Hd;
        dE = false;
        dN = false;
      }
    }
    // F loop: vertical gaps in rows [rloc, rhc]; the band's top row starts a fresh chain
    const int rloc = max(rlo, c - uband);
    const bool top = rloc == c - uband;
    const int Htop = __shfl(Hn, seg * B + min(max(rloc - rlo, 0), B - 1), 64);
    int rs = rloc;
    if (top) {
      G0 = Lv + open + ext;
      Lv = Htop;
      rs = rloc + 1;
    }
    const int A = (r >= rs && r <= rhc - 1) ? Hn + open - r * ext : kSent;
    const int A0 = max(G0, Lv + open) - (rs - 1) * ext;
    const int Xex = seg_shr1<B>(seg_scan_max<B>(A), kSent, sl);
    const int F = r * ext + max(A0, Xex);
    const int Fup = seg_shr1<B>(F, G0, sl);
    const int Lup = seg_shr1<B>(max(F, Hn), Lv, sl);
    const bool inF = act && r >= rs && r <= rhc;
    const int Fprev = (r == rs) ? G0 : Fup;
    const int Lprev = (r == rs) ? Lv : Lup;
    const bool vF = inF && (late ? (Fprev >= Lprev + open) : (Fprev > Lprev + open));
    const bool vN = inF && (late ? (F >= Hn) : (F > Hn));
    const int Hf = vN ? max(F, NEG) : Hn;
    const int Flast = __shfl(F, seg * B + min(max(rhc - rlo, 0), B - 1), 64);
    const uint64_t mH = ballot(act && dN && !vN), mV = ballot(vN), mE = ballot(act && dE), mF = ballot(vF);
    if (act) {
      H = Hf;
      E = En;
      if (sl == 0) FF[c] = (rhc >= rs) ? Flast : G0;
      if (sl == B - 1) pout[c] = (int16_t)Hf;
    }
    if (lane == 0) {
      uint64_t* d = wdirs + (size_t)t * 4;
      d[0] = mH;
      d[1] = mV;
      d[2] = mE;
      d[3] = mF;
    }
    if (k < nblk && ++o == stride) {
      o = 0;
      k++;
    }
  }
  __threadfence_block();
  __syncthreads();

  // ---- emission, one problem at a time with the whole wave ----
  for (int j = 0; j < NP; j++) {
    const int src = j * B;
    if (!__builtin_amdgcn_readlane((int)live, src)) continue;
    const int pj = __builtin_amdgcn_readlane(pid, src);
    const DevProblem Pj = probs[pj];
    const CarveSx cj = carve_sx(Pj.rlength, Pj.glength, B);
    unsigned char* bj = smem + (size_t)j * (size_t)slot;
    const SxDirs<B> dj{wdirs, Pj.lband, Pj.uband, Pj.rlength, Pj.glength, src};
    finish_dp(lane, Pj, pj, __builtin_amdgcn_readlane((int)simple, src) != 0, Pj.rlength, Pj.glength, dj,
              QView{qseq + Pj.qbase, 1}, QView{qseq_uc + Pj.qbase, 1},
              GClassView{reinterpret_cast<const uint8_t*>(bj + cj.gcls)}, constab, blocks, nwords, results, pairs);
  }
}

// ===========================================================================
// Dynprog_genome_gap (dynprog_genome.c:3288-3901), nosimd semantics, no
// splicing IIT.  One workgroup of two waves per problem:
//   1. genome_gap_simple (:3006) when !finalp && defect_rate < DEFECT_MEDQ
//      (wave 0): prefix sums of the two diagonals + a (score, rL) max-reduction;
//   2. otherwise the two fills run concurrently, wave 0 the R fill (reversed
//      query vs rev_gsequenceR, lband = lbandL, !jump_late_p, :3810), wave 1 the
//      L fill (:3801).  Each carries its side's bridge candidates along the band
//      rows (BridgeCarry), so no score matrix is ever stored;
//   3. bridge_intron_gap_site_level (:2469) on wave 0, one lane per row rL: the
//      reference's sequential "> score, or == score and > prob" scan is a
//      lexicographic max over (score, probL+probR, scan order), so each row's
//      A, best B and best C are merged in scan order and the rows by a wave
//      reduction;
//   4. traceback R, List_reverse, gap holder, traceback L, Pair_maxnegscore.
// ===========================================================================
struct CarveGG {
  size_t scL, scR, gclL, gclR, ldi, rdi, pL, pR, isc, flag, dirsL, dirsR, total;
};
// Global scratch of one genome-gap problem: the bridge candidates and diagonal of each fill
// (written once by the fill, read once by the bridge), then the direction planes unless in LDS.
struct ScratchGG {
  size_t partB, partC, diagL, diagR, dirsL, dirsR, total;
};

__host__ __device__ inline size_t gg_dirs_bytes(int glength, int R) { return (size_t)(glength + 1) * 4u * (size_t)R * 8u; }
// LDS direction planes of a one-word band (PackedDirs): 16 + 4 nhigh bytes per column
__host__ __device__ inline size_t gg_dirs_bytes_packed(int glength, int W) {
  return (size_t)(glength + 1) * (16u + 4u * (size_t)gg_dir_nhigh(W));
}

// LDS: per query row one word of 4-bit scores per side (as the packed kernel), genome classes,
// dinucleotide codes and splice probabilities per column; the query stays in HBM and genome
// characters derive from the classes.
__host__ __device__ inline CarveGG carve_gg(int rlength, int glengthL, int glengthR, int R, bool dirs_lds, int W = 64) {
  CarveGG cv;
  size_t off = 0;
  cv.pL = off;    off = align16(off + 8u * (size_t)glengthL);
  cv.pR = off;    off = align16(off + 8u * (size_t)glengthR);
  cv.scL = off;   off = align16(off + 4u * (size_t)(rlength + 2));
  cv.scR = off;   off = align16(off + 4u * (size_t)(rlength + 2));
  cv.gclL = off;  off = align16(off + (size_t)(glengthL + 2));
  cv.gclR = off;  off = align16(off + (size_t)(glengthR + 2));
  cv.ldi = off;   off = align16(off + (size_t)(glengthL + 2));
  cv.rdi = off;   off = align16(off + (size_t)(glengthR + 2));
  cv.isc = off;   off = align16(off + 64);
  cv.flag = off;  off = align16(off + 4);
  cv.dirsL = cv.dirsR = 0;
  if (dirs_lds) {  // one-word bands keep them packed (W: the wider side's band)
    cv.dirsL = off; off = align16(off + (R == 1 ? gg_dirs_bytes_packed(glengthL, W) : gg_dirs_bytes(glengthL, R)));
    cv.dirsR = off; off = align16(off + (R == 1 ? gg_dirs_bytes_packed(glengthR, W) : gg_dirs_bytes(glengthR, R)));
  }
  cv.total = off;
  return cv;
}

// Direction planes in global scratch packed as in LDS for one-word bands (GMAPDP_GG_PACK_GLOBAL builds,
// experiments): 20 B per column for the bench's ~37-lane bands instead of 32, but lane 0's packing sits on
// the column loop's issue path and gg_kernel<1, 0> measured 2.04 ms per launch against 1.93 unpacked
// (profiles/r06_seed), so the product stores the four 64-bit ballots.
#ifdef GMAPDP_GG_PACK_GLOBAL
constexpr bool kGgPackGlobal = true;
#else
constexpr bool kGgPackGlobal = false;
#endif
__host__ __device__ inline ScratchGG scratch_gg(int rlength, int glengthL, int glengthR, int R, bool dirs_lds,
                                                int W = 64) {
  ScratchGG sv;
  size_t off = 0;
  sv.partB = off; off = align16(off + 16u * (size_t)(rlength + 1));
  sv.partC = off; off = align16(off + 16u * (size_t)(rlength + 1));
  sv.diagL = off; off = align16(off + 4u * (size_t)(rlength + 1));
  sv.diagR = off; off = align16(off + 4u * (size_t)(rlength + 1));
  sv.dirsL = sv.dirsR = off;
  if (!dirs_lds) {
    const bool pk = R == 1 && kGgPackGlobal;
    sv.dirsL = off; off = align16(off + (pk ? gg_dirs_bytes_packed(glengthL, W) : gg_dirs_bytes(glengthL, R)));
    sv.dirsR = off; off = align16(off + (pk ? gg_dirs_bytes_packed(glengthR, W) : gg_dirs_bytes(glengthR, R)));
  }
  sv.total = off;
  return sv;
}

// GMAPDP_GGX_*: timing experiments only (make variant; outputs are garbage): NOSTAGE stages constants
// instead of loading, NOEMIT ends after the fills, WPE sets amdgpu_waves_per_eu.
#ifdef GMAPDP_GGX_WPE
#define GGX_ATTR __attribute__((amdgpu_waves_per_eu(GMAPDP_GGX_WPE)))
#else
#define GGX_ATTR
#endif
template <int R, bool DIRS_LDS>
__global__ __launch_bounds__(128) GGX_ATTR void gg_kernel(
    const DevGenomeProblem* __restrict__ probs, const int* __restrict__ order,
    const uint32_t* __restrict__ blocks, uint64_t nwords,
    const char* __restrict__ qseq, const char* __restrict__ qseq_uc, const double* __restrict__ sprob,
    const int8_t* __restrict__ sctab, const uint8_t* __restrict__ constab, const int8_t* __restrict__ isctab,
    gmapdp_genome_result* __restrict__ results, gmapdp_pair* __restrict__ pairs,
    unsigned char* __restrict__ gscratch, const uint8_t* __restrict__ known, const double* __restrict__ metab) {
  // sprob NULL: the splice probabilities are GMAP's MaxEnt models (metab) evaluated here while the
  // segments are staged (no probability arena written by a prologue kernel and read back)
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int pid = order[blockIdx.x];
  const DevGenomeProblem P = probs[pid];
  GG_MARK(0);
  const int rlen = P.rlength, gL = P.glengthL, gR = P.glengthR;
  const int flags = P.flags;
  const bool watson = flags & kFWatson;
  const int late = (flags & kFLate) ? 1 : 0;
  const int lband = P.lbandL, ubandL = P.ubandL, ubandR = P.ubandR;
  const int WL = lband + ubandL + 1, WR = lband + ubandR + 1;
  constexpr bool DPK = R == 1 && (DIRS_LDS || kGgPackGlobal);  // packed direction planes (PackedDirs)
  const CarveGG cv = carve_gg(rlen, gL, gR, R, DIRS_LDS, WL > WR ? WL : WR);
  const ScratchGG sv = scratch_gg(rlen, gL, gR, R, DIRS_LDS, WL > WR ? WL : WR);
  unsigned char* gbase = gscratch + P.dirs_offset;
  double* pL = reinterpret_cast<double*>(smem + cv.pL);
  double* pR = reinterpret_cast<double*>(smem + cv.pR);
  Part* partB = reinterpret_cast<Part*>(gbase + sv.partB);  // indexed by rR
  Part* partC = reinterpret_cast<Part*>(gbase + sv.partC);  // indexed by rL
  int* diagL = reinterpret_cast<int*>(gbase + sv.diagL);
  int* diagR = reinterpret_cast<int*>(gbase + sv.diagR);
  int32_t* scL = reinterpret_cast<int32_t*>(smem + cv.scL);
  int32_t* scR = reinterpret_cast<int32_t*>(smem + cv.scR);
  uint8_t* gclL = reinterpret_cast<uint8_t*>(smem + cv.gclL);
  uint8_t* gclR = reinterpret_cast<uint8_t*>(smem + cv.gclR);
  uint8_t* ldi = reinterpret_cast<uint8_t*>(smem + cv.ldi);
  uint8_t* rdi = reinterpret_cast<uint8_t*>(smem + cv.rdi);
  int8_t* isc = reinterpret_cast<int8_t*>(smem + cv.isc);
  int* done = reinterpret_cast<int*>(smem + cv.flag);
  uint64_t* dirsL = reinterpret_cast<uint64_t*>(DIRS_LDS ? smem + cv.dirsL : gbase + sv.dirsL);
  uint64_t* dirsR = reinterpret_cast<uint64_t*>(DIRS_LDS ? smem + cv.dirsR : gbase + sv.dirsR);
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
  const bool kn = flags & kGKnown;  // known splice sites (get_known_splicesites, dynprog_genome.c:405)
  const uint8_t* kb = kn ? known + P.known_offset : nullptr;

  // ---- stage (both waves): per query row the 4-bit score word in both DP orders, both genome
  //      segments as classes, dinucleotide codes, the splice probabilities, the intron scores ----
#ifdef GMAPDP_GGX_NOSTAGE
  for (int i = tid; i < rlen + 2; i += 128) scL[i] = scR[i] = 0x123456;
  for (int i = tid; i < gL + 2; i += 128) gclL[i] = i & 3;
  for (int i = tid; i < gR + 2; i += 128) gclR[i] = i & 3;
  for (int i = tid; i < gL; i += 128) pL[i] = 0.1;
  for (int i = tid; i < gR; i += 128) pR[i] = 0.1;
  if (tid < 64) isc[tid] = tid & 7;
  if (tid == 0) *done = 0;
  __syncthreads();
  if (false)
#endif
  for (int i = tid; i < rlen; i += 128) {
    const char c1 = qseq[P.qbase + i];
    const uint64_t row = *reinterpret_cast<const uint64_t*>(sct + (uint8_t)(c1 & 127) * kNClass);
    uint32_t w = 0;
#pragma unroll
    for (int g = 0; g < 6; g++) w |= (uint32_t)((row >> (8 * g)) & 0xfu) << (4 * g);
    scL[i + 1] = (int32_t)w;
    scR[rlen - i] = (int32_t)w;
  }
#ifndef GMAPDP_GGX_NOSTAGE
  if (tid < 2) {
    scL[tid ? rlen + 1 : 0] = 0;
    scR[tid ? rlen + 1 : 0] = 0;
  }
  // Both segments as one index space jj (L: i = jj, R: i = jj - gL), two items per thread per pass with
  // every load issued before any is used: segment_nt's bounds (Genome_get_segment_right/left) become a
  // class or a block address, then the flags word and the half word of each block are loaded together.
  {
    const int nG = gL + gR;
    for (int b0 = tid; b0 < nG; b0 += 256) {
      uint32_t wf[2], wv[2], bit[2];
      int cls[2];  // kStar / kN decided from the bounds, -1: decode the words
      double pv[2];
      bool rcv[2];
#pragma unroll
      for (int u = 0; u < 2; u++) {
        const int jj = b0 + 128 * u;
        const bool act = jj < nG;
        const bool rs = jj >= gL;
        const uint32_t i = (uint32_t)(rs ? jj - gL : jj), L = (uint32_t)(rs ? gR : gL);
        const uint64_t pos = rs ? P.segposR : P.segposL, bound = rs ? P.segboundR : P.segboundL;
        const bool left = rs ? (flags & kGSegRLeft) : (flags & kGSegLLeft);
        rcv[u] = rs ? (flags & kGSegRRc) : (flags & kGSegLRc);
        const uint64_t j = rcv[u] ? L - 1u - i : i;
        bool star;
        uint64_t g;
        if (!left) {  // Genome_get_segment_right(left = pos, L, chrhigh = bound)
          star = pos >= bound || (pos + L >= bound && j + (pos + L - bound) >= L);
          g = pos + j;
        } else {      // Genome_get_segment_left(right = pos, L, chroffset = bound)
          star = pos < bound || (pos < bound + L && j < bound + L - pos);
          g = pos - L + j;
        }
        const uint64_t ptr = (g >> 5) * 3u;
        cls[u] = star ? kStar : (ptr + 2 >= nwords ? kN : -1);  // beyond the allocation: 'N' (decode_nt)
        const uint64_t pp = (cls[u] < 0 && act) ? ptr : 0;
        bit[u] = (uint32_t)(g & 31u);
        wf[u] = blocks[pp + 2];
        wv[u] = blocks[pp + (bit[u] < 16 ? 1 : 0)];
        pv[u] = !act ? 0.0 : sprob ? sprob[P.prob_offset + jj] : gg_site_prob(P, blocks, nwords, metab, jj);
        // a known site has probability 1.0 in the bridge (dynprog_genome.c:2577-2578)
        if (kn && act && kb[jj]) pv[u] = 1.0;
      }
#pragma unroll
      for (int u = 0; u < 2; u++) {
        const int jj = b0 + 128 * u;
        if (jj >= nG) continue;
        int c = cls[u];
        if (c < 0) {
          const int x = (int)((wv[u] >> (2u * (bit[u] & 15u))) & 3u);
          c = ((wf[u] >> bit[u]) & 1u) ? kN : (rcv[u] ? 3 - x : x);  // complement of A C G T is 3 - code
        }
        if (jj < gL) {
          gclL[jj + 1] = (uint8_t)c;
          pL[jj] = pv[u];
        } else {
          gclR[gR - (jj - gL)] = (uint8_t)c;  // rev_gsequenceR[1-c] = segment[glengthR-c]
          pR[jj - gL] = pv[u];
        }
      }
    }
  }
  if (tid < 64) isc[tid] = isctab[(size_t)P.iclass * 128 + ((flags & kGFinal) ? 64 : 0) + tid];
  if (tid == 0) *done = 0;
  __syncthreads();
#endif
  // leftdi[cL] from gsequenceL[cL], [cL+1]; rightdi[cR] from rev_gsequenceR[-cR-1], [-cR] (:2518-2566)
  for (int c = tid; c <= gL; c += 128) ldi[c] = (c < gL - 1) ? left_dinucl(gchL[c + 1], gchL[c + 2]) : 0;
  for (int c = tid; c <= gR; c += 128) rdi[c] = (c < gR - 1) ? right_dinucl(gchR[c + 2], gchR[c + 1]) : 0;
  __syncthreads();
  GG_MARK(1);

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
                                     ldi, rdi, pL, pR, diagL, diagR, out, res, results,
                                     kn ? kb + gL + gR : nullptr, sprob ? sprob + P.prob_offset : nullptr, blocks,
                                     nwords, metab);
      if (lane == 0) *done = ok ? 1 : 0;
    }
    __syncthreads();
    if (*done) {
      GG_MARK_TO(2, 7);
      return;
    }
  }
  GG_MARK(2);

  // ---- 2. fills, concurrently: wave 0 R (feeds the B candidates), wave 1 L (the C candidates) ----
  const int rdist = P.rev_goffsetR - P.goffsetL;  // "cR < rightoffset - leftoffset - cL"
  {
    int br, bc;
    // (a band narrower than the wave's 64 R elements -- every bench genome gap: 37 -- takes the narrow-band
    // shifts; a wave-uniform choice per fill)
    if (wave == 0) {
      const BridgeCarry B{ldi, rdi, pL, pR, isc, rdist, partB, diagR};
      if (WR < 64 * R)
        fill_band<R, true, 64, true, false, DPK, true>(lane, rlen, gR, lband, ubandR, P.open, P.extend, 1 - late, 0,
                                                       reinterpret_cast<const int8_t*>(scR), 0, gclR, dirsR, &B, br,
                                                       bc);
      else
        fill_band<R, true, 64, true, false, DPK>(lane, rlen, gR, lband, ubandR, P.open, P.extend, 1 - late, 0,
                                                 reinterpret_cast<const int8_t*>(scR), 0, gclR, dirsR, &B, br, bc);
    } else {
      const BridgeCarry B{rdi, ldi, pR, pL, isc, rdist, partC, diagL};
      if (WL < 64 * R)
        fill_band<R, true, 64, true, false, DPK, true>(lane, rlen, gL, lband, ubandL, P.open, P.extend, late, 0,
                                                       reinterpret_cast<const int8_t*>(scL), 0, gclL, dirsL, &B, br,
                                                       bc);
      else
        fill_band<R, true, 64, true, false, DPK>(lane, rlen, gL, lband, ubandL, P.open, P.extend, late, 0,
                                                 reinterpret_cast<const int8_t*>(scL), 0, gclL, dirsL, &B, br, bc);
    }
  }
  __threadfence_block();
  __syncthreads();
  GG_MARK(3);
  if (wave != 0) return;
#ifdef GMAPDP_GGX_NOEMIT
  if (lane == 0) results[pid] = res;
  return;
#endif

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
    // B: cL = rL, best cR of R row rR (+ matrixL[rL][rL])
    const Part b = partB[rR];
    if (b.c >= 0 && lex_better(dL + b.s, b.p, rs, rp)) {
      rs = dL + b.s;
      rp = b.p;
      rcL = rL;
      rcR = b.c;
    }
    // C: cR = rR, best cL of L row rL (+ matrixR[rR][rR])
    const Part cpart = partC[rL];
    if (cpart.c >= 0 && lex_better(dR + cpart.s, cpart.p, rs, rp)) {
      rs = dR + cpart.s;
      rp = cpart.p;
      rcL = cpart.c;
      rcR = rR;
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
  // one lane's view is authoritative
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

  GG_MARK(4);
  if (finalscore < 0) {
    if (lane == 0) {
      res.traceback_score = -100;
      results[pid] = res;
    }
    GG_MARK_TO(5, 7);
    return;
  }

  // ---- 4. tracebacks around the intron gap holder ----
  res.left_prob = pL[bestcL];
  res.right_prob = pR[bestcR];
  const int new_left = P.goffsetL + (bestcL - 1);
  const int new_right = P.rev_goffsetR - (bestcR - 1);
  Tally t = {0, 0, 0, 0, 0, 0, 0, false};
  if constexpr (DPK) {
    const uint32_t* lo = reinterpret_cast<const uint32_t*>(dirsR);
    const PackedDirs dR{lo, lo + 4 * (gR + 1), WR, ubandR, gg_dir_nhigh(WR)};
    traceback_walk(lane, dR, bestrR, bestcR, GR, qR, qucR, gchR, cons, watson, P.chroffset, P.chrhigh, blocks, nwords,
                   out, t);
  } else {
    traceback_band<R>(lane, dirsR, WR, ubandR, bestrR, bestcR, GR, qR, qucR, gchR, cons, watson, P.chroffset,
                      P.chrhigh, blocks, nwords, out, t);
  }
  const int nR = t.count;
  reverse_records(lane, out, nR);
  GG_MARK(5);
  const int queryjump = (rev_roffset - bestrR) - (P.roffset + bestrL) + 1;
  if (lane == 0) put_pair(out, nR, -1, -1, new_right - new_left - 1, ' ', ' ', ' ', ' ');
  t.count += 1;
  if constexpr (DPK) {
    const uint32_t* lo = reinterpret_cast<const uint32_t*>(dirsL);
    const PackedDirs dL{lo, lo + 4 * (gL + 1), WL, ubandL, gg_dir_nhigh(WL)};
    traceback_walk(lane, dL, bestrL, bestcL, GL, qL, qucL, gchL, cons, watson, P.chroffset, P.chrhigh, blocks, nwords,
                   out, t);
  } else {
    traceback_band<R>(lane, dirsL, WL, ubandL, bestrL, bestcL, GL, qL, qucL, gchL, cons, watson, P.chroffset,
                      P.chrhigh, blocks, nwords, out, t);
  }
  GG_MARK(6);
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
  GG_MARK(7);
}

// ---- host-side launch table ----
template <int R, bool D, bool ROWS>
static void* kptr() {
  if constexpr (ROWS) return reinterpret_cast<void*>(&dpr_kernel<R, D>);
  else return reinterpret_cast<void*>(&dp_kernel<R, D>);
}

size_t lds_bytes_dp(int rlength, int glength, int R, bool dirs_lds) {
  return carve_dp(rlength, glength, R, dirs_lds).total;
}

hipError_t launch_dp(int R, bool dirs_lds, bool rows, int nblocks, size_t lds, hipStream_t stream,
                     const DevProblem* probs, const int* order, const uint32_t* blocks, uint64_t nwords,
                     const char* qseq, const char* qseq_uc, const int8_t* sctab, const uint8_t* constab,
                     gmapdp_result* results, gmapdp_pair* pairs, uint64_t* gdirs) {
  void* fn = nullptr;
#define GMAPDP_CASE(RR)                                          \
  case RR:                                                       \
    fn = dirs_lds ? kptr<RR, true, false>() : kptr<RR, false, false>();        \
    break;
#define GMAPDP_RCASE(RR)                                         \
  case RR:                                                       \
    fn = dirs_lds ? kptr<RR, true, true>() : kptr<RR, false, true>();        \
    break;
  if (rows) {
    switch (R) {  // 64 * 16 rows >= GMAPDP_MAX_RLENGTH + 1
      GMAPDP_RCASE(1)
      GMAPDP_RCASE(2)
      GMAPDP_RCASE(4)
      GMAPDP_RCASE(8)
      GMAPDP_RCASE(16)
      default: return hipErrorInvalidValue;
    }
  } else {
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
  }
#undef GMAPDP_CASE
#undef GMAPDP_RCASE
  if (lds > 64 * 1024) {
    hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
  }
  void* args[] = {(void*)&probs, (void*)&order, (void*)&blocks, (void*)&nwords, (void*)&qseq, (void*)&qseq_uc,
                  (void*)&sctab, (void*)&constab, (void*)&results, (void*)&pairs, (void*)&gdirs};
  return hipLaunchKernel(fn, dim3(nblocks), dim3(64), args, lds, stream);
}

size_t lds_slot_dpx(int rlength, int glength) { return carve_dpx(rlength, glength).total; }
size_t lds_dirs_dpx(int gmax) { return align16((size_t)(gmax + 1) * 4u * 8u); }

hipError_t launch_dpx(int S, int nproblems, int slot, int dirs_bytes, unsigned char* gdirs, hipStream_t stream,
                      const DevProblem* probs, const int* order, const uint32_t* blocks, uint64_t nwords,
                      const char* qseq, const char* qseq_uc, const int8_t* sctab, const uint8_t* constab,
                      gmapdp_result* results, gmapdp_pair* pairs) {
  if (S != 16 && S != 32) return hipErrorInvalidValue;
  void* fn;
  if (S == 16) fn = gdirs ? reinterpret_cast<void*>(&dpx_kernel<16, true>) : reinterpret_cast<void*>(&dpx_kernel<16, false>);
  else fn = gdirs ? reinterpret_cast<void*>(&dpx_kernel<32, true>) : reinterpret_cast<void*>(&dpx_kernel<32, false>);
  const int np = 64 / S;
  const size_t lds = (gdirs ? 0 : (size_t)dirs_bytes) + (size_t)slot * np;
  if (lds > 64 * 1024) {
    hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
  }
  const int nblocks = (nproblems + np - 1) / np;
  void* args[] = {(void*)&probs, (void*)&order, (void*)&nproblems, (void*)&slot, (void*)&dirs_bytes,
                  (void*)&gdirs, (void*)&blocks, (void*)&nwords, (void*)&qseq, (void*)&qseq_uc, (void*)&sctab,
                  (void*)&constab, (void*)&results, (void*)&pairs};
  return hipLaunchKernel(fn, dim3(nblocks), dim3(64), args, lds, stream);
}

size_t lds_slot_sx(int rlength, int glength, int B) { return carve_sx(rlength, glength, B).total; }
int steps_sx(int rlength, int lband, int uband, int B) { return sx_steps(rlength, lband, uband, B); }

hipError_t launch_sx(int B, int nproblems, int slot, long long wave_dirs_bytes, unsigned char* gdirs,
                     hipStream_t stream, const DevProblem* probs, const int* order, const uint32_t* blocks,
                     uint64_t nwords, const char* qseq, const char* qseq_uc, const int8_t* sctab,
                     const uint8_t* constab, gmapdp_result* results, gmapdp_pair* pairs) {
  if (B != 16 && B != 32) return hipErrorInvalidValue;
  void* fn = (B == 16) ? reinterpret_cast<void*>(&sx_kernel<16>) : reinterpret_cast<void*>(&sx_kernel<32>);
  const int np = 64 / B;
  const size_t lds = (size_t)slot * np;
  if (lds > 64 * 1024) {
    hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
  }
  const int nblocks = (nproblems + np - 1) / np;
  void* args[] = {(void*)&probs, (void*)&order, (void*)&nproblems, (void*)&slot, (void*)&wave_dirs_bytes,
                  (void*)&gdirs, (void*)&blocks, (void*)&nwords, (void*)&qseq, (void*)&qseq_uc, (void*)&sctab,
                  (void*)&constab, (void*)&results, (void*)&pairs};
  return hipLaunchKernel(fn, dim3(nblocks), dim3(64), args, lds, stream);
}

template <int R, bool D>
static void* gptr() { return reinterpret_cast<void*>(&gg_kernel<R, D>); }

size_t lds_bytes_gg(int rlength, int glengthL, int glengthR, int R, bool dirs_lds, int W) {
  return carve_gg(rlength, glengthL, glengthR, R, dirs_lds, W).total;
}
size_t scratch_bytes_gg(int rlength, int glengthL, int glengthR, int R, bool dirs_lds, int W) {
  return scratch_gg(rlength, glengthL, glengthR, R, dirs_lds, W).total;
}

hipError_t launch_gg(int R, bool dirs_lds, int nblocks, size_t lds, hipStream_t stream, const DevGenomeProblem* probs,
                     const int* order, const uint32_t* blocks, uint64_t nwords, const char* qseq,
                     const char* qseq_uc, const double* sprob, const int8_t* sctab, const uint8_t* constab,
                     const int8_t* isctab, gmapdp_genome_result* results, gmapdp_pair* pairs,
                     unsigned char* gscratch, const uint8_t* known, const double* metab) {
  void* fn = nullptr;
#define GMAPDP_CASE(RR)                                          \
  case RR:                                                       \
    fn = dirs_lds ? gptr<RR, true>() : gptr<RR, false>();        \
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
                  (void*)&sprob, (void*)&sctab, (void*)&constab, (void*)&isctab, (void*)&results, (void*)&pairs,
                  (void*)&gscratch, (void*)&known, (void*)&metab};
  return hipLaunchKernel(fn, dim3(nblocks), dim3(128), args, lds, stream);
}

}  // namespace gmapdp
