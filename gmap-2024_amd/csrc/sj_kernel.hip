// sj_kernel.hip -- CDNA4 (gfx950) kernels for GMAP's Dynprog_end5_splicejunction and
// Dynprog_end3_splicejunction (sj_kernel: nosimd semantics; usj_kernel: the SIMD builds' triangles
// and traceback_local_8/16_upper/_lower, dynprog_end.c:729-1137): the known-splice-site end alignments that
// Splicetrie_solve_end5/3 run for every candidate far exon (splicetrie.c, via Dynprog_end5/3_known,
// dynprog_end.c:2748/3009).
//
// Reference semantics restated (paths under the reference tree's src/):
//   Dynprog_end5/3_splicejunction          dynprog_end.c:1653-1919 / 2249-2498
//   find_best_endpoint_to_queryend_indels  dynprog_end.c:515-572
//   traceback_local_std                    dynprog_end.c:1138-1289
//   Pairpool_add_genomeskip (genomesequence given)  pairpool.c:1068-1154
//
// One 64-lane wave per problem, as dp_kernel: the band-lane fill (fill_band, ENDQ scores, END
// penalties, wide band) against the caller's junction string -- staged from the batch's junction
// arena instead of the packed genome -- then the two-piece local traceback (traceback_local): the
// far exon's piece down to column `contlength`, the known-splice gap holder, the anchor piece down
// to column 0.  The direction planes stay in LDS unless the band is very wide (global scratch).
#include "ux_device.h"

namespace gmapdp {

// The list's tail, shared by both builds' kernels: List_reverse, the INDEL records at the far end
// dropped, end5's second List_reverse, and the out-parameters (dynprog_end.c:1900-1917).
__device__ __forceinline__ void sj_finish(int lane, const DevSjProblem& P, int pid, const Tally& t, int known_push,
                                          gmapdp_pair* out, gmapdp_sj_result* __restrict__ results) {
  const bool end3 = P.end3p != 0;
  const int score = t.score + t.nmatches * kMatch + t.nmismatches * kMismatch;
  const int first = t.lead;
  const int npairs = t.count - first;
  int known = known_push - first;
  if (!end3) {
    if (npairs > 1) reverse_records(lane, out + first, npairs);
    known = npairs - 1 - known;
  }
  if (lane == 0) {
    gmapdp_sj_result res;
    res.npairs = npairs;
    res.pair_offset = P.pair_offset + first;
    res.traceback_score = score;
    res.missscore = score - P.rlength * kFullMatch;
    res.nmatches = t.nmatches;
    res.nmismatches = t.nmismatches;
    res.nopens = t.nopens;
    res.nindels = t.nindels;
    res.dynprogindex = P.dynprogindex + (P.dynprogindex > 0 ? 1 : -1);
    res.known_index = known;
    results[pid] = res;
  }
}

// a negative best endpoint: NULL, nothing written (dynprog_end.c:1798-1800)
__device__ __forceinline__ void sj_null(int lane, const DevSjProblem& P, int pid, gmapdp_sj_result* __restrict__ results) {
  if (lane == 0) {
    gmapdp_sj_result res;
    res.npairs = 0;
    res.pair_offset = P.pair_offset;
    res.dynprogindex = P.dynprogindex;
    res.known_index = -1;
    res.traceback_score = res.missscore = kUnset;
    res.nmatches = res.nmismatches = res.nopens = res.nindels = kUnset;
    results[pid] = res;
  }
}

template <int R, bool DIRS_LDS>
__global__ __launch_bounds__(64) void sj_kernel(const DevSjProblem* __restrict__ probs, const int* __restrict__ order,
                                                const char* __restrict__ qseq, const char* __restrict__ qseq_uc,
                                                const char* __restrict__ jseq, const int8_t* __restrict__ sctab,
                                                const uint8_t* __restrict__ constab, gmapdp_sj_result* __restrict__ results,
                                                gmapdp_pair* __restrict__ pairs, uint64_t* __restrict__ gdirs) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int lane = threadIdx.x;
  const int pid = order[blockIdx.x];
  const DevSjProblem P = probs[pid];
  const int rlen = P.rlength, glen = P.glength;
  const bool end3 = P.end3p != 0;
  const bool rev = !end3;  // end5 runs away from the anchor (revp)
  const Carve cv = carve_dp(rlen, glen, R, DIRS_LDS);
  int8_t* sc = reinterpret_cast<int8_t*>(smem + cv.sc);
  char* q = reinterpret_cast<char*>(smem + cv.q);
  char* quc = reinterpret_cast<char*>(smem + cv.quc);
  char* gch = reinterpret_cast<char*>(smem + cv.gch);
  uint8_t* gcl = reinterpret_cast<uint8_t*>(smem + cv.gcls);
  uint64_t* dirs = DIRS_LDS ? reinterpret_cast<uint64_t*>(smem + cv.dirs)
                            : reinterpret_cast<uint64_t*>(reinterpret_cast<unsigned char*>(gdirs) + P.dirs_offset);
  const int8_t* sct = sctab + (size_t)kMismatchEndQ * 128 * kNClass;
  const uint8_t* cons = constab + (size_t)P.genestrand * 128 * kNClass;
  const int srow = rlen + 2;

  // ---- query rows (end5: rev_rsequence walks backwards), score rows, junction columns ----
  // end3 fills on rsequenceuc, end5 on rev_rsequence as given (as the end gaps, dynprog_end.c:1788/2384)
  const int qstep = rev ? -1 : 1;
  for (int i = lane; i < rlen; i += 64) {
    const char c1 = qseq[P.qbase + qstep * i];
    const char c1u = qseq_uc[P.qbase + qstep * i];
    q[i + 1] = c1;
    quc[i + 1] = c1u;
    const uint64_t row = *reinterpret_cast<const uint64_t*>(sct + (uint8_t)((end3 ? c1u : c1) & 127) * kNClass);
#pragma unroll
    for (int g = 0; g < 6; g++) sc[g * srow + i + 1] = (int8_t)(row >> (8 * g));
  }
  if (lane < 6) {
    sc[lane * srow] = 0;
    sc[lane * srow + rlen + 1] = 0;
  }
  // column c is gsequence[c-1] (end3) / rev_gsequence[-(c-1)] (end5); jbase indexes column 1
  for (int i = lane; i < glen; i += 64) {
    const char c2 = jseq[P.jbase + qstep * i];
    gch[i + 1] = c2;
    gcl[i + 1] = gclass(c2);
  }
  __syncthreads();

  const int lband = P.lband, uband = P.uband;
  const int W = lband + uband + 1;
  int bestr = 0, bestc = 0, finalscore = kNegInf32;
  fill_band<R, false>(lane, rlen, glen, lband, uband, P.open, P.extend, P.late, /*track*/ 2, sc, srow, gcl, dirs,
                      nullptr, bestr, bestc, 0, nullptr, &finalscore);
  if (DIRS_LDS) __syncthreads();
  else __threadfence_block();

  if (finalscore < 0) {  // "Need a reasonable alignment to call a splice": nothing written
    sj_null(lane, P, pid, results);
    return;
  }

  gmapdp_pair* out = pairs + P.pair_offset;
  const BandDirs<R, uint64_t> d{dirs, W, uband, 0};
  Tally t = {0, 0, 0, 0, 0, 0, 0, false};
  int r = bestr, c = bestc;
  const char* qv = q;
  const char* qucv = quc;
  const char* gv = gch;
  {  // the far exon's piece (genome positions from goffset_far)
    const Geo G{P.roffset, P.goffset_far, rev ? -1 : 1};
    traceback_local(lane, d, r, c, P.contlength, lband, uband, G, qv, qucv, gv, cons, out, t);
  }
  const int known_push = t.count;  // Pairpool_push_gapholder(..., knownp = true)
  if (lane == 0) put_pair(out, t.count, -1, -1, P.known_jump, ' ', ' ', ' ', ' ');
  t.count += 1;
  t.seen = true;
  {  // the anchor piece
    const Geo G{P.roffset, P.goffset_anchor, rev ? -1 : 1};
    traceback_local(lane, d, r, c, 0, lband, uband, G, qv, qucv, gv, cons, out, t);
  }
  sj_finish(lane, P, pid, t, known_push, out, results);
}

// ---- traceback_local_{8,16}_upper / _lower (dynprog_end.c:729-1137), the SIMD builds' ----
// One triangle per walk (upper when bestc >= bestr, re-decided for the anchor piece with the
// updated cell).  Upper: HORIZ gaps only, the E chain bounded by endc (its post-decrement: a chain
// stopped by endc rather than by a DIAG cell skips one column further), a final lazy genome skip
// to endc; lower: VERT gaps only, the F chain unbounded (the diagonal reads DIAG), a final lazy
// query skip to row 0.  The last skips leave (r, c) where they were, as the reference's do.
template <typename QV, typename GV>
__device__ __forceinline__ void traceback_local_tri(int lane, const UxView& V, bool upper, int& r, int& c, int endc,
                                                    const Geo& G, const QV& q, const QV& quc, const GV& gch,
                                                    const uint8_t* __restrict__ cons, gmapdp_pair* out, Tally& t) {
  while (r > 0 && c > endc) {
    if (upper ? V(c, 0, r) : V(c, 1, r)) {
      int n = 0;
      if (upper) {
        for (int base = 0;; base += 64) {
          const int j = base + lane;
          const bool cont = (c - j > endc) && V(c - j, 2, r);
          const uint64_t stop = ~ballot(cont);
          if (stop) { n = base + __ffsll((long long)stop) - 1; break; }
        }
        const int dist = n + 1;
        const int cn = (c - n > endc) ? c - n - 1 : c - n;
        emit_genomeskip_seq(lane, r, cn + dist, dist, G, gch, out, t);
        c = cn;
      } else {
        for (int base = 0;; base += 64) {
          const int j = base + lane;
          const bool cont = (r - j >= 0) && V(c, 3, r - j);
          const uint64_t stop = ~ballot(cont);
          if (stop) { n = base + __ffsll((long long)stop) - 1; break; }
        }
        emit_queryskip(lane, r, c, n + 1, G, q, out, t);
        r = r - n - 1;
      }
    } else {
      int n = 0;
      for (int base = 0;; base += 64) {
        const int j = base + lane;
        const bool cont = (j == 0) || ((r - j >= 1) && (c - j > endc) &&
                                       !(upper ? V(c - j, 0, r - j) : V(c - j, 1, r - j)));
        const uint64_t stop = ~ballot(cont);
        if (stop) { n = base + __ffsll((long long)stop) - 1; break; }
      }
      emit_diag(lane, r, c, n, G, q, quc, gch, cons, out, t);
      r -= n;
      c -= n;
    }
  }
  if (upper) {
    if (c != endc) emit_genomeskip_seq(lane, /*LAZY_INDEL*/ 1, c, c - endc, G, gch, out, t);
  } else if (r != 0) {
    emit_queryskip(lane, r, endc + /*LAZY_INDEL*/ 1, r, G, q, out, t);
  }
}

// usj_kernel<B>: Dynprog_end5/3_splicejunction as GMAP's SIMD builds compute them
// (dynprog_end.c:1741-1878 / 2339-2470): the upper and lower triangles of uxe_kernel (8-bit when
// either length is below use8p_size[ENDQ], else 16-bit) against the junction string,
// find_best_endpoint_to_queryend_indels_8/16, then the two local triangle walks.
template <int B>
__global__ __launch_bounds__(64) void usj_kernel(const DevSjProblem* __restrict__ probs, const int* __restrict__ order,
                                                 unsigned char* __restrict__ gscratch, const char* __restrict__ qseq,
                                                 const char* __restrict__ qseq_uc, const char* __restrict__ jseq,
                                                 const int8_t* __restrict__ sctab, const uint8_t* __restrict__ constab,
                                                 gmapdp_sj_result* __restrict__ results,
                                                 gmapdp_pair* __restrict__ pairs) {
  constexpr int NEG = (B == 32) ? -128 : -32768;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int lane = threadIdx.x;
  const int pid = order[blockIdx.x];
  const DevSjProblem P = probs[pid];
  const int rlen = P.rlength, glen = P.glength;
  const bool end3 = P.end3p != 0;
  const bool rev = !end3;
  const int qstep = rev ? -1 : 1;
  const int8_t* sct = sctab + (size_t)kMismatchEndQ * 128 * kNClass;
  const uint8_t* cons = constab + (size_t)P.genestrand * 128 * kNClass;
  const CarveUx cv = carve_ux(rlen, glen, B, 0);
  uint8_t* gcl = smem + cv.gcl;
  for (int i = lane; i < glen; i += 64) gcl[i + 1] = gclass(jseq[P.jbase + qstep * i]);
  __syncthreads();
  ux_stage<B>(lane, smem, cv, rlen, glen, (end3 ? qseq_uc : qseq) + P.qbase, qstep, sct);
  __syncthreads();
  UxFill F[2];
  F[0] = ux_fill<B>(smem, cv, true, rlen, glen, P.uband, P.late, P.open, P.extend, 0);
  F[1] = ux_fill<B>(smem, cv, false, rlen, glen, P.lband, P.late, P.open, P.extend, 0);
  const int tmax = max(ux_steps(rlen, P.uband, B), ux_steps(glen, P.lband, B));
  uint64_t* wd = reinterpret_cast<uint64_t*>(gscratch + P.dirs_offset);
  int16_t* ws = reinterpret_cast<int16_t*>(gscratch + P.dirs_offset + 16 * (size_t)tmax);
  ux_run_fills<B>(lane, F, 2, tmax, wd, ws);
  __threadfence_block();
  __syncthreads();
  const UxView VU = ux_view(wd, ws, 0, B, F[0], true), VL = ux_view(wd, ws, 1, B, F[1], false);

  // find_best_endpoint_to_queryend_indels_8/16 on row rlength (as uxe_kernel's indels scan)
  const int late = P.late;
  uint64_t key = 0;
  {
    const int r = rlen;
    const int clo = max(1, r - P.lband), chigh = min(r + P.uband, glen), cend = max(r - 1, chigh);
    for (int c = clo + lane; c <= cend; c += 64) {
      const int s = (c < r) ? VL.cell(r, c) : VU.cell(r, c);
      if (late ? (s >= NEG) : (s > NEG)) {
        const uint32_t ord = ((uint32_t)r << 12) | (uint32_t)c;
        const uint64_t kk = ((uint64_t)(uint32_t)(s + (1 << 30)) << 24) | (late ? ord : 0xffffffu - ord);
        key = kk > key ? kk : key;
      }
    }
  }
  key = wave_max_u64(key);
  if (key == 0 || (int)(uint32_t)(key >> 24) - (1 << 30) < 0) {
    sj_null(lane, P, pid, results);
    return;
  }
  const uint32_t ord = late ? (uint32_t)(key & 0xffffffu) : 0xffffffu - (uint32_t)(key & 0xffffffu);
  int r = (int)(ord >> 12), c = (int)(ord & 4095u);

  gmapdp_pair* out = pairs + P.pair_offset;
  Tally t = {0, 0, 0, 0, 0, 0, 0, false};
  const QView qv{qseq + P.qbase, qstep}, qucv{qseq_uc + P.qbase, qstep};
  const GClassView gv{gcl};
  {
    const Geo G{P.roffset, P.goffset_far, rev ? -1 : 1};
    const bool up = c >= r;
    traceback_local_tri(lane, up ? VU : VL, up, r, c, P.contlength, G, qv, qucv, gv, cons, out, t);
  }
  const int known_push = t.count;
  if (lane == 0) put_pair(out, t.count, -1, -1, P.known_jump, ' ', ' ', ' ', ' ');
  t.count += 1;
  t.seen = true;
  {
    const Geo G{P.roffset, P.goffset_anchor, rev ? -1 : 1};
    const bool up = c >= r;  // re-decided with the cell the far piece ended on (dynprog_end.c:1827)
    traceback_local_tri(lane, up ? VU : VL, up, r, c, 0, G, qv, qucv, gv, cons, out, t);
  }
  sj_finish(lane, P, pid, t, known_push, out, results);
}

// ---- host-side launch table ----
size_t lds_bytes_sj(int rlength, int glength, int R, bool dirs_lds) { return carve_dp(rlength, glength, R, dirs_lds).total; }

hipError_t launch_sj(int R, bool dirs_lds, int nblocks, size_t lds, hipStream_t stream, const DevSjProblem* probs,
                     const int* order, const char* qseq, const char* qseq_uc, const char* jseq, const int8_t* sctab,
                     const uint8_t* constab, gmapdp_sj_result* results, gmapdp_pair* pairs, uint64_t* gdirs) {
  void* fn = nullptr;
#define GMAPDP_CASE(RR)                                                                                 \
  case RR:                                                                                              \
    fn = dirs_lds ? reinterpret_cast<void*>(&sj_kernel<RR, true>) : reinterpret_cast<void*>(&sj_kernel<RR, false>); \
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
  void* args[] = {(void*)&probs, (void*)&order, (void*)&qseq, (void*)&qseq_uc, (void*)&jseq,
                  (void*)&sctab, (void*)&constab, (void*)&results, (void*)&pairs, (void*)&gdirs};
  return hipLaunchKernel(fn, dim3(nblocks), dim3(64), args, lds, stream);
}

hipError_t launch_usj(int B, int nblocks, size_t lds, hipStream_t stream, const DevSjProblem* probs, const int* order,
                      unsigned char* gscratch, const char* qseq, const char* qseq_uc, const char* jseq,
                      const int8_t* sctab, const uint8_t* constab, gmapdp_sj_result* results, gmapdp_pair* pairs) {
  if (B != 16 && B != 32) return hipErrorInvalidValue;
  void* fn = (B == 16) ? reinterpret_cast<void*>(&usj_kernel<16>) : reinterpret_cast<void*>(&usj_kernel<32>);
  if (lds > 64 * 1024) {
    hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
  }
  void* args[] = {(void*)&probs, (void*)&order, (void*)&gscratch, (void*)&qseq, (void*)&qseq_uc, (void*)&jseq,
                  (void*)&sctab, (void*)&constab, (void*)&results, (void*)&pairs};
  return hipLaunchKernel(fn, dim3(nblocks), dim3(64), args, lds, stream);
}

}  // namespace gmapdp
