// sj_kernel.hip -- CDNA4 (gfx950) kernel for GMAP's Dynprog_end5_splicejunction and
// Dynprog_end3_splicejunction (nosimd semantics): the known-splice-site end alignments that
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
#include "dp_device.h"

namespace gmapdp {

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

  gmapdp_sj_result res;
  res.dynprogindex = P.dynprogindex;
  res.known_index = -1;
  res.pair_offset = P.pair_offset;
  if (finalscore < 0) {  // "Need a reasonable alignment to call a splice": nothing written
    if (lane == 0) {
      res.npairs = 0;
      res.traceback_score = res.missscore = kUnset;
      res.nmatches = res.nmismatches = res.nopens = res.nindels = kUnset;
      results[pid] = res;
    }
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
  const int score = t.score + t.nmatches * kMatch + t.nmismatches * kMismatch;
  // List_reverse, INDEL pairs at the far end dropped, and (end5) List_reverse again
  const int first = t.lead;
  const int npairs = t.count - first;
  int known = known_push - first;
  if (!end3) {
    if (npairs > 1) reverse_records(lane, out + first, npairs);
    known = npairs - 1 - known;
  }
  if (lane == 0) {
    res.npairs = npairs;
    res.pair_offset = P.pair_offset + first;
    res.traceback_score = score;
    res.missscore = score - rlen * kFullMatch;
    res.nmatches = t.nmatches;
    res.nmismatches = t.nmismatches;
    res.nopens = t.nopens;
    res.nindels = t.nindels;
    res.dynprogindex = P.dynprogindex + (P.dynprogindex > 0 ? 1 : -1);
    res.known_index = known;
    results[pid] = res;
  }
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

}  // namespace gmapdp
