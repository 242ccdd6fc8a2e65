// me_kernel.hip -- CDNA4 (gfx950) kernels for GMAP's MaxEnt splice-site probabilities on the device
// (SURVEY §8a a11, §8f-2), over the HBM-resident .genomecomp genome and model tables (me_device.h):
//   me_sites_kernel  a list of (splice_pos, model, chroffset): gmapdp_maxent_sites
//   me_gap_kernel    every probability entry of a set of Dynprog_genome_gap problems, the positions and
//                    models of bridge_intron_gap_site_level (dynprog_genome.c:2573-2660; the host lists
//                    them the same way in gmapdp_genome_splice_sites): left entry cL at
//                    chroffset + goffsetL + cL (plus strand) or chrhigh - goffsetL - cL + 1, right entry cR
//                    at chroffset + rev_goffsetR - cR + 1 or chrhigh - rev_goffsetR + cR; donor / acceptor
//                    models for cdna_direction > 0, antiacceptor / antidonor otherwise, mirrored on the minus
//                    strand.  One workgroup per problem; the entries are independent (6 table loads each).
#include "dp_device.h"
#include "me_device.h"

namespace gmapdp {

__global__ __launch_bounds__(256) void me_sites_kernel(const uint32_t* __restrict__ blocks, uint64_t nwords,
                                                       const double* __restrict__ T,
                                                       const gmapdp_coord_t* __restrict__ pos,
                                                       const uint8_t* __restrict__ models,
                                                       const gmapdp_coord_t* __restrict__ chroffsets, long long n,
                                                       double* __restrict__ out) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
    out[i] = maxent_prob(blocks, nwords, T, models[i] & 3, pos[i], chroffsets[i]);
}

__global__ __launch_bounds__(256) void me_gap_kernel(const DevGenomeProblem* __restrict__ probs,
                                                     const int* __restrict__ order, int n,
                                                     const uint32_t* __restrict__ blocks, uint64_t nwords,
                                                     const double* __restrict__ T, double* __restrict__ sprob) {
  const int k = blockIdx.x;
  if (k >= n) return;
  const DevGenomeProblem P = probs[order ? order[k] : k];
  double* out = sprob + P.prob_offset;
  const int total = P.glengthL + P.glengthR;
  for (int e = threadIdx.x; e < total; e += blockDim.x) out[e] = gg_site_prob(P, blocks, nwords, T, e);
}

hipError_t launch_me_sites(long long n, hipStream_t s, const uint32_t* blocks, uint64_t nwords, const double* T,
                           const gmapdp_coord_t* pos, const uint8_t* models, const gmapdp_coord_t* chroffsets,
                           double* out) {
  if (n <= 0) return hipSuccess;
  const long long nb = std::min<long long>((n + 255) / 256, 65536);
  hipLaunchKernelGGL(me_sites_kernel, dim3((unsigned)nb), dim3(256), 0, s, blocks, nwords, T, pos, models,
                     chroffsets, n, out);
  return hipGetLastError();
}

hipError_t launch_me_gap(int n, hipStream_t s, const DevGenomeProblem* probs, const int* order,
                         const uint32_t* blocks, uint64_t nwords, const double* T, double* sprob) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(me_gap_kernel, dim3(n), dim3(256), 0, s, probs, order, n, blocks, nwords, T, sprob);
  return hipGetLastError();
}

}  // namespace gmapdp
