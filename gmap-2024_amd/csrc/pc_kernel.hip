// pc_kernel.hip -- the compact pair stream ("run-length ops + per-record character codes, the host
// expands them into Pair_Ts").  The DP kernels write each call's Pair_T list as 16-B
// gmapdp_pair records (pairdef.h:8-42 flattened: querypos, genomepos, jump, cdna, comp, genome, genomealt) in
// List_T order; a caller that moves the pairs to the host (the drop-in, or the bench's like-for-like line)
// reads ~12 k records per 2-kb read.  Consecutive records of a list mostly step both positions by one (a
// diagonal run of matches and mismatches) or one of them (an indel run), and their characters are a few
// (cdna, comp, genome) combinations.  So each call's list becomes a byte stream of ops:
//   RUN  : 0x01, int32 querypos, int32 genomepos, int8 dq, int8 dg, uint16 len (13 B), then one byte per
//          record: cdna | genome << 2 | comp << 4 (cdna, genome in ACGT, comp one of '*' '|' ' ' ':',
//          genomealt = genome), or 0xFF and the record's four characters;
//   RAW  : 0x02 and the 16-B record (gap holders, records with a jump or a negative position).
// Stage 2's path pairs (gmapdp_path_pair, 20 B: querypos, genomepos, queryjump, genomejump, the four
// characters; stage2.c convert_to_nucleotides) take the same ops with a 21-B RAW (any jump or negative
// position); their lists are the plan's paths (gmapdp_path: pair_offset, npairs).
// Record k of a RUN sits at (querypos + k dq, genomepos + k dg).  A 10 000-read bench block's 94 M records
// (1.5 GB) take ~0.1 GB.  gmapdp_expand_pairs (gmapdp_engine.cpp) restores the records exactly.
//
// One wave per call, 64 records per step.  Record i continues the current run when neither it nor record i - 1
// is RAW, its step from i - 1 is within [-1, 1]^2, and either that step equals the step into i - 1 or i - 1
// had no step (it starts the list or follows a RAW record): every run's records then share the step of its
// second record, with no sequential decision.  A run's length and step are written when its end is seen
// (possibly a step later).  The first launch (WRITE = false) sizes every call's stream; a one-workgroup scan
// turns the sizes into offsets; the second writes.
#include "dp_device.h"

namespace gmapdp {

constexpr unsigned char kPcRun = 0x01, kPcRaw = 0x02, kPcEsc = 0xFF;
constexpr int kPcHeader = 13;

__device__ __forceinline__ int pc_nt(char c) {
  return c == 'A' ? 0 : c == 'C' ? 1 : c == 'G' ? 2 : c == 'T' ? 3 : -1;
}
__device__ __forceinline__ int pc_comp(char c) {
  return c == '*' ? 0 : c == '|' ? 1 : c == ' ' ? 2 : c == ':' ? 3 : -1;
}
// the record's one-byte code from its four characters (cdna, comp, genome, genomealt), or -1: escaped
__device__ __forceinline__ int pc_code(uint32_t ch) {
  const char cdna = (char)(ch & 0xFF), comp = (char)((ch >> 8) & 0xFF), gen = (char)((ch >> 16) & 0xFF),
             alt = (char)(ch >> 24);
  const int a = pc_nt(cdna), b = pc_nt(gen), c = pc_comp(comp);
  return (a < 0 || b < 0 || c < 0 || alt != gen) ? -1 : a | (b << 2) | (c << 4);
}

// the DP lists: n0 records of stride s0 bytes then n1 of stride s1 (gmapdp_result / gmapdp_genome_result:
// npairs at byte 0, pair_offset at byte 4); 16-B gmapdp_pair records
struct PcProblems {
  const unsigned char* r0;
  const unsigned char* r1;
  int n0, n1, s0, s1;
  const int4* pairs;
  static constexpr int kRaw = 17;
  __device__ __forceinline__ void list(int i, int& npairs, long long& off) const {
    const int* r = reinterpret_cast<const int*>(i < n0 ? r0 + (size_t)i * s0 : r1 + (size_t)(i - n0) * s1);
    npairs = r[0];
    off = r[1];
  }
  // record k of the list at `off`: positions, whether it must go RAW, its characters; raw bytes for RAW
  __device__ __forceinline__ void rec(long long off, int k, int& q, int& g, bool& jump, uint32_t& ch) const {
    const int4 r = pairs[off + k];
    q = r.x;
    g = r.y;
    jump = r.z != 0;
    ch = (uint32_t)r.w;
  }
  __device__ __forceinline__ const unsigned char* raw(long long off, int k) const {
    return reinterpret_cast<const unsigned char*>(pairs + off + k);
  }
};
// stage 2's path lists: the plan's paths (count in *npaths, at most the launch's grid), 20-B gmapdp_path_pair
struct PcPaths {
  const gmapdp_path* paths;
  const unsigned long long* npaths;
  const gmapdp_path_pair* pairs;
  unsigned long long pair_cap;
  static constexpr int kRaw = 21;
  __device__ __forceinline__ void list(int i, int& npairs, long long& off) const {
    npairs = 0;
    off = 0;
    if ((unsigned long long)i >= *npaths) return;
    const gmapdp_path p = paths[i];
    // (a call that overflowed the pools reports status -2; its records need not be in the pool)
    if (p.pair_offset < 0 || p.npairs < 0 || (unsigned long long)p.pair_offset + p.npairs > pair_cap) return;
    npairs = p.npairs;
    off = p.pair_offset;
  }
  __device__ __forceinline__ void rec(long long off, int k, int& q, int& g, bool& jump, uint32_t& ch) const {
    const int* r = reinterpret_cast<const int*>(pairs + off + k);
    q = r[0];
    g = r[1];
    jump = (r[2] | r[3]) != 0;
    ch = (uint32_t)r[4];
  }
  __device__ __forceinline__ const unsigned char* raw(long long off, int k) const {
    return reinterpret_cast<const unsigned char*>(pairs + off + k);
  }
};

template <bool WRITE, typename Src>
__global__ __launch_bounds__(64) void pc_kernel(Src P, unsigned long long* __restrict__ sizes_or_offsets,
                                               unsigned char* __restrict__ out) {
  const int lane = threadIdx.x;
  const int i = blockIdx.x;
  int npairs;
  long long off;
  P.list(i, npairs, off);
  npairs = max(npairs, 0);
  unsigned char* o = WRITE ? out + sizes_or_offsets[i] : nullptr;
  unsigned long long pos = 0;  // bytes written so far
  // carries: the previous record (q, g, raw), the step into it (valid?), the open run's header position
  int pq = 0, pg = 0, praw = 1, pdq = 0, pdg = 0, pstep = 0;
  long long hdr = -1;  // the open run's header offset (WRITE), -1: none
  int runlen = 0, rdq = 0, rdg = 0;
  for (int c0 = 0; c0 < npairs; c0 += 64) {
    const int k = c0 + lane;
    const bool v = k < npairs;
    int q = 0, g = 0;
    bool jump = false;
    uint32_t ch = 0;
    if (v) P.rec(off, k, q, g, jump, ch);
    const bool raw = v && (jump || q < 0 || g < 0);
    // the previous record (lane - 1, or the carry)
    int q1 = __shfl_up(q, 1, 64), g1 = __shfl_up(g, 1, 64);
    int raw1 = __shfl_up(raw ? 1 : 0, 1, 64);
    if (lane == 0) {
      q1 = pq;
      g1 = pg;
      raw1 = c0 == 0 ? 1 : praw;
    }
    const int dq = q - q1, dg = g - g1;
    const bool stepok = v && !raw && !raw1 && dq >= -1 && dq <= 1 && dg >= -1 && dg <= 1;
    // the step into the previous record (0: none)
    int s1q = __shfl_up(dq, 1, 64), s1g = __shfl_up(dg, 1, 64), s1v = __shfl_up(stepok ? 1 : 0, 1, 64);
    if (lane == 0) {
      s1q = pdq;
      s1g = pdg;
      s1v = c0 == 0 ? 0 : pstep;
    }
    const bool cont = stepok && (!s1v || (dq == s1q && dg == s1g));
    const bool start = v && !raw && !cont;
    const int code = v && !raw ? pc_code(ch) : 0;
    const int bytes = !v ? 0 : raw ? Src::kRaw : (start ? kPcHeader : 0) + (code < 0 ? 5 : 1);
    const int incl = wave_scan_add(lane, bytes);
    const unsigned long long at = pos + (unsigned long long)(incl - bytes);
    // run ends: the open run (from an earlier step, or a lane below) closes at the first record that does not
    // continue it
    const uint64_t sm = ballot(v && !cont);            // records that begin a run or are RAW
    if (WRITE) {
      if (raw) {
        o[at] = kPcRaw;
        const unsigned char* b = P.raw(off, k);
        for (int x = 0; x < Src::kRaw - 1; x++) o[at + 1 + x] = b[x];
      } else if (v) {
        unsigned long long p = at;
        if (start) {
          o[p] = kPcRun;
          const unsigned char* bq = reinterpret_cast<const unsigned char*>(&q);
          const unsigned char* bg = reinterpret_cast<const unsigned char*>(&g);
          for (int x = 0; x < 4; x++) {
            o[p + 1 + x] = bq[x];
            o[p + 5 + x] = bg[x];
          }
          p += kPcHeader;  // (step and length: written below when the run's end is seen)
        }
        if (code < 0) {
          o[p] = kPcEsc;
          for (int x = 0; x < 4; x++) o[p + 1 + x] = (unsigned char)(ch >> (8 * x));
        } else {
          o[p] = (unsigned char)code;
        }
      }
    }
    // run bookkeeping (wave-uniform): a run ends just before the next record that does not continue it
    {
      uint64_t starts = ballot(start);
      // the run open from the previous step continues through this step's lanes before its first
      // non-continuing record
      const int first_nc = sm ? __ffsll((long long)sm) - 1 : 64;
      if (hdr >= 0 || runlen > 0) {
        const int more = min(first_nc, max(0, min(64, npairs - c0)));
        // its step: the step of its second record (this step's lane 0 when the run had one record so far)
        if (runlen == 1 && more > 0) {
          rdq = __builtin_amdgcn_readlane(dq, 0);
          rdg = __builtin_amdgcn_readlane(dg, 0);
        }
        runlen += more;
        if (first_nc < 64 && first_nc < npairs - c0) {  // closed here
          if (WRITE && lane == 0 && hdr >= 0) {
            o[hdr + 9] = (unsigned char)(int8_t)(runlen > 1 ? rdq : 0);
            o[hdr + 10] = (unsigned char)(int8_t)(runlen > 1 ? rdg : 0);
            o[hdr + 11] = (unsigned char)(runlen & 0xFF);
            o[hdr + 12] = (unsigned char)(runlen >> 8);
          }
          hdr = -1;
          runlen = 0;
        }
      }
      // runs that start and end inside this step: written by their start lane below; the last start of the
      // step stays open
      while (starts) {
        const int s = __ffsll((long long)starts) - 1;
        starts &= starts - 1;
        const uint64_t above = s < 63 ? (sm >> (s + 1)) : 0ull;
        const int valid_end = min(64, npairs - c0);
        int len;
        bool closed;
        if (above && (__ffsll((long long)above) + s) < valid_end) {
          len = __ffsll((long long)above);
          closed = true;
        } else {
          len = valid_end - s;
          closed = valid_end < 64 ? true : false;  // the list ends in this step
          if (valid_end == 64 && c0 + 64 >= npairs) closed = true;
        }
        const int sdq = len > 1 ? __builtin_amdgcn_readlane(dq, min(s + 1, 63)) : 0;
        const int sdg = len > 1 ? __builtin_amdgcn_readlane(dg, min(s + 1, 63)) : 0;
        const unsigned long long h = pos + (unsigned long long)(__builtin_amdgcn_readlane(incl, s) -
                                                                __builtin_amdgcn_readlane(bytes, s));
        if (closed) {
          if (WRITE && lane == 0) {
            o[h + 9] = (unsigned char)(int8_t)sdq;
            o[h + 10] = (unsigned char)(int8_t)sdg;
            o[h + 11] = (unsigned char)(len & 0xFF);
            o[h + 12] = (unsigned char)(len >> 8);
          }
        } else {  // open into the next step
          hdr = (long long)h;
          runlen = len;
          rdq = sdq;
          rdg = sdg;
        }
      }
    }
    pos += (unsigned long long)__builtin_amdgcn_readlane(incl, 63);
    pq = __builtin_amdgcn_readlane(q, 63);
    pg = __builtin_amdgcn_readlane(g, 63);
    praw = __builtin_amdgcn_readlane(raw ? 1 : 0, 63);
    pdq = __builtin_amdgcn_readlane(dq, 63);
    pdg = __builtin_amdgcn_readlane(dg, 63);
    pstep = __builtin_amdgcn_readlane(stepok ? 1 : 0, 63);
  }
  if (WRITE && lane == 0 && hdr >= 0) {  // a run open at the list's end (its last step was full)
    o[hdr + 9] = (unsigned char)(int8_t)(runlen > 1 ? rdq : 0);
    o[hdr + 10] = (unsigned char)(int8_t)(runlen > 1 ? rdg : 0);
    o[hdr + 11] = (unsigned char)(runlen & 0xFF);
    o[hdr + 12] = (unsigned char)(runlen >> 8);
  }
  if (!WRITE && lane == 0) sizes_or_offsets[i] = pos;
}

// exclusive prefix sums of n sizes in place, n + 1 entries (the last: the total); one workgroup of 1024
__global__ __launch_bounds__(1024) void pc_scan_kernel(unsigned long long* __restrict__ v, int n) {
  __shared__ unsigned long long part[1024];
  const int t = threadIdx.x;
  const int per = (n + 1023) / 1024;
  const int lo = min(n, t * per), hi = min(n, lo + per);
  unsigned long long s = 0;
  for (int i = lo; i < hi; i++) s += v[i];
  part[t] = s;
  __syncthreads();
  for (int off = 1; off < 1024; off <<= 1) {
    const unsigned long long x = t >= off ? part[t - off] : 0ull;
    __syncthreads();
    part[t] += x;
    __syncthreads();
  }
  unsigned long long run = part[t] - s;
  for (int i = lo; i < hi; i++) {
    const unsigned long long x = v[i];
    v[i] = run;
    run += x;
  }
  if (t == 1023) v[n] = part[1023];
}

hipError_t launch_pc(const unsigned char* r0, int n0, int s0, const unsigned char* r1, int n1, int s1,
                     const gmapdp_pair* pairs, unsigned long long* offsets, unsigned char* out, hipStream_t stream) {
  PcProblems P{r0, r1, n0, n1, s0, s1, reinterpret_cast<const int4*>(pairs)};
  const int n = n0 + n1;
  if (n <= 0) return hipMemsetAsync(offsets, 0, sizeof(unsigned long long), stream);
  hipLaunchKernelGGL((pc_kernel<false, PcProblems>), dim3(n), dim3(64), 0, stream, P, offsets, (unsigned char*)nullptr);
  hipLaunchKernelGGL(pc_scan_kernel, dim3(1), dim3(1024), 0, stream, offsets, n);
  if (out) hipLaunchKernelGGL((pc_kernel<true, PcProblems>), dim3(n), dim3(64), 0, stream, P, offsets, out);
  return hipGetLastError();
}

// stage 2: path_cap lists (those past *npaths are empty), offsets path_cap + 1 entries
hipError_t launch_pc_paths(const gmapdp_path* paths, const unsigned long long* npaths, int path_cap,
                           const gmapdp_path_pair* pairs, unsigned long long pair_cap, unsigned long long* offsets,
                           unsigned char* out, hipStream_t stream) {
  PcPaths P{paths, npaths, pairs, pair_cap};
  if (path_cap <= 0) return hipMemsetAsync(offsets, 0, sizeof(unsigned long long), stream);
  hipLaunchKernelGGL((pc_kernel<false, PcPaths>), dim3(path_cap), dim3(64), 0, stream, P, offsets,
                     (unsigned char*)nullptr);
  hipLaunchKernelGGL(pc_scan_kernel, dim3(1), dim3(1024), 0, stream, offsets, path_cap);
  if (out) hipLaunchKernelGGL((pc_kernel<true, PcPaths>), dim3(path_cap), dim3(64), 0, stream, P, offsets, out);
  return hipGetLastError();
}

}  // namespace gmapdp
