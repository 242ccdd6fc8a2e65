// mx_kernel.hip -- CDNA4 (gfx950) kernels for Dynprog_microexon_int (SURVEY §8a a15;
// dynprog_single.c:900-1182), the microexon search stage 3 runs inside an intron (stage3.c:9664).
//
// mx_search_kernel, one wave per call:
//   - leftbound / rightbound (:1001-1047): mismatch flags of 64 query positions per step as one
//     ballot; the bound is the second mismatch (the popcount of the ballots so far);
//   - the cL with the intron's 5' dinucleotide (:1053-1062), 64 per ballot, visited in ascending
//     order; for each, the cR in [mincR, maxcR] with its 3' dinucleotide (:1063-1085);
//   - the exact search of the middle piece in the intron text (BoyerMoore_nt, boyer-moore.c:356:
//     every occurrence j in [0, textlen - querylen]; none when the piece holds anything but A/C/G/T):
//     64 offsets per step, lane l tests j = top - l so that the ballot order is the reference's hit
//     order (Intlist_push: descending j), each offset one compare of the piece's 2-bit codes (its
//     reverse complement on the minus strand) with the packed genome words, N flags and the
//     segment's chromosome bound included;
//   - the flank test (:1109-1116) and the candidate's two splice sites (:1120-1144).
//   Candidates collect in LDS and leave with one atomic per call; a call with more than kMxCap of
//   them reports its exact count and the host reruns it writing straight to its own region.
// mx_finish_kernel, one wave per call: the (float) prob2 + prob3 > best rule (:1147) over the
//   candidates in order, then make_microexon_pairs_double (:683) with every record placed by a ballot
//   rank (Pairpool_push drops negative positions, pairpool.c:188) in List_T order.
#include "dp_device.h"
#include "me_device.h"

namespace gmapdp {

constexpr int kMxMin = 3;       // MIN_MICROEXON_LENGTH (dynprog_single.c:83)
constexpr int kMxMax = 12;      // MAX_MICROEXON_LENGTH (:87, GMAP)
constexpr int kMxIntron = 9;    // MICROINTRON_LENGTH (:89)
constexpr int kMxCap = 256;     // candidates per call held in LDS

// 2-bit codes (A0 C1 G2 T3, first position in bits 1:0) of genome positions [lo, lo + ml), ml <= 12, straight
// from the packed .genomecomp words; false when one of them is an N (flags) or past the allocation
// (decode_nt reads those as N, which no A/C/G/T piece matches)
__device__ __forceinline__ bool mx_window(const uint32_t* __restrict__ blocks, uint64_t nwords, uint64_t lo, int ml,
                                          uint32_t& codes) {
  const uint64_t hi = lo + (uint64_t)ml - 1u;
  const uint64_t b0 = lo >> 5, b1 = hi >> 5;
  if (3 * b1 + 2 >= nwords) return false;
  uint64_t f = blocks[3 * b0 + 2];
  if (b1 != b0) f |= (uint64_t)blocks[3 * b1 + 2] << 32;
  if ((f >> (lo & 31u)) & ((1ull << ml) - 1ull)) return false;
  const uint64_t h = lo >> 4;  // half-words: even = low word (nt 0-15 of the block), odd = high word
  const uint32_t w0 = blocks[3 * (size_t)(h >> 1) + ((h & 1u) ? 0 : 1)];
  uint64_t x = w0;
  if ((lo & 15u) + (uint32_t)ml > 16u) {
    const uint64_t h1 = h + 1u;
    x |= (uint64_t)blocks[3 * (size_t)(h1 >> 1) + ((h1 & 1u) ? 0 : 1)] << 32;
  }
  codes = (uint32_t)(x >> (2u * (lo & 15u))) & ((1u << (2 * ml)) - 1u);
  return true;
}

// mx_window without its early return: the flag and code words are loaded together (addresses clamped in
// range), so the text scan below can have several steps' loads in flight instead of two dependent round
// trips per step
__device__ __forceinline__ bool mx_window_nb(const uint32_t* __restrict__ blocks, uint64_t nwords, uint64_t lo,
                                             int ml, uint32_t& codes) {
  const uint64_t hi = lo + (uint64_t)ml - 1u;
  const uint64_t b0 = lo >> 5, b1 = hi >> 5;
  const bool ok = 3 * b1 + 2 < nwords;
  // (b1 == b0: the window's flag bits all lie in the first word; the second word's bits land above them)
  const uint64_t f = (uint64_t)blocks[ok ? 3 * b0 + 2 : 2] | ((uint64_t)blocks[ok ? 3 * b1 + 2 : 2] << 32);
  const uint64_t h = lo >> 4, h1 = h + 1u;  // half-words: even = low word (nt 0-15 of the block), odd = high
  uint64_t i0 = 3 * (h >> 1) + ((h & 1u) ? 0 : 1), i1 = 3 * (h1 >> 1) + ((h1 & 1u) ? 0 : 1);
  if (!ok) i0 = 0;
  if (!ok || i1 >= nwords) i1 = 0;  // (only when the window does not reach half-word h1)
  const uint64_t x = (uint64_t)blocks[i0] | ((uint64_t)blocks[i1] << 32);
  codes = (uint32_t)(x >> (2u * (lo & 15u))) & ((1u << (2 * ml)) - 1u);
  return ok && !((f >> (lo & 31u)) & ((1ull << ml) - 1ull));
}

// the second mismatch among n flags produced 64 at a time by `flag(i)`; n - 1 when there is none
template <class F>
__device__ __forceinline__ int mx_second_mismatch(int n, int lane, F flag) {
  int seen = 0;
  for (int base = 0; base < n; base += 64) {
    const int i = base + lane;
    const uint64_t m = ballot(i < n && flag(i));
    const int c = __popcll(m);
    if (seen + c >= 2) {
      uint64_t x = m;
      if (seen == 0) x &= x - 1;  // drop the first mismatch of this step
      return base + __ffsll((long long)x) - 1;
    }
    seen += c;
  }
  return n - 1;
}

__global__ __launch_bounds__(64) void mx_search_kernel(const gmapdp_microexon_problem* __restrict__ probs, int n,
                                                       const uint32_t* __restrict__ blocks, uint64_t nwords,
                                                       const char* __restrict__ qseq,
                                                       const char* __restrict__ qseq_uc,
                                                       gmapdp_microexon_result* __restrict__ results,
                                                       gmapdp_microexon_candidate* __restrict__ cands,
                                                       unsigned long long cand_cap,
                                                       unsigned long long* __restrict__ counter,
                                                       const int64_t* __restrict__ direct) {
  __shared__ gmapdp_microexon_candidate lc[kMxCap];
  const int pi = blockIdx.x;
  if (pi >= n) return;
  const int lane = threadIdx.x;
  const gmapdp_microexon_problem P = probs[pi];
  const int64_t dst = direct ? direct[pi] : -1;  // rerun of an overflowing call: its own region
  if (direct && dst < 0) return;
  gmapdp_microexon_result R;
  R.ncandidates = 0;
  R.dynprogindex = P.dynprogindex;
  R.microintrontype = P.cdna_direction > 0 ? 0x20 : P.cdna_direction < 0 ? 0x04 : 0;
  R.npairs = -1;
  R.cand_offset = 0;
  R.pair_offset = 0;
  R.bestprob2 = R.bestprob3 = 0.0;
  const bool watson = P.watsonp != 0;
  const char* rs = qseq + P.qoff;
  const char* ruc = qseq_uc + P.qoff;
  int ncand = 0;
  if (P.cdna_direction != 0) {
    const char i1 = P.cdna_direction > 0 ? 'G' : 'C', i2 = 'T', i3 = 'A', i4 = P.cdna_direction > 0 ? 'G' : 'C';
    auto gnt = [&](int g) { return genomic_nt(blocks, nwords, g, P.chroffset, P.chrhigh, watson); };
    const int rl = P.rlength;
    const int leftbound = rl - 1 <= 0 ? -1
                                      : mx_second_mismatch(rl - 1, lane, [&](int i) { return ruc[i] != gnt(P.goffsetL + i); });
    const int rightbound = rl <= 0 ? -1
                                   : mx_second_mismatch(rl, lane, [&](int k) { return ruc[rl - 1 - k] != gnt(P.rev_goffsetR - k); });
    for (int base = 1; base <= leftbound; base += 64) {
      const int cl = base + lane;
      uint64_t mL = ballot(cl <= leftbound && gnt(P.goffsetL + cl) == i1 && gnt(P.goffsetL + cl + 1) == i2);
      while (mL) {
        const int cL = base + __ffsll((long long)mL) - 1;
        mL &= mL - 1;
        const int mincR = max(rl - kMxMax - cL, 1);
        const int maxcR = min(rl - kMxMin - cL, rightbound);
        for (int cR = mincR; cR <= maxcR; cR++) {
          if (gnt(P.rev_goffsetR - cR - 1) != i3 || gnt(P.rev_goffsetR - cR) != i4) continue;
          const int ml = rl - cL - cR;
          const int textleft = P.goffsetL + cL + kMxIntron;
          const int textright = P.rev_goffsetR - cR - kMxIntron;
          if (textright < textleft + ml) continue;
          // query_okay (boyer-moore.c:263) on the mixed-case piece
          const char qc = lane < ml ? rs[cL + lane] : 'A';
          if (ballot(qc != 'A' && qc != 'C' && qc != 'G' && qc != 'T')) continue;
          // the piece as 2-bit codes, and as the genome shows it on the minus strand (reverse complement)
          const uint32_t qcode = qc == 'A' ? 0u : qc == 'C' ? 1u : qc == 'G' ? 2u : 3u;
          uint32_t pat = 0, rcpat = 0;
          for (int k = 0; k < ml; k++) {
            const uint32_t ck = (uint32_t)__builtin_amdgcn_readlane((int)qcode, k);
            pat |= ck << (2 * k);
            rcpat |= (3u - ck) << (2 * (ml - 1 - k));
          }
          const int textlen = textright - textleft;
          // BoyerMoore_nt's text (Genome_get_segment_right / _left, boyer-moore.c:372-378): text[i] is
          // genome[chroffset + textleft + i] (plus; '*' from chrhigh on) or the complement of
          // genome[chrhigh - textleft - i] (minus; '*' below chroffset)
          const int64_t base = watson ? (int64_t)P.chroffset + textleft : (int64_t)P.chrhigh - textleft;
          // 2 048 offsets per step: lane l takes the 32 offsets j = J0 - k (J0 = top - 32 l, k = 0..31), whose
          // windows lie in 32 + ml - 1 genome positions from G0 -- decoded once from four half-words and three
          // flag words -- and tests them from registers.  Descending j is lane order, then k: the candidates
          // keep the reference's hit order (Intlist_push over descending j).  A lane whose positions run
          // outside the genome's words (or below 0) tests its offsets one by one as mx_window does.
          const uint32_t want = watson ? pat : rcpat;
          const uint32_t cmask = (1u << (2 * ml)) - 1u, fmask = (1u << ml) - 1u;
          for (int top = textlen - ml; top >= 0; top -= 64 * 32) {
            const int J0 = top - 32 * lane;
            uint32_t m = 0;  // bit k: offset J0 - k matches (window, N flags, chromosome bound)
            if (J0 >= 0) {
              const int kmax = min(31, J0);
              const int64_t G0 = watson ? base + J0 - 31 : base - J0 - (ml - 1);
              const uint64_t h0 = (uint64_t)G0 >> 4, b0 = (uint64_t)G0 >> 5;
              const uint64_t hlast = h0 + 3, wlast = 3 * (hlast >> 1) + ((hlast & 1u) ? 0 : 1);
              const bool fast = G0 >= 0 && wlast < nwords && 3 * (b0 + 2) + 2 < nwords;
              if (fast) {
                auto hw = [&](uint64_t h) { return (uint64_t)blocks[3 * (h >> 1) + ((h & 1u) ? 0 : 1)]; };
                const uint64_t A = hw(h0) | (hw(h0 + 1) << 32), B = hw(h0 + 2) | (hw(h0 + 3) << 32);
                const uint32_t sh = 2u * ((uint32_t)G0 & 15u);
                const uint64_t lo = sh ? (A >> sh) | (B << (64 - sh)) : A, hi = B >> sh;
                const uint64_t FA = (uint64_t)blocks[3 * b0 + 2] | ((uint64_t)blocks[3 * (b0 + 1) + 2] << 32);
                const uint64_t FB = blocks[3 * (b0 + 2) + 2];
                const uint32_t fs = (uint32_t)G0 & 31u;
                const uint64_t fl = fs ? (FA >> fs) | (FB << (64 - fs)) : FA;
#pragma unroll
                for (int k = 0; k < 32; k++) {
                  const int sidx = watson ? 31 - k : k;  // the window's first position, from G0
                  const int64_t st = G0 + sidx;
                  const bool inb = watson ? st + ml <= (int64_t)P.chrhigh : st >= (int64_t)P.chroffset;
                  const uint64_t w = sidx ? (lo >> (2 * sidx)) | (hi << (64 - 2 * sidx)) : lo;
                  const bool h = k <= kmax && inb && !((uint32_t)(fl >> sidx) & fmask) &&
                                 ((uint32_t)w & cmask) == want;
                  m |= (h ? 1u : 0u) << k;
                }
              } else {
                for (int k = 0; k <= kmax; k++) {
                  const int j = J0 - k;
                  const int64_t st = watson ? base + j : base - j - (ml - 1);
                  const bool inb = st >= 0 && (watson ? st + ml <= (int64_t)P.chrhigh : st >= (int64_t)P.chroffset);
                  uint32_t codes;
                  const bool w = mx_window_nb(blocks, nwords, inb ? (uint64_t)st : 0u, ml, codes);
                  if (inb && w && codes == want) m |= 1u << k;
                }
              }
              // the flanking dinucleotides of each match (rare: a few per call)
              for (uint32_t r = m; r; r &= r - 1) {
                const int k = __ffs(r) - 1;
                const int cand = textleft + J0 - k;
                if (!(gnt(cand - 2) == i3 && gnt(cand - 1) == i4 && gnt(cand + ml) == i1 && gnt(cand + ml + 1) == i2))
                  m &= ~(1u << k);
              }
            }
            const int cnt = __popc(m);
            const int incl = wave_scan_add(lane, cnt);
            int idx = ncand + incl - cnt;
            for (uint32_t r = m; r; r &= r - 1) {
              const int k = __ffs(r) - 1;
              const int cand = textleft + J0 - k;
              gmapdp_microexon_candidate c;
              c.cL = cL;
              c.cR = cR;
              c.candidate = cand;
              c.middlelength = ml;
              if (watson) {
                c.pos2 = P.chroffset + (uint64_t)(int64_t)(cand - 1) + 1u;  // Univcoord_T arithmetic
                c.pos3 = P.chroffset + (uint64_t)(int64_t)(cand + ml);
                c.model2 = P.cdna_direction > 0 ? GMAPDP_MAXENT_ACCEPTOR : GMAPDP_MAXENT_ANTIDONOR;
                c.model3 = P.cdna_direction > 0 ? GMAPDP_MAXENT_DONOR : GMAPDP_MAXENT_ANTIACCEPTOR;
              } else {
                c.pos2 = P.chrhigh - (uint64_t)(int64_t)(cand - 1);
                c.pos3 = P.chrhigh - (uint64_t)(int64_t)(cand + ml) + 1u;
                c.model2 = P.cdna_direction > 0 ? GMAPDP_MAXENT_ANTIACCEPTOR : GMAPDP_MAXENT_DONOR;
                c.model3 = P.cdna_direction > 0 ? GMAPDP_MAXENT_ANTIDONOR : GMAPDP_MAXENT_ACCEPTOR;
              }
              if (dst >= 0) cands[dst + idx] = c;
              else if (idx < kMxCap) lc[idx] = c;
              idx++;
            }
            ncand += __builtin_amdgcn_readlane(incl, 63);
          }
        }
      }
    }
  }
  R.ncandidates = ncand;
  if (dst >= 0) {
    R.cand_offset = dst;
  } else if (ncand > kMxCap) {
    R.cand_offset = -1;  // the host reruns this call with a region of ncand records
  } else if (ncand > 0) {
    unsigned long long b = 0;
    if (lane == 0) b = atomicAdd(counter, (unsigned long long)ncand);
    b = __shfl(b, 0);
    if (b + (unsigned long long)ncand <= cand_cap) {
      for (int k = lane; k < ncand; k += 64) cands[b + k] = lc[k];
      R.cand_offset = (int64_t)b;
    } else {
      R.cand_offset = -2;  // pool too small: the host grows it and reruns the batch
    }
  }
  if (lane == 0) results[pi] = R;
}

__global__ __launch_bounds__(64) void mx_finish_kernel(const gmapdp_microexon_problem* __restrict__ probs, int n,
                                                       const uint32_t* __restrict__ blocks, uint64_t nwords,
                                                       const char* __restrict__ qseq,
                                                       const char* __restrict__ qseq_uc,
                                                       const uint8_t* __restrict__ constab,
                                                       const gmapdp_microexon_candidate* __restrict__ cands,
                                                       const double* __restrict__ cand_probs,
                                                       const double* __restrict__ metab,
                                                       gmapdp_microexon_result* __restrict__ results,
                                                       gmapdp_pair* __restrict__ pairs,
                                                       const int64_t* __restrict__ poff) {
  const int pi = blockIdx.x;
  if (pi >= n) return;
  const int lane = threadIdx.x;
  const gmapdp_microexon_problem P = probs[pi];
  gmapdp_microexon_result R = results[pi];
  if (poff) R.pair_offset = poff[pi];
  if (R.ncandidates > 0 && R.cand_offset < 0) {  // a search whose candidates are not in the pool: the host reruns it
    R.npairs = -2;
    if (lane == 0) results[pi] = R;
    return;
  }
  R.dynprogindex = P.dynprogindex;
  R.npairs = -1;
  R.bestprob2 = R.bestprob3 = 0.0;
  R.microintrontype = P.cdna_direction > 0 ? 0x20 : P.cdna_direction < 0 ? 0x04 : 0;
  // the selection (:1147): float sums, strict >, candidates in order
  int best = -1;
  float bestprob = 0.0f, b2 = 0.0f, b3 = 0.0f;
  if (P.cdna_direction != 0 && cand_probs) {
    for (int k = 0; k < R.ncandidates; k++) {
      const float p2 = (float)cand_probs[2 * (R.cand_offset + k)];
      const float p3 = (float)cand_probs[2 * (R.cand_offset + k) + 1];
      if (p2 + p3 > bestprob) {
        best = k;
        b2 = p2;
        b3 = p3;
        bestprob = p2 + p3;
      }
    }
  } else if (P.cdna_direction != 0) {
    // device MaxEnt (me_device.h): the candidates' Maxent_hr_*_prob (:1120-1144) 64 at a time, one per lane;
    // the strict > over candidates in order keeps the first maximal sum above the running best
    for (int base = 0; base < R.ncandidates; base += 64) {
      const int k = base + lane;
      float p2 = 0.0f, p3 = 0.0f, sum = -1.0f;
      if (k < R.ncandidates) {
        const gmapdp_microexon_candidate C = cands[R.cand_offset + k];
        p2 = (float)maxent_prob(blocks, nwords, metab, C.model2 & 3, C.pos2, P.chroffset);
        p3 = (float)maxent_prob(blocks, nwords, metab, C.model3 & 3, C.pos3, P.chroffset);
        sum = p2 + p3;
      }
      float mx = sum;
      for (int off = 32; off >= 1; off >>= 1) mx = fmaxf(mx, __shfl_xor(mx, off, 64));
      if (mx > bestprob) {
        const int j = __ffsll((long long)ballot(sum == mx)) - 1;
        best = base + j;
        b2 = __shfl(p2, j, 64);
        b3 = __shfl(p3, j, 64);
        bestprob = mx;
      }
    }
  }
  if (best < 0) {
    R.microintrontype = 0;  // NONINTRON
    if (lane == 0) results[pi] = R;
    return;
  }
  const gmapdp_microexon_candidate C = cands[R.cand_offset + best];
  const bool watson = P.watsonp != 0;
  const char* rs = qseq + P.qoff;
  const char* ruc = qseq_uc + P.qoff;
  const uint8_t* cons = constab + (size_t)P.genestrand * 128 * kNClass;
  const char gapchar = P.cdna_direction > 0 ? '>' : '<';
  const int lenL = C.cL, lenM = C.middlelength, lenR = C.cR;
  const int goffsetM = C.candidate, goffsetR = P.rev_goffsetR - C.cR + 1;
  const int total = lenL + 1 + lenM + 1 + lenR;  // records in push order
  // valid records (Pairpool_push drops querypos < 0 or genomepos < 0; gap holders always stay)
  auto record = [&](int t, int& r, int& g, int& jump) {  // returns 0 pair, 1 gap holder
    if (t < lenL) {
      r = t;
      g = P.goffsetL + t;
      return 0;
    }
    if (t == lenL) {
      jump = goffsetM - (P.goffsetL + lenL);
      return 1;
    }
    if (t <= lenL + lenM) {
      r = lenL + (t - lenL - 1);
      g = goffsetM + (t - lenL - 1);
      return 0;
    }
    if (t == lenL + lenM + 1) {
      jump = goffsetR - (goffsetM + lenM);
      return 1;
    }
    r = lenL + lenM + (t - lenL - lenM - 2);
    g = goffsetR + (t - lenL - lenM - 2);
    return 0;
  };
  int nvalid = 0;
  for (int base = 0; base < total; base += 64) {
    const int t = base + lane;
    int r = 0, g = 0, jump = 0, kind = 0;
    if (t < total) kind = record(t, r, g, jump);
    const bool valid = t < total && (kind == 1 || (P.roffset + r >= 0 && g >= 0));
    nvalid += __popcll(ballot(valid));
  }
  gmapdp_pair* out = pairs + R.pair_offset;
  int rank0 = 0;
  for (int base = 0; base < total; base += 64) {
    const int t = base + lane;
    int r = 0, g = 0, jump = 0, kind = 0;
    if (t < total) kind = record(t, r, g, jump);
    const bool valid = t < total && (kind == 1 || (P.roffset + r >= 0 && g >= 0));
    const uint64_t m = ballot(valid);
    if (valid) {
      const int idx = nvalid - 1 - (rank0 + lanes_below(m, lane));  // List_T order: last push first
      if (kind == 1) {
        put_pair(out, idx, -1, -1, jump, ' ', gapchar, ' ', ' ');
      } else {
        const char c1 = rs[r], c1u = ruc[r];
        const char c2 = genomic_nt(blocks, nwords, g, P.chroffset, P.chrhigh, watson);
        const char comp = c1u == c2 ? '*' : cons[(uint8_t)(c1u & 127) * kNClass + gclass(c2)] ? ':' : ' ';
        put_pair(out, idx, P.roffset + r, g, 0, c1, comp, c2, c2);
      }
    }
    rank0 += __popcll(m);
  }
  R.npairs = nvalid;
  R.dynprogindex = P.dynprogindex + (P.dynprogindex > 0 ? 1 : -1);
  R.bestprob2 = (double)b2;
  R.bestprob3 = (double)b3;
  if (lane == 0) results[pi] = R;
}

hipError_t launch_mx_search(int n, hipStream_t s, const gmapdp_microexon_problem* probs, const uint32_t* blocks,
                            uint64_t nwords, const char* qseq, const char* qseq_uc, gmapdp_microexon_result* results,
                            gmapdp_microexon_candidate* cands, unsigned long long cap, unsigned long long* counter,
                            const int64_t* direct) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(mx_search_kernel, dim3(n), dim3(64), 0, s, probs, n, blocks, nwords, qseq, qseq_uc, results,
                     cands, cap, counter, direct);
  return hipGetLastError();
}

hipError_t launch_mx_finish(int n, hipStream_t s, const gmapdp_microexon_problem* probs, const uint32_t* blocks,
                            uint64_t nwords, const char* qseq, const char* qseq_uc, const uint8_t* constab,
                            const gmapdp_microexon_candidate* cands, const double* cand_probs, const double* metab,
                            gmapdp_microexon_result* results, gmapdp_pair* pairs, const int64_t* poff) {
  if (n <= 0) return hipSuccess;
  if (!cand_probs && !metab) return hipErrorInvalidValue;
  hipLaunchKernelGGL(mx_finish_kernel, dim3(n), dim3(64), 0, s, probs, n, blocks, nwords, qseq, qseq_uc, constab,
                     cands, cand_probs, metab, results, pairs, poff);
  return hipGetLastError();
}

}  // namespace gmapdp
