// s2c_kernel.hip -- CDNA4 (gfx950) kernel for GMAP's stage-2 chaining: what
// Stage2_compute (stage2.c:6325) does with the seeding that oi_kernel / oi_map_kernel leave in HBM.
//
// Reference semantics restated (paths under the reference tree's src/; GMAP's arguments, gmap.c:1208:
// localp, skip_repetitive_p, proceed_pctcoverage 0.3, favor_right_p false, max_nalignments 10; no
// cross-species canonical scoring, no SNPs, STANDARD mode):
//   Diag_update_coverage          diag.c:216
//   the proceed test              stage2.c:6521-6531
//   Diag_compute_bounds           diag.c:597 (assign_scores :521, compute_dominance :427,
//                                 keep_center_diagonal :493, the minactive / maxactive lines)
//   align_compute_scores_lookback stage2.c:3667 with score_querypos_lookback_one / _mult (:1073 / :1470),
//                                 revise_active_lookback (:2956) and the grand lookback (:3983-4020)
//   get_cells_fwd                 stage2.c:3437, the path loop of align_compute_lookback (:4465-4515)
//   traceback_one                 stage2.c:4140
//   convert_to_nucleotides        stage2.c:5334
//   Stage2_filter_unique          stage2.c:6013 (stage2_cmp, stage2pairs_overlap_p)
// glibc's qsort is a stable merge sort on this image, so every sort here is stable.
//
// Design.  One wave per Stage2_compute call.  The wave does the data-parallel parts: coverage and
// diagonal depth (difference arrays + wave prefix scans), the minactive / maxactive lines (a segment
// list, each segment filled by all lanes), the per-hit arrays (the hits of every query position laid
// out contiguously by a prefix scan of npositions, so a link is one index), the cell selection (a
// max-reduction, a compaction of the cells within FINAL_SCORE_TOLERANCE of the best, group maxima and
// ranks by lane), the duplicate filter and convert_to_nucleotides (per path entry record counts, a
// prefix scan, every record written in place in list order).  The querypos sweep of
// align_compute_scores_lookback and the pointer chase of traceback_one are inherently sequential; they
// run on lane 0 over the problem's L2-resident link arrays.  Scratch and outputs come from batch-wide
// pools (one atomic per problem); a problem that does not fit reports kS2Overflow and the host reruns
// the batch with larger pools.
#include "dp_device.h"

namespace gmapdp {

constexpr int kS2K = 8;                 // indexsize of GMAP's major oligoindex
constexpr int kS2EqualNotSplicing = 9;  // EQUAL_DISTANCE_NOT_SPLICING
constexpr int kS2EnoughConsec = 32;     // ENOUGH_CONSECUTIVE
constexpr int kS2GreedyConsec = 100;    // GREEDY_NCONSECUTIVE
constexpr int kS2ExonDefn = 30;         // EXON_DEFN
constexpr int kS2MinTerminal = 8;       // MIN_TERMINAL_NCONSECUTIVE
constexpr int kS2MaxNactive = 100;      // MAX_NACTIVE
constexpr int kS2MaxSkipped = 3;        // MAX_SKIPPED
constexpr int kS2ScoreRestrict = 10;    // SCORE_FOR_RESTRICT
constexpr int kS2TenThousand = 8192;    // TEN_THOUSAND
constexpr int kS2FinalTolerance = 20;   // FINAL_SCORE_TOLERANCE
constexpr int kS2MaxNalignments = 10;   // gmap.c:142
constexpr int kS2Sufflookback = 60, kS2Nsufflookback = 5;  // gmap.c:269-270
constexpr int kS2ExtraBounds = 20;      // diag.c:14

// result status
constexpr int kS2NoPositions = 0, kS2Coverage = 1, kS2Chained = 2, kS2Overflow = -2, kS2Domain = -3;

struct S2Hit {  // struct Link_T (stage2.c:363) + fwd_scores + active, one per (querypos, hit)
  uint32_t map;
  int consec, root, fpos, fhit, tracei, score, active, q;
};
struct S2Diag {  // struct Diag_T (diagdef.h)
  uint32_t diagonal;
  int querystart, queryend, nconsecutive, dominatedp, pad_;
  double score;
};
struct S2Path {
  int cell;          // end cell (hit index)
  int n;             // path entries after the 3'-end pruning
  uint32_t start, end;  // genomepos of the first and last pair of the converted list
};
struct S2Scratch {
  size_t diff, run, off, minact, maxact, first, proc, diags, ord, tmp, hits, cand, keep, paths, pq, ph, sbuf, total;
  int sortn;  // power of two >= every sorted array
};
__host__ __device__ inline int s2_pow2(int n) {
  int p = 64;
  while (p < n) p <<= 1;
  return p;
}
__host__ __device__ inline S2Scratch s2_scratch(int ql, int T, int nd) {
  S2Scratch s;
  const size_t Q = (size_t)ql + 1, D = (size_t)(nd > 0 ? nd : 1), H = (size_t)(T > 0 ? T : 1);
  s.diff = 0;
  s.run = align16(s.diff + 4 * Q);
  s.off = align16(s.run + 8 * Q);
  s.minact = align16(s.off + 4 * Q);
  s.maxact = align16(s.minact + 4 * Q);
  s.first = align16(s.maxact + 4 * Q);
  s.proc = align16(s.first + 4 * Q);
  s.diags = align16(s.proc + 4 * Q);
  s.ord = align16(s.diags + sizeof(S2Diag) * D);
  s.tmp = align16(s.ord + 4 * D);
  s.hits = align16(s.tmp + 4 * D);
  s.cand = align16(s.hits + sizeof(S2Hit) * H);
  s.keep = align16(s.cand + 4 * H);
  s.paths = align16(s.keep + 4 * H);
  s.pq = align16(s.paths + sizeof(S2Path) * H);
  s.ph = align16(s.pq + 4 * Q);
  s.sortn = s2_pow2((int)(H > D ? H : D));
  s.sbuf = align16(s.ph + 4 * Q);
  s.total = align16(s.sbuf + 4 * (size_t)s.sortn);
  return s;
}

// ---- wave primitives ----
__device__ __forceinline__ int wave_incl_sum(int x, int lane) {
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const int y = __shfl_up(x, off, 64);
    if (lane >= off) x += y;
  }
  return x;
}
__device__ __forceinline__ int wave_max_i(int x) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) x = max(x, __shfl_xor(x, off, 64));
  return x;
}
__device__ __forceinline__ int wave_sum_i(int x) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) x += __shfl_xor(x, off, 64);
  return x;
}
__device__ __forceinline__ void wave_sync() { __syncthreads(); }  // one wave per block: waitcnt + barrier

// Stable sort of in[0..n) into out[0..n) by `less` (a strict weak order on the values): a bitonic
// sort of the positions 0..n-1 in sbuf (padded with -1 = +infinity to a power of two), ties broken
// by position, which is the order a stable merge sort (glibc qsort) leaves.
template <class Less>
__device__ void wave_sort(int lane, int n, const int* in, int* out, int* sbuf, Less less) {
  if (n <= 0) return;
  const int NN = s2_pow2(n);
  for (int i = lane; i < NN; i += 64) sbuf[i] = i < n ? i : -1;
  wave_sync();
  auto lt = [&](int x, int y) {  // positions; -1 sorts last
    if (x < 0) return false;
    if (y < 0) return true;
    const int vx = in[x], vy = in[y];
    if (less(vx, vy)) return true;
    if (less(vy, vx)) return false;
    return x < y;
  };
  for (int size = 2; size <= NN; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int i = lane; i < NN; i += 64) {
        const int j = i ^ stride;
        if (j > i) {
          const int a = sbuf[i], b = sbuf[j];
          const bool up = (i & size) == 0;
          if (up ? lt(b, a) : lt(a, b)) {
            sbuf[i] = b;
            sbuf[j] = a;
          }
        }
      }
      wave_sync();
    }
  }
  for (int i = lane; i < n; i += 64) out[i] = in[sbuf[i]];
  wave_sync();
}

// fill dst[a..b] (inclusive) with f(q) by all lanes
template <class F>
__device__ __forceinline__ void fill_range(int lane, uint32_t* dst, int a, int b, F f) {
  for (int q = a + lane; q <= b; q += 64) dst[q] = f(q);
}

// ---- the sequential sweep (lane 0) ----
struct S2Best {
  int consec, root, pp, ph, score, tracei;
};
struct S2Chain {
  S2Hit* h;
  const int* off;
  int* first;
  int tracectr, splicingp;
  uint32_t maxintronlen;
  __device__ __forceinline__ S2Hit& at(int q, int hit) const { return h[off[q] + hit]; }
};

__device__ void s2_finish(S2Chain& C, int q, int hit, const S2Best& b) {
  S2Hit& x = C.at(q, hit);
  x.consec = b.consec;
  x.root = b.root;
  x.fpos = b.pp;
  x.fhit = b.ph;
  if (b.pp >= 0) {
    x.tracei = b.tracei;
    x.score = b.score;
  } else {  // localp
    x.tracei = ++C.tracectr;
    x.score = kS2K;
  }
}

// ranges 0-4 against processed query position pq from active hit ph; returns the range-1 frontier
__device__ int s2_ranges(S2Chain& C, S2Best& b, int q, uint32_t position, int pq, int ph, int& last_tr,
                         bool range1) {
  const int qd = q - pq, credit = -qd / kS2K;
  const S2Hit* H = C.h + C.off[pq];
  while (ph != -1 && H[ph].tracei == last_tr) ph = H[ph].active;
  if (ph != -1) last_tr = H[ph].tracei;
  if (range1)
    while (ph != -1 && H[ph].map + C.maxintronlen + (uint32_t)qd <= position) ph = H[ph].active;
  const int frontier = ph;
  while (ph != -1) {
    const uint32_t pp = H[ph].map;
    if (!(pp + (uint32_t)kS2EqualNotSplicing + (uint32_t)qd < position)) break;
    const int diff = (int)(position - pp) - qd;
    const int fs = H[ph].score + credit - (C.splicingp ? (diff / kS2TenThousand + 1) : (diff + 1));
    if (fs > b.score) {
      b.consec = (diff <= 0) ? H[ph].consec + qd : 0;
      b.root = H[ph].root;
      b.score = fs;
      b.pp = pq;
      b.ph = ph;
      b.tracei = ++C.tracectr;
    }
    ph = H[ph].active;
  }
  while (ph != -1) {
    const uint32_t pp = H[ph].map;
    if (!(pp + (uint32_t)kS2K <= position)) break;
    const int g = (int)(position - pp);
    const int diff = g > qd ? g - qd : qd - g;
    const int fs = H[ph].score + 1;
    if (fs > b.score) {
      b.consec = (diff <= 0) ? H[ph].consec + qd : 0;
      b.root = H[ph].root;
      b.score = fs;
      b.pp = pq;
      b.ph = ph;
      b.tracei = H[ph].tracei;
    }
    ph = H[ph].active;
  }
  return frontier;
}

__device__ __forceinline__ bool s2_adjacent(const S2Chain& C, int pq, int& ph, int qd, uint32_t position) {
  const S2Hit* H = C.h + C.off[pq];
  uint32_t pp = position;
  while (ph != -1 && (pp = H[ph].map) + (uint32_t)qd < position) ph = H[ph].active;
  return pp + (uint32_t)qd == position;
}

__device__ void s2_one(S2Chain& C, int q, int hit, const int* proc, int np) {
  const uint32_t position = C.at(q, hit).map;
  S2Best b = {kS2K, (int)position, -1, -1, 0, 0};
  int nlookback = kS2Nsufflookback, lookback = kS2Sufflookback;
  if (np > 0) {
    const int pq = proc[np - 1], qd = q - pq;
    int ph = C.first[pq];
    if (s2_adjacent(C, pq, ph, qd, position)) {
      const S2Hit& x = C.at(pq, ph);
      b.consec = x.consec + qd;
      b.root = x.root;
      b.score = x.score + qd;
      b.pp = pq;
      b.ph = ph;
      b.tracei = x.tracei;
      nlookback = 1;
      lookback = kS2Sufflookback / 2;
    }
  }
  bool donep = false;
  int last_tr = -1;
  for (int k = np - 1, nseen = 0; k >= 0 && b.consec < kS2EnoughConsec && !donep; k--, nseen++) {
    const int pq = proc[k], qd = q - pq;
    if (nseen > nlookback && qd - kS2K > lookback) donep = true;
    const int ph = C.first[pq];
    if (ph != -1) s2_ranges(C, b, q, position, pq, ph, last_tr, C.splicingp);
  }
  s2_finish(C, q, hit, b);
}

__device__ void s2_mult(S2Chain& C, int q, int low, int high, const int* proc, int np, int* frontier) {
  const int nhits = high - low;
  if (np == 0) {
    for (int i = 0; i < nhits; i++) {
      S2Hit& x = C.at(q, low + i);
      x.consec = kS2K;
      x.root = (int)x.map;
      x.fpos = x.fhit = -1;
      x.tracei = ++C.tracectr;
      x.score = kS2K;
    }
    return;
  }
  const int adj = proc[np - 1], adq = q - adj;
  int maxadj = 0, maxnon = 0, overall = 0;
  for (int n = 0; n < np; n++) {
    const int qd = q - proc[np - 1 - n];
    if (n <= 1 || qd - kS2K <= kS2Sufflookback / 2) maxadj = n;
    if (n <= kS2Nsufflookback || qd - kS2K <= kS2Sufflookback) maxnon = n;
    if (n > kS2Nsufflookback && n > 1 && qd - kS2K > kS2Sufflookback) break;  // later entries only shrink
    frontier[n] = C.first[proc[np - 1 - n]];
  }
  int adjf = C.first[adj];
  for (int i = 0; i < nhits; i++) {
    const uint32_t position = C.at(q, low + i).map;
    int ph = adjf;
    if (s2_adjacent(C, adj, ph, adq, position) && C.at(adj, ph).consec + adq > overall)
      overall = C.at(adj, ph).consec + adq;
    adjf = ph;
  }
  adjf = C.first[adj];
  for (int i = 0; i < nhits; i++) {
    const uint32_t position = C.at(q, low + i).map;
    int ph = adjf;
    S2Best b;
    int maxseen;
    if (s2_adjacent(C, adj, ph, adq, position)) {
      const S2Hit& x = C.at(adj, ph);
      b.consec = x.consec + adq;
      b.root = x.root;
      b.pp = adj;
      b.ph = ph;
      b.score = x.score + adq;
      b.tracei = x.tracei;
      maxseen = maxadj;
    } else {
      b.consec = kS2K;
      b.root = (int)position;
      b.pp = b.ph = -1;
      b.score = 0;
      b.tracei = -1;
      maxseen = maxnon;
    }
    adjf = ph;
    if (overall < kS2GreedyConsec) {
      int last_tr = -1;
      for (int k = np - 1, nseen = 0; k >= 0 && b.consec < kS2EnoughConsec && nseen <= maxseen; k--, nseen++) {
        const int ph0 = frontier[nseen];
        if (ph0 != -1) frontier[nseen] = s2_ranges(C, b, q, position, proc[k], ph0, last_tr, true);
      }
    }
    s2_finish(C, q, low + i, b);
  }
}

__device__ void s2_revise_active(S2Chain& C, int q, int low, int high) {
  if (low >= high) {
    C.first[q] = -1;
    return;
  }
  S2Hit* H = C.h + C.off[q];
  int best = H[low].score;
  for (int hit = low + 1; hit < high; hit++) best = max(best, H[hit].score);
  const int threshold = max(best - kS2ScoreRestrict, 0);
  int* ptr = &C.first[q];
  int hit = low;
  *ptr = -1;
  while (hit < high) {
    while (hit < high && H[hit].score <= threshold) hit++;
    *ptr = hit;
    if (hit < high) {
      ptr = &H[hit].active;
      hit++;
    }
  }
  *ptr = -1;
}

// align_compute_scores_lookback's sweep (stage2.c:3746-4080), lane 0
__device__ void s2_sweep(S2Chain& C, const int32_t* npq, int nq, const uint32_t* minact, const uint32_t* maxact,
                         int qstart, int qend, int* proc, int* frontier) {
  auto npos = [&](int q) { return q < nq ? npq[q] : 0; };
  int q, np = 0;
  for (q = 0; q < qstart; q++) C.first[q] = -1;
  while (q <= qend && npos(q) <= 0) C.first[q++] = -1;
  if (q <= qend) {
    const int n = npos(q);
    for (int hit = 0; hit < n; hit++) {
      S2Hit& x = C.at(q, hit);
      x.fpos = x.fhit = -1;
      x.consec = kS2K;
      x.tracei = -1;
      x.score = kS2K;
    }
    s2_revise_active(C, q, 0, n);
  }
  int grand_score = 0, grand_q = -1, grand_hit = -1, nskipped = 0, min_hits = 1000000, specific_q = -1,
      specific_low = 0, specific_high = 0;
  while (q <= qend) {
    const S2Hit* H = C.h + C.off[q];
    const int nq0 = npos(q);
    int hit = 0;
    while (hit < nq0 && H[hit].map < minact[q]) hit++;
    int low = hit;
    while (hit < nq0 && H[hit].map <= maxact[q]) hit++;
    int high = hit;
    if (high - low >= kS2MaxNactive && nskipped <= kS2MaxSkipped) {
      C.first[q] = -1;
      nskipped++;
      if (high - low < min_hits) {
        min_hits = high - low;
        specific_q = q;
        specific_low = low;
        specific_high = high;
      }
      q++;
      continue;
    }
    int next_q;
    if (nskipped > kS2MaxSkipped) {
      next_q = q;
      q = specific_q;
      low = specific_low;
      high = specific_high;
    } else {
      next_q = q + 1;
    }
    if (high - low > 0) {
      int best_score = 0, best_hit = -1;
      if (high - low == 1) {
        s2_one(C, q, low, proc, np);
        if (C.at(q, low).score > 0) {
          best_score = C.at(q, low).score;
          best_hit = low;
        }
      } else {
        s2_mult(C, q, low, high, proc, np, frontier);
        for (int h = low; h < high; h++)
          if (C.at(q, h).score > best_score) {
            best_score = C.at(q, h).score;
            best_hit = h;
          }
      }
      nskipped = 0;
      min_hits = 1000000;
      specific_q = -1;
      if (C.splicingp && best_hit >= 0 && C.at(q, best_hit).fhit < 0 && grand_q >= 0 && q >= grand_q + kS2K) {
        if ((best_score = C.at(grand_q, grand_hit).score - (q - grand_q)) > 0) {
          const uint32_t prevposition = C.at(grand_q, grand_hit).map;
          for (int h = low; h < high; h++) {
            S2Hit& x = C.at(q, h);
            if (x.map > prevposition + C.maxintronlen) continue;
            if (x.map >= prevposition + (uint32_t)kS2K) {
              x.consec = kS2K;
              x.fpos = grand_q;
              x.fhit = grand_hit;
              x.tracei = ++C.tracectr;
              x.score = best_score;
            }
          }
        }
      }
      if (best_hit >= 0 && best_score >= grand_score && C.at(q, best_hit).consec > kS2ExonDefn) {
        grand_score = best_score;
        grand_q = q;
        grand_hit = best_hit;
      }
    }
    s2_revise_active(C, q, low, high);
    if (npos(q) > 0) proc[np++] = q;  // q may be the specific position gone back to
    q = next_q;
  }
}

__device__ __forceinline__ char s2_genomic_nt(const uint32_t* __restrict__ blocks, uint64_t nwords, uint32_t chrpos,
                                              uint32_t chroffset, uint32_t chrhigh, bool plusp) {
  // get_genomic_nt (stage2.c:4124): no chromosome-bound check
  const char c = decode_nt(blocks, nwords, plusp ? chroffset + chrpos : chrhigh - chrpos);
  return plusp ? c : compl_nt(c);
}

// traceback_one (stage2.c:4140): drop the 3'-end links with fewer than MIN_TERMINAL_NCONSECUTIVE
// consecutive matches, then visit the path's hits 3' end first (Pairpool_push drops chrpos >= 2^31)
template <class F>
__device__ void s2_walk(const S2Hit* hits, const int* off, int gi, F visit) {
  while (gi >= 0 && hits[gi].consec < kS2MinTerminal) {
    const int fq = hits[gi].fpos;
    gi = fq >= 0 ? off[fq] + hits[gi].fhit : -1;
  }
  while (gi >= 0) {
    if ((int)hits[gi].map >= 0) visit(gi);
    const int fq = hits[gi].fpos;
    gi = fq >= 0 ? off[fq] + hits[gi].fhit : -1;
  }
}

// convert_to_nucleotides (stage2.c:5334) for path entry e (3' end first): fill pairs between it and
// the entry before, and whether a gap holder precedes them
__device__ __forceinline__ void s2_entry(const int* pathq, const int* pathg, int e, int& fill, int& gap) {
  gap = 0;
  if (e == 0) {
    fill = kS2K - 1;
    return;
  }
  const int qpos = pathq[e], gpos = pathg[e], lq = pathq[e - 1], lg = pathg[e - 1];
  const int qj = lq - 1 - qpos, gj = lg - 1 - gpos;
  if (qj == 0 && gj == 0) {
    fill = 0;
    return;
  }
  if (qpos + kS2K - 1 >= lq || gpos + kS2K - 1 >= lg)
    fill = (lq - qpos < lg - gpos) ? lq - qpos - 1 : lg - gpos - 1;
  else
    fill = kS2K - 1;
  gap = ((gj - fill) > 0 || (qj - fill) > 0) ? 1 : 0;
}

__global__ __launch_bounds__(64) void s2c_kernel(
    const DevStage2Problem* __restrict__ probs, const uint32_t* __restrict__ blocks, uint64_t nwords,
    const char* __restrict__ qseq, const char* __restrict__ quc, const gmapdp_oligo_result* __restrict__ ores,
    const int32_t* __restrict__ npos_all, const int32_t* __restrict__ map_all, const uint32_t* __restrict__ table_all,
    const int32_t* __restrict__ diag_all, unsigned char* __restrict__ scratch, unsigned long long* __restrict__ counters,
    unsigned long long scratch_cap, gmapdp_stage2_result* __restrict__ results, gmapdp_path* __restrict__ paths_out,
    unsigned long long path_cap, gmapdp_path_pair* __restrict__ pairs_out, unsigned long long pair_cap) {
  __shared__ int sh[8];
  const int lane = threadIdx.x;
  const DevStage2Problem P = probs[blockIdx.x];
  const int ql = P.querylength, nq = ql - kS2K + 1;
  const gmapdp_oligo_result O = ores[P.index];
  const int T = O.totalpositions, nd = O.ndiagonals;
  const int32_t* npq = npos_all + P.qoff;
  const int32_t* mpq = map_all + P.qoff;
  gmapdp_stage2_result R;
  R.nresults = 0;
  R.npaths = 0;
  R.ncovered = 0;
  R.status = kS2NoPositions;
  R.diag_querystart = R.diag_queryend = 0;
  R.path_offset = 0;
  R.npairs = 0;

  // ---- scratch ----
  const S2Scratch so = s2_scratch(ql, T, nd);
  unsigned long long base = 0;
  if (lane == 0) base = atomicAdd(&counters[0], (unsigned long long)so.total);
  base = __shfl(base, 0, 64);
  if (base + so.total > scratch_cap) {
    if (lane == 0) {
      R.status = kS2Overflow;
      results[P.index] = R;
    }
    return;
  }
  unsigned char* S = scratch + base;
  int* diff = reinterpret_cast<int*>(S + so.diff);
  double* run = reinterpret_cast<double*>(S + so.run);
  int* off = reinterpret_cast<int*>(S + so.off);
  uint32_t* minact = reinterpret_cast<uint32_t*>(S + so.minact);
  uint32_t* maxact = reinterpret_cast<uint32_t*>(S + so.maxact);
  int* first = reinterpret_cast<int*>(S + so.first);
  int* proc = reinterpret_cast<int*>(S + so.proc);
  S2Diag* dg = reinterpret_cast<S2Diag*>(S + so.diags);
  int* ord = reinterpret_cast<int*>(S + so.ord);
  int* tmp = reinterpret_cast<int*>(S + so.tmp);
  S2Hit* hits = reinterpret_cast<S2Hit*>(S + so.hits);
  int* cand = reinterpret_cast<int*>(S + so.cand);
  int* keep = reinterpret_cast<int*>(S + so.keep);
  S2Path* pth = reinterpret_cast<S2Path*>(S + so.paths);
  int* pathq = reinterpret_cast<int*>(S + so.pq);
  int* pathh = reinterpret_cast<int*>(S + so.ph);
  int* sbuf = reinterpret_cast<int*>(S + so.sbuf);

  // ---- Diag_update_coverage: depth per query position from a difference array ----
  for (int q = lane; q <= ql; q += 64) diff[q] = 0;
  for (int d = lane; d < nd; d += 64) {
    const int32_t* r = diag_all + 4 * (O.diag_offset + d);
    S2Diag x;
    x.diagonal = (uint32_t)r[0];
    x.querystart = r[1];
    x.queryend = r[2];
    x.nconsecutive = r[3];
    x.dominatedp = 0;
    x.pad_ = 0;
    x.score = 0.0;
    dg[d] = x;
  }
  wave_sync();
  for (int d = lane; d < nd; d += 64) {
    atomicAdd(&diff[dg[d].querystart], 1);
    atomicAdd(&diff[dg[d].queryend], -1);
  }
  wave_sync();
  int carry = 0, ncovered = 0;
  for (int cb = 0; cb < ql; cb += 64) {
    const int q = cb + lane;
    const int v = q < ql ? diff[q] : 0;
    const int depth = carry + wave_incl_sum(v, lane);
    carry = __shfl(depth, 63, 64);
    ncovered += wave_sum_i(q < ql && depth > 0 ? 1 : 0);
    if (q < ql) run[q] = depth > 0 ? 1.0 / (double)depth : 0.0;  // assign_scores' per-position term
  }
  R.ncovered = ncovered;
  const double pct = (double)ncovered / (double)ql;
  if (T == 0) {
    R.status = kS2NoPositions;
  } else if (ql > 150 && pct < 0.3 && ncovered < 200) {
    R.status = kS2Coverage;
  } else {
    R.status = kS2Chained;
  }
  if (R.status != kS2Chained) {
    if (lane == 0) results[P.index] = R;
    return;
  }
  wave_sync();

  // ---- Diag_compute_bounds ----
  const uint32_t chrinit = P.plusp ? P.chrstart : (P.chrhigh - P.chroffset) - P.chrend;
  const uint32_t chrterm = P.plusp ? P.chrend : (P.chrhigh - P.chroffset) - P.chrstart;
  const uint32_t genomiclength = P.chrend - P.chrstart;
  int qstart, qend;
  if (nd == 0) {
    fill_range(lane, minact, 0, ql - 1, [&](int) { return chrinit; });
    fill_range(lane, maxact, 0, ql - 1, [&](int) { return chrterm; });
    qstart = 0;
    qend = ql - 1;
  } else {
    // assign_scores: running sum in query order (sequential, as the reference rounds it)
    if (lane == 0) {
      double acc = 0.0;
      for (int q = 0; q < ql; q++) {
        acc += run[q];
        run[q] = acc;
      }
    }
    wave_sync();
    for (int d = lane; d < nd; d += 64) dg[d].score = run[dg[d].queryend] - run[dg[d].querystart];
    wave_sync();
    // gooddiagonals (List_push: reverse list order), else all in list order
    int ngood = 0;
    for (int cb = 0; cb < nd; cb += 64) {
      const int d = nd - 1 - (cb + lane);
      const bool g = (cb + lane < nd) && dg[d].score >= 10.0;
      const uint64_t m = ballot(g);
      if (g) ord[ngood + lanes_below(m, lane)] = d;
      ngood += __popcll(m);
    }
    if (ngood == 0) {
      for (int d = lane; d < nd; d += 64) ord[d] = d;
      ngood = nd;
    }
    wave_sync();
    // compute_dominance: stable sort by nconsecutive descending, then drop dominated diagonals
    wave_sort(lane, ngood, ord, tmp, sbuf, [&](int a, int b) { return dg[a].nconsecutive > dg[b].nconsecutive; });
    int nunique = ngood;
    for (int i = 0; i < nunique; i++) {
      const S2Diag sup = dg[tmp[i]];
      const int expected = sup.queryend + 1 - sup.querystart;
      int threshold;
      if (expected < 100 && sup.nconsecutive > expected - 10) {
        threshold = sup.nconsecutive - 20;
      } else if (expected >= 100 && sup.nconsecutive > expected * 0.90) {
        threshold = (int)(sup.nconsecutive * 0.80);
      } else {
        continue;
      }
      int k = i + 1;
      for (int cb = i + 1; cb < nunique; cb += 64) {
        const int j = cb + lane;
        int d = -1;
        bool live = false;
        if (j < nunique) {
          d = tmp[j];
          S2Diag& sub = dg[d];
          if (sub.querystart >= sup.querystart && sub.queryend <= sup.queryend && sub.nconsecutive < threshold)
            sub.dominatedp = 1;
          live = !sub.dominatedp;
        }
        const uint64_t m = ballot(live);
        wave_sync();
        if (live) tmp[k + lanes_below(m, lane)] = d;
        k += __popcll(m);
        wave_sync();
      }
      nunique = k;
    }
    // stable sort by diagonal
    wave_sort(lane, nunique, tmp, ord, sbuf, [&](int a, int b) { return dg[a].diagonal < dg[b].diagonal; });
    if (nunique > 100) {  // keep_center_diagonal
      if (lane == 0) {
        const uint32_t mind = dg[ord[0]].diagonal, maxd = dg[ord[nunique - 1]].diagonal;
        const int nbins = (int)((maxd - mind) / 10000) + 1;
        // bins by a sweep over the sorted diagonals (bin index is monotone in the order)
        int maxcount = 0, curbin = -1, curcount = 0;
        uint32_t center = 0;
        for (int i = 0; i <= nunique; i++) {
          const int b = i < nunique ? (int)((dg[ord[i]].diagonal - mind) / 10000) : nbins;
          if (b != curbin) {
            if (curbin >= 0 && curcount > maxcount) {
              maxcount = curcount;
              center = mind + 10000u * (uint32_t)curbin;
            }
            curbin = b;
            curcount = 0;
          }
          curcount++;
        }
        center += 5000;
        int j = 0;
        for (int i = 0; i < nunique; i++) {
          const uint32_t dd = dg[ord[i]].diagonal;
          if (!(dd + 10000 < center || dd > center + 10000)) ord[j++] = ord[i];
        }
        sh[0] = j;
      }
      wave_sync();
      nunique = sh[0];
    }
    const S2Diag d0 = dg[ord[0]], dl = dg[ord[nunique - 1]];
    qstart = ql - 1;
    qend = 0;
    {
      int mn = ql - 1, mx = 0;
      for (int i = lane; i < nunique; i += 64) {
        mn = min(mn, dg[ord[i]].querystart);
        mx = max(mx, dg[ord[i]].queryend);
      }
      qstart = -wave_max_i(-mn);
      qend = wave_max_i(mx);
    }
    auto minline = [&](uint32_t diagonal) {
      return [=](int q) {
        return (diagonal + (uint32_t)q < (uint32_t)kS2ExtraBounds) ? chrinit
                                                                    : chrinit + diagonal + (uint32_t)q - kS2ExtraBounds;
      };
    };
    auto maxline = [&](uint32_t diagonal) {
      return [=](int q) {
        const uint32_t position = diagonal + (uint32_t)q + kS2ExtraBounds;
        return (position > genomiclength) ? chrterm : chrinit + position;
      };
    };
    // minactive
    fill_range(lane, minact, 0, d0.querystart - 1, [&](int) { return 0u; });
    int q = d0.querystart;
    uint32_t diagonal = d0.diagonal;
    fill_range(lane, minact, q, d0.queryend, minline(diagonal));
    q = max(q, d0.queryend + 1);
    for (int i = 0, j; i < nunique; i = j) {
      const int qe_i = dg[ord[i]].queryend;
      for (j = i + 1; j < nunique && dg[ord[j]].queryend <= qe_i; j++) ;
      if (j < nunique) {
        diagonal = dg[ord[i]].diagonal;
        const int b = dg[ord[j]].queryend;
        fill_range(lane, minact, q, b, minline(diagonal));
        q = max(q, b + 1);
      }
    }
    {
      const uint32_t dlast = diagonal;
      fill_range(lane, minact, q, ql - 1, [=](int qq) {
        return (dlast + (uint32_t)qq < (uint32_t)kS2ExtraBounds) ? chrinit : chrinit + (uint32_t)qq - kS2ExtraBounds;
      });
    }
    // maxactive
    const int activeend = dl.queryend;
    fill_range(lane, maxact, activeend + 1, ql - 1, [&](int) { return chrterm; });
    q = min(ql - 1, activeend);
    diagonal = dl.diagonal;
    fill_range(lane, maxact, dl.querystart, q, maxline(diagonal));
    q = min(q, dl.querystart - 1);
    for (int i = nunique - 1, j; i >= 0; i = j) {
      const int qs_i = dg[ord[i]].querystart;
      for (j = i - 1; j >= 0 && dg[ord[j]].querystart > qs_i; j--) ;
      if (j >= 0) {
        diagonal = dg[ord[i]].diagonal;
        const int a = dg[ord[j]].querystart;
        fill_range(lane, maxact, a, q, maxline(diagonal));
        q = min(q, a - 1);
      }
    }
    fill_range(lane, maxact, 0, q, maxline(diagonal));
  }
  R.diag_querystart = qstart;
  R.diag_queryend = qend;

  // ---- per-hit arrays: the hits of query position q at hits[off[q] ...] (Linkmatrix_1d_new) ----
  carry = 0;
  for (int cb = 0; cb < ql; cb += 64) {
    const int q = cb + lane;
    const int v = q < nq ? npq[q] : 0;
    const int incl = carry + wave_incl_sum(v, lane);
    if (q < ql) off[q] = incl - v;
    carry = __shfl(incl, 63, 64);
  }
  if (lane == 0) off[ql] = carry;
  bool big = false;
  for (int q = lane; q < nq; q += 64) {
    const int n = npq[q];
    if (n <= 0) continue;
    const uint32_t* src = table_all + mpq[q];
    S2Hit* dst = hits + off[q];
    for (int k = 0; k < n; k++) {
      S2Hit x;
      x.map = src[k];
      big |= (x.map >= 0x80000000u);
      x.consec = x.root = x.fpos = x.fhit = x.tracei = x.score = x.active = 0;  // CALLOC
      x.q = q;
      dst[k] = x;
    }
  }
  if (ballot(big)) {  // chromosome positions past 2^31: Pairpool_push would drop them (outside the domain)
    if (lane == 0) {
      R.status = kS2Domain;
      results[P.index] = R;
    }
    return;
  }
  wave_sync();

  // ---- align_compute_scores_lookback: the sweep on lane 0 ----
  if (lane == 0) {
    S2Chain C;
    C.h = hits;
    C.off = off;
    C.first = first;
    C.tracectr = 0;
    C.splicingp = P.splicingp;
    C.maxintronlen = P.maxintronlen;
    s2_sweep(C, npq, nq, minact, maxact, qstart, qend, proc, pathh /* frontier (<= 70 entries used) */);
  }
  wave_sync();

  // ---- get_cells_fwd + the path loop: cells within FINAL_SCORE_TOLERANCE of the best, each the best
  // of its root position, in (score desc, root asc, querypos desc, hit asc) order ----
  const int h0 = off[qstart], h1 = off[qend + 1];
  int best = 0;
  for (int gi = h0 + lane; gi < h1; gi += 64) best = max(best, hits[gi].score);
  best = wave_max_i(best);
  int ncand = 0;
  if (best > 0) {
    for (int cb = h0; cb < h1; cb += 64) {
      const int gi = cb + lane;
      const bool c = gi < h1 && hits[gi].score > best - kS2FinalTolerance && hits[gi].score > 0;
      const uint64_t m = ballot(c);
      if (c) cand[ncand + lanes_below(m, lane)] = gi;
      ncand += __popcll(m);
    }
  }
  wave_sync();
  // get_cells_fwd: by (root asc, score desc, querypos desc, hit asc); each root's best cells are the
  // first of its group and those with the same score
  wave_sort(lane, ncand, cand, keep, sbuf, [&](int a, int b) {
    const S2Hit &x = hits[a], &y = hits[b];
    if (x.root != y.root) return x.root < y.root;
    if (x.score != y.score) return x.score > y.score;
    if (x.q != y.q) return x.q > y.q;
    return a < b;
  });
  int nkeep = 0, gcarry = 0;
  for (int cb = 0; cb < ncand; cb += 64) {
    const int i = cb + lane;
    int gi = -1, gstart = 0;
    if (i < ncand) {
      gi = keep[i];
      gstart = (i == 0 || hits[keep[i - 1]].root != hits[gi].root) ? i : 0;
    }
    int m = gstart;  // the group's first element: running maximum of the group starts
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int y = __shfl_up(m, o, 64);
      if (lane >= o) m = max(m, y);
    }
    m = max(m, gcarry);
    gcarry = __shfl(m, 63, 64);
    const bool k = i < ncand && hits[gi].score == hits[keep[m]].score;
    const uint64_t bm = ballot(k);
    if (k) cand[nkeep + lanes_below(bm, lane)] = gi;
    nkeep += __popcll(bm);
  }
  wave_sync();
  // Cell_score_cmp, stable over that order: (score desc, root asc, querypos desc, hit asc)
  wave_sort(lane, nkeep, cand, keep, sbuf, [&](int a, int b) {
    const S2Hit &x = hits[a], &y = hits[b];
    if (x.score != y.score) return x.score > y.score;
    if (x.root != y.root) return x.root < y.root;
    if (x.q != y.q) return x.q > y.q;
    return a < b;
  });
  for (int i = lane; i < nkeep; i += 64) cand[i] = keep[i];
  wave_sync();
  int npaths = 0;
  while (npaths < nkeep && (npaths < kS2MaxNalignments || hits[cand[npaths]].score == best)) npaths++;
  R.npaths = npaths;

  // ---- traceback_one per selected cell: length and extent of the converted list ----
  if (lane == 0) {
    for (int p = 0; p < npaths; p++) {
      int n = 0, top = -1, bottom = -1;
      s2_walk(hits, off, cand[p], [&](int gi) {
        if (n == 0) top = gi;
        bottom = gi;
        n++;
      });
      S2Path r;
      r.cell = cand[p];
      r.n = n;
      r.start = n ? hits[bottom].map : 0u;
      r.end = n ? hits[top].map + (uint32_t)(kS2K - 1) : 0u;
      pth[p] = r;
    }
  }
  wave_sync();

  // ---- Stage2_filter_unique: stable sort by (start, end), drop each path overlapping an earlier one ----
  int* pord = cand;  // the selected cells live on in pth[].cell
  for (int i = lane; i < npaths; i += 64) keep[i] = i;
  wave_sync();
  wave_sort(lane, npaths, keep, pord, sbuf, [&](int a, int b) {
    if (pth[a].start != pth[b].start) return pth[a].start < pth[b].start;
    return pth[a].end < pth[b].end;
  });
  for (int i = lane; i < npaths; i += 64) keep[i] = 0;  // eliminate flags, sorted order
  wave_sync();
  for (int i = 0; i < npaths; i++) {
    const S2Path x = pth[pord[i]];
    for (int j = i + 1 + lane; j < npaths; j += 64) {
      const S2Path y = pth[pord[j]];
      bool ov;
      if (y.start > x.end || x.start > y.end) {
        ov = false;
      } else if ((y.start < x.start && y.end >= x.end) || (y.start >= x.start && y.end < x.end)) {
        ov = true;  // subsumption
      } else {
        const uint32_t overlap = (y.start < x.start) ? y.end - x.start : x.end - y.start;
        const double fraction = (y.end - y.start < x.end - x.start) ? (double)overlap / (double)(y.end - y.start)
                                                                    : (double)overlap / (double)(x.end - x.start);
        ov = fraction > 0.5;
      }
      if (ov) keep[j] = 1;
    }
    wave_sync();
  }
  int nres = 0;
  for (int i = 0; i < npaths; i++) nres += keep[i] ? 0 : 1;
  R.nresults = nres;

  // ---- outputs: the kept results' path records and their pairs (convert_to_nucleotides) ----
  unsigned long long pbase = 0;
  if (lane == 0 && nres > 0) pbase = atomicAdd(&counters[1], (unsigned long long)nres);
  pbase = __shfl(pbase, 0, 64);
  if (nres > 0 && pbase + nres > path_cap) {
    if (lane == 0) {
      R.status = kS2Overflow;
      results[P.index] = R;
    }
    return;
  }
  R.path_offset = (int32_t)pbase;
  const bool plusp = P.plusp != 0;
  const char* qs = qseq + P.qoff;
  const char* qu = quc + P.qoff;
  int r = 0, allpairs = 0;
  for (int i = 0; i < npaths; i++) {
    if (keep[i]) continue;
    const S2Path x = pth[pord[i]];
    const int n = x.n;
    if (lane == 0) {  // entries, 3' end first
      int e = 0;
      s2_walk(hits, off, x.cell, [&](int gi) {
        pathq[e] = hits[gi].q;
        pathh[e] = (int)hits[gi].map;
        e++;
      });
    }
    wave_sync();
    // records per entry in generation (prepend) order: [gap holder], fills, the observed pair
    int total = 0;
    for (int cb = 0; cb < n; cb += 64) {
      const int e = cb + lane;
      int cnt = 0;
      if (e < n) {
        int fill, gap;
        s2_entry(pathq, pathh, e, fill, gap);
        cnt = gap + fill + 1;
      }
      total += wave_sum_i(cnt);
    }
    unsigned long long qb = 0;
    if (lane == 0) qb = atomicAdd(&counters[2], (unsigned long long)total);
    qb = __shfl(qb, 0, 64);
    if (qb + total > pair_cap) {
      if (lane == 0) {
        R.status = kS2Overflow;
        results[P.index] = R;
      }
      return;
    }
    gmapdp_path_pair* dst = pairs_out + qb;
    int gen = 0;
    for (int cb = 0; cb < n; cb += 64) {
      const int e = cb + lane;
      int cnt = 0, fill = 0, gap = 0;
      if (e < n) {
        s2_entry(pathq, pathh, e, fill, gap);
        cnt = gap + fill + 1;
      }
      const int incl = wave_incl_sum(cnt, lane);
      if (e < n) {
        int g = gen + incl - cnt;  // generation index of the entry's first record
        const int qpos = pathq[e], gpos = pathh[e];
        if (gap) {
          const int lq = pathq[e - 1], lg = pathh[e - 1];
          gmapdp_path_pair rr;
          rr.querypos = rr.genomepos = -1;
          rr.queryjump = (lq - 1 - qpos) - fill;
          rr.genomejump = (lg - 1 - gpos) - fill;
          rr.cdna = rr.comp = rr.genome = rr.genomealt = ' ';
          dst[total - 1 - g++] = rr;
        }
        for (int k = 0; k < fill; k++) {
          const int lq = qpos + fill - k, lg = gpos + fill - k;
          const char c = s2_genomic_nt(blocks, nwords, (uint32_t)lg, P.chroffset, P.chrhigh, plusp);
          gmapdp_path_pair rr;
          rr.querypos = lq;
          rr.genomepos = lg;
          rr.queryjump = rr.genomejump = 0;
          rr.cdna = qs[lq];
          rr.comp = '|';
          rr.genome = rr.genomealt = c;
          dst[total - 1 - g++] = rr;
        }
        gmapdp_path_pair rr;
        rr.querypos = qpos;
        rr.genomepos = gpos;
        rr.queryjump = rr.genomejump = 0;
        rr.cdna = qs[qpos];
        rr.comp = '|';
        rr.genome = rr.genomealt = qu[qpos];
        dst[total - 1 - g] = rr;
      }
      gen += __shfl(incl, 63, 64);
    }
    if (lane == 0) {
      gmapdp_path pr;
      pr.pair_offset = (int64_t)qb;
      pr.npairs = total;
      pr.pad_ = 0;
      paths_out[pbase + r] = pr;
    }
    r++;
    allpairs += total;
    wave_sync();
  }
  R.npairs = allpairs;
  if (lane == 0) results[P.index] = R;
}

size_t scratch_bytes_s2c(int querylength, int totalpositions, int ndiagonals) {
  return s2_scratch(querylength, totalpositions, ndiagonals).total;
}

hipError_t launch_s2c(int nproblems, hipStream_t stream, const DevStage2Problem* probs, const uint32_t* blocks,
                      uint64_t nwords, const char* qseq, const char* quc, const gmapdp_oligo_result* ores,
                      const int32_t* npos, const int32_t* map, const uint32_t* table, const int32_t* diags,
                      unsigned char* scratch, unsigned long long* counters, unsigned long long scratch_cap,
                      gmapdp_stage2_result* results, gmapdp_path* paths, unsigned long long path_cap,
                      gmapdp_path_pair* pairs, unsigned long long pair_cap) {
  void* args[] = {(void*)&probs, (void*)&blocks, (void*)&nwords, (void*)&qseq, (void*)&quc, (void*)&ores,
                  (void*)&npos, (void*)&map, (void*)&table, (void*)&diags, (void*)&scratch, (void*)&counters,
                  (void*)&scratch_cap, (void*)&results, (void*)&paths, (void*)&path_cap, (void*)&pairs,
                  (void*)&pair_cap};
  return hipLaunchKernel(reinterpret_cast<void*>(&s2c_kernel), dim3(nproblems), dim3(64), args, 0, stream);
}

}  // namespace gmapdp
