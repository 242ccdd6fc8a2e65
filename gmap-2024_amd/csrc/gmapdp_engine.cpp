// gmapdp_engine.cpp -- host side of libgmapdp: score tables, genome packing,
// batch planning and the C ABI of include/gmapdp.h.
//
// Reference interfaces mirrored (paths under the reference tree's src/):
//   Dynprog_init / permute_cases  dynprog.c:903-1197  (score + consistency tables)
//   Dynprog_compute_bands         dynprog.c:1247
//   Dynprog_single_gap prologue   dynprog_single.c:459-521 (penalties, size guard, segment)
//   Dynprog_end5/3_gap prologues  dynprog_end.c:1333-1411 / 1962-2027 (penalties, chopping,
//                                 NULL cases, segment orientation, bands per endalign)
//   Compress_create_blocks_comp   compress-write.c:754  (.genomecomp packing)
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <time.h>
#include <unistd.h>

#include <algorithm>
#include <climits>
#include <cctype>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <condition_variable>
#include <mutex>
#include <thread>
#include <atomic>
#include <sys/mman.h>
#include <string>
#include <tuple>
#include <utility>
#include <vector>

#include "gmapdp_internal.h"
#include "me_device.h"
#include "../../include/gmapdp.h"

namespace gmapdp {
size_t lds_bytes_dp(int rlength, int glength, int R, bool dirs_lds);
hipError_t launch_dp(int R, bool dirs_lds, bool rows, int nblocks, size_t lds, hipStream_t stream,
                     const DevProblem* probs, const int* order, const uint32_t* blocks, uint64_t nwords,
                     const char* qseq, const char* qseq_uc, const int8_t* sctab, const uint8_t* constab,
                     gmapdp_result* results, gmapdp_pair* pairs, uint64_t* gdirs);
size_t lds_slot_dpx(int rlength, int glength);
size_t lds_dirs_dpx(int gmax);
size_t lds_slot_sx(int rlength, int glength, int B);
int steps_sx(int rlength, int lband, int uband, int B);
hipError_t launch_sx(int B, int nproblems, int slot, long long wave_dirs_bytes, unsigned char* gdirs,
                     hipStream_t stream, const DevProblem* probs, const int* order, const uint32_t* blocks,
                     uint64_t nwords, const char* qseq, const char* qseq_uc, const int8_t* sctab,
                     const uint8_t* constab, gmapdp_result* results, gmapdp_pair* pairs);
hipError_t launch_dpx(int S, int nproblems, int slot, int dirs_bytes, unsigned char* gdirs, hipStream_t stream,
                      const DevProblem* probs, const int* order, const uint32_t* blocks, uint64_t nwords,
                      const char* qseq, const char* qseq_uc, const int8_t* sctab, const uint8_t* constab,
                      gmapdp_result* results, gmapdp_pair* pairs);
size_t lds_bytes_gg(int rlength, int glengthL, int glengthR, int R, bool dirs_lds, int W);
size_t scratch_bytes_gg(int rlength, int glengthL, int glengthR, int R, bool dirs_lds, int W);
hipError_t launch_gg(int R, bool dirs_lds, int nblocks, size_t lds, hipStream_t stream, const DevGenomeProblem* probs,
                     const int* order, const uint32_t* blocks, uint64_t nwords, const char* qseq,
                     const char* qseq_uc, const double* sprob, const int8_t* sctab, const uint8_t* constab,
                     const int8_t* isctab, gmapdp_genome_result* results, gmapdp_pair* pairs,
                     unsigned char* gscratch, const uint8_t* known, const double* metab);
size_t lds_bytes_sj(int rlength, int glength, int R, bool dirs_lds);
hipError_t launch_usj(int B, int nblocks, size_t lds, hipStream_t stream, const DevSjProblem* probs, const int* order,
                      unsigned char* gscratch, const char* qseq, const char* qseq_uc, const char* jseq,
                      const int8_t* sctab, const uint8_t* constab, gmapdp_sj_result* results, gmapdp_pair* pairs);
hipError_t launch_sj(int R, bool dirs_lds, int nblocks, size_t lds, hipStream_t stream, const DevSjProblem* probs,
                     const int* order, const char* qseq, const char* qseq_uc, const char* jseq, const int8_t* sctab,
                     const uint8_t* constab, gmapdp_sj_result* results, gmapdp_pair* pairs, uint64_t* gdirs);
size_t lds_bytes_uxe(int rlength, int glength, int B);
size_t scratch_bytes_uxe(int rlength, int glength, int lband, int uband, int B);
size_t lds_bytes_uxg(int rlength, int glengthL, int glengthR, int B);
size_t scratch_bytes_uxg(int rlength, int glengthL, int glengthR, int extraband, int B);
hipError_t launch_uxe(int B, int nproblems, size_t lds, hipStream_t stream, const DevProblem* probs, const int* order,
                      unsigned char* gscratch, const uint32_t* blocks, uint64_t nwords, const char* qseq,
                      const char* qseq_uc, const int8_t* sctab, const uint8_t* constab, gmapdp_result* results,
                      gmapdp_pair* pairs);
hipError_t launch_uxg(int B, int nproblems, size_t lds, hipStream_t stream, const DevGenomeProblem* probs,
                      const int* order, unsigned char* gscratch, const uint32_t* blocks, uint64_t nwords,
                      const char* qseq, const char* qseq_uc, const double* sprob, const int8_t* sctab,
                      const uint8_t* constab, const int8_t* isctab, gmapdp_genome_result* results,
                      gmapdp_pair* pairs, const uint8_t* known);
size_t lds_bytes_cg(int rlength, int glength, bool simd, int RB);
size_t scratch_bytes_cg(int rlength, int glength, int lband, int uband, bool simd, int RB);
hipError_t launch_cg(bool simd, int RB, int nproblems, size_t lds, hipStream_t stream, const DevCdnaProblem* probs,
                     const int* order, unsigned char* gscratch, const uint32_t* blocks, uint64_t nwords,
                     const char* qseq, const char* qseq_uc, const int8_t* sctab, const uint8_t* constab,
                     gmapdp_cdna_result* results, gmapdp_pair* pairs);
size_t lds_bytes_oi(int umax, bool wide);
size_t scratch_bytes_oi(int querylength, uint32_t genomiclength);
size_t scratch_bytes_oi_fallback(int querylength, uint32_t genomiclength);
size_t scratch_bytes_s2c(int querylength, int totalpositions, int ndiagonals);
// the chaining kernels' counters (paths, pairs, ...) followed by their launch order (one int per call)
// (then, per launch position, s2a's sweep-work estimate that re-orders the sweep)
inline size_t s2_counters_bytes(int n) {
  return 4 * sizeof(unsigned long long) + 2 * sizeof(int) * (size_t)(n > 0 ? n : 1);
}
hipError_t launch_s2c(int nproblems, hipStream_t stream, const DevStage2Problem* probs, const uint32_t* blocks,
                      uint64_t nwords, const char* qseq, const char* quc, const gmapdp_oligo_result* ores,
                      const int32_t* npos, const int32_t* map, const uint32_t* table, const int32_t* diags,
                      unsigned char* scratch, unsigned long long* counters, unsigned long long scratch_cap,
                      gmapdp_stage2_result* results, gmapdp_path* paths, unsigned long long path_cap,
                      gmapdp_path_pair* pairs, unsigned long long pair_cap, int phases = 7);
hipError_t launch_oi(bool wide, int nproblems, size_t lds, hipStream_t stream, const DevOligoProblem* probs,
                     const uint32_t* blocks, const char* quc, unsigned char* scratch, gmapdp_oligo_result* results,
                     int32_t* npos, int32_t* map, uint32_t* table, int32_t* diags, uint64_t* pool,
                     unsigned long long* pool_counter, unsigned long long pool_cap, int32_t* nhits_out);
size_t scratch_bytes_oi_hits(int querylength, size_t hitcap);
hipError_t launch_pc(const unsigned char* r0, int n0, int s0, const unsigned char* r1, int n1, int s1,
                     const gmapdp_pair* pairs, unsigned long long* offsets, unsigned char* out, hipStream_t stream);
hipError_t launch_pc_paths(const gmapdp_path* paths, const unsigned long long* npaths, int path_cap,
                           const gmapdp_path_pair* pairs, unsigned long long pair_cap, unsigned long long* offsets,
                           unsigned char* out, hipStream_t stream);
hipError_t launch_oi_split(int nproblems, int umax, hipStream_t stream, const DevOligoProblem* probs,
                           const uint32_t* blocks, const char* quc, unsigned char* scratch,
                           gmapdp_oligo_result* results, int32_t* npos, int32_t* map, uint32_t* table, int32_t* diags,
                           uint64_t* pool, unsigned long long* pool_counter, unsigned long long pool_cap);
hipError_t launch_mx_search(int n, hipStream_t s, const gmapdp_microexon_problem* probs, const uint32_t* blocks,
                            uint64_t nwords, const char* qseq, const char* qseq_uc, gmapdp_microexon_result* results,
                            gmapdp_microexon_candidate* cands, unsigned long long cap, unsigned long long* counter,
                            const int64_t* direct);
hipError_t launch_mx_finish(int n, hipStream_t s, const gmapdp_microexon_problem* probs, const uint32_t* blocks,
                            uint64_t nwords, const char* qseq, const char* qseq_uc, const uint8_t* constab,
                            const gmapdp_microexon_candidate* cands, const double* cand_probs, const double* metab,
                            gmapdp_microexon_result* results, gmapdp_pair* pairs, const int64_t* poff);
hipError_t launch_me_sites(long long n, hipStream_t s, const uint32_t* blocks, uint64_t nwords, const double* T,
                           const gmapdp_coord_t* pos, const uint8_t* models, const gmapdp_coord_t* chroffsets,
                           double* out);
hipError_t launch_me_gap(int n, hipStream_t s, const DevGenomeProblem* probs, const int* order,
                         const uint32_t* blocks, uint64_t nwords, const double* T, double* sprob);
static const int kUse8pSize[4] = {41, 63, 127, 24};  // use8p_size (dynprog.c:1022-1025)

// ---------------------------------------------------------------------------
// Score tables.  The reference builds pairdistance_array[4][128][128] and
// consistent_array[3][128][128]; the engine only ever scores a query byte
// against one of 6 genome classes (A C G T N *), so it keeps the
// [type][query byte][class] slice: 4 KB of scores + 3 KB of consistency.
// ---------------------------------------------------------------------------
enum { kHighQ = 0, kMedQ = 1, kLowQ = 2, kEndQ = 3 };
static const int kMismatchScore[4] = {-3, -2, -1, -5};  // MISMATCH_HIGHQ/MEDQ/LOWQ (dynprog.h), _ENDQ (dynprog.c:104)

struct Tables {
  short pd[4][128][128];
  unsigned char cons[3][128][128];
  int8_t sc[4][128][kNClass];
  uint8_t cs[3][128][kNClass];
  int8_t isc[3][2][64];  // intron_score_array_{sense,antisense,either}_{prelim,final}, [leftdi & rightdi]
};

// intron_score_setup (dynprog_genome.c:144-187) with the intron.h type codes.  The "either"
// arrays keep the reference's mix of FINAL and regular rewards.
static void build_intron_scores(Tables& T) {
  enum { GTAG_FWD = 0x20, GCAG_FWD = 0x10, ATAC_FWD = 0x08, GTAG_REV = 0x04, GCAG_REV = 0x02, ATAC_REV = 0x01 };
  const int canon = 14, final_canon = 16, gcag = 8, atac = 4, final_gcag = 10, final_atac = 8;
  std::memset(T.isc, 0, sizeof(T.isc));
  T.isc[0][1][GTAG_FWD] = final_canon; T.isc[0][1][GCAG_FWD] = final_gcag; T.isc[0][1][ATAC_FWD] = final_atac;
  T.isc[0][0][GTAG_FWD] = canon;       T.isc[0][0][GCAG_FWD] = gcag;       T.isc[0][0][ATAC_FWD] = atac;
  T.isc[1][1][GTAG_REV] = final_canon; T.isc[1][1][GCAG_REV] = final_gcag; T.isc[1][1][ATAC_REV] = final_atac;
  T.isc[1][0][GTAG_REV] = canon;       T.isc[1][0][GCAG_REV] = gcag;       T.isc[1][0][ATAC_REV] = atac;
  T.isc[2][1][GTAG_FWD] = final_canon; T.isc[2][1][GCAG_FWD] = final_gcag; T.isc[2][1][ATAC_FWD] = final_atac;
  T.isc[2][1][GTAG_REV] = canon;       T.isc[2][1][GCAG_REV] = final_gcag; T.isc[2][1][ATAC_REV] = final_atac;
  T.isc[2][0][GTAG_FWD] = final_canon; T.isc[2][0][GCAG_FWD] = gcag;       T.isc[2][0][ATAC_FWD] = atac;
  T.isc[2][0][GTAG_REV] = canon;       T.isc[2][0][GCAG_REV] = gcag;       T.isc[2][0][ATAC_REV] = atac;
}

static bool stranded(int mode) { return mode == 0 || mode == 1 || mode == 3 || mode == 5; }

static void build_tables(Tables& T, int mode) {
  std::memset(&T, 0, sizeof(T));
  // Mismatch everywhere in 'A'..'z' x 'A'..'y' (the reference's second loop bound is exclusive).
  for (int a = 'A'; a <= 'z'; a++)
    for (int b = 'A'; b < 'z'; b++)
      for (int t = 0; t < 4; t++) T.pd[t][a][b] = (short)kMismatchScore[t];
  auto mark = [&](int a, int b) {
    if (stranded(mode)) {
      T.cons[0][a][b] = 1;
    } else {
      T.cons[1][a][b] = 1;
      T.cons[2][a][b] = 1;
    }
  };
  // Symmetric assignment over upper/lower case variants (permute_cases).
  auto both = [&](int A, int B, short s) {
    const int a = std::tolower(A), b = std::tolower(B);
    const int v[4][2] = {{a, b}, {a, B}, {A, b}, {A, B}};
    for (auto& p : v) { mark(p[0], p[1]); mark(p[1], p[0]); }
    for (int t = 0; t < 4; t++)
      for (auto& p : v) { T.pd[t][p[0]][p[1]] = s; T.pd[t][p[1]][p[0]] = s; }
  };
  // One-directional assignment for the bisulfite / A-to-I modes (permute_cases_oneway).
  auto oneway = [&](int A, int B, short s, int strand) {
    const int a = std::tolower(A), b = std::tolower(B);
    const int v[4][2] = {{a, b}, {a, B}, {A, b}, {A, B}};
    for (auto& p : v) T.cons[strand][p[0]][p[1]] = 1;
    for (int t = 0; t < 4; t++)
      for (auto& p : v) T.pd[t][p[0]][p[1]] = s;
  };
  for (int ch = 'A'; ch < 'Z'; ch++) both(ch, ch, 3);  // FULLMATCH
  both('U', 'T', 3);
  const char* half[] = {"RA", "RG", "YT", "YC", "WA", "WT", "SG", "SC", "MA", "MC", "KG", "KT"};
  for (auto h : half) both(h[0], h[1], 1);  // HALFMATCH
  const char* amb[] = {"HA", "HT", "HC", "BG", "BC", "BT", "VG", "VA", "VC", "DG", "DA", "DT",
                       "NT", "NC", "NA", "NG", "XT", "XC", "XA", "XG", "NN", "XX"};
  for (auto h : amb) both(h[0], h[1], 3);  // AMBIGUOUS
  switch (mode) {
    case 1: oneway('T', 'C', 3, 0); break;
    case 2: oneway('T', 'C', 3, 1); oneway('A', 'G', 3, 2); break;
    case 3: oneway('G', 'A', 3, 0); break;
    case 4: oneway('G', 'A', 3, 1); oneway('C', 'T', 3, 2); break;
    case 5: oneway('C', 'T', 3, 0); break;
    case 6: oneway('C', 'T', 3, 1); oneway('G', 'A', 3, 2); break;
    default: break;
  }
  const char cls[kNClass] = {'A', 'C', 'G', 'T', 'N', '*', 0, 0};
  for (int t = 0; t < 4; t++)
    for (int a = 0; a < 128; a++)
      for (int g = 0; g < kNClass; g++) T.sc[t][a][g] = (int8_t)(cls[g] ? T.pd[t][a][(int)cls[g]] : 0);
  for (int s = 0; s < 3; s++)
    for (int a = 0; a < 128; a++)
      for (int g = 0; g < kNClass; g++) T.cs[s][a][g] = cls[g] ? T.cons[s][a][(int)cls[g]] : 0;
  build_intron_scores(T);
}

// ---------------------------------------------------------------------------
// Device buffer that only grows.
// ---------------------------------------------------------------------------
struct DevBuf {
  void* p = nullptr;
  size_t cap = 0;
  // tight: 1/8 headroom instead of doubling (the stage-2 plans' sizing arenas, tens of GB, about the same
  // size for every block of a run)
  hipError_t ensure(size_t bytes, bool tight = false) {
    if (bytes <= cap) return hipSuccess;
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    // doubling: a hipFree waits for the whole device (every stream of every context), so a buffer
    // should grow a handful of times per process, not per batch
    size_t want = std::max(bytes, (size_t)4096);
    want = tight ? want + want / 8 : want + want;
    hipError_t e = hipMalloc(&p, want);
    if (e == hipSuccess) cap = want;
    return e;
  }
  ~DevBuf() {
    if (p) (void)hipFree(p);
  }
};

// Pinned host staging (hipHostMalloc): the synchronous batch entry points gather every input into
// one of these and move it with one asynchronous copy each way.
struct HostBuf {
  void* p = nullptr;
  size_t cap = 0;
  hipError_t ensure(size_t bytes) {
    if (bytes <= cap) return hipSuccess;
    if (p) (void)hipHostFree(p);
    p = nullptr;
    cap = 0;
    size_t want = std::max(bytes, (size_t)65536);
    want = want + want;
    hipError_t e = hipHostMalloc(&p, want, hipHostMallocDefault);
    if (e == hipSuccess) cap = want;
    return e;
  }
  ~HostBuf() {
    if (p) (void)hipHostFree(p);
  }
};

}  // namespace gmapdp

using namespace gmapdp;

struct gmapdp_ctx {
  int device = 0;
  int mode = 0;
  int user_open = 0, user_extend = 0, user_dynprog_p = 0;
  hipStream_t stream = nullptr;
  // Side streams for the long-problem launch classes: a class of a few
  // thousand long fills runs as a latency-bound tail, so it overlaps the
  // bulk classes instead of following them (the launch order within a class
  // is longest-first already).
  static constexpr int kAux = 3;
  hipStream_t aux[kAux] = {nullptr, nullptr, nullptr};
  hipEvent_t ev_fork = nullptr;
  hipEvent_t ev_join[kAux] = {nullptr, nullptr, nullptr};
  Tables* tables = nullptr;
  int8_t* d_sc = nullptr;
  uint8_t* d_cs = nullptr;
  int8_t* d_isc = nullptr;
  uint32_t* d_genome = nullptr;
  uint64_t genome_words = 0;
  uint64_t genome_length = 0;
  bool genome_owned = true;  // false: another context's HBM genome (gmapdp_share_genome)
  bool one_stream = false;   // GMAPDP_CTX_ONE_STREAM: no side streams (callers that run many contexts)
  int plan_sides = kAux;     // side streams a plan's LPT spreads over (GMAPDP_CTX_TWO_SIDES: 2)
  hipEvent_t ev_block = nullptr;  // GMAPDP_CTX_BLOCKING_SYNC / _POLL_SYNC: batch completion waited on without spinning
  bool poll = false;              // GMAPDP_CTX_POLL_SYNC: ev_block is polled with sleeps in between
  DevBuf probs, order, qseq, qseq_uc, results, pairs, gdirs;
  DevBuf din, dout;    // run_batch: all inputs / all outputs of one synchronous batch
  HostBuf hin, hout;   // their pinned host images
  HostBuf hplan;       // a plan's descriptor upload (gmapdp_plan_create_all), staged pinned
  hipEvent_t ev_hplan = nullptr;  // the last upload from hplan (its copies may still be in flight)
  DevBuf gprobs, gorder, sprob, gresults;
  DevBuf cprobs, corder, cresults, cscratch;  // Dynprog_cdna_gap batches
  DevBuf sjprobs, sjorder, sjresults, sjseq, sjdirs;  // Dynprog_end5/3_splicejunction batches
  DevBuf oprobs, oresults, oscratch, onpos, omap, otable, odiag, opool, opoolctr;  // stage-2 seeding batches
  DevBuf onhits;  // stage-2 plans' sizing runs (with otable, odiag and the seeding scratch above)
  DevBuf s2probs, s2results, s2scratch, s2counters, s2paths, s2pairs, s2qseq;  // Stage2_compute batches
  DevBuf mxprobs, mxres, mxcands, mxcnt, mxdirect, mxprobs2, mxpairs;  // Dynprog_microexon_int batches
  std::string err;
};

// Wait for `s`: spinning (hipStreamSynchronize) by default; with GMAPDP_CTX_BLOCKING_SYNC the thread
// sleeps on a blocking-sync event instead, so that callers running many dispatcher threads next to
// their own compute threads (the GMAP drop-in) do not burn a core per waiting dispatcher.
// With GMAPDP_CTX_POLL_SYNC it polls an event every GMAPDP_POLL_US microseconds (default 10) and
// sleeps in between: the waiting thread gives its core to the caller's threads but still sees the
// batch end within a poll period (a blocking-sync wake-up measured slower).
static long poll_ns() {
  static const long v = (getenv("GMAPDP_POLL_US") ? atol(getenv("GMAPDP_POLL_US")) : 10L) * 1000L;
  return v;
}
static hipError_t ctx_sync(gmapdp_ctx* ctx, hipStream_t s) {
  if (!ctx->ev_block) return hipStreamSynchronize(s);
  hipError_t e = hipEventRecord(ctx->ev_block, s);
  if (e != hipSuccess || !ctx->poll) return e == hipSuccess ? hipEventSynchronize(ctx->ev_block) : e;
  const struct timespec ts = {0, poll_ns()};
  for (;;) {
    e = hipEventQuery(ctx->ev_block);
    if (e != hipErrorNotReady) return e;
    nanosleep(&ts, nullptr);
  }
}

// Large host mappings (transparent huge pages requested), recycled: get() hands out a free mapping of the
// size rounded up to 2 MB (the smallest that fits, if within 2x), else maps a new one; put() keeps it while
// the free ones total at most kKeep.  Process-wide, one mutex (a few calls per plan pass).
struct HugeCache {
  static constexpr size_t kKeep = size_t(2) << 30;
  std::mutex m;
  std::map<void*, size_t> live;              // mapping -> its size
  std::multimap<size_t, void*> free_by_size;
  size_t free_bytes = 0;
  void* get(size_t b) {
    b = (b + (size_t(2) << 20) - 1) & ~((size_t(2) << 20) - 1);
    {
      std::lock_guard<std::mutex> lk(m);
      auto it = free_by_size.lower_bound(b);
      if (it != free_by_size.end() && it->first <= 2 * b) {
        void* p = it->second;
        free_bytes -= it->first;
        free_by_size.erase(it);
        return p;
      }
    }
    void* p = mmap(nullptr, b, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
    if (p == MAP_FAILED) throw std::bad_alloc();
    (void)madvise(p, b, MADV_HUGEPAGE);
    std::lock_guard<std::mutex> lk(m);
    live[p] = b;
    return p;
  }
  void put(void* p) {
    std::unique_lock<std::mutex> lk(m);
    auto it = live.find(p);
    if (it == live.end()) return;
    const size_t b = it->second;
    if (free_bytes + b <= kKeep) {
      free_by_size.emplace(b, p);
      free_bytes += b;
      return;
    }
    live.erase(it);
    lk.unlock();
    munmap(p, b);
  }
};
static HugeCache& huge_cache() {
  static HugeCache* c = new HugeCache();  // never destroyed: arrays may be freed at process exit
  return *c;
}

// Host arrays a plan build fills completely: resize() leaves them uninitialised (zero-filling ~200 MB of
// descriptors for a 10 000-read block on one thread cost more than building them on 16).
template <typename T>
struct NoInitAlloc : std::allocator<T> {
  template <typename U>
  struct rebind {
    using other = NoInitAlloc<U>;
  };
  NoInitAlloc() = default;
  template <typename U>
  NoInitAlloc(const NoInitAlloc<U>&) {}
  // Large arrays (a 10 000-read block's descriptors: tens of MB each) come from their own mapping with
  // transparent huge pages requested, so that their first touch costs a fault per 2 MB rather than per
  // 4 KB page (the plan builders' passes were fault-bound on the GPU box).
  // A freed mapping is kept for the next plan's arrays (HugeCache): a block's plans free and re-create the
  // same ~300 MB of temporaries, and unmapping them (page frees, TLB shoot-downs across the plan's threads)
  // then faulting them in again cost milliseconds per plan.
  static constexpr size_t kHuge = size_t(4) << 20;
  T* allocate(size_t n) {
    const size_t b = n * sizeof(T);
    if (b < kHuge) return std::allocator<T>::allocate(n);
    return static_cast<T*>(huge_cache().get(b));
  }
  void deallocate(T* p, size_t n) {
    const size_t b = n * sizeof(T);
    if (b < kHuge) std::allocator<T>::deallocate(p, n);
    else huge_cache().put(p);
  }
  template <typename U>
  void construct(U* p) noexcept {
    ::new ((void*)p) U;
  }
  template <typename U, typename... A>
  void construct(U* p, A&&... a) {
    ::new ((void*)p) U(std::forward<A>(a)...);
  }
};
template <typename T>
using HostArray = std::vector<T, NoInitAlloc<T>>;

// A batch resolved on the host: GPU problems grouped into launch classes.
struct PlanCore {
  HostArray<DevProblem> dev;         // one per GPU problem (single / end)
  HostArray<int> dev_index;          // problem index -> dev slot (-1: resolved on host)
  HostArray<int> dev_problem;        // dev slot -> problem index
  HostArray<DevGenomeProblem> gdev;  // Dynprog_genome_gap problems on the GPU
  HostArray<int> gdev_index;         // genome problem index -> gdev slot (-1: resolved on host)
  HostArray<int> gdev_problem;       // gdev slot -> genome problem index
  // kDpx: 64/S narrow problems per wave, R = S; kSx: SIMD-build single gaps, 64/B problems per wave,
  // R = B; kUxe / kUxg: SIMD-build end / genome gaps (triangle fills), one wave per problem, R = B
  // kDpRows: dp_kernel's recurrence with lanes over query rows (dpr_kernel), R = row words
  enum Kind { kDp = 0, kGenomeGap = 1, kDpx = 2, kSx = 3, kUxe = 4, kUxg = 5, kDpRows = 7 };
  struct Launch {
    int kind;
    int R;           // band words per lane (kDp, kGenomeGap) or segment width S (kDpx)
    bool dirs_lds;
    size_t lds;      // LDS bucket per workgroup (kDpx: per problem slot)
    int first, count;
    double work;     // estimated wave-columns, for stream assignment
    double span;     // the longest single problem's estimate: the class's latency floor
    size_t extra;    // kDpx: bytes of the whole-wave direction words (per workgroup)
    size_t gdirs_offset;  // kDpx with !dirs_lds: the class's region of the global scratch
    int stream;      // 0: the caller's stream, 1..3: the context's side streams
  };
  std::vector<Launch> launches;
  std::vector<int> order;            // dev slots grouped by launch
  std::vector<int> gorder;           // gdev slots grouped by launch
  size_t pair_capacity = 0;
  size_t gdirs_bytes = 0;            // global scratch (spilled direction planes / bridge matrices)
};

static int fail(gmapdp_ctx* ctx, int code, const char* fmt, hipError_t e) {
  char buf[256];
  std::snprintf(buf, sizeof(buf), fmt, hipGetErrorString(e));
  if (ctx) ctx->err = buf;
  return code;
}

static int bad(gmapdp_ctx* ctx, const char* msg) {
  if (ctx) ctx->err = msg;
  return GMAPDP_EINVAL;
}

extern "C" {

void gmapdp_compute_bands(int* lband, int* uband, int rlength, int glength, int extraband, int widebandp) {
  if (!widebandp) {
    *lband = extraband;
    *uband = extraband;
  } else if (glength >= rlength) {
    *uband = glength - rlength + extraband;
    *lband = extraband;
  } else {
    *lband = rlength - glength + extraband;
    *uband = extraband;
  }
}

const char* gmapdp_last_error(gmapdp_ctx* ctx) { return ctx ? ctx->err.c_str() : "null context"; }

int gmapdp_create(gmapdp_ctx** out, int device, int mode, int user_open, int user_extend, int user_dynprog_p) {
  return gmapdp_create_ex(out, device, mode, user_open, user_extend, user_dynprog_p, 0);
}

int gmapdp_create_ex(gmapdp_ctx** out, int device, int mode, int user_open, int user_extend, int user_dynprog_p,
                     int flags) {
  if (!out || mode < 0 || mode > 6) return GMAPDP_EINVAL;
  *out = nullptr;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0 || device < 0 || device >= ndev) return GMAPDP_ENODEV;
  gmapdp_ctx* ctx = new gmapdp_ctx();
  ctx->device = device;
  ctx->mode = mode;
  ctx->user_open = user_open;
  ctx->user_extend = user_extend;
  ctx->user_dynprog_p = user_dynprog_p;
  ctx->one_stream = (flags & GMAPDP_CTX_ONE_STREAM) != 0;
  ctx->plan_sides = (flags & GMAPDP_CTX_TWO_SIDES) ? 2 : gmapdp_ctx::kAux;
  hipError_t e = hipSetDevice(device);
  int prio_least = 0, prio_greatest = 0;
  if (e == hipSuccess && (flags & (GMAPDP_CTX_PRIO_HIGH | GMAPDP_CTX_PRIO_LOW)))
    e = hipDeviceGetStreamPriorityRange(&prio_least, &prio_greatest);
  if (e == hipSuccess) {
    if (flags & GMAPDP_CTX_PRIO_HIGH)
      e = hipStreamCreateWithPriority(&ctx->stream, hipStreamNonBlocking, prio_greatest);
    else if (flags & GMAPDP_CTX_PRIO_LOW)
      e = hipStreamCreateWithPriority(&ctx->stream, hipStreamNonBlocking, prio_least);
    else
      e = hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking);
  }
  for (int i = 0; i < gmapdp_ctx::kAux && e == hipSuccess && !ctx->one_stream; i++) {
    e = hipStreamCreateWithFlags(&ctx->aux[i], hipStreamNonBlocking);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&ctx->ev_join[i], hipEventDisableTiming);
  }
  if (e == hipSuccess && !ctx->one_stream) e = hipEventCreateWithFlags(&ctx->ev_fork, hipEventDisableTiming);
  if (e == hipSuccess && (flags & GMAPDP_CTX_POLL_SYNC)) {
    e = hipEventCreateWithFlags(&ctx->ev_block, hipEventDisableTiming);
    ctx->poll = true;
  } else if (e == hipSuccess && (flags & GMAPDP_CTX_BLOCKING_SYNC)) {
    e = hipEventCreateWithFlags(&ctx->ev_block, hipEventDisableTiming | hipEventBlockingSync);
  }
  ctx->tables = new Tables();
  build_tables(*ctx->tables, mode);
  if (e == hipSuccess) e = hipMalloc(&ctx->d_sc, sizeof(ctx->tables->sc));
  if (e == hipSuccess) e = hipMalloc(&ctx->d_cs, sizeof(ctx->tables->cs));
  if (e == hipSuccess) e = hipMalloc(&ctx->d_isc, sizeof(ctx->tables->isc));
  if (e == hipSuccess) e = hipMemcpy(ctx->d_isc, ctx->tables->isc, sizeof(ctx->tables->isc), hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(ctx->d_sc, ctx->tables->sc, sizeof(ctx->tables->sc), hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(ctx->d_cs, ctx->tables->cs, sizeof(ctx->tables->cs), hipMemcpyHostToDevice);
  if (e != hipSuccess) {
    gmapdp_destroy(ctx);
    return GMAPDP_ENODEV;
  }
  *out = ctx;
  return GMAPDP_OK;
}

void gmapdp_destroy(gmapdp_ctx* ctx) {
  if (!ctx) return;
  (void)hipSetDevice(ctx->device);
  if (ctx->stream) (void)ctx_sync(ctx, ctx->stream);
  if (ctx->d_sc) (void)hipFree(ctx->d_sc);
  if (ctx->d_cs) (void)hipFree(ctx->d_cs);
  if (ctx->d_isc) (void)hipFree(ctx->d_isc);
  if (ctx->d_genome && ctx->genome_owned) (void)hipFree(ctx->d_genome);
  for (int i = 0; i < gmapdp_ctx::kAux; i++) {
    if (ctx->aux[i]) (void)hipStreamSynchronize(ctx->aux[i]);
    if (ctx->aux[i]) (void)hipStreamDestroy(ctx->aux[i]);
    if (ctx->ev_join[i]) (void)hipEventDestroy(ctx->ev_join[i]);
  }
  if (ctx->ev_fork) (void)hipEventDestroy(ctx->ev_fork);
  if (ctx->ev_block) (void)hipEventDestroy(ctx->ev_block);
  if (ctx->ev_hplan) {
    (void)hipEventSynchronize(ctx->ev_hplan);
    (void)hipEventDestroy(ctx->ev_hplan);
  }
  if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
  delete ctx->tables;
  delete ctx;
}

size_t gmapdp_genome_words(uint64_t length) { return (size_t)((length + 31) / 32) * 3 + 4; }

// Compress_create_blocks_comp (compress-write.c:754, put_compressed_one :293):
// 3 words per 32 nt, {high: nt 16..31, low: nt 0..15, flags}, 2 bits per nt
// (A0 C1 G2 T3), a set flag bit for any non-ACGT byte ('X' keeps code 3, all
// others code 0); the last (partial) block's tail and 4 trailing words are
// all-ones ('X' padding).
int gmapdp_pack_genome(const char* seq, uint64_t length, uint32_t* blocks) {
  if (!blocks || (!seq && length)) return GMAPDP_EINVAL;
  const uint64_t nblocks = (length + 31) / 32;
  const size_t nw = gmapdp_genome_words(length);
  std::memset(blocks, 0, nw * sizeof(uint32_t));
  for (int i = 0; i < 4; i++) blocks[3 * nblocks + i] = 0xFFFFFFFFu;
  // per byte: code in bits 0-1, flag in bit 2
  uint8_t lut[256];
  for (int c = 0; c < 256; c++) lut[c] = 4;                  // 'N' and anything else: A code + flag
  lut['A'] = lut['a'] = 0;
  lut['C'] = lut['c'] = 1;
  lut['G'] = lut['g'] = 2;
  lut['T'] = lut['t'] = 3;
  lut['X'] = lut['x'] = 3 | 4;                               // put_compressed_one: 'X' = T code + flag
  const unsigned char* s = (const unsigned char*)seq;
  for (uint64_t b = 0; b < nblocks; b++) {
    uint32_t high = 0, low = 0, flags = 0;
    const uint64_t base = b * 32;
    const int n = (int)std::min<uint64_t>(32, length - base);
    if (n == 32) {
      for (int j = 0; j < 16; j++) {
        const uint32_t v = lut[s[base + j]], w = lut[s[base + 16 + j]];
        low |= (v & 3u) << (2 * j);
        high |= (w & 3u) << (2 * j);
        flags |= ((v >> 2) << j) | ((w >> 2) << (j + 16));
      }
    } else {
      for (int j = 0; j < 32; j++) {
        const uint32_t v = j < n ? lut[s[base + j]] : (3 | 4);  // tail of the last block reads as 'X'
        if (j < 16) low |= (v & 3u) << (2 * j);
        else high |= (v & 3u) << (2 * (j - 16));
        flags |= (v >> 2) << j;
      }
    }
    blocks[3 * b] = high;
    blocks[3 * b + 1] = low;
    blocks[3 * b + 2] = flags;
  }
  return GMAPDP_OK;
}

int gmapdp_set_genome(gmapdp_ctx* ctx, const uint32_t* blocks, size_t nwords, uint64_t length) {
  if (!ctx || !blocks || nwords < (size_t)((length + 31) / 32) * 3) return GMAPDP_EINVAL;
  // coordinates are 64-bit (gmapdp_coord_t): gmapl genomes past 2^32 nt are supported
  (void)hipSetDevice(ctx->device);
  if (ctx->d_genome && ctx->genome_owned) (void)hipFree(ctx->d_genome);
  ctx->d_genome = nullptr;
  ctx->genome_owned = true;
  hipError_t e = hipMalloc(&ctx->d_genome, nwords * sizeof(uint32_t));
  if (e != hipSuccess) return fail(ctx, GMAPDP_ENOMEM, "hipMalloc genome: %s", e);
  e = hipMemcpy(ctx->d_genome, blocks, nwords * sizeof(uint32_t), hipMemcpyHostToDevice);
  if (e != hipSuccess) return fail(ctx, GMAPDP_ENOMEM, "genome upload: %s", e);
  ctx->genome_words = nwords;
  ctx->genome_length = length;
  return GMAPDP_OK;
}

int gmapdp_reserve(gmapdp_ctx* ctx, size_t bytes, int what) {
  if (!ctx) return GMAPDP_EINVAL;
  (void)hipSetDevice(ctx->device);
  hipError_t e = hipSuccess;
  auto dev = [&](DevBuf& b, size_t n) { if (e == hipSuccess) e = b.ensure(n); };
  auto host = [&](HostBuf& b, size_t n) { if (e == hipSuccess) e = b.ensure(n); };
  if (what & GMAPDP_RESERVE_DP) {
    host(ctx->hin, bytes);
    host(ctx->hout, bytes);
    dev(ctx->din, bytes);
    dev(ctx->dout, bytes);
    dev(ctx->gdirs, 4 * bytes);
  }
  if (what & GMAPDP_RESERVE_AUX) {
    for (DevBuf* b : {&ctx->mxprobs, &ctx->mxres, &ctx->mxcands, &ctx->mxcnt, &ctx->mxdirect, &ctx->mxprobs2,
                      &ctx->mxpairs, &ctx->cprobs, &ctx->corder, &ctx->cresults, &ctx->cscratch, &ctx->qseq_uc})
      dev(*b, bytes);
  }
  if (what & GMAPDP_RESERVE_STAGE2) {
    for (DevBuf* b : {&ctx->oprobs, &ctx->oresults, &ctx->oscratch, &ctx->onpos, &ctx->omap, &ctx->otable, &ctx->odiag,
                      &ctx->opool, &ctx->opoolctr, &ctx->qseq_uc, &ctx->s2probs, &ctx->s2results, &ctx->s2counters,
                      &ctx->s2paths, &ctx->s2pairs, &ctx->s2qseq})
      dev(*b, bytes);
    dev(ctx->s2scratch, 4 * bytes);
  }
  if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);  // this context only: other dispatchers keep running
  return e == hipSuccess ? GMAPDP_OK : fail(ctx, GMAPDP_ENOMEM, "reserve: %s", e);
}

struct gmapdp_dgenome {
  int device = 0;
  uint32_t* d = nullptr;
  uint64_t words = 0, length = 0;
};

int gmapdp_dgenome_create(int device, const uint32_t* blocks, size_t nwords, uint64_t length, gmapdp_dgenome** out) {
  if (!out || !blocks || nwords < (size_t)((length + 31) / 32) * 3) return GMAPDP_EINVAL;
  *out = nullptr;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev) return GMAPDP_ENODEV;
  if (hipSetDevice(device) != hipSuccess) return GMAPDP_ENODEV;
  gmapdp_dgenome* g = new gmapdp_dgenome();
  g->device = device;
  if (hipMalloc(&g->d, nwords * sizeof(uint32_t)) != hipSuccess) {
    delete g;
    return GMAPDP_ENOMEM;
  }
  if (hipMemcpy(g->d, blocks, nwords * sizeof(uint32_t), hipMemcpyHostToDevice) != hipSuccess) {
    (void)hipFree(g->d);
    delete g;
    return GMAPDP_ENOMEM;
  }
  g->words = nwords;
  g->length = length;
  *out = g;
  return GMAPDP_OK;
}

void gmapdp_dgenome_destroy(gmapdp_dgenome* g) {
  if (!g) return;
  (void)hipSetDevice(g->device);
  if (g->d) (void)hipFree(g->d);
  delete g;
}

int gmapdp_use_dgenome(gmapdp_ctx* ctx, const gmapdp_dgenome* g) {
  if (!ctx || !g || ctx->device != g->device) return GMAPDP_EINVAL;
  (void)hipSetDevice(ctx->device);
  if (ctx->d_genome && ctx->genome_owned) (void)hipFree(ctx->d_genome);
  ctx->d_genome = g->d;
  ctx->genome_words = g->words;
  ctx->genome_length = g->length;
  ctx->genome_owned = false;
  return GMAPDP_OK;
}

int gmapdp_share_genome(gmapdp_ctx* ctx, const gmapdp_ctx* owner) {
  if (!ctx || !owner || ctx == owner || ctx->device != owner->device) return GMAPDP_EINVAL;
  if (!owner->d_genome) return GMAPDP_ENOGENOME;
  (void)hipSetDevice(ctx->device);
  if (ctx->d_genome && ctx->genome_owned) (void)hipFree(ctx->d_genome);
  ctx->d_genome = owner->d_genome;
  ctx->genome_words = owner->genome_words;
  ctx->genome_length = owner->genome_length;
  ctx->genome_owned = false;
  return GMAPDP_OK;
}

}  // extern "C"

// ---------------------------------------------------------------------------
// Device MaxEnt (me_device.h): the reference's model tables (maxent_hr.c:25-24660), as
// tools/make_maxent_tables.py writes them, loaded once per process and uploaded once per device.
// ---------------------------------------------------------------------------
static std::mutex g_me_mu;
static std::vector<double> g_me_host;
static std::string g_me_path, g_me_err;
static double* g_me_dev[64];

static std::string me_path() {
  if (const char* e = getenv("GMAPDP_MAXENT_TABLES")) return e;
  Dl_info info;
  if (dladdr((void*)&gmapdp_genome_words, &info) && info.dli_fname) {
    const std::string so = info.dli_fname;
    const size_t k = so.rfind('/');
    return (k == std::string::npos ? std::string(".") : so.substr(0, k)) + "/maxent_hr_tables.bin";
  }
  return "maxent_hr_tables.bin";
}

static bool me_load_host_locked() {
  if (!g_me_host.empty()) return true;
  g_me_path = me_path();
  FILE* f = std::fopen(g_me_path.c_str(), "rb");
  if (!f) {
    g_me_err = "maxent tables: cannot open " + g_me_path + " (tools/make_maxent_tables.py writes it)";
    return false;
  }
  char magic[8];
  uint32_t hdr[2];
  bool ok = std::fread(magic, 1, 8, f) == 8 && std::memcmp(magic, "GMDPMXT1", 8) == 0 &&
            std::fread(hdr, 4, 2, f) == 2 && hdr[0] == 16;
  std::vector<double> all(kMeTotal);
  for (int t = 0; ok && t < 16; t++) {
    char name[32];
    uint32_t h[2];
    ok = std::fread(name, 1, 32, f) == 32 && std::fread(h, 4, 2, f) == 2 && (int)h[0] == kMeEntries[t] &&
         std::fread(all.data() + me_offset(t), sizeof(double), h[0], f) == h[0];
  }
  std::fclose(f);
  if (!ok) {
    g_me_err = "maxent tables: " + g_me_path + " is not a tools/make_maxent_tables.py table file";
    return false;
  }
  g_me_host.swap(all);
  return true;
}

// the device copy of the tables for ctx's device, or nullptr with ctx->err set
static const double* me_tables(gmapdp_ctx* ctx) {
  std::lock_guard<std::mutex> lk(g_me_mu);
  if (!me_load_host_locked()) {
    ctx->err = g_me_err;
    return nullptr;
  }
  if (ctx->device < 0 || ctx->device >= 64) return nullptr;
  if (!g_me_dev[ctx->device]) {
    double* d = nullptr;
    hipError_t e = hipMalloc(&d, sizeof(double) * kMeTotal);
    if (e == hipSuccess) e = hipMemcpy(d, g_me_host.data(), sizeof(double) * kMeTotal, hipMemcpyHostToDevice);
    if (e != hipSuccess) {
      if (d) (void)hipFree(d);
      ctx->err = std::string("maxent tables upload: ") + hipGetErrorString(e);
      return nullptr;
    }
    g_me_dev[ctx->device] = d;
  }
  return g_me_dev[ctx->device];
}

extern "C" {

int gmapdp_maxent_available(char* path, size_t path_bytes) {
  std::lock_guard<std::mutex> lk(g_me_mu);
  const bool ok = me_load_host_locked();
  if (path && path_bytes) std::snprintf(path, path_bytes, "%s", g_me_path.c_str());
  return ok ? 1 : 0;
}

int gmapdp_maxent_sites(gmapdp_ctx* ctx, const gmapdp_coord_t* positions, const uint8_t* models,
                        const gmapdp_coord_t* chroffsets, size_t n, double* out) {
  if (!ctx || (n && (!positions || !models || !chroffsets || !out))) return GMAPDP_EINVAL;
  if (!ctx->d_genome) return GMAPDP_ENOGENOME;
  if (n == 0) return GMAPDP_OK;
  (void)hipSetDevice(ctx->device);
  const double* T = me_tables(ctx);
  if (!T) return GMAPDP_EINVAL;
  const size_t o_pos = 0, o_chr = o_pos + 8 * n, o_mod = o_chr + 8 * n, in_bytes = o_mod + n;
  hipError_t e = ctx->din.ensure(in_bytes);
  if (e == hipSuccess) e = ctx->dout.ensure(8 * n);
  if (e != hipSuccess) return fail(ctx, GMAPDP_ENOMEM, "maxent buffers: %s", e);
  unsigned char* din = (unsigned char*)ctx->din.p;
  hipStream_t s = ctx->stream;
  e = hipMemcpyAsync(din + o_pos, positions, 8 * n, hipMemcpyHostToDevice, s);
  if (e == hipSuccess) e = hipMemcpyAsync(din + o_chr, chroffsets, 8 * n, hipMemcpyHostToDevice, s);
  if (e == hipSuccess) e = hipMemcpyAsync(din + o_mod, models, n, hipMemcpyHostToDevice, s);
  if (e == hipSuccess)
    e = launch_me_sites((long long)n, s, ctx->d_genome, ctx->genome_words, T, (const gmapdp_coord_t*)(din + o_pos),
                        din + o_mod, (const gmapdp_coord_t*)(din + o_chr), (double*)ctx->dout.p);
  if (e == hipSuccess) e = hipMemcpyAsync(out, ctx->dout.p, 8 * n, hipMemcpyDeviceToHost, s);
  if (e == hipSuccess) e = ctx_sync(ctx, s);
  return e == hipSuccess ? GMAPDP_OK : fail(ctx, GMAPDP_ELAUNCH, "maxent: %s", e);
}

}  // extern "C"

// ---------------------------------------------------------------------------
// Planning: resolve host-side cases, derive penalties, bands, orientation and
// segment extraction, pick the launch class and LDS footprint, and lay out
// the pair arena.
// ---------------------------------------------------------------------------
static const size_t kLdsBudget = 64 * 1024;  // per workgroup; keeps >= 2 problems resident per CU
// Packed workgroups keep their direction words in LDS while the workgroup's LDS stays within
// this; GMAPDP_DPX_LDS_DIRS_MAX overrides it (experiments).
static size_t env_size(const char* name, size_t dflt);
static size_t dpx_lds_dirs_max() {
  static const size_t v = env_size("GMAPDP_DPX_LDS_DIRS_MAX", 4 * 1024);
  return v;
}

static int pick_R(int W) {
  int R = 1;
  while (R * 64 < W) R <<= 1;
  return R;
}

static size_t lds_bucket(size_t lds) {
  static const size_t b[] = {4096, 8192, 16384, 32768, 49152, 65536, 98304, 163840};
  for (size_t x : b)
    if (lds <= x) return x;
  return lds;
}

// genome-gap workgroups: finer steps, since their LDS sets how many problems a CU holds
static size_t gg_lds_bucket(size_t lds) {
  static const size_t b[] = {4096,  6144,  8192,  10240, 12288, 14336, 16384, 20480, 24576,
                             28672, 32768, 40960, 49152, 65536, 98304, 163840};
  for (size_t x : b)
    if (lds <= x) return x;
  return lds;
}

static size_t env_size(const char* name, size_t dflt) {
  const char* e = getenv(name);
  return e ? (size_t)strtoull(e, nullptr, 10) : dflt;
}

// genome-gap direction planes stay in LDS while the workgroup's LDS stays within this; by default
// they always go to the L2-resident scratch, which measured fastest (more problems per CU).
// GMAPDP_GG_LDS_DIRS_MAX overrides it, for experiments.
static size_t gg_lds_dirs_max() { return env_size("GMAPDP_GG_LDS_DIRS_MAX", 0); }
// GMAPDP_DP_ROWS=0 keeps every single / end gap in the band layout (experiments, tests)
static bool rows_disabled() {
  static const bool v = env_size("GMAPDP_DP_ROWS", 1) == 0;
  return v;
}
// Batches of at most this many problems are planned for latency (classify); GMAPDP_LATENCY_BATCH
// overrides it.
static size_t latency_batch() {
  static const size_t v = env_size("GMAPDP_LATENCY_BATCH", 1024);
  return v;
}

// per-problem LDS slot of the packed kernel (64/S slots per workgroup)
static size_t slot_bucket(size_t b) {
  static const size_t s[] = {256, 384, 512, 768, 1024, 1536, 2048, 3072, 4096, 6144, 8192, 12288, 16384};
  for (size_t x : s)
    if (b <= x) return x;
  return 0;  // too big to pack
}

static void null_result(gmapdp_result& res, int score, int dpi) {
  res.npairs = 0;
  res.traceback_score = score;
  res.nmatches = res.nmismatches = res.nopens = res.nindels = 0;
  res.dynprogindex = dpi;
}

static int next_dpi(int dpi) { return dpi + (dpi > 0 ? 1 : -1); }

// Dynprog_single_gap (dynprog_single.c:459-592): returns 1 if the problem runs on the GPU.
static int convert_single(const gmapdp_ctx* ctx, const gmapdp_single_problem& p, gmapdp_result& res, DevProblem& d) {
  if (p.rlength <= 0 || p.glength <= 0 || p.rlength > GMAPDP_MAX_RLENGTH || p.glength > GMAPDP_MAX_GLENGTH) {
    null_result(res, GMAPDP_NEG_INFINITY_32, next_dpi(p.dynprogindex));  // size guard (:509-521)
    return 0;
  }
  std::memset(&d, 0, sizeof(d));
  d.kind = kSingle;
  d.qbase = p.qoff;
  d.rlength = p.rlength;
  d.glength = p.glength;
  d.roffset = p.roffset;
  d.goffset = p.goffset;
  d.chroffset = p.chroffset;
  d.chrhigh = p.chrhigh;
  const double dr = p.defect_rate;
  d.mismatchtype = dr < 0.003 ? kHighQ : (dr < 0.014 ? kMedQ : kLowQ);  // DEFECT_HIGHQ / DEFECT_MEDQ
  if (ctx->user_dynprog_p) {
    d.open = ctx->user_open;
    d.extend = ctx->user_extend;
  } else if (dr < 0.003) {
    d.open = -8; d.extend = -3;  // SINGLE_OPEN/EXTEND_HIGHQ
  } else if (dr < 0.014) {
    d.open = -7; d.extend = -2;
  } else {
    d.open = -6; d.extend = -1;
  }
  const bool watson = p.flags & GMAPDP_WATSON;
  d.flags = (watson ? kFWatson : 0) | ((p.flags & GMAPDP_JUMP_LATE) ? kFLate : 0) |
            ((p.flags & GMAPDP_SIMD) ? kFSimd : 0);
  if (watson) {
    d.segpos = p.chroffset + (uint64_t)(int64_t)p.goffset;  // Genome_get_segment_right(left, chrhigh)
    d.segbound = p.chrhigh;
  } else {
    d.segpos = p.chrhigh - (uint64_t)(int64_t)p.goffset + 1u;  // Genome_get_segment_left(right, chroffset), revcomp
    d.segbound = p.chroffset;
    d.flags |= kFSegLeft | kFSegRevcomp;
  }
  gmapdp_compute_bands(&d.lband, &d.uband, p.rlength, p.glength, p.extraband, p.flags & GMAPDP_WIDEBAND);
  if (!(p.flags & GMAPDP_SIMD)) {
    // stage3.c:9070-9077 passes extraband_single = |queryjump - genomejump|, so the band can be
    // ~3x glength wide.  Dynprog_standard only asks whether c - uband < 1 and c + lband > rlength
    // (dynprog.c:1411-1449), so a band past the matrix edges fills exactly the same cells as one
    // clamped to them: uband >= glength keeps every rlo at 1, lband >= rlength every rhigh at rlength.
    d.uband = std::min(d.uband, p.glength);
    d.lband = std::min(d.lband, p.rlength);
  }
  d.genestrand = p.genestrand;
  d.dynprogindex = p.dynprogindex;
  d.endalign = 0;
  return 1;
}

// Dynprog_end5_gap / Dynprog_end3_gap prologues (dynprog_end.c:1333-1411 / 1962-2027).
static int convert_end(const gmapdp_ctx* ctx, const gmapdp_end_problem& p, gmapdp_result& res, DevProblem& d,
                       int* err, const char** why) {
  *err = 0;
  auto bad = [why](const gmapdp_ctx*, const char* msg) {
    *why = msg;
    return GMAPDP_EINVAL;
  };
  const bool end3 = p.end3p != 0;
  const bool nogaps = p.endalign == kQueryendNogaps;
  if (p.endalign < 0 || p.endalign > 3) {
    *err = bad(ctx, "endalign out of range");
    return 0;
  }
  int rlength = p.rlength, glength = p.glength;
  if (rlength <= 0) { null_result(res, 0, p.dynprogindex); return 0; }
  if (!nogaps && rlength > GMAPDP_MAX_RLENGTH) rlength = GMAPDP_MAX_RLENGTH;
  if (!end3 && p.goffset < 0) { null_result(res, 0, p.dynprogindex); return 0; }
  if (glength <= 0) { null_result(res, 0, p.dynprogindex); return 0; }
  if (!nogaps && glength > GMAPDP_MAX_GLENGTH) glength = GMAPDP_MAX_GLENGTH;
  if (end3 && p.goffset < 0) {
    *err = bad(ctx, "Dynprog_end3_gap with goffset < 0 (the reference asserts)");
    return 0;
  }
  std::memset(&d, 0, sizeof(d));
  d.kind = end3 ? kEnd3 : kEnd5;
  d.endalign = p.endalign;
  d.rlength = rlength;
  d.glength = glength;
  d.roffset = p.roffset;
  d.goffset = p.goffset;
  d.chroffset = p.chroffset;
  d.chrhigh = p.chrhigh;
  d.mismatchtype = kEndQ;
  const double dr = p.defect_rate;
  if (ctx->user_dynprog_p) {
    d.open = ctx->user_open;
    d.extend = ctx->user_extend;
  } else {
    d.open = dr < 0.003 ? -10 : (dr < 0.014 ? -8 : -6);  // END_OPEN_HIGHQ/MEDQ/LOWQ
    d.extend = -2;                                        // END_EXTEND_*
  }
  const bool watson = p.flags & GMAPDP_WATSON;
  const bool jl = p.flags & GMAPDP_JUMP_LATE;
  d.flags = (watson ? kFWatson : 0) | (p.require_pos_score_p ? kFRequirePos : 0);
  if (end3) {
    d.qbase = p.qoff;
    d.flags |= (jl ? kFLate : 0) | kFScoreUC;  // end3 fills on rsequenceuc (dynprog_end.c:2061)
    if (watson) {
      d.segpos = p.chroffset + (uint64_t)(int64_t)p.goffset;
      d.segbound = p.chrhigh;
    } else {
      d.segpos = p.chrhigh - (uint64_t)(int64_t)p.goffset + 1u;
      d.segbound = p.chroffset;
      d.flags |= kFSegLeft | kFSegRevcomp;
    }
  } else {
    d.qbase = p.qoff + p.rlength - 1;          // rev_rsequence: the slice's last character
    d.flags |= (jl ? 0 : kFLate) | kFRev;      // fills with !jump_late_p, revp
    if (watson) {
      d.segpos = p.chroffset + (uint64_t)(int64_t)p.goffset + 1u;  // Genome_get_segment_left(right, chroffset)
      d.segbound = p.chroffset;
      d.flags |= kFSegLeft;
    } else {
      d.segpos = p.chrhigh - (uint64_t)(int64_t)p.goffset;  // Genome_get_segment_right(left, chrhigh), revcomp
      d.segbound = p.chrhigh;
      d.flags |= kFSegRevcomp;
    }
  }
  if (!nogaps)
    gmapdp_compute_bands(&d.lband, &d.uband, rlength, glength, p.extraband,
                         /*widebandp*/ p.endalign != kQueryendIndels);
  if ((p.flags & GMAPDP_SIMD) && !nogaps) {
    // The SIMD builds' triangles (QUERYEND_NOGAPS has no fill: the same path in every build).
    // find_best_endpoint_8/16 scans lower[r][c] for every c < r, so rlength > glength + 1 reads
    // columns past glength, which the reference fills from uninitialised pair scores.
    if (rlength > glength + 1) {
      *err = bad(ctx, "GMAPDP_SIMD end gap with rlength > glength + 1: the reference's lower-triangle scan "
                      "reads uninitialised pair scores there (stage3.c passes glength >= rlength)");
      return 0;
    }
    if (d.lband < 0 || d.uband < 0) {
      *err = bad(ctx, "negative band");
      return 0;
    }
    d.flags |= kFSimd;
  }
  d.genestrand = p.genestrand;
  d.dynprogindex = p.dynprogindex;
  return 1;
}

// Dynprog_genome_gap prologue (dynprog_genome.c:3351-3470): returns 1 if the problem runs on the GPU.
static int convert_genome(const gmapdp_ctx* ctx, const gmapdp_genome_problem& p, gmapdp_genome_result& res,
                          DevGenomeProblem& d, int* err, const char** why) {
  *err = 0;
  auto bad = [why](const gmapdp_ctx*, const char* msg) {
    *why = msg;
    return GMAPDP_EINVAL;
  };
  res.npairs = 0;
  res.pair_offset = 0;
  res.nmatches = res.nmismatches = res.nopens = res.nindels = 0;
  res.left_prob = res.right_prob = 0.0;
  res.introntype = 0;
  res.new_leftgenomepos = res.new_rightgenomepos = res.exonhead = GMAPDP_UNSET;
  res.gap_index = -1;
  res.gap_queryjump = 0;
  res.dynprogindex = p.dynprogindex;
  if (p.rlength <= 1) {
    res.traceback_score = GMAPDP_NEG_INFINITY_32;
    return 0;
  }
  const double dr = p.defect_rate;
  std::memset(&d, 0, sizeof(d));
  d.mismatchtype = dr < 0.003 ? kHighQ : (dr < 0.014 ? kMedQ : kLowQ);
  if (ctx->user_dynprog_p) {
    d.open = ctx->user_open;
    d.extend = ctx->user_extend;
  } else {
    // SINGLE_* when rlength > maxpeelback*4, else PAIRED_* (dynprog.h:62-76; equal values)
    d.open = dr < 0.003 ? -8 : (dr < 0.014 ? -7 : -6);
    d.extend = dr < 0.003 ? -3 : (dr < 0.014 ? -2 : -1);
  }
  if (p.rlength > GMAPDP_MAX_RLENGTH || p.glengthL > GMAPDP_MAX_GLENGTH || p.glengthR > GMAPDP_MAX_GLENGTH) {
    res.new_leftgenomepos = p.goffsetL - 1;  // size guard (:3405-3439)
    res.new_rightgenomepos = p.rev_goffsetR + 1;
    res.exonhead = p.roffset + p.rlength - 1;
    res.dynprogindex = next_dpi(p.dynprogindex);
    res.traceback_score = GMAPDP_NEG_INFINITY_32;
    return 0;
  }
  if (p.glengthL <= p.rlength || p.glengthR <= p.rlength) {
    *err = bad(ctx, "Dynprog_genome_gap needs glengthL, glengthR > rlength (the reference reads "
                    "uninitialised splice probabilities otherwise)");
    return 0;
  }
  if (p.extraband < 0) {
    *err = bad(ctx, "negative extraband_paired");
    return 0;
  }
  d.qbase = p.qoff;
  d.rlength = p.rlength;
  d.glengthL = p.glengthL;
  d.glengthR = p.glengthR;
  d.roffset = p.roffset;
  d.goffsetL = p.goffsetL;
  d.rev_goffsetR = p.rev_goffsetR;
  d.chroffset = p.chroffset;
  d.chrhigh = p.chrhigh;
  const bool watson = p.flags & GMAPDP_WATSON;
  d.flags = (watson ? kFWatson : 0) | ((p.flags & GMAPDP_JUMP_LATE) ? kFLate : 0) |
            ((p.flags & GMAPDP_HALFP) ? kGHalf : 0) | ((p.flags & GMAPDP_FINALP) ? kGFinal : 0);
  if (!(p.flags & GMAPDP_FINALP) && dr < 0.014) d.flags |= kGSimple;  // :3479
  if (p.flags & GMAPDP_SIMD) d.flags |= kGSimd;
  if (p.flags & GMAPDP_KNOWN_SITES) {
    if (p.known_offset < 0) {
      *err = bad(ctx, "negative known_offset");
      return 0;
    }
    d.flags |= kGKnown;
    d.known_offset = p.known_offset;
  }
  if (watson) {
    d.segposL = p.chroffset + (uint64_t)(int64_t)p.goffsetL;  // Genome_get_segment_right(left, chrhigh)
    d.segboundL = p.chrhigh;
    d.segposR = p.chroffset + (uint64_t)(int64_t)p.rev_goffsetR + 1u;  // Genome_get_segment_left(right, chroffset)
    d.segboundR = p.chroffset;
    d.flags |= kGSegRLeft;
  } else {
    d.segposL = p.chrhigh - (uint64_t)(int64_t)p.goffsetL + 1u;  // _left(right, chroffset), revcomp
    d.segboundL = p.chroffset;
    d.segposR = p.chrhigh - (uint64_t)(int64_t)p.rev_goffsetR;   // _right(left, chrhigh), revcomp
    d.segboundR = p.chrhigh;
    d.flags |= kGSegLLeft | kGSegLRc | kGSegRRc;
  }
  // Dynprog_compute_bands(widebandp true) with glength > rlength: lband = extraband,
  // uband = glength - rlength + extraband; these equal bridge_intron_gap's own bands (:2924-2928)
  d.lbandL = p.extraband;
  d.ubandL = p.glengthL - p.rlength + p.extraband;
  d.ubandR = p.glengthR - p.rlength + p.extraband;
  d.iclass = p.cdna_direction > 0 ? 0 : (p.cdna_direction < 0 ? 1 : 2);
  d.genestrand = p.genestrand;
  d.dynprogindex = p.dynprogindex;
  d.prob_offset = p.prob_offset;
  return 1;
}

// GMAPDP_PLAN_TIMING=1: the plan builders print their phase times (ms) to stderr (tools, not the product)
struct PlanTimer {
  const char* what;
  bool on;
  struct timespec t0;
  std::string line;
  explicit PlanTimer(const char* w) : what(w), on(getenv("GMAPDP_PLAN_TIMING") != nullptr) {
    if (on) clock_gettime(CLOCK_MONOTONIC, &t0);
  }
  void mark(const char* phase) {
    if (!on) return;
    struct timespec t1;
    clock_gettime(CLOCK_MONOTONIC, &t1);
    char b[96];
    std::snprintf(b, sizeof(b), " %s=%.1f", phase, (t1.tv_sec - t0.tv_sec) * 1e3 + (t1.tv_nsec - t0.tv_nsec) * 1e-6);
    line += b;
    t0 = t1;
  }
  ~PlanTimer() {
    if (!on) return;
    size_t fr = 0, tot = 0;
    // (=2: with the device's free memory; hipMemGetInfo takes milliseconds, so phase times are without it)
    if (std::atoi(getenv("GMAPDP_PLAN_TIMING")) >= 2) (void)hipMemGetInfo(&fr, &tot);
    std::fprintf(stderr, "[gmapdp plan timing] %s%s (device free %.1f of %.1f GB)\n", what, line.c_str(), fr * 1e-9,
                 tot * 1e-9);
  }
};

// ---- host threads of a plan build ----
// A batch of kPlanParallelMin problems or more (bench.py's 10 000-read blocks: ~840 000) is planned on
// GMAPDP_PLAN_THREADS host threads (default: min(16, hardware threads); a GPU-box job is given 16 cores);
// smaller batches (the drop-in's dispatcher batches) on the calling thread.  The plan is the same either
// way: per-problem work is independent, offsets are prefix sums taken in problem order, classes keep
// their members in problem order and sort them stably.
static const size_t kPlanParallelMin = 16384;
static int plan_threads(size_t n) {
  static const int v = [] {
    const char* e = getenv("GMAPDP_PLAN_THREADS");
    int t = e ? atoi(e) : 0;
    if (t <= 0) t = (int)std::min(16u, std::max(1u, std::thread::hardware_concurrency()));
    return t;
  }();
  return n >= kPlanParallelMin ? v : 1;
}
// The plan's worker threads, started once per process: a block's plans run ~15 parallel passes, and
// starting and joining 15 threads per pass cost milliseconds of a ~20-ms plan.  One caller at a time (a
// second concurrent caller, or a forked child, starts its own threads as before); workers sleep on a
// condition variable between passes.  Never destroyed: the threads end with the process.
struct PlanPool {
  std::mutex use;  // held by the pass being run
  std::mutex m;
  std::condition_variable cv;
  uint64_t gen = 0;
  int nchunks = 0;
  void (*call)(void*, int) = nullptr;
  void* arg = nullptr;
  std::atomic<int> left{0};
  int nthreads = 0;
  pid_t pid = 0;
  void start(int n) {
    pid = getpid();
    nthreads = n;
    for (int i = 1; i <= n; i++)
      std::thread([this, i] {
        uint64_t seen = 0;
        for (;;) {
          std::unique_lock<std::mutex> lk(m);
          cv.wait(lk, [&] { return gen != seen; });
          seen = gen;
          const bool mine = i < nchunks;
          void (*c)(void*, int) = call;
          void* a = arg;
          lk.unlock();
          if (mine) {
            c(a, i);
            left.fetch_sub(1, std::memory_order_acq_rel);
          }
        }
      }).detach();
  }
  // chunks 1..T-1 on the workers, chunk 0 on the caller; false: pool unavailable (caller spawns threads)
  template <typename G>
  bool run(int T, G& g) {
    if (T - 1 > nthreads || getpid() != pid || !use.try_lock()) return false;
    {
      std::lock_guard<std::mutex> lk(m);
      nchunks = T;
      call = [](void* a, int t) { (*static_cast<G*>(a))(t); };
      arg = &g;
      left.store(T - 1, std::memory_order_release);
      gen++;
    }
    cv.notify_all();
    g(0);
    while (left.load(std::memory_order_acquire) != 0) std::this_thread::yield();
    use.unlock();
    return true;
  }
};
static PlanPool* plan_pool(int T) {
  static PlanPool* p = [T] {
    PlanPool* q = new PlanPool();
    q->start(std::max(T, plan_threads(kPlanParallelMin)) - 1);
    return q;
  }();
  return p;
}
// f(begin, end, t) over T contiguous chunks of [0, n), chunk 0 on the calling thread
template <typename F>
static void plan_parallel(size_t n, int T, F&& f) {
  if (T <= 1 || n < 2) {
    f((size_t)0, n, 0);
    return;
  }
  const size_t per = (n + (size_t)T - 1) / (size_t)T;
  auto chunk = [&](int t) {
    const size_t lo = (size_t)t * per, hi = std::min(n, lo + per);
    if (lo < hi) f(lo, hi, t);
  };
  if (plan_pool(T)->run(T, chunk)) return;
  std::vector<std::thread> th;
  for (int t = 1; t < T; t++) th.emplace_back([&chunk, t] { chunk(t); });
  chunk(0);
  for (auto& x : th) x.join();
}
// ids ordered longest first by key(id): a stable counting sort on the key quantised to 16 steps per
// doubling (1 024 buckets, descending), threads over contiguous chunks (per-chunk histograms, then each chunk
// scatters its ids after the earlier chunks' of the same bucket).  The launch order only steers the tail of a
// launch, so 6 % key steps are as good as an exact sort; a comparison sort reading two random descriptors
// per comparison spent most of a 10 000-read plan on cache misses.
static inline int plan_bucket(uint64_t key) {
  if (key < 16) return (int)key;
  const int lg = 63 - __builtin_clzll(key);  // >= 4
  return std::min(1023, 16 * (lg - 3) + (int)((key >> (lg - 4)) & 15));
}
template <typename KF>
static void plan_sort_desc(std::vector<int>& ids, int T, KF key) {
  const size_t n = ids.size();
  if (n < 2) return;
  constexpr int NB = 1024;
  const int TT = n >= 65536 ? T : 1;
  std::vector<uint16_t> bk(n);
  std::vector<std::vector<uint32_t>> hist(TT, std::vector<uint32_t>(NB, 0));
  const size_t per = (n + (size_t)TT - 1) / (size_t)TT;
  plan_parallel(n, TT, [&](size_t lo, size_t hi, int t) {
    std::vector<uint32_t>& h = hist[t];
    for (size_t i = lo; i < hi; i++) {
      const int b = NB - 1 - plan_bucket(key(ids[i]));  // descending keys
      bk[i] = (uint16_t)b;
      h[b]++;
    }
  });
  std::vector<std::vector<uint32_t>> at(TT, std::vector<uint32_t>(NB));
  uint32_t run = 0;
  for (int b = 0; b < NB; b++)
    for (int t = 0; t < TT; t++) {
      at[t][b] = run;
      run += hist[t][b];
    }
  std::vector<int> out(n);
  plan_parallel(n, TT, [&](size_t lo, size_t hi, int t) {
    std::vector<uint32_t>& a = at[t];
    for (size_t i = lo; i < hi; i++) out[a[bk[i]]++] = ids[i];
  });
  (void)per;
  ids.swap(out);
}

// a launch class key ordered as the tuple (kind, R, dirs in LDS, LDS bucket)
static uint64_t class_key(int kind, int R, int dl, size_t bucket) {
  return ((uint64_t)kind << 48) | ((uint64_t)R << 32) | ((uint64_t)(dl ? 1 : 0) << 31) | (uint64_t)bucket;
}
struct ClassOf {  // (an aggregate: classify_dev / _gdev value-initialise it; arrays of it are left uninitialised)
  uint64_t key;
  size_t need;       // the problem's LDS bucket (a latency-mode class takes its largest member's)
  size_t pair;       // pair-arena records reserved
  size_t gdirs;      // bytes of the global direction scratch, 0: none
  const char* err;
  uint64_t len;      // the launch-order length (cells of the band) and work estimate (class_work)
  double one;
  int gm;
};

// A problem's launch-order length, work estimate and step count by its class (kind, R), filled in by the
// classification pass while its descriptor is in cache.
static void class_work(ClassOf& c, const DevProblem& d) {
  const int kind = (int)(c.key >> 48), R = (int)((c.key >> 32) & 0xFFFF);
  c.len = (uint64_t)d.glength * (uint64_t)(d.lband + d.uband + 1);
  c.gm = 0;
  if (kind == PlanCore::kUxe) {
    c.one = (double)(d.rlength + d.glength) + 0.5 * d.rlength;
  } else if (kind == PlanCore::kSx) {
    c.gm = steps_sx(d.rlength, d.lband, d.uband, R);
    c.one = (double)c.gm * R / 64.0 + 0.25 * (d.rlength + d.glength);
  } else {
    c.gm = (int)d.glength;
    c.one = (double)d.glength * (kind == PlanCore::kDpx ? R / 64.0 : R) + 0.25 * (d.rlength + d.glength);
  }
}
static void class_work(ClassOf& c, const DevGenomeProblem& d) {
  const int kind = (int)(c.key >> 48), R = (int)((c.key >> 32) & 0xFFFF);
  c.len = (uint64_t)(d.glengthL + d.glengthR) * (uint64_t)(2 * d.lbandL + d.ubandL + d.ubandR + 2);
  c.one = kind == PlanCore::kGenomeGap ? (double)std::max(d.glengthL, d.glengthR) * R + d.rlength
                                       : (double)(d.glengthL + d.glengthR + 2 * d.rlength) + 4.0 * d.rlength;
  c.gm = 0;
}

// one single / end gap's launch class (classify's rules)
static ClassOf classify_dev(DevProblem& d, bool latency) {
  ClassOf c{};
  c.pair = (size_t)d.rlength + (size_t)d.glength + 2;
  d.dirs_offset = 0;
  const bool nofill = d.kind != kSingle && d.endalign == kQueryendNogaps;
  if ((d.flags & kFSimd) && d.kind != kSingle) {
    // Dynprog_end5/3_gap of the SIMD builds (dynprog_end.c:1406 / 2027): 8-bit triangles when
    // either length is below use8p_size[ENDQ]
    const int B = (d.rlength < kUse8pSize[kEndQ] || d.glength < kUse8pSize[kEndQ]) ? 32 : 16;
    const size_t lds = lds_bytes_uxe(d.rlength, d.glength, B);
    if (lds > 160 * 1024) { c.err = "problem exceeds the LDS of a CU"; return c; }
    c.gdirs = (scratch_bytes_uxe(d.rlength, d.glength, d.lband, d.uband, B) + 255) & ~(size_t)255;
    c.need = gg_lds_bucket(lds);
    c.key = class_key((int)PlanCore::kUxe, B, 0, latency ? 0 : c.need);
    return c;
  }
  if (d.flags & kFSimd) {
    // Dynprog_single_gap of the SIMD builds (dynprog_single.c:593-631): 8-bit blocks of 32 rows when
    // both lengths are below use8p_size (dynprog.c:1022-1025), else 16-bit blocks of 16 rows
    static const int use8p[4] = {41, 63, 127, 24};
    const int B = (d.rlength < use8p[d.mismatchtype] && d.glength < use8p[d.mismatchtype]) ? 32 : 16;
    const size_t slot = gg_lds_bucket(lds_slot_sx(d.rlength, d.glength, B));
    if (slot * (64 / B) > 160 * 1024) { c.err = "problem exceeds the LDS of a CU"; return c; }
    c.need = slot;
    c.key = class_key((int)PlanCore::kSx, B, 0, latency ? 0 : slot);
    return c;
  }
  if (d.open > 0 && !nofill) { c.err = "positive gap-open penalty is not supported by the scan formulation"; return c; }
  if (d.lband < 0 || d.uband < 0) { c.err = "negative band"; return c; }
  const int W = d.lband + d.uband + 1;
  if (!latency && (nofill || W <= 32)) {  // narrow band: pack 64/S problems per wave
    const int S = (nofill || W <= 16) ? 16 : 32;
    const size_t slot = slot_bucket(lds_slot_dpx(d.rlength, d.glength));
    if (slot && slot * (64 / S) + lds_dirs_dpx(d.glength) <= kLdsBudget) {
      c.need = slot;
      c.key = class_key((int)PlanCore::kDpx, S, 1, slot);
      return c;
    }
  }
  int R = nofill ? 1 : pick_R(W);
  if (R > kMaxR) { c.err = "band wider than 4096"; return c; }
  // a band wider than the query: lanes over the query's rows cost fewer words per column
  const int Rrows = pick_R(d.rlength + 1);
  const bool rows = !nofill && Rrows < R && !rows_disabled();
  if (rows) R = Rrows;
  size_t lds = lds_bytes_dp(d.rlength, d.glength, R, !nofill);
  const bool dirs_lds = !nofill && lds <= kLdsBudget;
  if (!dirs_lds) {
    lds = lds_bytes_dp(d.rlength, d.glength, R, false);
    if (!nofill) c.gdirs = ((size_t)(d.glength + 1) * 4 * R * 8 + 255) & ~(size_t)255;
  }
  if (lds > 160 * 1024) { c.err = "problem exceeds the LDS of a CU"; return c; }
  c.need = lds_bucket(lds);
  c.key = class_key((int)(rows ? PlanCore::kDpRows : PlanCore::kDp), R, dirs_lds ? 1 : 0, latency ? 0 : c.need);
  return c;
}

// one genome gap's launch class
static ClassOf classify_gdev(DevGenomeProblem& d, bool latency, size_t lds_dirs_max) {
  ClassOf c{};
  // traceback R (<= r + gR records) + gap holder + traceback L (<= r + gL records)
  c.pair = 2 * (size_t)d.rlength + (size_t)d.glengthL + (size_t)d.glengthR + 4;
  if (d.flags & kGSimd) {
    // the SIMD builds' genome gap (dynprog_genome.c:3501-3507): 8-bit triangles when rlength, or
    // both glengths, are below use8p_size
    const int u = kUse8pSize[d.mismatchtype];
    const int B = (d.rlength < u || (d.glengthL < u && d.glengthR < u)) ? 32 : 16;
    const size_t lds = lds_bytes_uxg(d.rlength, d.glengthL, d.glengthR, B);
    if (lds > 160 * 1024) { c.err = "problem exceeds the LDS of a CU"; return c; }
    c.gdirs = (scratch_bytes_uxg(d.rlength, d.glengthL, d.glengthR, d.lbandL, B) + 255) & ~(size_t)255;
    c.need = gg_lds_bucket(lds);
    c.key = class_key((int)PlanCore::kUxg, B, 0, latency ? 0 : c.need);
    return c;
  }
  if (d.open > 0) { c.err = "positive gap-open penalty is not supported by the scan formulation"; return c; }
  const int WL = d.lbandL + d.ubandL + 1, WR = d.lbandL + d.ubandR + 1;
  const int R = pick_R(std::max(WL, WR));
  if (R > kMaxR) { c.err = "band wider than 4096"; return c; }
  size_t lds = lds_bytes_gg(d.rlength, d.glengthL, d.glengthR, R, true, std::max(WL, WR));
  const bool dirs_lds = lds <= lds_dirs_max;
  if (!dirs_lds) lds = lds_bytes_gg(d.rlength, d.glengthL, d.glengthR, R, false, std::max(WL, WR));
  // bridge candidates (+ direction planes) in global scratch
  c.gdirs = (scratch_bytes_gg(d.rlength, d.glengthL, d.glengthR, R, dirs_lds, std::max(WL, WR)) + 255) & ~(size_t)255;
  if (lds > 160 * 1024) { c.err = "problem exceeds the LDS of a CU"; return c; }
  c.need = gg_lds_bucket(lds);
  c.key = class_key((int)PlanCore::kGenomeGap, R, dirs_lds ? 1 : 0, latency ? 0 : c.need);
  return c;
}

static int classify(gmapdp_ctx* ctx, PlanCore& plan) {
  const size_t lds_dirs_max = gg_lds_dirs_max();  // read once per plan, not per genome-gap problem
  const size_t nd = plan.dev.size(), ng = plan.gdev.size();
  const int T = plan_threads(nd + ng);
  // Latency mode (small batches: the GMAP drop-in's dispatcher batches): one launch class per (kind, R,
  // direction placement) with the LDS of its largest member, and no packed narrow-band kernels, so a
  // batch is a few launches whose latencies do not add up class after class.
  const bool latency = nd + ng <= latency_batch();
  PlanTimer tm("classify");
  // per problem (threads): its class; slots 0..nd-1 single / end gaps, nd.. genome gaps
  HostArray<ClassOf> cls(nd + ng);
  std::vector<size_t> first_err(T, SIZE_MAX);  // per thread chunk: the first problem the engine rejects
  plan_parallel(nd + ng, T, [&](size_t lo, size_t hi, int t) {
    for (size_t s = lo; s < hi; s++) {
      ClassOf& c = cls[s];
      if (s < nd) {
        c = classify_dev(plan.dev[s], latency);
        if (!c.err) class_work(c, plan.dev[s]);
      } else {
        c = classify_gdev(plan.gdev[s - nd], latency, lds_dirs_max);
        if (!c.err) class_work(c, plan.gdev[s - nd]);
      }
      if (c.err && first_err[t] == SIZE_MAX) first_err[t] = s;
    }
  });
  tm.mark("classes");
  for (int t = 0; t < T; t++)  // the first problem in batch order that the engine rejects (chunks in order)
    if (first_err[t] != SIZE_MAX) return bad(ctx, cls[first_err[t]].err);
  // pair-arena and direction-scratch offsets in problem order (single / end gaps, then genome gaps): each
  // thread's chunk totals, then the chunk written from its prefix
  size_t pair_off = 0, gdirs_off = 0;
  {
    std::vector<size_t> tp(T, 0), tg(T, 0);
    plan_parallel(nd + ng, T, [&](size_t lo, size_t hi, int t) {
      size_t a = 0, b = 0;
      for (size_t s = lo; s < hi; s++) {
        a += cls[s].pair;
        b += cls[s].gdirs;
      }
      tp[t] = a;
      tg[t] = b;
    });
    std::vector<size_t> p0(T), g0(T);
    for (int t = 0; t < T; t++) {
      p0[t] = pair_off;
      g0[t] = gdirs_off;
      pair_off += tp[t];
      gdirs_off += tg[t];
    }
    plan_parallel(nd + ng, T, [&](size_t lo, size_t hi, int t) {
      size_t a = p0[t], b = g0[t];
      for (size_t s = lo; s < hi; s++) {
        const ClassOf& c = cls[s];
        if (s < nd) {
          plan.dev[s].pair_offset = (int32_t)a;
          if (c.gdirs) plan.dev[s].dirs_offset = (int64_t)b;
        } else {
          plan.gdev[s - nd].pair_offset = (int32_t)a;
          plan.gdev[s - nd].dirs_offset = (int64_t)b;
        }
        a += c.pair;
        b += c.gdirs;
      }
    });
  }
  tm.mark("offsets");
  // members per class in problem order (the classes in key order, as the tuple map kept them)
  std::vector<uint64_t> keys;
  {
    std::vector<std::vector<uint64_t>> tk(T);
    plan_parallel(nd + ng, T, [&](size_t lo, size_t hi, int t) {
      uint64_t last = ~0ull;
      for (size_t s = lo; s < hi; s++)
        if (cls[s].key != last) {
          last = cls[s].key;
          if (std::find(tk[t].begin(), tk[t].end(), last) == tk[t].end()) tk[t].push_back(last);
        }
    });
    for (auto& v : tk) keys.insert(keys.end(), v.begin(), v.end());
    std::sort(keys.begin(), keys.end());
    keys.erase(std::unique(keys.begin(), keys.end()), keys.end());
  }
  const size_t K = keys.size();
  auto class_index = [&](uint64_t k) { return (size_t)(std::lower_bound(keys.begin(), keys.end(), k) - keys.begin()); };
  // One pass (threads over contiguous chunks of problems): each problem's class, its bin -- the class and its
  // length quantised to 16 steps per doubling, longest first (plan_bucket: the launch order only steers the
  // tail of a launch) -- and the classes' work estimates (sums and maxima need no order); then the bins'
  // offsets (class-major; dev and genome classes into their own order arrays); then every problem scattered
  // to its slot (in problem order within a bin).  A comparison sort reading two random descriptors per
  // comparison spent most of a 10 000-read plan on cache misses.
  constexpr int NB = 1024;
  struct Acc {
    double work = 0.0, span = 0.0;
    int gm = 0;
    size_t need = 0;
  };
  std::vector<std::vector<uint32_t>> hist(T, std::vector<uint32_t>(K * NB, 0));
  std::vector<std::vector<Acc>> acc(T, std::vector<Acc>(K));
  HostArray<uint32_t> bin(nd + ng);
  plan_parallel(nd + ng, T, [&](size_t lo, size_t hi, int t) {
    std::vector<uint32_t>& h = hist[t];
    std::vector<Acc>& A = acc[t];
    size_t k = 0;
    uint64_t kk = ~0ull;
    for (size_t s = lo; s < hi; s++) {
      const ClassOf& c = cls[s];
      if (c.key != kk) {  // (runs of one class are common: a lookup per run)
        kk = c.key;
        k = class_index(kk);
      }
      const int kind = (int)(kk >> 48), R = (int)((kk >> 32) & 0xFFFF);
      const double one = c.one;
      const int gm = c.gm;
      const uint32_t bn = (uint32_t)(k * NB + (NB - 1 - plan_bucket(c.len)));
      bin[s] = bn;
      h[bn]++;
      Acc& a = A[k];
      a.work += one;
      // a packed wave's problems fill side by side: its latency is one problem's columns
      a.span = std::max(a.span, (kind == PlanCore::kDpx || kind == PlanCore::kSx) ? one * 64.0 / R : one);
      a.gm = std::max(a.gm, gm);
      a.need = std::max(a.need, cls[s].need);
    }
  });
  std::vector<std::vector<uint32_t>> at(T, std::vector<uint32_t>(K * NB));
  std::vector<size_t> first(K), count(K);
  {
    size_t run[2] = {0, 0};  // dev order, genome order
    for (size_t k = 0; k < K; k++) {
      const int kind = (int)(keys[k] >> 48);
      const int g = kind == PlanCore::kGenomeGap || kind == PlanCore::kUxg ? 1 : 0;
      first[k] = run[g];
      for (int b = 0; b < NB; b++)
        for (int t = 0; t < T; t++) {
          at[t][k * NB + b] = (uint32_t)run[g];
          run[g] += hist[t][k * NB + b];
        }
      count[k] = run[g] - first[k];
    }
    plan.order.resize(run[0]);
    plan.gorder.resize(run[1]);
  }
  plan_parallel(nd + ng, T, [&](size_t lo, size_t hi, int t) {
    std::vector<uint32_t>& a = at[t];
    for (size_t s = lo; s < hi; s++) {
      if (s < nd) plan.order[a[bin[s]]++] = (int)s;
      else plan.gorder[a[bin[s]]++] = (int)(s - nd);
    }
  });
  tm.mark("members");
  for (size_t k = 0; k < K; k++) {
    PlanCore::Launch L;
    const uint64_t key = keys[k];
    L.kind = (int)(key >> 48);
    L.R = (int)((key >> 32) & 0xFFFF);
    L.dirs_lds = ((key >> 31) & 1) != 0;
    L.lds = (size_t)(key & 0x7FFFFFFFull);
    L.count = (int)count[k];
    L.first = (int)first[k];
    Acc a;
    for (int t = 0; t < T; t++) {
      const Acc& x = acc[t][k];
      a.work += x.work;
      a.span = std::max(a.span, x.span);
      a.gm = std::max(a.gm, x.gm);
      a.need = std::max(a.need, x.need);
    }
    if (latency) L.lds = a.need;  // the class's LDS: its largest member's
    L.work = a.work;
    L.span = a.span;
    L.extra = 0;
    L.gdirs_offset = 0;
    if (L.kind == PlanCore::kSx) {  // per wave: 4 direction words per fill step (gm: the largest step count)
      L.extra = (size_t)a.gm * 32u;
      L.dirs_lds = false;
      L.gdirs_offset = gdirs_off;
      const size_t nblocks = ((size_t)L.count + (64 / L.R) - 1) / (64 / L.R);
      gdirs_off += (nblocks * L.extra + 255) & ~(size_t)255;
    }
    if (L.kind == PlanCore::kDpx) {
      L.extra = lds_dirs_dpx(a.gm);
      // direction words in LDS while the workgroup stays small; beyond that they go to an
      // L2-resident scratch so that more problems are resident per CU
      L.dirs_lds = L.extra + L.lds * (64 / L.R) <= dpx_lds_dirs_max();
      if (!L.dirs_lds) {
        L.gdirs_offset = gdirs_off;
        const size_t nblocks = ((size_t)L.count + (64 / L.R) - 1) / (64 / L.R);
        gdirs_off += (nblocks * L.extra + 255) & ~(size_t)255;
      }
    }
    L.stream = 0;
    plan.launches.push_back(L);
  }
  tm.mark("launches");
  // Independent classes share the GPU: longest-processing-time-first over the caller's stream and
  // the three side streams, so that LDS-heavy and LDS-light classes are co-resident on the CUs and
  // no launch's drain leaves the chip idle.  Launches are then kept in issue order (per stream,
  // largest first).
  {
    std::vector<int> idx(plan.launches.size());
    for (size_t i = 0; i < idx.size(); i++) idx[i] = (int)i;
    std::stable_sort(idx.begin(), idx.end(),
                     [&](int a, int b) { return plan.launches[a].work > plan.launches[b].work; });
    double load[1 + gmapdp_ctx::kAux] = {0.0, 0.0, 0.0, 0.0};
    for (int i : idx) {
      int best = 0;
      for (int k = 1; k <= ctx->plan_sides; k++)
        if (load[k] < load[best]) best = k;
      plan.launches[i].stream = best;
      load[best] += plan.launches[i].work;
    }
    // per stream, the classes with the longest single problems go first: they set the step's
    // critical path, so they start at the fork instead of after the bulk classes
    std::vector<int> byspan(idx);
    std::stable_sort(byspan.begin(), byspan.end(),
                     [&](int a, int b) { return plan.launches[a].span > plan.launches[b].span; });
    std::vector<PlanCore::Launch> sorted;
    for (int k = 0; k <= gmapdp_ctx::kAux; k++)
      for (int i : byspan)
        if (plan.launches[i].stream == k) sorted.push_back(plan.launches[i]);
    plan.launches.swap(sorted);
  }
  plan.pair_capacity = pair_off;
  plan.gdirs_bytes = gdirs_off;
  tm.mark("lpt");
  return GMAPDP_OK;
}

// Results: singles first, then ends (host_results); genome-gap results separately.  The per-problem
// prologues (penalties, size guards, bands, segment bounds) run on plan_threads() host threads; the GPU
// problems are then compacted in problem order.
static int build_plan(gmapdp_ctx* ctx, const gmapdp_single_problem* singles, int nsingle,
                      const gmapdp_end_problem* ends, int nend, const gmapdp_genome_problem* genomes, int ngenome,
                      gmapdp_result* results, gmapdp_genome_result* gresults, PlanCore& plan) {
  plan = PlanCore();
  PlanTimer tm("build_plan");
  const int n = nsingle + nend;
  const int T = plan_threads((size_t)n + (size_t)ngenome);
  std::vector<const char*> why(2 * T, nullptr);
  std::vector<int> errat(2 * T, INT32_MAX), errcode(2 * T, 0);
  // single and end gaps, then genome gaps: each descriptor converted once into a problem-order array
  // (threads), the GPU problems' slots by a prefix count, then moved into their slots (threads; the array
  // itself when every problem runs on the GPU)
  auto compact = [&](int m, int err_base, auto&& conv, auto& dev, auto& dev_index, auto& dev_problem) -> int {
    using D = typename std::decay_t<decltype(dev)>::value_type;
    std::vector<size_t> cnt(T, 0);
    HostArray<unsigned char> gpu(m);
    HostArray<D> tmp(m);
    plan_parallel((size_t)m, T, [&](size_t lo, size_t hi, int t) {
      size_t c = 0;
      for (size_t i = lo; i < hi; i++) {
        int err = 0;
        const char* w = nullptr;
        const int g = conv(i, &err, &w, &tmp[i]);
        if (err) {
          errat[err_base + t] = (int)i;
          errcode[err_base + t] = err;
          why[err_base + t] = w;
          return;
        }
        gpu[i] = (unsigned char)g;
        c += (size_t)g;
      }
      cnt[t] = c;
    });
    for (int t = 0; t < T; t++)
      if (errat[err_base + t] != INT32_MAX) return why[err_base + t] ? bad(ctx, why[err_base + t]) : errcode[err_base + t];
    std::vector<size_t> at(T);
    size_t total = 0;
    for (int t = 0; t < T; t++) {
      at[t] = total;
      total += cnt[t];
    }
    dev_index.resize(m);
    dev_problem.resize(total);
    if (total == (size_t)m) {
      dev.swap(tmp);
      plan_parallel((size_t)m, T, [&](size_t lo, size_t hi, int) {
        for (size_t i = lo; i < hi; i++) dev_index[i] = dev_problem[i] = (int)i;
      });
      return GMAPDP_OK;
    }
    dev.resize(total);
    plan_parallel((size_t)m, T, [&](size_t lo, size_t hi, int t) {
      size_t k = at[t];
      for (size_t i = lo; i < hi; i++) {
        if (!gpu[i]) {
          dev_index[i] = -1;
          continue;
        }
        dev[k] = tmp[i];
        dev_index[i] = (int)k;
        dev_problem[k++] = (int)i;
      }
    });
    return GMAPDP_OK;
  };
  int rc = compact(
      n, 0,
      [&](size_t i, int* err, const char** w, DevProblem* out) {
        DevProblem scratch;
        DevProblem& d = out ? *out : scratch;
        const int g = (int)i < nsingle ? convert_single(ctx, singles[i], results[i], d)
                                       : convert_end(ctx, ends[i - nsingle], results[i], d, err, w);
        results[i].pair_offset = 0;
        return g;
      },
      plan.dev, plan.dev_index, plan.dev_problem);
  if (rc) return rc;
  rc = compact(
      ngenome, T,
      [&](size_t j, int* err, const char** w, DevGenomeProblem* out) {
        DevGenomeProblem scratch;
        return convert_genome(ctx, genomes[j], gresults[j], out ? *out : scratch, err, w);
      },
      plan.gdev, plan.gdev_index, plan.gdev_problem);
  if (rc) return rc;
  tm.mark("convert");
  rc = classify(ctx, plan);
  if (rc) return rc;
  tm.mark("classify");
  plan_parallel(plan.dev.size() + plan.gdev.size(), T, [&](size_t lo, size_t hi, int) {
    for (size_t s = lo; s < hi; s++) {
      if (s < plan.dev.size()) results[plan.dev_problem[s]].pair_offset = plan.dev[s].pair_offset;
      else gresults[plan.gdev_problem[s - plan.dev.size()]].pair_offset = plan.gdev[s - plan.dev.size()].pair_offset;
    }
  });
  return GMAPDP_OK;
}

// Launches assigned to a side stream run concurrently with those on the caller's stream.
static bool launch_is_tail(const PlanCore::Launch& L) { return L.stream != 0; }

// Device-side inputs of one plan execution.
struct RunArgs {
  const DevProblem* d_probs;
  const int* d_order;
  const DevGenomeProblem* d_gprobs;
  const int* d_gorder;
  const char* d_q;
  const char* d_quc;
  const double* d_sprob;
  gmapdp_result* d_results;
  gmapdp_genome_result* d_gresults;
  gmapdp_pair* d_pairs;
  const uint8_t* d_known = nullptr;  // known-site arena (GMAPDP_KNOWN_SITES genome gaps)
  // device MaxEnt: each genome-gap class first fills its problems' entries of d_sprob (me_gap_kernel)
  const double* d_metab = nullptr;
};

// me_gap_kernel over a genome-gap launch class's problems, on the class's stream
static hipError_t launch_class_maxent(gmapdp_ctx* ctx, const PlanCore::Launch& L, const RunArgs& a, hipStream_t s) {
  if (!a.d_metab) return hipSuccess;
  return launch_me_gap(L.count, s, a.d_gprobs, a.d_gorder + L.first, ctx->d_genome, ctx->genome_words, a.d_metab,
                       const_cast<double*>(a.d_sprob));
}

// prologue = false: the launch's kernel alone (the MaxEnt prologue of a genome-gap class is skipped; the
// probabilities a previous full run computed stay in the arena)
static hipError_t launch_one(gmapdp_ctx* ctx, const PlanCore& plan, int li, const RunArgs& a, hipStream_t stream,
                             bool prologue = true) {
  const auto& L = plan.launches[li];
  if (L.kind == PlanCore::kUxe)
    return launch_uxe(L.R, L.count, L.lds, stream, a.d_probs, a.d_order + L.first, (unsigned char*)ctx->gdirs.p,
                      ctx->d_genome, ctx->genome_words, a.d_q, a.d_quc, ctx->d_sc, ctx->d_cs, a.d_results,
                      a.d_pairs);
  if (L.kind == PlanCore::kUxg) {
    if (!a.d_gresults || !a.d_sprob) return hipErrorInvalidValue;
    const hipError_t e = prologue ? launch_class_maxent(ctx, L, a, stream) : hipSuccess;
    if (e != hipSuccess) return e;
    return launch_uxg(L.R, L.count, L.lds, stream, a.d_gprobs, a.d_gorder + L.first, (unsigned char*)ctx->gdirs.p,
                      ctx->d_genome, ctx->genome_words, a.d_q, a.d_quc, a.d_sprob, ctx->d_sc, ctx->d_cs, ctx->d_isc,
                      a.d_gresults, a.d_pairs, a.d_known);
  }
  if (L.kind == PlanCore::kSx)
    return launch_sx(L.R, L.count, (int)L.lds, (long long)L.extra, (unsigned char*)ctx->gdirs.p + L.gdirs_offset,
                     stream, a.d_probs, a.d_order + L.first, ctx->d_genome, ctx->genome_words, a.d_q, a.d_quc,
                     ctx->d_sc, ctx->d_cs, a.d_results, a.d_pairs);
  if (L.kind == PlanCore::kDpx)
    return launch_dpx(L.R, L.count, (int)L.lds, (int)L.extra,
                      L.dirs_lds ? nullptr : (unsigned char*)ctx->gdirs.p + L.gdirs_offset, stream, a.d_probs,
                      a.d_order + L.first, ctx->d_genome, ctx->genome_words, a.d_q, a.d_quc, ctx->d_sc, ctx->d_cs,
                      a.d_results, a.d_pairs);
  if (L.kind == PlanCore::kDp || L.kind == PlanCore::kDpRows)
    return launch_dp(L.R, L.dirs_lds, L.kind == PlanCore::kDpRows, L.count, L.lds, stream, a.d_probs,
                     a.d_order + L.first, ctx->d_genome,
                     ctx->genome_words, a.d_q, a.d_quc, ctx->d_sc, ctx->d_cs, a.d_results, a.d_pairs,
                     (uint64_t*)ctx->gdirs.p);
  if (!a.d_gresults || !a.d_sprob) return hipErrorInvalidValue;
  // device MaxEnt: gg_kernel evaluates the models while it stages the segments (no me_gap_kernel prologue,
  // no probability arena written and read back); host probabilities: read from d_sprob
  return launch_gg(L.R, L.dirs_lds, L.count, L.lds, stream, a.d_gprobs, a.d_gorder + L.first, ctx->d_genome,
                   ctx->genome_words, a.d_q, a.d_quc, a.d_metab ? nullptr : a.d_sprob, ctx->d_sc, ctx->d_cs,
                   ctx->d_isc, a.d_gresults, a.d_pairs, (unsigned char*)ctx->gdirs.p, a.d_known, a.d_metab);
}

static int run_plan(gmapdp_ctx* ctx, const PlanCore& plan, const RunArgs& a, hipStream_t stream) {
  if (plan.gdirs_bytes) {
    hipError_t e = ctx->gdirs.ensure(plan.gdirs_bytes);
    if (e != hipSuccess) return fail(ctx, GMAPDP_ENOMEM, "direction scratch: %s", e);
  }
  // Fork: the side streams wait for everything already queued on `stream`; each launch goes to
  // its assigned stream; join: `stream` waits for the side streams.  A small batch (the drop-in's
  // dispatcher batches) runs on `stream` alone: a process has few hardware queues (GPU_MAX_HW_QUEUES)
  // and several dispatcher contexts share them.
  // (GMAPDP_SMALL_BATCH_STREAMS=1, experiments: small batches spread over the side streams too)
  static const bool small_streams = getenv("GMAPDP_SMALL_BATCH_STREAMS") != nullptr;
  const bool one_stream = ctx->one_stream || (!small_streams && plan.dev.size() + plan.gdev.size() < 2048);
  hipError_t e = one_stream ? hipSuccess : hipEventRecord(ctx->ev_fork, stream);
  bool used[gmapdp_ctx::kAux] = {false, false, false};
  for (size_t li = 0; li < plan.launches.size() && e == hipSuccess; li++) {
    const int k = one_stream ? 0 : plan.launches[li].stream;
    hipStream_t s = stream;
    if (k > 0) {
      s = ctx->aux[k - 1];
      if (!used[k - 1]) e = hipStreamWaitEvent(s, ctx->ev_fork, 0);
      used[k - 1] = true;
    }
    if (e == hipSuccess) e = launch_one(ctx, plan, (int)li, a, s);
  }
  for (int i = 0; i < gmapdp_ctx::kAux && e == hipSuccess; i++) {
    if (!used[i]) continue;
    e = hipEventRecord(ctx->ev_join[i], ctx->aux[i]);
    if (e == hipSuccess) e = hipStreamWaitEvent(stream, ctx->ev_join[i], 0);
  }
  if (e != hipSuccess) return fail(ctx, GMAPDP_ELAUNCH, "dp launch: %s", e);
  return GMAPDP_OK;
}

// Synchronous host-array batch (all entry-point families).
static int run_batch(gmapdp_ctx* ctx, const gmapdp_single_problem* singles, int nsingle,
                     const gmapdp_end_problem* ends, int nend, const gmapdp_genome_problem* genomes, int ngenome,
                     const char* qseq, const char* qseq_uc, size_t qbytes, const double* sprob, size_t nsprob,
                     gmapdp_result* results, gmapdp_genome_result* gresults, gmapdp_pair* pairs,
                     size_t pair_capacity, const uint8_t* known = nullptr, size_t nknown = 0) {
  const int n = nsingle + nend;
  if (!ctx || n < 0 || ngenome < 0 || (n && !results) || (ngenome && !gresults)) return GMAPDP_EINVAL;
  if (!ctx->d_genome) return GMAPDP_ENOGENOME;
  if (n + ngenome == 0) return GMAPDP_OK;
  (void)hipSetDevice(ctx->device);
  PlanCore plan;
  int rc = build_plan(ctx, singles, nsingle, ends, nend, genomes, ngenome, results, gresults, plan);
  if (rc) return rc;
  if (plan.pair_capacity > pair_capacity) return bad(ctx, "pair arena too small");
  for (size_t s = 0; s < plan.dev.size(); s++) {
    const int i = plan.dev_problem[s];
    const long lo = i < nsingle ? singles[i].qoff : ends[i - nsingle].qoff;
    const long len = i < nsingle ? singles[i].rlength : ends[i - nsingle].rlength;
    if (lo < 0 || (size_t)(lo + len) > qbytes) return bad(ctx, "query slice outside the query arena");
  }
  // splice_probs == NULL: the probability entries are evaluated on the device (me_gap_kernel)
  const bool dev_me = !sprob && !plan.gdev.empty();
  const double* metab = nullptr;
  if (dev_me) {
    nsprob = std::max(nsprob, gmapdp_genome_prob_entries(genomes, ngenome));
    if (!(metab = me_tables(ctx))) return GMAPDP_EINVAL;
  }
  for (size_t s = 0; s < plan.gdev.size(); s++) {
    const gmapdp_genome_problem& g = genomes[plan.gdev_problem[s]];
    if (g.qoff < 0 || (size_t)((long)g.qoff + g.rlength) > qbytes)
      return bad(ctx, "query slice outside the query arena");
    if (g.prob_offset < 0 || (size_t)g.prob_offset + (size_t)g.glengthL + (size_t)g.glengthR > nsprob)
      return bad(ctx, "splice probabilities outside the probability arena");
    if ((g.flags & GMAPDP_KNOWN_SITES) &&
        (!known || (size_t)g.known_offset + gmapdp_genome_known_bytes(&g) > nknown))
      return bad(ctx, "known-site flags outside the known-site arena");
  }
  const int ndev = (int)plan.dev.size(), ngdev = (int)plan.gdev.size();
  if (ndev + ngdev == 0) return GMAPDP_OK;
  const size_t nkn = (ngdev && known) ? nknown : 0;
  // one pinned image of every input and one of every output: a single copy each way
  auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
  const size_t o_probs = 0;
  const size_t o_order = o_probs + al(sizeof(DevProblem) * ndev);
  const size_t o_gprobs = o_order + al(sizeof(int) * ndev);
  const size_t o_gorder = o_gprobs + al(sizeof(DevGenomeProblem) * ngdev);
  const size_t o_sprob = o_gorder + al(sizeof(int) * ngdev);
  const size_t o_q = o_sprob + al(ngdev && !dev_me ? sizeof(double) * nsprob : 0);
  const size_t o_quc = o_q + al(qbytes);
  const size_t o_known = o_quc + al(qbytes);
  const size_t in_bytes = o_known + al(nkn);
  const size_t r_res = 0;
  const size_t r_gres = r_res + al(sizeof(gmapdp_result) * ndev);
  const size_t r_pairs = r_gres + al(sizeof(gmapdp_genome_result) * ngdev);
  const size_t out_bytes = r_pairs + al(sizeof(gmapdp_pair) * plan.pair_capacity);
  hipError_t e = ctx->hin.ensure(in_bytes);
  if (e == hipSuccess) e = ctx->din.ensure(in_bytes);
  if (e == hipSuccess) e = ctx->hout.ensure(out_bytes);
  if (e == hipSuccess) e = ctx->dout.ensure(out_bytes);
  if (e == hipSuccess && dev_me) e = ctx->sprob.ensure(sizeof(double) * nsprob);
  if (e != hipSuccess) return fail(ctx, GMAPDP_ENOMEM, "batch buffers: %s", e);
  unsigned char* hin = (unsigned char*)ctx->hin.p;
  unsigned char* din = (unsigned char*)ctx->din.p;
  unsigned char* hout = (unsigned char*)ctx->hout.p;
  unsigned char* dout = (unsigned char*)ctx->dout.p;
  if (ndev) {
    std::memcpy(hin + o_probs, plan.dev.data(), sizeof(DevProblem) * ndev);
    std::memcpy(hin + o_order, plan.order.data(), sizeof(int) * ndev);
  }
  if (ngdev) {
    std::memcpy(hin + o_gprobs, plan.gdev.data(), sizeof(DevGenomeProblem) * ngdev);
    std::memcpy(hin + o_gorder, plan.gorder.data(), sizeof(int) * ngdev);
    if (!dev_me) std::memcpy(hin + o_sprob, sprob, sizeof(double) * nsprob);
    if (nkn) std::memcpy(hin + o_known, known, nkn);
  }
  std::memcpy(hin + o_q, qseq, qbytes);
  std::memcpy(hin + o_quc, qseq_uc, qbytes);
  hipStream_t s = ctx->stream;
  e = hipMemcpyAsync(din, hin, in_bytes, hipMemcpyHostToDevice, s);
  if (e != hipSuccess) return fail(ctx, GMAPDP_ENOMEM, "upload: %s", e);
  RunArgs a;
  a.d_probs = (const DevProblem*)(din + o_probs);
  a.d_order = (const int*)(din + o_order);
  a.d_gprobs = (const DevGenomeProblem*)(din + o_gprobs);
  a.d_gorder = (const int*)(din + o_gorder);
  a.d_q = (const char*)(din + o_q);
  a.d_quc = (const char*)(din + o_quc);
  a.d_sprob = dev_me ? (const double*)ctx->sprob.p : (const double*)(din + o_sprob);
  a.d_metab = metab;
  a.d_results = (gmapdp_result*)(dout + r_res);
  a.d_gresults = (gmapdp_genome_result*)(dout + r_gres);
  a.d_pairs = (gmapdp_pair*)(dout + r_pairs);
  a.d_known = nkn ? (const uint8_t*)(din + o_known) : nullptr;
  rc = run_plan(ctx, plan, a, s);
  if (rc) return rc;
  e = hipMemcpyAsync(hout, dout, out_bytes, hipMemcpyDeviceToHost, s);
  if (e == hipSuccess) e = ctx_sync(ctx, s);
  if (e != hipSuccess) return fail(ctx, GMAPDP_ELAUNCH, "dp execution: %s", e);
  const gmapdp_result* dres = (const gmapdp_result*)(hout + r_res);
  const gmapdp_genome_result* gres = (const gmapdp_genome_result*)(hout + r_gres);
  if (pairs && plan.pair_capacity) std::memcpy(pairs, hout + r_pairs, sizeof(gmapdp_pair) * plan.pair_capacity);
  for (int d = 0; d < ndev; d++) results[plan.dev_problem[d]] = dres[d];
  for (int d = 0; d < ngdev; d++) gresults[plan.gdev_problem[d]] = gres[d];
  return GMAPDP_OK;
}

static size_t capacity(const gmapdp_single_problem* singles, int nsingle, const gmapdp_end_problem* ends, int nend) {
  size_t cap = 0;
  for (int i = 0; i < nsingle; i++)
    if (singles[i].rlength > 0 && singles[i].glength > 0 && singles[i].rlength <= GMAPDP_MAX_RLENGTH &&
        singles[i].glength <= GMAPDP_MAX_GLENGTH)
      cap += (size_t)singles[i].rlength + singles[i].glength + 2;
  for (int i = 0; i < nend; i++) {
    const bool nog = ends[i].endalign == kQueryendNogaps;
    const int r = nog ? ends[i].rlength : std::min(ends[i].rlength, GMAPDP_MAX_RLENGTH);
    const int g = nog ? ends[i].glength : std::min(ends[i].glength, GMAPDP_MAX_GLENGTH);
    if (r > 0 && g > 0) cap += (size_t)r + g + 2;
  }
  return cap;
}

extern "C" {

size_t gmapdp_single_pair_capacity(const gmapdp_single_problem* problems, int n) {
  return capacity(problems, n, nullptr, 0);
}
size_t gmapdp_end_pair_capacity(const gmapdp_end_problem* problems, int n) {
  return capacity(nullptr, 0, problems, n);
}
size_t gmapdp_genome_pair_capacity(const gmapdp_genome_problem* problems, int n) {
  size_t cap = 0;
  for (int i = 0; i < n; i++) {
    const gmapdp_genome_problem& p = problems[i];
    if (p.rlength > 1 && p.rlength <= GMAPDP_MAX_RLENGTH && p.glengthL <= GMAPDP_MAX_GLENGTH &&
        p.glengthR <= GMAPDP_MAX_GLENGTH && p.glengthL > 0 && p.glengthR > 0)
      cap += 2 * (size_t)p.rlength + (size_t)p.glengthL + (size_t)p.glengthR + 4;
  }
  return cap;
}

size_t gmapdp_genome_prob_entries(const gmapdp_genome_problem* problems, int n) {
  size_t m = 0;
  for (int i = 0; i < n; i++) {
    const gmapdp_genome_problem& p = problems[i];
    if (p.prob_offset < 0 || p.glengthL < 0 || p.glengthR < 0) continue;
    m = std::max(m, (size_t)p.prob_offset + (size_t)p.glengthL + (size_t)p.glengthR);
  }
  return m;
}

// The Maxent_hr_*_prob call of each probability entry (bridge_intron_gap_site_level,
// dynprog_genome.c:2573-2660; get_splicesite_probs :332-401).  Positions are 64-bit universal
// coordinates (gmapdp_coord_t), as gmapl's Univcoord_T.
int gmapdp_genome_splice_sites(const gmapdp_genome_problem* problems, int n, gmapdp_coord_t* positions, uint8_t* models,
                               size_t nentries) {
  if (n < 0 || (n && (!problems || !positions || !models))) return GMAPDP_EINVAL;
  if (gmapdp_genome_prob_entries(problems, n) > nentries) return GMAPDP_EINVAL;
  for (int i = 0; i < n; i++) {
    const gmapdp_genome_problem& p = problems[i];
    if (p.prob_offset < 0 || p.glengthL < 0 || p.glengthR < 0) return GMAPDP_EINVAL;
    const bool watson = p.flags & GMAPDP_WATSON;
    const bool sense = p.cdna_direction > 0;
    const uint64_t lo = (uint64_t)(int64_t)p.goffsetL, ro = (uint64_t)(int64_t)p.rev_goffsetR;
    gmapdp_coord_t* pos = positions + p.prob_offset;
    uint8_t* mod = models + p.prob_offset;
    for (int c = 0; c < p.glengthL; c++) {
      if (watson) {
        pos[c] = p.chroffset + lo + (uint64_t)c;
        mod[c] = sense ? GMAPDP_MAXENT_DONOR : GMAPDP_MAXENT_ANTIACCEPTOR;
      } else {
        pos[c] = p.chrhigh - lo - (uint64_t)c + 1u;
        mod[c] = sense ? GMAPDP_MAXENT_ANTIDONOR : GMAPDP_MAXENT_ACCEPTOR;
      }
    }
    pos += p.glengthL;
    mod += p.glengthL;
    for (int c = 0; c < p.glengthR; c++) {
      if (watson) {
        pos[c] = p.chroffset + ro - (uint64_t)c + 1u;
        mod[c] = sense ? GMAPDP_MAXENT_ACCEPTOR : GMAPDP_MAXENT_ANTIDONOR;
      } else {
        pos[c] = p.chrhigh - ro + (uint64_t)c;
        mod[c] = sense ? GMAPDP_MAXENT_ANTIACCEPTOR : GMAPDP_MAXENT_DONOR;
      }
    }
  }
  return GMAPDP_OK;
}

int gmapdp_single_gap_batch(gmapdp_ctx* ctx, const gmapdp_single_problem* problems, int n, const char* qseq,
                            const char* qseq_uc, size_t qbytes, gmapdp_result* results, gmapdp_pair* pairs,
                            size_t pair_capacity) {
  if (n > 0 && !problems) return GMAPDP_EINVAL;
  return run_batch(ctx, problems, n, nullptr, 0, nullptr, 0, qseq, qseq_uc, qbytes, nullptr, 0, results, nullptr,
                   pairs, pair_capacity);
}

int gmapdp_end_gap_batch(gmapdp_ctx* ctx, const gmapdp_end_problem* problems, int n, const char* qseq,
                         const char* qseq_uc, size_t qbytes, gmapdp_result* results, gmapdp_pair* pairs,
                         size_t pair_capacity) {
  if (n > 0 && !problems) return GMAPDP_EINVAL;
  return run_batch(ctx, nullptr, 0, problems, n, nullptr, 0, qseq, qseq_uc, qbytes, nullptr, 0, results, nullptr,
                   pairs, pair_capacity);
}

int gmapdp_genome_gap_batch(gmapdp_ctx* ctx, const gmapdp_genome_problem* problems, int n, const char* qseq,
                            const char* qseq_uc, size_t qbytes, const double* splice_probs, size_t nprobs,
                            gmapdp_genome_result* results, gmapdp_pair* pairs, size_t pair_capacity) {
  if (n > 0 && !problems) return GMAPDP_EINVAL;
  return run_batch(ctx, nullptr, 0, nullptr, 0, problems, n, qseq, qseq_uc, qbytes, splice_probs, nprobs, nullptr,
                   results, pairs, pair_capacity);
}

int gmapdp_genome_gap_batch_known(gmapdp_ctx* ctx, const gmapdp_genome_problem* problems, int n, const char* qseq,
                                  const char* qseq_uc, size_t qbytes, const double* splice_probs, size_t nprobs,
                                  const uint8_t* known_sites, size_t nknown, gmapdp_genome_result* results,
                                  gmapdp_pair* pairs, size_t pair_capacity) {
  if (n > 0 && !problems) return GMAPDP_EINVAL;
  return run_batch(ctx, nullptr, 0, nullptr, 0, problems, n, qseq, qseq_uc, qbytes, splice_probs, nprobs, nullptr,
                   results, pairs, pair_capacity, known_sites, nknown);
}

size_t gmapdp_genome_known_bytes(const gmapdp_genome_problem* p) {
  return (size_t)std::max(p->glengthL, 0) + (size_t)std::max(p->glengthR, 0) + 2 * (size_t)(std::max(p->rlength, 0) + 1);
}

int gmapdp_dynprog_batch(gmapdp_ctx* ctx, const gmapdp_single_problem* singles, int nsingle,
                         const gmapdp_end_problem* ends, int nend, const gmapdp_genome_problem* genomes, int ngenome,
                         const char* qseq, const char* qseq_uc, size_t qbytes, const double* splice_probs,
                         size_t nprobs, gmapdp_result* results, gmapdp_genome_result* genome_results,
                         gmapdp_pair* pairs, size_t pair_capacity) {
  if ((nsingle > 0 && !singles) || (nend > 0 && !ends) || (ngenome > 0 && !genomes)) return GMAPDP_EINVAL;
  return run_batch(ctx, singles, nsingle, ends, nend, genomes, ngenome, qseq, qseq_uc, qbytes, splice_probs, nprobs,
                   results, genome_results, pairs, pair_capacity);
}

}  // extern "C"

// ---------------------------------------------------------------------------
// Dynprog_cdna_gap (dynprog_cdna.c:787).  Rare in GMAP's pipeline, so it has its
// own synchronous batch path: the prologue on the host, one launch per (semantics, R or B) class.
// ---------------------------------------------------------------------------
static const int kInsertPairsHost = 9;  // INSERT_PAIRS (dynprog_cdna.c:40)
static size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

static bool cdna_on_host(const gmapdp_cdna_problem& p) {
  return p.glength <= 1 || p.glength > GMAPDP_MAX_GLENGTH || p.rlengthL > GMAPDP_MAX_RLENGTH ||
         p.rlengthR > GMAPDP_MAX_RLENGTH;
}

// Dynprog_cdna_gap prologue (:830-940): returns 1 if the problem runs on the GPU.
static int convert_cdna(gmapdp_ctx* ctx, const gmapdp_cdna_problem& p, size_t qbytes, gmapdp_cdna_result& res,
                        DevCdnaProblem& d, int* err) {
  *err = 0;
  std::memset(&res, 0, sizeof(res));
  res.traceback_score = GMAPDP_UNSET;
  res.dynprogindex = p.dynprogindex;
  res.gap_index = -1;
  if (p.glength <= 1) return 0;  // :830, dynprogindex unchanged
  if (cdna_on_host(p)) {         // size guard (:869-893)
    res.dynprogindex = next_dpi(p.dynprogindex);
    return 0;
  }
  if (p.rlengthL != p.rlengthR || p.rlengthL < p.glength) {
    *err = bad(ctx, "Dynprog_cdna_gap needs rlengthL == rlengthR >= glength (the reference's bridge reads "
                    "cells no fill wrote otherwise)");
    return 0;
  }
  if (p.extraband < 0) {
    *err = bad(ctx, "negative extraband_paired");
    return 0;
  }
  const long span = std::max<long>(p.rlengthL, (long)p.rev_roffsetR - p.roffsetL + 1);
  if (p.qoffL < 0 || p.qoffR - p.rlengthR + 1 < 0 || (size_t)(p.qoffL + span) > qbytes ||
      (size_t)p.qoffR >= qbytes) {
    *err = bad(ctx, "query pieces outside the query arena");
    return 0;
  }
  std::memset(&d, 0, sizeof(d));
  const double dr = p.defect_rate;
  d.mismatchtype = dr < 0.003 ? kHighQ : (dr < 0.014 ? kMedQ : kLowQ);
  d.open = -10;  // CDNA_OPEN_* / CDNA_EXTEND_* (:32-38), for every defect rate
  d.extend = -7;
  d.qbaseL = p.qoffL;
  d.qbaseR = p.qoffR;
  d.rlength = p.rlengthL;
  d.glength = p.glength;
  d.roffsetL = p.roffsetL;
  d.rev_roffsetR = p.rev_roffsetR;
  d.goffset = p.goffset;
  d.chroffset = p.chroffset;
  d.chrhigh = p.chrhigh;
  // Dynprog_compute_bands(widebandp) with glength <= rlength; equal to bridge_cdna_gap's own bands
  d.lband = p.rlengthL - p.glength + p.extraband;
  d.uband = p.extraband;
  const bool watson = p.flags & GMAPDP_WATSON;
  const uint32_t rev_goffset = (uint32_t)(p.goffset + p.glength - 1);
  d.flags = (watson ? kFWatson : 0) | ((p.flags & GMAPDP_JUMP_LATE) ? kFLate : 0) |
            ((p.flags & GMAPDP_SIMD) ? kCSimd : 0);
  if (watson) {  // :922-926
    d.segpos = p.chroffset + (uint64_t)(int64_t)p.goffset;  // Genome_get_segment_right(left, chrhigh)
    d.segbound = p.chrhigh;
    d.rsegpos = p.chroffset + rev_goffset + 1u;    // Genome_get_segment_left(right, chroffset)
    d.rsegbound = p.chroffset;
    d.flags |= kCRSegLeft;
  } else {       // :928-931
    d.rsegpos = p.chrhigh - rev_goffset;           // _right(left, chrhigh), revcomp
    d.rsegbound = p.chrhigh;
    d.segpos = p.chrhigh - (uint64_t)(int64_t)p.goffset + 1u;  // _left(right, chroffset), revcomp
    d.segbound = p.chroffset;
    d.flags |= kCSegLeft | kCSegRc | kCRSegRc;
  }
  d.genestrand = p.genestrand;
  d.dynprogindex = p.dynprogindex;
  return 1;
}

static size_t cdna_capacity_one(const gmapdp_cdna_problem& p) {
  if (cdna_on_host(p)) return 0;
  // two tracebacks (each <= rlength + glength records) + the 9 + 9 SHORTGAP block or a gap holder
  return 2 * ((size_t)p.rlengthL + (size_t)p.glength + 1) + 2 * kInsertPairsHost;
}

extern "C" {

size_t gmapdp_cdna_pair_capacity(const gmapdp_cdna_problem* problems, int n) {
  size_t cap = 0;
  for (int i = 0; i < n; i++) cap += cdna_capacity_one(problems[i]);
  return cap;
}

int gmapdp_cdna_gap_batch(gmapdp_ctx* ctx, const gmapdp_cdna_problem* problems, int n, const char* qseq,
                          const char* qseq_uc, size_t qbytes, gmapdp_cdna_result* results, gmapdp_pair* pairs,
                          size_t pair_capacity) {
  if (!ctx || n < 0 || (n > 0 && (!problems || !results))) return GMAPDP_EINVAL;
  if (!ctx->d_genome) return GMAPDP_ENOGENOME;
  if (n == 0) return GMAPDP_OK;
  (void)hipSetDevice(ctx->device);
  std::vector<DevCdnaProblem> dev;
  std::vector<int> dev_problem;
  // launch classes: (simd, R or B) -> device slots
  std::map<std::pair<int, int>, std::vector<int>> classes;
  size_t pair_off = 0, scratch_off = 0;
  for (int i = 0; i < n; i++) {
    DevCdnaProblem d;
    int err = 0;
    if (!convert_cdna(ctx, problems[i], qbytes, results[i], d, &err)) {
      if (err) return err;
      continue;
    }
    const bool simd = d.flags & kCSimd;
    const int W = d.lband + d.uband + 1;
    int RB;
    if (simd) {  // use8p (:909)
      const int u = kUse8pSize[d.mismatchtype];
      RB = (d.glength < u || (d.rlength < u && d.rlength <= u)) ? 32 : 16;
    } else {
      RB = pick_R(W);
      if (RB > kMaxR) return bad(ctx, "Dynprog_cdna_gap band wider than 4096 cells");
    }
    d.pair_offset = (int32_t)pair_off;
    pair_off += cdna_capacity_one(problems[i]);
    d.scratch_offset = (int64_t)scratch_off;
    scratch_off += align_up(scratch_bytes_cg(d.rlength, d.glength, d.lband, d.uband, simd, RB), 256);
    classes[{simd ? 1 : 0, RB}].push_back((int)dev.size());
    dev.push_back(d);
    dev_problem.push_back(i);
  }
  if (pair_off > pair_capacity) return bad(ctx, "pair arena too small");
  const int ndev = (int)dev.size();
  if (ndev == 0) return GMAPDP_OK;
  std::vector<int> order;
  order.reserve(ndev);
  struct CL {
    bool simd;
    int RB, first, count;
    size_t lds;
  };
  std::vector<CL> launches;
  for (auto& kv : classes) {
    CL L{kv.first.first != 0, kv.first.second, (int)order.size(), (int)kv.second.size(), 0};
    for (int s : kv.second) {
      L.lds = std::max(L.lds, lds_bytes_cg(dev[s].rlength, dev[s].glength, L.simd, L.RB));
      order.push_back(s);
    }
    launches.push_back(L);
  }
  hipError_t e = ctx->cprobs.ensure(sizeof(DevCdnaProblem) * ndev);
  if (e == hipSuccess) e = ctx->corder.ensure(sizeof(int) * ndev);
  if (e == hipSuccess) e = ctx->cresults.ensure(sizeof(gmapdp_cdna_result) * ndev);
  if (e == hipSuccess) e = ctx->cscratch.ensure(std::max<size_t>(scratch_off, 256));
  if (e == hipSuccess) e = ctx->qseq.ensure(qbytes);
  if (e == hipSuccess) e = ctx->qseq_uc.ensure(qbytes);
  if (e == hipSuccess) e = ctx->pairs.ensure(sizeof(gmapdp_pair) * std::max<size_t>(pair_off, 1));
  if (e != hipSuccess) return fail(ctx, GMAPDP_ENOMEM, "device buffers: %s", e);
  hipStream_t s = ctx->stream;
  e = hipMemcpyAsync(ctx->cprobs.p, dev.data(), sizeof(DevCdnaProblem) * ndev, hipMemcpyHostToDevice, s);
  if (e == hipSuccess) e = hipMemcpyAsync(ctx->corder.p, order.data(), sizeof(int) * ndev, hipMemcpyHostToDevice, s);
  if (e == hipSuccess) e = hipMemcpyAsync(ctx->qseq.p, qseq, qbytes, hipMemcpyHostToDevice, s);
  if (e == hipSuccess) e = hipMemcpyAsync(ctx->qseq_uc.p, qseq_uc, qbytes, hipMemcpyHostToDevice, s);
  if (e != hipSuccess) return fail(ctx, GMAPDP_ENOMEM, "upload: %s", e);
  for (const CL& L : launches) {
    e = launch_cg(L.simd, L.RB, L.count, L.lds, s, (const DevCdnaProblem*)ctx->cprobs.p,
                  (const int*)ctx->corder.p + L.first, (unsigned char*)ctx->cscratch.p, ctx->d_genome,
                  ctx->genome_words, (const char*)ctx->qseq.p, (const char*)ctx->qseq_uc.p, ctx->d_sc, ctx->d_cs,
                  (gmapdp_cdna_result*)ctx->cresults.p, (gmapdp_pair*)ctx->pairs.p);
    if (e != hipSuccess) return fail(ctx, GMAPDP_ELAUNCH, "cdna launch: %s", e);
  }
  std::vector<gmapdp_cdna_result> dres(ndev);
  e = hipMemcpyAsync(dres.data(), ctx->cresults.p, sizeof(gmapdp_cdna_result) * ndev, hipMemcpyDeviceToHost, s);
  if (e == hipSuccess && pairs)
    e = hipMemcpyAsync(pairs, ctx->pairs.p, sizeof(gmapdp_pair) * pair_off, hipMemcpyDeviceToHost, s);
  if (e == hipSuccess) e = ctx_sync(ctx, s);
  if (e != hipSuccess) return fail(ctx, GMAPDP_ELAUNCH, "cdna execution: %s", e);
  for (int d = 0; d < ndev; d++) results[dev_problem[d]] = dres[d];
  return GMAPDP_OK;
}

}  // extern "C"

// ---------------------------------------------------------------------------
// Dynprog_end5/3_splicejunction (dynprog_end.c:1653-1919 / 2249-2498)
// ---------------------------------------------------------------------------
static size_t sj_capacity_one(const gmapdp_sj_problem& p) {
  // every traceback step emits at most one record per row or column, plus the known gap holder
  return (size_t)std::max(p.rlength, 0) + (size_t)std::max(p.glength, 0) + 2;
}

// Prologue of the splice-junction end gaps: returns 1 if the problem runs on the GPU.
static int convert_sj(gmapdp_ctx* ctx, const gmapdp_sj_problem& p, size_t qbytes, const char* jseq, size_t jbytes,
                      gmapdp_sj_result& res, DevSjProblem& d, int* err) {
  *err = 0;
  res.npairs = 0;
  res.pair_offset = 0;
  res.known_index = -1;
  res.dynprogindex = p.dynprogindex;
  if (p.rlength <= 0 || p.rlength > GMAPDP_MAX_RLENGTH || p.glength <= 0 || p.glength > GMAPDP_MAX_GLENGTH) {
    res.traceback_score = 0;  // size guard (dynprog_end.c:1707-1722)
    res.nmatches = res.nmismatches = res.nopens = res.nindels = 0;
    res.missscore = -100;
    return 0;
  }
  const bool end3 = p.end3p != 0;
  if (p.qoff < 0 || (size_t)p.qoff + (size_t)p.rlength > qbytes || p.joff < 0 ||
      (size_t)p.joff + (size_t)p.glength > jbytes) {
    *err = bad(ctx, "splice-junction problem outside its query or junction arena");
    return 0;
  }
  for (int i = 0; i < p.glength; i++) {
    const char c = jseq[p.joff + i];
    if (c != 'A' && c != 'C' && c != 'G' && c != 'T' && c != 'N') {
      *err = bad(ctx, "junction characters must be A C G T or N");
      return 0;
    }
  }
  std::memset(&d, 0, sizeof(d));
  d.rlength = p.rlength;
  d.glength = p.glength;
  d.roffset = p.roffset;
  d.goffset_anchor = p.goffset_anchor;
  d.goffset_far = p.goffset_far;
  d.contlength = p.contlength;
  d.end3p = end3 ? 1 : 0;
  d.genestrand = p.genestrand;
  d.dynprogindex = p.dynprogindex;
  const bool jl = p.flags & GMAPDP_JUMP_LATE;
  if (end3) {
    d.qbase = p.qoff;
    d.jbase = p.joff;
    d.late = jl ? 1 : 0;
    d.known_jump = p.goffset_far - p.goffset_anchor;
  } else {
    d.qbase = p.qoff + p.rlength - 1;  // rev_rsequence / rev_gsequence: the slices' last characters
    d.jbase = p.joff + p.glength - 1;
    d.late = jl ? 0 : 1;               // "for revp true" !jump_late_p (dynprog_end.c:1792)
    d.known_jump = p.goffset_anchor - p.goffset_far;
  }
  const double dr = p.defect_rate;
  if (ctx->user_dynprog_p) {
    d.open = ctx->user_open;
    d.extend = ctx->user_extend;
  } else {
    d.open = dr < 0.003 ? -10 : (dr < 0.014 ? -8 : -6);  // END_OPEN_HIGHQ/MEDQ/LOWQ
    d.extend = -2;                                        // END_EXTEND_*
  }
  if (d.open > 0) {
    *err = bad(ctx, "positive gap-open penalty is not supported by the scan formulation");
    return 0;
  }
  gmapdp_compute_bands(&d.lband, &d.uband, p.rlength, p.glength, p.extraband, /*widebandp*/ 1);
  if (d.lband < 0 || d.uband < 0) {
    *err = bad(ctx, "negative band");
    return 0;
  }
  if (p.flags & GMAPDP_SIMD) {
    // the SIMD builds' endpoint scan reads lower[rlength][c] for c < rlength, past glength when
    // rlength > glength + 1 (uninitialised scores there; Splicetrie passes glength >= rlength)
    if (p.rlength > p.glength + 1) {
      *err = bad(ctx, "GMAPDP_SIMD splice junction with rlength > glength + 1");
      return 0;
    }
    d.simd = 1;
  }
  return 1;
}

extern "C" {

size_t gmapdp_sj_pair_capacity(const gmapdp_sj_problem* problems, int n) {
  size_t cap = 0;
  for (int i = 0; i < n; i++) cap += sj_capacity_one(problems[i]);
  return cap;
}

int gmapdp_end_splicejunction_batch(gmapdp_ctx* ctx, const gmapdp_sj_problem* problems, int n, const char* qseq,
                                    const char* qseq_uc, size_t qbytes, const char* jseq, size_t jbytes,
                                    gmapdp_sj_result* results, gmapdp_pair* pairs, size_t pair_capacity) {
  if (!ctx || n < 0 || (n > 0 && (!problems || !results))) return GMAPDP_EINVAL;
  if (n == 0) return GMAPDP_OK;
  (void)hipSetDevice(ctx->device);
  std::vector<DevSjProblem> dev;
  std::vector<int> dev_problem;
  std::map<std::pair<int, int>, std::vector<int>> classes;  // (R, dirs in LDS) -> device slots
  size_t pair_off = 0, dirs_off = 0;
  for (int i = 0; i < n; i++) {
    DevSjProblem d;
    int err = 0;
    if (!convert_sj(ctx, problems[i], qbytes, jseq, jbytes, results[i], d, &err)) {
      if (err) return err;
      continue;
    }
    d.pair_offset = (int32_t)pair_off;
    if (d.simd) {  // 8-bit triangles when either length is below use8p_size[ENDQ] (dynprog_end.c:1743)
      const int B = (d.rlength < kUse8pSize[kEndQ] || d.glength < kUse8pSize[kEndQ]) ? 32 : 16;
      d.dirs_offset = (int64_t)dirs_off;
      dirs_off += align_up(scratch_bytes_uxe(d.rlength, d.glength, d.lband, d.uband, B), 256);
      pair_off += sj_capacity_one(problems[i]);
      classes[{-B, 0}].push_back((int)dev.size());
      dev.push_back(d);
      dev_problem.push_back(i);
      continue;
    }
    const int W = d.lband + d.uband + 1;
    const int R = pick_R(W);
    if (R > kMaxR) return bad(ctx, "splice-junction band wider than 4096 cells");
    const bool dirs_lds = lds_bytes_sj(d.rlength, d.glength, R, true) <= kLdsBudget;
    if (!dirs_lds) {
      if (lds_bytes_sj(d.rlength, d.glength, R, false) > 160 * 1024) return bad(ctx, "problem exceeds the LDS of a CU");
      d.dirs_offset = (int64_t)dirs_off;
      dirs_off += align_up((size_t)(d.glength + 1) * 4 * R * 8, 256);
    }
    d.pair_offset = (int32_t)pair_off;
    pair_off += sj_capacity_one(problems[i]);
    classes[{R, dirs_lds ? 1 : 0}].push_back((int)dev.size());
    dev.push_back(d);
    dev_problem.push_back(i);
  }
  if (pair_off > pair_capacity) return bad(ctx, "pair arena too small");
  const int ndev = (int)dev.size();
  if (ndev == 0) return GMAPDP_OK;
  std::vector<int> order;
  order.reserve(ndev);
  struct CL {
    int R;
    bool dirs_lds;
    int first, count;
    size_t lds;
  };
  std::vector<CL> launches;
  for (auto& kv : classes) {
    CL L{kv.first.first, kv.first.second != 0, (int)order.size(), (int)kv.second.size(), 0};
    for (int s : kv.second) {
      L.lds = std::max(L.lds, L.R < 0 ? lds_bytes_uxe(dev[s].rlength, dev[s].glength, -L.R)
                                      : lds_bytes_sj(dev[s].rlength, dev[s].glength, L.R, L.dirs_lds));
      order.push_back(s);
    }
    if (L.lds > 160 * 1024) return bad(ctx, "problem exceeds the LDS of a CU");
    launches.push_back(L);
  }
  hipError_t e = ctx->sjprobs.ensure(sizeof(DevSjProblem) * ndev);
  if (e == hipSuccess) e = ctx->sjorder.ensure(sizeof(int) * ndev);
  if (e == hipSuccess) e = ctx->sjresults.ensure(sizeof(gmapdp_sj_result) * ndev);
  if (e == hipSuccess) e = ctx->sjdirs.ensure(std::max<size_t>(dirs_off, 256));
  if (e == hipSuccess) e = ctx->sjseq.ensure(jbytes);
  if (e == hipSuccess) e = ctx->qseq.ensure(qbytes);
  if (e == hipSuccess) e = ctx->qseq_uc.ensure(qbytes);
  if (e == hipSuccess) e = ctx->pairs.ensure(sizeof(gmapdp_pair) * std::max<size_t>(pair_off, 1));
  if (e != hipSuccess) return fail(ctx, GMAPDP_ENOMEM, "device buffers: %s", e);
  hipStream_t s = ctx->stream;
  e = hipMemcpyAsync(ctx->sjprobs.p, dev.data(), sizeof(DevSjProblem) * ndev, hipMemcpyHostToDevice, s);
  if (e == hipSuccess) e = hipMemcpyAsync(ctx->sjorder.p, order.data(), sizeof(int) * ndev, hipMemcpyHostToDevice, s);
  if (e == hipSuccess) e = hipMemcpyAsync(ctx->qseq.p, qseq, qbytes, hipMemcpyHostToDevice, s);
  if (e == hipSuccess) e = hipMemcpyAsync(ctx->qseq_uc.p, qseq_uc, qbytes, hipMemcpyHostToDevice, s);
  if (e == hipSuccess) e = hipMemcpyAsync(ctx->sjseq.p, jseq, jbytes, hipMemcpyHostToDevice, s);
  if (e != hipSuccess) return fail(ctx, GMAPDP_ENOMEM, "upload: %s", e);
  for (const CL& L : launches) {
    if (L.R < 0)  // SIMD-build semantics: key -B
      e = launch_usj(-L.R, L.count, L.lds, s, (const DevSjProblem*)ctx->sjprobs.p, (const int*)ctx->sjorder.p + L.first,
                     (unsigned char*)ctx->sjdirs.p, (const char*)ctx->qseq.p, (const char*)ctx->qseq_uc.p,
                     (const char*)ctx->sjseq.p, ctx->d_sc, ctx->d_cs, (gmapdp_sj_result*)ctx->sjresults.p,
                     (gmapdp_pair*)ctx->pairs.p);
    else
      e = launch_sj(L.R, L.dirs_lds, L.count, L.lds, s, (const DevSjProblem*)ctx->sjprobs.p,
                    (const int*)ctx->sjorder.p + L.first, (const char*)ctx->qseq.p, (const char*)ctx->qseq_uc.p,
                    (const char*)ctx->sjseq.p, ctx->d_sc, ctx->d_cs, (gmapdp_sj_result*)ctx->sjresults.p,
                    (gmapdp_pair*)ctx->pairs.p, (uint64_t*)ctx->sjdirs.p);
    if (e != hipSuccess) return fail(ctx, GMAPDP_ELAUNCH, "splice-junction launch: %s", e);
  }
  std::vector<gmapdp_sj_result> dres(ndev);
  e = hipMemcpyAsync(dres.data(), ctx->sjresults.p, sizeof(gmapdp_sj_result) * ndev, hipMemcpyDeviceToHost, s);
  if (e == hipSuccess && pairs)
    e = hipMemcpyAsync(pairs, ctx->pairs.p, sizeof(gmapdp_pair) * pair_off, hipMemcpyDeviceToHost, s);
  if (e == hipSuccess) e = ctx_sync(ctx, s);
  if (e != hipSuccess) return fail(ctx, GMAPDP_ELAUNCH, "splice-junction execution: %s", e);
  for (int d = 0; d < ndev; d++) results[dev_problem[d]] = dres[d];
  return GMAPDP_OK;
}

}  // extern "C"

// ---------------------------------------------------------------------------
// Device-resident path (bench / pipelined callers): the plan is built once on
// the host, then replayed against device-resident inputs.
// ---------------------------------------------------------------------------
struct gmapdp_plan {
  PlanCore in;
  int nsingle = 0, nend = 0, ngenome = 0;
  DevProblem* d_probs = nullptr;
  int* d_order = nullptr;
  DevGenomeProblem* d_gprobs = nullptr;
  int* d_gorder = nullptr;
  const double* d_sprob = nullptr;            // bound by gmapdp_plan_bind_genome
  gmapdp_genome_result* d_gresults = nullptr;
  const double* d_metab = nullptr;            // gmapdp_plan_bind_genome_maxent: each genome-gap class fills d_sprob
  void* d_base = nullptr;                     // one allocation holding d_probs, d_order, d_gprobs, d_gorder
  // the descriptors' upload, left in flight by gmapdp_plan_create_all (it overlaps the caller's next host
  // work: the stage-2 plan's build); the plan's first run waits for it
  hipEvent_t ev_up = nullptr;
  mutable std::atomic<bool> up_done{false};
};

static void plan_free(gmapdp_plan* p) {
  if (p->ev_up) {
    (void)hipEventSynchronize(p->ev_up);
    (void)hipEventDestroy(p->ev_up);
  }
  if (p->d_base) (void)hipFree(p->d_base);
  delete p;
}

// before a plan's descriptors are read on any stream
static hipError_t plan_uploaded(const gmapdp_plan* p) {
  if (!p->ev_up || p->up_done.load(std::memory_order_acquire)) return hipSuccess;
  const hipError_t e = hipEventSynchronize(p->ev_up);
  if (e == hipSuccess) p->up_done.store(true, std::memory_order_release);
  return e;
}

static RunArgs plan_args(const gmapdp_plan* plan, const char* d_qseq, const char* d_qseq_uc, gmapdp_result* d_results,
                         gmapdp_pair* d_pairs) {
  RunArgs a;
  a.d_probs = plan->d_probs;
  a.d_order = plan->d_order;
  a.d_gprobs = plan->d_gprobs;
  a.d_gorder = plan->d_gorder;
  a.d_q = d_qseq;
  a.d_quc = d_qseq_uc;
  a.d_sprob = plan->d_sprob;
  a.d_metab = plan->d_metab;
  a.d_results = d_results;
  a.d_gresults = plan->d_gresults;
  a.d_pairs = d_pairs;
  return a;
}

extern "C" {

int gmapdp_plan_create_all(gmapdp_ctx* ctx, const gmapdp_single_problem* singles, int nsingle,
                           const gmapdp_end_problem* ends, int nend, const gmapdp_genome_problem* genomes,
                           int ngenome, gmapdp_result* host_results, gmapdp_genome_result* host_genome_results,
                           gmapdp_plan** out) {
  if (!ctx || !out || nsingle < 0 || nend < 0 || ngenome < 0 || nsingle + nend + ngenome <= 0) return GMAPDP_EINVAL;
  if ((nsingle && !singles) || (nend && !ends) || (ngenome && !genomes)) return GMAPDP_EINVAL;
  if ((nsingle + nend && !host_results) || (ngenome && !host_genome_results)) return GMAPDP_EINVAL;
  (void)hipSetDevice(ctx->device);
  gmapdp_plan* p = new gmapdp_plan();
  PlanTimer tm("plan_create_all");
  p->nsingle = nsingle;
  p->nend = nend;
  p->ngenome = ngenome;
  int rc = build_plan(ctx, singles, nsingle, ends, nend, genomes, ngenome, host_results, host_genome_results, p->in);
  tm.mark("build_plan");
  if (rc) {
    delete p;
    return rc;
  }
  for (const DevGenomeProblem& g : p->in.gdev)
    if (g.flags & kGKnown) {  // the plan binds no known-site arena
      delete p;
      return bad(ctx, "GMAPDP_KNOWN_SITES genome gaps go through the synchronous batches, not plans");
    }
  const size_t nd = p->in.dev.size(), ng = p->in.gdev.size();
  // the four descriptor arrays in one device allocation (one hipMalloc per plan, not four)
  size_t o1 = align_up(sizeof(DevProblem) * std::max<size_t>(nd, 1), 256);
  size_t o2 = o1 + align_up(sizeof(int) * std::max<size_t>(nd, 1), 256);
  size_t o3 = o2 + align_up(sizeof(DevGenomeProblem) * std::max<size_t>(ng, 1), 256);
  const size_t dtot = o3 + align_up(sizeof(int) * std::max<size_t>(ng, 1), 256);
  hipError_t e = hipMalloc(&p->d_base, dtot);
  if (e == hipSuccess) {
    unsigned char* b = (unsigned char*)p->d_base;
    p->d_probs = (DevProblem*)b;
    p->d_order = (int*)(b + o1);
    p->d_gprobs = (DevGenomeProblem*)(b + o2);
    p->d_gorder = (int*)(b + o3);
  }
  tm.mark("alloc");
  // the four descriptor arrays (~115 MB for a 10 000-read block) copied into one pinned image on the plan's
  // threads, then moved with asynchronous copies (a pageable hipMemcpy stages through the runtime's own
  // buffers on one thread)
  {
    struct Part {
      void* dst;
      const void* src;
      size_t n, at;
    } parts[4] = {{p->d_probs, p->in.dev.data(), sizeof(DevProblem) * nd, 0},
                  {p->d_order, p->in.order.data(), sizeof(int) * nd, 0},
                  {p->d_gprobs, p->in.gdev.data(), sizeof(DevGenomeProblem) * ng, 0},
                  {p->d_gorder, p->in.gorder.data(), sizeof(int) * ng, 0}};
    size_t tot = 0;
    for (Part& x : parts) {
      x.at = tot;
      tot = align_up(tot + x.n, 256);
    }
    // (the previous plan's copies out of hplan first)
    if (e == hipSuccess && ctx->ev_hplan) e = hipEventSynchronize(ctx->ev_hplan);
    if (e == hipSuccess) e = ctx->hplan.ensure(std::max<size_t>(tot, 256));
    unsigned char* h = (unsigned char*)ctx->hplan.p;
    // in 8-MB pieces, so that each piece's DMA runs while the threads fill the next
    constexpr size_t kPiece = size_t(8) << 20;
    for (Part& x : parts)
      for (size_t o = 0; e == hipSuccess && o < x.n; o += kPiece) {
        const size_t m = std::min(kPiece, x.n - o);
        plan_parallel(m, plan_threads(m / 64), [&](size_t lo, size_t hi, int) {
          std::memcpy(h + x.at + o + lo, (const unsigned char*)x.src + o + lo, hi - lo);
        });
        e = hipMemcpyAsync((unsigned char*)x.dst + o, h + x.at + o, m, hipMemcpyHostToDevice, ctx->stream);
      }
    if (e == hipSuccess && !ctx->ev_hplan) e = hipEventCreateWithFlags(&ctx->ev_hplan, hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&p->ev_up, hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventRecord(ctx->ev_hplan, ctx->stream);
    if (e == hipSuccess) e = hipEventRecord(p->ev_up, ctx->stream);
  }
  if (e == hipSuccess && p->in.gdirs_bytes) e = ctx->gdirs.ensure(p->in.gdirs_bytes);
  tm.mark("upload");
  if (e != hipSuccess) {
    plan_free(p);
    return fail(ctx, GMAPDP_ENOMEM, "plan upload: %s", e);
  }
  *out = p;
  return GMAPDP_OK;
}

int gmapdp_plan_create(gmapdp_ctx* ctx, const gmapdp_single_problem* singles, int nsingle,
                       const gmapdp_end_problem* ends, int nend, gmapdp_result* host_results, gmapdp_plan** out) {
  return gmapdp_plan_create_all(ctx, singles, nsingle, ends, nend, nullptr, 0, host_results, nullptr, out);
}

int gmapdp_plan_single(gmapdp_ctx* ctx, const gmapdp_single_problem* problems, int n, gmapdp_result* host_results,
                       gmapdp_plan** out) {
  return gmapdp_plan_create(ctx, problems, n, nullptr, 0, host_results, out);
}

int gmapdp_plan_bind_genome(gmapdp_plan* plan, const double* d_splice_probs, gmapdp_genome_result* d_genome_results) {
  if (!plan) return GMAPDP_EINVAL;
  plan->d_sprob = d_splice_probs;
  plan->d_gresults = d_genome_results;
  plan->d_metab = nullptr;
  return GMAPDP_OK;
}

int gmapdp_plan_bind_genome_maxent(gmapdp_ctx* ctx, gmapdp_plan* plan, double* d_splice_probs,
                                   gmapdp_genome_result* d_genome_results) {
  if (!ctx || !plan || !d_splice_probs) return GMAPDP_EINVAL;
  (void)hipSetDevice(ctx->device);
  const double* T = me_tables(ctx);
  if (!T) return GMAPDP_EINVAL;
  plan->d_sprob = d_splice_probs;
  plan->d_gresults = d_genome_results;
  plan->d_metab = T;
  return GMAPDP_OK;
}

size_t gmapdp_plan_pair_capacity(const gmapdp_plan* plan) { return plan ? plan->in.pair_capacity : 0; }
int gmapdp_plan_gpu_problems(const gmapdp_plan* plan) { return plan ? (int)plan->in.dev.size() : 0; }
int gmapdp_plan_genome_gpu_problems(const gmapdp_plan* plan) { return plan ? (int)plan->in.gdev.size() : 0; }
int gmapdp_plan_dev_index(const gmapdp_plan* plan, int i) {
  return (plan && i >= 0 && i < (int)plan->in.dev_index.size()) ? plan->in.dev_index[i] : -1;
}
int gmapdp_plan_genome_dev_index(const gmapdp_plan* plan, int j) {
  return (plan && j >= 0 && j < (int)plan->in.gdev_index.size()) ? plan->in.gdev_index[j] : -1;
}
int gmapdp_plan_nlaunches(const gmapdp_plan* plan) { return plan ? (int)plan->in.launches.size() : 0; }

int gmapdp_plan_launch_info(const gmapdp_plan* plan, int li, int* R, int* dirs_lds, int* count, size_t* lds) {
  if (!plan || li < 0 || li >= (int)plan->in.launches.size()) return GMAPDP_EINVAL;
  const auto& L = plan->in.launches[li];
  if (R) *R = L.R;
  if (dirs_lds) *dirs_lds = L.dirs_lds ? 1 : 0;
  if (count) *count = L.count;
  if (lds) *lds = L.lds;
  return GMAPDP_OK;
}

int gmapdp_plan_launch_kind(const gmapdp_plan* plan, int li) {
  if (!plan || li < 0 || li >= (int)plan->in.launches.size()) return GMAPDP_EINVAL;
  return plan->in.launches[li].kind;
}

int gmapdp_plan_launch_stream(const gmapdp_plan* plan, int li) {
  if (!plan || li < 0 || li >= (int)plan->in.launches.size()) return GMAPDP_EINVAL;
  return plan->in.launches[li].stream;
}

int gmapdp_plan_launch_is_tail(const gmapdp_plan* plan, int li) {
  if (!plan || li < 0 || li >= (int)plan->in.launches.size()) return GMAPDP_EINVAL;
  return launch_is_tail(plan->in.launches[li]) ? 1 : 0;
}

int gmapdp_plan_launch_members(const gmapdp_plan* plan, int li, int* problem_indices) {
  if (!plan || li < 0 || li >= (int)plan->in.launches.size() || !problem_indices) return GMAPDP_EINVAL;
  const auto& L = plan->in.launches[li];
  for (int k = 0; k < L.count; k++) {
    const bool genome = L.kind == PlanCore::kGenomeGap || L.kind == PlanCore::kUxg;
    if (!genome) problem_indices[k] = plan->in.dev_problem[plan->in.order[L.first + k]];
    else problem_indices[k] = plan->nsingle + plan->nend + plan->in.gdev_problem[plan->in.gorder[L.first + k]];
  }
  return GMAPDP_OK;
}

int gmapdp_plan_run(gmapdp_ctx* ctx, const gmapdp_plan* plan, const char* d_qseq, const char* d_qseq_uc,
                    gmapdp_result* d_results, gmapdp_pair* d_pairs, void* stream) {
  if (!ctx || !plan) return GMAPDP_EINVAL;
  if (!ctx->d_genome) return GMAPDP_ENOGENOME;
  if (!plan->in.gdev.empty() && (!plan->d_sprob || !plan->d_gresults)) return bad(ctx, "genome-gap buffers not bound");
  if (const hipError_t eu = plan_uploaded(plan)) return fail(ctx, GMAPDP_ELAUNCH, "plan upload: %s", eu);
  return run_plan(ctx, plan->in, plan_args(plan, d_qseq, d_qseq_uc, d_results, d_pairs),
                  stream ? (hipStream_t)stream : ctx->stream);
}

static int plan_run_launch(gmapdp_ctx* ctx, const gmapdp_plan* plan, int li, const char* d_qseq,
                           const char* d_qseq_uc, gmapdp_result* d_results, gmapdp_pair* d_pairs, void* stream,
                           bool prologue) {
  if (!ctx || !plan || li < 0 || li >= (int)plan->in.launches.size()) return GMAPDP_EINVAL;
  if (!ctx->d_genome) return GMAPDP_ENOGENOME;
  if (plan->in.gdirs_bytes) {
    hipError_t e = ctx->gdirs.ensure(plan->in.gdirs_bytes);
    if (e != hipSuccess) return fail(ctx, GMAPDP_ENOMEM, "direction scratch: %s", e);
  }
  if (const hipError_t eu = plan_uploaded(plan)) return fail(ctx, GMAPDP_ELAUNCH, "plan upload: %s", eu);
  hipError_t e = launch_one(ctx, plan->in, li, plan_args(plan, d_qseq, d_qseq_uc, d_results, d_pairs),
                            stream ? (hipStream_t)stream : ctx->stream, prologue);
  if (e != hipSuccess) return fail(ctx, GMAPDP_ELAUNCH, "dp launch: %s", e);
  return GMAPDP_OK;
}

int gmapdp_plan_run_launch(gmapdp_ctx* ctx, const gmapdp_plan* plan, int li, const char* d_qseq,
                           const char* d_qseq_uc, gmapdp_result* d_results, gmapdp_pair* d_pairs, void* stream) {
  return plan_run_launch(ctx, plan, li, d_qseq, d_qseq_uc, d_results, d_pairs, stream, true);
}

// Host side of the compact pair stream: problem i's ops at stream[offsets[i], offsets[i + 1]) back to its
// npairs[i] records at out[pair_offsets[i]] (threads over the problems).  GMAPDP_EINVAL when a problem's
// ops do not decode to exactly its records and bytes.
}  // extern "C"

// (Rec: gmapdp_pair, 17-B RAW ops, or gmapdp_path_pair, 21-B RAW ops; list i: npairs_of(i) records at
// offset_of(i))
template <typename Rec, typename NP, typename OF>
static int expand_stream(const uint8_t* stream, const uint64_t* offsets, int n, NP&& npairs_of, OF&& offset_of,
                         Rec* out, int nthreads) {
  static const char nt[4] = {'A', 'C', 'G', 'T'}, cp[4] = {'*', '|', ' ', ':'};
  constexpr int kRaw = 1 + (int)sizeof(Rec);
  const int T = nthreads > 0 ? nthreads : plan_threads((size_t)n * 64);
  std::vector<int> bad_at(T, -1);
  plan_parallel((size_t)n, T, [&](size_t lo, size_t hi, int t) {
    for (size_t i = lo; i < hi; i++) {
      const uint8_t* p = stream + offsets[i];
      const uint8_t* end = stream + offsets[i + 1];
      const int m = std::max<int>(npairs_of(i), 0);
      Rec* o = m ? out + offset_of(i) : out;
      int k = 0;
      while (k < m && p < end) {
        if (*p == 0x02) {
          if (end - p < kRaw) break;
          std::memcpy(&o[k++], p + 1, sizeof(Rec));
          p += kRaw;
          continue;
        }
        if (*p != 0x01 || end - p < 13) break;
        int32_t q, g;
        std::memcpy(&q, p + 1, 4);
        std::memcpy(&g, p + 5, 4);
        const int dq = (int8_t)p[9], dg = (int8_t)p[10];
        const int len = p[11] | (p[12] << 8);
        p += 13;
        for (int r = 0; r < len && k < m && p < end; r++, k++) {
          Rec& x = o[k];
          x.querypos = q + r * dq;
          x.genomepos = g + r * dg;
          if constexpr (sizeof(Rec) == sizeof(gmapdp_pair)) {
            x.jump = 0;
          } else {
            x.queryjump = 0;
            x.genomejump = 0;
          }
          if (*p == 0xFF) {
            std::memcpy(&x.cdna, p + 1, 4);
            p += 5;
          } else {
            const uint8_t b = *p++;
            x.cdna = nt[b & 3];
            x.genome = x.genomealt = nt[(b >> 2) & 3];
            x.comp = cp[(b >> 4) & 3];
          }
        }
      }
      if (k != m || p != end) {
        bad_at[t] = (int)i;
        return;
      }
    }
  });
  for (int t = 0; t < T; t++)
    if (bad_at[t] >= 0) return GMAPDP_EINVAL;
  return GMAPDP_OK;
}

extern "C" {

int gmapdp_expand_pairs(const uint8_t* stream, const uint64_t* offsets, int n, const int32_t* npairs,
                        const int64_t* pair_offsets, gmapdp_pair* out, int nthreads) {
  if (n < 0 || (n && (!stream || !offsets || !npairs || !pair_offsets || !out))) return GMAPDP_EINVAL;
  return expand_stream(stream, offsets, n, [&](size_t i) { return npairs[i]; },
                       [&](size_t i) { return pair_offsets[i]; }, out, nthreads);
}

int gmapdp_expand_path_pairs(const uint8_t* stream, const uint64_t* offsets, int npaths, const gmapdp_path* paths,
                             gmapdp_path_pair* out, int nthreads) {
  if (npaths < 0 || (npaths && (!stream || !offsets || !paths || !out))) return GMAPDP_EINVAL;
  return expand_stream(stream, offsets, npaths, [&](size_t i) { return paths[i].npairs; },
                       [&](size_t i) { return paths[i].pair_offset; }, out, nthreads);
}

// The compact pair stream (pc_kernel.hip): the plan's GPU problems in dev-slot order, then its genome gaps.
size_t gmapdp_plan_compact_bound(const gmapdp_plan* plan) {
  return plan ? 17 * plan->in.pair_capacity + 64 : 0;
}
int gmapdp_plan_compact_pairs(gmapdp_ctx* ctx, const gmapdp_plan* plan, const gmapdp_result* d_results,
                              const gmapdp_pair* d_pairs, uint8_t* d_out, uint64_t* d_offsets, void* stream) {
  if (!ctx || !plan || !d_offsets || (!plan->in.dev.empty() && !d_results)) return GMAPDP_EINVAL;
  if (!plan->in.gdev.empty() && !plan->d_gresults) return bad(ctx, "genome-gap results not bound");
  (void)hipSetDevice(ctx->device);
  hipStream_t s = stream ? (hipStream_t)stream : ctx->stream;
  const hipError_t e = launch_pc((const unsigned char*)d_results, (int)plan->in.dev.size(), (int)sizeof(gmapdp_result),
                                 (const unsigned char*)plan->d_gresults, (int)plan->in.gdev.size(),
                                 (int)sizeof(gmapdp_genome_result), d_pairs, (unsigned long long*)d_offsets,
                                 (unsigned char*)d_out, s);
  return e == hipSuccess ? GMAPDP_OK : fail(ctx, GMAPDP_ELAUNCH, "pair compaction: %s", e);
}

int gmapdp_plan_run_launch_kernel(gmapdp_ctx* ctx, const gmapdp_plan* plan, int li, const char* d_qseq,
                                  const char* d_qseq_uc, gmapdp_result* d_results, gmapdp_pair* d_pairs, void* stream) {
  return plan_run_launch(ctx, plan, li, d_qseq, d_qseq_uc, d_results, d_pairs, stream, false);
}

void gmapdp_plan_destroy(gmapdp_plan* plan) {
  if (plan) plan_free(plan);
}

void* gmapdp_stream(gmapdp_ctx* ctx) { return ctx ? (void*)ctx->stream : nullptr; }

}  // extern "C"

// ---------------------------------------------------------------------------
// Stage-2 seeding: Oligoindex_hr_tally + Oligoindex_get_mappings as
// Stage2_compute calls them for GMAP (stage2.c:6480-6495).  Synchronous batch path.
// ---------------------------------------------------------------------------
static const int kOligoMaxDistinct = 16384;

// 8-mer starts the tally visits (count_positions_fwd/rev_std, oligoindex_hr.c:19268-19281)
static uint64_t oligo_window(const gmapdp_oligo_problem& p) {
  const uint64_t left = (uint64_t)p.chroffset + p.chrstart;
  uint64_t lpl = (uint64_t)p.chroffset + p.chrend + (p.plusp ? 0 : 1);
  lpl = lpl < 8 ? 0 : lpl - 8;
  return lpl > left ? lpl - left + 1 : 0;
}
static size_t oligo_table_cap(const gmapdp_oligo_problem& p) {
  if (p.querylength <= 8) return 0;
  return (size_t)std::min<uint64_t>(oligo_window(p), 255ull * (uint64_t)(p.querylength - 7));
}
// a good diagonal takes suffnconsecutive + 1 >= 11 hits, each query position at most 255
static size_t oligo_diag_cap(const gmapdp_oligo_problem& p) {
  if (p.querylength <= 8) return 0;
  return (size_t)(p.querylength - 7) * 24 + 1;
}
// distinct 8-mers of the query, as Oligoindex_set_inquery marks them (:33490-33515)
static int oligo_distinct(const char* q, int qlen, std::vector<uint32_t>& bm) {
  int n = 0, in_counter = 0;
  uint32_t oligo = 0;
  thread_local std::vector<uint32_t> touched;
  touched.clear();
  // (a table lookup per character: a four-way switch mispredicted on most characters)
  static const struct Lut {
    uint8_t v[256];
    Lut() {
      std::memset(v, 4, sizeof(v));
      v['A'] = 0;
      v['C'] = 1;
      v['G'] = 2;
      v['T'] = 3;
    }
  } lut;
  for (int i = 0; i < qlen; i++) {
    const uint32_t c = lut.v[(unsigned char)q[i]];
    if (c > 3) {
      oligo = 0;
      in_counter = 0;
      continue;
    }
    in_counter++;
    oligo = (oligo << 2) | c;
    if (in_counter == 8) {
      const uint32_t m = oligo & 0xFFFFu;
      if (!((bm[m >> 5] >> (m & 31)) & 1u)) {
        bm[m >> 5] |= 1u << (m & 31);
        touched.push_back(m >> 5);
        n++;
      }
      in_counter--;
    }
  }
  for (uint32_t w : touched) bm[w] = 0;
  return n;
}

extern "C" {

size_t gmapdp_oligo_positions_capacity(const gmapdp_oligo_problem* problems, int n) {
  size_t c = 0;
  for (int i = 0; i < n; i++) c += oligo_table_cap(problems[i]);
  return c;
}
size_t gmapdp_oligo_diagonal_capacity(const gmapdp_oligo_problem* problems, int n) {
  size_t c = 0;
  for (int i = 0; i < n; i++) c += oligo_diag_cap(problems[i]);
  return c;
}

}  // extern "C"

// A planned stage-2 batch: descriptors (in launch-class order) resident on the device, the launches, the
// scratch, the output capacities.  Launches are chunks of one launch class: each chunk's problems have their
// scratch regions and event-pool slots laid out from 0, and the chunks run one after another on the stream,
// so the scratch and the pool are sized for the largest chunk, not for the batch (a 214-kb stage-2 window,
// as GMAP's stage 1 extends a gregion by 100 kb each side, gregion.c:899, takes 1.7 MB of hit list and
// 7 MB of sequential-walk states).
struct gmapdp_oligo_plan {
  int n = 0;
  DevOligoProblem* d_probs = nullptr;
  unsigned char* d_scratch = nullptr;
  std::vector<std::pair<int, int>> launches;  // (first, count) per chunk
  std::vector<int> umax;                      // per chunk: 2 * umax + (32-bit counters)
  std::vector<int> keys;                      // per problem in launch order: its class key
  size_t table_cap = 0, diag_cap = 0, scratch_cap = 0;
  int32_t* d_nhits = nullptr;                 // sizing runs: each problem's hit-list length
  // Two seeding paths with the same results.  Device-resident plans (a stage-2 plan's sizing run and its
  // runs: bench.py's step, many calls beside the DP classes) take oi_kernel + oi_map_kernel, small-LDS
  // kernels that share the CUs with the DP launches; the synchronous batch APIs (the drop-in's dispatcher
  // batches: a few calls, latency-bound) take oi_scan_kernel + oi_build_kernel, four waves per call and
  // the table and the event sort in LDS (measured: DESIGN.md §5.7).
  bool split = false;
  // get_mappings' event pool (3 slots per hit, shared by a chunk through an atomic cursor; a problem that no
  // longer fits runs the sequential walk in its fallback region, or reports overflow when it has none)
  uint64_t* d_pool = nullptr;
  unsigned long long* d_pool_counter = nullptr;
  unsigned long long pool_cap = 0;
  // A plan made inside a synchronous batch call borrows the context's grow-only buffers: no
  // hipMalloc / hipFree per call (hipFree waits for the whole device, which would serialise the
  // shim's concurrent batches).  `ord` is the host image of d_probs, kept until the plan is freed.
  // A stage-2 plan's sizing run borrows them as well (tight growth): its upper-bound arenas, tens of GB, are
  // dropped right after the run, and a fresh hipMalloc of that size per plan took up to a second.
  bool borrowed = false, sizing = false;
  std::vector<DevOligoProblem> ord;
};

static constexpr int kOligoChunkProblems = 16384;
// scratch per launch chunk: 3 GB for the synchronous batches (a context keeps its grow-only scratch); a
// stage-2 plan's sizing run (window-sized hit lists and walk states, ~7 MB per 214-kb call) takes 32 GB
// chunks of the context's grow-only scratch: a 10 000-read block in 4 launches instead of 14 (a chunk of a
// thousand calls leaves most of the GPU idle); the process pays the first allocation once
static constexpr size_t kOligoChunkBytes = size_t(3) << 30;
static constexpr size_t kOligoSizingChunkBytes = size_t(32) << 30;

static void oligo_plan_free(gmapdp_oligo_plan* p) {
  if (!p) return;
  if (p->borrowed) {
    delete p;
    return;
  }
  if (p->d_probs) (void)hipFree(p->d_probs);
  if (p->d_scratch) (void)hipFree(p->d_scratch);
  if (p->d_pool) (void)hipFree(p->d_pool);
  if (p->d_pool_counter) (void)hipFree(p->d_pool_counter);
  if (p->d_nhits) (void)hipFree(p->d_nhits);
  delete p;
}

// Cut the launch-ordered problems into chunks and lay out each chunk's scratch (main region, then the
// sequential walk's region when `fallback`) and pool, and the table and diagonal arenas: slots[i], tcap[i],
// dcap[i] are what problem i may take of each.  `local`: the arenas too restart at 0 in every chunk (a
// sizing run, whose outputs are only its counts), else they are laid out over the whole plan.
static void oligo_layout(gmapdp_oligo_plan* P, const std::vector<size_t>& slots, bool fallback,
                         const std::vector<size_t>& tcap, const std::vector<size_t>& dcap, bool local,
                         const std::vector<size_t>* hcap = nullptr) {
  P->launches.clear();
  P->umax.clear();
  P->scratch_cap = 0;
  P->pool_cap = 0;
  P->table_cap = 0;
  P->diag_cap = 0;
  size_t cb = 0, cs = 0, ct = 0, cd = 0;
  int first = 0;
  auto close = [&](int end) {
    if (end > first) {
      P->launches.push_back({first, end - first});
      P->umax.push_back(P->keys[first]);
      P->scratch_cap = std::max(P->scratch_cap, cb);
      P->pool_cap = std::max<unsigned long long>(P->pool_cap, cs);
      P->table_cap = std::max(P->table_cap, ct);
      P->diag_cap = std::max(P->diag_cap, cd);
    }
    first = end;
    cb = cs = 0;
    if (local) ct = cd = 0;
  };
  for (int k = 0; k < (int)P->ord.size(); k++) {
    DevOligoProblem& d = P->ord[k];
    const uint32_t w = d.chrend > d.chrstart ? d.chrend - d.chrstart : 0;
    const size_t mb = align_up(hcap ? scratch_bytes_oi_hits(d.querylength, (*hcap)[d.index])
                                    : scratch_bytes_oi(d.querylength, w), 256);
    const size_t fb = fallback ? align_up(scratch_bytes_oi_fallback(d.querylength, w), 256) : 0;
    if (k > first && (P->keys[k] != P->keys[first] || k - first >= kOligoChunkProblems ||
                      cb + mb + fb > (local ? kOligoSizingChunkBytes : kOligoChunkBytes)))
      close(k);
    d.scratch_offset = (int64_t)cb;
    d.fallback_offset = fallback ? (int64_t)(cb + mb) : -1;
    d.table_offset = (int64_t)ct;
    d.diag_offset = (int64_t)cd;
    // (scratch_oi sizes the hit list from the window: one entry per 8-mer start, + 2)
    d.hit_cap = (uint32_t)std::min<size_t>(hcap ? (*hcap)[d.index] : (size_t)w + 2, 0xffffffffu);
    d.table_cap = (uint32_t)std::min<size_t>(tcap[d.index], 0xffffffffu);
    d.diag_cap = (uint32_t)std::min<size_t>(dcap[d.index], 0xffffffffu);
    cb += mb + fb;
    cs += slots[d.index];
    ct += tcap[d.index];
    cd += dcap[d.index];
  }
  close((int)P->ord.size());
}

static hipError_t oligo_buffers(gmapdp_ctx* ctx, gmapdp_oligo_plan* P) {
  const int n = P->n;
  hipError_t e = hipSuccess;
  if (P->borrowed) {
    const bool t = P->sizing;
    e = ctx->oprobs.ensure(sizeof(DevOligoProblem) * std::max(n, 1));
    if (e == hipSuccess) e = ctx->oscratch.ensure(std::max<size_t>(P->scratch_cap, 256), t);
    if (e == hipSuccess) e = ctx->opool.ensure(sizeof(uint64_t) * std::max<size_t>(P->pool_cap, 1), t);
    if (e == hipSuccess) e = ctx->opoolctr.ensure(sizeof(unsigned long long));
    P->d_probs = (DevOligoProblem*)ctx->oprobs.p;
    P->d_scratch = (unsigned char*)ctx->oscratch.p;
    P->d_pool = (uint64_t*)ctx->opool.p;
    P->d_pool_counter = (unsigned long long*)ctx->opoolctr.p;
    if (e == hipSuccess && n)
      e = hipMemcpyAsync(P->d_probs, P->ord.data(), sizeof(DevOligoProblem) * n, hipMemcpyHostToDevice, ctx->stream);
    return e;
  }
  for (void** b : {(void**)&P->d_scratch, (void**)&P->d_pool}) {
    if (*b) (void)hipFree(*b);
    *b = nullptr;
  }
  if (!P->d_probs) e = hipMalloc(&P->d_probs, sizeof(DevOligoProblem) * std::max(n, 1));
  if (e == hipSuccess) e = hipMalloc(&P->d_scratch, std::max<size_t>(P->scratch_cap, 256));
  if (e == hipSuccess) e = hipMalloc(&P->d_pool, sizeof(uint64_t) * std::max<size_t>(P->pool_cap, 1));
  if (e == hipSuccess && !P->d_pool_counter) e = hipMalloc(&P->d_pool_counter, sizeof(unsigned long long));
  if (e == hipSuccess && n)
    e = hipMemcpy(P->d_probs, P->ord.data(), sizeof(DevOligoProblem) * n, hipMemcpyHostToDevice);
  return e;
}

static int oligo_plan_build(gmapdp_ctx* ctx, const gmapdp_oligo_problem* problems, int n, const char* qseq_uc,
                            size_t qbytes, gmapdp_oligo_plan** plan, bool borrow, bool sizing = false) {
  if (!ctx || !plan || n < 0 || (n > 0 && (!problems || !qseq_uc))) return GMAPDP_EINVAL;
  *plan = nullptr;
  if (!ctx->d_genome) return GMAPDP_ENOGENOME;
  (void)hipSetDevice(ctx->device);
  std::vector<DevOligoProblem> dev(n);
  std::vector<size_t> slots(n), tcap(n), dcap(n);
  size_t toff = 0;
  static const int kBuckets[] = {1024, 2048, 4096, 8192, 16384};  // launch classes by LDS
  std::map<int, std::vector<int>> classes;
  const char* ev = std::getenv("GMAPDP_OLIGO_POOL_SLOTS");  // tests: a small pool forces the sequential walk
  // each query's distinct 8-mers (plan_threads() host threads: the sweep over a 10 000-read block's 15 850
  // queries was most of a stage-2 plan's host time), and the first problem the engine rejects
  std::vector<int> distinct(n, 0);
  std::vector<const char*> rej(n, nullptr);
  const int T = plan_threads((size_t)n * 128);
  plan_parallel((size_t)n, T, [&](size_t lo, size_t hi, int) {
    std::vector<uint32_t> bm(2048, 0u);
    for (size_t i = lo; i < hi; i++) {
      const gmapdp_oligo_problem& p = problems[i];
      if (p.querylength <= 8) {
        rej[i] = "stage-2 seeding needs querylength > 8 (Oligoindex_set_inquery)";
        continue;
      }
      if (p.qoff < 0 || (size_t)p.qoff + (size_t)p.querylength > qbytes) {
        rej[i] = "query outside the arena";
        continue;
      }
      distinct[i] = oligo_distinct(qseq_uc + p.qoff, p.querylength, bm);
    }
  });
  for (int i = 0; i < n; i++) {
    const gmapdp_oligo_problem& p = problems[i];
    if (rej[i]) return bad(ctx, rej[i]);
    const uint64_t win = oligo_window(p);
    if (win > 0) {  // the last 8-mer start's half-word and the one after it (window8)
      const uint64_t lpl = (uint64_t)p.chroffset + p.chrend + (p.plusp ? 0 : 1) - 8;
      const uint64_t h = (lpl >> 4) + 1;
      if (3 * (h >> 1) + 1 >= ctx->genome_words) return bad(ctx, "stage-2 window past the genome");
    }
    const int U = distinct[i];
    if (U > kOligoMaxDistinct) return bad(ctx, "query with more than 16384 distinct 8-mers");
    int umax = kBuckets[0];
    for (int b : kBuckets)
      if (U <= b) { umax = b; break; }
    DevOligoProblem& d = dev[i];
    std::memset(&d, 0, sizeof(d));
    d.qoff = p.qoff;
    d.querylength = p.querylength;
    d.chrstart = p.chrstart;
    d.chrend = p.chrend;
    d.chroffset = p.chroffset;
    d.chrhigh = p.chrhigh;
    d.plusp = p.plusp ? 1 : 0;
    d.minor = p.minor ? 1 : 0;
    d.umax = umax;
    d.index = i;
    tcap[i] = oligo_table_cap(p);
    dcap[i] = oligo_diag_cap(p);
    toff += tcap[i];
    // hits ~ the query's 8-mers once (the locus) plus the window's random matches (4^-8 per position each)
    const size_t est = (size_t)p.querylength * (2 + (size_t)(win >> 15)) + 256;
    slots[i] = 3 * std::min<size_t>(oligo_table_cap(p), est);
    // launch class: (umax, 32-bit counters); 16-bit counters when no count can reach 2^16
    classes[2 * umax + (win >= 65536 ? 1 : 0)].push_back(i);
  }
  gmapdp_oligo_plan* P = new gmapdp_oligo_plan();
  P->n = n;
  P->split = borrow;
  P->borrowed = borrow || sizing;
  P->sizing = sizing;
  P->ord.reserve(n);
  for (auto& kv : classes)
    for (int i : kv.second) {
      P->ord.push_back(dev[i]);
      P->keys.push_back(kv.first);
    }
  // (a sizing run keeps no sequential-walk region -- ~70 % of its scratch, the difference between one launch
  // and four for a 10 000-read block; a call that exhausts its chunk's event pool there reports overflow, and
  // the re-layout gives it the diagonal arena's upper bound instead of a measured count)
  oligo_layout(P, slots, !sizing, tcap, dcap, sizing);
  // (the kernels' mappings are relative to each problem's table_offset: the arena may pass 2^31 entries;
  // the public seeding API, whose mappings are absolute 32-bit indexes, checks its own total)
  (void)toff;
  if (ev) P->pool_cap = std::strtoull(ev, nullptr, 10);  // per chunk
  const hipError_t e = oligo_buffers(ctx, P);
  if (e != hipSuccess) {
    oligo_plan_free(P);
    return fail(ctx, GMAPDP_ENOMEM, "oligo plan: %s", e);
  }
  *plan = P;
  return GMAPDP_OK;
}

// After a measured run (the stage-2 plan's sizing run): every arena laid out from what the run wrote.  The
// table holds at most totalpositions entries per problem (each distinct 8-mer's hits, counted at least once
// over the query positions), the diagonal arena exactly ndiagonals records, the pool exactly 3 slots per hit
// (so no problem takes the sequential walk and no fallback region is kept); a rerun seeds the same way.
static hipError_t oligo_plan_relayout(gmapdp_ctx* ctx, gmapdp_oligo_plan* P, const gmapdp_oligo_problem* problems,
                                      const gmapdp_oligo_result* ores, const int32_t* nhits) {
  const int n = P->n;
  std::vector<size_t> slots(n), tcap(n), dcap(n), hcap(n);
  for (int i = 0; i < n; i++) {
    const size_t tp = (size_t)std::max(ores[i].totalpositions, 0);
    tcap[i] = std::min<size_t>(oligo_table_cap(problems[i]), tp);
    dcap[i] = ores[i].oned_matrix_p < 0 ? oligo_diag_cap(problems[i]) : (size_t)std::max(ores[i].ndiagonals, 0);
    slots[i] = 3 * tp;
    hcap[i] = (size_t)std::max(nhits[i], 0);
  }
  // 16-bit counters wherever the measured hit list is shorter than 2^16: a counter counts hits of its 8-mer
  // and a table offset sums wrapped counts, both bounded by the list's length (a 214-kb window: ~8 200).
  // The 32-bit class (chosen from the window alone) needs 8 B of LDS per distinct 8-mer, the 16-bit one 4:
  // for a 2-kb read 20 instead of 28 KB, 8 waves per CU instead of 5.
  {
    std::vector<int> key(n), idx(n);
    for (int k = 0; k < n; k++) {
      const int i = P->ord[k].index;
      key[k] = (P->keys[k] & 1) && nhits[i] >= 0 && nhits[i] < 65536 ? P->keys[k] - 1 : P->keys[k];
      idx[k] = k;
    }
    std::stable_sort(idx.begin(), idx.end(), [&](int a, int b) { return key[a] < key[b]; });
    std::vector<DevOligoProblem> ord(n);
    std::vector<int> keys(n);
    for (int k = 0; k < n; k++) {
      ord[k] = P->ord[idx[k]];
      keys[k] = key[idx[k]];
    }
    P->ord.swap(ord);
    P->keys.swap(keys);
  }
  // the hit lists sized as measured (a few % of a 214-kb window), so one launch holds most of a plan
  oligo_layout(P, slots, false, tcap, dcap, false, &hcap);
  if (P->borrowed) {  // the sizing run's borrowed buffers stay the context's; the plan allocates its own
    P->borrowed = P->sizing = false;
    P->d_probs = nullptr;
    P->d_scratch = nullptr;
    P->d_pool = nullptr;
    P->d_pool_counter = nullptr;
    P->d_nhits = nullptr;
  }
  return oligo_buffers(ctx, P);
}

extern "C" {

int gmapdp_oligo_plan_create(gmapdp_ctx* ctx, const gmapdp_oligo_problem* problems, int n, const char* qseq_uc,
                             size_t qbytes, gmapdp_oligo_plan** plan) {
  return oligo_plan_build(ctx, problems, n, qseq_uc, qbytes, plan, false);
}

// The device mappings are relative to each problem's table_offset; the host-array API hands out absolute
// 32-bit indexes into `positions` (the reference's mappings[q] pointers), so its table stays below 2^31.
static void oligo_absolute_mappings(const gmapdp_oligo_problem* problems, int n, const gmapdp_oligo_result* res,
                                    int32_t* mappings) {
  for (int i = 0; i < n; i++) {
    const int32_t t = (int32_t)res[i].table_offset;
    int32_t* m = mappings + problems[i].qoff;
    for (int q = 0; q < problems[i].querylength; q++)
      if (m[q] >= 0) m[q] += t;
  }
}

size_t gmapdp_oligo_plan_positions_capacity(const gmapdp_oligo_plan* plan) { return plan ? plan->table_cap : 0; }
size_t gmapdp_oligo_plan_diagonal_capacity(const gmapdp_oligo_plan* plan) { return plan ? plan->diag_cap : 0; }
int gmapdp_oligo_plan_nlaunches(const gmapdp_oligo_plan* plan) { return plan ? (int)plan->launches.size() : 0; }
void gmapdp_oligo_plan_destroy(gmapdp_oligo_plan* plan) { oligo_plan_free(plan); }

int gmapdp_oligo_plan_run(gmapdp_ctx* ctx, const gmapdp_oligo_plan* plan, const char* d_qseq_uc,
                          gmapdp_oligo_result* d_results, int32_t* d_npositions, int32_t* d_mappings,
                          uint32_t* d_positions, int32_t* d_diagonals, void* stream) {
  if (!ctx || !plan) return GMAPDP_EINVAL;
  if (plan->n == 0) return GMAPDP_OK;
  (void)hipSetDevice(ctx->device);
  hipStream_t s = stream ? (hipStream_t)stream : ctx->stream;
  for (size_t li = 0; li < plan->launches.size(); li++) {
    // the chunks reuse one scratch and one pool, in stream order
    if (hipMemsetAsync(plan->d_pool_counter, 0, sizeof(unsigned long long), s) != hipSuccess)
      return fail(ctx, GMAPDP_ELAUNCH, "oligo pool reset: %s", hipGetLastError());
    const int key = plan->umax[li];
    const hipError_t e =
        !plan->split
            ? launch_oi(key & 1, plan->launches[li].second, lds_bytes_oi(key >> 1, key & 1), s,
                        plan->d_probs + plan->launches[li].first, ctx->d_genome, d_qseq_uc, plan->d_scratch,
                        d_results, d_npositions, d_mappings, d_positions, d_diagonals, plan->d_pool,
                        plan->d_pool_counter, plan->pool_cap, plan->d_nhits)
            : launch_oi_split(plan->launches[li].second, key >> 1, s, plan->d_probs + plan->launches[li].first,
                              ctx->d_genome, d_qseq_uc, plan->d_scratch, d_results, d_npositions, d_mappings,
                              d_positions, d_diagonals, plan->d_pool, plan->d_pool_counter, plan->pool_cap);
    if (e != hipSuccess) return fail(ctx, GMAPDP_ELAUNCH, "oligo launch: %s", e);
  }
  return GMAPDP_OK;
}

int gmapdp_oligo_mappings_batch(gmapdp_ctx* ctx, const gmapdp_oligo_problem* problems, int n, const char* qseq_uc,
                                size_t qbytes, gmapdp_oligo_result* results, int32_t* npositions, int32_t* mappings,
                                uint32_t* positions, size_t positions_capacity, int32_t* diagonals,
                                size_t diagonal_capacity) {
  if (!ctx || n < 0 || (n > 0 && (!problems || !results || !qseq_uc || !npositions || !mappings)))
    return GMAPDP_EINVAL;
  if (!ctx->d_genome) return GMAPDP_ENOGENOME;
  if (n == 0) return GMAPDP_OK;
  {
    // npositions / mappings are written per problem at its query slice [qoff, qoff + querylength), and the
    // mappings turned absolute by adding that problem's table offset: two problems on overlapping slices
    // would overwrite each other's outputs (and have the offset added twice), so they are refused.
    std::vector<std::pair<int64_t, int64_t>> sl(n);
    for (int i = 0; i < n; i++) sl[i] = {problems[i].qoff, (int64_t)problems[i].qoff + problems[i].querylength};
    std::sort(sl.begin(), sl.end());
    for (int i = 1; i < n; i++)
      if (sl[i].first < sl[i - 1].second) return bad(ctx, "stage-2 seeding: two problems share query slots");
  }
  gmapdp_oligo_plan* plan = nullptr;
  int rc = oligo_plan_build(ctx, problems, n, qseq_uc, qbytes, &plan, true);
  if (rc) return rc;
  const size_t toff = plan->table_cap, doff = plan->diag_cap;
  if (toff > 0x7fffffffull) {  // absolute 32-bit mappings
    oligo_plan_free(plan);
    return bad(ctx, "stage-2 seeding: table arena beyond 2^31 entries (split the batch)");
  }
  if (toff > positions_capacity || doff > diagonal_capacity || (toff && !positions) || (doff && !diagonals)) {
    oligo_plan_free(plan);
    return bad(ctx, "positions or diagonal arena too small");
  }
  hipError_t e = ctx->oresults.ensure(sizeof(gmapdp_oligo_result) * n);
  if (e == hipSuccess) e = ctx->onpos.ensure(sizeof(int32_t) * qbytes);
  if (e == hipSuccess) e = ctx->omap.ensure(sizeof(int32_t) * qbytes);
  if (e == hipSuccess) e = ctx->otable.ensure(sizeof(uint32_t) * std::max<size_t>(toff, 1));
  if (e == hipSuccess) e = ctx->odiag.ensure(4 * sizeof(int32_t) * std::max<size_t>(doff, 1));
  if (e == hipSuccess) e = ctx->qseq_uc.ensure(qbytes);
  hipStream_t s = ctx->stream;
  if (e == hipSuccess) e = hipMemcpyAsync(ctx->qseq_uc.p, qseq_uc, qbytes, hipMemcpyHostToDevice, s);
  if (e == hipSuccess) e = hipMemsetAsync(ctx->onpos.p, 0, sizeof(int32_t) * qbytes, s);
  if (e == hipSuccess) e = hipMemsetAsync(ctx->omap.p, 0xff, sizeof(int32_t) * qbytes, s);
  if (e != hipSuccess) {
    oligo_plan_free(plan);
    return fail(ctx, GMAPDP_ENOMEM, "oligo buffers: %s", e);
  }
  rc = gmapdp_oligo_plan_run(ctx, plan, (const char*)ctx->qseq_uc.p, (gmapdp_oligo_result*)ctx->oresults.p,
                             (int32_t*)ctx->onpos.p, (int32_t*)ctx->omap.p, (uint32_t*)ctx->otable.p,
                             (int32_t*)ctx->odiag.p, nullptr);
  if (rc) {
    (void)ctx_sync(ctx, s);
    oligo_plan_free(plan);
    return rc;
  }
  e = hipMemcpyAsync(results, ctx->oresults.p, sizeof(gmapdp_oligo_result) * n, hipMemcpyDeviceToHost, s);
  if (e == hipSuccess) e = hipMemcpyAsync(npositions, ctx->onpos.p, sizeof(int32_t) * qbytes, hipMemcpyDeviceToHost, s);
  if (e == hipSuccess) e = hipMemcpyAsync(mappings, ctx->omap.p, sizeof(int32_t) * qbytes, hipMemcpyDeviceToHost, s);
  if (e == hipSuccess && toff)
    e = hipMemcpyAsync(positions, ctx->otable.p, sizeof(uint32_t) * toff, hipMemcpyDeviceToHost, s);
  if (e == hipSuccess && doff)
    e = hipMemcpyAsync(diagonals, ctx->odiag.p, 4 * sizeof(int32_t) * doff, hipMemcpyDeviceToHost, s);
  if (e == hipSuccess) e = ctx_sync(ctx, s);
  oligo_plan_free(plan);
  if (e != hipSuccess) return fail(ctx, GMAPDP_ELAUNCH, "oligo execution: %s", e);
  oligo_absolute_mappings(problems, n, results, mappings);
  return GMAPDP_OK;
}

}  // extern "C"

// ---------------------------------------------------------------------------
// Stage2_compute: seeding (oi_kernel + oi_map_kernel) then chaining (s2c_kernel)
// on the device; one synchronous batch.
// ---------------------------------------------------------------------------
extern "C" int gmapdp_stage2_batch(gmapdp_ctx* ctx, const gmapdp_stage2_problem* problems, int n, const char* qseq,
                                   const char* qseq_uc, size_t qbytes, gmapdp_stage2_result* results,
                                   gmapdp_path* paths, size_t path_cap, gmapdp_path_pair* pairs, size_t pair_cap,
                                   size_t* paths_needed, size_t* pairs_needed) {
  if (!ctx || n < 0 || (n > 0 && (!problems || !results || !qseq || !qseq_uc))) return GMAPDP_EINVAL;
  if (paths_needed) *paths_needed = 0;
  if (pairs_needed) *pairs_needed = 0;
  if (!ctx->d_genome) return GMAPDP_ENOGENOME;
  if (n == 0) return GMAPDP_OK;
  (void)hipSetDevice(ctx->device);
  std::vector<gmapdp_oligo_problem> op(n);
  std::vector<DevStage2Problem> dp(n);
  for (int i = 0; i < n; i++) {
    const gmapdp_stage2_problem& p = problems[i];
    if (p.maxintronlen < 0) return bad(ctx, "stage 2: negative maxintronlen");
    op[i].qoff = p.qoff;
    op[i].querylength = p.querylength;
    op[i].chrstart = p.chrstart;
    op[i].chrend = p.chrend;
    op[i].chroffset = p.chroffset;
    op[i].chrhigh = p.chrhigh;
    op[i].plusp = p.plusp ? 1 : 0;
    op[i].minor = 0;  // Stage2_compute takes oligoindices_major (gmap.c:1211)
    DevStage2Problem& d = dp[i];
    d.qoff = p.qoff;
    d.querylength = p.querylength;
    d.chrstart = p.chrstart;
    d.chrend = p.chrend;
    d.chroffset = p.chroffset;
    d.chrhigh = p.chrhigh;
    d.plusp = p.plusp ? 1 : 0;
    d.splicingp = p.splicingp ? 1 : 0;
    d.maxintronlen = (uint32_t)p.maxintronlen;
    d.index = i;
    d.scratch_offset = 0;
  }
  gmapdp_oligo_plan* plan = nullptr;
  int rc = oligo_plan_build(ctx, op.data(), n, qseq_uc, qbytes, &plan, true);
  if (rc) return rc;
  const size_t toff = plan->table_cap, doff = plan->diag_cap;
  hipStream_t s = ctx->stream;
  hipError_t e = ctx->oresults.ensure(sizeof(gmapdp_oligo_result) * n);
  if (e == hipSuccess) e = ctx->onpos.ensure(sizeof(int32_t) * qbytes);
  if (e == hipSuccess) e = ctx->omap.ensure(sizeof(int32_t) * qbytes);
  if (e == hipSuccess) e = ctx->otable.ensure(sizeof(uint32_t) * std::max<size_t>(toff, 1));
  if (e == hipSuccess) e = ctx->odiag.ensure(4 * sizeof(int32_t) * std::max<size_t>(doff, 1));
  if (e == hipSuccess) e = ctx->qseq_uc.ensure(qbytes);
  if (e == hipSuccess) e = ctx->s2qseq.ensure(qbytes);
  if (e == hipSuccess) e = ctx->s2probs.ensure(sizeof(DevStage2Problem) * n);
  if (e == hipSuccess) e = ctx->s2results.ensure(sizeof(gmapdp_stage2_result) * n);
  if (e == hipSuccess) e = ctx->s2counters.ensure(s2_counters_bytes(n));
  if (e == hipSuccess) e = hipMemcpyAsync(ctx->qseq_uc.p, qseq_uc, qbytes, hipMemcpyHostToDevice, s);
  if (e == hipSuccess) e = hipMemcpyAsync(ctx->s2qseq.p, qseq, qbytes, hipMemcpyHostToDevice, s);
  if (e == hipSuccess) e = hipMemcpyAsync(ctx->s2probs.p, dp.data(), sizeof(DevStage2Problem) * n, hipMemcpyHostToDevice, s);
  if (e == hipSuccess) e = hipMemsetAsync(ctx->onpos.p, 0, sizeof(int32_t) * qbytes, s);
  if (e == hipSuccess) e = hipMemsetAsync(ctx->omap.p, 0xff, sizeof(int32_t) * qbytes, s);
  if (e != hipSuccess) {
    oligo_plan_free(plan);
    return fail(ctx, GMAPDP_ENOMEM, "stage-2 buffers: %s", e);
  }
  rc = gmapdp_oligo_plan_run(ctx, plan, (const char*)ctx->qseq_uc.p, (gmapdp_oligo_result*)ctx->oresults.p,
                             (int32_t*)ctx->onpos.p, (int32_t*)ctx->omap.p, (uint32_t*)ctx->otable.p,
                             (int32_t*)ctx->odiag.p, nullptr);
  if (rc) {
    (void)ctx_sync(ctx, s);
    oligo_plan_free(plan);
    return rc;
  }
  // the chaining scratch is sized exactly from the seeding (totalpositions, ndiagonals per call)
  std::vector<gmapdp_oligo_result> ores(n);
  e = hipMemcpyAsync(ores.data(), ctx->oresults.p, sizeof(gmapdp_oligo_result) * n, hipMemcpyDeviceToHost, s);
  if (e == hipSuccess) e = ctx_sync(ctx, s);
  oligo_plan_free(plan);
  if (e != hipSuccess) return fail(ctx, GMAPDP_ELAUNCH, "stage-2 seeding: %s", e);
  size_t scratch = 0, qsum = 0;
  for (int i = 0; i < n; i++) {
    dp[i].scratch_offset = (int64_t)scratch;
    scratch += scratch_bytes_s2c(problems[i].querylength, ores[i].totalpositions, ores[i].ndiagonals);
    qsum += (size_t)problems[i].querylength;
  }
  e = hipMemcpyAsync(ctx->s2probs.p, dp.data(), sizeof(DevStage2Problem) * n, hipMemcpyHostToDevice, s);
  if (e != hipSuccess) return fail(ctx, GMAPDP_ELAUNCH, "stage-2 descriptors: %s", e);
  size_t pcap = 16 + 2 * (size_t)n, qcap = 64 + 2 * qsum;  // first guesses; grown on overflow
  for (int attempt = 0;; attempt++) {
    e = ctx->s2scratch.ensure(std::max<size_t>(scratch, 256));
    if (e == hipSuccess) e = ctx->s2paths.ensure(sizeof(gmapdp_path) * pcap);
    if (e == hipSuccess) e = ctx->s2pairs.ensure(sizeof(gmapdp_path_pair) * qcap);
    if (e == hipSuccess) e = hipMemsetAsync(ctx->s2counters.p, 0, 4 * sizeof(unsigned long long), s);
    if (e == hipSuccess)
      e = launch_s2c(n, s, (const DevStage2Problem*)ctx->s2probs.p, ctx->d_genome, ctx->genome_words,
                     (const char*)ctx->s2qseq.p, (const char*)ctx->qseq_uc.p, (const gmapdp_oligo_result*)ctx->oresults.p,
                     (const int32_t*)ctx->onpos.p, (const int32_t*)ctx->omap.p, (const uint32_t*)ctx->otable.p,
                     (const int32_t*)ctx->odiag.p, (unsigned char*)ctx->s2scratch.p,
                     (unsigned long long*)ctx->s2counters.p, (unsigned long long)scratch,
                     (gmapdp_stage2_result*)ctx->s2results.p, (gmapdp_path*)ctx->s2paths.p, pcap,
                     (gmapdp_path_pair*)ctx->s2pairs.p, qcap);
    unsigned long long cnt[4] = {0, 0, 0, 0};
    if (e == hipSuccess)
      e = hipMemcpyAsync(results, ctx->s2results.p, sizeof(gmapdp_stage2_result) * n, hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipMemcpyAsync(cnt, ctx->s2counters.p, sizeof(cnt), hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = ctx_sync(ctx, s);
    if (e != hipSuccess) return fail(ctx, GMAPDP_ELAUNCH, "stage-2 chaining: %s", e);
    bool overflow = false;
    for (int i = 0; i < n; i++) {
      if (results[i].status == -3) return bad(ctx, "stage 2: chromosome positions past 2^31");
      overflow |= results[i].status == -2;
    }
    if (!overflow) {
      if (paths_needed) *paths_needed = (size_t)cnt[1];
      if (pairs_needed) *pairs_needed = (size_t)cnt[2];
      if (cnt[1] > path_cap || cnt[2] > pair_cap || (cnt[1] && !paths) || (cnt[2] && !pairs)) return GMAPDP_ESPACE;
      if (cnt[1]) e = hipMemcpyAsync(paths, ctx->s2paths.p, sizeof(gmapdp_path) * cnt[1], hipMemcpyDeviceToHost, s);
      if (e == hipSuccess && cnt[2])
        e = hipMemcpyAsync(pairs, ctx->s2pairs.p, sizeof(gmapdp_path_pair) * cnt[2], hipMemcpyDeviceToHost, s);
      if (e == hipSuccess) e = ctx_sync(ctx, s);
      if (e != hipSuccess) return fail(ctx, GMAPDP_ELAUNCH, "stage-2 copy-out: %s", e);
      return GMAPDP_OK;
    }
    if (attempt >= 8) return fail(ctx, GMAPDP_ENOMEM, "stage-2 output pools keep overflowing%s", hipSuccess);
    pcap = std::max<size_t>(2 * pcap, (size_t)cnt[1] + 16);
    qcap = std::max<size_t>(2 * qcap, (size_t)cnt[2] + 64);
  }
}

// ---------------------------------------------------------------------------
// Dynprog_microexon_int (dynprog_single.c:900): candidate search, then selection + pairs
// (mx_kernel.hip).  Synchronous host-array batches.
// ---------------------------------------------------------------------------
static int mx_upload(gmapdp_ctx* ctx, const gmapdp_microexon_problem* problems, int n, const char* qseq,
                     const char* qseq_uc, size_t qbytes) {
  for (int i = 0; i < n; i++) {
    const gmapdp_microexon_problem& p = problems[i];
    if (p.rlength < 0 || p.qoff < 0 || (size_t)p.qoff + (size_t)p.rlength > qbytes)
      return bad(ctx, "microexon: query slice outside the query arena");
  }
  hipStream_t s = ctx->stream;
  hipError_t e = ctx->mxprobs.ensure(sizeof(gmapdp_microexon_problem) * n);
  if (e == hipSuccess) e = ctx->mxres.ensure(sizeof(gmapdp_microexon_result) * n);
  if (e == hipSuccess) e = ctx->qseq.ensure(std::max<size_t>(qbytes, 1));
  if (e == hipSuccess) e = ctx->qseq_uc.ensure(std::max<size_t>(qbytes, 1));
  if (e == hipSuccess)
    e = hipMemcpyAsync(ctx->mxprobs.p, problems, sizeof(gmapdp_microexon_problem) * n, hipMemcpyHostToDevice, s);
  if (e == hipSuccess && qbytes) e = hipMemcpyAsync(ctx->qseq.p, qseq, qbytes, hipMemcpyHostToDevice, s);
  if (e == hipSuccess && qbytes) e = hipMemcpyAsync(ctx->qseq_uc.p, qseq_uc, qbytes, hipMemcpyHostToDevice, s);
  if (e != hipSuccess) return fail(ctx, GMAPDP_ENOMEM, "microexon buffers: %s", e);
  return GMAPDP_OK;
}

extern "C" size_t gmapdp_microexon_pair_capacity(const gmapdp_microexon_problem* problems, int n) {
  size_t c = 0;
  for (int i = 0; i < n; i++) c += (size_t)std::max(problems[i].rlength, 0) + 2;
  return c;
}

extern "C" int gmapdp_microexon_search(gmapdp_ctx* ctx, const gmapdp_microexon_problem* problems, int n,
                                       const char* qseq, const char* qseq_uc, size_t qbytes,
                                       gmapdp_microexon_result* results, gmapdp_microexon_candidate* candidates,
                                       size_t cand_capacity, size_t* cands_needed) {
  if (!ctx || n < 0 || (n > 0 && (!problems || !results || !qseq || !qseq_uc))) return GMAPDP_EINVAL;
  if (cands_needed) *cands_needed = 0;
  if (!ctx->d_genome) return GMAPDP_ENOGENOME;
  if (n == 0) return GMAPDP_OK;
  (void)hipSetDevice(ctx->device);
  int rc = mx_upload(ctx, problems, n, qseq, qseq_uc, qbytes);
  if (rc) return rc;
  hipStream_t s = ctx->stream;
  size_t cap = std::max<size_t>(ctx->mxcands.cap / sizeof(gmapdp_microexon_candidate), 4096);
  unsigned long long cnt = 0;
  for (int attempt = 0;; attempt++) {
    hipError_t e = ctx->mxcands.ensure(sizeof(gmapdp_microexon_candidate) * cap);
    if (e == hipSuccess) e = ctx->mxcnt.ensure(sizeof(unsigned long long));
    if (e == hipSuccess) e = hipMemsetAsync(ctx->mxcnt.p, 0, sizeof(unsigned long long), s);
    if (e == hipSuccess)
      e = launch_mx_search(n, s, (const gmapdp_microexon_problem*)ctx->mxprobs.p, ctx->d_genome, ctx->genome_words,
                           (const char*)ctx->qseq.p, (const char*)ctx->qseq_uc.p,
                           (gmapdp_microexon_result*)ctx->mxres.p, (gmapdp_microexon_candidate*)ctx->mxcands.p, cap,
                           (unsigned long long*)ctx->mxcnt.p, nullptr);
    if (e == hipSuccess)
      e = hipMemcpyAsync(results, ctx->mxres.p, sizeof(gmapdp_microexon_result) * n, hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipMemcpyAsync(&cnt, ctx->mxcnt.p, sizeof(cnt), hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = ctx_sync(ctx, s);
    if (e != hipSuccess) return fail(ctx, GMAPDP_ELAUNCH, "microexon search: %s", e);
    bool regrow = false;
    for (int i = 0; i < n; i++) regrow |= results[i].cand_offset == -2;
    if (!regrow) break;
    if (attempt >= 8) return fail(ctx, GMAPDP_ENOMEM, "microexon candidate pool keeps overflowing%s", hipSuccess);
    cap = std::max<size_t>(2 * cap, (size_t)cnt + 64);
  }
  // calls with more candidates than the kernel holds in LDS: rerun them into regions of their own
  std::vector<int64_t> direct(n, -1);
  size_t total = (size_t)cnt;
  bool any = false;
  for (int i = 0; i < n; i++)
    if (results[i].cand_offset == -1) {
      direct[i] = (int64_t)total;
      total += (size_t)results[i].ncandidates;
      any = true;
    }
  hipError_t e = hipSuccess;
  if (any) {
    if (total > ctx->mxcands.cap / sizeof(gmapdp_microexon_candidate)) {
      // grow, keeping the candidates already found
      DevBuf keep;
      e = keep.ensure(sizeof(gmapdp_microexon_candidate) * std::max<size_t>(total, 1));
      if (e == hipSuccess && cnt)
        e = hipMemcpyAsync(keep.p, ctx->mxcands.p, sizeof(gmapdp_microexon_candidate) * cnt, hipMemcpyDeviceToDevice, s);
      if (e == hipSuccess) e = ctx_sync(ctx, s);
      if (e == hipSuccess) std::swap(keep.p, ctx->mxcands.p), std::swap(keep.cap, ctx->mxcands.cap);
    }
    if (e == hipSuccess) e = ctx->mxdirect.ensure(sizeof(int64_t) * n);
    if (e == hipSuccess)
      e = hipMemcpyAsync(ctx->mxdirect.p, direct.data(), sizeof(int64_t) * n, hipMemcpyHostToDevice, s);
    if (e == hipSuccess)
      e = launch_mx_search(n, s, (const gmapdp_microexon_problem*)ctx->mxprobs.p, ctx->d_genome, ctx->genome_words,
                           (const char*)ctx->qseq.p, (const char*)ctx->qseq_uc.p,
                           (gmapdp_microexon_result*)ctx->mxres.p, (gmapdp_microexon_candidate*)ctx->mxcands.p,
                           total, (unsigned long long*)ctx->mxcnt.p, (const int64_t*)ctx->mxdirect.p);
    if (e == hipSuccess)
      e = hipMemcpyAsync(results, ctx->mxres.p, sizeof(gmapdp_microexon_result) * n, hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = ctx_sync(ctx, s);
    if (e != hipSuccess) return fail(ctx, GMAPDP_ELAUNCH, "microexon search (large): %s", e);
  }
  if (cands_needed) *cands_needed = total;
  if (total > cand_capacity || (total && !candidates)) return GMAPDP_ESPACE;
  if (total) e = hipMemcpyAsync(candidates, ctx->mxcands.p, sizeof(gmapdp_microexon_candidate) * total,
                                hipMemcpyDeviceToHost, s);
  if (e == hipSuccess) e = ctx_sync(ctx, s);
  if (e != hipSuccess) return fail(ctx, GMAPDP_ELAUNCH, "microexon candidates: %s", e);
  return GMAPDP_OK;
}

extern "C" int gmapdp_microexon_finish(gmapdp_ctx* ctx, const gmapdp_microexon_problem* problems, int n,
                                       const char* qseq, const char* qseq_uc, size_t qbytes,
                                       const gmapdp_microexon_candidate* candidates, const double* cand_probs,
                                       size_t ncands, gmapdp_microexon_result* results, gmapdp_pair* pairs,
                                       size_t pair_capacity) {
  if (!ctx || n < 0 || (n > 0 && (!problems || !results || !qseq || !qseq_uc))) return GMAPDP_EINVAL;
  if (!ctx->d_genome) return GMAPDP_ENOGENOME;
  if (n == 0) return GMAPDP_OK;
  if (ncands && !candidates) return GMAPDP_EINVAL;
  size_t poff = 0;
  std::vector<gmapdp_microexon_result> res(results, results + n);
  for (int i = 0; i < n; i++) {
    if (res[i].ncandidates < 0 || (res[i].ncandidates > 0 && (res[i].cand_offset < 0 ||
                                                              (size_t)res[i].cand_offset + res[i].ncandidates > ncands)))
      return bad(ctx, "microexon: candidates outside the candidate array");
    res[i].pair_offset = (int64_t)poff;
    poff += (size_t)std::max(problems[i].rlength, 0) + 2;
  }
  if (poff > pair_capacity || !pairs) return bad(ctx, "microexon: pair arena too small");
  (void)hipSetDevice(ctx->device);
  // cand_probs NULL: the finish kernel evaluates the candidates' MaxEnt sites on the device
  const double* metab = nullptr;
  if (!cand_probs && !(metab = me_tables(ctx))) return GMAPDP_EINVAL;
  int rc = mx_upload(ctx, problems, n, qseq, qseq_uc, qbytes);
  if (rc) return rc;
  hipStream_t s = ctx->stream;
  hipError_t e = ctx->mxcands.ensure(sizeof(gmapdp_microexon_candidate) * std::max<size_t>(ncands, 1));
  if (e == hipSuccess) e = ctx->mxprobs2.ensure(sizeof(double) * 2 * std::max<size_t>(ncands, 1));
  if (e == hipSuccess) e = ctx->mxpairs.ensure(sizeof(gmapdp_pair) * std::max<size_t>(poff, 1));
  if (e == hipSuccess && ncands)
    e = hipMemcpyAsync(ctx->mxcands.p, candidates, sizeof(gmapdp_microexon_candidate) * ncands, hipMemcpyHostToDevice, s);
  if (e == hipSuccess && ncands && cand_probs)
    e = hipMemcpyAsync(ctx->mxprobs2.p, cand_probs, sizeof(double) * 2 * ncands, hipMemcpyHostToDevice, s);
  if (e == hipSuccess)
    e = hipMemcpyAsync(ctx->mxres.p, res.data(), sizeof(gmapdp_microexon_result) * n, hipMemcpyHostToDevice, s);
  if (e == hipSuccess)
    e = launch_mx_finish(n, s, (const gmapdp_microexon_problem*)ctx->mxprobs.p, ctx->d_genome, ctx->genome_words,
                         (const char*)ctx->qseq.p, (const char*)ctx->qseq_uc.p, ctx->d_cs,
                         (const gmapdp_microexon_candidate*)ctx->mxcands.p,
                         cand_probs ? (const double*)ctx->mxprobs2.p : nullptr, metab,
                         (gmapdp_microexon_result*)ctx->mxres.p, (gmapdp_pair*)ctx->mxpairs.p, nullptr);
  if (e == hipSuccess)
    e = hipMemcpyAsync(results, ctx->mxres.p, sizeof(gmapdp_microexon_result) * n, hipMemcpyDeviceToHost, s);
  if (e == hipSuccess) e = hipMemcpyAsync(pairs, ctx->mxpairs.p, sizeof(gmapdp_pair) * poff, hipMemcpyDeviceToHost, s);
  if (e == hipSuccess) e = ctx_sync(ctx, s);
  if (e != hipSuccess) return fail(ctx, GMAPDP_ELAUNCH, "microexon finish: %s", e);
  return GMAPDP_OK;
}

// The drop-in's dispatcher batch in one round trip (gmapdp_mixed_batch).  One pinned host image and
// one device image hold [inputs | outputs | device-only scratch]: the DP descriptors and launch orders,
// the query arena, the splice probabilities (unless the device evaluates them), the microexon
// searches, finishes and whole calls (the finishes' results, which their kernel updates in place, are
// the last input section), then the DP results and pairs, the searches' results and candidate pool,
// the finishes' and whole calls' results and pairs, then the whole calls' candidate pool (never copied).
// One copy up, the kernels, one copy down of the outputs, one wait.  A search that overflows the pool (a
// result with cand_offset -2) or holds more candidates than its LDS (-1) is rerun by
// gmapdp_microexon_search (a whole call then also by gmapdp_microexon_finish).
// GMAPDP_BATCH_TIMING=1: the mixed batches' host phases summed over the process (every dispatcher thread),
// printed at exit -- where a drop-in batch's wall time goes (tools, not the product)
struct BatchTiming {
  std::atomic<unsigned long long> n{0}, calls{0}, ns[5] = {};
  bool on = getenv("GMAPDP_BATCH_TIMING") != nullptr;
  BatchTiming() {
    if (on) atexit([] { print(); });
  }
  static void print();
  static unsigned long long now() {
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return (unsigned long long)t.tv_sec * 1000000000ull + (unsigned long long)t.tv_nsec;
  }
};
static BatchTiming g_bt;
void BatchTiming::print() {
  static const char* names[5] = {"plan", "stage", "gpu (upload + kernels + download + wait)", "unpack", "reruns"};
  const double n = (double)std::max<unsigned long long>(g_bt.n.load(), 1);
  std::fprintf(stderr, "[gmapdp batch timing] batches=%llu calls=%llu", g_bt.n.load(), g_bt.calls.load());
  for (int k = 0; k < 5; k++) std::fprintf(stderr, " %s=%.1fus", names[k], g_bt.ns[k].load() / n / 1e3);
  std::fprintf(stderr, " (mean per batch)\n");
}

extern "C" int gmapdp_mixed_batch(gmapdp_ctx* ctx, const char* qseq, const char* qseq_uc, size_t qbytes,
                                  gmapdp_mixed* m) {
  if (!ctx || !m) return GMAPDP_EINVAL;
  const int nsingle = m->nsingle, nend = m->nend, ngenome = m->ngenome, nxs = m->nsearch, nxf = m->nfinish;
  const int nxw = m->nwhole;
  if (nsingle < 0 || nend < 0 || ngenome < 0 || nxs < 0 || nxf < 0 || nxw < 0) return GMAPDP_EINVAL;
  if ((nsingle && !m->singles) || (nend && !m->ends) || (ngenome && !m->genomes) ||
      (nsingle + nend && !m->results) || (ngenome && !m->genome_results) || (nxs && (!m->searches || !m->search_results)) ||
      (nxf && (!m->finishes || !m->finish_results)) || (nxw && (!m->wholes || !m->whole_results)))
    return GMAPDP_EINVAL;
  m->candidates_needed = 0;
  if (!ctx->d_genome) return GMAPDP_ENOGENOME;
  if (nsingle + nend + ngenome + nxs + nxf + nxw == 0) return GMAPDP_OK;
  if (!qseq || !qseq_uc) return GMAPDP_EINVAL;
  (void)hipSetDevice(ctx->device);
  unsigned long long bt[6] = {g_bt.on ? BatchTiming::now() : 0, 0, 0, 0, 0, 0};
  auto mark = [&](int k) {
    if (g_bt.on) bt[k] = BatchTiming::now();
  };
  // ---- DP plan (as run_batch) ----
  PlanCore plan;
  size_t nsp = 0;
  bool dev_me = false;
  if (nsingle + nend + ngenome) {
    int rc = build_plan(ctx, m->singles, nsingle, m->ends, nend, m->genomes, ngenome, m->results, m->genome_results,
                        plan);
    if (rc) return rc;
    if (plan.pair_capacity > m->pair_capacity || (plan.pair_capacity && !m->pairs)) return bad(ctx, "pair arena too small");
    for (size_t s = 0; s < plan.dev.size(); s++) {
      const int i = plan.dev_problem[s];
      const long lo = i < nsingle ? m->singles[i].qoff : m->ends[i - nsingle].qoff;
      const long len = i < nsingle ? m->singles[i].rlength : m->ends[i - nsingle].rlength;
      if (lo < 0 || (size_t)(lo + len) > qbytes) return bad(ctx, "query slice outside the query arena");
    }
    dev_me = !m->splice_probs && !plan.gdev.empty();
    nsp = plan.gdev.empty() ? 0 : dev_me ? std::max(m->nprobs, gmapdp_genome_prob_entries(m->genomes, ngenome)) : m->nprobs;
    for (size_t s = 0; s < plan.gdev.size(); s++) {
      const gmapdp_genome_problem& g = m->genomes[plan.gdev_problem[s]];
      if (g.qoff < 0 || (size_t)((long)g.qoff + g.rlength) > qbytes) return bad(ctx, "query slice outside the query arena");
      if (g.prob_offset < 0 || (size_t)g.prob_offset + (size_t)g.glengthL + (size_t)g.glengthR > nsp)
        return bad(ctx, "splice probabilities outside the probability arena");
      if ((g.flags & GMAPDP_KNOWN_SITES) &&
          (!m->known_sites || (size_t)g.known_offset + gmapdp_genome_known_bytes(&g) > m->nknown))
        return bad(ctx, "known-site flags outside the known-site arena");
    }
  }
  const int ndev = (int)plan.dev.size(), ngdev = (int)plan.gdev.size();
  // ---- microexon sections (as gmapdp_microexon_search / _finish) ----
  for (int i = 0; i < nxs; i++) {
    const gmapdp_microexon_problem& p = m->searches[i];
    if (p.rlength < 0 || p.qoff < 0 || (size_t)p.qoff + (size_t)p.rlength > qbytes)
      return bad(ctx, "microexon: query slice outside the query arena");
  }
  std::vector<gmapdp_microexon_result> fres(m->finish_results, m->finish_results + nxf);
  size_t fpoff = 0;
  for (int i = 0; i < nxf; i++) {
    const gmapdp_microexon_problem& p = m->finishes[i];
    if (p.rlength < 0 || p.qoff < 0 || (size_t)p.qoff + (size_t)p.rlength > qbytes)
      return bad(ctx, "microexon: query slice outside the query arena");
    if (fres[i].ncandidates < 0 ||
        (fres[i].ncandidates > 0 && (fres[i].cand_offset < 0 ||
                                     (size_t)fres[i].cand_offset + fres[i].ncandidates > m->nfinish_candidates)))
      return bad(ctx, "microexon: candidates outside the candidate array");
    fres[i].pair_offset = (int64_t)fpoff;
    fpoff += (size_t)std::max(p.rlength, 0) + 2;
  }
  if (nxf && (fpoff > m->finish_pair_capacity || !m->finish_pairs)) return bad(ctx, "microexon: pair arena too small");
  if (m->nfinish_candidates && !m->finish_candidates) return GMAPDP_EINVAL;
  std::vector<int64_t> wpoff(nxw);
  size_t wpairs = 0;
  for (int i = 0; i < nxw; i++) {
    const gmapdp_microexon_problem& p = m->wholes[i];
    if (p.rlength < 0 || p.qoff < 0 || (size_t)p.qoff + (size_t)p.rlength > qbytes)
      return bad(ctx, "microexon: query slice outside the query arena");
    wpoff[i] = (int64_t)wpairs;
    wpairs += (size_t)p.rlength + 2;
  }
  if (nxw && (wpairs > m->whole_pair_capacity || !m->whole_pairs)) return bad(ctx, "microexon: whole-call pair arena too small");
  const bool fdev_me = nxf && !m->finish_probs;
  const double* metab = nullptr;
  if ((dev_me || fdev_me || nxw) && !(metab = me_tables(ctx))) return GMAPDP_EINVAL;
  const size_t nfc = nxf ? m->nfinish_candidates : 0;
  mark(1);
  const size_t pool = nxs ? std::max<size_t>(4096, 16 * (size_t)nxs) : 0;   // search candidates
  const size_t wpool = nxw ? std::max<size_t>(4096, 16 * (size_t)nxw) : 0;  // whole calls' candidates
  // ---- one image: inputs, then outputs, then device-only scratch ----
  auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
  size_t o = 0;
  const size_t o_probs = o;   o += al(sizeof(DevProblem) * ndev);
  const size_t o_order = o;   o += al(sizeof(int) * ndev);
  const size_t o_gprobs = o;  o += al(sizeof(DevGenomeProblem) * ngdev);
  const size_t o_gorder = o;  o += al(sizeof(int) * ngdev);
  const size_t o_sprob = o;   o += al(dev_me ? 0 : sizeof(double) * nsp);
  const size_t nkn = (ngdev && m->known_sites) ? m->nknown : 0;
  const size_t o_known = o;   o += al(nkn);
  const size_t o_q = o;       o += al(qbytes);
  const size_t o_quc = o;     o += al(qbytes);
  const size_t o_xs = o;      o += al(sizeof(gmapdp_microexon_problem) * nxs);
  const size_t o_xcnt = o;    o += al(2 * sizeof(unsigned long long));  // search pool, whole-call pool
  const size_t o_xf = o;      o += al(sizeof(gmapdp_microexon_problem) * nxf);
  const size_t o_xfc = o;     o += al(sizeof(gmapdp_microexon_candidate) * nfc);
  const size_t o_xfp = o;     o += al(fdev_me ? 0 : sizeof(double) * 2 * nfc);
  const size_t o_xw = o;      o += al(sizeof(gmapdp_microexon_problem) * nxw);
  const size_t o_xwpoff = o;  o += al(sizeof(int64_t) * nxw);
  const size_t o_xfres = o;   o += al(sizeof(gmapdp_microexon_result) * nxf);  // in and out
  const size_t in_bytes = o_xfres + sizeof(gmapdp_microexon_result) * nxf;
  const size_t r_res = o;     o += al(sizeof(gmapdp_result) * ndev);
  const size_t r_gres = o;    o += al(sizeof(gmapdp_genome_result) * ngdev);
  const size_t r_pairs = o;   o += al(sizeof(gmapdp_pair) * plan.pair_capacity);
  const size_t r_xsres = o;   o += al(sizeof(gmapdp_microexon_result) * nxs);
  const size_t r_xcand = o;   o += al(sizeof(gmapdp_microexon_candidate) * pool);
  const size_t r_xfpairs = o; o += al(sizeof(gmapdp_pair) * fpoff);
  const size_t r_xwres = o;   o += al(sizeof(gmapdp_microexon_result) * nxw);
  const size_t r_xwpairs = o; o += al(sizeof(gmapdp_pair) * wpairs);
  const size_t out_end = o;
  const size_t s_xwcand = o;  o += al(sizeof(gmapdp_microexon_candidate) * wpool);
  const size_t total = o;
  hipError_t e = ctx->hin.ensure(out_end);
  if (e == hipSuccess) e = ctx->din.ensure(total);
  if (e == hipSuccess && dev_me) e = ctx->sprob.ensure(sizeof(double) * nsp);
  if (e != hipSuccess) return fail(ctx, GMAPDP_ENOMEM, "batch buffers: %s", e);
  unsigned char* h = (unsigned char*)ctx->hin.p;
  unsigned char* d = (unsigned char*)ctx->din.p;
  if (ndev) {
    std::memcpy(h + o_probs, plan.dev.data(), sizeof(DevProblem) * ndev);
    std::memcpy(h + o_order, plan.order.data(), sizeof(int) * ndev);
  }
  if (ngdev) {
    std::memcpy(h + o_gprobs, plan.gdev.data(), sizeof(DevGenomeProblem) * ngdev);
    std::memcpy(h + o_gorder, plan.gorder.data(), sizeof(int) * ngdev);
    if (!dev_me) std::memcpy(h + o_sprob, m->splice_probs, sizeof(double) * nsp);
    if (nkn) std::memcpy(h + o_known, m->known_sites, nkn);
  }
  std::memcpy(h + o_q, qseq, qbytes);
  std::memcpy(h + o_quc, qseq_uc, qbytes);
  if (nxs) std::memcpy(h + o_xs, m->searches, sizeof(gmapdp_microexon_problem) * nxs);
  std::memset(h + o_xcnt, 0, 2 * sizeof(unsigned long long));
  if (nxf) {
    std::memcpy(h + o_xf, m->finishes, sizeof(gmapdp_microexon_problem) * nxf);
    std::memcpy(h + o_xfres, fres.data(), sizeof(gmapdp_microexon_result) * nxf);
  }
  if (nfc) {
    std::memcpy(h + o_xfc, m->finish_candidates, sizeof(gmapdp_microexon_candidate) * nfc);
    if (!fdev_me) std::memcpy(h + o_xfp, m->finish_probs, sizeof(double) * 2 * nfc);
  }
  if (nxw) {
    std::memcpy(h + o_xw, m->wholes, sizeof(gmapdp_microexon_problem) * nxw);
    std::memcpy(h + o_xwpoff, wpoff.data(), sizeof(int64_t) * nxw);
  }
  hipStream_t s = ctx->stream;
  mark(2);
  e = hipMemcpyAsync(d, h, in_bytes, hipMemcpyHostToDevice, s);
  if (e != hipSuccess) return fail(ctx, GMAPDP_ENOMEM, "upload: %s", e);
  // (GMAPDP_SMALL_BATCH_STREAMS with a multi-stream context, experiments: the microexon kernels on the last
  // side stream, beside the DP classes)
  static const bool small_streams = getenv("GMAPDP_SMALL_BATCH_STREAMS") != nullptr;
  const bool mxside = small_streams && !ctx->one_stream && (nxs || nxf || nxw);
  hipStream_t ms = s;
  if (mxside) {
    ms = ctx->aux[gmapdp_ctx::kAux - 1];
    e = hipEventRecord(ctx->ev_fork, s);
    if (e == hipSuccess) e = hipStreamWaitEvent(ms, ctx->ev_fork, 0);
    if (e != hipSuccess) return fail(ctx, GMAPDP_ELAUNCH, "mixed batch fork: %s", e);
  }
  if (ndev + ngdev) {
    RunArgs a;
    a.d_probs = (const DevProblem*)(d + o_probs);
    a.d_order = (const int*)(d + o_order);
    a.d_gprobs = (const DevGenomeProblem*)(d + o_gprobs);
    a.d_gorder = (const int*)(d + o_gorder);
    a.d_q = (const char*)(d + o_q);
    a.d_quc = (const char*)(d + o_quc);
    a.d_sprob = dev_me ? (const double*)ctx->sprob.p : (const double*)(d + o_sprob);
    a.d_metab = dev_me ? metab : nullptr;
    a.d_known = nkn ? (const uint8_t*)(d + o_known) : nullptr;
    a.d_results = (gmapdp_result*)(d + r_res);
    a.d_gresults = (gmapdp_genome_result*)(d + r_gres);
    a.d_pairs = (gmapdp_pair*)(d + r_pairs);
    const int rc = run_plan(ctx, plan, a, s);
    if (rc) return rc;
  }
  unsigned long long* cnt = (unsigned long long*)(d + o_xcnt);
  if (nxs)
    e = launch_mx_search(nxs, ms, (const gmapdp_microexon_problem*)(d + o_xs), ctx->d_genome, ctx->genome_words,
                         (const char*)(d + o_q), (const char*)(d + o_quc), (gmapdp_microexon_result*)(d + r_xsres),
                         (gmapdp_microexon_candidate*)(d + r_xcand), pool, cnt, nullptr);
  if (e == hipSuccess && nxf)
    e = launch_mx_finish(nxf, ms, (const gmapdp_microexon_problem*)(d + o_xf), ctx->d_genome, ctx->genome_words,
                         (const char*)(d + o_q), (const char*)(d + o_quc), ctx->d_cs,
                         (const gmapdp_microexon_candidate*)(d + o_xfc), fdev_me ? nullptr : (const double*)(d + o_xfp),
                         fdev_me ? metab : nullptr, (gmapdp_microexon_result*)(d + o_xfres),
                         (gmapdp_pair*)(d + r_xfpairs), nullptr);
  if (e == hipSuccess && nxw)
    e = launch_mx_search(nxw, ms, (const gmapdp_microexon_problem*)(d + o_xw), ctx->d_genome, ctx->genome_words,
                         (const char*)(d + o_q), (const char*)(d + o_quc), (gmapdp_microexon_result*)(d + r_xwres),
                         (gmapdp_microexon_candidate*)(d + s_xwcand), wpool, cnt + 1, nullptr);
  if (e == hipSuccess && nxw)
    e = launch_mx_finish(nxw, ms, (const gmapdp_microexon_problem*)(d + o_xw), ctx->d_genome, ctx->genome_words,
                         (const char*)(d + o_q), (const char*)(d + o_quc), ctx->d_cs,
                         (const gmapdp_microexon_candidate*)(d + s_xwcand), nullptr, metab,
                         (gmapdp_microexon_result*)(d + r_xwres), (gmapdp_pair*)(d + r_xwpairs),
                         (const int64_t*)(d + o_xwpoff));
  if (e == hipSuccess && mxside) {
    e = hipEventRecord(ctx->ev_join[gmapdp_ctx::kAux - 1], ms);
    if (e == hipSuccess) e = hipStreamWaitEvent(s, ctx->ev_join[gmapdp_ctx::kAux - 1], 0);
  }
  if (e == hipSuccess) e = hipMemcpyAsync(h + o_xfres, d + o_xfres, out_end - o_xfres, hipMemcpyDeviceToHost, s);
  if (e == hipSuccess) e = ctx_sync(ctx, s);
  if (e != hipSuccess) return fail(ctx, GMAPDP_ELAUNCH, "mixed batch: %s", e);
  mark(3);
  // ---- unpack ----
  const gmapdp_result* dres = (const gmapdp_result*)(h + r_res);
  const gmapdp_genome_result* gres = (const gmapdp_genome_result*)(h + r_gres);
  if (plan.pair_capacity) std::memcpy(m->pairs, h + r_pairs, sizeof(gmapdp_pair) * plan.pair_capacity);
  for (int k = 0; k < ndev; k++) m->results[plan.dev_problem[k]] = dres[k];
  for (int k = 0; k < ngdev; k++) m->genome_results[plan.gdev_problem[k]] = gres[k];
  if (nxf) {
    std::memcpy(m->finish_results, h + o_xfres, sizeof(gmapdp_microexon_result) * nxf);
    std::memcpy(m->finish_pairs, h + r_xfpairs, sizeof(gmapdp_pair) * fpoff);
  }
  if (nxw) {
    std::memcpy(m->whole_results, h + r_xwres, sizeof(gmapdp_microexon_result) * nxw);
    std::memcpy(m->whole_pairs, h + r_xwpairs, sizeof(gmapdp_pair) * wpairs);
  }
  // (the buffers of the reruns below are the context's own; the image above is consumed)
  mark(4);
  struct BtDone {  // the reruns' time, and the sums (on every return below)
    unsigned long long* bt;
    int ncalls;
    ~BtDone() {
      if (!g_bt.on) return;
      bt[5] = BatchTiming::now();
      g_bt.n++;
      g_bt.calls += (unsigned long long)ncalls;
      for (int k = 0; k < 5; k++) g_bt.ns[k] += bt[k + 1] - bt[k];
    }
  } bt_done{bt, nsingle + nend + ngenome + nxs + nxf + nxw};
  int rc = GMAPDP_OK;
  if (nxs) {
    const gmapdp_microexon_result* xr = (const gmapdp_microexon_result*)(h + r_xsres);
    bool rerun = false;
    size_t used = 0;
    for (int i = 0; i < nxs; i++) {
      rerun |= xr[i].cand_offset < 0 && xr[i].ncandidates > 0;  // -2: pool overflow, -1: past the LDS list
      if (xr[i].cand_offset >= 0) used = std::max(used, (size_t)xr[i].cand_offset + (size_t)xr[i].ncandidates);
    }
    if (rerun) {
      size_t need = 0;
      rc = gmapdp_microexon_search(ctx, m->searches, nxs, qseq, qseq_uc, qbytes, m->search_results, m->candidates,
                                   m->candidate_capacity, &need);
      m->candidates_needed = need;
    } else {
      std::memcpy(m->search_results, xr, sizeof(gmapdp_microexon_result) * nxs);
      m->candidates_needed = used;
      if (used > m->candidate_capacity || (used && !m->candidates)) rc = GMAPDP_ESPACE;
      else if (used) std::memcpy(m->candidates, h + r_xcand, sizeof(gmapdp_microexon_candidate) * used);
    }
  }
  // whole calls whose candidates did not fit (finish left npairs -2): search + finish again, alone -- also
  // when the searches section ran out of candidate room (GMAPDP_ESPACE leaves every other section filled)
  std::vector<int> redo;
  for (int i = 0; i < nxw; i++)
    if (m->whole_results[i].npairs == -2) redo.push_back(i);
  if (!redo.empty() && (rc == GMAPDP_OK || rc == GMAPDP_ESPACE)) {
    std::vector<gmapdp_microexon_problem> P(redo.size());
    for (size_t k = 0; k < redo.size(); k++) P[k] = m->wholes[redo[k]];
    const int nr = (int)redo.size();
    std::vector<gmapdp_microexon_result> R(nr);
    size_t need = 0;
    std::vector<gmapdp_microexon_candidate> C(4096);
    int r2 = gmapdp_microexon_search(ctx, P.data(), nr, qseq, qseq_uc, qbytes, R.data(), C.data(), C.size(), &need);
    if (r2 == GMAPDP_ESPACE) {
      C.resize(need);
      r2 = gmapdp_microexon_search(ctx, P.data(), nr, qseq, qseq_uc, qbytes, R.data(), C.data(), C.size(), &need);
    }
    std::vector<gmapdp_pair> pp(gmapdp_microexon_pair_capacity(P.data(), nr));
    if (r2 == GMAPDP_OK)
      r2 = gmapdp_microexon_finish(ctx, P.data(), nr, qseq, qseq_uc, qbytes, C.data(), nullptr, need, R.data(), pp.data(),
                                   pp.size());
    if (r2 != GMAPDP_OK) return r2;
    for (int k = 0; k < nr; k++) {
      const int i = redo[k];
      gmapdp_microexon_result x = R[k];
      x.pair_offset = wpoff[i];
      if (x.npairs > 0)
        std::memcpy(m->whole_pairs + wpoff[i], pp.data() + R[k].pair_offset, sizeof(gmapdp_pair) * (size_t)x.npairs);
      m->whole_results[i] = x;
    }
  }
  return rc;
}

// Device-resident microexon plan (bench / pipelined callers): the search is run once at plan time to
// size every call's candidate region exactly, so the plan's runs write candidates straight to fixed
// regions (no atomics, deterministic offsets) and the caller's probabilities line up with them.
struct gmapdp_microexon_plan {
  int n = 0;
  size_t ncands = 0, npairs = 0;
  gmapdp_microexon_problem* d_probs = nullptr;
  int64_t* d_direct = nullptr;
  int64_t* d_poff = nullptr;
  gmapdp_microexon_candidate* d_cands = nullptr;
  unsigned long long* d_counter = nullptr;
};

static void mx_plan_free(gmapdp_microexon_plan* P) {
  if (!P) return;
  for (void* b : {(void*)P->d_probs, (void*)P->d_direct, (void*)P->d_poff, (void*)P->d_cands, (void*)P->d_counter})
    if (b) (void)hipFree(b);
  delete P;
}

extern "C" int gmapdp_microexon_plan_create(gmapdp_ctx* ctx, const gmapdp_microexon_problem* problems, int n,
                                            const char* qseq, const char* qseq_uc, size_t qbytes,
                                            gmapdp_microexon_plan** plan) {
  if (!ctx || !plan || n < 0 || (n > 0 && (!problems || !qseq || !qseq_uc))) return GMAPDP_EINVAL;
  *plan = nullptr;
  if (!ctx->d_genome) return GMAPDP_ENOGENOME;
  std::vector<gmapdp_microexon_result> res(std::max(n, 1));
  size_t need = 0;
  int rc = gmapdp_microexon_search(ctx, problems, n, qseq, qseq_uc, qbytes, res.data(), nullptr, 0, &need);
  if (rc && rc != GMAPDP_ESPACE) return rc;
  std::vector<int64_t> direct(std::max(n, 1)), poff(std::max(n, 1));
  size_t c = 0, q = 0;
  for (int i = 0; i < n; i++) {
    direct[i] = (int64_t)c;
    c += (size_t)res[i].ncandidates;
    poff[i] = (int64_t)q;
    q += (size_t)std::max(problems[i].rlength, 0) + 2;
  }
  gmapdp_microexon_plan* P = new gmapdp_microexon_plan();
  P->n = n;
  P->ncands = c;
  P->npairs = q;
  hipError_t e = hipMalloc(&P->d_probs, sizeof(gmapdp_microexon_problem) * std::max(n, 1));
  if (e == hipSuccess) e = hipMalloc(&P->d_direct, sizeof(int64_t) * std::max(n, 1));
  if (e == hipSuccess) e = hipMalloc(&P->d_poff, sizeof(int64_t) * std::max(n, 1));
  if (e == hipSuccess) e = hipMalloc(&P->d_cands, sizeof(gmapdp_microexon_candidate) * std::max<size_t>(c, 1));
  if (e == hipSuccess) e = hipMalloc(&P->d_counter, sizeof(unsigned long long));
  if (e == hipSuccess && n)
    e = hipMemcpy(P->d_probs, problems, sizeof(gmapdp_microexon_problem) * n, hipMemcpyHostToDevice);
  if (e == hipSuccess && n) e = hipMemcpy(P->d_direct, direct.data(), sizeof(int64_t) * n, hipMemcpyHostToDevice);
  if (e == hipSuccess && n) e = hipMemcpy(P->d_poff, poff.data(), sizeof(int64_t) * n, hipMemcpyHostToDevice);
  if (e != hipSuccess) {
    mx_plan_free(P);
    return fail(ctx, GMAPDP_ENOMEM, "microexon plan: %s", e);
  }
  *plan = P;
  return GMAPDP_OK;
}

extern "C" size_t gmapdp_microexon_plan_candidates(const gmapdp_microexon_plan* plan) { return plan ? plan->ncands : 0; }
extern "C" size_t gmapdp_microexon_plan_pair_capacity(const gmapdp_microexon_plan* plan) {
  return plan ? plan->npairs : 0;
}

extern "C" int gmapdp_microexon_plan_run(gmapdp_ctx* ctx, const gmapdp_microexon_plan* plan, const char* d_qseq,
                                         const char* d_qseq_uc, const double* d_cand_probs,
                                         gmapdp_microexon_result* d_results, gmapdp_pair* d_pairs, int what,
                                         void* stream) {
  if (!ctx || !plan || !d_results) return GMAPDP_EINVAL;
  if (plan->n == 0) return GMAPDP_OK;
  if ((what & 2) && !d_pairs) return GMAPDP_EINVAL;
  (void)hipSetDevice(ctx->device);
  // d_cand_probs NULL: the finish evaluates the candidates' MaxEnt sites on the device
  const double* metab = nullptr;
  if ((what & 2) && !d_cand_probs && !(metab = me_tables(ctx))) return GMAPDP_EINVAL;
  hipStream_t s = stream ? (hipStream_t)stream : ctx->stream;
  hipError_t e = hipSuccess;
  if (what & 1)
    e = launch_mx_search(plan->n, s, plan->d_probs, ctx->d_genome, ctx->genome_words, d_qseq, d_qseq_uc,
                         d_results, plan->d_cands, plan->ncands, plan->d_counter, plan->d_direct);
  if (e == hipSuccess && (what & 2))
    e = launch_mx_finish(plan->n, s, plan->d_probs, ctx->d_genome, ctx->genome_words, d_qseq, d_qseq_uc, ctx->d_cs,
                         plan->d_cands, d_cand_probs, metab, d_results, d_pairs, plan->d_poff);
  if (e != hipSuccess) return fail(ctx, GMAPDP_ELAUNCH, "microexon plan launch: %s", e);
  return GMAPDP_OK;
}

extern "C" const gmapdp_microexon_candidate* gmapdp_microexon_plan_device_candidates(const gmapdp_microexon_plan* plan) {
  return plan ? plan->d_cands : nullptr;
}

extern "C" void gmapdp_microexon_plan_destroy(gmapdp_microexon_plan* plan) { mx_plan_free(plan); }

// Test instrumentation: the chaining scratch of the last gmapdp_stage2_batch (its layout is
// s2_scratch in s2c_kernel.hip; for a one-problem batch it starts at byte 0).
extern "C" int gmapdp_debug_stage2_scratch(gmapdp_ctx* ctx, void* out, size_t bytes) {
  if (!ctx || !out || bytes > ctx->s2scratch.cap) return GMAPDP_EINVAL;
  return hipMemcpy(out, ctx->s2scratch.p, bytes, hipMemcpyDeviceToHost) == hipSuccess ? GMAPDP_OK : GMAPDP_ELAUNCH;
}

// ---------------------------------------------------------------------------
// Stage2_compute, device-resident plan (bench / pipelined callers): the seeding plan plus the chaining
// kernel's pools, sized once by running the seeding at plan time.
// ---------------------------------------------------------------------------
struct gmapdp_stage2_plan {
  int n = 0;
  gmapdp_oligo_plan* oplan = nullptr;
  DevStage2Problem* d_probs = nullptr;
  gmapdp_oligo_result* d_ores = nullptr;
  int32_t *d_npos = nullptr, *d_map = nullptr, *d_diag = nullptr;
  uint32_t* d_table = nullptr;
  unsigned char* d_scratch = nullptr;
  unsigned long long* d_counters = nullptr;
  gmapdp_path* d_paths = nullptr;
  gmapdp_path_pair* d_pairs = nullptr;
  size_t qbytes = 0, scratch = 0, path_cap = 0, pair_cap = 0;
};

static void stage2_plan_free(gmapdp_stage2_plan* p) {
  if (!p) return;
  oligo_plan_free(p->oplan);
  void* bufs[] = {p->d_probs, p->d_ores, p->d_npos, p->d_map, p->d_diag, p->d_table, p->d_scratch, p->d_counters,
                  p->d_paths, p->d_pairs};
  for (void* b : bufs)
    if (b) (void)hipFree(b);
  delete p;
}

static int stage2_plan_launch(gmapdp_ctx* ctx, const gmapdp_stage2_plan* P, const char* d_qseq, const char* d_qseq_uc,
                              gmapdp_stage2_result* d_results, hipStream_t s, bool seed, int chain) {
  if (seed) {
    if (hipMemsetAsync(P->d_npos, 0, sizeof(int32_t) * P->qbytes, s) != hipSuccess)
      return fail(ctx, GMAPDP_ELAUNCH, "stage-2 plan: %s", hipGetLastError());
    int rc = gmapdp_oligo_plan_run(ctx, P->oplan, d_qseq_uc, P->d_ores, P->d_npos, P->d_map, P->d_table, P->d_diag, s);
    if (rc) return rc;
  }
  if (chain) {  // phases: 1 s2a, 2 s2b, 4 s2c (the pools restart with s2a or s2c)
    if ((chain & 5) && hipMemsetAsync(P->d_counters, 0, 4 * sizeof(unsigned long long), s) != hipSuccess)
      return fail(ctx, GMAPDP_ELAUNCH, "stage-2 plan: %s", hipGetLastError());
    hipError_t e = launch_s2c(P->n, s, P->d_probs, ctx->d_genome, ctx->genome_words, d_qseq, d_qseq_uc, P->d_ores,
                              P->d_npos, P->d_map, P->d_table, P->d_diag, P->d_scratch, P->d_counters, P->scratch,
                              d_results, P->d_paths, P->path_cap, P->d_pairs, P->pair_cap, chain);
    if (e != hipSuccess) return fail(ctx, GMAPDP_ELAUNCH, "stage-2 chaining launch: %s", e);
  }
  return GMAPDP_OK;
}

extern "C" {

int gmapdp_stage2_plan_create(gmapdp_ctx* ctx, const gmapdp_stage2_problem* problems, int n, const char* qseq,
                              const char* qseq_uc, size_t qbytes, gmapdp_stage2_plan** plan) {
  if (!ctx || !plan || n <= 0 || !problems || !qseq || !qseq_uc) return GMAPDP_EINVAL;
  *plan = nullptr;
  if (!ctx->d_genome) return GMAPDP_ENOGENOME;
  (void)hipSetDevice(ctx->device);
  std::vector<gmapdp_oligo_problem> op(n);
  std::vector<DevStage2Problem> dp(n);
  size_t qsum = 0;
  for (int i = 0; i < n; i++) {
    const gmapdp_stage2_problem& p = problems[i];
    if (p.maxintronlen < 0) return bad(ctx, "stage 2: negative maxintronlen");
    op[i] = gmapdp_oligo_problem{p.qoff, p.querylength, p.chrstart, p.chrend, p.chroffset, p.chrhigh,
                                 p.plusp ? 1 : 0, 0};
    dp[i] = DevStage2Problem{p.qoff, p.querylength, p.chrstart, p.chrend, p.chroffset, p.chrhigh, p.plusp ? 1 : 0,
                             p.splicingp ? 1 : 0, (uint32_t)p.maxintronlen, i, 0};
    qsum += (size_t)p.querylength;
  }
  gmapdp_stage2_plan* P = new gmapdp_stage2_plan();
  PlanTimer tm("stage2_plan_create");
  P->n = n;
  P->qbytes = qbytes;
  int rc = oligo_plan_build(ctx, op.data(), n, qseq_uc, qbytes, &P->oplan, false, /*sizing*/ true);
  tm.mark("oligo_plan_build");
  if (rc) {
    delete P;
    return rc;
  }
  const size_t toff = P->oplan->table_cap, doff = P->oplan->diag_cap;
  hipError_t e = hipMalloc(&P->d_probs, sizeof(DevStage2Problem) * n);
  if (e == hipSuccess) e = hipMalloc(&P->d_ores, sizeof(gmapdp_oligo_result) * n);
  if (e == hipSuccess) e = hipMalloc(&P->d_npos, sizeof(int32_t) * qbytes);
  if (e == hipSuccess) e = hipMalloc(&P->d_map, sizeof(int32_t) * qbytes);
  // the sizing run's upper-bound arenas: the context's grow-only buffers (see gmapdp_oligo_plan::borrowed)
  auto drop_sizing = [&]() {
    P->d_table = nullptr;
    P->d_diag = nullptr;
    P->oplan->d_nhits = nullptr;
  };
  if (e == hipSuccess) e = ctx->otable.ensure(sizeof(uint32_t) * std::max<size_t>(toff, 1), true);
  if (e == hipSuccess) e = ctx->odiag.ensure(4 * sizeof(int32_t) * std::max<size_t>(doff, 1), true);
  if (e == hipSuccess) e = ctx->onhits.ensure(sizeof(int32_t) * n);
  P->d_table = (uint32_t*)ctx->otable.p;
  P->d_diag = (int32_t*)ctx->odiag.p;
  P->oplan->d_nhits = (int32_t*)ctx->onhits.p;
  if (e == hipSuccess) e = hipMalloc(&P->d_counters, s2_counters_bytes(n));
  if (e == hipSuccess) e = hipMemcpy(P->d_probs, dp.data(), sizeof(DevStage2Problem) * n, hipMemcpyHostToDevice);
  if (e == hipSuccess) e = ctx->qseq_uc.ensure(qbytes);
  if (e == hipSuccess) e = hipMemcpy(ctx->qseq_uc.p, qseq_uc, qbytes, hipMemcpyHostToDevice);
  if (e != hipSuccess) {
    drop_sizing();
    stage2_plan_free(P);
    return fail(ctx, GMAPDP_ENOMEM, "stage-2 plan: %s", e);
  }
  tm.mark("buffers");
  // size the chaining scratch from one seeding run
  rc = stage2_plan_launch(ctx, P, nullptr, (const char*)ctx->qseq_uc.p, nullptr, ctx->stream, true, 0);
  std::vector<gmapdp_oligo_result> ores(n);
  std::vector<int32_t> nhits(n);
  if (!rc) {
    e = hipMemcpyAsync(ores.data(), P->d_ores, sizeof(gmapdp_oligo_result) * n, hipMemcpyDeviceToHost, ctx->stream);
    if (e == hipSuccess)
      e = hipMemcpyAsync(nhits.data(), P->oplan->d_nhits, sizeof(int32_t) * n, hipMemcpyDeviceToHost, ctx->stream);
    if (e == hipSuccess) e = ctx_sync(ctx, ctx->stream);
    if (e != hipSuccess) rc = fail(ctx, GMAPDP_ELAUNCH, "stage-2 plan seeding: %s", e);
  }
  drop_sizing();
  if (rc) {
    stage2_plan_free(P);
    return rc;
  }
  tm.mark("sizing_run");
  // The seeding's arenas were sized from upper bounds (a window's worth of positions and 24 diagonals per
  // query position: 19 GB for 10 000 5-kb reads).  Re-lay them out from this run's measured use
  // (oligo_plan_relayout) so the plan keeps only what its runs write.
  e = oligo_plan_relayout(ctx, P->oplan, op.data(), ores.data(), nhits.data());
  tm.mark("relayout");
  if (e == hipSuccess) e = hipMalloc(&P->d_table, sizeof(uint32_t) * std::max<size_t>(P->oplan->table_cap, 1));
  if (e == hipSuccess) e = hipMalloc(&P->d_diag, 4 * sizeof(int32_t) * std::max<size_t>(P->oplan->diag_cap, 1));
  if (e != hipSuccess) {
    stage2_plan_free(P);
    return fail(ctx, GMAPDP_ENOMEM, "stage-2 plan arenas: %s", e);
  }
  for (int i = 0; i < n; i++) {
    dp[i].scratch_offset = (int64_t)P->scratch;
    // (a call whose sizing run overflowed its event pool measured no diagonals: its arena's upper bound)
    const int nd = ores[i].oned_matrix_p < 0 ? (int)std::min<size_t>(oligo_diag_cap(op[i]), INT32_MAX)
                                             : ores[i].ndiagonals;
    P->scratch += scratch_bytes_s2c(problems[i].querylength, ores[i].totalpositions, nd);
  }
  P->path_cap = 16 + 4 * (size_t)n;
  P->pair_cap = 64 + 3 * qsum;
  e = hipMalloc(&P->d_scratch, std::max<size_t>(P->scratch, 256));
  if (e == hipSuccess) e = hipMemcpy(P->d_probs, dp.data(), sizeof(DevStage2Problem) * n, hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMalloc(&P->d_paths, sizeof(gmapdp_path) * P->path_cap);
  if (e == hipSuccess) e = hipMalloc(&P->d_pairs, sizeof(gmapdp_path_pair) * P->pair_cap);
  tm.mark("pools");
  if (e != hipSuccess) {
    stage2_plan_free(P);
    return fail(ctx, GMAPDP_ENOMEM, "stage-2 plan pools: %s", e);
  }
  *plan = P;
  return GMAPDP_OK;
}

// what: 1 seeding, 2 chaining, 3 both.  d_results: n gmapdp_stage2_result (problem order).  Outputs stay in
// the plan's pools (gmapdp_stage2_plan_outputs); a result with status -2 overflowed them.
int gmapdp_stage2_plan_run(gmapdp_ctx* ctx, const gmapdp_stage2_plan* plan, const char* d_qseq, const char* d_qseq_uc,
                           gmapdp_stage2_result* d_results, int what, void* stream) {
  if (!ctx || !plan || !d_qseq || !d_qseq_uc || !d_results) return GMAPDP_EINVAL;
  (void)hipSetDevice(ctx->device);
  // what: 1 seeding, 2 chaining; or one chaining kernel alone over a previous run's scratch: 4 s2a, 8 s2b, 16 s2c
  const int chain = (what & 2) ? 7 : ((what >> 2) & 7);
  return stage2_plan_launch(ctx, plan, d_qseq, d_qseq_uc, d_results, stream ? (hipStream_t)stream : ctx->stream,
                            (what & 1) != 0, chain);
}

int gmapdp_stage2_plan_seeding_results(gmapdp_ctx* ctx, const gmapdp_stage2_plan* plan, void* stream,
                                       gmapdp_oligo_result* out) {
  if (!ctx || !plan || !out) return GMAPDP_EINVAL;
  (void)hipSetDevice(ctx->device);
  hipStream_t s = stream ? (hipStream_t)stream : ctx->stream;
  hipError_t e = hipMemcpyAsync(out, plan->d_ores, sizeof(gmapdp_oligo_result) * plan->n, hipMemcpyDeviceToHost, s);
  if (e == hipSuccess) e = ctx_sync(ctx, s);
  return e == hipSuccess ? GMAPDP_OK : fail(ctx, GMAPDP_ELAUNCH, "stage-2 seeding results: %s", e);
}

int gmapdp_stage2_plan_outputs(const gmapdp_stage2_plan* plan, gmapdp_path** d_paths, gmapdp_path_pair** d_pairs,
                               unsigned long long** d_counters, size_t* scratch_bytes) {
  if (!plan) return GMAPDP_EINVAL;
  if (d_paths) *d_paths = plan->d_paths;
  if (d_pairs) *d_pairs = plan->d_pairs;
  if (d_counters) *d_counters = plan->d_counters;
  if (scratch_bytes) *scratch_bytes = plan->scratch;
  return GMAPDP_OK;
}

int gmapdp_stage2_plan_fetch(gmapdp_ctx* ctx, const gmapdp_stage2_plan* plan, const gmapdp_stage2_result* d_results,
                             void* stream, gmapdp_stage2_result* results, gmapdp_path* paths, size_t path_cap,
                             gmapdp_path_pair* pairs, size_t pair_cap, size_t* paths_needed, size_t* pairs_needed) {
  if (!ctx || !plan || !d_results || !results) return GMAPDP_EINVAL;
  if (paths_needed) *paths_needed = 0;
  if (pairs_needed) *pairs_needed = 0;
  (void)hipSetDevice(ctx->device);
  hipStream_t s = stream ? (hipStream_t)stream : ctx->stream;
  unsigned long long cnt[4] = {0, 0, 0, 0};
  hipError_t e = hipMemcpyAsync(results, d_results, sizeof(gmapdp_stage2_result) * plan->n, hipMemcpyDeviceToHost, s);
  if (e == hipSuccess) e = hipMemcpyAsync(cnt, plan->d_counters, sizeof(cnt), hipMemcpyDeviceToHost, s);
  if (e == hipSuccess) e = ctx_sync(ctx, s);
  if (e != hipSuccess) return fail(ctx, GMAPDP_ELAUNCH, "stage-2 plan fetch: %s", e);
  // the pools' atomics count past their capacity when calls overflow (those report status -2)
  const size_t np = std::min<size_t>(cnt[1], plan->path_cap), nq = std::min<size_t>(cnt[2], plan->pair_cap);
  if (paths_needed) *paths_needed = np;
  if (pairs_needed) *pairs_needed = nq;
  if (np > path_cap || nq > pair_cap || (np && !paths) || (nq && !pairs)) return GMAPDP_ESPACE;
  if (np) e = hipMemcpyAsync(paths, plan->d_paths, sizeof(gmapdp_path) * np, hipMemcpyDeviceToHost, s);
  if (e == hipSuccess && nq) e = hipMemcpyAsync(pairs, plan->d_pairs, sizeof(gmapdp_path_pair) * nq, hipMemcpyDeviceToHost, s);
  if (e == hipSuccess) e = ctx_sync(ctx, s);
  if (e != hipSuccess) return fail(ctx, GMAPDP_ELAUNCH, "stage-2 plan fetch: %s", e);
  return GMAPDP_OK;
}

// The compact stream of the plan's path pairs (pc_kernel.hip), one list per path record of the pool
size_t gmapdp_stage2_plan_compact_bound(const gmapdp_stage2_plan* plan, size_t* path_cap) {
  if (path_cap) *path_cap = plan ? plan->path_cap : 0;
  return plan ? 21 * plan->pair_cap + 64 : 0;
}
int gmapdp_stage2_plan_compact_pairs(gmapdp_ctx* ctx, const gmapdp_stage2_plan* plan, uint8_t* d_out,
                                     uint64_t* d_offsets, void* stream) {
  if (!ctx || !plan || !d_offsets) return GMAPDP_EINVAL;
  if (plan->path_cap > (size_t)INT32_MAX) return bad(ctx, "stage-2 compaction: too many path records");
  (void)hipSetDevice(ctx->device);
  hipStream_t s = stream ? (hipStream_t)stream : ctx->stream;
  const hipError_t e = launch_pc_paths(plan->d_paths, plan->d_counters + 1, (int)plan->path_cap, plan->d_pairs,
                                       plan->pair_cap, (unsigned long long*)d_offsets, (unsigned char*)d_out, s);
  return e == hipSuccess ? GMAPDP_OK : fail(ctx, GMAPDP_ELAUNCH, "path pair compaction: %s", e);
}

int gmapdp_stage2_plan_seeding_classes(const gmapdp_stage2_plan* plan, int* n16, int* n32) {
  if (!plan || !plan->oplan) return GMAPDP_EINVAL;
  int a = 0, b = 0;
  for (int k : plan->oplan->keys) (k & 1) ? b++ : a++;
  if (n16) *n16 = a;
  if (n32) *n32 = b;
  return GMAPDP_OK;
}

void gmapdp_stage2_plan_destroy(gmapdp_stage2_plan* plan) { stage2_plan_free(plan); }

}  // extern "C"
