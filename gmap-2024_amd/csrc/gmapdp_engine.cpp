// gmapdp_engine.cpp -- host side of libgmapdp: score tables, genome packing,
// batch planning and the C ABI of include/gmapdp.h.
//
// Reference interfaces mirrored (paths under the reference tree's src/):
//   Dynprog_init / permute_cases  dynprog.c:903-1197  (score + consistency tables)
//   Dynprog_compute_bands         dynprog.c:1247
//   Dynprog_single_gap prologue   dynprog_single.c:459-521 (penalties, size guard)
//   Compress_create_blocks_comp   compress-write.c:754  (.genomecomp packing)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cctype>
#include <cstdio>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "gmapdp_internal.h"
#include "../../include/gmapdp.h"

namespace gmapdp {
size_t lds_bytes_single(int rlength, int glength, int R, bool dirs_lds);
hipError_t launch_single(int R, bool dirs_lds, int nblocks, size_t lds, hipStream_t stream, const DevSingle* probs,
                         const int* order, const uint32_t* blocks, uint64_t nwords, const char* qseq,
                         const char* qseq_uc, const int8_t* sctab, const uint8_t* constab, gmapdp_result* results,
                         gmapdp_pair* pairs, uint64_t* gdirs);

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
};

static bool stranded(int mode) { return mode == 0 || mode == 1 || mode == 3 || mode == 5; }

static void build_tables(Tables& T, int mode) {
  std::memset(&T, 0, sizeof(T));
  // Mismatch everywhere in 'A'..'z' x 'A'..'y' (the reference's second loop bound is exclusive).
  for (int a = 'A'; a <= 'z'; a++)
    for (int b = 'A'; b < 'z'; b++)
      for (int t = 0; t < 4; t++) T.pd[t][a][b] = (short)kMismatchScore[t];
  auto mark = [&](int strandset, int a, int b) {
    if (stranded(mode)) {
      if (strandset) T.cons[0][a][b] = 1;
    } else if (strandset) {
      T.cons[1][a][b] = 1;
      T.cons[2][a][b] = 1;
    }
  };
  // Symmetric assignment over upper/lower case variants (permute_cases).
  auto both = [&](int A, int B, short s) {
    const int a = std::tolower(A), b = std::tolower(B);
    const int v[4][2] = {{a, b}, {a, B}, {A, b}, {A, B}};
    for (auto& p : v) { mark(1, p[0], p[1]); mark(1, p[1], p[0]); }
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
}

// ---------------------------------------------------------------------------
// Device buffer that only grows.
// ---------------------------------------------------------------------------
struct DevBuf {
  void* p = nullptr;
  size_t cap = 0;
  hipError_t ensure(size_t bytes) {
    if (bytes <= cap) return hipSuccess;
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    size_t want = std::max(bytes, (size_t)4096);
    want = want + want / 4;
    hipError_t e = hipMalloc(&p, want);
    if (e == hipSuccess) cap = want;
    return e;
  }
  ~DevBuf() {
    if (p) (void)hipFree(p);
  }
};

}  // namespace gmapdp

using namespace gmapdp;

struct gmapdp_ctx {
  int device = 0;
  int mode = 0;
  int user_open = 0, user_extend = 0, user_dynprog_p = 0;
  hipStream_t stream = nullptr;
  Tables* tables = nullptr;
  int8_t* d_sc = nullptr;
  uint8_t* d_cs = nullptr;
  uint32_t* d_genome = nullptr;
  uint64_t genome_words = 0;
  uint64_t genome_length = 0;
  DevBuf probs, order, qseq, qseq_uc, results, pairs, gdirs;
  std::string err;
};

struct gmapdp_plan_internal {
  std::vector<DevSingle> dev;        // one per GPU problem
  std::vector<int> dev_index;        // problem index -> dev slot (-1: resolved on host)
  std::vector<int> dev_problem;      // dev slot -> problem index
  struct Launch { int R; bool dirs_lds; size_t lds; int first, count; };
  std::vector<Launch> launches;
  std::vector<int> order;            // dev slots grouped by launch
  size_t pair_capacity = 0;
  size_t gdirs_bytes = 0;
};

static int fail(gmapdp_ctx* ctx, int code, const char* fmt, hipError_t e) {
  char buf[256];
  std::snprintf(buf, sizeof(buf), fmt, hipGetErrorString(e));
  if (ctx) ctx->err = buf;
  return code;
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
  hipError_t e = hipSetDevice(device);
  if (e == hipSuccess) e = hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking);
  ctx->tables = new Tables();
  build_tables(*ctx->tables, mode);
  if (e == hipSuccess) e = hipMalloc(&ctx->d_sc, sizeof(ctx->tables->sc));
  if (e == hipSuccess) e = hipMalloc(&ctx->d_cs, sizeof(ctx->tables->cs));
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
  if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
  if (ctx->d_sc) (void)hipFree(ctx->d_sc);
  if (ctx->d_cs) (void)hipFree(ctx->d_cs);
  if (ctx->d_genome) (void)hipFree(ctx->d_genome);
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
  if (nblocks) {
    blocks[3 * nblocks - 3] = blocks[3 * nblocks - 2] = blocks[3 * nblocks - 1] = 0xFFFFFFFFu;
  }
  for (int i = 0; i < 4; i++) blocks[3 * nblocks + i] = 0xFFFFFFFFu;
  for (uint64_t b = 0; b < nblocks; b++) {
    uint32_t high = 0, low = 0, flags = 0;
    const uint64_t base = b * 32;
    const int n = (int)std::min<uint64_t>(32, length - base);
    for (int j = 0; j < n; j++) {
      uint32_t code;
      switch (seq[base + j]) {
        case 'A': case 'a': code = 0; break;
        case 'C': case 'c': code = 1; break;
        case 'G': case 'g': code = 2; break;
        case 'T': case 't': code = 3; break;
        case 'X': case 'x': code = 3; flags |= 1u << j; break;  // put_compressed_one: 'X' = T code + flag
        default: code = 0; flags |= 1u << j; break;            // 'N' and anything else: A code + flag
      }
      if (j < 16) low |= code << (2 * j);
      else high |= code << (2 * (j - 16));
    }
    if (n < 32) {  // tail of the last block reads as 'X' (all bits set)
      for (int j = n; j < 32; j++) {
        flags |= 1u << j;
        if (j < 16) low |= 3u << (2 * j);
        else high |= 3u << (2 * (j - 16));
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
  (void)hipSetDevice(ctx->device);
  if (ctx->d_genome) (void)hipFree(ctx->d_genome);
  ctx->d_genome = nullptr;
  hipError_t e = hipMalloc(&ctx->d_genome, nwords * sizeof(uint32_t));
  if (e != hipSuccess) return fail(ctx, GMAPDP_ENOMEM, "hipMalloc genome: %s", e);
  e = hipMemcpy(ctx->d_genome, blocks, nwords * sizeof(uint32_t), hipMemcpyHostToDevice);
  if (e != hipSuccess) return fail(ctx, GMAPDP_ENOMEM, "genome upload: %s", e);
  ctx->genome_words = nwords;
  ctx->genome_length = length;
  return GMAPDP_OK;
}

}  // extern "C"

// ---------------------------------------------------------------------------
// Planning: resolve host-side cases (size guard), derive penalties and bands
// (dynprog_single.c:459-521, dynprog.c:1247), pick the launch class and LDS
// footprint, and lay out the pair arena.
// ---------------------------------------------------------------------------
static const size_t kLdsBudget = 64 * 1024;  // per workgroup; keeps >= 2 problems resident per CU

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

static int plan_single(gmapdp_ctx* ctx, const gmapdp_single_problem* pr, int n, gmapdp_result* results,
                       gmapdp_plan_internal& plan) {
  plan.dev.clear();
  plan.dev_index.assign(n, -1);
  plan.dev_problem.clear();
  plan.launches.clear();
  plan.order.clear();
  size_t pair_off = 0, gdirs_off = 0;
  std::map<std::tuple<int, int, size_t>, std::vector<int>> classes;
  for (int i = 0; i < n; i++) {
    const gmapdp_single_problem& p = pr[i];
    gmapdp_result& res = results[i];
    const int dpi_next = p.dynprogindex + (p.dynprogindex > 0 ? 1 : -1);
    res.pair_offset = (int32_t)pair_off;
    if (p.rlength <= 0 || p.glength <= 0 || p.rlength > GMAPDP_MAX_RLENGTH || p.glength > GMAPDP_MAX_GLENGTH) {
      // size guard (dynprog_single.c:509-521)
      res.npairs = 0;
      res.traceback_score = GMAPDP_NEG_INFINITY_32;
      res.nmatches = res.nmismatches = res.nopens = res.nindels = 0;
      res.dynprogindex = dpi_next;
      continue;
    }
    DevSingle d;
    d.qoff = p.qoff;
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
    if (d.open > 0) {
      ctx->err = "positive gap-open penalty is not supported by the scan formulation";
      return GMAPDP_EINVAL;
    }
    int lb, ub;
    gmapdp_compute_bands(&lb, &ub, p.rlength, p.glength, p.extraband, p.flags & GMAPDP_WIDEBAND);
    if (lb < 0 || ub < 0) {
      ctx->err = "negative band";
      return GMAPDP_EINVAL;
    }
    d.lband = lb;
    d.uband = ub;
    d.flags = p.flags;
    d.genestrand = p.genestrand;
    d.dynprogindex = p.dynprogindex;
    d.pair_offset = (int32_t)pair_off;
    const int W = lb + ub + 1;
    const int R = pick_R(W);
    if (R > kMaxR) {
      ctx->err = "band wider than 4096";
      return GMAPDP_EINVAL;
    }
    size_t lds = lds_bytes_single(p.rlength, p.glength, R, true);
    bool dirs_lds = lds <= kLdsBudget;
    d.dirs_offset = 0;
    if (!dirs_lds) {
      lds = lds_bytes_single(p.rlength, p.glength, R, false);
      d.dirs_offset = (int64_t)gdirs_off;
      gdirs_off += ((size_t)(p.glength + 1) * 4 * R * 8 + 255) & ~(size_t)255;
    }
    plan.dev_index[i] = (int)plan.dev.size();
    plan.dev_problem.push_back(i);
    classes[std::make_tuple(R, dirs_lds ? 1 : 0, lds_bucket(lds))].push_back((int)plan.dev.size());
    plan.dev.push_back(d);
    pair_off += (size_t)p.rlength + (size_t)p.glength + 2;
  }
  for (auto& kv : classes) {
    gmapdp_plan_internal::Launch L;
    L.R = std::get<0>(kv.first);
    L.dirs_lds = std::get<1>(kv.first) != 0;
    L.lds = std::get<2>(kv.first);
    L.first = (int)plan.order.size();
    L.count = (int)kv.second.size();
    // longest problems first, so the tail of the launch is short work
    std::vector<int> ids = kv.second;
    std::stable_sort(ids.begin(), ids.end(), [&](int a, int b) {
      return (size_t)plan.dev[a].glength * (plan.dev[a].lband + plan.dev[a].uband + 1) >
             (size_t)plan.dev[b].glength * (plan.dev[b].lband + plan.dev[b].uband + 1);
    });
    plan.order.insert(plan.order.end(), ids.begin(), ids.end());
    plan.launches.push_back(L);
  }
  plan.pair_capacity = pair_off;
  plan.gdirs_bytes = gdirs_off;
  return GMAPDP_OK;
}

static int run_plan(gmapdp_ctx* ctx, const gmapdp_plan_internal& plan, const DevSingle* d_probs, const int* d_order,
                    const char* d_q, const char* d_quc, gmapdp_result* d_results, gmapdp_pair* d_pairs,
                    hipStream_t stream) {
  if (plan.gdirs_bytes) {
    hipError_t e = ctx->gdirs.ensure(plan.gdirs_bytes);
    if (e != hipSuccess) return fail(ctx, GMAPDP_ENOMEM, "direction scratch: %s", e);
  }
  for (const auto& L : plan.launches) {
    hipError_t e = launch_single(L.R, L.dirs_lds, L.count, L.lds, stream, d_probs, d_order + L.first, ctx->d_genome,
                                 ctx->genome_words, d_q, d_quc, ctx->d_sc, ctx->d_cs, d_results, d_pairs,
                                 (uint64_t*)ctx->gdirs.p);
    if (e != hipSuccess) return fail(ctx, GMAPDP_ELAUNCH, "single_gap launch: %s", e);
  }
  return GMAPDP_OK;
}

extern "C" {

size_t gmapdp_single_pair_capacity(const gmapdp_single_problem* problems, int n) {
  size_t cap = 0;
  for (int i = 0; i < n; i++)
    if (problems[i].rlength > 0 && problems[i].glength > 0) cap += (size_t)problems[i].rlength + problems[i].glength + 2;
  return cap;
}

int gmapdp_single_gap_batch(gmapdp_ctx* ctx, const gmapdp_single_problem* problems, int n, const char* qseq,
                            const char* qseq_uc, size_t qbytes, gmapdp_result* results, gmapdp_pair* pairs,
                            size_t pair_capacity) {
  if (!ctx || n < 0 || (n && (!problems || !results))) return GMAPDP_EINVAL;
  if (!ctx->d_genome) return GMAPDP_ENOGENOME;
  if (n == 0) return GMAPDP_OK;
  (void)hipSetDevice(ctx->device);
  gmapdp_plan_internal plan;
  int rc = plan_single(ctx, problems, n, results, plan);
  if (rc) return rc;
  if (plan.pair_capacity > pair_capacity) {
    ctx->err = "pair arena too small";
    return GMAPDP_EINVAL;
  }
  for (int i = 0; i < n; i++) {
    if (plan.dev_index[i] < 0) continue;
    if (problems[i].qoff < 0 || (size_t)problems[i].qoff + (size_t)problems[i].rlength > qbytes) {
      ctx->err = "query slice outside the query arena";
      return GMAPDP_EINVAL;
    }
  }
  const int ndev = (int)plan.dev.size();
  if (ndev == 0) return GMAPDP_OK;
  hipError_t e = hipSuccess;
  if (e == hipSuccess) e = ctx->probs.ensure(sizeof(DevSingle) * ndev);
  if (e == hipSuccess) e = ctx->order.ensure(sizeof(int) * ndev);
  if (e == hipSuccess) e = ctx->qseq.ensure(qbytes);
  if (e == hipSuccess) e = ctx->qseq_uc.ensure(qbytes);
  if (e == hipSuccess) e = ctx->results.ensure(sizeof(gmapdp_result) * ndev);
  if (e == hipSuccess) e = ctx->pairs.ensure(sizeof(gmapdp_pair) * std::max<size_t>(plan.pair_capacity, 1));
  if (e != hipSuccess) return fail(ctx, GMAPDP_ENOMEM, "device buffers: %s", e);
  // results are written per dev slot; map dev slot -> original index afterwards
  std::vector<DevSingle> dev = plan.dev;
  hipStream_t s = ctx->stream;
  e = hipMemcpyAsync(ctx->probs.p, dev.data(), sizeof(DevSingle) * ndev, hipMemcpyHostToDevice, s);
  if (e == hipSuccess) e = hipMemcpyAsync(ctx->order.p, plan.order.data(), sizeof(int) * ndev, hipMemcpyHostToDevice, s);
  if (e == hipSuccess) e = hipMemcpyAsync(ctx->qseq.p, qseq, qbytes, hipMemcpyHostToDevice, s);
  if (e == hipSuccess) e = hipMemcpyAsync(ctx->qseq_uc.p, qseq_uc, qbytes, hipMemcpyHostToDevice, s);
  if (e != hipSuccess) return fail(ctx, GMAPDP_ENOMEM, "upload: %s", e);
  rc = run_plan(ctx, plan, (const DevSingle*)ctx->probs.p, (const int*)ctx->order.p, (const char*)ctx->qseq.p,
                (const char*)ctx->qseq_uc.p, (gmapdp_result*)ctx->results.p, (gmapdp_pair*)ctx->pairs.p, s);
  if (rc) return rc;
  std::vector<gmapdp_result> dres(ndev);
  e = hipMemcpyAsync(dres.data(), ctx->results.p, sizeof(gmapdp_result) * ndev, hipMemcpyDeviceToHost, s);
  if (e == hipSuccess && pairs && plan.pair_capacity)
    e = hipMemcpyAsync(pairs, ctx->pairs.p, sizeof(gmapdp_pair) * plan.pair_capacity, hipMemcpyDeviceToHost, s);
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  if (e != hipSuccess) return fail(ctx, GMAPDP_ELAUNCH, "single_gap execution: %s", e);
  for (int i = 0; i < n; i++) {
    const int d = plan.dev_index[i];
    if (d >= 0) results[i] = dres[d];
  }
  return GMAPDP_OK;
}

}  // extern "C"

// ---------------------------------------------------------------------------
// Device-resident path (bench / pipelined callers): the plan is built once on
// the host, then replayed against device-resident inputs.
// ---------------------------------------------------------------------------
struct gmapdp_plan {
  gmapdp_plan_internal in;
  DevSingle* d_probs = nullptr;
  int* d_order = nullptr;
};

extern "C" {

int gmapdp_plan_single(gmapdp_ctx* ctx, const gmapdp_single_problem* problems, int n, gmapdp_result* host_results,
                       gmapdp_plan** out) {
  if (!ctx || !out || n <= 0 || !problems || !host_results) return GMAPDP_EINVAL;
  (void)hipSetDevice(ctx->device);
  gmapdp_plan* p = new gmapdp_plan();
  int rc = plan_single(ctx, problems, n, host_results, p->in);
  if (rc) {
    delete p;
    return rc;
  }
  // device results are indexed by dev slot; keep problem order == dev order for this API
  const size_t nd = p->in.dev.size();
  hipError_t e = hipMalloc(&p->d_probs, sizeof(DevSingle) * std::max<size_t>(nd, 1));
  if (e == hipSuccess) e = hipMalloc(&p->d_order, sizeof(int) * std::max<size_t>(nd, 1));
  if (e == hipSuccess && nd) e = hipMemcpy(p->d_probs, p->in.dev.data(), sizeof(DevSingle) * nd, hipMemcpyHostToDevice);
  if (e == hipSuccess && nd) e = hipMemcpy(p->d_order, p->in.order.data(), sizeof(int) * nd, hipMemcpyHostToDevice);
  if (e == hipSuccess && p->in.gdirs_bytes) e = ctx->gdirs.ensure(p->in.gdirs_bytes);
  if (e != hipSuccess) {
    if (p->d_probs) (void)hipFree(p->d_probs);
    if (p->d_order) (void)hipFree(p->d_order);
    delete p;
    return fail(ctx, GMAPDP_ENOMEM, "plan upload: %s", e);
  }
  *out = p;
  return GMAPDP_OK;
}

size_t gmapdp_plan_pair_capacity(const gmapdp_plan* plan) { return plan ? plan->in.pair_capacity : 0; }
int gmapdp_plan_gpu_problems(const gmapdp_plan* plan) { return plan ? (int)plan->in.dev.size() : 0; }
int gmapdp_plan_dev_index(const gmapdp_plan* plan, int i) {
  return (plan && i >= 0 && i < (int)plan->in.dev_index.size()) ? plan->in.dev_index[i] : -1;
}
int gmapdp_plan_nlaunches(const gmapdp_plan* plan) { return plan ? (int)plan->in.launches.size() : 0; }

int gmapdp_plan_run(gmapdp_ctx* ctx, const gmapdp_plan* plan, const char* d_qseq, const char* d_qseq_uc,
                    gmapdp_result* d_results, gmapdp_pair* d_pairs, void* stream) {
  if (!ctx || !plan) return GMAPDP_EINVAL;
  if (!ctx->d_genome) return GMAPDP_ENOGENOME;
  return run_plan(ctx, plan->in, plan->d_probs, plan->d_order, d_qseq, d_qseq_uc, d_results, d_pairs,
                  stream ? (hipStream_t)stream : ctx->stream);
}

int gmapdp_plan_launch_info(const gmapdp_plan* plan, int li, int* R, int* dirs_lds, int* count, size_t* lds) {
  if (!plan || li < 0 || li >= (int)plan->in.launches.size()) return GMAPDP_EINVAL;
  const auto& L = plan->in.launches[li];
  if (R) *R = L.R;
  if (dirs_lds) *dirs_lds = L.dirs_lds ? 1 : 0;
  if (count) *count = L.count;
  if (lds) *lds = L.lds;
  return GMAPDP_OK;
}

int gmapdp_plan_launch_members(const gmapdp_plan* plan, int li, int* problem_indices) {
  if (!plan || li < 0 || li >= (int)plan->in.launches.size() || !problem_indices) return GMAPDP_EINVAL;
  const auto& L = plan->in.launches[li];
  for (int k = 0; k < L.count; k++) problem_indices[k] = plan->in.dev_problem[plan->in.order[L.first + k]];
  return GMAPDP_OK;
}

int gmapdp_plan_run_launch(gmapdp_ctx* ctx, const gmapdp_plan* plan, int li, const char* d_qseq,
                           const char* d_qseq_uc, gmapdp_result* d_results, gmapdp_pair* d_pairs, void* stream) {
  if (!ctx || !plan || li < 0 || li >= (int)plan->in.launches.size()) return GMAPDP_EINVAL;
  if (!ctx->d_genome) return GMAPDP_ENOGENOME;
  const auto& L = plan->in.launches[li];
  hipError_t e = launch_single(L.R, L.dirs_lds, L.count, L.lds, stream ? (hipStream_t)stream : ctx->stream,
                               plan->d_probs, plan->d_order + L.first, ctx->d_genome, ctx->genome_words, d_qseq,
                               d_qseq_uc, ctx->d_sc, ctx->d_cs, d_results, d_pairs, (uint64_t*)ctx->gdirs.p);
  if (e != hipSuccess) return fail(ctx, GMAPDP_ELAUNCH, "single_gap launch: %s", e);
  return GMAPDP_OK;
}

void gmapdp_plan_destroy(gmapdp_plan* plan) {
  if (!plan) return;
  if (plan->d_probs) (void)hipFree(plan->d_probs);
  if (plan->d_order) (void)hipFree(plan->d_order);
  delete plan;
}

void* gmapdp_stream(gmapdp_ctx* ctx) { return ctx ? (void*)ctx->stream : nullptr; }

}  // extern "C"
