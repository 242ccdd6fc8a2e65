// tools/plan_bench.cpp -- host-only timing of the DP plan build (build_plan: per-problem prologues and launch
// classification) on a dumped block of descriptors; no GPU is touched.  Diagnostic, not the product:
//   make -C gmap-2024_amd && hipcc -O3 -std=c++17 -o /tmp/plan_bench tools/plan_bench.cpp \
//       gmap-2024_amd/build/{dp,ux,cg,oi,s2c,mx,sj,me}_kernel.hip.o
//   /tmp/plan_bench <dir with single.bin end.bin genome.bin> [reps]
#include "../gmap-2024_amd/csrc/gmapdp_engine.cpp"

#include <chrono>

template <typename T>
static std::vector<T> load(const std::string& path) {
  std::vector<T> v;
  FILE* f = std::fopen(path.c_str(), "rb");
  if (!f) return v;
  std::fseek(f, 0, SEEK_END);
  const long n = std::ftell(f) / (long)sizeof(T);
  std::fseek(f, 0, SEEK_SET);
  v.resize(n);
  if (std::fread(v.data(), sizeof(T), n, f) != (size_t)n) v.clear();
  std::fclose(f);
  return v;
}

int main(int argc, char** argv) {
  const std::string dir = argc > 1 ? argv[1] : "/tmp/planb";
  const int reps = argc > 2 ? std::atoi(argv[2]) : 3;
  auto sp = load<gmapdp_single_problem>(dir + "/single.bin");
  auto ep = load<gmapdp_end_problem>(dir + "/end.bin");
  auto gp = load<gmapdp_genome_problem>(dir + "/genome.bin");
  std::printf("problems: %zu single, %zu end, %zu genome\n", sp.size(), ep.size(), gp.size());
  gmapdp_ctx ctx;
  ctx.plan_sides = 2;
  std::vector<gmapdp_result> res(sp.size() + ep.size());
  std::vector<gmapdp_genome_result> gres(gp.size());
  for (int r = 0; r < reps; r++) {
    PlanCore plan;
    const auto t0 = std::chrono::steady_clock::now();
    const int rc = build_plan(&ctx, sp.data(), (int)sp.size(), ep.data(), (int)ep.size(), gp.data(), (int)gp.size(),
                              res.data(), gres.data(), plan);
    const auto t1 = std::chrono::steady_clock::now();
    std::printf("build_plan rc %d: %.1f ms (%zu launches, %zu + %zu GPU problems)\n", rc,
                std::chrono::duration<double, std::milli>(t1 - t0).count(), plan.launches.size(), plan.dev.size(),
                plan.gdev.size());
  }
  return 0;
}
