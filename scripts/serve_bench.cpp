// serve_bench.cpp -- native serving load for the request coalescer (pyr_index_set_coalescing).
//
// The reference serves one VEC.SEARCH per call from many Garnet session threads
// (Extensions/VectorCommandSet.cs:457-459).  This client does the same against the C ABI: T threads,
// each in a closed loop calling pyr_index_search with nq queries (host buffers, PCIe-inclusive) for a
// few seconds; reported per setting: QPS and per-call latency p50 / p99.  No Python, no GIL: what the
// library itself sustains.  Index: IVF_FLAT d=128 N rows of the bench generator, nlist 1024, nprobe 32.
//
//   g++ -O2 -std=c++17 -Iinclude scripts/serve_bench.cpp -Lpyrope_amd -lpyrope_hip -lpthread \
//       -Wl,-rpath,'$ORIGIN/../pyrope_amd' -o scripts/serve_bench      (scripts/build_serve_bench.sh)
//   scripts/serve_bench [N] [seconds]   -> one JSON object on stdout
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <thread>
#include <vector>

#include "pyrope_ann.h"

#define CHK(x)                                                                          \
  do {                                                                                  \
    pyr_status s_ = (x);                                                                \
    if (s_ != PYR_OK) {                                                                 \
      std::fprintf(stderr, "%s failed: %d %s\n", #x, (int)s_, pyr_last_error());      \
      std::exit(1);                                                                     \
    }                                                                                   \
  } while (0)

using clk = std::chrono::steady_clock;

struct Result {
  int nq, threads, wait_us;
  double qps, p50, p99;
  long calls;
};

static Result run(pyr_index *idx, const std::vector<float> &qs, int nq_total, int dim, int nq, int threads,
                  int max_batch, int wait_us, double seconds) {
  CHK(pyr_index_set_coalescing(idx, max_batch, wait_us));
  pyr_search_params prm{32, 0, -1};
  std::vector<std::vector<double>> lat(threads);
  std::vector<long> done(threads, 0);
  const auto stop = clk::now() + std::chrono::duration<double>(seconds);
  std::vector<std::thread> th;
  const auto t0 = clk::now();
  for (int t = 0; t < threads; ++t)
    th.emplace_back([&, t] {
      std::vector<float> s((size_t)nq * 10);
      std::vector<int64_t> l((size_t)nq * 10);
      uint32_t r = 12345u + 7919u * (uint32_t)t;
      while (clk::now() < stop) {
        r = r * 1664525u + 1013904223u;
        const int a = (int)(r % (uint32_t)(nq_total - nq + 1));
        const auto c0 = clk::now();
        CHK(pyr_index_search(idx, qs.data() + (size_t)a * dim, nq, 10, &prm, s.data(), l.data(), nullptr));
        lat[t].push_back(std::chrono::duration<double, std::milli>(clk::now() - c0).count());
        done[t] += nq;
      }
    });
  for (auto &x : th) x.join();
  const double wall = std::chrono::duration<double>(clk::now() - t0).count();
  std::vector<double> all;
  long q = 0;
  for (int t = 0; t < threads; ++t) {
    all.insert(all.end(), lat[t].begin(), lat[t].end());
    q += done[t];
  }
  std::sort(all.begin(), all.end());
  auto pct = [&](double p) { return all.empty() ? 0.0 : all[std::min(all.size() - 1, (size_t)(p * all.size()))]; };
  return Result{nq, threads, wait_us, q / wall, pct(0.5), pct(0.99), (long)all.size()};
}

int main(int argc, char **argv) {
  const int64_t n = argc > 1 ? std::atoll(argv[1]) : 10000000;
  const double seconds = argc > 2 ? std::atof(argv[2]) : 3.0;
  const int dim = 128, nlist = 1024;
  std::vector<float> x((size_t)n * dim);
  CHK(pyr_generate_synthetic_blocked(0, n, dim, 42, 65536, x.data()));
  std::vector<float> cents((size_t)nlist * dim);
  int32_t kout = 0;
  CHK(pyr_kmeans_train(0, x.data(), n, dim, nlist, PYR_L2, 10, 42, cents.data(), &kout));
  pyr_index_desc d{};
  d.kind = PYR_IVF_FLAT;
  d.dim = dim;
  d.metric = PYR_L2;
  d.nlist = nlist;
  pyr_index *idx = nullptr;
  CHK(pyr_index_create(&d, &idx));
  CHK(pyr_index_set_centroids(idx, cents.data(), kout));
  CHK(pyr_index_reserve(idx, n));
  std::vector<int64_t> labels(n);
  for (int64_t i = 0; i < n; ++i) labels[i] = i;
  for (int64_t a = 0; a < n; a += 2000000) {
    const int64_t c = std::min<int64_t>(2000000, n - a);
    CHK(pyr_index_add(idx, x.data() + (size_t)a * dim, c, labels.data() + a));
  }
  CHK(pyr_index_build(idx));
  std::vector<float>().swap(x);
  const int nqt = 20000;
  std::vector<float> qs((size_t)nqt * dim);
  CHK(pyr_generate_synthetic(nqt, dim, 1337, qs.data()));
  std::fprintf(stderr, "index ready: N=%lld\n", (long long)n);

  struct Cfg {
    int nq, threads, wait_us;
  };
  const Cfg cfgs[] = {{1, 64, 0}, {1, 64, 200}, {1, 64, 2000}, {1, 256, 200}, {16, 64, 0}, {16, 64, 200},
                      {128, 32, 0}, {128, 32, 200}, {1000, 8, 0}, {1000, 8, 200}};
  std::printf("{\"index\": \"IVF_FLAT d=128 N=%lld nlist=1024 nprobe=32 k=10\", \"client\": \"native C++ threads "
              "over the C ABI (pyr_index_search, host buffers, PCIe-inclusive)\", \"max_batch\": 4096, \"results\": [",
              (long long)n);
  bool first = true;
  for (const Cfg &c : cfgs) {
    const Result r = run(idx, qs, nqt, dim, c.nq, c.threads, 4096, c.wait_us, seconds);
    std::fprintf(stderr, "nq %d x %d threads, wait %d us: %.0f QPS, p50 %.3f ms, p99 %.3f ms (%ld calls)\n", r.nq,
                 r.threads, r.wait_us, r.qps, r.p50, r.p99, r.calls);
    std::printf("%s{\"nq_per_call\": %d, \"threads\": %d, \"coalescing_wait_us\": %d, \"qps\": %.1f, \"p50_ms\": %.4f, "
                "\"p99_ms\": %.4f, \"calls\": %ld}",
                first ? "" : ", ", r.nq, r.threads, r.wait_us, r.qps, r.p50, r.p99, r.calls);
    first = false;
    std::fflush(stdout);
  }
  std::printf("]}\n");
  pyr_index_destroy(idx);
  return 0;
}
