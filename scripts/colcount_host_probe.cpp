// Host probe: the LADIES draw's column count (cnt[c] += 1 per entry of U = lap[rows, :]) on an
// ogbn-products-sized count array, with T threads counting their own batches at once (as the
// batch producer's sampler threads do). Forms:
//   direct  — one increment per entry straight into the N-wide array (sampler.cpp add_row)
//   bkt<S>  — entries appended to per-window buckets of 2^S columns (2-byte offsets), then each
//             window's increments applied at once (the window stays in the core's L2)
// Synthetic rows: 17,000 rows x 250 sorted random columns (4.25 M entries: the products batch's
// count volume). Prints ms per batch per thread (median over the repeats).
//   g++ -O3 -march=x86-64-v2 -pthread scripts/colcount_host_probe.cpp -o /tmp/ccp && /tmp/ccp 2449029
#include <algorithm>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <thread>
#include <vector>

namespace {

constexpr size_t kRows = 17000, kDeg = 250;

struct Counter {
  size_t n;
  std::vector<uint32_t> idx;
  std::vector<int32_t> cnt;
  std::vector<std::vector<uint16_t>> bk;
  Counter(size_t n_, uint32_t seed) : n(n_), idx(kRows * kDeg), cnt(n_, 0) {
    std::mt19937 g(seed);
    for (size_t r = 0; r < kRows; ++r) {
      for (size_t k = 0; k < kDeg; ++k) idx[r * kDeg + k] = g() % n;
      std::sort(idx.begin() + r * kDeg, idx.begin() + (r + 1) * kDeg);
    }
  }
  int64_t direct() {
    for (const uint32_t c : idx) ++cnt[c];
    return 0;
  }
  int64_t bucketed(int shift) {
    bk.resize((n + ((size_t)1 << shift) - 1) >> shift);
    for (const uint32_t c : idx) bk[c >> shift].push_back((uint16_t)(c & ((1u << shift) - 1)));
    for (size_t b = 0; b < bk.size(); ++b) {
      int32_t* const w = cnt.data() + (b << shift);
      for (const uint16_t o : bk[b]) ++w[o];
      bk[b].clear();
    }
    return 0;
  }
  int64_t reset() {  // checksum + clear (outside the timed region)
    int64_t s = 0;
    for (size_t c = 0; c < n; c += 4099) s += cnt[c];
    std::fill(cnt.begin(), cnt.end(), 0);
    return s;
  }
};

}  // namespace

int main(int argc, char** argv) {
  const size_t n = argc > 1 ? (size_t)atol(argv[1]) : 2449029;
  const int reps = 6;
  for (const int T : {1, 8, 14}) {
    std::vector<Counter*> cs;
    for (int t = 0; t < T; ++t) cs.push_back(new Counter(n, 1u + t));
    for (const int form : {0, 14, 15, 16}) {
      std::vector<double> per(T * reps);
      std::vector<int64_t> sums(T);
      std::vector<std::thread> th;
      for (int t = 0; t < T; ++t)
        th.emplace_back([&, t] {
          for (int r = 0; r < reps; ++r) {
            const auto a = std::chrono::steady_clock::now();
            form ? cs[t]->bucketed(form) : cs[t]->direct();
            per[t * reps + r] = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - a).count();
            sums[t] += cs[t]->reset();
          }
        });
      for (auto& x : th) x.join();
      std::sort(per.begin(), per.end());
      printf("N=%zu T=%2d %-6s%s median %.2f ms/batch (min %.2f)  sum %lld\n", n, T, form ? "bkt" : "direct",
             form ? std::to_string(form).c_str() : "", per[per.size() / 2], per[0], (long long)sums[0]);
      fflush(stdout);
    }
    for (auto* c : cs) delete c;
  }
}
