// Native LADIES sampler (include/gnn_sampler.h): host C++ restatement of the per-batch
// numpy/scipy work of ladies_sampler (reference sampler.py:90-160), bit-identical to it.
//
// The costs the numpy path pays per layer (csr row slicing, sp.linalg.norm, N-wide cumsum
// per choice round, np.unique, scipy column indexing) become linear passes over the touched
// rows plus O(#nonzero columns) work per choice round, on scratch arrays owned by the call —
// so batches sample concurrently on host threads (ctypes releases the GIL).
#include "gnn_sampler.h"
#include "sampler_internal.h"

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdarg>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <emmintrin.h>
#include <memory>
#include <new>
#include <string>
#include <vector>

using gnn_smp::Layer;

namespace {

thread_local std::string g_err;

// Optional phase timers (GNN_SAMPLER_PROFILE=1): nanoseconds per phase summed over all threads,
// read by gnn_sampler_profile (scripts/sampler_probe.py). One clock read per phase per layer.
enum Phase { P_SCRATCH, P_ROWPTR, P_COUNT, P_DRAW, P_AFTER, P_EXTRACT, P_TAIL, P_CALLS, P_NPHASE };
std::atomic<int64_t> g_prof[P_NPHASE];
const bool g_prof_on = [] {
  const char* e = getenv("GNN_SAMPLER_PROFILE");
  return e && atoi(e) != 0;
}();

struct PhaseClock {
  std::chrono::steady_clock::time_point t;
  PhaseClock() : t(g_prof_on ? std::chrono::steady_clock::now() : std::chrono::steady_clock::time_point{}) {}
  void lap(Phase p) {
    if (!g_prof_on) return;
    const auto n = std::chrono::steady_clock::now();
    g_prof[p].fetch_add(std::chrono::duration_cast<std::chrono::nanoseconds>(n - t).count(), std::memory_order_relaxed);
    t = n;
  }
};

int fail(const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  g_err = buf;
  return -22;
}

// numpy's legacy MT19937 (RandomState): init_genrand seeding (mt19937_seed), the reference
// generator, and random_sample's 53-bit double from two draws (mt19937_next_double).
class MT19937 {
 public:
  explicit MT19937(uint32_t s) {
    for (int i = 0; i < kN; ++i) {
      key_[i] = s;
      s = 1812433253u * (s ^ (s >> 30)) + (uint32_t)i + 1u;
    }
    pos_ = kN;
  }
  uint32_t next32() {
    if (pos_ == kN) gen();
    uint32_t y = key_[pos_++];
    y ^= (y >> 11);
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= (y >> 18);
    return y;
  }
  double next_double() {
    const int32_t a = (int32_t)(next32() >> 5);
    const int32_t b = (int32_t)(next32() >> 6);
    return (a * 67108864.0 + b) / 9007199254740992.0;
  }

 private:
  static constexpr int kN = 624, kM = 397;
  static constexpr uint32_t kA = 0x9908b0dfu, kUp = 0x80000000u, kLo = 0x7fffffffu;
  void gen() {
    int i = 0;
    uint32_t y;
    for (; i < kN - kM; ++i) {
      y = (key_[i] & kUp) | (key_[i + 1] & kLo);
      key_[i] = key_[i + kM] ^ (y >> 1) ^ ((0u - (y & 1u)) & kA);
    }
    for (; i < kN - 1; ++i) {
      y = (key_[i] & kUp) | (key_[i + 1] & kLo);
      key_[i] = key_[i + (kM - kN)] ^ (y >> 1) ^ ((0u - (y & 1u)) & kA);
    }
    y = (key_[kN - 1] & kUp) | (key_[0] & kLo);
    key_[kN - 1] = key_[kM - 1] ^ (y >> 1) ^ ((0u - (y & 1u)) & kA);
    pos_ = 0;
  }
  uint32_t key_[kN];
  int pos_;
};


// RandomState.choice(N, size, p=p, replace=False) (numpy mtrand.pyx, legacy): rounds of
// `rand(size - n_uniq)` draws, p of the already found entries zeroed, cdf = cumsum(p) /
// cdf[-1], searchsorted(side='right'), de-duplicated in first-occurrence order.
// cumsum over the zero entries adds +0.0 (exact) and searchsorted('right') never lands on a
// zero-probability index, so both run over the ascending list of non-zero entries live[0..n)
// (pv[i] = p[live[i]]) with identical results. Three more exact shortcuts:
//  - the cdf is never divided: the search compares x against cdf[j] / last at its probe points
//    only (the same correctly rounded quotient numpy stores, so the same comparisons);
//  - a round's cumsum is recomputed only from the first position whose p changed (the smallest
//    index found in the previous round): the prefix below it sums the same terms in the same
//    order, so it is bit-identical;
//  - base is cumsum(pv) with nothing taken: the first round reads it, later rounds write their
//    suffixes to `work` (cdf[i] = i < wfrom ? base[i] : work[i]); FastGCN's base is shared by
//    every call over the same p, LADIES' is computed with pv in one pass (base == work).
// The searches of a round run kSearchLanes at a time, branch-free and in lock step, so their
// cache misses overlap. pv_mutable: found entries' pv is zeroed in place (a per-call pv);
// otherwise taken[] stands in for the zeroing (a shared pv).
// taken[] must be all zero on entry; found entries are left set (make_after clears them).
constexpr int kSearchLanes = 16;

void choice_without_replacement(MT19937& rng, const int64_t* live, double* pv, bool pv_mutable, const double* base,
                                size_t n, int64_t size, std::vector<uint8_t>& taken, std::vector<int64_t>& found,
                                std::vector<double>& work, std::vector<double>& xs, std::vector<uint32_t>& js) {
  found.clear();
  if (size <= 0 || n == 0) return;
  found.reserve((size_t)size);
  if (work.size() < n) work.resize(n);
  double* const wk = work.data();
  size_t wfrom = base == wk ? 0 : n;
  size_t dirty = n;  // the smallest position whose p changed since the cdf was computed
  double last = base[n - 1];
  while ((int64_t)found.size() < size) {
    const size_t m = (size_t)(size - (int64_t)found.size());
    xs.resize(m);
    js.resize(m);
    for (size_t i = 0; i < m; ++i) xs[i] = rng.next_double();
    if (dirty < n) {  // p[found] = 0: cumsum again from the first changed position
      double s = dirty ? (dirty - 1 < wfrom ? base[dirty - 1] : wk[dirty - 1]) : 0.0;
      if (pv_mutable) {
        for (size_t i = dirty; i < n; ++i) {
          s += pv[i];
          wk[i] = s;
        }
      } else {
        for (size_t i = dirty; i < n; ++i) {
          s += taken[(size_t)live[i]] ? 0.0 : pv[i];
          wk[i] = s;
        }
      }
      wfrom = std::min(wfrom, dirty);
      last = s;
      dirty = n;
    }
    // upper_bound: the first j with x < cdf[j] / last. Branch-free halving keeps the answer in
    // [lo, lo + len]; at len == 1 it is lo or lo + 1.
    for (size_t i0 = 0; i0 < m; i0 += kSearchLanes) {
      const int lanes = (int)std::min<size_t>(kSearchLanes, m - i0);
      size_t lo[kSearchLanes];
      double x[kSearchLanes];
      for (int g = 0; g < lanes; ++g) {
        lo[g] = 0;
        x[g] = xs[i0 + (size_t)g];
      }
      for (size_t len = n; len > 1;) {
        const size_t half = len >> 1;
        for (int g = 0; g < lanes; ++g) {
          const size_t mid = lo[g] + half - 1;
          const double c = mid < wfrom ? base[mid] : wk[mid];
          lo[g] = (x[g] < c / last) ? lo[g] : lo[g] + half;
        }
        len -= half;
      }
      for (int g = 0; g < lanes; ++g) {
        const double c = lo[g] < wfrom ? base[lo[g]] : wk[lo[g]];
        size_t j = (x[g] < c / last) ? lo[g] : lo[g] + 1;
        js[i0 + (size_t)g] = (uint32_t)(j < n ? j : n - 1);  // j == n cannot happen for x < 1; guard
      }
    }
    for (size_t i = 0; i < m; ++i) {  // first-occurrence order
      const size_t j = js[i];
      const int64_t v = live[j];
      if (!taken[(size_t)v]) {
        taken[(size_t)v] = 1;
        found.push_back(v);
        if (pv_mutable) pv[j] = 0.0;
        dirty = std::min(dirty, j);
      }
    }
  }
}

struct Graph {
  const int64_t* indptr;
  const int32_t* indices;
  const float* data;
  size_t N;
};

// Per-call scratch (N-sized arrays) and the steps both samplers are built from. One Work
// per sampler thread, reused across calls (acquire): fresh multi-MB allocations are served
// by mmap and pay a page fault per 4 KB on first touch — the layer extraction's scratch
// alone (up to 23 MB per layer) cost ~40 % of a Reddit batch before it was reused.
// Bumped by gnn_fastgcn_p_changed(): invalidates every thread's FastGCN candidate cache.
std::atomic<uint64_t> g_fastgcn_generation{0};

class Work {
 public:
  explicit Work(const Graph& g) : g_(g), cnt(g.N, 0), bits((g.N + 63) / 64), wrank((g.N + 63) / 64),
                                  taken(g.N, 0), in_prev(g.N, 0), counted(g.N, 0) {}

  // This thread's Work for graph g, in the state of a freshly constructed one. A call that
  // finished (finish()) left taken / in_prev clear and recorded what it set in cnt (live) and
  // counted (counted_list): only those entries are reset — N-wide fills cost ~3 ms a batch on a
  // 2.4 M-node graph. After a call that failed part-way everything is refilled.
  static Work& acquire(const Graph& g) {
    static thread_local std::unique_ptr<Work> tw;
    if (!tw || tw->g_.N != g.N) {
      tw.reset(new Work(g));
    } else {
      tw->g_ = g;
      if (!tw->clean_) {
        std::fill(tw->cnt.begin(), tw->cnt.end(), 0);
        std::fill(tw->cnt16.begin(), tw->cnt16.end(), (uint16_t)0);
        std::fill(tw->taken.begin(), tw->taken.end(), 0);
        std::fill(tw->in_prev.begin(), tw->in_prev.end(), 0);
        std::fill(tw->counted.begin(), tw->counted.end(), 0);
      } else {
        tw->reset_counts();
        for (int64_t v : tw->counted_list) tw->counted[(size_t)v] = 0;
      }
      tw->counted_list.clear();
      tw->live.clear();
      tw->found.clear();
      tw->has_live_cnt = false;
    }
    tw->in16 = false;
    tw->rows16 = 0;
    tw->clean_ = false;
    return *tw;
  }

  // The call ends with taken / in_prev clear (every successful sampler path restores them).
  void finish() { clean_ = true; }

  // Row pointers of U = lap[rows, :] into fullrowptr; returns nnz(U) or -1 if >= 2^31.
  int64_t row_pointers(const std::vector<int64_t>& rows, std::vector<int32_t>& fullrowptr) const {
    fullrowptr.resize(rows.size() + 1);
    fullrowptr[0] = 0;
    int64_t unnz = 0;
    for (size_t r = 0; r < rows.size(); ++r) {
      unnz += g_.indptr[rows[r] + 1] - g_.indptr[rows[r]];
      if (unnz >= ((int64_t)1 << 31)) return -1;
      fullrowptr[r + 1] = (int32_t)unnz;
    }
    return unnz;
  }

  // Column nonzero counts of U = lap[rows, :] (sp.linalg.norm(U, ord=0, axis=0)); `live` =
  // ascending columns with a non-zero count (one sequential scan, no sort); returns the sum.
  int64_t count_columns(const std::vector<int64_t>& rows) {
    if (start16((int64_t)rows.size())) {
      for (size_t r = 0; r < rows.size(); ++r) {
        prefetch_row(rows, r + kPrefetchRows);
        add_row16(rows[r]);
      }
      return scan_counts16();
    }
    for (size_t r = 0; r < rows.size(); ++r) {
      prefetch_row(rows, r + kPrefetchRows);
      add_row(rows[r]);
    }
    return scan_counts();
  }

  // 16-bit counters (default; GNN_SAMPLER_CNT16=0: int32 only): a column's count is at most the
  // number of rows counted
  // (each row of the canonical CSR holds a column once), so while fewer than 65,535 rows are
  // counted the counts fit 16 bits and the random increments hit an array half the size of cnt
  // (Reddit: 0.47 MB against 0.93 MB — inside a core's L2). The scan writes the live columns'
  // counts into cnt, which the rest of the draw reads: the same integers, the same draw. On the
  // box's EPYC 9575F (scripts/sampler_probe.py, one thread, Reddit): count phase 4.83 / 4.88 ms
  // per batch against 5.38 / 5.28, the draw 10.9 / 10.8 against 11.5 / 11.2 ms; ogbn-products
  // (2.45 M columns: 4.9 MB against 9.8 MB) 8.99 / 9.16 against 10.87 / 10.44 ms, the draw 19.7 /
  // 19.9 against 21.0 / 20.5 ms; same checksums (profiles/round6/producer/, products/).
  std::vector<uint16_t> cnt16;
  bool in16 = false;     // this call's counts are in cnt16 (live ones mirrored into cnt)
  int64_t rows16 = 0;    // rows counted into cnt16 since the last clear
  static bool cnt16_enabled() {
    static const bool on = [] {
      const char* e = getenv("GNN_SAMPLER_CNT16");
      return !(e && atoi(e) == 0);
    }();
    return on;
  }
  // Whether the next `add` rows are counted in 16 bits; leaving the 16-bit form (too many rows)
  // keeps the counts so far: cnt already holds every live column's count.
  bool start16(int64_t add) {
    const bool fits = cnt16_enabled() && !g_.data && rows16 + add < 65535;
    if (fits) {
      if (cnt16.size() != g_.N) cnt16.assign(g_.N, 0);
      in16 = true;
      rows16 += add;
      return true;
    }
    if (in16) {
      for (int64_t c : live) cnt16[(size_t)c] = 0;
      in16 = false;
    }
    return false;
  }
  void add_row16(int64_t v) {
    const int64_t b = g_.indptr[v], e = g_.indptr[v + 1];
    uint16_t* const c16 = cnt16.data();
    for (int64_t k = b; k < e; ++k) ++c16[(uint32_t)g_.indices[k]];
  }
  // scan_counts over cnt16: live, the sum, and cnt[live] = cnt16[live]
  int64_t scan_counts16() {
    int64_t isum = 0;
    has_live_cnt = false;
    live.clear();
    const uint16_t* const c16 = cnt16.data();
    int32_t* const c32 = cnt.data();
    const size_t N = g_.N, N16 = N & ~(size_t)15;
    const __m128i z = _mm_setzero_si128();
    auto visit = [&](size_t c0, uint32_t mask) {
      for (; mask; mask &= mask - 1) {
        const size_t c = c0 + (size_t)__builtin_ctz(mask);
        const int32_t v = c16[c];
        isum += v;
        c32[c] = v;
        live.push_back((int64_t)c);
      }
    };
    for (size_t c0 = 0; c0 < N16; c0 += 16) {
      const __m128i* q = reinterpret_cast<const __m128i*>(c16 + c0);
      const __m128i za = _mm_cmpeq_epi16(_mm_loadu_si128(q), z), zb = _mm_cmpeq_epi16(_mm_loadu_si128(q + 1), z);
      const uint32_t zm = (uint32_t)_mm_movemask_epi8(_mm_packs_epi16(za, zb));
      if (zm != 0xFFFFu) visit(c0, ~zm & 0xFFFFu);
    }
    uint32_t tail = 0;
    for (size_t c = N16; c < N; ++c) tail |= (uint32_t)(c16[c] != 0) << (c - N16);
    visit(N16, tail);
    return isum;
  }

  // the first lines of a row's entries (rows are scattered over the graph's index array: one
  // DRAM miss each), requested kPrefetchRows rows ahead of the walk
  static constexpr size_t kPrefetchRows = 6;
  void prefetch_row(const std::vector<int64_t>& rows, size_t r) const {
    if (r < rows.size()) {
      const int32_t* q = g_.indices + g_.indptr[rows[r]];
      __builtin_prefetch(q);
      __builtin_prefetch(q + 16);
    }
  }

  // Same counts when rows ⊇ the rows already counted (LADIES: each layer's rows are the
  // previous layer's rows plus the newly sampled ones, sampler.py:131) — only the rows not
  // counted yet are added; the counts are kept across layers (the layer-2 U has 5.7 M
  // entries of which 3.5 M are the layer-1 rows').
  int64_t count_columns_nested(const std::vector<int64_t>& rows) {
    if (cnt16_enabled()) {
      newrows.clear();
      for (int64_t v : rows)
        if (!counted[(size_t)v]) newrows.push_back(v);
      if (start16((int64_t)newrows.size())) {
        for (size_t r = 0; r < newrows.size(); ++r) {
          prefetch_row(newrows, r + kPrefetchRows);
          counted[(size_t)newrows[r]] = 1;
          counted_list.push_back(newrows[r]);
          add_row16(newrows[r]);
        }
        return scan_counts16();
      }
    }
    for (size_t r = 0; r < rows.size(); ++r) {
      const int64_t v = rows[r];
      if (!counted[(size_t)v]) {
        prefetch_row(rows, r + kPrefetchRows);
        counted[(size_t)v] = 1;
        counted_list.push_back(v);
        add_row(v);
      }
    }
    return scan_counts();
  }

  // The same counts summed on the device (gnn_colcount_api): the rows not counted yet (nested)
  // or all rows go to the GPU, live and cnt[live] come back. Returns the sum, or -1 (rc set).
  int64_t count_columns_device(const std::vector<int64_t>& rows, bool nested, const gnn_colcount_api* cc, void* ctx,
                               int* rc) {
    const std::vector<int64_t>* send = &rows;
    if (nested) {
      newrows.clear();
      for (int64_t v : rows) {
        if (!counted[(size_t)v]) {
          counted[(size_t)v] = 1;
          counted_list.push_back(v);
          newrows.push_back(v);
        }
      }
      send = &newrows;
    }
    int64_t nlive = 0;
    const uint64_t* bits = nullptr;
    const int32_t* counts = nullptr;
    *rc = cc->add(ctx, send->data(), (int64_t)send->size(), &nlive, &bits, &counts);
    if (*rc) return -1;
    // live from the bitmap, cnt[live] from the counts (ascending stores); the counts also stay
    // contiguous in live order for the draw's p (choose_by_counts)
    live.resize((size_t)nlive);
    live_cnt.assign(counts, counts + nlive);
    int64_t* const lp = live.data();
    int32_t* const cp = cnt.data();
    int64_t i = 0;
    const size_t W = (g_.N + 63) / 64;
    for (size_t wi = 0; wi < W; ++wi) {
      uint64_t x = bits[wi];
      if (!x) continue;
      if (i + __builtin_popcountll(x) > nlive) {
        *rc = -5;
        return -1;
      }
      for (; x; x &= x - 1) {
        const size_t c = (wi << 6) + (size_t)__builtin_ctzll(x);
        lp[i] = (int64_t)c;
        cp[c] = counts[i];
        ++i;
      }
    }
    if (i != nlive || (nlive > 0 && (size_t)lp[nlive - 1] >= g_.N)) {
      *rc = -5;
      return -1;
    }
    int64_t isum = 0;
    for (int64_t k = 0; k < nlive; ++k) isum += counts[k];
    has_live_cnt = true;
    return isum;
  }

  // cnt[c] += entries of row v in column c (one random increment per entry: the sampler's
  // costliest loop on large graphs — nothing else is done per entry)
  void add_row(int64_t v) {
    const int64_t b = g_.indptr[v], e = g_.indptr[v + 1];
    if (g_.data) {
      for (int64_t k = b; k < e; ++k) cnt[(uint32_t)g_.indices[k]] += (g_.data[k] != 0.0f);
    } else {
      for (int64_t k = b; k < e; ++k) ++cnt[(uint32_t)g_.indices[k]];
    }
  }

  // live = the columns with a non-zero count, ascending; returns their sum. 16 counts per
  // step compared at once; only the non-zero ones are visited (no per-column branch).
  int64_t scan_counts() {
    int64_t isum = 0;
    has_live_cnt = false;
    live.clear();
    const int32_t* const c32 = cnt.data();
    const size_t N = g_.N, N16 = N & ~(size_t)15;
    const __m128i z = _mm_setzero_si128();
    auto visit = [&](size_t c0, uint32_t mask) {
      for (; mask; mask &= mask - 1) {
        const size_t c = c0 + (size_t)__builtin_ctz(mask);
        isum += c32[c];
        live.push_back((int64_t)c);
      }
    };
    for (size_t c0 = 0; c0 < N16; c0 += 16) {
      const __m128i* q = reinterpret_cast<const __m128i*>(c32 + c0);
      const uint32_t zm = (uint32_t)_mm_movemask_ps(_mm_castsi128_ps(_mm_cmpeq_epi32(_mm_loadu_si128(q), z))) |
                          (uint32_t)_mm_movemask_ps(_mm_castsi128_ps(_mm_cmpeq_epi32(_mm_loadu_si128(q + 1), z))) << 4 |
                          (uint32_t)_mm_movemask_ps(_mm_castsi128_ps(_mm_cmpeq_epi32(_mm_loadu_si128(q + 2), z))) << 8 |
                          (uint32_t)_mm_movemask_ps(_mm_castsi128_ps(_mm_cmpeq_epi32(_mm_loadu_si128(q + 3), z))) << 12;
      if (zm != 0xFFFFu) visit(c0, ~zm & 0xFFFFu);
    }
    uint32_t tail = 0;
    for (size_t c = N16; c < N; ++c) tail |= (uint32_t)(c32[c] != 0) << (c - N16);
    visit(N16, tail);
    return isum;
  }

  // every non-zero count is in live (the last scan saw them all: counts only grow between scans,
  // and clear_counts empties them)
  void reset_counts() {
    for (int64_t c : live) cnt[(size_t)c] = 0;
    if (!cnt16.empty())
      for (int64_t c : live) cnt16[(size_t)c] = 0;
  }

  // LADIES: choice over live with p[v] = pi[v] / sum(pi), the column counts (sampler.py:122);
  // p and its cumsum in one pass (the divide and the add chain overlap)
  void choose_by_counts(MT19937& rng, double total, int64_t s_num) {
    const size_t n = live.size();
    pv.resize(n);
    if (cdf_work.size() < n) cdf_work.resize(n);
    double s = 0.0;
    if (has_live_cnt) {  // device counts: already contiguous in live order
      const int32_t* lc = live_cnt.data();
      for (size_t i = 0; i < n; ++i) {
        const double q = (double)lc[i] / total;
        pv[i] = q;
        s += q;
        cdf_work[i] = s;
      }
    } else {
      for (size_t i = 0; i < n; ++i) {
        const double q = (double)cnt[(size_t)live[i]] / total;
        pv[i] = q;
        s += q;
        cdf_work[i] = s;
      }
    }
    choice_without_replacement(rng, live.data(), pv.data(), true, cdf_work.data(), n, s_num, taken, found, cdf_work,
                               xs, js);
  }

  // FastGCN: choice over the nodes with p > 0 (NaN p never live), layer-independent: the
  // candidate list, their p and the untouched cdf are kept per thread for the p array they
  // came from (identified by its address, length, 64 sampled values and the process-wide
  // generation that gnn_fastgcn_p_changed() bumps: a caller that rewrites p in place, or frees
  // it and allocates another, announces it there, so no stale candidate list is reused).
  void choose_by_p(MT19937& rng, const double* p, int64_t s_num) {
    const size_t N = g_.N;
    uint64_t sig = 1469598103934665603ull;
    for (size_t k = 0; k < 64; ++k) {
      uint64_t b;
      std::memcpy(&b, &p[(k * (N - 1)) / 63], 8);
      sig = (sig ^ b) * 1099511628211ull;
    }
    const uint64_t gen = g_fastgcn_generation.load(std::memory_order_acquire);
    if (fg_p != p || fg_n != N || fg_sig != sig || fg_gen != gen) {
      fg_live.clear();
      fg_pv.clear();
      for (size_t v = 0; v < N; ++v) {
        if (p[v] > 0.0) {
          fg_live.push_back((int64_t)v);
          fg_pv.push_back(p[v]);
        }
      }
      fg_base.resize(fg_pv.size());
      double s = 0.0;
      for (size_t i = 0; i < fg_pv.size(); ++i) {
        s += fg_pv[i];
        fg_base[i] = s;
      }
      fg_p = p;
      fg_n = N;
      fg_sig = sig;
      fg_gen = gen;
    }
    choice_without_replacement(rng, fg_live.data(), fg_pv.data(), false, fg_base.data(), fg_live.size(),
                               std::min<int64_t>((int64_t)fg_live.size(), s_num), taken, found, cdf_work, xs, js);
  }

  size_t fastgcn_candidates() const { return fg_live.size(); }

  void clear_counts() {
    for (int64_t c : live) cnt[(size_t)c] = 0;
    if (!cnt16.empty())
      for (int64_t c : live) cnt16[(size_t)c] = 0;
    in16 = false;
    rows16 = 0;
    for (int64_t v : counted_list) counted[(size_t)v] = 0;
    counted_list.clear();
  }

  // after = unique(concat(found, prev)), ascending; then the membership bitmap of `after`
  // with per-word rank prefixes (N/8 + N/16 bytes: L1/L2-resident, unlike an N-entry int32
  // map): the new column of c is rank[c / 64] + popcount(bits[c / 64] below bit c % 64).
  void make_after(const std::vector<int64_t>& prev, std::vector<int64_t>& after, bool columns = true) {
    after.assign(found.begin(), found.end());
    after.insert(after.end(), prev.begin(), prev.end());
    std::sort(after.begin(), after.end());
    after.erase(std::unique(after.begin(), after.end()), after.end());
    for (int64_t v : found) taken[(size_t)v] = 0;
    if (columns) set_columns(after);
  }

  // A layer left to the GPU extraction: its rows and columns as int32 node ids, and from the
  // column counts of U (structural: data == NULL) the exact nnz of U[:, after] and its CSC
  // column pointer — colptr[j + 1] - colptr[j] = count of U's column after[j].
  // colseg: the offsets of lapᵀ's rows of `after` concatenated (the transposed extraction's
  // segments), from indptr_t (lapᵀ's row pointer; the graph's own when NULL = symmetric).
  // Returns false if they reach 2^31 entries.
  bool device_layer(const std::vector<int64_t>& prev, const std::vector<int64_t>& after, const int64_t* indptr_t,
                    Layer& L) const {
    L.on_device = true;
    L.rows.assign(prev.begin(), prev.end());
    L.cols.assign(after.begin(), after.end());
    L.colptr.resize(after.size() + 1);
    L.colseg.resize(after.size() + 1);
    const int64_t* pt = indptr_t ? indptr_t : g_.indptr;
    int64_t acc = 0, seg = 0;
    L.colptr[0] = 0;
    L.colseg[0] = 0;
    for (size_t j = 0; j < after.size(); ++j) {
      acc += cnt[(size_t)after[j]];
      L.colptr[j + 1] = (int32_t)acc;
      seg += pt[after[j] + 1] - pt[after[j]];
      if (seg >= ((int64_t)1 << 31)) return false;
      L.colseg[j + 1] = (int32_t)seg;
    }
    L.nnz = acc;
    return true;
  }

  void set_columns(const std::vector<int64_t>& cols) {
    std::fill(bits.begin(), bits.end(), 0ull);
    for (int64_t a : cols) bits[(size_t)a >> 6] |= 1ull << (a & 63);
    int32_t acc = 0;
    for (size_t wi = 0; wi < bits.size(); ++wi) {
      wrank[wi] = acc;
      acc += (int32_t)__builtin_popcountll(bits[wi]);
    }
  }

  // adj = lap[rows, :][:, cols] (scipy column indexing with sorted unique cols): per row,
  // the entries whose column is a member, renumbered (branch-free compaction).
  void extract(const std::vector<int64_t>& rows, int64_t unnz, Layer& L) {
    L.rowptr.resize(rows.size() + 1);
    L.rowptr[0] = 0;
    if (ecap < (size_t)unnz + 1) {  // reused across calls, never value-initialised
      ecap = ((size_t)unnz + 1) * 5 / 4;
      ebuf.reset(new int32_t[ecap]);
    }
    int32_t* const base = ebuf.get();
    int32_t* w = base;
    for (size_t r = 0; r < rows.size(); ++r) {
      const int64_t v = rows[r];
      prefetch_row(rows, r + kPrefetchRows);
      for (int64_t k = g_.indptr[v], e = g_.indptr[v + 1]; k < e; ++k) {
        const uint32_t c = (uint32_t)g_.indices[k];
        const uint64_t word = bits[c >> 6];
        const uint32_t sh = c & 63u;
        *w = wrank[c >> 6] + (int32_t)__builtin_popcountll(word & ((1ull << sh) - 1ull));
        w += (word >> sh) & 1ull;
      }
      L.rowptr[r + 1] = (int32_t)(w - base);
    }
    L.colidx.assign(base, w);
    L.nnz = (int64_t)L.colidx.size();
  }

  // normfact = 1 / float32(clip(s_num * p[cols], 1e-10, 1))  (sampler.py:137: float32 division)
  void normfact(const std::vector<int64_t>& cols, double total, int64_t s_num, Layer& L) const {
    L.normfact.resize(cols.size());
    const double sn = (double)s_num;
    for (size_t j = 0; j < cols.size(); ++j) {
      double q = sn * ((double)cnt[(size_t)cols[j]] / total);
      q = q < 1e-10 ? 1e-10 : (q > 1.0 ? 1.0 : q);  // NaN passes through, as np.clip
      L.normfact[j] = 1.0f / (float)q;
    }
  }

  // same, with p given: 1 / float32(clip(s_num * p[cols], 1e-10, 1))
  static void normfact_p(const std::vector<int64_t>& cols, const double* p, int64_t s_num, Layer& L) {
    L.normfact.resize(cols.size());
    const double sn = (double)s_num;
    for (size_t j = 0; j < cols.size(); ++j) {
      double q = sn * p[cols[j]];
      q = q < 1e-10 ? 1e-10 : (q > 1.0 ? 1.0 : q);
      L.normfact[j] = 1.0f / (float)q;
    }
  }

  // sampled_nodes = where(isin(after, prev))
  void positions(const std::vector<int64_t>& after, const std::vector<int64_t>& prev, Layer& L) {
    for (int64_t v : prev) in_prev[(size_t)v] = 1;
    L.sampled.clear();
    for (size_t j = 0; j < after.size(); ++j)
      if (in_prev[(size_t)after[j]]) L.sampled.push_back((int64_t)j);
    for (int64_t v : prev) in_prev[(size_t)v] = 0;
  }

  Graph g_;
  std::unique_ptr<int32_t[]> ebuf;  // extract scratch (unnz + 1 entries)
  size_t ecap = 0;
  std::vector<int32_t> cnt;  // column nonzero counts of U (< nnz < 2^31)
  std::vector<uint64_t> bits;
  std::vector<int32_t> wrank;
  std::vector<uint8_t> taken, in_prev, counted;
  std::vector<int64_t> live, found, counted_list, newrows;
  std::vector<double> pv, cdf_work, xs;  // choice scratch
  std::vector<uint32_t> js;
  std::vector<int32_t> live_cnt;  // cnt[live[i]] in live order (device counts)
  bool has_live_cnt = false;
  std::vector<int64_t> fg_live;          // FastGCN candidates (see choose_by_p)
  std::vector<double> fg_pv, fg_base;
  const double* fg_p = nullptr;
  size_t fg_n = 0;
  uint64_t fg_sig = 0;
  uint64_t fg_gen = ~0ull;
  bool clean_ = true;
};

int check_inputs(const char* who, const int64_t* indptr, const int32_t* indices, int64_t num_nodes,
                 const int64_t* batch_nodes, int64_t batch_size, const int64_t* samp_num, const int32_t* orders,
                 int32_t num_layers, void* out) {
  if (!out) return fail("%s: out is NULL", who);
  if (num_nodes <= 0 || num_nodes >= (int64_t)1 << 31) return fail("%s: num_nodes out of range", who);
  if (!indptr || !indices) return fail("%s: NULL graph", who);
  if (batch_size < 0 || (batch_size > 0 && !batch_nodes)) return fail("%s: bad batch", who);
  if (num_layers < 0 || (num_layers > 0 && (!samp_num || !orders))) return fail("%s: bad layers", who);
  for (int64_t i = 0; i < batch_size; ++i)
    if (batch_nodes[i] < 0 || batch_nodes[i] >= num_nodes) return fail("%s: batch node out of range", who);
  return 0;
}

}  // namespace


namespace gnn_smp {

void layer_csc(const Layer& L, int32_t* colptr, int32_t* rows) {
  // stable counting sort of the entries by column: rows come out ascending in each column
  std::fill(colptr, colptr + L.K + 1, 0);
  for (int32_t c : L.colidx) ++colptr[c + 1];
  for (int64_t c = 0; c < L.K; ++c) colptr[c + 1] += colptr[c];
  std::vector<int32_t> cur(colptr, colptr + L.K);
  for (int64_t i = 0; i < L.M; ++i)
    for (int32_t k = L.rowptr[(size_t)i]; k < L.rowptr[(size_t)i + 1]; ++k) rows[cur[(size_t)L.colidx[(size_t)k]]++] = (int32_t)i;
}

void set_error(const std::string& msg) { g_err = msg; }

}  // namespace gnn_smp

extern "C" {

const char* gnn_sampler_last_error(void) { return g_err.c_str(); }

int gnn_sampler_profile(double* out, int32_t n, int32_t reset) {
  if (!out || n < 0) return fail("gnn_sampler_profile: bad arguments");
  for (int32_t i = 0; i < n && i < P_NPHASE; ++i) {
    const int64_t v = reset ? g_prof[i].exchange(0) : g_prof[i].load();
    out[i] = i == P_CALLS ? (double)v : (double)v * 1e-9;
  }
  return g_prof_on ? 0 : 1;
}

int gnn_mt19937_random_sample(uint32_t seed, int64_t n, double* out) {
  if (n < 0 || (n > 0 && !out)) return fail("gnn_mt19937_random_sample: bad arguments");
  MT19937 rng(seed);
  for (int64_t i = 0; i < n; ++i) out[i] = rng.next_double();
  return 0;
}

int gnn_ladies_sample(const int64_t* indptr, const int32_t* indices, const float* data, int64_t num_nodes,
                      const int64_t* batch_nodes, int64_t batch_size, const int64_t* samp_num,
                      const int32_t* orders, int32_t num_layers, uint32_t seed, gnn_ladies_result** out) {
  return gnn_ladies_sample_dev(indptr, indices, data, nullptr, num_nodes, batch_nodes, batch_size, samp_num, orders,
                               num_layers, seed, 0, out);
}

int gnn_ladies_sample_dev(const int64_t* indptr, const int32_t* indices, const float* data, const int64_t* indptr_t,
                          int64_t num_nodes,
                          const int64_t* batch_nodes, int64_t batch_size, const int64_t* samp_num,
                          const int32_t* orders, int32_t num_layers, uint32_t seed, int32_t device_extract,
                          gnn_ladies_result** out) {
  return gnn_ladies_sample_cc(indptr, indices, data, indptr_t, num_nodes, batch_nodes, batch_size, samp_num, orders,
                              num_layers, seed, device_extract, nullptr, nullptr, out);
}

int gnn_ladies_sample_cc(const int64_t* indptr, const int32_t* indices, const float* data, const int64_t* indptr_t,
                         int64_t num_nodes, const int64_t* batch_nodes, int64_t batch_size, const int64_t* samp_num,
                         const int32_t* orders, int32_t num_layers, uint32_t seed, int32_t device_extract,
                         const gnn_colcount_api* cc, void* cc_ctx, gnn_ladies_result** out) {
  if (int rc = check_inputs("gnn_ladies_sample", indptr, indices, num_nodes, batch_nodes, batch_size, samp_num,
                            orders, num_layers, out))
    return rc;
  if (device_extract && data)
    return fail("gnn_ladies_sample_dev: device extraction needs a graph without stored zeros (data == NULL)");
  if (cc && (!cc_ctx || !cc->add || !cc->reset || data))
    return fail("gnn_ladies_sample_cc: device counting needs a context and a graph without stored zeros");
  *out = nullptr;
  try {
    const Graph g{indptr, indices, data, (size_t)num_nodes};
    PhaseClock clk;
    Work& w = Work::acquire(g);
    std::unique_ptr<gnn_ladies_result> res(new gnn_ladies_result());
    res->layers.resize((size_t)num_layers);
    MT19937 rng(seed);
    std::vector<int64_t> prev(batch_nodes, batch_nodes + batch_size), after;
    clk.lap(P_SCRATCH);
    if (g_prof_on) g_prof[P_CALLS].fetch_add(1, std::memory_order_relaxed);
    // A batch with repeated nodes repeats rows of U (counted twice); later layers' rows are
    // unique. Counts carry over between layers only when every layer's rows are unique.
    bool nested = true;
    for (int64_t v : prev) {
      if (w.in_prev[(size_t)v]) nested = false;
      w.in_prev[(size_t)v] = 1;
    }
    for (int64_t v : prev) w.in_prev[(size_t)v] = 0;
    if (cc) {
      if (int rc = cc->reset(cc_ctx)) return fail("gnn_ladies_sample: device column count reset failed (%d)", rc);
    }
    bool top = true;  // the first sampled layer: its rows are the batch (any order, repeats)
    for (int32_t d = 0; d < num_layers; ++d) {
      Layer& L = res->layers[(size_t)(num_layers - 1 - d)];  // stored bottom-up
      if (orders[num_layers - 1 - d] == 0) continue;         // orders1 = orders[::-1]
      L.present = true;
      // below the top layer rows = np.unique(...) of the layer above; device_extract is a mask
      // over the (bottom-up) layer index, -1 = every layer below the top one
      const bool dev = !top && ((device_extract >> (num_layers - 1 - d)) & 1);
      top = false;
      clk.lap(P_TAIL);
      const int64_t unnz = w.row_pointers(prev, L.fullrowptr);  // U = lap[prev, :]
      if (unnz < 0) return fail("gnn_ladies_sample: sub-graph nnz >= 2^31");
      clk.lap(P_ROWPTR);
      // p = pi / sum(pi): exact integer sum
      int cc_rc = 0;
      const int64_t isum = cc ? w.count_columns_device(prev, nested, cc, cc_ctx, &cc_rc)
                              : (nested ? w.count_columns_nested(prev) : w.count_columns(prev));
      if (cc_rc) return fail("gnn_ladies_sample: device column count failed (%d)", cc_rc);
      clk.lap(P_COUNT);
      if (isum == 0)  // p = 0/0: numpy's choice raises "probabilities contain NaN"
        return fail("gnn_ladies_sample: probabilities contain NaN (layer %d: no entries in U)", d);
      const double total = (double)isum;
      const int64_t s_num = std::min<int64_t>((int64_t)w.live.size(), samp_num[d]);
      L.s_num = s_num;
      w.choose_by_counts(rng, total, s_num);
      clk.lap(P_DRAW);
      w.make_after(prev, after, !dev);
      clk.lap(P_AFTER);
      if (dev) {
        if (!w.device_layer(prev, after, indptr_t, L) || L.nnz >= ((int64_t)1 << 31))
          return fail("gnn_ladies_sample: sub-graph nnz >= 2^31");
      } else {
        w.extract(prev, unnz, L);
      }
      clk.lap(P_EXTRACT);
      w.normfact(after, total, s_num, L);
      w.positions(after, prev, L);
      L.M = (int64_t)prev.size();
      L.K = (int64_t)after.size();
      if (!nested) {
        w.clear_counts();
        nested = true;  // after = unique(...): from here on every layer's rows are unique
        if (cc) {
          if (int rc = cc->reset(cc_ctx)) return fail("gnn_ladies_sample: device column count reset failed (%d)", rc);
        }
      }
      prev.swap(after);  // after ⊇ prev: the next layer's counts extend these
    }
    res->input_nodes = prev;
    *out = res.release();
    w.finish();
    clk.lap(P_TAIL);
    return 0;
  } catch (const std::bad_alloc&) {
    return fail("gnn_ladies_sample: out of host memory");
  }
}

int gnn_subgraph_sample(const int64_t* indptr, const int32_t* indices, const float* data, int64_t num_nodes,
                        const int64_t* batch_nodes, int64_t batch_size, const int64_t* samp_num,
                        const int32_t* orders, int32_t num_layers, uint32_t seed, gnn_ladies_result** out) {
  if (int rc = check_inputs("gnn_subgraph_sample", indptr, indices, num_nodes, batch_nodes, batch_size, samp_num,
                            orders, num_layers, out))
    return rc;
  *out = nullptr;
  try {
    const Graph g{indptr, indices, data, (size_t)num_nodes};
    Work& w = Work::acquire(g);
    std::unique_ptr<gnn_ladies_result> res(new gnn_ladies_result());
    res->layers.resize((size_t)num_layers);
    MT19937 rng(seed);
    const std::vector<int64_t> batch(batch_nodes, batch_nodes + batch_size);
    std::vector<int64_t> after;
    // One importance draw from the batch's neighbourhood (sampler.py:19-38) ...
    Layer first;
    const int64_t unnz = w.row_pointers(batch, first.fullrowptr);
    if (unnz < 0) return fail("gnn_subgraph_sample: sub-graph nnz >= 2^31");
    const int64_t isum = w.count_columns(batch);
    if (isum == 0) return fail("gnn_subgraph_sample: probabilities contain NaN (no entries in U)");
    const double total = (double)isum;
    const int64_t s_num = std::min<int64_t>((int64_t)w.live.size(), samp_num[0]);
    w.choose_by_counts(rng, total, s_num);
    w.make_after(batch, after);
    // ... the top-most layer with a non-zero order takes U[:, after] (sampler.py:42-53) ...
    int32_t d = 0;
    for (; d < num_layers; ++d) {
      if (orders[num_layers - 1 - d] == 0) continue;
      Layer& L = res->layers[(size_t)(num_layers - 1 - d)];
      L = std::move(first);
      L.present = true;
      L.s_num = s_num;
      w.extract(batch, unnz, L);
      w.normfact(after, total, s_num, L);
      w.positions(after, batch, L);
      L.M = (int64_t)batch.size();
      L.K = (int64_t)after.size();
      ++d;
      break;
    }
    // ... and EVERY layer below it (whatever its order, sampler.py:55-69) the square
    // sub-graph lap[after, :][:, after], same normfact, sampled_nodes = arange(len(after)).
    for (; d < num_layers; ++d) {
      Layer& L = res->layers[(size_t)(num_layers - 1 - d)];
      L.present = true;
      L.s_num = s_num;
      const int64_t n2 = w.row_pointers(after, L.fullrowptr);
      if (n2 < 0) return fail("gnn_subgraph_sample: sub-graph nnz >= 2^31");
      w.extract(after, n2, L);
      w.normfact(after, total, s_num, L);
      L.sampled.resize(after.size());
      for (size_t j = 0; j < after.size(); ++j) L.sampled[j] = (int64_t)j;
      L.M = L.K = (int64_t)after.size();
    }
    res->input_nodes = after;
    *out = res.release();
    w.finish();
    return 0;
  } catch (const std::bad_alloc&) {
    return fail("gnn_subgraph_sample: out of host memory");
  }
}

void gnn_fastgcn_p_changed(void) { g_fastgcn_generation.fetch_add(1, std::memory_order_acq_rel); }

int gnn_fastgcn_sample(const int64_t* indptr, const int32_t* indices, const float* data, int64_t num_nodes,
                       const double* p, const int64_t* batch_nodes, int64_t batch_size, const int64_t* samp_num,
                       const int32_t* orders, int32_t num_layers, uint32_t seed, gnn_ladies_result** out) {
  if (int rc = check_inputs("gnn_fastgcn_sample", indptr, indices, num_nodes, batch_nodes, batch_size, samp_num,
                            orders, num_layers, out))
    return rc;
  if (!p) return fail("gnn_fastgcn_sample: p is NULL");
  *out = nullptr;
  try {
    const Graph g{indptr, indices, data, (size_t)num_nodes};
    PhaseClock clk;
    Work& w = Work::acquire(g);
    if (g_prof_on) g_prof[P_CALLS].fetch_add(1, std::memory_order_relaxed);
    std::unique_ptr<gnn_ladies_result> res(new gnn_ladies_result());
    res->layers.resize((size_t)num_layers);
    MT19937 rng(seed);
    std::vector<int64_t> prev(batch_nodes, batch_nodes + batch_size), after;
    for (int32_t d = 0; d < num_layers; ++d) {
      Layer& L = res->layers[(size_t)(num_layers - 1 - d)];
      if (orders[num_layers - 1 - d] == 0) continue;
      L.present = true;
      clk.lap(P_TAIL);
      const int64_t unnz = w.row_pointers(prev, L.fullrowptr);  // U = lap[prev, :]
      clk.lap(P_ROWPTR);
      if (unnz < 0) return fail("gnn_fastgcn_sample: sub-graph nnz >= 2^31");
      // the layer-independent importance: candidates = ascending nodes with p > 0
      w.choose_by_p(rng, p, samp_num[d]);
      clk.lap(P_DRAW);
      const int64_t s_num = std::min<int64_t>((int64_t)w.fastgcn_candidates(), samp_num[d]);
      L.s_num = s_num;
      // after = unique(sampled): layers are sampled independently (no union with prev)
      after.assign(w.found.begin(), w.found.end());
      std::sort(after.begin(), after.end());
      for (int64_t v : w.found) w.taken[(size_t)v] = 0;
      w.set_columns(after);
      clk.lap(P_AFTER);
      w.extract(prev, unnz, L);
      clk.lap(P_EXTRACT);
      Work::normfact_p(after, p, s_num, L);
      w.positions(after, prev, L);
      L.M = (int64_t)prev.size();
      L.K = (int64_t)after.size();
      prev.swap(after);
    }
    res->input_nodes = prev;
    *out = res.release();
    w.finish();
    return 0;
  } catch (const std::bad_alloc&) {
    return fail("gnn_fastgcn_sample: out of host memory");
  }
}

int gnn_ladies_layer_dims(const gnn_ladies_result* r, int32_t layer, int64_t dims[5]) {
  if (!r || !dims || layer < 0 || (size_t)layer >= r->layers.size()) return fail("gnn_ladies_layer_dims: bad args");
  const Layer& L = r->layers[(size_t)layer];
  dims[0] = L.M;
  dims[1] = L.K;
  dims[2] = L.nnz;
  dims[3] = (int64_t)L.sampled.size();
  dims[4] = L.s_num;
  return L.present ? 0 : 1;
}

int gnn_ladies_layer_copy(const gnn_ladies_result* r, int32_t layer, int32_t* fullrowptr, int32_t* rowptr,
                          int32_t* colidx, float* normfact, int64_t* sampled) {
  if (!r || layer < 0 || (size_t)layer >= r->layers.size()) return fail("gnn_ladies_layer_copy: bad args");
  const Layer& L = r->layers[(size_t)layer];
  auto cp = [](void* dst, const void* src, size_t bytes) {
    if (dst && bytes) std::memcpy(dst, src, bytes);
  };
  // (on_device layers: fullrowptr / rowptr / colidx are not made; nothing is copied for them)
  cp(fullrowptr, L.fullrowptr.data(), L.fullrowptr.size() * 4);
  cp(rowptr, L.rowptr.data(), L.rowptr.size() * 4);
  cp(colidx, L.colidx.data(), L.colidx.size() * 4);
  cp(normfact, L.normfact.data(), L.normfact.size() * 4);
  cp(sampled, L.sampled.data(), L.sampled.size() * 8);
  return 0;
}

int gnn_ladies_layer_device(const gnn_ladies_result* r, int32_t layer, int32_t* rows, int32_t* cols,
                            int32_t* colptr, int32_t* rowseg, int32_t* colseg) {
  if (!r || layer < 0 || (size_t)layer >= r->layers.size()) return fail("gnn_ladies_layer_device: bad args");
  const Layer& L = r->layers[(size_t)layer];
  if (!L.present || !L.on_device) return 1;
  if (rows && !L.rows.empty()) std::memcpy(rows, L.rows.data(), L.rows.size() * 4);
  if (cols && !L.cols.empty()) std::memcpy(cols, L.cols.data(), L.cols.size() * 4);
  if (colptr) std::memcpy(colptr, L.colptr.data(), L.colptr.size() * 4);
  if (rowseg) std::memcpy(rowseg, L.fullrowptr.data(), L.fullrowptr.size() * 4);
  if (colseg) std::memcpy(colseg, L.colseg.data(), L.colseg.size() * 4);
  return 0;
}

int gnn_ladies_layer_csc(const gnn_ladies_result* r, int32_t layer, int32_t* colptr, int32_t* rows) {
  if (!r || layer < 0 || (size_t)layer >= r->layers.size()) return fail("gnn_ladies_layer_csc: bad args");
  const Layer& L = r->layers[(size_t)layer];
  if (!L.present) return fail("gnn_ladies_layer_csc: layer %d has no sub-graph", layer);
  if (L.on_device) return fail("gnn_ladies_layer_csc: layer %d is extracted on the device", layer);
  if (!colptr || (!rows && !L.colidx.empty())) return fail("gnn_ladies_layer_csc: NULL output");
  gnn_smp::layer_csc(L, colptr, rows);
  return 0;
}

int64_t gnn_ladies_num_input_nodes(const gnn_ladies_result* r) { return r ? (int64_t)r->input_nodes.size() : -1; }

int gnn_ladies_input_nodes(const gnn_ladies_result* r, int64_t* out) {
  if (!r || (!out && !r->input_nodes.empty())) return fail("gnn_ladies_input_nodes: bad args");
  if (!r->input_nodes.empty()) std::memcpy(out, r->input_nodes.data(), r->input_nodes.size() * 8);
  return 0;
}

void gnn_ladies_free(gnn_ladies_result* r) { delete r; }

int gnn_host_gather_rows_f32(const float* src, int64_t ld_src, int64_t num_src_rows, const int64_t* idx, int64_t n,
                             int64_t F, float* dst, int64_t ld_dst) {
  if (n < 0 || F < 0 || F > ld_src || F > ld_dst || (n > 0 && (!src || !idx || !dst)))
    return fail("gnn_host_gather_rows_f32: bad arguments");
  for (int64_t i = 0; i < n; ++i)
    if (idx[i] < 0 || idx[i] >= num_src_rows) return fail("gnn_host_gather_rows_f32: index %lld out of range", (long long)idx[i]);
  for (int64_t i = 0; i < n; ++i) {
    float* d = dst + i * ld_dst;
    std::memcpy(d, src + idx[i] * ld_src, (size_t)F * sizeof(float));
    if (ld_dst > F) std::memset(d + F, 0, (size_t)(ld_dst - F) * sizeof(float));
  }
  return 0;
}

}  // extern "C"
