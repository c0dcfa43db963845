// colcount.hip — the LADIES draw's column counts of U = lap[rows, :] on the GPU
// (include/gnn_extract.h: gnn_colcount_*).
//
// Reference: sampler.py:116-122 — pi = sp.linalg.norm(U, ord=0, axis=0), p = pi / sum(pi). The
// host sampler counts U's columns with one random increment per graph entry (4.2 M per
// ogbn-products batch: half of the host's per-batch time on the box), while the graph is already
// resident in HBM for the layer extraction (gnn_ladies_extract_f32). Here a producer thread hands
// over the rows a layer adds (the LADIES layers are nested: each layer's rows extend the previous
// layer's, so the counts carry over), the GPU adds their entries into a per-context count array,
// and the thread gets back what the draw needs: the bitmap of non-zero columns (N / 8 bytes) and
// their counts in ascending column order — the host's `live` list and cnt[live], exactly (integer
// counts; the draw itself stays on the host, bit-identical).
//
// Per call: rows H2D (int32), hist (a wave per row, one integer atomicAdd per entry — counts are
// order-independent, so the result is deterministic), live_count (per 4096-column block: ballots
// of cnt > 0), one scan, live_write (bitmap words + compacted counts), D2H of the bitmap and the
// total, then of the counts. Everything on the context's own stream; two host waits per call.
#include <hip/hip_runtime.h>

#include <climits>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <vector>

#include "common.h"
#include "gnn_extract.h"

namespace {

using gnn::ceil_div;

#define GNN_TRY_CC(x)     \
  do {                    \
    int rc_ = (x);        \
    if (rc_) return rc_;  \
  } while (0)

constexpr int CC_WAVES = 4;                      // waves per workgroup
constexpr int CC_ITERS = 16;                     // 64-column chunks per wave
constexpr int CC_BLOCK = CC_WAVES * CC_ITERS * 64;  // columns per workgroup (4096)

// cnt[c] += 1 for every entry of the given rows (a wave per row, grid-stride over rows)
__global__ __launch_bounds__(256) void cc_hist_kernel(const int32_t* __restrict__ rows, int n,
                                                      const int64_t* __restrict__ indptr,
                                                      const int32_t* __restrict__ indices, int32_t* __restrict__ cnt) {
  const int lane = threadIdx.x & 63;
  const int wave = (int)((blockIdx.x * blockDim.x + threadIdx.x) >> 6);
  const int nwaves = (int)((gridDim.x * blockDim.x) >> 6);
  for (int r = wave; r < n; r += nwaves) {
    const int64_t v = rows[r];
    const int64_t b = indptr[v], e = indptr[v + 1];
    for (int64_t k = b + lane; k < e; k += 64) atomicAdd(&cnt[indices[k]], 1);
  }
}

// blk[b] = number of columns with cnt > 0 in workgroup b's 4096 columns
__global__ __launch_bounds__(256) void cc_live_count_kernel(const int32_t* __restrict__ cnt, int64_t N,
                                                            int32_t* __restrict__ blk) {
  __shared__ int wsum[CC_WAVES];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t base = (int64_t)blockIdx.x * CC_BLOCK + (int64_t)w * CC_ITERS * 64;
  int s = 0;
#pragma unroll 4
  for (int it = 0; it < CC_ITERS; ++it) {
    const int64_t c = base + it * 64 + lane;
    const bool nz = c < N && cnt[c] > 0;
    s += __popcll(__ballot(nz));
  }
  if (lane == 0) wsum[w] = s;
  __syncthreads();
  if (threadIdx.x == 0) blk[blockIdx.x] = (wsum[0] + wsum[1]) + (wsum[2] + wsum[3]);
}

// bitmap words and the counts of the non-zero columns at their ascending-column positions
__global__ __launch_bounds__(256) void cc_live_write_kernel(const int32_t* __restrict__ cnt, int64_t N,
                                                            const int32_t* __restrict__ blk_off,
                                                            uint64_t* __restrict__ bits, int32_t* __restrict__ out) {
  __shared__ int wsum[CC_WAVES];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t base = (int64_t)blockIdx.x * CC_BLOCK + (int64_t)w * CC_ITERS * 64;
  int32_t v[CC_ITERS];
  uint64_t m[CC_ITERS];
  int s = 0;
#pragma unroll
  for (int it = 0; it < CC_ITERS; ++it) {
    const int64_t c = base + it * 64 + lane;
    v[it] = c < N ? cnt[c] : 0;
    m[it] = __ballot(v[it] > 0);
    s += __popcll(m[it]);
  }
  if (lane == 0) wsum[w] = s;
  __syncthreads();
  int off = blk_off[blockIdx.x];
  for (int j = 0; j < w; ++j) off += wsum[j];
  const uint64_t below = (1ull << lane) - 1ull;
#pragma unroll
  for (int it = 0; it < CC_ITERS; ++it) {
    const int64_t c0 = base + it * 64;
    if (c0 < N && lane == 0) bits[c0 >> 6] = m[it];
    if (v[it] > 0) out[off + __popcll(m[it] & below)] = v[it];
    off += __popcll(m[it]);
  }
}

struct ColCount {
  int device = 0;
  int64_t N = 0, W = 0, NB = 0;
  const int64_t* indptr = nullptr;
  const int32_t* indices = nullptr;
  hipStream_t st = nullptr;
  int32_t* cnt = nullptr;      // device [N]
  uint64_t* bits = nullptr;    // device [W]
  int32_t* blk = nullptr;      // device [NB]
  int32_t* blk_off = nullptr;  // device [NB + 1]
  int32_t* out = nullptr;      // device [N]
  int32_t* rows_d = nullptr;   // device [rows_cap]
  int64_t rows_cap = 0;
  int32_t* rows_h = nullptr;   // pinned [rows_cap]
  uint64_t* bits_h = nullptr;  // pinned [W]
  int32_t* total_h = nullptr;  // pinned [1]
  int32_t* out_h = nullptr;    // pinned [N]

  ~ColCount() {
    if (st) (void)hipStreamSynchronize(st);
    for (void* p : {(void*)cnt, (void*)bits, (void*)blk, (void*)blk_off, (void*)out, (void*)rows_d})
      if (p) (void)hipFree(p);
    for (void* p : {(void*)rows_h, (void*)bits_h, (void*)total_h, (void*)out_h})
      if (p) (void)hipHostFree(p);
    if (st) (void)hipStreamDestroy(st);
  }
};

int grow_rows(ColCount* c, int64_t n) {
  if (n <= c->rows_cap) return 0;
  const int64_t cap = n + n / 2 + 1024;
  if (c->rows_d) GNN_HIP(hipFree(c->rows_d), "hipFree");
  if (c->rows_h) GNN_HIP(hipHostFree(c->rows_h), "hipHostFree");
  c->rows_d = nullptr;
  c->rows_h = nullptr;
  c->rows_cap = 0;
  GNN_HIP(hipMalloc(&c->rows_d, (size_t)cap * 4), "hipMalloc");
  GNN_HIP(hipHostMalloc(&c->rows_h, (size_t)cap * 4, hipHostMallocDefault), "hipHostMalloc");
  c->rows_cap = cap;
  return 0;
}

}  // namespace

extern "C" {

int gnn_colcount_create(int32_t device, int64_t num_nodes, const int64_t* indptr, const int32_t* indices, void** ctx) {
  GNN_REQUIRE(ctx != nullptr, "gnn_colcount_create: ctx is NULL");
  *ctx = nullptr;
  GNN_REQUIRE(num_nodes > 0 && num_nodes < INT32_MAX && indptr && indices, "gnn_colcount_create: bad graph");
  GNN_HIP(hipSetDevice(device), "hipSetDevice");
  std::unique_ptr<ColCount> c(new ColCount());
  c->device = device;
  c->N = num_nodes;
  c->W = ceil_div(num_nodes, 64);
  c->NB = ceil_div(num_nodes, CC_BLOCK);
  c->indptr = indptr;
  c->indices = indices;
  // The producers' counting runs beside the training step. GNN_CC_CUS = n > 0 puts it on a
  // CU-masked stream over n of the device's CUs (spread evenly; n = all CUs: a mask of every CU),
  // which gets a hardware queue of its own: the products-shaped GPU step then runs at 957-977
  // mini-batches/s instead of 450-480 when the two overlap — but in the end-to-end run the counts
  // (~1.2 ms of kernels and copies per batch) then take more of the GPU from the step and the rate
  // drops 453-470 -> 404-436 (profiles/round5/configs/, r5ah, r5an) — so by default (0) the streams
  // are plain ones.
  int cus = 0;
  if (const char* e = getenv("GNN_CC_CUS")) cus = atoi(e);
  int ncu = 0;
  GNN_HIP(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, device), "hipDeviceGetAttribute");
  if (cus > 0 && cus <= ncu) {
    std::vector<uint32_t> mask((size_t)(ncu + 31) / 32, 0u);
    const int stride = ncu / cus;
    for (int i = 0, k = 0; i < ncu && k < cus; i += stride, ++k) mask[(size_t)i / 32] |= 1u << (i % 32);
    if (hipExtStreamCreateWithCUMask(&c->st, (uint32_t)mask.size(), mask.data()) != hipSuccess) {
      (void)hipGetLastError();
      c->st = nullptr;
    }
  }
  if (!c->st) GNN_HIP(hipStreamCreateWithFlags(&c->st, hipStreamNonBlocking), "hipStreamCreateWithFlags");
  GNN_HIP(hipMalloc(&c->cnt, (size_t)c->N * 4), "hipMalloc");
  GNN_HIP(hipMalloc(&c->bits, (size_t)c->W * 8), "hipMalloc");
  GNN_HIP(hipMalloc(&c->blk, (size_t)c->NB * 4), "hipMalloc");
  GNN_HIP(hipMalloc(&c->blk_off, (size_t)(c->NB + 1) * 4), "hipMalloc");
  GNN_HIP(hipMalloc(&c->out, (size_t)c->N * 4), "hipMalloc");
  GNN_HIP(hipHostMalloc(&c->bits_h, (size_t)c->W * 8, hipHostMallocDefault), "hipHostMalloc");
  GNN_HIP(hipHostMalloc(&c->total_h, 4, hipHostMallocDefault), "hipHostMalloc");
  GNN_HIP(hipHostMalloc(&c->out_h, (size_t)c->N * 4, hipHostMallocDefault), "hipHostMalloc");
  GNN_HIP(hipMemsetAsync(c->cnt, 0, (size_t)c->N * 4, c->st), "hipMemsetAsync");
  GNN_HIP(hipStreamSynchronize(c->st), "hipStreamSynchronize");
  *ctx = c.release();
  return 0;
}

int gnn_colcount_add(void* ctx, const int64_t* rows, int64_t n, int64_t* nlive, const uint64_t** bits,
                     const int32_t** counts) {
  ColCount* c = static_cast<ColCount*>(ctx);
  GNN_REQUIRE(c && nlive && bits && counts && n >= 0 && (n == 0 || rows), "gnn_colcount_add: bad arguments");
  GNN_HIP(hipSetDevice(c->device), "hipSetDevice");
  if (n > 0) {
    GNN_TRY_CC(grow_rows(c, n));
    for (int64_t i = 0; i < n; ++i) {
      GNN_REQUIRE(rows[i] >= 0 && rows[i] < c->N, "gnn_colcount_add: row %lld out of range", (long long)rows[i]);
      c->rows_h[i] = (int32_t)rows[i];
    }
    GNN_HIP(hipMemcpyAsync(c->rows_d, c->rows_h, (size_t)n * 4, hipMemcpyHostToDevice, c->st), "hipMemcpyAsync");
    const int64_t waves = n < 8192 ? n : 8192;
    cc_hist_kernel<<<dim3((unsigned)ceil_div(waves, 4)), dim3(256), 0, c->st>>>(c->rows_d, (int)n, c->indptr,
                                                                                c->indices, c->cnt);
    GNN_LAUNCHED("cc_hist_kernel");
  }
  cc_live_count_kernel<<<dim3((unsigned)c->NB), dim3(256), 0, c->st>>>(c->cnt, c->N, c->blk);
  GNN_LAUNCHED("cc_live_count_kernel");
  GNN_TRY_CC(gnn::launch_scan_exclusive(c->blk, (int)c->NB, c->blk_off, c->st));
  cc_live_write_kernel<<<dim3((unsigned)c->NB), dim3(256), 0, c->st>>>(c->cnt, c->N, c->blk_off, c->bits, c->out);
  GNN_LAUNCHED("cc_live_write_kernel");
  GNN_HIP(hipMemcpyAsync(c->bits_h, c->bits, (size_t)c->W * 8, hipMemcpyDeviceToHost, c->st), "hipMemcpyAsync");
  GNN_HIP(hipMemcpyAsync(c->total_h, c->blk_off + c->NB, 4, hipMemcpyDeviceToHost, c->st), "hipMemcpyAsync");
  GNN_HIP(hipStreamSynchronize(c->st), "hipStreamSynchronize");
  const int64_t total = *c->total_h;
  GNN_REQUIRE(total >= 0 && total <= c->N, "gnn_colcount_add: bad live count %lld", (long long)total);
  if (total > 0) {
    GNN_HIP(hipMemcpyAsync(c->out_h, c->out, (size_t)total * 4, hipMemcpyDeviceToHost, c->st), "hipMemcpyAsync");
    GNN_HIP(hipStreamSynchronize(c->st), "hipStreamSynchronize");
  }
  *nlive = total;
  *bits = c->bits_h;
  *counts = c->out_h;
  return 0;
}

int gnn_colcount_reset(void* ctx) {
  ColCount* c = static_cast<ColCount*>(ctx);
  GNN_REQUIRE(c != nullptr, "gnn_colcount_reset: ctx is NULL");
  GNN_HIP(hipSetDevice(c->device), "hipSetDevice");
  GNN_HIP(hipMemsetAsync(c->cnt, 0, (size_t)c->N * 4, c->st), "hipMemsetAsync");
  return 0;
}

void gnn_colcount_destroy(void* ctx) {
  ColCount* c = static_cast<ColCount*>(ctx);
  if (!c) return;
  (void)hipSetDevice(c->device);
  delete c;
}

}  // extern "C"
