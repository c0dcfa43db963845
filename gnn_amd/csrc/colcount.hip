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
// Per call: rows H2D (int32), the histogram, live_count (per 4096-column block: ballots of
// cnt > 0), one scan, live_write (bitmap words + compacted counts), D2H of the bitmap and the
// total, then of the counts. Everything on the context's own stream; two host waits per call.
//
// The histogram (counts are integers and order-independent: every form below gives the same
// cnt). One global atomicAdd per entry (cc_hist_kernel) executes at the memory side, not in L2
// (MI355X_MICROARCH.md §Global float atomics): ~90 µs per products-shaped call, and that traffic
// crosses the fabric while the training step runs. The default form partitions instead: the
// entries' columns are split into buckets of 2^13 columns (cc_part_count: an LDS histogram of the
// buckets per workgroup, one LDS add per run of same-bucket lanes; a chunked scan gives every
// (bucket, workgroup) its slot range; cc_part_scatter: the 13-bit offsets written there), then one
// workgroup per bucket adds its entries in LDS and writes its 8,192 columns' sums into cnt
// (cc_bucket_add) — no global atomics. Its kernels take longer in isolation (≈130 µs per call
// against 90: the partition reads every row twice), but the products-shaped end-to-end rate is 4 %
// higher with it (A/B pairs on six boxes, profiles/round5/colcount_part/). The offsets buffer
// grows to the largest call seen: a call with more entries than it holds runs the atomic kernel
// instead (cc_hist_guard, which does nothing otherwise). GNN_CC_HIST=atomic selects the atomic form.
// The (bucket, workgroup) offsets are int32, so the call's entry total is also summed in int64
// (cc_part_count) and every partition kernel checks THAT against the capacity (itself at most
// INT32_MAX): a call of 2^31 or more entries runs the atomic form instead of wrapping an offset.
#include <hip/hip_runtime.h>

#include <atomic>

#include <algorithm>
#include <climits>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <vector>

#include "common.h"
#include "gnn_extract.h"

// gnn_colcount_set_cus: the CU mask of the streams of contexts created from now on (0: plain)
static std::atomic<int> g_cc_cus{0};

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

constexpr int CB_SHIFT = 13;                // columns per bucket: 2^13 (32 KB of LDS counters)
constexpr int CB_COLS = 1 << CB_SHIFT;
constexpr int CB_MAX = 8192;                 // buckets (32 KB of LDS in the partition kernels)
constexpr int CP_WAVES = 4;                  // waves per partition workgroup, a wave per row
constexpr int CP_U = 16;                     // 64-entry pieces of a row loaded at once

// A row's columns are ascending, so the lanes of one 64-entry piece that fall in one bucket are
// consecutive: each run's first lane adds the run's length (one LDS atomic per run, not per entry
// — per-entry adds to the same counter serialise up to 64-way).
struct Run {
  int bk;     // the lane's bucket (-1: past the row's end)
  int head;   // lane of the run's first entry
  int len;    // entries in the run (valid on the head lane)
  bool is_head;
};

__device__ __forceinline__ Run bucket_run(int c, bool valid, int lane, int nvalid) {
  Run r;
  r.bk = valid ? (c >> CB_SHIFT) : -1;
  const int prev = __shfl_up(r.bk, 1);
  r.is_head = valid && (lane == 0 || prev != r.bk);
  const uint64_t hm = __ballot(r.is_head);
  const uint64_t incl = lane == 63 ? ~0ull : ((2ull << lane) - 1ull);
  const uint64_t above = hm & ~incl;
  const int next = above ? __ffsll((unsigned long long)above) - 1 : nvalid;
  r.len = next - lane;
  r.head = 63 - __clzll(hm & incl);
  return r;
}

// part[b * G + g] = entries of workgroup g's rows (grid-stride over rows, a wave per row) whose
// column lies in bucket b
__global__ __launch_bounds__(256) void cc_part_count_kernel(const int32_t* __restrict__ rows, int n,
                                                             const int64_t* __restrict__ indptr,
                                                             const int32_t* __restrict__ indices, int B,
                                                             int32_t* __restrict__ part,
                                                             unsigned long long* __restrict__ total) {
  extern __shared__ int h[];
  __shared__ unsigned long long wtot[CP_WAVES];
  for (int i = threadIdx.x; i < B; i += blockDim.x) h[i] = 0;
  __syncthreads();
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  unsigned long long mine = 0;  // this wave's entries (the call's int64 total, below)
  for (int r = blockIdx.x * CP_WAVES + w; r < n; r += gridDim.x * CP_WAVES) {
    const int64_t v = rows[r];
    const int64_t b = indptr[v], e = indptr[v + 1];
    mine += (unsigned long long)(e - b);
    for (int64_t k0 = b; k0 < e; k0 += 64 * CP_U) {  // CP_U pieces' loads in flight at once
      int cu[CP_U];
#pragma unroll
      for (int u = 0; u < CP_U; ++u) {
        const int64_t k = k0 + u * 64 + lane;
        cu[u] = k < e ? indices[k] : 0;
      }
#pragma unroll
      for (int u = 0; u < CP_U; ++u) {
        const int64_t ku = k0 + u * 64;
        if (ku >= e) break;
        const int nvalid = (int)(e - ku < 64 ? e - ku : 64);
        const bool valid = lane < nvalid;
        const Run ru = bucket_run(cu[u], valid, lane, nvalid);
        if (ru.is_head) atomicAdd(&h[ru.bk], ru.len);
      }
    }
  }
  if (lane == 0) wtot[w] = mine;
  __syncthreads();
  for (int i = threadIdx.x; i < B; i += blockDim.x) part[(int64_t)i * gridDim.x + blockIdx.x] = h[i];
  if (threadIdx.x == 0) {
    unsigned long long t = 0;
    for (int j = 0; j < CP_WAVES; ++j) t += wtot[j];
    atomicAdd(total, t);
  }
}

// keys[slot] = column & (2^13 - 1), each entry at a slot of its (bucket, workgroup) range (the
// same rows per workgroup as cc_part_count; a run's head reserves the run's slots); nothing when
// the entries exceed the capacity
__global__ __launch_bounds__(256) void cc_part_scatter_kernel(const int32_t* __restrict__ rows, int n,
                                                               const int64_t* __restrict__ indptr,
                                                               const int32_t* __restrict__ indices, int B,
                                                               const int32_t* __restrict__ off, int64_t cap,
                                                               const unsigned long long* __restrict__ total,
                                                               uint16_t* __restrict__ keys) {
  extern __shared__ int h[];
  if (*total > (unsigned long long)cap) return;
  for (int i = threadIdx.x; i < B; i += blockDim.x) h[i] = off[(int64_t)i * gridDim.x + blockIdx.x];
  __syncthreads();
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  for (int r = blockIdx.x * CP_WAVES + w; r < n; r += gridDim.x * CP_WAVES) {
    const int64_t v = rows[r];
    const int64_t b = indptr[v], e = indptr[v + 1];
    for (int64_t k0 = b; k0 < e; k0 += 64 * CP_U) {
      int cu[CP_U];
#pragma unroll
      for (int u = 0; u < CP_U; ++u) {
        const int64_t k = k0 + u * 64 + lane;
        cu[u] = k < e ? indices[k] : 0;
      }
#pragma unroll
      for (int u = 0; u < CP_U; ++u) {
        const int64_t ku = k0 + u * 64;
        if (ku >= e) break;
        const int nvalid = (int)(e - ku < 64 ? e - ku : 64);
        const bool valid = lane < nvalid;
        const int c = cu[u];
        const Run ru = bucket_run(c, valid, lane, nvalid);
        int base = 0;
        if (ru.is_head) base = atomicAdd(&h[ru.bk], ru.len);
        base = __shfl(base, valid ? ru.head : 0);
        if (valid) keys[base + (lane - ru.head)] = (uint16_t)(c & (CB_COLS - 1));
      }
    }
  }
}

// The (bucket, workgroup) counts' exclusive scan over all CUs: workgroup j scans its 8,192
// counts and leaves their sum in csum[j]; the sums' scan (one workgroup: a few dozen) gives each
// chunk's start, which cc_chunk_add adds (and writes the total at out[n]).
constexpr int CS_ITEMS = 8;
constexpr int CS_CHUNK = 1024 * CS_ITEMS;

__global__ __launch_bounds__(1024) void cc_chunk_scan_kernel(const int32_t* __restrict__ in, int n,
                                                             int32_t* __restrict__ out, int32_t* __restrict__ csum) {
  __shared__ int wsum[16];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int base = blockIdx.x * CS_CHUNK + tid * CS_ITEMS;
  int v[CS_ITEMS];
  int tsum = 0;
#pragma unroll
  for (int k = 0; k < CS_ITEMS; ++k) {
    v[k] = base + k < n ? in[base + k] : 0;
    tsum += v[k];
  }
  int x = tsum;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const int y = __shfl_up(x, d);
    if (lane >= d) x += y;
  }
  if (lane == 63) wsum[wave] = x;
  __syncthreads();
  if (wave == 0) {
    int w = lane < 16 ? wsum[lane] : 0;
#pragma unroll
    for (int d = 1; d < 16; d <<= 1) {
      const int y = __shfl_up(w, d);
      if (lane >= d) w += y;
    }
    if (lane < 16) wsum[lane] = w;
  }
  __syncthreads();
  int excl = (wave ? wsum[wave - 1] : 0) + x - tsum;
#pragma unroll
  for (int k = 0; k < CS_ITEMS; ++k) {
    if (base + k < n) out[base + k] = excl;
    excl += v[k];
  }
  if (tid == 0) csum[blockIdx.x] = wsum[15];
}

__global__ __launch_bounds__(256) void cc_chunk_add_kernel(int32_t* __restrict__ out, int n,
                                                           const int32_t* __restrict__ coff, int nchunks) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i < n) out[i] += coff[i / CS_CHUNK];
  if (i == 0) out[n] = coff[nchunks];
}

// workgroup b: cnt[b * 2^13 + i] += the bucket's entries with offset i (LDS sums, then one
// read-modify-write per non-zero column; the workgroup owns its columns)
__global__ __launch_bounds__(256) void cc_bucket_add_kernel(const uint16_t* __restrict__ keys,
                                                            const int32_t* __restrict__ off, int G, int B,
                                                            int64_t cap, const unsigned long long* __restrict__ total,
                                                            int64_t N, int32_t* __restrict__ cnt) {
  __shared__ int h[CB_COLS];
  if (*total > (unsigned long long)cap) return;
  for (int i = threadIdx.x; i < CB_COLS; i += blockDim.x) h[i] = 0;
  __syncthreads();
  const int64_t beg = off[(int64_t)blockIdx.x * G];
  const int64_t end = off[(int64_t)(blockIdx.x + 1) * G];
  for (int64_t i = beg + threadIdx.x; i < end; i += blockDim.x) atomicAdd(&h[keys[i]], 1);
  __syncthreads();
  const int64_t c0 = (int64_t)blockIdx.x << CB_SHIFT;
  for (int i = threadIdx.x; i < CB_COLS && c0 + i < N; i += blockDim.x)
    if (h[i]) cnt[c0 + i] += h[i];
}

// the atomic histogram for a call whose entries exceed the offsets buffer (returns at once
// otherwise)
__global__ __launch_bounds__(256) void cc_hist_guard_kernel(const int32_t* __restrict__ rows, int n,
                                                            const int64_t* __restrict__ indptr,
                                                            const int32_t* __restrict__ indices,
                                                            const unsigned long long* __restrict__ total,
                                                            int64_t cap, int32_t* __restrict__ cnt) {
  if (*total <= (unsigned long long)cap) return;
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
  int32_t* total_h = nullptr;  // pinned [1]: live columns
  unsigned long long* ent = nullptr;    // device [1]: the call's entries, int64 (partitioned form)
  unsigned long long* ent_h = nullptr;  // pinned [1]: its copy
  int32_t* out_h = nullptr;    // pinned [N]
  bool part = false;           // partitioned histogram (else the atomic one)
  int64_t B = 0;               // buckets of 2^13 columns
  int32_t* pcnt = nullptr;     // device [B * CP_GRID]: entries per (bucket, workgroup)
  int32_t* poff = nullptr;     // device [B * CP_GRID + 1]: their first slots, then the total
  int32_t* csum = nullptr;     // device [chunks + 1] x 2: the chunk sums and their scan
  uint16_t* keys = nullptr;    // device [keys_cap]
  int64_t keys_cap = 0;

  ~ColCount() {
    if (st) (void)hipStreamSynchronize(st);
    for (void* p : {(void*)cnt, (void*)bits, (void*)blk, (void*)blk_off, (void*)out, (void*)rows_d, (void*)pcnt,
                    (void*)poff, (void*)csum, (void*)keys, (void*)ent})
      if (p) (void)hipFree(p);
    for (void* p : {(void*)rows_h, (void*)bits_h, (void*)total_h, (void*)out_h, (void*)ent_h})
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

constexpr int CP_GRID = 2048;  // partition workgroups (the scan covers B * CP_GRID counts)

// the partition kernels' grid for n rows: a row per wave, at most CP_GRID workgroups
int part_grid(int64_t n) {
  const int64_t g = ceil_div(n, (int64_t)CP_WAVES);
  return (int)(g < 1 ? 1 : (g > CP_GRID ? CP_GRID : g));
}

}  // namespace

extern "C" {

int gnn_colcount_set_cus(int32_t cus) {
  GNN_REQUIRE(cus >= 0, "gnn_colcount_set_cus: cus must be >= 0");
  g_cc_cus.store(cus);
  return 0;
}

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
  int cus = g_cc_cus.load();
  if (const char* e = getenv("GNN_CC_CUS")) cus = atoi(e);
  int ncu = 0;
  GNN_HIP(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, device), "hipDeviceGetAttribute");
  if (cus > ncu) cus = ncu;
  if (cus > 0) {
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
  GNN_HIP(hipHostMalloc(&c->total_h, 8, hipHostMallocDefault), "hipHostMalloc");
  GNN_HIP(hipHostMalloc(&c->out_h, (size_t)c->N * 4, hipHostMallocDefault), "hipHostMalloc");
  // GNN_CC_HIST=atomic: the one-atomic-per-entry histogram; GNN_CC_KEYS: the offsets buffer's
  // initial capacity in entries (default 4 M: 8 MB)
  const char* hist = getenv("GNN_CC_HIST");
  c->B = ceil_div(c->N, (int64_t)CB_COLS);
  c->part = !(hist && strcmp(hist, "atomic") == 0) && c->B <= CB_MAX;
  if (c->part) {
    int64_t cap = (int64_t)1 << 22;
    if (const char* e = getenv("GNN_CC_KEYS")) cap = atoll(e);
    c->keys_cap = cap > 0 ? std::min<int64_t>(cap, INT32_MAX) : 1;  // int32 offsets
    GNN_HIP(hipMalloc(&c->ent, 8), "hipMalloc");
    GNN_HIP(hipHostMalloc(&c->ent_h, 8, hipHostMallocDefault), "hipHostMalloc");
    *c->ent_h = 0;
    GNN_HIP(hipMalloc(&c->pcnt, (size_t)(c->B * CP_GRID) * 4), "hipMalloc");
    GNN_HIP(hipMalloc(&c->poff, (size_t)(c->B * CP_GRID + 1) * 4), "hipMalloc");
    GNN_HIP(hipMalloc(&c->csum, (size_t)(ceil_div(c->B * CP_GRID, (int64_t)CS_CHUNK) + 1) * 8), "hipMalloc");
    GNN_HIP(hipMalloc(&c->keys, (size_t)c->keys_cap * 2), "hipMalloc");
  }
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
    if (c->part) {
      const int G = part_grid(n);
      const int B = (int)c->B;
      const size_t lds = (size_t)B * 4;
      GNN_HIP(hipMemsetAsync(c->ent, 0, 8, c->st), "hipMemsetAsync");
      cc_part_count_kernel<<<dim3((unsigned)G), dim3(64 * CP_WAVES), lds, c->st>>>(c->rows_d, (int)n, c->indptr, c->indices, B,
                                                                         c->pcnt, c->ent);
      GNN_LAUNCHED("cc_part_count_kernel");
      const int np = B * G, nch = (int)ceil_div(np, CS_CHUNK);
      int32_t* const coff = c->csum + nch + 1;
      cc_chunk_scan_kernel<<<dim3((unsigned)nch), dim3(1024), 0, c->st>>>(c->pcnt, np, c->poff, c->csum);
      GNN_LAUNCHED("cc_chunk_scan_kernel");
      GNN_TRY_CC(gnn::launch_scan_exclusive(c->csum, nch, coff, c->st));
      cc_chunk_add_kernel<<<dim3((unsigned)ceil_div(np, 256)), dim3(256), 0, c->st>>>(c->poff, np, coff, nch);
      GNN_LAUNCHED("cc_chunk_add_kernel");
      cc_part_scatter_kernel<<<dim3((unsigned)G), dim3(64 * CP_WAVES), lds, c->st>>>(c->rows_d, (int)n, c->indptr, c->indices,
                                                                           B, c->poff, c->keys_cap, c->ent, c->keys);
      GNN_LAUNCHED("cc_part_scatter_kernel");
      cc_bucket_add_kernel<<<dim3((unsigned)B), dim3(256), 0, c->st>>>(c->keys, c->poff, G, B, c->keys_cap, c->ent,
                                                                       c->N, c->cnt);
      GNN_LAUNCHED("cc_bucket_add_kernel");
      cc_hist_guard_kernel<<<dim3((unsigned)std::min<int64_t>(ceil_div(waves, 4), 512)), dim3(256), 0, c->st>>>(
          c->rows_d, (int)n, c->indptr, c->indices, c->ent, c->keys_cap, c->cnt);
      GNN_LAUNCHED("cc_hist_guard_kernel");
      GNN_HIP(hipMemcpyAsync(c->ent_h, c->ent, 8, hipMemcpyDeviceToHost, c->st), "hipMemcpyAsync");
    } else {
      cc_hist_kernel<<<dim3((unsigned)ceil_div(waves, 4)), dim3(256), 0, c->st>>>(c->rows_d, (int)n, c->indptr,
                                                                                  c->indices, c->cnt);
      GNN_LAUNCHED("cc_hist_kernel");
    }
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
  if (c->part && n > 0 && *c->ent_h > (unsigned long long)c->keys_cap && c->keys_cap < INT32_MAX) {
    // this call ran the atomic form: grow (the int32 offsets cap the buffer at INT32_MAX entries;
    // calls beyond that keep the atomic form)
    const unsigned long long want = *c->ent_h + *c->ent_h / 2;
    const int64_t cap = (int64_t)std::min<unsigned long long>(want, (unsigned long long)INT32_MAX);
    GNN_HIP(hipStreamSynchronize(c->st), "hipStreamSynchronize");
    GNN_HIP(hipFree(c->keys), "hipFree");
    c->keys = nullptr;
    c->keys_cap = 0;
    GNN_HIP(hipMalloc(&c->keys, (size_t)cap * 2), "hipMalloc");
    c->keys_cap = cap;
  }
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
