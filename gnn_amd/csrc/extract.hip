// extract.hip — the LADIES layer extraction adj = lap[rows, :][:, cols] on the GPU, fused with
// create_coo_tensor's values (include/gnn_extract.h).
//
// Reference (sampler.py:113-139): per sampled layer the host slices U = lap_matrix[previous, :]
// (scipy row indexing), draws the next layer's nodes, slices adj = U[:, after_nodes] (scipy
// column indexing), ships rowptr / int16 colidx / normfact to the GPU, and create_coo_tensor
// (cuda_spmm.cu:787-827) computes val = (1/deg_full(row)) * normfact[col] there.
//
// Here the host keeps only the draw (it needs the column counts of U, which it has without
// materialising U) and everything that touches the sub-graph's entries runs on the GPU, reading
// the graph's CSR resident in HBM. Both outputs are "filtered gathers" of graph rows:
//   forward   A:  segment i = lap row rows[i],   keep node c if c is in cols (position j) -> col j
//   transpose Aᵀ: segment j = lapᵀ row cols[j],  keep node r if r is in rows (position i) -> row i
// with value (float)((1.0 / deg(row node)) * (double)normfact[j]) either way (bit-identical to
// gnn_build_operand_f32 / gnn_build_operand_t_f32 on host-extracted pieces). The segment offsets
// (S = U's row pointer; the offsets of lapᵀ's rows of cols) come from the host, which has them
// from the draw.
//  * Balance: graph rows follow a power law and LADIES draws the high-degree nodes, so a wave per
//    row leaves a long tail (one 20 k-entry row = 80 dependent rounds on one wave: 195 us for the
//    Reddit layer 0). The concatenated segments are cut into XW equal contiguous entry ranges,
//    one per wave; a wave holds its range's segment table in registers (lane q: segment sb + q's
//    offsets and graph position), so a round of 64 * XU consecutive entries — across segment
//    boundaries — issues all its index loads at once, then all its membership lookups.
//  * Latency: the walks are chains of dependent loads, so everything a wave would otherwise
//    search for (its first / last segment, each segment's graph position) is made once by a prep
//    kernel; per wave: one load for its segment range, one round trip for the segment table, then
//    two per round (indices, membership).
//  * Membership: a bitmap of the sorted id set with a rank per 64-bit word (12 bytes per 64
//    nodes; built from the sorted list without atomics: rank[w] = lower_bound(ids, 64 w)).
// Measured (Reddit LADIES layer 0, 5.7 M graph entries, MI355X): wave per row 195 us; entry
// ranges with per-lane segment search 161; staging the table in LDS cost more (the copy) than
// the lookups it saved; an int node -> position map instead of the bitmap: same time.
// Launches: 1. prep  2. count (per wave kept entries; per (row, 64-entry group) one integer
// atomicAdd — deterministic)  3. scan (wave offsets per direction, rowptr)  4. write (compacted in
// order by ballot + mbcnt at wave offset + rank: CSR order for A, canonical order for Aᵀ —
// segments ascending, graph rows ascending, rows sorted).
// Every size the host needs (nnz, grid) is known before launch; no state survives a call.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>
#include <cstdint>
#include <cstdlib>

#include "common.h"
#include "gnn_extract.h"

namespace {

using gnn::ceil_div;

constexpr int XW_MAX = 16384;   // waves per direction (contiguous entry ranges): the default
constexpr int XW_DEFAULT = 8192;
constexpr int XU = 8;           // entries per lane per round (512 per wave round)
constexpr int SCAN_ITEMS = 16;  // scan: items per thread per pass (1024 threads)

__device__ __forceinline__ int below_me(unsigned long long mask) {
  return (int)__builtin_amdgcn_mbcnt_hi((unsigned)(mask >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)mask, 0u));
}

__device__ __forceinline__ int rl(int x, int l) { return __builtin_amdgcn_readlane(x, l); }

// One direction of the extraction (device pointers).
struct Side {
  const int64_t* ptr;          // graph indptr (lap or lapᵀ)
  const int* idx;              // graph indices
  const int* src;              // segment source nodes [R]
  const int* S;                // [R+1] segment offsets (host)
  const int* ids;              // the sorted output index set (cols for A, rows for Aᵀ)
  unsigned long long* bits;    // [words] membership bitmap of ids
  int* rank;                   // [words] ids below each 64-bit word
  int64_t* segbase;            // [R] ptr[src[i]]: graph position of segment i (prep kernel)
  int2* wseg;                  // [XW] first / last segment of each wave's entry range (prep kernel)
  int* segcnt;                 // A: [R] kept entries per row (-> rowptr); Aᵀ: unused
  int* wavecnt;                // [XW]
  int* waveoff;                // [XW+1]
  int* out_idx;                // col (A) / rows_t (Aᵀ)
  float* out_val;
  int R;                       // segments
  int nids;
  int words;                   // ceil(N / 64)
  int transpose;               // 0: A (segment = row i), 1: Aᵀ (segment = column j)
  int nnz;                     // host-known entry count
};

struct Sides {
  Side s[2];
  int n;      // 1 or 2
  int xw;     // waves per direction
  int flags;  // experiments: 1 = skip the membership lookups (traversal cost alone)
};

// Everything the walks look up per wave or per segment, made once per call, one thread per item:
//   [0, n * words)        membership bitmap + word ranks of the sorted id lists: rank[w] = #ids
//                         below 64 w (a lower bound), bits[w] = the ids in [64 w, 64 w + 64)
//   next M                segcnt = 0
//   next R0 (+ R1)        segbase[i] = ptr[src[i]]
//   next n * XW           wseg[w] = (first segment with an entry >= a_w, last with one < b_w)
__global__ __launch_bounds__(256) void lx_prep_kernel(Sides sd, int* __restrict__ segcnt, int M) {
  int i = blockIdx.x * 256 + threadIdx.x;
  const int words = sd.s[0].words;
  if (i < words * sd.n) {
    const int side = i / words;
    const int w = i - side * words;
    const Side& s = sd.s[side];
    const int lo64 = w * 64;
    int lo = 0, hi = s.nids;  // first id >= 64 w
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (s.ids[mid] < lo64) lo = mid + 1;
      else hi = mid;
    }
    unsigned long long b = 0ull;
    for (int k = lo; k < s.nids && s.ids[k] < lo64 + 64; ++k) b |= 1ull << (s.ids[k] - lo64);
    s.bits[w] = b;
    s.rank[w] = lo;
    return;
  }
  i -= words * sd.n;
  if (i < M) {
    segcnt[i] = 0;
    return;
  }
  i -= M;
  for (int k = 0; k < sd.n; ++k) {
    const Side& s = sd.s[k];
    if (i < s.R) {
      s.segbase[i] = s.ptr[s.src[i]];
      return;
    }
    i -= s.R;
  }
  const int XW = sd.xw;
  if (i >= XW * sd.n) return;
  const int side = i / XW;
  const int w = i - side * XW;
  const Side& s = sd.s[side];
  const int T = s.S[s.R];
  const int a = (int)((int64_t)T * w / XW);
  const int b = (int)((int64_t)T * (w + 1) / XW);
  int2 r = make_int2(0, -1);
  if (a < b) {
    // first q with S[q+1] > a, then first q with S[q+1] >= b
    int lo = 0, hi = s.R;
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (s.S[mid + 1] > a) hi = mid;
      else lo = mid + 1;
    }
    r.x = lo;
    hi = s.R;
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (s.S[mid + 1] >= b) hi = mid;
      else lo = mid + 1;
    }
    r.y = lo;
  }
  s.wseg[w] = r;
}

// Exclusive scan of int32 arrays, one workgroup per array.
__device__ void scan_block(const int* __restrict__ in, int n, int* __restrict__ out, int* wsum) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  int carry = 0;
  for (int base = 0; base < n; base += 1024 * SCAN_ITEMS) {
    int v[SCAN_ITEMS];
    int tsum = 0;
#pragma unroll
    for (int k = 0; k < SCAN_ITEMS; ++k) {
      const int idx = base + tid * SCAN_ITEMS + k;
      v[k] = (idx < n) ? in[idx] : 0;
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
      int w = (lane < 16) ? wsum[lane] : 0;
#pragma unroll
      for (int d = 1; d < 16; d <<= 1) {
        const int y = __shfl_up(w, d);
        if (lane >= d) w += y;
      }
      if (lane < 16) wsum[lane] = w;
    }
    __syncthreads();
    int excl = carry + (wave ? wsum[wave - 1] : 0) + x - tsum;
#pragma unroll
    for (int k = 0; k < SCAN_ITEMS; ++k) {
      const int idx = base + tid * SCAN_ITEMS + k;
      if (idx < n) out[idx] = excl;
      excl += v[k];
    }
    carry += wsum[15];
    __syncthreads();
  }
  if (tid == 0) out[n] = carry;
}

struct ScanJobs {
  const int* in[3];
  int* out[3];
  int n[3];
  int count;
};

__global__ __launch_bounds__(1024) void lx_scan_kernel(ScanJobs j) {
  __shared__ int wsum[16];
  const int b = blockIdx.x;
  if (b < j.count) scan_block(j.in[b], j.n[b], j.out[b], wsum);
}

// Position of node c in the sorted id set, -1 if absent (bits and rank loaded together: no
// dependent second load).
__device__ __forceinline__ int lookup(const unsigned long long* bits, const int* rank, int c) {
  const unsigned long long b = bits[c >> 6];
  const int r = rank[c >> 6];
  const unsigned sh = (unsigned)c & 63u;
  return ((b >> sh) & 1ull) ? r + __builtin_popcountll(b & ((1ull << sh) - 1ull)) : -1;
}

// Walks the kept entries of wave w's entry range. WRITE = false: counts (returns the total,
// adds per-row counts into segcnt); WRITE = true: writes them from position `out`.
template <bool WRITE>
__device__ __forceinline__ int walk(const Side& s, const unsigned long long* bits, const int* rank, int w, int lane,
                                    const int64_t* __restrict__ deg_ptr, const float* __restrict__ normfact,
                                    int out, int XW, int flags) {
  const int2 ws = s.wseg[w];
  const int s0 = ws.x, s1 = ws.y;
  if (s0 > s1) return 0;
  const int T = s.S[s.R];
  const int a = (int)((int64_t)T * w / XW);
  const int b = (int)((int64_t)T * (w + 1) / XW);
  const int out0 = out;
  const int lim = s.nnz;
  for (int sb = s0; sb <= s1; sb += 64) {
    // the segment table of up to 64 segments: offsets, graph positions, (Aᵀ) normfact
    const int sj = sb + lane;
    int Sj = INT_MAX, Sj1 = INT_MAX;
    int64_t gj = 0;
    float nfj = 0.0f;
    if (sj <= s1) {
      Sj = s.S[sj];
      Sj1 = s.S[sj + 1];
      gj = s.segbase[sj];
      if (WRITE && s.transpose) nfj = normfact[sj];
    }
    const int nseg = min(64, s1 - sb + 1);
    const int ta = max(a, rl(Sj, 0));
    const int tb = min(b, rl(Sj1, nseg - 1));
    for (int off = ta; off < tb; off += 64 * XU) {
      int node[XU], m[XU], sq[XU];
#pragma unroll
      for (int t = 0; t < XU; ++t) {
        const int k = off + t * 64 + lane;
        int q = 0;  // the table segment holding entry k (empty segments are skipped past)
        for (int u = 1; u < nseg; ++u) q += (k >= rl(Sj, u)) ? 1 : 0;
        sq[t] = q;
        const int segS = __shfl(Sj, q);
        const int64_t g = ((int64_t)__shfl((int)(gj >> 32), q) << 32) | (uint32_t)__shfl((int)(uint32_t)gj, q);
        node[t] = (k < tb) ? s.idx[g + (k - segS)] : -1;
      }
#pragma unroll
      for (int t = 0; t < XU; ++t)
        m[t] = node[t] >= 0 ? ((flags & 1) ? ((node[t] & 3) ? -1 : node[t]) : lookup(bits, rank, node[t])) : -1;
#pragma unroll
      for (int t = 0; t < XU; ++t) {
        const bool keep = m[t] >= 0;
        const unsigned long long km = __ballot(keep);
        if (WRITE) {
          const int pos = out + below_me(km);
          const int segS = __shfl(Sj, sq[t]);
          const int segE = __shfl(Sj1, sq[t]);
          const float nfs = __shfl(nfj, sq[t]);
          if (keep && pos < lim) {
            double inv;
            float nf;
            if (s.transpose) {  // segment = column j, kept node = A's row node
              inv = 1.0 / (double)(deg_ptr[node[t] + 1] - deg_ptr[node[t]]);
              nf = nfs;
            } else {            // segment = row i: its length is the row's full degree
              inv = 1.0 / (double)(segE - segS);
              nf = normfact[m[t]];
            }
            s.out_idx[pos] = m[t];
            s.out_val[pos] = (float)(inv * (double)nf);
          }
        } else if (s.segcnt && km) {
          // one integer atomicAdd per (segment, 64-entry group): the lanes of a segment are contiguous
          unsigned long long live = __ballot(node[t] >= 0);
          while (live) {
            const int leader = __builtin_ctzll(live);
            const int qq = __builtin_amdgcn_readlane(sq[t], leader);
            const unsigned long long same = __ballot(sq[t] == qq) & live;
            const int c = __builtin_popcountll(same & km);
            if (c && lane == leader) atomicAdd(&s.segcnt[sb + qq], c);
            live &= ~same;
          }
        }
        out += __builtin_popcountll(km);
      }
    }
  }
  return out - out0;
}

__global__ __launch_bounds__(256) void lx_count_kernel(Sides sd) {
  const int lane = threadIdx.x & 63;
  const int gw = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int XW = sd.xw;
  const int side = gw / XW;  // workgroup-uniform (XW % 4 == 0)
  if (side >= sd.n) return;
  const Side& s = sd.s[side];
  const int w = gw - side * XW;
  const int total = walk<false>(s, s.bits, s.rank, w, lane, nullptr, nullptr, 0, XW, sd.flags);
  if (lane == 0) s.wavecnt[w] = total;
}

__global__ __launch_bounds__(256) void lx_write_kernel(Sides sd, const int64_t* __restrict__ deg_ptr,
                                                       const float* __restrict__ normfact, int* __restrict__ err) {
  const int lane = threadIdx.x & 63;
  const int gw = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int XW = sd.xw;
  const int side = gw / XW;
  if (side >= sd.n) return;
  const Side& s = sd.s[side];
  const int w = gw - side * XW;
  if (w == 0 && lane == 0 && err && s.waveoff[XW] != s.nnz) atomicOr(err, 1 << side);
  walk<true>(s, s.bits, s.rank, w, lane, deg_ptr, normfact, s.waveoff[w], XW, sd.flags);
}

int64_t table_words(int64_t num_nodes) { return (num_nodes + 63) / 64; }

}  // namespace

extern "C" {

size_t gnn_ladies_extract_workspace_bytes(int64_t num_nodes, int64_t M, int64_t K, int32_t transpose) {
  const int64_t words = table_words(num_nodes > 0 ? num_nodes : 1);
  const size_t table = gnn::align_up((size_t)words * 8, 256) + gnn::align_up((size_t)words * 4, 256);
  const size_t waves = gnn::align_up((size_t)XW_MAX * 4, 256) + gnn::align_up((size_t)(XW_MAX + 1) * 4, 256) +
                       gnn::align_up((size_t)XW_MAX * 8, 256);
  const size_t segs = gnn::align_up((size_t)(M > 0 ? M : 1) * 8, 256) +
                      (transpose ? gnn::align_up((size_t)(K > 0 ? K : 1) * 8, 256) : 0);
  return (waves + table) * (transpose ? 2 : 1) + segs + gnn::align_up((size_t)(M > 0 ? M : 1) * 4, 256);
}

int gnn_ladies_extract_f32(const int64_t* indptr, const int32_t* indices, int64_t num_nodes, const int64_t* indptr_t,
                           const int32_t* indices_t, const int32_t* rows, int64_t M, const int32_t* cols, int64_t K,
                           const float* normfact, int64_t nnz, const int32_t* rowseg, const int32_t* colseg,
                           const int32_t* colptr_t, int32_t* rowptr, int32_t* col, float* val, int32_t* rows_t,
                           float* val_t, void* workspace, size_t workspace_bytes, int32_t* err_flag, void* stream) {
  GNN_REQUIRE(M >= 0 && K >= 0 && nnz >= 0 && num_nodes > 0, "gnn_ladies_extract_f32: negative size / empty graph");
  GNN_REQUIRE(M < INT_MAX && K < INT_MAX && nnz < INT_MAX && num_nodes < INT_MAX - 64,
              "gnn_ladies_extract_f32: sizes must be < 2^31");
  GNN_REQUIRE(rowptr && rowseg, "gnn_ladies_extract_f32: NULL rowptr / rowseg");
  GNN_REQUIRE(M == 0 || (indptr && indices && rows), "gnn_ladies_extract_f32: NULL graph / rows");
  GNN_REQUIRE(K == 0 || (cols && normfact), "gnn_ladies_extract_f32: NULL cols / normfact");
  GNN_REQUIRE(nnz == 0 || (col && val), "gnn_ladies_extract_f32: NULL col / val");
  const bool tr = colptr_t != nullptr;
  GNN_REQUIRE(!tr || (colseg && indptr_t && indices_t && (nnz == 0 || (rows_t && val_t))),
              "gnn_ladies_extract_f32: transpose requested with NULL colseg / lap^T / rows_t / val_t");
  const size_t need = gnn_ladies_extract_workspace_bytes(num_nodes, M, K, tr);
  GNN_REQUIRE(workspace && workspace_bytes >= need, "gnn_ladies_extract_f32: workspace too small (%zu < %zu)",
              workspace_bytes, need);
  hipStream_t st = (hipStream_t)stream;
  const int64_t words = table_words(num_nodes);
  char* w = (char*)workspace;
  auto take = [&](size_t bytes) {
    char* p = w;
    w += gnn::align_up(bytes, 256);
    return p;
  };
  int* segcnt = (int*)take((size_t)(M > 0 ? M : 1) * 4);
  Sides sd{};
  sd.n = tr ? 2 : 1;
  for (int k = 0; k < sd.n; ++k) {
    Side& s = sd.s[k];
    s.ptr = k == 0 ? indptr : indptr_t;
    s.idx = k == 0 ? indices : indices_t;
    s.src = k == 0 ? rows : cols;
    s.S = k == 0 ? rowseg : colseg;
    s.ids = k == 0 ? cols : rows;  // A keeps the nodes of cols, Aᵀ those of rows
    s.R = (int)(k == 0 ? M : K);
    s.nids = (int)(k == 0 ? K : M);
    s.wavecnt = (int*)take((size_t)XW_MAX * 4);
    s.waveoff = (int*)take((size_t)(XW_MAX + 1) * 4);
    s.wseg = (int2*)take((size_t)XW_MAX * 8);
    s.segbase = (int64_t*)take((size_t)(s.R > 0 ? s.R : 1) * 8);
    s.bits = (unsigned long long*)take((size_t)words * 8);
    s.rank = (int*)take((size_t)words * 4);
    s.segcnt = k == 0 ? segcnt : nullptr;
    s.out_idx = k == 0 ? col : rows_t;
    s.out_val = k == 0 ? val : val_t;
    s.R = (int)(k == 0 ? M : K);
    s.words = (int)words;
    s.transpose = k;
    s.nnz = (int)nnz;
  }
  // experiment knobs (benchmarks only): GNN_LX_XW waves per direction, GNN_LX_FLAGS (Sides::flags)
  sd.xw = XW_DEFAULT;
  if (const char* e = getenv("GNN_LX_XW")) sd.xw = std::min(XW_MAX, std::max(4, atoi(e) / 4 * 4));
  if (const char* e = getenv("GNN_LX_FLAGS")) sd.flags = atoi(e);
  const int XW = sd.xw;
  const int64_t nprep = words * sd.n + M + M + (tr ? K : 0) + (int64_t)XW * sd.n;
  lx_prep_kernel<<<dim3((unsigned)ceil_div(nprep, 256)), dim3(256), 0, st>>>(sd, segcnt, (int)M);
  GNN_LAUNCHED("lx_prep_kernel");
  lx_count_kernel<<<dim3((unsigned)(XW / 4 * sd.n)), dim3(256), 0, st>>>(sd);
  GNN_LAUNCHED("lx_count_kernel");
  ScanJobs sc{};
  sc.count = 1 + sd.n;
  sc.in[0] = segcnt;
  sc.out[0] = rowptr;
  sc.n[0] = (int)M;
  for (int k = 0; k < sd.n; ++k) {
    sc.in[1 + k] = sd.s[k].wavecnt;
    sc.out[1 + k] = sd.s[k].waveoff;
    sc.n[1 + k] = XW;
  }
  lx_scan_kernel<<<dim3((unsigned)sc.count), dim3(1024), 0, st>>>(sc);
  GNN_LAUNCHED("lx_scan_kernel");
  lx_write_kernel<<<dim3((unsigned)(XW / 4 * sd.n)), dim3(256), 0, st>>>(sd, indptr, normfact, err_flag);
  GNN_LAUNCHED("lx_write_kernel");
  return 0;
}

}  // extern "C"
