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
// the graph's CSR resident in HBM:
//   1. map[cols[j]] = j                      (node -> column position, -1 elsewhere)
//   2. per row: count of entries whose column is mapped       (wave per row)
//   3. exclusive scan -> rowptr
//   4. per row: the mapped entries, compacted in order (ballot + mbcnt), their value
//      (float)((1.0 / deg(row node)) * (double)normfact[j]) — the create_coo_tensor formula,
//      bit-identical to gnn_build_operand_f32 on the host-extracted pieces
//   5. map reset; then, for the backward's operand Aᵀ (rows ascending — every layer below the
//      top, whose rows are np.unique output), map[rows[i]] = i and a wave per column j walks
//      lapᵀ's row cols[j]: the mapped entries ARE Aᵀ's row j in canonical (ascending) order,
//      written at the host-known offset colptr[j] (colptr[j+1] - colptr[j] = the column count
//      of U the draw already used), values by the same formula.
// No sort, no atomics on the data path; the only atomics raise an error flag on a count that
// disagrees with the host's (then the writes stay clamped inside their segments).
#include <hip/hip_runtime.h>

#include <climits>
#include <cstdint>

#include "common.h"
#include "gnn_extract.h"

namespace {

using gnn::ceil_div;

__device__ __forceinline__ int below_me(unsigned long long mask) {
  return (int)__builtin_amdgcn_mbcnt_hi((unsigned)(mask >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)mask, 0u));
}

__global__ __launch_bounds__(256) void lx_map_kernel(const int* __restrict__ ids, int n, int* __restrict__ map,
                                                     int set) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i < n) map[ids[i]] = set ? i : -1;
}

// Entries per pass: 4 chunks of 64 loaded before any is used (4 independent index -> map
// chains in flight per lane).
constexpr int LX_U = 4;

__global__ __launch_bounds__(256) void lx_count_kernel(const int64_t* __restrict__ indptr,
                                                       const int* __restrict__ indices, const int* __restrict__ rows,
                                                       int M, const int* __restrict__ map, int* __restrict__ cnt) {
  const int lane = threadIdx.x & 63;
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= M) return;
  const int v = rows[r];
  const int64_t b = indptr[v], e = indptr[v + 1];
  int n = 0;
  for (int64_t base = b; base < e; base += 64 * LX_U) {
    int m[LX_U];
#pragma unroll
    for (int t = 0; t < LX_U; ++t) {
      const int64_t k = base + t * 64 + lane;
      m[t] = (k < e) ? indices[k] : -1;
    }
#pragma unroll
    for (int t = 0; t < LX_U; ++t) m[t] = (m[t] >= 0) ? map[m[t]] : -1;
#pragma unroll
    for (int t = 0; t < LX_U; ++t) n += __builtin_popcountll(__ballot(m[t] >= 0));
  }
  if (lane == 0) cnt[r] = n;
}

__global__ __launch_bounds__(256) void lx_write_kernel(const int64_t* __restrict__ indptr,
                                                       const int* __restrict__ indices, const int* __restrict__ rows,
                                                       int M, const int* __restrict__ map,
                                                       const float* __restrict__ normfact,
                                                       const int* __restrict__ rowptr, int nnz, int* __restrict__ col,
                                                       float* __restrict__ val, int* __restrict__ err) {
  const int lane = threadIdx.x & 63;
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= M) return;
  if (r == M - 1 && err && lane == 0 && rowptr[M] != nnz) atomicOr(err, 1);
  const int v = rows[r];
  const int64_t b = indptr[v], e = indptr[v + 1];
  const double inv = 1.0 / (double)(e - b);  // deg_full(row): fullrowptr[r+1] - fullrowptr[r]
  int out = rowptr[r];
  const int lim = min(rowptr[r + 1], nnz);
  for (int64_t base = b; base < e; base += 64 * LX_U) {
    int m[LX_U];
#pragma unroll
    for (int t = 0; t < LX_U; ++t) {
      const int64_t k = base + t * 64 + lane;
      m[t] = (k < e) ? indices[k] : -1;
    }
#pragma unroll
    for (int t = 0; t < LX_U; ++t) m[t] = (m[t] >= 0) ? map[m[t]] : -1;
#pragma unroll
    for (int t = 0; t < LX_U; ++t) {
      const bool keep = m[t] >= 0;
      const unsigned long long mask = __ballot(keep);
      const int pos = out + below_me(mask);
      if (keep && pos < lim) {
        col[pos] = m[t];
        val[pos] = (float)(inv * (double)normfact[m[t]]);
      }
      out += __builtin_popcountll(mask);
    }
  }
}

// Aᵀ row j (= column j of A): the entries of lapᵀ's row cols[j] whose node is one of A's rows
// (map: node -> row position), in node order = row order (rows ascending).
__global__ __launch_bounds__(256) void lx_write_t_kernel(
    const int64_t* __restrict__ indptr, const int64_t* __restrict__ indptr_t, const int* __restrict__ indices_t,
    const int* __restrict__ cols, int K, const int* __restrict__ map, const float* __restrict__ normfact,
    const int* __restrict__ colptr, int nnz, int* __restrict__ rows_t, float* __restrict__ val_t,
    int* __restrict__ err) {
  const int lane = threadIdx.x & 63;
  const int j = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (j >= K) return;
  const int u = cols[j];
  const int64_t b = indptr_t[u], e = indptr_t[u + 1];
  const double nf = (double)normfact[j];
  int out = colptr[j];
  const int end = colptr[j + 1];
  const int lim = min(end, nnz);
  for (int64_t base = b; base < e; base += 64 * LX_U) {
    int node[LX_U], m[LX_U];
#pragma unroll
    for (int t = 0; t < LX_U; ++t) {
      const int64_t k = base + t * 64 + lane;
      node[t] = (k < e) ? indices_t[k] : -1;
    }
#pragma unroll
    for (int t = 0; t < LX_U; ++t) m[t] = (node[t] >= 0) ? map[node[t]] : -1;
#pragma unroll
    for (int t = 0; t < LX_U; ++t) {
      const bool keep = m[t] >= 0;
      const unsigned long long mask = __ballot(keep);
      const int pos = out + below_me(mask);
      if (keep && pos < lim) {
        const double inv = 1.0 / (double)(indptr[node[t] + 1] - indptr[node[t]]);
        rows_t[pos] = m[t];
        val_t[pos] = (float)(inv * nf);
      }
      out += __builtin_popcountll(mask);
    }
  }
  if (err && lane == 0 && out != end) atomicOr(err, 2);
}

}  // namespace

extern "C" {

int gnn_ladies_extract_f32(const int64_t* indptr, const int32_t* indices, int64_t num_nodes, const int64_t* indptr_t,
                           const int32_t* indices_t, const int32_t* rows, int64_t M, const int32_t* cols, int64_t K,
                           const float* normfact, int64_t nnz, const int32_t* colptr_t, int32_t* node_map,
                           int32_t* rowptr, int32_t* col, float* val, int32_t* rowcnt, int32_t* rows_t, float* val_t,
                           int32_t* err_flag, void* stream) {
  GNN_REQUIRE(M >= 0 && K >= 0 && nnz >= 0 && num_nodes >= 0, "gnn_ladies_extract_f32: negative size");
  GNN_REQUIRE(M < INT_MAX && K < INT_MAX && nnz < INT_MAX && num_nodes < INT_MAX,
              "gnn_ladies_extract_f32: sizes must be < 2^31");
  GNN_REQUIRE(rowptr != nullptr, "gnn_ladies_extract_f32: rowptr is NULL");
  GNN_REQUIRE(M == 0 || (indptr && indices && rows && node_map && rowcnt),
              "gnn_ladies_extract_f32: NULL graph / rows / node_map / rowcnt");
  GNN_REQUIRE(K == 0 || (cols && normfact), "gnn_ladies_extract_f32: NULL cols / normfact");
  GNN_REQUIRE(nnz == 0 || (col && val), "gnn_ladies_extract_f32: NULL col / val");
  const bool tr = colptr_t != nullptr;
  GNN_REQUIRE(!tr || (indptr_t && indices_t && (nnz == 0 || (rows_t && val_t))),
              "gnn_ladies_extract_f32: transpose requested with NULL lap^T / rows_t / val_t");
  hipStream_t st = (hipStream_t)stream;
  const unsigned gm = (unsigned)ceil_div(M > 0 ? M : 1, 4);
  if (K > 0) {
    lx_map_kernel<<<dim3((unsigned)ceil_div(K, 256)), dim3(256), 0, st>>>(cols, (int)K, node_map, 1);
    GNN_LAUNCHED("lx_map_kernel");
  }
  if (M > 0) {
    lx_count_kernel<<<dim3(gm), dim3(256), 0, st>>>(indptr, indices, rows, (int)M, node_map, rowcnt);
    GNN_LAUNCHED("lx_count_kernel");
  }
  if (int rc = gnn::launch_scan_exclusive(rowcnt, (int)M, rowptr, st)) return rc;
  if (M > 0) {
    lx_write_kernel<<<dim3(gm), dim3(256), 0, st>>>(indptr, indices, rows, (int)M, node_map, normfact, rowptr,
                                                     (int)nnz, col, val, err_flag);
    GNN_LAUNCHED("lx_write_kernel");
  }
  if (K > 0) {
    lx_map_kernel<<<dim3((unsigned)ceil_div(K, 256)), dim3(256), 0, st>>>(cols, (int)K, node_map, 0);
    GNN_LAUNCHED("lx_map_kernel");
  }
  if (tr && K > 0) {
    if (M > 0) {
      lx_map_kernel<<<dim3((unsigned)ceil_div(M, 256)), dim3(256), 0, st>>>(rows, (int)M, node_map, 1);
      GNN_LAUNCHED("lx_map_kernel");
    }
    lx_write_t_kernel<<<dim3((unsigned)ceil_div(K, 4)), dim3(256), 0, st>>>(
        indptr, indptr_t, indices_t, cols, (int)K, node_map, normfact, colptr_t, (int)nnz, rows_t, val_t, err_flag);
    GNN_LAUNCHED("lx_write_t_kernel");
    if (M > 0) {
      lx_map_kernel<<<dim3((unsigned)ceil_div(M, 256)), dim3(256), 0, st>>>(rows, (int)M, node_map, 0);
      GNN_LAUNCHED("lx_map_kernel");
    }
  }
  return 0;
}

}  // extern "C"
