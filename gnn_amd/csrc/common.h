// common.h — shared host helpers of libgnn_spmm.so (error reporting, sizes).
#pragma once

#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

#define GNN_EINVAL (-22)

namespace gnn {

// Records the message for gnn_last_error() (thread-local) and returns `code`.
int fail(int code, const char* fmt, ...);

inline size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }
inline int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }

// out[0..n] = exclusive prefix of in[0..n) (out[n] = total), one workgroup (spmm.hip).
int launch_scan_exclusive(const int* in, int n, int* out, hipStream_t st);

// Whether gnn_spmm_csr_f32(_ex) runs this call shape as spmm_row_kernel with one wave per row
// (every output a C fmaf chain over the row in CSR order): the executor then may fold the call
// into its consumer (gnn_sage_norm_bwd_agg_f32) with bit-identical values.
bool spmm_row_chain(int64_t M, int64_t K, int64_t nnz, int64_t F, int64_t ldx, int64_t ldy, const void* X,
                    const void* Y);

// gnn_gemm_f32_split3 with the split-k and tail-tile choices made for a batch of split_nbatch
// products (gemm.hip): product batch_index of that batch launched on its own (nbatch = 1),
// bit-identical to its result in the batched launch.
int gemm_split3_as_batch(int a_kmajor, int b_kmajor, int64_t M, int64_t N, int64_t K, int nbatch, int split_nbatch,
                         int batch_index, const float* const* A, int64_t lda, const float* const* B, int64_t ldb,
                         float* const* C, int64_t ldc, void* workspace, size_t workspace_bytes, void* stream);

// gnn_gemm_f32_split3 with row-indexed operands: A's row m is A[ia[b][m]] (m-major A, a_rows
// source rows), B's row k is B[ib[b][k]] (k-major B, b_rows source rows); NULL arrays / entries:
// not indexed. Same sums as the split3 product of the gathered operands (gemm.hip).
int gemm_split3_indexed(int a_kmajor, int b_kmajor, int64_t M, int64_t N, int64_t K, int nbatch,
                        const float* const* A, int64_t lda, const int64_t* const* ia, int64_t a_rows,
                        const float* const* B, int64_t ldb, const int64_t* const* ib, int64_t b_rows,
                        float* const* C, int64_t ldc, void* workspace, size_t workspace_bytes, void* stream);

}  // namespace gnn

#define GNN_REQUIRE(cond, ...)                              \
  do {                                                      \
    if (!(cond)) return ::gnn::fail(GNN_EINVAL, __VA_ARGS__); \
  } while (0)

#define GNN_LAUNCHED(name)                                                                       \
  do {                                                                                           \
    hipError_t e_ = hipGetLastError();                                                           \
    if (e_ != hipSuccess) return ::gnn::fail((int)e_, "%s launch: %s", name, hipGetErrorString(e_)); \
  } while (0)

// A failed runtime call is reported by status code and also cleared from HIP's per-thread
// last-error slot: the caller gets the RuntimeError once, and later unrelated calls (torch's
// own error checks) do not pick up the stale error.
#define GNN_HIP(call, name)                                                                \
  do {                                                                                     \
    hipError_t e_ = (call);                                                                \
    if (e_ != hipSuccess) {                                                                \
      (void)hipGetLastError();                                                             \
      return ::gnn::fail((int)e_, "%s: %s", name, hipGetErrorString(e_));                  \
    }                                                                                      \
  } while (0)
