/*
 * gnn_spmm.h — C ABI of the MI355X-native SpMM-aggregation path (libgnn_spmm.so).
 *
 * This is the drop-in boundary for the reference's CUDA extension `spmm`
 * (reference: spmm_cpp/spmm.cpp:52-56, bound in custom_sparse_ops.py:8). Every entry
 * point takes plain device pointers, sizes and a hipStream_t (passed as void*), launches
 * stream-ordered work only (no host synchronisation, no allocation, graph-capturable),
 * and returns 0 on success or a non-zero status whose text is gnn_last_error().
 *
 * Status codes: 0 = ok; GNN_EINVAL (-22) = bad argument (shape, alignment, workspace);
 * any positive value = the hipError_t of a failed launch.
 *
 * Index types: CSR row pointers and column indices are int32 (the reference narrows its
 * int64 COO indices to int32 too: cuda_spmm.cu:620-621), so M, K and nnz must be < 2^31.
 */
#ifndef GNN_SPMM_H
#define GNN_SPMM_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GNN_EINVAL (-22)

/* Text of the last error raised on the calling thread ("" if none). */
const char* gnn_last_error(void);

/* Library version string (build id). */
const char* gnn_version(void);

/* ---------------------------------------------------------------------------------
 * SpMM forward / backward:  Y[M, F] = A[M, K] · X[K, F]   (fp32, CSR operand)
 *
 * Replaces: spmm_load_balance(sparseMat, denseMat)   spmm_cpp/spmm.cpp:23-27
 *           -> spmm_cuda_v2                           spmm_cpp/cuda_spmm.cu:619-704
 *           and spmm_naive (spmm.cpp:38-42, same math, no load balance).
 * The reference's backward is the same call on A^T (custom_sparse_ops.py:33-37); here the
 * caller passes the CSR of A^T produced by gnn_csr_transpose.
 *
 * X rows are read with stride ldx (elements), Y rows written with stride ldy; F <= ldx,
 * F <= ldy. Every one of the M rows of Y (columns [0, F)) is written (empty rows get 0),
 * so Y needs no zero-fill. Work is cut into units of `unit_nnz` consecutive nonzeros; a row
 * of at most unit_nnz entries is summed whole, in CSR order, by the unit holding its first
 * entry (bit for bit a C fmaf chain); longer rows are summed per unit and their pieces added
 * in unit order by a second kernel — deterministic (bitwise reproducible run to run).
 *
 * `workspace` must hold gnn_spmm_workspace_bytes(M, nnz, F, unit_nnz) bytes (device
 * memory); unit_nnz <= 0 selects gnn_spmm_default_unit_nnz(M, nnz, F).
 * ------------------------------------------------------------------------------- */
int64_t gnn_spmm_default_unit_nnz(int64_t M, int64_t nnz, int64_t F);
size_t gnn_spmm_workspace_bytes(int64_t M, int64_t nnz, int64_t F, int64_t unit_nnz);
int gnn_spmm_csr_f32(const int32_t* rowptr, const int32_t* col, const float* val,
                     int64_t M, int64_t K, int64_t nnz,
                     const float* X, int64_t ldx,
                     float* Y, int64_t ldy, int64_t F,
                     void* workspace, size_t workspace_bytes, int64_t unit_nnz,
                     void* stream);

/* Same, plus a row-mapped residual fused into the stores:
 *     Y[r, :] = (A · X)[r, :] + (rmap[r] >= 0 ? R[rmap[r], :] : 0)
 * rmap (int32, M entries, device) may be NULL (then R is ignored). This is the backward of
 * GraphSageConvolution's two inputs (models.py:18-21): d(x) = A^T · d(A·x) + scatter of
 * d(x[sampled]) — the scatter is the residual with rmap = inverse of the sampled-row map.
 * R rows are read with stride ldr (F <= ldr) and must be aligned like Y. */
int gnn_spmm_csr_f32_ex(const int32_t* rowptr, const int32_t* col, const float* val,
                        int64_t M, int64_t K, int64_t nnz,
                        const float* X, int64_t ldx,
                        float* Y, int64_t ldy, int64_t F,
                        const float* R, int64_t ldr, const int32_t* rmap,
                        void* workspace, size_t workspace_bytes, int64_t unit_nnz,
                        void* stream);

/* Describe the kernel configuration gnn_spmm_csr_f32 would pick (vector width, lanes per
 * column group, column chunks per lane, column tiles, units). For diagnostics/benchmarks. */
int gnn_spmm_config(int64_t M, int64_t K, int64_t nnz, int64_t F, int64_t ldx, int64_t ldy,
                    const void* X, const void* Y, int64_t unit_nnz, int32_t out[6]);

/* The name of the main aggregation kernel gnn_spmm_csr_f32(_ex) would launch for this call, as
 * rocprofv3 lists it: "spmm_unit_kernel<VW, G, NJ, U, RES>" (nnz work units + the combine of
 * cut rows) or, for small operands (up to 64 k nonzeros, unit_nnz == 0: the layer-2 calls),
 * "spmm_row_kernel<VW, NJ, U, WPR, RES>" (a workgroup of WPR waves per (row, column slice), no
 * combine launch). residual != 0 names the row-mapped residual variant. */
int gnn_spmm_kernel_name(int64_t M, int64_t K, int64_t nnz, int64_t F, int64_t ldx, int64_t ldy,
                         const void* X, const void* Y, int64_t unit_nnz, int residual, char* out,
                         size_t out_bytes);

/* Optional timing hook: when set, the NEXT gnn_spmm_csr_f32 call on this thread launches its
 * main aggregation kernel with `start` / `stop` as the dispatch's own start and end timestamps
 * (hipExtLaunchKernel: hipEventElapsedTime(start, stop) = the kernel's duration, as rocprofv3
 * reports it), then clears the hook. Events are hipEvent_t (created with timing) as void*. */
void gnn_spmm_set_timing_events(void* start, void* stop);

/* ---------------------------------------------------------------------------------
 * Sampled-adjacency operand builder.
 *
 * Replaces: create_coo_tensor(fullrowptr, rowptr, colidx, normfact, nrows, ncols)
 *           spmm_cpp/spmm.cpp:44-50 -> to_coo_tensor / _create_coo_tensor_kernel
 *           spmm_cpp/cuda_spmm.cu:787-827 (called from sampler.py:135-139).
 * For row r and each entry i in [rowptr[r], rowptr[r+1]):
 *     val[i] = (float)((1.0 / (double)(fullrowptr[r+1] - fullrowptr[r])) * (double)normfact[col[i]])
 * (double arithmetic, single rounding to fp32, as cuda_spmm.cu:800).
 * colidx may be int16 (colidx_bytes = 2, sign-extended like the reference's int16
 * accessor), int32 (4) or int64 (8). Rows whose columns are not ascending are sorted
 * (key = column, payload = value), which is what the reference's .coalesce() does
 * (cuda_spmm.cu:825). A repeated column within a row (never made by scipy slicing or the
 * reference's samplers) is NOT merged here — merging changes nnz, which the host would have to
 * read back — but flagged: the workspace's second int64 word is nonzero after the call iff a row
 * repeats a column (checked after sorting), so a caller can coalesce lazily at a point that
 * synchronises anyway (gnn_amd.custom_sparse_ops: the first aggregation on the tensor).
 * Outputs: csr_col (int32, nnz), csr_val (fp32, nnz) and, if coo_indices != NULL, the
 * coalesced COO indices int64[2][nnz] (row-major: all rows then all columns).
 * `workspace` (device, 8-byte aligned, >= gnn_build_operand_workspace_bytes()) holds the
 * call's "unsorted row seen" and "repeated column seen" words, zeroed on `stream` by the call itself: the library keeps
 * no device state and allocates nothing, so the call is graph-capturable and concurrent
 * calls on different streams need different workspaces.
 * ------------------------------------------------------------------------------- */
size_t gnn_segsort_workspace_bytes(int64_t nseg);
size_t gnn_build_operand_workspace_bytes(void);
int gnn_build_operand_f32(const int32_t* fullrowptr, const int32_t* rowptr,
                          const void* colidx, int colidx_bytes,
                          const float* normfact, int64_t nrows, int64_t ncols, int64_t nnz,
                          int32_t* csr_col, float* csr_val, int64_t* coo_indices,
                          void* workspace, size_t workspace_bytes, void* stream);

/* Same, for rows the caller guarantees column-ascending (e.g. gnn_ladies_sample output): no
 * unsorted-row check pass is launched (one launch instead of two). */
int gnn_build_operand_sorted_f32(const int32_t* fullrowptr, const int32_t* rowptr,
                                 const void* colidx, int colidx_bytes,
                                 const float* normfact, int64_t nrows, int64_t ncols, int64_t nnz,
                                 int32_t* csr_col, float* csr_val, int64_t* coo_indices, void* stream);

/* ---------------------------------------------------------------------------------
 * Format conversions (replace the per-call preprocessing of cuda_spmm.cu:620-667 and the
 * backward's A.transpose(0,1).coalesce() of custom_sparse_ops.py:34).
 * ------------------------------------------------------------------------------- */

/* Values of the TRANSPOSED operand (Aᵀ, K x M) when the caller already has A's CSC
 * structure (colptr int32[K+1], rows int32[nnz], rows ascending inside each column — e.g.
 * from gnn_ladies_layer_csc): val_t[i] = (float)((1.0/deg_full(rows[i])) * normfact[c]) for
 * the entries of column c, the forward's value of the same entry bit for bit. Then
 * (colptr, rows, val_t) is the canonical transpose (what gnn_csr_transpose builds on the GPU
 * and custom_sparse_ops.py:34 `A.transpose(0,1).coalesce()` computes). */
int gnn_build_operand_t_f32(const int32_t* fullrowptr, const int32_t* colptr, const int32_t* rows,
                            const float* normfact, int64_t nrows, int64_t ncols, int64_t nnz, float* val_t,
                            void* stream);

/* Coalesced COO (int64 row and column index arrays, rows ascending) -> CSR row pointer
 * (int32, M+1) and int32 column indices. `col32` may be NULL to skip the narrowing. */
int gnn_coo_to_csr(const int64_t* row, const int64_t* col, int64_t nnz, int64_t M,
                   int32_t* rowptr, int32_t* col32, void* stream);

/* CSR (M x K) -> CSR of the transpose (K x M), canonical: rows ascending inside every
 * output row, i.e. identical to A.t().coalesce(). Deterministic.
 * tr_rowptr: int32[K+1], tr_col: int32[nnz], tr_val: fp32[nnz].
 * `workspace` >= gnn_csr_transpose_workspace_bytes(M, K, nnz). */
size_t gnn_csr_transpose_workspace_bytes(int64_t M, int64_t K, int64_t nnz);
int gnn_csr_transpose(const int32_t* rowptr, const int32_t* col, const float* val,
                      int64_t M, int64_t K, int64_t nnz,
                      int32_t* tr_rowptr, int32_t* tr_col, float* tr_val,
                      void* workspace, size_t workspace_bytes, void* stream);

/* ---------------------------------------------------------------------------------
 * Feature staging (replaces the masked gathers of main.py:129-134).
 * dst[dst_idx[i], 0:F] = src[src_idx[i], 0:F] for i in [0, n). A NULL src_idx / dst_idx
 * means the identity. Row strides in elements. Indices int64.
 * ------------------------------------------------------------------------------- */
int gnn_gather_rows_f32(const float* src, int64_t ld_src, const int64_t* src_idx,
                        float* dst, int64_t ld_dst, const int64_t* dst_idx,
                        int64_t n, int64_t F, void* stream);

/* Two sources in one launch (round 6): dst[pos0[i]] = src0[idx0[i]] for i < n0, then
 * dst[pos1[i]] = src1[idx1[i]] for i < n1 — the own feature-buffer rows and the batch's host
 * rows of one X0 (main.py:129-134). NULL idx / pos = identity. */
int gnn_gather_rows2_f32(const float* src0, int64_t ld0, const int64_t* idx0, const int64_t* pos0, int64_t n0,
                         const float* src1, int64_t ld1, const int64_t* idx1, const int64_t* pos1, int64_t n1,
                         float* dst, int64_t ld_dst, int64_t F, void* stream);

/* Zero-copy variant for the non-buffered rows (replaces the pageable
 * feat_data[idx_cpu].to(device) of main.py:134): `host_src` is host memory registered with
 * gnn_host_register (pinned, device-mapped); the GPU reads the rows over PCIe, so no host
 * thread copies them. src_idx / dst_idx are device int64 arrays (NULL = identity). A small
 * persistent grid keeps the gather's CU footprint low beside the compute stream. */
int gnn_gather_rows_host_f32(const float* host_src, int64_t ld_src, const int64_t* src_idx,
                             float* dst, int64_t ld_dst, const int64_t* dst_idx,
                             int64_t n, int64_t F, void* stream);

/* Pin + map a host range for device access (hipHostRegister, mapped) / undo it. */
int gnn_host_register(void* host, size_t bytes);
int gnn_host_unregister(void* host);

/* Peer feature buffers read directly over xGMI (replaces the per-peer
 * gpu_buffers[i][idx].to(device) P2P copies of main.py:129-133 without any per-step collective):
 * each rank exports its buffer ONCE — an IPC handle of the allocation holding `ptr` and the byte
 * offset of `ptr` in that allocation — the peers open it ONCE (peer access to `peer_device`
 * enabled when it is another GPU), and gnn_gather_rows_f32 then reads a batch's peer rows
 * straight from the mapped pointer into X0. The buffer must stay allocated and unchanged while
 * peers hold it mapped; gnn_ipc_close undoes gnn_ipc_open. */
#define GNN_IPC_HANDLE_BYTES 64
int gnn_ipc_export(const void* ptr, void* handle_out, int64_t* offset_out);
int gnn_ipc_open(const void* handle, int64_t offset, int peer_device, void** ptr_out);
int gnn_ipc_close(void* ptr, int64_t offset);

/* A stream whose kernels run only on `cus` of the device's CUs, spread evenly over its CU
 * numbering (hipExtStreamCreateWithCUMask; a blocking stream) — experiments with the X0 staging
 * stream (GNN_STAGE_CUS). gnn_stream_destroy releases it. */
int gnn_stream_create_cu_masked(int32_t device, int32_t cus, int32_t priority, void** stream_out);
int gnn_stream_destroy(void* stream);

/* One stream-ordered host-to-device copy (hipMemcpyAsync): the upload of a native loader's
 * batch blob (gnn_sampler.h) — every per-batch array of main.py:115-134 in one transfer. */
int gnn_memcpy_h2d_async(void* dst, const void* src, size_t bytes, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* GNN_SPMM_H */
