/* gnn_extract.h — C ABI of the GPU-side LADIES layer extraction (libgnn_spmm.so, gfx950).
 *
 * Replaces, for every sampled layer whose rows are unique and ascending (all layers below the
 * top one: their rows are the np.unique output of the layer above), the host half of
 *   reference sampler.py:114   U = lap_matrix[previous_nodes, :]
 *   reference sampler.py:133   adj = U[:, after_nodes]
 *   reference sampler.py:135-139  rowptr / colidx / normfact -> create_coo_tensor
 * and the device half, create_coo_tensor (spmm_cpp/spmm.cpp:44-50 -> cuda_spmm.cu:787-827),
 * in one stream-ordered call that reads the graph's CSR resident in device memory. The host
 * sampler keeps the draw (np.random.choice over the column counts of U) and hands over the rows
 * (previous_nodes), the columns (after_nodes), normfact, and — from the same column counts —
 * the exact nnz and the CSC column pointer of adj.
 *
 * Conventions as gnn_spmm.h: device pointers, a hipStream_t as void*, no host syncs, no
 * allocation (graph-capturable), 0 on success / negative or hipError_t code with the message in
 * gnn_last_error().
 */
#ifndef GNN_EXTRACT_H
#define GNN_EXTRACT_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* The operand of one sampled layer and, optionally, its transpose.
 *
 * Graph (device): the lap matrix as canonical CSR (indptr int64[num_nodes+1], indices int32,
 * columns ascending per row, no duplicates); indptr_t / indices_t: the same for lap^T (may alias
 * indptr / indices when the structure is symmetric). deg(v) = indptr[v+1] - indptr[v]; degree
 * int32[num_nodes] holds it (required with the transpose: its values' row degrees).
 * rows  int32[M]: U's rows (node ids) in order; cols int32[K]: after_nodes, strictly ascending;
 * normfact fp32[K]; nnz = number of entries of U[:, cols] (the sum of U's column counts over cols).
 * rowseg int32[M+1] = U's row pointer (exclusive scan of deg(rows[i])); colseg int32[K+1] = the
 * exclusive scan of lapᵀ's row lengths of cols (transpose only) — both host-known (the draw).
 * workspace: gnn_ladies_extract_workspace_bytes(num_nodes, M, K, transpose, rowseg_total,
 * colseg_total) bytes (8 bytes per graph entry scanned plus tables; no state is kept between
 * calls: concurrent calls on different streams need different workspaces).
 * Outputs: rowptr int32[M+1], col int32[nnz] (positions into cols, ascending per row),
 * val fp32[nnz] = (float)((1.0 / deg(rows[i])) * (double)normfact[col]) — identical to
 * gnn_build_operand_f32 on the host-extracted pieces with fullrowptr = rowseg.
 * Transpose (colptr_t != NULL; rows must then be unique and ascending): rows_t int32[nnz] /
 * val_t fp32[nnz] receive the canonical CSR of adj^T (rows ascending in each column) whose row
 * pointer is colptr_t, the host's CSC column pointer (its column counts; not read here) — what
 * gnn_csr_transpose / A.t().coalesce() would produce.
 * rowseg_total = rowseg[M] and colseg_total = colseg[K] (transpose only; ignored otherwise): the
 * graph entries scanned per direction, host-known like the offsets (they size the launch).
 * Work is balanced over entries, not rows (power-law rows): each direction's concatenated graph
 * rows are cut into equal contiguous ranges, one per wave, and every entry is read ONCE (the
 * kept entries of a range go to a gapped buffer, then to their place after a scan of the
 * per-range counts); membership of a node in cols / rows is a bitmap + per-word rank table.
 * err_flag (device int32, optional): OR-ed with 1 / 2 if the kept entries of A / A^T do not add up
 * to nnz (or a segment total differs from the device offsets). The outputs then stay safe to
 * read: writes stay below nnz, entries past the kept ones are zero-filled (column / row 0, value
 * 0) and rowptr is clamped to nnz. */
size_t gnn_ladies_extract_workspace_bytes(int64_t num_nodes, int64_t M, int64_t K, int32_t transpose,
                                          int64_t rowseg_total, int64_t colseg_total);
int gnn_ladies_extract_f32(const int64_t* indptr, const int32_t* indices, const int32_t* degree, int64_t num_nodes,
                           const int64_t* indptr_t, const int32_t* indices_t, const int32_t* rows, int64_t M, const int32_t* cols, int64_t K,
                           const float* normfact, int64_t nnz, const int32_t* rowseg, const int32_t* colseg,
                           const int32_t* colptr_t, int64_t rowseg_total, int64_t colseg_total, int32_t* rowptr,
                           int32_t* col, float* val, int32_t* rows_t, float* val_t, void* workspace,
                           size_t workspace_bytes, int32_t* err_flag, void* stream);

/* U's column counts for the LADIES draw on the GPU (reference sampler.py:116-122,
 * pi = norm(U, ord=0, axis=0)), for a host sampler thread (gnn_sampler.h: gnn_colcount_api).
 * A context belongs to ONE host thread: its own stream, a device count array over the graph's
 * nodes, pinned result buffers. Unlike the rest of this library these calls synchronise with
 * their own stream (the host draw needs the result) and gnn_colcount_create allocates.
 * create: graph = the lap matrix's canonical CSR in device memory (as gnn_ladies_extract_f32;
 *   no stored zeros), device = the HIP device it lives on.
 * add: count the entries of lap rows rows[0..n) (host node ids; repeats count again) into the
 *   context's counts, then return the non-zero columns: *bits = bitmap (host, ceil(N/64) words,
 *   bit c%64 of word c/64), *counts = their counts in ascending column order (host, *nlive
 *   entries). Both stay valid until the next call on the context.
 * reset: zero the counts (stream-ordered before the next add).
 * The counts are summed without global atomics (a bucket partition + LDS histograms) unless
 * GNN_CC_HIST=atomic is set when the context is created; same counts either way. GNN_CC_CUS=n:
 * the context's stream on n of the device's CUs (own hardware queue; default: a plain stream).
 * Note: hipExtStreamCreateWithCUMask makes a BLOCKING stream (the default is non-blocking), so
 * with GNN_CC_CUS set the counter's work also orders against legacy null-stream work; the bench's
 * producers issue none (torch and the library use explicit streams), off by default.
 * A call's entry total is carried in int64; a call of 2^31 or more entries (beyond the int32
 * partition offsets) runs the atomic form instead. */
int gnn_colcount_create(int32_t device, int64_t num_nodes, const int64_t* indptr, const int32_t* indices, void** ctx);
/* The stream of the contexts created after this call (process-wide): cus = 0 a plain stream
 * (default), cus > 0 a stream over that many CUs (>= the device's: all of them) — a CU-masked
 * stream gets a hardware queue of its own instead of sharing one with the training step's streams
 * (GPU_MAX_HW_QUEUES is 4). GNN_CC_CUS, when set, overrides. Returns 0, or -22 for cus < 0. */
int gnn_colcount_set_cus(int32_t cus);
int gnn_colcount_add(void* ctx, const int64_t* rows, int64_t n, int64_t* nlive, const uint64_t** bits,
                     const int32_t** counts);
int gnn_colcount_reset(void* ctx);
void gnn_colcount_destroy(void* ctx);

#ifdef __cplusplus
}
#endif

#endif /* GNN_EXTRACT_H */
