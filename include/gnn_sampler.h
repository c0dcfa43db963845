/*
 * gnn_sampler.h — native LADIES layer-wise sampler (host C++, libgnn_sampler.so).
 *
 * Replaces the per-batch numpy/scipy work of ladies_sampler (sampler.py:90-160): for each
 * layer, top-down, U = lap[previous, :] (sampler.py:112), column nonzero counts of U
 * (sp.linalg.norm(U, ord=0, axis=0), :117), p = counts / sum (:122),
 * s_num = min(#(p > 0), samp_num) (:126), np.random.choice(N, s_num, p=p, replace=False)
 * under np.random.seed(seed) (:96, :128 — numpy's legacy MT19937 stream and its
 * without-replacement loop restated exactly), after = unique(sampled ∪ previous) (:131),
 * the sub-graph U[:, after] as CSR (:133-136, int32 columns instead of int16),
 * normfact = 1 / float32(clip(s_num * p[after], 1e-10, 1)) (:137) and
 * sampled_nodes = positions of previous in after (:143).
 * Results are bit-identical to the numpy path (tests/test_sampler_native.py).
 *
 * The graph is CSR with sorted, duplicate-free column indices per row (scipy canonical
 * format: the reference's sp.linalg.norm canonicalises U in place before U[:, after]).
 * `data` may be NULL (every stored entry non-zero); otherwise entries equal to 0 are kept
 * in the structure but not counted, as sp.linalg.norm(ord=0) does.
 *
 * Thread-safe: independent calls may run concurrently (each owns its scratch). Returns 0 or
 * a non-zero status; text via gnn_sampler_last_error() (thread-local).
 */
#ifndef GNN_SAMPLER_H
#define GNN_SAMPLER_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct gnn_ladies_result gnn_ladies_result;

const char* gnn_sampler_last_error(void);

/* Sample one mini-batch. orders[num_layers] bottom-up as the reference's `orders`;
 * samp_num[num_layers] indexed top-down as samp_num_list[d] (sampler.py:124). A layer with
 * order 0 yields no sub-graph (sampler.py:107-110). On success *out owns the result. */
int gnn_ladies_sample(const int64_t* indptr, const int32_t* indices, const float* data, int64_t num_nodes,
                      const int64_t* batch_nodes, int64_t batch_size, const int64_t* samp_num,
                      const int32_t* orders, int32_t num_layers, uint32_t seed, gnn_ladies_result** out);

/* Same draw (bit-identical RNG stream, sampled nodes, normfact), with device_extract a mask over
 * the bottom-up layer index (-1: all): every selected layer below the top one (its rows are the
 * ascending, unique `after` of the layer above) is NOT extracted on the host — the host keeps only what the draw needs (U's column counts) and records
 * the layer's rows, columns, exact nnz and CSC column pointer for gnn_ladies_extract_f32
 * (include/gnn_extract.h), which builds adj = U[:, after] and its transpose on the GPU from the
 * graph resident there. Requires data == NULL (no stored zeros: the column counts are then the
 * structural counts the extraction keeps). The top layer (rows = the batch) is host-extracted.
 * indptr_t: lapᵀ's row pointer (NULL: the structure is symmetric, lapᵀ's = indptr) — for the
 * offsets of the transposed extraction's segments. */
int gnn_ladies_sample_dev(const int64_t* indptr, const int32_t* indices, const float* data, const int64_t* indptr_t,
                          int64_t num_nodes,
                          const int64_t* batch_nodes, int64_t batch_size, const int64_t* samp_num,
                          const int32_t* orders, int32_t num_layers, uint32_t seed, int32_t device_extract,
                          gnn_ladies_result** out);

/* Optional device column counting for the LADIES draw: libgnn_spmm.so's gnn_colcount_* entry
 * points (include/gnn_extract.h), bound by address — this library stays free of the GPU runtime —
 * and the graph's CSR in device memory (no stored zeros). With it U's column counts (the
 * draw's p, sampler.py:116-122) are summed on the GPU from the rows each layer adds; the draw,
 * and so every output, is unchanged. ctx: from create(device, num_nodes, indptr, indices, &ctx)
 * on the calling thread (a context belongs to one thread). */
typedef struct gnn_colcount_api {
  int (*create)(int32_t device, int64_t num_nodes, const int64_t* indptr, const int32_t* indices, void** ctx);
  int (*add)(void* ctx, const int64_t* rows, int64_t n, int64_t* nlive, const uint64_t** bits, const int32_t** counts);
  int (*reset)(void* ctx);
  void (*destroy)(void* ctx);
  int32_t device;
  const int64_t* indptr;  /* device */
  const int32_t* indices; /* device */
} gnn_colcount_api;

/* gnn_ladies_sample_dev with U's column counts on the device (cc, cc_ctx; both NULL: on the host). */
int gnn_ladies_sample_cc(const int64_t* indptr, const int32_t* indices, const float* data, const int64_t* indptr_t,
                         int64_t num_nodes, const int64_t* batch_nodes, int64_t batch_size, const int64_t* samp_num,
                         const int32_t* orders, int32_t num_layers, uint32_t seed, int32_t device_extract,
                         const gnn_colcount_api* cc, void* cc_ctx, gnn_ladies_result** out);

/* subgraph_sampler (sampler.py:7-88): ONE importance draw from the batch's neighbourhood
 * (same p, s_num = min(#(p > 0), samp_num[0]), same RNG use), after = unique(sampled ∪ batch);
 * the top-most layer with a non-zero order gets lap[batch, :][:, after]; every layer below it
 * (whatever its order — reference behaviour) gets the square lap[after, :][:, after] with the
 * same normfact and sampled_nodes = arange(len(after)). Same result object as LADIES. */
int gnn_subgraph_sample(const int64_t* indptr, const int32_t* indices, const float* data, int64_t num_nodes,
                        const int64_t* batch_nodes, int64_t batch_size, const int64_t* samp_num,
                        const int32_t* orders, int32_t num_layers, uint32_t seed, gnn_ladies_result** out);

/* FastGCN layer-wise sampler (Chen et al. 2018; NOT in the reference — BASELINE config 5;
 * parity unpinned): p is the caller's layer-independent importance over all nodes
 * (fastgcn_probability: column sums of lap∘lap, normalised); per layer, top-down,
 * U = lap[prev, :], s_num = min(#(p > 0), samp_num[d]), np.random.choice(N, s_num, p=p,
 * replace=False) on the same RNG stream as LADIES, after = unique(sampled) (no union with
 * prev), adj = U[:, after], normfact = 1 / float32(clip(s_num * p[after], 1e-10, 1)).
 * Same result object as LADIES. */
int gnn_fastgcn_sample(const int64_t* indptr, const int32_t* indices, const float* data, int64_t num_nodes,
                       const double* p, const int64_t* batch_nodes, int64_t batch_size, const int64_t* samp_num,
                       const int32_t* orders, int32_t num_layers, uint32_t seed, gnn_ladies_result** out);

/* The FastGCN draw keeps, per sampler thread, the candidate list and base cdf of the p array it
 * last saw (keyed by its address, length and a sample of its values). A caller that rewrites a
 * p array in place — or frees one and passes another that may reuse the address — calls this
 * first: every thread rebuilds its cache on its next draw. Thread-safe. */
void gnn_fastgcn_p_changed(void);

/* dims of layer `layer` (bottom-up, as the returned adjs): {M, K, nnz, n_sampled, s_num}.
 * Returns 1 if the layer has order 0 (no sub-graph), 0 otherwise. */
int gnn_ladies_layer_dims(const gnn_ladies_result* r, int32_t layer, int64_t dims[5]);

/* Copy layer arrays out: fullrowptr int32[M+1] (indptr of U), rowptr int32[M+1] (indptr of
 * U[:, after]), colidx int32[nnz], normfact float32[K], sampled int64[n_sampled]. Any
 * pointer may be NULL to skip that array. */
int gnn_ladies_layer_copy(const gnn_ladies_result* r, int32_t layer, int32_t* fullrowptr, int32_t* rowptr,
                          int32_t* colidx, float* normfact, int64_t* sampled);

/* A layer left to the device extraction: rows int32[M] (U's rows, node ids), cols int32[K]
 * (after_nodes, ascending), colptr int32[K+1] (CSC column pointer of adj; colptr[K] = nnz),
 * rowseg int32[M+1] (U's row pointer = the offsets of lap's rows of `rows` concatenated),
 * colseg int32[K+1] (the offsets of lapᵀ's rows of `cols` concatenated).
 * Returns 0 and copies (NULL pointers skip) for such a layer, 1 for a host-extracted or absent
 * layer (nothing copied). rowptr / colidx of gnn_ladies_layer_copy are not made for it;
 * fullrowptr (= rowseg), normfact and sampled are. */
int gnn_ladies_layer_device(const gnn_ladies_result* r, int32_t layer, int32_t* rows, int32_t* cols,
                            int32_t* colptr, int32_t* rowseg, int32_t* colseg);

/* CSC structure of layer `layer`'s sub-graph (= CSR of its transpose, canonical: rows
 * ascending inside each column): colptr int32[K+1], rows int32[nnz]. Lets the training
 * pipeline hand the backward aggregation its operand without a GPU transpose
 * (custom_sparse_ops.py:34 `A.transpose(0,1).coalesce()`). */
int gnn_ladies_layer_csc(const gnn_ladies_result* r, int32_t layer, int32_t* colptr, int32_t* rows);

/* The layer-0 input node ids (the last `after`, sorted). */
int64_t gnn_ladies_num_input_nodes(const gnn_ladies_result* r);
int gnn_ladies_input_nodes(const gnn_ladies_result* r, int64_t* out);

void gnn_ladies_free(gnn_ladies_result* r);

/* ---------------------------------------------------------------------------------------
 * Native batch producer (loader.cpp): prepare_data's thread pool (sampler.py:163-210) plus the
 * host half of the feature staging (main.py:129-134) in C++ threads that never take the Python
 * GIL. Each batch becomes ONE contiguous blob (pinned through the process's HIP runtime when it
 * is loaded and `pinned` != 0) described by an int64 descriptor:
 *   header  [GNN_BLOB_HEADER] slots GNN_H_*;
 *   layer li (bottom-up) at GNN_BLOB_HEADER + li * GNN_BLOB_LAYER_SLOTS: scalars GNN_L_* and
 *     sections (byte offset, element count) at the GNN_L_* section slots;
 *   batch sections at GNN_BLOB_HEADER + num_layers * GNN_BLOB_LAYER_SLOTS + GNN_B_*, then per
 *     peer j (world entries): peer_pos at + GNN_BLOB_BATCH_SLOTS + 4 j, peer_src at + 2.
 * Sections are 256-byte aligned; absent sections have count 0. Element types: int32 for
 * fullrowptr / rowptr / colidx / csc_colptr / csc_rows / rows / cols / rmap, fp32 for normfact,
 * labels [batch x classes] and host_rows [n_host x ld_x0] (zero-padded rows of the feature
 * table), int64 for sampled and every placement list. Layer semantics as gnn_ladies_sample_dev
 * (device-extracted layers carry rows / cols / csc_colptr / fullrowptr (= rowseg) / colseg
 * instead of the CSR pieces, int32); rmap[K]
 * (layers >= 1): rmap[sampled[i]] = i, -1 elsewhere. */
#define GNN_BLOB_VERSION 1
#define GNN_BLOB_MAX_LAYERS 16
#define GNN_BLOB_HEADER 16
#define GNN_BLOB_LAYER_SLOTS 32
#define GNN_BLOB_BATCH_SLOTS 16
enum {
  GNN_H_VERSION = 0, GNN_H_LAYERS = 1, GNN_H_BYTES = 2, GNN_H_BATCH = 3, GNN_H_CLASSES = 4, GNN_H_INPUTS = 5,
  GNN_H_WORLD = 6, GNN_H_LD_X0 = 7, GNN_H_SEED = 8, GNN_H_PINNED = 9
};
enum {
  GNN_L_PRESENT = 0, GNN_L_ON_DEVICE = 1, GNN_L_M = 2, GNN_L_K = 3, GNN_L_NNZ = 4, GNN_L_SNUM = 5,
  GNN_L_NSAMPLED = 6, GNN_L_HAS_RMAP = 7, GNN_L_FULLROWPTR = 8, GNN_L_ROWPTR = 10, GNN_L_COLIDX = 12,
  GNN_L_NORMFACT = 14, GNN_L_CSC_COLPTR = 16, GNN_L_CSC_ROWS = 18, GNN_L_ROWS = 20, GNN_L_COLS = 22,
  GNN_L_SAMPLED = 24, GNN_L_RMAP = 26, GNN_L_COLSEG = 28
};
enum {
  GNN_B_LABELS = 0, GNN_B_HOST_ROWS = 2, GNN_B_OWN_POS = 4, GNN_B_OWN_SRC = 6, GNN_B_HOST_POS = 8,
  GNN_B_HOST_SRC = 10, GNN_B_INPUT_NODES = 12
};
enum { GNN_SAMPLER_LADIES = 0, GNN_SAMPLER_SUBGRAPH = 1, GNN_SAMPLER_FASTGCN = 2 };

typedef struct gnn_loader gnn_loader;
typedef struct gnn_batch gnn_batch;

/* Borrowed arrays (the caller keeps them alive until gnn_loader_destroy): the graph as for the
 * samplers; labels as CSR (int64 indptr, int32 indices, fp32 values, num_classes columns);
 * the placement of this rank (device_id_of_nodes / idx_of_nodes_on_device, main.py:95-103),
 * devices[world]; feat (NULL: no host-row gather, e.g. zero-copy staging) with row stride
 * ld_feat, F features, host rows written ld_x0 wide. kind GNN_SAMPLER_*; fastgcn_p for FastGCN;
 * device_extract as gnn_ladies_sample_dev; host-extracted layers >= csc_from also get their CSC.
 * Returns NULL on bad arguments (message in gnn_sampler_last_error). */
gnn_loader* gnn_loader_create(const int64_t* indptr, const int32_t* indices, const float* data,
                              const int64_t* indptr_t, int64_t num_nodes,
                              const int64_t* label_indptr, const int32_t* label_indices, const float* label_values,
                              int64_t num_classes, const int64_t* device_id_of_nodes,
                              const int64_t* idx_of_nodes_on_device, int32_t rank, int32_t world,
                              const int64_t* devices, const float* feat, int64_t ld_feat, int64_t F, int64_t ld_x0,
                              const int64_t* samp_num, const int32_t* orders, int32_t num_layers, int32_t kind,
                              const double* fastgcn_p, int32_t device_extract, int32_t csc_from, int32_t workers,
                              int32_t pinned);
/* LADIES loaders: count U's columns on the device (each worker thread makes its own context on
 * first use). Call before the first gnn_loader_submit; api is copied. */
int gnn_loader_set_colcount(gnn_loader* ld, const gnn_colcount_api* api);
/* With gnn_loader_set_colcount: only worker threads 0 .. workers-1 count on the device, the others
 * on the host (0 = all of them; the batches are the same either way: the counts are exact). Device
 * counts cost the GPU ~1.2 ms per ogbn-products-sized batch beside the step, host counts ~9 ms of a
 * worker's CPU: a mix keeps both the GPU and the producers below their bound. GNN_CC_WORKERS, when
 * set, overrides. Call before the first gnn_loader_submit. */
int gnn_loader_set_colcount_workers(gnn_loader* ld, int32_t workers);
/* Queue one batch (node ids copied); batches come out of gnn_loader_next in submission order. */
int gnn_loader_submit(gnn_loader* ld, uint32_t seed, const int64_t* nodes, int64_t n);
/* Block until the oldest submitted batch is ready. On a sampling error returns its status (the
 * message in gnn_sampler_last_error) and *out = NULL. */
int gnn_loader_next(gnn_loader* ld, gnn_batch** out);
const int64_t* gnn_batch_desc(const gnn_batch* b, int64_t* n);
void* gnn_batch_blob(const gnn_batch* b);
/* Return the blob to its pool (call once the device copy that reads it has completed). */
void gnn_batch_release(gnn_batch* b);
/* Stops the threads (queued batches are dropped); batches already handed out stay valid. */
void gnn_loader_destroy(gnn_loader* ld);

/* Host half of the layer-0 feature staging (main.py:134, `feat_data[idx_cpu]`): copy rows
 * src[idx[i], 0:F] into dst row i (stride ld_dst, columns [F, ld_dst) zeroed) — typically a
 * pinned buffer that one hipMemcpyAsync then moves to the GPU. */
int gnn_host_gather_rows_f32(const float* src, int64_t ld_src, int64_t num_src_rows, const int64_t* idx, int64_t n,
                             int64_t F, float* dst, int64_t ld_dst);

/* LADIES draw phase timers, summed over all threads since the last reset, when the process runs
 * with GNN_SAMPLER_PROFILE=1 (returns 1 otherwise): out[0..n) = seconds in scratch reset, U's
 * row pointer, U's column counts, the draw, unique(sampled ∪ prev), the extraction (or the
 * device-layer metadata), normfact / positions; out[7] = calls. */
int gnn_sampler_profile(double* out, int32_t n, int32_t reset);

/* numpy legacy RandomState(seed).random_sample(n) — exposed for the RNG-stream tests. */
int gnn_mt19937_random_sample(uint32_t seed, int64_t n, double* out);

#ifdef __cplusplus
}
#endif

#endif /* GNN_SAMPLER_H */
