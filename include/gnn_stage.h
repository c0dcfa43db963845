/* gnn_stage.h — one native call that stages a batch of the native loader on the device
 * (libgnn_spmm.so; gnn_amd/csrc/stage.hip).
 *
 * Replaces the host side of the reference's per-batch staging (main.py:129-134: X0 assembled
 * from the GPU buffers and the host rows; sampler.py:135-139: create_coo_tensor per layer) as
 * the training thread issued it through ~25 Python / ctypes calls per batch (staging.Stager.issue
 * + loader.NativeBatch.to_device + sampler.DeviceBatch.build_operands): the batch blob's upload,
 * X0's own-buffer and host rows (gnn_gather_rows2_f32), every layer's operand — extracted from the
 * graph resident in HBM (gnn_ladies_extract_f32, with its transpose from layer csc_from up) or
 * built from the blob's CSR (gnn_build_operand_sorted_f32 + gnn_build_operand_t_f32 on the
 * blob's CSC) — and the copy of the extraction error flag into pinned host memory. The same
 * library calls with the same arguments as the Python path, so the outputs are bit-identical.
 *
 * The blob is the one gnn_loader_next hands out (gnn_sampler.h: descriptor GNN_BLOB_* / GNN_H_* /
 * GNN_L_* / GNN_B_*); host copy pinned, device copy of GNN_H_BYTES bytes (256-byte aligned).
 * Stream-ordered, no allocation, no host synchronisation (graph-capturable when the upload is
 * skipped). Returns 0 or a status (text: gnn_last_error()).
 *
 * Arguments: an int64 array of GNN_STAGE_SLOTS slots (GNN_ST_*; pointers stored as integers):
 *   DESC / HOST_BLOB / DEV_BLOB   the batch's descriptor (host), blob (host, pinned) and its device
 *                                 copy; UPLOAD = 1: copy host -> device first (0: already there)
 *   BUFFER, LD_BUFFER             this rank's GPU feature buffer (rows of the own-buffer inputs)
 *   X0, LD_X0, F                  X0 (n_inputs x LD_X0 floats) and the row width the gathers copy
 *                                 (the padded width: buffer rows, host rows and X0 rows all hold it)
 *   INDPTR, INDICES, DEGREE, NUM_NODES, INDPTR_T, INDICES_T, ERR
 *                                 the graph on the device (sampler.DeviceGraph) for GPU-extracted
 *                                 layers, and its error flag; ERR_HOST: pinned int32 the flag is
 *                                 copied to after the extractions (0: no copy)
 *   GATE                          a hipEvent_t the gathers and operand builds wait for (0: none);
 *                                 the upload goes ahead of it
 *   CSC_FROM                      layers >= CSC_FROM get their transpose
 *   ARENA, ARENA_BYTES            the outputs (operand arrays, extraction workspace), laid out by
 *                                 gnn_stage_plan
 * gnn_stage_plan writes, per layer li, GNN_STAGE_OUT_SLOTS int64 at out[li * GNN_STAGE_OUT_SLOTS]:
 * the arena byte offsets of the operand's rowptr, col, val and of its transpose's rows and values
 * (GNN_SO_*), -1 where the array is a section of the blob (rowptr of a host-built layer; the
 * transpose's colptr is always the blob's GNN_L_CSC_COLPTR, its rows for a host-built layer the
 * blob's GNN_L_CSC_ROWS) or absent, and in layer 0's GNN_SO_WORKSPACE slot the offset of the
 * extraction workspace (-1: none); it returns the arena bytes (0 on error).
 */
#ifndef GNN_STAGE_H
#define GNN_STAGE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GNN_STAGE_SLOTS 24
#define GNN_STAGE_OUT_SLOTS 6

enum {
  GNN_ST_DESC = 0, GNN_ST_HOST_BLOB = 1, GNN_ST_DEV_BLOB = 2, GNN_ST_UPLOAD = 3, GNN_ST_BUFFER = 4,
  GNN_ST_LD_BUFFER = 5, GNN_ST_X0 = 6, GNN_ST_LD_X0 = 7, GNN_ST_F = 8, GNN_ST_INDPTR = 9, GNN_ST_INDICES = 10,
  GNN_ST_DEGREE = 11, GNN_ST_NUM_NODES = 12, GNN_ST_INDPTR_T = 13, GNN_ST_INDICES_T = 14, GNN_ST_ERR = 15,
  GNN_ST_ERR_HOST = 16, GNN_ST_GATE = 17, GNN_ST_CSC_FROM = 18, GNN_ST_ARENA = 19, GNN_ST_ARENA_BYTES = 20
};

enum { GNN_SO_ROWPTR = 0, GNN_SO_COL = 1, GNN_SO_VAL = 2, GNN_SO_ROWS_T = 3, GNN_SO_VAL_T = 4, GNN_SO_WORKSPACE = 5 };

/* Arena layout of a batch (see above); `out` holds GNN_BLOB_MAX_LAYERS * GNN_STAGE_OUT_SLOTS. */
size_t gnn_stage_plan(const int64_t* args, int64_t* out);

/* Stage the batch on `stream` (hipStream_t). */
int gnn_stage_batch_f32(const int64_t* args, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* GNN_STAGE_H */
