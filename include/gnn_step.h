/* gnn_step.h — native executor of a GraphSAGE / GCN training step's forward + backward
 * (libgnn_spmm.so, gfx950; gnn_amd/csrc/step.hip).
 *
 * Replaces the host side of the reference's step (main.py:122-146: model(x0, adjs,
 * sampled_nodes) -> utils.loss -> loss.backward(); models.py:6-97, utils.py:129-140) — the
 * ~45 autograd Functions / ctypes calls per step of gnn_amd.models' fused path — with ONE call
 * that issues the same kernels (aggregation gnn_spmm_csr_f32[_ex], row gather, split3 / rocBLAS
 * GEMMs, gnn_sage_norm_*, gnn_head_bce_*) with the same routing and dropout seeds. Gradients
 * are written into caller-provided buffers; clip / all-reduce / Adam stay with the caller
 * (gnn_optim.h). Stream-ordered; every intermediate lives in one caller-provided workspace of
 * gnn_train_step_workspace_bytes(desc) bytes (256-byte aligned). Returns 0 or a status (text:
 * gnn_last_error()).
 *
 * The descriptor is an int64 array: a header of GNN_STEP_HEADER slots (GNN_SH_*), then
 * GNN_STEP_LAYER_SLOTS slots per layer, bottom-up (GNN_SL_*). Pointers are device pointers
 * stored as integers; float scalars as their IEEE bits.
 *   header: kind (GNN_STEP_SAGE: cat[linearB(x[sampled]), linearW(A·x)]; GNN_STEP_GCN:
 *     linear(A·x)), layers, nhid N, x0 (K0 x F0, row stride ldx0: the staged X0), the head
 *     (W C x D, bias, their gradient buffers), labels (M_top x C, row stride ldl), the head's
 *     dropout seed, p (dropout), training (0: no dropout), loss (device float out), and
 *     optionally timing: a HOST int64 array T, T[0] = capacity in records, then records of
 *     GNN_STEP_TIMING_SLOTS slots; the caller puts a hipEvent_t pair in slots 0-1 of each, and
 *     the step arms them around its aggregation kernels in call order (forward layers bottom-up,
 *     then the backward aggregations top-down) and writes slots 2-14: kind (0 fwd, 1 bwd),
 *     layer, M, K, nnz, F, padded F, ldx, ldy, X, Y (device addresses), residual rows, 1;
 *     and optionally gradient-ready events: a HOST int64 array E, E[0] = entries, E[1] = a
 *     hipEvent_t recorded once the head's gradients are final, E[2 + l] = one recorded once
 *     layer l's gradients (weights, biases, scale, offset) are final (0 = none): the caller's
 *     data-parallel exchange starts on a bucket while the backward of the layers below runs;
 *     and optionally a staging gate: a hipEvent_t (GNN_SH_STAGE_EVENT, 0 = none) recorded on the
 *     step's stream right after layer GNN_SH_STAGE_LAYER's forward aggregation — the caller's
 *     staging stream waits on it before the next batches' row gathers and layer extractions, so
 *     those gather-bound kernels run beside the GEMMs and tails instead of competing with the
 *     aggregation for L2 (main.py:129-137's staging, overlapped with the step);
 *     and the phase (GNN_SH_PHASE): 0 = the whole step; 1 = only layer 0's forward aggregation
 *     A_0·x0, into the workspace (a data-parallel caller issues the NEXT batch's while this
 *     step's gradient all-reduce runs: it reads only the batch, never a parameter); 2 = the step
 *     of a batch whose layer-0 aggregation a phase-1 call with the same descriptor already issued
 *     into the same workspace (it is not issued again). 0 and 1 + 2 give the same results.
 *   layer l: the operand A (rowptr / col / val, M x K, nnz) and its transpose (K x M, layers >= 1),
 *     sampled (int64 [M], SAGE) and rmap (int32 [K], rmap[sampled[i]] = i, SAGE layers >= 1),
 *     weights W_W / W_B (N x F row-major), biases, scale / offset, their gradient buffers, the
 *     dropout seed. Layer l >= 1 reads layer l-1's output (K_l must equal M_{l-1}).
 */
#ifndef GNN_STEP_H
#define GNN_STEP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GNN_STEP_VERSION 1
#define GNN_STEP_MAX_LAYERS 4
#define GNN_STEP_HEADER 24
#define GNN_STEP_LAYER_SLOTS 32
#define GNN_STEP_SAGE 0
#define GNN_STEP_GCN 1
#define GNN_STEP_TIMING_SLOTS 16

enum {
  GNN_SH_VERSION = 0, GNN_SH_LAYERS = 1, GNN_SH_KIND = 2, GNN_SH_X0 = 3, GNN_SH_LDX0 = 4, GNN_SH_F0 = 5,
  GNN_SH_HEAD_W = 6, GNN_SH_HEAD_B = 7, GNN_SH_HEAD_GW = 8, GNN_SH_HEAD_GB = 9, GNN_SH_CLASSES = 10,
  GNN_SH_LABELS = 11, GNN_SH_LDL = 12, GNN_SH_HEAD_SEED = 13, GNN_SH_PDROP_BITS = 14, GNN_SH_TRAINING = 15,
  GNN_SH_LOSS = 16, GNN_SH_NHID = 17, GNN_SH_TIMING = 18, GNN_SH_GRAD_EVENTS = 19, GNN_SH_STAGE_EVENT = 20,
  GNN_SH_STAGE_LAYER = 21, GNN_SH_PHASE = 22
};
enum {
  GNN_SL_ROWPTR = 0, GNN_SL_COL = 1, GNN_SL_VAL = 2, GNN_SL_M = 3, GNN_SL_K = 4, GNN_SL_NNZ = 5,
  GNN_SL_TROWPTR = 6, GNN_SL_TCOL = 7, GNN_SL_TVAL = 8, GNN_SL_SAMPLED = 9, GNN_SL_NSAMPLED = 10,
  GNN_SL_RMAP = 11, GNN_SL_WW = 12, GNN_SL_BW = 13, GNN_SL_WB = 14, GNN_SL_BB = 15, GNN_SL_SCALE = 16,
  GNN_SL_OFFSET = 17, GNN_SL_GWW = 18, GNN_SL_GBW = 19, GNN_SL_GWB = 20, GNN_SL_GBB = 21, GNN_SL_GSCALE = 22,
  GNN_SL_GOFFSET = 23, GNN_SL_SEED = 24
};

size_t gnn_train_step_workspace_bytes(const int64_t* desc);
int gnn_train_step_f32(const int64_t* desc, void* workspace, size_t workspace_bytes, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* GNN_STEP_H */
