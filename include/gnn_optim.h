/*
 * gnn_optim.h — gradient clipping + Adam for the data-parallel step (libgnn_spmm.so).
 *
 * Replaces, per rank, torch.nn.utils.clip_grad_norm_(params, max_norm) and
 * torch.optim.Adam.step() of the reference's training loop (main.py:146-170), whose
 * semantics are kept: the clip uses the rank's own gradients (before the cross-rank sum),
 * the gradients are summed (not averaged) across ranks, Adam is torch's (amsgrad off, no
 * weight decay). Tensors are passed as HOST arrays of device pointers (count <= 32 per
 * call); n[i] = element count. Partial sums are per 8192-element chunk:
 * gnn_optim_chunks(count, n) floats of device workspace.
 *
 *  N = 1:  gnn_grad_sqnorm_f32  ->  gnn_adam_f32(partial, max_norm)   (clip applied inside)
 *  N > 1:  gnn_grad_sqnorm_f32  ->  gnn_clip_scale_into_f32 (clipped grads into the flat
 *          all-reduce buffer)  ->  all-reduce(SUM)  ->  gnn_adam_f32(partial = NULL) on the
 *          flat buffer's views.
 */
#ifndef GNN_OPTIM_H
#define GNN_OPTIM_H

#include <stddef.h>
#include <stdint.h>

#define GNN_OPTIM_MAX_TENSORS 32

#ifdef __cplusplus
extern "C" {
#endif

int64_t gnn_optim_chunks(int count, const int64_t* n);

/* partial[c] = sum of g^2 over chunk c (fixed order inside the chunk). */
int gnn_grad_sqnorm_f32(int count, const float* const* g, const int64_t* n, float* partial, void* stream);

/* flat[off_i + e] = g_i[e] * min(1, max_norm / (||g|| + 1e-6)) (max_norm <= 0: no clip);
 * off_i = sum of n before i. scale_out (device float, may be NULL) receives the factor. */
int gnn_clip_scale_into_f32(int count, const float* const* g, const int64_t* n, const float* partial,
                            float max_norm, float* flat, float* scale_out, void* stream);

/* One Adam step (torch semantics, step = 1-based count) with the gradient scaled by the clip
 * factor computed from `partial` (nchunks_partial entries) when partial != NULL and
 * max_norm > 0. */
int gnn_adam_f32(int count, float* const* p, const float* const* g, float* const* m, float* const* v,
                 const int64_t* n, const float* partial, int64_t nchunks_partial, float max_norm, float lr,
                 float beta1, float beta2, float eps, int64_t step, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* GNN_OPTIM_H */
