/*
 * gnn_optim.h — gradient clipping + Adam for the data-parallel step (libgnn_spmm.so).
 *
 * Replaces, per rank, torch.nn.utils.clip_grad_norm_(params, max_norm) and
 * torch.optim.Adam.step() of the reference's training loop (main.py:146-170), whose
 * semantics are kept: the clip uses the rank's own gradients (before the cross-rank sum),
 * the gradients are summed (not averaged) across ranks, Adam is torch's (amsgrad off, no
 * weight decay). Tensors are passed as HOST arrays of device pointers (count <= 32 per
 * call); n[i] = element count. Partial sums are per 1024-element chunk:
 * gnn_optim_chunks(count, n) floats of device workspace.
 *
 *  N = 1:  gnn_grad_sqnorm_f32 -> gnn_clip_scale_f32 -> gnn_adam_f32(scale)   (clip inside)
 *  N > 1:  gnn_grad_sqnorm_f32 -> gnn_clip_scale_f32 -> gnn_scale_into_f32 (clipped grads into
 *          the flat all-reduce buffer) -> all-reduce(SUM) -> gnn_adam_f32(scale = NULL) on the
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

/* *scale = min(1, max_norm / (sqrt(sum of the nchunks partials) + 1e-6)); max_norm > 0. */
int gnn_clip_scale_f32(const float* partial, int64_t nchunks, float max_norm, float* scale, void* stream);

/* flat[off_i + e] = g_i[e] * (*scale) (scale may be NULL: 1); off_i = sum of n before i. */
int gnn_scale_into_f32(int count, const float* const* g, const int64_t* n, const float* scale, float* flat,
                       void* stream);

/* One Adam step (torch semantics, step = 1-based count), the gradient multiplied by *scale
 * (device float; NULL = 1) as it is read. */
int gnn_adam_f32(int count, float* const* p, const float* const* g, float* const* m, float* const* v,
                 const int64_t* n, const float* scale, float lr, float beta1, float beta2, float eps, int64_t step,
                 void* stream);

#ifdef __cplusplus
}
#endif

#endif /* GNN_OPTIM_H */
