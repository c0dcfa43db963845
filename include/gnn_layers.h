/*
 * gnn_layers.h — fused epilogue of the GraphSAGE / GCN convolution (libgnn_spmm.so).
 *
 * Replaces the elementwise tail of GraphSageConvolution.forward (models.py:18-25) and
 * GraphConvolution.forward (models.py:58-64), plus the dropout GraphSage/GCN apply to each
 * layer's output (models.py:43,82):
 *     h   = cat([hB + biasB, hW + biasW], 1)      (GCN: h = hW + biasW, D1 = 0)
 *     o   = elu(h)
 *     y   = (o - mean(o)) * scale * rsqrt(var(o) + 1e-9) + offset     (biased var, per row)
 *     out = dropout(y, p)                          (training only; inverted scaling)
 * in ONE pass over the rows (one wave per row, the row held in registers), and its
 * backward in one more pass plus a deterministic column reduction for d(scale), d(offset)
 * and the linear biases' gradients d(biasB), d(biasW) (hB / hW are the bias-free linear
 * outputs; biases may be NULL, then their gradients are not written).
 * Dropout masks come from a counter-based hash of (seed, row * D + col): nothing is stored,
 * backward regenerates them.
 *
 * All pointers are device pointers; row strides in elements; D = D1 + D2, D1 % 4 == 0,
 * D <= 2048. Returns 0 or a non-zero status (text: gnn_last_error()).
 */
#ifndef GNN_LAYERS_H
#define GNN_LAYERS_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

int gnn_sage_norm_fwd_f32(const float* hB, int64_t ldb, int64_t D1, const float* hW, int64_t ldw, int64_t D2,
                          const float* biasB, const float* biasW, const float* scale, const float* offset, int64_t M,
                          float p_drop, uint64_t seed, int training, float* Y, int64_t ldy, float* mean_out,
                          float* rstd_out, void* stream);

size_t gnn_sage_norm_bwd_workspace_bytes(int64_t M, int64_t D);

int gnn_sage_norm_bwd_f32(const float* gY, int64_t ldg, const float* hB, int64_t ldb, int64_t D1, const float* hW,
                          int64_t ldw, int64_t D2, const float* biasB, const float* biasW, const float* scale,
                          const float* mean, const float* rstd, int64_t M, float p_drop, uint64_t seed, int training,
                          float* dhB, float* dhW, float* dscale, float* doffset, float* dbiasB, float* dbiasW,
                          void* workspace, size_t workspace_bytes, void* stream);

/* gnn_sage_norm_bwd_f32 whose output gradient is not a dense gY but the aggregation of the layer
 * above, computed per row as the tail reads it:
 *   gY[r] = Σ_e t_val[e] · G[t_col[e]]  (e over Aᵀ's row r, a C fmaf chain from 0 in CSR order)
 *           + R[rmap[r]]               (when rmap[r] >= 0; rmap NULL: no residual)
 * — the same values gnn_spmm_csr_f32_ex produces for this operand with its row kernel (one wave
 * per row), bit for bit. Replaces the backward aggregation of the top layer (custom_sparse_ops.py:
 * 33-37, A.t().coalesce() @ G, and GraphSAGE's x[sampled] gradient scatter) when Aᵀ's rows are
 * short: the 35 MB gradient is never written nor read back. G and R: 16-byte aligned rows of at
 * least D floats. */
int gnn_sage_norm_bwd_agg_f32(const int32_t* t_rowptr, const int32_t* t_col, const float* t_val, const float* G,
                              int64_t ldG, const float* R, int64_t ldr, const int32_t* rmap, const float* hB,
                              int64_t ldb, int64_t D1, const float* hW, int64_t ldw, int64_t D2, const float* biasB,
                              const float* biasW, const float* scale, const float* mean, const float* rstd, int64_t M,
                              float p_drop, uint64_t seed, int training, float* dhB, float* dhW, float* dscale,
                              float* doffset, float* dbiasB, float* dbiasW, void* workspace, size_t workspace_bytes,
                              void* stream);

/* ---------------------------------------------------------------------------------
 * fp32 GEMMs of the layers on gfx950 MFMA (gemm.hip): C[b] = A[b] · B[b] for b < nbatch
 * (1..4 problems of one shape in one launch; A, B, C are HOST arrays of device pointers).
 *   A(m, k) = a_kmajor ? A[k*lda + m] : A[m*lda + k]      (M x K)
 *   B(k, n) = b_kmajor ? B[k*ldb + n] : B[n*ldb + k]      (K x N)
 *   C(m, n) = C[m*ldc + n]                                 (M x N, row-major)
 * Replaces the torch.nn.Linear products of GraphSageConvolution / GraphConvolution
 * (models.py:18-21, 58-61) and their backward: forward X·Wᵀ (0, 0), input gradient G·W
 * (0, 1), weight gradient Gᵀ·X (1, 1). Exact fp32 (each output a k-ordered fmaf chain per
 * k-split; splits added in order: deterministic). lda, ldb even and A, B 8-byte aligned
 * (16-byte loads when lda/ldb are multiples of 4 and the pointers 16-byte aligned). When gnn_gemm_f32_workspace_bytes(M, N, K, nbatch) > 0 the k dimension is split
 * and `workspace` must hold that many bytes of device memory.
 * ------------------------------------------------------------------------------- */
size_t gnn_gemm_f32_workspace_bytes(int64_t M, int64_t N, int64_t K, int nbatch);
int gnn_gemm_f32(int a_kmajor, int b_kmajor, int64_t M, int64_t N, int64_t K, int nbatch, const float* const* A,
                 int64_t lda, const float* const* B, int64_t ldb, float* const* C, int64_t ldc, void* workspace,
                 size_t workspace_bytes, void* stream);

/* The same contract on the bf16 matrix cores ("split3", gemm.hip): every fp32 operand is cut
 * EXACTLY into three bf16 pieces by truncation (x = h + m + l) and each output accumulates in
 * fp32 the six largest piece products h·h + h·m + m·h + h·l + m·m + l·h per k (each exact in
 * fp32); the dropped products are below 3·2^-24·|a||b|, i.e. fp32-level accuracy (bounded
 * against fp64 by the same tolerance as gnn_gemm_f32 in tests/test_gemm_gpu.py), at 2.67x the
 * f32-input matrix rate. Deterministic (fixed accumulation order, k-splits added in order). */
size_t gnn_gemm_f32_split3_workspace_bytes(int64_t M, int64_t N, int64_t K, int nbatch);
int gnn_gemm_f32_split3(int a_kmajor, int b_kmajor, int64_t M, int64_t N, int64_t K, int nbatch,
                        const float* const* A, int64_t lda, const float* const* B, int64_t ldb, float* const* C,
                        int64_t ldc, void* workspace, size_t workspace_bytes, void* stream);

/* gnn_gemm_f32_split3 with row-indexed operands: row m of an m-major A is A[ia[b][m]] (a_rows
 * source rows), row k of a k-major B is B[ib[b][k]] (b_rows source rows); ia / ib or entries NULL
 * = not indexed (an indexed k-major A or m-major B is rejected). Bit-identical to the split3
 * product of the gathered operands — GraphSAGE's x[sampled] (models.py:18-21) read in place. */
int gnn_gemm_f32_split3_indexed(int a_kmajor, int b_kmajor, int64_t M, int64_t N, int64_t K, int nbatch,
                                const float* const* A, int64_t lda, const int64_t* const* ia, int64_t a_rows,
                                const float* const* B, int64_t ldb, const int64_t* const* ib, int64_t b_rows,
                                float* const* C, int64_t ldc, void* workspace, size_t workspace_bytes, void* stream);

/* split3 over operands split ONCE into their three bf16 pieces ("p3"): gnn_gemm_p3_pack_f32 writes
 * an operand viewed as R rows (M for A, N for B) by K — element (r, k) = src[row(r)*ld + k]
 * (kmajor = 0) or src[row(k)*ld + r] (kmajor = 1), row() through idx when given — as three
 * zero-padded planes [piece][k tile of 16][R rounded up to 128][16] bf16
 * (gnn_gemm_p3_packed_bytes(R, K) bytes, 16-byte aligned); gnn_gemm_p3 then computes
 * C[b] (M x N, row stride ldc) = A[b] · B[b]ᵀ-as-packed with the split3 kernel's tile, k steps
 * and MFMA order: bit-identical to gnn_gemm_f32_split3 on the same operands for shapes without
 * split3's tail tiles (gnn_gemm_f32_split3 sums the last 1-32 tiles past a multiple of 256 as k
 * pieces when GNN_GEMM_TAIL is on; p3 has no tail mode — equal there with GNN_GEMM_TAIL=0). */
size_t gnn_gemm_p3_packed_bytes(int64_t R, int64_t K);
int gnn_gemm_p3_pack_f32(const float* src, int64_t ld, int kmajor, const int64_t* idx, int64_t R, int64_t K,
                         void* out, size_t out_bytes, void* stream);
size_t gnn_gemm_p3_workspace_bytes(int64_t M, int64_t N, int64_t K, int nbatch);
int gnn_gemm_p3(int64_t M, int64_t N, int64_t K, int nbatch, const void* const* Ap, const void* const* Bp,
                float* const* C, int64_t ldc, void* workspace, size_t workspace_bytes, void* stream);

/* ---------------------------------------------------------------------------------
 * Classifier head + loss (head.hip). Replaces GNN.forward's tail (models.py:90-97:
 * F.normalize(x, 2, 1) -> dropout(p) -> nn.Linear(D, C)) and utils.loss with sigmoid_loss
 * (utils.py:129-140: BCEWithLogitsLoss(weight = 1/M per row, reduction "sum")):
 *   xd = dropout(x / max(||x||, 1e-12))  -> stored M x D (row stride D) for dW = dzᵀ·xd
 *   z  = xd·Wᵀ + bias                    -> stored M x C (logits)
 *   *loss = Σ_rows Σ_j (max(z,0) - z y + log1p(exp(-|z|))) / M   (rows summed in fixed order)
 * norm[M] = ||x|| per row, rowloss[M] = the per-row terms (workspace). W is C x D row-major
 * (nn.Linear.weight), labels M x C with row stride ldl; bias may be NULL. D % 4 == 0,
 * D <= 2048, C <= 256; X, W, xd 16-byte aligned. Dropout: the counter hash of (seed, r*D+c)
 * (as gnn_sage_norm_*), training = 0 or p = 0 disables it.
 * Backward: dz = (*grad_loss) (sigmoid(z) - y) / M (M x C, written for dW / db), and
 * dX = d/dx of the normalisation applied to mask · (dz·W). grad_loss may be NULL (1).
 * ------------------------------------------------------------------------------- */
int gnn_head_bce_fwd_f32(const float* X, int64_t ldx, int64_t M, int64_t D, const float* W, const float* bias,
                         int64_t C, const float* labels, int64_t ldl, float p, uint64_t seed, int training,
                         float* xd, float* z, float* norm, float* rowloss, float* loss, void* stream);
int gnn_head_bce_bwd_f32(const float* X, int64_t ldx, int64_t M, int64_t D, const float* W, int64_t C,
                         const float* labels, int64_t ldl, const float* grad_loss, float p, uint64_t seed,
                         int training, const float* z, const float* norm, float* dz, float* dX, int64_t lddx,
                         void* stream);

#ifdef __cplusplus
}
#endif

#endif /* GNN_LAYERS_H */
