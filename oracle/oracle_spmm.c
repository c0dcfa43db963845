/*
 * oracle_spmm.c — TEST INFRASTRUCTURE ONLY (CPU restatement of the reference's SpMM path).
 *
 * Used exclusively by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg as
 * the checker. Never linked into, called by, or shipped as part of the gnn_amd product.
 *
 * Parity anchor: the reference's executable SpMM is CUDA-only (spmm_cpp/cuda_spmm.cu) and
 * cannot run here; its CPU path is torch.sparse.mm (custom_sparse_ops.py:25,36, commented
 * out upstream). These functions restate the math and are pinned against golden vectors
 * captured from the reference's Python (tests/golden/make_golden.py, torch.sparse.mm).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

/* Operand builder, restating _create_coo_tensor_kernel (cuda_spmm.cu:795-802):
 *   value[i] = 1. / (fullrowptr[r+1] - fullrowptr[r]) * normfact[colidx[i]]
 * evaluated in double and stored as float; then .coalesce() (cuda_spmm.cu:825) orders the
 * entries of each row by column: a stable insertion sort here. */
void oracle_build_operand(const int32_t* fullrowptr, const int32_t* rowptr, const int32_t* colidx,
                          const float* normfact, int64_t nrows, int32_t* out_col, float* out_val) {
  for (int64_t r = 0; r < nrows; ++r) {
    const int32_t b = rowptr[r], e = rowptr[r + 1];
    const double inv = 1. / (double)(fullrowptr[r + 1] - fullrowptr[r]);
    for (int32_t i = b; i < e; ++i) {
      out_col[i] = colidx[i];
      out_val[i] = (float)(inv * (double)normfact[colidx[i]]);
    }
    for (int32_t i = b + 1; i < e; ++i) {
      const int32_t c = out_col[i];
      const float v = out_val[i];
      int32_t j = i - 1;
      while (j >= b && out_col[j] > c) {
        out_col[j + 1] = out_col[j];
        out_val[j + 1] = out_val[j];
        --j;
      }
      out_col[j + 1] = c;
      out_val[j + 1] = v;
    }
  }
}

/* Y = A·X, fp32, one fused multiply-add per nonzero in CSR order (the order in which a
 * single work unit of the HIP kernel accumulates a row). */
void oracle_spmm_csr_f32(const int32_t* rowptr, const int32_t* col, const float* val, int64_t M,
                         const float* X, int64_t ldx, int64_t F, float* Y, int64_t ldy) {
  for (int64_t r = 0; r < M; ++r) {
    float* y = Y + r * ldy;
    for (int64_t c = 0; c < F; ++c) y[c] = 0.0f;
    for (int32_t i = rowptr[r]; i < rowptr[r + 1]; ++i) {
      const float v = val[i];
      const float* x = X + (int64_t)col[i] * ldx;
      for (int64_t c = 0; c < F; ++c) y[c] = fmaf(v, x[c], y[c]);
    }
  }
}

/* Same product accumulated in double (error reference): Y64 = A·X exactly rounded once. */
void oracle_spmm_csr_f64(const int32_t* rowptr, const int32_t* col, const float* val, int64_t M,
                         const float* X, int64_t ldx, int64_t F, double* Y, int64_t ldy) {
  for (int64_t r = 0; r < M; ++r) {
    double* y = Y + r * ldy;
    for (int64_t c = 0; c < F; ++c) y[c] = 0.0;
    for (int32_t i = rowptr[r]; i < rowptr[r + 1]; ++i) {
      const double v = (double)val[i];
      const float* x = X + (int64_t)col[i] * ldx;
      for (int64_t c = 0; c < F; ++c) y[c] += v * (double)x[c];
    }
  }
}

/* Sum over rows of |a|·|x| per output element — the scale for a relative error bound. */
void oracle_spmm_abs_f64(const int32_t* rowptr, const int32_t* col, const float* val, int64_t M,
                         const float* X, int64_t ldx, int64_t F, double* Y, int64_t ldy) {
  for (int64_t r = 0; r < M; ++r) {
    double* y = Y + r * ldy;
    for (int64_t c = 0; c < F; ++c) y[c] = 0.0;
    for (int32_t i = rowptr[r]; i < rowptr[r + 1]; ++i) {
      const double v = fabs((double)val[i]);
      const float* x = X + (int64_t)col[i] * ldx;
      for (int64_t c = 0; c < F; ++c) y[c] += v * fabs((double)x[c]);
    }
  }
}

/* Canonical transpose, i.e. A.transpose(0,1).coalesce() of custom_sparse_ops.py:34:
 * counting sort by column, rows visited in ascending order (stable). */
void oracle_csr_transpose(const int32_t* rowptr, const int32_t* col, const float* val, int64_t M, int64_t K,
                          int32_t* tr_rowptr, int32_t* tr_col, float* tr_val) {
  memset(tr_rowptr, 0, (size_t)(K + 1) * sizeof(int32_t));
  const int32_t nnz = rowptr[M];
  for (int32_t i = 0; i < nnz; ++i) tr_rowptr[col[i] + 1]++;
  for (int64_t c = 0; c < K; ++c) tr_rowptr[c + 1] += tr_rowptr[c];
  int32_t* cur = (int32_t*)malloc((size_t)(K > 0 ? K : 1) * sizeof(int32_t));
  memcpy(cur, tr_rowptr, (size_t)K * sizeof(int32_t));
  for (int64_t r = 0; r < M; ++r) {
    for (int32_t i = rowptr[r]; i < rowptr[r + 1]; ++i) {
      const int32_t p = cur[col[i]]++;
      tr_col[p] = (int32_t)r;
      tr_val[p] = val[i];
    }
  }
  free(cur);
}

/* Row gather of the feature staging (main.py:129-134): dst[dst_idx[i]] = src[src_idx[i]]. */
void oracle_gather_rows(const float* src, int64_t ld_src, const int64_t* src_idx, float* dst, int64_t ld_dst,
                        const int64_t* dst_idx, int64_t n, int64_t F) {
  for (int64_t i = 0; i < n; ++i) {
    const int64_t s = src_idx ? src_idx[i] : i;
    const int64_t d = dst_idx ? dst_idx[i] : i;
    memcpy(dst + d * ld_dst, src + s * ld_src, (size_t)F * sizeof(float));
  }
}
