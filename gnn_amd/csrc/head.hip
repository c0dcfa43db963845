// head.hip — the classifier head and its loss as one row pass each way (gnn_layers.h).
//
// Reference: GNN.forward's tail (models.py:90-97): F.normalize(x, p=2, dim=1) -> dropout ->
// nn.Linear(nhid, num_classes), then utils.loss (utils.py:129-140):
// BCEWithLogitsLoss(weight = 1/batch per row, reduction = "sum"). In torch that is ~12
// launches forward and ~14 backward for a 512 x 1024 input. Here four waves share a row: the
// row norm by shuffles + LDS, the inverted-dropout mask from a counter hash (regenerated in the
// backward, nothing stored), the C <= 256 logits as wave dot products against W (L2-resident:
// 168 KB for 41 classes x 1024, 704 KB for ogbn-papers' 172), and the per-row loss; a one-workgroup launch adds the rows in a fixed order. The
// backward recomputes the normalised row, forms dz = w (sigmoid(z) - y), back-projects it
// through W and the normalisation; dW = dzᵀ·xd and db = Σ dz are a small GEMM + sum.
#include <hip/hip_runtime.h>

#include <climits>
#include <cstdint>

#include "common.h"
#include "gnn_layers.h"

namespace {

using gnn::ceil_div;

typedef float f4 __attribute__((ext_vector_type(4)));

constexpr int HEAD_MAXC = 256;  // classes: lane j holds classes j, j + 64, j + 128, j + 192
constexpr int HEAD_CQ = HEAD_MAXC / 64;
constexpr int HEAD_MAXV = 8;    // 4-float pieces per lane: D <= 64 * 4 * 8 = 2048

__device__ __forceinline__ float wave_sum(float x) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) x += __shfl_xor(x, m);
  return x;
}

__device__ __forceinline__ uint32_t mix32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  x *= 0x846ca68bu;
  x ^= x >> 16;
  return x;
}

__device__ __forceinline__ bool keep_elem(uint64_t seed, uint64_t idx, float p) {
  const uint32_t h = mix32((uint32_t)idx ^ mix32((uint32_t)(idx >> 32) ^ mix32((uint32_t)seed ^ 0x9e3779b9u) ^
                                                 (uint32_t)(seed >> 32)));
  return (float)(h >> 8) * (1.0f / 16777216.0f) >= p;
}

// dropout multiplier of element (r, c): 0 or 1 / (1 - p) (training), 1 otherwise
__device__ __forceinline__ float drop_mult(uint64_t seed, int64_t r, int64_t D, int c, float p, bool training,
                                           float inv_keep) {
  if (!training) return 1.0f;
  return keep_elem(seed, (uint64_t)(r * D + c), p) ? inv_keep : 0.0f;
}

// Four waves per row: wave w holds the row's 4-float pieces t = w, w + 4, ... (one per lane
// for D = 1024), so a 512-row batch runs 2048 waves; the per-class partial dot products and
// the partial sums of squares meet in LDS.
constexpr int WPR = 4;
constexpr int CB = 8;  // classes per block: 8 rows of W in flight, 8 reductions interleaved

// PV = 4-float pieces per lane (1: D <= 1024, 2: D <= 2048)
template <int PV>
__device__ __forceinline__ void load_w_block(f4 (&wv)[CB][PV], const float* __restrict__ W, int j0, int C, int D,
                                             int w, int lane) {
#pragma unroll
  for (int u = 0; u < CB; ++u)
#pragma unroll
    for (int i = 0; i < PV; ++i) {
      const int c = ((w + i * WPR) * 64 + lane) * 4;
      wv[u][i] = (j0 + u < C && c < D) ? *reinterpret_cast<const f4*>(W + (int64_t)(j0 + u) * D + c) : f4(0.0f);
    }
}

template <int PV>
__global__ __launch_bounds__(256) void head_fwd_kernel(const float* __restrict__ X, int64_t ldx, int M, int D,
                                                       const float* __restrict__ W, const float* __restrict__ bias,
                                                       int C, const float* __restrict__ Y, int64_t ldy_lab,
                                                       float row_weight, float p, uint64_t seed, int training,
                                                       float* __restrict__ XD, float* __restrict__ Z,
                                                       float* __restrict__ nrm, float* __restrict__ rowloss) {
  __shared__ float part[WPR][HEAD_MAXC + 1];  // [w][j] class partials, [w][HEAD_MAXC] sum of squares
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int r = blockIdx.x;
  const float inv_keep = 1.0f / (1.0f - p);
  const bool tr = training != 0 && p > 0.0f;
  f4 x[PV];
  float ss = 0.0f;
#pragma unroll
  for (int i = 0; i < PV; ++i) {
    const int c = ((w + i * WPR) * 64 + lane) * 4;
    x[i] = f4(0.0f);
    if (c < D) {
      x[i] = *reinterpret_cast<const f4*>(X + (int64_t)r * ldx + c);
      ss += x[i].x * x[i].x + x[i].y * x[i].y + x[i].z * x[i].z + x[i].w * x[i].w;
    }
  }
  ss = wave_sum(ss);
  if (lane == 0) part[w][HEAD_MAXC] = ss;
  __syncthreads();
  const float norm = sqrtf((part[0][HEAD_MAXC] + part[1][HEAD_MAXC]) + (part[2][HEAD_MAXC] + part[3][HEAD_MAXC]));
  const float inv = 1.0f / fmaxf(norm, 1e-12f);  // F.normalize: x / max(||x||, eps)
#pragma unroll
  for (int i = 0; i < PV; ++i) {
    const int c = ((w + i * WPR) * 64 + lane) * 4;
    if (c < D) {
      f4 v = x[i] * inv;
      v.x *= drop_mult(seed, r, D, c + 0, p, tr, inv_keep);
      v.y *= drop_mult(seed, r, D, c + 1, p, tr, inv_keep);
      v.z *= drop_mult(seed, r, D, c + 2, p, tr, inv_keep);
      v.w *= drop_mult(seed, r, D, c + 3, p, tr, inv_keep);
      x[i] = v;
      *reinterpret_cast<f4*>(XD + (int64_t)r * D + c) = v;
    }
  }
  // software-pipelined over blocks of 8 classes: the next block's W loads are in flight while
  // this block is reduced
  f4 wn[CB][PV];
  load_w_block<PV>(wn, W, 0, C, D, w, lane);
  for (int j0 = 0; j0 < C; j0 += CB) {
    f4 wc[CB][PV];
#pragma unroll
    for (int u = 0; u < CB; ++u)
#pragma unroll
      for (int i = 0; i < PV; ++i) wc[u][i] = wn[u][i];
    if (j0 + CB < C) load_w_block<PV>(wn, W, j0 + CB, C, D, w, lane);
    float s[CB];
#pragma unroll
    for (int u = 0; u < CB; ++u) {
      s[u] = 0.0f;
#pragma unroll
      for (int i = 0; i < PV; ++i)
        s[u] += wc[u][i].x * x[i].x + wc[u][i].y * x[i].y + wc[u][i].z * x[i].z + wc[u][i].w * x[i].w;
    }
    // reduce-scatter over the wave: 4 + 2 + 1 exchanges halve the class set per step, then
    // 3 more finish the sums; lane 8u ends with class j0 + u (10 shuffles for 8 classes, not 48)
    float t4[4], t2[2];
    const bool h32 = lane & 32, h16 = lane & 16, h8 = lane & 8;
#pragma unroll
    for (int u = 0; u < 4; ++u) t4[u] = (h32 ? s[u + 4] : s[u]) + __shfl_xor(h32 ? s[u] : s[u + 4], 32);
#pragma unroll
    for (int u = 0; u < 2; ++u) t2[u] = (h16 ? t4[u + 2] : t4[u]) + __shfl_xor(h16 ? t4[u] : t4[u + 2], 16);
    float t1 = (h8 ? t2[1] : t2[0]) + __shfl_xor(h8 ? t2[0] : t2[1], 8);
    t1 += __shfl_xor(t1, 4);
    t1 += __shfl_xor(t1, 2);
    t1 += __shfl_xor(t1, 1);
    if ((lane & 7) == 0 && j0 + (lane >> 3) < C) part[w][j0 + (lane >> 3)] = t1;
  }
  __syncthreads();
  if (w != 0) return;
  // lane j: logits j, j + 64, ... and their BCE terms
  float term = 0.0f;
#pragma unroll
  for (int q = 0; q < HEAD_CQ; ++q) {
    const int j = lane + 64 * q;
    if (j < C) {
      const float z = ((part[0][j] + part[1][j]) + (part[2][j] + part[3][j])) + (bias ? bias[j] : 0.0f);
      Z[(int64_t)r * C + j] = z;
      const float y = Y[(int64_t)r * ldy_lab + j];
      // BCE with logits, stable form: max(z, 0) - z y + log1p(exp(-|z|))
      term += fmaxf(z, 0.0f) - z * y + log1pf(expf(-fabsf(z)));
    }
  }
  const float loss = wave_sum(term);
  if (lane == 0) {
    nrm[r] = norm;
    rowloss[r] = loss * row_weight;
  }
}

__global__ __launch_bounds__(256) void head_loss_sum_kernel(const float* __restrict__ rowloss, int M,
                                                            float* __restrict__ out) {
  __shared__ float red[4];
  float s = 0.0f;
  for (int i = threadIdx.x; i < M; i += 256) s += rowloss[i];
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) *out = (red[0] + red[1]) + (red[2] + red[3]);
}

template <int PV>
__global__ __launch_bounds__(256) void head_bwd_kernel(const float* __restrict__ X, int64_t ldx, int M, int D,
                                                       const float* __restrict__ W, int C,
                                                       const float* __restrict__ Y, int64_t ldy_lab,
                                                       float row_weight, const float* __restrict__ gloss, float p,
                                                       uint64_t seed, int training, const float* __restrict__ Z,
                                                       const float* __restrict__ nrm, float* __restrict__ DZ,
                                                       float* __restrict__ DX, int64_t lddx) {
  __shared__ float dots[WPR];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int r = blockIdx.x;
  const float inv_keep = 1.0f / (1.0f - p);
  const bool tr = training != 0 && p > 0.0f;
  const float g = gloss ? *gloss : 1.0f;
  // dz_j = g * w * (sigmoid(z_j) - y_j), classes lane + 64 q per lane, in every wave
  float dz[HEAD_CQ];
#pragma unroll
  for (int q = 0; q < HEAD_CQ; ++q) {
    const int j = lane + 64 * q;
    dz[q] = 0.0f;
    if (j < C) {
      const float z = Z[(int64_t)r * C + j];
      const float sg = 1.0f / (1.0f + expf(-z));
      dz[q] = g * row_weight * (sg - Y[(int64_t)r * ldy_lab + j]);
      if (w == 0) DZ[(int64_t)r * C + j] = dz[q];
    }
  }
  // this wave's pieces of dxd = Wᵀ dz, then through dropout and the normalisation
  f4 dxd[PV], xn[PV];
#pragma unroll
  for (int i = 0; i < PV; ++i) dxd[i] = f4(0.0f);
  f4 wn[CB][PV];
  load_w_block<PV>(wn, W, 0, C, D, w, lane);
  for (int j0 = 0; j0 < C; j0 += CB) {
    f4 wc[CB][PV];
#pragma unroll
    for (int u = 0; u < CB; ++u)
#pragma unroll
      for (int i = 0; i < PV; ++i) wc[u][i] = wn[u][i];
    if (j0 + CB < C) load_w_block<PV>(wn, W, j0 + CB, C, D, w, lane);
    const int qb = j0 >> 6;  // a block of CB classes lies in one 64-class slot
    const float dzq = qb == 0 ? dz[0] : qb == 1 ? dz[1] : qb == 2 ? dz[2] : dz[3];
#pragma unroll
    for (int u = 0; u < CB; ++u) {
      const float dzj = __shfl(dzq, (j0 + u) & 63);  // classes >= C hold 0
#pragma unroll
      for (int i = 0; i < PV; ++i) dxd[i] += dzj * wc[u][i];
    }
  }
  const float norm = nrm[r];
  const float inv = 1.0f / fmaxf(norm, 1e-12f);
  float dot = 0.0f;
#pragma unroll
  for (int i = 0; i < PV; ++i) {
    const int c = ((w + i * WPR) * 64 + lane) * 4;
    xn[i] = f4(0.0f);
    if (c < D) {
      xn[i] = *reinterpret_cast<const f4*>(X + (int64_t)r * ldx + c) * inv;
      f4 d = dxd[i];
      d.x *= drop_mult(seed, r, D, c + 0, p, tr, inv_keep);
      d.y *= drop_mult(seed, r, D, c + 1, p, tr, inv_keep);
      d.z *= drop_mult(seed, r, D, c + 2, p, tr, inv_keep);
      d.w *= drop_mult(seed, r, D, c + 3, p, tr, inv_keep);
      dxd[i] = d;  // now d(xn)
      dot += d.x * xn[i].x + d.y * xn[i].y + d.z * xn[i].z + d.w * xn[i].w;
    }
  }
  dot = wave_sum(dot);
  if (lane == 0) dots[w] = dot;
  __syncthreads();
  dot = (dots[0] + dots[1]) + (dots[2] + dots[3]);
  const bool clamped = !(norm > 1e-12f);  // below eps the denominator is the constant eps
#pragma unroll
  for (int i = 0; i < PV; ++i) {
    const int c = ((w + i * WPR) * 64 + lane) * 4;
    if (c < D) {
      const f4 dx = clamped ? dxd[i] * inv : (dxd[i] - xn[i] * dot) * inv;
      *reinterpret_cast<f4*>(DX + (int64_t)r * lddx + c) = dx;
    }
  }
}

}  // namespace

extern "C" {

int gnn_head_bce_fwd_f32(const float* X, int64_t ldx, int64_t M, int64_t D, const float* W, const float* bias,
                         int64_t C, const float* labels, int64_t ldl, float p, uint64_t seed, int training,
                         float* xd, float* z, float* norm, float* rowloss, float* loss, void* stream) {
  GNN_REQUIRE(M >= 0 && D > 0 && C > 0, "gnn_head_bce_fwd_f32: bad sizes");
  GNN_REQUIRE(D % 4 == 0 && D <= 64 * 4 * HEAD_MAXV, "gnn_head_bce_fwd_f32: D must be a multiple of 4, <= %d",
              64 * 4 * HEAD_MAXV);
  GNN_REQUIRE(C <= HEAD_MAXC, "gnn_head_bce_fwd_f32: at most %d classes", HEAD_MAXC);
  GNN_REQUIRE(ldx % 4 == 0 && (uintptr_t)X % 16 == 0 && (uintptr_t)W % 16 == 0 && (uintptr_t)xd % 16 == 0,
              "gnn_head_bce_fwd_f32: X, W, xd must be 16-byte aligned with ldx % 4 == 0");
  GNN_REQUIRE(M < INT_MAX && p >= 0.0f && p < 1.0f, "gnn_head_bce_fwd_f32: bad M or p");
  GNN_REQUIRE(loss && rowloss && z && norm && labels, "gnn_head_bce_fwd_f32: NULL output");
  hipStream_t st = (hipStream_t)stream;
  if (M > 0) {
    auto k = D <= 64 * 4 * WPR ? head_fwd_kernel<1> : head_fwd_kernel<2>;
    k<<<dim3((unsigned)M), dim3(64 * WPR), 0, st>>>(X, ldx, (int)M, (int)D, W, bias, (int)C, labels, ldl,
                                                    1.0f / (float)M, p, seed, training, xd, z, norm, rowloss);
    GNN_LAUNCHED("head_fwd_kernel");
  }
  head_loss_sum_kernel<<<dim3(1), dim3(256), 0, st>>>(rowloss, (int)M, loss);
  GNN_LAUNCHED("head_loss_sum_kernel");
  return 0;
}

int gnn_head_bce_bwd_f32(const float* X, int64_t ldx, int64_t M, int64_t D, const float* W, int64_t C,
                         const float* labels, int64_t ldl, const float* grad_loss, float p, uint64_t seed,
                         int training, const float* z, const float* norm, float* dz, float* dX, int64_t lddx,
                         void* stream) {
  GNN_REQUIRE(M >= 0 && D > 0 && C > 0 && C <= HEAD_MAXC && D % 4 == 0 && D <= 64 * 4 * HEAD_MAXV,
              "gnn_head_bce_bwd_f32: bad sizes");
  GNN_REQUIRE(lddx % 4 == 0 && (uintptr_t)dX % 16 == 0 && ldx % 4 == 0 && (uintptr_t)X % 16 == 0,
              "gnn_head_bce_bwd_f32: X / dX must be 16-byte aligned");
  if (M == 0) return 0;
  auto k = D <= 64 * 4 * WPR ? head_bwd_kernel<1> : head_bwd_kernel<2>;
  k<<<dim3((unsigned)M), dim3(64 * WPR), 0, (hipStream_t)stream>>>(
      X, ldx, (int)M, (int)D, W, (int)C, labels, ldl, 1.0f / (float)M, grad_loss, p, seed, training, z, norm, dz,
      dX, lddx);
  GNN_LAUNCHED("head_bwd_kernel");
  return 0;
}

}  // extern "C"
