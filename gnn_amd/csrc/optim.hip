// optim.hip — the training step's tail in three launches: global gradient-norm clipping and
// Adam, over all parameter tensors at once (multi-tensor: one workgroup per 1K-element chunk
// of any tensor, the tensor list passed by value in the kernel arguments).
//
// Reference (main.py:146-170): clip_grad_norm_(params, 5) on each rank's gradients, the
// per-rank sum of the clipped gradients, then torch.optim.Adam (lr, betas (0.9, 0.999),
// eps 1e-8, no weight decay). torch runs the clip as ~6 launches (per-tensor norms, stack,
// norm, clamp, scale) and Adam as a multi-tensor kernel that moves the 4 state streams at
// ~1.6 TB/s; here: a partial-sum-of-squares launch, a one-workgroup launch that turns the
// partials into the clip factor (fixed-order sum: deterministic), and one Adam launch that
// applies the factor to the gradient as it reads it.
#include <hip/hip_runtime.h>

#include <climits>
#include <cmath>
#include <cstdint>

#include "common.h"
#include "gnn_optim.h"

namespace {

using gnn::ceil_div;

constexpr int MAXT = GNN_OPTIM_MAX_TENSORS;
constexpr int CHUNK = 1024;  // elements per workgroup: 4 per thread, enough workgroups to fill the chip

struct TensorList {
  float* p[MAXT];
  const float* g[MAXT];
  float* m[MAXT];
  float* v[MAXT];
  int64_t n[MAXT];
  int64_t chunk0[MAXT + 1];  // first chunk of tensor i (exclusive prefix of ceil(n / CHUNK))
  int count;
};

typedef float f4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ bool aligned16(const void* q) { return ((uintptr_t)q & 15u) == 0; }

__device__ __forceinline__ int tensor_of(const TensorList& L, int64_t chunk) {
  int i = 0;
  while (i + 1 < L.count && L.chunk0[i + 1] <= chunk) ++i;  // <= 32 entries, uniform
  return i;
}

__device__ __forceinline__ float block_sum(float s, float* red) {
  for (int o = 32; o >= 1; o >>= 1) s += __shfl_xor(s, o);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (lane == 0) red[w] = s;
  __syncthreads();
  float t = 0.0f;
  if (threadIdx.x == 0) t = (red[0] + red[1]) + (red[2] + red[3]);  // fixed order
  return t;
}

// partial[chunk] = sum of squares of the gradient elements of that chunk
__global__ __launch_bounds__(256) void grad_sqnorm_kernel(TensorList L, float* __restrict__ partial) {
  __shared__ float red[4];
  const int64_t chunk = blockIdx.x;
  const int i = tensor_of(L, chunk);
  const int64_t base = (chunk - L.chunk0[i]) * CHUNK;
  const int64_t end = min(base + (int64_t)CHUNK, L.n[i]);
  const float* g = L.g[i];
  float s = 0.0f;
  if (end - base == CHUNK && aligned16(g + base)) {  // full chunk: one float4 per thread
    const f4 x = reinterpret_cast<const f4*>(g + base)[threadIdx.x];
    s = fmaf(x.w, x.w, fmaf(x.z, x.z, fmaf(x.y, x.y, x.x * x.x)));
  } else {
    for (int64_t e = base + threadIdx.x; e < end; e += 256) {
      const float x = g[e];
      s = fmaf(x, x, s);
    }
  }
  const float t = block_sum(s, red);
  if (threadIdx.x == 0) partial[chunk] = t;
}

// scale = min(1, max_norm / (sqrt(sum partial) + 1e-6)) (torch: clip_coef clamped to 1), one
// workgroup, partials summed in a fixed order.
__global__ __launch_bounds__(256) void clip_scale_kernel(const float* __restrict__ partial, int64_t nchunks,
                                                         float max_norm, float* __restrict__ scale) {
  __shared__ float red[4];
  float s = 0.0f;
  for (int64_t c = threadIdx.x; c < nchunks; c += 256) s += partial[c];
  const float t = block_sum(s, red);
  if (threadIdx.x == 0) {
    const float coef = max_norm / (sqrtf(t) + 1e-6f);
    *scale = coef < 1.0f ? coef : 1.0f;
  }
}

__global__ __launch_bounds__(256) void scale_into_kernel(TensorList L, const float* __restrict__ scale,
                                                         float* __restrict__ flat) {
  const float sc = scale ? *scale : 1.0f;
  const int64_t chunk = blockIdx.x;
  const int i = tensor_of(L, chunk);
  const int64_t base = (chunk - L.chunk0[i]) * CHUNK;
  const int64_t end = min(base + (int64_t)CHUNK, L.n[i]);
  // flat offset of tensor i = sum of the sizes before it (its views in the flat buffer)
  int64_t off = 0;
  for (int j = 0; j < i; ++j) off += L.n[j];
  for (int64_t e = base + threadIdx.x; e < end; e += 256) flat[off + e] = L.g[i][e] * sc;
}

__global__ __launch_bounds__(256) void adam_kernel(TensorList L, const float* __restrict__ scale, float beta1,
                                                   float beta2, float eps, float step_size, float bc2_sqrt) {
  const float sc = scale ? *scale : 1.0f;
  const int64_t chunk = blockIdx.x;
  const int i = tensor_of(L, chunk);
  const int64_t base = (chunk - L.chunk0[i]) * CHUNK;
  const int64_t end = min(base + (int64_t)CHUNK, L.n[i]);
  float* __restrict__ p = L.p[i];
  const float* __restrict__ g = L.g[i];
  float* __restrict__ m = L.m[i];
  float* __restrict__ v = L.v[i];
  // torch (_fused_adam / _multi_tensor_adam, amsgrad=False, weight_decay=0):
  //   m = lerp(m, g, 1 - beta1); v = beta2 * v + (1 - beta2) * g * g
  //   p -= (lr / bc1) * m / (sqrt(v) / sqrt(bc2) + eps)
  auto upd = [&](float gr, float mo, float vo, float po, float& mn, float& vn, float& pn) {
    mn = mo + (1.0f - beta1) * (gr - mo);
    vn = beta2 * vo + (1.0f - beta2) * gr * gr;
    const float denom = sqrtf(vn) / bc2_sqrt + eps;
    pn = po - step_size * (mn / denom);
  };
  if (end - base == CHUNK && aligned16(p + base) && aligned16(g + base) && aligned16(m + base) &&
      aligned16(v + base)) {  // full chunk: one float4 of each stream per thread (same per-element math)
    const int64_t e = base + 4 * threadIdx.x;
    const f4 g4 = *reinterpret_cast<const f4*>(g + e) * sc;
    const f4 m4 = *reinterpret_cast<const f4*>(m + e);
    const f4 v4 = *reinterpret_cast<const f4*>(v + e);
    const f4 p4 = *reinterpret_cast<const f4*>(p + e);
    float mn[4], vn[4], pn[4];
    upd(g4.x, m4.x, v4.x, p4.x, mn[0], vn[0], pn[0]);
    upd(g4.y, m4.y, v4.y, p4.y, mn[1], vn[1], pn[1]);
    upd(g4.z, m4.z, v4.z, p4.z, mn[2], vn[2], pn[2]);
    upd(g4.w, m4.w, v4.w, p4.w, mn[3], vn[3], pn[3]);
    *reinterpret_cast<f4*>(m + e) = f4{mn[0], mn[1], mn[2], mn[3]};
    *reinterpret_cast<f4*>(v + e) = f4{vn[0], vn[1], vn[2], vn[3]};
    *reinterpret_cast<f4*>(p + e) = f4{pn[0], pn[1], pn[2], pn[3]};
    return;
  }
  for (int64_t e = base + threadIdx.x; e < end; e += 256) {
    float mn, vn, pn;
    upd(g[e] * sc, m[e], v[e], p[e], mn, vn, pn);
    m[e] = mn;
    v[e] = vn;
    p[e] = pn;
  }
}

int fill_list(TensorList& L, int count, float* const* p, const float* const* g, float* const* m, float* const* v,
              const int64_t* n) {
  GNN_REQUIRE(count >= 1 && count <= MAXT, "optimizer: 1..%d tensors per call (got %d)", MAXT, count);
  L.count = count;
  L.chunk0[0] = 0;
  for (int i = 0; i < count; ++i) {
    GNN_REQUIRE(n[i] >= 0 && g[i] != nullptr, "optimizer: bad tensor %d", i);
    L.p[i] = p ? p[i] : nullptr;
    L.g[i] = g[i];
    L.m[i] = m ? m[i] : nullptr;
    L.v[i] = v ? v[i] : nullptr;
    L.n[i] = n[i];
    L.chunk0[i + 1] = L.chunk0[i] + ceil_div(n[i], (int64_t)CHUNK);
  }
  for (int i = count; i < MAXT; ++i) {
    L.p[i] = nullptr;
    L.g[i] = nullptr;
    L.m[i] = nullptr;
    L.v[i] = nullptr;
    L.n[i] = 0;
    L.chunk0[i + 1] = L.chunk0[count];
  }
  return 0;
}

}  // namespace

extern "C" {

int64_t gnn_optim_chunks(int count, const int64_t* n) {
  int64_t c = 0;
  for (int i = 0; i < count; ++i) c += ceil_div(n[i], (int64_t)CHUNK);
  return c;
}

int gnn_grad_sqnorm_f32(int count, const float* const* g, const int64_t* n, float* partial, void* stream) {
  TensorList L;
  if (int rc = fill_list(L, count, nullptr, g, nullptr, nullptr, n)) return rc;
  const int64_t nch = L.chunk0[count];
  GNN_REQUIRE(partial != nullptr || nch == 0, "gnn_grad_sqnorm_f32: NULL partial");
  if (nch == 0) return 0;
  GNN_REQUIRE(nch < INT_MAX, "gnn_grad_sqnorm_f32: too many chunks");
  grad_sqnorm_kernel<<<dim3((unsigned)nch), dim3(256), 0, (hipStream_t)stream>>>(L, partial);
  GNN_LAUNCHED("grad_sqnorm_kernel");
  return 0;
}

int gnn_clip_scale_f32(const float* partial, int64_t nchunks, float max_norm, float* scale, void* stream) {
  GNN_REQUIRE(scale != nullptr && (partial != nullptr || nchunks == 0), "gnn_clip_scale_f32: NULL argument");
  GNN_REQUIRE(max_norm > 0.0f, "gnn_clip_scale_f32: max_norm must be > 0");
  clip_scale_kernel<<<dim3(1), dim3(256), 0, (hipStream_t)stream>>>(partial, nchunks, max_norm, scale);
  GNN_LAUNCHED("clip_scale_kernel");
  return 0;
}

int gnn_scale_into_f32(int count, const float* const* g, const int64_t* n, const float* scale, float* flat,
                       void* stream) {
  TensorList L;
  if (int rc = fill_list(L, count, nullptr, g, nullptr, nullptr, n)) return rc;
  const int64_t nch = L.chunk0[count];
  if (nch == 0) return 0;
  GNN_REQUIRE(flat != nullptr, "gnn_scale_into_f32: NULL flat");
  GNN_REQUIRE(nch < INT_MAX, "gnn_scale_into_f32: too many chunks");
  scale_into_kernel<<<dim3((unsigned)nch), dim3(256), 0, (hipStream_t)stream>>>(L, scale, flat);
  GNN_LAUNCHED("scale_into_kernel");
  return 0;
}

int gnn_adam_f32(int count, float* const* p, const float* const* g, float* const* m, float* const* v,
                 const int64_t* n, const float* scale, float lr, float beta1, float beta2, float eps, int64_t step,
                 void* stream) {
  TensorList L;
  if (int rc = fill_list(L, count, p, g, m, v, n)) return rc;
  for (int i = 0; i < count; ++i) GNN_REQUIRE(p[i] && m[i] && v[i], "gnn_adam_f32: NULL tensor %d", i);
  GNN_REQUIRE(step >= 1, "gnn_adam_f32: step must be >= 1");
  const int64_t nch = L.chunk0[count];
  if (nch == 0) return 0;
  GNN_REQUIRE(nch < INT_MAX, "gnn_adam_f32: too many chunks");
  const double bc1 = 1.0 - std::pow((double)beta1, (double)step);
  const double bc2 = 1.0 - std::pow((double)beta2, (double)step);
  const float step_size = (float)(lr / bc1);
  const float bc2_sqrt = (float)std::sqrt(bc2);
  adam_kernel<<<dim3((unsigned)nch), dim3(256), 0, (hipStream_t)stream>>>(L, scale, beta1, beta2, eps, step_size,
                                                                         bc2_sqrt);
  GNN_LAUNCHED("adam_kernel");
  return 0;
}

}  // extern "C"
