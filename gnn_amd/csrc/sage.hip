// sage.hip — fused GraphSAGE / GCN layer epilogue (forward + backward), gfx950.
//
// Reference (models.py:16-25, 58-64, 43, 82): after the two linear layers, torch runs
// bias-add -> cat -> elu -> mean -> var -> sub -> mul(scale) -> rsqrt -> mul -> add(offset) ->
// dropout, each a separate pass over the (M x 1024) activation, and about twice as many
// passes in backward (plus one column-sum kernel per linear bias). Here one wave owns one
// row: the row (<= 2048 floats, <= 8 float4 per lane) is read once into registers, the
// linear biases added, ELU'd, reduced twice with wave shuffles (mean, then the centred
// second moment: the same two-pass variance torch computes), normalised, scaled, dropped
// out and stored once. Backward re-reads the bias-free linear outputs and the saved per-row
// mean and rstd, regenerates the dropout mask from its counter hash, and writes the two
// input gradients in one pass; d(scale), d(offset) and d(bias) are column sums reduced per
// workgroup into a slab and then summed over workgroups in a fixed order (deterministic).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>
#include <cstdint>
#include <cstdlib>

#include "common.h"
#include "gnn_layers.h"

namespace {

using gnn::ceil_div;
typedef float f4 __attribute__((ext_vector_type(4)));

constexpr int SN_MAXV = 8;   // float4 per lane: D <= 64 * 4 * 8 = 2048
constexpr int BWD_MAX_GRID = 768;  // 3 workgroups per CU (158 VGPRs at D = 1024): rows overlap their latencies

// backward grid cap (env GNN_SAGE_BWD_GRID overrides, for sweeps; the workspace is sized by
// the larger of the two)
int bwd_grid_cap() {
  static const int cap = [] {
    const char* e = std::getenv("GNN_SAGE_BWD_GRID");
    const int v = e ? std::atoi(e) : 0;
    return v > 0 && v <= 4096 ? v : BWD_MAX_GRID;
  }();
  return cap;
}
constexpr int NRED = 3;      // column sums: d(scale), d(offset), d(bias)

__device__ __forceinline__ float wave_sum(float x) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) x += __shfl_xor(x, m);
  return x;
}

__device__ __forceinline__ uint32_t mix32(uint32_t x) {  // "lowbias32" integer hash
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  x *= 0x846ca68bu;
  x ^= x >> 16;
  return x;
}

// Keep-mask of inverted dropout for element `idx` (row * D + col): P(keep) = 1 - p.
__device__ __forceinline__ bool keep_elem(uint64_t seed, uint64_t idx, float p) {
  const uint32_t h = mix32((uint32_t)idx ^ mix32((uint32_t)(idx >> 32) ^ mix32((uint32_t)seed ^ 0x9e3779b9u) ^
                                                 (uint32_t)(seed >> 32)));
  return (float)(h >> 8) * (1.0f / 16777216.0f) >= p;
}

// The same mask, computed per row: the inner hash of the element index's high word is the same
// for every element of a row (or takes two values when the row straddles a multiple of 2^32), so
// it is hashed twice per row instead of once per element, and the keep test is one integer
// compare against the threshold T << 8, T = ceil(p * 2^24) (x * 2^-24 >= p <=> x >= T for the
// integer x = h >> 8 < 2^24; T = 2^24, i.e. p >= 1, keeps nothing). Bit-identical to keep_elem.
__device__ __forceinline__ uint32_t drop_key(uint64_t seed) {
  return mix32((uint32_t)seed ^ 0x9e3779b9u) ^ (uint32_t)(seed >> 32);
}

struct DropThr {
  uint32_t thr;
  bool none;
};

__device__ __forceinline__ DropThr drop_thr(float p) {
  const float t = ceilf(p * 16777216.0f);
  if (!(t < 16777216.0f)) return DropThr{0u, true};
  return DropThr{t <= 0.0f ? 0u : ((uint32_t)t) << 8, false};
}

struct RowDrop {
  uint32_t lo0, in0, in1;
  __device__ __forceinline__ RowDrop(uint32_t key, uint64_t e0) : lo0((uint32_t)e0) {
    const uint32_t hi0 = (uint32_t)(e0 >> 32);
    in0 = mix32(hi0 ^ key);
    in1 = mix32((hi0 + 1u) ^ key);
  }
  // keep_elem(seed, e0 + off, p)
  __device__ __forceinline__ bool keep(uint32_t off, DropThr t) const {
    const uint32_t lo = lo0 + off;
    return !t.none && mix32(lo ^ (lo < lo0 ? in1 : in0)) >= t.thr;
  }
};

// expm1 evaluated for every element (of min(h, 0): the same value where it is kept) and then
// selected: as `h > 0 ? h : expm1f(h)` the compiler wraps each element's expm1f in an exec-masked
// branch (saveexec / cbranch / restore per element; 90 branches in the forward kernel against 62).
__device__ __forceinline__ float elu1(float h) {
  const float e = expm1f(fminf(h, 0.0f));
  return h > 0.0f ? h : e;
}
// d elu(h) / dh from the activation o = elu(h): 1 for h > 0 (o > 0), else exp(h) = o + 1
// (one rounding of expm1(h) + 1 instead of a second exponential).
__device__ __forceinline__ float elu1_grad_from_out(float o) { return o > 0.0f ? 1.0f : o + 1.0f; }

// Pre-activation of column c of row r: the linear output plus its bias (when given).
__device__ __forceinline__ f4 load_h(const float* hB, int64_t ldb, const float* bB, int D1, const float* hW,
                                     int64_t ldw, const float* bW, int r, int c) {
  if (c < D1) {
    f4 h = *reinterpret_cast<const f4*>(hB + (int64_t)r * ldb + c);
    if (bB) h += *reinterpret_cast<const f4*>(bB + c);
    return h;
  }
  f4 h = *reinterpret_cast<const f4*>(hW + (int64_t)r * ldw + (c - D1));
  if (bW) h += *reinterpret_cast<const f4*>(bW + (c - D1));
  return h;
}

// The output gradient of a row: a dense row of gY, or (AGG) computed on the fly as the
// aggregation Aᵀ·G of the layer above plus its row-mapped residual — the layer-2 backward
// aggregation fused into the layer-1 tail (gnn_sage_norm_bwd_agg_f32): Aᵀ's rows are short
// (1.7 nonzeros on average for the Reddit batch) and G is L2-resident, so the tail reads those
// few G rows instead of a 35 MB gradient that a separate launch would write and this kernel
// read back. Per element the same operations in the same order as spmm_row_kernel with one wave
// per row (a C fmaf chain over the row in CSR order from 0, then + the residual): bit-identical.
struct GradSrc {
  const float* gY;
  int64_t ldg;
  const int* rp;  // Aᵀ (rows = this layer's rows), CSR
  const int* col;
  const float* val;
  const float* G;  // the dense operand Aᵀ multiplies (rows of the layer above)
  int64_t ldG;
  const float* R;  // residual rows R[rmap[r]] (rmap NULL: none)
  int64_t ldr;
  const int* rmap;
};

__device__ __forceinline__ f4 fma4(float v, f4 x, f4 a) {
  return f4{__builtin_fmaf(v, x.x, a.x), __builtin_fmaf(v, x.y, a.y), __builtin_fmaf(v, x.z, a.z),
            __builtin_fmaf(v, x.w, a.w)};
}

// g[k] for columns cbase + (lane + 64 k) * 4 < cend of row r.
template <bool AGG, int NV>
__device__ __forceinline__ void grad_row(const GradSrc& s, int r, int lane, int cbase, int cend, f4 (&g)[NV]) {
  if constexpr (!AGG) {
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      const int c = cbase + (lane + 64 * k) * 4;
      g[k] = c < cend ? *reinterpret_cast<const f4*>(s.gY + (int64_t)r * s.ldg + c) : f4(0.0f);
    }
  } else {
    const int q = s.rmap ? s.rmap[r] : -1;
#pragma unroll
    for (int k = 0; k < NV; ++k) g[k] = f4(0.0f);
    const int rb = s.rp[r], re = s.rp[r + 1];
    // two nonzeros per round: both G rows in flight before the FMAs (added in CSR order)
    for (int e = rb; e < re; e += 2) {
      const bool two = e + 1 < re;  // wave-uniform
      const float* x0 = s.G + (int64_t)s.col[e] * s.ldG;  // wave-uniform: scalar loads of (col, val)
      const float v0 = s.val[e];
      const float* x1 = two ? s.G + (int64_t)s.col[e + 1] * s.ldG : x0;
      const float v1 = two ? s.val[e + 1] : 0.0f;
      f4 xs0[NV], xs1[NV];
#pragma unroll
      for (int k = 0; k < NV; ++k) {
        const int c = cbase + (lane + 64 * k) * 4;
        xs0[k] = c < cend ? *reinterpret_cast<const f4*>(x0 + c) : f4(0.0f);
        xs1[k] = (two && c < cend) ? *reinterpret_cast<const f4*>(x1 + c) : f4(0.0f);
      }
#pragma unroll
      for (int k = 0; k < NV; ++k) g[k] = fma4(v0, xs0[k], g[k]);
      if (two) {
#pragma unroll
        for (int k = 0; k < NV; ++k) g[k] = fma4(v1, xs1[k], g[k]);
      }
    }
    if (q >= 0) {
#pragma unroll
      for (int k = 0; k < NV; ++k) {
        const int c = cbase + (lane + 64 * k) * 4;
        if (c < cend) g[k] += *reinterpret_cast<const f4*>(s.R + (int64_t)q * s.ldr + c);
      }
    }
  }
}

// The folded gradient's dependent chain, loaded one row ahead (AGG, split-row backward): the next
// row's Aᵀ range and residual slot at the top of an iteration, its first two (col, val) at the end
// (the range has arrived by then), so a row's own chain is only its G rows (+ the residual row).
// The values travel in vector registers (lane 0 / 1 / 2: row start / end / residual slot; lane j <
// 2: entry rb + j) and are read with readlane where used: vector loads retire in order, so using
// them waits for nothing issued later (scalar loads may return out of order, and any use of one
// waits for every scalar load in flight).
struct Ahead {
  int rv;    // lane 0: rb, lane 1: re, lane 2: q (rmap[r] or -1)
  int cv;    // lane j < 2: col[rb + j]
  float vv;  // lane j < 2: val[rb + j]
};

__device__ __forceinline__ int rdl(int x, int l) { return __builtin_amdgcn_readlane(x, l); }
__device__ __forceinline__ float rdlf(float x, int l) {
  return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, x), l));
}

__device__ __forceinline__ void ahead_range(const GradSrc& s, int r, int M, int lane, Ahead& a) {
  a.rv = lane == 2 ? -1 : 0;
  if (r < M) {
    if (lane < 2) a.rv = s.rp[r + lane];
    else if (lane == 2 && s.rmap) a.rv = s.rmap[r];
  }
}

__device__ __forceinline__ void ahead_pairs(const GradSrc& s, int lane, Ahead& a) {
  const int rb = rdl(a.rv, 0), re = rdl(a.rv, 1);
  const int e = rb + (lane & 1);
  a.cv = 0;
  a.vv = 0.0f;
  if (lane < 2 && e < re) {
    a.cv = s.col[e];
    a.vv = s.val[e];
  }
}

// The same values as grad_row<true>: the fmaf chain in CSR order from 0, then + the residual.
template <int NV>
__device__ __forceinline__ void grad_row_ahead(const GradSrc& s, const Ahead& a, int lane, int cbase, int cend,
                                               f4 (&g)[NV]) {
#pragma unroll
  for (int k = 0; k < NV; ++k) g[k] = f4(0.0f);
  const int rb = rdl(a.rv, 0), re = rdl(a.rv, 1), q = rdl(a.rv, 2);
  for (int e = rb; e < re; e += 2) {
    const bool first = e == rb;  // wave-uniform
    const bool two = e + 1 < re;
    const int c0 = first ? rdl(a.cv, 0) : s.col[e];
    const float v0 = first ? rdlf(a.vv, 0) : s.val[e];
    const int c1 = first ? rdl(a.cv, 1) : (two ? s.col[e + 1] : 0);
    const float v1 = first ? rdlf(a.vv, 1) : (two ? s.val[e + 1] : 0.0f);
    const float* x0 = s.G + (int64_t)c0 * s.ldG;
    const float* x1 = s.G + (int64_t)(two ? c1 : c0) * s.ldG;
    f4 xs0[NV], xs1[NV];
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      const int c = cbase + (lane + 64 * k) * 4;
      xs0[k] = c < cend ? *reinterpret_cast<const f4*>(x0 + c) : f4(0.0f);
      xs1[k] = (two && c < cend) ? *reinterpret_cast<const f4*>(x1 + c) : f4(0.0f);
    }
#pragma unroll
    for (int k = 0; k < NV; ++k) g[k] = fma4(v0, xs0[k], g[k]);
    if (two) {
#pragma unroll
      for (int k = 0; k < NV; ++k) g[k] = fma4(v1, xs1[k], g[k]);
    }
  }
  if (q >= 0) {
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      const int c = cbase + (lane + 64 * k) * 4;
      if (c < cend) g[k] += *reinterpret_cast<const f4*>(s.R + (int64_t)q * s.ldr + c);
    }
  }
}

template <int NV>
__global__ __launch_bounds__(256) void sage_norm_fwd_kernel(const float* __restrict__ hB, int64_t ldb,
                                                            const float* __restrict__ bB, int D1,
                                                            const float* __restrict__ hW, int64_t ldw,
                                                            const float* __restrict__ bW, int D,
                                                            const float* __restrict__ scale,
                                                            const float* __restrict__ offset, int M, float p,
                                                            float inv_keep, uint64_t seed, int training,
                                                            float* __restrict__ Y, int64_t ldy,
                                                            float* __restrict__ mean_out, float* __restrict__ rstd_out) {
  const int lane = threadIdx.x & 63;
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= M) return;
  f4 o[NV];
  float s = 0.0f;
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    const int c = (lane + 64 * k) * 4;
    if (c < D) {
      const f4 h = load_h(hB, ldb, bB, D1, hW, ldw, bW, r, c);
      o[k] = f4{elu1(h.x), elu1(h.y), elu1(h.z), elu1(h.w)};
      s += (o[k].x + o[k].y) + (o[k].z + o[k].w);
    } else {
      o[k] = f4(0.0f);
    }
  }
  const float mean = wave_sum(s) / (float)D;
  float q = 0.0f;
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    const int c = (lane + 64 * k) * 4;
    if (c < D) {
      const f4 d = o[k] - mean;
      q += (d.x * d.x + d.y * d.y) + (d.z * d.z + d.w * d.w);
    }
  }
  const float var = wave_sum(q) / (float)D + 1e-9f;
  const float rstd = rsqrtf(var);
  const DropThr dt = drop_thr(p);
  const RowDrop rd(drop_key(seed), (uint64_t)r * (uint64_t)D);
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    const int c = (lane + 64 * k) * 4;
    if (c < D) {
      const f4 sc = *reinterpret_cast<const f4*>(scale + c);
      const f4 of = *reinterpret_cast<const f4*>(offset + c);
      f4 y = (o[k] - mean) * sc * rstd + of;
      if (training) {
        y.x = rd.keep(c + 0, dt) ? y.x * inv_keep : 0.0f;
        y.y = rd.keep(c + 1, dt) ? y.y * inv_keep : 0.0f;
        y.z = rd.keep(c + 2, dt) ? y.z * inv_keep : 0.0f;
        y.w = rd.keep(c + 3, dt) ? y.w * inv_keep : 0.0f;
      }
      *reinterpret_cast<f4*>(Y + (int64_t)r * ldy + c) = y;
    }
  }
  if (lane == 0) {
    mean_out[r] = mean;
    rstd_out[r] = rstd;
  }
}

template <int NV, bool AGG>
__global__ __launch_bounds__(256) void sage_norm_bwd_kernel(
    GradSrc src, const float* __restrict__ hB, int64_t ldb,
    const float* __restrict__ bB, int D1, const float* __restrict__ hW, int64_t ldw, const float* __restrict__ bW,
    int D, const float* __restrict__ scale, const float* __restrict__ mean, const float* __restrict__ rstd, int M,
    float p, float inv_keep, uint64_t seed, int training, float* __restrict__ dhB, float* __restrict__ dhW,
    float* __restrict__ partial) {
  extern __shared__ __attribute__((aligned(16))) float red[];  // [4 waves][D], reused per sum
  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;
  f4 ds[NV], db[NV], dbi[NV];
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    ds[k] = f4(0.0f);
    db[k] = f4(0.0f);
    dbi[k] = f4(0.0f);
  }
  const DropThr dt = drop_thr(p);
  const uint32_t dkey = drop_key(seed);
  for (int r = blockIdx.x * 4 + w; r < M; r += gridDim.x * 4) {
    const float m = mean[r];
    const float rs = rstd[r];
    const RowDrop rd(dkey, (uint64_t)r * (uint64_t)D);
    f4 h[NV], xh[NV], gx[NV];
#pragma unroll
    for (int k = 0; k < NV; ++k) {  // pre-activations first (overlapping the gradient's chain)
      const int c = (lane + 64 * k) * 4;
      h[k] = c < D ? load_h(hB, ldb, bB, D1, hW, ldw, bW, r, c) : f4(0.0f);
    }
    grad_row<AGG, NV>(src, r, lane, 0, D, gx);  // gx holds the output gradient until it is scaled
    float a = 0.0f, b = 0.0f;
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      const int c = (lane + 64 * k) * 4;
      if (c < D) {
        const f4 hk = h[k];
        const f4 o = f4{elu1(hk.x), elu1(hk.y), elu1(hk.z), elu1(hk.w)};
        h[k] = f4{elu1_grad_from_out(o.x), elu1_grad_from_out(o.y), elu1_grad_from_out(o.z),
                  elu1_grad_from_out(o.w)};  // h[k] now holds the ELU derivative
        xh[k] = (o - m) * rs;
        f4 g = gx[k];
        if (training) {
          g.x = rd.keep(c + 0, dt) ? g.x * inv_keep : 0.0f;
          g.y = rd.keep(c + 1, dt) ? g.y * inv_keep : 0.0f;
          g.z = rd.keep(c + 2, dt) ? g.z * inv_keep : 0.0f;
          g.w = rd.keep(c + 3, dt) ? g.w * inv_keep : 0.0f;
        }
        db[k] += g;
        ds[k] += g * xh[k];
        gx[k] = g * *reinterpret_cast<const f4*>(scale + c);
        const f4 gxx = gx[k] * xh[k];
        a += (gx[k].x + gx[k].y) + (gx[k].z + gx[k].w);
        b += (gxx.x + gxx.y) + (gxx.z + gxx.w);
      } else {
        h[k] = xh[k] = gx[k] = f4(0.0f);
      }
    }
    a = wave_sum(a) / (float)D;
    b = wave_sum(b) / (float)D;
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      const int c = (lane + 64 * k) * 4;
      if (c < D) {
        const f4 dxo = rs * (gx[k] - a - xh[k] * b);
        const f4 dh = dxo * h[k];
        dbi[k] += dh;
        if (c < D1) {
          *reinterpret_cast<f4*>(dhB + (int64_t)r * D1 + c) = dh;
        } else {
          *reinterpret_cast<f4*>(dhW + (int64_t)r * (D - D1) + (c - D1)) = dh;
        }
      }
    }
  }
  // workgroup column sums -> partial[blockIdx.x][q][D], q = 0 d(scale), 1 d(offset), 2 d(bias)
#pragma unroll
  for (int q = 0; q < NRED; ++q) {
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      const int c = (lane + 64 * k) * 4;
      if (c < D) *reinterpret_cast<f4*>(red + w * D + c) = (q == 0) ? ds[k] : (q == 1) ? db[k] : dbi[k];
    }
    __syncthreads();
    for (int c = threadIdx.x; c < D; c += 256) {
      partial[((int64_t)blockIdx.x * NRED + q) * D + c] = (red[c] + red[D + c]) + (red[2 * D + c] + red[3 * D + c]);
    }
    __syncthreads();
  }
}

// Split-row backward (D % 8 == 0, D >= 512): two waves per row, each holding half of it
// (half the registers: ~2x the rows in flight per CU, the 1-wave form is latency-bound at
// 3 workgroups per CU); the row sums meet in LDS (half 0 + half 1, fixed order) behind one
// barrier per row pair, double-buffered by iteration parity.
constexpr int BWD2_MAX_GRID = 1024;
// The folded form (AGG) at 2,048 workgroups measured 36.7 vs 37.6 us for the kernel but +6 us of
// finalize over twice the partial rows (profiles/round4/fold/, r4f): both forms keep 1,024;
// GNN_SAGE_BWD2_GRID(_AGG) override it for sweeps (the workspace is sized for up to 2,048).
constexpr int BWD2_GRID_SWEEP_MAX = 2048;
int bwd2_grid_cap(bool agg) {
  const char* e = std::getenv(agg ? "GNN_SAGE_BWD2_GRID_AGG" : "GNN_SAGE_BWD2_GRID");
  const int v = e ? std::atoi(e) : 0;
  return v > 0 && v <= BWD2_GRID_SWEEP_MAX ? v : BWD2_MAX_GRID;
}

// 4 workgroups per CU at D <= 1024 (<= 128 VGPRs with the next row's loads held)
template <int NVH, bool AGG>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(NVH <= 2 ? 4 : 1))) void sage_norm_bwd2_kernel(
    GradSrc src, const float* __restrict__ hB, int64_t ldb,
    const float* __restrict__ bB, int D1, const float* __restrict__ hW, int64_t ldw, const float* __restrict__ bW,
    int D, const float* __restrict__ scale, const float* __restrict__ mean, const float* __restrict__ rstd, int M,
    float p, float inv_keep, uint64_t seed, int training, float* __restrict__ dhB, float* __restrict__ dhW,
    float* __restrict__ partial) {
  extern __shared__ __attribute__((aligned(16))) float red[];  // [2 row slots][D]
  __shared__ float rsum[2][4][2];
  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;
  const int slot = w >> 1, half = w & 1;
  const int Dh = D >> 1;
  const int cbase = half * Dh;
  const int cend = half ? D : Dh;
  f4 ds[NVH], db[NVH], dbi[NVH];
#pragma unroll
  for (int k = 0; k < NVH; ++k) {
    ds[k] = f4(0.0f);
    db[k] = f4(0.0f);
    dbi[k] = f4(0.0f);
  }
  const DropThr dt = drop_thr(p);
  const uint32_t dkey = drop_key(seed);
  int it = 0;
  Ahead nx{};  // AGG: the chain of this wave's next row, loaded one iteration ahead
  if constexpr (AGG) {
    ahead_range(src, blockIdx.x * 2 + slot, M, lane, nx);
    ahead_pairs(src, lane, nx);
  }
  // The next row's pre-activations, saved statistics and (dense form) output gradient are loaded
  // one iteration ahead: they arrive while this row is reduced, exchanged and stored (the kernel
  // is latency-bound at 4 workgroups per CU; loads stay in flight across the LDS barrier).
  const int rstride = gridDim.x * 2;
  f4 hn[NVH], gn[NVH];
  float mn = 0.0f, rsn = 0.0f;
  auto load_next = [&](int rr) {
    if (rr < M) {
      mn = mean[rr];
      rsn = rstd[rr];
#pragma unroll
      for (int k = 0; k < NVH; ++k) {
        const int c = cbase + (lane + 64 * k) * 4;
        hn[k] = c < cend ? load_h(hB, ldb, bB, D1, hW, ldw, bW, rr, c) : f4(0.0f);
      }
      if constexpr (!AGG) grad_row<false, NVH>(src, rr, lane, cbase, cend, gn);
    }
  };
  load_next(blockIdx.x * 2 + slot);
  for (int r0 = blockIdx.x * 2; r0 < M; r0 += rstride, ++it) {
    const int r = r0 + slot;
    const bool live = r < M;
    f4 gx[NVH];
    float a = 0.0f, b = 0.0f;
    const float m = mn, rs = rsn;
    f4 hv[NVH];
#pragma unroll
    for (int k = 0; k < NVH; ++k) {
      hv[k] = hn[k];
      if constexpr (!AGG) gx[k] = gn[k];
    }
    Ahead cur{};
    if constexpr (AGG) cur = nx;
    load_next(r + rstride);
    if constexpr (AGG) {
      ahead_range(src, r + rstride, M, lane, nx);  // the next row's range
      if (live) grad_row_ahead<NVH>(src, cur, lane, cbase, cend, gx);  // the output gradient, scaled below
    }
    // the next row's first (col, val) pairs: its range arrived while this row's G rows were awaited,
    // and the pairs now have the rest of this iteration (reductions, barrier, stores) to arrive
    if constexpr (AGG) ahead_pairs(src, lane, nx);
    const RowDrop rd(dkey, (uint64_t)r * (uint64_t)D);
#pragma unroll
    for (int k = 0; k < NVH; ++k) {
      const int c = cbase + (lane + 64 * k) * 4;
      if (live && c < cend) {
        const f4 hk = hv[k];
        const f4 o = f4{elu1(hk.x), elu1(hk.y), elu1(hk.z), elu1(hk.w)};
        hv[k] = o;  // the activation: xh and the ELU derivative are recomputed from it below
        const f4 xh = (o - m) * rs;
        f4 g = gx[k];
        if (training) {
          g.x = rd.keep(c + 0, dt) ? g.x * inv_keep : 0.0f;
          g.y = rd.keep(c + 1, dt) ? g.y * inv_keep : 0.0f;
          g.z = rd.keep(c + 2, dt) ? g.z * inv_keep : 0.0f;
          g.w = rd.keep(c + 3, dt) ? g.w * inv_keep : 0.0f;
        }
        db[k] += g;
        ds[k] += g * xh;
        gx[k] = g * *reinterpret_cast<const f4*>(scale + c);
        const f4 gxx = gx[k] * xh;
        a += (gx[k].x + gx[k].y) + (gx[k].z + gx[k].w);
        b += (gxx.x + gxx.y) + (gxx.z + gxx.w);
      } else {
        hv[k] = gx[k] = f4(0.0f);
      }
    }
    a = wave_sum(a);
    b = wave_sum(b);
    const int buf = it & 1;
    if (lane == 0) {
      rsum[buf][w][0] = a;
      rsum[buf][w][1] = b;
    }
    __syncthreads();
    const float A = (rsum[buf][2 * slot][0] + rsum[buf][2 * slot + 1][0]) / (float)D;
    const float B = (rsum[buf][2 * slot][1] + rsum[buf][2 * slot + 1][1]) / (float)D;
    if (live) {
#pragma unroll
      for (int k = 0; k < NVH; ++k) {
        const int c = cbase + (lane + 64 * k) * 4;
        if (c < cend) {
          const f4 o = hv[k];
          const f4 xh = (o - m) * rs;
          const f4 eg = f4{elu1_grad_from_out(o.x), elu1_grad_from_out(o.y), elu1_grad_from_out(o.z),
                           elu1_grad_from_out(o.w)};
          const f4 dh = rs * (gx[k] - A - xh * B) * eg;
          dbi[k] += dh;
          if (c < D1) {
            *reinterpret_cast<f4*>(dhB + (int64_t)r * D1 + c) = dh;
          } else {
            *reinterpret_cast<f4*>(dhW + (int64_t)r * (D - D1) + (c - D1)) = dh;
          }
        }
      }
    }
  }
  // workgroup column sums -> partial[blockIdx.x][q][D]: slot 0 + slot 1 (fixed order)
#pragma unroll
  for (int q = 0; q < NRED; ++q) {
#pragma unroll
    for (int k = 0; k < NVH; ++k) {
      const int c = cbase + (lane + 64 * k) * 4;
      if (c < cend) *reinterpret_cast<f4*>(red + slot * D + c) = (q == 0) ? ds[k] : (q == 1) ? db[k] : dbi[k];
    }
    __syncthreads();
    for (int c = threadIdx.x; c < D; c += 256) partial[((int64_t)blockIdx.x * NRED + q) * D + c] = red[c] + red[D + c];
    __syncthreads();
  }
}

// Column sums over the G workgroup partials: a workgroup owns FIN_COLS of the NRED*D
// columns (192 workgroups at D = 1024, not 48: the sum is latency-bound); thread t sums
// column t % FIN_COLS over the partial rows g = t / FIN_COLS (mod 16), 16 loads in flight,
// and the 16 group sums are added in a fixed order through LDS (deterministic).
constexpr int FIN_COLS = 16;

__global__ __launch_bounds__(256) void sage_norm_bwd_finalize_kernel(const float* __restrict__ partial, int G, int D,
                                                                     int D1, float* __restrict__ dscale,
                                                                     float* __restrict__ doffset,
                                                                     float* __restrict__ dbB,
                                                                     float* __restrict__ dbW) {
  __shared__ float qs[16][FIN_COLS];
  const int cl = threadIdx.x % FIN_COLS;
  const int grp = threadIdx.x / FIN_COLS;  // 0..15
  const int i = blockIdx.x * FIN_COLS + cl;
  float s = 0.0f;
  if (i < NRED * D) {
    const int64_t stride = (int64_t)NRED * D;
    int g = grp;
    // 16 loads in flight per thread (the sum is latency-bound: 64 partial rows per thread at
    // G = 1024), added in row order as they arrive
    for (; g + 240 < G; g += 256) {
      float a[16];
#pragma unroll
      for (int k = 0; k < 16; ++k) a[k] = partial[(int64_t)(g + 16 * k) * stride + i];
#pragma unroll
      for (int k = 0; k < 16; ++k) s += a[k];
    }
    for (; g + 48 < G; g += 64) {
      const float a0 = partial[(int64_t)(g + 0) * stride + i];
      const float a1 = partial[(int64_t)(g + 16) * stride + i];
      const float a2 = partial[(int64_t)(g + 32) * stride + i];
      const float a3 = partial[(int64_t)(g + 48) * stride + i];
      s += a0;
      s += a1;
      s += a2;
      s += a3;
    }
    for (; g < G; g += 16) s += partial[(int64_t)g * stride + i];
  }
  qs[grp][cl] = s;
  __syncthreads();
  if (grp == 0 && i < NRED * D) {
    float t = 0.0f;
#pragma unroll
    for (int q = 0; q < 16; ++q) t += qs[q][cl];
    const int q = i / D, c = i % D;
    if (q == 0) {
      dscale[c] = t;
    } else if (q == 1) {
      doffset[c] = t;
    } else if (c < D1) {
      if (dbB) dbB[c] = t;
    } else if (dbW) {
      dbW[c - D1] = t;
    }
  }
}

using FwdFn = void (*)(const float*, int64_t, const float*, int, const float*, int64_t, const float*, int,
                       const float*, const float*, int, float, float, uint64_t, int, float*, int64_t, float*, float*);
using BwdFn = void (*)(GradSrc, const float*, int64_t, const float*, int, const float*, int64_t,
                       const float*, int, const float*, const float*, const float*, int, float, float, uint64_t, int,
                       float*, float*, float*);

FwdFn fwd_fn(int nv) {
  switch (nv) {
    case 1: return &sage_norm_fwd_kernel<1>;
    case 2: return &sage_norm_fwd_kernel<2>;
    case 3: return &sage_norm_fwd_kernel<3>;
    case 4: return &sage_norm_fwd_kernel<4>;
    case 5: return &sage_norm_fwd_kernel<5>;
    case 6: return &sage_norm_fwd_kernel<6>;
    case 7: return &sage_norm_fwd_kernel<7>;
    case 8: return &sage_norm_fwd_kernel<8>;
    default: return nullptr;
  }
}

template <bool AGG>
BwdFn bwd2_fn(int nvh) {
  switch (nvh) {
    case 1: return &sage_norm_bwd2_kernel<1, AGG>;
    case 2: return &sage_norm_bwd2_kernel<2, AGG>;
    case 3: return &sage_norm_bwd2_kernel<3, AGG>;
    case 4: return &sage_norm_bwd2_kernel<4, AGG>;
    default: return nullptr;
  }
}

// the split-row form applies (and its grid G, which sizes the partial slab)
bool use_bwd2(int64_t D) { return D % 8 == 0 && D >= 512 && std::getenv("GNN_SAGE_BWD1") == nullptr; }

int64_t bwd_grid(int64_t M, int64_t D, bool agg = false) {
  if (use_bwd2(D)) return std::max<int64_t>(1, std::min<int64_t>(ceil_div(M, 2), bwd2_grid_cap(agg)));
  const int64_t cap = bwd_grid_cap();
  return std::max<int64_t>(1, ceil_div(M, 4) < cap ? ceil_div(M, 4) : cap);
}

template <bool AGG>
BwdFn bwd_fn(int nv) {
  switch (nv) {
    case 1: return &sage_norm_bwd_kernel<1, AGG>;
    case 2: return &sage_norm_bwd_kernel<2, AGG>;
    case 3: return &sage_norm_bwd_kernel<3, AGG>;
    case 4: return &sage_norm_bwd_kernel<4, AGG>;
    case 5: return &sage_norm_bwd_kernel<5, AGG>;
    case 6: return &sage_norm_bwd_kernel<6, AGG>;
    case 7: return &sage_norm_bwd_kernel<7, AGG>;
    case 8: return &sage_norm_bwd_kernel<8, AGG>;
    default: return nullptr;
  }
}

int check_shapes(const char* fn, int64_t D1, int64_t D2, int64_t M, const void* hB, int64_t ldb, const void* hW,
                 int64_t ldw, const void* bB, const void* bW) {
  GNN_REQUIRE(M >= 0 && D1 >= 0 && D2 >= 0, "%s: negative size", fn);
  GNN_REQUIRE(M < INT_MAX, "%s: M too large", fn);
  GNN_REQUIRE(D1 % 4 == 0 && D2 % 4 == 0, "%s: D1 and D2 must be multiples of 4", fn);
  GNN_REQUIRE(D1 + D2 > 0 && D1 + D2 <= SN_MAXV * 256, "%s: D = %lld outside (0, 2048]", fn,
              (long long)(D1 + D2));
  GNN_REQUIRE(D1 == 0 || (hB && ldb % 4 == 0 && (uintptr_t)hB % 16 == 0), "%s: hB must be 16-byte aligned rows", fn);
  GNN_REQUIRE(D2 == 0 || (hW && ldw % 4 == 0 && (uintptr_t)hW % 16 == 0), "%s: hW must be 16-byte aligned rows", fn);
  GNN_REQUIRE((uintptr_t)bB % 16 == 0 && (uintptr_t)bW % 16 == 0, "%s: biases must be 16-byte aligned", fn);
  return 0;
}

}  // namespace

extern "C" {

int gnn_sage_norm_fwd_f32(const float* hB, int64_t ldb, int64_t D1, const float* hW, int64_t ldw, int64_t D2,
                          const float* biasB, const float* biasW, const float* scale, const float* offset, int64_t M,
                          float p_drop, uint64_t seed, int training, float* Y, int64_t ldy, float* mean_out,
                          float* rstd_out, void* stream) {
  int rc = check_shapes("gnn_sage_norm_fwd_f32", D1, D2, M, hB, ldb, hW, ldw, biasB, biasW);
  if (rc) return rc;
  if (M == 0) return 0;
  GNN_REQUIRE(scale && offset && Y && mean_out && rstd_out, "gnn_sage_norm_fwd_f32: NULL pointer");
  GNN_REQUIRE(ldy % 4 == 0 && (uintptr_t)Y % 16 == 0, "gnn_sage_norm_fwd_f32: Y must be 16-byte aligned rows");
  GNN_REQUIRE(p_drop >= 0.0f && p_drop < 1.0f, "gnn_sage_norm_fwd_f32: p_drop must be in [0, 1)");
  const int D = (int)(D1 + D2);
  const int nv = (int)ceil_div(D, 256);
  hipStream_t st = (hipStream_t)stream;
  const float inv_keep = 1.0f / (1.0f - p_drop);
  hipLaunchKernelGGL(fwd_fn(nv), dim3((unsigned)ceil_div(M, 4)), dim3(256), 0, st, hB ? hB : hW, ldb, biasB,
                     (int)D1, hW, ldw, biasW, D, scale, offset, (int)M, p_drop, inv_keep, seed, training, Y, ldy,
                     mean_out, rstd_out);
  GNN_LAUNCHED("sage_norm_fwd_kernel");
  return 0;
}

size_t gnn_sage_norm_bwd_workspace_bytes(int64_t M, int64_t D) {
  // sized for the largest grid a sweep may ask for
  const int64_t G = M <= 0 ? 1 : (use_bwd2(D) ? std::max<int64_t>(1, std::min<int64_t>(ceil_div(M, 2),
                                                                                        BWD2_GRID_SWEEP_MAX))
                                              : bwd_grid(M, D));
  return gnn::align_up((size_t)G * NRED * (size_t)(D > 0 ? D : 1) * sizeof(float), 256);
}

}  // extern "C"

namespace {

int sage_norm_bwd(const GradSrc& src, bool agg, const float* hB, int64_t ldb, int64_t D1, const float* hW,
                  int64_t ldw, int64_t D2, const float* biasB, const float* biasW, const float* scale,
                  const float* mean, const float* rstd, int64_t M, float p_drop, uint64_t seed, int training,
                  float* dhB, float* dhW, float* dscale, float* doffset, float* dbiasB, float* dbiasW,
                  void* workspace, size_t workspace_bytes, void* stream) {
  const float* gY = agg ? src.G : src.gY;
  const int64_t ldg = agg ? 4 : src.ldg;
  int rc = check_shapes("gnn_sage_norm_bwd_f32", D1, D2, M, hB, ldb, hW, ldw, biasB, biasW);
  if (rc) return rc;
  GNN_REQUIRE(scale && dscale && doffset, "gnn_sage_norm_bwd_f32: NULL pointer");
  GNN_REQUIRE(p_drop >= 0.0f && p_drop < 1.0f, "gnn_sage_norm_bwd_f32: p_drop must be in [0, 1)");
  const int D = (int)(D1 + D2);
  hipStream_t st = (hipStream_t)stream;
  if (M == 0) {
    GNN_HIP(hipMemsetAsync(dscale, 0, (size_t)D * 4, st), "dscale memset");
    GNN_HIP(hipMemsetAsync(doffset, 0, (size_t)D * 4, st), "doffset memset");
    if (dbiasB && D1) GNN_HIP(hipMemsetAsync(dbiasB, 0, (size_t)D1 * 4, st), "dbiasB memset");
    if (dbiasW && D2) GNN_HIP(hipMemsetAsync(dbiasW, 0, (size_t)D2 * 4, st), "dbiasW memset");
    return 0;
  }
  GNN_REQUIRE(gY && mean && rstd && (D1 == 0 || dhB) && (D2 == 0 || dhW), "gnn_sage_norm_bwd_f32: NULL pointer");
  GNN_REQUIRE(ldg % 4 == 0 && (uintptr_t)gY % 16 == 0, "gnn_sage_norm_bwd_f32: gY must be 16-byte aligned rows");
  GNN_REQUIRE(D1 == 0 || (uintptr_t)dhB % 16 == 0, "gnn_sage_norm_bwd_f32: dhB not 16-byte aligned");
  GNN_REQUIRE(D2 == 0 || (uintptr_t)dhW % 16 == 0, "gnn_sage_norm_bwd_f32: dhW not 16-byte aligned");
  GNN_REQUIRE(workspace && workspace_bytes >= gnn_sage_norm_bwd_workspace_bytes(M, D),
              "gnn_sage_norm_bwd_f32: workspace too small");
  const int64_t G = bwd_grid(M, D, agg);
  const float inv_keep = 1.0f / (1.0f - p_drop);
  float* partial = (float*)workspace;
  if (use_bwd2(D)) {
    hipLaunchKernelGGL(agg ? bwd2_fn<true>((int)ceil_div(D / 2, 256)) : bwd2_fn<false>((int)ceil_div(D / 2, 256)),
                       dim3((unsigned)G), dim3(256), (size_t)2 * D * sizeof(float), st, src, hB ? hB : hW, ldb, biasB,
                       (int)D1, hW, ldw, biasW, D, scale, mean, rstd, (int)M, p_drop, inv_keep, seed, training,
                       dhB ? dhB : dhW, dhW, partial);
  } else {
    hipLaunchKernelGGL(agg ? bwd_fn<true>((int)ceil_div(D, 256)) : bwd_fn<false>((int)ceil_div(D, 256)),
                       dim3((unsigned)G), dim3(256), (size_t)4 * D * sizeof(float), st, src, hB ? hB : hW, ldb, biasB,
                       (int)D1, hW, ldw, biasW, D, scale, mean, rstd, (int)M, p_drop, inv_keep, seed, training,
                       dhB ? dhB : dhW, dhW, partial);
  }
  GNN_LAUNCHED("sage_norm_bwd_kernel");
  sage_norm_bwd_finalize_kernel<<<dim3((unsigned)ceil_div(NRED * D, FIN_COLS)), dim3(256), 0, st>>>(
      partial, (int)G, D, (int)D1, dscale, doffset, dbiasB, dbiasW);
  GNN_LAUNCHED("sage_norm_bwd_finalize_kernel");
  return 0;
}

}  // namespace

extern "C" {

int gnn_sage_norm_bwd_f32(const float* gY, int64_t ldg, const float* hB, int64_t ldb, int64_t D1, const float* hW,
                          int64_t ldw, int64_t D2, const float* biasB, const float* biasW, const float* scale,
                          const float* mean, const float* rstd, int64_t M, float p_drop, uint64_t seed, int training,
                          float* dhB, float* dhW, float* dscale, float* doffset, float* dbiasB, float* dbiasW,
                          void* workspace, size_t workspace_bytes, void* stream) {
  GradSrc src{};
  src.gY = gY;
  src.ldg = ldg;
  return sage_norm_bwd(src, false, hB, ldb, D1, hW, ldw, D2, biasB, biasW, scale, mean, rstd, M, p_drop, seed,
                       training, dhB, dhW, dscale, doffset, dbiasB, dbiasW, workspace, workspace_bytes, stream);
}

int gnn_sage_norm_bwd_agg_f32(const int32_t* t_rowptr, const int32_t* t_col, const float* t_val, const float* G,
                              int64_t ldG, const float* R, int64_t ldr, const int32_t* rmap, const float* hB,
                              int64_t ldb, int64_t D1, const float* hW, int64_t ldw, int64_t D2, const float* biasB,
                              const float* biasW, const float* scale, const float* mean, const float* rstd, int64_t M,
                              float p_drop, uint64_t seed, int training, float* dhB, float* dhW, float* dscale,
                              float* doffset, float* dbiasB, float* dbiasW, void* workspace, size_t workspace_bytes,
                              void* stream) {
  const int64_t D = D1 + D2;
  GNN_REQUIRE(M == 0 || (t_rowptr && G), "gnn_sage_norm_bwd_agg_f32: NULL t_rowptr / G");
  GNN_REQUIRE(ldG % 4 == 0 && (uintptr_t)G % 16 == 0 && ldG >= D, "gnn_sage_norm_bwd_agg_f32: G must be 16-byte "
              "aligned rows of at least D floats");
  GNN_REQUIRE(rmap == nullptr || (R && ldr % 4 == 0 && (uintptr_t)R % 16 == 0 && ldr >= D),
              "gnn_sage_norm_bwd_agg_f32: R must be 16-byte aligned rows of at least D floats");
  GradSrc src{};
  src.rp = t_rowptr;
  src.col = t_col;
  src.val = t_val;
  src.G = G;
  src.ldG = ldG;
  src.R = R;
  src.ldr = ldr;
  src.rmap = rmap;
  return sage_norm_bwd(src, true, hB, ldb, D1, hW, ldw, D2, biasB, biasW, scale, mean, rstd, M, p_drop, seed,
                       training, dhB, dhW, dscale, doffset, dbiasB, dbiasW, workspace, workspace_bytes, stream);
}

}  // extern "C"
