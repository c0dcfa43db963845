// spmm.hip — MI355X (gfx950, CDNA4) kernels and C ABI of the SpMM aggregation path.
//
// What the reference does (spmm_cpp/cuda_spmm.cu:619-704): per call it converts the COO
// indices to int32, zero-fills Y, builds a row pointer and a "virtual row" split of every
// row into <=64-nnz chunks with a Blelloch scan (5-6 device syncs, 3 .item() reads, raw
// cudaMalloc/cudaFree), then runs one 32-thread half-block per virtual row that gathers
// X rows with scalar 4-byte loads and atomically adds each 64-column tile into Y.
//
// What this file does instead (design: DESIGN.md §Kernels):
//  * The operand is CSR (int32 rowptr/col, fp32 val), built once per sampled layer by
//    gnn_build_operand_f32 (the create_coo_tensor replacement) — no per-call conversion.
//  * Load balance without a scan: the nonzeros are cut into fixed work units of S
//    consecutive entries (S = unit_nnz). One 64-lane wave owns one unit; it finds its
//    first/last row with a 64-way parallel search of rowptr and walks the rows in order.
//    A row of at most S nonzeros is owned whole by the unit holding its first nonzero and
//    stored straight to Y (empty rows store zeros, so Y is never memset); only longer rows
//    are cut at unit boundaries: their pieces go to a slab and a small second kernel adds
//    them in unit order. No atomics: results are deterministic.
//  * Inside a wave, G lanes span the feature columns with VW-wide (8 or 16 byte) loads,
//    NJ column chunks per lane, and the 64/G lane groups take different nonzeros of the
//    same row; U nonzeros are issued back to back so U*NJ row loads are in flight per lane
//    before the FMAs (memory-level parallelism for an HBM/Infinity-Cache bound gather).
//  * Everything is stream-ordered on the caller's stream: no host syncs, no allocation.
#include <hip/hip_runtime.h>
#include <vector>
#include <hip/hip_ext.h>

#include <climits>
#include <cstdarg>
#include <cstdint>
#include <cstring>
#include <cstdio>
#include <cstdlib>
#include <algorithm>
#include <atomic>
#include <mutex>
#include <string>

#include "gnn_spmm.h"
#include "common.h"

#ifndef GNN_BUILD_ID
#define GNN_BUILD_ID "dev"
#endif

namespace gnn {
thread_local std::string g_err;

int fail(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}
}  // namespace gnn

namespace {

using gnn::align_up;
using gnn::ceil_div;
using gnn::fail;
using gnn::g_err;

thread_local hipEvent_t g_ev_start = nullptr;
thread_local hipEvent_t g_ev_stop = nullptr;

// ---------------------------------------------------------------------------------
// Vector types: clang ext vectors give global_load_dwordx2/x4 and per-lane packed FMA.
// ---------------------------------------------------------------------------------
typedef float f2 __attribute__((ext_vector_type(2)));
typedef float f4 __attribute__((ext_vector_type(4)));
template <int VW> struct Vec;
template <> struct Vec<1> { using T = float; };
template <> struct Vec<2> { using T = f2; };
template <> struct Vec<4> { using T = f4; };

template <int VW>
__device__ __forceinline__ typename Vec<VW>::T vzero() { return typename Vec<VW>::T(0.0f); }

// acc + v * x with one rounding per element (matches a C fmaf chain bit for bit).
__device__ __forceinline__ float vfma(float v, float x, float acc) { return __builtin_fmaf(v, x, acc); }
__device__ __forceinline__ f2 vfma(float v, f2 x, f2 acc) {
  return f2{__builtin_fmaf(v, x.x, acc.x), __builtin_fmaf(v, x.y, acc.y)};
}
__device__ __forceinline__ f4 vfma(float v, f4 x, f4 acc) {
  return f4{__builtin_fmaf(v, x.x, acc.x), __builtin_fmaf(v, x.y, acc.y),
            __builtin_fmaf(v, x.z, acc.z), __builtin_fmaf(v, x.w, acc.w)};
}

__device__ __forceinline__ float shfl_xor_v(float x, int m) { return __shfl_xor(x, m); }
__device__ __forceinline__ f2 shfl_xor_v(f2 x, int m) { return f2{__shfl_xor(x.x, m), __shfl_xor(x.y, m)}; }
__device__ __forceinline__ f4 shfl_xor_v(f4 x, int m) {
  return f4{__shfl_xor(x.x, m), __shfl_xor(x.y, m), __shfl_xor(x.z, m), __shfl_xor(x.w, m)};
}

__device__ __forceinline__ int readlane_i(int x, int l) { return __builtin_amdgcn_readlane(x, l); }
__device__ __forceinline__ float readlane_f(float x, int l) {
  return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, x), l));
}

// Smallest r in [lo, hi) with pred(r) true (pred monotone false..true), hi if none.
// 64 probes per round: ceil(log64(hi-lo)) dependent rounds (3 for 250k rows).
template <class Pred>
__device__ __forceinline__ int wave_first_true(int lo, int hi, int lane, Pred pred) {
  while (lo < hi) {
    const int n = hi - lo;
    const int step = (n + 63) >> 6;
    const int r = lo + lane * step;
    const bool p = (r < hi) && pred(r);
    const unsigned long long b = __ballot(p);
    if (b == 0ull) {
      lo = lo + ((n - 1) / step) * step + 1;
    } else {
      const int f = __builtin_ctzll(b);
      hi = lo + f * step;
      lo = (f == 0) ? hi : lo + (f - 1) * step + 1;
    }
  }
  return lo;
}

// ---------------------------------------------------------------------------------
// SpMM main kernel. One wave per work unit of S consecutive nonzeros.
//   VW: floats per load (1/2/4); G: lanes per column group (64/32/16); NJ: column chunks
//   per lane; U: nonzeros per lane group issued back to back.
// Column of chunk j for a lane: tile_base + (lane % G) * VW + j * G * VW.
// Slab layout: [nunits][2][ldslab]; slot 0 = piece of a row that began in an earlier unit,
// slot 1 = piece of a row that begins in this unit and continues past it.
// Empty rows are not walked by the nonzero units: ROW_UNIT-row "row units" appended to the
// grid store them (zeros, or the residual row). Left to the unit holding their position, a
// run of empty rows (a FastGCN layer's transpose: most of its 8 k rows) serialised on one
// wave — 54 us for a 17 MB output.
// ---------------------------------------------------------------------------------
constexpr int ROW_UNIT = 64;

// Workgroup -> (unit block, column tile). The launch is 1-D; workgroups are dealt to the 8
// XCDs round-robin (b and b + 8 share one, MI355X_MICROARCH.md §Workgroup dispatch), and
// each XCD has its own 4 MiB L2. In tile-major order (xcd_chunk == 0) all 8 XCDs sweep the
// same column tile at once, so every L2 must hold that tile's whole slice of X. With the
// XCD map the tile-major list of W = gx * tiles items is cut into 8 contiguous chunks of
// xcd_chunk items and workgroup b works on item (b % 8) * xcd_chunk + b / 8: each XCD walks
// its own chunk in order, i.e. its own tile at a time, and holds only that tile's slice.
struct WorkMap {
  int gx;         // unit blocks per column tile (incl. the row-unit blocks)
  int items;      // gx * tiles
  int xcd_chunk;  // 0: tile-major order; else ceil(items / 8)
  __device__ __forceinline__ bool locate(unsigned b, int& ub, int& tile) const {
    int w = (int)b;
    if (xcd_chunk) {
      w = (int)(b & 7u) * xcd_chunk + (int)(b >> 3);
      if (w >= items) return false;
    }
    tile = w / gx;
    ub = w - tile * gx;
    return true;
  }
};

// One column chunk per lane: held to 8 waves per SIMD (<= 64 VGPRs; the slot-skip branches
// below otherwise take 66); wider instantiations keep the compiler's choice (no spills).
template <int VW, int G, int NJ, int U, bool RES>
__global__ __launch_bounds__(256, (NJ == 1 && U <= 4) ? 8 : 1) void spmm_unit_kernel(
    const int* __restrict__ rowptr, const int* __restrict__ col, const float* __restrict__ val,
    int M, int nnz, int S, int nunits,
    const float* __restrict__ X, int64_t ldx,
    float* __restrict__ Y, int64_t ldy,
    float* __restrict__ slab, int64_t ldslab, int F,
    const float* __restrict__ R, int64_t ldr, const int* __restrict__ rmap, WorkMap wm) {
  using V = typename Vec<VW>::T;
  constexpr int P = 64 / G;            // nonzeros taken side by side per step
  constexpr int COVER = VW * G * NJ;   // columns covered by one column tile
  const int lane = threadIdx.x & 63;
  int ub, tile;
  if (!wm.locate(blockIdx.x, ub, tile)) return;
  const int u = ub * 4 + (threadIdx.x >> 6);  // wave-uniform; no block barriers below
  const int sub = lane / G;
  const int c0 = tile * COVER + (lane % G) * VW;
  if (u >= nunits) {  // row unit: the empty rows among ROW_UNIT consecutive rows
    const int r0 = (u - nunits) * ROW_UNIT;
    if (r0 >= M) return;
    const int rl = r0 + lane;
    unsigned long long em = __ballot(rl < M && rowptr[rl] == rowptr[rl + 1]);
    while (em) {
      const int r = r0 + __builtin_ctzll(em);
      em &= em - 1;
      const float* res = nullptr;
      if constexpr (RES) {
        const int q = rmap[r];
        if (q >= 0) res = R + (int64_t)q * ldr;
      }
      float* dst = Y + (int64_t)r * ldy;
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int cc = c0 + j * G * VW;
        if ((j % P) == sub && cc < F) {
          V a = vzero<VW>();
          if constexpr (RES) {
            if (res) a = *reinterpret_cast<const V*>(res + cc);
          }
          *reinterpret_cast<V*>(dst + cc) = a;
        }
      }
    }
    return;
  }

  const int ustart = u * S;  // host guarantees nunits * S fits in int
  const int uend = min(ustart + S, nnz);

  // Row ownership: a row of at most S nonzeros belongs wholly to the unit holding its first
  // nonzero (it may run past uend, by < S); only longer rows are cut at unit boundaries.
  // rlo = the row containing position ustart (or the first row starting at/after it).
  const int rlo = wave_first_true(0, M, lane, [&](int r) {
    return rowptr[r + 1] > ustart || rowptr[r] >= ustart;
  });
  // (rows starting at or after uend belong to later units; trailing empty rows start at nnz)
  const int rhi = wave_first_true(rlo, M, lane, [&](int r) { return rowptr[r] >= uend; });

  for (int r = rlo; r < rhi; ++r) {
    const int rb = rowptr[r];
    const int re = rowptr[r + 1];
    if (rb == re) {  // empty: a row unit stores it; skip the whole run of empty rows at rb
      r = wave_first_true(r + 1, rhi, lane, [&](int q) { return rowptr[q + 1] > rb; }) - 1;
      continue;
    }
    const bool cut = re - rb > S;  // wave-uniform
    if (rb < ustart && !cut) continue;  // short row owned by an earlier unit
    const int b = max(rb, ustart);
    const int e = cut ? min(re, uend) : re;
    V acc[NJ];
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[j] = vzero<VW>();

    for (int base = b; base < e; base += 64) {
      const int n = min(64, e - base);
      int mc = 0;
      float mv = 0.0f;
      if (lane < n) {
        mc = col[base + lane];
        mv = val[base + lane];
      }
      const int last_c = __shfl(mc, n - 1);
      for (int k = 0; k < n; k += P * U) {
        V xs[U][NJ];
        float vs[U];
#pragma unroll
        for (int t = 0; t < U; ++t) {
          const int idx = k + t * P + sub;
          int c;
          float v;
          // idx may run past the chunk (and past lane 63, where lane selects wrap):
          // such padded slots get v = 0 and re-read a row already in flight.
          if constexpr (P == 1) {
            c = readlane_i(mc, idx & 63);  // idx is wave-uniform: scalar row address
            v = readlane_f(mv, idx & 63);
          } else {
            c = __shfl(mc, idx & 63);
            v = __shfl(mv, idx & 63);
          }
          if (idx >= n) {
            c = last_c;
            v = 0.0f;
          }
          vs[t] = v;
          const float* xr = X + (int64_t)c * ldx;
          // a slot past the row end for every lane group (the row's last, partly empty round:
          // 6-7 % of the slots on the Reddit layers) issues no load; its FMA adds 0 * 0, as the
          // loaded-and-masked slot added 0 * x: bit-identical (A/B: layer-0 forward -1 %)
          if (k + t * P >= n) {  // wave-uniform
#pragma unroll
            for (int j = 0; j < NJ; ++j) xs[t][j] = vzero<VW>();
            continue;
          }
          // Columns past F load the row's last vector instead (same cache lines, no
          // branch, no extra HBM bytes); those accumulator slots are never stored.
#pragma unroll
          for (int j = 0; j < NJ; ++j) {
            const int cc = min(c0 + j * G * VW, F - VW);
            xs[t][j] = *reinterpret_cast<const V*>(xr + cc);
          }
        }
        // keep all U * NJ row loads ahead of the FMAs (the scheduler otherwise interleaves
        // them to raise occupancy, leaving fewer loads in flight per wave)
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int t = 0; t < U; ++t) {
#pragma unroll
          for (int j = 0; j < NJ; ++j) acc[j] = vfma(vs[t], xs[t][j], acc[j]);
        }
      }
    }

    if constexpr (P > 1) {
#pragma unroll
      for (int m = G; m < 64; m <<= 1) {
#pragma unroll
        for (int j = 0; j < NJ; ++j) acc[j] += shfl_xor_v(acc[j], m);
      }
    }

    float* dst;
    const float* res = nullptr;  // residual row added to a complete output row
    if (!cut) {
      dst = Y + (int64_t)r * ldy;
      if constexpr (RES) {
        const int q = rmap[r];
        if (q >= 0) res = R + (int64_t)q * ldr;
      }
    } else {
      dst = slab + ((int64_t)u * 2 + (rb < ustart ? 0 : 1)) * ldslab;
    }
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int cc = c0 + j * G * VW;
      if ((j % P) == sub && cc < F) {
        V a = acc[j];
        if constexpr (RES) {
          if (res) a += *reinterpret_cast<const V*>(res + cc);
        }
        *reinterpret_cast<V*>(dst + cc) = a;
      }
    }
  }
}

// Adds the unit pieces of every cut row (> S nonzeros), in unit order. A workgroup covers
// `rows` rows (<= 64): every wave loads their rowptr pairs at once (one dependent round, not one
// per row) and ballots the cut ones; the (cut row, 64*VW-column pass) items are dealt to the 4
// waves, so a cluster of long rows still spreads over the workgroup. 4 rows per workgroup (1 for
// operands under 512 rows): more, smaller workgroups finish sooner beside the concurrent staging
// kernels — combines per step 50.9 (16 rows) vs 45.4 (4 rows) vs 71.9 (32) us, and the layer-2
// forward's 10.7 -> 6.0 us (A/B/A/B under the bench, profiles/round3/spmm/combine_rows_*).
constexpr int COMBINE_ROWS = 4;
constexpr int COMBINE_LOADS = 4;  // pieces of a cut row loaded before they are added
int combine_rows(int64_t M) { return M >= 512 ? COMBINE_ROWS : 1; }

template <int VW, int COMBINE_BATCH>
__global__ __launch_bounds__(256) void spmm_combine_kernel(
    const int* __restrict__ rowptr, int M, int S,
    const float* __restrict__ slab, int64_t ldslab,
    float* __restrict__ Y, int64_t ldy, int F,
    const float* __restrict__ R, int64_t ldr, const int* __restrict__ rmap, int rows) {
  using V = typename Vec<VW>::T;
  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;
  const int r0 = blockIdx.x * rows;
  const int rl = r0 + lane;
  const bool is_cut = lane < rows && rl < M && (rowptr[rl + 1] - rowptr[rl]) > S;  // ownership rule
  const unsigned long long cutmask = __ballot(is_cut);
  if (cutmask == 0ull) return;
  const int npass = (F + 64 * VW - 1) / (64 * VW);
  const int items = __builtin_popcountll(cutmask) * npass;
  for (int it = w; it < items; it += 4) {
    unsigned long long m = cutmask;
    for (int k = it / npass; k > 0; --k) m &= m - 1;  // the (it / npass)-th cut row
    const int r = r0 + __builtin_ctzll(m);
    const int cc = (it % npass) * 64 * VW + lane * VW;
    if (cc >= F) continue;
    const int rb = rowptr[r];
    const int re = rowptr[r + 1];
    const int u0 = rb / S;
    const int u1 = (re - 1) / S;
    const int q = rmap ? rmap[r] : -1;
    {
      // pieces in unit order: slot 1 of u0, then slot 0 of u0 + 1 .. u1, added in that order,
      // COMBINE_BATCH pieces' loads in flight at once (A/B of 2 / 4 / 8 / 16 under the bench,
      // profiles/round3/spmm/combine_loads_r3ar_r3as/: 4 and 8 equal, 2 and 16 slower)
      const int np = u1 - u0 + 1;  // wave-uniform
      V s = vzero<VW>();
      for (int b = 0; b < np; b += COMBINE_BATCH) {
        V a[COMBINE_BATCH];
#pragma unroll
        for (int k = 0; k < COMBINE_BATCH; ++k) {
          const int p = b + k;
          if (p < np) a[k] = *reinterpret_cast<const V*>(slab + ((int64_t)(u0 + p) * 2 + (p == 0 ? 1 : 0)) * ldslab + cc);
        }
#pragma unroll
        for (int k = 0; k < COMBINE_BATCH; ++k) {
          const int p = b + k;
          if (p < np) s = p == 0 ? a[k] : s + a[k];
        }
      }
      if (q >= 0) s += *reinterpret_cast<const V*>(R + (int64_t)q * ldr + cc);
      *reinterpret_cast<V*>(Y + (int64_t)r * ldy + cc) = s;
    }
  }
}

// ---------------------------------------------------------------------------------
// Small operands (the layer-2 calls: 15 k nonzeros, F = 1024): one workgroup of WPR waves per
// (row, column slice of 64 * VW * NJ floats), no work units, no slab, no combine launch.
// The unit kernel's parallelism comes from many equal units; on a 15 k-entry operand it has a
// few thousand short waves, each a chain of dependent loads (row search, (col, val), gathers
// in rounds of U, store) with 4 row loads in flight: 24-25 us per call + a combine launch for
// the cut rows, latency-bound. Here a wave owns one row (WPR = 1) or a contiguous 1/WPR of it
// (long rows: the layer-2 forward's 512 rows reach 484 nonzeros), issues U row loads per lane
// before its FMAs, and the WPR partial rows are added in wave order through LDS by wave 0.
// WPR = 1: every output element is a C fmaf chain over the row in CSR order (bit-identical to
// the oracle); WPR > 1: WPR such chains added in order (deterministic). Empty rows store zeros
// (or the residual row).
// ---------------------------------------------------------------------------------
template <int VW, int NJ, int U, int WPR, bool RES>
__global__ __launch_bounds__(64 * WPR) void spmm_row_kernel(
    const int* __restrict__ rowptr, const int* __restrict__ col, const float* __restrict__ val, int M,
    const float* __restrict__ X, int64_t ldx, float* __restrict__ Y, int64_t ldy, int F, int slices,
    const float* __restrict__ R, int64_t ldr, const int* __restrict__ rmap) {
  using V = typename Vec<VW>::T;
  constexpr int COVER = 64 * VW * NJ;
  __shared__ V part[WPR > 1 ? WPR - 1 : 1][NJ][64];
  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;
  const int r = (int)(blockIdx.x / (unsigned)slices);
  const int s = (int)(blockIdx.x - (unsigned)r * (unsigned)slices);
  if (r >= M) return;
  const int c0 = s * COVER + lane * VW;
  int q = -1;
  if constexpr (RES) q = rmap[r];  // issued early: its latency overlaps the walk
  const int rb = rowptr[r];
  const int re = rowptr[r + 1];
  const int per = (re - rb + WPR - 1) / WPR;
  const int b = rb + w * per;
  const int e = min(re, b + per);
  V acc[NJ];
#pragma unroll
  for (int j = 0; j < NJ; ++j) acc[j] = vzero<VW>();
  for (int base = b; base < e; base += 64) {
    const int n = min(64, e - base);
    int mc = 0;
    float mv = 0.0f;
    if (lane < n) {
      mc = col[base + lane];
      mv = val[base + lane];
    }
    for (int k = 0; k < n; k += U) {
      V xs[U][NJ];
      float vs[U];
#pragma unroll
      for (int t = 0; t < U; ++t) {
        const int idx = k + t;  // wave-uniform
        if (idx >= n) {        // past the chunk: no load, the FMA adds 0 * 0
          vs[t] = 0.0f;
#pragma unroll
          for (int j = 0; j < NJ; ++j) xs[t][j] = vzero<VW>();
          continue;
        }
        const int c = readlane_i(mc, idx);  // scalar row address
        vs[t] = readlane_f(mv, idx);
        const float* xr = X + (int64_t)c * ldx;
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
          const int cc = min(c0 + j * 64 * VW, F - VW);  // past F: the row's last vector (unstored)
          xs[t][j] = *reinterpret_cast<const V*>(xr + cc);
        }
      }
      __builtin_amdgcn_sched_barrier(0);  // all U * NJ row loads ahead of the FMAs
#pragma unroll
      for (int t = 0; t < U; ++t) {
#pragma unroll
        for (int j = 0; j < NJ; ++j) acc[j] = vfma(vs[t], xs[t][j], acc[j]);
      }
    }
  }
  if constexpr (WPR > 1) {
    if (w > 0) {
#pragma unroll
      for (int j = 0; j < NJ; ++j) part[w - 1][j][lane] = acc[j];
    }
    __syncthreads();
    if (w > 0) return;
#pragma unroll
    for (int p = 0; p < WPR - 1; ++p) {  // wave order: deterministic
#pragma unroll
      for (int j = 0; j < NJ; ++j) acc[j] += part[p][j][lane];
    }
  }
  float* dst = Y + (int64_t)r * ldy;
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int cc = c0 + j * 64 * VW;
    if (cc < F) {
      V a = acc[j];
      if constexpr (RES) {
        if (q >= 0) a += *reinterpret_cast<const V*>(R + (int64_t)q * ldr + cc);
      }
      *reinterpret_cast<V*>(dst + cc) = a;
    }
  }
}

// ---------------------------------------------------------------------------------
// Operand builder: value = (float)((1.0 / full_degree(row)) * (double)normfact[col]),
// the formula of cuda_spmm.cu:800 evaluated in double. A flat nnz-balanced pass builds
// every entry; rows found out of column order (never from a scipy-sliced sub-graph, but a
// caller may pass them) are redone by a row-per-wave pass that also sorts them.
// ---------------------------------------------------------------------------------
// Bitonic sort helpers, "all comparators ascending" form: positions >= L act as +inf.
constexpr int SEG_WAVE_LDS = 512;
constexpr int SEG_BLOCK_LDS = 16384;

__device__ __forceinline__ void cmpx_reg(int& k, float& v, int lane, int mask) {
  const int pk = __shfl_xor(k, mask);
  const float pv = __shfl_xor(v, mask);
  const bool lower = lane < (lane ^ mask);
  const bool take = lower ? (pk < k) : (pk > k);
  if (take) {
    k = pk;
    v = pv;
  }
}

// Pair p of a bitonic step -> element positions (i < j).
__device__ __forceinline__ void bitonic_pair(int p, int size, int d, bool flip, int& i, int& j) {
  if (flip) {
    const int half = size >> 1;
    i = (p / half) * size + (p % half);
    j = i ^ (size - 1);
  } else {
    i = (p / d) * (2 * d) + (p % d);
    j = i + d;
  }
}

// One row by one wave: values, a sortedness check and, for an unsorted row, the sort that
// restores the coalesced (column-ascending) order the reference gets from .coalesce():
// in registers (<= 64 entries), in the wave's LDS (<= 512) or in place in global memory.
template <typename CT>
__device__ void build_operand_row(const int* __restrict__ fullrowptr, const int* __restrict__ rowptr,
                                  const CT* __restrict__ colidx, const float* __restrict__ normfact, int r,
                                  int* __restrict__ out_col, float* __restrict__ out_val, int* sk, float* sv,
                                  int lane, unsigned long long* __restrict__ dflag, unsigned long long gen) {
  const int b = rowptr[r];
  const int e = rowptr[r + 1];
  if (b == e) return;
  const double inv = 1.0 / (double)(fullrowptr[r + 1] - fullrowptr[r]);
  bool bad = false;
  for (int i = b + lane; i < e; i += 64) {
    const int c = (int)colidx[i];
    if (i + 1 < e) bad |= c > (int)colidx[i + 1];
    out_col[i] = c;
    out_val[i] = (float)(inv * (double)normfact[c]);
  }
  if (__ballot(bad) == 0ull) return;
  const int L = e - b;
  if (L <= 64) {
    // this wave wrote the row above; re-read it (same lanes' own stores) and sort in registers
    int k = INT_MAX;
    float v = 0.0f;
    if (lane < L) {
      k = (int)colidx[b + lane];
      v = (float)(inv * (double)normfact[k]);
    }
    for (int size = 2; size <= 64; size <<= 1) {
      cmpx_reg(k, v, lane, size - 1);
      for (int d = size >> 2; d >= 1; d >>= 1) cmpx_reg(k, v, lane, d);
    }
    if (lane < L) {
      out_col[b + lane] = k;
      out_val[b + lane] = v;
    }
    // a repeated column, adjacent once sorted: flagged for the caller's lazy coalesce
    const int kn = __shfl_down(k, 1);
    if (dflag && __ballot(lane + 1 < L && k == kn) != 0ull && lane == 0) atomicMax(dflag, gen);
    return;
  }
  // Longer unsorted rows (never produced by scipy slicing, kept for generality): bitonic
  // sort of (column, value) by this wave, in its LDS region (<= 512) or in place in global
  // memory (the lanes' own stores are made visible to the wave by a workgroup fence).
  int n = 1;
  while (n < L) n <<= 1;
  if (L <= SEG_WAVE_LDS) {
    for (int i = lane; i < n; i += 64) {
      const int c = (i < L) ? (int)colidx[b + i] : INT_MAX;
      sk[i] = c;
      sv[i] = (i < L) ? (float)(inv * (double)normfact[c]) : 0.0f;
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
  __builtin_amdgcn_wave_barrier();
  for (int size = 2; size <= n; size <<= 1) {
    for (int d = size >> 1; d >= 1; d >>= 1) {
      const bool flip = (d == (size >> 1));
      for (int p = lane; p < (n >> 1); p += 64) {
        int i, j;
        bitonic_pair(p, size, d, flip, i, j);
        if (L <= SEG_WAVE_LDS) {
          const int ki = sk[i], kj = sk[j];
          if (kj < ki) {
            const float vi = sv[i], vj = sv[j];
            sk[i] = kj;
            sk[j] = ki;
            sv[i] = vj;
            sv[j] = vi;
          }
        } else if (j < L) {
          const int ki = out_col[b + i], kj = out_col[b + j];
          if (kj < ki) {
            const float vi = out_val[b + i], vj = out_val[b + j];
            out_col[b + i] = kj;
            out_col[b + j] = ki;
            out_val[b + i] = vj;
            out_val[b + j] = vi;
          }
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
      __builtin_amdgcn_wave_barrier();
    }
  }
  bool dup = false;
  if (L <= SEG_WAVE_LDS) {
    for (int i = lane; i < L; i += 64) {
      out_col[b + i] = sk[i];
      out_val[b + i] = sv[i];
      dup |= i + 1 < L && sk[i] == sk[i + 1];
    }
  } else {
    for (int i = lane; i + 1 < L; i += 64) dup |= out_col[b + i] == out_col[b + i + 1];
  }
  if (dflag && __ballot(dup) != 0ull && lane == 0) atomicMax(dflag, gen);
}

// Row-per-wave build with the sort fallback; grid-stride over rows. With `flag`, a no-op
// unless the flat builder of the same call (generation `gen`) saw an unsorted row.
template <typename CT>
__global__ __launch_bounds__(256) void build_operand_kernel(
    const int* __restrict__ fullrowptr, const int* __restrict__ rowptr,
    const CT* __restrict__ colidx, const float* __restrict__ normfact, int nrows,
    int* __restrict__ out_col, float* __restrict__ out_val,
    unsigned long long* __restrict__ flag, unsigned long long gen) {
  __shared__ int sk[4][SEG_WAVE_LDS];
  __shared__ float sv[4][SEG_WAVE_LDS];
  if (flag && flag[0] < gen) return;
  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;
  for (int r = blockIdx.x * 4 + w; r < nrows; r += gridDim.x * 4)
    build_operand_row<CT>(fullrowptr, rowptr, colidx, normfact, r, out_col, out_val, sk[w], sv[w], lane,
                          flag ? flag + 1 : nullptr, gen);
}

// nonzeros per wave in the flat operand builders (a multiple of 64)
#ifndef GNN_BUILD_CHUNK
#define GNN_BUILD_CHUNK 64
#endif
constexpr int BUILD_CHUNK = GNN_BUILD_CHUNK;

// Flat build: a wave per 256 consecutive nonzeros (nnz-balanced, ~4 loads in flight per
// lane), each lane finding its row by a short binary search between the chunk's first and
// last rows. Writes col/val for every entry and raises `flag` to `gen` if any row is out of
// order (then the row-per-wave kernel above re-does those rows with their sort).
template <typename CT>
__global__ __launch_bounds__(256) void build_operand_flat_kernel(
    const int* __restrict__ fullrowptr, const int* __restrict__ rowptr,
    const CT* __restrict__ colidx, const float* __restrict__ normfact, int nrows, int nnz,
    int* __restrict__ out_col, float* __restrict__ out_val,
    unsigned long long* __restrict__ flag, unsigned long long gen) {
  const int lane = threadIdx.x & 63;
  const int cs = (blockIdx.x * 4 + (threadIdx.x >> 6)) * BUILD_CHUNK;
  if (cs >= nnz) return;
  const int ce = min(cs + BUILD_CHUNK, nnz);
  const int rf = wave_first_true(0, nrows, lane, [&](int r) { return rowptr[r + 1] > cs; });
  // The ends of rows rf, rf+1, ... one per lane; entry i is in row rf + #{ends <= i}. When
  // fewer than 64 row ends fall inside the chunk that count is a uniform loop over them
  // (no per-entry search of rowptr in global memory).
  const int e = (rf + 1 + lane <= nrows) ? rowptr[rf + 1 + lane] : INT_MAX;
  const int nin = __popcll(__ballot(e < ce));
  int rl = rf;
  if (nin == 64) rl = wave_first_true(rf, nrows, lane, [&](int r) { return rowptr[r + 1] >= ce; });
  bool bad = false, dup = false;
#pragma unroll
  for (int t = 0; t < BUILD_CHUNK / 64; ++t) {
    const int i = cs + t * 64 + lane;
    int k = 0;
    if (nin < 64) {
      for (int j = 0; j < nin; ++j) k += (i >= __builtin_amdgcn_readlane(e, j)) ? 1 : 0;
    }
    const int rend = __shfl(e, k < 64 ? k : 63);
    if (i < ce) {
      int lo = rf + k, end = rend;
      if (nin == 64) {  // the largest r with rowptr[r] <= i is the row holding i
        int hi = rl;
        while (lo < hi) {
          const int mid = (lo + hi + 1) >> 1;
          if (rowptr[mid] <= i) lo = mid; else hi = mid - 1;
        }
        end = rowptr[lo + 1];
      }
      const int c = (int)colidx[i];
      if (i + 1 < end) {
        const int cn = (int)colidx[i + 1];
        bad |= c > cn;
        dup |= c == cn;
      }
      const double inv = 1.0 / (double)(fullrowptr[lo + 1] - fullrowptr[lo]);
      out_col[i] = c;
      out_val[i] = (float)(inv * (double)normfact[c]);
    }
  }
  if (flag && __ballot(bad) != 0ull && lane == 0) atomicMax(flag, gen);
  // word 1: a repeated column in an already ascending row (unsorted rows: checked after their sort)
  if (flag && __ballot(dup) != 0ull && lane == 0) atomicMax(flag + 1, gen);
}

// Values of the transposed operand from its CSR structure (the CSC of A): entry i of
// transposed row c (a column of A) is A's entry (rows[i], c), value
// (float)((1.0 / full_degree(rows[i])) * (double)normfact[c]) — bit-identical to the
// forward operand's value of that entry, so (colptr, rows, val) IS the canonical transpose.
__global__ __launch_bounds__(256) void build_operand_t_kernel(
    const int* __restrict__ fullrowptr, const int* __restrict__ colptr, const int* __restrict__ rows,
    const float* __restrict__ normfact, int ncols, int nnz, float* __restrict__ out_val) {
  const int lane = threadIdx.x & 63;
  const int cs = (blockIdx.x * 4 + (threadIdx.x >> 6)) * BUILD_CHUNK;
  if (cs >= nnz) return;
  const int ce = min(cs + BUILD_CHUNK, nnz);
  const int cf = wave_first_true(0, ncols, lane, [&](int c) { return colptr[c + 1] > cs; });
  // column ends one per lane, as in build_operand_flat_kernel
  const int e = (cf + 1 + lane <= ncols) ? colptr[cf + 1 + lane] : INT_MAX;
  const int nin = __popcll(__ballot(e < ce));
  int cl = cf;
  if (nin == 64) cl = wave_first_true(cf, ncols, lane, [&](int c) { return colptr[c + 1] >= ce; });
#pragma unroll
  for (int t = 0; t < BUILD_CHUNK / 64; ++t) {
    const int i = cs + t * 64 + lane;
    if (i < ce) {
      const int r = rows[i];
      int lo = cf;
      if (nin < 64) {
        for (int j = 0; j < nin; ++j) lo += (i >= __builtin_amdgcn_readlane(e, j)) ? 1 : 0;
      } else {
        int hi = cl;
        while (lo < hi) {
          const int mid = (lo + hi + 1) >> 1;
          if (colptr[mid] <= i) lo = mid; else hi = mid - 1;
        }
      }
      const double inv = 1.0 / (double)(fullrowptr[r + 1] - fullrowptr[r]);
      out_val[i] = (float)(inv * (double)normfact[lo]);
    }
  }
}

// COO index image of a CSR: indices[0][i] = row(i), indices[1][i] = col[i].
__global__ __launch_bounds__(256) void csr_to_coo_indices_kernel(
    const int* __restrict__ rowptr, const int* __restrict__ col, int nrows, int64_t nnz,
    int64_t* __restrict__ indices) {
  const int lane = threadIdx.x & 63;
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= nrows) return;
  const int b = rowptr[r];
  const int e = rowptr[r + 1];
  for (int i = b + lane; i < e; i += 64) {
    indices[i] = r;
    indices[nnz + i] = col[i];
  }
}

// Sorted COO rows -> CSR row pointer by gap filling (thread i owns rows (row[i-1], row[i]]).
__global__ __launch_bounds__(256) void coo_rowptr_kernel(const int64_t* __restrict__ row, int64_t nnz,
                                                         int M, int* __restrict__ rowptr) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i > nnz) return;
  const int64_t prev = (i == 0) ? -1 : row[i - 1];
  const int64_t cur = (i == nnz) ? (int64_t)M : row[i];
  for (int64_t k = prev + 1; k <= cur; ++k) rowptr[k] = (int)i;
}

__global__ __launch_bounds__(256) void narrow_index_kernel(const int64_t* __restrict__ in, int64_t n,
                                                           int* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n) out[i] = (int)in[i];
}

// ---------------------------------------------------------------------------------
// Exclusive scan of n int32 counts into out[0..n] (out[n] = total), one workgroup.
// Optionally also writes the exclusive prefix into out2[0..n-1] (transpose cursors).
// ---------------------------------------------------------------------------------
__global__ __launch_bounds__(1024) void scan_exclusive_kernel(const int* __restrict__ in, int n,
                                                              int* __restrict__ out,
                                                              int* __restrict__ out2) {
  constexpr int ITEMS = 8;
  __shared__ int wsum[16];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  int carry = 0;
  for (int base = 0; base < n; base += 1024 * ITEMS) {
    int v[ITEMS];
    int tsum = 0;
#pragma unroll
    for (int k = 0; k < ITEMS; ++k) {
      const int idx = base + tid * ITEMS + k;
      v[k] = (idx < n) ? in[idx] : 0;
      tsum += v[k];
    }
    int x = tsum;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const int y = __shfl_up(x, d);
      if (lane >= d) x += y;
    }
    if (lane == 63) wsum[wave] = x;
    __syncthreads();
    if (wave == 0) {
      int w = (lane < 16) ? wsum[lane] : 0;
#pragma unroll
      for (int d = 1; d < 16; d <<= 1) {
        const int y = __shfl_up(w, d);
        if (lane >= d) w += y;
      }
      if (lane < 16) wsum[lane] = w;
    }
    __syncthreads();
    int excl = carry + (wave ? wsum[wave - 1] : 0) + x - tsum;
#pragma unroll
    for (int k = 0; k < ITEMS; ++k) {
      const int idx = base + tid * ITEMS + k;
      if (idx < n) {
        out[idx] = excl;
        if (out2) out2[idx] = excl;
      }
      excl += v[k];
    }
    carry += wsum[15];
    __syncthreads();
  }
  if (tid == 0) out[n] = carry;
}

// ---------------------------------------------------------------------------------
// Transpose helpers.
// ---------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void col_count_kernel(const int* __restrict__ col, int64_t nnz,
                                                        int* __restrict__ cnt) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < nnz) atomicAdd(&cnt[col[i]], 1);
}

// Wave per source row: each entry claims a slot in its column's output row. The slot
// order inside an output row is arbitrary here; segsort restores ascending row order.
__global__ __launch_bounds__(256) void transpose_scatter_kernel(
    const int* __restrict__ rowptr, const int* __restrict__ col, const float* __restrict__ val,
    int M, int* __restrict__ cursor, int* __restrict__ tr_col, float* __restrict__ tr_val) {
  const int lane = threadIdx.x & 63;
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= M) return;
  const int b = rowptr[r];
  const int e = rowptr[r + 1];
  for (int i = b + lane; i < e; i += 64) {
    const int pos = atomicAdd(&cursor[col[i]], 1);
    tr_col[pos] = r;
    tr_val[pos] = val[i];
  }
}

// ---------------------------------------------------------------------------------
// Tiled transpose (K <= TR_MAX_K): a stable counting sort by column with no global atomics
// and no sort pass. The nonzeros are cut into T tiles of TS consecutive entries (CSR order).
//  1. tr_tile_hist:   per tile, an LDS histogram of its columns -> hist[t][0..K).
//  2. tr_col_prefix:  per column, exclusive prefix of hist over tiles (in place) -> the
//                     offset of tile t's first entry inside output row c; totals -> cnt.
//     (then scan_exclusive_kernel turns cnt into tr_rowptr.)
//  3. tr_tile_scatter: per tile, LDS cursors cur[c] = tr_rowptr[c] + hist[t][c]; ONE wave
//                     walks the tile's rows in order, one row segment per LDS access, so
//                     the lanes of an access hold distinct columns and rows are placed in
//                     ascending order: the result is the canonical (coalesced) transpose.
// ---------------------------------------------------------------------------------
constexpr int TR_MAX_K = 32 * 1024;   // cursor / histogram array in LDS (128 KiB)
constexpr int TR_MAX_TS = 4 * 1024;   // tile entries preloaded in LDS (32 KiB)

__global__ __launch_bounds__(256) void tr_tile_hist_kernel(const int* __restrict__ col, int nnz, int TS, int K,
                                                           int* __restrict__ hist) {
  extern __shared__ __attribute__((aligned(16))) int lds_i[];
  const int t = blockIdx.x;
  for (int c = threadIdx.x; c < K; c += 256) lds_i[c] = 0;
  __syncthreads();
  const int b = t * TS;
  const int e = min(b + TS, nnz);
  for (int i = b + threadIdx.x; i < e; i += 256) atomicAdd(&lds_i[col[i]], 1);
  __syncthreads();
  int* h = hist + (int64_t)t * K;
  for (int c = threadIdx.x; c < K; c += 256) h[c] = lds_i[c];
}

__global__ __launch_bounds__(256) void tr_col_prefix_kernel(int* __restrict__ hist, int T, int K,
                                                            int* __restrict__ cnt) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= K) return;
  int run = 0;
  int t = 0;
  for (; t + 4 <= T; t += 4) {
    const int64_t o = (int64_t)t * K + c;
    const int h0 = hist[o], h1 = hist[o + K], h2 = hist[o + 2 * (int64_t)K], h3 = hist[o + 3 * (int64_t)K];
    hist[o] = run;
    hist[o + K] = run + h0;
    hist[o + 2 * (int64_t)K] = run + h0 + h1;
    hist[o + 3 * (int64_t)K] = run + h0 + h1 + h2;
    run += h0 + h1 + h2 + h3;
  }
  for (; t < T; ++t) {
    const int64_t o = (int64_t)t * K + c;
    const int h = hist[o];
    hist[o] = run;
    run += h;
  }
  cnt[c] = run;
}

__global__ __launch_bounds__(256) void tr_tile_scatter_kernel(
    const int* __restrict__ rowptr, const int* __restrict__ col, const float* __restrict__ val, int M, int nnz,
    int TS, int K, const int* __restrict__ hist, const int* __restrict__ tr_rowptr, int* __restrict__ tr_col,
    float* __restrict__ tr_val) {
  // LDS: cur[K] cursors, then the tile's columns and values (preloaded by all 4 waves so
  // the ordered walk below reads only LDS and registers).
  extern __shared__ __attribute__((aligned(16))) int cur[];
  int* tcol = cur + ((K + 3) & ~3);
  float* tval = reinterpret_cast<float*>(tcol + TS);
  const int t = blockIdx.x;
  const int b = t * TS;
  const int e = min(b + TS, nnz);
  const int* h = hist + (int64_t)t * K;
  for (int c = threadIdx.x; c < K; c += 256) cur[c] = tr_rowptr[c] + h[c];
  for (int i = b + threadIdx.x; i < e; i += 256) {
    tcol[i - b] = col[i];
    tval[i - b] = val[i];
  }
  __syncthreads();
  if (threadIdx.x >= 64) return;
  const int lane = threadIdx.x;
  // first row with an entry at position >= b; row ends rowptr[r+1..r+64] held in a register
  int r = wave_first_true(0, M, lane, [&](int rr) { return rowptr[rr + 1] > b; });
  int wbase = r;
  int rp = rowptr[min(r + 1 + lane, M)];
  for (int base = b; base < e; base += 64) {
    const int i = base + lane;
    const bool valid = i < e;
    const int c = valid ? tcol[i - b] : 0;
    const float v = valid ? tval[i - b] : 0.0f;
    const int last = min(base + 64, e);  // one past the chunk's last entry
    bool todo = valid;
    while (true) {
      if (r - wbase >= 64) {
        wbase = r;
        rp = rowptr[min(r + 1 + lane, M)];
      }
      const int rend = readlane_i(rp, r - wbase);  // rowptr[r + 1], wave-uniform
      const bool mine = todo && i < rend;
      if (mine) {
        const int p = cur[c];
        cur[c] = p + 1;
        tr_col[p] = r;
        tr_val[p] = v;
      }
      todo = todo && !mine;
      if (rend >= last) break;  // row r continues into (or ends at) the next chunk
      ++r;
    }
  }
}

// ---------------------------------------------------------------------------------
// Segmented sort, ascending by int32 key with an fp32 payload, in place.
// Bitonic network in its "all comparators ascending" form (first step of every merge
// compares mirrored positions), so positions >= L can be treated as +inf and skipped.
// Segments: <=64 in registers, <=512 in a per-wave LDS region, <=16384 by one 1024-thread
// workgroup in LDS, longer ones by one workgroup in global memory. (Helpers: above the
// operand builder, which uses the same network.)
// ---------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void segsort_wave_kernel(const int* __restrict__ ptr, int nseg,
                                                           int* __restrict__ key, float* __restrict__ val,
                                                           int* __restrict__ counters,
                                                           int* __restrict__ list_mid,
                                                           int* __restrict__ list_long) {
  __shared__ int sk[4][SEG_WAVE_LDS];
  __shared__ float sv[4][SEG_WAVE_LDS];
  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;
  const int s = blockIdx.x * 4 + w;
  if (s >= nseg) return;
  const int b = ptr[s];
  const int L = ptr[s + 1] - b;
  if (L <= 1) return;
  // already ascending?
  bool bad = false;
  for (int i = lane; i + 1 < L; i += 64) bad |= key[b + i] > key[b + i + 1];
  if (__ballot(bad) == 0ull) return;

  if (L <= 64) {
    int k = (lane < L) ? key[b + lane] : INT_MAX;
    float v = (lane < L) ? val[b + lane] : 0.0f;
    for (int size = 2; size <= 64; size <<= 1) {
      cmpx_reg(k, v, lane, size - 1);
      for (int d = size >> 2; d >= 1; d >>= 1) cmpx_reg(k, v, lane, d);
    }
    if (lane < L) {
      key[b + lane] = k;
      val[b + lane] = v;
    }
    return;
  }
  if (L <= SEG_WAVE_LDS) {
    int n = 1;
    while (n < L) n <<= 1;
    for (int i = lane; i < n; i += 64) {
      sk[w][i] = (i < L) ? key[b + i] : INT_MAX;
      sv[w][i] = (i < L) ? val[b + i] : 0.0f;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    for (int size = 2; size <= n; size <<= 1) {
      for (int d = size >> 1; d >= 1; d >>= 1) {
        const bool flip = (d == (size >> 1));
        for (int p = lane; p < (n >> 1); p += 64) {
          int i, j;
          bitonic_pair(p, size, d, flip, i, j);
          const int ki = sk[w][i], kj = sk[w][j];
          if (kj < ki) {
            const float vi = sv[w][i], vj = sv[w][j];
            sk[w][i] = kj;
            sk[w][j] = ki;
            sv[w][i] = vj;
            sv[w][j] = vi;
          }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      }
    }
    for (int i = lane; i < L; i += 64) {
      key[b + i] = sk[w][i];
      val[b + i] = sv[w][i];
    }
    return;
  }
  if (lane == 0) {
    if (L <= SEG_BLOCK_LDS) {
      list_mid[atomicAdd(&counters[0], 1)] = s;
    } else {
      list_long[atomicAdd(&counters[1], 1)] = s;
    }
  }
}

__global__ __launch_bounds__(1024) void segsort_block_kernel(const int* __restrict__ ptr,
                                                             int* __restrict__ key, float* __restrict__ val,
                                                             const int* __restrict__ counters,
                                                             const int* __restrict__ list) {
  __shared__ int sk[SEG_BLOCK_LDS];
  __shared__ float sv[SEG_BLOCK_LDS];
  const int count = counters[0];
  for (int t = blockIdx.x; t < count; t += gridDim.x) {
    const int s = list[t];
    const int b = ptr[s];
    const int L = ptr[s + 1] - b;
    int n = 1;
    while (n < L) n <<= 1;
    for (int i = threadIdx.x; i < n; i += 1024) {
      sk[i] = (i < L) ? key[b + i] : INT_MAX;
      sv[i] = (i < L) ? val[b + i] : 0.0f;
    }
    __syncthreads();
    for (int size = 2; size <= n; size <<= 1) {
      for (int d = size >> 1; d >= 1; d >>= 1) {
        const bool flip = (d == (size >> 1));
        for (int p = threadIdx.x; p < (n >> 1); p += 1024) {
          int i, j;
          bitonic_pair(p, size, d, flip, i, j);
          const int ki = sk[i], kj = sk[j];
          if (kj < ki) {
            const float vi = sv[i], vj = sv[j];
            sk[i] = kj;
            sk[j] = ki;
            sv[i] = vj;
            sv[j] = vi;
          }
        }
        __syncthreads();
      }
    }
    for (int i = threadIdx.x; i < L; i += 1024) {
      key[b + i] = sk[i];
      val[b + i] = sv[i];
    }
    __syncthreads();
  }
}

__global__ __launch_bounds__(1024) void segsort_global_kernel(const int* __restrict__ ptr,
                                                              int* __restrict__ key, float* __restrict__ val,
                                                              const int* __restrict__ counters,
                                                              const int* __restrict__ list) {
  const int count = counters[1];
  for (int t = blockIdx.x; t < count; t += gridDim.x) {
    const int s = list[t];
    const int b = ptr[s];
    const int L = ptr[s + 1] - b;
    int64_t n = 1;
    while (n < L) n <<= 1;
    int* K = key + b;
    float* Vv = val + b;
    for (int64_t size = 2; size <= n; size <<= 1) {
      for (int64_t d = size >> 1; d >= 1; d >>= 1) {
        const bool flip = (d == (size >> 1));
        for (int64_t p = threadIdx.x; p < (n >> 1); p += 1024) {
          int64_t i, j;
          if (flip) {
            const int64_t half = size >> 1;
            i = (p / half) * size + (p % half);
            j = i ^ (size - 1);
          } else {
            i = (p / d) * (2 * d) + (p % d);
            j = i + d;
          }
          if (j < L) {
            const int ki = K[i], kj = K[j];
            if (kj < ki) {
              const float vi = Vv[i], vj = Vv[j];
              K[i] = kj;
              K[j] = ki;
              Vv[i] = vj;
              Vv[j] = vi;
            }
          }
        }
        __syncthreads();
      }
    }
  }
}

// ---------------------------------------------------------------------------------
// Feature staging gather/scatter: one wave per row.
// ---------------------------------------------------------------------------------
template <int VW>
__global__ __launch_bounds__(256) void gather_rows_kernel(const float* __restrict__ src, int64_t ld_src,
                                                          const int64_t* __restrict__ src_idx,
                                                          float* __restrict__ dst, int64_t ld_dst,
                                                          const int64_t* __restrict__ dst_idx,
                                                          int64_t n, int F) {
  using V = typename Vec<VW>::T;
  const int lane = threadIdx.x & 63;
  const int64_t i = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (i >= n) return;
  const int64_t s = src_idx ? src_idx[i] : i;
  const int64_t d = dst_idx ? dst_idx[i] : i;
  const float* sr = src + s * ld_src;
  float* dr = dst + d * ld_dst;
  for (int c = lane * VW; c < F; c += 64 * VW) {
    *reinterpret_cast<V*>(dr + c) = *reinterpret_cast<const V*>(sr + c);
  }
}

// X0 from two sources in one launch (round 6): rows [0, n0) from (src0, idx0) and
// rows [n0, n0 + n1) from (src1, idx1), to dst rows pos0 / pos1 — the own feature-buffer rows and
// the batch's host rows of a staging issue. A wave per row with every load of the row issued
// before its stores (608-float rows: 3 float4 per lane).
template <int VW, int NL>
__global__ __launch_bounds__(256) void gather_rows2_kernel(const float* __restrict__ src0, int64_t ld0,
                                                           const int64_t* __restrict__ idx0,
                                                           const int64_t* __restrict__ pos0, int64_t n0,
                                                           const float* __restrict__ src1, int64_t ld1,
                                                           const int64_t* __restrict__ idx1,
                                                           const int64_t* __restrict__ pos1, int64_t n1,
                                                           float* __restrict__ dst, int64_t ld_dst, int F) {
  using V = typename Vec<VW>::T;
  const int lane = threadIdx.x & 63;
  int64_t i = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (i >= n0 + n1) return;
  const bool second = i >= n0;  // wave-uniform
  if (second) i -= n0;
  const float* sr;
  int64_t d;
  if (!second) {
    sr = src0 + (idx0 ? idx0[i] : i) * ld0;
    d = pos0 ? pos0[i] : i;
  } else {
    sr = src1 + (idx1 ? idx1[i] : i) * ld1;
    d = pos1 ? pos1[i] : i;
  }
  float* dr = dst + d * ld_dst;
  V v[NL];
#pragma unroll
  for (int k = 0; k < NL; ++k) {
    const int c = (lane + 64 * k) * VW;
    if (c < F) v[k] = *reinterpret_cast<const V*>(sr + c);
  }
#pragma unroll
  for (int k = 0; k < NL; ++k) {
    const int c = (lane + 64 * k) * VW;
    if (c < F) *reinterpret_cast<V*>(dr + c) = v[k];
  }
}

// Rows read straight from pinned, device-mapped host memory (zero-copy over PCIe): a small
// persistent grid (each wave two rows per pass, every load of both rows issued before the
// first store) keeps a few MB of PCIe reads in flight while holding few CU slots, so the
// gather runs on the staging stream beside the compute kernels.
// Measured on MI355X (Reddit batch, 31 MB of host rows): 46-51 GB/s at 32-128 workgroups,
// 24 GB/s at 8 — but the PCIe reads slow the concurrent compute kernels (GPU step 2.18 ->
// 2.50-2.64 ms at every grid tried), so bench.py defaults to the pinned-copy path.
constexpr int HOST_GATHER_GRID = 32;

template <int VW>
__global__ __launch_bounds__(256) void gather_rows_host_kernel(const float* __restrict__ src, int64_t ld_src,
                                                               const int64_t* __restrict__ src_idx,
                                                               float* __restrict__ dst, int64_t ld_dst,
                                                               const int64_t* __restrict__ dst_idx, int64_t n, int F) {
  using V = typename Vec<VW>::T;
  constexpr int CH = 3;  // 64 * VW-float chunks per row held in registers (608 floats at VW 4)
  const int lane = threadIdx.x & 63;
  const int64_t w = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int64_t nw = (int64_t)gridDim.x * 4;
  for (int64_t i0 = 2 * w; i0 < n; i0 += 2 * nw) {
    V v[2][CH];
    const float* sr[2];
    float* dr[2];
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int64_t i = min(i0 + q, n - 1);  // an odd last row is simply copied twice
      sr[q] = src + (src_idx ? src_idx[i] : i) * ld_src;
      dr[q] = dst + (dst_idx ? dst_idx[i] : i) * ld_dst;
    }
#pragma unroll
    for (int q = 0; q < 2; ++q)
#pragma unroll
      for (int j = 0; j < CH; ++j) {
        const int c = (lane + 64 * j) * VW;
        if (c < F) v[q][j] = *reinterpret_cast<const V*>(sr[q] + c);
      }
#pragma unroll
    for (int q = 0; q < 2; ++q) {
#pragma unroll
      for (int j = 0; j < CH; ++j) {
        const int c = (lane + 64 * j) * VW;
        if (c < F) *reinterpret_cast<V*>(dr[q] + c) = v[q][j];
      }
      for (int c = (lane + 64 * CH) * VW; c < F; c += 64 * VW)  // rows wider than CH chunks
        *reinterpret_cast<V*>(dr[q] + c) = *reinterpret_cast<const V*>(sr[q] + c);
    }
  }
}

// ---------------------------------------------------------------------------------
// Host-side configuration and dispatch.
// ---------------------------------------------------------------------------------
struct SpmmCfg {
  int vw, g, nj, tiles;
  int64_t unit, nunits, ldslab;
  // small operands: spmm_row_kernel<vw, rnj, ru, wpr> over M * slices workgroups (wpr == 0: the
  // unit kernel above)
  int wpr, rnj, ru, slices;
  // small operands cut into 256-float column tiles (small_tiles): 16 nonzeros in flight per lane
  // instead of 4 (their units are short chains of latency-bound rounds)
  bool u16;
};

// The row kernel takes operands whose nonzeros are too few to fill the chip with units: up to
// ROWK_MAX_NNZ nonzeros and ROWK_MAX_WG workgroups (GNN_SPMM_ROWK=0 / 1 forces it off / on when
// the caller did not fix the unit size).
constexpr int64_t ROWK_MAX_NNZ = 65536;
constexpr int64_t ROWK_MAX_WG = 1 << 20;

void pick_row_kernel(SpmmCfg& c, int64_t M, int64_t nnz, int64_t F, int64_t unit) {
  c.wpr = 0;
  if (unit > 0 || M <= 0 || F <= 0) return;  // a fixed unit size asks for the unit kernel
  const char* env = getenv("GNN_SPMM_ROWK");
  const int mode = env ? atoi(env) : -1;
  if (mode == 0) return;
  const int64_t chunks = ceil_div(F, (int64_t)64 * c.vw);  // 64-lane column chunks covering F
  // many rows: whole rows per wave, up to 4 chunks per lane; few rows: one chunk per slice
  int nj = 1;
  if (c.vw == 4 && M >= 4096) nj = chunks >= 4 ? 4 : (chunks >= 2 ? 2 : 1);
  const int64_t slices = ceil_div(chunks, (int64_t)nj);
  const double avg = (double)nnz / (double)M;
  // Measured on the layer-2 calls (profiles/round4/layer2/): short rows (the backward's Aᵀ, 1.7
  // nonzeros per row) 12.7-13.7 us with 1-2 waves per row against 25 us for units + combine;
  // long-tailed rows (the forward's A, 29 per row, up to 484) 20.4 us at best (8 waves per row)
  // against 19.5 for units + combine — so by default only short-row operands take this kernel,
  // with one wave per row (each output a C fmaf chain: the executor folds such a call into the
  // tail that consumes it, gnn_sage_norm_bwd_agg_f32, bit for bit).
  // (round 5: a dynamic form, one wave per 8 nonzeros of a row up to 16 per workgroup, took the
  // layer-2 forward to 49 us in the step against 23 for units + combine: not kept)
  if (mode != 1 && avg >= 12.0) return;
  int wpr = avg >= 48.0 ? 8 : (avg >= 12.0 ? 4 : 1);
  if (const char* e = getenv("GNN_SPMM_ROWK_WPR")) {  // experiments
    const int v = atoi(e);
    if (v == 1 || v == 2 || v == 4 || v == 8) wpr = v;
  }
  if (mode != 1 && (nnz > ROWK_MAX_NNZ || M * slices > ROWK_MAX_WG)) return;
  if (M * slices >= (int64_t)INT_MAX) return;
  c.wpr = wpr;
  c.rnj = nj;
  c.ru = nj == 1 ? 16 : (nj == 2 ? 8 : 4);
  c.slices = (int)slices;
}

int pick_vw(int64_t F, int64_t ldx, int64_t ldy, const void* X, const void* Y) {
  const uintptr_t px = (uintptr_t)X, py = (uintptr_t)Y;
  if (F % 4 == 0 && ldx % 4 == 0 && ldy % 4 == 0 && px % 16 == 0 && py % 16 == 0) return 4;
  if (F % 2 == 0 && ldx % 2 == 0 && ldy % 2 == 0 && px % 8 == 0 && py % 8 == 0) return 2;
  return 1;
}

// About 2.4 rows' worth of nonzeros as a power of two in [16, 256] (see default_unit).
int64_t row_unit(int64_t M, int64_t nnz) {
  int64_t s = 256;
  if (M > 0) {
    const double want = 2.4 * (double)nnz / (double)M;
    while (s > 16 && (double)s > want * 1.41421356) s >>= 1;
  }
  return s;
}

// Small operands (fewer than 2048 row-sized units) take their parallelism from 256-float
// column tiles before cutting rows into pieces: the layer-2 forward (512 rows of ~30
// nonzeros, F = 1024) had 2048 units of 8 nonzeros, every row cut and recombined (14 + 17 us).
// (Operands with < 16 nonzeros per row keep their two-rows-per-unit path.)
int64_t small_tiles(int64_t M, int64_t nnz, int64_t F) {
  if (F < 512 || nnz <= 0 || nnz < 16 * M || ceil_div(nnz, row_unit(M, nnz)) >= 2048) return 1;
  return std::min<int64_t>(F / 256, 8);
}

int64_t default_unit(int64_t M, int64_t nnz, int64_t F) {
  // Units are equal-sized (S nonzeros), which balances power-law rows by construction.
  // Measured on the Reddit LADIES layers (scripts/spmm_microbench.py, with L2 column
  // tiles): S = 256 is the sweet spot between per-row flush/search overhead (small S) and
  // too few waves per column-tile pass (large S: layer-1 forward 262 us at S = 404 vs
  // 208 us at 256). Small problems keep >= 2048 units for parallelism, S >= 16. Operands
  // with < 16 nonzeros per row on average are mostly output rows to write (the layer-2
  // backward: 8.7 k rows, 1.7 nonzeros each): about two rows per unit, S >= 4 (18 vs 23 us).
  // About 2.4 rows per unit, as a power of two in [16, 256]: the layer-1 backward operand
  // (54 nonzeros per row) 199 us at S = 128 vs 209 at 256; the forward operands (98-114 per
  // row) keep 256.
  int64_t s = row_unit(M, nnz);
  const int64_t t = small_tiles(M, nnz, F);
  if (ceil_div(nnz, s) * t < 2048) s = ceil_div(nnz * t, 2048);
  if (s < 16) s = 16;
  if (M > 0 && nnz < 16 * M) {
    const int64_t r = 2 * nnz / M;
    s = std::min<int64_t>(s, r < 4 ? 4 : r);
  }
  return s;
}

SpmmCfg make_cfg(int64_t M, int64_t K, int64_t nnz, int64_t F, int64_t ldx, int64_t ldy, const void* X,
                 const void* Y, int64_t unit) {
  SpmmCfg c{};
  c.vw = pick_vw(F, ldx, ldy, X, Y);
  double best = -1.0;
  const int gs[3] = {64, 32, 16};
  for (int gi = 0; gi < 3; ++gi) {
    const int g = gs[gi];
    const int64_t lanecols = (int64_t)c.vw * g;
    const int64_t tiles = ceil_div(F, lanecols * 8) > 0 ? ceil_div(F, lanecols * 8) : 1;
    int64_t nj = ceil_div(F, lanecols * tiles);
    if (nj < 1) nj = 1;
    const double util = (double)F / (double)(tiles * lanecols * nj);
    if (util > best + 1e-9) {
      best = util;
      c.g = g;
      c.nj = (int)nj;
      c.tiles = (int)tiles;
    }
  }
  // L2-sized column tiles. Each XCD's 4 MiB L2 sees random rows of X; when X rows are
  // re-read many times (nnz/K >= 8) cut the columns into tiles whose slice of X
  // (K rows x tile width) is about one L2, processed tile after tile (grid.y is the slow
  // dispatch dimension), so re-reads hit L2 instead of the Infinity Cache. Measured on the
  // Reddit LADIES layers: 1.3-1.9x.
  if (K > 0 && nnz >= 8 * K) {
    const double target_cols = (4.0 * 1024 * 1024 / 4.0) / (double)K;  // floats per row slice
    int64_t cols = (int64_t)c.vw * 16;                                    // smallest: G=16, NJ=1
    while (cols * 2 <= F && (double)(cols * 2) <= target_cols * 1.41421356) cols *= 2;
    if (cols < F) {
      const int64_t per = cols / c.vw;  // lanes x chunks
      c.g = per >= 64 ? 64 : (int)per;
      c.nj = per >= 64 ? (int)(per / 64) : 1;
      if (c.nj > 8) c.nj = 8;
      c.tiles = (int)ceil_div(F, (int64_t)c.vw * c.g * c.nj);
    }
  }
  // Small operands: 256-float column tiles (G = 64, one chunk) for parallelism (small_tiles).
  c.u16 = false;
  if (c.vw == 4 && c.tiles == 1) {
    const int64_t t = small_tiles(M, nnz, F);
    if (t > 1) {
      c.g = 64;
      c.nj = 1;
      c.tiles = (int)ceil_div(F, (int64_t)256);
      const char* e = getenv("GNN_SPMM_SMALL_U16");  // A/B
      c.u16 = !(e && atoi(e) == 0);
    }
  }
  // Experiment override (benchmarks only): GNN_SPMM_G / GNN_SPMM_NJ force the lane group
  // and column chunks; F is then covered by ceil(F / (VW*G*NJ)) column tiles (grid.y).
  if (const char* eg = getenv("GNN_SPMM_G")) {
    const int g = atoi(eg);
    const char* en = getenv("GNN_SPMM_NJ");
    const int nj = en ? atoi(en) : 1;
    const char* ev = getenv("GNN_SPMM_VW");
    if (ev && atoi(ev) >= 1 && atoi(ev) < c.vw && (atoi(ev) & (atoi(ev) - 1)) == 0) c.vw = atoi(ev);
    if ((g == 8 || g == 16 || g == 32 || g == 64) && nj >= 1 && nj <= 8) {
      c.g = g;
      c.nj = nj;
      c.tiles = (int)ceil_div(F, (int64_t)c.vw * g * nj);
    }
  }
  c.unit = unit > 0 ? unit : default_unit(M, nnz, F);
  c.nunits = nnz > 0 ? ceil_div(nnz, c.unit) : 1;
  c.ldslab = (int64_t)align_up((size_t)(F > 0 ? F : 1), 4);
  pick_row_kernel(c, M, nnz, F, unit);
  return c;
}

// The XCD map pays when a column tile's slice of X is re-read (several tiles, many units);
// GNN_SPMM_XCD=0/1 forces it off/on (measurements).
WorkMap work_map(const SpmmCfg& c, int64_t M) {
  WorkMap wm{};
  wm.gx = (int)ceil_div(c.nunits + ceil_div(M, (int64_t)ROW_UNIT), 4);
  wm.items = wm.gx * c.tiles;
  bool on = c.tiles > 1;
  if (const char* e = getenv("GNN_SPMM_XCD")) on = atoi(e) != 0;
  wm.xcd_chunk = on ? (int)ceil_div(wm.items, 8) : 0;
  return wm;
}

using MainFn = void (*)(const int*, const int*, const float*, int, int, int, int, const float*, int64_t,
                        float*, int64_t, float*, int64_t, int, const float*, int64_t, const int*, WorkMap);

#ifndef GNN_SPMM_U1  // nonzeros in flight per lane group for one column chunk (experiments: -DGNN_SPMM_U1=n)
#define GNN_SPMM_U1 4
#endif
constexpr int pick_u(int nj) { return nj <= 1 ? GNN_SPMM_U1 : (nj <= 4 ? 4 : (nj == 5 ? 3 : 2)); }

template <int VW, int G, int NJ>
MainFn main_ptr(bool res) {
  return res ? &spmm_unit_kernel<VW, G, NJ, pick_u(NJ), true> : &spmm_unit_kernel<VW, G, NJ, pick_u(NJ), false>;
}

template <int VW, int G>
MainFn main_by_nj(int nj, bool res) {
  switch (nj) {
    case 1: return main_ptr<VW, G, 1>(res);
    case 2: return main_ptr<VW, G, 2>(res);
    case 3: return main_ptr<VW, G, 3>(res);
    case 4: return main_ptr<VW, G, 4>(res);
    case 5: return main_ptr<VW, G, 5>(res);
    case 6: return main_ptr<VW, G, 6>(res);
    case 7: return main_ptr<VW, G, 7>(res);
    case 8: return main_ptr<VW, G, 8>(res);
    default: return nullptr;
  }
}

template <int VW>
MainFn main_by_g(int g, int nj, bool res) {
  switch (g) {
    case 64: return main_by_nj<VW, 64>(nj, res);
    case 32: return main_by_nj<VW, 32>(nj, res);
    case 16: return main_by_nj<VW, 16>(nj, res);
    case 8: return main_by_nj<VW, 8>(nj, res);
    default: return nullptr;
  }
}

// res: the row-mapped residual variant (gnn_spmm_csr_f32_ex); a separate instantiation, so
// the plain aggregation carries no residual code and the two show up apart in rocprofv3.
MainFn select_main(const SpmmCfg& c, bool res) {
  if (c.u16 && c.vw == 4 && c.g == 64 && c.nj == 1)
    return res ? &spmm_unit_kernel<4, 64, 1, 16, true> : &spmm_unit_kernel<4, 64, 1, 16, false>;
  switch (c.vw) {
    case 4: return main_by_g<4>(c.g, c.nj, res);
    case 2: return main_by_g<2>(c.g, c.nj, res);
    case 1: return main_by_g<1>(c.g, c.nj, res);
    default: return nullptr;
  }
}

using RowFn = void (*)(const int*, const int*, const float*, int, const float*, int64_t, float*, int64_t, int, int,
                      const float*, int64_t, const int*);

template <int VW, int NJ, int U>
RowFn row_by_wpr(int wpr, bool res) {
  switch (wpr) {
    case 1: return res ? &spmm_row_kernel<VW, NJ, U, 1, true> : &spmm_row_kernel<VW, NJ, U, 1, false>;
    case 2: return res ? &spmm_row_kernel<VW, NJ, U, 2, true> : &spmm_row_kernel<VW, NJ, U, 2, false>;
    case 4: return res ? &spmm_row_kernel<VW, NJ, U, 4, true> : &spmm_row_kernel<VW, NJ, U, 4, false>;
    case 8: return res ? &spmm_row_kernel<VW, NJ, U, 8, true> : &spmm_row_kernel<VW, NJ, U, 8, false>;
    default: return nullptr;
  }
}

RowFn select_row(const SpmmCfg& c, bool res) {
  if (c.vw == 4) {
    if (c.rnj == 4) return row_by_wpr<4, 4, 4>(c.wpr, res);
    if (c.rnj == 2) return row_by_wpr<4, 2, 8>(c.wpr, res);
    return row_by_wpr<4, 1, 16>(c.wpr, res);
  }
  if (c.rnj != 1) return nullptr;
  if (c.vw == 2) return row_by_wpr<2, 1, 16>(c.wpr, res);
  return row_by_wpr<1, 1, 16>(c.wpr, res);
}

// The main kernel's name as rocprofv3 lists it (bench.py's per-kernel roofline).
std::string main_kernel_name(const SpmmCfg& c, bool res) {
  char b[96];
  if (c.wpr)
    snprintf(b, sizeof b, "spmm_row_kernel<%d, %d, %d, %d, %s>", c.vw, c.rnj, c.ru, c.wpr, res ? "true" : "false");
  else
    snprintf(b, sizeof b, "spmm_unit_kernel<%d, %d, %d, %d, %s>", c.vw, c.g, c.nj,
             (c.u16 && c.vw == 4 && c.g == 64 && c.nj == 1) ? 16 : pick_u(c.nj), res ? "true" : "false");
  return b;
}

void tr_tiles(int64_t nnz, int64_t& TS, int64_t& T) {
  TS = ceil_div(nnz, 256);
  if (TS < 1024) TS = 1024;
  if (TS > TR_MAX_TS) TS = TR_MAX_TS;
  T = nnz > 0 ? ceil_div(nnz, TS) : 0;
}

size_t segsort_ws(int64_t nseg) { return 256 + align_up((size_t)(nseg > 0 ? nseg : 1) * 4, 256) * 2; }

struct SegLists {
  int* counters;
  int* list_mid;
  int* list_long;
};

SegLists seg_lists(void* ws, int64_t nseg) {
  char* w = (char*)ws;
  return SegLists{(int*)w, (int*)(w + 256), (int*)(w + 256 + align_up((size_t)(nseg > 0 ? nseg : 1) * 4, 256))};
}

// Sort the queued segments: the workgroup (LDS) sorter for counters[0] entries, the
// global-memory sorter for counters[1]. Small grids: they loop over the (usually empty)
// lists, reading the counts on the device (no host synchronisation).
int run_list_sorters(const int* ptr, int* key, float* val, const SegLists& l, hipStream_t st) {
  segsort_block_kernel<<<dim3(16), dim3(1024), 0, st>>>(ptr, key, val, l.counters, l.list_mid);
  GNN_LAUNCHED("segsort_block_kernel");
  segsort_global_kernel<<<dim3(4), dim3(1024), 0, st>>>(ptr, key, val, l.counters, l.list_long);
  GNN_LAUNCHED("segsort_global_kernel");
  return 0;
}

int run_segsort(const int* ptr, int64_t nseg, int* key, float* val, void* ws, hipStream_t st) {
  if (nseg <= 0) return 0;
  const SegLists l = seg_lists(ws, nseg);
  GNN_HIP(hipMemsetAsync(l.counters, 0, 16, st), "segsort counters memset");
  segsort_wave_kernel<<<dim3((unsigned)ceil_div(nseg, 4)), dim3(256), 0, st>>>(ptr, (int)nseg, key, val, l.counters,
                                                                            l.list_mid, l.list_long);
  GNN_LAUNCHED("segsort_wave_kernel");
  int rc = run_list_sorters(ptr, key, val, l, st);
  if (rc) return rc;
  return 0;
}

}  // namespace

bool gnn::spmm_row_chain(int64_t M, int64_t K, int64_t nnz, int64_t F, int64_t ldx, int64_t ldy, const void* X,
                         const void* Y) {
  const SpmmCfg c = make_cfg(M, K, nnz, F, ldx, ldy, X, Y, 0);
  return c.wpr == 1 && c.vw == 4;
}

int gnn::launch_scan_exclusive(const int* in, int n, int* out, hipStream_t st) {
  scan_exclusive_kernel<<<dim3(1), dim3(1024), 0, st>>>(in, n, out, nullptr);
  GNN_LAUNCHED("scan_exclusive_kernel");
  return 0;
}

// =================================================================================
// C ABI
// =================================================================================
extern "C" {

const char* gnn_last_error(void) { return g_err.c_str(); }

const char* gnn_version(void) { return "gnn_spmm gfx950 " GNN_BUILD_ID; }

int64_t gnn_spmm_default_unit_nnz(int64_t M, int64_t nnz, int64_t F) { return default_unit(M, nnz, F); }

size_t gnn_spmm_workspace_bytes(int64_t M, int64_t nnz, int64_t F, int64_t unit_nnz) {
  const SpmmCfg c = make_cfg(M, 0, nnz, F, F, F, nullptr, nullptr, unit_nnz);
  // (the row kernel needs none; the size stays the unit kernel's, which a call with other
  // strides / alignment may take)
  return align_up((size_t)c.nunits * 2 * (size_t)c.ldslab * sizeof(float), 256);
}

int gnn_spmm_kernel_name(int64_t M, int64_t K, int64_t nnz, int64_t F, int64_t ldx, int64_t ldy, const void* X,
                         const void* Y, int64_t unit_nnz, int residual, char* out, size_t out_bytes) {
  GNN_REQUIRE(out != nullptr && out_bytes > 0, "gnn_spmm_kernel_name: out is NULL");
  const std::string n = main_kernel_name(make_cfg(M, K, nnz, F, ldx, ldy, X, Y, unit_nnz), residual != 0);
  snprintf(out, out_bytes, "%s", n.c_str());
  return 0;
}

int gnn_spmm_config(int64_t M, int64_t K, int64_t nnz, int64_t F, int64_t ldx, int64_t ldy, const void* X,
                    const void* Y, int64_t unit_nnz, int32_t out[6]) {
  GNN_REQUIRE(out != nullptr, "gnn_spmm_config: out is NULL");
  const SpmmCfg c = make_cfg(M, K, nnz, F, ldx, ldy, X, Y, unit_nnz);
  out[0] = c.vw;
  out[1] = c.g;
  out[2] = c.nj;
  out[3] = c.tiles;
  out[4] = (int32_t)c.unit;
  out[5] = (int32_t)c.nunits;
  return 0;
}

void gnn_spmm_set_timing_events(void* start, void* stop) {
  g_ev_start = (hipEvent_t)start;
  g_ev_stop = (hipEvent_t)stop;
}

int gnn_spmm_csr_f32(const int32_t* rowptr, const int32_t* col, const float* val, int64_t M, int64_t K,
                     int64_t nnz, const float* X, int64_t ldx, float* Y, int64_t ldy, int64_t F,
                     void* workspace, size_t workspace_bytes, int64_t unit_nnz, void* stream) {
  return gnn_spmm_csr_f32_ex(rowptr, col, val, M, K, nnz, X, ldx, Y, ldy, F, nullptr, 0, nullptr, workspace,
                             workspace_bytes, unit_nnz, stream);
}

int gnn_spmm_csr_f32_ex(const int32_t* rowptr, const int32_t* col, const float* val, int64_t M, int64_t K,
                        int64_t nnz, const float* X, int64_t ldx, float* Y, int64_t ldy, int64_t F,
                        const float* R, int64_t ldr, const int32_t* rmap, void* workspace, size_t workspace_bytes,
                        int64_t unit_nnz, void* stream) {
  hipEvent_t ev0 = g_ev_start, ev1 = g_ev_stop;
  g_ev_start = g_ev_stop = nullptr;
  GNN_REQUIRE(M >= 0 && K >= 0 && nnz >= 0 && F >= 0, "gnn_spmm_csr_f32: negative size");
  GNN_REQUIRE(M < INT_MAX && K < INT_MAX && nnz < INT_MAX, "gnn_spmm_csr_f32: M, K, nnz must be < 2^31");
  GNN_REQUIRE(F <= ldx || K == 0, "gnn_spmm_csr_f32: F (%lld) > ldx (%lld)", (long long)F, (long long)ldx);
  GNN_REQUIRE(F <= ldy || M == 0, "gnn_spmm_csr_f32: F (%lld) > ldy (%lld)", (long long)F, (long long)ldy);
  if (M == 0 || F == 0) return 0;
  GNN_REQUIRE(rowptr && Y, "gnn_spmm_csr_f32: NULL rowptr/Y");
  GNN_REQUIRE(nnz == 0 || (col && val && X), "gnn_spmm_csr_f32: NULL col/val/X");
  GNN_REQUIRE(rmap == nullptr || (R != nullptr && F <= ldr), "gnn_spmm_csr_f32_ex: rmap needs R with F <= ldr");
  const SpmmCfg c = make_cfg(M, K, nnz, F, ldx, ldy, X, Y, unit_nnz);
  hipStream_t st = (hipStream_t)stream;
  if (c.wpr) {  // small operand: one workgroup per (row, column slice), nothing to combine
    GNN_REQUIRE(rmap == nullptr || (ldr % c.vw == 0 && (uintptr_t)R % (4 * c.vw) == 0),
                "gnn_spmm_csr_f32_ex: R (ldr %lld) not aligned for %d-wide vectors", (long long)ldr, c.vw);
    RowFn fn = select_row(c, rmap != nullptr);
    GNN_REQUIRE(fn != nullptr, "gnn_spmm_csr_f32: no row kernel for vw=%d nj=%d wpr=%d", c.vw, c.rnj, c.wpr);
    // timing (gnn_spmm_set_timing_events): the events take the dispatch's own start / end
    // timestamps (hipExtLaunchKernel), the kernel's duration as rocprofv3 reports it — not an
    // event pair around the launch, which also brackets the queue's event packets (~7 us each)
    if (ev0 || ev1)
      hipExtLaunchKernelGGL(fn, dim3((unsigned)(M * c.slices)), dim3(64 * c.wpr), 0, st, ev0, ev1, 0, rowptr, col, val,
                            (int)M, X, ldx, Y, ldy, (int)F, c.slices, R, ldr, (const int*)rmap);
    else
      hipLaunchKernelGGL(fn, dim3((unsigned)(M * c.slices)), dim3(64 * c.wpr), 0, st, rowptr, col, val, (int)M, X, ldx,
                         Y, ldy, (int)F, c.slices, R, ldr, (const int*)rmap);
    GNN_LAUNCHED("spmm_row_kernel");
    return 0;
  }
  GNN_REQUIRE(c.nunits * c.unit < (int64_t)INT_MAX + c.unit, "gnn_spmm_csr_f32: unit overflow");
  GNN_REQUIRE(c.nunits <= (int64_t)INT_MAX / 2, "gnn_spmm_csr_f32: too many units");
  const size_t need = align_up((size_t)c.nunits * 2 * (size_t)c.ldslab * sizeof(float), 256);
  const bool any_split = c.nunits > 1;
  GNN_REQUIRE(!any_split || (workspace && workspace_bytes >= need),
              "gnn_spmm_csr_f32: workspace too small (%zu < %zu)", workspace_bytes, need);
  GNN_REQUIRE((uintptr_t)workspace % 16 == 0, "gnn_spmm_csr_f32: workspace not 16-byte aligned");
  GNN_REQUIRE(rmap == nullptr || (ldr % c.vw == 0 && (uintptr_t)R % (4 * c.vw) == 0),
              "gnn_spmm_csr_f32_ex: R (ldr %lld) not aligned for %d-wide vectors", (long long)ldr, c.vw);
  MainFn fn = select_main(c, rmap != nullptr);
  GNN_REQUIRE(fn != nullptr, "gnn_spmm_csr_f32: no kernel for vw=%d g=%d nj=%d", c.vw, c.g, c.nj);
  float* slab = (float*)workspace;
  GNN_REQUIRE(ceil_div(c.nunits + ceil_div(M, (int64_t)ROW_UNIT), 4) * c.tiles < (int64_t)INT_MAX - 8,
              "gnn_spmm_csr_f32: grid too large");
  const WorkMap wm = work_map(c, M);
  const dim3 grid((unsigned)(wm.xcd_chunk ? 8 * (int64_t)wm.xcd_chunk : wm.items));
  if (ev0 || ev1)  // the dispatch's own start / end timestamps (see the row kernel above)
    hipExtLaunchKernelGGL(fn, grid, dim3(256), 0, st, ev0, ev1, 0, rowptr, col, val, (int)M, (int)nnz, (int)c.unit,
                          (int)c.nunits, X, ldx, Y, ldy, slab, c.ldslab, (int)F, R, ldr, (const int*)rmap, wm);
  else
    hipLaunchKernelGGL(fn, grid, dim3(256), 0, st, rowptr, col, val, (int)M, (int)nnz, (int)c.unit,
                       (int)c.nunits, X, ldx, Y, ldy, slab, c.ldslab, (int)F, R, ldr, (const int*)rmap, wm);
  GNN_LAUNCHED("spmm_unit_kernel");
  if (any_split) {
    int crows = combine_rows(M);
    if (const char* e = getenv("GNN_SPMM_CROWS")) crows = std::min(64, std::max(1, atoi(e)));  // A/B
    const dim3 g2((unsigned)ceil_div(M, (int64_t)crows));
    auto combine = [&](auto kern) {
      kern<<<g2, dim3(256), 0, st>>>(rowptr, (int)M, (int)c.unit, slab, c.ldslab, Y, ldy, (int)F, R, ldr,
                                     (const int*)rmap, crows);
    };
    // (round 5: for the layer-2 forward, every piece of a pass in flight and a row per workgroup
    // measured equal under the bench — 573.5 / 570.8 vs 574.0 / 570.7 gpu_step: not kept)
    if (c.vw == 4) combine(spmm_combine_kernel<4, COMBINE_LOADS>);
    else if (c.vw == 2) combine(spmm_combine_kernel<2, COMBINE_LOADS>);
    else combine(spmm_combine_kernel<1, COMBINE_LOADS>);
    GNN_LAUNCHED("spmm_combine_kernel");
  }
  return 0;
}

size_t gnn_segsort_workspace_bytes(int64_t nseg) { return segsort_ws(nseg); }

namespace {
int build_operand(const int32_t* fullrowptr, const int32_t* rowptr, const void* colidx, int colidx_bytes,
                  const float* normfact, int64_t nrows, int64_t ncols, int64_t nnz, int32_t* csr_col, float* csr_val,
                  int64_t* coo_indices, unsigned long long* flag, void* stream);
}  // namespace

size_t gnn_build_operand_workspace_bytes(void) { return 256; }

int gnn_build_operand_f32(const int32_t* fullrowptr, const int32_t* rowptr, const void* colidx, int colidx_bytes,
                          const float* normfact, int64_t nrows, int64_t ncols, int64_t nnz, int32_t* csr_col,
                          float* csr_val, int64_t* coo_indices, void* workspace, size_t workspace_bytes,
                          void* stream) {
  // the "unsorted row seen" and "repeated column seen" words live in the caller's workspace,
  // zeroed on the call's stream: no allocation inside the library, no state shared between
  // concurrent calls
  GNN_REQUIRE(nrows == 0 || nnz == 0 || (workspace != nullptr && workspace_bytes >= 16 && (uintptr_t)workspace % 8 == 0),
              "gnn_build_operand_f32: needs an 8-byte aligned workspace of gnn_build_operand_workspace_bytes() bytes");
  return build_operand(fullrowptr, rowptr, colidx, colidx_bytes, normfact, nrows, ncols, nnz, csr_col, csr_val,
                       coo_indices, (unsigned long long*)workspace, stream);
}

int gnn_build_operand_sorted_f32(const int32_t* fullrowptr, const int32_t* rowptr, const void* colidx,
                                 int colidx_bytes, const float* normfact, int64_t nrows, int64_t ncols, int64_t nnz,
                                 int32_t* csr_col, float* csr_val, int64_t* coo_indices, void* stream) {
  return build_operand(fullrowptr, rowptr, colidx, colidx_bytes, normfact, nrows, ncols, nnz, csr_col, csr_val,
                       coo_indices, nullptr, stream);
}

}  // extern "C"

namespace {
int build_operand(const int32_t* fullrowptr, const int32_t* rowptr, const void* colidx, int colidx_bytes,
                  const float* normfact, int64_t nrows, int64_t ncols, int64_t nnz, int32_t* csr_col, float* csr_val,
                  int64_t* coo_indices, unsigned long long* flag, void* stream) {
  // flag == nullptr: rows guaranteed column-ascending (no check, no fix pass)
  GNN_REQUIRE(nrows >= 0 && ncols >= 0 && nnz >= 0, "gnn_build_operand_f32: negative size");
  GNN_REQUIRE(nrows < INT_MAX && ncols < INT_MAX && nnz < INT_MAX, "gnn_build_operand_f32: sizes must be < 2^31");
  GNN_REQUIRE(colidx_bytes == 2 || colidx_bytes == 4 || colidx_bytes == 8,
              "gnn_build_operand_f32: colidx_bytes must be 2, 4 or 8 (got %d)", colidx_bytes);
  if (nrows == 0 || nnz == 0) return 0;
  GNN_REQUIRE(fullrowptr && rowptr && colidx && normfact && csr_col && csr_val, "gnn_build_operand_f32: NULL input");
  hipStream_t st = (hipStream_t)stream;
  const dim3 grid((unsigned)ceil_div(nrows, 4));
  const bool sorted = flag == nullptr;
  const unsigned long long gen = 1;
  if (!sorted) GNN_HIP(hipMemsetAsync(flag, 0, 2 * sizeof(*flag), st), "operand flag memset");
  const dim3 gflat((unsigned)ceil_div(nnz, 4 * BUILD_CHUNK));  // 4 waves x BUILD_CHUNK nonzeros
  const dim3 gfix(16);  // usually a no-op (gated): keep the launch small
  switch (colidx_bytes) {
    case 2:
      build_operand_flat_kernel<int16_t><<<gflat, dim3(256), 0, st>>>(
          fullrowptr, rowptr, (const int16_t*)colidx, normfact, (int)nrows, (int)nnz, csr_col, csr_val, flag, gen);
      GNN_LAUNCHED("build_operand_flat_kernel");
      if (!sorted)
        build_operand_kernel<int16_t><<<gfix, dim3(256), 0, st>>>(fullrowptr, rowptr, (const int16_t*)colidx, normfact,
                                                                (int)nrows, csr_col, csr_val, flag, gen);
      break;
    case 4:
      build_operand_flat_kernel<int32_t><<<gflat, dim3(256), 0, st>>>(
          fullrowptr, rowptr, (const int32_t*)colidx, normfact, (int)nrows, (int)nnz, csr_col, csr_val, flag, gen);
      GNN_LAUNCHED("build_operand_flat_kernel");
      if (!sorted)
        build_operand_kernel<int32_t><<<gfix, dim3(256), 0, st>>>(fullrowptr, rowptr, (const int32_t*)colidx, normfact,
                                                                (int)nrows, csr_col, csr_val, flag, gen);
      break;
    default:
      build_operand_flat_kernel<int64_t><<<gflat, dim3(256), 0, st>>>(
          fullrowptr, rowptr, (const int64_t*)colidx, normfact, (int)nrows, (int)nnz, csr_col, csr_val, flag, gen);
      GNN_LAUNCHED("build_operand_flat_kernel");
      if (!sorted)
        build_operand_kernel<int64_t><<<gfix, dim3(256), 0, st>>>(fullrowptr, rowptr, (const int64_t*)colidx, normfact,
                                                                (int)nrows, csr_col, csr_val, flag, gen);
      break;
  }
  GNN_LAUNCHED("build_operand_kernel");
  if (coo_indices) {
    csr_to_coo_indices_kernel<<<grid, dim3(256), 0, st>>>(rowptr, csr_col, (int)nrows, nnz, coo_indices);
    GNN_LAUNCHED("csr_to_coo_indices_kernel");
  }
  return 0;
}
}  // namespace

extern "C" {

int gnn_build_operand_t_f32(const int32_t* fullrowptr, const int32_t* colptr, const int32_t* rows,
                            const float* normfact, int64_t nrows, int64_t ncols, int64_t nnz, float* val_t,
                            void* stream) {
  GNN_REQUIRE(nrows >= 0 && ncols >= 0 && nnz >= 0, "gnn_build_operand_t_f32: negative size");
  GNN_REQUIRE(nrows < INT_MAX && ncols < INT_MAX && nnz < INT_MAX, "gnn_build_operand_t_f32: sizes must be < 2^31");
  if (ncols == 0 || nnz == 0) return 0;
  GNN_REQUIRE(fullrowptr && colptr && rows && normfact && val_t, "gnn_build_operand_t_f32: NULL input");
  build_operand_t_kernel<<<dim3((unsigned)ceil_div(nnz, 4 * BUILD_CHUNK)), dim3(256), 0, (hipStream_t)stream>>>(
      fullrowptr, colptr, rows, normfact, (int)ncols, (int)nnz, val_t);
  GNN_LAUNCHED("build_operand_t_kernel");
  return 0;
}

int gnn_coo_to_csr(const int64_t* row, const int64_t* col, int64_t nnz, int64_t M, int32_t* rowptr, int32_t* col32,
                   void* stream) {
  GNN_REQUIRE(nnz >= 0 && M >= 0, "gnn_coo_to_csr: negative size");
  GNN_REQUIRE(nnz < INT_MAX && M < INT_MAX, "gnn_coo_to_csr: sizes must be < 2^31");
  GNN_REQUIRE(rowptr != nullptr, "gnn_coo_to_csr: NULL rowptr");
  GNN_REQUIRE(nnz == 0 || row != nullptr, "gnn_coo_to_csr: NULL row");
  hipStream_t st = (hipStream_t)stream;
  coo_rowptr_kernel<<<dim3((unsigned)ceil_div(nnz + 1, 256)), dim3(256), 0, st>>>(row, nnz, (int)M, rowptr);
  GNN_LAUNCHED("coo_rowptr_kernel");
  if (col32 && nnz > 0) {
    GNN_REQUIRE(col != nullptr, "gnn_coo_to_csr: NULL col");
    narrow_index_kernel<<<dim3((unsigned)ceil_div(nnz, 256)), dim3(256), 0, st>>>(col, nnz, col32);
    GNN_LAUNCHED("narrow_index_kernel");
  }
  return 0;
}

size_t gnn_csr_transpose_workspace_bytes(int64_t M, int64_t K, int64_t nnz) {
  (void)M;
  const size_t fallback = align_up((size_t)(K > 0 ? K : 1) * 4, 256) + segsort_ws(K);
  if (K > TR_MAX_K) return fallback;
  int64_t TS = 0, T = 0;
  tr_tiles(nnz, TS, T);
  const size_t tiled = align_up((size_t)T * (size_t)K * 4, 256) + align_up((size_t)(K > 0 ? K : 1) * 4, 256);
  return tiled > fallback ? tiled : fallback;
}

int gnn_csr_transpose(const int32_t* rowptr, const int32_t* col, const float* val, int64_t M, int64_t K, int64_t nnz,
                      int32_t* tr_rowptr, int32_t* tr_col, float* tr_val, void* workspace, size_t workspace_bytes,
                      void* stream) {
  GNN_REQUIRE(M >= 0 && K >= 0 && nnz >= 0, "gnn_csr_transpose: negative size");
  GNN_REQUIRE(M < INT_MAX && K < INT_MAX && nnz < INT_MAX, "gnn_csr_transpose: sizes must be < 2^31");
  GNN_REQUIRE(tr_rowptr != nullptr, "gnn_csr_transpose: NULL tr_rowptr");
  hipStream_t st = (hipStream_t)stream;
  if (K == 0) return 0;
  if (nnz == 0 || M == 0) {
    GNN_HIP(hipMemsetAsync(tr_rowptr, 0, (size_t)(K + 1) * 4, st), "transpose memset");
    return 0;
  }
  GNN_REQUIRE(rowptr && col && val && tr_col && tr_val, "gnn_csr_transpose: NULL input/output");
  GNN_REQUIRE(workspace && workspace_bytes >= gnn_csr_transpose_workspace_bytes(M, K, nnz),
              "gnn_csr_transpose: workspace too small");
  char* w = (char*)workspace;
  if (K <= TR_MAX_K) {
    int64_t TS = 0, T = 0;
    tr_tiles(nnz, TS, T);
    int* hist = (int*)w;
    int* cnt = (int*)(w + align_up((size_t)T * (size_t)K * 4, 256));
    const size_t lds = (size_t)K * 4;
    static bool attr_set = false;
    if (!attr_set) {
      GNN_HIP(hipFuncSetAttribute((const void*)tr_tile_hist_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  TR_MAX_K * 4), "hipFuncSetAttribute(tr_tile_hist)");
      GNN_HIP(hipFuncSetAttribute((const void*)tr_tile_scatter_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  TR_MAX_K * 4 + TR_MAX_TS * 8), "hipFuncSetAttribute(tr_tile_scatter)");
      attr_set = true;
    }
    tr_tile_hist_kernel<<<dim3((unsigned)T), dim3(256), lds, st>>>(col, (int)nnz, (int)TS, (int)K, hist);
    GNN_LAUNCHED("tr_tile_hist_kernel");
    tr_col_prefix_kernel<<<dim3((unsigned)ceil_div(K, 256)), dim3(256), 0, st>>>(hist, (int)T, (int)K, cnt);
    GNN_LAUNCHED("tr_col_prefix_kernel");
    scan_exclusive_kernel<<<dim3(1), dim3(1024), 0, st>>>(cnt, (int)K, tr_rowptr, nullptr);
    GNN_LAUNCHED("scan_exclusive_kernel");
    const size_t lds3 = (size_t)((K + 3) & ~3) * 4 + (size_t)TS * 8;
    tr_tile_scatter_kernel<<<dim3((unsigned)T), dim3(256), lds3, st>>>(rowptr, col, val, (int)M, (int)nnz, (int)TS,
                                                                     (int)K, hist, tr_rowptr, tr_col, tr_val);
    GNN_LAUNCHED("tr_tile_scatter_kernel");
    return 0;
  }
  // Large K: atomic slot claim + segmented sort (also canonical and deterministic).
  int* cnt = (int*)w;
  void* ssws = w + align_up((size_t)K * 4, 256);
  GNN_HIP(hipMemsetAsync(cnt, 0, (size_t)K * 4, st), "transpose count memset");
  col_count_kernel<<<dim3((unsigned)ceil_div(nnz, 256)), dim3(256), 0, st>>>(col, nnz, cnt);
  GNN_LAUNCHED("col_count_kernel");
  scan_exclusive_kernel<<<dim3(1), dim3(1024), 0, st>>>(cnt, (int)K, tr_rowptr, cnt);
  GNN_LAUNCHED("scan_exclusive_kernel");
  transpose_scatter_kernel<<<dim3((unsigned)ceil_div(M, 4)), dim3(256), 0, st>>>(rowptr, col, val, (int)M, cnt,
                                                                               tr_col, tr_val);
  GNN_LAUNCHED("transpose_scatter_kernel");
  return run_segsort(tr_rowptr, K, tr_col, tr_val, ssws, st);
}

int gnn_gather_rows_f32(const float* src, int64_t ld_src, const int64_t* src_idx, float* dst, int64_t ld_dst,
                        const int64_t* dst_idx, int64_t n, int64_t F, void* stream) {
  GNN_REQUIRE(n >= 0 && F >= 0, "gnn_gather_rows_f32: negative size");
  GNN_REQUIRE(F <= ld_src && F <= ld_dst, "gnn_gather_rows_f32: F exceeds a row stride");
  GNN_REQUIRE(F < INT_MAX, "gnn_gather_rows_f32: F too large");
  if (n == 0 || F == 0) return 0;
  GNN_REQUIRE(src && dst, "gnn_gather_rows_f32: NULL src/dst");
  hipStream_t st = (hipStream_t)stream;
  const int vw = pick_vw(F, ld_src, ld_dst, src, dst);
  const dim3 grid((unsigned)ceil_div(n, 4));
  switch (vw) {
    case 4:
      gather_rows_kernel<4><<<grid, dim3(256), 0, st>>>(src, ld_src, src_idx, dst, ld_dst, dst_idx, n, (int)F);
      break;
    case 2:
      gather_rows_kernel<2><<<grid, dim3(256), 0, st>>>(src, ld_src, src_idx, dst, ld_dst, dst_idx, n, (int)F);
      break;
    default:
      gather_rows_kernel<1><<<grid, dim3(256), 0, st>>>(src, ld_src, src_idx, dst, ld_dst, dst_idx, n, (int)F);
      break;
  }
  GNN_LAUNCHED("gather_rows_kernel");
  return 0;
}

int gnn_gather_rows2_f32(const float* src0, int64_t ld0, const int64_t* idx0, const int64_t* pos0, int64_t n0,
                         const float* src1, int64_t ld1, const int64_t* idx1, const int64_t* pos1, int64_t n1,
                         float* dst, int64_t ld_dst, int64_t F, void* stream) {
  GNN_REQUIRE(n0 >= 0 && n1 >= 0 && F >= 0, "gnn_gather_rows2_f32: negative size");
  GNN_REQUIRE(F < INT_MAX && n0 + n1 < (int64_t)INT_MAX * 4, "gnn_gather_rows2_f32: too large");
  if (n0 + n1 == 0 || F == 0) return 0;
  GNN_REQUIRE(dst && (n0 == 0 || src0) && (n1 == 0 || src1), "gnn_gather_rows2_f32: NULL src/dst");
  GNN_REQUIRE(F <= ld_dst && (n0 == 0 || F <= ld0) && (n1 == 0 || F <= ld1),
              "gnn_gather_rows2_f32: F exceeds a row stride");
  hipStream_t st = (hipStream_t)stream;
  // 16-byte loads when every row of both sources and of dst allows them
  int vw = pick_vw(F, n0 ? ld0 : ld1, ld_dst, n0 ? src0 : src1, dst);
  if (n0 && n1) vw = std::min(vw, pick_vw(F, ld1, ld_dst, src1, dst));
  const dim3 grid((unsigned)ceil_div(n0 + n1, (int64_t)4));
  const int per = (int)ceil_div(F, (int64_t)64 * vw);  // loads per lane
#define GNN_G2(VW, NL) \
  gather_rows2_kernel<VW, NL><<<grid, dim3(256), 0, st>>>(src0, ld0, idx0, pos0, n0, src1, ld1, idx1, pos1, n1, dst, ld_dst, (int)F)
  if (vw == 4 && per <= 3) GNN_G2(4, 3);
  else if (vw == 4 && per <= 8) GNN_G2(4, 8);
  else if (vw == 2 && per <= 8) GNN_G2(2, 8);
  else if (vw == 1 && per <= 16) GNN_G2(1, 16);
  else {  // wide rows: the one-source kernel per source
    const int rc = gnn_gather_rows_f32(src0, ld0, idx0, dst, ld_dst, pos0, n0, F, stream);
    if (rc) return rc;
    return gnn_gather_rows_f32(src1, ld1, idx1, dst, ld_dst, pos1, n1, F, stream);
  }
#undef GNN_G2
  GNN_LAUNCHED("gather_rows2_kernel");
  return 0;
}

int gnn_host_register(void* host, size_t bytes) {
  GNN_REQUIRE(host && bytes > 0, "gnn_host_register: NULL or empty range");
  GNN_HIP(hipHostRegister(host, bytes, hipHostRegisterMapped), "hipHostRegister");
  return 0;
}

int gnn_host_unregister(void* host) {
  GNN_REQUIRE(host, "gnn_host_unregister: NULL");
  GNN_HIP(hipHostUnregister(host), "hipHostUnregister");
  return 0;
}

int gnn_stream_create_cu_masked(int32_t device, int32_t cus, int32_t priority, void** stream_out) {
  GNN_REQUIRE(stream_out, "gnn_stream_create_cu_masked: NULL stream_out");
  *stream_out = nullptr;
  GNN_HIP(hipSetDevice(device), "hipSetDevice");
  int ncu = 0;
  GNN_HIP(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, device), "hipDeviceGetAttribute");
  GNN_REQUIRE(cus > 0 && cus <= ncu, "gnn_stream_create_cu_masked: cus must be in [1, %d]", ncu);
  std::vector<uint32_t> mask((size_t)(ncu + 31) / 32, 0u);
  const int stride = ncu / cus;  // spread over the device's CU numbering (every XCD gets its share)
  for (int i = 0, k = 0; i < ncu && k < cus; i += stride, ++k) mask[(size_t)i / 32] |= 1u << (i % 32);
  hipStream_t st = nullptr;
  GNN_HIP(hipExtStreamCreateWithCUMask(&st, (uint32_t)mask.size(), mask.data()), "hipExtStreamCreateWithCUMask");
  (void)priority;
  *stream_out = (void*)st;
  return 0;
}

int gnn_stream_destroy(void* stream) {
  if (stream) GNN_HIP(hipStreamDestroy((hipStream_t)stream), "hipStreamDestroy");
  return 0;
}

int gnn_memcpy_h2d_async(void* dst, const void* src, size_t bytes, void* stream) {
  if (bytes == 0) return 0;
  GNN_REQUIRE(dst && src, "gnn_memcpy_h2d_async: NULL pointer");
  GNN_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, (hipStream_t)stream), "hipMemcpyAsync");
  return 0;
}

int gnn_ipc_export(const void* ptr, void* handle_out, int64_t* offset_out) {
  GNN_REQUIRE(ptr && handle_out && offset_out, "gnn_ipc_export: NULL argument");
  static_assert(sizeof(hipIpcMemHandle_t) == GNN_IPC_HANDLE_BYTES, "IPC handle size");
  void* base = nullptr;
  size_t size = 0;
  GNN_HIP(hipMemGetAddressRange(&base, &size, const_cast<void*>(ptr)), "hipMemGetAddressRange");
  hipIpcMemHandle_t h;
  GNN_HIP(hipIpcGetMemHandle(&h, base), "hipIpcGetMemHandle");
  std::memcpy(handle_out, &h, sizeof(h));
  *offset_out = (int64_t)((const char*)ptr - (const char*)base);
  return 0;
}

int gnn_ipc_open(const void* handle, int64_t offset, int peer_device, void** ptr_out) {
  GNN_REQUIRE(handle && ptr_out && offset >= 0, "gnn_ipc_open: bad argument");
  int cur = 0;
  GNN_HIP(hipGetDevice(&cur), "hipGetDevice");
  if (peer_device >= 0 && peer_device != cur) {
    int can = 0;
    GNN_HIP(hipDeviceCanAccessPeer(&can, cur, peer_device), "hipDeviceCanAccessPeer");
    GNN_REQUIRE(can, "gnn_ipc_open: this GPU cannot access the peer GPU's memory");
    const hipError_t e = hipDeviceEnablePeerAccess(peer_device, 0);
    if (e == hipErrorPeerAccessAlreadyEnabled) (void)hipGetLastError();
    else GNN_HIP(e, "hipDeviceEnablePeerAccess");
  }
  hipIpcMemHandle_t h;
  std::memcpy(&h, handle, sizeof(h));
  void* base = nullptr;
  GNN_HIP(hipIpcOpenMemHandle(&base, h, hipIpcMemLazyEnablePeerAccess), "hipIpcOpenMemHandle");
  *ptr_out = (char*)base + offset;
  return 0;
}

int gnn_ipc_close(void* ptr, int64_t offset) {
  GNN_REQUIRE(ptr && offset >= 0, "gnn_ipc_close: bad argument");
  GNN_HIP(hipIpcCloseMemHandle((char*)ptr - offset), "hipIpcCloseMemHandle");
  return 0;
}

int gnn_gather_rows_host_f32(const float* host_src, int64_t ld_src, const int64_t* src_idx, float* dst,
                             int64_t ld_dst, const int64_t* dst_idx, int64_t n, int64_t F, void* stream) {
  GNN_REQUIRE(n >= 0 && F >= 0, "gnn_gather_rows_host_f32: negative size");
  GNN_REQUIRE(F <= ld_src && F <= ld_dst, "gnn_gather_rows_host_f32: F exceeds a row stride");
  GNN_REQUIRE(F < INT_MAX, "gnn_gather_rows_host_f32: F too large");
  if (n == 0 || F == 0) return 0;
  GNN_REQUIRE(host_src && dst, "gnn_gather_rows_host_f32: NULL src/dst");
  void* dsrc = nullptr;
  GNN_HIP(hipHostGetDevicePointer(&dsrc, (void*)host_src, 0),
          "hipHostGetDevicePointer (host_src must be pinned, device-mapped host memory)");
  const float* src = (const float*)dsrc;
  hipStream_t st = (hipStream_t)stream;
  const int vw = pick_vw(F, ld_src, ld_dst, src, dst);
  const dim3 grid((unsigned)std::min<int64_t>(ceil_div(n, 8), HOST_GATHER_GRID));
  switch (vw) {
    case 4:
      gather_rows_host_kernel<4><<<grid, dim3(256), 0, st>>>(src, ld_src, src_idx, dst, ld_dst, dst_idx, n, (int)F);
      break;
    case 2:
      gather_rows_host_kernel<2><<<grid, dim3(256), 0, st>>>(src, ld_src, src_idx, dst, ld_dst, dst_idx, n, (int)F);
      break;
    default:
      gather_rows_host_kernel<1><<<grid, dim3(256), 0, st>>>(src, ld_src, src_idx, dst, ld_dst, dst_idx, n, (int)F);
      break;
  }
  GNN_LAUNCHED("gather_rows_host_kernel");
  return 0;
}

}  // extern "C"
