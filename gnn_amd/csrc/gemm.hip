// gemm.hip — fp32 GEMMs of the GraphSAGE / GCN layers on gfx950 MFMA (v_mfma_f32_32x32x2_f32).
//
// The layers' dense products (models.py:18-21, 58-61 and their backward) are fp32 in the
// reference and stay exact fp32 here: f32-input MFMA is a k-ordered fmaf chain per output
// (no xf32 on gfx950), at the f32 matrix rate (157 TF/s dense). One kernel covers the three
// shapes of a layer through operand layouts:
//   forward     H  = X · Wᵀ   A = X  (row m contiguous in k), B = Wᵀ (row n of W contiguous in k)
//   input grad  dX = G · W    A = G  (m-major),               B = W  (row k contiguous in n)
//   weight grad dW = Gᵀ · X   A = Gᵀ (row k of G contiguous in m), B = X (k-major)
// The weight gradient reduces over the sampled rows (8-16 k) into a small 512 × F output, so
// it is split over k into partial tiles that a second kernel adds in split order
// (deterministic; no atomics).
//
// Tiling: 256-thread workgroup = 2 × 2 waves, 128 × 128 output tile, k staged 16 at a time in
// double-buffered LDS (next tile's global loads in flight during the current tile's MFMAs,
// one barrier per k tile); each wave owns 64 × 64 = 2 × 2 MFMA blocks (64 accumulator VGPRs).
// LDS images follow the source layout, padded so the MFMA operand reads are conflict-free:
// k-major [16][128 + 32] (the two lane halves read rows 160 floats apart: banks offset by 32),
// m/n-major [128][16 + 2] (row stride ≡ 2 mod 4: 32 rows × 2 k land on 64 distinct banks).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>
#include <cstdint>
#include <cstdlib>

#include "common.h"
#include "gnn_layers.h"

namespace {

using gnn::ceil_div;

typedef float f2 __attribute__((ext_vector_type(2)));
typedef float f4 __attribute__((ext_vector_type(4)));
typedef float f16v __attribute__((ext_vector_type(16)));

constexpr int BM = 128, BN = 128;
constexpr int KM_LD = BM + 32;  // k-major LDS row (BM == BN)
constexpr int MAX_BATCH = 4;

// k depth of one LDS stage; m/n-major LDS rows are BKT + 2 floats (≡ 2 mod 4)
template <int BKT>
struct Stage {
  static constexpr int MM_LD = BKT + 2;
  static constexpr int FLOATS = (BKT * KM_LD > BM * MM_LD) ? BKT * KM_LD : BM * MM_LD;
  static constexpr int NP = BKT / 8;  // 4-float pieces per thread per operand tile
};

struct Batch {
  const float* A[MAX_BATCH];
  const float* B[MAX_BATCH];
  float* C[MAX_BATCH];
  // split3 only: row indices of A / B (NULL: none). An indexed operand's row r is the source's
  // row idx[r] — A's rows m (m-major A) or B's rows k (k-major B): the GraphSAGE x[sampled]
  // operand read in place instead of gathered first.
  const int64_t* ia[MAX_BATCH];
  const int64_t* ib[MAX_BATCH];
};

// Four consecutive floats of a row: one 16-byte load (VEC 4) or two 8-byte loads (VEC 2,
// for rows whose stride is only even, e.g. 602 features).
template <int VEC>
__device__ __forceinline__ f4 load4(const float* p) {
  if constexpr (VEC == 4) {
    return *reinterpret_cast<const f4*>(p);
  } else {
    const f2 lo = *reinterpret_cast<const f2*>(p);
    const f2 hi = *reinterpret_cast<const f2*>(p + 2);
    return f4{lo.x, lo.y, hi.x, hi.y};
  }
}

// One operand tile (BKT x 128 of a k-major source, or 128 x BKT of an m-major source) as NP
// 4-float pieces per thread.
//  * Interior k tiles (GUARD = false) are branch-free: an m/n coordinate past the matrix
//    edge is clamped to a valid address — it only feeds accumulator rows/columns that are
//    never stored — so every piece is one unconditional vector load.
//  * The k-tail tile (GUARD = true) reads k >= klim as 0, element by element.
template <bool KMAJ, int VEC, int BKT, bool GUARD>
__device__ __forceinline__ void load_tile(const float* __restrict__ P, int64_t ld, int r0, int rlim, int k0, int klim,
                                          int t, f4 v[Stage<BKT>::NP]) {
#pragma unroll
  for (int j = 0; j < Stage<BKT>::NP; ++j) {
    if constexpr (KMAJ) {
      const int k = k0 + (t >> 5) + 8 * j;
      const int m = r0 + (t & 31) * 4;
      if constexpr (!GUARD) {
        const float* row = P + (int64_t)k * ld;
        if constexpr (VEC == 4) {
          // ld % 4 == 0 and ld >= rlim: a piece starting at a multiple of 4 below rlim stays in the
          // row (its elements >= rlim feed unstored columns); pieces past rlim re-read the last one
          v[j] = load4<4>(row + min(m, ((rlim - 1) >> 2) << 2));
        } else {
          const int mc = ((rlim - 1) >> 1) << 1;  // last even column start below rlim (ld even >= rlim)
          const f2 lo = *reinterpret_cast<const f2*>(row + min(m, mc));
          const f2 hi = *reinterpret_cast<const f2*>(row + min(m + 2, mc));
          v[j] = f4{lo.x, lo.y, hi.x, hi.y};
        }
      } else {
        f4 x = f4(0.0f);
        if (k < klim) {
          const float* row = P + (int64_t)k * ld;
          if (m + 0 < rlim) x.x = row[m + 0];
          if (m + 1 < rlim) x.y = row[m + 1];
          if (m + 2 < rlim) x.z = row[m + 2];
          if (m + 3 < rlim) x.w = row[m + 3];
        }
        v[j] = x;
      }
    } else {
      constexpr int TPR = BKT / 4;  // threads per row
      const int m = min(r0 + t / TPR + (256 / TPR) * j, rlim - 1);
      const int k = k0 + (t % TPR) * 4;
      const float* q = P + (int64_t)m * ld + k;
      if constexpr (!GUARD) {
        v[j] = load4<VEC>(q);
      } else {
        f4 x = f4(0.0f);
        if (k + 0 < klim) x.x = q[0];
        if (k + 1 < klim) x.y = q[1];
        if (k + 2 < klim) x.z = q[2];
        if (k + 3 < klim) x.w = q[3];
        v[j] = x;
      }
    }
  }
}

template <bool KMAJ, int BKT>
__device__ __forceinline__ void store_tile(float* __restrict__ S, int t, const f4 v[Stage<BKT>::NP]) {
#pragma unroll
  for (int j = 0; j < Stage<BKT>::NP; ++j) {
    if constexpr (KMAJ) {
      const int kk = (t >> 5) + 8 * j, m = (t & 31) * 4;
      *reinterpret_cast<f4*>(S + kk * KM_LD + m) = v[j];
    } else {
      constexpr int TPR = BKT / 4;
      const int m = t / TPR + (256 / TPR) * j, kk = (t % TPR) * 4;
      float* p = S + m * Stage<BKT>::MM_LD + kk;  // 8-byte aligned (MM_LD even)
      *reinterpret_cast<f2*>(p) = f2{v[j].x, v[j].y};
      *reinterpret_cast<f2*>(p + 2) = f2{v[j].z, v[j].w};
    }
  }
}

// MFMA operand of lane (i, kk): element (row i of the block, k = 2s + kk).
template <bool KMAJ, int BKT>
__device__ __forceinline__ float frag(const float* __restrict__ S, int r, int k) {
  if constexpr (KMAJ) return S[k * KM_LD + r];
  else return S[r * Stage<BKT>::MM_LD + k];
}

// C (or a split-k partial) = A · B over k in [kbeg, kend) for one 128 x 128 tile.
template <bool AK, bool BKM, int VA, int VB, int BKT>
__global__ __launch_bounds__(256) void gemm_f32_kernel(Batch bt, int M, int N, int K, int64_t lda, int64_t ldb,
                                                          int64_t ldc, int splits, int klen, float* __restrict__ part) {
  __shared__ __attribute__((aligned(16))) float As[2][Stage<BKT>::FLOATS];
  __shared__ __attribute__((aligned(16))) float Bs[2][Stage<BKT>::FLOATS];
  const int t = threadIdx.x;
  const int lane = t & 63;
  const int wid = t >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int b = blockIdx.z / splits;
  const int split = blockIdx.z % splits;
  const int m0 = blockIdx.y * BM;
  const int n0 = blockIdx.x * BN;
  const int kbeg = split * klen;
  const int kend = min(K, kbeg + klen);
  const float* __restrict__ A = bt.A[b];
  const float* __restrict__ B = bt.B[b];

  f16v acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f16v(0.0f);

  const int nk = kend > kbeg ? (kend - kbeg + BKT - 1) / BKT : 0;
  f4 ra[Stage<BKT>::NP], rb[Stage<BKT>::NP];
  auto load_ab = [&](int k0) {  // uniform branch: only the k-tail tile takes the guarded path
    if (k0 + BKT <= kend) {
      load_tile<AK, VA, BKT, false>(A, lda, m0, M, k0, kend, t, ra);
      load_tile<BKM, VB, BKT, false>(B, ldb, n0, N, k0, kend, t, rb);
    } else {
      load_tile<AK, VA, BKT, true>(A, lda, m0, M, k0, kend, t, ra);
      load_tile<BKM, VB, BKT, true>(B, ldb, n0, N, k0, kend, t, rb);
    }
  };
  if (nk > 0) {
    load_ab(kbeg);
    store_tile<AK, BKT>(As[0], t, ra);
    store_tile<BKM, BKT>(Bs[0], t, rb);
  }
  __syncthreads();
  const int li = lane & 31, lk = lane >> 5;
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) load_ab(kbeg + (kt + 1) * BKT);
    const float* Sa = As[cur];
    const float* Sb = Bs[cur];
#pragma unroll
    for (int s = 0; s < BKT / 2; ++s) {
      const int k = 2 * s + lk;
      const float a0 = frag<AK, BKT>(Sa, wm * 64 + li, k);
      const float a1 = frag<AK, BKT>(Sa, wm * 64 + 32 + li, k);
      const float b0 = frag<BKM, BKT>(Sb, wn * 64 + li, k);
      const float b1 = frag<BKM, BKT>(Sb, wn * 64 + 32 + li, k);
      acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b0, acc[0][0], 0, 0, 0);
      acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b1, acc[0][1], 0, 0, 0);
      acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b0, acc[1][0], 0, 0, 0);
      acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b1, acc[1][1], 0, 0, 0);
    }
    if (kt + 1 < nk) {
      store_tile<AK, BKT>(As[cur ^ 1], t, ra);
      store_tile<BKM, BKT>(Bs[cur ^ 1], t, rb);
    }
    __syncthreads();
  }

  // C/D map of the 32x32 MFMA: column = lane & 31, row = (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5).
  float* __restrict__ Cb;
  int64_t ldo;
  if (splits > 1) {
    Cb = part + (int64_t)blockIdx.z * M * N;
    ldo = N;
  } else {
    Cb = bt.C[b];
    ldo = ldc;
  }
#pragma unroll
  for (int i = 0; i < 2; ++i) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int n = n0 + wn * 64 + j * 32 + li;
      if (n >= N) continue;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = m0 + wm * 64 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * lk;
        if (m < M) Cb[(int64_t)m * ldo + n] = acc[i][j][r];
      }
    }
  }
}

// C[b] = sum over splits of the partial tiles, in split order; 4 consecutive outputs per thread
// (C rows contiguous: ldc == N, M*N % 4 == 0, 16-byte aligned).
__global__ __launch_bounds__(256) void gemm_splitk_reduce4_kernel(Batch bt, const float* __restrict__ part, int64_t MN,
                                                                  int splits, int nbatch) {
  const int64_t n4 = MN / 4;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < n4 * nbatch; e += (int64_t)gridDim.x * 256) {
    const int b = (int)(e / n4);
    const int64_t o = (e - (int64_t)b * n4) * 4;
    const float* p = part + (int64_t)b * splits * MN + o;
    f4 acc = *reinterpret_cast<const f4*>(p);
    int q = 1;
    for (; q + 3 < splits; q += 4) {  // 4 partial tiles in flight, added in split order
      const f4 v0 = *reinterpret_cast<const f4*>(p + (int64_t)q * MN);
      const f4 v1 = *reinterpret_cast<const f4*>(p + (int64_t)(q + 1) * MN);
      const f4 v2 = *reinterpret_cast<const f4*>(p + (int64_t)(q + 2) * MN);
      const f4 v3 = *reinterpret_cast<const f4*>(p + (int64_t)(q + 3) * MN);
      acc += v0;
      acc += v1;
      acc += v2;
      acc += v3;
    }
    for (; q < splits; ++q) acc += *reinterpret_cast<const f4*>(p + (int64_t)q * MN);
    *reinterpret_cast<f4*>(bt.C[b] + o) = acc;
  }
}

// C[b] = sum over splits of the partial tiles, in split order.
__global__ __launch_bounds__(256) void gemm_splitk_reduce_kernel(Batch bt, const float* __restrict__ part, int M, int N,
                                                                 int64_t ldc, int splits, int nbatch) {
  const int64_t MN = (int64_t)M * N;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < MN * nbatch; e += (int64_t)gridDim.x * 256) {
    const int b = (int)(e / MN);
    const int64_t o = e - (int64_t)b * MN;
    const float* p = part + (int64_t)b * splits * MN + o;
    float s = p[0];
    for (int q = 1; q < splits; ++q) s += p[(int64_t)q * MN];
    const int m = (int)(o / N), n = (int)(o - (int64_t)m * N);
    bt.C[b][(int64_t)m * ldc + n] = s;
  }
}

// ---------------------------------------------------------------------------------------------
// fp32 GEMM on the bf16 matrix cores by an exact three-way split ("split3").
//
// Every fp32 operand is cut into three bf16 pieces by truncation, x = h + m + l EXACTLY
// (h keeps the top 8 significant bits, m the next 8 bits of the remainder, l the remaining
// <= 8 bits), and a·b is accumulated in fp32 as the six largest piece products
//   h·h + h·m + m·h + h·l + m·m + l·h
// on v_mfma_f32_32x32x16_bf16 (each bf16 x bf16 product is exact in fp32). The three dropped
// products (m·l, l·m, l·l) are below 3·2^-24 |a||b| — the size of one fp32 rounding — so the
// result has fp32-level accuracy (tests/test_gemm_gpu.py bounds it against fp64 with the same
// tolerance as the f32-input kernel above). Six bf16 MFMAs (6 × 32 cycles per 32×32×16) do
// the work of eight f32-input ones (8 × 64 cycles): 2.67× the matrix rate.
//
// Tiling: 256-thread workgroup = 2 × 2 waves, 128 × 128 output tile, k staged 16 deep in
// double-buffered LDS (48 KB: three workgroups per CU). Each operand tile is loaded as 8
// floats of one row per thread — k-contiguous sources by two 16-byte (or four 8-byte) loads,
// k-major sources by eight 4-byte loads whose wave instruction covers 64 consecutive columns —
// split into its pieces in registers and stored as three k-contiguous images [128][16] bf16
// (one 16-byte store per piece; the MFMA operand of lane (r, h) is the 16 bytes at row r,
// k 8h, read with ds_read_b128 from a bank-swizzled image). Operands are read by buffer loads
// (per-thread VGPR offset + scalar k offset) two k tiles ahead of the MFMAs.
// ---------------------------------------------------------------------------------------------
typedef __bf16 bf8v __attribute__((ext_vector_type(8)));
typedef unsigned int u4v __attribute__((ext_vector_type(4)));

constexpr int S3_BK = 16;                  // k per LDS stage
constexpr int S3_PIECE = BM * S3_BK;       // bf16 per piece image
constexpr int S3_OPER = 3 * S3_PIECE;      // bf16 per operand stage

// Buffer resource over one operand (raw, byte offsets; the host guarantees extents < 2^31 B).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t s3_rsrc(const float* p, int64_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)p, (short)0, (int)bytes, 0x00020000);
}

// 8 floats of one operand row (row rr of the tile, k = kh*8 .. kh*8+7 of the stage), by buffer
// loads whose per-thread part (column / row start) is a fixed VGPR offset and whose k part is
// a scalar offset: no per-load 64-bit address arithmetic.
//   k-major source: thread t holds column m = t & 127 (a wave instruction reads 64 consecutive
//     floats of one k row); the k half kh = t >> 7 is wave-uniform.
//   k-contiguous source: thread t holds row t >> 1, k half t & 1 (two 16-byte or four 8-byte loads).
// IX (k-major sources): row k of the operand is the source's row idx[k] (a wave-uniform scalar
// load per row); m-major sources take their row index in the fixed offset (s3_voff).
template <bool KMAJ, int VEC, bool GUARD, bool IX = false>
__device__ __forceinline__ void s3_load(__amdgpu_buffer_rsrc_t rs, const float* __restrict__ P, int64_t ld, int voff,
                                        int r0, int rlim, int k0, int klim, int t, float v[8],
                                        const int64_t* __restrict__ idx = nullptr) {
  if constexpr (KMAJ) {
    const int kb = k0 + __builtin_amdgcn_readfirstlane((t >> 7) * 8);
    if constexpr (GUARD) {
      const int m = min(r0 + (t & 127), rlim - 1);
#pragma unroll
      for (int i = 0; i < 8; ++i)
        v[i] = (kb + i < klim) ? P[(IX ? idx[kb + i] : (int64_t)(kb + i)) * ld + m] : 0.0f;
    } else {
#pragma unroll
      for (int i = 0; i < 8; ++i)
        v[i] = __builtin_bit_cast(
            float, __builtin_amdgcn_raw_buffer_load_b32(
                       rs, voff, (int)((IX ? idx[kb + i] : (int64_t)(kb + i)) * ld * 4), 0));
    }
  } else {
    if constexpr (GUARD) {
      const int m = min(r0 + (t >> 1), rlim - 1);
      const int kb = k0 + (t & 1) * 8;
      const float* q = P + (IX ? idx[m] : (int64_t)m) * ld + kb;
#pragma unroll
      for (int i = 0; i < 8; ++i) v[i] = (kb + i < klim) ? q[i] : 0.0f;
    } else {
      const int so = k0 * 4;
      if constexpr (VEC == 4) {
        const f4 a = __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(rs, voff, so, 0));
        const f4 b = __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(rs, voff + 16, so, 0));
        v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
        v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
      } else {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const f2 a = __builtin_bit_cast(f2, __builtin_amdgcn_raw_buffer_load_b64(rs, voff + 8 * i, so, 0));
          v[2 * i] = a.x;
          v[2 * i + 1] = a.y;
        }
      }
    }
  }
}

// The thread's fixed VGPR byte offset for s3_load (rows past the edge clamped to the last row).
template <bool KMAJ>
__device__ __forceinline__ int s3_voff(int64_t ld, int r0, int rlim, int t, const int64_t* __restrict__ idx = nullptr) {
  if constexpr (KMAJ) return min(r0 + (t & 127), rlim - 1) * 4;
  else {
    const int r = min(r0 + (t >> 1), rlim - 1);
    return (int)(((idx ? idx[r] : (int64_t)r) * ld + (t & 1) * 8) * 4);
  }
}

// Offset (in bf16 units) of the 16-byte chunk (row, k half h) in a piece image. The half is
// swizzled by bit 3 of the row so that every 16-lane group of a ds_read_b128 (lanes
// {0-3,12-15,20-27}, {4-11,16-19,28-31}, ...: MI355X_MICROARCH.md §LDS) covers all 64 banks
// (unswizzled, rows r and r + 8 of a group share banks: 2-way conflicts, measured).
// k-major sources store one row per lane with a wave-uniform half, so their images are laid
// out half-major, [h][row]: a ds_write_b128 group of 8 lanes then covers 128 contiguous bytes
// (the [row][h] image was 2-way: 0.33 of the LDS cycles of the weight-gradient kernels), and
// each ds_read_b128 group {0-3,12-15,20-27} / {4-11,16-19,28-31} still covers 64 banks.
template <bool KMAJ>
__device__ __forceinline__ int s3_chunk(int row, int h) {
  if constexpr (KMAJ) return (h * BM + row) * 8;
  else return (2 * row + (h ^ ((row >> 3) & 1))) * 8;
}

// Split 8 floats into their three bf16 pieces and store them into the stage's images.
template <bool KMAJ>
__device__ __forceinline__ void s3_store(unsigned short* __restrict__ S, int t, const float v[8]) {
  const int rr = KMAJ ? (t & 127) : (t >> 1);
  const int kh = KMAJ ? (t >> 7) : (t & 1);
  // per pair of elements: 4 v_and, 4 v_sub_f32 and 3 v_perm (one per piece, packing the two high
  // halves). The kernel is bound by the SIMD's issue port (VALU + MFMA issue); the subtractions
  // stay scalar: the packed form (v_pk_add_f32, two elements per instruction) measured 2-5 %
  // slower on every layer pair (profiles/round5/gemm_split/), the element-wise and/or form
  // (and + or_sdwa + lshr + and_or + moves, 214 VALU per two k tiles) slower still.
  u4v ph, pm, pl;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const float x0 = v[2 * j], x1 = v[2 * j + 1];
    const unsigned int h0 = __float_as_uint(x0) & 0xffff0000u, h1 = __float_as_uint(x1) & 0xffff0000u;
    const float r0 = x0 - __uint_as_float(h0), r1 = x1 - __uint_as_float(h1);  // exact
    const unsigned int m0 = __float_as_uint(r0) & 0xffff0000u, m1 = __float_as_uint(r1) & 0xffff0000u;
    const float l0 = r0 - __uint_as_float(m0), l1 = r1 - __uint_as_float(m1);  // exact, <= 8 significant bits
    // bytes {lo.2, lo.3, hi.2, hi.3}: the bf16 (high half) of element 2j low, of 2j+1 high
    ph[j] = __builtin_amdgcn_perm(h1, h0, 0x07060302u);
    pm[j] = __builtin_amdgcn_perm(m1, m0, 0x07060302u);
    pl[j] = __builtin_amdgcn_perm(__float_as_uint(l1), __float_as_uint(l0), 0x07060302u);
  }
  const int off = s3_chunk<KMAJ>(rr, kh);
  *reinterpret_cast<u4v*>(S + off) = ph;
  *reinterpret_cast<u4v*>(S + S3_PIECE + off) = pm;
  *reinterpret_cast<u4v*>(S + 2 * S3_PIECE + off) = pl;
}

template <bool KMAJ>
__device__ __forceinline__ bf8v s3_frag(const unsigned short* __restrict__ S, int piece, int row, int h) {
  return __builtin_bit_cast(bf8v, *reinterpret_cast<const u4v*>(S + piece * S3_PIECE + s3_chunk<KMAJ>(row, h)));
}

// The six piece products of one k16 step into the wave's 2 x 2 accumulators (small terms first).
template <bool AK, bool BKM>
__device__ __forceinline__ void s3_mma(const unsigned short* __restrict__ Sa, const unsigned short* __restrict__ Sb,
                                       int ra0, int rb0, int li, int lh, f16v acc[2][2]) {
  bf8v a[2][3], bb[2][3];
#pragma unroll
  for (int p = 0; p < 3; ++p)
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      a[i][p] = s3_frag<AK>(Sa, p, ra0 + i * 32 + li, lh);
      bb[i][p] = s3_frag<BKM>(Sb, p, rb0 + i * 32 + li, lh);
    }
  constexpr int PA[6] = {2, 1, 0, 1, 0, 0};
  constexpr int PB[6] = {0, 1, 2, 0, 1, 0};
#pragma unroll
  for (int q = 0; q < 6; ++q)
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i][PA[q]], bb[j][PB[q]], acc[i][j], 0, 0, 0);
}

// three workgroups per CU: LDS 48 KB each, registers capped at 168 (3 waves per SIMD)
template <bool AK, bool BKM, int VA, int VB, bool IDX = false>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(3, 3))) void gemm_s3_kernel(Batch bt, int M, int N, int K, int64_t lda, int64_t ldb,
                                                         int64_t ldc, int splits, int klen, float* __restrict__ part,
                                                         int64_t abytes, int64_t bbytes, int xcd_map,
                                                         int tail_base = 0, int tail_s = 0) {
  __shared__ __attribute__((aligned(16))) unsigned short As[2][S3_OPER];
  __shared__ __attribute__((aligned(16))) unsigned short Bs[2][S3_OPER];
  const int t = threadIdx.x;
  const int lane = t & 63;
  const int wid = t >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  // Tile of this workgroup. xcd_map: consecutive tiles (the n tiles of one m row panel)
  // go to one XCD (workgroups are dealt to the 8 XCDs round-robin), so a row panel of A is
  // fetched into one L2 instead of up to four.
  int tx = blockIdx.x, ty = blockIdx.y, tz = blockIdx.z;
  int b, split;
  int piece = -1;  // tail mode: this workgroup's k piece of a tail tile (slot in the piece slab)
  if (tail_s > 0) {
    // 1-D grid: tiles [0, tail_base) whole (XCD map over them), then each tail tile as tail_s
    // k pieces (see tail_plan)
    const int gx = (N + BN - 1) / BN, gy = (M + BM - 1) / BM;
    const int hw = blockIdx.x;
    int lg;
    if (hw < tail_base) {
      const int per = tail_base >> 3;
      lg = xcd_map ? (hw & 7) * per + (hw >> 3) : hw;
      split = 0;
    } else {
      piece = hw - tail_base;
      lg = tail_base + piece / tail_s;
      split = piece % tail_s;
    }
    tx = lg % gx;
    ty = (lg / gx) % gy;
    b = lg / (gx * gy);
  } else {
    if (xcd_map) {
      const int gx = gridDim.x, gy = gridDim.y;
      const int total = gx * gy * gridDim.z;
      const int hw = blockIdx.x + gx * (blockIdx.y + gy * blockIdx.z);
      const int per = total >> 3;
      const int lg = hw < per * 8 ? (hw & 7) * per + (hw >> 3) : hw;
      tx = lg % gx;
      ty = (lg / gx) % gy;
      tz = lg / (gx * gy);
    }
    b = tz / splits;
    split = tz % splits;
  }
  const int m0 = ty * BM;
  const int n0 = tx * BN;
  const bool whole = tail_s > 0 && piece < 0;
  const int kbeg = whole ? 0 : split * klen;
  const int kend = whole ? K : min(K, kbeg + klen);
  const float* __restrict__ A = bt.A[b];
  const float* __restrict__ B = bt.B[b];
  const __amdgpu_buffer_rsrc_t rsa = s3_rsrc(A, abytes), rsb = s3_rsrc(B, bbytes);
  // IDX instantiations: A indexed when m-major, B when k-major (the two GraphSAGE x[sampled] uses)
  const int64_t* __restrict__ ia = (IDX && !AK) ? bt.ia[b] : nullptr;
  const int64_t* __restrict__ ib = (IDX && BKM) ? bt.ib[b] : nullptr;
  const int voa = s3_voff<AK>(lda, m0, M, t, ia), vob = s3_voff<BKM>(ldb, n0, N, t);

  f16v acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f16v(0.0f);

  // Two register sets: tile kt+2's loads are in flight while tile kt is multiplied and tile
  // kt+1 (loaded one tile earlier) is split into the other LDS stage.
  float ra[2][8], rb[2][8];
  // The main loop runs over the full k tiles with branch-free loads: a prefetch past the last
  // full tile re-reads that tile (never multiplied). A divergent guarded load inside the loop
  // made the compiler join two register sets and wait for ALL loads (vmcnt(0)) before the
  // MFMAs, i.e. no prefetch at all. The k tail (K % 16) runs once after the loop.
  const int nfull = (kend - kbeg) / S3_BK;
  auto load_ab = [&](int kt, float(&xa)[8], float(&xb)[8]) {
    const int k0 = kbeg + min(kt, nfull - 1) * S3_BK;
    s3_load<AK, VA, false>(rsa, A, lda, voa, m0, M, k0, kend, t, xa);
    if (IDX && BKM && ib)
      s3_load<BKM, VB, false, true>(rsb, B, ldb, vob, n0, N, k0, kend, t, xb, ib);
    else
      s3_load<BKM, VB, false>(rsb, B, ldb, vob, n0, N, k0, kend, t, xb);
  };
  auto store_ab = [&](int stage, const float(&xa)[8], const float(&xb)[8]) {
    s3_store<AK>(As[stage], t, xa);
    s3_store<BKM>(Bs[stage], t, xb);
  };
  const int li = lane & 31, lh = lane >> 5;
  if (nfull > 0) {
    load_ab(0, ra[0], rb[0]);
    load_ab(1, ra[1], rb[1]);
    store_ab(0, ra[0], rb[0]);
    __syncthreads();
    int kt = 0;
    for (; kt + 1 < nfull; kt += 2) {
      // tile kt from stage 0; tile kt+1 (set 1) -> stage 1; set 0 <- tile kt+2
      load_ab(kt + 2, ra[0], rb[0]);
      s3_mma<AK, BKM>(As[0], Bs[0], wm * 64, wn * 64, li, lh, acc);
      store_ab(1, ra[1], rb[1]);
      __syncthreads();
      // tile kt+1 from stage 1; tile kt+2 (set 0) -> stage 0; set 1 <- tile kt+3
      load_ab(kt + 3, ra[1], rb[1]);
      s3_mma<AK, BKM>(As[1], Bs[1], wm * 64, wn * 64, li, lh, acc);
      store_ab(0, ra[0], rb[0]);
      __syncthreads();
    }
    if (nfull & 1) {  // odd count: the last full tile is in stage 0
      s3_mma<AK, BKM>(As[0], Bs[0], wm * 64, wn * 64, li, lh, acc);
      __syncthreads();
    }
  }
  if (kbeg + nfull * S3_BK < kend) {  // k tail
    const int k0 = kbeg + nfull * S3_BK;
    if (IDX && !AK && ia)
      s3_load<AK, VA, true, true>(rsa, A, lda, voa, m0, M, k0, kend, t, ra[0], ia);
    else
      s3_load<AK, VA, true>(rsa, A, lda, voa, m0, M, k0, kend, t, ra[0]);
    if (IDX && BKM && ib)
      s3_load<BKM, VB, true, true>(rsb, B, ldb, vob, n0, N, k0, kend, t, rb[0], ib);
    else
      s3_load<BKM, VB, true>(rsb, B, ldb, vob, n0, N, k0, kend, t, rb[0]);
    store_ab(0, ra[0], rb[0]);
    __syncthreads();
    s3_mma<AK, BKM>(As[0], Bs[0], wm * 64, wn * 64, li, lh, acc);
  }

  if (piece >= 0) {  // a tail tile's k piece: the whole 128 x 128 tile, tile-local, into its slab slot
    float* __restrict__ P = part + (int64_t)piece * (BM * BN);
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r)
          P[(wm * 64 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh) * BN + wn * 64 + j * 32 + li] = acc[i][j][r];
    return;
  }
  float* __restrict__ Cb;
  int64_t ldo;
  if (splits > 1) {
    Cb = part + (int64_t)tz * M * N;
    ldo = N;
  } else {
    Cb = bt.C[b];
    ldo = ldc;
  }
#pragma unroll
  for (int i = 0; i < 2; ++i) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int n = n0 + wn * 64 + j * 32 + li;
      if (n >= N) continue;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = m0 + wm * 64 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
        if (m < M) Cb[(int64_t)m * ldo + n] = acc[i][j][r];
      }
    }
  }
}

// ---------------------------------------------------------------------------------------------
// "split3w": the split3 kernel with twice the output per wave (round 6).
//
// The 128 x 128 split3 tile gives each wave a 64 x 64 output: per k16 stage 24 MFMAs against 12
// ds_read_b128, 16 split floats per thread and one barrier. Here the tile is 128 x 256 (the same
// 2 x 2 waves, each 64 x 128 = 2 x 4 blocks of 32 x 32): per stage 48 MFMAs against 18 reads, 24
// split floats per thread and still one barrier — a quarter fewer LDS reads and split
// instructions per MFMA and half the barriers. The price is the register file: 128 accumulators,
// so two workgroups per CU (8 waves) instead of three, and LDS 72 KB per workgroup. The B operand
// of a stage is two 128-row halves, each loaded, split and stored exactly as split3 does its B.
// Every output element accumulates the same pieces in the same order as split3 (per k16 step the
// six products h·h .. l·h, small terms first): whole tiles are bit-identical to split3's.
// ---------------------------------------------------------------------------------------------
constexpr int W_BN = 2 * BN;  // 256

// piece-image chunk offset (bf16 units) for an image of R rows (split3's s3_chunk at R = 128)
template <bool KMAJ, int R>
__device__ __forceinline__ int s3w_chunk(int row, int h) {
  if constexpr (KMAJ) return (h * R + row) * 8;
  else return (2 * row + (h ^ ((row >> 3) & 1))) * 8;
}

// split 8 floats of (row rr, k half kh) into the three piece images (each R x 16 bf16)
template <bool KMAJ, int R>
__device__ __forceinline__ void s3w_store(unsigned short* __restrict__ S, int rr, int kh, const float v[8]) {
  u4v ph, pm, pl;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const float x0 = v[2 * j], x1 = v[2 * j + 1];
    const unsigned int h0 = __float_as_uint(x0) & 0xffff0000u, h1 = __float_as_uint(x1) & 0xffff0000u;
    const float r0 = x0 - __uint_as_float(h0), r1 = x1 - __uint_as_float(h1);
    const unsigned int m0 = __float_as_uint(r0) & 0xffff0000u, m1 = __float_as_uint(r1) & 0xffff0000u;
    const float l0 = r0 - __uint_as_float(m0), l1 = r1 - __uint_as_float(m1);
    ph[j] = __builtin_amdgcn_perm(h1, h0, 0x07060302u);
    pm[j] = __builtin_amdgcn_perm(m1, m0, 0x07060302u);
    pl[j] = __builtin_amdgcn_perm(__float_as_uint(l1), __float_as_uint(l0), 0x07060302u);
  }
  const int off = s3w_chunk<KMAJ, R>(rr, kh);
  *reinterpret_cast<u4v*>(S + off) = ph;
  *reinterpret_cast<u4v*>(S + R * S3_BK + off) = pm;
  *reinterpret_cast<u4v*>(S + 2 * R * S3_BK + off) = pl;
}

template <bool KMAJ, int R>
__device__ __forceinline__ bf8v s3w_frag(const unsigned short* __restrict__ S, int piece, int row, int h) {
  return __builtin_bit_cast(bf8v, *reinterpret_cast<const u4v*>(S + piece * R * S3_BK + s3w_chunk<KMAJ, R>(row, h)));
}

// one k16 step: the wave's 2 x 4 blocks, per B block its three pieces, the six products in
// split3's order
template <bool AK, bool BKM>
__device__ __forceinline__ void s3w_mma(const unsigned short* __restrict__ Sa, const unsigned short* __restrict__ Sb,
                                        int ra0, int rb0, int li, int lh, f16v acc[2][4]) {
  bf8v a[2][3];
#pragma unroll
  for (int p = 0; p < 3; ++p)
#pragma unroll
    for (int i = 0; i < 2; ++i) a[i][p] = s3w_frag<AK, BM>(Sa, p, ra0 + i * 32 + li, lh);
  constexpr int PA[6] = {2, 1, 0, 1, 0, 0};
  constexpr int PB[6] = {0, 1, 2, 0, 1, 0};
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    bf8v bb[3];
#pragma unroll
    for (int p = 0; p < 3; ++p) bb[p] = s3w_frag<BKM, W_BN>(Sb, p, rb0 + j * 32 + li, lh);
#pragma unroll
    for (int q = 0; q < 6; ++q)
#pragma unroll
      for (int i = 0; i < 2; ++i)
        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i][PA[q]], bb[PB[q]], acc[i][j], 0, 0, 0);
  }
}

// two workgroups per CU: LDS 72 KB each, up to 256 registers (2 waves per SIMD)
template <bool AK, bool BKM, int VA, int VB, bool IDX = false>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2, 2))) void gemm_s3w_kernel(
    Batch bt, int M, int N, int K, int64_t lda, int64_t ldb, int64_t ldc, int splits, int klen, float* __restrict__ part,
    int64_t abytes, int64_t bbytes, int xcd_map) {
  __shared__ __attribute__((aligned(16))) unsigned short As[2][S3_OPER];
  __shared__ __attribute__((aligned(16))) unsigned short Bs[2][2 * S3_OPER];
  const int t = threadIdx.x;
  const int lane = t & 63;
  const int wid = t >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  int tx = blockIdx.x, ty = blockIdx.y, tz = blockIdx.z;
  if (xcd_map) {  // consecutive tiles on one XCD (split3's map)
    const int gx = gridDim.x, gy = gridDim.y;
    const int total = gx * gy * gridDim.z;
    const int hw = blockIdx.x + gx * (blockIdx.y + gy * blockIdx.z);
    const int per = total >> 3;
    const int lg = hw < per * 8 ? (hw & 7) * per + (hw >> 3) : hw;
    tx = lg % gx;
    ty = (lg / gx) % gy;
    tz = lg / (gx * gy);
  }
  const int b = tz / splits;
  const int split = tz % splits;
  const int m0 = ty * BM;
  const int n0 = tx * W_BN;
  const int kbeg = split * klen;
  const int kend = min(K, kbeg + klen);
  const float* __restrict__ A = bt.A[b];
  const float* __restrict__ B = bt.B[b];
  const __amdgpu_buffer_rsrc_t rsa = s3_rsrc(A, abytes), rsb = s3_rsrc(B, bbytes);
  const int64_t* __restrict__ ia = (IDX && !AK) ? bt.ia[b] : nullptr;
  const int64_t* __restrict__ ib = (IDX && BKM) ? bt.ib[b] : nullptr;
  const int voa = s3_voff<AK>(lda, m0, M, t, ia);
  const int vob0 = s3_voff<BKM>(ldb, n0, N, t), vob1 = s3_voff<BKM>(ldb, n0 + BN, N, t);
  const int ar = AK ? (t & 127) : (t >> 1), ah = AK ? (t >> 7) : (t & 1);     // A's (row, k half)
  const int br = BKM ? (t & 127) : (t >> 1), bh = BKM ? (t >> 7) : (t & 1);  // B's, per 128-row half

  f16v acc[2][4];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f16v(0.0f);

  float ra[2][8], rb[2][16];
  const int nfull = (kend - kbeg) / S3_BK;
  auto load_b = [&](int k0, int half, int vob, float* xb, bool guard) {
    if (guard) {
      if (IDX && BKM && ib)
        s3_load<BKM, VB, true, true>(rsb, B, ldb, vob, n0 + half * BN, N, k0, kend, t, xb, ib);
      else
        s3_load<BKM, VB, true>(rsb, B, ldb, vob, n0 + half * BN, N, k0, kend, t, xb);
    } else {
      if (IDX && BKM && ib)
        s3_load<BKM, VB, false, true>(rsb, B, ldb, vob, n0 + half * BN, N, k0, kend, t, xb, ib);
      else
        s3_load<BKM, VB, false>(rsb, B, ldb, vob, n0 + half * BN, N, k0, kend, t, xb);
    }
  };
  auto load_ab = [&](int kt, float(&xa)[8], float(&xb)[16]) {
    const int k0 = kbeg + min(kt, nfull - 1) * S3_BK;
    s3_load<AK, VA, false>(rsa, A, lda, voa, m0, M, k0, kend, t, xa);
    load_b(k0, 0, vob0, xb, false);
    load_b(k0, 1, vob1, xb + 8, false);
  };
  auto store_ab = [&](int stage, const float(&xa)[8], const float(&xb)[16]) {
    s3w_store<AK, BM>(As[stage], ar, ah, xa);
    s3w_store<BKM, W_BN>(Bs[stage], br, bh, xb);
    s3w_store<BKM, W_BN>(Bs[stage], br + BN, bh, xb + 8);
  };
  const int li = lane & 31, lh = lane >> 5;
  if (nfull > 0) {
    load_ab(0, ra[0], rb[0]);
    load_ab(1, ra[1], rb[1]);
    store_ab(0, ra[0], rb[0]);
    __syncthreads();
    int kt = 0;
    for (; kt + 1 < nfull; kt += 2) {
      load_ab(kt + 2, ra[0], rb[0]);
      s3w_mma<AK, BKM>(As[0], Bs[0], wm * 64, wn * 128, li, lh, acc);
      store_ab(1, ra[1], rb[1]);
      __syncthreads();
      load_ab(kt + 3, ra[1], rb[1]);
      s3w_mma<AK, BKM>(As[1], Bs[1], wm * 64, wn * 128, li, lh, acc);
      store_ab(0, ra[0], rb[0]);
      __syncthreads();
    }
    if (nfull & 1) {
      s3w_mma<AK, BKM>(As[0], Bs[0], wm * 64, wn * 128, li, lh, acc);
      __syncthreads();
    }
  }
  if (kbeg + nfull * S3_BK < kend) {  // k tail
    const int k0 = kbeg + nfull * S3_BK;
    if (IDX && !AK && ia)
      s3_load<AK, VA, true, true>(rsa, A, lda, voa, m0, M, k0, kend, t, ra[0], ia);
    else
      s3_load<AK, VA, true>(rsa, A, lda, voa, m0, M, k0, kend, t, ra[0]);
    load_b(k0, 0, vob0, rb[0], true);
    load_b(k0, 1, vob1, rb[0] + 8, true);
    store_ab(0, ra[0], rb[0]);
    __syncthreads();
    s3w_mma<AK, BKM>(As[0], Bs[0], wm * 64, wn * 128, li, lh, acc);
  }
  float* __restrict__ Cb;
  int64_t ldo;
  if (splits > 1) {
    Cb = part + (int64_t)tz * M * N;
    ldo = N;
  } else {
    Cb = bt.C[b];
    ldo = ldc;
  }
#pragma unroll
  for (int i = 0; i < 2; ++i) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int n = n0 + wn * 128 + j * 32 + li;
      if (n >= N) continue;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = m0 + wm * 64 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
        if (m < M) Cb[(int64_t)m * ldo + n] = acc[i][j][r];
      }
    }
  }
}

// ---------------------------------------------------------------------------------

// The tail tiles' k pieces summed in piece order into C: 16 workgroups per tile, a float4 of the
// tile per thread.
__global__ __launch_bounds__(256) void gemm_tail_reduce_kernel(Batch bt, const float* __restrict__ part, int M, int N,
                                                               int64_t ldc, int tail_base, int tail_s) {
  const int tile = blockIdx.x >> 4;
  const int e4 = (blockIdx.x & 15) * 256 + threadIdx.x;  // float4 of the tile, 0 .. 4095
  const int ml = e4 >> 5, nl = (e4 & 31) * 4;
  const float* p = part + (int64_t)tile * tail_s * (BM * BN) + ml * BN + nl;
  f4 acc = *reinterpret_cast<const f4*>(p);
  for (int q = 1; q < tail_s; ++q) acc += *reinterpret_cast<const f4*>(p + (int64_t)q * (BM * BN));
  const int gx = (N + BN - 1) / BN, gy = (M + BM - 1) / BM;
  const int lg = tail_base + tile;
  const int m = ((lg / gx) % gy) * BM + ml, n = (lg % gx) * BN + nl;
  if (m >= M) return;
  float* c = bt.C[lg / (gx * gy)] + (int64_t)m * ldc + n;
  if (n + 0 < N) c[0] = acc.x;
  if (n + 1 < N) c[1] = acc.y;
  if (n + 2 < N) c[2] = acc.z;
  if (n + 3 < N) c[3] = acc.w;
}

// "p3": split3 on operands split ONCE into their three bf16 pieces in HBM (gnn_gemm_p3_pack_f32)
// instead of in every workgroup's registers. The split3 kernel spends ~3 of its ~5 vector
// instructions per MFMA on the split (and/sub/perm), and it is bound by the SIMD's issue port
// (profiles/round1/gemm_split3_pmc_summary.txt: MFMA busy 0.42-0.51, issue stalls 0.45-0.53); a
// packed operand costs 1.5x the fp32 bytes per tile but no vector work. Packed layout (per
// operand, viewed as R rows — M for A, N for B — by K): three planes [piece][k tile][R_pad][16]
// bf16, rows and k zero-padded to 128 / 16, so a thread's 16 bytes of (row, k half) are one
// coalesced load and the GEMM needs no guards. The pieces are the split3 kernel's (truncation,
// exact) and the MFMA schedule is the same (same k16 steps, same six products in the same
// order): results bit-identical to gnn_gemm_f32_split3 on shapes without split3's tail tiles
// (tail_plan; with GNN_GEMM_TAIL=0 on every shape).
// ---------------------------------------------------------------------------------
__device__ __forceinline__ void split_piece8(const float v[8], u4v& ph, u4v& pm, u4v& pl) {
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const f2 x = f2{v[2 * j], v[2 * j + 1]};
    const unsigned int h0 = __float_as_uint(x.x) & 0xffff0000u, h1 = __float_as_uint(x.y) & 0xffff0000u;
    const f2 r = x - f2{__uint_as_float(h0), __uint_as_float(h1)};
    const unsigned int m0 = __float_as_uint(r.x) & 0xffff0000u, m1 = __float_as_uint(r.y) & 0xffff0000u;
    const f2 l = r - f2{__uint_as_float(m0), __uint_as_float(m1)};
    ph[j] = __builtin_amdgcn_perm(h1, h0, 0x07060302u);
    pm[j] = __builtin_amdgcn_perm(m1, m0, 0x07060302u);
    pl[j] = __builtin_amdgcn_perm(__float_as_uint(l.y), __float_as_uint(l.x), 0x07060302u);
  }
}

// One (128-row block, k tile) per workgroup. m-major source (element (r, k) = src[row(r)*ld + k]):
// thread t takes row t >> 1, k half t & 1; k-major source (element (r, k) = src[row(k)*ld + r]):
// row t & 127, the wave-uniform k half t >> 7 (each of the 8 loads is one coalesced k row).
// idx (optional): the source's row index (r for m-major, k for k-major).
__global__ __launch_bounds__(256) void p3_pack_kernel(const float* __restrict__ src, int64_t ld, int kmajor,
                                                      const int64_t* __restrict__ idx, int R, int K, int Rp, int KT,
                                                      unsigned short* __restrict__ out) {
  const int t = threadIdx.x;
  const int r0 = blockIdx.x * 128;
  const int kt = blockIdx.y;
  const int rr = kmajor ? (t & 127) : (t >> 1);
  const int kh = kmajor ? (t >> 7) : (t & 1);
  const int r = r0 + rr;
  const int kb = kt * 16 + kh * 8;
  float v[8];
  if (!kmajor) {
    const float* q = (r < R) ? src + (idx ? idx[r] : (int64_t)r) * ld : nullptr;
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = (q && kb + i < K) ? q[kb + i] : 0.0f;
  } else {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int k = kb + i;
      v[i] = (r < R && k < K) ? src[(idx ? idx[k] : (int64_t)k) * ld + r] : 0.0f;
    }
  }
  u4v ph, pm, pl;
  split_piece8(v, ph, pm, pl);
  const int64_t plane = (int64_t)KT * Rp * 16;
  const int64_t o = ((int64_t)kt * Rp + r) * 16 + kh * 8;
  *reinterpret_cast<u4v*>(out + o) = ph;
  *reinterpret_cast<u4v*>(out + plane + o) = pm;
  *reinterpret_cast<u4v*>(out + 2 * plane + o) = pl;
}

struct PBatch {
  const unsigned short* A[MAX_BATCH];
  const unsigned short* B[MAX_BATCH];
  float* C[MAX_BATCH];
};

// The split3 kernel's tile, pipeline and MFMA schedule over packed operands: 3 x 16 bytes per
// operand per thread per k tile (one per piece) straight into the LDS images (m-major form).
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(3, 3))) void gemm_p3_kernel(
    PBatch bt, int M, int N, int Mp, int Np, int KT, int64_t ldc, int splits, int ktlen, float* __restrict__ part,
    int xcd_map) {
  __shared__ __attribute__((aligned(16))) unsigned short As[2][S3_OPER];
  __shared__ __attribute__((aligned(16))) unsigned short Bs[2][S3_OPER];
  const int t = threadIdx.x;
  const int lane = t & 63;
  const int wid = t >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  int tx = blockIdx.x, ty = blockIdx.y, tz = blockIdx.z;
  if (xcd_map) {
    const int gx = gridDim.x, gy = gridDim.y;
    const int total = gx * gy * gridDim.z;
    const int hw = blockIdx.x + gx * (blockIdx.y + gy * blockIdx.z);
    const int per = total >> 3;
    const int lg = hw < per * 8 ? (hw & 7) * per + (hw >> 3) : hw;
    tx = lg % gx;
    ty = (lg / gx) % gy;
    tz = lg / (gx * gy);
  }
  const int b = tz / splits;
  const int split = tz % splits;
  const int m0 = ty * BM;
  const int n0 = tx * BN;
  const int ktb = split * ktlen;
  const int kte = min(KT, ktb + ktlen);
  const int64_t aplane = (int64_t)KT * Mp * 16, bplane = (int64_t)KT * Np * 16;  // bf16 units
  const __amdgpu_buffer_rsrc_t rsa = __builtin_amdgcn_make_buffer_rsrc((void*)bt.A[b], (short)0,
                                                                      (int)(3 * aplane * 2), 0x00020000);
  const __amdgpu_buffer_rsrc_t rsb = __builtin_amdgcn_make_buffer_rsrc((void*)bt.B[b], (short)0,
                                                                      (int)(3 * bplane * 2), 0x00020000);
  const int rr = t >> 1, kh = t & 1;
  const int voa = ((m0 + rr) * 16 + kh * 8) * 2, vob = ((n0 + rr) * 16 + kh * 8) * 2;  // bytes
  const int off = s3_chunk<false>(rr, kh);

  f16v acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f16v(0.0f);

  u4v ra[2][3], rb[2][3];
  const int nfull = kte - ktb;
  auto load_ab = [&](int kt, u4v(&xa)[3], u4v(&xb)[3]) {
    const int k = ktb + min(kt, nfull - 1);
#pragma unroll
    for (int p = 0; p < 3; ++p) {
      xa[p] = __builtin_bit_cast(u4v, __builtin_amdgcn_raw_buffer_load_b128(
                                          rsa, voa, (int)((p * aplane + (int64_t)k * Mp * 16) * 2), 0));
      xb[p] = __builtin_bit_cast(u4v, __builtin_amdgcn_raw_buffer_load_b128(
                                          rsb, vob, (int)((p * bplane + (int64_t)k * Np * 16) * 2), 0));
    }
  };
  auto store_ab = [&](int stage, const u4v(&xa)[3], const u4v(&xb)[3]) {
#pragma unroll
    for (int p = 0; p < 3; ++p) {
      *reinterpret_cast<u4v*>(As[stage] + p * S3_PIECE + off) = xa[p];
      *reinterpret_cast<u4v*>(Bs[stage] + p * S3_PIECE + off) = xb[p];
    }
  };
  const int li = lane & 31, lh = lane >> 5;
  if (nfull > 0) {
    load_ab(0, ra[0], rb[0]);
    load_ab(1, ra[1], rb[1]);
    store_ab(0, ra[0], rb[0]);
    __syncthreads();
    int kt = 0;
    for (; kt + 1 < nfull; kt += 2) {
      load_ab(kt + 2, ra[0], rb[0]);
      s3_mma<false, false>(As[0], Bs[0], wm * 64, wn * 64, li, lh, acc);
      store_ab(1, ra[1], rb[1]);
      __syncthreads();
      load_ab(kt + 3, ra[1], rb[1]);
      s3_mma<false, false>(As[1], Bs[1], wm * 64, wn * 64, li, lh, acc);
      store_ab(0, ra[0], rb[0]);
      __syncthreads();
    }
    if (nfull & 1) {
      s3_mma<false, false>(As[0], Bs[0], wm * 64, wn * 64, li, lh, acc);
      __syncthreads();
    }
  }
  float* __restrict__ Cb;
  int64_t ldo;
  if (splits > 1) {
    Cb = part + (int64_t)tz * M * N;
    ldo = N;
  } else {
    Cb = bt.C[b];
    ldo = ldc;
  }
#pragma unroll
  for (int i = 0; i < 2; ++i) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int n = n0 + wn * 64 + j * 32 + li;
      if (n >= N) continue;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = m0 + wm * 64 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
        if (m < M) Cb[(int64_t)m * ldo + n] = acc[i][j][r];
      }
    }
  }
}

// Workgroup slots of the chip at each kernel's occupancy: f32-input kernel 2 per CU (80 KB of
// LDS each), split3 kernel 3 per CU (48 KB).
constexpr int64_t SLOTS_F32 = 2 * 256;
constexpr int64_t SLOTS_S3 = 3 * 256;

// Split count: the weight-gradient shapes have few output tiles and a long k, so split k
// until the tiles x splits fill the slots once — never past them: a second, nearly empty
// round of workgroups costs almost a full round (measured: 40 tiles x 12 splits = 480
// workgroups 190 µs, x 13 = 520 workgroups 255 µs). Each split keeps >= 256 of k.
int pick_splits(int64_t M, int64_t N, int64_t K, int nbatch, int64_t slots) {
  if (const char* e = getenv("GNN_GEMM_SPLITS")) return std::max(1, atoi(e));  // experiments
  const int64_t tiles = ceil_div(M, (int64_t)BM) * ceil_div(N, (int64_t)BN) * nbatch;
  if (tiles * 2 > slots) return 1;
  int64_t s = slots / tiles;
  s = std::min<int64_t>(s, std::max<int64_t>(1, K / 256));
  return (int)std::max<int64_t>(1, std::min<int64_t>(s, 64));
}

// The wide split3 kernel (128 x 256 tiles, two workgroups per CU). Measured per layer pair against
// split3 (scripts/gemm_bench.py, profiles/round6/gemm_wide/): the same rate per CU, so it wins only
// where its tile count fills the chip's 512 slots once while split3's 128 x 128 tiles need a second,
// partial round — the layer-0 forward (496 wide tiles against 992 on 768 slots: 118.8 vs 130.7 µs);
// it loses where it leaves half the slots empty (layer-1 forward, 272 tiles: 146.6 vs 101.6 µs) or
// spills into a second round (layer-1 input gradient, 544: 133.4 vs 109.1). In the training step the
// layer-0 gain does not survive the staging kernels beside it (their 58 KB LDS tables leave room for
// one 72 KB wide workgroup per CU: 175 µs under rocprofv3 against split3's 144; gpu_step 603.9 / 604.9
// vs 603.0 / 602.6 interleaved), so the default is off. GNN_GEMM_WIDE = -1: wide when k is not split
// and its tiles fill 85-100 % of the slots; 1: every product with N >= 256; 0 (default): never. A pure function of the shape and the batch count the split choice is made
// for, so a product launched alone (gemm_split3_as_batch) takes the same kernel and k splits as inside
// its batch, and the workspace query agrees with the launch.
constexpr int64_t SLOTS_S3W = 2 * 256;

bool use_wide(int64_t M, int64_t N, int64_t K, int nbatch) {
  const char* e = getenv("GNN_GEMM_WIDE");  // per call (tests and benches toggle it)
  const int mode = e ? atoi(e) : 0;
  if (mode == 0 || N < W_BN || K <= 0) return false;
  if (mode == 1) return true;
  if (getenv("GNN_GEMM_SPLITS")) return false;  // split experiments keep split3
  const int64_t tw = ceil_div(M, (int64_t)BM) * ceil_div(N, (int64_t)W_BN) * nbatch;
  return tw * 100 >= SLOTS_S3W * 85 && tw <= SLOTS_S3W;
}

int pick_splits_wide(int64_t M, int64_t N, int64_t K, int nbatch) {
  if (const char* e = getenv("GNN_GEMM_SPLITS")) return std::max(1, atoi(e));
  const int64_t tiles = ceil_div(M, (int64_t)BM) * ceil_div(N, (int64_t)W_BN) * nbatch;
  if (tiles * 2 > SLOTS_S3W) return 1;
  int64_t s = SLOTS_S3W / tiles;
  s = std::min<int64_t>(s, std::max<int64_t>(1, K / 256));
  return (int)std::max<int64_t>(1, std::min<int64_t>(s, 64));
}

// Tail tiles (split3, unsplit k): a launch of T tiles over 256 CUs whose last partial round holds
// only rem = T mod 256 tiles (the layer-1 forward's 544 = 2 x 256 + 32) pays for that round almost
// like a full one (scripts/gemm_tiles_probe.py: 512 tiles 104 us, 544 126 us, 768 139 us). The
// first T - rem tiles run whole and each tail tile is cut into S = 4 k pieces (>= 4 k tiles each),
// small pieces beside the whole tiles of 4 rem CUs; gemm_tail_reduce_kernel adds a tail tile's
// pieces in order (deterministic; those tiles are summed in S chains instead of one). rem <= 32
// only: at the layer-1 input gradient's 64 (1,088 tiles) the pieces + their reduction cost more
// than the round they save (profiles/round4/gemm_tail/); GNN_GEMM_TAIL=0 turns it off (A/B).
struct TailPlan {
  int base = 0;  // whole tiles
  int s = 0;     // pieces per tail tile (0: off)
  int rem = 0;
};

TailPlan tail_plan(int64_t M, int64_t N, int64_t K, int nbatch) {
  TailPlan tp;
  const int64_t T = ceil_div(M, (int64_t)BM) * ceil_div(N, (int64_t)BN) * nbatch;
  if (T <= 256 || T >= INT_MAX / 2) return tp;
  const int64_t rem = T % 256;
  if (rem == 0 || rem > 32) return tp;
  const int64_t S = std::min<int64_t>(std::min<int64_t>(256 / rem, 4), ceil_div(K, (int64_t)16) / 4);
  if (S < 2) return tp;
  tp.base = (int)(T - rem);
  tp.s = (int)S;
  tp.rem = (int)rem;
  return tp;
}

bool tail_enabled() {
  const char* e = getenv("GNN_GEMM_TAIL");  // per call (tests toggle it)
  return !(e && atoi(e) == 0);
}

size_t tail_bytes(const TailPlan& tp) { return (size_t)tp.rem * tp.s * BM * BN * sizeof(float); }

enum Algo { ALGO_F32 = 0, ALGO_S3 = 1 };

int64_t slots_of(int algo) { return algo == ALGO_S3 ? SLOTS_S3 : SLOTS_F32; }

// split_nbatch: the batch count the split-k choice is made for (0: nbatch). A product launched
// alone with split_nbatch = n sums in exactly the order it would inside a batch of n.
// Indexed operands (split3): ia / ib (per batch entry, NULL entries allowed) with the source's row
// count a_rows / b_rows (its extent for the buffer range); A is indexable when m-major, B when
// k-major.
struct RowIndex {
  const int64_t* const* ia = nullptr;
  int64_t a_rows = 0;
  const int64_t* const* ib = nullptr;
  int64_t b_rows = 0;
};

// batch_index (with split_nbatch > 0): which product of the mimicked batch this launch is, so that
// its tiles that the batched launch would run as tail pieces (tail_plan over the whole batch) run
// as the same pieces here — the same sums, bit for bit.
int gemm_run(int algo, int a_kmajor, int b_kmajor, int64_t M, int64_t N, int64_t K, int nbatch, const float* const* A,
             int64_t lda, const float* const* B, int64_t ldb, float* const* C, int64_t ldc, void* workspace,
             size_t workspace_bytes, void* stream, int split_nbatch = 0, const RowIndex* ri = nullptr,
             int batch_index = -1) {
  GNN_REQUIRE(M >= 0 && N >= 0 && K >= 0, "gnn_gemm_f32: negative size");
  GNN_REQUIRE(M < INT_MAX && N < INT_MAX && K < INT_MAX, "gnn_gemm_f32: sizes must be < 2^31");
  GNN_REQUIRE(nbatch >= 1 && nbatch <= MAX_BATCH, "gnn_gemm_f32: nbatch must be 1..%d", MAX_BATCH);
  if (M == 0 || N == 0) return 0;
  GNN_REQUIRE(A && B && C, "gnn_gemm_f32: NULL pointer array");
  GNN_REQUIRE(ldc >= N, "gnn_gemm_f32: ldc < N");
  GNN_REQUIRE(lda >= (a_kmajor ? M : K) && ldb >= (b_kmajor ? N : K), "gnn_gemm_f32: lda/ldb too small");
  GNN_REQUIRE(lda % 2 == 0 && ldb % 2 == 0, "gnn_gemm_f32: lda and ldb must be even (8-byte rows)");
  Batch bt{};
  int va = 4, vb = 4;  // 16-byte loads where every row allows them, else 8-byte
  for (int b = 0; b < nbatch; ++b) {
    GNN_REQUIRE(C[b] && (K == 0 || (A[b] && B[b])), "gnn_gemm_f32: NULL operand %d", b);
    GNN_REQUIRE((uintptr_t)A[b] % 8 == 0 && (uintptr_t)B[b] % 8 == 0, "gnn_gemm_f32: A/B not 8-byte aligned");
    if (lda % 4 || (uintptr_t)A[b] % 16) va = 2;
    if (ldb % 4 || (uintptr_t)B[b] % 16) vb = 2;
    bt.A[b] = A[b];
    bt.B[b] = B[b];
    bt.C[b] = C[b];
    bt.ia[b] = ri && ri->ia ? ri->ia[b] : nullptr;
    bt.ib[b] = ri && ri->ib ? ri->ib[b] : nullptr;
  }
  bool idx = false;
  for (int b = 0; b < nbatch; ++b) idx = idx || bt.ia[b] || bt.ib[b];
  GNN_REQUIRE(!idx || (algo == ALGO_S3 && (!ri->ia || !a_kmajor) && (!ri->ib || b_kmajor)),
              "gnn_gemm: row indices need split3, an m-major A or a k-major B");
  // split3 addresses operands by 32-bit buffer offsets: operands of >= 2 GiB take the f32-input kernel
  const int64_t arows = (ri && ri->ia) ? ri->a_rows : (a_kmajor ? K : M);
  const int64_t brows = (ri && ri->ib) ? ri->b_rows : (b_kmajor ? K : N);
  const int64_t abytes = K == 0 ? 0 : (arows - 1) * lda * 4 + (a_kmajor ? M : K) * 4;
  const int64_t bbytes = K == 0 ? 0 : (brows - 1) * ldb * 4 + (b_kmajor ? N : K) * 4;
  if (algo == ALGO_S3 && (abytes >= INT_MAX || bbytes >= INT_MAX)) {
    GNN_REQUIRE(!idx, "gnn_gemm: indexed operand of >= 2 GiB");
    algo = ALGO_F32;
  }
  hipStream_t st = (hipStream_t)stream;
  if (algo == ALGO_S3 && K > 0 && use_wide(M, N, K, split_nbatch > 0 ? split_nbatch : nbatch)) {
    const int splits = pick_splits_wide(M, N, K, split_nbatch > 0 ? split_nbatch : nbatch);
    int xcdm = 1;
    if (const char* e = getenv("GNN_GEMM_XCD")) xcdm = atoi(e) != 0;
    const int klen = splits > 1 ? (int)(ceil_div(ceil_div(K, (int64_t)splits), (int64_t)S3_BK) * S3_BK) : (int)K;
    if (splits > 1) {
      const size_t need = (size_t)splits * nbatch * M * N * sizeof(float);
      GNN_REQUIRE(workspace && workspace_bytes >= need, "gnn_gemm_f32: workspace too small (%zu < %zu)",
                  workspace_bytes, need);
    }
    const dim3 grid((unsigned)ceil_div(N, (int64_t)W_BN), (unsigned)ceil_div(M, (int64_t)BM),
                    (unsigned)(nbatch * splits));
    float* part = (float*)workspace;
#define GNN_GEMMW_LAUNCH(AK, BK, VA, VB)                                                                        \
  do {                                                                                                          \
    if (idx)                                                                                                    \
      gemm_s3w_kernel<AK, BK, VA, VB, true><<<grid, dim3(256), 0, st>>>(bt, (int)M, (int)N, (int)K, lda, ldb,   \
                                                                        ldc, splits, klen, part, abytes, bbytes, \
                                                                        xcdm);                                   \
    else                                                                                                        \
      gemm_s3w_kernel<AK, BK, VA, VB><<<grid, dim3(256), 0, st>>>(bt, (int)M, (int)N, (int)K, lda, ldb, ldc,    \
                                                                  splits, klen, part, abytes, bbytes, xcdm);    \
  } while (0)
#define GNN_GEMMW_V(AK, BK)                                    \
  do {                                                         \
    if (va == 4 && vb == 4) GNN_GEMMW_LAUNCH(AK, BK, 4, 4);    \
    else if (va == 4) GNN_GEMMW_LAUNCH(AK, BK, 4, 2);          \
    else if (vb == 4) GNN_GEMMW_LAUNCH(AK, BK, 2, 4);          \
    else GNN_GEMMW_LAUNCH(AK, BK, 2, 2);                       \
  } while (0)
    if (a_kmajor && b_kmajor) GNN_GEMMW_V(true, true);
    else if (a_kmajor) GNN_GEMMW_V(true, false);
    else if (b_kmajor) GNN_GEMMW_V(false, true);
    else GNN_GEMMW_V(false, false);
#undef GNN_GEMMW_V
#undef GNN_GEMMW_LAUNCH
    GNN_LAUNCHED("gemm_s3w_kernel");
    if (splits > 1) {
      const int64_t total = (int64_t)M * N * nbatch;
      bool vec4 = ldc == N && (M * N) % 4 == 0;
      for (int b = 0; b < nbatch; ++b) vec4 = vec4 && (uintptr_t)C[b] % 16 == 0;
      if (vec4) {
        const unsigned g = (unsigned)std::min<int64_t>(ceil_div(total / 4, (int64_t)256), 2048);
        gemm_splitk_reduce4_kernel<<<dim3(g), dim3(256), 0, st>>>(bt, part, M * N, splits, nbatch);
        GNN_LAUNCHED("gemm_splitk_reduce4_kernel");
      } else {
        const unsigned g = (unsigned)std::min<int64_t>(ceil_div(total, (int64_t)256), 2048);
        gemm_splitk_reduce_kernel<<<dim3(g), dim3(256), 0, st>>>(bt, part, (int)M, (int)N, ldc, splits, nbatch);
        GNN_LAUNCHED("gemm_splitk_reduce_kernel");
      }
    }
    return 0;
  }
  const int splits = K == 0 ? 1 : pick_splits(M, N, K, split_nbatch > 0 ? split_nbatch : nbatch, slots_of(algo));
  // XCD-aware tile map for split3 (2-8 % per layer pair, scripts/gemm_bench.py); GNN_GEMM_XCD=0 turns it off
  int xcdm = 1;
  if (const char* e = getenv("GNN_GEMM_XCD")) xcdm = atoi(e) != 0;
  int bkt = algo == ALGO_S3 ? S3_BK : 32;
  if (algo == ALGO_F32)
    if (const char* e = getenv("GNN_GEMM_BKT")) bkt = atoi(e) == 16 ? 16 : 32;  // experiments
  TailPlan tp;
  if (algo == ALGO_S3 && splits == 1 && split_nbatch == 0 && K > 0 && tail_enabled()) tp = tail_plan(M, N, K, nbatch);
  if (algo == ALGO_S3 && splits == 1 && split_nbatch > 0 && nbatch == 1 && batch_index >= 0 && K > 0 &&
      tail_enabled()) {
    // one product of a batch of split_nbatch, launched alone: the batch's tail tiles that are this
    // product's tiles [batch_index * T1, (batch_index + 1) * T1) run as the same k pieces
    const TailPlan full = tail_plan(M, N, K, split_nbatch);
    const int64_t T1 = ceil_div(M, (int64_t)BM) * ceil_div(N, (int64_t)BN);
    const int64_t lo = (int64_t)batch_index * T1;
    if (full.s > 0 && full.base < lo + T1) {
      tp.base = (int)std::max<int64_t>(0, full.base - lo);
      tp.s = full.s;
      tp.rem = (int)(T1 - tp.base);
      if (tp.base % 8) xcdm = 0;  // the kernel's XCD map of the whole tiles needs base % 8 == 0 (speed only)
    }
  }
  int klen = splits > 1 ? (int)(ceil_div(ceil_div(K, (int64_t)splits), (int64_t)bkt) * bkt) : (int)K;
  if (tp.s > 0) klen = (int)(ceil_div(ceil_div(K, (int64_t)tp.s), (int64_t)bkt) * bkt);
  if (splits > 1 || tp.s > 0) {
    const size_t need = splits > 1 ? (size_t)splits * nbatch * M * N * sizeof(float) : tail_bytes(tp);
    GNN_REQUIRE(workspace && workspace_bytes >= need, "gnn_gemm_f32: workspace too small (%zu < %zu)",
                workspace_bytes, need);
  }
  const dim3 grid = tp.s > 0 ? dim3((unsigned)(tp.base + tp.rem * tp.s))
                             : dim3((unsigned)ceil_div(N, (int64_t)BN), (unsigned)ceil_div(M, (int64_t)BM),
                                    (unsigned)(nbatch * splits));
  float* part = (float*)workspace;
#define GNN_GEMM_LAUNCH(AK, BK, VA, VB)                                                                     \
  do {                                                                                                        \
    if (algo == ALGO_S3 && idx)                                                                               \
      gemm_s3_kernel<AK, BK, VA, VB, true><<<grid, dim3(256), 0, st>>>(bt, (int)M, (int)N, (int)K, lda, ldb,  \
                                                                       ldc, splits, klen, part, abytes, bbytes, \
                                                                       xcdm, tp.base, tp.s);                    \
    else if (algo == ALGO_S3)                                                                                 \
      gemm_s3_kernel<AK, BK, VA, VB><<<grid, dim3(256), 0, st>>>(bt, (int)M, (int)N, (int)K, lda, ldb, ldc,  \
                                                                 splits, klen, part, abytes, bbytes, xcdm,    \
                                                                 tp.base, tp.s);                              \
    else if (bkt == 16)                                                                                       \
      gemm_f32_kernel<AK, BK, VA, VB, 16>                                                                     \
          <<<grid, dim3(256), 0, st>>>(bt, (int)M, (int)N, (int)K, lda, ldb, ldc, splits, klen, part);        \
    else                                                                                                      \
      gemm_f32_kernel<AK, BK, VA, VB, 32>                                                                     \
          <<<grid, dim3(256), 0, st>>>(bt, (int)M, (int)N, (int)K, lda, ldb, ldc, splits, klen, part);        \
  } while (0)
#define GNN_GEMM_V(AK, BK)                                    \
  do {                                                        \
    if (va == 4 && vb == 4) GNN_GEMM_LAUNCH(AK, BK, 4, 4);    \
    else if (va == 4) GNN_GEMM_LAUNCH(AK, BK, 4, 2);          \
    else if (vb == 4) GNN_GEMM_LAUNCH(AK, BK, 2, 4);          \
    else GNN_GEMM_LAUNCH(AK, BK, 2, 2);                       \
  } while (0)
  if (a_kmajor && b_kmajor) GNN_GEMM_V(true, true);
  else if (a_kmajor) GNN_GEMM_V(true, false);
  else if (b_kmajor) GNN_GEMM_V(false, true);
  else GNN_GEMM_V(false, false);
#undef GNN_GEMM_V
#undef GNN_GEMM_LAUNCH
  GNN_LAUNCHED(algo == ALGO_S3 ? "gemm_s3_kernel" : "gemm_f32_kernel");
  if (tp.s > 0) {
    gemm_tail_reduce_kernel<<<dim3((unsigned)(tp.rem * 16)), dim3(256), 0, st>>>(bt, part, (int)M, (int)N, ldc,
                                                                                tp.base, tp.s);
    GNN_LAUNCHED("gemm_tail_reduce_kernel");
  }
  if (splits > 1) {
    const int64_t total = (int64_t)M * N * nbatch;
    bool vec4 = ldc == N && (M * N) % 4 == 0;
    for (int b = 0; b < nbatch; ++b) vec4 = vec4 && (uintptr_t)C[b] % 16 == 0;
    if (vec4) {
      const unsigned g = (unsigned)std::min<int64_t>(ceil_div(total / 4, (int64_t)256), 2048);
      gemm_splitk_reduce4_kernel<<<dim3(g), dim3(256), 0, st>>>(bt, part, M * N, splits, nbatch);
      GNN_LAUNCHED("gemm_splitk_reduce4_kernel");
    } else {
      const unsigned g = (unsigned)std::min<int64_t>(ceil_div(total, (int64_t)256), 2048);
      gemm_splitk_reduce_kernel<<<dim3(g), dim3(256), 0, st>>>(bt, part, (int)M, (int)N, ldc, splits, nbatch);
      GNN_LAUNCHED("gemm_splitk_reduce_kernel");
    }
  }
  return 0;
}

size_t workspace_bytes_of(int algo, int64_t M, int64_t N, int64_t K, int nbatch) {
  if (M <= 0 || N <= 0 || K <= 0 || nbatch <= 0) return 0;
  if (algo == ALGO_S3 && use_wide(M, N, K, nbatch)) {
    const int s = pick_splits_wide(M, N, K, nbatch);
    return s > 1 ? (size_t)s * nbatch * M * N * sizeof(float) : 0;
  }
  const int s = pick_splits(M, N, K, nbatch, slots_of(algo));
  if (s > 1) return (size_t)s * nbatch * M * N * sizeof(float);
  return algo == ALGO_S3 ? tail_bytes(tail_plan(M, N, K, nbatch)) : 0;  // whatever GNN_GEMM_TAIL says
}

}  // namespace

extern "C" {

size_t gnn_gemm_f32_workspace_bytes(int64_t M, int64_t N, int64_t K, int nbatch) {
  return workspace_bytes_of(ALGO_F32, M, N, K, nbatch);
}

int gnn_gemm_f32(int a_kmajor, int b_kmajor, int64_t M, int64_t N, int64_t K, int nbatch, const float* const* A,
                 int64_t lda, const float* const* B, int64_t ldb, float* const* C, int64_t ldc, void* workspace,
                 size_t workspace_bytes, void* stream) {
  return gemm_run(ALGO_F32, a_kmajor, b_kmajor, M, N, K, nbatch, A, lda, B, ldb, C, ldc, workspace, workspace_bytes,
                  stream);
}

size_t gnn_gemm_p3_packed_bytes(int64_t R, int64_t K) {
  if (R <= 0 || K <= 0) return 0;
  return (size_t)3 * (size_t)ceil_div(K, (int64_t)16) * (size_t)(ceil_div(R, (int64_t)128) * 128) * 16 * 2;
}

int gnn_gemm_p3_pack_f32(const float* src, int64_t ld, int kmajor, const int64_t* idx, int64_t R, int64_t K,
                         void* out, size_t out_bytes, void* stream) {
  GNN_REQUIRE(R >= 0 && K >= 0 && R < INT_MAX && K < INT_MAX, "gnn_gemm_p3_pack_f32: bad size");
  if (R == 0 || K == 0) return 0;
  GNN_REQUIRE(src && out, "gnn_gemm_p3_pack_f32: NULL pointer");
  GNN_REQUIRE(out_bytes >= gnn_gemm_p3_packed_bytes(R, K), "gnn_gemm_p3_pack_f32: output too small");
  GNN_REQUIRE((uintptr_t)out % 16 == 0, "gnn_gemm_p3_pack_f32: output not 16-byte aligned");
  GNN_REQUIRE(gnn_gemm_p3_packed_bytes(R, K) < (size_t)INT_MAX, "gnn_gemm_p3_pack_f32: packed operand >= 2 GiB");
  const int Rp = (int)(ceil_div(R, (int64_t)128) * 128), KT = (int)ceil_div(K, (int64_t)16);
  p3_pack_kernel<<<dim3((unsigned)(Rp / 128), (unsigned)KT), dim3(256), 0, (hipStream_t)stream>>>(
      src, ld, kmajor, idx, (int)R, (int)K, Rp, KT, (unsigned short*)out);
  GNN_LAUNCHED("p3_pack_kernel");
  return 0;
}

size_t gnn_gemm_p3_workspace_bytes(int64_t M, int64_t N, int64_t K, int nbatch) {
  return workspace_bytes_of(ALGO_S3, M, N, K, nbatch);
}

int gnn_gemm_p3(int64_t M, int64_t N, int64_t K, int nbatch, const void* const* Ap, const void* const* Bp,
                float* const* C, int64_t ldc, void* workspace, size_t workspace_bytes, void* stream) {
  GNN_REQUIRE(M >= 0 && N >= 0 && K >= 0 && M < INT_MAX && N < INT_MAX && K < INT_MAX, "gnn_gemm_p3: bad size");
  GNN_REQUIRE(nbatch >= 1 && nbatch <= MAX_BATCH, "gnn_gemm_p3: nbatch must be 1..%d", MAX_BATCH);
  if (M == 0 || N == 0) return 0;
  GNN_REQUIRE(Ap && Bp && C && ldc >= N, "gnn_gemm_p3: NULL pointer array or ldc < N");
  PBatch bt{};
  for (int b = 0; b < nbatch; ++b) {
    GNN_REQUIRE(C[b] && (K == 0 || (Ap[b] && Bp[b])), "gnn_gemm_p3: NULL operand %d", b);
    GNN_REQUIRE((uintptr_t)Ap[b] % 16 == 0 && (uintptr_t)Bp[b] % 16 == 0, "gnn_gemm_p3: packed operands 16-byte aligned");
    bt.A[b] = (const unsigned short*)Ap[b];
    bt.B[b] = (const unsigned short*)Bp[b];
    bt.C[b] = C[b];
  }
  GNN_REQUIRE(gnn_gemm_p3_packed_bytes(M, K) < (size_t)INT_MAX && gnn_gemm_p3_packed_bytes(N, K) < (size_t)INT_MAX,
              "gnn_gemm_p3: packed operand >= 2 GiB");
  hipStream_t st = (hipStream_t)stream;
  const int Mp = (int)(ceil_div(M, (int64_t)128) * 128), Np = (int)(ceil_div(N, (int64_t)128) * 128);
  const int KT = (int)ceil_div(K, (int64_t)16);
  const int splits = K == 0 ? 1 : pick_splits(M, N, K, nbatch, SLOTS_S3);
  // the split3 kernel's k ranges: ceil(ceil(K / splits) / 16) k tiles per split
  const int ktlen = splits > 1 ? (int)ceil_div(ceil_div(K, (int64_t)splits), (int64_t)S3_BK) : KT;
  if (splits > 1) {
    const size_t need = (size_t)splits * nbatch * M * N * sizeof(float);
    GNN_REQUIRE(workspace && workspace_bytes >= need, "gnn_gemm_p3: workspace too small (%zu < %zu)", workspace_bytes,
                need);
  }
  int xcdm = 1;
  if (const char* e = getenv("GNN_GEMM_XCD")) xcdm = atoi(e) != 0;
  const dim3 grid((unsigned)(Np / BN), (unsigned)(Mp / BM), (unsigned)(nbatch * splits));
  float* part = (float*)workspace;
  gemm_p3_kernel<<<grid, dim3(256), 0, st>>>(bt, (int)M, (int)N, Mp, Np, KT, ldc, splits, ktlen, part, xcdm);
  GNN_LAUNCHED("gemm_p3_kernel");
  if (splits > 1) {
    Batch cb{};
    for (int b = 0; b < nbatch; ++b) cb.C[b] = C[b];
    const int64_t total = (int64_t)M * N * nbatch;
    bool vec4 = ldc == N && (M * N) % 4 == 0;
    for (int b = 0; b < nbatch; ++b) vec4 = vec4 && (uintptr_t)C[b] % 16 == 0;
    if (vec4) {
      const unsigned g = (unsigned)std::min<int64_t>(ceil_div(total / 4, (int64_t)256), 2048);
      gemm_splitk_reduce4_kernel<<<dim3(g), dim3(256), 0, st>>>(cb, part, M * N, splits, nbatch);
      GNN_LAUNCHED("gemm_splitk_reduce4_kernel");
    } else {
      const unsigned g = (unsigned)std::min<int64_t>(ceil_div(total, (int64_t)256), 2048);
      gemm_splitk_reduce_kernel<<<dim3(g), dim3(256), 0, st>>>(cb, part, (int)M, (int)N, ldc, splits, nbatch);
      GNN_LAUNCHED("gemm_splitk_reduce_kernel");
    }
  }
  return 0;
}

size_t gnn_gemm_f32_split3_workspace_bytes(int64_t M, int64_t N, int64_t K, int nbatch) {
  return workspace_bytes_of(ALGO_S3, M, N, K, nbatch);
}

int gnn_gemm_f32_split3(int a_kmajor, int b_kmajor, int64_t M, int64_t N, int64_t K, int nbatch,
                        const float* const* A, int64_t lda, const float* const* B, int64_t ldb, float* const* C,
                        int64_t ldc, void* workspace, size_t workspace_bytes, void* stream) {
  return gemm_run(ALGO_S3, a_kmajor, b_kmajor, M, N, K, nbatch, A, lda, B, ldb, C, ldc, workspace, workspace_bytes,
                  stream);
}

int gnn_gemm_f32_split3_indexed(int a_kmajor, int b_kmajor, int64_t M, int64_t N, int64_t K, int nbatch,
                                const float* const* A, int64_t lda, const int64_t* const* ia, int64_t a_rows,
                                const float* const* B, int64_t ldb, const int64_t* const* ib, int64_t b_rows,
                                float* const* C, int64_t ldc, void* workspace, size_t workspace_bytes, void* stream) {
  GNN_REQUIRE((!ia || a_rows > 0) && (!ib || b_rows > 0), "gnn_gemm_f32_split3_indexed: source rows");
  return gnn::gemm_split3_indexed(a_kmajor, b_kmajor, M, N, K, nbatch, A, lda, ia, a_rows, B, ldb, ib, b_rows, C, ldc,
                                  workspace, workspace_bytes, stream);
}

}  // extern "C"

namespace gnn {

int gemm_split3_as_batch(int a_kmajor, int b_kmajor, int64_t M, int64_t N, int64_t K, int nbatch, int split_nbatch,
                         int batch_index, const float* const* A, int64_t lda, const float* const* B, int64_t ldb,
                         float* const* C, int64_t ldc, void* workspace, size_t workspace_bytes, void* stream) {
  return gemm_run(ALGO_S3, a_kmajor, b_kmajor, M, N, K, nbatch, A, lda, B, ldb, C, ldc, workspace, workspace_bytes,
                  stream, split_nbatch, nullptr, batch_index);
}

int gemm_split3_indexed(int a_kmajor, int b_kmajor, int64_t M, int64_t N, int64_t K, int nbatch,
                        const float* const* A, int64_t lda, const int64_t* const* ia, int64_t a_rows,
                        const float* const* B, int64_t ldb, const int64_t* const* ib, int64_t b_rows,
                        float* const* C, int64_t ldc, void* workspace, size_t workspace_bytes, void* stream) {
  RowIndex ri;
  ri.ia = ia;
  ri.a_rows = a_rows;
  ri.ib = ib;
  ri.b_rows = b_rows;
  return gemm_run(ALGO_S3, a_kmajor, b_kmajor, M, N, K, nbatch, A, lda, B, ldb, C, ldc, workspace, workspace_bytes,
                  stream, 0, &ri);
}

}  // namespace gnn
