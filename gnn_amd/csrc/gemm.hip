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

// Workgroup slots of the chip at the kernel's occupancy (2 per CU: 80 KB of LDS each).
constexpr int64_t SLOTS = 2 * 256;

// Split count: the weight-gradient shapes have few output tiles and a long k, so split k
// until the tiles x splits fill the slots once — never past them: a second, nearly empty
// round of workgroups costs almost a full round (measured: 40 tiles x 12 splits = 480
// workgroups 190 µs, x 13 = 520 workgroups 255 µs). Each split keeps >= 256 of k.
int pick_splits(int64_t M, int64_t N, int64_t K, int nbatch) {
  if (const char* e = getenv("GNN_GEMM_SPLITS")) return std::max(1, atoi(e));  // experiments
  const int64_t tiles = ceil_div(M, (int64_t)BM) * ceil_div(N, (int64_t)BN) * nbatch;
  if (tiles * 2 > SLOTS) return 1;
  int64_t s = SLOTS / tiles;
  s = std::min<int64_t>(s, std::max<int64_t>(1, K / 256));
  return (int)std::max<int64_t>(1, std::min<int64_t>(s, 64));
}

}  // namespace

extern "C" {

size_t gnn_gemm_f32_workspace_bytes(int64_t M, int64_t N, int64_t K, int nbatch) {
  if (M <= 0 || N <= 0 || K <= 0 || nbatch <= 0) return 0;
  const int s = pick_splits(M, N, K, nbatch);
  return s > 1 ? (size_t)s * nbatch * M * N * sizeof(float) : 0;
}

int gnn_gemm_f32(int a_kmajor, int b_kmajor, int64_t M, int64_t N, int64_t K, int nbatch, const float* const* A,
                 int64_t lda, const float* const* B, int64_t ldb, float* const* C, int64_t ldc, void* workspace,
                 size_t workspace_bytes, void* stream) {
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
  }
  hipStream_t st = (hipStream_t)stream;
  const int splits = K == 0 ? 1 : pick_splits(M, N, K, nbatch);
  int bkt = 32;
  if (const char* e = getenv("GNN_GEMM_BKT")) bkt = atoi(e) == 16 ? 16 : 32;  // experiments
  const int klen = splits > 1 ? (int)(ceil_div(ceil_div(K, (int64_t)splits), (int64_t)bkt) * bkt) : (int)K;
  if (splits > 1) {
    const size_t need = (size_t)splits * nbatch * M * N * sizeof(float);
    GNN_REQUIRE(workspace && workspace_bytes >= need, "gnn_gemm_f32: workspace too small (%zu < %zu)",
                workspace_bytes, need);
  }
  const dim3 grid((unsigned)ceil_div(N, (int64_t)BN), (unsigned)ceil_div(M, (int64_t)BM), (unsigned)(nbatch * splits));
  float* part = (float*)workspace;
#define GNN_GEMM_LAUNCH(AK, BK, VA, VB)                                                                     \
  do {                                                                                                        \
    if (bkt == 16)                                                                                            \
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
  GNN_LAUNCHED("gemm_f32_kernel");
  if (splits > 1) {
    const int64_t total = (int64_t)M * N * nbatch;
    const unsigned g = (unsigned)std::min<int64_t>(ceil_div(total, (int64_t)256), 2048);
    gemm_splitk_reduce_kernel<<<dim3(g), dim3(256), 0, st>>>(bt, part, (int)M, (int)N, ldc, splits, nbatch);
    GNN_LAUNCHED("gemm_splitk_reduce_kernel");
  }
  return 0;
}

}  // extern "C"
