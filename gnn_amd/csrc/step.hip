// step.hip — native executor of one GraphSAGE / GCN training step's forward + backward
// (include/gnn_step.h).
//
// Reference (main.py:122-146): output = model(x0, adjs, sampled_nodes); loss = utils.loss(...);
// loss.backward() — GraphSageConvolution / GraphConvolution (models.py:6-64) per layer, GNN's
// head (models.py:86-97) and the BCE loss (utils.py:129-140), autograd for the backward.
//
// The Python path (gnn_amd.models fused=True) already runs every piece as a hand-written HIP
// kernel, but through ~45 autograd Functions and ctypes calls per step: 1.2-1.5 ms of host time
// against a 1.8 ms GPU step. This executor issues the same kernel sequence from C++ — one
// call per step, every intermediate carved from one caller-provided workspace — with the same
// numerics: the same kernels with the same arguments and routing (the split3 GEMM where its
// tiles fill the chip, the vendor GEMM (rocBLAS) for the small products), the same dropout
// seeds. Only the two products torch would run through its own reduction (the head's bias
// gradient, a column sum) use a fixed-order kernel here.
//
// Sequence (L layers, bottom-up index l; layer 0's input is the features, so it has no input
// gradient):
//   forward  l = 0..L-1:  feat = A_l·X (gnn_spmm_csr_f32);  [SAGE] xs = X[sampled] (row gather)
//                         [hB,] hW = [xs, feat]·[W_B, W_W]ᵀ  (one batched split3 launch or rocBLAS)
//                         Y_l = sage_norm(hB + b_B, hW + b_W)  (ELU, row standardise, scale/offset, dropout)
//   head:                 loss, z = BCE(linear(dropout(normalize(Y_{L-1}))))
//   backward head:        dz, dY_{L-1};  dW_h = dzᵀ·xd (rocBLAS), db_h = colsum(dz)
//   backward l = L-1..0:  dhB, dhW, dscale, doffset, dbB, dbW = sage_norm_bwd(dY_l)
//                         dW_B, dW_W = [dhB, dhW]ᵀ·[xs, feat]  (split-k split3 from 2048 rows)
//                         l >= 1: dxs, dfeat = [dhB, dhW]·[W_B, W_W];
//                                 dY_{l-1} = A_lᵀ·dfeat (+ dxs scattered through rmap, SAGE)
#include <hip/hip_runtime.h>
#include <rocblas/rocblas.h>

#include <algorithm>
#include <climits>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <string>

#include "common.h"
#include "gnn_layers.h"
#include "gnn_spmm.h"
#include "gnn_step.h"

namespace {

using gnn::align_up;
using gnn::ceil_div;

// db = Σ_rows dz (M x C, row-major): one workgroup per column, each thread a strided set of
// rows, then a fixed-order tree (deterministic). A thread per column summing all M rows in a
// dependent chain took ~48 us for 512 x 41.
__global__ __launch_bounds__(256) void colsum_kernel(const float* __restrict__ dz, int M, int C,
                                                     float* __restrict__ out) {
  __shared__ float red[4];
  const int c = blockIdx.x;
  float s = 0.0f;
  for (int r = threadIdx.x; r < M; r += 256) s += dz[(int64_t)r * C + c];
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) s += __shfl_xor(s, m);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) out[c] = (red[0] + red[1]) + (red[2] + red[3]);
}

// A bump allocator over the workspace; with base == nullptr it only measures.
struct Arena {
  char* base;
  size_t off = 0;
  template <typename T>
  T* take(int64_t count) {
    const size_t bytes = align_up((size_t)(count > 0 ? count : 1) * sizeof(T), 256);
    T* p = base ? (T*)(base + off) : nullptr;
    off += bytes;
    return p;
  }
};

int64_t L(const int64_t* d, int l, int f) { return d[GNN_STEP_HEADER + l * GNN_STEP_LAYER_SLOTS + f]; }
template <typename T>
T* P(const int64_t* d, int l, int f) {
  return (T*)(uintptr_t)L(d, l, f);
}
template <typename T>
T* HP(const int64_t* d, int f) {
  return (T*)(uintptr_t)d[f];
}

// The split3 GEMM takes an unsplit product when its 128 x 128 tiles cover the CUs
// (gnn_amd/fused.py _mfma_fills) and every operand meets its contract (_gemm_ok).
bool fills(int64_t M, int64_t N, int n) { return ceil_div(M, 128) * ceil_div(N, 128) * n >= 256; }
bool gemm_ok(const void* p, int64_t ld) { return ((uintptr_t)p % 8) == 0 && (ld % 2) == 0; }

std::mutex g_blas_mu;
rocblas_handle g_blas[64][2] = {};

// which = 0: the step's stream; 1: the aux stream (its own handle, so the two streams' small
// products never share a handle's workspace)
int blas_handle(rocblas_handle* h, int which = 0) {
  int dev = 0;
  GNN_HIP(hipGetDevice(&dev), "hipGetDevice");
  GNN_REQUIRE(dev >= 0 && dev < 64, "gnn_train_step: device index %d", dev);
  std::lock_guard<std::mutex> g(g_blas_mu);
  if (!g_blas[dev][which]) {
    if (rocblas_create_handle(&g_blas[dev][which]) != rocblas_status_success)
      return gnn::fail(-1, "rocblas_create_handle failed");
  }
  *h = g_blas[dev][which];
  return 0;
}

// The aux stream of a (device, priority): the work of a layer that does not depend on its
// aggregation — the x[sampled] gather and its GEMM in the forward, the weight-gradient GEMMs in
// the backward — can run there, beside the L2-gather-bound SpMM on the caller's stream. Forked and joined with events from a small
// per-stream pool; the pool's mutex is held for the whole step (events are re-recorded per call).
struct Aux {
  hipStream_t s = nullptr;
  hipEvent_t ev[24] = {};
  int next = 0;
  std::mutex mu;
  hipEvent_t take() { return ev[next++ % 24]; }
};
std::mutex g_aux_mu;
Aux* g_aux[64][4] = {};

int aux_of(hipStream_t st, Aux** out) {
  int dev = 0;
  GNN_HIP(hipGetDevice(&dev), "hipGetDevice");
  GNN_REQUIRE(dev >= 0 && dev < 64, "gnn_train_step: device index %d", dev);
  int prio = 0, lo = 0, hi = 0;
  GNN_HIP(hipStreamGetPriority(st, &prio), "hipStreamGetPriority");
  GNN_HIP(hipDeviceGetStreamPriorityRange(&lo, &hi), "hipDeviceGetStreamPriorityRange");
  const int slot = std::min(3, std::max(0, lo - prio));  // lo = least urgent
  std::lock_guard<std::mutex> g(g_aux_mu);
  Aux*& a = g_aux[dev][slot];
  if (!a) {
    std::unique_ptr<Aux> n(new Aux());
    GNN_HIP(hipStreamCreateWithPriority(&n->s, hipStreamNonBlocking, prio), "hipStreamCreateWithPriority");
    for (auto& e : n->ev) GNN_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming), "hipEventCreateWithFlags");
    a = n.release();
  }
  *out = a;
  return 0;
}

// `to` waits for everything issued so far on `from`
int fork_join(Aux* a, hipStream_t from, hipStream_t to) {
  hipEvent_t e = a->take();
  GNN_HIP(hipEventRecord(e, from), "hipEventRecord");
  GNN_HIP(hipStreamWaitEvent(to, e, 0), "hipStreamWaitEvent");
  return 0;
}

// GNN_STEP_GATHER=1: gather x[sampled] first even where the GEMMs could read it in place (A/B)
bool no_index() {
  // read per call, as f32_gemm() below (bench.py's `gemm_ab` pass toggles GNN_GEMM_ALGO)
  const char* e = getenv("GNN_STEP_GATHER");
  const char* a = getenv("GNN_GEMM_ALGO");
  return (e && atoi(e) != 0) || (a && std::string(a) == "f32");  // the f32 kernel has no indexed form
}

// GNN_GEMM_ALGO=f32: the layer GEMMs on the f32-input MFMA kernel (gnn_gemm_f32, exact fp32)
// instead of split3 — the same routing, x[sampled] gathered (no row-indexed operands), no aux
// stream. For the end-to-end A/B of the two kernels (gnn_amd.fused reads the same variable).
bool f32_gemm() {
  const char* e = getenv("GNN_GEMM_ALGO");  // read per call (bench.py's `gemm_ab` pass toggles it)
  return e && std::string(e) == "f32";
}

int gemm(int ak, int bk, int64_t M, int64_t N, int64_t K, int nb, const float* const* A, int64_t lda,
         const float* const* B, int64_t ldb, float* const* C, int64_t ldc, void* ws, size_t wsb, hipStream_t st) {
  if (f32_gemm()) return gnn_gemm_f32(ak, bk, M, N, K, nb, A, lda, B, ldb, C, ldc, ws, wsb, st);
  return gnn_gemm_f32_split3(ak, bk, M, N, K, nb, A, lda, B, ldb, C, ldc, ws, wsb, st);
}

size_t gemm_ws(int64_t M, int64_t N, int64_t K, int nb) {
  return std::max(gnn_gemm_f32_split3_workspace_bytes(M, N, K, nb), gnn_gemm_f32_workspace_bytes(M, N, K, nb));
}

// GNN_STEP_OVERLAP=1 turns the aux stream on. Off by default: measured on the Reddit config-2
// step it changed nothing (550 mini-batches/s either way; the layer-0/1 aggregations slowed from
// 239 to 261 us while the GEMMs ran beside them — the CUs are already saturated).
// GNN_STEP_FUSE_AGG=0: launch the top layer's backward aggregation on its own instead of folding
// it into the layer-1 tail backward (A/B; the values are bit-identical either way)
bool fuse_agg_enabled() {
  const char* e = getenv("GNN_STEP_FUSE_AGG");  // read per step (tests toggle it in-process)
  return !(e && atoi(e) == 0);
}

// GNN_STEP_SMALL_OVERLAP=0 keeps everything on the step's stream. By default the top layer's
// small, latency-bound pieces that do not depend on each other run on the aux stream: in the
// forward x[sampled] + linearB beside the aggregation + linearW; in the backward the head's and
// the top layer's weight gradients beside the input gradients and the layer below (same kernels,
// same handles' results: bit-identical).
bool small_overlap_enabled() {
  const char* e = getenv("GNN_STEP_SMALL_OVERLAP");
  return !(e && atoi(e) == 0);
}

bool overlap_enabled() {
  const char* e = getenv("GNN_STEP_OVERLAP");  // read per step (tests toggle it in-process)
  return e && atoi(e) != 0;
}

// Row-major products on rocBLAS (column-major underneath): the small layer-2 / head products.
int sgemm(rocblas_handle h, rocblas_operation ta, rocblas_operation tb, int64_t m, int64_t n, int64_t k,
          const float* A, int64_t lda, const float* B, int64_t ldb, float* C, int64_t ldc) {
  const float one = 1.0f, zero = 0.0f;
  if (rocblas_sgemm(h, ta, tb, (rocblas_int)m, (rocblas_int)n, (rocblas_int)k, &one, A, (rocblas_int)lda, B,
                    (rocblas_int)ldb, &zero, C, (rocblas_int)ldc) != rocblas_status_success)
    return gnn::fail(-1, "rocblas_sgemm failed (m %lld n %lld k %lld)", (long long)m, (long long)n, (long long)k);
  return 0;
}
// out (M x N) = x (M x K) · Wᵀ (W: N x K)
int mm_xwt(rocblas_handle h, const float* x, int64_t ldx, const float* W, int64_t ldw, float* out, int64_t ldo,
           int64_t M, int64_t N, int64_t K) {
  return sgemm(h, rocblas_operation_transpose, rocblas_operation_none, N, M, K, W, ldw, x, ldx, out, ldo);
}
// out (M x K) = g (M x N) · W (N x K)
int mm_gw(rocblas_handle h, const float* g, int64_t ldg, const float* W, int64_t ldw, float* out, int64_t ldo,
          int64_t M, int64_t K, int64_t N) {
  return sgemm(h, rocblas_operation_none, rocblas_operation_none, K, M, N, W, ldw, g, ldg, out, ldo);
}
// out (N x K) = gᵀ (g: M x N) · x (M x K)
int mm_gtx(rocblas_handle h, const float* g, int64_t ldg, const float* x, int64_t ldx, float* out, int64_t ldo,
           int64_t N, int64_t K, int64_t M) {
  return sgemm(h, rocblas_operation_none, rocblas_operation_transpose, K, N, M, x, ldx, g, ldg, out, ldo);
}

// The per-layer buffers of one step (carved in a fixed order: sizing and running share it).
struct LayerBufs {
  int64_t M, K, nnz, F, Fk, ldx, ldo, N, D;
  bool xs_gathered;  // false: x[sampled] is read in place by the split3 GEMMs (row-indexed X)
  const float* X;
  float *feat, *xs, *hB, *hW, *Y, *mean, *rstd;
  float *dY, *dhB, *dhW, *dxs, *dfeat;
  void *ws_fwd, *ws_bwd, *ws_norm, *ws_gemm_f, *ws_gemm_f2, *ws_gemm_dx, *ws_gemm_dw;
  size_t b_fwd, b_bwd, b_norm, b_gemm_f, b_gemm_dx, b_gemm_dw;
  // dY given as the aggregation of the layer above (its backward SpMM folded into this layer's
  // tail backward, gnn_sage_norm_bwd_agg_f32) instead of a dense buffer
  bool dy_agg;
  const int32_t *agg_rp, *agg_col, *agg_rmap;
  const float *agg_val, *agg_G, *agg_R;
};

struct Plan {
  int nl = 0, sage = 1;
  LayerBufs lb[GNN_STEP_MAX_LAYERS];
  float *xd, *z, *nrm, *rowloss, *dz, *dXh;
  int64_t Mh = 0, Dh = 0, C = 0;
};

int plan(const int64_t* d, Arena& ar, Plan& pl) {
  GNN_REQUIRE(d[GNN_SH_VERSION] == GNN_STEP_VERSION, "gnn_train_step: descriptor version %lld",
              (long long)d[GNN_SH_VERSION]);
  pl.nl = (int)d[GNN_SH_LAYERS];
  pl.sage = d[GNN_SH_KIND] == GNN_STEP_SAGE;
  GNN_REQUIRE(pl.nl >= 1 && pl.nl <= GNN_STEP_MAX_LAYERS, "gnn_train_step: %d layers", pl.nl);
  const int64_t N = d[GNN_SH_NHID];
  const int n = pl.sage ? 2 : 1;
  for (int l = 0; l < pl.nl; ++l) {
    LayerBufs& b = pl.lb[l];
    b.dy_agg = false;
    b.M = L(d, l, GNN_SL_M);
    b.K = L(d, l, GNN_SL_K);
    b.nnz = L(d, l, GNN_SL_NNZ);
    b.N = N;
    b.D = n * N;
    if (l == 0) {
      b.X = HP<const float>(d, GNN_SH_X0);
      b.ldx = d[GNN_SH_LDX0];
      b.F = d[GNN_SH_F0];
    } else {
      const LayerBufs& p = pl.lb[l - 1];
      GNN_REQUIRE(b.K == p.M, "gnn_train_step: layer %d has K = %lld, layer %d M = %lld", l, (long long)b.K, l - 1,
                  (long long)p.M);
      b.X = p.Y;
      b.ldx = p.D;
      b.F = p.D;
    }
    GNN_REQUIRE(b.F <= b.ldx && b.F > 0 && b.M > 0 && b.K > 0, "gnn_train_step: layer %d shape", l);
    // the aggregation's padded width (custom_sparse_ops.spmm_csr): 16-byte loads over whole
    // line-aligned rows when the input rows are padded (the 602-wide features in 608-float rows)
    b.Fk = b.F;
    if (b.F % 4 && b.ldx % 4 == 0 && ((uintptr_t)b.X % 16 == 0 || !ar.base) && b.ldx >= b.F + (4 - b.F % 4))
      b.Fk = b.F + (4 - b.F % 4);
    b.ldo = (b.Fk != b.F && b.ldx <= 2 * b.Fk) ? b.ldx : b.Fk;
    b.feat = ar.take<float>(b.M * b.ldo);
    b.xs = pl.sage ? ar.take<float>(b.M * b.ldo) : nullptr;
    b.hB = pl.sage ? ar.take<float>(b.M * N) : nullptr;
    b.hW = ar.take<float>(b.M * N);
    b.Y = ar.take<float>(b.M * b.D);
    b.mean = ar.take<float>(b.M);
    b.rstd = ar.take<float>(b.M);
    b.b_fwd = gnn_spmm_workspace_bytes(b.M, b.nnz, b.Fk, 0);
    b.ws_fwd = ar.take<char>((int64_t)b.b_fwd);
    b.b_gemm_f = gemm_ws(b.M, N, b.F, n);
    b.ws_gemm_f = ar.take<char>((int64_t)b.b_gemm_f);
    b.ws_gemm_f2 = pl.sage ? ar.take<char>((int64_t)b.b_gemm_f) : nullptr;  // the aux stream's product
  }
  const LayerBufs& top = pl.lb[pl.nl - 1];
  pl.Mh = top.M;
  pl.Dh = top.D;
  pl.C = d[GNN_SH_CLASSES];
  GNN_REQUIRE(pl.C > 0 && pl.C <= 256 && pl.Dh % 4 == 0 && pl.Dh <= 2048, "gnn_train_step: head %lld x %lld",
              (long long)pl.Dh, (long long)pl.C);
  pl.xd = ar.take<float>(pl.Mh * pl.Dh);
  pl.z = ar.take<float>(pl.Mh * pl.C);
  pl.nrm = ar.take<float>(pl.Mh);
  pl.rowloss = ar.take<float>(pl.Mh);
  pl.dz = ar.take<float>(pl.Mh * pl.C);
  pl.dXh = ar.take<float>(pl.Mh * pl.Dh);
  for (int l = pl.nl - 1; l >= 0; --l) {
    LayerBufs& b = pl.lb[l];
    b.dY = (l == pl.nl - 1) ? pl.dXh : pl.lb[l + 1].dfeat;  // placeholder, set below for l < nl-1
    b.dhB = pl.sage ? ar.take<float>(b.M * N) : nullptr;
    b.dhW = ar.take<float>(b.M * N);
    b.b_norm = gnn_sage_norm_bwd_workspace_bytes(b.M, b.D);
    b.ws_norm = ar.take<char>((int64_t)b.b_norm);
    b.b_gemm_dw = gemm_ws(N, b.F, b.M, n);
    b.ws_gemm_dw = ar.take<char>((int64_t)b.b_gemm_dw);
    if (l >= 1) {
      b.dxs = pl.sage ? ar.take<float>(b.M * b.F) : nullptr;
      b.dfeat = ar.take<float>(b.M * b.F);
      b.b_gemm_dx = gemm_ws(b.M, b.F, N, n);
      b.ws_gemm_dx = ar.take<char>((int64_t)b.b_gemm_dx);
      b.b_bwd = gnn_spmm_workspace_bytes(b.K, b.nnz, b.F, 0);
      b.ws_bwd = ar.take<char>((int64_t)b.b_bwd);
    } else {
      b.dxs = b.dfeat = nullptr;
      b.ws_gemm_dx = b.ws_bwd = nullptr;
      b.b_gemm_dx = b.b_bwd = 0;
    }
  }
  // dY of layer l < nl-1 is the input gradient of layer l+1 (K_{l+1} x F_{l+1} = M_l x D_l)
  for (int l = 0; l < pl.nl - 1; ++l) pl.lb[l].dY = ar.take<float>(pl.lb[l].M * pl.lb[l].D);
  return 0;
}

#define GNN_TRY(x)        \
  do {                    \
    int rc_ = (x);        \
    if (rc_) return rc_;  \
  } while (0)

}  // namespace

extern "C" {

size_t gnn_train_step_workspace_bytes(const int64_t* desc) {
  if (!desc) return 0;
  Arena ar{nullptr};
  Plan pl;
  if (plan(desc, ar, pl)) return 0;
  return ar.off;
}

int gnn_train_step_f32(const int64_t* d, void* workspace, size_t workspace_bytes, void* stream) {
  GNN_REQUIRE(d != nullptr, "gnn_train_step: NULL descriptor");
  Arena ar{(char*)workspace};
  Plan pl;
  {
    Arena dry{nullptr};
    Plan tmp;
    GNN_TRY(plan(d, dry, tmp));
    GNN_REQUIRE(workspace && workspace_bytes >= dry.off, "gnn_train_step: workspace too small (%zu < %zu)",
                workspace_bytes, dry.off);
    GNN_REQUIRE((uintptr_t)workspace % 256 == 0, "gnn_train_step: workspace not 256-byte aligned");
  }
  GNN_TRY(plan(d, ar, pl));
  hipStream_t st = (hipStream_t)stream;
  rocblas_handle h = nullptr;
  GNN_TRY(blas_handle(&h));
  if (rocblas_set_stream(h, st) != rocblas_status_success) return gnn::fail(-1, "rocblas_set_stream failed");
  const int n = pl.sage ? 2 : 1;
  const float p = [&] {
    float f;
    const int32_t bits = (int32_t)d[GNN_SH_PDROP_BITS];
    std::memcpy(&f, &bits, 4);
    return f;
  }();
  const int training = (int)d[GNN_SH_TRAINING];
  Aux* aux = nullptr;
  const bool big_ov = overlap_enabled() && !f32_gemm();  // the big layers' GEMMs beside their SpMMs (off)
  const bool small_ov = small_overlap_enabled();
  if (big_ov || small_ov) GNN_TRY(aux_of(st, &aux));
  std::unique_lock<std::mutex> aux_lock;
  if (aux) aux_lock = std::unique_lock<std::mutex>(aux->mu);
  bool aux_used = false;
  rocblas_handle ha = nullptr;  // the aux stream's handle (small products there)
  if (aux && small_ov) {
    GNN_TRY(blas_handle(&ha, 1));
    if (rocblas_set_stream(ha, aux->s) != rocblas_status_success) return gnn::fail(-1, "rocblas_set_stream failed");
  }
  // optional per-aggregation timing (GNN_SH_TIMING): arm the caller's event pair for the next
  // SpMM launch (gnn_spmm_set_timing_events) and record the call's shape beside it
  int64_t* const T = HP<int64_t>(d, GNN_SH_TIMING);
  int64_t nrec = 0;
  auto arm = [&](int64_t kind, int64_t l, int64_t M, int64_t K, int64_t nnz, int64_t F, int64_t Fk, int64_t ldx,
                 int64_t ldo, const void* X, const void* Y, int64_t res_rows) {
    if (!T || nrec >= T[0]) return;
    int64_t* r = T + 1 + GNN_STEP_TIMING_SLOTS * nrec++;
    gnn_spmm_set_timing_events((void*)r[0], (void*)r[1]);
    const int64_t v[] = {kind, l, M, K, nnz, F, Fk, ldx, ldo, (int64_t)(uintptr_t)X, (int64_t)(uintptr_t)Y, res_rows, 1};
    std::memcpy(r + 2, v, sizeof v);
  };
  // the staging gate (GNN_SH_STAGE_EVENT): recorded right after the chosen layer's forward
  // aggregation is issued
  auto stage_gate = [&](int l) -> int {
    if (d[GNN_SH_STAGE_EVENT] && l == (int)d[GNN_SH_STAGE_LAYER])
      GNN_HIP(hipEventRecord((hipEvent_t)d[GNN_SH_STAGE_EVENT], st), "hipEventRecord (stage gate)");
    return 0;
  };
  // phase (GNN_SH_PHASE): 1 = only layer 0's forward aggregation, into this workspace (a data-
  // parallel caller issues the next batch's while the gradient all-reduce runs); 2 = the step with
  // that aggregation already issued into this workspace by a phase-1 call (same descriptor plan)
  const int64_t phase = d[GNN_SH_PHASE];
  GNN_REQUIRE(phase >= 0 && phase <= 2, "gnn_train_step: phase %lld", (long long)phase);
  auto first_agg = [&]() -> int {
    const LayerBufs& b = pl.lb[0];
    return gnn_spmm_csr_f32(P<const int32_t>(d, 0, GNN_SL_ROWPTR), P<const int32_t>(d, 0, GNN_SL_COL),
                            P<const float>(d, 0, GNN_SL_VAL), b.M, b.K, b.nnz, b.X, b.ldx, b.feat, b.ldo, b.Fk,
                            b.ws_fwd, b.b_fwd, 0, st);
  };
  if (phase == 1) {
    GNN_TRY(first_agg());
    return stage_gate(0);
  }
  // ------------------------------------------------------------------ forward
  for (int l = 0; l < pl.nl; ++l) {
    LayerBufs& b = pl.lb[l];
    const int64_t N = b.N;
    const float* WB = P<const float>(d, l, GNN_SL_WB);
    const float* WW = P<const float>(d, l, GNN_SL_WW);
    if (pl.sage)
      GNN_REQUIRE(L(d, l, GNN_SL_NSAMPLED) == b.M, "gnn_train_step: layer %d sampled %lld != M %lld", l,
                  (long long)L(d, l, GNN_SL_NSAMPLED), (long long)b.M);
    const bool ok = gemm_ok(b.feat, b.ldo) && gemm_ok(WW, b.F) && (!pl.sage || gemm_ok(WB, b.F));
    // the top layer's small products (rocBLAS): x[sampled] + linearB on the aux stream beside A·X
    const bool small_side = ha && pl.sage && !(ok && fills(b.M, N, n));
    if (big_ov && pl.sage && ok && fills(b.M, N, n)) {
      // x[sampled] and linearB on the aux stream beside A·X and linearW; each product launched
      // alone with the split choice of the pair, so the sums are those of the batched launch
      b.xs_gathered = true;
      GNN_TRY(fork_join(aux, st, aux->s));
      GNN_TRY(gnn_gather_rows_f32(b.X, b.ldx, P<const int64_t>(d, l, GNN_SL_SAMPLED), b.xs, b.ldo, nullptr, b.M, b.F,
                                  aux->s));
      const float* Ab[1] = {b.xs};
      const float* Bb[1] = {WB};
      float* Cb[1] = {b.hB};
      GNN_TRY(gnn::gemm_split3_as_batch(0, 0, b.M, N, b.F, 1, 2, 0, Ab, b.ldo, Bb, b.F, Cb, N, b.ws_gemm_f2, b.b_gemm_f,
                                        aux->s));
      if (phase != 2 || l != 0) {
        arm(0, l, b.M, b.K, b.nnz, b.F, b.Fk, b.ldx, b.ldo, b.X, b.feat, 0);
        GNN_TRY(gnn_spmm_csr_f32(P<const int32_t>(d, l, GNN_SL_ROWPTR), P<const int32_t>(d, l, GNN_SL_COL),
                                 P<const float>(d, l, GNN_SL_VAL), b.M, b.K, b.nnz, b.X, b.ldx, b.feat, b.ldo, b.Fk,
                                 b.ws_fwd, b.b_fwd, 0, st));
        GNN_TRY(stage_gate(l));
      }
      const float* Aw[1] = {b.feat};
      const float* Bw[1] = {WW};
      float* Cw[1] = {b.hW};
      GNN_TRY(gnn::gemm_split3_as_batch(0, 0, b.M, N, b.F, 1, 2, 1, Aw, b.ldo, Bw, b.F, Cw, N, b.ws_gemm_f, b.b_gemm_f, st));
      GNN_TRY(fork_join(aux, aux->s, st));
    } else if (small_side) {
      b.xs_gathered = true;
      GNN_TRY(fork_join(aux, st, aux->s));  // aux sees X complete
      GNN_TRY(gnn_gather_rows_f32(b.X, b.ldx, P<const int64_t>(d, l, GNN_SL_SAMPLED), b.xs, b.ldo, nullptr, b.M,
                                  b.F, aux->s));
      GNN_TRY(mm_xwt(ha, b.xs, b.ldo, WB, b.F, b.hB, N, b.M, N, b.F));
      if (phase != 2 || l != 0) {
        arm(0, l, b.M, b.K, b.nnz, b.F, b.Fk, b.ldx, b.ldo, b.X, b.feat, 0);
        GNN_TRY(gnn_spmm_csr_f32(P<const int32_t>(d, l, GNN_SL_ROWPTR), P<const int32_t>(d, l, GNN_SL_COL),
                                 P<const float>(d, l, GNN_SL_VAL), b.M, b.K, b.nnz, b.X, b.ldx, b.feat, b.ldo, b.Fk,
                                 b.ws_fwd, b.b_fwd, 0, st));
        GNN_TRY(stage_gate(l));
      }
      GNN_TRY(mm_xwt(h, b.feat, b.ldo, WW, b.F, b.hW, N, b.M, N, b.F));
      GNN_TRY(fork_join(aux, aux->s, st));  // the tail reads hB
    } else {
      if (phase != 2 || l != 0) {
        arm(0, l, b.M, b.K, b.nnz, b.F, b.Fk, b.ldx, b.ldo, b.X, b.feat, 0);
        GNN_TRY(gnn_spmm_csr_f32(P<const int32_t>(d, l, GNN_SL_ROWPTR), P<const int32_t>(d, l, GNN_SL_COL),
                                 P<const float>(d, l, GNN_SL_VAL), b.M, b.K, b.nnz, b.X, b.ldx, b.feat, b.ldo, b.Fk,
                                 b.ws_fwd, b.b_fwd, 0, st));
        GNN_TRY(stage_gate(l));
      }
      // x[sampled] feeds only linearB and its weight gradient: when both run on split3 (and X's
      // rows have the aggregation output's stride) the GEMMs read X's rows through the index
      // instead of a gathered copy (bit-identical operands)
      b.xs_gathered = !(pl.sage && ok && fills(b.M, N, n) && b.M >= 2048 && b.ldx == b.ldo && !no_index());
      if (pl.sage && b.xs_gathered)
        GNN_TRY(gnn_gather_rows_f32(b.X, b.ldx, P<const int64_t>(d, l, GNN_SL_SAMPLED), b.xs, b.ldo, nullptr, b.M,
                                    b.F, st));
    }
    if ((big_ov && pl.sage && ok && fills(b.M, N, n)) || small_side) {
      // done above
    } else if (ok && fills(b.M, N, n) && !b.xs_gathered) {
      const float* A[2] = {b.X, b.feat};
      const int64_t* IA[2] = {P<const int64_t>(d, l, GNN_SL_SAMPLED), nullptr};
      const float* B[2] = {WB, WW};
      float* Cc[2] = {b.hB, b.hW};
      GNN_TRY(gnn::gemm_split3_indexed(0, 0, b.M, N, b.F, n, A, b.ldo, IA, b.K, B, b.F, nullptr, 0, Cc, N,
                                       b.ws_gemm_f, b.b_gemm_f, st));
    } else if (ok && fills(b.M, N, n)) {
      const float* A[2] = {pl.sage ? b.xs : b.feat, b.feat};
      const float* B[2] = {pl.sage ? WB : WW, WW};
      float* Cc[2] = {pl.sage ? b.hB : b.hW, b.hW};
      GNN_TRY(gemm(0, 0, b.M, N, b.F, n, A + (pl.sage ? 0 : 1), b.ldo, B + (pl.sage ? 0 : 1), b.F,
                                  Cc + (pl.sage ? 0 : 1), N, b.ws_gemm_f, b.b_gemm_f, st));
    } else {
      if (pl.sage) GNN_TRY(mm_xwt(h, b.xs, b.ldo, WB, b.F, b.hB, N, b.M, N, b.F));
      GNN_TRY(mm_xwt(h, b.feat, b.ldo, WW, b.F, b.hW, N, b.M, N, b.F));
    }
    GNN_TRY(gnn_sage_norm_fwd_f32(pl.sage ? b.hB : nullptr, pl.sage ? N : 4, pl.sage ? N : 0, b.hW, N, N,
                                  pl.sage ? P<const float>(d, l, GNN_SL_BB) : nullptr, P<const float>(d, l, GNN_SL_BW),
                                  P<const float>(d, l, GNN_SL_SCALE), P<const float>(d, l, GNN_SL_OFFSET), b.M, p,
                                  (uint64_t)L(d, l, GNN_SL_SEED), training, b.Y, b.D, b.mean, b.rstd, st));
  }
  // ------------------------------------------------------------------ head + loss
  const LayerBufs& top = pl.lb[pl.nl - 1];
  const float* Wh = HP<const float>(d, GNN_SH_HEAD_W);
  const uint64_t hseed = (uint64_t)d[GNN_SH_HEAD_SEED];
  const float* labels = HP<const float>(d, GNN_SH_LABELS);
  const int64_t ldl = d[GNN_SH_LDL];
  GNN_TRY(gnn_head_bce_fwd_f32(top.Y, top.D, pl.Mh, pl.Dh, Wh, HP<const float>(d, GNN_SH_HEAD_B), pl.C, labels, ldl, p,
                               hseed, training, pl.xd, pl.z, pl.nrm, pl.rowloss, HP<float>(d, GNN_SH_LOSS), st));
  // ------------------------------------------------------------------ backward
  GNN_TRY(gnn_head_bce_bwd_f32(top.Y, top.D, pl.Mh, pl.Dh, Wh, pl.C, labels, ldl, nullptr, p, hseed, training, pl.z,
                               pl.nrm, pl.dz, pl.dXh, pl.Dh, st));
  // gradient-ready events (GNN_SH_GRAD_EVENTS): the caller's DP exchange of a bucket starts there
  const int64_t* const E = HP<const int64_t>(d, GNN_SH_GRAD_EVENTS);
  auto grads_ready = [&](int64_t slot, hipStream_t s) -> int {
    if (E && slot < E[0] && E[slot]) GNN_HIP(hipEventRecord((hipEvent_t)E[slot], s), "hipEventRecord (grad event)");
    return 0;
  };
  // the head's weight and bias gradients (their inputs are final here). With the aux stream they
  // go there with the first small weight-gradient products of the backward below, behind the same
  // fork: every event recorded on or awaited by the step's stream costs it a ~7 us bubble between
  // kernels (profiles/round4/trace/), so the backward forks once, not twice.
  bool head_pending = true;
  auto head_grads = [&](hipStream_t s, rocblas_handle hh) -> int {
    GNN_TRY(mm_gtx(hh, pl.dz, pl.C, pl.xd, pl.Dh, HP<float>(d, GNN_SH_HEAD_GW), pl.Dh, pl.C, pl.Dh, pl.Mh));
    if (HP<float>(d, GNN_SH_HEAD_GB)) {
      colsum_kernel<<<dim3((unsigned)pl.C), dim3(256), 0, s>>>(pl.dz, (int)pl.Mh, (int)pl.C,
                                                             HP<float>(d, GNN_SH_HEAD_GB));
      GNN_LAUNCHED("colsum_kernel");
    }
    GNN_TRY(grads_ready(1, s));
    head_pending = false;
    return 0;
  };
  if (!ha) GNN_TRY(head_grads(st, h));
  for (int l = pl.nl - 1; l >= 0; --l) {
    LayerBufs& b = pl.lb[l];
    const int64_t N = b.N;
    const float* WB = P<const float>(d, l, GNN_SL_WB);
    const float* WW = P<const float>(d, l, GNN_SL_WW);
    if (b.dy_agg)  // the layer above's backward aggregation, computed as this tail reads its rows
      GNN_TRY(gnn_sage_norm_bwd_agg_f32(b.agg_rp, b.agg_col, b.agg_val, b.agg_G, b.D, b.agg_R, b.D, b.agg_rmap,
                                        pl.sage ? b.hB : nullptr, pl.sage ? N : 4, pl.sage ? N : 0, b.hW, N, N,
                                        pl.sage ? P<const float>(d, l, GNN_SL_BB) : nullptr,
                                        P<const float>(d, l, GNN_SL_BW), P<const float>(d, l, GNN_SL_SCALE), b.mean,
                                        b.rstd, b.M, p, (uint64_t)L(d, l, GNN_SL_SEED), training, b.dhB, b.dhW,
                                        P<float>(d, l, GNN_SL_GSCALE), P<float>(d, l, GNN_SL_GOFFSET),
                                        pl.sage ? P<float>(d, l, GNN_SL_GBB) : nullptr, P<float>(d, l, GNN_SL_GBW),
                                        b.ws_norm, b.b_norm, st));
    else
      GNN_TRY(gnn_sage_norm_bwd_f32(b.dY, b.D, pl.sage ? b.hB : nullptr, pl.sage ? N : 4, pl.sage ? N : 0, b.hW, N, N,
                                    pl.sage ? P<const float>(d, l, GNN_SL_BB) : nullptr, P<const float>(d, l, GNN_SL_BW),
                                    P<const float>(d, l, GNN_SL_SCALE), b.mean, b.rstd, b.M, p,
                                    (uint64_t)L(d, l, GNN_SL_SEED), training, b.dhB, b.dhW,
                                    P<float>(d, l, GNN_SL_GSCALE), P<float>(d, l, GNN_SL_GOFFSET),
                                    pl.sage ? P<float>(d, l, GNN_SL_GBB) : nullptr, P<float>(d, l, GNN_SL_GBW),
                                    b.ws_norm, b.b_norm, st));
    const bool ok = gemm_ok(b.feat, b.ldo) && gemm_ok(WW, b.F) && (!pl.sage || gemm_ok(WB, b.F));
    const float* G[2] = {pl.sage ? b.dhB : b.dhW, b.dhW};
    const int o = pl.sage ? 0 : 1;
    if (l >= 1) {  // input gradients (layer 0's input is the features)
      if (ok && fills(b.M, b.F, n)) {
        const float* B[2] = {pl.sage ? WB : WW, WW};
        float* Cc[2] = {pl.sage ? b.dxs : b.dfeat, b.dfeat};
        GNN_TRY(gemm(0, 1, b.M, b.F, N, n, G + o, N, B + o, b.F, Cc + o, b.F, b.ws_gemm_dx,
                                    b.b_gemm_dx, st));
      } else {
        if (pl.sage) GNN_TRY(mm_gw(h, b.dhB, N, WB, b.F, b.dxs, b.F, b.M, b.F, N));
        GNN_TRY(mm_gw(h, b.dhW, N, WW, b.F, b.dfeat, b.F, b.M, b.F, N));
      }
    }
    // weight gradients: split over the sampled rows on split3 from 2048 rows, else rocBLAS; on
    // the aux stream (joined at the end of the step) beside the input-gradient GEMM + A_lᵀ·dfeat
    float* gWB = pl.sage ? P<float>(d, l, GNN_SL_GWB) : nullptr;
    float* gWW = P<float>(d, l, GNN_SL_GWW);
    if (ok && b.M >= 2048) {
      const float* X[2] = {pl.sage ? (b.xs_gathered ? b.xs : b.X) : b.feat, b.feat};
      const int64_t* IB[2] = {pl.sage && !b.xs_gathered ? P<const int64_t>(d, l, GNN_SL_SAMPLED) : nullptr, nullptr};
      float* Cc[2] = {pl.sage ? gWB : gWW, gWW};
      hipStream_t sw = st;
      if (big_ov && l >= 1) {
        GNN_TRY(fork_join(aux, st, aux->s));
        sw = aux->s;
        aux_used = true;
      }
      if (pl.sage && !b.xs_gathered)
        GNN_TRY(gnn::gemm_split3_indexed(1, 1, N, b.F, b.M, n, G + o, N, nullptr, 0, X + o, b.ldo, IB + o, b.K,
                                         Cc + o, b.F, b.ws_gemm_dw, b.b_gemm_dw, sw));
      else
        GNN_TRY(gemm(1, 1, N, b.F, b.M, n, G + o, N, X + o, b.ldo, Cc + o, b.F, b.ws_gemm_dw,
                                    b.b_gemm_dw, sw));
      GNN_TRY(grads_ready(2 + l, sw));  // sw follows st's norm backward (fork_join)
    } else {
      // the small weight-gradient products (rocBLAS): on the aux stream beside the input gradients
      // and the layer below (their inputs are final: the norm backward and x[sampled] / A·X)
      hipStream_t sw = st;
      rocblas_handle hw = h;
      if (ha) {
        GNN_TRY(fork_join(aux, st, aux->s));
        sw = aux->s;
        hw = ha;
        aux_used = true;
        if (head_pending) GNN_TRY(head_grads(aux->s, ha));
      }
      if (pl.sage) GNN_TRY(mm_gtx(hw, b.dhB, N, b.xs, b.ldo, gWB, b.F, N, b.F, b.M));
      GNN_TRY(mm_gtx(hw, b.dhW, N, b.feat, b.ldo, gWW, b.F, N, b.F, b.M));
      GNN_TRY(grads_ready(2 + l, sw));
    }
    if (l >= 1) {  // dY_{l-1} = A_lᵀ·dfeat (+ dxs through rmap: the x[sampled] gradient)
      LayerBufs& prev = pl.lb[l - 1];
      GNN_REQUIRE(P<const int32_t>(d, l, GNN_SL_TROWPTR) != nullptr, "gnn_train_step: layer %d has no transpose", l);
      if (pl.sage) GNN_REQUIRE(P<const int32_t>(d, l, GNN_SL_RMAP) != nullptr, "gnn_train_step: layer %d has no row map", l);
      // short-row transposes (the top layer's: 1.7 nonzeros per row on the Reddit batch) that a
      // standalone call would run as one fmaf chain per row: folded into layer l-1's tail
      // backward, which computes each dY row as it reads it (no dY write / read back, no launch)
      if (fuse_agg_enabled() && prev.D == b.F &&
          gnn::spmm_row_chain(b.K, b.M, b.nnz, b.F, b.F, b.F, b.dfeat, prev.dY)) {
        prev.dy_agg = true;
        prev.agg_rp = P<const int32_t>(d, l, GNN_SL_TROWPTR);
        prev.agg_col = P<const int32_t>(d, l, GNN_SL_TCOL);
        prev.agg_val = P<const float>(d, l, GNN_SL_TVAL);
        prev.agg_G = b.dfeat;
        prev.agg_R = pl.sage ? b.dxs : nullptr;
        prev.agg_rmap = pl.sage ? P<const int32_t>(d, l, GNN_SL_RMAP) : nullptr;
      } else if (pl.sage) {
        GNN_REQUIRE(P<const int32_t>(d, l, GNN_SL_RMAP) != nullptr, "gnn_train_step: layer %d has no row map", l);
        arm(1, l, b.K, b.M, b.nnz, b.F, b.F, b.F, b.F, b.dfeat, prev.dY, b.M);
        GNN_TRY(gnn_spmm_csr_f32_ex(P<const int32_t>(d, l, GNN_SL_TROWPTR), P<const int32_t>(d, l, GNN_SL_TCOL),
                                    P<const float>(d, l, GNN_SL_TVAL), b.K, b.M, b.nnz, b.dfeat, b.F, prev.dY, b.F,
                                    b.F, b.dxs, b.F, P<const int32_t>(d, l, GNN_SL_RMAP), b.ws_bwd, b.b_bwd, 0, st));
      } else {
        arm(1, l, b.K, b.M, b.nnz, b.F, b.F, b.F, b.F, b.dfeat, prev.dY, 0);
        GNN_TRY(gnn_spmm_csr_f32(P<const int32_t>(d, l, GNN_SL_TROWPTR), P<const int32_t>(d, l, GNN_SL_TCOL),
                                 P<const float>(d, l, GNN_SL_TVAL), b.K, b.M, b.nnz, b.dfeat, b.F, prev.dY, b.F, b.F,
                                 b.ws_bwd, b.b_bwd, 0, st));
      }
    }
  }
  if (head_pending) {  // no small weight-gradient fork above: the head's own
    GNN_TRY(fork_join(aux, st, aux->s));
    GNN_TRY(head_grads(aux->s, ha));
    aux_used = true;
  }
  if (aux_used) GNN_TRY(fork_join(aux, aux->s, st));
  return 0;
}

}  // extern "C"
