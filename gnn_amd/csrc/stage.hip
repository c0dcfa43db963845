// stage.hip — a batch of the native loader staged on the device by one call (include/gnn_stage.h).
//
// Reference: main.py:129-134 (X0 from the GPU buffers and the host rows) and sampler.py:135-139
// (create_coo_tensor per layer). The Python pipeline issued the same work as ~25 interpreter /
// ctypes calls per batch on the training thread (staging.Stager.issue, loader.NativeBatch.
// to_device, sampler.DeviceBatch.build_operands): 0.2-0.3 ms per step, doubling when the host
// runs slow. Here the training thread makes two calls (plan, stage) and this file issues, on the
// staging stream, the library calls the Python path made, with the same arguments:
//   blob upload -> [gate] -> X0 gather (own-buffer + host rows, gnn_gather_rows2_f32) ->
//   per layer: gnn_ladies_extract_f32 (GPU-extracted) | gnn_build_operand_sorted_f32 (+ _t on the
//   blob's CSC) -> the extraction error flag into pinned host memory.
// No kernels of its own; nothing allocated (the caller's arena holds every output and the
// extraction workspace, which the layers reuse one after the other on the stream).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>

#include "common.h"
#include "gnn_extract.h"
#include "gnn_sampler.h"
#include "gnn_spmm.h"
#include "gnn_stage.h"

#define GNN_STAGE_TRY(x)  \
  do {                    \
    const int rc_ = (x);  \
    if (rc_) return rc_;  \
  } while (0)

namespace {

constexpr size_t kAlign = 256;

template <typename T>
T* AP(const int64_t* a, int slot) {
  return reinterpret_cast<T*>((uintptr_t)a[slot]);
}

// One batch as the descriptor describes it (host view of the section table).
struct BlobView {
  const int64_t* d;
  const char* host;
  char* dev;
  int nl;
  int64_t layer(int li) const { return GNN_BLOB_HEADER + (int64_t)li * GNN_BLOB_LAYER_SLOTS; }
  int64_t batch() const { return GNN_BLOB_HEADER + (int64_t)nl * GNN_BLOB_LAYER_SLOTS; }
  int64_t count(int64_t slot) const { return d[slot + 1]; }
  template <typename T>
  const T* h(int64_t slot) const {
    return reinterpret_cast<const T*>(host + d[slot]);
  }
  template <typename T>
  T* dv(int64_t slot) const {
    return reinterpret_cast<T*>(dev + d[slot]);
  }
};

// The totals a GPU-extracted layer's launch is sized by (the host's copies, as the Python path
// read them from the blob: U's row pointer at M and the lapᵀ segment offsets at K).
void seg_totals(const BlobView& b, int li, bool tr, int64_t& rowseg_total, int64_t& colseg_total) {
  const int64_t L = b.layer(li);
  const int64_t M = b.d[L + GNN_L_M], K = b.d[L + GNN_L_K];
  rowseg_total = b.h<int32_t>(L + GNN_L_FULLROWPTR)[M];
  colseg_total = tr ? b.h<int32_t>(L + GNN_L_COLSEG)[K] : 0;
}

// The arena layout; returns the bytes (0: invalid descriptor, error recorded).
size_t plan(const int64_t* a, int64_t* out) {
  const int64_t* d = AP<const int64_t>(a, GNN_ST_DESC);
  if (!d || !a[GNN_ST_HOST_BLOB]) {
    gnn::fail(GNN_EINVAL, "gnn_stage: NULL descriptor / blob");
    return 0;
  }
  if (d[GNN_H_VERSION] != GNN_BLOB_VERSION || d[GNN_H_LAYERS] < 0 || d[GNN_H_LAYERS] > GNN_BLOB_MAX_LAYERS) {
    gnn::fail(GNN_EINVAL, "gnn_stage: blob version %lld / layers %lld", (long long)d[GNN_H_VERSION],
              (long long)d[GNN_H_LAYERS]);
    return 0;
  }
  BlobView b{d, AP<const char>(a, GNN_ST_HOST_BLOB), nullptr, (int)d[GNN_H_LAYERS]};
  const int64_t csc_from = a[GNN_ST_CSC_FROM];
  size_t off = 0, ws = 0;
  auto take = [&](int64_t bytes) {
    const int64_t o = (int64_t)off;
    off += gnn::align_up((size_t)std::max<int64_t>(bytes, 1), kAlign);
    return o;
  };
  for (int li = 0; li < b.nl; ++li) {
    int64_t* o = out + (int64_t)li * GNN_STAGE_OUT_SLOTS;
    for (int k = 0; k < GNN_STAGE_OUT_SLOTS; ++k) o[k] = -1;
    const int64_t L = b.layer(li);
    if (!d[L + GNN_L_PRESENT]) continue;
    const int64_t M = d[L + GNN_L_M], K = d[L + GNN_L_K], nnz = d[L + GNN_L_NNZ];
    if (M < 0 || K < 0 || nnz < 0) {
      gnn::fail(GNN_EINVAL, "gnn_stage: layer %d has a negative size", li);
      return 0;
    }
    if (d[L + GNN_L_ON_DEVICE]) {
      const bool tr = li >= csc_from;
      if (b.count(L + GNN_L_FULLROWPTR) != M + 1 || (tr && b.count(L + GNN_L_COLSEG) != K + 1)) {
        gnn::fail(GNN_EINVAL, "gnn_stage: layer %d segment offsets do not match its shape", li);
        return 0;
      }
      int64_t rt, ct;
      seg_totals(b, li, tr, rt, ct);
      ws = std::max(ws, gnn_ladies_extract_workspace_bytes(a[GNN_ST_NUM_NODES], M, K, tr, rt, ct));
      o[GNN_SO_ROWPTR] = take((M + 1) * 4);
      o[GNN_SO_COL] = take(nnz * 4);
      o[GNN_SO_VAL] = take(nnz * 4);
      if (tr) {
        o[GNN_SO_ROWS_T] = take(nnz * 4);
        o[GNN_SO_VAL_T] = take(nnz * 4);
      }
    } else {
      if (b.count(L + GNN_L_COLIDX) != nnz || b.count(L + GNN_L_ROWPTR) != M + 1) {
        gnn::fail(GNN_EINVAL, "gnn_stage: layer %d CSR does not match its shape", li);
        return 0;
      }
      o[GNN_SO_COL] = take(nnz * 4);
      o[GNN_SO_VAL] = take(nnz * 4);
      if (b.count(L + GNN_L_CSC_COLPTR) > 0) o[GNN_SO_VAL_T] = take(nnz * 4);
    }
  }
  // the extraction workspace, after the outputs (layer 0's GNN_SO_WORKSPACE slot records where)
  if (b.nl > 0) out[GNN_SO_WORKSPACE] = ws ? take((int64_t)ws) : -1;
  return off > 0 ? off : kAlign;
}

}  // namespace

extern "C" {

size_t gnn_stage_plan(const int64_t* args, int64_t* out) {
  if (!args || !out) {
    gnn::fail(GNN_EINVAL, "gnn_stage_plan: NULL argument");
    return 0;
  }
  return plan(args, out);
}

int gnn_stage_batch_f32(const int64_t* a, void* stream) {
  GNN_REQUIRE(a, "gnn_stage_batch_f32: NULL arguments");
  // the layout the caller sized the arena by (gnn_stage_plan), recomputed: a few integer ops per layer
  int64_t out[GNN_BLOB_MAX_LAYERS * GNN_STAGE_OUT_SLOTS];
  const size_t need = plan(a, out);
  if (need == 0) return GNN_EINVAL;
  char* arena = AP<char>(a, GNN_ST_ARENA);
  GNN_REQUIRE(arena && (size_t)a[GNN_ST_ARENA_BYTES] >= need, "gnn_stage_batch_f32: arena too small (%lld < %zu)",
              (long long)a[GNN_ST_ARENA_BYTES], need);
  GNN_REQUIRE((uintptr_t)arena % kAlign == 0, "gnn_stage_batch_f32: arena not %zu-byte aligned", kAlign);
  const int64_t* d = AP<const int64_t>(a, GNN_ST_DESC);
  BlobView b{d, AP<const char>(a, GNN_ST_HOST_BLOB), AP<char>(a, GNN_ST_DEV_BLOB), (int)d[GNN_H_LAYERS]};
  GNN_REQUIRE(b.dev && (uintptr_t)b.dev % 16 == 0, "gnn_stage_batch_f32: device blob NULL or not 16-byte aligned");
  hipStream_t st = (hipStream_t)stream;
  // 1. the blob, one copy (the copy engine goes ahead of the gate)
  if (a[GNN_ST_UPLOAD]) GNN_STAGE_TRY(gnn_memcpy_h2d_async(b.dev, b.host, (size_t)d[GNN_H_BYTES], stream));
  if (a[GNN_ST_GATE]) GNN_HIP(hipStreamWaitEvent(st, (hipEvent_t)a[GNN_ST_GATE], 0), "hipStreamWaitEvent (gate)");
  // 2. X0: own-buffer rows and host rows in one launch
  const int64_t B = b.batch();
  const int64_t n_own = b.count(B + GNN_B_OWN_POS), nh = b.count(B + GNN_B_HOST_POS);
  const int64_t ld_x0 = a[GNN_ST_LD_X0];
  float* x0 = AP<float>(a, GNN_ST_X0);
  GNN_REQUIRE(x0 && ld_x0 == d[GNN_H_LD_X0], "gnn_stage_batch_f32: X0 NULL or its stride %lld != the blob's %lld",
              (long long)ld_x0, (long long)d[GNN_H_LD_X0]);
  GNN_REQUIRE(nh == 0 || b.count(B + GNN_B_HOST_ROWS) == nh * ld_x0,
              "gnn_stage_batch_f32: the blob holds no host rows (zero-copy batches stage through Python)");
  GNN_REQUIRE(n_own == 0 || a[GNN_ST_BUFFER], "gnn_stage_batch_f32: NULL feature buffer");
  GNN_STAGE_TRY(gnn_gather_rows2_f32(AP<const float>(a, GNN_ST_BUFFER), a[GNN_ST_LD_BUFFER],
                               b.dv<const int64_t>(B + GNN_B_OWN_SRC), b.dv<const int64_t>(B + GNN_B_OWN_POS), n_own,
                               nh ? b.dv<const float>(B + GNN_B_HOST_ROWS) : x0, ld_x0, nullptr,
                               b.dv<const int64_t>(B + GNN_B_HOST_POS), nh, x0, ld_x0, a[GNN_ST_F], stream));
  // 3. the operands
  const int64_t csc_from = a[GNN_ST_CSC_FROM];
  const int64_t ws_off = b.nl > 0 ? out[GNN_SO_WORKSPACE] : -1;
  bool extracted = false;
  for (int li = 0; li < b.nl; ++li) {
    const int64_t L = b.layer(li);
    if (!d[L + GNN_L_PRESENT]) continue;
    const int64_t* o = out + (int64_t)li * GNN_STAGE_OUT_SLOTS;
    const int64_t M = d[L + GNN_L_M], K = d[L + GNN_L_K], nnz = d[L + GNN_L_NNZ];
    auto O = [&](int k) -> void* { return o[k] >= 0 ? (void*)(arena + o[k]) : nullptr; };
    if (d[L + GNN_L_ON_DEVICE]) {
      const bool tr = li >= csc_from;
      GNN_REQUIRE(a[GNN_ST_INDPTR] && a[GNN_ST_INDICES] && a[GNN_ST_ERR] && ws_off >= 0,
                  "gnn_stage_batch_f32: a GPU-extracted layer needs the graph on the device");
      int64_t rt, ct;
      seg_totals(b, li, tr, rt, ct);
      const size_t wsb = gnn_ladies_extract_workspace_bytes(a[GNN_ST_NUM_NODES], M, K, tr, rt, ct);
      GNN_STAGE_TRY(gnn_ladies_extract_f32(
          AP<const int64_t>(a, GNN_ST_INDPTR), AP<const int32_t>(a, GNN_ST_INDICES), AP<const int32_t>(a, GNN_ST_DEGREE),
          a[GNN_ST_NUM_NODES], AP<const int64_t>(a, GNN_ST_INDPTR_T), AP<const int32_t>(a, GNN_ST_INDICES_T),
          b.dv<const int32_t>(L + GNN_L_ROWS), M, b.dv<const int32_t>(L + GNN_L_COLS), K,
          b.dv<const float>(L + GNN_L_NORMFACT), nnz, b.dv<const int32_t>(L + GNN_L_FULLROWPTR),
          tr ? b.dv<const int32_t>(L + GNN_L_COLSEG) : nullptr, tr ? b.dv<const int32_t>(L + GNN_L_CSC_COLPTR) : nullptr,
          rt, ct, (int32_t*)O(GNN_SO_ROWPTR), (int32_t*)O(GNN_SO_COL), (float*)O(GNN_SO_VAL),
          (int32_t*)O(GNN_SO_ROWS_T), (float*)O(GNN_SO_VAL_T), arena + ws_off, wsb, AP<int32_t>(a, GNN_ST_ERR),
          stream));
      extracted = true;
    } else {
      GNN_STAGE_TRY(gnn_build_operand_sorted_f32(b.dv<const int32_t>(L + GNN_L_FULLROWPTR),
                                           b.dv<const int32_t>(L + GNN_L_ROWPTR), b.dv<const void>(L + GNN_L_COLIDX),
                                           4, b.dv<const float>(L + GNN_L_NORMFACT), M, K, nnz,
                                           (int32_t*)O(GNN_SO_COL), (float*)O(GNN_SO_VAL), nullptr, stream));
      if (b.count(L + GNN_L_CSC_COLPTR) > 0)
        GNN_STAGE_TRY(gnn_build_operand_t_f32(b.dv<const int32_t>(L + GNN_L_FULLROWPTR),
                                        b.dv<const int32_t>(L + GNN_L_CSC_COLPTR),
                                        b.dv<const int32_t>(L + GNN_L_CSC_ROWS), b.dv<const float>(L + GNN_L_NORMFACT),
                                        M, K, nnz, (float*)O(GNN_SO_VAL_T), stream));
    }
  }
  // 4. the extraction error flag as it stands after this batch's extractions (read by the host
  //    once the staging has completed, before the step that consumes the operands is issued)
  if (extracted && a[GNN_ST_ERR_HOST])
    GNN_HIP(hipMemcpyAsync(AP<void>(a, GNN_ST_ERR_HOST), AP<const void>(a, GNN_ST_ERR), 4, hipMemcpyDeviceToHost, st),
            "hipMemcpyAsync (error flag)");
  return 0;
}

}  // extern "C"
