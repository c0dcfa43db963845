// spmm_ext.cpp — the reference's native module `spmm` as a PyTorch-ROCm extension, plus the
// aggregation as registered torch operators (torch.ops.gnn.*), both over libgnn_spmm.so's C ABI.
//
// Reference: custom_sparse_ops.py:8 builds a pybind module named `spmm` at import time
// (torch.utils.cpp_extension.load over spmm_cpp/spmm.cpp + cuda_spmm.cu) exporting
// (spmm.cpp:52-56):
//   spmm_load_balance(Tensor sparse_coo, Tensor dense) -> Tensor      (spmm.cpp:23-27)
//   spmm_naive(Tensor sparse_coo, Tensor dense) -> Tensor             (spmm.cpp:38-42)
//   create_coo_tensor(Tensor fullrowptr, Tensor rowptr, Tensor colidx, Tensor normfact,
//                     int nrows, int ncols) -> sparse COO              (spmm.cpp:44-50)
// This module has the same name, functions, argument meaning and TORCH_CHECK errors
// (spmm.cpp:10-21): a maintainer replaces the load(...) call with `import spmm`. Underneath,
// every call is the HIP path of gnn_spmm.h on torch's current HIP stream (no host syncs).
//
// Registered operators (TORCH_LIBRARY gnn; fake shapes and autograd are registered from
// Python, gnn_amd/torch_ops.py), so torch.compile / the dispatcher see the aggregation as one
// op instead of an opaque ctypes call:
//   gnn::spmm_csr(rowptr, col, val, M, K, dense) -> Tensor          Y = A·X on a CSR operand
//   gnn::csr_transpose(rowptr, col, val, M, K) -> (rowptr_t, col_t, val_t)   canonical Aᵀ
//   gnn::spmm(rowptr, col, val, t_rowptr, t_col, t_val, M, K, dense) -> Tensor
//        the autograd-carrying form (custom_sparse_ops.py:16-37: backward = Aᵀ·G on the given
//        transpose, no gradient to the sparse values)
#include <torch/extension.h>

#include <ATen/hip/HIPContext.h>
#include <c10/core/DeviceGuard.h>

#include "gnn_spmm.h"

namespace {

void check_rc(int rc, const char* what) { TORCH_CHECK(rc == 0, what, " failed: ", gnn_last_error()); }

void* current_stream(const at::Tensor& t) { return (void*)at::hip::getCurrentHIPStream(t.device().index()).stream(); }

void check_csr(const at::Tensor& rowptr, const at::Tensor& col, const at::Tensor& val, int64_t M) {
  TORCH_CHECK(rowptr.is_cuda() && col.is_cuda() && val.is_cuda(), "CSR operand must be CUDA tensors");
  TORCH_CHECK(rowptr.scalar_type() == at::kInt && col.scalar_type() == at::kInt, "rowptr / col must be int32");
  TORCH_CHECK(val.scalar_type() == at::kFloat, "val must be float32");
  TORCH_CHECK(rowptr.is_contiguous() && col.is_contiguous() && val.is_contiguous(), "CSR arrays must be contiguous");
  TORCH_CHECK(rowptr.numel() == M + 1 && col.numel() == val.numel(), "CSR array sizes do not match M / nnz");
}

// Y (M x F) = A · X for a CSR operand; X rows may be padded (stride(0) >= F, stride(1) == 1).
at::Tensor spmm_csr(const at::Tensor& rowptr, const at::Tensor& col, const at::Tensor& val, int64_t M, int64_t K,
                    const at::Tensor& dense) {
  check_csr(rowptr, col, val, M);
  TORCH_CHECK(dense.is_cuda(), "denseMat must be a CUDA tensor");
  TORCH_CHECK(dense.dim() == 2 && dense.size(0) == K, "size mismatch: sparse (", M, ", ", K, ") @ dense ",
              dense.sizes());
  TORCH_CHECK(dense.scalar_type() == at::kFloat, "denseMat must be float32");
  TORCH_CHECK(dense.stride(1) == 1 || dense.size(1) <= 1, "denseMat must be contiguous");
  TORCH_CHECK(dense.device() == val.device(), "sparseMat and denseMat must be on the same device");
  c10::DeviceGuard guard(dense.device());
  const int64_t F = dense.size(1), nnz = col.numel();
  at::Tensor out = at::empty({M, F}, dense.options());
  if (M == 0 || F == 0) return out;
  const int64_t ldx = dense.size(0) > 1 ? dense.stride(0) : std::max<int64_t>(F, 1);
  const size_t wsb = gnn_spmm_workspace_bytes(M, nnz, F, 0);
  at::Tensor ws = at::empty({(int64_t)std::max<size_t>(wsb, 256)}, dense.options().dtype(at::kByte));
  check_rc(gnn_spmm_csr_f32(rowptr.data_ptr<int32_t>(), col.data_ptr<int32_t>(), val.data_ptr<float>(), M, K, nnz,
                            dense.data_ptr<float>(), ldx, out.data_ptr<float>(), F, F, ws.data_ptr(), wsb, 0,
                            current_stream(dense)),
           "gnn_spmm_csr_f32");
  return out;
}

std::tuple<at::Tensor, at::Tensor, at::Tensor> csr_transpose(const at::Tensor& rowptr, const at::Tensor& col,
                                                             const at::Tensor& val, int64_t M, int64_t K) {
  check_csr(rowptr, col, val, M);
  c10::DeviceGuard guard(val.device());
  const int64_t nnz = col.numel();
  at::Tensor trp = at::empty({K + 1}, rowptr.options()), tc = at::empty({nnz}, col.options()),
             tv = at::empty({nnz}, val.options());
  const size_t wsb = gnn_csr_transpose_workspace_bytes(M, K, nnz);
  at::Tensor ws = at::empty({(int64_t)std::max<size_t>(wsb, 1)}, val.options().dtype(at::kByte));
  check_rc(gnn_csr_transpose(rowptr.data_ptr<int32_t>(), col.data_ptr<int32_t>(), val.data_ptr<float>(), M, K, nnz,
                             trp.data_ptr<int32_t>(), tc.data_ptr<int32_t>(), tv.data_ptr<float>(), ws.data_ptr(), wsb,
                             current_stream(val)),
           "gnn_csr_transpose");
  return {trp, tc, tv};
}

// The forward of gnn::spmm (its backward, registered from Python, is spmm_csr on the transpose).
at::Tensor spmm_with_t(const at::Tensor& rowptr, const at::Tensor& col, const at::Tensor& val, const at::Tensor&,
                       const at::Tensor&, const at::Tensor&, int64_t M, int64_t K, const at::Tensor& dense) {
  return spmm_csr(rowptr, col, val, M, K, dense);
}

// CSR image of a coalesced COO operand (the reference's per-call preprocessing,
// cuda_spmm.cu:620-667, in one stream-ordered call).
std::tuple<at::Tensor, at::Tensor> coo_to_csr(const at::Tensor& sparse) {
  const int64_t M = sparse.size(0), nnz = sparse._nnz();
  at::Tensor idx = sparse._indices().contiguous();
  at::Tensor rowptr = at::empty({M + 1}, idx.options().dtype(at::kInt));
  at::Tensor col = at::empty({nnz}, idx.options().dtype(at::kInt));
  check_rc(gnn_coo_to_csr(nnz ? idx.data_ptr<int64_t>() : nullptr, nnz ? idx.data_ptr<int64_t>() + nnz : nullptr, nnz,
                          M, rowptr.data_ptr<int32_t>(), nnz ? col.data_ptr<int32_t>() : nullptr,
                          current_stream(sparse)),
           "gnn_coo_to_csr");
  return {rowptr, col};
}

// spmm.cpp:23-27 (and :38-42): the same preconditions and messages as the reference's checks.
at::Tensor spmm_load_balance(const at::Tensor& sparseMat, const at::Tensor& denseMat) {
  TORCH_CHECK(sparseMat.is_cuda(), "sparseMat must be a CUDA tensor");
  TORCH_CHECK(sparseMat.is_sparse(), "sparseMat must be a sparse COO tensor");
  TORCH_CHECK(sparseMat.is_coalesced(), "sparseMat must be coalesced");
  TORCH_CHECK(denseMat.is_cuda(), "denseMat must be a CUDA tensor");
  TORCH_CHECK(denseMat.is_contiguous(), "denseMat must be contiguous");
  TORCH_CHECK(sparseMat.scalar_type() == at::kFloat, "sparseMat must be float32");
  TORCH_CHECK(sparseMat.size(0) < INT32_MAX && sparseMat.size(1) < INT32_MAX && sparseMat._nnz() < INT32_MAX,
              "sparseMat dims and nnz must be < 2^31");
  c10::DeviceGuard guard(denseMat.device());
  auto [rowptr, col] = coo_to_csr(sparseMat);
  return spmm_csr(rowptr, col, sparseMat._values().contiguous(), sparseMat.size(0), sparseMat.size(1), denseMat);
}

// spmm.cpp:44-50 -> cuda_spmm.cu:787-827: val = (float)((1.0/deg_full(row)) * (double)normfact[col]),
// a coalesced sparse COO (int64 indices [2, nnz], float32 values) of shape (nrows, ncols).
// Contract: the tensor is marked coalesced without a host read. A repeated (row, col) pair in the
// inputs (never made by the reference's samplers) is merged by the first spmm_load_balance on it,
// or by gnn_amd.custom_sparse_ops.finalize_coalesce(t); other torch operators see the unmerged
// entries until then.
py::object create_coo_tensor(const at::Tensor& fullrowptr, const at::Tensor& rowptr, const at::Tensor& colidx,
                             const at::Tensor& normfact, int64_t nrows, int64_t ncols) {
  for (const at::Tensor* t : {&fullrowptr, &rowptr, &colidx, &normfact})
    TORCH_CHECK(t->is_cuda(), "create_coo_tensor inputs must be CUDA tensors");
  TORCH_CHECK(fullrowptr.scalar_type() == at::kInt && rowptr.scalar_type() == at::kInt, "row pointers must be int32");
  TORCH_CHECK(normfact.scalar_type() == at::kFloat, "normfact must be float32");
  const auto ct = colidx.scalar_type();
  TORCH_CHECK(ct == at::kShort || ct == at::kInt || ct == at::kLong, "colidx must be int16/int32/int64");
  TORCH_CHECK(rowptr.numel() == nrows + 1 && fullrowptr.numel() == nrows + 1, "row pointer length != nrows + 1");
  c10::DeviceGuard guard(colidx.device());
  at::Tensor fr = fullrowptr.contiguous(), rp = rowptr.contiguous(), ci = colidx.contiguous(),
             nf = normfact.contiguous();
  const int64_t nnz = ci.numel();
  at::Tensor col32 = at::empty({nnz}, rp.options());
  at::Tensor val = at::empty({nnz}, nf.options());
  at::Tensor idx = at::empty({2, nnz}, rp.options().dtype(at::kLong));
  const size_t wsb = gnn_build_operand_workspace_bytes();
  at::Tensor ws = at::empty({(int64_t)std::max<size_t>(wsb, 8)}, rp.options().dtype(at::kByte));
  check_rc(gnn_build_operand_f32(fr.data_ptr<int32_t>(), rp.data_ptr<int32_t>(), ci.data_ptr(), (int)ci.element_size(),
                                 nf.data_ptr<float>(), nrows, ncols, nnz, col32.data_ptr<int32_t>(), val.data_ptr<float>(),
                                 idx.data_ptr<int64_t>(), ws.data_ptr(), wsb, current_stream(ci)),
           "gnn_build_operand_f32");
  at::Tensor out = at::_sparse_coo_tensor_unsafe(idx, val, {nrows, ncols}, nf.options())._coalesced_(true);
  // Columns come out ascending per row. A repeated (row, col) pair (never made by the reference's
  // samplers) is flagged by the builder on the GPU (the workspace's second word) without a host
  // read here — the call stays stream-ordered and graph-capturable; the first spmm_load_balance on
  // the tensor reads the flag and, if set, sums the duplicates in place as the reference's
  // .coalesce() does (cuda_spmm.cu:825).
  py::object t = py::cast(out);
  if (nrows > 0 && nnz > 1) t.attr("_gnn_dup") = py::cast(ws.view(at::kLong).narrow(0, 1, 1));
  // The CSR the builder already made (rowptr, int32 columns; values shared with the COO), kept on
  // the tensor with the identity of its indices: spmm_load_balance then skips the per-call COO->CSR
  // of the reference's driver (cuda_spmm.cu:620-667). A coalesce of duplicates replaces the
  // indices, and with them the key, so the CSR is rebuilt from the merged entries.
  t.attr("_gnn_ext_csr") = py::make_tuple(py::cast(rp), py::cast(col32), py::int_((int64_t)(intptr_t)idx.data_ptr()),
                                          py::int_(nnz));
  return t;
}

// The deferred half of create_coo_tensor's coalesce (above): read the repeated-column flag once
// (one synchronisation, as the reference's coalesce) and coalesce the tensor in place if set.
at::Tensor resolve_duplicates(const py::object& sparse) {
  at::Tensor sp = sparse.cast<at::Tensor>();
  if (!py::hasattr(sparse, "_gnn_dup")) return sp;
  py::object w = sparse.attr("_gnn_dup");
  if (w.is_none()) return sp;
  sparse.attr("_gnn_dup") = py::none();
  if (w.cast<at::Tensor>().item<int64_t>() != 0)
    sp.copy_(at::_sparse_coo_tensor_unsafe(sp._indices(), sp._values(), sp.sizes()).coalesce());
  return sp;
}

at::Tensor spmm_load_balance_py(const py::object& sparseMat, const at::Tensor& denseMat) {
  at::Tensor sp = resolve_duplicates(sparseMat);
  if (py::hasattr(sparseMat, "_gnn_ext_csr")) {  // create_coo_tensor's own CSR, if still current
    py::tuple c = sparseMat.attr("_gnn_ext_csr").cast<py::tuple>();
    if (sp.is_sparse() && sp.is_coalesced() && sp._nnz() == c[3].cast<int64_t>() &&
        (int64_t)(intptr_t)sp._indices().data_ptr() == c[2].cast<int64_t>()) {
      TORCH_CHECK(denseMat.is_cuda(), "denseMat must be a CUDA tensor");
      TORCH_CHECK(denseMat.is_contiguous(), "denseMat must be contiguous");
      c10::DeviceGuard guard(denseMat.device());
      return spmm_csr(c[0].cast<at::Tensor>(), c[1].cast<at::Tensor>(), sp._values().contiguous(), sp.size(0),
                      sp.size(1), denseMat);
    }
  }
  return spmm_load_balance(sp, denseMat);
}

}  // namespace

TORCH_LIBRARY(gnn, m) {
  m.def("spmm_csr(Tensor rowptr, Tensor col, Tensor val, int M, int K, Tensor dense) -> Tensor");
  m.def("csr_transpose(Tensor rowptr, Tensor col, Tensor val, int M, int K) -> (Tensor, Tensor, Tensor)");
  m.def("spmm(Tensor rowptr, Tensor col, Tensor val, Tensor t_rowptr, Tensor t_col, Tensor t_val, int M, int K, "
        "Tensor dense) -> Tensor");
}

TORCH_LIBRARY_IMPL(gnn, CUDA, m) {
  m.impl("spmm_csr", &spmm_csr);
  m.impl("csr_transpose", &csr_transpose);
  m.impl("spmm", &spmm_with_t);
}

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  m.doc() = "MI355X (gfx950) sparse aggregation: the reference's `spmm` module over libgnn_spmm.so";
  m.def("spmm_load_balance", &spmm_load_balance_py, "Y = A·X (A sparse COO, coalesced; X dense) on the GPU",
        py::arg("sparseMat"), py::arg("denseMat"));
  m.def("spmm_naive", &spmm_load_balance_py, "same as spmm_load_balance (one kernel serves both, spmm.cpp:38-42)",
        py::arg("sparseMat"), py::arg("denseMat"));
  m.def("create_coo_tensor", &create_coo_tensor, "sampled-adjacency builder (spmm.cpp:44-50)", py::arg("fullrowptr"),
        py::arg("rowptr"), py::arg("colidx"), py::arg("normfact"), py::arg("nrows"), py::arg("ncols"));
  m.def("version", []() { return std::string(gnn_version()); });
}
