// sampler_internal.h — the sampled-batch result shared by sampler.cpp (the samplers) and
// loader.cpp (the native batch producer) inside libgnn_sampler.so. Not part of the C ABI.
#pragma once

#include <cstdint>
#include <string>
#include <vector>

#include "gnn_sampler.h"

namespace gnn_smp {

struct Layer {
  bool present = false;
  bool on_device = false;  // entries left to the GPU extraction (gnn_ladies_extract_f32)
  int64_t M = 0, K = 0, s_num = 0, nnz = 0;
  std::vector<int32_t> fullrowptr, rowptr, colidx;
  std::vector<float> normfact;
  std::vector<int64_t> sampled;
  std::vector<int32_t> rows, cols, colptr;  // on_device: U's rows, after_nodes, CSC column pointer
  std::vector<int32_t> colseg;              // on_device: offsets of lapᵀ's rows of after_nodes (K+1)
};

// Stable counting sort of a host-extracted layer's entries by column: the CSC (colptr[K+1],
// rows[nnz], rows ascending per column) = the CSR of its canonical transpose.
void layer_csc(const Layer& L, int32_t* colptr, int32_t* rows);

// The sampler's thread-local error message (gnn_sampler_last_error).
void set_error(const std::string& msg);

}  // namespace gnn_smp

struct gnn_ladies_result {
  std::vector<gnn_smp::Layer> layers;  // bottom-up
  std::vector<int64_t> input_nodes;
};
