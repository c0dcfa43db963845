// gather_shape.hip — the SpMM aggregation's memory access shape with nothing else in it
// (pin the kernel's ceiling with a microbenchmark of its exact shape).
//
// spmm_unit_kernel<VW=4, G, NJ=1, U> (gnn_amd/csrc/spmm.hip) gathers, per wave instruction, 64/G
// row pieces of G * 16 bytes (G lanes x one 16-byte load each) of X, with U such instructions in
// flight per lane before it uses them, 32 waves per CU, all waves sweeping the same column tile
// of X (so the tile's slice, K rows x G * 16 bytes, is what each XCD's L2 must hold). This
// program issues exactly that load stream — random rows of a K-row table with 608-float rows,
// row ids read from memory 64 at a time and broadcast by lane shuffles — and only sums what it
// loads (one FMA-free add per loaded float4, one store per lane at the end), so its rate is the
// rate of the access shape itself. Reported: algorithmic bytes (row pieces x G x 16) per second,
// median of 20 launches timed with HIP events.
//
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 scripts/gather_shape.hip -o scripts/bin/gather_shape
// Run:   scripts/bin/gather_shape > gather_shape.json     (one JSON line per case)
//        scripts/bin/gather_shape K G U                     (one case: bench.py's live ceiling)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#define CHECK(x)                                                                     \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) {                                                          \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      std::exit(1);                                                                  \
    }                                                                                \
  } while (0)

constexpr int LD = 608;  // floats per X row (X0's padded stride)

// Each wave owns `per_wave` consecutive row ids of `idx` (a multiple of 64). Per round a lane
// loads one id; group g (lanes g*G .. g*G+G-1) then takes ids u * (64/G) + g for u < U' (U' = the
// ids per round / (64/G)), issuing U loads before summing them.
template <int G, int U, bool VAL = false>
__global__ __launch_bounds__(256) void gather_kernel(const float4* __restrict__ X, const int* __restrict__ idx,
                                                     int per_wave, int tile4, float* __restrict__ out) {
  constexpr int GROUPS = 64 / G;
  constexpr int PER_ROUND = GROUPS * U;  // row pieces per round per wave (<= 64)
  static_assert(PER_ROUND <= 64, "one id load per lane per round");
  const int lane = threadIdx.x & 63;
  const int64_t wave = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  const int grp = lane / G, gl = lane % G;
  const int* my = idx + wave * per_wave;
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int base = 0; base < per_wave; base += PER_ROUND) {
    const int id = lane < PER_ROUND ? my[base + lane] : 0;
    const float wv = VAL ? (float)(id & 7) * 0.25f : 1.0f;  // a per-piece value, as the operand's
    float4 v[U];
    float w[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int r = __shfl(id, u * GROUPS + grp);
      w[u] = VAL ? __shfl(wv, u * GROUPS + grp) : 1.0f;
      v[u] = X[(int64_t)r * (LD / 4) + tile4 + gl];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      acc.x = __builtin_fmaf(w[u], v[u].x, acc.x);
      acc.y = __builtin_fmaf(w[u], v[u].y, acc.y);
      acc.z = __builtin_fmaf(w[u], v[u].z, acc.z);
      acc.w = __builtin_fmaf(w[u], v[u].w, acc.w);
    }
  }
  out[wave * 64 + lane] = acc.x + acc.y + acc.z + acc.w;
}

template <int G, int U, bool VAL = false>
double run(const float4* X, const int* idx, int waves, int per_wave, int tile4, float* out, int wpb) {
  const dim3 block(64 * wpb), grid(waves / wpb);
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  for (int w = 0; w < 3; ++w) gather_kernel<G, U, VAL><<<grid, block>>>(X, idx, per_wave, tile4, out);
  CHECK(hipGetLastError());
  std::vector<float> ms;
  for (int rep = 0; rep < 20; ++rep) {
    CHECK(hipEventRecord(a));
    gather_kernel<G, U, VAL><<<grid, block>>>(X, idx, per_wave, tile4, out);
    CHECK(hipEventRecord(b));
    CHECK(hipEventSynchronize(b));
    float t = 0;
    CHECK(hipEventElapsedTime(&t, a, b));
    ms.push_back(t);
  }
  CHECK(hipEventDestroy(a));
  CHECK(hipEventDestroy(b));
  std::sort(ms.begin(), ms.end());
  return ms[ms.size() / 2] * 1e-3;
}

template <int G>
double run_u(int U, const float4* X, const int* idx, int waves, int per_wave, float* out) {
  switch (U) {
    case 2: return run<G, 2>(X, idx, waves, per_wave, 0, out, 4);
    case 8: return run<G, 8>(X, idx, waves, per_wave, 0, out, 4);
    default: return run<G, 4>(X, idx, waves, per_wave, 0, out, 4);
  }
}

int main(int argc, char** argv) {
  int dev_count = 0;
  CHECK(hipGetDeviceCount(&dev_count));
  if (dev_count < 1) return 1;
  hipDeviceProp_t prop;
  CHECK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  const int64_t KMAX = 44352;
  // X: KMAX rows of 608 floats, deterministic contents
  std::vector<float> hx((size_t)KMAX * LD);
  for (size_t i = 0; i < hx.size(); ++i) hx[i] = (float)((i * 2654435761u) % 1000) * 1e-3f;
  float4* X = nullptr;
  CHECK(hipMalloc(&X, hx.size() * sizeof(float)));
  CHECK(hipMemcpy(X, hx.data(), hx.size() * sizeof(float), hipMemcpyHostToDevice));
  // about 1.9 M row pieces per launch (the layer-0 operand's nonzero count)
  const char* pw = std::getenv("PER_WAVE");  // row pieces per wave (a multiple of 64): launch length
  const int per_wave = pw ? std::max(64, atoi(pw) / 64 * 64) : 256;
  const int waves_per_cu = 32;
  const int waves = cus * waves_per_cu;  // one full round of the chip
  const int64_t rows = (int64_t)waves * per_wave;
  int* idx = nullptr;
  float* out = nullptr;
  CHECK(hipMalloc(&idx, rows * sizeof(int)));
  CHECK(hipMalloc(&out, (size_t)waves * 64 * sizeof(float)));
  std::vector<int> hi(rows);
  std::mt19937 rng(7);
  if (argc >= 4) {  // one case: K rows, G lanes per row piece, U pieces in flight per lane group
    const int64_t K = std::max<int64_t>(1, std::min<int64_t>(KMAX, atoll(argv[1])));
    const int g = atoi(argv[2]), u = atoi(argv[3]);
    std::uniform_int_distribution<int> d(0, (int)K - 1);
    for (auto& v : hi) v = d(rng);
    CHECK(hipMemcpy(idx, hi.data(), rows * sizeof(int), hipMemcpyHostToDevice));
    double s = 0;
    if (g == 8) s = run_u<8>(u, X, idx, waves, per_wave, out);
    else if (g == 32) s = run_u<32>(u, X, idx, waves, per_wave, out);
    else if (g == 64) s = run_u<64>(u, X, idx, waves, per_wave, out);
    else s = run_u<16>(u, X, idx, waves, per_wave, out);
    const int gg = (g == 8 || g == 32 || g == 64) ? g : 16;
    std::printf("{\"K\": %lld, \"G\": %d, \"U\": %d, \"slice_MB\": %.2f, \"us\": %.1f, \"GBps\": %.1f}\n",
                (long long)K, gg, u, K * gg * 16 / 1e6, s * 1e6, (double)rows * gg * 16 / s / 1e9);
    return 0;
  }
  const int64_t Ks[] = {512, 4096, 11008, 16384, 22176, 44352};
  for (int64_t K : Ks) {
    std::uniform_int_distribution<int> d(0, (int)K - 1);
    for (auto& v : hi) v = d(rng);
    CHECK(hipMemcpy(idx, hi.data(), rows * sizeof(int), hipMemcpyHostToDevice));
    struct Case { int g, u, wpb; double s; };
    std::vector<Case> cs;
    cs.push_back({16, 4, 4, run<16, 4>(X, idx, waves, per_wave, 0, out, 4)});
    cs.push_back({16, -4, 4, run<16, 4, true>(X, idx, waves, per_wave, 0, out, 4)});  // U = -4: + value shuffle, FMA
    cs.push_back({16, 2, 4, run<16, 2>(X, idx, waves, per_wave, 0, out, 4)});
    cs.push_back({16, 8, 4, run<16, 8>(X, idx, waves, per_wave, 0, out, 4)});
    cs.push_back({16, 16, 4, run<16, 16>(X, idx, waves, per_wave, 0, out, 4)});
    cs.push_back({8, 4, 4, run<8, 4>(X, idx, waves, per_wave, 0, out, 4)});
    cs.push_back({8, 8, 4, run<8, 8>(X, idx, waves, per_wave, 0, out, 4)});
    cs.push_back({32, 4, 4, run<32, 4>(X, idx, waves, per_wave, 0, out, 4)});
    cs.push_back({64, 4, 4, run<64, 4>(X, idx, waves, per_wave, 0, out, 4)});
    cs.push_back({64, 8, 4, run<64, 8>(X, idx, waves, per_wave, 0, out, 4)});
    for (const Case& c : cs) {
      const double bytes = (double)rows * c.g * 16;
      std::printf("{\"K\": %lld, \"slice_MB\": %.2f, \"G\": %d, \"piece_B\": %d, \"U\": %d, \"waves_per_cu\": %d, "
                  "\"row_pieces\": %lld, \"us\": %.1f, \"GBps\": %.1f, \"GBps_per_cu\": %.1f}\n",
                  (long long)K, K * c.g * 16 / 1e6, c.g, c.g * 16, c.u, waves_per_cu, (long long)rows, c.s * 1e6,
                  bytes / c.s / 1e9, bytes / c.s / 1e9 / cus);
      std::fflush(stdout);
    }
  }
  // sequential control: every wave reads consecutive rows (no gather), G = 16
  for (int64_t i = 0; i < rows; ++i) hi[i] = (int)(i % 4096);
  CHECK(hipMemcpy(idx, hi.data(), rows * sizeof(int), hipMemcpyHostToDevice));
  const double s = run<16, 4>(X, idx, waves, per_wave, 0, out, 4);
  std::printf("{\"K\": 4096, \"order\": \"sequential\", \"G\": 16, \"U\": 4, \"us\": %.1f, \"GBps\": %.1f}\n", s * 1e6,
              (double)rows * 256 / s / 1e9);
  CHECK(hipFree(X));
  CHECK(hipFree(idx));
  CHECK(hipFree(out));
  return 0;
}
