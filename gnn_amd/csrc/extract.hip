// extract.hip — the LADIES layer extraction adj = lap[rows, :][:, cols] on the GPU, fused with
// create_coo_tensor's values (include/gnn_extract.h).
//
// Reference (sampler.py:113-139): per sampled layer the host slices U = lap_matrix[previous, :]
// (scipy row indexing), draws the next layer's nodes, slices adj = U[:, after_nodes] (scipy
// column indexing), ships rowptr / int16 colidx / normfact to the GPU, and create_coo_tensor
// (cuda_spmm.cu:787-827) computes val = (1/deg_full(row)) * normfact[col] there.
//
// Here the host keeps only the draw (it needs the column counts of U, which it has without
// materialising U) and everything that touches the sub-graph's entries runs on the GPU, reading
// the graph's CSR resident in HBM. Both outputs are "filtered gathers" of graph rows:
//   forward   A:  segment i = lap row rows[i],   keep node c if c is in cols (position j) -> col j
//   transpose Aᵀ: segment j = lapᵀ row cols[j],  keep node r if r is in rows (position i) -> row i
// with value (float)((1.0 / deg(row node)) * (double)normfact[j]) either way (bit-identical to
// gnn_build_operand_f32 / gnn_build_operand_t_f32 on host-extracted pieces). The segment offsets
// (S = U's row pointer; the offsets of lapᵀ's rows of cols) come from the host, which has them
// from the draw, and so do their totals T (the graph entries scanned per side).
//
// ONE walk per graph entry (round 3; round 2 walked every entry twice: a count pass, a scan, then
// a write pass over the same entries), and no wave ever waits for another:
//  * Balance: graph rows follow a power law and LADIES draws the high-degree nodes, so the
//    concatenated segments are cut into XW equal contiguous entry ranges ("chunks"), one per wave
//    (at most 64 * XU entries: entry a + 64 t + lane of the range sits in register slot t).
//  * Per wave, all latency chains issued at once for the whole range: the segment table (offsets,
//    graph positions, row lengths / normfact — prep kernel), the graph indices, the membership
//    lookups, the value inputs (normfact[col] or deg(row node)).
//  * The kept entries leave compacted (ballot + mbcnt) into a GAPPED buffer at the chunk's own
//    entry position (a chunk keeps at most its range), with the chunk's count; A's row pointer
//    gets, for each segment starting in the chunk, the kept entries of the chunk before it.
//  * Every chunk adds its count to its group's total (groups of 64 chunks; one agent-scope add,
//    nothing awaited); a compaction pass (a wave per chunk: its prefix from the lower chunks of
//    its group + the lower groups' totals, coalesced copies of its entries to that prefix,
//    rowptr += prefix) finishes.
//    Measured on the Reddit layer 0 (13 M graph entries with the transpose): a single walk that
//    waited for the lower chunks' counts (chained or two-level prefix) spent ~45 % of its time
//    waiting — every wave of a launch ends its walk at about the same time — while the gapped
//    buffer costs one extra coalesced read and write of the kept entries (~29 MB).
//  * Membership: a bitmap of the sorted id set with a rank per 32-bit word, one 8-byte load per
//    lookup (built from the sorted list without atomics: rank[w] = lower_bound(ids, 32 w)). When
//    the table fits 64 KB (N <= 262 k: Reddit) every workgroup of 16 waves copies it into LDS
//    first: the lookups are random 8-byte reads, one cache line each from global memory (the
//    walk's main cost), a few LDS cycles each from the copy (layer 0: 148 -> 128 us).
// Launches: 1. prep (tables, segment positions, chunk -> first segment) 2. walk 3. compact.
// Every size the host needs (grid, workspace) follows from the host-known nnz and
// segment totals; no state survives a call. If the device's kept count differs from the host's
// nnz the error flag is raised, writes stay below nnz, the tail of the outputs is zero-filled and
// rowptr is clamped to nnz, so a consumer never reads outside the operand.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>
#include <cstdint>
#include <cstdlib>

#include "common.h"
#include "gnn_extract.h"

namespace {

using gnn::ceil_div;

constexpr int XW_MAX = 65536;        // chunks (waves) per direction
constexpr int XW_DEFAULT = 8192;     // default chunk count, unless a chunk would exceed 64 * XU
constexpr int MIN_PER_WAVE = 256;    // ... or fall under this many entries

__device__ __forceinline__ int below_me(unsigned long long mask) {
  return (int)__builtin_amdgcn_mbcnt_hi((unsigned)(mask >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)mask, 0u));
}

__device__ __forceinline__ int rl(int x, int l) { return __builtin_amdgcn_readlane(x, l); }

__device__ __forceinline__ int64_t shfl64(int64_t v, int src) {
  const int hi = __shfl((int)(v >> 32), src), lo = __shfl((int)(uint32_t)v, src);
  return ((int64_t)hi << 32) | (uint32_t)lo;
}

// Pointers read from the kernel's argument structs are generic; every array here lives in device
// memory, so accesses go through global-address-space views (global_load/store, not flat).
template <typename T>
__device__ __forceinline__ __attribute__((address_space(1))) T* G(T* p) {
  return (__attribute__((address_space(1))) T*)p;
}

__device__ __forceinline__ int wave_sum(int x) {
#pragma unroll
  for (int off = 32; off; off >>= 1) x += __shfl_xor(x, off);
  return x;
}

// Membership word of the sorted id set (one 8-byte load, global or LDS): x = the ids in
// [32 w, 32 w + 32) as bits, y = the number of ids below 32 w.
using Word = uint2;
constexpr int WORD_NODES = 32;
// The table goes to LDS (one copy per workgroup of LDS_WAVES waves) when it is at most this
// big: N <= 262,144 nodes (Reddit: 233 k -> 58 KB, two workgroups per CU).
constexpr size_t LDS_TABLE_MAX = 64 * 1024;
constexpr int LDS_WAVES = 16;  // waves per workgroup in LDS mode (2 x 1024 threads per CU)
constexpr int GLB_WAVES = 4;   // ... in global mode
constexpr int LDS_CPW = 2;     // chunks per wave in LDS mode (one table copy per 32 chunks)
constexpr int CHUNK_ALIGN = 32;  // chunk counts are multiples of every workgroup's chunk block
constexpr int GROUP = 64;        // chunks per group (the compaction's two-level prefix)
constexpr int COMPACT_CPW = 2;   // chunks per compaction wave (4 * it divides CHUNK_ALIGN)

// One direction of the extraction (device pointers).
struct Side {
  const int64_t* ptr;          // graph indptr (lap or lapᵀ)
  const int* idx;              // graph indices
  const int* src;              // segment source nodes [R]
  const int* S;                // [R+1] segment offsets (host)
  const int* ids;              // the sorted output index set (cols for A, rows for Aᵀ)
  Word* tab;                   // [words] membership table of ids (prep)
  int64_t* segbase;            // [R] ptr[src[i]]: graph position of segment i (prep)
  int* qs;                     // [xw+1] first segment starting at or after each chunk's start (prep)
  unsigned long long* gap;     // [T] kept entries (index | value bits << 32) at their chunk's entry position
  int* cnt;                    // [xw] kept entries per chunk
  int* gcnt;                   // [xw / GROUP] arrivals per group of chunks (zeroed by prep; GSUM = false)
  int* gsum;                   // [xw / GROUP] kept entries per group (zeroed by prep)
  int* rowptr;                 // A: the output row pointer [R+1]; Aᵀ: NULL (host colptr)
  int* out_idx;                // col (A) / rows_t (Aᵀ)
  float* out_val;
  int R;                       // segments
  int nids;
  int transpose;               // 0: A (segment = row i), 1: Aᵀ (segment = column j)
  int nnz;                     // host-known kept entries
  int T;                       // host-known graph entries scanned (S[R])
  int xw;                      // chunks (waves), a multiple of CHUNK_ALIGN
};

struct Sides {
  Side s[2];
  int n;      // 1 or 2
  int words;  // ceil(N / 32)
};

// Chunk w's entry range [a, b) of a side.
__device__ __forceinline__ int chunk_lo(int T, int xw, int w) { return (int)((int64_t)T * w / xw); }

// The chunk that owns entry position p: the largest w < xw with chunk_lo(w) <= p.
__device__ __forceinline__ int owner_of(int T, int xw, int p) {
  if (T <= 0) return xw - 1;
  const int64_t w = ((int64_t)(p + 1) * xw - 1) / T;
  return (int)(w < xw - 1 ? w : xw - 1);
}

// Prep, one thread per item:
//   [0, n * words)         membership table of the sorted id lists (32 nodes per word)
//   next (R0 + 1) (+ R1+1) per segment q: segbase[q] = ptr[src[q]]; qs[w] = q for the chunks w
//                          whose first segment (first q with S[q] >= chunk_lo(w)) is q
//   next ng0 (+ ng1)       group arrival counters zeroed
__global__ __launch_bounds__(256) void lx_prep_kernel(Sides sd) {
  int i = blockIdx.x * 256 + threadIdx.x;
  const int words = sd.words;
  if (i < words * sd.n) {
    const int side = i / words;
    const int w = i - side * words;
    const Side& s = sd.s[side];
    const int lo32 = w * WORD_NODES;
    int lo = 0, hi = s.nids;  // first id >= 32 w
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (s.ids[mid] < lo32) lo = mid + 1;
      else hi = mid;
    }
    unsigned b = 0u;
    for (int k = lo; k < s.nids && s.ids[k] < lo32 + WORD_NODES; ++k) b |= 1u << (s.ids[k] - lo32);
    s.tab[w] = make_uint2(b, (unsigned)lo);
    return;
  }
  i -= words * sd.n;
  for (int k = 0; k < sd.n; ++k) {
    const Side& s = sd.s[k];
    if (i <= s.R) {
      const int q = i;
      if (q < s.R) s.segbase[q] = s.ptr[s.src[q]];
      const int T = s.T, xw = s.xw;
      const int o = (q == s.R) ? xw - 1 : owner_of(T, xw, min(max(s.S[q], 0), T));
      const int op = (q == 0) ? -1 : owner_of(T, xw, min(max(s.S[q - 1], 0), T));
      for (int w = op + 1; w <= o; ++w) s.qs[w] = q;
      if (q == s.R) s.qs[xw] = s.R + 1;
      return;
    }
    i -= s.R + 1;
  }
  for (int k = 0; k < sd.n; ++k) {
    const Side& s = sd.s[k];
    const int ng = (s.xw + GROUP - 1) / GROUP;
    if (i < ng) {
      s.gcnt[i] = 0;
      s.gsum[i] = 0;
      return;
    }
    i -= ng;
  }
}

// Position of node c in the sorted id set, -1 if absent: one 8-byte load from the global table or
// from its LDS copy.
__device__ __forceinline__ int from_word(Word wd, int c) {
  const unsigned sh = (unsigned)c & (WORD_NODES - 1);
  return ((wd.x >> sh) & 1u) ? (int)wd.y + __builtin_popcount(wd.x & ((1u << sh) - 1u)) : -1;
}

__device__ __forceinline__ int lookup(const Word* tab, int c) {
  const auto* p = G(tab) + (c >> 5);
  Word wd;
  wd.x = p->x;
  wd.y = p->y;
  return from_word(wd, c);
}

// The table lane holding entry k: the last u < nseg with S(u) <= k (empty segments skipped past).
__device__ __forceinline__ int seg_of(int k, int Sj, int nseg) {
  int q = 0;
  if (nseg <= 6) {
    for (int u = 1; u < nseg; ++u) q += (k >= rl(Sj, u)) ? 1 : 0;
  } else {
#pragma unroll
    for (int step = 32; step; step >>= 1) {
      const int c = q + step;
      const int v = __shfl(Sj, c & 63);
      if (c < nseg && v <= k) q = c;
    }
  }
  return q;
}

// Segments with entries in chunk w's range [a, b): s0 .. s1 (s0 > s1: none).
__device__ __forceinline__ void chunk_segments(const Side& s, int w, int a, int& s0, int& s1) {
  const int q0 = min(max(G(s.qs)[w], 0), s.R), q1 = min(max(G(s.qs)[w + 1], q0), s.R + 1);
  s0 = (q0 > 0 && (q0 >= s.R || G(s.S)[q0] > a)) ? q0 - 1 : q0;
  s1 = min(q1 - 1, s.R - 1);
}

// One chunk w of side s by one wave (see the file comment).
template <int XU, bool LDS, bool GSUM>
__device__ __forceinline__ void walk_chunk(const Side& s, int w, int lane, const Word* ltab,
                                           const int* __restrict__ degree, const float* __restrict__ normfact) {
  const int T = s.T;
  const int a = chunk_lo(T, s.xw, w), b = chunk_lo(T, s.xw, w + 1);
  int s0, s1;
  chunk_segments(s, w, a, s0, s1);

  // 1. graph indices of the range (and per entry: its row length (A) / its column's normfact (Aᵀ))
  int node[XU], aux[XU];
#pragma unroll
  for (int t = 0; t < XU; ++t) node[t] = -1;
  for (int sb = s0; sb <= s1; sb += 64) {
    const int sj = sb + lane;
    int Sj = INT_MAX, Sj1 = INT_MAX, auxj = 0;
    int64_t gj = 0;
    if (sj <= s1) {
      Sj = G(s.S)[sj];
      Sj1 = G(s.S)[sj + 1];
      gj = G(s.segbase)[sj];
      auxj = s.transpose ? __float_as_int(G(normfact)[sj]) : Sj1 - Sj;
    }
    const int nseg = min(64, s1 - sb + 1);
    const int ta = max(a, rl(Sj, 0)), tb = min(b, rl(Sj1, nseg - 1));
    if (ta >= tb) continue;
#pragma unroll
    for (int t = 0; t < XU; ++t) {
      const int k = a + t * 64 + lane;
      if (__builtin_amdgcn_readfirstlane(a + t * 64) < tb && a + t * 64 + 63 >= ta) {  // slot group overlaps
        const int q = seg_of(k, Sj, nseg);
        const int segS = __shfl(Sj, q);
        const int64_t g = shfl64(gj, q);
        const int ax = __shfl(auxj, q);
        if (k >= ta && k < tb) {
          node[t] = G(s.idx)[g + (k - segS)];
          aux[t] = ax;
        }
      }
    }
  }
  // 2. membership: the output index of each entry, -1 if dropped
  int m[XU];
#pragma unroll
  for (int t = 0; t < XU; ++t) m[t] = node[t] >= 0 ? (LDS ? from_word(ltab[node[t] >> 5], node[t])
                                                          : lookup(s.tab, node[t])) : -1;
  // 3. values (float)((1.0 / deg(row node)) * (double)normfact[col]) of the kept entries
  float val[XU];
  if (s.transpose) {
    int dg[XU];
#pragma unroll
    for (int t = 0; t < XU; ++t) dg[t] = m[t] >= 0 ? degree[node[t]] : 1;
#pragma unroll
    for (int t = 0; t < XU; ++t) val[t] = (float)((1.0 / (double)dg[t]) * (double)__int_as_float(aux[t]));
  } else {
    float nf[XU];
#pragma unroll
    for (int t = 0; t < XU; ++t) nf[t] = m[t] >= 0 ? normfact[m[t]] : 0.0f;
#pragma unroll
    for (int t = 0; t < XU; ++t) val[t] = (float)((1.0 / (double)(m[t] >= 0 ? aux[t] : 1)) * (double)nf[t]);
  }
  // 4. the chunk's count, then its kept entries compacted into the gapped buffer at the chunk's
  //    entry position
  unsigned long long km[XU];
  int total = 0;
#pragma unroll
  for (int t = 0; t < XU; ++t) {
    km[t] = __ballot(m[t] >= 0);
    total += __builtin_popcountll(km[t]);
  }
  const int g = w / GROUP;
  if constexpr (GSUM) {
    // the group's total by one agent-scope add per chunk, no returned value awaited: nothing in
    // this launch reads it (the compaction, a later launch, does), so no wave waits for its stores
    // or for another wave (round 3, late; was: count stores drained, then an arrival counter whose
    // last adder summed the group's counts)
    if (lane == 0) {
      G(s.cnt)[w] = total;
      __hip_atomic_fetch_add(G(s.gsum) + g, total, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  {
    int run = 0;
#pragma unroll
    for (int t = 0; t < XU; ++t) {
      const int pos = a + run + below_me(km[t]);
      if (m[t] >= 0) G(s.gap)[pos] = (unsigned)m[t] | ((unsigned long long)__float_as_uint(val[t]) << 32);
      run += __builtin_popcountll(km[t]);
    }
  }
  if constexpr (!GSUM) {
    // the count, and the group's total by the group's last arriving chunk (MI355X_MICROARCH.md,
    // Valid forms, table row 1: sc1 count stores drained before the agent-scope counter add; the
    // last adder reads the counts with sc1 loads after its add returned)
    if (lane == 0) __hip_atomic_store(G(s.cnt) + w, total, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const int gsize = min(GROUP, s.xw - g * GROUP);
    int last = 0;
    if (lane == 0)
      last = __hip_atomic_fetch_add(G(s.gcnt) + g, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gsize - 1;
    if (__builtin_amdgcn_readfirstlane(last)) {
      const int c = lane < gsize ? __hip_atomic_load(G(s.cnt) + g * GROUP + lane, __ATOMIC_RELAXED,
                                                     __HIP_MEMORY_SCOPE_AGENT) : 0;
      const int gs = wave_sum(c);
      if (lane == 0) G(s.gsum)[g] = gs;
    }
  }
  // 5. A: for the segments starting in this range (the last chunk: up to R), the kept entries of
  //    the range before them (the compaction adds the chunk's prefix)
  if (s.rowptr) {
    const int q0 = min(max(G(s.qs)[w], 0), s.R), q1 = min(max(G(s.qs)[w + 1], q0), s.R + 1);
    for (int qb = q0; qb < q1; qb += 64) {
      const int q = qb + lane;
      if (q < q1) {
        const int p = min(max(G(s.S)[q], a), T);
        int kb = 0;
#pragma unroll
        for (int t = 0; t < XU; ++t) {
          const int n = p - a - t * 64;
          const unsigned long long mk = n <= 0 ? 0ull : (n >= 64 ? ~0ull : ((1ull << n) - 1ull));
          kb += __builtin_popcountll(km[t] & mk);
        }
        G(s.rowptr)[q] = kb;
      }
    }
  }
}

// A workgroup of WGW waves walks WGW * CPW consecutive chunks of one side (each wave CPW of them,
// one after the other), sharing one LDS copy of the membership table in LDS mode.
template <int XU, int WGW, int CPW, bool LDS, bool GSUM>
__global__ __launch_bounds__(64 * WGW, XU == 8 ? 8 : 4) void lx_walk_kernel(Sides sd, const int* __restrict__ degree,
                                                           const float* __restrict__ normfact) {
  extern __shared__ __attribute__((aligned(16))) Word ltab[];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform
  int w0 = blockIdx.x * WGW * CPW;
  const bool second = w0 >= sd.s[0].xw;  // chunk counts are multiples of WGW * CPW
  const int side = second ? 1 : 0;
  if (second) w0 -= sd.s[0].xw;
  if (side >= sd.n) return;  // workgroup-uniform
  const Side s = second ? sd.s[1] : sd.s[0];  // a uniform select of kernel arguments (no scratch copy)
  if (LDS) {  // the side's membership table, once per workgroup
    for (int i = threadIdx.x; i < sd.words; i += 64 * WGW) {
      const auto* p = G(s.tab) + i;
      ltab[i] = make_uint2(p->x, p->y);
    }
    __syncthreads();
  }
#pragma unroll 1
  for (int c = 0; c < CPW; ++c) {
    const int w = w0 + c * WGW + wave;
    if (w < s.xw) walk_chunk<XU, LDS, GSUM>(s, w, lane, ltab, degree, normfact);
  }
}

// A wave per chunk: its prefix (the counts of the lower chunks of its group + the totals of the
// lower groups: at most 63 + xw / 64 loads, no waiting — the walk launch has finished), its kept
// entries from the gapped buffer to their final positions (coalesced), A's row pointer += the
// prefix; the last chunk checks the totals (see the file comment).
template <int COMPACT_CPW>
__global__ __launch_bounds__(256) void lx_compact_kernel(Sides sd, int* __restrict__ err) {
  const int lane = threadIdx.x & 63;
  // a wave per COMPACT_CPW consecutive chunks (fewer, fuller waves beside the compute stream)
  int w0 = (blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6)) * COMPACT_CPW;
  const bool second = blockIdx.x * 4 * COMPACT_CPW >= sd.s[0].xw;  // xw0 is a multiple of 4 COMPACT_CPW
  const int side = second ? 1 : 0;
  if (second) w0 -= sd.s[0].xw;
  if (side >= sd.n) return;
  const Side s = second ? sd.s[1] : sd.s[0];
  if (w0 >= s.xw) return;
  const int T = s.T, lim = s.nnz;
  // the first chunk's prefix: its group's lower chunks + the lower groups' totals
  const int g = w0 / GROUP, gl = w0 - g * GROUP;
  int c = lane < gl ? G(s.cnt)[g * GROUP + lane] : 0;
  for (int h = lane; h < g; h += 64) c += G(s.gsum)[h];
  int ex = wave_sum(c);
  int ns[COMPACT_CPW];
#pragma unroll
  for (int k = 0; k < COMPACT_CPW; ++k) ns[k] = w0 + k < s.xw ? G(s.cnt)[w0 + k] : 0;
#pragma unroll 1
  for (int k = 0; k < COMPACT_CPW && w0 + k < s.xw; ++k) {
    const int w = w0 + k, n = ns[k];
    const int a = chunk_lo(T, s.xw, w);
    for (int i = lane; i < n; i += 64) {
      const int pos = ex + i;
      if (pos < lim) {
        const unsigned long long e = G(s.gap)[a + i];
        G(s.out_idx)[pos] = (int)(unsigned)e;
        G(s.out_val)[pos] = __uint_as_float((unsigned)(e >> 32));
      }
    }
    if (s.rowptr) {
      const int q0 = min(max(G(s.qs)[w], 0), s.R), q1 = min(max(G(s.qs)[w + 1], q0), s.R + 1);
      for (int q = q0 + lane; q < q1; q += 64) G(s.rowptr)[q] = min(G(s.rowptr)[q] + ex, lim);
    }
    if (w == s.xw - 1) {
      const int incl = ex + n;
      if (incl != lim || G(s.S)[s.R] != T) {
        if (lane == 0 && err) atomicOr(err, 1 << side);
        for (int p = incl + lane; p < lim; p += 64) {  // nothing reads garbage past the kept entries
          G(s.out_idx)[p] = 0;
          G(s.out_val)[p] = 0.0f;
        }
      }
    }
    ex += n;
  }
}

int64_t table_words(int64_t num_nodes) { return (num_nodes + WORD_NODES - 1) / WORD_NODES; }

// Chunks for T entries at XU slots per lane: XW_DEFAULT, or more if a chunk would exceed 64 XU
// entries, or fewer if a chunk would fall under MIN_PER_WAVE; a multiple of CHUNK_ALIGN (every
// workgroup's waves on one side) in [CHUNK_ALIGN, XW_MAX].
int64_t chunks_for(int64_t T, int XU, int64_t want) {
  const int64_t need = ceil_div(T, 64 * XU);
  int64_t xw = want > 0 ? want : std::min<int64_t>(XW_DEFAULT, ceil_div(T, MIN_PER_WAVE));
  xw = std::max<int64_t>(std::max<int64_t>(xw, need), CHUNK_ALIGN);
  return (xw + CHUNK_ALIGN - 1) / CHUNK_ALIGN * CHUNK_ALIGN;
}

}  // namespace

extern "C" {

size_t gnn_ladies_extract_workspace_bytes(int64_t num_nodes, int64_t M, int64_t K, int32_t transpose,
                                          int64_t rowseg_total, int64_t colseg_total) {
  const int64_t words = table_words(num_nodes > 0 ? num_nodes : 1);
  const size_t per_side = gnn::align_up((size_t)words * sizeof(Word), 256) +
                          2 * gnn::align_up((size_t)(XW_MAX + 1) * 4, 256) +
                          2 * gnn::align_up((size_t)(XW_MAX / GROUP) * 4, 256);
  const size_t segs = gnn::align_up((size_t)(M > 0 ? M : 1) * 8, 256) +
                      (transpose ? gnn::align_up((size_t)(K > 0 ? K : 1) * 8, 256) : 0);
  const size_t gaps = gnn::align_up((size_t)std::max<int64_t>(rowseg_total, 1) * 8, 256) +
                      (transpose ? gnn::align_up((size_t)std::max<int64_t>(colseg_total, 1) * 8, 256) : 0);
  return per_side * (transpose ? 2 : 1) + segs + gaps;
}

int gnn_ladies_extract_f32(const int64_t* indptr, const int32_t* indices, const int32_t* degree, int64_t num_nodes,
                           const int64_t* indptr_t, const int32_t* indices_t, const int32_t* rows, int64_t M,
                           const int32_t* cols, int64_t K, const float* normfact, int64_t nnz, const int32_t* rowseg,
                           const int32_t* colseg, const int32_t* colptr_t, int64_t rowseg_total, int64_t colseg_total,
                           int32_t* rowptr, int32_t* col, float* val, int32_t* rows_t, float* val_t, void* workspace,
                           size_t workspace_bytes, int32_t* err_flag, void* stream) {
  GNN_REQUIRE(M >= 0 && K >= 0 && nnz >= 0 && num_nodes > 0, "gnn_ladies_extract_f32: negative size / empty graph");
  GNN_REQUIRE(M < INT_MAX && K < INT_MAX && nnz < INT_MAX && num_nodes < INT_MAX - 64,
              "gnn_ladies_extract_f32: sizes must be < 2^31");
  GNN_REQUIRE(rowptr && rowseg, "gnn_ladies_extract_f32: NULL rowptr / rowseg");
  GNN_REQUIRE(M == 0 || (indptr && indices && rows), "gnn_ladies_extract_f32: NULL graph / rows");
  GNN_REQUIRE(K == 0 || (cols && normfact), "gnn_ladies_extract_f32: NULL cols / normfact");
  GNN_REQUIRE(nnz == 0 || (col && val), "gnn_ladies_extract_f32: NULL col / val");
  const bool tr = colptr_t != nullptr;
  GNN_REQUIRE(!tr || (colseg && indptr_t && indices_t && degree && (nnz == 0 || (rows_t && val_t))),
              "gnn_ladies_extract_f32: transpose requested with NULL colseg / lap^T / degree / rows_t / val_t");
  GNN_REQUIRE(rowseg_total >= 0 && rowseg_total < INT_MAX && (!tr || (colseg_total >= 0 && colseg_total < INT_MAX)),
              "gnn_ladies_extract_f32: segment totals must be in [0, 2^31)");
  GNN_REQUIRE(nnz <= rowseg_total && (!tr || nnz <= colseg_total),
              "gnn_ladies_extract_f32: nnz exceeds the graph entries scanned");
  const size_t need = gnn_ladies_extract_workspace_bytes(num_nodes, M, K, tr, rowseg_total, colseg_total);
  GNN_REQUIRE(workspace && workspace_bytes >= need, "gnn_ladies_extract_f32: workspace too small (%zu < %zu)",
              workspace_bytes, need);
  hipStream_t st = (hipStream_t)stream;
  const int64_t words = table_words(num_nodes);
  char* wp = (char*)workspace;
  auto take = [&](size_t bytes) {
    char* p = wp;
    wp += gnn::align_up(bytes, 256);
    return p;
  };
  // chunk counts per side (experiment knobs: GNN_LX_XW chunks per side, GNN_LX_XU=16, GNN_LX_LDS=0)
  int64_t want = 0;
  if (const char* e = getenv("GNN_LX_XW")) want = atoll(e);
  const int64_t Ts[2] = {rowseg_total, tr ? colseg_total : 0};
  int XU = 8;
  for (int k = 0; k < (tr ? 2 : 1); ++k)
    if (chunks_for(Ts[k], 8, want) > XW_MAX) XU = 16;
  if (const char* e = getenv("GNN_LX_XU"))
    if (atoi(e) == 16) XU = 16;
  Sides sd{};
  sd.n = tr ? 2 : 1;
  sd.words = (int)words;
  for (int k = 0; k < sd.n; ++k) {
    Side& s = sd.s[k];
    const int64_t xw = chunks_for(Ts[k], XU, want);
    GNN_REQUIRE(xw <= XW_MAX, "gnn_ladies_extract_f32: %lld graph entries per side exceed the %d x %d limit",
                (long long)Ts[k], XW_MAX, 64 * XU);
    s.ptr = k == 0 ? indptr : indptr_t;
    s.idx = k == 0 ? indices : indices_t;
    s.src = k == 0 ? rows : cols;
    s.S = k == 0 ? rowseg : colseg;
    s.ids = k == 0 ? cols : rows;  // A keeps the nodes of cols, Aᵀ those of rows
    s.R = (int)(k == 0 ? M : K);
    s.nids = (int)(k == 0 ? K : M);
    s.tab = (Word*)take((size_t)words * sizeof(Word));
    s.qs = (int*)take((size_t)(XW_MAX + 1) * 4);
    s.cnt = (int*)take((size_t)XW_MAX * 4);
    s.gcnt = (int*)take((size_t)(XW_MAX / GROUP) * 4);
    s.gsum = (int*)take((size_t)(XW_MAX / GROUP) * 4);
    s.segbase = (int64_t*)take((size_t)(s.R > 0 ? s.R : 1) * 8);
    s.gap = (unsigned long long*)take((size_t)std::max<int64_t>(Ts[k], 1) * 8);
    s.rowptr = k == 0 ? rowptr : nullptr;
    s.out_idx = k == 0 ? col : rows_t;
    s.out_val = k == 0 ? val : val_t;
    s.transpose = k;
    s.nnz = (int)nnz;
    s.T = (int)Ts[k];
    s.xw = (int)xw;
  }
  int64_t nprep = words * sd.n;
  for (int k = 0; k < sd.n; ++k) nprep += sd.s[k].R + 1 + (sd.s[k].xw + GROUP - 1) / GROUP;
  lx_prep_kernel<<<dim3((unsigned)ceil_div(nprep, 256)), dim3(256), 0, st>>>(sd);
  GNN_LAUNCHED("lx_prep_kernel");
  const int64_t waves = sd.s[0].xw + (tr ? sd.s[1].xw : 0);
  const size_t tab_bytes = (size_t)words * sizeof(Word);
  bool lds = tab_bytes <= LDS_TABLE_MAX;
  if (const char* e = getenv("GNN_LX_LDS")) lds = lds && atoi(e) != 0;
  const int wgw = lds ? LDS_WAVES : GLB_WAVES, cpw = lds ? LDS_CPW : 1;
  const dim3 grid((unsigned)(waves / (wgw * cpw))), block((unsigned)(64 * wgw));
  const size_t shm = lds ? tab_bytes : 0;
  bool gsum = true;  // GNN_LX_GSUM=0: the last-arriver group sums (A/B)
  if (const char* e = getenv("GNN_LX_GSUM")) gsum = atoi(e) != 0;
  if (XU == 8 && lds && gsum)
    lx_walk_kernel<8, LDS_WAVES, LDS_CPW, true, true><<<grid, block, shm, st>>>(sd, degree, normfact);
  else if (XU == 8 && lds)
    lx_walk_kernel<8, LDS_WAVES, LDS_CPW, true, false><<<grid, block, shm, st>>>(sd, degree, normfact);
  else if (XU == 8)
    lx_walk_kernel<8, GLB_WAVES, 1, false, true><<<grid, block, 0, st>>>(sd, degree, normfact);
  else if (lds)
    lx_walk_kernel<16, LDS_WAVES, LDS_CPW, true, true><<<grid, block, shm, st>>>(sd, degree, normfact);
  else
    lx_walk_kernel<16, GLB_WAVES, 1, false, true><<<grid, block, 0, st>>>(sd, degree, normfact);
  GNN_LAUNCHED("lx_walk_kernel");
  int ccpw = COMPACT_CPW;
  if (const char* e = getenv("GNN_LX_CCPW")) ccpw = atoi(e);
  if (ccpw == 8)
    lx_compact_kernel<8><<<dim3((unsigned)(waves / 32)), dim3(256), 0, st>>>(sd, err_flag);
  else if (ccpw == 1)
    lx_compact_kernel<1><<<dim3((unsigned)(waves / 4)), dim3(256), 0, st>>>(sd, err_flag);
  else
    lx_compact_kernel<COMPACT_CPW><<<dim3((unsigned)(waves / (4 * COMPACT_CPW))), dim3(256), 0, st>>>(sd, err_flag);
  GNN_LAUNCHED("lx_compact_kernel");
  return 0;
}

}  // extern "C"
