// loader.cpp — native mini-batch producer of libgnn_sampler.so (include/gnn_sampler.h,
// gnn_loader_*).
//
// Reference: prepare_data (sampler.py:163-210) submits ladies_sampler calls to a Python
// ThreadPoolExecutor; each call returns the sub-graph pieces, the feature-placement masks and
// index lists (sampler.py:150-158) and the dense labels (sampler.py:160), and the training loop
// then gathers the non-buffered feature rows on the host (main.py:129-134).
//
// Here worker threads (std::thread, never touching the Python interpreter) run the whole
// per-batch host side — the draw (gnn_ladies_sample_dev & co.), the CSC of host-extracted
// layers, the residual row maps, the placement split of the layer-0 inputs (own buffer / host /
// peers), the dense labels and the gather of the host feature rows — and write everything into
// ONE contiguous (pinned, when the HIP runtime is loaded) "batch blob" whose layout a small
// int64 descriptor describes. The training thread uploads a blob with a single host-to-device
// copy and takes device views of its sections. Batches come out in submission order.
#include <dlfcn.h>

#include <algorithm>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <new>
#include <string>
#include <thread>
#include <vector>

#include <emmintrin.h>
#include <xmmintrin.h>

#include "gnn_sampler.h"
#include "sampler_internal.h"

using gnn_smp::Layer;

namespace {

constexpr int64_t kAlign = 256;

int64_t align_up(int64_t x) { return (x + kAlign - 1) / kAlign * kAlign; }

// Descriptor layout (int64): see gnn_sampler.h (GNN_BLOB_*).
struct Sec {
  int slot;       // descriptor slot of (offset, count)
  int64_t count;  // elements
  int64_t esize;  // bytes per element
};

using HostMallocFn = int (*)(void**, size_t, unsigned int);
using HostFreeFn = int (*)(void*);

class Pool {
 public:
  explicit Pool(bool want_pinned) {
    if (want_pinned) {
      // the HIP runtime the process already has loaded (torch's), never a second copy
      void* h = dlopen("libamdhip64.so.7", RTLD_NOW | RTLD_NOLOAD);
      if (h) {
        halloc_ = (HostMallocFn)dlsym(h, "hipHostMalloc");
        hfree_ = (HostFreeFn)dlsym(h, "hipHostFree");
        if (!halloc_ || !hfree_) halloc_ = nullptr, hfree_ = nullptr;
      }
    }
  }
  ~Pool() {
    for (auto& a : all_) release(a.first, a.second);
  }
  bool pinned() const { return halloc_ != nullptr; }

  char* get(size_t need, size_t& cap) {
    {
      std::lock_guard<std::mutex> g(mu_);
      auto it = free_.lower_bound(need);
      if (it != free_.end() && it->first <= need * 2 + (64u << 20)) {
        cap = it->first;
        char* p = it->second;
        free_.erase(it);
        return p;
      }
    }
    cap = (need + need / 8 + (1u << 20)) & ~(size_t)((1u << 20) - 1);
    char* p = nullptr;
    bool pin = false;
    if (halloc_) {
      void* q = nullptr;
      if (halloc_(&q, cap, 0) == 0 && q) p = (char*)q, pin = true;
    }
    if (!p) {
      void* q = nullptr;
      if (posix_memalign(&q, 4096, cap) != 0) throw std::bad_alloc();
      p = (char*)q;
    }
    std::lock_guard<std::mutex> g(mu_);
    all_.emplace_back(p, pin);
    return p;
  }

  void put(char* p, size_t cap) {
    std::lock_guard<std::mutex> g(mu_);
    free_.emplace(cap, p);
  }

 private:
  void release(char* p, bool pin) {
    if (pin && hfree_) hfree_(p);
    else free(p);
  }
  std::mutex mu_;
  std::multimap<size_t, char*> free_;
  std::vector<std::pair<char*, bool>> all_;
  HostMallocFn halloc_ = nullptr;
  HostFreeFn hfree_ = nullptr;
};

struct Job {
  uint64_t id;
  uint32_t seed;
  std::vector<int64_t> nodes;
};

}  // namespace

struct gnn_batch {
  uint64_t id = 0;
  std::shared_ptr<Pool> pool;  // the pool the blob goes back to (outlives the loader if needed)
  char* blob = nullptr;
  size_t cap = 0;
  std::vector<int64_t> desc;
  int rc = 0;
  std::string err;
};

struct gnn_loader {
  // graph + features + placement (borrowed: the caller keeps them alive)
  const int64_t* indptr;
  const int32_t* indices;
  const float* data;
  const int64_t* indptr_t;
  int64_t N;
  const int64_t* lab_ptr;
  const int32_t* lab_idx;
  const float* lab_val;
  int64_t C;
  const int64_t* dev_of;
  const int64_t* idx_on;
  int32_t rank, world;
  std::vector<int64_t> devices;
  const float* feat;
  int64_t ld_feat, F, ld_x0;
  std::vector<int64_t> samp;
  std::vector<int32_t> orders;
  int32_t kind, device_extract, csc_from;
  const double* fastgcn_p;
  gnn_colcount_api cc{};  // device column counting (cc.add == NULL: on the host)
  int cc_workers = 0;     // workers 0 .. cc_workers-1 count on the device (0: all)
  // machinery
  std::shared_ptr<Pool> pool;
  std::vector<std::thread> threads;
  std::mutex mu;
  std::condition_variable cv_job, cv_done;
  std::deque<Job> jobs;
  std::map<uint64_t, gnn_batch*> done;
  uint64_t next_id = 0, next_out = 0;
  bool stop = false;

  void run(int worker);
  gnn_batch* produce(const Job& job, void** cc_ctx, bool device_counts);
};

namespace {

bool getenv_off(const char* name) {
  static const bool off = [name] {
    const char* e = getenv(name);
    return e && atoi(e) == 0;
  }();
  return off;
}

// One feature row (F floats) into an ld-wide row of the pinned blob, zero padded, by 16-byte
// non-temporal stores: the blob is read once, by the copy engine, so its lines need no
// read-for-ownership and should not evict the graph the sampler walks (the host rows are a
// quarter of a Reddit batch's producer time). Byte-identical to memcpy + memset.
inline void copy_row_nt(float* dst, const float* src, int64_t F, int64_t ld) {
  int64_t c = 0;
  for (; c + 4 <= F; c += 4)
    _mm_stream_si128(reinterpret_cast<__m128i*>(dst + c), _mm_loadu_si128(reinterpret_cast<const __m128i*>(src + c)));
  for (; c < ld; c += 4) {
    alignas(16) float t[4];
    for (int k = 0; k < 4; ++k) t[k] = c + k < F ? src[c + k] : 0.0f;
    _mm_stream_si128(reinterpret_cast<__m128i*>(dst + c), _mm_load_si128(reinterpret_cast<const __m128i*>(t)));
  }
}

// Fill the blob of one sampled batch (layout in gnn_sampler.h).
void fill(gnn_loader& ld, const gnn_ladies_result& res, const Job& job, gnn_batch& b) {
  const int nl = (int)ld.orders.size();
  const int64_t W = ld.world;
  b.desc.assign((size_t)(GNN_BLOB_HEADER + nl * GNN_BLOB_LAYER_SLOTS + GNN_BLOB_BATCH_SLOTS + 4 * W), 0);
  int64_t* d = b.desc.data();
  const std::vector<int64_t>& inp = res.input_nodes;
  const int64_t n_in = (int64_t)inp.size();
  const int64_t bs = (int64_t)job.nodes.size();
  // the placement split of the layer-0 inputs (sampler.py:150-158)
  std::vector<int64_t> own_pos, own_src, host_pos, host_src;
  std::vector<std::vector<int64_t>> peer_pos((size_t)W), peer_src((size_t)W);
  const int64_t own_dev = ld.devices[(size_t)ld.rank];
  for (int64_t i = 0; i < n_in; ++i) {
    const int64_t v = inp[(size_t)i];
    const int64_t dv = ld.dev_of[v];
    if (dv == -1) {
      host_pos.push_back(i);
      host_src.push_back(v);
    } else if (dv == own_dev) {
      own_pos.push_back(i);
      own_src.push_back(ld.idx_on[v]);
    } else {
      for (int64_t j = 0; j < W; ++j)
        if (ld.devices[(size_t)j] == dv) {
          peer_pos[(size_t)j].push_back(i);
          peer_src[(size_t)j].push_back(ld.idx_on[v]);
          break;
        }
    }
  }
  std::vector<Sec> secs;
  for (int li = 0; li < nl; ++li) {
    const Layer& L = res.layers[(size_t)li];
    int64_t* s = d + GNN_BLOB_HEADER + li * GNN_BLOB_LAYER_SLOTS;
    const int base = GNN_BLOB_HEADER + li * GNN_BLOB_LAYER_SLOTS;
    s[GNN_L_PRESENT] = L.present;
    if (!L.present) continue;
    s[GNN_L_ON_DEVICE] = L.on_device;
    s[GNN_L_M] = L.M;
    s[GNN_L_K] = L.K;
    s[GNN_L_NNZ] = L.nnz;
    s[GNN_L_SNUM] = L.s_num;
    s[GNN_L_NSAMPLED] = (int64_t)L.sampled.size();
    const bool want_t = li >= ld.csc_from;
    const bool rmap = li >= 1 && !L.sampled.empty();
    s[GNN_L_HAS_RMAP] = rmap;
    secs.push_back({base + GNN_L_NORMFACT, L.K, 4});
    secs.push_back({base + GNN_L_SAMPLED, (int64_t)L.sampled.size(), 8});
    if (rmap) secs.push_back({base + GNN_L_RMAP, L.K, 4});
    if (L.on_device) {
      secs.push_back({base + GNN_L_ROWS, L.M, 4});
      secs.push_back({base + GNN_L_COLS, L.K, 4});
      secs.push_back({base + GNN_L_CSC_COLPTR, L.K + 1, 4});
      secs.push_back({base + GNN_L_FULLROWPTR, L.M + 1, 4});
      secs.push_back({base + GNN_L_COLSEG, L.K + 1, 4});
    } else {
      secs.push_back({base + GNN_L_FULLROWPTR, L.M + 1, 4});
      secs.push_back({base + GNN_L_ROWPTR, L.M + 1, 4});
      secs.push_back({base + GNN_L_COLIDX, L.nnz, 4});
      if (want_t) {
        secs.push_back({base + GNN_L_CSC_COLPTR, L.K + 1, 4});
        secs.push_back({base + GNN_L_CSC_ROWS, L.nnz, 4});
      }
    }
  }
  const int bb = GNN_BLOB_HEADER + nl * GNN_BLOB_LAYER_SLOTS;
  secs.push_back({bb + GNN_B_LABELS, bs * ld.C, 4});
  secs.push_back({bb + GNN_B_HOST_ROWS, ld.feat ? (int64_t)host_src.size() * ld.ld_x0 : 0, 4});
  secs.push_back({bb + GNN_B_OWN_POS, (int64_t)own_pos.size(), 8});
  secs.push_back({bb + GNN_B_OWN_SRC, (int64_t)own_src.size(), 8});
  secs.push_back({bb + GNN_B_HOST_POS, (int64_t)host_pos.size(), 8});
  secs.push_back({bb + GNN_B_HOST_SRC, (int64_t)host_src.size(), 8});
  secs.push_back({bb + GNN_B_INPUT_NODES, n_in, 8});
  for (int64_t j = 0; j < W; ++j) {
    secs.push_back({bb + GNN_BLOB_BATCH_SLOTS + 4 * (int)j, (int64_t)peer_pos[(size_t)j].size(), 8});
    secs.push_back({bb + GNN_BLOB_BATCH_SLOTS + 4 * (int)j + 2, (int64_t)peer_src[(size_t)j].size(), 8});
  }
  int64_t off = 0;
  for (const Sec& s : secs) {
    d[s.slot] = off;
    d[s.slot + 1] = s.count;
    off += align_up(s.count * s.esize);
  }
  const int64_t total = off > 0 ? off : kAlign;
  b.pool = ld.pool;
  b.blob = ld.pool->get((size_t)total, b.cap);
  char* blob = b.blob;
  auto at = [&](int slot) { return blob + d[slot]; };
  auto put = [&](int slot, const void* src, int64_t bytes) {
    if (bytes) std::memcpy(at(slot), src, (size_t)bytes);
  };
  for (int li = 0; li < nl; ++li) {
    const Layer& L = res.layers[(size_t)li];
    if (!L.present) continue;
    const int base = GNN_BLOB_HEADER + li * GNN_BLOB_LAYER_SLOTS;
    put(base + GNN_L_NORMFACT, L.normfact.data(), L.K * 4);
    put(base + GNN_L_SAMPLED, L.sampled.data(), (int64_t)L.sampled.size() * 8);
    if (d[base + GNN_L_HAS_RMAP]) {  // rmap[sampled[i]] = i, -1 elsewhere (the fused residual's row map)
      int32_t* r = (int32_t*)at(base + GNN_L_RMAP);
      std::fill(r, r + L.K, -1);
      for (size_t i = 0; i < L.sampled.size(); ++i) r[L.sampled[i]] = (int32_t)i;
    }
    if (L.on_device) {
      put(base + GNN_L_ROWS, L.rows.data(), L.M * 4);
      put(base + GNN_L_COLS, L.cols.data(), L.K * 4);
      put(base + GNN_L_CSC_COLPTR, L.colptr.data(), (L.K + 1) * 4);
      put(base + GNN_L_FULLROWPTR, L.fullrowptr.data(), (L.M + 1) * 4);
      put(base + GNN_L_COLSEG, L.colseg.data(), (L.K + 1) * 4);
    } else {
      put(base + GNN_L_FULLROWPTR, L.fullrowptr.data(), (L.M + 1) * 4);
      put(base + GNN_L_ROWPTR, L.rowptr.data(), (L.M + 1) * 4);
      put(base + GNN_L_COLIDX, L.colidx.data(), L.nnz * 4);
      if (d[base + GNN_L_CSC_ROWS + 1] || d[base + GNN_L_CSC_COLPTR + 1])
        gnn_smp::layer_csc(L, (int32_t*)at(base + GNN_L_CSC_COLPTR), (int32_t*)at(base + GNN_L_CSC_ROWS));
    }
  }
  // labels_full[batch_nodes].todense() (sampler.py:160), float32
  float* lab = (float*)at(bb + GNN_B_LABELS);
  std::fill(lab, lab + bs * ld.C, 0.0f);
  for (int64_t i = 0; i < bs; ++i) {
    const int64_t v = job.nodes[(size_t)i];
    for (int64_t k = ld.lab_ptr[v]; k < ld.lab_ptr[v + 1]; ++k) lab[i * ld.C + ld.lab_idx[k]] += ld.lab_val[k];
  }
  put(bb + GNN_B_OWN_POS, own_pos.data(), (int64_t)own_pos.size() * 8);
  put(bb + GNN_B_OWN_SRC, own_src.data(), (int64_t)own_src.size() * 8);
  put(bb + GNN_B_HOST_POS, host_pos.data(), (int64_t)host_pos.size() * 8);
  put(bb + GNN_B_HOST_SRC, host_src.data(), (int64_t)host_src.size() * 8);
  put(bb + GNN_B_INPUT_NODES, inp.data(), n_in * 8);
  for (int64_t j = 0; j < W; ++j) {
    put(bb + GNN_BLOB_BATCH_SLOTS + 4 * (int)j, peer_pos[(size_t)j].data(), (int64_t)peer_pos[(size_t)j].size() * 8);
    put(bb + GNN_BLOB_BATCH_SLOTS + 4 * (int)j + 2, peer_src[(size_t)j].data(),
        (int64_t)peer_src[(size_t)j].size() * 8);
  }
  // the non-buffered feature rows (main.py:133), ld_x0-wide rows with zero padding
  if (ld.feat) {
    float* rows = (float*)at(bb + GNN_B_HOST_ROWS);
    const bool nt = ld.ld_x0 % 4 == 0 && (uintptr_t)rows % 16 == 0 && !getenv_off("GNN_LOADER_NT");
    constexpr size_t kAhead = 4;  // source rows prefetched ahead (random rows of the feature table)
    for (size_t i = 0; i < host_src.size(); ++i) {
      if (i + kAhead < host_src.size()) {
        const char* p = reinterpret_cast<const char*>(ld.feat + host_src[i + kAhead] * ld.ld_feat);
        _mm_prefetch(p, _MM_HINT_T0);
        _mm_prefetch(p + 64, _MM_HINT_T0);
      }
      float* dst = rows + (int64_t)i * ld.ld_x0;
      const float* src = ld.feat + host_src[i] * ld.ld_feat;
      if (nt) {
        copy_row_nt(dst, src, ld.F, ld.ld_x0);
      } else {
        std::memcpy(dst, src, (size_t)ld.F * 4);
        if (ld.ld_x0 > ld.F) std::memset(dst + ld.F, 0, (size_t)(ld.ld_x0 - ld.F) * 4);
      }
    }
    if (nt) _mm_sfence();  // the stores are visible before the batch is handed over
  }
  d[GNN_H_VERSION] = GNN_BLOB_VERSION;
  d[GNN_H_LAYERS] = nl;
  d[GNN_H_BYTES] = total;
  d[GNN_H_BATCH] = bs;
  d[GNN_H_CLASSES] = ld.C;
  d[GNN_H_INPUTS] = n_in;
  d[GNN_H_WORLD] = W;
  d[GNN_H_LD_X0] = ld.ld_x0;
  d[GNN_H_SEED] = job.seed;
  d[GNN_H_PINNED] = ld.pool->pinned();
}

}  // namespace

gnn_batch* gnn_loader::produce(const Job& job, void** cc_ctx, bool device_counts) {
  std::unique_ptr<gnn_batch> b(new gnn_batch());
  b->id = job.id;
  gnn_ladies_result* res = nullptr;
  const int nl = (int)orders.size();
  int rc = 0;
  const bool use_cc = device_counts && cc.add != nullptr && kind == GNN_SAMPLER_LADIES;
  if (use_cc && !*cc_ctx) {  // this worker's context, made on its first batch
    rc = cc.create(cc.device, N, cc.indptr, cc.indices, cc_ctx);
    if (rc != 0) {
      b->rc = rc;
      b->err = "gnn_loader: gnn_colcount_create failed";
      return b.release();
    }
  }
  if (kind == GNN_SAMPLER_FASTGCN)
    rc = gnn_fastgcn_sample(indptr, indices, data, N, fastgcn_p, job.nodes.data(), (int64_t)job.nodes.size(),
                            samp.data(), orders.data(), nl, job.seed, &res);
  else if (kind == GNN_SAMPLER_SUBGRAPH)
    rc = gnn_subgraph_sample(indptr, indices, data, N, job.nodes.data(), (int64_t)job.nodes.size(), samp.data(),
                             orders.data(), nl, job.seed, &res);
  else
    rc = gnn_ladies_sample_cc(indptr, indices, data, indptr_t, N, job.nodes.data(), (int64_t)job.nodes.size(),
                              samp.data(), orders.data(), nl, job.seed, device_extract, use_cc ? &cc : nullptr,
                              use_cc ? *cc_ctx : nullptr, &res);
  if (rc != 0) {
    b->rc = rc;
    b->err = gnn_sampler_last_error();
    return b.release();
  }
  std::unique_ptr<gnn_ladies_result, void (*)(gnn_ladies_result*)> hold(res, gnn_ladies_free);
  try {
    fill(*this, *res, job, *b);
  } catch (const std::bad_alloc&) {
    b->rc = -12;
    b->err = "gnn_loader: out of host memory";
  }
  return b.release();
}

void gnn_loader::run(int worker) {
  void* cc_ctx = nullptr;
  struct Close {
    gnn_loader* ld;
    void** ctx;
    ~Close() {
      if (*ctx && ld->cc.destroy) ld->cc.destroy(*ctx);
    }
  } close{this, &cc_ctx};
  for (;;) {
    Job job;
    {
      std::unique_lock<std::mutex> lk(mu);
      cv_job.wait(lk, [&] { return stop || !jobs.empty(); });
      if (stop) return;
      job = std::move(jobs.front());
      jobs.pop_front();
    }
    // gnn_loader_set_colcount_workers (read after the job: set before the first submission;
    // GNN_CC_WORKERS overrides for experiments)
    int k = cc_workers;
    if (const char* e = getenv("GNN_CC_WORKERS")) k = atoi(e);
    gnn_batch* b = produce(job, &cc_ctx, k <= 0 || worker < k);
    {
      std::lock_guard<std::mutex> lk(mu);
      done[b->id] = b;
    }
    cv_done.notify_all();
  }
}

extern "C" {

gnn_loader* gnn_loader_create(const int64_t* indptr, const int32_t* indices, const float* data,
                              const int64_t* indptr_t, int64_t num_nodes,
                              const int64_t* label_indptr, const int32_t* label_indices, const float* label_values,
                              int64_t num_classes, const int64_t* device_id_of_nodes,
                              const int64_t* idx_of_nodes_on_device, int32_t rank, int32_t world,
                              const int64_t* devices, const float* feat, int64_t ld_feat, int64_t F, int64_t ld_x0,
                              const int64_t* samp_num, const int32_t* orders, int32_t num_layers, int32_t kind,
                              const double* fastgcn_p, int32_t device_extract, int32_t csc_from, int32_t workers,
                              int32_t pinned) {
  if (!indptr || !indices || num_nodes <= 0 || !label_indptr || (num_classes > 0 && (!label_indices || !label_values))
      || !device_id_of_nodes || !idx_of_nodes_on_device || world < 1 || rank < 0 || rank >= world || !devices
      || num_layers < 0 || num_layers > GNN_BLOB_MAX_LAYERS || (num_layers > 0 && (!samp_num || !orders))
      || workers < 1 || (kind == GNN_SAMPLER_FASTGCN && !fastgcn_p) || (feat && (F < 0 || F > ld_feat || F > ld_x0))) {
    gnn_smp::set_error("gnn_loader_create: bad arguments");
    return nullptr;
  }
  try {
    std::unique_ptr<gnn_loader> ld(new gnn_loader());
    ld->indptr = indptr;
    ld->indices = indices;
    ld->data = data;
    ld->indptr_t = indptr_t;
    ld->N = num_nodes;
    ld->lab_ptr = label_indptr;
    ld->lab_idx = label_indices;
    ld->lab_val = label_values;
    ld->C = num_classes;
    ld->dev_of = device_id_of_nodes;
    ld->idx_on = idx_of_nodes_on_device;
    ld->rank = rank;
    ld->world = world;
    ld->devices.assign(devices, devices + world);
    ld->feat = feat;
    ld->ld_feat = ld_feat;
    ld->F = F;
    ld->ld_x0 = ld_x0;
    ld->samp.assign(samp_num, samp_num + num_layers);
    ld->orders.assign(orders, orders + num_layers);
    ld->kind = kind;
    ld->device_extract = data ? 0 : device_extract;
    ld->csc_from = csc_from;
    ld->fastgcn_p = fastgcn_p;
    ld->pool.reset(new Pool(pinned != 0));
    for (int i = 0; i < workers; ++i) ld->threads.emplace_back([p = ld.get(), i] { p->run(i); });
    return ld.release();
  } catch (const std::exception& e) {
    gnn_smp::set_error(std::string("gnn_loader_create: ") + e.what());
    return nullptr;
  }
}

int gnn_loader_set_colcount(gnn_loader* ld, const gnn_colcount_api* api) {
  if (!ld || !api || !api->create || !api->add || !api->reset || !api->destroy || !api->indptr || !api->indices
      || ld->data) {
    gnn_smp::set_error("gnn_loader_set_colcount: bad arguments (or a graph with stored zeros)");
    return -22;
  }
  std::lock_guard<std::mutex> lk(ld->mu);
  if (ld->next_id != 0) {
    gnn_smp::set_error("gnn_loader_set_colcount: batches already submitted");
    return -22;
  }
  ld->cc = *api;
  return 0;
}

int gnn_loader_set_colcount_workers(gnn_loader* ld, int32_t workers) {
  if (!ld || workers < 0) {
    gnn_smp::set_error("gnn_loader_set_colcount_workers: bad arguments");
    return -22;
  }
  std::lock_guard<std::mutex> lk(ld->mu);
  if (ld->next_id != 0) {
    gnn_smp::set_error("gnn_loader_set_colcount_workers: batches already submitted");
    return -22;
  }
  ld->cc_workers = workers;
  return 0;
}

int gnn_loader_submit(gnn_loader* ld, uint32_t seed, const int64_t* nodes, int64_t n) {
  if (!ld || n < 0 || (n > 0 && !nodes)) {
    gnn_smp::set_error("gnn_loader_submit: bad arguments");
    return -22;
  }
  for (int64_t i = 0; i < n; ++i)
    if (nodes[i] < 0 || nodes[i] >= ld->N) {
      gnn_smp::set_error("gnn_loader_submit: batch node out of range");
      return -22;
    }
  {
    std::lock_guard<std::mutex> lk(ld->mu);
    ld->jobs.push_back(Job{ld->next_id++, seed, std::vector<int64_t>(nodes, nodes + n)});
  }
  ld->cv_job.notify_one();
  return 0;
}

int gnn_loader_next(gnn_loader* ld, gnn_batch** out) {
  if (!ld || !out) {
    gnn_smp::set_error("gnn_loader_next: bad arguments");
    return -22;
  }
  gnn_batch* b = nullptr;
  {
    std::unique_lock<std::mutex> lk(ld->mu);
    if (ld->next_out >= ld->next_id) {
      gnn_smp::set_error("gnn_loader_next: nothing submitted");
      return -22;
    }
    const uint64_t want = ld->next_out;
    ld->cv_done.wait(lk, [&] { return ld->done.count(want) != 0; });
    b = ld->done[want];
    ld->done.erase(want);
    ld->next_out++;
  }
  if (b->rc != 0) {
    gnn_smp::set_error(b->err);
    const int rc = b->rc;
    gnn_batch_release(b);
    *out = nullptr;
    return rc;
  }
  *out = b;
  return 0;
}

const int64_t* gnn_batch_desc(const gnn_batch* b, int64_t* n) {
  if (!b) return nullptr;
  if (n) *n = (int64_t)b->desc.size();
  return b->desc.data();
}

void* gnn_batch_blob(const gnn_batch* b) { return b ? b->blob : nullptr; }

void gnn_batch_release(gnn_batch* b) {
  if (!b) return;
  if (b->blob) b->pool->put(b->blob, b->cap);
  delete b;
}

void gnn_loader_destroy(gnn_loader* ld) {
  if (!ld) return;
  {
    std::lock_guard<std::mutex> lk(ld->mu);
    ld->stop = true;
  }
  ld->cv_job.notify_all();
  for (auto& t : ld->threads) t.join();
  for (auto& kv : ld->done) gnn_batch_release(kv.second);
  delete ld;
}

}  // extern "C"
