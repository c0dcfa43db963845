"""Host-side probe: one sampler thread's draw time per batch (native LADIES / FastGCN, samp 8192,
batch 512, 3 layers) on a synthetic graph, with a checksum of every output array so a change to
the sampler can be checked for identical results as well as timed.

    python scripts/sampler_probe.py products ladies,ladies-dx,fastgcn 20
"""
import hashlib
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gnn_amd import graphs, sampler  # noqa: E402
from gnn_amd._lib import sampler_lib  # noqa: E402

spec = {"reddit": graphs.REDDIT, "products": graphs.PRODUCTS, "papers": graphs.PAPERS_SCALED,
        "products-test": graphs.PRODUCTS_TEST}[sys.argv[1] if len(sys.argv) > 1 else "reddit"]
kinds = (sys.argv[2] if len(sys.argv) > 2 else "ladies,ladies-dx,fastgcn").split(",")
n = int(sys.argv[3]) if len(sys.argv) > 3 else 20
cache = os.environ.get("GNN_PROBE_CACHE", "")  # directory: keep the graph arrays between runs


class _Cached:
    """NativeGraph's fields as saved by an earlier run (GraphSAGE: symmetric structure, no zeros)."""

    def __init__(self, z):
        self.indptr, self.indices, self.num_nodes = z["indptr"], z["indices"], int(z["indptr"].size - 1)
        self.data, self.transpose_structure = None, (True, None, None)
        self.fastgcn_p = z["p"] if "p" in z else None


t0 = time.perf_counter()
cpath = os.path.join(cache, f"{spec.name}.npz") if cache else ""
if cache:
    os.makedirs(cache, exist_ok=True)
if cpath and os.path.exists(cpath) and "fastgcn" not in kinds:
    z = np.load(cpath)
    train, A = z["train"], None
    print(f"graph {spec.name} from {cpath}", flush=True)
else:
    A, labels, feats, nc, train, *_ = graphs.make_dataset(spec, seed=0, with_features=False)
    print(f"graph {spec.name}: {A.shape[0]} nodes {A.nnz} entries ({time.perf_counter() - t0:.1f} s)", flush=True)
batches = sampler.rank_batches(train, 512, 0, 1, n + 2)[: n + 2]
for kind in kinds:
    model = "gcn" if kind == "fastgcn" else "graphsage"
    if A is None:
        g = _Cached(z)
    else:
        g = sampler.native_graph(graphs.lap_matrix(A, model))
        if cpath and model == "graphsage" and not os.path.exists(cpath):
            np.savez(cpath, indptr=g.indptr, indices=g.indices, train=np.asarray(train))
    cc = None
    if kind.startswith("ladies-dx"):
        g.transpose_structure
    if kind == "ladies-dx-cc":  # U's column counts on the GPU (needs a GPU)
        cc = sampler.ColumnCounter(g, "cuda:0")
    if kind == "fastgcn":
        g.fastgcn_p
    h = hashlib.sha256()
    ts = []
    for i, b in enumerate(batches):
        t = time.perf_counter()
        layers, sampled, inp, _ = sampler._native_layers(1000 + i, b, [8192] * 3, g, [1, 1, 1],
                                                         kind="fastgcn" if kind == "fastgcn" else "ladies",
                                                         device_extract=kind.startswith("ladies-dx"), colcount=cc)
        dt = time.perf_counter() - t
        if i >= 2:
            ts.append(dt)
        for L in layers:
            for f in ("fullrowptr", "rowptr", "colidx", "normfact", "csc_colptr", "csc_rows", "rows", "cols", "colseg"):
                a = getattr(L, f, None)
                if a is not None:
                    h.update(np.ascontiguousarray(a).tobytes())
        for s in sampled:
            h.update(np.ascontiguousarray(s).tobytes())
        h.update(np.ascontiguousarray(inp).tobytes())
    ts = np.array(ts) * 1e3
    prof = np.zeros(8)
    if sampler_lib().gnn_sampler_profile(prof.ctypes.data, 8, 1) == 0 and prof[7] > 0:
        names = ["scratch", "rowptr", "count", "draw", "after", "extract", "tail"]
        print("  ms/call: " + " ".join(f"{nm} {1e3 * prof[i] / prof[7]:.2f}" for i, nm in enumerate(names)), flush=True)
    print(f"{kind}: {ts.mean():.2f} ms/batch (median {np.median(ts):.2f}, min {ts.min():.2f})  sha {h.hexdigest()[:16]}",
          flush=True)
