"""Host probe: are the synthetic graphs and the LADIES draws the same on this machine as on another?
Prints sha256 prefixes of the generated graph (indptr + indices + data) and of three native LADIES
batches per geometry, and checks batch 0 of each against the numpy restatement bit for bit.

    python scripts/host_fingerprint.py reddit products
"""
import hashlib
import os
import platform
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gnn_amd import graphs, sampler  # noqa: E402


def sha(*arrays):
    h = hashlib.sha256()
    for a in arrays:
        h.update(np.ascontiguousarray(a).tobytes())
    return h.hexdigest()[:16]


def batch_sha(b):
    arrs = []
    for L in b.layers:
        if L is not None:
            arrs += [L.fullrowptr, L.rowptr, L.colidx, L.normfact]
    arrs += [np.asarray(s, np.int64) for s in b.sampled_nodes] + [b.input_nodes]
    return sha(*arrs)


print(platform.processor() or platform.machine(), "numpy", np.__version__, flush=True)
w = np.random.default_rng(0).lognormal(0.0, 1.3, 100000)
print("lognormal", sha(w), "cumsum", sha(np.cumsum(w / w.sum())), flush=True)
for name in sys.argv[1:] or ["reddit"]:
    spec = {"reddit": graphs.REDDIT, "products": graphs.PRODUCTS}[name]
    A, labels, _, nc, train, *_ = graphs.make_dataset(spec, seed=0, with_features=False)
    lap = graphs.lap_matrix(A, "graphsage")
    print(name, "graph", A.shape[0], A.nnz, sha(A.indptr, A.indices, A.data), "lap", sha(lap.indptr, lap.indices, lap.data),
          flush=True)
    N = A.shape[0]
    lab = labels if labels is not None else None
    batches = sampler.rank_batches(train, 512, 0, 1, 3)[:3]
    dev_of = np.zeros(N, np.int64)
    idx_on = np.arange(N)
    out = []
    for i, bn in enumerate(batches):
        args = (1000 + i, bn, np.array([8192] * 3), N, lap, lab, [1, 1, 1], dev_of, idx_on, None, 1.0, [0])
        nb = sampler.ladies_sample_host(*args, native=True)
        out.append(batch_sha(nb))
        if i == 0:
            pb = sampler.ladies_sample_host(*args, native=False)
            out.append("numpy-equal" if batch_sha(pb) == out[0] else "numpy-DIFFERS " + batch_sha(pb))
    print(name, "ladies", " ".join(out), flush=True)
