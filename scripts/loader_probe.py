"""Host-side probe: BatchLoader throughput (native LADIES + pinned host staging) vs worker count."""
import time, numpy as np, torch, sys
import os; sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gnn_amd import _lib
if os.environ.get("GNN_SAMPLER_LIB"):  # A/B another build of libgnn_sampler.so
    _lib.SAMPLER_PATH = os.environ["GNN_SAMPLER_LIB"]
from gnn_amd import graphs, sampler, placement, staging, loader
A, labels, feats, nc, train, *_ = graphs.make_dataset(graphs.REDDIT, seed=0)
lap = graphs.row_normalize(A); lap.sum_duplicates()
N = A.shape[0]
pl = placement.create_buffer(lap, train, int(0.1*N), [0], 3, alpha=0)
store = staging.FeatureStore(feats, pl.gpu_buffer_group[0], "cpu", 0)
for w in [int(x) for x in sys.argv[1].split(",")]:
    for use_store in (False, True):
        ld = loader.BatchLoader(lap, labels, train, 8192, 512, [1,1,1], pl.device_id_of_nodes_group[0], pl.idx_of_nodes_on_device_group[0], store=store if use_store else None, workers=w)
        it = ld.forever()
        for _ in range(2*w): next(it)
        t=time.perf_counter(); n=int(sys.argv[2]) if len(sys.argv) > 2 else 120
        for _ in range(n): next(it)
        dt=time.perf_counter()-t
        ld.close()
        print(f"workers {w} store {use_store}: {n/dt:.1f} batches/s", flush=True)
