"""Host-side probe: batch producer throughput (Reddit LADIES samp 8192 / batch 512, host staging)
vs worker count — the Python BatchLoader (native sampler called from Python threads) against
the NativeLoader (C++ worker threads, one blob per batch), with and without GPU extraction."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gnn_amd import graphs, loader, placement, staging  # noqa: E402

A, labels, feats, nc, train, *_ = graphs.make_dataset(graphs.REDDIT, seed=0)
lap = graphs.row_normalize(A)
lap.sum_duplicates()
N = A.shape[0]
pl = placement.create_buffer(lap, train, int(0.1 * N), [0], 3, alpha=0)
store = staging.FeatureStore(feats, pl.gpu_buffer_group[0], "cpu", 0)
n = int(sys.argv[2]) if len(sys.argv) > 2 else 120
kinds = sys.argv[3].split(",") if len(sys.argv) > 3 else ["python", "python-dx", "native", "native-dx"]
for w in [int(x) for x in sys.argv[1].split(",")]:
    for kind in kinds:
        cls = loader.NativeLoader if kind.startswith("native") else loader.BatchLoader
        ld = cls(lap, labels, train, 8192, 512, [1, 1, 1], pl.device_id_of_nodes_group[0],
                 pl.idx_of_nodes_on_device_group[0], store=store, workers=w, device_extract=kind.endswith("-dx"))
        it = ld.forever()
        for _ in range(2 * w):
            next(it)
        t = time.perf_counter()
        for _ in range(n):
            next(it)
        dt = time.perf_counter() - t
        ld.close()
        print(f"workers {w} {kind}: {n / dt:.1f} batches/s", flush=True)
