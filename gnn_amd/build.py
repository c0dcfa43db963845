"""In-tree build of libgnn_spmm.so (hipcc, gfx950). No JIT cache: the .so lives next to
the package so it travels with the repository snapshot to the GPU box."""
from __future__ import annotations

import hashlib
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
SRCS = [os.path.join(HERE, "csrc", f) for f in ("spmm.hip", "sage.hip")]
HDRS = [os.path.join(REPO, "include", f) for f in ("gnn_spmm.h", "gnn_layers.h")] + [
    os.path.join(HERE, "csrc", "common.h")]
OUT = os.path.join(HERE, "libgnn_spmm.so")
ARCH = os.environ.get("GNN_OFFLOAD_ARCH", "gfx950")


def _build_id() -> str:
    h = hashlib.sha1()
    for p in SRCS + HDRS:
        with open(p, "rb") as f:
            h.update(f.read())
    return h.hexdigest()[:12]


def build_library(force: bool = False, verbose: bool = False) -> str:
    bid = _build_id()
    stamp = OUT + ".buildid"
    if not force and os.path.exists(OUT) and os.path.exists(stamp):
        with open(stamp) as f:
            if f.read().strip() == bid:
                return OUT
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    cmd = [hipcc, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared",
           f"-I{os.path.join(REPO, 'include')}", f'-DGNN_BUILD_ID="{bid}"', "-o", OUT + ".tmp"] + SRCS
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(OUT + ".tmp", OUT)
    with open(stamp, "w") as f:
        f.write(bid)
    return OUT


if __name__ == "__main__":
    print(build_library(force=True, verbose=True))
