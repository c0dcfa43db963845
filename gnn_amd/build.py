"""In-tree builds: libgnn_spmm.so (hipcc, gfx950), libgnn_sampler.so (g++, host only) and the
PyTorch-ROCm extension module `spmm` (g++ against torch + libgnn_spmm.so), and the
measurement probe scripts/bin/gather_shape (bench.py's access-shape ceiling).
No JIT cache: the .so files live next to the package so they travel with the repository
snapshot to the GPU box."""
from __future__ import annotations

import hashlib
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
SRCS = [os.path.join(HERE, "csrc", f) for f in ("spmm.hip", "sage.hip", "gemm.hip", "optim.hip", "head.hip", "extract.hip", "step.hip", "colcount.hip", "stage.hip")]
HDRS = [os.path.join(REPO, "include", f) for f in ("gnn_spmm.h", "gnn_layers.h", "gnn_optim.h", "gnn_extract.h", "gnn_step.h", "gnn_stage.h")] + [
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
           f"-I{os.path.join(REPO, 'include')}", f'-DGNN_BUILD_ID="{bid}"', "-o", OUT + ".tmp"] + SRCS + ["-lrocblas"]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(OUT + ".tmp", OUT)
    with open(stamp, "w") as f:
        f.write(bid)
    return OUT


SAMPLER_SRCS = [os.path.join(HERE, "csrc", f) for f in ("sampler.cpp", "loader.cpp")]
SAMPLER_HDRS = [os.path.join(REPO, "include", "gnn_sampler.h"), os.path.join(HERE, "csrc", "sampler_internal.h")]
SAMPLER_OUT = os.path.join(HERE, "libgnn_sampler.so")


def build_sampler(force: bool = False, verbose: bool = False) -> str:
    h = hashlib.sha1()
    for p in SAMPLER_SRCS + SAMPLER_HDRS:
        with open(p, "rb") as f:
            h.update(f.read())
    bid = h.hexdigest()[:12]
    stamp = SAMPLER_OUT + ".buildid"
    if not force and os.path.exists(SAMPLER_OUT) and os.path.exists(stamp):
        with open(stamp) as f:
            if f.read().strip() == bid:
                return SAMPLER_OUT
    # x86-64-v2 (SSE4.2 + POPCNT), not -march=native: the GPU box's host CPU may differ
    cmd = [os.environ.get("CXX", "g++"), "-O3", "-march=x86-64-v2", "-std=c++17", "-fPIC", "-shared", "-Wall",
           f"-I{os.path.join(REPO, 'include')}", "-pthread", "-o", SAMPLER_OUT + ".tmp"] + SAMPLER_SRCS + ["-ldl"]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(SAMPLER_OUT + ".tmp", SAMPLER_OUT)
    with open(stamp, "w") as f:
        f.write(bid)
    return SAMPLER_OUT


EXT_SRC = os.path.join(HERE, "csrc", "spmm_ext.cpp")


def ext_path() -> str:
    """The reference's native module name `spmm`, built next to the repository root so that
    `import spmm` (custom_sparse_ops.py:8's load(name='spmm', ...)) finds it."""
    import sysconfig

    return os.path.join(REPO, "spmm" + sysconfig.get_config_var("EXT_SUFFIX"))


def build_torch_ext(force: bool = False, verbose: bool = False) -> str:
    """The PyTorch-ROCm extension (gnn_amd/csrc/spmm_ext.cpp): pybind module `spmm` + the
    torch.ops.gnn operators, host C++ linked against torch and libgnn_spmm.so (built first)."""
    import sysconfig

    import torch
    import torch.utils.cpp_extension as ce

    build_library(verbose=verbose)
    out = ext_path()
    h = hashlib.sha1()
    for p in (EXT_SRC, os.path.join(REPO, "include", "gnn_spmm.h")):
        with open(p, "rb") as f:
            h.update(f.read())
    h.update(torch.__version__.encode())
    bid = h.hexdigest()[:12]
    stamp = out + ".buildid"
    if not force and os.path.exists(out) and os.path.exists(stamp):
        with open(stamp) as f:
            if f.read().strip() == bid:
                return out
    incs = ce.include_paths(device_type="cuda") + [sysconfig.get_paths()["include"], os.path.join(REPO, "include")]
    libdirs = ce.library_paths(device_type="cuda")
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    cmd = [os.environ.get("CXX", "g++"), "-O2", "-std=c++17", "-fPIC", "-shared", "-Wall", "-Wno-unused-function",
           "-D__HIP_PLATFORM_AMD__=1", "-DUSE_ROCM=1", f"-D_GLIBCXX_USE_CXX11_ABI={abi}",
           "-DTORCH_EXTENSION_NAME=spmm", "-DTORCH_API_INCLUDE_EXTENSION_H"]
    cmd += [f"-I{d}" for d in incs] + [EXT_SRC, "-o", out + ".tmp"]
    cmd += [f"-L{d}" for d in libdirs] + [f"-L{HERE}", "-lgnn_spmm", "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu",
                                           "-ltorch_hip", "-ltorch_python", "-lamdhip64"]
    cmd += [f"-Wl,-rpath,{libdirs[0]}", "-Wl,-rpath,$ORIGIN/gnn_amd"]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(out + ".tmp", out)
    with open(stamp, "w") as f:
        f.write(bid)
    return out


PROBE_SRC = os.path.join(REPO, "scripts", "gather_shape.hip")
PROBE_OUT = os.path.join(REPO, "scripts", "bin", "gather_shape")


def build_probe(force: bool = False, verbose: bool = False) -> str:
    """The access-shape microbenchmark bench.py runs for its live gather ceiling (a stand-alone
    HIP program: the aggregation's load stream with nothing else in it)."""
    with open(PROBE_SRC, "rb") as f:
        bid = hashlib.sha1(f.read()).hexdigest()[:12]
    stamp = PROBE_OUT + ".buildid"
    if not force and os.path.exists(PROBE_OUT) and os.path.exists(stamp):
        with open(stamp) as f:
            if f.read().strip() == bid:
                return PROBE_OUT
    os.makedirs(os.path.dirname(PROBE_OUT), exist_ok=True)
    cmd = [os.environ.get("HIPCC", "/opt/rocm/bin/hipcc"), f"--offload-arch={ARCH}", "-O3", "-std=c++17", PROBE_SRC,
           "-o", PROBE_OUT + ".tmp"]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(PROBE_OUT + ".tmp", PROBE_OUT)
    with open(stamp, "w") as f:
        f.write(bid)
    return PROBE_OUT


if __name__ == "__main__":
    print(build_library(force=True, verbose=True))
    print(build_sampler(force=True, verbose=True))
    print(build_torch_ext(force=True, verbose=True))
    print(build_probe(force=True, verbose=True))
