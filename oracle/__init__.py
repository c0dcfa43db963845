"""TEST INFRASTRUCTURE — the CPU oracle of the SpMM aggregation path.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this
package, and only as the checker / CPU baseline. The gnn_amd product never imports it.

Contents:
  * oracle_spmm.c (+ Makefile -> liboracle.so): C restatement of the operand builder
    (cuda_spmm.cu:795-802 + coalesce), CSR SpMM (fp32 fmaf chain and fp64), the canonical
    transpose (custom_sparse_ops.py:34) and the feature-row gather (main.py:129-134).
  * cpu_reference.py: the reference's CPU path — torch.sparse.mm autograd op
    (custom_sparse_ops.py:25,36) driving the GraphSAGE/GCN modules — for the training-step
    parity tests and the CPU baseline.

Parity pinning: golden vectors captured from the reference's own Python in this container
(tests/golden/make_golden.py) — LADIES sampler outputs, placement maps, torch.sparse.mm
forward/backward outputs and a seeded GraphSAGE training step.
"""
from .oracle import *  # noqa: F401,F403
