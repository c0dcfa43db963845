"""Data-parallel training step (main.py:122-170), one process per GPU.

Reference: per-rank threads in one process; grads flattened with torch.cat, published in a
shared list, ``threading.Barrier``, summed with P2P ``.to(device)`` copies (main.py:149-168);
per-rank clip_grad_norm_(5) BEFORE the sum and no averaging (main.py:146,159).

Here: one process per GPU with torch.distributed (backend "nccl" = RCCL over xGMI). By default
the per-rank clip writes the clipped gradients straight into one flat fp32 buffer (one kernel,
gnn_amd.optim), summed with ONE in-place ``all_reduce(SUM)``, and Adam reads them as views of
that buffer; at N = 1 the clip factor is applied inside the Adam launch. With the native step
executor and GNN_DP_BUCKETS=1 the exchange is bucketed per backward stage and overlapped with
the backward instead (gnn_amd.dp: all-to-all of unscaled shards as each stage finishes, then
the ranks' clip factors, the weighted shard sums and one gather — the same
per-rank-clip-then-sum, bit-identical at world 2); bench.py times both at N > 1. (On the CPU
— the gloo tests — the same semantics run through torch's clip_grad_norm_ and Adam.)
Gradients are reset to None each step, so autograd hands its freshly computed tensors over
instead of accumulating into old ones. Initial weights are broadcast from rank 0 (the
reference never syncs them: SURVEY.md Appendix B, F).
"""
from __future__ import annotations

import os
from typing import Optional

import torch
from torch._utils import _flatten_dense_tensors, _unflatten_dense_tensors

from .models import loss as loss_fn


class Trainer:
    def __init__(self, model: torch.nn.Module, lr: float, device, group=None, sigmoid_loss: bool = True,
                 clip: float = 5.0):
        self.model = model
        self.device = torch.device(device)
        self.sigmoid_loss = sigmoid_loss
        self.clip = clip
        self.group = group
        self.params = [p for p in model.parameters() if p.requires_grad]
        # The reference's default Adam (main.py:102) and clip_grad_norm_(5) (main.py:146).
        self.native = self.device.type == "cuda"
        if self.native:
            # The layer GEMMs (15k x 602..1024 x 512, fp32): rocBLAS ("cublas" on ROCm builds)
            # measured faster than hipBLASLt on MI355X (317 vs 294 mini-batches/s, same box).
            torch.backends.cuda.preferred_blas_library("cublas")
            # clip + Adam in two HIP launches (gnn_amd.optim, include/gnn_optim.h)
            from .optim import ClipAdam

            self.optimizer = ClipAdam(self.params, lr=lr, max_norm=clip)
        else:
            self.optimizer = torch.optim.Adam(self.params, lr=lr)
        # the whole forward + backward as one native call when the model allows it
        # (gnn_amd.executor, include/gnn_step.h); GNN_NATIVE_STEP=0 keeps the autograd path
        self.executor = None
        if self.native:
            from . import executor as ex

            if ex.enabled():
                try:
                    self.executor = ex.NativeStep(model)
                except ValueError:
                    self.executor = None
        self.world = 1
        if torch.distributed.is_available() and torch.distributed.is_initialized():
            self.world = torch.distributed.get_world_size(group)
        # the data-parallel branch of step() (clip into the flat buffer, all-reduce, Adam on the
        # sum): every N > 1 run; tests/test_rccl_gpu.py also drives it through a 1-rank RCCL group
        self.dp = self.world > 1
        if self.world > 1:
            self.broadcast_parameters()
        # N > 1 with the executor: the gradient exchange bucketed per backward stage and started
        # while the backward runs (gnn_amd.dp), built whenever possible; used when
        # GNN_DP_BUCKETS=1 (default: one flat all-reduce after the backward — bench.py times
        # both at N > 1, since neither is measured over RCCL / xGMI on a one-GPU box)
        self.bucketed = None
        if self.world > 1 and self.executor is not None:
            from .dp import BucketedExchange

            try:
                self.bucketed = BucketedExchange(self.executor, self.optimizer, group)
            except ValueError:
                self.bucketed = None
        self.exchange = self.bucketed if os.environ.get("GNN_DP_BUCKETS", "0") == "1" else None
        # (event, layer): recorded by the executor after that layer's forward aggregation; the
        # staging of later batches waits on it (staging.Stager.gate, set by the caller)
        self.stage_gate = None

    @property
    def num_params(self) -> int:
        return sum(p.numel() for p in self.params)

    def broadcast_parameters(self):
        flat = _flatten_dense_tensors([p.detach() for p in self.params])
        torch.distributed.broadcast(flat, src=0, group=self.group)
        with torch.no_grad():
            for p, v in zip(self.params, _unflatten_dense_tensors(flat, self.params)):
                p.copy_(v)

    def param_digest(self) -> str:
        """sha256 (first 16 hex digits) over every parameter's bytes, in parameter order."""
        import hashlib

        h = hashlib.sha256()
        for p in self.params:
            h.update(p.detach().contiguous().cpu().numpy().tobytes())
        return h.hexdigest()[:16]

    def check_ranks_agree(self) -> dict:
        """Cross-rank consistency of the data-parallel step (main.py:146-170): after the summed
        gradient and the same Adam update on every rank, all ranks must hold bit-identical
        parameters. Collective (every rank of the group). Returns {"identical", "digests"}."""
        d = self.param_digest()
        dist = torch.distributed
        if not (dist.is_available() and dist.is_initialized()):
            return {"identical": True, "digests": [d]}
        digests = [None] * dist.get_world_size(self.group)
        torch.distributed.all_gather_object(digests, d, group=self.group)
        return {"identical": all(x == digests[0] for x in digests), "digests": digests}

    def allreduce_grads(self) -> Optional[torch.Tensor]:
        """Σ over ranks of the (already clipped) gradients, in one flat buffer."""
        if not self.dp:
            return None
        grads = [p.grad for p in self.params]
        flat = _flatten_dense_tensors(grads)
        torch.distributed.all_reduce(flat, op=torch.distributed.ReduceOp.SUM, group=self.group)
        for p, g in zip(self.params, _unflatten_dense_tensors(flat, grads)):
            p.grad = g
        return flat

    def _next_batch(self, prefetch):
        """The next batch (x0, adjs, sampled_nodes, labels) for the executor's layer-0 prefetch, or
        None: data-parallel runs only (there the all-reduce leaves the compute stream idle), the
        flat exchange, not while the per-aggregation timing runs, GNN_PREFETCH_L0=0 turns it off."""
        if prefetch is None or self.executor is None or os.environ.get("GNN_PREFETCH_L0", "1") == "0":
            return None
        from . import custom_sparse_ops as cso

        if cso.timing_enabled():
            return None
        nxt = prefetch() if callable(prefetch) else prefetch
        if nxt is None or not self.executor.supports(*nxt):
            return None
        return nxt

    def step(self, x0, adjs, sampled_nodes, labels, prefetch=None) -> torch.Tensor:
        """One training step. ``prefetch``: the next batch (x0, adjs, sampled_nodes, labels), or a
        callable returning it, whose layer-0 forward aggregation a data-parallel run issues while
        this step's gradient all-reduce is in flight (gnn_amd.executor.NativeStep.prefetch; the
        next step then skips it). Results are the same with or without it."""
        if not self.model.training:  # module.train() walks every submodule: ~50 µs of host time
            self.model.train()
        if self.executor is not None and self.executor.supports(x0, adjs, sampled_nodes, labels):
            if self.exchange is not None:  # buckets leave while the lower layers' backward runs
                loss = self.executor.step(x0, adjs, sampled_nodes, labels, grad_events=self.exchange.events,
                                          stage_gate=self.stage_gate)
                self.exchange.issue()
                self.exchange.finish()  # this rank's clip, Σ_r c_r g_r into the flat gradient
                self.optimizer.step(clipped=True)
                return loss
            loss = self.executor.step(x0, adjs, sampled_nodes, labels,  # grads into the flat buffer
                                      stage_gate=self.stage_gate)
            if self.dp:
                flat = self.optimizer.clip_to_flat()
                # the all-reduce is issued first, on the collective's stream: fetching the next
                # batch may wait on the host for its staging event (GNN_EXTRACT_CHECK=step), which
                # must not hold the collective back on this rank. The next batch's layer-0
                # aggregation (no parameter in it) then fills the compute stream meanwhile, and the
                # optimizer step waits for the sum (Work.wait: a stream wait, not a host one)
                work = torch.distributed.all_reduce(flat, op=torch.distributed.ReduceOp.SUM, group=self.group,
                                                    async_op=True)
                nxt = self._next_batch(prefetch)
                if nxt is not None:
                    self.executor.prefetch(*nxt, stage_gate=self.stage_gate)
                work.wait()
                self.optimizer.step(clipped=True)
            else:
                # N = 1 takes no prefetch: issuing it with the clip + Adam kernels moved to a side
                # stream beside it measured 0.5-0.8 % slower (two cross-stream events per step
                # against ~30 us of small launches; profiles/round5/prefetch_l0/)
                self.optimizer.step()
            return loss
        for p in self.params:
            p.grad = None
        if hasattr(self.model, "forward_loss"):
            loss, _ = self.model.forward_loss(x0, adjs, sampled_nodes, labels, self.sigmoid_loss)
        else:
            out = self.model(x0, adjs, sampled_nodes)
            loss = loss_fn(out, labels, self.sigmoid_loss, self.device)
        if self.native:
            # d(loss)/d(loss) = 1 from a cached device scalar (no fill launch per step)
            one = getattr(self, "_one", None)
            if one is None or one.device != loss.device:
                one = self._one = torch.ones((), dtype=loss.dtype, device=loss.device)
            loss.backward(one)
        else:
            loss.backward()
        if self.native:
            if self.dp:
                flat = self.optimizer.clip_to_flat()  # this rank's clip, into the all-reduce buffer
                torch.distributed.all_reduce(flat, op=torch.distributed.ReduceOp.SUM, group=self.group)
                self.optimizer.step(clipped=True)
            else:
                self.optimizer.step()  # clip applied inside the Adam launch
            return loss.detach()
        torch.nn.utils.clip_grad_norm_(self.params, self.clip)
        self.allreduce_grads()
        self.optimizer.step()
        return loss.detach()


DEFAULT_TIMEOUT_S = 180.0


def collective_timeout():
    """How long any collective of this package may wait for its peers (GNN_DIST_TIMEOUT_S,
    default 180 s) before the rank fails. The reference's threads wait on a
    ``threading.Barrier`` with no timeout (main.py:158,214), and torch's defaults are 10 min
    (RCCL) and 30 min (gloo): a stalled collective must instead end the run, non-zero, well
    inside a driver's time limit, with the rank and the call in the log."""
    import datetime

    s = float(os.environ.get("GNN_DIST_TIMEOUT_S", DEFAULT_TIMEOUT_S))
    if not s > 0:
        raise ValueError(f"GNN_DIST_TIMEOUT_S must be > 0, got {s}")
    return datetime.timedelta(seconds=s)


def init_group(backend: str, rank: Optional[int] = None, world: Optional[int] = None, local: int = 0):
    """init_process_group with this package's collective timeout. RCCL ("nccl"): the watchdog's
    asynchronous error handling stays on (TORCH_NCCL_ASYNC_ERROR_HANDLING, set to 1 = abort the
    communicator and end the process unless the caller chose otherwise), so a collective that
    does not complete within the timeout takes the rank down with the watchdog's report of the
    rank, the operation and its sequence number instead of hanging; its heartbeat monitor is
    held to the timeout + 60 s. gloo: every collective raises RuntimeError after the timeout."""
    timeout = collective_timeout()
    kw = {"timeout": timeout}
    if rank is not None:
        kw.update(rank=rank, world_size=world)
    if backend == "nccl":
        os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "1")
        os.environ.setdefault("TORCH_NCCL_HEARTBEAT_TIMEOUT_SEC", str(int(timeout.total_seconds()) + 60))
        torch.distributed.init_process_group(backend, device_id=torch.device("cuda", local), **kw)
    else:
        from .staging import stdout_to_stderr

        with stdout_to_stderr():  # gloo's connection lines go to stderr, not into the bench's stdout
            torch.distributed.init_process_group(backend, **kw)


def new_gloo_group():
    """A gloo side group (host metadata, IPC handle exchange) with the same timeout."""
    from .staging import stdout_to_stderr

    with stdout_to_stderr():  # gloo prints its connection lines on stdout (bench: one JSON line)
        return torch.distributed.new_group(backend="gloo", timeout=collective_timeout())


def init_distributed(backend: Optional[str] = None):
    """Initialise torch.distributed from torchrun's environment; returns (rank, world, local_rank)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1 and not torch.distributed.is_initialized():
        be = backend or os.environ.get("GNN_DIST_BACKEND") or ("nccl" if torch.cuda.is_available() else "gloo")
        if torch.cuda.is_available():
            # one GPU per local rank (torchrun); more ranks than GPUs (a rehearsal on a smaller
            # box, gloo backend: RCCL refuses two ranks on one GPU) share them round-robin
            local = local % max(torch.cuda.device_count(), 1)
            torch.cuda.set_device(local)
        init_group(be, local=local)
    return rank, world, local
