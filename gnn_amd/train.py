"""Data-parallel training step (main.py:122-170), one process per GPU.

Reference: per-rank threads in one process; grads flattened with torch.cat, published in a
shared list, ``threading.Barrier``, summed with P2P ``.to(device)`` copies (main.py:149-168);
per-rank clip_grad_norm_(5) BEFORE the sum and no averaging (main.py:146,159).

Here: one process per GPU with torch.distributed (backend "nccl" = RCCL over xGMI). The
gradients live in ONE flat fp32 buffer from the start (every ``param.grad`` is a view of it),
so the exchange is a single in-place ``all_reduce(SUM)`` — no cat/split copies — after the
same per-rank clip. Initial weights are broadcast from rank 0 (the reference never syncs
them: quirk F in SURVEY.md Appendix B).
"""
from __future__ import annotations

from typing import Optional

import torch

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
        n = sum(p.numel() for p in self.params)
        self.flat_grad = torch.zeros(n, dtype=torch.float32, device=self.device)
        off = 0
        for p in self.params:
            p.grad = self.flat_grad[off: off + p.numel()].view_as(p)
            off += p.numel()
        self.optimizer = torch.optim.Adam(self.params, lr=lr)
        self.world = 1
        if group is not None or (torch.distributed.is_available() and torch.distributed.is_initialized()):
            self.world = torch.distributed.get_world_size(group)
        if self.world > 1:
            self.broadcast_parameters()

    @property
    def num_params(self) -> int:
        return self.flat_grad.numel()

    def broadcast_parameters(self):
        flat = torch.cat([p.detach().reshape(-1) for p in self.params])
        torch.distributed.broadcast(flat, src=0, group=self.group)
        off = 0
        with torch.no_grad():
            for p in self.params:
                p.copy_(flat[off: off + p.numel()].view_as(p))
                off += p.numel()

    def step(self, x0, adjs, sampled_nodes, labels, exchange: bool = True) -> torch.Tensor:
        self.flat_grad.zero_()
        self.model.train()
        out = self.model(x0, adjs, sampled_nodes)
        loss = loss_fn(out, labels, self.sigmoid_loss, self.device)
        loss.backward()
        torch.nn.utils.clip_grad_norm_(self.params, self.clip)
        if exchange and self.world > 1:
            torch.distributed.all_reduce(self.flat_grad, op=torch.distributed.ReduceOp.SUM, group=self.group)
        self.optimizer.step()
        return loss.detach()


def init_distributed(backend: Optional[str] = None):
    """Initialise torch.distributed from torchrun's environment; returns (rank, world, local_rank)."""
    import os

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1 and not torch.distributed.is_initialized():
        be = backend or ("nccl" if torch.cuda.is_available() else "gloo")
        if be == "nccl":
            torch.cuda.set_device(local)
            torch.distributed.init_process_group(be, device_id=torch.device("cuda", local))
        else:
            torch.distributed.init_process_group(be)
    return rank, world, local
