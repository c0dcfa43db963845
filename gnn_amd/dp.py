"""Data-parallel gradient exchange, bucketed and overlapped with the backward.

Reference semantics (main.py:146-170): every rank clips its OWN gradient with
clip_grad_norm_(5) (factor c_r = min(1, 5 / (||g_r|| + 1e-6))), the clipped gradients are
SUMMED over ranks (no averaging), then Adam. The reference exchanges flattened gradients by
P2P copies after the whole backward.

The clip factor of a rank is known only when its whole backward has finished, so the sum
Σ_r c_r g_r cannot be all-reduced bucket by bucket as the buckets become ready. It is split
instead into the two halves of a ring all-reduce, with the reduction moved after the clip:
  1. per bucket, as soon as the step executor records that the bucket's gradients are final
     (GNN_SH_GRAD_EVENTS, include/gnn_step.h): an all-to-all on a side stream sends shard j of
     this rank's UNSCALED bucket to rank j — while the layers below are still in their
     backward on the compute stream (RCCL over xGMI beside the compute kernels). The LAST
     bucket (layer 0, final when the backward ends) travels after the backward, straight from
     the flat gradient, and the ranks' clip factors by one all-gather of W floats;
  2. per bucket: rank r sums its shard over the ranks in rank order, Σ_j c_j * g_j[shard r]
     (each product rounded in fp32 as the reference's clip-then-add);
  3. ONE all-to-all returns every rank's summed shards of every bucket (an all-gather with
     unequal shards), and one copy puts them into the flat gradient, which Adam reads.
So three collectives follow the backward, two of them tiny or small (the flat path: one
all-reduce of the whole gradient), and the reduce-scatter half of the traffic of the other
buckets is off the critical path.
Buckets = backward stages: [head + top layer], [layer L-2], ..., [layer 0].
"""
from __future__ import annotations

from typing import List

import torch


class BucketedExchange:
    def __init__(self, executor, optimizer, group=None):
        import torch.distributed as dist

        self.dist = dist
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.ex = executor
        self.opt = optimizer
        flat = executor.flat_grad
        dev = self.device = flat.device
        offs, o = [], 0
        for p in executor.params:
            offs.append((o, o + p.numel()))
            o += p.numel()
        stages = executor.grad_stages()
        # the head joins the top layer's bucket (ready right after it); a bucket must be one
        # contiguous range of the flat gradient
        groups = [stages[0] + stages[1]] + stages[2:]
        self.buckets = []
        for idx in groups:
            lo = min(offs[i][0] for i in idx)
            hi = max(offs[i][1] for i in idx)
            if sum(offs[i][1] - offs[i][0] for i in idx) != hi - lo:
                raise ValueError("BucketedExchange: a backward stage's gradients are not contiguous in the flat buffer")
            self.buckets.append((lo, hi))
        # the buckets must tile the whole flat gradient: finish() writes back only the bucket
        # positions, so an element outside every bucket would keep this rank's unclipped local
        # gradient and the ranks would silently diverge (the Trainer then uses the flat exchange)
        cover = sorted(self.buckets)
        if (not cover or cover[0][0] != 0 or cover[-1][1] != flat.numel()
                or any(a[1] != b[0] for a, b in zip(cover, cover[1:]))):
            raise ValueError(f"BucketedExchange: buckets {cover} do not tile the flat gradient [0, {flat.numel()})")
        W, r = self.world, self.rank
        # shard j of bucket b: [lo + off_b[j], lo + off_b[j] + sz_b[j])
        self.sz = []
        for lo, hi in self.buckets:
            n = hi - lo
            self.sz.append([n // W + (1 if j < n % W else 0) for j in range(W)])
        self.off = [[sum(s[:j]) for j in range(W)] for s in self.sz]
        self.recv = [torch.empty(W * s[r], dtype=torch.float32, device=dev) for s in self.sz]
        self.fac = torch.empty(W, dtype=torch.float32, device=dev)  # every rank's clip factor
        # the gather phase: this rank's summed shards of every bucket, one copy per destination
        self.mine = sum(s[r] for s in self.sz)
        self.red = torch.empty(self.mine, dtype=torch.float32, device=dev)
        self.gsend = torch.empty(W * self.mine, dtype=torch.float32, device=dev)
        self.gsizes = [sum(s[j] for s in self.sz) for j in range(W)]
        self.grecv = torch.empty(sum(self.gsizes), dtype=torch.float32, device=dev)
        # flat position of every element of grecv (source j's shards of buckets 0..B-1)
        pos = []
        for j in range(W):
            for (lo, _), s, of in zip(self.buckets, self.sz, self.off):
                pos.append(torch.arange(lo + of[j], lo + of[j] + s[j], dtype=torch.int64))
        self.gpos = torch.cat(pos).to(dev)
        self.stream = torch.cuda.Stream(device=dev)
        nl = len(stages) - 1
        # events per stage, in the executor's order: [head, layer 0, ..., layer L-1]
        self.events = [torch.cuda.Event() for _ in range(1 + nl)]
        # the event that makes bucket b ready: [top layer, L-2, ..., 0]
        self.ready = [self.events[1 + (nl - 1 - b)] for b in range(len(self.buckets))]
        self.works: List = []

    def issue(self):
        """After the executor call (its events recorded in order): start the all-to-all of every
        bucket but the last on the side stream, each waiting only for its own gradients."""
        flat = self.ex.flat_grad
        self.works = []
        for b in range(len(self.buckets) - 1):
            lo, hi = self.buckets[b]
            self.stream.wait_event(self.ready[b])
            with torch.cuda.stream(self.stream):
                w = self.dist.all_to_all_single(self.recv[b], flat[lo:hi], output_split_sizes=[self.sz[b][self.rank]] *
                                                self.world, input_split_sizes=self.sz[b], group=self.group,
                                                async_op=True)
            self.works.append(w)

    def finish(self):
        """This rank's clip factor, the last bucket + the factors, the weighted shard sums, the
        gather back into the flat gradient: the parameters' .grad then hold Σ_r c_r g_r."""
        dist, W, r, flat = self.dist, self.world, self.rank, self.ex.flat_grad
        from . import _lib

        if self.opt.max_norm > 0:
            self.opt._clip_scale([p.grad for p in self.opt.params], _lib.stream_of(self.device))
            c = self.opt.scale
        else:
            c = torch.ones(1, dtype=torch.float32, device=self.device)
        dist.all_gather_into_tensor(self.fac, c.view(1), group=self.group)
        fac = self.fac.view(W, 1)  # c_j of every rank
        lo, hi = self.buckets[-1]
        dist.all_to_all_single(self.recv[-1], flat[lo:hi], output_split_sizes=[self.sz[-1][r]] * W,
                               input_split_sizes=self.sz[-1], group=self.group)
        for w in self.works:
            w.wait()  # the current stream waits for the side stream's all-to-alls
        torch.cuda.current_stream(self.device).wait_stream(self.stream)
        o = 0
        for b in range(len(self.buckets)):
            q = self.sz[b][r]
            torch.sum(self.recv[b].view(W, q) * fac, dim=0, out=self.red[o:o + q])
            o += q
        self.gsend.view(W, self.mine).copy_(self.red.view(1, self.mine).expand(W, self.mine))
        dist.all_to_all_single(self.grecv, self.gsend, output_split_sizes=self.gsizes,
                               input_split_sizes=[self.mine] * W, group=self.group)
        flat.index_copy_(0, self.gpos, self.grecv)
        self.works = []
