"""GraphSAGE / GCN encoders and the GNN head — the callers of the aggregation operator.

Restates models.py:1-97 of the reference module-for-module (same parameter creation order,
so a seeded torch RNG yields the same initial weights). The aggregation is
``custom_sparse_ops.spmm(adj, x)`` (models.py:18,60); everything else is dense torch work
(rocBLAS/hipBLASLt GEMMs, elementwise) and is not part of the hand-written HIP path.

``spmm_fn`` lets the CPU baseline (oracle/) run the same modules with torch.sparse.mm.
``fused=True`` (GPU training) runs each layer's elementwise tail — ELU, row standardise,
scale/offset and the following dropout — as one HIP kernel (gnn_amd.fused.sage_norm)
instead of ~15 torch kernels; the math is the same (tests/test_fused_gpu.py).
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import custom_sparse_ops


def _default_spmm(adj, x):
    return custom_sparse_ops.spmm(adj, x)


class GraphSageConvolution(nn.Module):
    """models.py:6-25: cat[linearB(x[self]), linearW(A·x)] -> ELU -> row standardise."""

    def __init__(self, n_in, n_out, order, bias=True, spmm_fn=None):
        super().__init__()
        self.n_in = n_in
        self.n_out = n_out
        self.linearW = nn.Linear(n_in, n_out)
        self.linearB = nn.Linear(n_in, n_out)
        self.offset = nn.Parameter(torch.zeros((1 + order) * n_out))
        self.scale = nn.Parameter(torch.ones((1 + order) * n_out))
        self.order = order
        self.spmm_fn = spmm_fn or _default_spmm

    def forward(self, x, adj, sampled_nodes):
        if self.order > 0:
            feat = self.spmm_fn(adj, x)
            feat = torch.cat([self.linearB(x[sampled_nodes]), self.linearW(feat)], 1)
        else:
            feat = self.linearW(x)
        out = F.elu(feat)
        mean = out.mean(dim=1).view(out.shape[0], 1)
        var = out.var(dim=1, unbiased=False).view(out.shape[0], 1) + 1e-9
        return (out - mean) * self.scale * torch.rsqrt(var) + self.offset

    def forward_fused(self, x, adj, sampled_nodes, p, training):
        from .fused import index_rows, linear_pair, sage_aggregate, sage_norm

        bB, bW = self.linearB.bias, self.linearW.bias
        if self.order > 0:
            if self.spmm_fn is _default_spmm:
                feat, xs = sage_aggregate(adj, x, sampled_nodes)
            else:
                feat, xs = self.spmm_fn(adj, x), index_rows(x, sampled_nodes)
            hB, hW = linear_pair([xs, feat], [self.linearB.weight, self.linearW.weight])
            return sage_norm(hB, hW, self.scale, self.offset, p, training, bB, bW)
        (hW,) = linear_pair([x], [self.linearW.weight])
        return sage_norm(None, hW, self.scale, self.offset, p, training, None, bW)


class GraphSage(nn.Module):
    """models.py:27-44."""

    def __init__(self, nfeat, nhid, orders, dropout, spmm_fn=None, fused=False):
        super().__init__()
        layers = len(orders)
        self.fused = fused
        self.nhid = (1 + orders[-1]) * nhid
        self.gcs = nn.ModuleList()
        self.gcs.append(GraphSageConvolution(nfeat, nhid, orders[0], spmm_fn=spmm_fn))
        self.dropout = nn.Dropout(dropout)
        for i in range(layers - 1):
            self.gcs.append(GraphSageConvolution((1 + orders[i]) * nhid, nhid, orders[i + 1], spmm_fn=spmm_fn))

    def forward(self, x, adjs, sampled_nodes):
        for idx in range(len(self.gcs)):
            if self.fused:
                x = self.gcs[idx].forward_fused(x, adjs[idx], sampled_nodes[idx], self.dropout.p, self.training)
            else:
                x = self.dropout(self.gcs[idx](x, adjs[idx], sampled_nodes[idx]))
        return x


class GraphConvolution(nn.Module):
    """models.py:48-64: linear(A·x) -> ELU -> row standardise."""

    def __init__(self, n_in, n_out, order, bias=True, spmm_fn=None):
        super().__init__()
        self.n_in = n_in
        self.n_out = n_out
        self.linear = nn.Linear(n_in, n_out)
        self.offset = nn.Parameter(torch.zeros(n_out))
        self.scale = nn.Parameter(torch.ones(n_out))
        self.order = order
        self.spmm_fn = spmm_fn or _default_spmm

    def forward(self, x, adj):
        feat = x
        if self.order > 0:
            feat = self.spmm_fn(adj, feat)
        out = F.elu(self.linear(feat))
        mean = out.mean(dim=1).view(out.shape[0], 1)
        var = out.var(dim=1, unbiased=False).view(out.shape[0], 1) + 1e-9
        return (out - mean) * self.scale * torch.rsqrt(var) + self.offset

    def forward_fused(self, x, adj, p, training):
        from .fused import linear_pair, sage_norm

        feat = self.spmm_fn(adj, x) if self.order > 0 else x
        (h,) = linear_pair([feat], [self.linear.weight])
        return sage_norm(None, h, self.scale, self.offset, p, training, None, self.linear.bias)


class GCN(nn.Module):
    """models.py:67-83."""

    def __init__(self, nfeat, nhid, orders, dropout, spmm_fn=None, fused=False):
        super().__init__()
        layers = len(orders)
        self.fused = fused
        self.nhid = nhid
        self.gcs = nn.ModuleList()
        self.gcs.append(GraphConvolution(nfeat, nhid, orders[0], spmm_fn=spmm_fn))
        self.dropout = nn.Dropout(dropout)
        for i in range(layers - 1):
            self.gcs.append(GraphConvolution(nhid, nhid, orders[i + 1], spmm_fn=spmm_fn))

    def forward(self, x, adjs, sampled_nodes):
        for idx in range(len(self.gcs)):
            if self.fused:
                x = self.gcs[idx].forward_fused(x, adjs[idx], self.dropout.p, self.training)
            else:
                x = self.dropout(self.gcs[idx](x, adjs[idx]))
        return x


class GNN(nn.Module):
    """models.py:86-97: encoder -> L2 normalise -> dropout -> linear."""

    def __init__(self, encoder, num_classes, dropout, inp):
        super().__init__()
        self.encoder = encoder
        self.dropout = nn.Dropout(dropout)
        self.linear = nn.Linear(self.encoder.nhid, num_classes)

    def forward(self, feat, adjs, sampled_nodes):
        x = self.encoder(feat, adjs, sampled_nodes)
        x = F.normalize(x, p=2, dim=1)
        x = self.dropout(x)
        x = self.linear(x)
        return x

    def forward_loss(self, feat, adjs, sampled_nodes, labels, sigmoid_loss: bool = True):
        """(loss, logits) = (utils.loss(forward(...), labels), forward(...)). With the fused
        GPU encoder and the sigmoid loss, the head (normalize, dropout, linear) and the BCE run
        as one HIP pass each way (gnn_amd.fused.head_bce_loss); otherwise as the modules above."""
        x = self.encoder(feat, adjs, sampled_nodes)
        if sigmoid_loss and getattr(self.encoder, "fused", False) and x.is_cuda:
            from .fused import head_bce_loss, head_supported

            if head_supported(x, self.linear.weight, labels):
                return head_bce_loss(x, self.linear.weight, self.linear.bias, labels, self.dropout.p,
                                     self.training)
        out = self.linear(self.dropout(F.normalize(x, p=2, dim=1)))
        return loss(out, labels, sigmoid_loss, x.device), out


def loss(preds, labels, sigmoid_loss, device):
    """utils.py:129-140: BCE-with-logits (or CE) weighted by 1/batch, summed."""
    norm_loss = torch.ones(preds.shape[0], device=device)
    norm_loss /= preds.shape[0]
    if sigmoid_loss:
        norm_loss = norm_loss.unsqueeze(1)
        return torch.nn.BCEWithLogitsLoss(weight=norm_loss, reduction="sum")(preds, labels)
    _ls = torch.nn.CrossEntropyLoss(reduction="none")(preds, labels)
    return (norm_loss * _ls).sum()


def build_model(name: str, nfeat: int, nhid: int, orders, num_classes: int, dropout: float = 0.1, spmm_fn=None,
                fused: bool = False):
    """main.py:91-97."""
    if name == "graphsage":
        enc = GraphSage(nfeat=nfeat, nhid=nhid, orders=orders, dropout=dropout, spmm_fn=spmm_fn, fused=fused)
    elif name == "gcn":
        enc = GCN(nfeat=nfeat, nhid=nhid, orders=orders, dropout=dropout, spmm_fn=spmm_fn, fused=fused)
    else:
        raise ValueError(f"unknown model {name!r} (graphsage/gcn)")
    return GNN(encoder=enc, num_classes=num_classes, dropout=dropout, inp=nfeat)
