"""Policies with the reference's constructors and call contracts (reference: policy.py:14-129).

``ForwardPolicy`` restates the reference's GATv2 -> GATv2 -> mean-pool -> fc network
(policy.py:14-73) in plain torch ops (no torch_geometric).  It is the logit producer of
the rollout, NOT part of the HIP hot path yet, and its numerics
are "parity unpinned": the reference's PyG version is unpinned and PyG is not installed,
so no golden vectors exist for it.  GATv2 semantics restated: per head
e_ij = att . leaky_relu(W_l x_j + W_r x_i + W_e a_ij, 0.2), softmax over the incoming
edges of i, out_i = sum_j alpha_ij W_l x_j (+ bias); self-loops replaced by loops whose
edge attribute is the mean of the node's incoming attributes (fill_value="mean").
``BackwardPolicy`` is the reference's LSTM policy (policy.py:75-129), batched.
"""
from __future__ import annotations

from typing import Tuple

import torch
import torch.nn.functional as F
from torch import Tensor, nn


class GATv2Layer(nn.Module):
    def __init__(self, in_channels: int, out_channels: int, heads: int = 1, edge_dim: int = 1,
                 negative_slope: float = 0.2):
        super().__init__()
        self.h, self.c, self.slope = heads, out_channels, negative_slope
        self.lin_l = nn.Linear(in_channels, heads * out_channels)
        self.lin_r = nn.Linear(in_channels, heads * out_channels)
        self.lin_edge = nn.Linear(edge_dim, heads * out_channels, bias=False)
        self.att = nn.Parameter(torch.empty(1, heads, out_channels))
        self.bias = nn.Parameter(torch.zeros(heads * out_channels))
        for lin in (self.lin_l, self.lin_r, self.lin_edge):
            nn.init.xavier_uniform_(lin.weight)
            if lin.bias is not None:
                nn.init.zeros_(lin.bias)
        nn.init.xavier_uniform_(self.att)

    def forward(self, x: Tensor, edge_index: Tensor, edge_attr: Tensor) -> Tensor:
        n = x.size(0)
        src, dst = edge_index[0], edge_index[1]
        ea = edge_attr.reshape(-1, 1).to(x.dtype)
        keep = src != dst
        src, dst, ea = src[keep], dst[keep], ea[keep]
        deg = torch.zeros(n, device=x.device, dtype=x.dtype).index_add_(0, dst, torch.ones_like(dst, dtype=x.dtype))
        loop_attr = torch.zeros(n, 1, device=x.device, dtype=x.dtype).index_add_(0, dst, ea) / deg.clamp(min=1).view(-1, 1)
        ar = torch.arange(n, device=x.device)
        src, dst, ea = torch.cat([src, ar]), torch.cat([dst, ar]), torch.cat([ea, loop_attr])
        xl = self.lin_l(x).view(n, self.h, self.c)
        xr = self.lin_r(x).view(n, self.h, self.c)
        e = F.leaky_relu(xl[src] + xr[dst] + self.lin_edge(ea).view(-1, self.h, self.c), self.slope)
        score = (e * self.att).sum(-1)  # [E', H]
        smax = torch.full((n, self.h), float("-inf"), device=x.device, dtype=score.dtype)
        smax = smax.scatter_reduce(0, dst.view(-1, 1).expand_as(score), score, reduce="amax", include_self=True)
        ex = torch.exp(score - smax[dst])
        den = torch.zeros(n, self.h, device=x.device, dtype=ex.dtype).index_add_(0, dst, ex)
        alpha = ex / den[dst]
        out = torch.zeros(n, self.h, self.c, device=x.device, dtype=x.dtype)
        out = out.index_add_(0, dst, xl[src] * alpha.unsqueeze(-1))
        return out.reshape(n, self.h * self.c) + self.bias


class BasePolicy(nn.Module):
    def __init__(self, node_features: int, hidden_dim: int):
        super().__init__()
        self.node_features = node_features
        self.hid = hidden_dim
        self.in_head = 4
        self.out_head = 1
        # the reference uses a lazy (-1) input width; the state graph's x is ones(2N, 1)
        self.gat1 = GATv2Layer(node_features if node_features > 0 else 1, self.hid, heads=self.in_head)


class ForwardPolicy(BasePolicy):
    def __init__(self, node_features: int, hidden_dim: int, max_num_actions: int):
        super().__init__(node_features, hidden_dim)
        self.gat2 = GATv2Layer(self.hid * self.in_head, self.hid, heads=self.out_head)
        self.fc = nn.Linear(self.hid, max_num_actions)
        self.alpha = nn.Parameter(torch.tensor(0.0))

    def logits(self, data) -> Tuple[Tensor, Tensor]:
        """Unmasked logits [1, E+1] and sigmoid(alpha): everything of forward() but the mask."""
        x, edge_index, edge_attr = data.x, data.edge_index, data.edge_attr
        num_actions = edge_attr.size(0) + 1
        x = torch.relu(self.gat1(x, edge_index, edge_attr))
        x = torch.relu(self.gat2(x, edge_index, edge_attr))
        x = x.mean(dim=0, keepdim=True)
        return self.fc(x)[:, :num_actions], torch.sigmoid(self.alpha)

    def forward(self, data, actions: Tensor) -> Tuple[Tensor, Tensor]:
        x, a = self.logits(data)
        if actions.numel() > 0:
            blocked = torch.zeros_like(x, dtype=torch.bool)
            blocked[:, actions.to(x.device)] = True
            x = x.masked_fill(blocked, float("-inf"))
        return torch.softmax(x, dim=1), a


class BackwardPolicy(nn.Module):
    """LSTM over each trajectory's action ids; softmax over its first n_valid fc outputs,
    padded with 1.0 to the trajectory length (policy.py:87-129), all samples in one call."""

    def __init__(self, input_dim: int, hidden_dim: int, max_num_actions: int):
        super().__init__()
        self.hidden_dim = hidden_dim
        self.max_num_actions = max_num_actions
        self.lstm = nn.LSTM(input_dim, hidden_dim, batch_first=True)
        self.fc = nn.Linear(hidden_dim, max_num_actions)

    def forward(self, trajectories: Tensor) -> Tensor:
        B, T = trajectories.shape
        n = (trajectories != -1).sum(1)
        packed = nn.utils.rnn.pack_padded_sequence(trajectories.float().unsqueeze(-1), n.cpu(), batch_first=True,
                                                   enforce_sorted=False)
        _, (h, _) = self.lstm(packed)
        out = self.fc(h[-1])
        width = min(T, out.shape[1])
        pos = torch.arange(width, device=out.device)
        valid = pos.view(1, -1) < n.view(-1, 1)
        p = torch.softmax(out[:, :width].masked_fill(~valid, float("-inf")), dim=1)
        res = torch.ones(B, T, device=out.device, dtype=out.dtype)
        res[:, :width] = torch.where(valid, p, torch.ones((), device=out.device, dtype=out.dtype))
        return res.unsqueeze(1)
