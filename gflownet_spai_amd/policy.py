"""Policies with the reference's constructors and call contracts (reference: policy.py:14-129).

``ForwardPolicy`` is the reference's GATv2 -> GATv2 -> mean-pool -> fc network
(policy.py:14-73) without torch_geometric: its forward runs on the gfx950 kernels of
``spai_policy_logits`` (csrc/policy.hip); ``GATv2Layer`` below is the torch restatement
that holds the parameters, gives the gradients and is the fp32 test reference.  The PyG
version the reference ran is unpinned and PyG is not installed, so the GATv2 semantics
are pinned by the numpy restatement in oracle/ and by a known answer (with x = ones, as
state_to_data builds it, every node's output is W_l 1 + b_l + bias whatever the
attention weights).  GATv2 semantics restated: per head
e_ij = att . leaky_relu(W_l x_j + W_r x_i + W_e a_ij, 0.2), softmax over the incoming
edges of i, out_i = sum_j alpha_ij W_l x_j (+ bias); self-loops replaced by loops whose
edge attribute is the mean of the node's incoming attributes (fill_value="mean").
``BackwardPolicy`` is the reference's LSTM policy (policy.py:75-129), batched, with the
recurrence (forward and BPTT) on the gfx950 kernels of csrc/train.hip.
"""
from __future__ import annotations

from typing import Tuple

import torch
import torch.nn.functional as F
from torch import Tensor, nn

from . import _lib, kernels


def _small_linear(x: Tensor, weight: Tensor, bias: Tensor | None) -> Tensor:
    """nn.Linear for a small input width, as in_features broadcast multiply-adds."""
    out = weight[:, 0].unsqueeze(0) * x[:, 0:1]
    if bias is not None:
        out = out + bias
    for k in range(1, x.shape[1]):
        out = torch.addcmul(out, x[:, k:k + 1], weight[:, k].unsqueeze(0))
    return out


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
        # the three linears as broadcast multiply-adds (K = in_channels <= 16, edge_dim 1): the
        # BLAS tiles these skinny GEMMs badly (~8 ms each at C4), elementwise they are bandwidth
        xl = _small_linear(x, self.lin_l.weight, self.lin_l.bias).view(n, self.h, self.c)
        xr = _small_linear(x, self.lin_r.weight, self.lin_r.bias).view(n, self.h, self.c)
        xe = _small_linear(ea, self.lin_edge.weight, None).view(-1, self.h, self.c)
        e = F.leaky_relu(xl[src] + xr[dst] + xe, self.slope)
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


def graph_csr(x: Tensor, edge_index: Tensor, edge_attr: Tensor):
    """The state graph as the CSR by target that spai_policy_logits reads: self loops
    removed, one loop per node re-added with the mean incoming attribute (GATv2Conv
    add_self_loops(fill_value="mean")), edges grouped by target (edge_index[1]) in their
    original order.  Built once per state graph (the graph is fixed within a rollout)."""
    n = x.size(0)
    dev = x.device
    src, dst = edge_index[0].to(dev), edge_index[1].to(dev)
    ea = edge_attr.reshape(-1).to(device=dev, dtype=torch.float32)
    if src.numel() and (int(src.min()) < 0 or int(max(src.max(), dst.max())) >= n or int(dst.min()) < 0):
        raise ValueError("edge_index out of range for x")
    keep = src != dst
    src, dst, ea = src[keep], dst[keep], ea[keep]
    deg = torch.bincount(dst, minlength=n)
    loop = torch.zeros(n, dtype=torch.float32, device=dev).index_add_(0, dst, ea) / deg.clamp(min=1).float()
    ar = torch.arange(n, device=dev)
    src, dst, ea = torch.cat([src, ar]), torch.cat([dst, ar]), torch.cat([ea, loop])
    order = torch.sort(dst, stable=True).indices
    rowptr = torch.zeros(n + 1, dtype=torch.int32, device=dev)
    rowptr[1:] = torch.cumsum(torch.bincount(dst, minlength=n), 0).to(torch.int32)
    return rowptr, src[order].to(torch.int32).contiguous(), ea[order].contiguous()


def skinny_linear(h: Tensor, weight: Tensor, bias: Tensor, width: int) -> Tensor:
    """nn.Linear(h)[:, :width] for a short hidden size: the first ``width`` output columns only,
    as hid broadcast multiply-adds over [rows, width] (bandwidth-bound elementwise work, and so
    is its autograd), instead of a full [rows, max_num_actions] GEMM whose skinny shape
    (K = hid = 4) the BLAS tiles badly."""
    out = bias[:width].unsqueeze(0).expand(h.shape[0], width)
    for k in range(h.shape[1]):
        out = torch.addcmul(out, h[:, k:k + 1], weight[:width, k].unsqueeze(0))
    return out


def _pack(layer: GATv2Layer) -> Tensor:
    """Packed parameter block of one layer in the order spai_policy_logits reads (cached
    until a parameter is modified in place, e.g. by an optimizer step)."""
    ps = (layer.lin_l.weight, layer.lin_l.bias, layer.lin_r.weight, layer.lin_r.bias, layer.lin_edge.weight,
          layer.att, layer.bias)
    key = tuple((p.data_ptr(), p._version) for p in ps)
    hit = getattr(layer, "_packed", None)
    if hit is not None and hit[0] == key:
        return hit[1]
    packed = torch.cat([layer.lin_l.weight.reshape(-1), layer.lin_l.bias, layer.lin_r.weight.reshape(-1),
                      layer.lin_r.bias, layer.lin_edge.weight.reshape(-1), layer.att.reshape(-1),
                      layer.bias]).detach().float().contiguous()
    layer._packed = (key, packed)
    return packed


def reverse_csr(src: Tensor, n: int):
    """The target-CSR edges grouped by SOURCE node (stable): rev_ptr [n+1], rev_eid [E'] = edge
    positions in the target CSR.  The policy backward gathers each source's gradient messages
    through it in a fixed order (no atomics)."""
    s = src.long()
    rev_eid = torch.sort(s, stable=True).indices.to(torch.int32).contiguous()
    rev_ptr = torch.zeros(n + 1, dtype=torch.int32, device=src.device)
    rev_ptr[1:] = torch.cumsum(torch.bincount(s, minlength=n), 0).to(torch.int32)
    return rev_ptr, rev_eid


class _HipLogits(torch.autograd.Function):
    """Forward on the gfx950 kernels.  Backward on the gfx950 kernels too (spai_policy_backward,
    hid 4 or 8 and node_features 1/2/4: the GATv2 softmax and message gradients, fc, pooling);
    other sizes differentiate the torch restatement ForwardPolicy.torch_logits on the device.
    The gradient path of the TB loss, not the sampler's hot path."""

    @staticmethod
    def forward(ctx, policy, data, B, *params):
        ctx.policy, ctx.data = policy, data
        logits, lmax = policy._hip_logits(data, B)
        ctx.mark_non_differentiable(lmax)
        return logits, lmax

    @staticmethod
    def backward(ctx, g, _g_lmax):
        pol = ctx.policy
        if pol._hip_backward_ok(ctx.data):
            grads = pol._hip_backward(ctx.data, g.reshape(-1))
            return (None, None, None, *[grads.get(id(p)) if p.requires_grad else None for p in pol.parameters()])
        return _HipLogits._torch_backward(ctx, g)

    @staticmethod
    def _torch_backward(ctx, g):
        params = [p for p in ctx.policy.parameters()]
        with torch.enable_grad():
            out, _ = ctx.policy.torch_logits(ctx.data)
            need = [p for p in params if p.requires_grad]
            grads = torch.autograd.grad(out.reshape(-1), need, g.reshape(-1), allow_unused=True)
        it = iter(grads)
        full = [next(it) if p.requires_grad else None for p in params]
        return (None, None, None, *full)


class ForwardPolicy(BasePolicy):
    """policy.py:24-73 on the MI355X: ``logits``/``forward`` run the gfx950 kernels of
    spai_policy_logits (GATv2 layer 1, GATv2 layer 2 + mean pool, fc + max); there is no CPU
    path (``torch_logits`` is the torch restatement used for gradients and as the fp32
    test reference).  When every row of x is the same (state_to_data's ones(2N, 1),
    gflownet.py:247) the two GATv2 layers give every node the same output whatever the
    attention weights, and spai_policy_logits evaluates that closed form instead of the
    graph kernels (detected on the device once per x)."""

    supports_defer_max = True  # logits_and_max(..., defer_max=True): kernels.PendingMax

    def __init__(self, node_features: int, hidden_dim: int, max_num_actions: int):
        super().__init__(node_features, hidden_dim)
        self.gat2 = GATv2Layer(self.hid * self.in_head, self.hid, heads=self.out_head)
        self.fc = nn.Linear(self.hid, max_num_actions)
        self.alpha = nn.Parameter(torch.tensor(0.0))
        self._csr = {}
        # x with identical rows (the reference's ones(2N, 1)) takes the closed form of the GATv2
        # stack (spai_policy_logits const_rows); False forces the general kernels (tests)
        self.const_fast_path = True
        self._const = None  # (x key, rows-constant flag): checked once per x tensor version

    def torch_logits(self, data) -> Tuple[Tensor, Tensor]:
        """Unmasked logits [1, E+1] and sigmoid(alpha) with torch ops (gradient path)."""
        x, edge_index, edge_attr = data.x, data.edge_index, data.edge_attr
        num_actions = edge_attr.size(0) + 1
        x = torch.relu(self.gat1(x, edge_index, edge_attr))
        x = torch.relu(self.gat2(x, edge_index, edge_attr))
        x = x.mean(dim=0, keepdim=True)
        return skinny_linear(x, self.fc.weight, self.fc.bias, num_actions), torch.sigmoid(self.alpha)

    def _graph(self, data):
        x, ei = data.x, data.edge_index
        key = (ei.data_ptr(), ei.shape[1], data.edge_attr.data_ptr(), x.shape[0], str(x.device))
        hit = self._csr.get(key)
        if hit is None:
            hit = self._csr[key] = (data,) + graph_csr(x, ei, data.edge_attr)  # data pins the key's storage
            if len(self._csr) > 4:
                self._csr.pop(next(iter(self._csr)))
        return hit[1:]

    def rows_constant(self, x: Tensor) -> bool:
        """True when every row of x equals its first row (spai_policy_rows_constant; one host
        sync per new x tensor or in-place modification, cached on (storage, version, shape))."""
        key = (x.data_ptr(), x._version, tuple(x.shape), x.dtype, str(x.device))
        if self._const is not None and self._const[0] == key:
            return self._const[1]
        if torch.cuda.is_current_stream_capturing():
            # no host sync inside a HIP-graph capture: an x first seen here takes the general
            # GATv2 kernels (same logits up to fp32 rounding, capturable); warm the cache eagerly
            return False
        xf = x.detach().float().contiguous()
        flag = torch.empty(1, dtype=torch.int32, device=x.device)
        lib = _lib.load()
        _lib.check(lib.spai_policy_rows_constant(xf.shape[0], xf.shape[1], _lib.ptr(xf), _lib.ptr(flag),
                                                 _lib.stream_ptr(x.device)), "spai_policy_rows_constant")
        const = bool(int(flag.item()) == 1)
        self._const = (key, const, x)  # x pins the storage the key names
        return const

    def _hip_logits(self, data, B: int, defer_max: bool = False):
        x = data.x
        _lib.require_device(x)
        n, fin = x.shape
        num_actions = data.edge_attr.size(0) + 1
        if num_actions > self.fc.out_features:
            raise ValueError(f"{num_actions} actions > max_num_actions={self.fc.out_features}")
        const = self.const_fast_path and self.rows_constant(x)
        rowptr, src, ea = (None, None, None) if const else self._graph(data)
        xf = x.detach().float().contiguous()
        w = self.fc.weight.detach()
        if w.dtype != torch.float32 or not w.is_contiguous():
            w = w.float().contiguous()
        fb = self.fc.bias.detach().float().contiguous()
        p1, p2 = _pack(self.gat1), _pack(self.gat2)
        lib = _lib.load()
        if p1.numel() != lib.spai_policy_params(1, fin, self.hid) or p2.numel() != lib.spai_policy_params(2, fin, self.hid):
            raise ValueError("policy parameter shapes do not match node_features/hidden_dim")
        logits = torch.empty(1, num_actions, dtype=torch.float32, device=x.device)
        lmax = torch.empty(B, dtype=torch.float32, device=x.device)
        # defer_max: the fc block maxima only (B = 0); the rollout's select reduces them (PendingMax)
        buf = torch.empty(lib.spai_policy_lmax_parts(num_actions), dtype=torch.float32, device=x.device) \
            if defer_max else lmax
        ws = _lib.workspace(lib.spai_policy_workspace_bytes(n, self.hid, num_actions), x.device, "policy")
        with kernels._timed("policy"):
            st = lib.spai_policy_logits(n, fin, self.hid, _lib.ptr(xf), _lib.ptr(rowptr), _lib.ptr(src),
                                          _lib.ptr(ea), _lib.ptr(p1), _lib.ptr(p2), _lib.ptr(w), _lib.ptr(fb),
                                          num_actions, _lib.ptr(logits), _lib.ptr(buf), 0 if defer_max else B,
                                          int(const), _lib.ptr(ws), ws.numel(), _lib.stream_ptr(x.device))
        _lib.check(st, "spai_policy_logits")
        return logits, (kernels.PendingMax(lmax, buf) if defer_max else lmax)

    def _hip_backward_ok(self, data) -> bool:
        return self.hid in (4, 8) and data.x.shape[1] in (1, 2, 4)

    def _hip_backward(self, data, g: Tensor) -> dict:
        """{id(parameter): gradient} of sum_a g_a logit_a by spai_policy_backward."""
        x = data.x
        n, fin = x.shape
        A = g.numel()
        rowptr, src, ea = self._graph(data)
        key = (rowptr.data_ptr(), src.data_ptr())
        rev = getattr(self, "_rev", None)
        if rev is None or rev[0] != key:
            rev = self._rev = (key, *reverse_csr(src, n))
        rev_ptr, rev_eid = rev[1], rev[2]
        xf = x.detach().float().contiguous()
        p1, p2 = _pack(self.gat1), _pack(self.gat2)
        w = self.fc.weight.detach()
        if w.dtype != torch.float32 or not w.is_contiguous():
            w = w.float().contiguous()
        gf = g.detach().float().contiguous()
        g1, g2 = torch.empty_like(p1), torch.empty_like(p2)
        dW = torch.empty(A, self.hid, dtype=torch.float32, device=x.device)
        db = torch.empty(A, dtype=torch.float32, device=x.device)
        lib = _lib.load()
        ne = src.numel()
        ws = _lib.workspace(lib.spai_policy_backward_workspace_bytes(n, ne, fin, self.hid, A), x.device,
                            "policy_bwd")
        with kernels._timed("policy_backward"):
            st = lib.spai_policy_backward(n, ne, fin, self.hid, _lib.ptr(xf), _lib.ptr(rowptr), _lib.ptr(src),
                                          _lib.ptr(ea), _lib.ptr(rev_ptr), _lib.ptr(rev_eid), _lib.ptr(p1),
                                          _lib.ptr(p2), _lib.ptr(w), A, _lib.ptr(gf), _lib.ptr(g1), _lib.ptr(g2),
                                          _lib.ptr(dW), _lib.ptr(db), _lib.ptr(ws), ws.numel(),
                                          _lib.stream_ptr(x.device))
        _lib.check(st, "spai_policy_backward")
        grads = {}
        for layer, flat in ((self.gat1, g1), (self.gat2, g2)):
            off = 0
            for p in (layer.lin_l.weight, layer.lin_l.bias, layer.lin_r.weight, layer.lin_r.bias,
                      layer.lin_edge.weight, layer.att, layer.bias):
                grads[id(p)] = flat[off:off + p.numel()].view(p.shape).to(p.dtype)
                off += p.numel()
        fw = torch.zeros_like(self.fc.weight)
        fw[:A] = dW.to(fw.dtype)
        fb = torch.zeros_like(self.fc.bias)
        fb[:A] = db.to(fb.dtype)
        grads[id(self.fc.weight)], grads[id(self.fc.bias)] = fw, fb
        return grads

    def logits_and_max(self, data, B: int = 1, defer_max: bool = False) -> Tuple[Tensor, Tensor, Tensor]:
        """(logits [1, E+1], sigmoid(alpha), lmax [B]) — everything of forward() but the mask,
        plus the logits' maximum for the sampler (no separate statistics pass).  defer_max (no
        autograd): lmax is a kernels.PendingMax the throughput rollout's select completes."""
        params = tuple(self.parameters())
        if torch.is_grad_enabled() and any(p.requires_grad for p in params):
            logits, lmax = _HipLogits.apply(self, data, B, *params)
            return logits, torch.sigmoid(self.alpha), lmax
        logits, lmax = self._hip_logits(data, B, defer_max)
        return logits, self._sigmoid_alpha(), lmax

    def _sigmoid_alpha(self) -> Tensor:
        """sigmoid(alpha) without autograd, cached until alpha is modified in place (an
        optimizer step bumps its version): a rollout does not relaunch the 1-element kernel."""
        key = (self.alpha.data_ptr(), self.alpha._version)
        hit = getattr(self, "_sig_alpha", None)
        if hit is None or hit[0] != key:
            hit = self._sig_alpha = (key, torch.sigmoid(self.alpha.detach()))
        return hit[1]

    def logits(self, data) -> Tuple[Tensor, Tensor]:
        """Unmasked logits [1, E+1] and sigmoid(alpha)."""
        logits, a, _ = self.logits_and_max(data)
        return logits, a

    def forward(self, data, actions: Tensor) -> Tuple[Tensor, Tensor]:
        x, a = self.logits(data)
        if actions.numel() > 0:
            blocked = torch.zeros_like(x, dtype=torch.bool)
            blocked[:, actions.to(x.device)] = True
            x = x.masked_fill(blocked, float("-inf"))
        return torch.softmax(x, dim=1), a


class _LstmLast(torch.autograd.Function):
    """h at each row's last valid step of nn.LSTM(1, H) on the gfx950 kernels: forward
    spai_lstm_forward (keeping (h_t, c_t) when a gradient is needed), backward
    spai_lstm_backward (BPTT, per-sample fp64 rows summed here in sample order)."""

    @staticmethod
    def forward(ctx, traj, lengths, w_ih, w_hh, b_ih, b_hh):
        need = any(ctx.needs_input_grad[2:])
        h, states = kernels.lstm_forward(traj, lengths, w_ih, w_hh, b_ih, b_hh, keep_states=need)
        if need:
            ctx.save_for_backward(traj, lengths, w_ih, w_hh, b_ih, b_hh, states)
        return h

    @staticmethod
    def backward(ctx, dh):
        traj, lengths, w_ih, w_hh, b_ih, b_hh, states = ctx.saved_tensors
        H = w_hh.shape[1]
        rows = kernels.lstm_backward(traj, lengths, w_ih, w_hh, b_ih, b_hh, states, dh)
        g = rows.sum(0)
        R = 4 * H
        d_ih = g[:R].view(R, 1).to(w_ih.dtype)
        d_hh = g[R:R + R * H].view(R, H).to(w_hh.dtype)
        d_b = g[R + R * H:].to(b_ih.dtype)
        return None, None, d_ih, d_hh, d_b, d_b.clone()


class BackwardPolicy(nn.Module):
    """LSTM over each trajectory's action ids; softmax over its first n_valid fc outputs,
    padded with 1.0 to the trajectory length (policy.py:75-129), all samples in one call.
    The recurrence runs on the gfx950 kernels (spai_lstm_forward / spai_lstm_backward);
    the fc GEMM and the masked softmax are torch ops on the device.  ``torch_forward`` is
    the nn.LSTM restatement (the fp32 test reference), not a fallback."""

    def __init__(self, input_dim: int, hidden_dim: int, max_num_actions: int):
        super().__init__()
        self.hidden_dim = hidden_dim
        self.max_num_actions = max_num_actions
        self.lstm = nn.LSTM(input_dim, hidden_dim, batch_first=True)
        self.fc = nn.Linear(hidden_dim, max_num_actions)

    def _head(self, h: Tensor, n: Tensor, T: int) -> Tensor:
        B = h.shape[0]
        width = min(T, self.fc.out_features)
        out = skinny_linear(h, self.fc.weight, self.fc.bias, width)
        pos = torch.arange(width, device=out.device)
        valid = pos.view(1, -1) < n.view(-1, 1)
        p = torch.softmax(out[:, :width].masked_fill(~valid, float("-inf")), dim=1)
        res = torch.ones(B, T, device=out.device, dtype=out.dtype)
        res[:, :width] = torch.where(valid, p, torch.ones((), device=out.device, dtype=out.dtype))
        return res.unsqueeze(1)

    def forward(self, trajectories: Tensor) -> Tensor:
        _lib.require_device(trajectories)
        if self.lstm.input_size != 1:
            raise ValueError("the trajectory is one feature per step (policy.py:100): input_dim must be 1")
        B, T = trajectories.shape
        n = (trajectories != -1).sum(1)
        if bool((n == 0).any()):  # pack_padded_sequence rejects empty rows (one host sync)
            raise RuntimeError("Length of all samples has to be greater than 0")
        lstm = self.lstm
        h = _LstmLast.apply(trajectories, n, lstm.weight_ih_l0, lstm.weight_hh_l0, lstm.bias_ih_l0, lstm.bias_hh_l0)
        return self._head(h, n, T)

    def torch_forward(self, trajectories: Tensor) -> Tensor:
        """The same network with nn.LSTM over packed sequences (test reference)."""
        B, T = trajectories.shape
        n = (trajectories != -1).sum(1)
        packed = nn.utils.rnn.pack_padded_sequence(trajectories.float().unsqueeze(-1), n.cpu(), batch_first=True,
                                                   enforce_sorted=False)
        _, (h, _) = self.lstm(packed)
        return self._head(h[-1], n, T)
