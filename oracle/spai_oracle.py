"""CPU ORACLE for the SPAI-via-GFlowNet hot path — TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may import this module, and only as the checker / the timed CPU baseline.
The product (``gflownet_spai_amd``) never imports it and has no CPU fallback.

It is a plain restatement (numpy / scipy / torch-CPU) of the reference's
algorithm for the hot path, each function citing the reference file:line it
follows (reference = tonylizza/gflownet-spai @ 2024-10-24), plus the
north-star extensions that have no reference counterpart (marked
"PARITY UNPINNED BY THE REFERENCE": pinned instead by numpy ``lstsq`` /
stacked Householder QR and by the reference's own ``calculate_residual`` via the
symmetric-A identity ||AM-I|| = ||M^T A - I||).

Pinning: ``tests/test_oracle_golden.py`` checks every function here against the
golden vectors captured from the reference itself (``tests/golden/make_golden.py``).

Contents
  * pattern layout: raw COO -> action ids / lines      (preconditioner.py:12-25)
  * reference-parity rollout (sequential, torch noise)  (gflownet/gflownet.py:125-197, log.py:24-121)
  * throughput rollout (Gumbel-top-k, Philox4x32-10)   (distributional restatement of gflownet.py:148)
  * copy fill + ||MA-I||_F                             (utils.py:295-356, 89-126; preconditioner.py:79-93)
  * reward                                              (preconditioner.py:55-66, 68-77, 137-165)
  * least-squares fill + ||AM-I||_F                    (north-star extension; parity unpinned by the reference)
  * trajectory balance loss                             (gflownet/utils.py:228-278)
  * logged-probability gradient w.r.t. the logits       (log.py:70 + policy.py:65-73 under autograd)
  * BackwardPolicy LSTM forward / BPTT                  (policy.py:75-129, torch nn.LSTM semantics)
"""
from __future__ import annotations

import numpy as np
import scipy.sparse as sp
import torch

# --------------------------------------------------------------------------------------
# Pattern / layout
# --------------------------------------------------------------------------------------


def lines_from_coo(rows, cols, vals, n, orient, width=None):
    """Line-major ELL view of a raw COO matrix.

    orient == "row": line i lists (col k, value, action id) of row i    (MA side, CSR)
    orient == "col": line j lists (row r, value, action id) of column j (AM side, CSC)
    The action id of an entry is its position in the raw COO order
    (preconditioner.py:23-25: edge_index = matrix._indices()).
    Entries inside a line are sorted by the other index.  Raises on duplicates.
    """
    rows = np.asarray(rows, np.int64)
    cols = np.asarray(cols, np.int64)
    vals = np.asarray(vals)
    line, other = (rows, cols) if orient == "row" else (cols, rows)
    order = np.lexsort((other, line))
    ls, os_ = line[order], other[order]
    if ls.size and np.any((ls[1:] == ls[:-1]) & (os_[1:] == os_[:-1])):
        raise ValueError("duplicate (row, col) entries are not supported")
    counts = np.bincount(ls, minlength=n)
    w = int(counts.max()) if counts.size else 0
    if width is None:
        width = max(w, 1)
    if w > width:
        raise ValueError(f"line width {w} exceeds {width}")
    start = np.concatenate([[0], np.cumsum(counts)[:-1]])
    slot = np.arange(ls.size) - start[ls]
    idx = np.full((n, width), -1, np.int32)
    act = np.full((n, width), -1, np.int32)
    val = np.zeros((n, width), vals.dtype)
    idx[ls, slot] = os_
    act[ls, slot] = order
    val[ls, slot] = vals[order]
    return idx, act, val


def poisson2d(grid, dtype=np.float32):
    t = sp.diags([-np.ones(grid - 1), 2 * np.ones(grid), -np.ones(grid - 1)], [-1, 0, 1])
    i = sp.identity(grid)
    a = (sp.kron(i, t) + sp.kron(t, i)).tocoo().astype(dtype)
    order = np.lexsort((a.col, a.row))
    return a.row[order].astype(np.int64), a.col[order].astype(np.int64), a.data[order], grid * grid


def poisson3d(grid, dtype=np.float64):
    t = sp.diags([-np.ones(grid - 1), 2 * np.ones(grid), -np.ones(grid - 1)], [-1, 0, 1])
    i = sp.identity(grid)
    a = (sp.kron(sp.kron(i, i), t) + sp.kron(sp.kron(i, t), i) + sp.kron(sp.kron(t, i), i)).tocoo().astype(dtype)
    order = np.lexsort((a.col, a.row))
    return a.row[order].astype(np.int64), a.col[order].astype(np.int64), a.data[order], grid ** 3


# --------------------------------------------------------------------------------------
# Reference-parity rollout (gflownet/gflownet.py:125-197 with the fixed-logit policy
# contract of policy.py:63-73; log.py:24-89)
# --------------------------------------------------------------------------------------


def parity_rollout(logits, B, generator=None, max_steps=None):
    """Sequential rollout with exactly the reference's torch ops and noise stream
    (``max_steps``: stop after that many steps — the prefix of the full rollout, for long golden
    trajectories whose O(T^2) history masking would take minutes here).

    Per step: each sample's probs = softmax(logits masked by its history)
    (policy.py:65-73) -> stack [B,1,E+1] -> row renormalisation when B > 1
    (gflownet.py:116-120) -> Categorical(probs).sample() (gflownet.py:148) which is
    argmax(p / q), q ~ Exp(1) drawn B*(E+1) per step from the default generator.
    Returns actions [T,B] int64 (-1 after done), fwd_probs [B,T] fp32 (1 after done).
    """
    logits = torch.as_tensor(logits, dtype=torch.float32).view(1, -1)
    A1 = logits.shape[1]
    E = A1 - 1
    done = torch.zeros(B, dtype=torch.bool)
    hist = []  # list of [B] int64 (log._actions)
    fwd = []
    while not bool(done.all()) and (max_steps is None or len(hist) < max_steps):
        a_all, probs_all = reference_step(logits, B, hist, generator)
        mask_active = ~done
        fp = torch.ones(B)
        gathered = probs_all.gather(2, a_all.unsqueeze(1)).view(B)
        fp[mask_active] = gathered[mask_active]
        fwd.append(fp)
        la = -torch.ones(B, dtype=torch.long)
        la[mask_active] = a_all.view(B)[mask_active]
        hist.append(la)
        term = (a_all.view(B) == E)
        done[mask_active] = term[mask_active]
    return torch.stack(hist, 0), torch.stack(fwd, 0).t().contiguous()


def reference_step(logits, B, hist, generator=None):
    """One step of the reference's sampler with its torch-CPU ops: per sample the policy's
    masked softmax over the action history (policy.py:65-73), stacked [B,1,E+1], renormalised
    when B > 1 (gflownet.py:116-120), then Categorical(probs).sample() (gflownet.py:148), i.e.
    multinomial's fast path argmax(p / q), q ~ Exp(1) of shape [B, E+1] from the generator.
    Returns (actions [B,1], probs_all [B,1,E+1])."""
    A1 = logits.shape[1]
    acts = torch.stack(hist, 1) if hist else torch.empty(B, 0, dtype=torch.long)
    probs = []
    for b in range(B):
        x = logits
        if acts.shape[1] > 0:
            mask = torch.ones_like(x, dtype=torch.bool)
            mask[:, acts[b]] = 0
            x = x.masked_fill(~mask, float("-inf"))
        probs.append(torch.softmax(x, dim=1))
    probs_all = torch.stack(probs, 0)  # [B,1,E+1]
    if B > 1:
        s = probs_all.sum(2)
        s[s == 0] = 1
        probs_all = probs_all / s.unsqueeze(1)
    # torch.distributions.Categorical(probs).sample() == multinomial(p/sum, 1, True)
    p2 = probs_all.reshape(-1, A1)
    p2 = p2 / p2.sum(-1, keepdim=True)
    q = torch.empty_like(p2).exponential_(1, generator=generator)
    return torch.argmax(p2 / q, dim=-1).view(B, 1), probs_all


def reference_update_residual(rows, cols, vals, removed_b, n, A_t):
    """One sample of env.update with the reference's torch-CPU ops: the kept edges as a fresh
    COO M (utils.py:315-353: keep mask over E, coalesce), ||M A - I||_F by sparse torch.mm,
    the fp64 identity subtraction and torch.norm (preconditioner.py:79-93).  A_t: A as a torch
    sparse COO tensor (fp32)."""
    keep = ~torch.as_tensor(removed_b)
    ind = torch.stack([torch.as_tensor(rows)[keep], torch.as_tensor(cols)[keep]])
    M = torch.sparse_coo_tensor(ind, torch.as_tensor(vals)[keep].float(), (n, n)).coalesce()
    i = torch.arange(n)
    eye = torch.sparse_coo_tensor(torch.stack([i, i]), torch.ones(n, dtype=torch.float64), (n, n))
    return float(torch.norm(torch.mm(M, A_t) - eye))


# --------------------------------------------------------------------------------------
# Throughput rollout: Gumbel-top-k with counter-based Philox4x32-10.
# Distributionally identical to the sequential process of gflownet.py:148 (sampling
# without replacement until the terminal id is drawn == Plackett-Luce order of
# keys l_a + Gumbel_a; removed set = {a : key_a > key_E}); not pathwise identical.
# Everything below is defined bit-for-bit so that the HIP kernels reproduce it.
# --------------------------------------------------------------------------------------

_PHILOX_M0, _PHILOX_M1 = np.uint64(0xD2511F53), np.uint64(0xCD9E8D57)
_PHILOX_W0, _PHILOX_W1 = 0x9E3779B9, 0xBB67AE85
_MASK32 = np.uint64(0xFFFFFFFF)


def philox4x32_10(c0, c1, c2, c3, k0, k1):
    """Random123 Philox4x32-10 on uint32 arrays (returned as uint64 arrays < 2^32)."""
    c0, c1, c2, c3 = (np.asarray(x, np.uint64) & _MASK32 for x in (c0, c1, c2, c3))
    k0, k1 = int(k0) & 0xFFFFFFFF, int(k1) & 0xFFFFFFFF
    for r in range(10):
        p0 = _PHILOX_M0 * c0
        p1 = _PHILOX_M1 * c2
        hi0, lo0 = p0 >> np.uint64(32), p0 & _MASK32
        hi1, lo1 = p1 >> np.uint64(32), p1 & _MASK32
        c0, c1, c2, c3 = hi1 ^ c1 ^ np.uint64(k0), lo1, hi0 ^ c3 ^ np.uint64(k1), lo0
        k0 = (k0 + _PHILOX_W0) & 0xFFFFFFFF
        k1 = (k1 + _PHILOX_W1) & 0xFFFFFFFF
    return c0, c1, c2, c3


_LOG_C = np.array([0x3f800000, 0xbefffffc, 0x3eaaabc8, 0xbe8002d3, 0x3e4c5c05,
                   0xbe2994df, 0x3e191428, 0xbe13394f, 0x3db31375], np.uint32).view(np.float32)
_LN2F = np.array([0x3f317218], np.uint32).view(np.float32)[0]


def fma32(a, b, c):
    """IEEE single-rounded fp32 fused multiply-add, elementwise (the device's v_fma_f32 /
    v_pk_fma_f32 and C fmaf).  a*b is exact in fp64; the fp64 sum s = a*b + c is rounded
    once, and rounding s to fp32 can only differ from rounding the exact sum when s lands
    exactly on a midpoint between two fp32 values - the exact TwoSum error of s then
    decides the side."""
    a = np.asarray(a, np.float32)
    b = np.asarray(b, np.float32)
    c = np.asarray(c, np.float32)
    p = a.astype(np.float64) * b.astype(np.float64)
    c64 = c.astype(np.float64)
    s = p + c64
    bb = s - p
    err = (p - (s - bb)) + (c64 - bb)
    r = s.astype(np.float32)
    d = s - r.astype(np.float64)
    # neighbour of r on the side of s, and the midpoint between them (exact in fp64)
    n = np.nextafter(r, np.where(d > 0, np.float32(np.inf), np.float32(-np.inf))).astype(np.float32)
    mid = (r.astype(np.float64) + n.astype(np.float64)) * 0.5
    fix = (d != 0) & (s == mid) & (err != 0) & (np.sign(err) == np.sign(d))
    return np.where(fix, n, r).astype(np.float32)


def det_logf(x):
    """Deterministic natural log of positive normal float32 values.

    Exponent/mantissa split by bit operations, m in [sqrt(.5), sqrt(2)), t = m - 1
    (exact), ln(1+t) = t * Q(t) with a degree-8 Q evaluated by Horner in single-rounded
    fp32 FMAs, then fma(e, ln2, t * Q).  The HIP kernels (spai_device.h: det_logf /
    det_logf2, the latter two lanes per packed v_pk_fma_f32) perform the identical op
    sequence.
    """
    x = np.asarray(x, np.float32)
    bits = x.view(np.uint32)
    e = (bits >> np.uint32(23)).astype(np.int32) - 127
    mb = (bits & np.uint32(0x7FFFFF)) | np.uint32(0x3F800000)
    big = mb > np.uint32(0x3FB504F3)
    mb = np.where(big, mb - np.uint32(0x00800000), mb).astype(np.uint32)
    e = e + big.astype(np.int32)
    t = mb.view(np.float32) - np.float32(1.0)
    p = np.full_like(t, _LOG_C[8])
    for c in _LOG_C[7::-1]:
        p = fma32(p, t, c)
    p = p * t
    return fma32(e.astype(np.float32), _LN2F, p)


_EXP_C = np.array([0x3f800000, 0x3f800000, 0x3f000000, 0x3e2aaaab, 0x3d2aaaab, 0x3c088889, 0x3ab60b61,
                   0x39500d01], np.uint32).view(np.float32)  # 1/i! for i = 0..7
_LOG2EF = np.array([0x3fb8aa3b], np.uint32).view(np.float32)[0]
_LN2_HI = np.array([0x3f317200], np.uint32).view(np.float32)[0]
_LN2_LO = np.array([0x35bfbe8e], np.uint32).view(np.float32)[0]


def det_expf(x):
    """Deterministic e^x of float32 values (spai_device.h det_expf, op for op).

    k = rint(x * log2 e) in fp32, r = x - k ln2 by two single-rounded FMAs (ln2 split in a
    head and a tail), e^r by a degree-7 Taylor Horner in fp32 FMAs, times 2^k (ldexp, exact:
    the results stay normal).  x > 88.72 gives +inf, x < -87.33 gives 0.
    """
    x = np.asarray(x, np.float32)
    xc = np.clip(x, np.float32(-87.33), np.float32(88.72))
    k = np.rint(xc * _LOG2EF).astype(np.float32)
    r = fma32(-k, _LN2_HI, xc)
    r = fma32(-k, _LN2_LO, r)
    p = np.full_like(r, _EXP_C[7])
    for c in _EXP_C[6::-1]:
        p = fma32(p, r, c)
    out = np.ldexp(p, k.astype(np.int32)).astype(np.float32)
    out = np.where(x > np.float32(88.72), np.float32(np.inf), out)
    return np.where(x < np.float32(-87.33), np.float32(0.0), out).astype(np.float32)


def philox_u(n, b_global, seed, stream):
    """u_a for a = 0..n-1: counter = (a >> 2, b_global, stream_lo, stream_hi), key = (seed_lo,
    seed_hi), output word a & 3; u = (2*(w >> 9) + 1) * 2^-24 in (0, 1), exact in fp32."""
    a = np.arange(n, dtype=np.uint64)
    w = philox4x32_10(a >> np.uint64(2), np.full_like(a, b_global), np.full_like(a, stream & 0xFFFFFFFF),
                      np.full_like(a, (stream >> 32) & 0xFFFFFFFF), seed & 0xFFFFFFFF, (seed >> 32) & 0xFFFFFFFF)
    sel = (a & np.uint64(3)).astype(np.int64)
    word = np.choose(sel, w).astype(np.uint64)
    k = (word >> np.uint64(9)).astype(np.uint32)
    return (np.float32(2.0) * k.astype(np.float32) + np.float32(1.0)) * np.float32(2.0 ** -24)


def inverse_rates(logits):
    """r_a = e^(l_E - l_a) (det_expf of the fp32 difference), r_E = 1 exactly."""
    logits = np.asarray(logits, np.float32)
    return det_expf(logits[-1] - logits)


def arrival_times(logits, b_global, seed, stream):
    """Exponential race of sample b_global: t_a = q_a * r_a in fp32 for a = 0..E (E = terminal),
    q_a = -ln u_a (det_logf) ~ Exp(1), r_a = inverse_rates.  t_a < t_E <=> the Gumbel key
    l_a - ln q_a exceeds the terminal's, and ascending t is the Plackett-Luce order of
    sequential sampling without replacement (gflownet.py:135-179)."""
    logits = np.asarray(logits, np.float32)
    q = -det_logf(philox_u(logits.size, b_global, seed, stream))
    return (q * inverse_rates(logits)).astype(np.float32)


def throughput_rollout(logits, B, seed, stream, sample_base=0):
    """Removed sets, ordered trajectories and forward probabilities for B samples.

    Returns (removed [B,E] bool, actions [T,B] int64, fwd_probs [B,T] fp32, counts [B]).
    Removed: t_a < t_E (arrival_times); order: t ascending, ties by action id ascending;
    trajectory = winners then E.
    fwd_probs[t] = w_{a_t} / (W_rest + sum_{s>=t} w_{a_s}), w = exp(l - lmax) in fp64 and
    W_rest the mass of the actions never removed (terminal included): the masked-softmax
    probability the sequential reference assigns to that step (policy.py:65-73, log.py:70),
    formed from the remaining mass directly (no Z - prefix cancellation).
    """
    logits = np.asarray(logits, np.float32)
    E = logits.size - 1
    lmax = np.float64(logits.max())
    w = np.exp(logits.astype(np.float64) - lmax)
    removed = np.zeros((B, E), np.bool_)
    orders, probs = [], []
    for b in range(B):
        t = arrival_times(logits, sample_base + b, seed, stream)
        win = np.flatnonzero(t[:E] < t[E])
        removed[b, win] = True
        o = win[np.lexsort((win, t[win]))]
        ww = w[o]
        rest = w[E] + w[:E][~removed[b]].sum()
        suffix = np.cumsum(ww[::-1])[::-1]
        p = np.concatenate([ww / (rest + suffix), [w[E] / rest]])
        orders.append(np.concatenate([o, [E]]))
        probs.append(p)
    counts = np.array([len(o) - 1 for o in orders])
    T = int(counts.max()) + 1
    actions = -np.ones((T, B), np.int64)
    fwd = np.ones((B, T), np.float32)
    for b in range(B):
        actions[:len(orders[b]), b] = orders[b]
        fwd[b, :len(probs[b])] = probs[b].astype(np.float32)
    return removed, actions, fwd, counts


def removal_from_actions(actions_bt, E):
    """Removed-set bitmap from a [B,T] action list (preconditioner.py:37-43, utils.py:315-323)."""
    a = np.asarray(actions_bt)
    B = a.shape[0]
    removed = np.zeros((B, E), np.bool_)
    for b in range(B):
        x = a[b]
        x = x[(x >= 0) & (x < E)]
        removed[b, x] = True
    return removed


# --------------------------------------------------------------------------------------
# Copy fill + residual + reward (reference parity)
# --------------------------------------------------------------------------------------


def copy_fill_coo(rows, cols, vals, removed_b, n):
    """M = initial matrix minus removed edges, values copied as fp32 (utils.py:331-353)."""
    keep = ~np.asarray(removed_b, bool)
    return rows[keep], cols[keep], np.asarray(vals)[keep].astype(np.float32)


def residual_ma_torch(m_rows, m_cols, m_vals, a_rows, a_cols, a_vals, n):
    """||M A - I||_F with the reference's torch ops (preconditioner.py:79-93)."""
    M = torch.sparse_coo_tensor(torch.from_numpy(np.stack([m_rows, m_cols]).astype(np.int64)),
                                torch.from_numpy(np.asarray(m_vals, np.float32)), (n, n)).coalesce()
    A = torch.sparse_coo_tensor(torch.from_numpy(np.stack([a_rows, a_cols]).astype(np.int64)),
                                torch.from_numpy(np.asarray(a_vals)), (n, n))
    i = torch.arange(n)
    eye = torch.sparse_coo_tensor(torch.stack([i, i]), torch.ones(n, dtype=torch.float64), (n, n))
    return float(torch.norm(torch.mm(M, A) - eye))


def residual_fro_fp64(X: sp.spmatrix, Y: sp.spmatrix):
    """||X Y - I||_F with fp64 products and sums (scipy)."""
    P = (X.astype(np.float64) @ Y.astype(np.float64)).tocsr()
    P = P - sp.identity(P.shape[0], format="csr")
    return float(np.sqrt((P.data.astype(np.float64) ** 2).sum()))


def reward(residual, nnz_m, alpha, r0, f0, n):
    """preconditioner.py:55-66 + 68-77 + 137-165, with alpha taken from the argument.

    Mirrors torch's type promotion exactly: alpha is a 0-d fp32 tensor, the
    residual ratio a 0-d fp64 tensor, the flop ratio a python float, so
    (1 - alpha) * (1 - flop_ratio) is computed in fp32 and the sum in fp64.
    """
    alpha = torch.as_tensor(alpha, dtype=torch.float32)
    res = torch.as_tensor(residual, dtype=torch.float64)
    r0 = torch.as_tensor(r0, dtype=torch.float64)
    rr = res / r0 if float(r0) != 0 else float("inf")
    flops = int(nnz_m) * n * 2
    cr = flops / f0 if f0 != 0 else float("inf")
    perf = alpha * (1 - rr) + (1 - alpha) * (1 - cr)
    return float(perf.to(torch.float64) * 1000)


# --------------------------------------------------------------------------------------
# Exact residual sums (the build's multi-GPU reduction; no reference counterpart: the reference
# sums ||M A - I||_F^2 inside one torch.norm, preconditioner.py:90).  Restates spai_device.h
# fixed_add / fixed_value (spai_hip.h SPAI_RES2_LIMBS): every partial truncated toward zero to a
# multiple of 2^-96, summed as integers, rounded once.
# --------------------------------------------------------------------------------------

RES2_LIMBS = 8


def fixed_limbs(x: float) -> np.ndarray:
    """int64 [8] slots of one fp64 partial: six signed 32-bit limbs (value = sum L_i 2^(32i-96)),
    then the NaN (<< 32) / inf-or-|x|>=2^94 count, then a pad."""
    L = np.zeros(RES2_LIMBS, dtype=np.int64)
    x = float(x)
    if np.isnan(x):
        L[6] = 1 << 32
        return L
    if np.isinf(x) or abs(x) >= 2.0 ** 94:
        L[6] = 1
        return L
    F = int(abs(x) * 2.0 ** 96)  # |x| 2^96 is exact (a power-of-two scaling); int() truncates toward 0
    for i in range(6):
        c = (F >> (32 * i)) & 0xFFFFFFFF
        L[i] = -c if x < 0 else c
    return L


def fixed_value(L) -> float:
    """fp64 value of summed slots (carry-normalise, then Horner from the top limb, as the kernel)."""
    L = [int(v) for v in L]
    if L[6] >> 32:
        return float("nan")
    if L[6]:
        return float("inf")
    c = L[:6]
    for i in range(5):
        carry = c[i] >> 32
        c[i] -= carry << 32
        c[i + 1] += carry
    v = float(c[5])
    for i in range(4, -1, -1):
        v = v * 4294967296.0 + float(c[i])  # the kernel's fma: v * 2^32 is exact, one rounding
    return v * 2.0 ** -96


def fixed_sum(partials) -> float:
    """The exact sum of fp64 partials as the GPU reduction returns it (partition-invariant)."""
    acc = np.zeros(RES2_LIMBS, dtype=object)
    for x in partials:
        acc = acc + fixed_limbs(x).astype(object)
    return fixed_value(acc)


# --------------------------------------------------------------------------------------
# Least-squares fill (north-star extension) — PARITY UNPINNED BY THE REFERENCE.
# m_j = argmin || A[:, J_j] m - e_j ||_2, J_j = kept pattern rows of column j.
# Oracle: stacked Householder QR in fp64 (numpy), cross-checked by lstsq.
# --------------------------------------------------------------------------------------


def lsq_fill(pat_idx, keep, a_idx, a_val, line_ids=None):
    """Column-wise LS fill.  pat_idx [N,W] (rows of each column, -1 pad), keep [N,W] bool,
    a_idx/a_val [N,WA]: column lines of A.  Returns m [len(line_ids), W] fp64 (0 where not kept).

    Uses stacked dense Householder QR over the local row set I_j = union of rows of
    A[:, J_j]; singular systems are not expected (A nonsingular => columns independent).
    """
    N, W = pat_idx.shape
    WA = a_idx.shape[1]
    if line_ids is None:
        line_ids = np.arange(N)
    line_ids = np.asarray(line_ids)
    n = line_ids.size
    J = np.where(keep[line_ids], pat_idx[line_ids], -1)  # [n, W]
    Jc = np.where(J >= 0, J, 0)
    rows = a_idx[Jc]  # [n, W, WA]
    vals = a_val[Jc].astype(np.float64)
    valid = (J[:, :, None] >= 0) & (rows >= 0)
    rows = np.where(valid, rows, -1)
    vals = np.where(valid, vals, 0.0)
    flat = rows.reshape(n, W * WA)
    srt = np.sort(np.where(flat >= 0, flat, np.iinfo(np.int32).max), axis=1)
    first = np.ones_like(srt, bool)
    first[:, 1:] = srt[:, 1:] != srt[:, :-1]
    first &= srt != np.iinfo(np.int32).max
    IMAX = max(int(first.sum(1).max()) if n else 1, 1)
    uniq = np.full((n, IMAX), -1, np.int64)
    pos = np.cumsum(first, 1) - 1
    r_i, c_i = np.nonzero(first)
    uniq[r_i, pos[r_i, c_i]] = srt[r_i, c_i]
    # local row index of each (p, s) entry
    dense = np.zeros((n, IMAX, W))
    for p in range(W):
        for s in range(WA):
            r = rows[:, p, s]
            ok = r >= 0
            loc = np.argmax(uniq == r[:, None], axis=1)
            dense[np.nonzero(ok)[0], loc[ok], p] += vals[ok, p, s]
    rhs = (uniq == line_ids[:, None]).astype(np.float64)
    # columns not kept are zero columns; replace by unit vectors on an extra row so QR
    # stays nonsingular, and force their coefficients to 0 afterwards.
    kept = J >= 0
    ext = np.zeros((n, IMAX + W, W))
    ext[:, :IMAX, :] = dense
    ii = np.arange(W)
    ext[:, IMAX + ii, ii] = np.where(kept, 0.0, 1.0)
    rhs_ext = np.zeros((n, IMAX + W))
    rhs_ext[:, :IMAX] = rhs
    q, r = np.linalg.qr(ext)
    qtb = np.einsum("nij,ni->nj", q, rhs_ext)
    m = np.linalg.solve(r, qtb[..., None])[..., 0]
    m = np.where(kept, m, 0.0)
    return m


def lsq_fill_lstsq(pat_idx, keep, A_csc: sp.csc_matrix, j):
    """Per-column numpy lstsq cross-check of lsq_fill (small cases only)."""
    J = pat_idx[j][keep[j] & (pat_idx[j] >= 0)]
    if J.size == 0:
        return np.zeros(0), J
    sub = A_csc[:, J].toarray().astype(np.float64)
    e = np.zeros(A_csc.shape[0])
    e[j] = 1.0
    m, *_ = np.linalg.lstsq(sub, e, rcond=None)
    return m, J


def m_to_csc(pat_idx, m, n, dtype=np.float32):
    """Assemble M (column lines of values aligned with pat_idx) as a scipy CSC matrix."""
    N, W = pat_idx.shape
    cols = np.repeat(np.arange(N), W)
    rows = pat_idx.reshape(-1)
    v = np.asarray(m, dtype).reshape(-1)
    ok = rows >= 0
    return sp.csc_matrix((v[ok], (rows[ok], cols[ok])), shape=(n, n))


# --------------------------------------------------------------------------------------
# Trajectory balance loss (gflownet/utils.py:228-278)
# --------------------------------------------------------------------------------------


def trajectory_balance_loss(total_flow, rewards, fwd_probs, back_probs):
    eps = 1e-9
    total_flow = total_flow.to(fwd_probs.device).to(fwd_probs.dtype)
    rewards = rewards.to(fwd_probs.device).to(fwd_probs.dtype)
    back_probs = back_probs.to(fwd_probs.device).to(fwd_probs.dtype)
    lf = torch.log(fwd_probs + eps).sum(dim=-1)
    lb = torch.log(back_probs + eps).sum(dim=-1)
    lf = lf - lf.max(dim=0, keepdim=True)[0]
    lb = lb - lb.max(dim=0, keepdim=True)[0]
    lhs = torch.log(total_flow + eps) + lf
    rhs = torch.log(rewards + eps) + lb
    return ((lhs - rhs) ** 2).mean()


# --------------------------------------------------------------------------------------
# Gradient of the logged forward probabilities w.r.t. the logits: what autograd computes
# through the reference's per-step masked softmax (policy.py:65-73) and the gather of
# log.py:70, in closed form.  p_t = w_{a_t} / R_t, R_t = untouched mass + sum_{s>=t} w_{a_s}:
#   dL/dl_{a_t} += G_t - w_{a_t} S_t,  dL/dl_a += -w_a S_last (a untouched, a < E),
#   G_t = gp_t p_t,  S_t = sum_{s<=t} G_s p_s / w_{a_s}.
# Pinned by the reference's own logits.grad in the golden rollouts (tests/golden).
# --------------------------------------------------------------------------------------


def logp_grad(logits, actions_bt, probs_bt, gprobs_bt):
    l = np.asarray(logits, np.float64).reshape(-1)
    w = np.exp(l - l.max())
    E = l.size - 1
    grad = np.zeros(E + 1)
    for a, p, g in zip(np.asarray(actions_bt), np.asarray(probs_bt, np.float64), np.asarray(gprobs_bt, np.float64)):
        valid = a >= 0
        av, pv, gv = a[valid], p[valid], g[valid]
        G = gv * pv
        S = np.cumsum(np.where(w[av] > 0, G * pv / np.where(w[av] > 0, w[av], 1.0), 0.0))
        grad[av] += G - w[av] * S  # actions are distinct within one trajectory
        untouched = np.ones(E + 1, np.bool_)
        untouched[av] = False
        untouched[E] = False
        if S.size:
            grad[untouched] -= w[untouched] * S[-1]
    return grad


# --------------------------------------------------------------------------------------
# BackwardPolicy LSTM (policy.py:75-129): nn.LSTM(1, H) over each row's entries != -1
# (pack_padded_sequence keeps the first n of them), gate order i, f, g, o (torch), then
# fc(h_last) -> softmax over the first n outputs, padded with 1.  fp64 numpy restatement;
# the BPTT gives d w_ih [4H, 1], d w_hh [4H, H], d bias [4H] (= d b_ih = d b_hh).
# --------------------------------------------------------------------------------------


def _sig(x):
    return 1.0 / (1.0 + np.exp(-x))


def lstm_forward(traj, w_ih, w_hh, b_ih, b_hh):
    """(h_last [B, H], per-row lists of (h_t, c_t)) in fp64."""
    w_ih, w_hh = np.asarray(w_ih, np.float64).reshape(-1), np.asarray(w_hh, np.float64)
    bias = np.asarray(b_ih, np.float64) + np.asarray(b_hh, np.float64)
    H = w_hh.shape[1]
    outs, states = [], []
    for row in np.asarray(traj):
        n = int((row != -1).sum())
        h, c, st = np.zeros(H), np.zeros(H), []
        for t in range(n):
            z = w_ih * float(row[t]) + bias + w_hh @ h
            i, f, g, o = _sig(z[:H]), _sig(z[H:2 * H]), np.tanh(z[2 * H:3 * H]), _sig(z[3 * H:])
            c = f * c + i * g
            h = o * np.tanh(c)
            st.append((h.copy(), c.copy()))
        outs.append(h)
        states.append(st)
    return np.stack(outs), states


def lstm_backward(traj, w_ih, w_hh, b_ih, b_hh, dh_last):
    """Summed over rows: (d w_ih [4H, 1], d w_hh [4H, H], d bias [4H]) for dL/dh_last."""
    w_ih1, w_hh = np.asarray(w_ih, np.float64).reshape(-1), np.asarray(w_hh, np.float64)
    bias = np.asarray(b_ih, np.float64) + np.asarray(b_hh, np.float64)
    H = w_hh.shape[1]
    _, states = lstm_forward(traj, w_ih, w_hh, b_ih, b_hh)
    g_ih, g_hh, g_b = np.zeros(4 * H), np.zeros((4 * H, H)), np.zeros(4 * H)
    for row, st, dh0 in zip(np.asarray(traj), states, np.asarray(dh_last, np.float64)):
        dh, dc = dh0.copy(), np.zeros(H)
        for t in range(len(st) - 1, -1, -1):
            hp, cp = (st[t - 1] if t > 0 else (np.zeros(H), np.zeros(H)))
            x = float(row[t])
            z = w_ih1 * x + bias + w_hh @ hp
            i, f, g, o = _sig(z[:H]), _sig(z[H:2 * H]), np.tanh(z[2 * H:3 * H]), _sig(z[3 * H:])
            tc = np.tanh(st[t][1])
            dcc = dc + dh * o * (1 - tc * tc)
            da = np.concatenate([dcc * g * i * (1 - i), dcc * cp * f * (1 - f), dcc * i * (1 - g * g),
                                 dh * tc * o * (1 - o)])
            g_ih += da * x
            g_b += da
            g_hh += np.outer(da, hp)
            dc = dcc * f
            dh = w_hh.T @ da
    return g_ih.reshape(-1, 1), g_hh, g_b


def backward_probs(traj, w_ih, w_hh, b_ih, b_hh, fc_w, fc_b):
    """BackwardPolicy.forward (policy.py:87-129) -> [B, 1, T] in fp64."""
    traj = np.asarray(traj)
    B, T = traj.shape
    h, _ = lstm_forward(traj, w_ih, w_hh, b_ih, b_hh)
    out = h @ np.asarray(fc_w, np.float64).T + np.asarray(fc_b, np.float64)
    res = np.ones((B, T))
    for b in range(B):
        n = min(int((traj[b] != -1).sum()), out.shape[1], T)
        z = out[b, :n] - out[b, :n].max()
        res[b, :n] = np.exp(z) / np.exp(z).sum()
    return res[:, None, :]


# --------------------------------------------------------------------------------------
# ForwardPolicy logits (policy.py:14-73) — GATv2Conv restated from PyG's published
# algorithm (torch_geometric.nn.GATv2Conv, 2.x: lin_l / lin_r source and target
# transforms, lin_edge without bias, leaky_relu 0.2, softmax over the incoming edges of
# each target, concat heads, + bias; add_self_loops after remove_self_loops with
# fill_value="mean" over edge_index[1]).  PARITY UNPINNED BY THE REFERENCE: PyG is not
# installed and its version is unpinned (requirements.txt lists none), so this restatement
# is pinned by the known answer gatv2_layer_ones_answer (x = ones, as state_to_data builds
# it, gflownet/gflownet.py:247) and by the test-side torch restatement.
# --------------------------------------------------------------------------------------


def gatv2_layer(x, edge_index, edge_attr, W_l, b_l, W_r, b_r, W_e, att, bias, heads):
    """One GATv2Conv (fp64, sequential loops over targets).  x [n, F]; W_l/W_r [H*C, F];
    W_e [H*C, 1]; att [H, C]; bias [H*C].  Returns [n, H*C]."""
    x = np.asarray(x, np.float64)
    n = x.shape[0]
    src, dst = np.asarray(edge_index[0]), np.asarray(edge_index[1])
    ea = np.asarray(edge_attr, np.float64).reshape(-1)
    keep = src != dst
    src, dst, ea = src[keep], dst[keep], ea[keep]
    deg = np.bincount(dst, minlength=n)
    loop = np.bincount(dst, weights=ea, minlength=n) / np.maximum(deg, 1)
    src = np.concatenate([src, np.arange(n)])
    dst = np.concatenate([dst, np.arange(n)])
    ea = np.concatenate([ea, loop])
    HC = W_l.shape[0]
    C = HC // heads
    xl = (x @ np.asarray(W_l, np.float64).T + b_l).reshape(n, heads, C)
    xr = (x @ np.asarray(W_r, np.float64).T + b_r).reshape(n, heads, C)
    we = np.asarray(W_e, np.float64).reshape(heads, C)
    att = np.asarray(att, np.float64).reshape(heads, C)
    out = np.zeros((n, heads, C))
    order = np.argsort(dst, kind="stable")
    starts = np.searchsorted(dst[order], np.arange(n + 1))
    for i in range(n):
        es = order[starts[i]:starts[i + 1]]
        if es.size == 0:
            continue
        z = xl[src[es]] + xr[i][None] + ea[es][:, None, None] * we[None]
        z = np.where(z > 0, z, 0.2 * z)
        s = (z * att[None]).sum(-1)  # [deg, H]
        s = np.exp(s - s.max(0, keepdims=True))
        a = s / s.sum(0, keepdims=True)
        out[i] = (a[:, :, None] * xl[src[es]]).sum(0)
    return out.reshape(n, HC) + np.asarray(bias, np.float64)


def gatv2_layer_ones_answer(W_l, b_l, bias, n):
    """Known answer for x = ones(n, 1): every node's incoming sources carry the same
    W_l 1 + b_l, and the attention weights of a target sum to 1, so out_i = W_l 1 + b_l + bias
    whatever the graph, edge attributes, att and W_e are."""
    row = np.asarray(W_l, np.float64).sum(1) + np.asarray(b_l, np.float64) + np.asarray(bias, np.float64)
    return np.tile(row, (n, 1))


def forward_policy_logits(x, edge_index, edge_attr, p1, p2, fc_w, fc_b, num_actions):
    """logits[a] = fc(mean_pool(relu(gat2(relu(gat1(x))))))[a], a < num_actions
    (policy.py:40-69).  p1/p2: dicts with W_l b_l W_r b_r W_e att bias (numpy)."""
    h = np.maximum(gatv2_layer(x, edge_index, edge_attr, heads=4, **p1), 0.0)
    h = np.maximum(gatv2_layer(h, edge_index, edge_attr, heads=1, **p2), 0.0)
    pooled = h.mean(0)
    return (np.asarray(fc_w, np.float64)[:num_actions] @ pooled + np.asarray(fc_b, np.float64)[:num_actions])
