"""World-size-2 gloo tests of the multi-GPU layout on CPU (no GPU needed).

The per-shard compute is played by the CPU oracle; the collectives and the shard
bookkeeping are the product code used on the GPU box (gflownet_spai_amd/distributed.py).
"""
import os
import socket

import numpy as np
import pytest
import scipy.sparse as sp
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from gflownet_spai_amd.distributed import (LINE_ALIGN, LineGather, PackPlan, allgather_lines, allreduce_res2,
                                           exchange_packed, exchange_parts, gather_rewards, gather_slices,
                                           pack_bits_reference, select_best_samples, shard_lines, word_spans)
from oracle import spai_oracle as O


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        out = {}
        # column-sharded LSQ fill + ||AM - I||^2 of 3 candidates of a 12x12 Poisson matrix
        r, c, v, n = O.poisson2d(12, np.float64)
        idx, act, _ = O.lines_from_coo(r, c, v, n, "col")
        a_idx, _, a_val = O.lines_from_coo(r, c, v, n, "col")
        A = sp.csc_matrix((v, (r, c)), shape=(n, n))
        rng = np.random.default_rng(5)
        B = 3
        removed = rng.random((B, len(r))) < 0.3
        b0, b1 = shard_lines(n, rank, world)
        lines = np.arange(b0, b1)
        res2 = torch.zeros(B, dtype=torch.float64)
        m_loc = torch.zeros(B, b1 - b0, idx.shape[1], dtype=torch.float64)
        for b in range(B):
            keep = (idx >= 0) & ~removed[b][np.clip(act, 0, None)]
            m = O.lsq_fill(idx, keep, a_idx, a_val, lines)
            m_loc[b] = torch.from_numpy(m)
            sub = idx[lines]
            ok = sub >= 0
            cols = np.repeat(np.arange(len(lines)), sub.shape[1]).reshape(sub.shape)
            M = sp.csc_matrix((m[ok], (sub[ok], cols[ok])), shape=(n, len(lines)))  # columns b0..b1
            P = (A @ M).tocoo()
            diag = P.data[P.row == lines[P.col]].sum()
            res2[b] = (P.data ** 2).sum() - 2 * diag + len(lines)
        allreduce_res2(res2)
        full_m = allgather_lines(m_loc, n)
        out["res2"] = res2.numpy()
        out["m"] = full_m.numpy()
        # the pipelined form (bench.py's per-step assembly): two gathers through the same buffers
        lgth = LineGather(n, align=LINE_ALIGN)
        b0a, b1a = shard_lines(n, rank, world, LINE_ALIGN)
        ma = torch.arange(2 * (b1a - b0a) * 5, dtype=torch.float32).view(2, b1a - b0a, 5) + 1000 * rank
        lgth.start(ma)
        lgth.start(ma + 1)
        out["m_pipe"] = lgth.result().numpy()
        lgth.start(ma + 1, rows=torch.tensor([1]))  # one candidate, selected into the send buffer
        out["m_row"] = lgth.result().numpy()
        out["rewards"] = gather_rewards(torch.arange(B, dtype=torch.float64) + 10 * rank).numpy()
        # the slices split's exchange: each part fills the bucket weight sums and winner counts
        # of its own bucket range (zero elsewhere, the exchange array's [B][2][kMaxB] layout)
        # and its lines' exact residual limbs go into the B x 8 trailing slots; one all_reduce
        # of the int64 bit patterns in place
        full_bs, partials = _split_fixture()
        B3, nb = full_bs.shape[0], full_bs.shape[2]
        k0, k1 = nb * rank // world, nb * (rank + 1) // world
        xch = torch.zeros(full_bs.numel() + B3 * O.RES2_LIMBS, dtype=torch.float64)
        bs = xch[:full_bs.numel()].view_as(full_bs)
        bs[:, :, k0:k1] = full_bs[:, :, k0:k1]
        mine = partials[:, rank::world]  # this rank's per-block partials of every sample
        limbs = torch.from_numpy(np.stack([sum(O.fixed_limbs(x) for x in row) for row in mine]))
        summed = exchange_parts(xch, limbs)
        out["r2"] = [O.fixed_value(row) for row in summed.numpy()]
        out["bs"] = bs.numpy()
        out["cols"] = _columns_exchange(rank, world)
        out["cols_win"] = _columns_exchange(rank, world, mode="auto")
        # the samples split: 2 local candidates per rank, global best's M reduced to rank 0
        rw = torch.tensor([[0.5, 2.5], [1.5, -1.0]], dtype=torch.float64)[rank]
        ml = torch.arange(2 * 3 * 4, dtype=torch.float64).view(2, 3, 4) + 100 * rank
        allr, best, mbest = select_best_samples(rw, ml)
        out["samples"] = (allr.numpy(), int(best), mbest.numpy())
        # the split log: rank q holds slice [bounds[b,0], bounds[b,1]) of each trajectory
        acts, fwd, cuts, T = _slices_fixture()
        bounds = torch.stack([cuts[:, rank], cuts[:, rank + 1]], 1)
        mine_a = torch.full_like(acts, -99)
        mine_f = torch.full_like(fwd, -99.0)
        for b in range(acts.shape[0]):
            s0, e0 = int(bounds[b, 0]), int(bounds[b, 1])
            mine_a[b, s0:e0] = acts[b, s0:e0]
            mine_f[b, s0:e0] = fwd[b, s0:e0]
        ga, gf = gather_slices(mine_a, mine_f, bounds, T)
        out["slices"] = (ga.numpy(), gf.numpy())
        q.put((rank, out))
    finally:
        dist.destroy_process_group()


def _split_fixture():
    g = torch.Generator().manual_seed(3)
    sums = torch.rand(3, 1, 37, generator=g, dtype=torch.float64) * 1e3
    counts = torch.randint(0, 5000, (3, 1, 37), generator=g).double()
    partials = np.random.default_rng(3).random((3, 11)) * np.logspace(-12, 6, 11)  # per-block partials
    return torch.cat([sums, counts], 1), partials


class _Pattern:
    """The attributes distributed.PackPlan / word_spans read from a PreconditionerEnv (CPU
    stand-in); ``perm_seed``: the raw COO entries shuffled, i.e. a numbering whose action ids are
    scattered over the whole bitmap (thermal2's file order, BASELINE C5)."""

    def __init__(self, grid, perm_seed=None):
        r, c, v, n = O.poisson2d(grid)
        if perm_seed is not None:
            o = np.random.default_rng(perm_seed).permutation(len(r))
            r, c, v = r[o], c[o], v[o]
        idx, act, _ = O.lines_from_coo(r, c, v, n, "col")
        self.matrix_size, self.E = n, len(r)
        self.pattern = type("P", (), {"act": torch.from_numpy(act), "idx": torch.from_numpy(idx)})()


def _columns_fixture(world, bl, perm_seed=None):
    env = _Pattern(24, perm_seed)  # 576 lines: 256-line blocks split 2 + 1 over two ranks
    words = (env.E + 31) // 32
    rng = np.random.default_rng(7)
    bits = rng.integers(0, 2 ** 32, size=(world * bl, words), dtype=np.uint64).astype(np.uint32).view(np.int32)
    counts = rng.integers(0, env.E, size=world * bl).astype(np.int32)
    return env, words, torch.from_numpy(bits), torch.from_numpy(counts)


def _columns_exchange(rank, world, bl=3, perm_seed=None, mode="gather"):
    """The columns split's all_to_all: rank r holds candidates r*bl .. and sends every rank q the
    bits of q's line-major action ids packed 32 per word, plus the counts (spai_bitmap_pack,
    restated in torch); it receives every candidate's packed row of its own shard.  mode="auto"
    on a stencil numbering: the word windows instead (spai_window_pack)."""
    env, words, bits, counts = _columns_fixture(world, bl, perm_seed)
    plan = PackPlan(env, world, mode)
    mine = slice(rank * bl, (rank + 1) * bl)
    send = pack_bits_reference(bits[mine], counts[mine], plan, bl)
    assert send.numel() == plan.send_words(bl)
    recv = torch.full((world * bl, plan.wq[rank] + 1), -7, dtype=torch.int32)
    exchange_packed(send, recv, plan, bl, rank).wait()
    return plan.wq, recv.numpy(), plan.mode, getattr(plan, "lo_words", None)


def _unpack_expected(env, bits, lines):
    """[B, m] removal bits of the line-major action ids of lines [b, e) (the receiver's view)."""
    b, e = lines
    a = env.pattern.act[b:e].reshape(-1)
    a = a[a >= 0].long()
    return ((bits[:, a >> 5].long() >> (a & 31)) & 1).numpy()


def _unpack(recv, m):
    w = recv[:, :-1].astype(np.uint32)
    return ((w[:, :, None] >> np.arange(32, dtype=np.uint32)) & 1).reshape(len(recv), -1)[:, :m]


def _slices_fixture():
    g = torch.Generator().manual_seed(4)
    B, T = 3, 50
    acts = torch.randint(0, 1000, (B, T), generator=g)
    fwd = torch.rand(B, T, generator=g)
    cuts = torch.tensor([[0, 20, T], [0, 0, T], [0, 50, T]])  # empty slices at either end too
    return acts, fwd, cuts, T


def test_shard_lines_partition():
    for n in (1, 7, 256, 1048576):
        for world in (1, 2, 3, 8):
            rngs = [shard_lines(n, r, world) for r in range(world)]
            assert rngs[0][0] == 0 and rngs[-1][1] == n
            assert all(rngs[i][1] == rngs[i + 1][0] for i in range(world - 1))
            sizes = [e - b for b, e in rngs]
            assert max(sizes) - min(sizes) <= 1


def test_world2_column_sharded_reward_and_assembly():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # reference: the unsharded computation
    r, c, v, n = O.poisson2d(12, np.float64)
    idx, act, _ = O.lines_from_coo(r, c, v, n, "col")
    a_idx, _, a_val = O.lines_from_coo(r, c, v, n, "col")
    A = sp.csc_matrix((v, (r, c)), shape=(n, n))
    removed = np.random.default_rng(5).random((3, len(r))) < 0.3
    for b in range(3):
        keep = (idx >= 0) & ~removed[b][np.clip(act, 0, None)]
        m = O.lsq_fill(idx, keep, a_idx, a_val)
        full = O.residual_fro_fp64(A, O.m_to_csc(idx, m, n, np.float64)) ** 2
        for rank in (0, 1):
            assert res[rank]["res2"][b] == pytest.approx(full, rel=1e-12)
            np.testing.assert_allclose(res[rank]["m"][b], m, rtol=1e-12, atol=1e-15)
    np.testing.assert_array_equal(res[0]["rewards"], [0, 1, 2, 10, 11, 12])
    blocks = []
    for q_ in (0, 1):
        b0a, b1a = shard_lines(n, q_, 2, LINE_ALIGN)
        blocks.append(torch.arange(2 * (b1a - b0a) * 5, dtype=torch.float32).view(2, b1a - b0a, 5) + 1000 * q_ + 1)
    for rank in (0, 1):  # the second of two pipelined gathers, on every rank
        assert np.array_equal(res[rank]["m_pipe"], torch.cat(blocks, 1).numpy())
        assert np.array_equal(res[rank]["m_row"], torch.cat(blocks, 1).numpy()[1:2])
    full_bs, partials = _split_fixture()
    acts, fwd, _, _ = _slices_fixture()
    env, words, bits, counts = _columns_fixture(2, 3)
    lines = [shard_lines(env.matrix_size, q, 2, LINE_ALIGN) for q in (0, 1)]
    assert lines == [(0, 512), (512, 576)]
    for rank in (0, 1):
        assert np.array_equal(res[rank]["bs"], full_bs.numpy())  # bit-exact: one non-zero term each
        for b in range(3):  # exact sums: the same bits as one process summing every partial
            assert res[rank]["r2"][b] == O.fixed_sum(partials[b])
        wq, recv, mode, _ = res[rank]["cols"]
        b0, b1 = lines[rank]
        m = int((env.pattern.act[b0:b1] >= 0).sum())
        assert mode == "gather" and wq[rank] == (m + 31) // 32 and recv.shape == (6, wq[rank] + 1)
        # every candidate (global order): exactly the bits of this rank's actions, line-major
        assert np.array_equal(_unpack(recv, m), _unpack_expected(env, bits, lines[rank]))
        assert np.array_equal(recv[:, -1], counts.numpy())
        # the stencil numbering's word windows (auto -> window): the rank's contiguous bitmap words,
        # every one of its action ids a read as bit a - 32 lo of the received rows
        wq, recv, mode, lo = res[rank]["cols_win"]
        assert mode == "window" and recv.shape == (6, wq[rank] + 1)
        assert np.array_equal(recv[:, :-1], bits.numpy()[:, lo[rank]:lo[rank] + wq[rank]])
        a = env.pattern.act[b0:b1].reshape(-1)
        a = (a[a >= 0].long() - 32 * lo[rank]).numpy()
        assert a.min() >= 0 and a.max() < 32 * wq[rank]
        assert np.array_equal(_unpack(recv, 32 * wq[rank])[:, a], _unpack_expected(env, bits, lines[rank]))
        assert np.array_equal(recv[:, -1], counts.numpy())
        assert wq[rank] <= 1.25 * ((m + 31) // 32) + 2
        assert np.array_equal(res[rank]["slices"][0], acts.numpy())
        allr, best, mbest = res[rank]["samples"]
        np.testing.assert_array_equal(allr, [0.5, 2.5, 1.5, -1.0])
        assert best == 1
        assert np.array_equal(res[rank]["slices"][1], fwd.numpy())
    np.testing.assert_array_equal(res[0]["samples"][2], np.arange(24, dtype=np.float64).reshape(2, 3, 4)[1])


def test_shard_lines_aligned():
    for n in (1, 255, 256, 576, 1048576, 262144 + 17):
        for world in (1, 2, 3, 8):
            rngs = [shard_lines(n, r, world, LINE_ALIGN) for r in range(world)]
            assert rngs[0][0] == 0 and rngs[-1][1] == n
            assert all(rngs[i][1] == rngs[i + 1][0] for i in range(world - 1))
            assert all(b % LINE_ALIGN == 0 or b == n for b, _ in rngs)


def test_fixed_point_sums_are_partition_invariant():
    """The oracle restatement of the exact residual sums (spai_device.h fixed_add/fixed_value):
    any split of the partials sums to the same bits, close to the fp64 sum, NaN / inf flagged."""
    rng = np.random.default_rng(11)
    x = rng.random(500) * np.logspace(-20, 8, 500)
    x[::7] *= -1
    whole = O.fixed_sum(x)
    assert abs(whole - x.sum()) <= 1e-12 * np.abs(x).sum()
    for cut in (1, 17, 250, 499):
        a = sum(O.fixed_limbs(v).astype(object) for v in x[:cut])
        b = sum(O.fixed_limbs(v).astype(object) for v in x[cut:])
        assert O.fixed_value(a + b) == whole
    assert O.fixed_value(O.fixed_limbs(2.0 ** -100)) == 0.0  # below 2^-96: truncated
    assert O.fixed_value(O.fixed_limbs(1.5) + O.fixed_limbs(float("inf"))) == float("inf")
    assert np.isnan(O.fixed_value(O.fixed_limbs(float("nan")) + O.fixed_limbs(float("inf"))))


def _worker3(rank, world, port, q):
    """Three ranks (a non-power-of-two world): the packed bitmap exchange on a PERMUTED numbering
    (the windows of word_spans would be whole bitmaps there) and the pipelined M gather with the
    256-line-aligned shards GFlowNet uses for both splits (unequal: 1000 lines = 4 blocks, 2+1+1)."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        out = {"cols": _columns_exchange(rank, world, bl=2, perm_seed=3, mode="auto")}  # auto -> gather here
        n = 1000
        b0, b1 = shard_lines(n, rank, world, LINE_ALIGN)
        lg = LineGather(n, align=LINE_ALIGN)
        m = torch.arange(2 * (b1 - b0) * 5, dtype=torch.float32).view(2, b1 - b0, 5) + 1e4 * rank
        lg.start(m)
        lg.start(m + 1)
        out["m"] = lg.result().numpy()
        q.put((rank, out))
    finally:
        dist.destroy_process_group()


def test_world3_packed_exchange_on_permuted_numbering_and_aligned_gather():
    world = 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker3, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    env, words, bits, counts = _columns_fixture(world, 2, perm_seed=3)
    lines = [shard_lines(env.matrix_size, r, world, LINE_ALIGN) for r in range(world)]
    spans = word_spans(env, world)
    for rank in range(world):
        wq, recv, mode, _ = res[rank]["cols"]
        assert mode == "gather"
        m = int((env.pattern.act[lines[rank][0]:lines[rank][1]] >= 0).sum())
        assert np.array_equal(_unpack(recv, m), _unpack_expected(env, bits, lines[rank]))
        assert np.array_equal(recv[:, -1], counts.numpy())
        # ~1/P of each bitmap per rank (its own nnz), where the word windows are ~whole bitmaps
        assert wq[rank] <= -(-env.E // 32) * (lines[rank][1] - lines[rank][0]) // env.matrix_size + 2
        assert spans[rank][1] - spans[rank][0] > 0.9 * words
    blocks = []
    for r in range(world):
        b0, b1 = shard_lines(1000, r, world, LINE_ALIGN)
        blocks.append(torch.arange(2 * (b1 - b0) * 5, dtype=torch.float32).view(2, b1 - b0, 5) + 1e4 * r + 1)
    for rank in range(world):
        assert np.array_equal(res[rank]["m"], torch.cat(blocks, 1).numpy())
