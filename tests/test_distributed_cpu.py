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

from gflownet_spai_amd.distributed import (allgather_lines, allreduce_res2, exchange_parts, gather_rewards,
                                           gather_slices, select_best_samples, shard_lines)
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
        out["rewards"] = gather_rewards(torch.arange(B, dtype=torch.float64) + 10 * rank).numpy()
        # the split rollout's exchange: each part fills the bucket weight sums and winner counts
        # of its own bucket range (zero elsewhere, the exchange array's [B][2][kMaxB] layout)
        # and its lines' residual partials go into the B trailing slots; one all_reduce in place
        full_bs, full_r2 = _split_fixture()
        B3, nb = full_bs.shape[0], full_bs.shape[2]
        k0, k1 = nb * rank // world, nb * (rank + 1) // world
        xch = torch.zeros(full_bs.numel() + B3, dtype=torch.float64)
        bs = xch[:full_bs.numel()].view_as(full_bs)
        bs[:, :, k0:k1] = full_bs[:, :, k0:k1]
        r2 = full_r2 * (0.25 if rank == 0 else 0.75)
        out["r2"] = exchange_parts(xch, r2).clone().numpy()
        out["bs"] = bs.numpy()
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
    return torch.cat([sums, counts], 1), torch.rand(3, generator=g, dtype=torch.float64)


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
    full_bs, full_r2 = _split_fixture()
    acts, fwd, _, _ = _slices_fixture()
    for rank in (0, 1):
        assert np.array_equal(res[rank]["bs"], full_bs.numpy())  # bit-exact: one non-zero term each
        np.testing.assert_allclose(res[rank]["r2"], full_r2.numpy(), rtol=1e-15)
        assert np.array_equal(res[rank]["slices"][0], acts.numpy())
        allr, best, mbest = res[rank]["samples"]
        np.testing.assert_array_equal(allr, [0.5, 2.5, 1.5, -1.0])
        assert best == 1
        assert np.array_equal(res[rank]["slices"][1], fwd.numpy())
    np.testing.assert_array_equal(res[0]["samples"][2], np.arange(24, dtype=np.float64).reshape(2, 3, 4)[1])
