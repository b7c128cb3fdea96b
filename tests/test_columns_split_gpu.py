"""The multi-GPU column split (distributed.py) on the one GPU of the box.

1. In one process, P ranks played by P select calls with their own Philox sample ids, the
   all_to_all played by slicing the send buffers: the per-rank windows + 256-line-aligned line
   shards + integer-limb sums reproduce the one-process batch BIT FOR BIT (bitmaps, counts,
   squared residuals, rewards, M).
2. The product path itself in two processes (gloo on the one GPU, device tensors host-staged
   by distributed.py): GFlowNet(shard=..., split="columns") and split="slices" end to end,
   compared bit for bit with one process rolling out the same candidates.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

DEV = "cuda"


class EdgeLogits(torch.nn.Module):
    """Fixed-logit stand-in with ForwardPolicy's `logits` contract (module level: picklable)."""

    def __init__(self, logits):
        super().__init__()
        self.l = torch.nn.Parameter(torch.as_tensor(logits).view(1, -1).clone(), requires_grad=False)
        self.a = torch.tensor(0.25)

    def logits(self, data):
        return self.l.to(DEV), self.a.to(DEV)


def _logits(E, seed, terminal=1.5):
    lg = torch.randn(E + 1, generator=torch.Generator().manual_seed(seed))
    lg[E] = terminal
    return lg


_ENVS = {}


def _env(kind):
    from gflownet_spai_amd import PreconditionerEnv, axial_pattern_3d, poisson_2d, poisson_3d
    if kind == "c4":  # BASELINE configs[3]: 1024^2 Poisson, fp32, ||AM - I||, LSQ fill (built once)
        if kind not in _ENVS:
            A = poisson_2d(1024)
            _ENVS[kind] = (PreconditionerEnv(A.shape[0], A, A, side="AM", fill="lsq", keep_m=True), A, A)
        return _ENVS[kind]
    if kind == "2d":
        A = poisson_2d(96)
        return PreconditionerEnv(A.shape[0], A, A, side="AM", fill="lsq", keep_m=True), A, A
    if kind == "thermal":  # the C5 stand-in's randomly permuted numbering (fp64, 7 per line), QR fill
        from gflownet_spai_amd import thermal_like
        A = thermal_like(160, 0, torch.float64)
        return PreconditionerEnv(A.shape[0], A, A, side="AM", fill="qr", keep_m=True), A, A
    A = poisson_3d(12)
    P = axial_pattern_3d(12, 2, torch.float64)
    return PreconditionerEnv(A.shape[0], P, A, side="AM", fill="lsq", keep_m=True), P, A


@pytest.mark.parametrize("kind,P,bl,mode", [("2d", 2, 3, "auto"), ("2d", 3, 2, "auto"), ("2d", 8, 1, "auto"),
                                            ("3d", 3, 2, "auto"), ("c4", 2, 1, "auto"), ("c4", 4, 1, "auto"),
                                            ("c4", 8, 1, "auto"), ("c4", 3, 2, "auto"), ("thermal", 8, 1, "auto"),
                                            ("thermal", 3, 2, "auto"), ("2d", 3, 2, "gather"), ("c4", 8, 1, "gather"),
                                            ("c4", 3, 2, "gather")])
def test_columns_split_in_process_bit_identical(kind, P, bl, mode):
    """P ranks in one process (C4 geometry included: 1024^2, E = 5,238,784, P = 2/4/8 with one
    candidate per rank, and P = 3 whose shards are not equal; and the C5 stand-in's randomly
    PERMUTED numbering, whose action ids scatter every shard over the whole bitmap): the packed
    line-major exchange (spai_bitmap_pack == its torch restatement), 256-line shards and the
    shard-local action tables reproduce the one-process batch bit for bit, and every rank receives
    exactly nnz(shard) bits per candidate (~1/P of a bitmap) whatever the numbering.  mode "auto"
    picks the word windows (spai_window_pack, no gather) for the stencil numberings and the packed
    gather for the permuted one; "gather" forces the packed exchange on a stencil."""
    from gflownet_spai_amd import kernels
    from gflownet_spai_amd.distributed import LINE_ALIGN, PackPlan, pack_bits_reference, shard_lines, word_spans
    env, _, _ = _env(kind)
    n, E = env.matrix_size, env.num_actions - 1
    words = (E + 31) // 32
    B = P * bl
    lg, lmax, _ = kernels.logits_stats(_logits(E, 5).to(DEV), B)
    seed, stream = 77, 3
    # one process, the whole batch
    removed1, counts1, _ = kernels.rollout_select(lg, B, lmax, seed, stream)
    res2_1 = env.fill_partial(removed1)
    m1 = env.last_m.clone()
    alpha = torch.tensor(0.4)
    rw1 = env.rewards_from_res2(res2_1, counts1, alpha)
    # P ranks: own candidates, then the all_to_all of packed rows + counts
    plan = PackPlan(env, P, mode)
    # auto: windows for the 2-D stencils (the 12^3 3-D pattern's halo is wide next to its shards:
    # either layout), the gather for the permuted numbering
    want = mode if mode != "auto" else {"thermal": "gather", "3d": plan.mode}.get(kind, "window")
    assert plan.mode == want
    if mode == "auto":
        assert env.pack_plan(P).mode == plan.mode  # the plan the GFlowNet step uses
    sends = []
    for r in range(P):
        sel = torch.empty(bl * words + bl, dtype=torch.int32, device=DEV)
        rm, ct, _ = kernels.rollout_select(lg[: E + 1], bl, lmax[:bl], seed, stream, r * bl, out=sel, ws_tag=f"r{r}")
        assert torch.equal(rm, removed1[r * bl:(r + 1) * bl]) and torch.equal(ct, counts1[r * bl:(r + 1) * bl])
        send = kernels.bitmap_pack(rm, ct, plan)
        assert torch.equal(send, pack_bits_reference(rm, ct, plan, bl))
        sends.append(send)
    nnz = [int(plan.seg[q + 1] - plan.seg[q]) for q in range(P)]
    assert sum(nnz) == E
    for q in range(P):  # exactly the shard's bits (windows: within 1.25x of them): ~1/P of a bitmap per candidate
        b, e = shard_lines(n, q, P, LINE_ALIGN)
        assert nnz[q] == int((env.pattern.act[b:e] >= 0).sum())
        if plan.mode == "gather":
            assert plan.wq[q] == -(-nnz[q] // 32)
    if plan.mode == "window":
        assert sum(plan.wq) <= 1.25 * sum(-(-x // 32) for x in nnz)
    if kind == "thermal":  # the word windows of this numbering would be whole bitmaps
        spans = word_spans(env, P)
        assert all(w1 - w0 > 0.95 * words for w0, w1 in spans)
        assert max(plan.wq) <= words // P + 64
    offs = np.cumsum([0] + [bl * (w + 1) for w in plan.wq])
    limbs, blocks = [], []
    for q in range(P):
        recv = torch.cat([sends[r][offs[q]:offs[q + 1]] for r in range(P)]).view(B, plan.wq[q] + 1)
        assert torch.equal(recv[:, plan.wq[q]], counts1)
        b, e = shard_lines(n, q, P, LINE_ALIGN)
        limbs.append(env.fill_partial(recv, b, e, limbs=True, pattern=plan.local_pattern(env, q)))
        blocks.append(env.last_m.clone())
    res2 = kernels.res2_from_limbs(sum(limbs))
    assert torch.equal(res2, res2_1)  # bit for bit, whatever P and the numbering
    assert torch.equal(torch.cat(blocks, 1), m1)
    assert torch.equal(env.rewards_from_res2(res2, counts1, alpha), rw1)


def test_exact_reduce_matches_oracle_and_shards():
    """spai_fill_reduce's integer-limb sums: the one-launch residuals equal the limbs of any
    256-aligned line partition summed, and the oracle's exact sum of the kernel's partials."""
    from gflownet_spai_amd import kernels
    from gflownet_spai_amd.distributed import LINE_ALIGN, shard_lines
    from oracle import spai_oracle as O
    env, _, _ = _env("2d")
    n, E = env.matrix_size, env.num_actions - 1
    rng = np.random.default_rng(2)
    acts = torch.from_numpy(np.where(rng.random((3, E)) < 0.3, np.arange(E), -1))
    removed, _ = kernels.actions_to_removed(acts.to(DEV), E)
    whole = env.fill_partial(removed)
    for P in (2, 5, 7):
        lb = sum(env.fill_partial(removed, *shard_lines(n, q, P, LINE_ALIGN), limbs=True) for q in range(P))
        assert torch.equal(kernels.res2_from_limbs(lb), whole)
    # the per-block partials the kernel sums (workspace after a fill over all lines)
    lim = env.fill_partial(removed, limbs=True)
    ws = torch.empty(0)
    from gflownet_spai_amd import _lib
    ws = _lib._ws_cache[("fill", str(removed.device), torch.cuda.current_stream().cuda_stream)]
    nparts = -(-n // 256)
    partials = ws[: 8 * 3 * nparts].view(torch.float64).view(3, nparts).cpu().numpy()
    for b in range(3):
        assert float(whole[b]) == O.fixed_sum(partials[b])
        assert np.array_equal(lim[b].cpu().numpy(), sum(O.fixed_limbs(x) for x in partials[b]).astype(np.int64))


# ---------------------------------------------------------------- two processes, gloo, one GPU
def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _by_value(x, back=False):
    """Tensors <-> numpy arrays through the result queue: numpy pickles by value, while CPU
    tensors travel as shared-memory file descriptors that a rank which has already exited can no
    longer hand over (a race that failed this test once)."""
    if isinstance(x, dict):
        return {k: _by_value(v, back) for k, v in x.items()}
    if back and isinstance(x, np.ndarray):
        return torch.from_numpy(x)
    if not back and isinstance(x, torch.Tensor):
        return x.numpy()
    return x


def _rccl_world1_main(port, q):
    """RCCL (backend "nccl") with one rank: the device-tensor branch of every collective the splits
    use (no host staging), on the dtypes and shapes they send."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1")
    import torch.distributed as dist
    from gflownet_spai_amd.distributed import (LINE_ALIGN, LineGather, all_reduce_, allgather_lines,
                                               exchange_bitmaps, select_best_samples)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", device_id=dev)
    out = {"backend": dist.get_backend()}
    try:
        bl, w0, w1 = 3, 5, 40
        send = torch.arange(bl * (w1 - w0 + 1), dtype=torch.int32, device=dev)
        recv = torch.empty(bl, w1 - w0 + 1, dtype=torch.int32, device=dev)
        exchange_bitmaps(send, recv, [(w0, w1)], bl, 0, async_op=True).wait()
        out["a2a"] = bool(torch.equal(recv.view(-1), send))
        limbs = torch.arange(8 * bl, dtype=torch.int64, device=dev).view(bl, 8) * (1 << 40)
        ref = limbs.clone()
        all_reduce_(limbs)
        out["allreduce"] = bool(torch.equal(limbs, ref))
        n = 1000
        m = torch.randn(bl, n, 5, device=dev)
        lg = LineGather(n, align=LINE_ALIGN)
        lg.start(m)
        lg.start(m * 2)  # the second waits for the first before reusing its buffers
        out["allgather"] = bool(torch.equal(allgather_lines(m, n, align=LINE_ALIGN), m)
                                and torch.equal(lg.result(), m * 2))
        rw = torch.tensor([0.5, 2.0, 1.0], dtype=torch.float64, device=dev)
        r, best, mb = select_best_samples(rw, m)
        out["best"] = bool(torch.equal(r, rw) and int(best) == 1 and torch.equal(mb, m[1]))
        torch.cuda.synchronize()
    finally:
        dist.destroy_process_group()
    q.put(out)


def test_rccl_one_rank_collectives():
    """The RCCL branch of the split collectives (all_to_all_single with uneven splits, int64
    all_reduce, all_gather_into_tensor, the samples split's all_gather + reduce) executed on the
    GPU with one rank: two ranks cannot share one GPU under RCCL (duplicate-GPU check), so the
    multi-rank tests above run gloo; this is the device-tensor path they skip."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_rccl_world1_main, args=(_free_port(), q))
    p.start()
    out = q.get(timeout=240)
    p.join(timeout=60)
    assert p.exitcode == 0
    assert out == {"backend": "nccl", "a2a": True, "allreduce": True, "allgather": True, "best": True}, out


def _rank_main(rank, world, port, bl, q):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from gflownet_spai_amd import GFlowNet
        from gflownet_spai_amd.distributed import LINE_ALIGN, allgather_lines
        env, Pm, _ = _env("2d")
        E = env.num_actions - 1
        pol = EdgeLogits(_logits(E, 9)).to(DEV)
        out = {}
        with torch.no_grad():
            g = GFlowNet(pol, None, env, mode="throughput", seed=21, shard=(rank, world, None), split="columns")
            logs = [g.sample_states([Pm] * bl, return_log=True) for _ in range(2)]  # two steps: streams 0, 1
            log = logs[-1]
            best = torch.argmax(log.rewards_all).view(1)
            m = allgather_lines(env.last_m.index_select(0, best), env.matrix_size, align=LINE_ALIGN)
            out["columns"] = dict(rewards_all=log.rewards_all.cpu(), rewards=log.rewards.cpu(),
                                  actions=log.actions.cpu(), fwd=log.fwd_probs.cpu(), m_best=m.cpu(),
                                  best=int(best), residual=env.last_residual.cpu(), rollouts=g.rollouts)
            gs = GFlowNet(pol, None, env, mode="throughput", seed=21, shard=(rank, world, None), split="slices")
            log = gs.sample_states([Pm] * (world * bl), return_log=True)
            try:
                log.actions
                out["slices_guard"] = False
            except RuntimeError:
                out["slices_guard"] = True  # the full log needs the explicit collective
            log.gather_parts()
            out["slices"] = dict(rewards=log.rewards.cpu(), actions=log.actions.cpu(), fwd=log.fwd_probs.cpu())
        q.put((rank, _by_value(out)))
    finally:
        dist.destroy_process_group()


def test_two_processes_columns_and_slices_match_one_process():
    from gflownet_spai_amd import GFlowNet
    world, bl = 2, 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, world, port, bl, q)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        res = {r: _by_value(o, back=True) for r, o in (q.get(timeout=240) for _ in procs)}
    finally:
        for p in procs:
            p.join(timeout=60)
    assert all(p.exitcode == 0 for p in procs)
    # one process rolling out the same P*bl candidates (sample ids 0 .. P*bl-1), two steps
    env, Pm, _ = _env("2d")
    E = env.num_actions - 1
    pol = EdgeLogits(_logits(E, 9)).to(DEV)
    with torch.no_grad():
        g1 = GFlowNet(pol, None, env, mode="throughput", seed=21)
        logs = [g1.sample_states([Pm] * (world * bl), return_log=True) for _ in range(2)]
    one = logs[-1]
    rw = one.rewards_all.cpu()
    for r in range(world):
        c = res[r]["columns"]
        assert torch.equal(c["rewards_all"], rw)
        assert torch.equal(c["rewards"], one.rewards.cpu()[r * bl:(r + 1) * bl])
        assert torch.equal(c["residual"], env.last_residual.cpu())
        mine = slice(r * bl, (r + 1) * bl)
        a1 = one.actions.cpu()[:, mine]
        T = int((a1 >= 0).sum(0).max())
        assert torch.equal(c["actions"][:T], a1[:T]) and bool((c["actions"][T:] == -1).all())
        assert torch.equal(c["fwd"][:, :T], one.fwd_probs.cpu()[mine, :T])
        assert c["best"] == int(torch.argmax(rw))
        assert torch.equal(c["m_best"][0], env.last_m[c["best"]].cpu())
        assert c["rollouts"] == 2
        s = res[r]["slices"]
        assert res[r]["slices_guard"]
        assert torch.equal(s["actions"], res[0]["slices"]["actions"])
    # the slices split draws the one-process candidates of ITS first rollout (stream 0)
    with torch.no_grad():
        g0 = GFlowNet(pol, None, env, mode="throughput", seed=21)
        ref = g0.sample_states([Pm] * (world * bl), return_log=True)
    for r in range(world):
        s = res[r]["slices"]
        assert torch.equal(s["actions"], ref.actions.cpu())
        assert torch.equal(s["fwd"], ref.fwd_probs.cpu())
        assert torch.equal(s["rewards"], ref.rewards.cpu())
