"""Drop-in ``GFlowNet`` (reference: gflownet/gflownet.py:12-257) with the MI355X sampler.

``sample_states(s0, return_log=True) -> Log`` keeps the reference's contract.  The
policy's logits are state-independent within a rollout (gflownet.py:133,145: data_list
is built once from s0 and only the action mask changes), so they are produced ONCE per
rollout and the T-step loop runs on the device:

  mode="parity"     the reference's sampler step for step: per step B*(E+1) Exp(1) noise
                    from the torch CPU generator (exactly what Categorical(probs).sample()
                    draws, gflownet.py:148) and one fused masked-argmax kernel; bit-exact
                    actions vs the reference given the same torch seed.  O(T*B*E).
  mode="throughput" one-pass Gumbel-top-k (Philox, no host noise): all trajectories in
                    O(B*E) — distributionally identical to the sequential sampler.
Then ``env.update`` semantics: removal bitmaps -> fill -> residual -> rewards.
"""
from __future__ import annotations

import contextlib
from typing import List

import torch
from torch import Tensor, nn

from . import kernels
from .log import Log, trajectory_probs
from .preconditioner import Data


class GFlowNet(nn.Module):
    def __init__(self, forward_policy, backward_policy, env, *, mode: str = "parity", seed: int | None = None,
                 sample_base: int = 0, shard: tuple | None = None, split: str | None = None,
                 overlap: bool | str = "sort", pipeline: bool = False):
        super().__init__()
        if mode not in ("parity", "throughput"):
            raise ValueError("mode must be 'parity' or 'throughput'")
        if split not in (None, "columns", "slices"):
            raise ValueError("split must be 'columns' or 'slices'")
        self.register_buffer("total_flow", torch.ones(1))
        self.forward_policy = forward_policy
        self.backward_policy = backward_policy
        self.env = env
        self.mode = mode
        self._alpha_mean = None  # (key, mean over the batch of a constant sigmoid(alpha), pin)
        self.seed = int(torch.initial_seed() if seed is None else seed) & (2**64 - 1)
        self.sample_base = sample_base
        self._rollouts0 = 0  # Philox stream id of the first throughput rollout
        self._ctr = None     # the stream id on the device (advanced by the select phase itself)
        self._data_cache = {}
        self._bufs = {}      # persistent exchange buffers of the columns split (graph-replay safe)
        # one GPU, throughput mode: run the fill + rewards on a second stream beside the trajectory
        # sort (the two chains share only the select phase's outputs); "sort" / True: the sort is
        # launched first, "fill": the fill first, False: one stream, fill then sort
        if overlap not in (False, True, "sort", "fill", "select"):
            raise ValueError("overlap must be False, True, 'sort', 'fill' or 'select'")
        self.overlap = "sort" if overlap is True else overlap
        self._side = None
        # pipeline=True (one GPU, throughput mode, a fixed policy): consecutive steps alternate
        # between two stream lanes, and step k+1 waits only for step k's select phase (the Philox
        # stream counter it advances), so its policy and select run beside step k's sort, fill and
        # padding.  Every step still does all of its work, in the same order within the step, on
        # buffers of its own lane.  The lanes are forked from the caller's stream once; results are
        # complete after pipeline_join() (or a device synchronisation).
        self.pipeline = bool(pipeline)
        self._pl = None
        # (rank, world, group): the multi-GPU split of DESIGN.md §6 (throughput mode)
        #   split="columns": rank r rolls out its own len(s0) candidates (global sample ids
        #     sample_base + r*len(s0) ..), one all_to_all ships each rank the bitmap words of its
        #     256-line-aligned column shard for EVERY candidate, every rank fills its lines of all
        #     P*len(s0) candidates, one all_reduce sums the exact residual limbs (distributed.py).
        #   split="slices": every rank draws the same B candidates and orders one slice of every
        #     trajectory; one all_reduce of the bucket sums + residual partials.
        #   The two splits read s0 differently (this rank's candidates vs the whole batch), so a
        #   sharded GFlowNet must name its split: an old slices-era call site fails loudly.
        # a one-rank shard is dropped (the one-GPU step) unless a split is named explicitly: then
        # the split's phases run with their collectives on a one-rank group (bench.py --dist)
        self.shard = shard if shard is not None and (shard[1] > 1 or split is not None) else None
        if self.shard is not None and split is None:
            raise ValueError("a sharded GFlowNet needs split='columns' (s0 = this rank's own candidates) or "
                             "split='slices' (s0 = the whole batch on every rank); INTEGRATION.md §4")
        self.split = split if self.shard is not None else None
        if self.shard is not None:
            if mode != "throughput":
                raise ValueError("a sharded GFlowNet needs mode='throughput'")
            from .distributed import LINE_ALIGN, shard_lines
            rank, world, _ = self.shard
            # 256-line-aligned shards for both splits: the per-block fp64 partials of the fill
            # start at the shard's first line, so only aligned shards sum to one GPU's bits
            self.lines = shard_lines(env.matrix_size, rank, world, LINE_ALIGN) if env is not None else None

    @property
    def rollouts(self) -> int:
        """Philox stream id of the next throughput rollout.  The device counter is the only source
        of truth once a rollout ran (graph replays advance it without the host): reading it syncs."""
        return self._rollouts0 if self._ctr is None else int(self._ctr.item())

    @rollouts.setter
    def rollouts(self, value: int) -> None:
        self._rollouts0 = int(value)
        if self._ctr is not None:
            self._ctr.fill_(int(value))  # replays from here draw stream ids value, value + 1, ...

    # ------------------------------------------------------------------ policy
    def policy_logits(self, data, batch_size: int, defer_max: bool = False):
        """(logits [E+1] fp32, alpha 0-d, lmax [B] or None) for this rollout.

        Uses ``forward_policy.logits_and_max(data, B)`` (ForwardPolicy here: the gfx950
        kernels also return the logits' maximum), else ``.logits(data)``, else the reference
        call contract ``forward(data, empty)`` -> probs and logits = log(probs) (a constant
        shift, irrelevant to sampling).  alpha is the mean of the B per-sample
        sigmoid(alpha) values, as gflownet.py:89."""
        lmax = None
        if hasattr(self.forward_policy, "logits_and_max"):
            if defer_max:  # (the throughput rollout's select forms the maximum: kernels.PendingMax)
                logits, a, lmax = self.forward_policy.logits_and_max(data, batch_size, defer_max=True)
            else:
                logits, a, lmax = self.forward_policy.logits_and_max(data, batch_size)
        elif hasattr(self.forward_policy, "logits"):
            logits, a = self.forward_policy.logits(data)
        else:
            probs, a = self.forward_policy(data, torch.empty(0, dtype=torch.long))
            logits = torch.log(probs)
        if a.requires_grad or a._version != 0:
            alpha = torch.stack([a] * batch_size, dim=0).mean()
        else:  # a constant (the policy's cached sigmoid): its batch mean is cached with it
            key = (id(a), a.data_ptr(), batch_size)
            hit = self._alpha_mean
            if hit is None or hit[0] != key:
                hit = self._alpha_mean = (key, torch.stack([a] * batch_size, dim=0).mean(), a)  # a pins the id
            alpha = hit[1]
        return logits.reshape(-1), alpha, lmax

    def forward_probs(self, s, data_list, actions=None):
        """gflownet.py:47-123 (reference API; per-sample policy calls, not the hot path)."""
        if actions is None or len(actions) == 0:
            actions = torch.empty(0)
        else:
            actions = torch.stack(list(actions), dim=1) if torch.is_tensor(actions[0]) else torch.tensor(actions).t()
        probs, alphas = [], []
        for i, data in enumerate(data_list):
            act = actions[i, :] if actions.numel() > 0 else torch.empty(0, dtype=torch.long)
            p, a = self.forward_policy(data, act)
            probs.append(p)
            alphas.append(a)
        probs = torch.stack(probs, dim=0)
        if probs.size(0) > 1:
            tot = probs.sum(2)
            tot[tot == 0] = 1
            probs = probs / tot.unsqueeze(1)
        return probs, torch.stack(alphas, dim=0).mean()

    def state_to_data(self, s: List[Tensor]) -> list:
        """gflownet.py:223-257: one Data(x=ones(2N,1), edge_index, edge_attr) per state."""
        out = []
        for i, m in enumerate(s):
            if not m.is_sparse:
                raise ValueError(f"Tensor at index {i} is not a sparse tensor.")
            key = (m._indices().data_ptr(), m._values().data_ptr(), m._nnz(), self.env.matrix_size)
            hit = self._data_cache.get(key)
            if hit is None:  # states are never modified by a rollout: build each graph once
                dev = self.env.device
                d = Data(x=torch.ones((self.env.matrix_size * 2, 1), device=dev),
                         edge_index=m._indices().to(dev), edge_attr=m._values().float().to(dev))
                hit = self._data_cache[key] = (m, d)  # holding m pins its storage (key stays unique)
                if len(self._data_cache) > 8:
                    self._data_cache.pop(next(iter(self._data_cache)))
            out.append(hit[1])
        return out

    def _same_states(self, s0) -> bool:
        """True when every initial state is the same matrix (the drivers pass clones of one
        matrix, GFlowNet100.py:276): same storage, or equal indices and values (compared once per
        set of storages and versions).  Then one policy call serves every sample (the logits
        depend on the state only)."""
        key = tuple((m._indices().data_ptr(), m._values().data_ptr(), m._values()._version, m._nnz())
                    if m.is_sparse else id(m) for m in s0)
        memo = getattr(self, "_same_memo", None)
        if memo is not None and memo[0] == key:
            return memo[1]
        same = self._compare_states(s0)
        self._same_memo = (key, same, list(s0))  # the list pins the storages the key names
        return same

    @staticmethod
    def _compare_states(s0) -> bool:
        m0 = s0[0]
        for m in s0[1:]:
            if m is m0:
                continue
            if not (m.is_sparse and m0.is_sparse) or m.shape != m0.shape or m._nnz() != m0._nnz():
                return False
            i0, v0, i1, v1 = m0._indices(), m0._values(), m._indices(), m._values()
            if i0.data_ptr() == i1.data_ptr() and v0.data_ptr() == v1.data_ptr():
                continue
            if not (torch.equal(i0, i1.to(i0.device)) and torch.equal(v0, v1.to(v0.device))):
                return False
        return True

    def _rewards(self, removed, counts, alpha):
        return self.env.rewards_from_removed(removed, counts, alpha)

    # ------------------------------------------------------------------ sampler
    def sample_states(self, s0, return_log: bool = False):
        """gflownet.py:125-197: sample B trajectories from the initial states, score them, log."""
        if self.mode == "throughput":
            st = {"s0": s0}
            for phase, kind in self.rollout_phases():
                self.run_phase(phase, kind, st)
            return st["log"] if return_log else None
        env = self.env
        B = len(s0)
        E = env.num_actions - 1
        log = Log(s0, self.backward_policy, self.total_flow, env)
        logits, alpha, lg, lmax, z = self._logits(s0, need_z=True)
        actions_bt, fwd_bt = self._parity_rollout(lg, B, lmax, z)
        removed, counts = kernels.actions_to_removed(actions_bt, E)
        self._rewards(removed, counts, alpha)
        log._set_rollout(logits, actions_bt, fwd_bt, lmax=lmax)
        log.removed, log.counts = removed, counts
        log.rewards = env.last_reward32
        return log if return_log else None

    def _logits(self, s0, need_z: bool = False, defer_max: bool = False):
        """(logits, alpha, sampler logits fp32 on the device, lmax [B], z [B] or None).  defer_max:
        lmax may come back as a kernels.PendingMax (the ForwardPolicy's fc block maxima, no reduction
        launch), which kernels.rollout_select completes."""
        env = self.env
        B = len(s0)
        E = env.num_actions - 1
        if self._same_states(s0):
            data_list = self.state_to_data(s0[:1])
            defer = (defer_max and not need_z and not torch.is_grad_enabled()
                     and getattr(self.forward_policy, "supports_defer_max", False))
            logits, alpha, lmax = self.policy_logits(data_list[0], B, defer_max=defer)
            if logits.numel() != E + 1:
                raise ValueError(f"policy produced {logits.numel()} logits for {E + 1} actions")
        else:
            # distinct initial states: one policy call per sample (gflownet.py:70-74 builds one
            # Data per sample), per-sample logit rows [B, E+1] for the sampler
            rows, alphas = [], []
            for d in self.state_to_data(s0):
                l, a, _ = self.policy_logits(d, 1)
                if l.numel() != E + 1:
                    raise ValueError(f"policy produced {l.numel()} logits for {E + 1} actions")
                rows.append(l)
                alphas.append(a)
            logits, alpha, lmax = torch.stack(rows, 0), torch.stack(alphas).mean(), None
        if lmax is not None and not need_z and logits.is_cuda and logits.dtype == torch.float32:
            return logits, alpha, logits.detach(), lmax, None  # the policy kernels produced the maximum
        lg, lmax, z = kernels.logits_stats(logits.detach().to(env.device), B)
        return logits, alpha, lg, lmax, z

    # ------------------------------------------------------------------ throughput step
    # The throughput step as a list of phases (``rollout_phases``), so a caller can capture the
    # collective-free ones in HIP graphs (bench.py).  No phase synchronises with the host; the
    # Philox stream id lives on the device and the select phase advances it, so a replayed graph
    # draws a fresh rollout.  Every phase takes the step's state dict (``{"s0": s0}`` to start;
    # the last phase leaves the Log in ``st["log"]``).
    # Phase kinds: False = device work on the current stream; True = a collective (eager under
    # bench.py's graphs); "side" = device work on the side stream, forked from the current stream at
    # its position; "join" = device work on the current stream after the side stream's work.  A
    # "side" phase is a graph segment of its own, replayed on the side stream, so it runs beside the
    # collectives and device phases between it and the join.
    def rollout_phases(self) -> list:
        """[(phase, kind)] in execution order."""
        if self.split == "columns":
            return [(self._c_select, False), (self._c_pack, False), (self._c_order, "side"), (self._c_send, True),
                    (self._c_recv, True), (self._c_fill, False), (self._c_reduce, True), (self._c_end, "join")]
        if self.split == "slices":
            return [(self._begin, False), (self.rollout_exchange, True), (self._end, False)]
        return [(self._begin, False), (self.rollout_exchange, False), (self._end, False)]

    def run_phase(self, fn, kind, st: dict, timer: str | None = None) -> None:
        """Run one phase eagerly with its kind's stream order (timer: kernels._timed name, recorded
        on the stream the phase runs on)."""
        tm = kernels._timed(timer) if timer else contextlib.nullcontext()
        if kind == "side":
            dev = st["dev"]
            side = self._side_stream(dev)
            side.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(side), tm:
                fn(st)
            return
        if kind == "join":
            torch.cuda.current_stream(st["dev"]).wait_stream(self._side_stream(st["dev"]))
        with tm:
            fn(st)

    def _fork_fill(self, st: dict) -> None:
        """fill + rewards of all lines on the side stream, after everything the current stream has
        issued (the select phase, and with overlap="sort" the trajectory sort's launch) — or, with
        overlap="select", after the select phase only (its event), though issued after the sort."""
        dev = st["lg"].device
        side = st["lane"][1] if "lane" in st else self._side_stream(dev)
        ev = st.pop("select_done", None)
        if ev is not None:
            side.wait_event(ev)
        else:
            side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side):
            st["rewards"] = self.env.fill_rewards(st["removed"], st["counts"], st["alpha"])
        st["join"] = side

    def _side_stream(self, dev):
        if self._side is None or self._side.device != dev:
            # high priority: HIP multiplexes streams onto GPU_MAX_HW_QUEUES (4) hardware queues, and a
            # default-priority stream can land on the current stream's queue, where its work runs
            # strictly after everything queued before it (measured: the columns split's sort, no
            # overlap); a high-priority stream gets a queue of its own
            self._side = torch.cuda.Stream(dev, priority=-1)
        return self._side

    def _counter(self, dev):
        if self._ctr is None or self._ctr.device != dev:
            self._ctr = torch.tensor([self._rollouts0], dtype=torch.int64, device=dev)
        return self._ctr

    def _buf(self, key, shape, dtype, dev):
        t = self._bufs.get(key)
        if t is None or t.shape != torch.Size(shape) or t.dtype != dtype or t.device != dev:
            t = self._bufs[key] = torch.empty(shape, dtype=dtype, device=dev)
        return t

    # one GPU, or the slices split
    def rollout_begin(self, s0) -> dict:
        st = {"s0": s0}
        self._begin(st)
        return st

    def _lane(self, dev):
        """The pipelined step's lane: (stream, side stream), alternating per step, forked from the
        caller's stream (under graph capture only lanes that carry work are forked and joined)."""
        pl = self._pl
        if pl is None or pl["dev"] != dev:
            mk = lambda: torch.cuda.Stream(dev, priority=-1)  # (own hardware queues: see _side_stream)
            pl = self._pl = {"dev": dev, "lanes": [(mk(), mk()), (mk(), mk())], "i": 0, "sel": None, "used": []}
        p = pl["i"]
        pl["i"] ^= 1
        lane = pl["lanes"][p]
        # every dependency between lanes goes through the caller's stream: it waits for the previous
        # step's select, and the lane forks from it (HIP's stream capture crashed on lanes waiting
        # on each other's events directly, scripts/pipeline_capture_diag.py); the caller's stream
        # carries no work of its own in between, so the lanes still overlap
        cur = torch.cuda.current_stream(dev)
        if pl["sel"] is not None:
            cur.wait_event(pl["sel"])
        lane[0].wait_stream(cur)
        if p not in pl["used"]:
            pl["used"].append(p)
        return lane

    def pipeline_join(self) -> None:
        """The caller's stream waits for every pipelined step issued so far (required before a
        graph capture ends and before the host reads a pipelined step's results)."""
        pl = self._pl
        if pl is None:
            return
        cur = torch.cuda.current_stream(pl["dev"])
        for p in pl["used"]:  # (each step joins its fill's side stream into its lane)
            cur.wait_stream(pl["lanes"][p][0])
        pl["used"] = []
        pl["sel"] = None

    def _begin(self, st: dict) -> None:
        if self.pipeline and self.mode == "throughput" and self.shard is None:
            ln, sd = self._lane(torch.device(self.env.device))  # (after the previous step's select: the
            pl = self._pl                                         # stream counter it advances)
            # (no second-level fork: HIP's stream capture fails on a stream forked from a forked stream
            # — scripts/pipeline_capture_diag.py — so a lane runs its fill after its sort, in order,
            # and the concurrency comes from the other lane's step)
            st["lane"] = (ln, sd)
            st["no_fork"] = True
            with torch.cuda.stream(ln):
                self._begin_body(st)
                ev = torch.cuda.Event()
                ev.record(ln)
                pl["sel"] = ev
            return
        self._begin_body(st)

    def _begin_body(self, st: dict) -> None:
        env, s0 = self.env, st["s0"]
        B = len(s0)
        E = env.num_actions - 1
        logits, alpha, lg, lmax, _ = self._logits(s0, defer_max=True)
        rank, world, group = self.shard if self.shard is not None else (0, 1, None)
        removed, counts, ws = kernels.rollout_select(lg, B, lmax, self.seed, 0, self.sample_base, self._counter(lg.device),
                                                     rank, world)
        if isinstance(lmax, kernels.PendingMax):
            lmax = lmax.out  # written by the select
        st.update(B=B, E=E, logits=logits, alpha=alpha, lg=lg, lmax=lmax, removed=removed, counts=counts, ws=ws,
                  part=(rank, world, group))
        if world == 1:  # all lines here: fill, exact sums and rewards (one launch after the fill)
            if st.get("no_fork"):
                st["fill_after_sort"] = "inline"
            elif self.overlap == "fill":
                # the fill needs only the removal bitmaps and the sort only the staged records: the
                # fill + rewards run on a second stream beside rollout_sort / rollout_finish (under
                # HIP-graph capture: two parallel branches), joined in _end
                self._fork_fill(st)
            elif self.overlap:  # "sort": the same branches, the sort launched first (_end forks the fill)
                st["fill_after_sort"] = True
                if self.overlap == "select":  # the fill depends on the select only, issued after the sort
                    ev = torch.cuda.Event()
                    ev.record(torch.cuda.current_stream(lg.device))
                    st["select_done"] = ev
            else:
                st["rewards"] = env.fill_rewards(removed, counts, alpha)
        else:  # a split sums exact limbs of its lines
            st["res2_part"] = env.fill_partial(removed, *self.lines, limbs=True)

    def rollout_exchange(self, st: dict) -> None:
        """The slices split's ONE all_reduce, in place on the rollout workspace's exchange array:
        the parts' bucket weight sums and winner counts (disjoint supports: the sum is exact and
        equals the one-GPU array) and the lines' exact residual limbs (the same bits as one GPU).
        Nothing on one GPU."""
        rank, world, group = st["part"]
        if world == 1:
            return
        from .distributed import exchange_parts
        limbs = exchange_parts(kernels.exchange_array(st["ws"], st["E"], st["B"]), st["res2_part"], group)
        st["res2"] = kernels.res2_from_limbs(limbs)

    def rollout_end(self, st: dict) -> Log:
        self._end(st)
        return st["log"]

    def _end(self, st: dict) -> None:
        if "lane" in st:
            with torch.cuda.stream(st["lane"][0]):
                self._end_body(st)
            return
        self._end_body(st)

    def _end_body(self, st: dict) -> None:
        env = self.env
        rank, world, group = st["part"]
        B, E, lg, lmax, counts, ws = st["B"], st["E"], st["lg"], st["lmax"], st["counts"], st["ws"]
        if world > 1:  # counts, T and the bucket positions need every part's buckets
            kernels.rollout_merge(lg, B, lmax, ws, rank, world, counts)
        actions, fwd = kernels.rollout_sort(lg, B, lmax, ws, rank, world)
        fas = st.pop("fill_after_sort", False)
        if fas == "inline":  # (pipelined lane: the fill in order after the sort)
            st["rewards"] = env.fill_rewards(st["removed"], st["counts"], st["alpha"])
        elif fas:
            self._fork_fill(st)
        t_dev = kernels.rollout_finish(lg, B, lmax, counts, ws, actions, fwd, rank, world)
        if "join" in st:  # the fill's stream (rollout_begin) rejoins before anything reads its outputs
            torch.cuda.current_stream(lg.device).wait_stream(st.pop("join"))
        rewards = st["rewards"] if world == 1 else env.rewards_from_res2(st["res2"], counts, st["alpha"])
        log = Log(st["s0"], self.backward_policy, self.total_flow, env)
        log._set_rollout(st["logits"], actions, fwd, t_dev, lmax=lmax)
        if world > 1:
            log._set_part(rank, world, group, kernels.part_bounds(ws, E, B, rank, world))
        log.removed, log.counts = st["removed"], counts
        log.rewards = env.last_reward32
        log.rewards_all = rewards
        st["log"] = log

    # the columns split: rollouts by candidates, fill + residual by column shards
    def _c_select(self, st: dict) -> None:
        env, s0 = self.env, st["s0"]
        rank, world, group = self.shard
        bl = len(s0)
        E = env.num_actions - 1
        words = (E + 31) // 32
        logits, alpha, lg, lmax, _ = self._logits(s0, defer_max=True)
        dev = lg.device
        sel = self._buf("select" + st.get("bt", ""), (bl * words + bl,), torch.int32, dev)
        removed, counts, ws = kernels.rollout_select(lg, bl, lmax, self.seed, 0, self.sample_base + rank * bl,
                                                     self._counter(dev), out=sel)
        if isinstance(lmax, kernels.PendingMax):
            lmax = lmax.out  # written by the select
        st.update(B=bl, E=E, logits=logits, alpha=alpha, lg=lg, lmax=lmax, removed=removed, counts=counts, ws=ws,
                  dev=dev, part=(rank, world, group))

    def _c_pack(self, st: dict) -> None:
        rank, world, _ = st["part"]
        bl, dev = st["B"], st["dev"]
        plan = self.env.pack_plan(world)
        send = self._buf("send" + st.get("bt", ""), (plan.send_words(bl),), torch.int32, dev)
        kernels.bitmap_pack(st["removed"], st["counts"], plan, out=send)  # line-major packed bits per destination
        recv = self._buf("recv" + st.get("bt", ""), (world * bl, plan.wq[rank] + 1), torch.int32, dev)
        st.update(send=send, recv=recv, plan=plan)

    def _c_send(self, st: dict) -> None:
        from .distributed import exchange_packed
        rank, _, group = st["part"]
        st["a2a"] = exchange_packed(st["send"], st["recv"], st["plan"], st["B"], rank, group, async_op=True)

    def _c_order(self, st: dict) -> None:
        # this rank's own trajectories (side stream), beside the exchange and the fill
        B, lg, lmax, ws = st["B"], st["lg"], st["lmax"], st["ws"]
        actions, fwd = kernels.rollout_sort(lg, B, lmax, ws, 0, 1)
        st["traj"] = (actions, fwd, kernels.rollout_finish(lg, B, lmax, st["counts"], ws, actions, fwd, 0, 1))

    def _c_recv(self, st: dict) -> None:
        st.pop("a2a").wait()

    def _c_fill(self, st: dict) -> None:
        rank = st["part"][0]
        plan, recv = st["plan"], st["recv"]
        st["limbs"] = self.env.fill_partial(recv, *self.lines, limbs=True, pattern=plan.local_pattern(self.env, rank))
        st["counts_all"] = recv[:, plan.wq[rank]].contiguous()

    def _c_reduce(self, st: dict) -> None:
        from .distributed import all_reduce_
        all_reduce_(st["limbs"], st["part"][2])

    def _c_end(self, st: dict) -> None:
        env = self.env
        rank, world, group = st["part"]
        bl = st["B"]
        res2 = kernels.res2_from_limbs(st["limbs"])
        rewards = env.rewards_from_res2(res2, st["counts_all"], st["alpha"])  # all P*bl candidates
        actions, fwd, t_dev = st["traj"]
        log = Log(st["s0"], self.backward_policy, self.total_flow, env)
        log._set_rollout(st["logits"], actions, fwd, t_dev, lmax=st["lmax"])
        removed, counts = st["removed"], st["counts"]
        if not torch.cuda.is_current_stream_capturing():
            # views into the persistent exchange buffer: copied, so a later step cannot overwrite
            # this Log's bitmaps (a captured graph keeps the views: valid until the next replay)
            removed, counts = removed.clone(), counts.clone()
        log.removed, log.counts = removed, counts
        log.rewards = env.last_reward32[rank * bl:(rank + 1) * bl]
        log.rewards_all = rewards  # [P*bl] fp64, global sample order (the M lines of every one are here)
        st["log"] = log

    def _parity_rollout(self, lg: Tensor, B: int, lmax: Tensor, z: Tensor):
        E1 = lg.shape[-1]
        dev = lg.device
        chosen = torch.zeros(B, (E1 + 31) // 32, dtype=torch.int32, device=dev)
        active = torch.ones(B, dtype=torch.uint8, device=dev)
        zrem = z.clone()
        acts, probs = [], []
        while True:
            # exactly the draws of Categorical(probs).sample() -> multinomial fast path
            noise = torch.empty(B, E1).exponential_(1)
            a, p = kernels.parity_step(lg, B, noise, lmax, chosen, active, zrem)
            acts.append(a)
            probs.append(p)
            if not bool(active.any()):
                break
        actions_bt = torch.stack(acts, 1)
        # logged probabilities from the remaining mass (no running-sum cancellation)
        return actions_bt, trajectory_probs(lg, actions_bt)
