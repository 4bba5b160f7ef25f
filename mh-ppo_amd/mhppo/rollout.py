"""GPU rollout collector: one PPO iteration's episodes for N envs at once.

Batched form of `Env_rollout.iterations_rand` (Coop-MH-PPO-scalable.py:357-517;
coop driver Coop-MH-PPO.ipynb cell 0): every env plays one 80-step episode;
the choice head is sampled once at t=0 (ped_traffic never changes, so
`need_new_d` is only true at the start); each step runs the
MFMA policy kernel and the fused sample+env-step kernel.  The per-step records are
written time-major, [t, env, slot] (each step's writes are one contiguous block
in HBM); RolloutBatch exposes them as [env, slot, t] views, and bucket_segments
gathers (env, slot) segments over t into the reference's episode-major,
car-major, time-ascending batch order.

Noise: in perf mode the standard normals (MVN eps) and the Categorical
uniforms come from Philox keyed by (seed, iteration) with counters built from
the GLOBAL env id, so a sharded run draws the same noise per env as a single
GPU.  In parity mode callers pass the reference's recorded draws instead.
"""
import ctypes
import os

import torch

from . import _lib

NF_C = 13
_CTR_STEP = 1 << 40  # counter stride between time steps (global env*slot index below it)


class RolloutBatch:
    """Views of one iteration's rollout buffers (all on the env's device).  With the compact
    record layout (rec_of set: the scalable env, whose absent car slots store no records) obs_c /
    act / logp / rew are gathered from the time-major records on first access, absent segments
    zero — a full copy, not a view: at config 4 (524 288 segments x 80 steps) obs_c alone is
    2.2 GB, and the gather needs about twice that in temporaries.  The product path never touches
    them (bucket_segments reads the *_tm records through rec_of); they are for tests and tools."""

    _REC = ("obs_c", "act", "logp", "rew")

    def __init__(self, **kw):
        self.__dict__.update(kw)

    def __getattr__(self, name):
        if name not in RolloutBatch._REC or self.__dict__.get("rec_of") is None:
            raise AttributeError(name)
        N, S, T = self.N, self.S, self.T
        ro = self.rec_of.long()
        x = getattr(self, name + "_tm").reshape(T, N * S, -1).index_select(1, ro.clamp_min(0))
        x = torch.where((ro >= 0).reshape(1, -1, 1), x, torch.zeros((), dtype=x.dtype, device=x.device))
        x = x.reshape(T, N, S, -1).permute(1, 2, 0, 3)
        v = x if name == "obs_c" else x[..., 0]
        self.__dict__[name] = v
        return v


# Envs per part below which the rollout runs as one chain (parts = 1): with fewer than ~256 waves of
# envs per part the launches are too small for two streams to gain anything
PART_MIN_ENVS = 16384


def default_parts(n_envs, valu_policy=False):
    """2 (two independent step chains on two streams, RolloutGPU.collect) for large env counts,
    else 1.  MHPPO_ROLLOUT_PARTS overrides (A/B)."""
    import os
    env = os.environ.get("MHPPO_ROLLOUT_PARTS")
    if env:
        return max(1, int(env))
    return 2 if (not valu_policy and n_envs >= 2 * PART_MIN_ENVS) else 1


def default_graph():
    """Replay the one-chain step loop from a captured HIP graph (RolloutGPU.collect) unless
    MHPPO_ROLLOUT_GRAPH=0; =2 also captures the two-stream parts loop (measured no faster at
    config 3: 64.5-65.2 us per step either way, profiles/r04_host/graph_parts_ab.txt)."""
    import os
    return {"0": 0, "2": 2}.get(os.environ.get("MHPPO_ROLLOUT_GRAPH", "1"), 1)


class RolloutGPU:
    def __init__(self, venv, T=None, valu_policy=False, parts=None):
        if venv.variant == "4cars2":
            raise ValueError("4cars2 is an env-level variant only: the reference has no driver for it and its "
                             "PPO-driven followers earn no reward (Env_hybrid_multi_coop_4cars2.py:836-847)")
        self.venv = venv
        self.T = T or venv.max_episode
        N, S, P = venv.n_envs, venv.n_slots, venv.nb_ped
        self.N, self.S, self.P = N, S, P
        self.dc = _lib.lib().mhppo_choice_dim(venv.handle)
        dev = venv.device
        f32, f64, i32 = torch.float32, torch.float64, torch.int32
        z = lambda shape, dt: torch.zeros(shape, dtype=dt, device=dev)
        self.feat_d = z((N, S, P, self.dc), f32)
        self.probs_d = z((N, S, P, 2), f32)
        self.logp_d = z((N, S, P), f32)
        self.a_d = z((N, S, P), i32)
        self.closest = z((N, S), i32)
        self.feat_c = z((N, S, P, NF_C), f32)
        self.out_c = z((N, S, P), f32)
        self.obs = z((N, venv.obs_dim), f32)
        # time-major records [T, N, S(, 13)] (include/mhppo.h mhppo_rollout_bufs)
        self.obs_c = z((self.T, N, S, NF_C), f32)
        self.act = z((self.T, N, S), f32)
        self.logp = z((self.T, N, S), f32)
        self.rew = z((self.T, N, S), f64)
        self.ep_min = z((N, S), f64)
        self.exist = z((N, S), torch.uint8)
        self.eps = z((self.T, N, S), f32)
        self.u = z((N, S, P), f32)
        # the compact record layout (include/mhppo.h mhppo_rollout_bufs.rec_of) where car slots can
        # be absent (the scalable env): absent segments store no records, present ones are
        # contiguous (MHPPO_COMPACT_RECORDS=0: the identity layout)
        self.compact = venv.variant == "scalable" and os.environ.get("MHPPO_COMPACT_RECORDS", "1") != "0"
        self.rec_buf = z(N * S + N + 1, i32) if self.compact else None  # segment ranks | per-env prefix
        self.rec_of = self.rec_buf[:N * S] if self.compact else None
        self.parts = default_parts(N, valu_policy) if parts is None else int(parts)
        if self.parts > 1 and valu_policy:
            raise ValueError("parts > 1 runs the MFMA policy kernel only")
        # head-sorted policy rows (filled by mhppo_rollout_begin) + the parts' bounds in them
        self.rows = z(N * S * P + 2 + 2 * (self.parts + 1), i32)
        self.status = z(1, i32)  # NaN flags of the policy draws (mhppo_rollout_check)
        b = _lib.RolloutBufs()
        for name in ("feat_d", "probs_d", "logp_d", "a_d", "closest", "feat_c", "out_c", "obs", "obs_c", "act",
                     "logp", "rew", "ep_min", "exist", "rows", "status"):
            setattr(b, name, ctypes.c_void_p(getattr(self, name).data_ptr()))
        b.T = self.T
        b.rec_of = ctypes.c_void_p(self.rec_buf.data_ptr()) if self.compact else None
        # policy step on the VALU reference kernels instead of the MFMA one (bit-identical; tests, with
        # the test build of the library: MHPPO_LIB=tests/lib/libmhppo_test.so); "unsorted": the
        # one-lane-per-row kernel
        b.flags = {False: 0, True: 1, "unsorted": 3}[valu_policy]  # MHPPO_ROLLOUT_VALU_POLICY
        b.parts = self.parts
        self._bufs = b
        # captured one-chain step loops, keyed by what their launches bake in (collect)
        self._graphs = {}
        self._cap_stream = None  # the graph capture stream, on the env's device (created at first capture)
        self.use_graph = default_graph() if dev.type == "cuda" else 0
        # parts > 1: part p > 0 steps on its own stream (created once), part 0 on the caller's
        self._side = [torch.cuda.Stream(device=dev) for _ in range(self.parts - 1)] if dev.type == "cuda" else []

    def evaluate(self, actor_cross, actor_wait, actor_choice, episodes=1, choix=False):
        """Deterministic evaluation (Env_rollout.iterations :152-252): `episodes` consecutive
        episodes in every env (env e's episodes continue its own random stream).
        Returns the five tensors iterations returns, env-major (env 0's episodes first),
        on the env's device: obs [N*K*T, obs_dim], acts [N*K*T, S], rews_c [N*K*T, S]
        (float32), rews_d [saves, S], waiting [saves * P].  choix=True plays the scripted
        choix_test scenario (:629-633) after every reset (scalable env only)."""
        L = _lib.lib()
        venv, N, S, P, T = self.venv, self.N, self.S, self.P, self.T
        dev = venv.device
        z = lambda shape, dt: torch.zeros(shape, dtype=dt, device=dev)
        E = dict(obs=z((N, venv.obs_dim), torch.float32), a_d=z((N, S, P), torch.int32),
                 trig=z(N, torch.uint8), ep_min=z((N, S), torch.float64))
        hist = {k: [] for k in ("obs", "acts", "rews_c", "rews_d", "waiting", "saved")}
        mc, tc = actor_cross.mlp_desc()
        mw, tw = actor_wait.mlp_desc()
        md, td = actor_choice.mlp_desc()
        st = _lib.stream_ptr(device=venv.device)
        for _ in range(episodes):
            R = dict(obs_hist=z((T, N, venv.obs_dim), torch.float32), acts=z((T, N, S), torch.float32),
                     rews_c=z((T, N, S), torch.float32), rews_d=z((T, N, S), torch.float32),
                     waiting=z((T, N, P), torch.float32), saved=z((T, N), torch.uint8))
            b = _lib.EvalBufs()
            for k, v in list(E.items()) + list(R.items()):
                setattr(b, k, ctypes.c_void_p(v.data_ptr()))
            b.T = T
            _lib.check(L.mhppo_env_reset(venv.handle, _lib.ptr(E["obs"]), st))
            if choix:  # iterations(choix=True): choix_test + get_state (:170-172)
                _lib.check(L.mhppo_env_choix_test(venv.handle, _lib.ptr(E["obs"]), st))
            for t in range(T):
                _lib.check(L.mhppo_eval_step(venv.handle, ctypes.byref(mc), ctypes.byref(mw), ctypes.byref(md), t,
                                             ctypes.byref(b), st))
            hist["obs"].append(R["obs_hist"].transpose(0, 1))  # [N, T, od]
            for k in ("acts", "rews_c", "rews_d", "waiting", "saved"):
                hist[k].append(R[k].transpose(0, 1))
        cat = {k: torch.stack(v, 1) for k, v in hist.items()}  # [N, K, T, ...]
        saved = cat["saved"].reshape(-1).bool()
        return (cat["obs"].reshape(-1, venv.obs_dim), cat["acts"].reshape(-1, S), cat["rews_c"].reshape(-1, S),
                cat["rews_d"].reshape(-1, S)[saved], cat["waiting"].reshape(-1, P)[saved].reshape(-1))

    def check(self):
        """Raise MhppoNaNError (a ValueError, as the reference's torch.distributions raise) if
        a NaN policy output was sampled since the last check.  Synchronises the stream."""
        _lib.check(_lib.lib().mhppo_rollout_check(ctypes.byref(self._bufs), _lib.stream_ptr(device=self.venv.device)))

    def draw_noise(self, seed, iteration):
        """Philox perf-mode noise for one iteration (global-env-id counters)."""
        L = _lib.lib()
        key = (int(seed) * 1000003 + int(iteration)) & 0xFFFFFFFFFFFFFFFF
        off = int(self.venv.cfg.env_id_offset)
        st = _lib.stream_ptr(device=self.venv.device)
        _lib.check(L.mhppo_philox_uniform(key, off * self.S * self.P, _lib.ptr(self.u), self.u.numel(), st))
        # step t's normals from counters (t + 1) * 2^40 + global (env, slot): one launch
        _lib.check(L.mhppo_philox_normal_2d(key, _CTR_STEP + off * self.S, _CTR_STEP, _lib.ptr(self.eps), self.T,
                                            self.eps[0].numel(), st))

    def _step_loop(self, L, mx, mw, st, step_events):
        """The T steps as one chain on stream `st`: policy + env step."""
        for t in range(self.T):
            if self.P == 1:  # features straight into the step's record (include/mhppo.h)
                self._bufs.feat_c = self.obs_c[t].data_ptr()
            _lib.check(L.mhppo_rollout_policy(self.venv.handle, ctypes.byref(mx), ctypes.byref(mw),
                                              ctypes.byref(self._bufs), st))
            if step_events is not None:  # HIP events bracketing the env-step kernel on this stream
                step_events[t][0].record()
            _lib.check(L.mhppo_rollout_sample_env(self.venv.handle, _lib.ptr(self.eps[t]), t,
                                                  ctypes.byref(self._bufs), st))
            if step_events is not None:
                step_events[t][1].record()

    def _parts_loop(self, L, mx, mw, nparts, main):
        """Two-stream rollout: the parts' step chains (policy -> env step -> policy ...) are
        independent, so one part's policy MFMA work fills the CUs that another part's
        latency-bound env step leaves idle (one wave per SIMD, the launch lasting as long as its
        slowest wave).  Part 0 on `main`, part p > 0 on side stream p - 1, forked from and joined
        back to `main`.  The same kernels and results as the one-chain loop."""
        forked = torch.cuda.Event()
        forked.record(main)
        for side in self._side[:nparts - 1]:
            side.wait_event(forked)
        streams = [main.cuda_stream] + [side.cuda_stream for side in self._side[:nparts - 1]]
        for t in range(self.T):
            if self.P == 1:  # features straight into the step's record (include/mhppo.h)
                self._bufs.feat_c = self.obs_c[t].data_ptr()
            for part, sp in enumerate(streams):
                _lib.check(L.mhppo_rollout_policy_part(self.venv.handle, ctypes.byref(mx), ctypes.byref(mw),
                                                       ctypes.byref(self._bufs), part, sp))
                _lib.check(L.mhppo_rollout_sample_env_part(self.venv.handle, _lib.ptr(self.eps[t]), t,
                                                           ctypes.byref(self._bufs), part, sp))
        for side in self._side[:nparts - 1]:
            main.wait_stream(side)

    def collect(self, actor_cross, actor_wait, actor_choice, seed=0, iteration=0, forced_choice=None,
                eps_tape=None, step_events=None, parts=None, graph=None):
        """Run one episode in every env.  forced_choice int32 [N,S,P] / eps_tape float32 [T,N,S]
        replay recorded draws (parity mode); otherwise Philox noise is drawn.  parts: 1 forces the
        one-chain loop for this call (default: self.parts); step_events implies it.  step_events
        brackets each step's env-step launch.  graph: replay the step loop
        from a captured HIP graph (default: self.use_graph; pass False while mhppo_kernel_timing is
        on — graph nodes carry no timing events)."""
        L = _lib.lib()
        nparts = self.parts if parts is None else min(int(parts), self.parts)
        if step_events is not None:
            nparts = 1
        self._bufs.parts = nparts
        if forced_choice is None or eps_tape is None:
            self.draw_noise(seed, iteration)
        if eps_tape is not None:
            self.eps.copy_(eps_tape.to(self.eps.device, torch.float32))
        fa = None
        if forced_choice is not None:
            fa = forced_choice.to(self.a_d.device, torch.int32).contiguous()
        mc, tc = actor_choice.mlp_desc()
        mx, tx = actor_cross.mlp_desc()
        mw, tw = actor_wait.mlp_desc()
        dev = self.venv.device
        st = _lib.stream_ptr(device=dev)
        _lib.check(L.mhppo_rollout_begin(self.venv.handle, ctypes.byref(mc), _lib.ptr(self.u), _lib.ptr(fa),
                                         ctypes.byref(self._bufs), st))
        if graph is None:  # the default: the one-chain loop (and with MHPPO_ROLLOUT_GRAPH=2 the parts loop)
            graph = bool(self.use_graph) and (nparts == 1 or self.use_graph == 2)
        graph = bool(graph) and dev.type == "cuda"
        if step_events is None and graph:
            # The step loop's launches (one chain: 160; parts: 160 per part on their
            # streams, forked from and joined back to the capture stream) as one captured HIP
            # graph, replayed: the same kernels and arguments (the pointers, step indices and the
            # actors' mean / std are baked into the graph's nodes and key it), without the
            # per-launch host work — which at small N is the step's time, and at large N keeps the
            # host from queueing the bucketing until the rollout has nearly finished.
            # Capture and replay with the env's device current and on a capture stream OF that
            # device: torch.cuda.graph's default capture stream is created once, on whichever
            # device was current at its first use, and a launch on another device's stream would
            # run eagerly outside the capture (an empty graph, replayed silently).  The replay
            # goes to dev's current stream, ordered after mhppo_rollout_begin above.
            key = (nparts, mx.packed, mw.packed, mx.mean, mx.std, mw.mean, mw.std)
            with torch.cuda.device(dev):
                g = self._graphs.get(key)
                if g is None:
                    if self._cap_stream is None:
                        self._cap_stream = torch.cuda.Stream(device=dev)
                    g = torch.cuda.CUDAGraph()
                    with torch.cuda.graph(g, stream=self._cap_stream):
                        cap = torch.cuda.current_stream(dev)
                        assert cap == self._cap_stream, "graph capture must run on the env's device"
                        if nparts == 1:
                            self._step_loop(L, mx, mw, cap.cuda_stream, None)
                        else:
                            self._parts_loop(L, mx, mw, nparts, cap)
                    if len(self._graphs) > 8:
                        self._graphs.clear()
                    self._graphs[key] = g
                g.replay()
        elif nparts == 1:
            self._step_loop(L, mx, mw, st, step_events)
        else:
            self._parts_loop(L, mx, mw, nparts, torch.cuda.current_stream(dev))
        del tc, tx, tw, fa  # keep the packed weights alive until the launches are queued
        # obs_c/act/logp/rew: [N, S, T(, 13)] views of the time-major buffers (*_tm)
        views = {} if self.compact else dict(obs_c=self.obs_c.permute(1, 2, 0, 3), act=self.act.permute(1, 2, 0),
                                             logp=self.logp.permute(1, 2, 0), rew=self.rew.permute(1, 2, 0))
        return RolloutBatch(feat_d=self.feat_d, probs_d=self.probs_d, logp_d=self.logp_d, a_d=self.a_d,
                            closest=self.closest, **views, obs_c_tm=self.obs_c,
                            act_tm=self.act, logp_tm=self.logp, rew_tm=self.rew, ep_min=self.ep_min, rec_of=self.rec_of,
                            exist=self.exist, N=self.N, S=self.S, P=self.P, T=self.T)


def returns_scan_tm(rew_tm, gamma=0.99):
    """futur_rewards over time-major records: rew float64 [T, ...] (one segment per column)
    -> float32 [T, ...]."""
    T = rew_tm.shape[0]
    r = rew_tm.reshape(T, -1).contiguous()
    out = torch.empty(r.shape, dtype=torch.float32, device=rew_tm.device)
    with torch.cuda.device(rew_tm.device):  # the records' device and its current stream
        _lib.check(_lib.lib().mhppo_returns_scan_tm(_lib.ptr(r), _lib.ptr(out), r.shape[1], T, gamma,
                                                    _lib.stream_ptr(device=rew_tm.device)))
    return out.reshape(rew_tm.shape)


def returns_scan(rew, gamma=0.99):
    """futur_rewards (:658-684): float64 reverse discounted scan per [.., T] row -> float32."""
    T = rew.shape[-1]
    r = rew.reshape(-1, T).contiguous()
    out = torch.empty(r.shape, dtype=torch.float32, device=rew.device)
    with torch.cuda.device(rew.device):
        _lib.check(_lib.lib().mhppo_returns_scan(_lib.ptr(r), _lib.ptr(out), r.shape[0], T, gamma,
                                                 _lib.stream_ptr(device=rew.device)))
    return out.reshape(rew.shape)


NAN_STATUS_MSG = {1: "Categorical probs of the choice actor, :409",
                  2: "MultivariateNormal loc of the continuous actors, :451"}


def raise_if_nan_status(st):
    """The host side of mhppo_rollout_check for a status word already read back: raise
    MhppoNaNError (a ValueError, as the reference's torch.distributions raise) when set."""
    st = int(st)
    if st:
        what = "; ".join(m for b, m in NAN_STATUS_MSG.items() if st & b)
        raise _lib.MhppoNaNError(f"NaN policy output sampled ({what}): the reference raises ValueError here")


def bucket_segments(batch, fix_bucket=False, status=None):
    """Split (env, slot) episode segments into the reference's cross/wait/choice batches.
    fix_bucket=True (opt-in bug fix) buckets car i by ITS closest
    pedestrian's decision action_d[i*P + closest_i] instead of the flat action_d[i].

    Bucket rule (:489-507): only existing cars (scalable driver); cross when
    action_d[i] <= 0 where action_d is the per-(car, ped) array indexed by the CAR
    index i.  Choice sample per existing car: the closest pedestrian's
    features, action and log-prob, reward = episodic min of reward_light.

    One host synchronisation: the three bucket sizes (and, when `status` -- the rollout's
    NaN-flag word, int32 [1] on the device -- is given, that word, raised on as
    RolloutGPU.check would) come back in one read; the segment lists are then built with
    nonzero_static at the known sizes.
    """
    N, S, P, T = batch.N, batch.S, batch.P, batch.T
    a_flat = batch.a_d.reshape(N, S * P)
    if fix_bucket:
        a_car = batch.a_d.reshape(N, S, P).gather(2, batch.closest.reshape(N, S, 1).long()).reshape(N, S)
        action_d_i = 2 * a_car.to(torch.int32) - 1
    else:
        action_d_i = 2 * a_flat[:, :S].to(torch.int32) - 1  # action_d[i], i < S
    exist = batch.exist.bool().reshape(-1)
    cross = exist & (action_d_i <= 0).reshape(-1)
    wait = exist & (action_d_i > 0).reshape(-1)
    NS = N * S
    # Everything is queued before the one host sync, so the GPU runs it while the host waits for
    # the sizes: the returns scan; each segment's bucket position (its rank among its bucket's
    # segments in (env, slot) order = the nonzero order); the bucket scatter into buffers with
    # room for every segment; the choice batch gathered over all segment slots (existing ones
    # first: nonzero_static pads with slot 0); the choice action counts.  After the sync the
    # batches are leading views of those buffers.
    # Both buckets share ONE buffer of NS + 3 segments (not one of NS each: that doubled the
    # bucketing's peak memory): cross segments from slot 0, wait segments from slot w0 = the cross
    # count rounded up to a multiple of 4, computed on the device, so the wait bucket's observation
    # rows start 16-byte aligned at any T (the train kernels' LDS-DMA rows; 4 T 52 B = 16 T 13 B).
    ret = returns_scan_tm(batch.rew_tm)  # [T, N, S]
    cc, cw = torch.cumsum(cross, 0), torch.cumsum(wait, 0)
    w0 = torch.div(cc[-1] + 3, 4, rounding_mode="floor") * 4
    pos = torch.where(cross, cc - 1, torch.where(wait, w0 + cw - 1, -1))
    bucket = torch.zeros(NS, dtype=torch.int8, device=pos.device)
    rec_of = getattr(batch, "rec_of", None)
    if rec_of is not None:  # the compact layout: the scatter's positions are per record
        idx = torch.where(rec_of >= 0, rec_of, NS).long()
        pos = torch.full((NS + 1,), -1, dtype=pos.dtype, device=pos.device).scatter_(0, idx, pos)[:NS]
    (both,) = scatter_positions(pos, bucket, (NS + 3,), NS, T, batch.obs_c_tm, batch.act_tm, batch.logp_tm, ret,
                                batch.rew_tm)
    seg_all = torch.nonzero_static(exist, size=NS, fill_value=0).squeeze(1)
    cl = batch.closest.reshape(NS).long().index_select(0, seg_all)
    base = seg_all * P + cl
    dc = batch.feat_d.shape[-1]
    a_sel = batch.a_d.reshape(-1).index_select(0, base)
    choice = dict(
        obs=batch.feat_d.reshape(NS * P, dc).index_select(0, base),
        act=a_sel,
        logp=batch.logp_d.reshape(-1).index_select(0, base),
        ret=batch.ep_min.reshape(-1).index_select(0, seg_all).float(),
    )
    a_car = batch.a_d.reshape(NS, P).gather(1, batch.closest.reshape(NS, 1).long()).reshape(-1)
    counts = torch.stack([(exist & (a_car == 0)).sum(), (exist & (a_car == 1)).sum()]).to(torch.float64)
    sizes = [cc[-1], cw[-1], exist.sum()]
    if status is not None:
        sizes.append(status.reshape(-1)[0].to(torch.int64))
    sizes = torch.stack(sizes).tolist()
    if status is not None:
        if sizes[3]:
            status.zero_()
        raise_if_nan_status(sizes[3])
    n_cross, n_wait, n_all = sizes[:3]
    c0 = (n_cross + 3) // 4 * 4  # = w0
    cross_r = {k: both[k][:n_cross * T] for k in ("obs", "act", "logp", "ret", "rew")}
    wait_r = {k: both[k][c0 * T:(c0 + n_wait) * T] for k in ("obs", "act", "logp", "ret", "rew")}
    cross_r["n_seg"], wait_r["n_seg"] = n_cross, n_wait
    choice = {k: v[:n_all] for k, v in choice.items()}
    choice["n_seg"] = n_all
    choice["counts"] = counts  # float64 [2] on the device: (act == 0).sum(), (act == 1).sum()
    return cross_r, wait_r, choice


def scatter_buckets(seg0, seg1, NS, T, obs_tm, act_tm, logp_tm, ret_tm, rew_tm):
    """Two segment-major buckets of time-major records (mhppo_bucket_scatter): row
    (k, t) = k*T + t of bucket b is record t*NS + seg_b[k] (segments disjoint)."""
    dev = obs_tm.device
    pos = torch.full((NS,), -1, dtype=torch.int64, device=dev)
    bucket = torch.zeros(NS, dtype=torch.int8, device=dev)
    for b, seg in enumerate((seg0, seg1)):
        pos[seg] = torch.arange(int(seg.numel()), dtype=torch.int64, device=dev)
        bucket[seg] = b
    return scatter_positions(pos, bucket, (int(seg0.numel()), int(seg1.numel())), NS, T, obs_tm, act_tm, logp_tm,
                             ret_tm, rew_tm)


def scatter_positions(pos, bucket, sizes, NS, T, obs_tm, act_tm, logp_tm, ret_tm, rew_tm):
    """scatter_buckets with the segments given as positions: segment s goes to row block pos[s]
    of bucket bucket[s] (pos < 0: no bucket); sizes = the two buckets' segment counts."""
    dev = obs_tm.device
    outs, dst = [], (_lib.BucketDst * 2)()  # one size: bucket 1 unused (every bucket[s] = 0)
    for b, n in enumerate(sizes):
        o = dict(obs=torch.empty(n * T, NF_C, dtype=torch.float32, device=dev),
                 act=torch.empty(n * T, dtype=torch.float32, device=dev),
                 logp=torch.empty(n * T, dtype=torch.float32, device=dev),
                 ret=torch.empty(n * T, dtype=torch.float32, device=dev),
                 rew=torch.empty(n * T, dtype=torch.float64, device=dev), n_seg=n)
        dst[b] = _lib.BucketDst(*[o[k].data_ptr() for k in ("obs", "act", "logp", "ret", "rew")])
        outs.append(o)
    srcs = [x.contiguous() for x in (obs_tm, act_tm, logp_tm, ret_tm, rew_tm)]
    _lib.check(_lib.lib().mhppo_bucket_scatter(_lib.ptr(pos), _lib.ptr(bucket), NS, T, *[_lib.ptr(x) for x in srcs],
                                               dst, _lib.stream_ptr(device=dev)))
    return outs
