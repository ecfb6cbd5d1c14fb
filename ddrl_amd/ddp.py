"""Data-parallel learner for the shared-policy configurations (C4
SharedDecentral, C5 DecentralShared_Graph).  One process per GPU, torch.distributed over
RCCL ("nccl") on the GPU box or gloo for the CPU tests.

Per iteration (RLlib semantics restated for G ranks that each own N / G envs):
  * rollout on the rank's own envs with its own MeanStdFilter (like an RLlib worker);
  * synchronize_filters (P_Local:160): every rank's pushes since the last sync (the filter
    "buffer", `ddrl_filter_delta_get`) are all-gathered and merged into the synced filter
    with RunningStat.update in rank order -- identical on every rank;
  * StandardizeFields over the union batch: all-reduce of fp64 (sum adv, sum adv^2, n);
  * minibatch SGD: per step every rank computes the gradient of its share of the
    minibatch (`ddrl_ppo_grad`, scaled by 1 / sgd_minibatch_size), one all-reduce(sum)
    of the flat gradient, then clip_by_global_norm + Adam locally (`ddrl_ppo_apply`),
    identical on every rank;
      mode "split": the global minibatch of 128 rows is 128 / G rows per rank -- the
                    sum of the rank gradients IS the single-process minibatch gradient
                    (the parity mode);
      mode "local": every rank contributes 128 rows (global minibatch 128 G, gradient
                    averaged over ranks), G times fewer sequential steps per epoch;
  * update_kl from the all-reduced mean KL of the last epoch.
Independent-policy configurations (Local, C3) need none of this: every rank is a replica.

The learner drives a backend with grad / apply / stats (`HipBackend` wraps the C-ABI
context); the collectives go through torch.distributed.  On RCCL the whole minibatch loop
can instead run inside the library (`NativeDataParallelLearner`: the context's own RCCL
communicator from `ddrl_comm_init`, `ddrl_ppo_update_ddp` enqueues grad -> ncclAllReduce ->
Adam per step with no Python between them).
"""
from __future__ import annotations

import numpy as np


def merge_running_stats(base, deltas):
    """RunningStat.update (Chan et al.) of every delta (n, M, S) into base, in order."""
    n, M, S = float(base[0]), np.array(base[1], np.float64), np.array(base[2], np.float64)
    for dn, dM, dS in deltas:
        dn = float(dn)
        if dn == 0:
            continue
        tot = n + dn
        delta = M - np.asarray(dM, np.float64)
        M = (n * M + dn * np.asarray(dM, np.float64)) / tot
        S = S + np.asarray(dS, np.float64) + delta * delta * n * dn / tot
        n = tot
    return n, M, S


def standardize_constants(sums):
    """(mean, max(1e-4, std)) from fp64 (sum, sum of squares, count) exactly as the GAE
    finalize kernel computes them (population std, fp32 results)."""
    s1, s2, n = (float(v) for v in sums)
    mean = s1 / n
    var = max(s2 / n - mean * mean, 0.0)
    return np.float32(mean), max(np.float32(1e-4), np.float32(np.sqrt(var)))


class Comm:
    """torch.distributed helpers on numpy arrays (tensors live on `device`: cuda for RCCL,
    cpu for gloo)."""

    def __init__(self, device="cpu", group=None):
        import torch
        import torch.distributed as dist
        self.torch, self.dist, self.group = torch, dist, group
        self.device = device
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)

    def all_reduce_np(self, arr, op="sum"):
        t = self.torch.as_tensor(np.ascontiguousarray(arr)).to(self.device)
        self.dist.all_reduce(t, op=getattr(self.dist.ReduceOp, op.upper()), group=self.group)
        return t.cpu().numpy()

    def all_gather_np(self, arr):
        t = self.torch.as_tensor(np.ascontiguousarray(arr)).to(self.device)
        out = [self.torch.empty_like(t) for _ in range(self.world)]
        self.dist.all_gather(out, t, group=self.group)
        return [o.cpu().numpy() for o in out]

    def all_reduce_(self, tensor):
        if self.world > 1:
            self.dist.all_reduce(tensor, group=self.group)


def sync_filters(comm, base, delta):
    """All-gather every rank's filter delta and merge them into `base` in rank order."""
    D = len(delta[1])
    packed = np.concatenate([[delta[0]], delta[1], delta[2]]).astype(np.float64)
    parts = comm.all_gather_np(packed)
    deltas = [(p[0], p[1:1 + D], p[1 + D:1 + 2 * D]) for p in parts]
    return merge_running_stats(base, deltas)


def sync_standardize(comm, sums):
    """Global StandardizeFields constants from every rank's fp64 advantage sums."""
    return standardize_constants(comm.all_reduce_np(np.asarray(sums, np.float64)))


def gather_records(comm, src, dst):
    """Gather mode: every rank's record buffer `src` ([rows][stride] fp32, device) into the
    union buffer `dst` of the learner context, rank-major (rank r's rows at r * rows).  The union
    is a row permutation of one process's time-major batch over all envs, and the update's
    shuffle is a random permutation, so the two are the same SGD problem.  `comm` None: one
    process (a plain copy).  RCCL gathers straight into `dst`; gloo goes through host memory."""
    if comm is None or comm.world == 1:
        dst.copy_(src)
        return
    if dst.shape[0] != src.shape[0] * comm.world or dst.shape[1:] != src.shape[1:]:
        raise ValueError(f"union buffer {tuple(dst.shape)} is not {comm.world} x {tuple(src.shape)}")
    torch = comm.torch
    if comm.device == "cpu":   # gloo
        parts = [torch.empty_like(src, device="cpu") for _ in range(comm.world)]
        comm.dist.all_gather(parts, src.cpu(), group=comm.group)
        dst.copy_(torch.cat(parts).to(dst.device))
    else:
        comm.dist.all_gather_into_tensor(dst, src, group=comm.group)


class HipBackend:
    """The C-ABI context as a learner backend."""

    def __init__(self, ctx):
        self.ctx = ctx

    def grad(self, pid, rows, n_rows, kl, grad, stats_step):
        self.ctx.ppo_grad(pid, rows, n_rows, kl, grad, stats_step)

    def apply(self, pid, grad):
        self.ctx.ppo_apply(pid, grad)

    def stats(self, pid, n, first=0):
        return self.ctx.ppo_stats(pid, n, first)

    def snapshot(self, pid):
        """Weights, Adam m / v and beta powers of the policy (restored if the update fails)."""
        return self.ctx.params_get(pid), self.ctx.adam_get(pid)

    def restore(self, pid, snap):
        theta, (m, v, b1, b2) = snap
        self.ctx.params_set(pid, theta)
        self.ctx.adam_set(pid, m, v, b1, b2)


def native_comm_init(ctx, comm):
    """Give the C-ABI context its own RCCL communicator over the ranks of `comm`: rank 0 makes
    the unique id, a torch.distributed broadcast hands it to the others."""
    from . import native
    uid = native.comm_unique_id() if comm.rank == 0 else bytes(native.COMM_ID_BYTES)
    t = comm.torch.tensor(list(uid), dtype=comm.torch.uint8, device=comm.device)
    if comm.world > 1:
        comm.dist.broadcast(t, src=0, group=comm.group)
    ctx.comm_init(bytes(t.cpu().tolist()), comm.rank, comm.world)


class DataParallelLearner:
    def __init__(self, backend, comm, pid=0, minibatch=128, mode="split"):
        if mode not in ("split", "local"):
            raise ValueError("mode must be 'split' or 'local'")
        if mode == "split" and minibatch % comm.world:
            raise ValueError("split mode needs sgd_minibatch_size divisible by the world size")
        self.backend, self.comm, self.pid, self.mode = backend, comm, pid, mode
        self.rows_per_rank = minibatch // comm.world if mode == "split" else minibatch
        self.grad_scale = 1.0 if mode == "split" else 1.0 / comm.world
        self.stats_first = 0   # the row of the last epoch's first step in the learner statistics

    def n_minibatches(self, rows_local):
        """Steps per epoch: every rank must run the same number (the smallest shard wins).
        A shard without one full minibatch share is refused on every rank, as
        ddrl_ppo_update refuses a batch smaller than one minibatch (a gradient launch reads
        rows_per_rank rows of the shuffle)."""
        nb = rows_local // self.rows_per_rank
        nb = int(self.comm.all_reduce_np(np.array([nb], np.int64), op="min")[0])
        if nb < 1:
            raise ValueError(f"a rank holds fewer rows than one minibatch share of {self.rows_per_rank}")
        return nb

    def schedule(self, rng, rows_local, epochs):
        nb = self.n_minibatches(rows_local)
        shuffle = rng.permutation(rows_local).astype(np.int32)
        perms = np.stack([rng.permutation(nb) for _ in range(epochs)]).astype(np.int32)
        return shuffle, perms

    def learn(self, shuffle, perms, kl_coeff, grad):
        """shuffle: rank-local row permutation (device tensor for the HIP backend),
        perms: host int array [epochs][nb], grad: flat gradient buffer (device tensor).
        Returns the all-reduced mean KL of the last epoch."""
        E, nb = perms.shape
        m = self.rows_per_rank
        snap = self.backend.snapshot(self.pid) if hasattr(self.backend, "snapshot") else None
        err = None
        for e in range(E):
            last = e == E - 1
            for b in range(nb):
                s = int(perms[e, b]) * m
                if err is None:
                    try:
                        self.backend.grad(self.pid, shuffle[s:s + m], m, kl_coeff, grad, b if last else -1)
                    except Exception as ex:   # DdrlError of a failed launch: stop computing,
                        err = ex              # keep joining the collectives (zero contribution)
                if err is not None:
                    grad.zero_()
                self.comm.all_reduce_(grad)
                if self.grad_scale != 1.0:
                    grad.mul_(self.grad_scale)
                if err is None:
                    try:
                        self.backend.apply(self.pid, grad)
                    except Exception as ex:
                        err = ex
        return self._kl(nb, err, snap)

    def _kl(self, nb, err=None, snap=None):
        """All-reduced mean KL of the last epoch.  The error state of every rank is exchanged
        first (max of a flag): a rank whose gradient / apply launch or update kernel reported
        an error (e.g. an exchange timeout) makes every rank raise, instead of the others
        blocking in their next collective while it unwinds.  A failing rank keeps joining
        every step's all-reduce with a zero gradient, and on failure every rank restores the
        weights / Adam state it held before the update (`snap`), so they stay identical."""
        kl_local = 0.0
        if err is None:
            try:
                st = (self.backend.stats(self.pid, nb, self.stats_first) if self.stats_first else
                      self.backend.stats(self.pid, nb))
                kl_local = float(np.mean(st[:, 3].astype(np.float64)))
            except Exception as e:   # the backend's own error (DdrlError from the C-ABI)
                err = e
        red = self.comm.all_reduce_np(np.array([kl_local, 1.0 if err is not None else 0.0]))
        if red[1] > 0:
            if snap is not None:
                self.backend.restore(self.pid, snap)
            if err is not None:
                raise err
            raise RuntimeError(f"data-parallel update failed on {int(red[1])} other rank(s)")
        return float(red[0]) / self.comm.world


class NativeDataParallelLearner(DataParallelLearner):
    """DataParallelLearner whose per-step loop runs inside the library: ddrl_ppo_update_ddp
    enqueues gradient -> RCCL all-reduce -> Adam for every minibatch from C++, on the
    context's stream and communicator (`native_comm_init`), the same arithmetic in the same
    order as `learn` above (which it is tested against bit for bit)."""

    def __init__(self, ctx, comm, pid=0, minibatch=128, mode="split"):
        super().__init__(HipBackend(ctx), comm, pid, minibatch, mode)
        self.ctx = ctx

    def learn(self, shuffle, perms, kl_coeff, grad=None):
        perms = np.asarray(perms, np.int32)
        self.ctx.ppo_update_ddp(self.pid, shuffle, perms, self.rows_per_rank, kl_coeff, self.grad_scale)
        return self._kl(perms.shape[1])


def _device_key(torch):
    """An id of this process's current GPU that is the same in every process using that GPU (its
    UUID or PCI bus id; device indexes differ between processes with different visible-device
    lists), -1 without a GPU."""
    if not torch.cuda.is_available():
        return -1
    props = torch.cuda.get_device_properties(torch.cuda.current_device())
    for attr in ("uuid", "pci_bus_id"):
        v = getattr(props, attr, None)
        if v is not None:
            import zlib
            return zlib.crc32(str(v).encode()) & 0x7FFFFFFF
    return torch.cuda.current_device()


def peer_init(ctx, comm):
    """Peer mode: rank 0 allocates the shared outboxes (fine-grained device memory) and exports
    an IPC handle, a torch.distributed broadcast hands it to rank 1, which maps it; both attach.
    Returns the outbox pointer in this process."""
    from . import native
    if comm.world != 2:
        raise ValueError("peer mode splits the minibatch over exactly two ranks")
    # which GPU each rank's context is on: every test ran both ranks on one GPU; the cross-GPU
    # path (system-scope stores over xGMI into the peer's fine-grained HBM, IPC mapping across
    # devices) has not run on hardware, so it is flagged, and PeerLearner checks the
    # ranks' weights after every update
    pci = comm.all_gather_np(np.array([_device_key(comm.torch)], np.int64))
    if len({int(p[0]) for p in pci}) > 1:
        import warnings
        warnings.warn("peer mode across two GPUs is experimental: its cross-device exchange has not run on "
                      "hardware; the ranks' weights are compared after every update and a mismatch falls back "
                      "to the all-reduce learner")
    if comm.rank == 0:
        gx, h = ctx.peer_alloc(export=True)
    else:
        h = bytes(native.PEER_HANDLE_BYTES)
    t = comm.torch.tensor(list(h), dtype=comm.torch.uint8, device=comm.device)
    comm.dist.broadcast(t, src=0, group=comm.group)
    if comm.rank == 1:
        gx = ctx.peer_open(bytes(t.cpu().tolist()))
    _peer_arm(ctx, comm, gx)
    return gx


def _peer_arm(ctx, comm, gx):
    """Rank 0's attach clears the outboxes; rank 1 attaches after it (a collective between)."""
    if comm.rank == 0:
        ctx.peer_attach(gx, 0, 2)
    comm.all_reduce_np(np.zeros(1))
    if comm.rank == 1:
        ctx.peer_attach(gx, 1, 2)


class PeerLearner(DataParallelLearner):
    """Two ranks' "split" minibatch SGD as ONE fused update split across them
    (ddrl_ppo_update_peer): rank r's persistent launch runs row half r of every 128-row minibatch
    (its own 64 rows) and swaps partial gradients with the peer's launch every step through the
    shared outboxes -- device-initiated stores (xGMI between GPUs), no collective call and no
    launch per step.  Both ranks then run the same clip + Adam, so their weights stay
    bit-identical, and equal to one fused update over the union batch whose minibatch b is
    [rank 0's rows | rank 1's rows] (tests/test_gpu_peer.py).  The launches wait for each other
    (3 s bound), so both must be enqueued close together: the StandardizeFields all-reduce and
    the minibatch-count all-reduce the trainer runs just before are the rendezvous.
    A failure on either rank (a wait abandoned at the bound, a refused launch) makes both ranks
    see it (the flag exchange of `_kl`) with the state of before the call restored; both then
    fall back to the per-step all-reduce learner (DataParallelLearner over `comm`), this update
    included, for the rest of the run.  `backend` defaults to the context (HipBackend)."""

    def __init__(self, ctx, comm, pid=0, minibatch=128, backend=None):
        if minibatch != 128:
            raise ValueError("peer mode splits the fused update's 128-row minibatch")
        super().__init__(backend if backend is not None else HipBackend(ctx), comm, pid, minibatch, "split")
        self.ctx = ctx
        self.fallback = None
        self.gx = peer_init(ctx, comm)

    def learn(self, shuffle, perms, kl_coeff, grad=None):
        if self.fallback is not None:
            return self.fallback.learn(shuffle, perms, kl_coeff, grad)
        torch = self.comm.torch
        perms = np.asarray(perms, np.int32)
        E, nb = perms.shape
        self.stats_first = (E - 1) * nb
        snap = self.backend.snapshot(self.pid) if hasattr(self.backend, "snapshot") else None
        pe = torch.from_numpy(np.ascontiguousarray(perms)).to(getattr(shuffle, "device", "cpu"))
        err = None
        try:
            self.ctx.ppo_update_peer(self.pid, shuffle, pe, kl_coeff)
            self.ctx.synchronize()
        except Exception as e:   # DdrlError: this rank's state is already restored
            err = e
        # both ranks must hold bit-identical weights after a completed peer update; a mismatch (a
        # partial the peer never saw) is a failure like an abandoned exchange: both restore the
        # snapshot and fall back
        digest = np.zeros(2)
        if err is None:
            theta = np.asarray(self.ctx.params_get(self.pid))
            digest = np.array([float(np.sum(theta, dtype=np.float64)),
                               float(np.dot(theta.astype(np.float64), np.arange(1, theta.size + 1)))])
        both = self.comm.all_gather_np(digest)
        if err is None and not np.array_equal(both[0], both[1]) and np.all(np.isfinite(both)):
            if not any(np.all(b == 0) for b in both):   # the other rank failed: its error wins below
                err = RuntimeError("peer update: the two ranks' weights differ after the fused update (the peer's "
                                   "partials were not seen); the state of before the call is restored")
                if snap is not None:
                    self.backend.restore(self.pid, snap)
        try:
            return self._kl(nb, err, snap)
        except Exception as e:
            import warnings
            warnings.warn(f"peer update failed on rank {self.comm.rank} or its peer ({e}); this update and "
                          "the following ones run on the per-step all-reduce learner")
            self.stats_first = 0
            self.fallback = DataParallelLearner(self.backend, self.comm, self.pid, 128, "split")
            if grad is None:
                grad = torch.zeros(int(self.ctx.n_params[self.pid]), dtype=torch.float32,
                                   device=getattr(shuffle, "device", "cpu"))
            return self.fallback.learn(shuffle, perms, kl_coeff, grad)
