"""Data-parallel learner (ddrl_amd.ddp) on CPU: world_size-2 and -4 gloo process groups.

The learner is driven with an oracle backend (gradients / clip + Adam from the numpy
oracle, scaled to 1 / sgd_minibatch_size like ddrl_ppo_grad), so these tests check the
distributed logic itself -- row shares, gradient all-reduce, identical Adam on every rank,
filter synchronization, cross-rank StandardizeFields, KL all-reduce -- against a
single-process oracle run on the union of the ranks' data.
Tolerances: fp64 statistics 1e-12 relative; parameters as the GPU learner tests
(>= 99.9 % within 1e-5, max <= 2 lr steps) since the two-half gradient sum differs from
the one-pass sum by fp32 rounding only.
"""
import os
import socket
import tempfile

import numpy as np
import pytest

from oracle import ddrl_oracle as O

D, A, MB = 19, 2, 128


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _rank_batch(rank, rows):
    rng = np.random.default_rng(10 + rank)
    f = np.float32
    logits = np.concatenate([rng.normal(size=(rows, A)) * 0.3, rng.normal(size=(rows, A)) * 0.1 - 0.5], 1)
    return dict(obs=rng.normal(size=(rows, D)).astype(f), actions=rng.normal(size=(rows, A)).astype(f),
                logits=logits.astype(f), logp=(rng.normal(size=rows) - 2).astype(f),
                vf_preds=rng.normal(size=rows).astype(f), adv=rng.normal(size=rows).astype(f),
                vt=rng.normal(size=rows).astype(f))


class OracleBackend:
    def __init__(self, params, shapes, batch, cap):
        self.shapes, self.batch = shapes, batch
        self.theta = O.pack(params, shapes)
        self.adam = O.Adam(self.theta.size)
        self.st = np.zeros((cap, 8), np.float32)

    def grad(self, pid, rows, n_rows, kl, grad, stats_step):
        import torch
        rows = np.asarray(rows)
        b = {k: v[rows] for k, v in self.batch.items()}
        p = O.unpack(self.theta, self.shapes)
        logits, value, cache = O.ffn_forward(p, b["obs"])
        dl, dv, st = O.ppo_loss_rows(logits, value, b["actions"], b["logits"], b["logp"], b["vf_preds"],
                                     b["adv"], b["vt"], np.float32(kl))
        s = np.float32(n_rows / MB)          # oracle averages over n_rows; ppo_grad uses 1/128
        g = O.pack(O.ffn_backward(p, cache, dl * s, dv * s), self.shapes)
        grad.copy_(torch.from_numpy(g))
        if stats_step >= 0:
            self.st[stats_step, 3] = st["kl"]

    def apply(self, pid, grad):
        clipped, _ = O.clip_by_global_norm([grad.numpy()], 0.5)
        self.theta = self.adam.apply(self.theta, clipped[0])

    def stats(self, pid, n):
        return self.st[:n]


def _worker(rank, world, port, out_dir, mode, rows_local, epochs):
    import torch
    import torch.distributed as dist
    from ddrl_amd.ddp import Comm, DataParallelLearner, sync_filters, sync_standardize
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    comm = Comm("cpu")
    # --- filter synchronization: base filter + each rank's pushes since the sync
    rng = np.random.default_rng(0)
    base_rs = O.RunningStat((43,))
    for x in rng.normal(size=(50, 43)):
        base_rs.push(x)
    mine = O.RunningStat((43,))
    for x in np.random.default_rng(100 + rank).normal(size=(30 + 7 * rank, 43)) * 2 + rank:
        mine.push(x)
    merged = sync_filters(comm, (base_rs.n, base_rs.M, base_rs.S), (mine.n, mine.M, mine.S))
    # --- StandardizeFields over the union
    adv = np.random.default_rng(200 + rank).normal(size=500 + 100 * rank).astype(np.float32) * 3 + 1
    sums = np.array([np.sum(adv, dtype=np.float64), np.sum(adv.astype(np.float64) ** 2), adv.size])
    mean, den = sync_standardize(comm, sums)
    # --- minibatch SGD
    params = O.ffn_init(np.random.default_rng(7), D, 2 * A)
    shapes = O.ffn_param_shapes(D, 2 * A)
    batch = _rank_batch(rank, rows_local)
    be = OracleBackend(params, shapes, batch, cap=1024)
    learner = DataParallelLearner(be, comm, minibatch=MB, mode=mode)
    shuffle, perms = learner.schedule(np.random.default_rng(300 + rank), rows_local, epochs)
    grad = torch.zeros(be.theta.size)
    kl = learner.learn(shuffle, perms, 0.2, grad)
    np.savez(os.path.join(out_dir, f"r{rank}.npz"), theta=be.theta, shuffle=shuffle, perms=perms,
             n=merged[0], M=merged[1], S=merged[2], mean=mean, den=den, kl=kl)
    dist.destroy_process_group()


def _run(mode, rows_local, epochs, world=2):
    import torch.multiprocessing as mp
    out = tempfile.mkdtemp()
    mp.spawn(_worker, args=(world, _free_port(), out, mode, rows_local, epochs), nprocs=world, join=True)
    return [dict(np.load(os.path.join(out, f"r{r}.npz"))) for r in range(world)]


def _reference(res, mode, rows_local, epochs):
    """Single process: the union of every rank's rows per step, one 128-row (split) or
    128 G-row (local) minibatch gradient, clip + Adam."""
    world = len(res)
    m = MB // world if mode == "split" else MB
    batches = [_rank_batch(r, rows_local) for r in range(world)]
    full = {k: np.concatenate([b[k] for b in batches]) for k in batches[0]}
    params = O.ffn_init(np.random.default_rng(7), D, 2 * A)
    shapes = O.ffn_param_shapes(D, 2 * A)
    theta = O.pack(params, shapes)
    adam = O.Adam(theta.size)
    E, nb = res[0]["perms"].shape
    kls = []
    for e in range(E):
        for b in range(nb):
            rows = np.concatenate([r * rows_local + res[r]["shuffle"][int(res[r]["perms"][e, b]) * m:
                                                                      int(res[r]["perms"][e, b]) * m + m]
                                   for r in range(world)])
            p = O.unpack(theta, shapes)
            sl = {k: v[rows] for k, v in full.items()}
            logits, value, cache = O.ffn_forward(p, sl["obs"])
            dl, dv, st = O.ppo_loss_rows(logits, value, sl["actions"], sl["logits"], sl["logp"],
                                         sl["vf_preds"], sl["adv"], sl["vt"], np.float32(0.2))
            g = O.pack(O.ffn_backward(p, cache, dl, dv), shapes)   # mean over the union rows
            clipped, _ = O.clip_by_global_norm([g], 0.5)
            theta = adam.apply(theta, clipped[0])
            if e == E - 1:
                kls.append(st["kl"])
    return theta, float(np.mean(kls))


def _params_close(got, ref, steps):
    diff = np.abs(got - ref)
    assert np.mean(diff <= 1e-5 + 1e-5 * np.abs(ref)) >= 0.999, diff.max()
    assert diff.max() <= 2 * 3e-4 * steps + 1e-5


@pytest.mark.parametrize("world,mode", [(2, "split"), (2, "local"), (4, "split"), (4, "local")])
def test_ddp_learner(world, mode):
    """World 2 and world 4 (the ranks beyond two of the driver's 8-GPU run)."""
    rows_local, epochs = 512, 2
    res = _run(mode, rows_local, epochs, world)
    # identical parameters on every rank (same all-reduced gradient, same Adam)
    for r in range(1, world):
        np.testing.assert_array_equal(res[0]["theta"], res[r]["theta"])
        assert res[0]["kl"] == res[r]["kl"]
    ref, kl_ref = _reference(res, mode, rows_local, epochs)
    steps = res[0]["perms"].size
    _params_close(res[0]["theta"], ref, steps)
    np.testing.assert_allclose(res[0]["kl"], kl_ref, rtol=1e-5)
    if mode == "split":
        # filter sync == one RunningStat over base + every rank's pushes, in rank order
        rs = O.RunningStat((43,))
        for x in np.random.default_rng(0).normal(size=(50, 43)):
            rs.push(x)
        for r in range(world):
            for x in np.random.default_rng(100 + r).normal(size=(30 + 7 * r, 43)) * 2 + r:
                rs.push(x)
        for r in range(world):
            assert res[r]["n"] == rs.n
            np.testing.assert_allclose(res[r]["M"], rs.M, rtol=1e-12, atol=1e-12)
            np.testing.assert_allclose(res[r]["S"], rs.S, rtol=1e-11)
        adv = np.concatenate([np.random.default_rng(200 + r).normal(size=500 + 100 * r).astype(np.float32) * 3 + 1
                              for r in range(world)])
        _, mean, std = O.standardize(adv)
        for r in range(1, world):
            assert res[0]["mean"] == res[r]["mean"] and res[0]["den"] == res[r]["den"]
        np.testing.assert_allclose(res[0]["mean"], mean, rtol=1e-6)
        np.testing.assert_allclose(res[0]["den"], max(np.float32(1e-4), std), rtol=1e-6)


def _gather_worker(rank, world, port, out_dir):
    import torch
    import torch.distributed as dist
    from ddrl_amd.ddp import Comm, gather_records, sync_standardize
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    comm = Comm("cpu")
    rows, stride = 200 * 12, 32
    src = torch.from_numpy(np.random.default_rng(50 + rank).normal(size=(rows, stride)).astype(np.float32))
    dst = torch.full((rows * world, stride), np.nan)
    gather_records(comm, src, dst)
    adv = src[:, 27].double()
    mean, den = sync_standardize(comm, [adv.sum().item(), (adv * adv).sum().item(), adv.numel()])
    bad = None
    try:
        gather_records(comm, src, torch.empty((rows * world + 1, stride)))
    except ValueError as e:
        bad = str(e)
    np.savez(os.path.join(out_dir, f"g{rank}.npz"), dst=dst.numpy(), mean=mean, den=den, bad=bad or "")
    dist.destroy_process_group()


def test_gather_records_world4():
    """Gather mode's record exchange at world 4 (gloo): every rank ends with the same union batch,
    rank-major, and the same StandardizeFields constants as one process over the union; a
    mis-sized union buffer is refused before any collective."""
    import torch.multiprocessing as mp
    from ddrl_amd.ddp import standardize_constants
    world = 4
    out = tempfile.mkdtemp()
    mp.spawn(_gather_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    res = [dict(np.load(os.path.join(out, f"g{r}.npz"))) for r in range(world)]
    union = np.concatenate([np.random.default_rng(50 + r).normal(size=(2400, 32)).astype(np.float32)
                            for r in range(world)])
    a = union[:, 27].astype(np.float64)
    mean, den = standardize_constants([a.sum(), (a * a).sum(), a.size])
    for r in range(world):
        np.testing.assert_array_equal(res[r]["dst"], union)
        assert res[r]["mean"] == res[0]["mean"] and res[r]["den"] == res[0]["den"]
        np.testing.assert_allclose([res[r]["mean"], res[r]["den"]], [mean, den], rtol=1e-6)
        assert "union buffer" in str(res[r]["bad"])


def test_merge_running_stats_order_and_identity():
    from ddrl_amd.ddp import merge_running_stats
    rng = np.random.default_rng(1)
    a, b = O.RunningStat((5,)), O.RunningStat((5,))
    for x in rng.normal(size=(20, 5)):
        a.push(x)
    for x in rng.normal(size=(13, 5)) + 3:
        b.push(x)
    n, M, S = merge_running_stats((a.n, a.M, a.S), [(0, np.zeros(5), np.zeros(5)), (b.n, b.M, b.S)])
    ref = O.RunningStat((5,))
    ref.n, ref.M[:], ref.S[:] = a.n, a.M, a.S
    ref.update(b)
    assert n == ref.n
    np.testing.assert_allclose(M, ref.M, rtol=1e-14)
    np.testing.assert_allclose(S, ref.S, rtol=1e-14)


class _RecordingCtx:
    """Stands in for native.Context: records the ddrl_ppo_update_ddp call and serves stats."""

    def __init__(self, kl_rows):
        self.calls, self.kl_rows = [], kl_rows

    def ppo_update_ddp(self, pid, shuffle, perms, m, kl, gscale):
        self.calls.append((pid, shuffle, perms, m, kl, gscale))

    def ppo_stats(self, pid, n, first=0):
        st = np.zeros((n, 8), np.float32)
        st[:, 3] = self.kl_rows[:n]
        return st


@pytest.mark.parametrize("mode,m,gscale", [("split", 128, 1.0), ("local", 128, 1.0)])
def test_native_learner_plumbing_world1(mode, m, gscale, monkeypatch):
    """NativeDataParallelLearner hands the schedule to the library as the Python learner
    would run it: int32 [epochs][nb] slots, rows per rank and gradient scale by mode, and the
    KL of the last epoch's statistics (world 1: the all-reduce is the identity)."""
    import torch.distributed as dist
    from ddrl_amd.ddp import Comm, NativeDataParallelLearner
    monkeypatch.setenv("MASTER_ADDR", "127.0.0.1")
    monkeypatch.setenv("MASTER_PORT", str(_free_port()))
    dist.init_process_group("gloo", rank=0, world_size=1)
    try:
        ctx = _RecordingCtx(np.array([0.01, 0.03, 0.02], np.float32))
        lr = NativeDataParallelLearner(ctx, Comm("cpu"), 0, 128, mode)
        sh, pe = lr.schedule(np.random.default_rng(0), 3 * 128, 2)
        assert pe.shape == (2, 3) and pe.dtype == np.int32
        kl = lr.learn(sh, pe.astype(np.int64), 0.2)
        (pid, shuffle, perms, rows, klc, gs), = ctx.calls
        assert pid == 0 and shuffle is sh and rows == m and klc == 0.2 and gs == gscale
        assert perms.dtype == np.int32 and perms.flags.c_contiguous and np.array_equal(perms, pe)
        np.testing.assert_allclose(kl, np.mean([0.01, 0.03, 0.02]), rtol=1e-6)
    finally:
        dist.destroy_process_group()


class _CommInitCtx:
    def __init__(self):
        self.args = None

    def comm_init(self, uid, rank, world):
        self.args = (bytes(uid), rank, world)


def _comm_init_worker(rank, world, port, out_dir):
    import torch.distributed as dist
    from ddrl_amd import ddp, native
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    # rank 0's id: a recognizable pattern instead of ncclGetUniqueId (no GPU here)
    native.comm_unique_id = lambda: bytes((7 * i + 3) % 256 for i in range(native.COMM_ID_BYTES))
    ctx = _CommInitCtx()
    ddp.native_comm_init(ctx, ddp.Comm("cpu"))
    uid, r, w = ctx.args
    np.savez(os.path.join(out_dir, f"c{rank}.npz"), uid=np.frombuffer(uid, np.uint8), rank=r, world=w)
    dist.destroy_process_group()


def test_native_comm_init_broadcasts_rank0_id_world2():
    """native_comm_init at world 2 (gloo): every rank joins with rank 0's unique id, its own
    rank and the world size (the RCCL join itself needs GPUs and runs on the GPU box)."""
    import torch.multiprocessing as mp
    out = tempfile.mkdtemp()
    mp.spawn(_comm_init_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    want = np.array([(7 * i + 3) % 256 for i in range(128)], np.uint8)
    for r in range(2):
        got = np.load(os.path.join(out, f"c{r}.npz"))
        np.testing.assert_array_equal(got["uid"], want)
        assert int(got["rank"]) == r and int(got["world"]) == 2


class _FailingBackend:
    """Gradient adds 1 to every entry, apply adds the all-reduced gradient to a weight vector;
    on the failing rank `where` ("stats" | "grad" | "apply") raises, as ddrl_ppo_stats does
    when the update kernel's error word is set (exchange timeout) or a launch fails."""

    def __init__(self, fail, where="stats"):
        self.fail, self.where, self.calls = fail, where, 0
        self.theta = np.zeros(4)

    def _maybe(self, what):
        self.calls += 1
        if self.fail and self.where == what and (what == "stats" or self.calls >= 3):
            from ddrl_amd.native import DdrlError
            raise DdrlError(f"update kernel: {what} failed (exchange timed out)")

    def grad(self, pid, rows, n_rows, kl, grad, stats_step):
        self._maybe("grad")
        grad.fill_(1.0)

    def apply(self, pid, grad):
        self._maybe("apply")
        self.theta = self.theta + grad.numpy()

    def stats(self, pid, n):
        self._maybe("stats")
        return np.zeros((n, 8), np.float32)

    def snapshot(self, pid):
        return self.theta.copy()

    def restore(self, pid, snap):
        self.theta = snap.copy()


def _error_worker(rank, world, port, out_dir, where="stats"):
    import torch
    import torch.distributed as dist
    from ddrl_amd.ddp import Comm, DataParallelLearner
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    comm = Comm("cpu")
    be = _FailingBackend(rank == 1, where)
    be.theta[:] = 5.0
    learner = DataParallelLearner(be, comm, 0, MB, "split")
    grad = torch.zeros(4)
    msg = "no error"
    try:
        learner.learn(np.arange(256, dtype=np.int32), np.array([[0, 1], [1, 0]], np.int32), 0.2, grad)
    except Exception as e:   # every rank must get here, none may hang in a collective
        msg = f"{type(e).__name__}: {e}"
    # one more collective after the failure: both ranks are still in step
    t = torch.ones(1)
    dist.all_reduce(t)
    with open(os.path.join(out_dir, f"e{rank}.txt"), "w") as f:
        f.write(f"{msg}\n{float(t[0])}\n{be.theta.tolist()}")
    dist.destroy_process_group()


@pytest.mark.parametrize("where", ["stats", "grad", "apply"])
def test_learner_error_raises_on_every_rank_world2(where):
    """an update error on one rank -- its stats (the kernel's error word), or a
    gradient / apply launch in the middle of the loop -- makes every rank raise after the
    learn loop (the error flag is all-reduced with the KL; a failing rank keeps joining each
    step's all-reduce with a zero gradient), every rank restores the weights it held before
    the update, and the ranks stay in step for the next collective."""
    import torch.multiprocessing as mp
    out = tempfile.mkdtemp()
    mp.spawn(_error_worker, args=(2, _free_port(), out, where), nprocs=2, join=True)
    msgs = [open(os.path.join(out, f"e{r}.txt")).read().splitlines() for r in range(2)]
    assert msgs[1][0].startswith("DdrlError") and "timed out" in msgs[1][0]
    assert msgs[0][0].startswith("RuntimeError") and "other rank" in msgs[0][0]
    assert msgs[0][1] == msgs[1][1] == "2.0"
    assert msgs[0][2] == msgs[1][2] == str([5.0] * 4)   # weights as before the update


class _FakePeerCtx:
    """Stands in for native.Context in peer mode: the peer launch of `fail_rank` is refused, the
    other rank's launch then abandons its waits (its synchronize raises), as on the GPU."""

    def __init__(self, rank, fail_rank, n_params):
        self.rank, self.fail_rank, self.n_params, self.calls = rank, fail_rank, [n_params], []

    def peer_alloc(self, export=False):
        self.calls.append("alloc")
        return 4096, bytes(64)

    def peer_open(self, handle):
        self.calls.append("open")
        return 8192

    def peer_attach(self, gx, rank, nranks=2):
        self.calls.append(("attach", gx, rank))

    def ppo_update_peer(self, pid, shuffle, perm, kl, max_steps=-1):
        from ddrl_amd.native import DdrlError
        self.calls.append(("update", tuple(perm.shape)))
        if self.rank == self.fail_rank:
            raise DdrlError("refused (simulated)")

    def synchronize(self):
        from ddrl_amd.native import DdrlError
        if self.fail_rank >= 0:
            raise DdrlError("update kernel: an exchange ... was abandoned (simulated)")

    def params_get(self, pid):
        # fail_rank < 0: both launches "complete" but the ranks' weights differ (a partial the
        # peer never saw), which the learner's digest exchange must catch
        return np.full(self.n_params[0], 1.0 + self.rank, np.float32)


def _peer_fallback_worker(rank, world, port, out_dir, rows_local, epochs, fail_rank=1):
    import torch
    import torch.distributed as dist
    from ddrl_amd.ddp import Comm, PeerLearner
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    params = O.ffn_init(np.random.default_rng(7), D, 2 * A)
    shapes = O.ffn_param_shapes(D, 2 * A)
    be = OracleBackend(params, shapes, _rank_batch(rank, rows_local), cap=1024)
    ctx = _FakePeerCtx(rank, fail_rank, be.theta.size)
    learner = PeerLearner(ctx, Comm("cpu"), 0, MB, backend=be)
    shuffle, perms = learner.schedule(np.random.default_rng(300 + rank), rows_local, epochs)
    with pytest.warns(UserWarning, match="per-step all-reduce"):
        kl = learner.learn(shuffle, perms, 0.2, torch.zeros(be.theta.size))
    assert learner.fallback is not None and learner.stats_first == 0
    np.savez(os.path.join(out_dir, f"r{rank}.npz"), theta=be.theta, shuffle=shuffle, perms=perms, kl=kl,
             calls=np.array([str(c) for c in ctx.calls]))
    dist.destroy_process_group()


@pytest.mark.parametrize("fail_rank", [1, -1])
def test_peer_learner_falls_back_to_allreduce_loop_world2(fail_rank):
    """PeerLearner over gloo with a stand-in context: rank 0 allocates and attaches before rank 1
    opens the handle and attaches; a refused peer launch on rank 1 (rank 0's waits abandoned) --
    or (fail_rank -1) two launches that complete with different weights on the two ranks, caught
    by the learner's weight-digest exchange -- makes BOTH ranks fall back to the
    per-step all-reduce learner for the same update, which then matches the single-process union
    reference like test_ddp_learner[2-split]."""
    import torch.multiprocessing as mp
    rows_local, epochs = 512, 2
    out = tempfile.mkdtemp()
    mp.spawn(_peer_fallback_worker, args=(2, _free_port(), out, rows_local, epochs, fail_rank), nprocs=2,
             join=True)
    res = [dict(np.load(os.path.join(out, f"r{r}.npz"))) for r in range(2)]
    assert list(res[0]["calls"][:2]) == ["alloc", "('attach', 4096, 0)"]
    assert list(res[1]["calls"][:2]) == ["open", "('attach', 8192, 1)"]
    assert res[0]["calls"][2] == res[1]["calls"][2] == "('update', (2, 8))"
    np.testing.assert_array_equal(res[0]["theta"], res[1]["theta"])
    ref, kl_ref = _reference(res, "split", rows_local, epochs)
    _params_close(res[0]["theta"], ref, res[0]["perms"].size)
    np.testing.assert_allclose(res[0]["kl"], kl_ref, rtol=1e-5)
