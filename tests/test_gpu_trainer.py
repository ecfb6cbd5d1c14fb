"""Trainer-level GPU tests: one PPOTrainer.train() iteration per architecture through the
HIP path (synthetic env), and the data-parallel learner's HIP backend (world size 1
process group) against the oracle.

Tolerances: learner parameters as the fused-update tests (>= 99.9 % within 1e-5 after
a few steps; the DDP apply kernel divides exactly where the fused kernel uses the hardware
reciprocal, so the two HIP paths agree to rounding, not bitwise).
"""
import os
import socket

import numpy as np
import pytest

from oracle import ddrl_oracle as O
from tests.gpu_harness import init_params, make_ctx, run_rollout

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from ddrl_amd import build
    build.build()


@pytest.fixture()
def pg1():
    """A world-size-1 gloo process group for the data-parallel code paths."""
    import torch.distributed as dist
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=0, world_size=1)
    yield
    dist.destroy_process_group()


@pytest.mark.parametrize("env,n,model", [("QuantrupedMultiEnv_Local", 64, None),
                                         ("QuantrupedMultiEnv_SharedDecentral", 48, None),
                                         ("QuantrupedMultiEnv_DecentralShared_Graph", 24, None),
                                         ("QuantrupedMultiEnv_Centralized", 32, None),
                                         ("QuantrupedMultiEnv_SharedDecentralLegID", 32, "cup"),
                                         ("QuantrupedMultiEnv_DecentralShared_Graph", 24, "gnn:gcn"),
                                         ("QuantrupedMultiEnv_DecentralShared_Graph", 24, "gnn:mpnn2"),
                                         ("QuantrupedMultiEnv_DecentralShared_Graph", 24, "gnn:gat1")])
def test_trainer_iteration(env, n, model):
    from ddrl_amd.trainer import PPOTrainer
    extra = {}
    if model:
        name, _, layer = model.partition(":")
        extra = {"model": {"custom_model": name, **({"gnn_layer": layer} if layer else {})}}
    tr = PPOTrainer({"env": env, "rollout_fragment_length": 8, **extra}, n_envs=n, seed=3)
    w0 = {k: v.copy() for k, v in tr.get_weights().items()}
    r = tr.train()
    assert r["timesteps_total"] == 8 * n
    for pid, st in r["info"]["learner"].items():
        for k in ("total_loss", "policy_loss", "vf_loss", "kl", "entropy"):
            assert np.isfinite(st[k]), (pid, k)
        assert not np.array_equal(tr.get_weights()[pid], w0[pid]), "weights did not move"
    tr.stop()


def test_trainer_ddp_world1(pg1, tmp_path):
    """The data-parallel trainer path (filter sync, global standardization, per-step
    grad / all-reduce / apply) on one rank; save / restore round trip."""
    from ddrl_amd.trainer import PPOTrainer
    tr = PPOTrainer({"env": "QuantrupedMultiEnv_SharedDecentral", "rollout_fragment_length": 8,
                     "parallel": "ddp", "observation_filter": "MeanStdFilter"}, n_envs=32, seed=1)
    assert tr.parallel == "ddp"
    r = tr.train()
    st = r["info"]["learner"]["policy_legs"] if "policy_legs" in r["info"]["learner"] else \
        next(iter(r["info"]["learner"].values()))
    assert np.isfinite(st["kl"]) and st["num_ranks"] == 1
    n, M, S = tr.ctx.filter_get()
    assert n == 32 * 9   # reset + 8 steps pushed, synced into the base filter
    pn, _, _ = tr.ctx.policy_filter_get(0)
    assert pn == 32 * 4 * 9 and tr.ctx.policy_filter_get(0, delta=True)[0] == 0   # synced, delta reset
    path = tr.save(str(tmp_path / "ck.npz"))
    w = tr.get_weights()
    tr.train()
    tr.restore(path)
    for k in w:
        np.testing.assert_array_equal(tr.get_weights()[k], w[k])
    tr.stop()


def test_ddp_learner_hip_backend_matches_oracle(pg1):
    import torch
    from ddrl_amd.ddp import Comm, DataParallelLearner, HipBackend
    env, n, T = "QuantrupedMultiEnv_SharedDecentral", 32, 4
    ctx, cfg, inst = make_ctx(env, n, T)
    rng = np.random.default_rng(6)
    params = init_params(ctx, cfg, 12, head_scale=1.0)
    filt = (1000.0, rng.normal(size=43) * 0.3, np.abs(rng.normal(size=43)) * 999.0 + 10.0)
    orc, norms, _, _ = run_rollout(ctx, cfg, inst, params, rng, filt, T)
    lay = ctx.layout[0]
    rec = orc.flat_records(0, lay)
    ctx.records_set(0, rec)
    ctx.adv_norm_set(0, *norms[0])
    learner = DataParallelLearner(HipBackend(ctx), Comm("cpu"), 0, 128, "split")
    sh, pe = O.sgd_schedule(np.random.default_rng(2), rec.shape[0], 128, 2)   # 2 epochs x 4 steps
    grad = torch.zeros(ctx.n_params[0], device="cuda")
    kl = learner.learn(torch.from_numpy(sh).cuda(), pe, 0.2, grad)
    ctx.synchronize()
    mean, den = norms[0]
    batch = dict(obs=rec[:, :19], actions=rec[:, lay["act"]:lay["act"] + 2],
                 logits=rec[:, lay["logit"]:lay["logit"] + 4], logp=rec[:, lay["logp"]],
                 vf_preds=rec[:, lay["vf"]], adv=((rec[:, lay["adv"]] - mean) / den).astype(np.float32),
                 vt=rec[:, lay["vt"]])
    shapes = O.ffn_param_shapes(19, 4)
    adam = O.Adam(ctx.n_params[0])
    new, stats = O.ppo_update("ffn", params[0], shapes, adam, batch, sh, pe, np.float32(0.2), {})
    ref = O.pack(new, shapes)
    got = ctx.params_get(0)
    diff = np.abs(got - ref)
    assert np.mean(diff <= 1e-5 + 1e-5 * np.abs(ref)) >= 0.999 and diff.max() <= 2 * 3e-4 * 8 + 1e-5
    kl_ref = np.mean([s["kl"] for s in stats[-pe.shape[1]:]])
    np.testing.assert_allclose(kl, kl_ref, rtol=1e-4)
    ctx.close()


def _ddp_rank(rank, world, port, out_dir):
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)          # both ranks share the one GPU of the box
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from ddrl_amd.trainer import PPOTrainer
    tr = PPOTrainer({"env": "QuantrupedMultiEnv_SharedDecentral", "rollout_fragment_length": 8,
                     "parallel": "ddp", "observation_filter": "MeanStdFilter"}, n_envs=32, seed=5)
    w0 = tr.get_weights()["policy_legs"] if "policy_legs" in tr.policy_ids else next(iter(tr.get_weights().values()))
    r = tr.train()
    pid = tr.policy_ids[0]
    np.savez(os.path.join(out_dir, f"r{rank}.npz"), rec=tr.ctx.records_get(0), w0=w0, w1=tr.get_weights()[pid],
             env_filter_n=np.array([tr.ctx.filter_get()[0]]), env_filter_M=tr.ctx.filter_get()[1],
             pf_M=tr.ctx.policy_filter_get(0)[1], kl=np.array([r["info"]["learner"][pid]["kl"]]))
    tr.stop()
    dist.destroy_process_group()


def test_trainer_ddp_world2_ranks_sample_differently_and_agree_on_weights():
    """two data-parallel ranks (gloo, sharing the box's GPU) sample DIFFERENT
    trajectories (env and exploration seeds offset by rank) and hold IDENTICAL weights after an
    update (gradient all-reduce, identical Adam); RLlib's per-policy filter is synchronized,
    the env-side filter stays rank-local (a per-process singleton in the reference)."""
    import tempfile
    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    out = tempfile.mkdtemp()
    mp.spawn(_ddp_rank, args=(2, port, out), nprocs=2, join=True)
    a, b = (np.load(os.path.join(out, f"r{r}.npz")) for r in range(2))
    np.testing.assert_array_equal(a["w0"], b["w0"])              # same init
    assert not np.array_equal(a["rec"], b["rec"])                # different trajectories
    assert not np.array_equal(a["w1"], a["w0"])                  # the update moved the weights
    np.testing.assert_array_equal(a["w1"], b["w1"])              # ... identically on both ranks
    np.testing.assert_array_equal(a["pf_M"], b["pf_M"])          # per-policy filter synced
    assert a["env_filter_n"][0] == b["env_filter_n"][0] == 32 * 9   # env filter: own pushes only
    assert not np.array_equal(a["env_filter_M"], b["env_filter_M"])
    assert a["kl"][0] == b["kl"][0]                              # all-reduced KL


def test_trainer_continues_from_published_local_checkpoint():
    """PPOTrainer.load_policy_states (the back end of restore_rllib) with the published Local
    policies (tests/golden/ckpt_local_1250.npz): weights, Adam state, filters and KL
    coefficients land in the context, and a training iteration continues from them."""
    import json
    from ddrl_amd.trainer import PPOTrainer
    z = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "ckpt_local_1250.npz"),
                allow_pickle=False)
    pids = json.loads(bytes(z["policy_ids"]).decode())
    states = {pid: {"weights": z[f"{pid}/weights"], "adam_m": z[f"{pid}/adam_m"], "adam_v": z[f"{pid}/adam_v"],
                    "beta_powers": tuple(float(x) for x in z[f"{pid}/beta_powers"]),
                    "filter": (float(z[f"{pid}/filter_n"][0]), z[f"{pid}/filter_M"], z[f"{pid}/filter_S"]),
                    "kl_coeff": float(z[f"{pid}/kl_coeff"][0])} for pid in pids}
    tr = PPOTrainer({"env": "QuantrupedMultiEnv_Local", "rollout_fragment_length": 8,
                     "observation_filter": "MeanStdFilter"}, n_envs=32, seed=2)
    assert tr.load_policy_states(states) == tr.policy_ids
    for p, pid in enumerate(tr.policy_ids):
        np.testing.assert_array_equal(tr.ctx.params_get(p), states[pid]["weights"])
        m, v, b1, b2 = tr.ctx.adam_get(p)
        np.testing.assert_array_equal(v, states[pid]["adam_v"])
        assert tr.kl_coeff[p] == states[pid]["kl_coeff"]
        assert tr.ctx.policy_filter_get(p)[0] == states[pid]["filter"][0]
    r = tr.train()
    for pid, st in r["info"]["learner"].items():
        assert np.isfinite(st["total_loss"]) and st["cur_kl_coeff"] == pytest.approx(states[pid]["kl_coeff"], rel=1e-6)
    tr.stop()


@pytest.mark.parametrize("env,extra", [
    ("QuantrupedMultiEnv_Local", {"observation_filter": "MeanStdFilter"}),
    ("QuantrupedMultiEnv_SharedDecentralLegID", {"model": {"custom_model": "cup"}}),
    ("QuantrupedMultiEnv_DecentralShared_Graph", {"model": {"custom_model": "gnn"}}),
])
def test_trainer_rllib_checkpoint_round_trip(tmp_path, env, extra):
    """f2 writer: PPOTrainer.save_rllib after one iteration writes the Ray 1.0.1 checkpoint
    layout (tests/test_checkpoint.py pins the writer byte for byte against the published files);
    a fresh trainer's restore_rllib of it restores weights, Adam m / v, beta powers, filters and
    KL coefficients bit for bit, and the learner statistics in the file are the iteration's."""
    from ddrl_amd import rllib_checkpoint as RC
    from ddrl_amd.trainer import PPOTrainer
    cfg = {"env": env, "rollout_fragment_length": 8, **extra}
    tr = PPOTrainer(cfg, n_envs=32, seed=4)
    r = tr.train()
    path = tr.save_rllib(str(tmp_path))
    ck = RC.read_checkpoint(path)
    assert RC.policy_ids(ck) == sorted(tr.policy_ids)
    for pid, st in r["info"]["learner"].items():
        got = ck["train_exec_impl"]["info"]["learner"][pid]
        assert float(got["kl"]) == float(np.float32(st["kl"]))
        assert float(got["total_loss"]) == float(np.float32(st["total_loss"]))
    assert ck["train_exec_impl"]["counters"]["num_steps_sampled"] == tr.timesteps_total
    tr2 = PPOTrainer(cfg, n_envs=32, seed=9)
    assert tr2.restore_rllib(path) == tr2.policy_ids
    for p in range(len(tr.policy_ids)):
        np.testing.assert_array_equal(tr2.ctx.params_get(p), tr.ctx.params_get(p))
        m1, v1, a1, b1 = tr.ctx.adam_get(p)
        m2, v2, a2, b2 = tr2.ctx.adam_get(p)
        np.testing.assert_array_equal(m1, m2)
        np.testing.assert_array_equal(v1, v2)
        assert (a1, b1) == (a2, b2)
        assert tr2.kl_coeff[p] == pytest.approx(tr.kl_coeff[p], rel=1e-7)   # update_kl of the saved coefficient
        if tr.cfg.policy_filter:
            n1, M1, S1 = tr.ctx.policy_filter_get(p)
            n2, M2, S2 = tr2.ctx.policy_filter_get(p)
            assert n1 == n2
            np.testing.assert_array_equal(M1, M2)
    tr.stop()
    tr2.stop()


def _gather_rank(rank, world, port, out_dir, env):
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)          # both ranks share the one GPU of the box
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from ddrl_amd.trainer import PPOTrainer
    tr = PPOTrainer({"env": env, "rollout_fragment_length": 8, "parallel": "gather",
                     "observation_filter": "MeanStdFilter"}, n_envs=32, seed=5)
    P = tr.cfg.n_policies
    w0 = [tr.ctx.params_get(p) for p in range(P)]
    # the schedule the trainer will draw (its generator is the same on every rank)
    sched = np.random.default_rng(5 + 7919)
    r = tr.train()
    out = {"w0_%d" % p: w0[p] for p in range(P)}
    for p in range(P):
        out[f"w1_{p}"] = tr.get_weights()[tr.policy_ids[p]]
        out[f"rec_{p}"] = tr.rctx.records_get(p)
        out[f"union_{p}"] = tr.ctx.records_get(p)
        out[f"norm_{p}"] = tr.ctx.adv_norm_get(p)
        out[f"roll_w_{p}"] = tr.rctx.params_get(p)
        out[f"kl_{p}"] = np.array([r["info"]["learner"][tr.policy_ids[p]]["kl"]])
    np.savez(os.path.join(out_dir, f"g{rank}.npz"), **out)
    tr.stop()
    dist.destroy_process_group()


@pytest.mark.parametrize("env", ["QuantrupedMultiEnv_SharedDecentral", "QuantrupedMultiEnv_Local"])
def test_trainer_gather_world2_equals_single_process_union_update(env):
    """VERDICT r2 item 4, the shared-policy multi-GPU mode with no per-step collective
    ("parallel": "gather"): two ranks (gloo, sharing the box's GPU) roll out DIFFERENT envs,
    all-gather their records once (rank-major union batch) and both run the fused update over
    it with the same schedule.  Their weights are bit-identical, and bit-identical to a
    single-process fused update of a fresh context over the same union batch, initial
    weights, advantage standardization and schedule; the rollout context carries the new
    weights into the next iteration."""
    import tempfile
    import torch
    import torch.multiprocessing as mp
    from ddrl_amd.spec import make_cfg
    from ddrl_amd import native as N
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    out = tempfile.mkdtemp()
    mp.spawn(_gather_rank, args=(2, port, out, env), nprocs=2, join=True)
    a, b = (np.load(os.path.join(out, f"g{r}.npz")) for r in range(2))
    P = len([k for k in a.files if k.startswith("w0_")])
    # reference: one process, one context over all 64 envs, the gathered union batch
    cfg, _ = make_cfg(env, 64, 8, {"observation_filter": "MeanStdFilter"})
    ctx = N.Context(cfg, 0, torch.cuda.current_stream().cuda_stream)
    rng = np.random.default_rng(5 + 7919)
    sh, pe = [], []
    for p in range(P):
        np.testing.assert_array_equal(a[f"w0_{p}"], b[f"w0_{p}"])
        assert not np.array_equal(a[f"rec_{p}"], b[f"rec_{p}"])                  # different envs
        union = np.concatenate([a[f"rec_{p}"], b[f"rec_{p}"]])
        np.testing.assert_array_equal(a[f"union_{p}"], union)                     # rank-major gather
        np.testing.assert_array_equal(b[f"union_{p}"], union)
        ctx.params_set(p, a[f"w0_{p}"])
        ctx.records_set(p, union)
        ctx.adv_norm_set(p, *a[f"norm_{p}"])
        R = union.shape[0]
        nb = R // 128
        sh.append(torch.from_numpy(rng.permutation(R).astype(np.int32)).cuda())
        pe.append(torch.from_numpy(np.stack([rng.permutation(nb) for _ in range(cfg.num_sgd_iter)])
                                   .astype(np.int32)).cuda())
    ctx.ppo_update((1 << P) - 1, sh, pe, [0.2] * P)
    ctx.synchronize()
    for p in range(P):
        ref = ctx.params_get(p)
        assert not np.array_equal(ref, a[f"w0_{p}"])
        np.testing.assert_array_equal(a[f"w1_{p}"], ref)
        np.testing.assert_array_equal(b[f"w1_{p}"], ref)
        np.testing.assert_array_equal(a[f"roll_w_{p}"], ref)
        assert a[f"kl_{p}"][0] == b[f"kl_{p}"][0]
    ctx.close()


def test_trainer_rllib_save_after_restore_keeps_kl_coeff(tmp_path):
    """restore_rllib -> save_rllib -> restore_rllib is the identity on the KL
    coefficient (the saved row carries the restored file's cur_kl_coeff and kl, not kl = 0
    next to the already-updated coefficient), and an npz restore followed by save_rllib writes
    no kl, so a reload keeps the coefficient; "restore_kl_coeff": "config" reproduces RLlib
    1.0.1's restart from config["kl_coeff"]."""
    from ddrl_amd import rllib_checkpoint as RC
    from ddrl_amd.trainer import PPOTrainer
    cfg = {"env": "QuantrupedMultiEnv_Local", "rollout_fragment_length": 8, "kl_coeff": 0.3}
    tr = PPOTrainer(cfg, n_envs=32, seed=4)
    tr.train()
    tr.kl_coeff = [0.45, 0.3, 0.15, 0.6]   # distinct per policy, so a mix-up shows
    tr.last_learner = {pid: {**st, "cur_kl_coeff": c, "kl": k} for (pid, st), c, k in
                       zip(tr.last_learner.items(), (0.3, 0.2, 0.3, 0.4), (0.05, 0.02, 0.001, 0.03))}
    p1 = tr.save_rllib(str(tmp_path / "a"))
    tr2 = PPOTrainer(cfg, n_envs=32, seed=9)
    tr2.restore_rllib(p1)
    k2 = list(tr2.kl_coeff)
    assert k2 == pytest.approx([0.45, 0.2, 0.15, 0.6])   # update_kl(cur, kl) per policy
    p2 = tr2.save_rllib(str(tmp_path / "b"))
    tr3 = PPOTrainer(cfg, n_envs=32, seed=11)
    tr3.restore_rllib(p2)
    assert tr3.kl_coeff == k2
    # npz restore, then save_rllib without training: no kl in the row, coefficient kept
    npz = tr2.save(str(tmp_path / "c.npz"))
    tr4 = PPOTrainer(cfg, n_envs=32, seed=12)
    tr4.restore(npz)
    assert tr4.kl_coeff == k2
    p4 = tr4.save_rllib(str(tmp_path / "d"))
    row = RC.read_checkpoint(p4)["train_exec_impl"]["info"]["learner"][tr4.policy_ids[0]]
    assert "kl" not in row
    tr5 = PPOTrainer(cfg, n_envs=32, seed=13)
    tr5.restore_rllib(p4)
    assert tr5.kl_coeff == pytest.approx(k2, rel=1e-7)
    tr6 = PPOTrainer({**cfg, "restore_kl_coeff": "config"}, n_envs=32, seed=14)
    tr6.restore_rllib(p1)
    assert tr6.kl_coeff == [0.3] * 4
    for t in (tr, tr2, tr3, tr4, tr5, tr6):
        t.stop()


def test_trainer_gather_restore_keeps_policy_filter_and_set_weights_reaches_rollout(tmp_path):
    """in "gather" mode (one rank) restore() makes the restored per-policy
    RunningStat the base of the next filter sync (its count keeps growing from the restored
    value), and set_weights writes the rollout context as well as the learner's."""
    from ddrl_amd.trainer import PPOTrainer
    cfg = {"env": "QuantrupedMultiEnv_Local", "rollout_fragment_length": 8, "parallel": "gather",
           "observation_filter": "MeanStdFilter"}
    tr = PPOTrainer(cfg, n_envs=32, seed=4)
    tr.train()
    tr.train()
    n_saved = tr.ctx.policy_filter_get(0)[0]
    assert n_saved == 2 * 8 * 32 + 32   # reset + 16 steps of 32 envs, one agent per policy
    path = tr.save(str(tmp_path / "g.npz"))
    tr2 = PPOTrainer(cfg, n_envs=32, seed=7)
    tr2.restore(path)
    assert tr2.ctx.policy_filter_get(0)[0] == n_saved
    tr2.train()
    assert tr2.ctx.policy_filter_get(0)[0] == n_saved + 8 * 32   # grows from the restored n
    w = {pid: np.full_like(v, 0.01) for pid, v in tr2.get_weights().items()}
    tr2.set_weights(w)
    for p in range(tr2.cfg.n_policies):
        np.testing.assert_array_equal(tr2.rctx.params_get(p), w[tr2.policy_ids[p]])
    for t in (tr, tr2):
        t.stop()


def test_trainer_host_backend_runs_the_reference_curriculum_callback():
    """a TVel trainer over the host env plane with a 2-velocity list
    (every env draws its own on each reset) and train_experiment_1's on_train_result callback
    unchanged (:171-178: trainer.workers.foreach_worker(... env.update_environment_after_epoch
    ...)), which resets every env after every iteration while the velocities stay."""
    from ddrl_amd.trainer import PPOTrainer
    seen = []

    def on_train_result(info):   # the reference script's callback, verbatim in behaviour
        result = info["result"]
        trainer = info["trainer"]
        timesteps_res = result["timesteps_total"]
        before = trainer.backend.target_velocities
        trainer.workers.foreach_worker(
            lambda ev: ev.foreach_env(lambda env: env.update_environment_after_epoch(timesteps_res)))
        seen.append((before, trainer.backend.target_velocities))

    tr = PPOTrainer({"env": "QuantrupedMultiEnv_Local", "rollout_fragment_length": 8, "env_backend": "host",
                     "env_config": {"target_velocity": [0.5, 1.5]},
                     "callbacks": {"on_train_result": on_train_result}}, n_envs=64, seed=2)
    tv0 = tr.backend.target_velocities
    assert set(np.unique(tv0)) == {0.5, 1.5}
    assert tr.cfg.obs_full_dim == 44
    r = tr.train()
    assert len(seen) == 1 and r["timesteps_total"] == 8 * 64
    np.testing.assert_array_equal(seen[0][1], seen[0][0])   # the reset keeps every env's velocity
    for pid, st in r["info"]["learner"].items():
        assert np.isfinite(st["total_loss"]), pid
    tr.train()
    assert len(seen) == 2
    tr.stop()
