"""f2: the no-code reader of the reference's RLlib checkpoints (ddrl_amd/rllib_checkpoint.py).

The reader walks the pickle opcode stream (pickletools.genops) and evaluates it symbolically;
nothing in a file is imported or called.  Pinned here against the reference's own data:
  * every one of the 120 published checkpoints (when /root/reference is present) reads, and
    every policy's variables come in the Keras order the C-ABI takes (ddrl_params_set,
    include/ddrl_hip.h) with the oracle's shapes (ffn_param_shapes(d, 2A)), Adam slots in the
    same order, fp32, plus an RLlib RunningStat of width d;
  * the committed fixture tests/golden/ckpt_local_1250.npz (made by make_checkpoint_fixture.py)
    equals a fresh read, and its learner statistics satisfy RLlib 1.0's loss identity
    total = policy + kl_coeff * kl + vf_coeff * vf (train_exec_impl.info.learner);
  * a crafted pickle naming os.system stays an inert marker.
"""
import glob
import json
import os
import pickle

import numpy as np
import pytest

from ddrl_amd import rllib_checkpoint as RC
from oracle import ddrl_oracle as O

HERE = os.path.dirname(os.path.abspath(__file__))
FIX = os.path.join(HERE, "golden", "ckpt_local_1250.npz")
REF = "/root/reference/Results"
have_ref = pytest.mark.skipif(not os.path.isdir(REF), reason="reference checkpoints not in this container")


def _fixture():
    z = np.load(FIX, allow_pickle=False)
    pids = json.loads(bytes(z["policy_ids"]).decode())
    return z, pids


def test_fixture_layout_matches_oracle_and_cabi_order():
    z, pids = _fixture()
    assert pids == ["policy_FL", "policy_FR", "policy_HL", "policy_HR"]
    shapes = O.ffn_param_shapes(35, 4)
    n = sum(int(np.prod(s)) for _, s in shapes)
    assert n == 13253   # d = 35 -> 13,253 (= ddrl_param_count of the Local context)
    for pid in pids:
        w, m, v = z[f"{pid}/weights"], z[f"{pid}/adam_m"], z[f"{pid}/adam_v"]
        assert w.dtype == m.dtype == v.dtype == np.float32 and w.shape == m.shape == v.shape == (n,)
        assert np.isfinite(w).all() and (v >= 0).all()
        p = O.unpack(w, shapes)
        assert np.abs(p["fc_1/kernel"]).max() > 0.05        # trained weights, not an init
        assert z[f"{pid}/filter_M"].shape == z[f"{pid}/filter_S"].shape == (35,)
        assert int(z[f"{pid}/filter_n"][0]) > 2e7 - 1e5
        b1p, b2p = z[f"{pid}/beta_powers"]
        assert 0.0 <= b1p < 1 and 0.0 <= b2p < 1         # 1.56M Adam steps: both underflow to 0 in fp32


def test_fixture_learner_stats_satisfy_loss_identity():
    z, pids = _fixture()
    for pid in pids:
        st = json.loads(bytes(z[f"{pid}/learner_stats"]).decode())
        kl = float(z[f"{pid}/kl_coeff"][0])
        assert kl == pytest.approx(st["cur_kl_coeff"])
        tot = st["policy_loss"] + kl * st["kl"] + 0.5 * st["vf_loss"] - st["entropy_coeff"] * st["entropy"]
        assert tot == pytest.approx(st["total_loss"], rel=2e-6)


def test_crafted_pickle_stays_inert(tmp_path):
    marker = tmp_path / "executed"

    class Evil:
        def __reduce__(self):
            return (os.system, (f"touch {marker}",))

    data = pickle.dumps({"worker": Evil()}, protocol=4)   # dumps runs __reduce__, never os.system
    tree = RC.walk(data)
    call = tree["worker"]
    assert isinstance(call, RC.Call) and call.func.qualname in ("posix.system", "os.system")
    out = RC.to_data(tree)
    assert out["worker"]["__class__"] in ("posix.system", "os.system")
    assert not marker.exists()


def test_reader_rejects_non_numeric_array_payloads():
    data = pickle.dumps(np.array(["a", "b"], dtype=object), protocol=4)
    with pytest.raises(RC.CheckpointFormatError):
        RC.to_data(RC.walk(data))


def test_reader_round_trips_numpy_arrays_and_scalars():
    src = {"a": np.arange(12, dtype=np.float32).reshape(3, 4), "b": np.float64(2.5), "c": [1, (2, 3)],
           "d": np.asfortranarray(np.arange(6, dtype=np.int64).reshape(2, 3)), "e": np.zeros(0, ">f8")}
    out = RC.to_data(RC.walk(pickle.dumps(src, protocol=4)))
    np.testing.assert_array_equal(out["a"], src["a"])
    assert out["b"] == 2.5 and out["c"] == [1, (2, 3)]
    np.testing.assert_array_equal(out["d"], src["d"])
    assert out["e"].shape == (0,)


@have_ref
def test_fixture_equals_fresh_read():
    from tests.golden.make_checkpoint_fixture import LOCAL
    z, pids = _fixture()
    ck = RC.read_checkpoint(os.path.join(REF, LOCAL))
    assert RC.policy_ids(ck) == pids
    for pid in pids:
        s = RC.policy_state(ck, pid)
        np.testing.assert_array_equal(s["weights"], z[f"{pid}/weights"])
        np.testing.assert_array_equal(s["adam_m"], z[f"{pid}/adam_m"])
        np.testing.assert_array_equal(s["filter"][1], z[f"{pid}/filter_M"])


@have_ref
def test_every_published_checkpoint_reads_in_cabi_order():
    files = sorted(glob.glob(os.path.join(REF, "**/checkpoint-1250"), recursive=True))
    assert len(files) == 120
    keys = [n for n, _ in O.ffn_param_shapes(1, 2)]
    seen = set()
    for f in files:
        ck = RC.read_checkpoint(f)
        for pid in RC.policy_ids(ck):
            s = RC.policy_state(ck, pid)
            d, out = s["shapes"][0][1][0], s["shapes"][8][1][1]
            seen.add((d, out))
            assert s["variable_order"] == [f"{pid}/{k}" for k in keys]          # Keras = C-ABI order
            assert [tuple(sh) for _, sh in s["shapes"]] == [sh for _, sh in O.ffn_param_shapes(d, out)]
            slots = [f"{pid}/beta1_power", f"{pid}/beta2_power"] + [
                f"{pid}/{pid}/{k}/{a}" for k in keys for a in ("Adam", "Adam_1")]
            assert s["optimizer_order"] == slots
            assert s["weights"].size == s["adam_m"].size == s["adam_v"].size == sum(
                int(np.prod(sh)) for _, sh in O.ffn_param_shapes(d, out))
            assert s["filter"][1].shape == (d,)
    # d in {19, 27, 35, 43} and TVel {20, 28, 36, 44}, A in {2, 4, 8}
    assert {d for d, _ in seen} == {19, 20, 27, 28, 35, 36, 43, 44}
    assert {o // 2 for _, o in seen} == {2, 4, 8}


# ---- writer (f2, second half) -------------------------------------------------------------
DIGEST = os.path.join(HERE, "golden", "ckpt_local_1250_digest.json")


def _fixture_policies():
    z, pids = _fixture()
    pols = {}
    for pid in pids:
        n = int(z[f"{pid}/filter_n"][0])
        pols[pid] = {"weights": z[f"{pid}/weights"], "adam_m": z[f"{pid}/adam_m"], "adam_v": z[f"{pid}/adam_v"],
                     "beta_powers": tuple(np.float32(b) for b in z[f"{pid}/beta_powers"]),
                     "filter": (n, z[f"{pid}/filter_M"], z[f"{pid}/filter_S"]), "filter_buffer": None,
                     "shapes": RC.ffn_shapes(35, 4)}
    learner = {pid: json.loads(bytes(z[f"{pid}/learner_stats"]).decode()) for pid in pids}
    return pols, learner


def test_writer_rebuilds_published_local_checkpoint_byte_for_byte(tmp_path):
    """The committed fixture (weights, Adam m / v, beta powers, RunningStat, learner stats of the
    published Local policies) written by write_checkpoint gives the published checkpoint-1250
    and its .tune_metadata byte for byte (SHA-256 recorded by make_checkpoint_fixture.py
    --digest): same opcode skeleton, GLOBAL names, key order, dtypes, shapes, memo layout and
    framing as Ray 1.0.1's pickler -- no reference file needed at test time."""
    import hashlib
    dg = json.load(open(DIGEST))
    pols, learner = _fixture_policies()
    md = dg["metadata"]
    path = RC.write_checkpoint(str(tmp_path), 1250, pols, learner, dg["counters"]["num_steps_sampled"],
                               time_total=md["time_total"], episodes_total=md["episodes_total"],
                               experiment_id=md["experiment_id"], ray_version=md["ray_version"])
    assert path.endswith("checkpoint_1250/checkpoint-1250")
    raw = open(path, "rb").read()
    assert len(raw) == dg["bytes"]
    assert hashlib.sha256(raw).hexdigest() == dg["sha256"]
    assert hashlib.sha256(open(path + ".tune_metadata", "rb").read()).hexdigest() == dg["metadata_sha256"]
    assert os.path.exists(os.path.join(os.path.dirname(path), ".is_checkpoint"))


def test_writer_round_trips_through_the_reader(tmp_path):
    """Arbitrary state (cup-model fcnet with the coupling table, d = 19, A = 2, NoFilter on one
    policy) written, then read back with read_checkpoint / policy_state: bit-exact."""
    rng = np.random.default_rng(5)
    shapes = RC.ffn_shapes(19, 4) + [("leg_coupling", (4, 2))]
    n = sum(int(np.prod(s)) for _, s in shapes)
    pols = {}
    for k, pid in enumerate(["policy_legs", "policy_other"]):
        pols[pid] = {"weights": rng.normal(size=n).astype(np.float32), "adam_m": rng.normal(size=n).astype(np.float32),
                     "adam_v": rng.random(n).astype(np.float32), "beta_powers": (np.float32(0.9 ** 7), np.float32(0.999 ** 7)),
                     "filter": (12345, rng.normal(size=19), rng.random(19) * 5) if k == 0 else None,
                     "filter_buffer": None, "shapes": shapes}
    pols["policy_other"]["filter_kind"] = "NoFilter"
    learner = {pid: {"cur_kl_coeff": 0.3, "cur_lr": 3e-4, "total_loss": 1.5, "policy_loss": -0.01, "vf_loss": 3.0,
                     "vf_explained_var": 0.2, "kl": 0.012, "entropy": 1.1, "entropy_coeff": 0.0} for pid in pols}
    path = RC.write_checkpoint(str(tmp_path), 7, pols, learner, 4096 * 200 * 7, experiment_id="x")
    ck = RC.read_checkpoint(path)
    assert RC.policy_ids(ck) == list(pols)
    s = RC.policy_state(ck, "policy_legs")
    np.testing.assert_array_equal(s["weights"], pols["policy_legs"]["weights"])
    assert [k for k, _ in s["shapes"]] == [k for k, _ in shapes]
    w = ck["worker"]["state"]["policy_legs"]
    np.testing.assert_array_equal(w["policy_legs/leg_coupling"].reshape(-1), pols["policy_legs"]["weights"][n - 8:])
    np.testing.assert_array_equal(s["adam_m"], pols["policy_legs"]["adam_m"])
    np.testing.assert_array_equal(s["adam_v"], pols["policy_legs"]["adam_v"])
    assert s["beta_powers"] == (float(np.float32(0.9 ** 7)), float(np.float32(0.999 ** 7)))
    assert s["filter"][0] == 12345
    np.testing.assert_array_equal(s["filter"][1], pols["policy_legs"]["filter"][1])
    assert s["kl_coeff"] == 0.3 and s["learner_stats"]["kl"] == pytest.approx(0.012)
    assert ck["worker"]["filters"]["policy_other"]["__class__"] == "ray.rllib.utils.filter.NoFilter"
    assert ck["train_exec_impl"]["counters"]["num_steps_trained"] == 4096 * 200 * 7
    md = RC.to_data(RC.walk(open(path + ".tune_metadata", "rb").read()))
    assert md["iteration"] == 7 and md["ray_version"] == "1.0.1"


def test_emit_inverts_walk_on_crafted_streams():
    """emit(walk(x)) == x for pickles CPython writes with protocol 4: nested containers, shared
    references, long strings / bytes past the 64 KiB frame, large ints, batches > 1000."""
    shared = ("s", 1)
    obj = {"a": [1, 2.5, None, True, False, -7, 70000, 2 ** 40, -(2 ** 70)], "b": shared, "c": shared,
           "big": b"x" * 70000, "str": "y" * 300, "many": list(range(2500)), "d": {str(i): i for i in range(1200)},
           "t": (1, 2, 3, 4), "e": (), "arr": np.arange(6, dtype=np.float32).reshape(2, 3)}
    data = pickle.dumps(obj, protocol=4)
    assert RC.emit(RC.walk(data)) == data


@have_ref
def test_writer_rebuilds_every_published_checkpoint():
    """All 120 published checkpoints (+ metadata): emit(walk(file)) is the file, and
    write-from-contents (published_policies + learner stats + counters) is the file."""
    files = sorted(glob.glob(os.path.join(REF, "**/checkpoint-1250"), recursive=True))
    assert len(files) == 120
    for f in files:
        raw = open(f, "rb").read()
        assert RC.emit(RC.walk(raw)) == raw, f
        ck = RC.read_checkpoint(f)
        inner = RC.emit(RC.worker_tree(RC.published_policies(ck)))
        t = ck["train_exec_impl"]
        assert RC.emit(RC.checkpoint_tree(inner, t["info"]["learner"], t["counters"]["num_steps_sampled"])) == raw, f
        md_raw = open(f + ".tune_metadata", "rb").read()
        md = RC.to_data(RC.walk(md_raw))
        assert RC.emit(RC.metadata_tree(md["iteration"], md["time_total"], md["episodes_total"],
                                        md["experiment_id"], md["ray_version"])) == md_raw, f


@pytest.mark.parametrize("layer", O.GNN_LAYERS)
def test_gnn_variable_names_agree_between_writer_and_oracle(layer):
    """One naming for the GNN variables: the Keras attribute names of models/gcn.py:19,46-47,
    102-103,159-160 (msg_transform, node_update, linear, pre_att_linear, att_linear) in the
    writer's layout (rllib_checkpoint.gnn_shapes) and in the oracle's parameter dicts."""
    assert [(n, tuple(s)) for n, s in RC.gnn_shapes(4, layer=layer)] == \
        [(n, tuple(s)) for n, s in O.gnn_param_shapes(4, layer=layer)]
