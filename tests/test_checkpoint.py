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
