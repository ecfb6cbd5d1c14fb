"""Fixture (SURVEY 8(c) plan item i): the published QuantrupedMultiEnv_Local policies at
checkpoint 1250 (Results/experiment_1_models_architectures_on_flat/HF_10_QuantrupedMultiEnv_Local/
PPO_..._00000_0_.../checkpoint_1250/checkpoint-1250, 20M env steps), read with the no-code reader
ddrl_amd/rllib_checkpoint.py (pickletools opcode walk; nothing in the file is executed):
per policy the Keras-order weights, Adam m / v, beta powers, the RLlib MeanStdFilter RunningStat
(n, M, S) and the KL coefficient, plus the variable / optimizer-slot order and shapes of one
checkpoint of every published architecture (JSON).

    python tests/golden/make_checkpoint_fixture.py            # in the container (needs /root/reference)
    python tests/golden/make_checkpoint_fixture.py --digest   # + ckpt_local_1250_digest.json (writer test)
"""
import glob
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
from ddrl_amd.rllib_checkpoint import policy_ids, policy_state, read_checkpoint  # noqa: E402

REF = "/root/reference/Results"
LOCAL = "experiment_1_models_architectures_on_flat/HF_10_QuantrupedMultiEnv_Local/" \
        "PPO_QuantrupedMultiEnv_Local_1a49c_00000_0_2020-12-04_12-08-56/checkpoint_1250/checkpoint-1250"


def main():
    ck = read_checkpoint(os.path.join(REF, LOCAL))
    out = {}
    for pid in policy_ids(ck):
        s = policy_state(ck, pid)
        out[f"{pid}/weights"] = s["weights"]
        out[f"{pid}/adam_m"], out[f"{pid}/adam_v"] = s["adam_m"], s["adam_v"]
        out[f"{pid}/beta_powers"] = np.array(s["beta_powers"], np.float32)
        n, M, S = s["filter"]
        out[f"{pid}/filter_n"], out[f"{pid}/filter_M"], out[f"{pid}/filter_S"] = np.array([n]), M, S
        out[f"{pid}/kl_coeff"] = np.array([s["kl_coeff"]])
        out[f"{pid}/learner_stats"] = np.frombuffer(json.dumps(s["learner_stats"]).encode(), np.uint8)
    out["policy_ids"] = np.frombuffer(json.dumps(policy_ids(ck)).encode(), np.uint8)
    out["source"] = np.frombuffer(LOCAL.encode(), np.uint8)
    np.savez_compressed(os.path.join(HERE, "ckpt_local_1250.npz"), **out)

    # variable / slot order and shapes of every published architecture (one trial each)
    orders = {}
    for f in sorted(glob.glob(os.path.join(REF, "**/checkpoint-1250"), recursive=True)):
        arch = f.split("/")[-4]
        if arch in orders:
            continue
        ck = read_checkpoint(f)
        orders[arch] = {pid: {"variables": [[k, list(v)] for k, v in policy_state(ck, pid)["shapes"]],
                              "variable_order": policy_state(ck, pid)["variable_order"],
                              "optimizer_order": policy_state(ck, pid)["optimizer_order"]}
                        for pid in policy_ids(ck)}
    with open(os.path.join(HERE, "ckpt_layouts.json"), "w") as fh:
        json.dump(orders, fh, indent=0)
    print("wrote ckpt_local_1250.npz and ckpt_layouts.json for", len(orders), "architectures")


def digests():
    """ckpt_local_1250_digest.json: what the writer test needs besides the npz to rebuild the
    published Local checkpoint byte for byte -- the SHA-256 of checkpoint-1250 and of its
    .tune_metadata, the metadata fields, the trainer counters and the (empty) filter buffers."""
    import hashlib
    from ddrl_amd.rllib_checkpoint import to_data, walk
    path = os.path.join(REF, LOCAL)
    ck = read_checkpoint(path)
    raw = open(path, "rb").read()
    md_raw = open(path + ".tune_metadata", "rb").read()
    buffers = {}
    for pid in policy_ids(ck):
        b = ck["worker"]["filters"][pid]["state"]["buffer"]["state"]
        assert b["_n"] == 0 and not np.any(b["_M"]) and not np.any(b["_S"])
        buffers[pid] = {"n": 0, "width": int(b["_M"].shape[0])}
    out = {"source": LOCAL, "sha256": hashlib.sha256(raw).hexdigest(), "bytes": len(raw),
           "metadata_sha256": hashlib.sha256(md_raw).hexdigest(), "metadata": to_data(walk(md_raw)),
           "counters": ck["train_exec_impl"]["counters"], "filter_buffers": buffers}
    with open(os.path.join(HERE, "ckpt_local_1250_digest.json"), "w") as fh:
        json.dump(out, fh, indent=1)
    print("wrote ckpt_local_1250_digest.json")


if __name__ == "__main__":
    if "--digest" in sys.argv:
        digests()
    else:
        main()
