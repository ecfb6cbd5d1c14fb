"""Generate the committed golden fixtures under tests/golden/ from the reference snapshot.

This script is test infrastructure.  It runs only in the build container, where
/root/reference exists.  It never imports or executes reference code:

* Layout tables.  The reference's Python sources are parsed as TEXT with `ast`.  We take
  the literal field lists OBS_FIELDS / ACTION_FIELDS / CONTACT_FORCE_FIELDS
  (simulation_envs/quantruped_v3.py:68-112).  We also take every
  `get_obs_indices([...])`, `get_action_indices([...])` and
  `get_contact_force_indices([...], weights=[...])` call with literal arguments, for
  each env class in simulation_envs/*.py.  The index tables are then computed with the
  reference's prefix algorithm (quantruped_v3.py:282-341), restated here on its own so
  that it cross-checks ddrl_amd/simulation_envs/layouts.py.
* Recorded learner statistics (known-answer vectors for the PPO loss composition).
  These come from experiment_state-*.json (plain JSON).  Each scalar is stored there as
  a hex pickle byte-string ("CLOUDPICKLE_FALLBACK").  We do NOT unpickle it.  The float
  is the 4-byte payload of the SHORT_BINBYTES opcode ('C' = 0x43, length 0x04) that
  numpy's scalar reconstruction carries.  We cut those 4 bytes out with a regex and
  decode them as little-endian float32.
* The recorded PPO configuration (params.json, plain JSON) of the Local run.

Usage:  python tests/golden/make_golden.py   (writes tests/golden/*.json)
"""
import ast
import glob
import json
import os
import re
import struct

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))


def _literal_list_assign(tree, cls_name, attr):
    for node in ast.walk(tree):
        if isinstance(node, ast.ClassDef) and node.name == cls_name:
            for stmt in node.body:
                if isinstance(stmt, ast.Assign) and any(
                        isinstance(t, ast.Name) and t.id == attr for t in stmt.targets):
                    return ast.literal_eval(stmt.value)
    raise KeyError((cls_name, attr))


def _prefix_indices(fields, prefixes):
    # Restatement of quantruped_v3.py:282-300 (order follows the prefix list; inside one
    # prefix the order is the field order).
    out = []
    for p in prefixes:
        out.extend(i for i, f in enumerate(fields) if f.startswith(p))
    return out


def _contact_indices(fields, prefixes, weights):
    # Restatement of quantruped_v3.py:318-341.
    idx, w = [], []
    if weights is None:
        weights = [1.0] * len(prefixes)
    for p, wt in zip(prefixes, weights):
        sel = [i for i, f in enumerate(fields) if f.startswith(p)]
        idx.extend(sel)
        w.extend([float(wt)] * len(sel))
    return idx, w


def _call_name(call):
    f = call.func
    return f.attr if isinstance(f, ast.Attribute) else None


def _table_key(target):
    # self.obs_indices["agent_FL"]  ->  ("obs_indices", "agent_FL")
    if isinstance(target, ast.Subscript) and isinstance(target.value, ast.Attribute):
        key = target.slice
        if isinstance(key, ast.Constant):
            return target.value.attr, key.value
    return None


def _const(node):
    """Evaluate a literal, allowing constant arithmetic such as `1./4.` (no names, no calls)."""
    if isinstance(node, ast.BinOp) and isinstance(node.op, (ast.Add, ast.Sub, ast.Mult, ast.Div)):
        a, b = _const(node.left), _const(node.right)
        return {ast.Add: a + b, ast.Sub: a - b, ast.Mult: a * b,
                ast.Div: a / b if b else None}[type(node.op)]
    if isinstance(node, (ast.List, ast.Tuple)):
        return [_const(e) for e in node.elts]
    return ast.literal_eval(node)


def _eval_call(call, tabs):
    name = _call_name(call)
    args = [_const(a) for a in call.args]
    kw = {k.arg: _const(k.value) for k in call.keywords}
    prefixes = args[0] if args else None
    if name == "get_obs_indices":
        return ("obs", prefixes)
    if name == "get_action_indices":
        return ("act", prefixes)
    if name == "get_contact_force_indices":
        return ("contact", prefixes, kw.get("weights", args[1] if len(args) > 1 else None))
    return None


def extract_env_tables():
    v3 = ast.parse(open(os.path.join(REF, "simulation_envs/quantruped_v3.py")).read())
    obs_fields = _literal_list_assign(v3, "QuAntrupedEnv", "OBS_FIELDS")
    act_fields = _literal_list_assign(v3, "QuAntrupedEnv", "ACTION_FIELDS")
    cf_fields = _literal_list_assign(v3, "QuAntrupedEnv", "CONTACT_FORCE_FIELDS")
    tvel_fields = _literal_list_assign(v3, "QuAntrupedTVelEnv", "OBS_FIELDS")

    classes = {}
    for path in sorted(glob.glob(os.path.join(REF, "simulation_envs", "*.py"))):
        tree = ast.parse(open(path).read())
        for cls in [n for n in tree.body if isinstance(n, ast.ClassDef)]:
            info = {"file": os.path.relpath(path, REF), "line": cls.lineno,
                    "bases": [ast.unparse(b) for b in cls.bases]}
            specs = {"obs_indices": {}, "action_indices": {}, "contact_force_indices": {}}
            for stmt in cls.body:
                if isinstance(stmt, ast.Assign) and len(stmt.targets) == 1 and \
                        isinstance(stmt.targets[0], ast.Name) and \
                        stmt.targets[0].id in ("policy_names", "agent_names"):
                    info[stmt.targets[0].id] = ast.literal_eval(stmt.value)
                if isinstance(stmt, ast.FunctionDef) and stmt.name == "__init__":
                    for node in ast.walk(stmt):
                        if not isinstance(node, ast.Assign) or len(node.targets) != 1:
                            continue
                        tgt = node.targets[0]
                        # self.X = { 'agent': self.env.get_*(...) , ... }
                        if isinstance(tgt, ast.Attribute) and tgt.attr in specs and \
                                isinstance(node.value, ast.Dict):
                            for k, v in zip(node.value.keys, node.value.values):
                                if isinstance(v, ast.Call):
                                    specs[tgt.attr][ast.literal_eval(k)] = _eval_call(v, specs)
                        # self.X["agent"] = self.env.get_*(...)  or alias of another entry
                        tk = _table_key(tgt)
                        if tk and tk[0] in specs:
                            if isinstance(node.value, ast.Call):
                                specs[tk[0]][tk[1]] = _eval_call(node.value, specs)
                            else:
                                src = _table_key(node.value)
                                if src:
                                    specs[tk[0]][tk[1]] = ("alias", src[1])
            tables = {}
            for tab, entries in specs.items():
                res = {}
                for agent, spec in entries.items():
                    while spec[0] == "alias":
                        spec = entries[spec[1]]
                    if spec[0] == "obs":
                        res[agent] = {"prefixes": spec[1],
                                      "indices": list(range(len(obs_fields))) if spec[1] is None
                                      else _prefix_indices(obs_fields, spec[1])}
                    elif spec[0] == "act":
                        res[agent] = {"prefixes": spec[1],
                                      "indices": list(range(len(act_fields))) if spec[1] is None
                                      else _prefix_indices(act_fields, spec[1])}
                    else:
                        if spec[1] is None:
                            i, w = list(range(len(cf_fields))), [1.0] * len(cf_fields)
                        else:
                            i, w = _contact_indices(cf_fields, spec[1], spec[2])
                        res[agent] = {"prefixes": spec[1], "weights_in": spec[2],
                                      "indices": i, "weights": w}
                if res:
                    tables[tab] = res
            info["tables"] = tables
            classes[cls.name] = info
    return {
        "source": "parsed as text from /root/reference/simulation_envs/*.py (ast); never imported",
        "OBS_FIELDS": obs_fields, "ACTION_FIELDS": act_fields,
        "CONTACT_FORCE_FIELDS": cf_fields, "TVEL_OBS_FIELDS": tvel_fields,
        "classes": classes,
    }


_F32 = re.compile(r"4304([0-9a-f]{8})94")


def _decode_scalar(hexstr):
    m = _F32.search(hexstr)
    if not m:
        return None
    return struct.unpack("<f", bytes.fromhex(m.group(1)))[0]


def extract_learner_stats():
    """Known-answer learner stats: last checkpointed result of each exp-3 TVel trial."""
    rows = []
    for path in sorted(glob.glob(os.path.join(
            REF, "Results/experiment_3_models_curriculum_tvel/*/experiment_state-*.json"))):
        d = json.load(open(path))
        for trial in d.get("checkpoints", []):
            if isinstance(trial, str):
                trial = json.loads(trial)
            res = trial.get("last_result") or {}
            learner = ((res.get("info") or {}).get("learner")) or {}
            for pid, st in learner.items():
                rec = {"file": os.path.relpath(path, REF), "trial": trial.get("trial_id"),
                       "policy": pid, "cur_kl_coeff": st.get("cur_kl_coeff"),
                       "cur_lr": st.get("cur_lr"), "entropy_coeff": st.get("entropy_coeff")}
                ok = True
                for k in ("total_loss", "policy_loss", "vf_loss", "kl", "entropy",
                          "vf_explained_var"):
                    v = st.get(k)
                    if isinstance(v, dict) and "value" in v:
                        v = _decode_scalar(v["value"])
                    if v is None:
                        ok = False
                    rec[k] = v
                if ok:
                    rows.append(rec)
            timers = res.get("timers")
            if timers and learner:
                rows.append({"file": os.path.relpath(path, REF), "trial": trial.get("trial_id"),
                             "timers": timers, "n_policies": len(learner),
                             "sampler_perf": res.get("sampler_perf")})
    return rows


def extract_params():
    path = glob.glob(os.path.join(
        REF, "Results/experiment_1_models_architectures_on_flat/HF_10_QuantrupedMultiEnv_Local/"
        "PPO_QuantrupedMultiEnv_Local_1a49c_00000_*/params.json"))[0]
    d = json.load(open(path))
    d.pop("multiagent", None)
    d.pop("callbacks", None)
    d["_source"] = os.path.relpath(path, REF)
    return d


def main():
    with open(os.path.join(OUT, "layout_tables.json"), "w") as f:
        json.dump(extract_env_tables(), f, indent=1)
    with open(os.path.join(OUT, "learner_stats.json"), "w") as f:
        json.dump(extract_learner_stats(), f, indent=1)
    with open(os.path.join(OUT, "ppo_params_local.json"), "w") as f:
        json.dump(extract_params(), f, indent=1, sort_keys=True)
    print("wrote", os.listdir(OUT))


if __name__ == "__main__":
    main()
