"""Reader of the reference's published RLlib checkpoints that executes nothing.

The checkpoints (`Results/**/checkpoint_1250/checkpoint-1250`, consumed by
evaluation/evaluate_trained_policies_pd.py:93-96 through `PPOTrainer.restore`) are pickles
written by Ray 1.0.1: an outer dict whose "worker" entry holds a second pickle with the
rollout worker's state -- per policy the TF variables (`<pid>/fc_1/kernel`, ..., the Adam slots
`.../Adam`, `.../Adam_1`, `<pid>/beta1_power`, `<pid>/beta2_power`) and the RLlib
MeanStdFilter / RunningStat of every policy.

Unpickling would import and call whatever the stream names.  This module never does: it walks
the opcode stream with `pickletools.genops` and evaluates it *symbolically* -- GLOBAL /
STACK_GLOBAL become inert `Global(module, name)` markers, REDUCE / NEWOBJ become inert
`Call` records, BUILD attaches the state to them -- so the result is a tree of dicts, lists,
tuples, scalars, bytes and markers.  Only afterwards are three known marker shapes turned
into numpy data, from their raw little-endian payload bytes: `numpy.core.multiarray._reconstruct`
(+ BUILD state (version, shape, dtype, fortran, raw)), `numpy.core.multiarray.scalar`
(dtype, raw) and `numpy.dtype(str, 0, 1)` (+ BUILD state with the byte order).  Nothing in
the file is imported, called or executed.

    ck = read_checkpoint(path)              # {"worker": {...}, "optimizer": ..., ...}
    pol = policy_state(ck, "policy_FL")     # weights / Adam / beta powers / filter, Keras order
"""
from __future__ import annotations

import pickletools
from dataclasses import dataclass, field

import numpy as np


@dataclass
class Global:
    module: str
    name: str

    @property
    def qualname(self):
        return f"{self.module}.{self.name}"


@dataclass
class Call:
    """An inert REDUCE / NEWOBJ record: func(*args), plus BUILD state and SETITEM(S) items."""
    func: object
    args: tuple
    state: object = None
    items: dict = field(default_factory=dict)
    appended: list = field(default_factory=list)


class _Mark:
    pass


_MARK = _Mark()


class CheckpointFormatError(ValueError):
    pass


def _pop_mark(stack):
    for i in range(len(stack) - 1, -1, -1):
        if stack[i] is _MARK:
            items = stack[i + 1:]
            del stack[i:]
            return items
    raise CheckpointFormatError("MARK expected")


def walk(data: bytes):
    """Symbolic evaluation of one pickle opcode stream (protocol <= 5).  Returns the object
    tree with Global / Call markers in place of anything the stream would construct."""
    stack, memo = [], {}
    for op, arg, pos in pickletools.genops(data):
        n = op.name
        if n in ("PROTO", "FRAME"):
            continue
        if n == "STOP":
            if len(stack) != 1:
                raise CheckpointFormatError(f"stack holds {len(stack)} items at STOP")
            return stack[0]
        if n == "MARK":
            stack.append(_MARK)
        elif n in ("EMPTY_DICT",):
            stack.append({})
        elif n in ("EMPTY_LIST",):
            stack.append([])
        elif n == "EMPTY_TUPLE":
            stack.append(())
        elif n in ("SHORT_BINUNICODE", "BINUNICODE", "BINUNICODE8", "UNICODE", "SHORT_BINSTRING",
                   "BINSTRING", "STRING", "BININT", "BININT1", "BININT2", "INT", "LONG", "LONG1",
                   "LONG4", "BINFLOAT", "FLOAT", "SHORT_BINBYTES", "BINBYTES", "BINBYTES8",
                   "BYTEARRAY8"):
            stack.append(bytes(arg) if n == "BYTEARRAY8" else arg)
        elif n == "NONE":
            stack.append(None)
        elif n == "NEWTRUE":
            stack.append(True)
        elif n == "NEWFALSE":
            stack.append(False)
        elif n == "TUPLE":
            stack.append(tuple(_pop_mark(stack)))
        elif n in ("TUPLE1", "TUPLE2", "TUPLE3"):
            k = int(n[-1])
            t = tuple(stack[-k:])
            del stack[-k:]
            stack.append(t)
        elif n == "LIST":
            stack.append(list(_pop_mark(stack)))
        elif n == "DICT":
            items = _pop_mark(stack)
            stack.append({items[i]: items[i + 1] for i in range(0, len(items), 2)})
        elif n == "APPEND":
            v = stack.pop()
            _append(stack[-1], [v])
        elif n == "APPENDS":
            items = _pop_mark(stack)
            _append(stack[-1], items)
        elif n == "SETITEM":
            v = stack.pop()
            k = stack.pop()
            _setitems(stack[-1], [k, v])
        elif n == "SETITEMS":
            items = _pop_mark(stack)
            _setitems(stack[-1], items)
        elif n == "MEMOIZE":
            memo[len(memo)] = stack[-1]
        elif n in ("BINPUT", "LONG_BINPUT", "PUT"):
            memo[arg] = stack[-1]
        elif n in ("BINGET", "LONG_BINGET", "GET"):
            stack.append(memo[arg])
        elif n == "STACK_GLOBAL":
            name = stack.pop()
            module = stack.pop()
            stack.append(Global(module, name))
        elif n == "GLOBAL":
            module, name = arg.split(" ", 1)
            stack.append(Global(module, name))
        elif n == "REDUCE":
            args = stack.pop()
            func = stack.pop()
            stack.append(Call(func, tuple(args)))
        elif n == "NEWOBJ":
            args = stack.pop()
            cls = stack.pop()
            stack.append(Call(cls, tuple(args)))
        elif n == "BUILD":
            state = stack.pop()
            obj = stack[-1]
            if not isinstance(obj, Call):
                raise CheckpointFormatError(f"BUILD on {type(obj).__name__} at byte {pos}")
            obj.state = state
        else:
            raise CheckpointFormatError(f"opcode {n} at byte {pos} is not part of the checkpoint format")
    raise CheckpointFormatError("no STOP opcode")


def _append(target, items):
    if isinstance(target, list):
        target.extend(items)
    elif isinstance(target, Call):
        target.appended.extend(items)
    else:
        raise CheckpointFormatError("APPEND to a non-list")


def _setitems(target, items):
    if len(items) % 2:
        raise CheckpointFormatError("odd SETITEMS")
    dst = target if isinstance(target, dict) else target.items if isinstance(target, Call) else None
    if dst is None:
        raise CheckpointFormatError("SETITEM on a non-dict")
    for i in range(0, len(items), 2):
        dst[items[i]] = items[i + 1]


# ---- numpy payloads (data only: dtype strings and raw bytes) -----------------------------
_RECONSTRUCT = {"numpy.core.multiarray._reconstruct", "numpy._core.multiarray._reconstruct"}
_SCALAR = {"numpy.core.multiarray.scalar", "numpy._core.multiarray.scalar"}
_DTYPE = {"numpy.dtype"}
_ALLOWED_DTYPES = {"f2", "f4", "f8", "i1", "i2", "i4", "i8", "u1", "u2", "u4", "u8", "b1"}


def _dtype_of(c):
    if not (isinstance(c, Call) and isinstance(c.func, Global) and c.func.qualname in _DTYPE):
        raise CheckpointFormatError(f"expected a numpy dtype, got {c!r}"[:200])
    code = c.args[0]
    if code not in _ALLOWED_DTYPES:
        raise CheckpointFormatError(f"dtype {code!r} is not a plain numeric type")
    order = "<"
    if isinstance(c.state, tuple) and len(c.state) > 1 and c.state[1] in ("<", ">", "|", "="):
        order = "<" if c.state[1] in ("|", "=") else c.state[1]
    return np.dtype(order + code)


def to_data(x):
    """Replace the numpy markers of a walked tree by arrays / scalars; dicts, lists and tuples
    are converted recursively; any other Call is kept as {"__class__": name, "state": ...}."""
    if isinstance(x, dict):
        return {k: to_data(v) for k, v in x.items()}
    if isinstance(x, list):
        return [to_data(v) for v in x]
    if isinstance(x, tuple):
        return tuple(to_data(v) for v in x)
    if isinstance(x, Call) and isinstance(x.func, Global):
        q = x.func.qualname
        if q in _RECONSTRUCT:
            st = x.state
            if not (isinstance(st, tuple) and len(st) == 5):
                raise CheckpointFormatError("ndarray state must be (version, shape, dtype, fortran, raw)")
            _, shape, dt, fortran, raw = st
            dt = _dtype_of(dt)
            if not isinstance(raw, (bytes, bytearray)):
                raise CheckpointFormatError("ndarray payload is not raw bytes (object array?)")
            a = np.frombuffer(bytes(raw), dt).reshape(shape, order="F" if fortran else "C")
            return a.astype(dt.newbyteorder("="), copy=True)
        if q in _SCALAR:
            dt = _dtype_of(x.args[0])
            return np.frombuffer(bytes(x.args[1]), dt)[0].astype(dt.newbyteorder("="))
        if q in _DTYPE:
            return _dtype_of(x)
        if q == "collections.OrderedDict":
            d = {}
            for pair in (x.args[0] if x.args else []):
                d[pair[0]] = to_data(pair[1])
            d.update({k: to_data(v) for k, v in x.items.items()})
            return d
        return {"__class__": q, "args": to_data(x.args), "state": to_data(x.state)}
    return x


def read_checkpoint(path):
    """The checkpoint as plain data; the nested "worker" pickle is walked too."""
    with open(path, "rb") as f:
        outer = to_data(walk(f.read()))
    if isinstance(outer, dict) and isinstance(outer.get("worker"), (bytes, bytearray)):
        outer["worker"] = to_data(walk(bytes(outer["worker"])))
    return outer


FFN_KEYS = ["fc_1/kernel", "fc_1/bias", "fc_value_1/kernel", "fc_value_1/bias", "fc_2/kernel", "fc_2/bias",
            "fc_value_2/kernel", "fc_value_2/bias", "fc_out/kernel", "fc_out/bias", "value_out/kernel",
            "value_out/bias"]


def _weights_dict(worker, pid):
    st = worker.get("state", {}).get(pid)
    if st is None:
        raise KeyError(f"checkpoint has no state for policy {pid!r}: {sorted(worker.get('state', {}))}")
    w = st[0] if isinstance(st, (tuple, list)) else st
    return w if isinstance(w, dict) else st


def policy_state(ck, pid):
    """One policy's state in the C-ABI's order (ddrl_params_set / ddrl_adam_set /
    ddrl_policy_filter_set): flat fp32 weights, Adam m and v in the same order, beta powers, and
    the RLlib MeanStdFilter's RunningStat (n, M, S) in fp64 (None if the policy has none)."""
    worker = ck["worker"]
    w = _weights_dict(worker, pid)
    # TF1 optimizer slots: "<pid>/beta1_power", "<pid>/<pid>/fc_1/kernel/Adam", ".../Adam_1"
    opt = w.get("_optimizer_variables", {})

    def var(name):
        k = f"{pid}/{name}"
        if k in w:
            return np.asarray(w[k])
        raise KeyError(f"{pid}: no variable {name!r}")

    def slot(name):
        for k in (f"{pid}/{pid}/{name}", f"{pid}/{name}"):
            if k in opt:
                return np.asarray(opt[k])
        raise KeyError(f"{pid}: no optimizer variable {name!r}")

    names = [k for k in w if k != "_optimizer_variables"]
    shapes = [(k, var(k).shape) for k in FFN_KEYS]
    flat = np.concatenate([var(k).astype(np.float32).reshape(-1) for k in FFN_KEYS])
    m = np.concatenate([slot(k + "/Adam").astype(np.float32).reshape(-1) for k in FFN_KEYS])
    v = np.concatenate([slot(k + "/Adam_1").astype(np.float32).reshape(-1) for k in FFN_KEYS])
    b1p, b2p = float(np.float32(opt[f"{pid}/beta1_power"])), float(np.float32(opt[f"{pid}/beta2_power"]))
    learner = ck.get("train_exec_impl", {}) or {}
    learner = (learner.get("info") or {}).get("learner", {}).get(pid, {})
    filt = None
    f = worker.get("filters", {}).get(pid)
    if isinstance(f, dict) and f.get("__class__", "").endswith("MeanStdFilter"):
        rs = f["state"]["rs"]["state"]
        filt = (float(rs["_n"]), np.asarray(rs["_M"], np.float64), np.asarray(rs["_S"], np.float64))
    return {"weights": flat, "adam_m": m, "adam_v": v, "beta_powers": (b1p, b2p), "filter": filt,
            "kl_coeff": float(learner["cur_kl_coeff"]) if "cur_kl_coeff" in learner else None,
            "learner_stats": {k: float(v) for k, v in learner.items() if np.ndim(v) == 0 and
                              isinstance(v, (float, int, np.floating, np.integer))},
            "shapes": shapes, "variable_order": names, "optimizer_order": list(opt.keys())}


def policy_ids(ck):
    """Policy ids of the checkpoint's worker state, in the file's order."""
    return list(ck["worker"]["state"].keys())
