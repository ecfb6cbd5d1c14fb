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


@dataclass(eq=False)
class Call:
    """An inert REDUCE / NEWOBJ record: func(*args), plus BUILD state and SETITEM(S) items.
    newobj: the stream built it with NEWOBJ (cls.__new__(cls, *args)) rather than REDUCE."""
    func: object
    args: tuple
    state: object = None
    items: dict = field(default_factory=dict)
    appended: list = field(default_factory=list)
    newobj: bool = False


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
            stack.append(Call(cls, tuple(args), newobj=True))
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
    # the file's variable order: Keras order (= FFN_KEYS for every published fcnet checkpoint,
    # tests/test_checkpoint.py; "cup" adds leg_coupling, "gnn" its actor / critic variables)
    keys = [k[len(pid) + 1:] for k in names if k.startswith(pid + "/")]
    shapes = [(k, var(k).shape) for k in keys]
    flat = np.concatenate([var(k).astype(np.float32).reshape(-1) for k in keys])
    m = np.concatenate([slot(k + "/Adam").astype(np.float32).reshape(-1) for k in keys])
    v = np.concatenate([slot(k + "/Adam_1").astype(np.float32).reshape(-1) for k in keys])
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


# ---- writer (second half) ------------------------------------------------
# The inverse of walk(): an object tree of dicts, lists, tuples, scalars, bytes and Global /
# Call markers is written as a protocol-4 opcode stream by the same rules CPython's pickler
# follows (Lib/pickle.py, which Ray 1.0.1 used through cloudpickle for these files): 64 KiB
# frames, every str / bytes / non-empty tuple / dict / list / global / constructed object
# memoized by identity on first write and re-referenced with BINGET afterwards, SETITEMS /
# APPENDS in batches of 1000, STACK_GLOBAL for globals.  No class is imported or pickled:
# the markers name the module / qualname as plain strings.  emit(walk(data)) == data for
# every published checkpoint and metadata file (tests/test_checkpoint.py).
import struct as _struct

_FRAME_TARGET = 64 * 1024
_BATCH = 1000


class _Emitter:
    def __init__(self):
        self.out = bytearray()
        self.frame = bytearray()
        self.memo = {}
        self.keep = []   # objects memoized by id stay alive for the whole dump

    # framing: CPython's _Framer (a frame is committed at the start of a save() once it has
    # reached the target; large str / bytes payloads go straight to the file)
    def commit(self, force=False):
        if self.frame is not None and (len(self.frame) >= _FRAME_TARGET or force):
            if len(self.frame) >= 4:
                self.out += b"\x95" + _struct.pack("<Q", len(self.frame))
            self.out += self.frame
            self.frame = bytearray()

    def write(self, b):
        (self.frame if self.frame is not None else self.out).extend(b)

    def write_large(self, header, payload):
        self.commit(force=True)
        self.out += header
        self.out += payload

    def memoize(self, obj):
        self.write(b"\x94")   # MEMOIZE
        self.memo[id(obj)] = len(self.memo)
        self.keep.append(obj)

    def get(self, i):
        self.write(b"h" + _struct.pack("<B", i) if i < 256 else b"j" + _struct.pack("<I", i))

    def dump(self, obj):
        self.out += b"\x80\x04"   # PROTO 4, outside the first frame
        self.save(obj)
        self.write(b".")          # STOP
        self.commit(force=True)
        self.frame = None
        return bytes(self.out)

    def save(self, obj):
        self.commit()
        i = self.memo.get(id(obj))
        if i is not None:
            self.get(i)
            return
        if obj is None:
            self.write(b"N")
        elif obj is True:
            self.write(b"\x88")
        elif obj is False:
            self.write(b"\x89")
        elif isinstance(obj, int):
            self._int(obj)
        elif isinstance(obj, float):
            self.write(b"G" + _struct.pack(">d", obj))
        elif isinstance(obj, str):
            e = obj.encode("utf-8", "surrogatepass")
            if len(e) <= 0xFF:
                self.write(b"\x8c" + _struct.pack("<B", len(e)) + e)
            elif len(e) >= _FRAME_TARGET:
                self.write_large(b"X" + _struct.pack("<I", len(e)), e)
            else:
                self.write(b"X" + _struct.pack("<I", len(e)) + e)
            self.memoize(obj)
        elif isinstance(obj, (bytes, bytearray)):
            b = bytes(obj)
            if len(b) <= 0xFF:
                self.write(b"C" + _struct.pack("<B", len(b)) + b)
            elif len(b) >= _FRAME_TARGET:
                self.write_large(b"B" + _struct.pack("<I", len(b)), b)
            else:
                self.write(b"B" + _struct.pack("<I", len(b)) + b)
            self.memoize(obj)
        elif isinstance(obj, tuple):
            self._tuple(obj)
        elif isinstance(obj, list):
            self.write(b"]")
            self.memoize(obj)
            self._appends(obj)
        elif isinstance(obj, dict):
            self.write(b"}")
            self.memoize(obj)
            self._setitems(list(obj.items()))
        elif isinstance(obj, Global):
            self.save(obj.module)
            self.save(obj.name)
            self.write(b"\x93")   # STACK_GLOBAL
            self.memoize(obj)
        elif isinstance(obj, Call):
            self.save(obj.func)
            self.save(obj.args)
            self.write(b"\x81" if obj.newobj else b"R")   # NEWOBJ / REDUCE
            self.memoize(obj)
            if obj.appended:
                self._appends(obj.appended)
            if obj.items:
                self._setitems(list(obj.items.items()))
            if obj.state is not None:
                self.save(obj.state)
                self.write(b"b")   # BUILD
        else:
            raise CheckpointFormatError(f"cannot write a {type(obj).__name__}")

    def _int(self, x):
        if 0 <= x <= 0xFF:
            self.write(b"K" + _struct.pack("<B", x))
        elif 0 <= x <= 0xFFFF:
            self.write(b"M" + _struct.pack("<H", x))
        elif -0x80000000 <= x <= 0x7FFFFFFF:
            self.write(b"J" + _struct.pack("<i", x))
        else:
            e = x.to_bytes((x.bit_length() + 8) // 8, "little", signed=True) if x else b""
            self.write(b"\x8a" + _struct.pack("<B", len(e)) + e if len(e) < 256 else
                       b"\x8b" + _struct.pack("<i", len(e)) + e)

    def _tuple(self, t):
        if not t:
            self.write(b")")   # EMPTY_TUPLE, never memoized
            return
        if len(t) <= 3:
            for x in t:
                self.save(x)
            if id(t) in self.memo:   # recursive reference (never in these files)
                self.write(b"0" * len(t))
                self.get(self.memo[id(t)])
                return
            self.write({1: b"\x85", 2: b"\x86", 3: b"\x87"}[len(t)])
            self.memoize(t)
            return
        self.write(b"(")
        for x in t:
            self.save(x)
        self.write(b"t")
        self.memoize(t)

    def _appends(self, items):
        for k in range(0, max(len(items), 1), _BATCH):
            chunk = items[k:k + _BATCH]
            if len(chunk) > 1:
                self.write(b"(")
                for x in chunk:
                    self.save(x)
                self.write(b"e")
            elif chunk:
                self.save(chunk[0])
                self.write(b"a")

    def _setitems(self, items):
        for k in range(0, max(len(items), 1), _BATCH):
            chunk = items[k:k + _BATCH]
            if len(chunk) > 1:
                self.write(b"(")
                for kk, v in chunk:
                    self.save(kk)
                    self.save(v)
                self.write(b"u")
            elif chunk:
                self.save(chunk[0][0])
                self.save(chunk[0][1])
                self.write(b"s")


def emit(tree) -> bytes:
    """The protocol-4 pickle opcode stream of a marker tree (the inverse of walk())."""
    return _Emitter().dump(tree)


# ---- Ray 1.0.1 checkpoint layout ---------------------------------------------------------
class _Np:
    """Marker builders for numpy data in the form numpy 1.x pickled it (module
    numpy.core.multiarray), sharing the global / dtype objects the way one pickler run does."""

    def __init__(self):
        self.scalar = Global("numpy.core.multiarray", "scalar")
        self.reconstruct = Global("numpy.core.multiarray", "_reconstruct")
        self.ndarray = Global("numpy", "ndarray")
        self.dtype_g = Global("numpy", "dtype")
        self.dtypes = {}
        self.b = b"b"

    def dtype(self, code):
        if code not in self.dtypes:
            # a fresh state tuple per dtype (one pickler run memoizes by identity)
            self.dtypes[code] = Call(self.dtype_g, (code, 0, 1), state=tuple([3, "<", None, None, None, -1, -1, 0]))
        return self.dtypes[code]

    def scalar_of(self, value, code):
        raw = np.asarray(value, dtype="<" + code).tobytes()
        return Call(self.scalar, (self.dtype(code), raw))

    def array_of(self, a, code):
        a = np.ascontiguousarray(np.asarray(a, dtype="<" + code))
        return Call(self.reconstruct, (self.ndarray, tuple([0]), self.b),
                    state=(1, tuple(int(s) for s in a.shape), self.dtype(code), False, a.tobytes()))


_LEARNER_KEYS = (("cur_kl_coeff", "f8"), ("cur_lr", "f8"), ("total_loss", "f4"), ("policy_loss", "f4"),
                 ("vf_loss", "f4"), ("vf_explained_var", "f4"), ("kl", "f4"), ("entropy", "f4"),
                 ("entropy_coeff", "f8"))


def _split_flat(flat, shapes):
    out, o = [], 0
    for _, sh in shapes:
        n = int(np.prod(sh))
        out.append(np.asarray(flat[o:o + n], np.float32).reshape(sh))
        o += n
    if o != len(flat):
        raise ValueError(f"flat vector holds {len(flat)} values, the layout {o}")
    return out


def ffn_shapes(d, n_out, hidden=64):
    """Keras variable order / shapes of the fcnet (models/fcnet_glorot_uniform_init.py:39-118)."""
    h = hidden
    return [("fc_1/kernel", (d, h)), ("fc_1/bias", (h,)), ("fc_value_1/kernel", (d, h)), ("fc_value_1/bias", (h,)),
            ("fc_2/kernel", (h, h)), ("fc_2/bias", (h,)), ("fc_value_2/kernel", (h, h)), ("fc_value_2/bias", (h,)),
            ("fc_out/kernel", (h, n_out)), ("fc_out/bias", (n_out,)), ("value_out/kernel", (h, 1)),
            ("value_out/bias", (1,))]


def gnn_shapes(n_out, hidden=64, feat=19, layer="mpnn"):
    """Variable order / shapes of the "gnn" model (models/shared_graphnet_glorot_uniform_init.py:
    32-33: actor GraphNet then critic GraphNet; models/graph_net.py:14-29 state_enc, MPNN
    msg_transform / node_update (models/gcn.py:46-47, no bias), linear_out).  No GNN checkpoint
    is published, so these names are not pinned by a reference file."""
    names = {"mpnn": ["mpnn/msg_transform", "mpnn/node_update"], "gcn": ["gcn/linear"],
             "mpnn2": ["mpnn2/msg_transform", "mpnn2/node_update"],
             "gat1": ["gat1/pre_att_linear", "gat1/att_linear"]}[layer]
    kshapes = {"mpnn": [(hidden, hidden)] * 2, "gcn": [(hidden, hidden)], "mpnn2": [(2 * hidden, hidden)] * 2,
               "gat1": [(hidden, hidden), (2 * hidden, 1)]}[layer]
    out = []
    for net, no in (("actor", n_out), ("critic", 1)):
        out += [(f"{net}/state_enc/kernel", (4, feat * hidden)), (f"{net}/state_enc/bias", (feat * hidden,))]
        out += [(f"{net}/{nm}/kernel", sh) for nm, sh in zip(names, kshapes)]
        out += [(f"{net}/linear_out/kernel", (hidden, no)), (f"{net}/linear_out/bias", (no,))]
    return out


def worker_tree(policies, shapes_of=None):
    """The rollout worker's state (RolloutWorker.save in Ray 1.0.1): {"filters": {pid:
    MeanStdFilter}, "state": {pid: OrderedDict{"<pid>/<var>": ndarray f4, ...,
    "_optimizer_variables": OrderedDict{"<pid>/beta1_power", "<pid>/beta2_power",
    "<pid>/<pid>/<var>/Adam", ".../Adam_1"}}}}.

    policies: {pid: {"weights", "adam_m", "adam_v" (flat, Keras order), "beta_powers" (b1, b2),
    "filter" (n, M, S) or None (then an empty RunningStat of width d is written), "filter_buffer"
    (n, M, S) or None, "shapes" [(name, shape)] in Keras order, optional "obs_dim" (filter
    width, default the first kernel's rows) and "filter_kind" ("MeanStdFilter" | "NoFilter")}}"""
    np_ = _Np()
    mod = "ray.rllib.utils.filter"
    msf, rsg = Global(mod, "MeanStdFilter"), Global(mod, "RunningStat")
    odict = Global("collections", "OrderedDict")
    filters, state, fshape = {}, {}, {}
    for pid, st in policies.items():
        shapes = st.get("shapes") or shapes_of(pid, st)
        d = int(st.get("obs_dim") or shapes[0][1][0])
        fshape.setdefault(d, tuple([d]))   # one observation-space shape object per width

        def rstat(f):
            n, M, S = f if f is not None else (0, np.zeros(d), np.zeros(d))
            return Call(rsg, (), newobj=True, state={"_n": int(n), "_M": np_.array_of(M, "f8"),
                                                     "_S": np_.array_of(S, "f8")})

        if st.get("filter_kind", "MeanStdFilter") == "NoFilter":   # observation_filter: NoFilter
            filters[pid] = Call(Global(mod, "NoFilter"), (), newobj=True)
            continue
        filters[pid] = Call(msf, (), newobj=True, state={
            "shape": fshape[d], "demean": True, "destd": True, "clip": None,
            "rs": rstat(st.get("filter")), "buffer": rstat(st.get("filter_buffer"))})
    for pid, st in policies.items():
        shapes = st.get("shapes") or shapes_of(pid, st)
        w = {}
        for (name, _), a in zip(shapes, _split_flat(st["weights"], shapes)):
            w[f"{pid}/{name}"] = np_.array_of(a, "f4")
        b1, b2 = st["beta_powers"]
        opt = {f"{pid}/beta1_power": np_.scalar_of(b1, "f4"), f"{pid}/beta2_power": np_.scalar_of(b2, "f4")}
        ms, vs = _split_flat(st["adam_m"], shapes), _split_flat(st["adam_v"], shapes)
        for (name, _), m, v in zip(shapes, ms, vs):
            opt[f"{pid}/{pid}/{name}/Adam"] = np_.array_of(m, "f4")
            opt[f"{pid}/{pid}/{name}/Adam_1"] = np_.array_of(v, "f4")
        w["_optimizer_variables"] = Call(odict, (), items=opt)
        state[pid] = Call(odict, (), items=w)   # TFPolicy.get_state: an OrderedDict
    return {"filters": filters, "state": state}


def checkpoint_tree(worker_bytes, learner, timesteps):
    """The outer dict of PPOTrainer.save (Ray 1.0.1 Trainer.__getstate__): the worker's pickle
    as bytes, then train_exec_impl {counters, info: {learner: {pid: stats}}, timers: None}."""
    np_ = _Np()
    ln = {}
    for pid, s in learner.items():
        # a statistic absent from the row (e.g. "kl" when no iteration has run on the saved
        # weights) is left out rather than written as 0.0, which a reader would take as a kl
        row = {k: np_.scalar_of(s[k], code) for k, code in _LEARNER_KEYS if k in s}
        row["model"] = {}
        ln[pid] = row
    return {"worker": worker_bytes,
            "train_exec_impl": {"counters": {"num_steps_sampled": int(timesteps), "num_steps_trained": int(timesteps)},
                                "info": {"learner": ln}, "timers": None}}


def metadata_tree(iteration, time_total, episodes_total, experiment_id, ray_version="1.0.1"):
    """checkpoint-<i>.tune_metadata (Tune Trainable.save), read by Trainable.restore."""
    return {"experiment_id": experiment_id, "iteration": int(iteration), "timesteps_total": None,
            "time_total": float(time_total), "episodes_total": int(episodes_total), "ray_version": ray_version,
            "saved_as_dict": False}


def write_checkpoint(checkpoint_dir, iteration, policies, learner, timesteps, time_total=0.0, episodes_total=0,
                     experiment_id=None, ray_version="1.0.1"):
    """Write <checkpoint_dir>/checkpoint_<i>/checkpoint-<i> (+ .tune_metadata, .is_checkpoint) in
    the layout PPOTrainer.restore of Ray 1.0.1 reads (evaluation/evaluate_trained_policies_pd.py:93-96).
    policies: see worker_tree; learner: {pid: {cur_kl_coeff, cur_lr, total_loss, policy_loss,
    vf_loss, vf_explained_var, kl, entropy, entropy_coeff}}.  Returns the checkpoint file path."""
    import os
    import uuid
    d = os.path.join(checkpoint_dir, f"checkpoint_{iteration}")
    os.makedirs(d, exist_ok=True)
    path = os.path.join(d, f"checkpoint-{iteration}")
    inner = emit(worker_tree(policies))
    with open(path, "wb") as f:
        f.write(emit(checkpoint_tree(inner, learner, timesteps)))
    with open(path + ".tune_metadata", "wb") as f:
        f.write(emit(metadata_tree(iteration, time_total, episodes_total, experiment_id or uuid.uuid4().hex,
                                   ray_version)))
    open(os.path.join(d, ".is_checkpoint"), "wb").close()
    return path


def published_policies(ck):
    """{pid: worker_tree input} of a read checkpoint (weights, Adam, beta powers, both filter
    stats, Keras shapes), so that a published file can be written back."""
    out = {}
    worker = ck["worker"]
    for pid in policy_ids(ck):
        s = policy_state(ck, pid)
        f = worker["filters"][pid]["state"]
        buf = f["buffer"]["state"]
        out[pid] = {"weights": s["weights"], "adam_m": s["adam_m"], "adam_v": s["adam_v"],
                    "beta_powers": tuple(np.float32(opt) for opt in s["beta_powers"]),
                    "filter": s["filter"], "filter_buffer": (buf["_n"], buf["_M"], buf["_S"]),
                    "shapes": [(k, tuple(sh)) for k, sh in s["shapes"]]}
    return out
