"""ctypes binding of libddrl_hip.so (include/ddrl_hip.h).

The HIP library is the only compute path: if it is missing or fails to load, every entry
point raises.  There is no CPU fallback.  Device buffers are passed as raw pointers (for
example torch tensors' data_ptr()); torch is plumbing for memory and streams only.
"""
from __future__ import annotations

import ctypes as C
import os
import re

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libddrl_hip.so")
HEADER = os.path.join(os.path.dirname(HERE), "include", "ddrl_hip.h")

MAX_P, MAX_AG, MAX_OBS = 4, 4, 48
MODEL_FFN, MODEL_GNN = 0, 1
REWARD_PER_LEG, REWARD_GLOBAL, REWARD_NORM = 0, 1, 2
VF_CLIP_RAY10, VF_CLIP_SQUARED = 0, 1
# message-passing layer of the "gnn" model (models/graph_net.py:20 selects one of models/gcn.py's)
GNN_LAYERS = {"mpnn": 0, "gcn": 1, "mpnn2": 2, "gat1": 3}

i32, f32 = C.c_int32, C.c_float


class DdrlCfg(C.Structure):
    _fields_ = [
        ("n_envs", i32), ("frag_len", i32), ("obs_full_dim", i32), ("n_agents", i32),
        ("n_policies", i32), ("model_kind", i32), ("act_dim", i32),
        ("agent_policy", i32 * MAX_AG), ("obs_dim", i32 * MAX_P),
        ("obs_index", (i32 * MAX_OBS) * MAX_AG), ("act_index", (i32 * 8) * MAX_AG),
        ("n_contact", i32 * MAX_AG), ("contact_index", (i32 * 14) * MAX_AG),
        ("contact_weight", (f32 * 14) * MAX_AG), ("leg_angle_deg", f32 * MAX_AG),
        ("filter_enabled", i32), ("filter_update", i32), ("filter_clip", f32),
        ("reward_mode", i32), ("ctrl_cost_weight", f32), ("contact_cost_weight", f32),
        ("gamma", f32), ("lambda_", f32), ("clip_param", f32), ("vf_clip_param", f32),
        ("vf_loss_coeff", f32), ("entropy_coeff", f32), ("lr", f32), ("grad_clip", f32),
        ("adam_beta1", f32), ("adam_beta2", f32), ("adam_eps", f32),
        ("vf_clip_mode", i32), ("sgd_minibatch_size", i32), ("num_sgd_iter", i32),
        ("act_negate", (i32 * 8) * MAX_AG), ("policy_filter", i32),
        ("leg_coupling", i32), ("gnn_layer", i32),
    ]


VP = C.c_void_p
_SIGS = {
    "ddrl_abi_version": ([], C.c_int),
    "ddrl_last_error": ([], C.c_char_p),
    "ddrl_ctx_create": ([C.POINTER(DdrlCfg), C.c_int, C.POINTER(VP)], C.c_int),
    "ddrl_ctx_destroy": ([VP], C.c_int),
    "ddrl_set_stream": ([VP, VP], C.c_int),
    "ddrl_synchronize": ([VP], C.c_int),
    "ddrl_param_count": ([VP, C.c_int, C.POINTER(C.c_int64)], C.c_int),
    "ddrl_record_layout": ([VP, C.c_int, C.POINTER(i32)], C.c_int),
    "ddrl_params_set": ([VP, C.c_int, VP, C.c_size_t], C.c_int),
    "ddrl_params_get": ([VP, C.c_int, VP, C.c_size_t], C.c_int),
    "ddrl_adam_set": ([VP, C.c_int, VP, VP, C.c_size_t, f32, f32], C.c_int),
    "ddrl_adam_get": ([VP, C.c_int, VP, VP, C.c_size_t, C.POINTER(f32), C.POINTER(f32)], C.c_int),
    "ddrl_filter_set": ([VP, C.c_double, VP, VP], C.c_int),
    "ddrl_filter_get": ([VP, C.POINTER(C.c_double), VP, VP], C.c_int),
    "ddrl_filter_delta_get": ([VP, C.POINTER(C.c_double), VP, VP], C.c_int),
    "ddrl_filter_delta_reset": ([VP], C.c_int),
    "ddrl_adv_sums_get": ([VP, C.c_int, VP], C.c_int),
    "ddrl_policy_filter_set": ([VP, C.c_int, C.c_double, VP, VP], C.c_int),
    "ddrl_policy_filter_get": ([VP, C.c_int, C.POINTER(C.c_double), VP, VP], C.c_int),
    "ddrl_policy_filter_delta_get": ([VP, C.c_int, C.POINTER(C.c_double), VP, VP], C.c_int),
    "ddrl_policy_filter_delta_reset": ([VP], C.c_int),
    "ddrl_observe": ([VP, VP], C.c_int),
    "ddrl_act": ([VP, C.c_int, VP, VP], C.c_int),
    "ddrl_reward": ([VP, C.c_int, VP, VP, VP, VP], C.c_int),
    "ddrl_bootstrap": ([VP], C.c_int),
    "ddrl_step_host": ([VP, C.c_int, VP, VP, VP], C.c_int),
    "ddrl_act_host": ([VP, C.c_int, VP, VP], C.c_int),
    "ddrl_rollout_fragment": ([VP, VP, VP, VP, VP, VP, VP], C.c_int),
    "ddrl_env_step_host": ([VP, C.c_int, VP, VP, VP, VP], C.c_int),
    "ddrl_gae": ([VP], C.c_int),
    "ddrl_ppo_update": ([VP, C.c_int, C.POINTER(VP), C.POINTER(VP), C.POINTER(f32), C.c_int], C.c_int),
    "ddrl_ppo_update_from": ([VP, C.c_int, C.POINTER(VP), C.POINTER(VP), C.POINTER(f32), C.c_int, C.c_int], C.c_int),
    "ddrl_ppo_stats": ([VP, C.c_int, VP, C.c_size_t], C.c_int),
    "ddrl_ppo_stats_range": ([VP, C.c_int, C.c_size_t, C.c_size_t, VP], C.c_int),
    "ddrl_ppo_grad": ([VP, C.c_int, VP, C.c_int, f32, VP, C.c_int], C.c_int),
    "ddrl_ppo_apply": ([VP, C.c_int, VP], C.c_int),
    "ddrl_comm_unique_id": ([VP, C.c_size_t], C.c_int),
    "ddrl_comm_init": ([VP, VP, C.c_int, C.c_int], C.c_int),
    "ddrl_comm_allreduce": ([VP, VP, C.c_size_t], C.c_int),
    "ddrl_ppo_update_ddp": ([VP, C.c_int, VP, VP, C.c_int, C.c_int, C.c_int, f32, f32], C.c_int),
    "ddrl_peer_alloc": ([VP, C.POINTER(VP), VP], C.c_int),
    "ddrl_peer_open": ([VP, VP, C.POINTER(VP)], C.c_int),
    "ddrl_peer_attach": ([VP, VP, C.c_int, C.c_int], C.c_int),
    "ddrl_ppo_update_peer": ([VP, C.c_int, VP, VP, C.c_int, C.c_int, f32, C.c_int], C.c_int),
    "ddrl_policy_forward": ([VP, C.c_int, VP, VP, C.c_int, VP, VP], C.c_int),
    "ddrl_gnn_one_launch": ([VP, C.POINTER(C.c_int)], C.c_int),
    "ddrl_device_buffers": ([VP, C.c_int, C.POINTER(VP), C.POINTER(VP), C.POINTER(VP), C.POINTER(VP)], C.c_int),
    "ddrl_records_get": ([VP, C.c_int, VP, C.c_size_t], C.c_int),
    "ddrl_records_set": ([VP, C.c_int, VP, C.c_size_t], C.c_int),
    "ddrl_adv_norm_get": ([VP, C.c_int, VP], C.c_int),
    "ddrl_adv_norm_set": ([VP, C.c_int, f32, f32], C.c_int),
    "ddrl_last_values_get": ([VP, C.c_int, VP, C.c_size_t], C.c_int),
    "ddrl_last_values_set": ([VP, C.c_int, VP, C.c_size_t], C.c_int),
    "ddrl_done_set": ([VP, VP, C.c_size_t], C.c_int),
    "ddrl_observe_range": ([VP, VP, C.c_int, C.c_int], C.c_int),
    "ddrl_act_range": ([VP, C.c_int, C.c_int, C.c_int, VP, VP], C.c_int),
    "ddrl_reward_range": ([VP, C.c_int, C.c_int, C.c_int, VP, VP, VP, VP], C.c_int),
    "ddrl_hostenv_last_error": ([], C.c_char_p),
    "ddrl_hostenv_create": ([C.c_int, C.c_int, C.c_int, C.c_uint64, f32, C.POINTER(VP)], C.c_int),
    "ddrl_hostenv_destroy": ([VP], C.c_int),
    "ddrl_hostenv_buffers": ([VP, C.POINTER(VP), C.POINTER(VP), C.POINTER(VP), C.POINTER(VP), C.POINTER(VP)],
                             C.c_int),
    "ddrl_hostenv_reset": ([VP], C.c_int),
    "ddrl_hostenv_step": ([VP, C.c_int, C.c_int], C.c_int),
    "ddrl_hostenv_threads": ([VP], C.c_int),
    "ddrl_hostenv_set_target_velocities": ([VP, C.POINTER(C.c_float), C.c_int], C.c_int),
    "ddrl_hostenv_target_velocities": ([VP, C.POINTER(C.c_float), C.c_int], C.c_int),
    "ddrl_hostenv_reset_state": ([VP], C.c_int),
    "ddrl_rollout_hostenv": ([VP, VP, C.c_int, VP, C.c_int], C.c_int),
}

_lib = None


class DdrlError(RuntimeError):
    pass


def header_symbols(path=HEADER):
    """Function names declared in include/ddrl_hip.h."""
    txt = open(path).read()
    return sorted(set(re.findall(r"^\s*(?:int|const char\*)\s+(ddrl_\w+)\s*\(", txt, re.M)))


ABI_VERSION = 4   # DDRL_ABI_VERSION of include/ddrl_hip.h (ddrl_cfg layout, record layout)
COMM_ID_BYTES = 128   # DDRL_COMM_ID_BYTES (sizeof ncclUniqueId)
PEER_HANDLE_BYTES = 64   # DDRL_PEER_HANDLE_BYTES (sizeof hipIpcMemHandle_t)


def comm_unique_id():
    """A fresh RCCL unique id (rank 0 makes it, the caller hands it to the other ranks)."""
    buf = (C.c_uint8 * COMM_ID_BYTES)()
    _ck(load().ddrl_comm_unique_id(buf, COMM_ID_BYTES))
    return bytes(buf)


def load(path: str = LIB_PATH):
    """The HIP library.  DDRL_LIB names an alternative in-tree build of the same ABI (the
    diagnostic variants of ddrl_amd/build.py, e.g. libddrl_hip_atomic.so) for A/B timing."""
    global _lib
    if _lib is not None:
        return _lib
    if path == LIB_PATH and os.environ.get("DDRL_LIB"):
        path = os.path.join(HERE, os.path.basename(os.environ["DDRL_LIB"]))
    if not os.path.exists(path):
        raise DdrlError(f"{path} is missing: build it with `python -m ddrl_amd.build` "
                        "(the HIP library is the only compute path; there is no fallback)")
    # torch ships its own libamdhip64.so.7 (same soname as /opt/rocm's): import it first so
    # this library binds to the process's single HIP runtime instead of starting a second one
    import torch  # noqa: F401
    lib = C.CDLL(path)
    for name, (args, res) in _SIGS.items():
        fn = getattr(lib, name)
        fn.argtypes = args
        fn.restype = res
    if lib.ddrl_abi_version() != ABI_VERSION:
        raise DdrlError(f"{path} has ABI {lib.ddrl_abi_version()}, this binding expects {ABI_VERSION}: "
                        "rebuild with `python -m ddrl_amd.build`")
    _lib = lib
    return lib


def _ck(rc):
    if rc != 0:
        raise DdrlError(load().ddrl_last_error().decode())


def _ptr(x):
    """Device/host pointer of a torch tensor, numpy array, int or None."""
    if x is None:
        return None
    if isinstance(x, int):
        return x
    if isinstance(x, np.ndarray):
        assert x.flags["C_CONTIGUOUS"]
        return x.ctypes.data
    if hasattr(x, "data_ptr"):
        assert x.is_contiguous()
        return x.data_ptr()
    raise TypeError(type(x))


class Context:
    """One device + stream + rollout shard (a ddrl_ctx)."""

    def __init__(self, cfg: DdrlCfg, device: int = 0, stream: int | None = None):
        self.lib = load()
        self.cfg = cfg
        h = VP()
        _ck(self.lib.ddrl_ctx_create(C.byref(cfg), device, C.byref(h)))
        self.h = h
        self.device = device
        if stream is not None:
            self.set_stream(stream)
        self.n_params = []
        self.layout = []
        for p in range(cfg.n_policies):
            n = C.c_int64()
            _ck(self.lib.ddrl_param_count(h, p, C.byref(n)))
            self.n_params.append(int(n.value))
            lay = (i32 * 11)()
            _ck(self.lib.ddrl_record_layout(h, p, lay))
            self.layout.append(dict(zip(
                ["stride", "obs", "act", "logit", "logp", "vf", "adv", "vt", "rew", "C", "leg"], list(lay))))

    def close(self):
        if getattr(self, "h", None):
            self.lib.ddrl_ctx_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_stream(self, stream: int):
        _ck(self.lib.ddrl_set_stream(self.h, stream))

    def synchronize(self):
        _ck(self.lib.ddrl_synchronize(self.h))

    # ---- state ----
    def params_set(self, pid, flat):
        a = np.ascontiguousarray(flat, np.float32)
        _ck(self.lib.ddrl_params_set(self.h, pid, a.ctypes.data, a.size))

    def params_get(self, pid):
        a = np.empty(self.n_params[pid], np.float32)
        _ck(self.lib.ddrl_params_get(self.h, pid, a.ctypes.data, a.size))
        return a

    def adam_set(self, pid, m, v, b1p, b2p):
        m = np.ascontiguousarray(m, np.float32)
        v = np.ascontiguousarray(v, np.float32)
        _ck(self.lib.ddrl_adam_set(self.h, pid, m.ctypes.data, v.ctypes.data, m.size, b1p, b2p))

    def adam_get(self, pid):
        n = self.n_params[pid]
        m, v = np.empty(n, np.float32), np.empty(n, np.float32)
        b1, b2 = f32(), f32()
        _ck(self.lib.ddrl_adam_get(self.h, pid, m.ctypes.data, v.ctypes.data, n, C.byref(b1), C.byref(b2)))
        return m, v, b1.value, b2.value

    def filter_set(self, n, M, S):
        M = np.ascontiguousarray(M, np.float64)
        S = np.ascontiguousarray(S, np.float64)
        _ck(self.lib.ddrl_filter_set(self.h, float(n), M.ctypes.data, S.ctypes.data))

    def filter_get(self):
        D = self.cfg.obs_full_dim
        n = C.c_double()
        M, S = np.empty(D), np.empty(D)
        _ck(self.lib.ddrl_filter_get(self.h, C.byref(n), M.ctypes.data, S.ctypes.data))
        return n.value, M, S

    def filter_delta_get(self):
        """Pushes since the last filter_delta_reset as (n, M, S)."""
        D = self.cfg.obs_full_dim
        n = C.c_double()
        M, S = np.empty(D), np.empty(D)
        _ck(self.lib.ddrl_filter_delta_get(self.h, C.byref(n), M.ctypes.data, S.ctypes.data))
        return n.value, M, S

    def filter_delta_reset(self):
        _ck(self.lib.ddrl_filter_delta_reset(self.h))

    def policy_filter_set(self, pid, n, M, S):
        M = np.ascontiguousarray(M, np.float64)
        S = np.ascontiguousarray(S, np.float64)
        _ck(self.lib.ddrl_policy_filter_set(self.h, pid, float(n), M.ctypes.data, S.ctypes.data))

    def policy_filter_get(self, pid, delta=False):
        d = self.cfg.obs_dim[pid]
        n = C.c_double()
        M, S = np.empty(d), np.empty(d)
        fn = self.lib.ddrl_policy_filter_delta_get if delta else self.lib.ddrl_policy_filter_get
        _ck(fn(self.h, pid, C.byref(n), M.ctypes.data, S.ctypes.data))
        return n.value, M, S

    def policy_filter_delta_reset(self):
        _ck(self.lib.ddrl_policy_filter_delta_reset(self.h))

    def adv_sums_get(self, pid):
        """fp64 (sum adv, sum adv^2, count) of the last gae() for policy pid."""
        a = np.empty(3, np.float64)
        _ck(self.lib.ddrl_adv_sums_get(self.h, pid, a.ctypes.data))
        return a

    def records_get(self, pid):
        lay = self.layout[pid]
        a = np.empty((self.cfg.frag_len * lay["C"], lay["stride"]), np.float32)
        _ck(self.lib.ddrl_records_get(self.h, pid, a.ctypes.data, a.size))
        return a

    def records_tensor(self, pid):
        """The policy's device record buffer [T * C][stride] as a torch tensor (no copy: a
        view over ddrl_device_buffers' pointer through __cuda_array_interface__)."""
        import torch
        rec, lv, par, an = VP(), VP(), VP(), VP()
        _ck(self.lib.ddrl_device_buffers(self.h, pid, C.byref(rec), C.byref(lv), C.byref(par), C.byref(an)))
        lay = self.layout[pid]
        shape = (self.cfg.frag_len * lay["C"], lay["stride"])

        class _View:
            __cuda_array_interface__ = {"shape": shape, "typestr": "<f4", "data": (rec.value, False),
                                        "version": 3, "strides": None}
        return torch.as_tensor(_View(), device=torch.device("cuda", self.device))

    def records_set(self, pid, rec):
        a = np.ascontiguousarray(rec, np.float32)
        _ck(self.lib.ddrl_records_set(self.h, pid, a.ctypes.data, a.size))

    def adv_norm_get(self, pid):
        a = np.empty(2, np.float32)
        _ck(self.lib.ddrl_adv_norm_get(self.h, pid, a.ctypes.data))
        return a

    def adv_norm_set(self, pid, mean, den):
        _ck(self.lib.ddrl_adv_norm_set(self.h, pid, mean, den))

    def last_values_get(self, pid):
        a = np.empty(self.layout[pid]["C"], np.float32)
        _ck(self.lib.ddrl_last_values_get(self.h, pid, a.ctypes.data, a.size))
        return a

    def last_values_set(self, pid, values):
        a = np.ascontiguousarray(values, np.float32)
        _ck(self.lib.ddrl_last_values_set(self.h, pid, a.ctypes.data, a.size))

    def done_set(self, done_tn):
        a = np.ascontiguousarray(done_tn, np.uint8)
        _ck(self.lib.ddrl_done_set(self.h, a.ctypes.data, a.size))

    # ---- rollout ----
    def observe(self, obs_dev):
        _ck(self.lib.ddrl_observe(self.h, _ptr(obs_dev)))

    def act(self, t, eps_dev, actions_dev):
        _ck(self.lib.ddrl_act(self.h, t, _ptr(eps_dev), _ptr(actions_dev)))

    def reward(self, t, fw_dev, cfrc_dev, actions_dev, done_dev=None):
        _ck(self.lib.ddrl_reward(self.h, t, _ptr(fw_dev), _ptr(cfrc_dev), _ptr(actions_dev), _ptr(done_dev)))

    def bootstrap(self):
        _ck(self.lib.ddrl_bootstrap(self.h))

    def step_host(self, t, obs_host, eps_host, actions_host):
        _ck(self.lib.ddrl_step_host(self.h, t, _ptr(obs_host), _ptr(eps_host), _ptr(actions_host)))

    def rollout_fragment(self, obs_dev, eps_dev, fw_dev, cfrc_dev, done_dev, actions_dev):
        _ck(self.lib.ddrl_rollout_fragment(self.h, _ptr(obs_dev), _ptr(eps_dev), _ptr(fw_dev), _ptr(cfrc_dev),
                                           _ptr(done_dev), _ptr(actions_dev)))

    def act_host(self, t, eps_host, actions_host):
        _ck(self.lib.ddrl_act_host(self.h, t, _ptr(eps_host), _ptr(actions_host)))

    def env_step_host(self, t, fw_host, cfrc_host, done_host, obs_next_host):
        _ck(self.lib.ddrl_env_step_host(self.h, t, _ptr(fw_host), _ptr(cfrc_host), _ptr(done_host),
                                        _ptr(obs_next_host)))

    def gae(self):
        _ck(self.lib.ddrl_gae(self.h))

    # ---- learner ----
    def ppo_update(self, mask, shuffles, perms, kl_coeffs, max_steps=-1, step0=0):
        """The fused minibatch SGD (ddrl_ppo_update); step0 > 0 resumes the schedule at that step
        (ddrl_ppo_update_from), bit-identical to the same steps of one uninterrupted launch."""
        P = self.cfg.n_policies
        sh = (VP * MAX_P)(*[_ptr(shuffles[p]) if shuffles[p] is not None else None for p in range(P)])
        pe = (VP * MAX_P)(*[_ptr(perms[p]) if perms[p] is not None else None for p in range(P)])
        kl = (f32 * MAX_P)(*[float(k) for k in kl_coeffs])
        if step0:
            _ck(self.lib.ddrl_ppo_update_from(self.h, mask, sh, pe, kl, step0, max_steps))
        else:
            _ck(self.lib.ddrl_ppo_update(self.h, mask, sh, pe, kl, max_steps))

    def ppo_stats(self, pid, n_steps, first=0):
        """Learner statistics rows [first, first + n_steps) of the last update (8 floats each)."""
        a = np.empty((n_steps, 8), np.float32)
        _ck(self.lib.ddrl_ppo_stats_range(self.h, pid, first, n_steps, a.ctypes.data))
        return a

    def ppo_grad(self, pid, rows_dev, n_rows, kl_coeff, grad_dev, stats_step=-1):
        _ck(self.lib.ddrl_ppo_grad(self.h, pid, _ptr(rows_dev), n_rows, kl_coeff, _ptr(grad_dev),
                                   stats_step))

    def ppo_apply(self, pid, grad_dev):
        _ck(self.lib.ddrl_ppo_apply(self.h, pid, _ptr(grad_dev)))

    def comm_init(self, unique_id, rank, nranks):
        """Join the RCCL communicator named by `unique_id` (bytes from comm_unique_id())."""
        buf = (C.c_uint8 * COMM_ID_BYTES).from_buffer_copy(bytes(unique_id))
        _ck(self.lib.ddrl_comm_init(self.h, buf, rank, nranks))

    def comm_allreduce(self, buf_dev):
        _ck(self.lib.ddrl_comm_allreduce(self.h, _ptr(buf_dev), buf_dev.numel()))

    def peer_alloc(self, export=False):
        """Rank 0: the shared outboxes of peer mode; (device pointer, IPC handle bytes or None)."""
        p = VP()
        h = (C.c_uint8 * PEER_HANDLE_BYTES)() if export else None
        _ck(self.lib.ddrl_peer_alloc(self.h, C.byref(p), h))
        return p.value, (bytes(h) if export else None)

    def peer_open(self, handle):
        """Rank 1 in another process: map rank 0's outboxes from its IPC handle."""
        buf = (C.c_uint8 * PEER_HANDLE_BYTES).from_buffer_copy(bytes(handle))
        p = VP()
        _ck(self.lib.ddrl_peer_open(self.h, buf, C.byref(p)))
        return p.value

    def peer_attach(self, gx_ptr, rank, nranks=2):
        _ck(self.lib.ddrl_peer_attach(self.h, VP(gx_ptr), rank, nranks))

    def ppo_update_peer(self, pid, shuffle_dev, perm_dev, kl_coeff, max_steps=-1):
        """One fused update with this rank's 64 rows of every minibatch (ddrl_ppo_update_peer);
        perm_dev: [n_epochs][nb] device int32, shuffle_dev: this rank's nb * 64 row indices."""
        E, nb = int(perm_dev.shape[0]), int(perm_dev.shape[1])
        _ck(self.lib.ddrl_ppo_update_peer(self.h, pid, _ptr(shuffle_dev), _ptr(perm_dev), E, nb, float(kl_coeff),
                                          max_steps))

    def gnn_one_launch(self):
        """True when the GraphNet minibatch step runs as one launch (reduction + clip + Adam in
        the gradient launch's tail), False for the three-launch step or an fcnet context."""
        on = C.c_int()
        _ck(self.lib.ddrl_gnn_one_launch(self.h, C.byref(on)))
        return bool(on.value)

    def ppo_update_ddp(self, pid, shuffle_dev, perms, rows_per_rank, kl_coeff, grad_scale):
        """The data-parallel minibatch loop in C++ (gradient -> RCCL all-reduce -> Adam per step)."""
        perms = np.ascontiguousarray(perms, np.int32)
        E, nb = perms.shape
        _ck(self.lib.ddrl_ppo_update_ddp(self.h, pid, _ptr(shuffle_dev), perms.ctypes.data, E, nb,
                                         rows_per_rank, kl_coeff, grad_scale))

    # ---- ranged rollout calls (env groups of a pipelined host env plane) ----
    def observe_range(self, obs_dev, e0, e1):
        _ck(self.lib.ddrl_observe_range(self.h, _ptr(obs_dev), e0, e1))

    def act_range(self, t, e0, e1, eps_dev, actions_dev):
        _ck(self.lib.ddrl_act_range(self.h, t, e0, e1, _ptr(eps_dev), _ptr(actions_dev)))

    def reward_range(self, t, e0, e1, fw_dev, cfrc_dev, actions_dev, done_dev=None):
        _ck(self.lib.ddrl_reward_range(self.h, t, e0, e1, _ptr(fw_dev), _ptr(cfrc_dev), _ptr(actions_dev),
                                       _ptr(done_dev)))

    def rollout_hostenv(self, env, eps_dev, groups=2, reset=False):
        """A fragment with the envs stepped on the host (HostEnv), pipelined over env groups."""
        _ck(self.lib.ddrl_rollout_hostenv(self.h, env.h, groups, _ptr(eps_dev), 1 if reset else 0))

    def policy_forward(self, pid, obs_dev, n, logits_dev, values_dev, node_dev=None):
        _ck(self.lib.ddrl_policy_forward(self.h, pid, _ptr(obs_dev), _ptr(node_dev), n,
                                         _ptr(logits_dev), _ptr(values_dev)))


class HostEnv:
    """The host env plane (hostenv.cpp): N QuAntruped stand-in envs stepped by a pool of host
    threads into pinned buffers, exposed here as numpy views (obs [N][D], act [N][8], fw [N],
    cfrc [N][14][6], done [N])."""

    def __init__(self, n_envs, obs_dim=43, n_threads=1, seed=0, target_velocity=0.0):
        """target_velocity: one value, or a list every env draws its episode's velocity from on
        each reset (the adaptor's random.choice, quantruped_adaptor_multi_environment.py:50, 216)."""
        self.lib = load()
        h = VP()
        tvs = [float(v) for v in (target_velocity if np.ndim(target_velocity) else [target_velocity])]
        if self.lib.ddrl_hostenv_create(n_envs, obs_dim, n_threads, seed, tvs[0], C.byref(h)) != 0:
            raise DdrlError(self.lib.ddrl_hostenv_last_error().decode())
        if len(tvs) > 1:
            arr = (C.c_float * len(tvs))(*tvs)
            if self.lib.ddrl_hostenv_set_target_velocities(h, arr, len(tvs)) != 0:
                err = self.lib.ddrl_hostenv_last_error().decode()
                self.lib.ddrl_hostenv_destroy(h)
                raise DdrlError(err)
        self.h, self.n, self.obs_dim = h, n_envs, obs_dim
        ptrs = [VP() for _ in range(5)]
        self._ck(self.lib.ddrl_hostenv_buffers(h, *[C.byref(p) for p in ptrs]))
        view = lambda p, ct, shape: np.ctypeslib.as_array(C.cast(p, C.POINTER(ct)), shape=shape)
        self.obs = view(ptrs[0], C.c_float, (n_envs, obs_dim))
        self.act = view(ptrs[1], C.c_float, (n_envs, 8))
        self.fw = view(ptrs[2], C.c_float, (n_envs,))
        self.cfrc = view(ptrs[3], C.c_float, (n_envs, 14, 6))
        self.done = view(ptrs[4], C.c_uint8, (n_envs,))
        self.threads = self.lib.ddrl_hostenv_threads(h)

    def _ck(self, rc):
        if rc != 0:
            raise DdrlError(self.lib.ddrl_hostenv_last_error().decode())

    def _live(self):
        if not getattr(self, "h", None):
            raise DdrlError("host env plane is closed")

    def reset(self):
        """Reset every env; returns a COPY of the observations (self.obs is the live pinned
        buffer that the next step() overwrites in place)."""
        self._live()
        self._ck(self.lib.ddrl_hostenv_reset(self.h))
        return self.obs.copy()

    def step(self, e0=0, e1=None):
        """Step the envs [e0, e1) with the actions in self.act (written by the caller)."""
        self._live()
        self._ck(self.lib.ddrl_hostenv_step(self.h, e0, self.n if e1 is None else e1))

    def reset_state(self):
        """update_environment_after_epoch's env.reset(): every env's state and TimeLimit count
        restart; target velocities, done flags and self.obs are left as they are."""
        self._live()
        self._ck(self.lib.ddrl_hostenv_reset_state(self.h))

    @property
    def target_velocities(self):
        """Each env's current target velocity (the draw of its current episode)."""
        self._live()
        out = np.zeros(self.n, np.float32)
        self._ck(self.lib.ddrl_hostenv_target_velocities(self.h, out.ctypes.data_as(C.POINTER(C.c_float)), self.n))
        return out

    def close(self):
        """Free the pinned buffers.  The numpy views over them are dropped first (set to None),
        so no attribute of this object can read freed memory afterwards; copies made by the
        caller stay valid."""
        if getattr(self, "h", None):
            self.obs = self.act = self.fw = self.cfrc = self.done = None
            self.lib.ddrl_hostenv_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
