"""Mirror of the reference's model registry (models/__init__.py:7-13) over the HIP path.

ModelCatalog names: "ffn" and "fc_glorot_uniform_init" -> fcnet with Glorot-uniform init
(models/fcnet_glorot_uniform_init.py:10-125); "cup" -> fcnet + trainable leg coupling
(models/coupling_net_glorot_uniform_init.py:11-137); "gnn" -> GraphNet actor/critic
(models/shared_graphnet_glorot_uniform_init.py:14-58).  A model instance exposes the
ModelV2 surface the reference's plugins implement: forward(input_dict, state, seq_lens)
-> (logits, state) and value_function() -> [B]; the arithmetic runs in libddrl_hip.so.
"""
from __future__ import annotations

import math

import numpy as np

from . import native as N

_CATALOG = {}


class ModelCatalog:
    @staticmethod
    def register_custom_model(name, cls):
        _CATALOG[name] = cls

    @staticmethod
    def get(name):
        try:
            return _CATALOG[name]
        except KeyError:
            raise KeyError(f"unknown custom_model {name!r}; registered: {sorted(_CATALOG)}") from None


def gnn_layer_kernel_shapes(layer, hidden=64):
    """Kernels of the message-passing layer in Keras creation order (models/gcn.py: MPNN
    msg_transform + node_update :46-47, GCN linear :19, MPNN2 msg_transform + node_update on
    concatenations :102-103, GAT1 pre_att_linear + att_linear :159-160)."""
    return {"mpnn": [(hidden, hidden), (hidden, hidden)], "gcn": [(hidden, hidden)],
            "mpnn2": [(2 * hidden, hidden), (2 * hidden, hidden)],
            "gat1": [(hidden, hidden), (2 * hidden, 1)]}[layer]


def glorot_gnn_flat(rng, A, hidden=64, feat=19, layer="mpnn"):
    """GraphNet init: state_enc / layer kernels Glorot(1.0) (GAT1's Keras default
    glorot_uniform is the same law), linear_out Glorot(0.01), biases 0; actor then critic."""
    def g(fi, fo, s):
        lim = math.sqrt(6.0 * s / (fi + fo))
        return rng.uniform(-lim, lim, size=(fi, fo)).astype(np.float32)
    out = []
    for n_out in (2 * A, 1):
        out += [g(4, feat * hidden, 1.0), np.zeros(feat * hidden, np.float32)]
        out += [g(fi, fo, 1.0) for fi, fo in gnn_layer_kernel_shapes(layer, hidden)]
        out += [g(hidden, n_out, 0.01), np.zeros(n_out, np.float32)]
    return np.concatenate([o.reshape(-1) for o in out])


class _HipModel:
    kind = N.MODEL_FFN

    def __init__(self, obs_space, action_space, num_outputs, model_config, name, ctx=None, pid=0):
        hid = model_config.get("fcnet_hiddens", [64, 64])
        if list(hid) != [64, 64]:
            raise ValueError("the HIP kernels implement fcnet_hiddens = [64, 64] (the reference's setting)")
        if model_config.get("fcnet_activation", "tanh") != "tanh":
            raise ValueError("the HIP kernels implement fcnet_activation = tanh")
        if model_config.get("free_log_std"):
            raise ValueError("free_log_std is not used by the reference's configs")
        self.obs_space, self.action_space = obs_space, action_space
        self.num_outputs, self.name = num_outputs, name
        self.ctx, self.pid = ctx, pid
        self._value_out = None

    def _need_ctx(self):
        if self.ctx is None:
            raise RuntimeError("model is not bound to a ddrl context (PPOTrainer binds it)")

    def value_function(self):
        return self._value_out


class FullyConnectedNetwork_GlorotUniformInitializer(_HipModel):
    def forward(self, input_dict, state, seq_lens):
        import torch
        self._need_ctx()
        x = input_dict["obs_flat"] if "obs_flat" in input_dict else input_dict["obs"]
        x = torch.as_tensor(x, dtype=torch.float32, device="cuda").contiguous()
        n = x.shape[0]
        logits = torch.empty((n, self.num_outputs), dtype=torch.float32, device="cuda")
        values = torch.empty((n,), dtype=torch.float32, device="cuda")
        self.ctx.policy_forward(self.pid, x, n, logits, values)
        self._value_out = values
        return logits, state


class FullyConnectedNetwork_GNN_GlorotUniformInitializer(_HipModel):
    kind = N.MODEL_GNN

    def forward(self, input_dict, state, seq_lens):
        import torch
        self._need_ctx()
        node, X, _adj = input_dict["obs"]
        X = torch.as_tensor(X, dtype=torch.float32, device="cuda").contiguous()
        node = torch.as_tensor(node, device="cuda").reshape(-1).to(torch.int32).contiguous()
        n = X.shape[0]
        logits = torch.empty((n, self.num_outputs), dtype=torch.float32, device="cuda")
        values = torch.empty((n,), dtype=torch.float32, device="cuda")
        self.ctx.policy_forward(self.pid, X, n, logits, values, node_dev=node)
        self._value_out = values
        return logits, state


class FullyConnectedNetwork_Coupling_GlorotUniformInitializer(_HipModel):
    """"cup" (models/coupling_net_glorot_uniform_init.py:32-137): the fcnet on the features
    of the (leg index, features) observation, whose action means are scaled by the trainable
    leg_coupling row of the leg index (LegCoupling, :11-30)."""

    def forward(self, input_dict, state, seq_lens):
        import torch
        self._need_ctx()
        leg, x = input_dict["obs"]
        x = torch.as_tensor(x, dtype=torch.float32, device="cuda").contiguous()
        leg = torch.as_tensor(leg, device="cuda").reshape(-1).to(torch.int32).contiguous()
        if leg.numel() and (int(leg.min()) < 0 or int(leg.max()) > 3):
            raise ValueError("leg index out of range [0, 3]")
        n = x.shape[0]
        logits = torch.empty((n, self.num_outputs), dtype=torch.float32, device="cuda")
        values = torch.empty((n,), dtype=torch.float32, device="cuda")
        self.ctx.policy_forward(self.pid, x, n, logits, values, node_dev=leg)
        self._value_out = values
        return logits, state


ModelCatalog.register_custom_model("ffn", FullyConnectedNetwork_GlorotUniformInitializer)
ModelCatalog.register_custom_model("cup", FullyConnectedNetwork_Coupling_GlorotUniformInitializer)
ModelCatalog.register_custom_model("gnn", FullyConnectedNetwork_GNN_GlorotUniformInitializer)
ModelCatalog.register_custom_model("fc_glorot_uniform_init", FullyConnectedNetwork_GlorotUniformInitializer)
