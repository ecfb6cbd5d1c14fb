"""QuAntruped observation / action / contact-force layouts.

Field names are the reference's data tables (simulation_envs/quantruped_v3.py:68-112;
TVel adds `body_target_x_vel`, :351-384).  The lookup rules restate
QuAntrupedEnv.get_obs_indices / get_action_indices / get_contact_force_indices
(quantruped_v3.py:282-341): prefixes are matched with `str.startswith`, the output order
follows the prefix list, and within one prefix it follows the field order.  The real
index order is therefore body-first; the inline comments in the
reference's env files disagree with the code, and the code is what we follow.
"""
from __future__ import annotations

import numpy as np

OBS_FIELDS = [
    'body_height',
    'body_qpos_x', 'body_qpos_y', 'body_qpos_z', 'body_qpos_w',
    'fl_hip', 'fl_knee', 'hl_hip', 'hl_knee', 'hr_hip', 'hr_knee', 'fr_hip', 'fr_knee',
    'body_vel_x', 'body_vel_y', 'body_vel_z',
    'body_rot_vel_x', 'body_rot_vel_y', 'body_rot_vel_z',
    'fl_hip_vel', 'fl_knee_vel', 'hl_hip_vel', 'hl_knee_vel',
    'hr_hip_vel', 'hr_knee_vel', 'fr_hip_vel', 'fr_knee_vel',
    'fl_hip_pforce', 'fl_knee_pforce', 'hl_hip_pforce', 'hl_knee_pforce',
    'hr_hip_pforce', 'hr_knee_pforce', 'fr_hip_pforce', 'fr_knee_pforce',
    'fr_hip_hist_ctrl', 'fr_knee_vel_hist_ctrl', 'fl_hip_hist_ctrl', 'fl_knee_vel_hist_ctrl',
    'hl_hip_hist_ctrl', 'hl_knee_vel_hist_ctrl', 'hr_hip_hist_ctrl', 'hr_knee_vel_hist_ctrl',
]
TVEL_OBS_FIELDS = OBS_FIELDS + ['body_target_x_vel']

ACTION_FIELDS = ['fr_hip', 'fr_knee', 'fl_hip', 'fl_knee', 'hl_hip', 'hl_knee', 'hr_hip', 'hr_knee']

CONTACT_FORCE_FIELDS = [
    'body_floor', 'body',
    'fl_hip', 'fl_leg', 'fl_foot', 'hl_hip', 'hl_leg', 'hl_foot',
    'hr_hip', 'hr_leg', 'hr_foot', 'fr_hip', 'fr_leg', 'fr_foot',
]

OBS_FULL_DIM = len(OBS_FIELDS)          # 43
ACT_FULL_DIM = len(ACTION_FIELDS)       # 8
N_CONTACT_BODIES = len(CONTACT_FORCE_FIELDS)  # 14 bodies x 6 (cfrc_ext)


def get_obs_indices(prefixes=None, fields=OBS_FIELDS):
    if prefixes is None:
        return list(range(len(fields)))
    out = []
    for p in prefixes:
        out.extend(int(i) for i in np.where([f.startswith(p) for f in fields])[0])
    return out


def get_action_indices(prefixes=None):
    if prefixes is None:
        return list(range(len(ACTION_FIELDS)))
    out = []
    for p in prefixes:
        out.extend(int(i) for i in np.where([f.startswith(p) for f in ACTION_FIELDS])[0])
    return out


def get_contact_force_indices(prefixes=None, weights=None):
    """Returns (indices, weights) with one weight per selected body."""
    if prefixes is None:
        n = len(CONTACT_FORCE_FIELDS)
        return list(range(n)), [1.0] * n
    if weights is None:
        weights = [1.0] * len(prefixes)
    idx, w = [], []
    for p, wt in zip(prefixes, weights):
        sel = [int(i) for i in np.where([f.startswith(p) for f in CONTACT_FORCE_FIELDS])[0]]
        idx.extend(sel)
        w.extend([float(wt)] * len(sel))
    return idx, w
