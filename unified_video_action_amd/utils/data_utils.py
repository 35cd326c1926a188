"""Batch -> device-resident VAE input / trajectories (reference: utils/data_utils.py).

The reference resizes all T=32 horizon frames to 256x256 (resize_image, :19-83), scales by
255, selects 8 frames (select_frames, :140-158) and normalises to [-1, 1] (:206-226).  Here
the selection happens first and resize+scale+normalise+NCHW->NHWC run in ONE HIP kernel
(uva_resize_select); bilinear resize is per frame, so selecting first is bit-identical and
4x cheaper.  Frame/trajectory index arithmetic is bit-exact with the reference.
"""
import random
from itertools import combinations_with_replacement

import numpy as np
import torch

from ..native import ops
from ..runtime import cdt

# 4-tuples over range(16) ending in 15 (data_utils.py:14-16)
COMBINATIONS = [c for c in combinations_with_replacement(range(16), 4) if c[-1] == 15]


def select_frame_indices(T, eval=False, select_timesteps=4, different_history_freq=False, rng_choice=None):
    if eval:
        idx = np.arange(0, T, T // select_timesteps) + select_timesteps - 1
    else:
        idx = np.arange(0, T, T // (select_timesteps * 2)) + select_timesteps - 1
        if different_history_freq:
            comb = rng_choice if rng_choice is not None else random.choice(COMBINATIONS)
            idx = np.concatenate([np.asarray(comb), idx[idx.shape[0] // 2:]])
    return idx.astype(np.int64)


def image_key(task_name):
    if "libero" in task_name:
        return "agentview_rgb"
    if "umi" in task_name:
        return "camera0_rgb"
    if "toolhang" in task_name:
        return "sideview_image"  # (data_utils.py:47-58: resize_image renames it to "image")
    return "image"


def vae_images(obs_image, sel, cin_pad=8):
    """[B, T, 3, H, W] fp32 in [0,1] -> NHWC [B*len(sel), 256, 256, cin_pad] (compute dtype),
    future-half frames of every sample first, then history-half frames."""
    B = obs_image.shape[0]
    out = torch.empty(B * len(sel), 256, 256, cin_pad, dtype=cdt(), device=obs_image.device)
    sel_t = torch.as_tensor(np.asarray(sel), dtype=torch.int32, device=obs_image.device)
    ops.resize_select(obs_image.float().contiguous(), sel_t, out, cin_pad)
    return out


def get_trajectory(nactions, T, shift_action, use_history_action=False):
    """data_utils.py:368-388."""
    if nactions is None:
        return None, None
    if use_history_action:
        if shift_action:
            return nactions[:, :T // 2], nactions[:, T // 2:-1]
        h, t = torch.chunk(nactions[:, 1:], 2, dim=1)
        return h, t
    if shift_action:
        return None, nactions[:, T // 2 - 1:-1]
    h, t = torch.chunk(nactions, 2, dim=1)
    return h, t


def umi_proprioception(obs, indices=None, different_history_freq=False, train=True):
    """process_data's UMI branch (data_utils.py:291-360): split history/pred halves and gather the
    history at the loaded image indices."""
    keys = ["robot0_eef_pos", "robot0_eef_rot_axis_angle", "robot0_gripper_width",
            "robot0_eef_rot_axis_angle_wrt_start"]
    out = {}
    for k in keys:
        if train:
            hist, pred = torch.chunk(obs[k], 2, dim=1)
        else:
            hist, pred = obs[k], None
        if different_history_freq and indices is not None:
            length = indices.shape[1] // 2 if train else indices.shape[1]
            bi = torch.arange(indices.shape[0], device=indices.device)[:, None].expand(-1, length)
            hist = hist[bi, indices[:, :length].long()]
        out[k] = hist
        out[k + "_pred"] = pred
    return out
