"""legged_gym/utils/math.py:38-55 (host-side helpers for user code; the kernel has its own)."""
import numpy as np
import torch


def _quat_apply(a, b):
    shape = b.shape
    a = a.reshape(-1, 4)
    b = b.reshape(-1, 3)
    xyz = a[:, :3]
    t = xyz.cross(b, dim=-1) * 2
    return (b + a[:, 3:] * t + xyz.cross(t, dim=-1)).view(shape)


def quat_apply_yaw(quat, vec):
    q = quat.clone().view(-1, 4)
    q[:, :2] = 0.0
    q = q / q.norm(p=2, dim=-1).clamp(min=1e-9).unsqueeze(-1)
    return _quat_apply(q, vec)


def wrap_to_pi(angles):
    angles %= 2 * np.pi
    angles -= 2 * np.pi * (angles > np.pi)
    return angles


def torch_rand_sqrt_float(lower, upper, shape, device):
    r = 2 * torch.rand(*shape, device=device) - 1
    r = torch.where(r < 0.0, -torch.sqrt(-r), torch.sqrt(r))
    r = (r + 1.0) / 2.0
    return (upper - lower) * r + lower
