"""Bind one buffer layout to both the CPU oracle (numpy) and liblgx.so (torch on the GPU,
or host tensors for the library's host backend, device="cpu") so parity tests can run both
on identical inputs and diff every field."""
import numpy as np

import driver


def _torchable(v):
    return v.view(np.int32) if v.dtype == np.uint32 else v


class Twin:
    def __init__(self, P, M_struct, num_reward_slots, terrain=None, device="cuda"):
        """terrain: None or (height_samples, mesh_words[, levels, types, origins]);
        device: "cuda" (HIP kernels) or "cpu" (liblgx.so's host backend, lgx_create(-1))."""
        import torch
        from legged_gym_custom_amd import _native
        self.torch = torch
        self.o = driver.OracleEnv(P, M_struct, num_reward_slots)
        if terrain is not None:
            self.o.set_terrain(*terrain)
        self.t = {}
        for k, v in self.o.a.items():
            self.t[k] = None if v is None else torch.from_numpy(_torchable(v).copy()).to(device)
        self.device = device
        self.native = _native.NativeEnv(M_struct, P, 0 if device == "cuda" else -1)
        self.native.bind(self.t)
        self.P = P

    def enable_curriculum(self, d):
        """Bind the command-curriculum buffers (initial ranges from fixture d) on both sides."""
        import golden_util as G
        G.enable_curriculum(self.o, d)
        for k in ("command_ranges", "curriculum_vals", "command_range_log"):
            self.t[k] = self.torch.from_numpy(self.o.a[k].copy()).to(self.device)
        self.native.bind(self.t)

    @property
    def a(self):
        return self.o.a

    def push(self):
        """numpy (oracle) state -> GPU buffers."""
        for k, v in self.o.a.items():
            if v is not None:
                self.t[k].copy_(self.torch.from_numpy(_torchable(v)))

    def pull(self):
        """GPU buffers -> numpy (oracle) state, in place (the oracle holds pointers to them)."""
        for k, v in self.o.a.items():
            if v is not None:
                v[...] = self.gpu(k)

    def gpu(self, k):
        v = self.t[k].cpu().numpy()
        return v.view(self.o.a[k].dtype) if self.o.a[k] is not None else v

    def stream(self):
        return self.torch.cuda.current_stream().cuda_stream if self.device == "cuda" else 0

    def sync(self):
        if self.device == "cuda":
            self.torch.cuda.synchronize()
