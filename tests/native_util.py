"""Bind one buffer layout to both the CPU oracle (numpy) and liblgx.so (torch on the GPU)
so parity tests can run both on identical inputs and diff every field."""
import numpy as np

import driver


class Twin:
    def __init__(self, P, M_struct, num_reward_slots):
        import torch
        from legged_gym_custom_amd import _native
        self.torch = torch
        self.o = driver.OracleEnv(P, M_struct, num_reward_slots)
        self.t = {}
        for k, v in self.o.a.items():
            self.t[k] = None if v is None else torch.from_numpy(v.copy()).cuda()
        self.native = _native.NativeEnv(M_struct, P, 0)
        self.native.bind(self.t)
        self.P = P

    @property
    def a(self):
        return self.o.a

    def push(self):
        """numpy (oracle) state -> GPU buffers."""
        for k, v in self.o.a.items():
            if v is not None:
                self.t[k].copy_(self.torch.from_numpy(v))

    def gpu(self, k):
        return self.t[k].cpu().numpy()

    def stream(self):
        return self.torch.cuda.current_stream().cuda_stream

    def sync(self):
        self.torch.cuda.synchronize()
