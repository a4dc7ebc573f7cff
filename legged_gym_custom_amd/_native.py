"""ctypes binding of liblgx.so (include/lgx.h). The product path calls ONLY this
library for the env step; if it is missing it raises. A HIP device index runs the
kernels (buffers on that device); device -1 runs the library's host backend (buffers in
host memory) — chosen explicitly by --sim_device=cpu, never as a fallback."""
import ctypes as C
import os

from . import _abi

LIB_PATH = os.environ.get("LGX_LIB") or os.path.join(os.path.dirname(os.path.abspath(__file__)), "lib", "liblgx.so")
_lib = None


class LgxError(RuntimeError):
    pass


def lib():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise LgxError(f"liblgx.so not built ({LIB_PATH}); run `python -m legged_gym_custom_amd.build_native`")
    L = C.CDLL(LIB_PATH)
    vp, u64, i32 = C.c_void_p, C.c_uint64, C.c_int32
    L.lgx_abi_version.restype = i32
    L.lgx_create.argtypes = [vp, vp, i32, C.POINTER(vp)]
    L.lgx_create.restype = C.c_int
    L.lgx_bind.argtypes = [vp, vp]
    L.lgx_step.argtypes = [vp, u64, u64, vp]
    L.lgx_step_dev.argtypes = [vp, u64, vp, vp]
    L.lgx_post_physics.argtypes = [vp, u64, u64, vp]
    L.lgx_physics.argtypes = [vp, vp]
    L.lgx_reset_envs.argtypes = [vp, vp, u64, u64, vp]
    L.lgx_episode_extras.argtypes = [vp, vp, vp, vp, vp, vp]
    L.lgx_command_curriculum.argtypes = [vp, u64, u64, vp, vp, vp]
    L.lgx_set_envs_per_wave.argtypes = [vp, i32]
    L.lgx_last_error.argtypes = [vp]
    L.lgx_last_error.restype = C.c_char_p
    L.lgx_destroy.argtypes = [vp]
    L.lgx_destroy.restype = None
    if L.lgx_abi_version() != _abi.ABI_VERSION:
        raise LgxError("liblgx ABI version mismatch; rebuild")
    _abi.check_layout(L, "lgx_sizeof_")
    _lib = L
    return L


EXPORTED = ["lgx_abi_version", "lgx_sizeof_model", "lgx_sizeof_task_params", "lgx_sizeof_buffers", "lgx_create",
            "lgx_bind", "lgx_step", "lgx_step_dev", "lgx_post_physics", "lgx_physics", "lgx_reset_envs", "lgx_last_error",
            "lgx_destroy", "lgx_episode_extras", "lgx_command_curriculum", "lgx_set_envs_per_wave"]


class NativeEnv:
    """Owns one lgx_env handle; buffers are torch tensors owned by the caller."""

    def __init__(self, model_struct, params_struct, device_index):
        self._L = lib()
        self.model = model_struct
        self.params = params_struct
        self.device_index = int(device_index)
        self._dev_type = "cpu" if self.device_index < 0 else "cuda"
        self.handle = C.c_void_p()
        rc = self._L.lgx_create(C.byref(model_struct), C.byref(params_struct), device_index, C.byref(self.handle))
        self._check(rc, "lgx_create")
        self.buffers = _abi.Buffers()
        self._keep = {}

    def _check(self, rc, what):
        if rc != 0:
            msg = self._L.lgx_last_error(self.handle).decode() if self.handle else "?"
            raise LgxError(f"{what} failed ({rc}): {msg}")

    def bind(self, tensors):
        """tensors: dict field -> torch tensor (contiguous; on the HIP device, or on the CPU for
        device -1) or None."""
        for name in _abi.BUFFER_FIELDS:
            t = tensors.get(name)
            if t is None:
                setattr(self.buffers, name, None)
                continue
            if not t.is_contiguous():
                raise LgxError(f"buffer {name} must be contiguous")
            if t.device.type != self._dev_type:
                where = "host memory (device -1)" if self._dev_type == "cpu" else "the HIP device"
                raise LgxError(f"buffer {name} must live in {where} (got {t.device})")
            setattr(self.buffers, name, t.data_ptr())
            self._keep[name] = t
        self._check(self._L.lgx_bind(self.handle, C.byref(self.buffers)), "lgx_bind")

    def set_envs_per_wave(self, n):
        """lgx_set_envs_per_wave: 2 (default where it applies), 1, or 0 (default)."""
        self._check(self._L.lgx_set_envs_per_wave(self.handle, int(n)), "lgx_set_envs_per_wave")

    def step(self, seed, step_counter, stream):
        self._check(self._L.lgx_step(self.handle, seed, step_counter, C.c_void_p(stream)), "lgx_step")

    def step_dev(self, seed, step_counter_tensor, stream):
        """lgx_step_dev: the step counter lives in a device uint64/int64 scalar tensor."""
        self._check(self._L.lgx_step_dev(self.handle, seed, C.c_void_p(step_counter_tensor.data_ptr()),
                                         C.c_void_p(stream)), "lgx_step_dev")

    def post_physics(self, seed, step_counter, stream):
        self._check(self._L.lgx_post_physics(self.handle, seed, step_counter, C.c_void_p(stream)), "lgx_post_physics")

    def reset_envs(self, mask, seed, call, stream):
        self._keep["_mask"] = mask
        self._check(self._L.lgx_reset_envs(self.handle, C.c_void_p(mask.data_ptr()), seed, call, C.c_void_p(stream)),
                    "lgx_reset_envs")

    def command_curriculum(self, seed, step, global_sum_count, stream):
        """lgx_command_curriculum; `step`: a device int64 scalar (the step counter lgx_step_dev
        read) or an int; global_sum_count: None or a device float64 [2] {sum, count}."""
        p = lambda t: None if t is None else C.c_void_p(t.data_ptr())  # noqa: E731
        dev = hasattr(step, "data_ptr")
        self._check(self._L.lgx_command_curriculum(self.handle, seed, 0 if dev else int(step), p(step) if dev else None,
                                                   p(global_sum_count), C.c_void_p(stream)), "lgx_command_curriculum")

    def episode_extras(self, means, level_mean, time_outs, stream, step_dev=None):
        """lgx_episode_extras into the given device tensors (level_mean / time_outs: None = skip);
        consumes episode_stats and, with step_dev (a device int64 scalar), advances it by one."""
        p = lambda t: None if t is None else C.c_void_p(t.data_ptr())  # noqa: E731
        self._check(self._L.lgx_episode_extras(self.handle, p(means), p(level_mean), p(time_outs), p(step_dev),
                                               C.c_void_p(stream)), "lgx_episode_extras")

    def __del__(self):
        try:
            if self.handle:
                self._L.lgx_destroy(self.handle)
                self.handle = C.c_void_p()
        except Exception:
            pass
