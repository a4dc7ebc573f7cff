"""The product learner fails loudly when its HIP libraries are missing: with
the S8 update / fused act selected (the defaults) a missing or broken liblgx_s8.so raises from
the executors' `supported` checks instead of quietly selecting the older GEMM core, so neither
the GPU tests nor bench.py can pass on a different code path than the one they claim."""
import types

import pytest

from legged_gym_custom_amd.rsl_rl.algorithms import s8_act, s8_update
from legged_gym_custom_amd.rsl_rl.modules import hip_s8


def _broken(monkeypatch):
    def load(*a, **k):
        raise hip_s8.S8LibError("liblgx_s8.so not built (test)")
    monkeypatch.setattr(hip_s8, "_lib", None)
    monkeypatch.setattr(hip_s8, "load", load)


def test_s8_update_raises_without_library(monkeypatch):
    _broken(monkeypatch)
    alg = types.SimpleNamespace(on_gpu=True)
    with pytest.raises(hip_s8.S8LibError):
        s8_update.S8Minibatch.supported(alg, 24576)


def test_fused_act_raises_without_library(monkeypatch):
    _broken(monkeypatch)
    alg = types.SimpleNamespace(on_gpu=True)
    with pytest.raises(hip_s8.S8LibError):
        s8_act.S8Act.supported(alg)


def test_cpu_learner_never_needs_the_library(monkeypatch):
    """The CPU learner (--rl_device=cpu) is a selected path, not a fallback: it never loads it."""
    _broken(monkeypatch)
    alg = types.SimpleNamespace(on_gpu=False)
    assert s8_update.S8Minibatch.supported(alg, 24576) is False
    assert s8_act.S8Act.supported(alg) is False
