"""The C-ABI libraries load and export every symbol their headers declare; the ctypes
mirrors have the compiled struct layouts. No compute calls (no GPU needed)."""
import ctypes as C
import os
import re

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

HEADERS = {"lgx.h": "liblgx.so", "lgx_mlp.h": "liblgx_mlp.so", "lgx_s8.h": "liblgx_s8.so"}


def _declared(header):
    src = open(os.path.join(REPO, "include", header)).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    src = re.sub(r"//[^\n]*", "", src)
    return sorted(set(re.findall(r"\b(lgx_\w+)\s*\(", src)) - {"lgx_gemm_args"})


@pytest.fixture(scope="module")
def libs():
    from legged_gym_custom_amd import build_native
    build_native.build()  # no-op when up to date (hipcc cross-compiles gfx950 here)
    return {h: C.CDLL(os.path.join(REPO, "legged_gym_custom_amd", "lib", lib)) for h, lib in HEADERS.items()}


@pytest.mark.parametrize("header", sorted(HEADERS))
def test_every_declared_symbol_is_exported(libs, header):
    names = _declared(header)
    assert len(names) >= 4
    missing = [n for n in names if not hasattr(libs[header], n)]
    assert not missing, f"{HEADERS[header]} lacks {missing}"


def test_python_bindings_cover_the_headers():
    from legged_gym_custom_amd import _native
    from legged_gym_custom_amd.rsl_rl.modules import hip_mlp
    assert set(_declared("lgx.h")) <= set(_native.EXPORTED) | {n for n in _declared("lgx.h") if n.startswith("lgx_sizeof")}
    assert set(_declared("lgx_mlp.h")) == set(hip_mlp.EXPORTED)
    from legged_gym_custom_amd.rsl_rl.modules import hip_s8
    assert set(_declared("lgx_s8.h")) == set(hip_s8.EXPORTED)


def test_struct_layouts_and_abi_versions(libs):
    from legged_gym_custom_amd import _abi, _native
    from legged_gym_custom_amd.rsl_rl.modules import hip_mlp
    L = _native.lib()  # checks abi version + lgx_sizeof_{model,task_params,buffers}
    assert L.lgx_abi_version() == _abi.ABI_VERSION
    M = hip_mlp.lib()  # checks abi version + sizeof(lgx_gemm_args)
    assert M.lgx_mlp_sizeof_gemm_args() == C.sizeof(hip_mlp.GemmArgs)
    from legged_gym_custom_amd.rsl_rl.modules import hip_s8
    S8 = hip_s8.lib()  # checks abi version + sizeof(lgx_s8_gemm_args)
    assert S8.lgx_s8_sizeof_gemm_args() == C.sizeof(hip_s8.GemmArgs)


def test_gemm_rejects_bad_arguments_without_touching_the_device(libs):
    from legged_gym_custom_amd.rsl_rl.modules import hip_mlp
    L = hip_mlp.lib()
    a = hip_mlp.GemmArgs(M=-1, N=1, K=1)
    assert L.lgx_gemm(C.byref(a), None) < 0
    assert b"negative" in L.lgx_mlp_last_error()
    a = hip_mlp.GemmArgs(M=4, N=4, K=4, A=16, B=16, C=16, epilogue=hip_mlp.EPI_BIAS)
    assert L.lgx_gemm(C.byref(a), None) < 0 and b"bias" in L.lgx_mlp_last_error()
    assert L.lgx_mlp_pick_split(512, 627, 24576) >= 2
