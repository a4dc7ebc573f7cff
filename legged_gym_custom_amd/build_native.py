"""Build the HIP libraries in-tree for gfx950 with hipcc:
  lib/liblgx.so      env step (csrc/lgx_env.hip, include/lgx.h) + its host backend
                     (csrc/lgx_env_host.cpp, g++ -fopenmp, linked in: lgx_create(device=-1))
  lib/liblgx_mlp.so  learner MLP GEMMs (csrc/lgx_mlp.hip, include/lgx_mlp.h)
  lib/liblgx_s8.so   the update's GEMM core on pre-split operands (csrc/lgx_s8.hip) and the rollout's
                     act networks in one launch (csrc/lgx_act.hip), include/lgx_s8.h"""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
INC = os.path.join(os.path.dirname(HERE), "include")
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950")
LIBS = {
    "liblgx.so": (["lgx_env.hip"], ["lgx_device.h", "lgx_host.h", "lgx_env_host.cpp", "lgx_knobs.h"], ["lgx.h"]),
    "liblgx_mlp.so": (["lgx_mlp.hip"], ["lgx_knobs.h"], ["lgx_mlp.h"]),
    "liblgx_s8.so": (["lgx_s8.hip", "lgx_act.hip", "lgx_s8chain.hip"], ["lgx_knobs.h"], ["lgx_s8.h"]),
}
OUT = os.path.join(HERE, "lib", "liblgx.so")
OUT_MLP = os.path.join(HERE, "lib", "liblgx_mlp.so")


def _paths(name):
    srcs, hdrs, incs = LIBS[name]
    src = [os.path.join(HERE, "csrc", s) for s in srcs]
    deps = src + [os.path.join(HERE, "csrc", h) for h in hdrs] + [os.path.join(INC, h) for h in incs]
    return src, deps, os.path.join(HERE, "lib", name)


def needs_build(name="liblgx.so"):
    src, deps, out = _paths(name)
    if not os.path.exists(out):
        return True
    t = os.path.getmtime(out)
    return any(os.path.getmtime(d) > t for d in deps)


def _host_objects(name, verbose):
    """liblgx.so's host backend: compiled by g++ with OpenMP (libgomp, as torch's CPU ops)."""
    if name != "liblgx.so":
        return []
    src = os.path.join(HERE, "csrc", "lgx_env_host.cpp")
    obj = os.path.join(HERE, "lib", "lgx_env_host.o")
    cmd = ["g++", "-O3", "-std=c++17", "-fPIC", "-fopenmp", "-ffp-contract=off", "-fno-fast-math", "-Wall",
           "-c", "-o", obj, src]
    if verbose:
        print(" ".join(cmd))
    subprocess.run(cmd, check=True)
    gomp = subprocess.run(["g++", "-print-file-name=libgomp.so"], check=True, capture_output=True,
                          text=True).stdout.strip()
    return [obj, gomp]


def build_one(name, force=False, verbose=False):
    """Compile one library if a source is newer than it (or force). Returns (path, compiled?)."""
    src, _, out = _paths(name)
    if not force and not needs_build(name):
        return out, False
    os.makedirs(os.path.dirname(out), exist_ok=True)
    hip = ["hipcc", f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off"]
    extra = _host_objects(name, verbose)
    if extra:  # compile the HIP source alone (hipcc reads inputs after a .hip file as HIP), then link
        obj = out[:-3] + "_hip.o"
        cmds = [hip + ["-c", "-o", obj] + src, ["hipcc", "-shared", "-o", out + ".tmp", obj] + extra]
    else:
        cmds = [hip + ["-shared", "-o", out + ".tmp"] + src]
    for cmd in cmds:
        if verbose:
            print(" ".join(cmd))
        subprocess.run(cmd, check=True)
    os.replace(out + ".tmp", out)
    return out, True


def build_variant(name, out, flags, verbose=True):
    """A dev build of one library (e.g. liblgx_s8.so with -DLGX_DEV_KNOBS or -DLGX_S8_CLOCK) at `out`;
    the product path never loads it (bench.py refuses LGX_*_LIB overrides)."""
    src, _, _ = _paths(name)
    hip = ["hipcc", f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off"] + list(flags)
    if name == "liblgx.so":
        return build_env_variant(out, flags, verbose)
    cmd = hip + ["-shared", "-o", out] + src
    if verbose:
        print(" ".join(cmd))
    subprocess.run(cmd, check=True)
    return out


def build_env_variant(out, flags, verbose=True):
    """A dev build of liblgx.so with extra compile flags (e.g. -DLGX_PHASE_CLOCK) at `out`."""
    src, _, _ = _paths("liblgx.so")
    obj = out[:-3] + "_hip.o"
    hip = ["hipcc", f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off"] + list(flags)
    for cmd in (hip + ["-c", "-o", obj] + src, ["hipcc", "-shared", "-o", out, obj] + _host_objects("liblgx.so", verbose)):
        if verbose:
            print(" ".join(cmd))
        subprocess.run(cmd, check=True)
    return out


def build(force=False, verbose=False):
    for name in LIBS:
        out, compiled = build_one(name, force=force, verbose=verbose)
        if verbose:
            print(f"build_native: {name}: {'compiled' if compiled else 'reused (up to date)'} -> {out}")
    return OUT


if __name__ == "__main__":
    build(force="--force" in sys.argv, verbose=True)
    print(OUT, OUT_MLP)
