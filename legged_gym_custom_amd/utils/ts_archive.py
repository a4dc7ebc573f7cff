"""Weights of a TorchScript archive (torch.jit.save / export_policy_as_jit, helpers.py:180-214)
read WITHOUT deserialising it: no TorchScript, no unpickling, nothing constructed or executed.

The archive is a zip: `<root>/data.pkl` describes the module tree, `<root>/data/<key>` holds
each tensor's raw little-endian storage. data.pkl is walked as a flat opcode stream with
pickletools (a parser): a module is `key, GLOBAL __torch__.<class>, ..., BUILD`, a tensor
is `attr, GLOBAL torch._utils _rebuild_tensor_v2, (storage, FloatStorage, key, cpu, numel),
offset, (sizes), (strides), ...`. The result maps each tensor's dotted module path (the
state_dict key, e.g. `0.weight`, `scan_encoder.2.bias`, `conv_layers.0.weight`) to a float32
array. Contiguous FloatStorage tensors only; anything else raises.

Used to read the reference's trained deploy networks (deploy/networks/go2/*/{policy,
adaptation_module,estimator,scan_encoder}.pt) into this build's modules in a test that runs
only where those files exist; no weights are stored in this repository.
"""
import collections
import io
import pickletools
import zipfile

import numpy as np


def _ops(pkl):
    """(kind, value) tokens: S string, I int, G global, M mark, T tuple, P persid, B build;
    memo'd strings/globals resolved on BINGET."""
    memo, last = {}, None
    for op, arg, _ in pickletools.genops(io.BytesIO(pkl)):
        n = op.name
        tok = None
        if n in ("BINUNICODE", "SHORT_BINUNICODE", "UNICODE", "BINUNICODE8"):
            tok = ("S", arg)
        elif n in ("GLOBAL", "STACK_GLOBAL"):
            tok = ("G", arg)
        elif n in ("BINPUT", "LONG_BINPUT", "PUT"):
            memo[arg] = last
            continue
        elif n == "MEMOIZE":
            memo[len(memo)] = last
            continue
        elif n in ("BINGET", "LONG_BINGET", "GET"):
            tok = memo.get(arg)
        elif n in ("BININT", "BININT1", "BININT2", "INT", "LONG1"):
            tok = ("I", int(arg))
        elif n == "MARK":
            tok = ("M", None)
        elif n in ("TUPLE", "TUPLE1", "TUPLE2", "TUPLE3", "EMPTY_TUPLE"):
            tok = ("T", None)
        elif n == "BINPERSID":
            tok = ("P", None)
        elif n == "BUILD":
            tok = ("B", None)
        last = tok
        if tok is not None:
            yield tok


def read_state(path):
    """OrderedDict {dotted path: float32 ndarray} of the archive's tensors, in file order."""
    z = zipfile.ZipFile(path)
    root = z.namelist()[0].split("/")[0]
    toks = list(_ops(z.read(f"{root}/data.pkl")))
    out = collections.OrderedDict()
    stack = []  # module path
    i = 0
    while i < len(toks):
        kind, val = toks[i]
        if kind == "G" and val.startswith("__torch__."):
            prev = toks[i - 1] if i > 0 else None
            stack.append(prev[1] if prev is not None and prev[0] == "S" else "")
        elif kind == "B":
            if stack:
                stack.pop()
        elif kind == "G" and val == "torch._utils _rebuild_tensor_v2":
            attr = toks[i - 1][1]
            k = i + 1
            while toks[k] != ("S", "storage"):
                k += 1
            if toks[k + 1] != ("G", "torch FloatStorage"):
                raise ValueError(f"{path}: unsupported storage {toks[k + 1]}")
            key = toks[k + 2][1]
            numel = toks[k + 4][1]
            while toks[k][0] != "P":
                k += 1
            offset = toks[k + 1][1]
            assert toks[k + 2][0] == "M", toks[k + 2]
            k += 3
            size = []
            while toks[k][0] == "I":
                size.append(toks[k][1])
                k += 1
            k += 2  # TUPLE, MARK of the strides
            stride = []
            while toks[k][0] == "I":
                stride.append(toks[k][1])
                k += 1
            want = [int(np.prod(size[d + 1:])) for d in range(len(size))]
            if stride != want:
                raise ValueError(f"{path}: {attr} is not contiguous (sizes {size}, strides {stride})")
            raw = np.frombuffer(z.read(f"{root}/data/{key}"), dtype="<f4")
            if raw.size < offset + int(np.prod(size)) or numel < int(np.prod(size)):
                raise ValueError(f"{path}: storage {key} too small for {attr}")
            name = ".".join([p for p in stack[1:] if p] + [attr])
            out[name] = raw[offset:offset + int(np.prod(size))].reshape(size).copy()
            i = k
            continue
        i += 1
    return out
