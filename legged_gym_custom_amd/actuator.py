"""ANYmal series-elastic actuator network (anymal.py:24-81).

The reference loads `resources/actuator_nets/anydrive_v3_lstm.pt` with torch.jit.load and
calls it once per joint per physics substep:

    tau, (h, c) = net(x, (h, c)),  x[N*12, 1, 2] = (a * action_scale + q0 - q, qd)

The archive's own TorchScript source (code/__torch__/models.py) defines the net as
    x0 = x * in_scale                      in_scale [1, 1, 2]
    y, (h, c) = LSTM(x0, (h, c))           2 layers, hidden 8, batch_first, gates i f g o
    tau = out_scale * squeeze(Linear(y))   Linear 8 -> 1, out_scale [1]
with state h, c [2, N*12, 8].

Here the archive named by cfg.control.actuator_net_file is read at env creation, as the
reference does, but never deserialised (no TorchScript, no unpickling): the tensor
storages are raw little-endian fp32 files in the zip, and the name -> storage mapping
is read by walking data.pkl's opcodes with pickletools (a parser; nothing is executed
or constructed). No trained weights ship with this package: the user's own archive is
read in place, and the tests use synthetic nets of the same architecture (saved with
torch.jit.save, so the reader is pinned against torch's own serializer). The env kernel
evaluates the net per joint lane inside each substep (lgx_env.hip `sea_torque`);
`SeaLSTM` below is the torch restatement used as the fp32 reference in tests.
"""
import io
import os
import pickletools
import zipfile
from typing import Tuple

import numpy as np
import torch

SEA_KEYS = ["in_scale", "out_scale", "lstm.weight_ih_l0", "lstm.weight_hh_l0", "lstm.bias_ih_l0", "lstm.bias_hh_l0",
            "lstm.weight_ih_l1", "lstm.weight_hh_l1", "lstm.bias_ih_l1", "lstm.bias_hh_l1", "linear.weight",
            "linear.bias"]
SEA_SHAPES = {"in_scale": (1, 1, 2), "out_scale": (1,), "lstm.weight_ih_l0": (32, 2), "lstm.weight_hh_l0": (32, 8),
              "lstm.bias_ih_l0": (32,), "lstm.bias_hh_l0": (32,), "lstm.weight_ih_l1": (32, 8),
              "lstm.weight_hh_l1": (32, 8), "lstm.bias_ih_l1": (32,), "lstm.bias_hh_l1": (32,),
              "linear.weight": (1, 8), "linear.bias": (1,)}


def _tokens(pkl_bytes):
    """Flatten a pickle opcode stream into ('S', str) / ('I', int) / ('M',) / ('T',) /
    ('P',) / ('G', module name) tokens, resolving memo'd strings. Parse only."""
    memo, out, last = {}, [], None
    for op, arg, _ in pickletools.genops(io.BytesIO(pkl_bytes)):
        name = op.name
        if name in ("BINUNICODE", "SHORT_BINUNICODE", "UNICODE"):
            out.append(("S", arg))
            last = ("S", arg)
        elif name in ("BINPUT", "LONG_BINPUT", "PUT"):
            memo[arg] = last
        elif name == "MEMOIZE":
            memo[len(memo)] = last
        elif name in ("BINGET", "LONG_BINGET", "GET"):
            v = memo.get(arg)
            if v is not None:
                out.append(v)
            last = v
        elif name in ("BININT", "BININT1", "BININT2", "INT", "LONG1"):
            out.append(("I", int(arg)))
            last = None
        elif name == "MARK":
            out.append(("M",))
        elif name in ("TUPLE", "TUPLE1", "TUPLE2", "TUPLE3"):
            out.append(("T",))
        elif name == "BINPERSID":
            out.append(("P",))
        elif name in ("GLOBAL", "STACK_GLOBAL"):
            out.append(("G", arg))
            last = ("G", arg)
        else:
            last = None
    return out


def read_torchscript_tensors(path):
    """{attribute path: float32 array} of a TorchScript archive's tensors, from the raw
    storages (contiguous tensors, FloatStorage only)."""
    z = zipfile.ZipFile(path)
    names = z.namelist()
    root = names[0].split("/")[0]
    toks = _tokens(z.read(f"{root}/data.pkl"))
    tensors = {}
    i = 0
    while i < len(toks):
        t = toks[i]
        if t == ("S", "storage") and i + 2 < len(toks) and toks[i + 1][0] == "G" and toks[i + 2][0] == "S":
            if not toks[i + 1][1].endswith("FloatStorage"):
                raise ValueError(f"unsupported storage type {toks[i + 1][1]}")
            key = toks[i + 2][1]
            # attribute name: nearest preceding plain string
            j = i - 1
            while j >= 0 and not (toks[j][0] == "S" and toks[j][1] not in ("storage", "cpu") and
                                  not toks[j][1].isdigit()):
                j -= 1
            attr = toks[j][1]
            # sizes: the first MARK ... TUPLE of ints after BINPERSID + offset
            k = i
            while toks[k] != ("P",):
                k += 1
            k += 2  # BINPERSID, storage offset int
            assert toks[k] == ("M",), toks[k]
            k += 1
            size = []
            while toks[k][0] == "I":
                size.append(toks[k][1])
                k += 1
            raw = np.frombuffer(z.read(f"{root}/data/{key}"), dtype="<f4")
            tensors[attr] = (raw[:int(np.prod(size))] if size else raw[:1]).reshape(size).copy()
            i = k
        else:
            i += 1
    # qualify the LSTM / Linear members by their module (the archive nests them)
    out = {}
    for attr, v in tensors.items():
        if attr.startswith(("weight_ih", "weight_hh", "bias_ih", "bias_hh")):
            out["lstm." + attr] = v
        elif attr in ("weight", "bias"):
            out["linear." + attr] = v
        else:
            out[attr] = v
    return out


def load_sea_lstm(path):
    """Weights of the SEA net in the TorchScript archive at `path` (anymal.py:24)."""
    if not os.path.exists(path):
        raise FileNotFoundError(f"actuator network archive not found: {path} (cfg.control.actuator_net_file)")
    if not zipfile.is_zipfile(path):
        raise ValueError(f"{path} is not a TorchScript archive")
    w = read_torchscript_tensors(path)
    for k in SEA_KEYS:
        if k not in w or tuple(w[k].shape) != SEA_SHAPES[k]:
            raise ValueError(f"actuator net {path}: {k} missing or not {SEA_SHAPES[k]}")
    return {k: np.ascontiguousarray(w[k], dtype=np.float32) for k in SEA_KEYS}


def random_sea_weights(seed=0, scale=0.5):
    """Synthetic SEA net weights (tests): the reference architecture, random values."""
    g = np.random.default_rng(seed)
    w = {k: (g.standard_normal(SEA_SHAPES[k]) * scale).astype(np.float32) for k in SEA_KEYS}
    w["in_scale"] = np.array([[[4.0, 0.1]]], np.float32)
    w["out_scale"] = np.array([20.0], np.float32)
    return w


def save_sea_archive(w, path):
    """Write `w` as a TorchScript archive of SeaLSTM (test fixtures; our own file)."""
    torch.jit.save(torch.jit.script(SeaLSTM(w)), path)


def fill_task_params(P, w):
    """Copy the weights into lgx_task_params (sea_*), read by the kernel per substep."""
    P.actuator_net = 1
    P.sea_in_scale[:] = w["in_scale"].reshape(2).tolist()
    P.sea_out_scale = float(w["out_scale"][0])
    flat = lambda a: a.reshape(-1).tolist()  # noqa: E731
    P.sea_w_ih0[:] = flat(w["lstm.weight_ih_l0"])
    P.sea_w_hh0[:] = flat(w["lstm.weight_hh_l0"])
    P.sea_b_ih0[:] = flat(w["lstm.bias_ih_l0"])
    P.sea_b_hh0[:] = flat(w["lstm.bias_hh_l0"])
    P.sea_w_ih1[:] = flat(w["lstm.weight_ih_l1"])
    P.sea_w_hh1[:] = flat(w["lstm.weight_hh_l1"])
    P.sea_b_ih1[:] = flat(w["lstm.bias_ih_l1"])
    P.sea_b_hh1[:] = flat(w["lstm.bias_hh_l1"])
    P.sea_lin_w[:] = flat(w["linear.weight"])
    P.sea_lin_b = float(w["linear.bias"][0])


class SeaLSTM(torch.nn.Module):
    """torch restatement of the archive's LSTMsea (models.py above): same call signature
    as the TorchScript module, `net(x, (h, c)) -> (tau, (h, c))`."""

    def __init__(self, w):
        super().__init__()
        self.register_buffer("in_scale", torch.from_numpy(w["in_scale"].copy()))
        self.register_buffer("out_scale", torch.from_numpy(w["out_scale"].copy()))
        self.lstm = torch.nn.LSTM(2, 8, num_layers=2, batch_first=True)
        self.linear = torch.nn.Linear(8, 1)
        with torch.no_grad():
            for k in SEA_KEYS[2:]:
                mod, name = k.split(".")
                getattr(getattr(self, mod), name).copy_(torch.from_numpy(w[k]))

    def forward(self, x: torch.Tensor, hc: Tuple[torch.Tensor, torch.Tensor]):
        y, (h, c) = self.lstm(x * self.in_scale, hc)
        return self.out_scale * torch.squeeze(self.linear(y)), (h, c)
