"""Why the isolated weight-gradient group (bench.py roofline_learner: 10 back-to-back replays)
runs slower than the same launch inside the runner: time ONE replay of the
17-layer dW group (24,576 rows, graph-captured) after different cache states:
  cold   - a 1 GiB buffer written just before (L2 and the 256 MiB Infinity Cache hold none of
           the operands)
  dy     - the output gradients (202 MB) rewritten just before, as the runner's backward
           input-gradient launches write them right before the dW launch
  dy+x   - the output gradients and the actor/critic layer inputs rewritten just before
  back2back - the bench's method: 10 replays in one graph, mean per replay
Usage (GPU): python tools/dw_cache_probe.py"""
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
from legged_gym_custom_amd.rsl_rl.modules import hip_mlp as H  # noqa: E402

dev = "cuda:0"
rows = 24576
layers = [(627, 512), (512, 256), (256, 128), (128, 12), (736, 512), (512, 256), (256, 128), (128, 1),
          (29, 64), (64, 20), (20, 20), (132, 128), (128, 64), (64, 32), (572, 128), (128, 64), (64, 3)]
g = torch.Generator(device=dev).manual_seed(7)
data = [(torch.randn(rows, o, device=dev, generator=g), torch.randn(rows, i, device=dev, generator=g),
         torch.zeros(o, i, device=dev), torch.zeros(o, device=dev)) for i, o in layers]
flush = torch.empty(1 << 28, device=dev)  # 1 GiB


def once():
    with H.deferred_weight_grads():
        for dy, x, dW, db in data:
            H.linear_weight_grad(dy, x, dW, db, accumulate=True)


side = torch.cuda.Stream(dev)
side.wait_stream(torch.cuda.current_stream(dev))
with torch.cuda.stream(side):
    for _ in range(3):
        once()
torch.cuda.current_stream(dev).wait_stream(side)
g1 = torch.cuda.CUDAGraph()
with torch.cuda.graph(g1):
    once()
g10 = torch.cuda.CUDAGraph()
with torch.cuda.graph(g10):
    for _ in range(10):
        once()
st = torch.cuda.current_stream(dev)


def timed(prep, graph, n=1):
    ts = []
    for _ in range(12):
        prep()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record(st)
        graph.replay()
        e.record(st)
        torch.cuda.synchronize(dev)
        ts.append(s.elapsed_time(e) * 1e3 / n)
    return statistics.median(ts[2:])


def cold():
    flush.fill_(1.0)


def touch_dy():
    cold()
    for dy, _, _, _ in data:
        dy.mul_(1.0)


def touch_dy_x():
    touch_dy()
    for k in (0, 4):
        data[k][1].mul_(1.0)


res = {"cold": timed(cold, g1), "dy": timed(touch_dy, g1), "dy+x": timed(touch_dy_x, g1),
       "back2back": timed(lambda: None, g10, 10)}
print(" ".join(f"{k} {v:.1f}us" for k, v in res.items()), flush=True)
