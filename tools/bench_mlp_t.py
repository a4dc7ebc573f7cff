"""Graph-replay GPU timer shared by the GEMM dev tools."""
import torch  # noqa: E402

B = 24576
layers = [(627, 512), (512, 256), (256, 128), (128, 12), (736, 512), (572, 128), (128, 64), (132, 128), (29, 64)]


def t(fn, it=20):
    """GPU time per call: `it` calls captured in one hipGraph, replayed (no host overhead)."""
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        for _ in range(3):
            fn()
    torch.cuda.current_stream().wait_stream(side)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(it):
            fn()
    g.replay()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(3):
        g.replay()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / (3 * it) * 1e3


