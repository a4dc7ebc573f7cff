"""Dev check (GPU): the go2 update's 17 weight-gradient GEMMs as one deferred group, against
fp64, for the liblgx_mlp build / knobs of this process (e.g. LGX_DW_SB1=1). Prints the worst
|err| / bound per layer. Usage: python tools/check_dw_group.py [rows]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
from legged_gym_custom_amd.rsl_rl.modules import hip_mlp as H  # noqa: E402

rows = int(sys.argv[1]) if len(sys.argv) > 1 else 24576
layers = [(627, 512), (512, 256), (256, 128), (128, 12), (736, 512), (512, 256), (256, 128), (128, 1),
          (29, 64), (64, 20), (20, 20), (132, 128), (128, 64), (64, 32), (572, 128), (128, 64), (64, 3)]
g = torch.Generator(device="cuda").manual_seed(3)
data = [(torch.randn(rows, o, device="cuda", generator=g), torch.randn(rows, i, device="cuda", generator=g),
         torch.zeros(o, i, device="cuda"), torch.zeros(o, device="cuda")) for i, o in layers]
print("splits", H.pick_split_group([(o, i, rows) for i, o in layers]))
for rep in range(3):
    for _, _, dW, db in data:
        dW.zero_()
        db.zero_()
    with H.deferred_weight_grads():
        for dy, x, dW, db in data:
            H.linear_weight_grad(dy, x, dW, db, accumulate=True)
    torch.cuda.synchronize()
    worst = []
    for (i, o), (dy, x, dW, db) in zip(layers, data):
        ref = dy.double().t() @ x.double()
        bound = 3e-5 * (dy.double().abs().t() @ x.double().abs()) + 1e-6
        e = float(((dW.double() - ref).abs() / bound).max())
        eb = float(((db.double() - dy.double().sum(0)).abs()).max())
        worst.append((f"{i}x{o}", round(e, 3), round(eb, 6)))
    print(rep, worst, flush=True)
