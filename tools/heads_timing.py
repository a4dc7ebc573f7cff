"""Loss-head kernels at the go2 minibatch shape (dev tool; run under rocprofv3 --kernel-trace
--stats): 50 x {ppo_head, aux_losses, fused loss_heads}, forward + backward each."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
from legged_gym_custom_amd.rsl_rl.modules import hip_mlp as H  # noqa: E402

dev = "cuda"
g = torch.Generator(device=dev).manual_seed(41)
B, A = int(os.environ.get("B", "24576")), 12
r = lambda *s: torch.randn(*s, device=dev, generator=g)  # noqa: E731
b = dict(actions=r(B, A), old_logp=r(B, 1), adv=r(B, 1), tv=r(B, 1), ret=r(B, 1), old_mu=r(B, A),
         old_sigma=r(B, A).abs() + 0.5, a=r(B, 20), t=r(B, 3))
leaves = [r(B, A), r(B, 1), r(A).abs() + 0.5, r(B, 20), r(B, 3)]
seeds = torch.tensor([1.0, 1.3, -0.01, 0.05, 1.0], device=dev)
for it in range(50):
    mu, v, std, pl, pr = [x.clone().requires_grad_(True) for x in leaves]
    s1, v1, e1, _k = H.ppo_head(mu, v, std, b["actions"], b["old_logp"], b["adv"], b["tv"], b["ret"],
                                b["old_mu"], b["old_sigma"], 0.2, True)
    rg, es = H.aux_losses(pl, b["a"], pr, b["t"])
    torch.autograd.backward([s1, v1, e1, rg, es], list(seeds.unbind()))
    mu, v, std, pl, pr = [x.clone().requires_grad_(True) for x in leaves]
    outs = H.loss_heads(mu, v, std, b["actions"], b["old_logp"], b["adv"], b["tv"], b["ret"], b["old_mu"],
                        b["old_sigma"], 0.2, True, pl, b["a"], pr, b["t"])
    torch.autograd.backward([outs[0], outs[1], outs[2], outs[4], outs[5]], list(seeds.unbind()))
torch.cuda.synchronize()
print("done")
