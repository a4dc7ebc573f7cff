"""Physics plausibility with the reference's TRAINED deploy networks.

The reference ships a policy trained in Isaac Gym / PhysX for go2_parkour
(deploy/networks/go2/<run>/{policy, adaptation_module, estimator, scan_encoder}.pt, composed
as in deploy/base/deploy_base.py:248-264). Those weights are read in place with the
parse-only reader (legged_gym_custom_amd/utils/ts_archive.py; nothing is deserialised, nothing
is stored in this repository) and drive this build's physics, stepped by the CPU oracle (the
same model as the HIP kernel: tests/test_gpu_trajectory.py pins the two together), on flat
ground with the parkour task's control and observation settings, a forward command and no
observation noise. If the build's contact/actuator physics is close to what the policy was
trained in, the robot walks: it survives, holds the trotting height the reference's recorded
deploy scan implies (deploy/base/SCAN_v12_ft_iii.txt: scan = z - 0.3 = -0.0040 on flat ground,
z = 0.296 m), tracks the command and steps in phase with the gait clock.

In-container dev tool (the reference tree is not on the GPU box):
  python tools/trained_policy_rollout.py [run] [N] [steps] [vx]
"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
NETS = "/root/reference/deploy/networks/go2"
SCAN = "/root/reference/deploy/base/SCAN_v12_ft_iii.txt"


def _seq(state, prefix=""):
    """Linear/ELU stack from a state dict of `<prefix><i>.weight` entries."""
    import torch.nn as nn
    idx = sorted({int(k[len(prefix):].split(".")[0]) for k in state if k.startswith(prefix)})
    layers = []
    for n, i in enumerate(idx):
        w, b = state[f"{prefix}{i}.weight"], state[f"{prefix}{i}.bias"]
        lin = nn.Linear(w.shape[1], w.shape[0])
        lin.weight.data.copy_(torch.from_numpy(w))
        lin.bias.data.copy_(torch.from_numpy(b))
        layers.append(lin)
        if n < len(idx) - 1:
            layers.append(nn.ELU())
    return nn.Sequential(*layers)


def load_nets(run):
    from legged_gym_custom_amd.utils import ts_archive as ts
    from legged_gym_custom_amd.rsl_rl.modules.support_networks import AdaptationEncoderTS
    d = os.path.join(NETS, run)
    pol = _seq(ts.read_state(os.path.join(d, "policy.pt")))
    est = _seq(ts.read_state(os.path.join(d, "estimator.pt")), "estimator.")
    sp = os.path.join(d, "scan_encoder.pt")  # flat-terrain runs (cheetah_*) have no scan latent
    scan = _seq(ts.read_state(sp), "scan_encoder.").eval() if os.path.exists(sp) else None
    ad_state = ts.read_state(os.path.join(d, "adaptation_module.pt"))
    ad = AdaptationEncoderTS(ad_state["fc_encoder.0.weight"].shape[1], 10, ad_state["fc_final.0.weight"].shape[0])
    ad.load_state_dict({k: torch.from_numpy(v) for k, v in ad_state.items()})
    return pol.eval(), est.eval(), scan, ad.eval()


def scan_trace_height():
    """Base height implied by the recorded deploy scan trace (deploy_base.py:66-83: a phase
    sync point, then 132-point scan frames of an obstacle approach): its first frame is flat
    ground (scan = z - 0.3 - h, h = 0)."""
    import re
    frames = [np.array(b.split(), float) for b in re.findall(r"\[([^\]]*)\]", open(SCAN).read())]
    first = next(f for f in frames if f.size == 132)
    return 0.3 + float(np.median(first))


def rollout(run="parkour_v12_ft_iii", n=64, steps=1000, vx=1.0, seed=3, est_source="net", period=None):
    """est_source: "net" (the shipped estimator.pt, as deploy_base.py:248-264) or "true" (the
    env's true estimated observation, v_body * lin_vel scale — what a trained estimator
    approximates: PPO.update trains it toward exactly that, ppo.py:224-231)."""
    import driver
    from legged_gym_custom_amd.envs import task_registry_configs
    from legged_gym_custom_amd import model as mdl, params as prm
    from legged_gym_custom_amd import _abi  # noqa: F401
    # parkour runs: the go2_parkour_finetune settings (gait clock, commands); flat runs: go2
    task = "go2_parkour_finetune" if os.path.exists(os.path.join(NETS, run, "scan_encoder.pt")) else "go2"
    cfg, _ = task_registry_configs(task)
    cfg.terrain.mesh_type = "plane"
    cfg.terrain.curriculum = False
    cfg.noise.add_noise = False
    cfg.domain_rand.push_robots = False
    cfg.commands.user_command = [vx, 0.0, 0.0, 0.0]
    if period is not None:  # gait clock (the deploy config's is 0.35 s, deploy/configs/go2.yaml:21)
        cfg.env.period = period
    cfg.env.num_envs = n
    m = mdl.load_model(cfg.asset.file, cfg.asset.foot_name)
    P = prm.build_task_params(cfg, m, n, go2=True)
    o = driver.OracleEnv(P, mdl.to_struct(m), P.num_reward_terms + P.has_termination_reward)
    a = o.a
    a["friction"][:] = cfg.terrain.static_friction
    side = int(np.ceil(np.sqrt(n)))
    a["env_origins"][:, 0] = 3.0 * (np.arange(n) // side)
    a["env_origins"][:, 1] = 3.0 * (np.arange(n) % side)
    o.reset_envs(np.ones(n, bool), seed, 0)
    pol, est, scan, ad = load_nets(run)
    H, Pp = P.history_len, P.num_proprio
    feet = list(P.feet_idx[:4])
    z, vxs, vest, contact, phase, fell = [], [], [], [], [], np.zeros(n, bool)
    x0 = a["root_states"][:, 0].copy()
    with torch.no_grad():
        for k in range(steps):
            obs = torch.from_numpy(a["obs"].copy())
            hist = obs[:, :H * Pp].reshape(n, H, Pp)
            e_net = est(obs)
            e = e_net if est_source == "net" else torch.from_numpy(a["est"].copy())
            parts = [obs, ad(hist)] + ([scan(torch.from_numpy(a["scan"].copy()))] if scan is not None else []) + [e]
            x = torch.cat(parts, dim=-1)
            a["actions_in"][:] = pol(x).numpy()
            o.step(seed, k + 1)
            fell |= (a["reset"] != 0) & (a["time_out"] == 0)
            if k >= 100:  # after the start transient
                z.append(a["root_states"][:, 2].copy())
                vxs.append(a["base_lin_vel"][:, 0].copy())
                vest.append(e_net[:, 0].numpy() / cfg.normalization.obs_scales.lin_vel)
                contact.append(a["contact_forces"][:, feet, 2] > 1.0)
                phase.append(a["rpy_phase"][:, 3:7].copy())  # fl fr bl br, [0, 1)
    z, vxs, vest, contact, phase = map(np.array, (z, vxs, vest, contact, phase))
    alive = ~fell
    # stance when sin(2 pi phase) <= 2 * percent_time_on_ground - 1 (go2.py _reward_phase_contact_match)
    thr = 2.0 * cfg.rewards.percent_time_on_ground - 1.0
    stance = np.sin(2 * np.pi * phase) <= thr
    return {
        "run": run, "estimator_input": est_source, "task_settings": task, "gait_period": cfg.env.period, "envs": n, "steps": steps, "command_vx": vx,
        "survival": float(alive.mean()),
        "base_height_mean": float(z[:, alive].mean()), "base_height_std": float(z[:, alive].std()),
        "scan_trace_height": scan_trace_height(),
        "vx_mean": float(vxs[:, alive].mean()),
        "vx_estimated_mean": float(vest[:, alive].mean()),  # the policy's own velocity estimator
        "distance_x_mean": float((a["root_states"][alive, 0] - x0[alive]).mean()),
        "duty_cycle": contact[:, alive].mean(axis=(0, 1)).round(3).tolist(),
        "contact_matches_gait_clock": float((contact[:, alive] == stance[:, alive]).mean()),
    }


if __name__ == "__main__":
    args = sys.argv[1:]
    est_source = "true" if "--true-est" in args else "net"
    period = None
    if "--period" in args:
        i = args.index("--period")
        period = float(args[i + 1])
        del args[i:i + 2]
    args = [x for x in args if x != "--true-est"]
    res = rollout(args[0] if args else "parkour_v12_ft_iii", *(int(v) for v in args[1:3]),
                  *(float(v) for v in args[3:4]), est_source=est_source, period=period)
    for k, v in res.items():
        print(f"{k:28s} {v}")
