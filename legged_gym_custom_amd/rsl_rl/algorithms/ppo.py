"""PPO + ROA (regularised online adaptation) — drop-in for rsl_rl/algorithms/ppo.py:10-349.

Same hyper-parameters, losses, schedules, optimizers and param groups:
  optimizer            Adam([actor, critic, privileged_encoder_, std, scan_encoder]) lr
  adaptation_optimizer Adam(adaptation_encoder_) lr
  estimator_optimizer  Adam(estimator) estimator_learning_rate

MI355X execution of the same math (DESIGN.md "Learner"):
  * gradients live in ONE flat fp32 buffer (`FlatGrads`): p.grad are views into it, so
    zero_grad is one memset, grad clipping is one norm over a slice, and the multi-GPU
    all-reduce is one RCCL call per minibatch over [main | estimator | kl] (mean over ranks);
  * the adaptive-KL learning-rate schedule (ppo.py:230-246) runs on the device (fp64
    master, same branches), so a minibatch needs no host round trip;
  * on the GPU, parameters and Adam moments are views into flat buffers with the same
    layout, and each optimizer step is one lgx_adam_step launch over its segment with the
    clip_grad_norm_ coefficient folded in (torch's Adam objects remain the containers:
    param groups, state_dict and load_state_dict in the reference's format);
  * on a HIP device the whole 5x4-minibatch update is captured once as a hipGraph and
    replayed per iteration (world_size 1), or as per-minibatch graphs around the RCCL
    all-reduce (world_size > 1). The first two updates run eagerly (warm-up), and any
    optimizer/model state load drops the graphs.
The estimator step is issued after the main backward instead of before it: the two
losses share no parameters, so the result is identical (the ROA update uses the TRUE
estimated obs, ppo.py:190).
Reference quirk kept: clip_grad_norm_(actor_critic.parameters()) also sees the
adaptation encoder's stale DAgger gradients (never zeroed by `optimizer`), and scales them.
"""
import copy
import os

import torch
import torch.distributed as dist
import torch.optim as optim

from legged_gym_custom_amd.rsl_rl.modules import ActorCritic, hip_mlp
from legged_gym_custom_amd.rsl_rl.modules.support_networks import MlpEstimator
from legged_gym_custom_amd.rsl_rl.storage import RolloutStorage

from .s8_act import S8Act
from .s8_update import S8Minibatch

# the GPU minibatch on the pre-split GEMM core (s8_update.py); "0" selects the autograd path
USE_S8 = os.environ.get("LGX_S8_UPDATE", "1") != "0"
# the rollout's act networks in one launch (s8_act.py); "0" selects the grouped launches
USE_FUSED_ACT = os.environ.get("LGX_FUSED_ACT", "1") != "0"
# under RCCL ("nccl"), "1" captures the per-minibatch gradient all-reduce inside the one update
# graph. Default "0": the phased graphs (per-minibatch replays around host-issued all-reduces),
# the mode the 2-rank tests exercise, until a multi-GPU run has shown the captured collective
# equal to eager (tests/test_gpu_graph_allreduce.py covers it on a 1-rank group only)
GRAPH_ALLREDUCE = os.environ.get("LGX_GRAPH_ALLREDUCE", "0") != "0"
# the DAgger minibatch as one fused launch (lgx_adaptation_train) + one reduce, instead of the
# adaptation encoder's autograd graph
DAGGER_FUSED = os.environ.get("LGX_DAGGER_FUSED", "1") != "0"
# dev knob: LGX_POST_STEP=0 launches the transition row and the episode bookkeeping separately
POST_STEP_FUSED = os.environ.get("LGX_POST_STEP", "1") != "0"
DAGGER_BLOCKS = 512  # lgx_adaptation_train's block budget (two per CU: <= 80 KB of LDS each)


def _distributed():
    return dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1


def allreduce_grads(params):
    """Average the gradients of `params` over ranks with ONE all-reduce (flat bucket)."""
    if not _distributed():
        return
    grads = [p.grad for p in params if p.grad is not None]
    if not grads:
        return
    flat = torch.cat([g.reshape(-1) for g in grads])
    dist.all_reduce(flat)
    flat /= dist.get_world_size()
    off = 0
    for g in grads:
        n = g.numel()
        g.copy_(flat[off:off + n].view_as(g))
        off += n


class FlatGrads:
    """p.grad of every parameter as a view into one contiguous fp32 buffer.

    `segments` = [(name, params | int)]: a parameter list, or a number of plain scalar
    slots (e.g. the KL riding along in the all-reduce). Backward accumulates in place
    into a defined .grad, so the views stay bound as long as nothing sets .grad to None
    (PPO never calls optimizer.zero_grad())."""

    def __init__(self, segments):
        self._segments = segments
        sizes = [(name, (sum(p.numel() for p in ps) if not isinstance(ps, int) else ps)) for name, ps in segments]
        dev = next(ps for _, ps in segments if not isinstance(ps, int))[0].device
        self.buf = torch.zeros(sum(n for _, n in sizes), device=dev)
        self.slices = {}
        self._ptrs = []
        off = 0
        for (name, ps), (_, n) in zip(segments, sizes):
            self.slices[name] = (off, off + n)
            if not isinstance(ps, int):
                o = off
                for p in ps:
                    p.grad = self.buf[o:o + p.numel()].view_as(p)
                    self._ptrs.append((p, p.grad.data_ptr()))
                    o += p.numel()
            off += n

    def segment(self, name):
        a, b = self.slices[name]
        return self.buf[a:b]

    def span(self, first, last):
        return self.buf[self.slices[first][0]:self.slices[last][1]]

    def check(self):
        """True while every p.grad is still the view installed at construction."""
        return all(p.grad is not None and p.grad.data_ptr() == ptr for p, ptr in self._ptrs)

    def rebind(self):
        """Re-install the views (e.g. after copy.deepcopy, which copies p.grad and the
        buffer separately); the buffer keeps its values."""
        off = 0
        self._ptrs = []
        for name, ps in self._segments:
            a, b = self.slices[name]
            if not isinstance(ps, int):
                o = a
                for p in ps:
                    p.grad = self.buf[o:o + p.numel()].view_as(p)
                    self._ptrs.append((p, p.grad.data_ptr()))
                    o += p.numel()
            off = b


def _clip_coef(segs, max_norm):
    """clip_grad_norm_'s coefficient over the concatenation of `segs`
    (torch/nn/utils/clip_grad.py): clamp(max_norm / (||g||_2 + 1e-6), max=1). No host sync."""
    if len(segs) == 1:
        total = torch.linalg.vector_norm(segs[0])
    else:
        total = torch.linalg.vector_norm(torch.stack([torch.linalg.vector_norm(s) for s in segs]))
    return torch.clamp(max_norm / (total + 1e-6), max=1.0)


def _clip_(segs, max_norm):
    """clip_grad_norm_ in place: g *= coef."""
    coef = _clip_coef(segs, max_norm)
    for s in segs:
        s.mul_(coef)
    return coef


def export_adam_state(opt):
    """Optimizer state_dict in the reference's format (plain torch Adam, float lr,
    CPU fp32 `step`), whatever execution flags this build runs Adam with."""
    sd = copy.deepcopy(opt.state_dict())
    for g in sd["param_groups"]:
        if isinstance(g.get("lr"), torch.Tensor):
            g["lr"] = float(g["lr"])
        g["capturable"] = False
        g["fused"] = None
    for st in sd["state"].values():
        if "step" in st:
            st["step"] = torch.tensor(float(st["step"]), dtype=torch.float32)
        for k in ("exp_avg", "exp_avg_sq", "max_exp_avg_sq"):
            if k in st:
                st[k] = st[k].cpu()
    return sd


class PPO:
    actor_critic: ActorCritic
    estimator: MlpEstimator

    def __init__(self, actor_critic, estimator, num_learning_epochs=1, num_mini_batches=1, clip_param=0.2,
                 gamma=0.998, lam=0.95, value_loss_coef=1.0, entropy_coef=0.0, learning_rate=1e-3,
                 estimator_learning_rate=1e-3, max_grad_norm=1.0, use_clipped_value_loss=True, schedule="fixed",
                 desired_kl=0.01, resume=False, device="cpu", use_graphs=None):
        self.device = device
        self.desired_kl = desired_kl
        self.schedule = schedule
        self.learning_rate = learning_rate
        self.estimator_learning_rate = estimator_learning_rate
        # ROA regularisation schedule (ppo.py:41-43)
        self.start_val, self.end_val, self.start_step, self.duration = 0.0, 0.05, 5000, 10000
        if resume:
            self.start_val, self.end_val, self.start_step, self.duration = 0.0, 0.1, 0, 1
        self.actor_critic = actor_critic.to(self.device)
        self.storage = None
        self.act_dst = None  # optional [num_envs, A] device buffer the act head also writes (the env's input)
        # optional (seed, device step counter, global env offset) of the env: the act head then
        # draws the exploration noise per (global env, env step) in the kernel (Philox) instead
        # of torch.randn_like, so env shards on several ranks sample what one GPU would
        self.act_noise = None
        self.estimator = estimator.to(self.device)
        ac = self.actor_critic
        self.on_gpu = str(device).startswith("cuda")
        self.use_graphs = self.on_gpu if use_graphs is None else (use_graphs and self.on_gpu)

        main_groups = [list(ac.actor.parameters()), list(ac.critic.parameters()),
                       list(ac.privileged_encoder_.parameters()), [ac.std], list(ac.scan_encoder.parameters())]
        self._main_params = [p for g in main_groups for p in g]
        self._adapt_params = list(ac.adaptation_encoder_.parameters())
        self._est_params = list(self.estimator.parameters())
        # [main | estimator | kl] is the contiguous all-reduce span; adaptation after it
        self.grads = FlatGrads([("main", self._main_params), ("estimator", self._est_params), ("kl", 1),
                                ("adaptation", self._adapt_params)])

        # learning rate: fp64 master on the device (KL schedule), fp32 copy read by the Adam kernel
        self._lr64 = torch.tensor(float(learning_rate), dtype=torch.float64, device=device)
        self._lr32 = torch.tensor(float(learning_rate), dtype=torch.float32, device=device) if self.on_gpu else None
        self._adapt_lr = float(learning_rate)  # adaptation_optimizer keeps its construction lr (ppo.py:65)
        self.optimizer = optim.Adam([{"params": g} for g in main_groups], lr=learning_rate)
        self.adaptation_optimizer = optim.Adam(self._adapt_params, lr=learning_rate)
        self.estimator_optimizer = optim.Adam(self._est_params, lr=estimator_learning_rate)
        self._segment_of = {"optimizer": "main", "estimator_optimizer": "estimator",
                            "adaptation_optimizer": "adaptation"}
        if self.on_gpu:
            self._flatten_params_and_moments()
        self.transition = RolloutStorage.Transition()
        self.clip_param = clip_param
        self.num_learning_epochs = num_learning_epochs
        self.num_mini_batches = num_mini_batches
        self.value_loss_coef = value_loss_coef
        self.entropy_coef = entropy_coef
        self.gamma = gamma
        self.lam = lam
        self.max_grad_norm = max_grad_norm
        self.use_clipped_value_loss = use_clipped_value_loss
        self.total_updates = 0.0
        # update-step device state (static addresses: captured by the graphs)
        self._reg_coef = torch.zeros((), device=device)
        self._losses = torch.zeros(4, device=device)   # value, surrogate, regularisation, estimator
        self._sums = torch.zeros(4, device=device)
        if self.on_gpu:  # fixed-address loss outputs and tail scratch (read by the captured tail)
            self._head_out = torch.zeros(4, device=device)   # surrogate, value, entropy, kl
            self._aux_out = torch.zeros(2, device=device)    # regularisation, estimator
            self._tail_ws = torch.zeros(2 * 512 + 8, device=device)
            self._tail_counter = torch.zeros(1, dtype=torch.int32, device=device)
            # the backward seeds d loss / d {surrogate, value, entropy, regularisation, estimator}
            # back to back in one buffer: the loss-head backward kernels read them in place
            self._seeds = torch.tensor([1.0, float(value_loss_coef), -float(entropy_coef), 0.0, 1.0], device=device)
            self._g_one, self._g_value, self._g_ent, self._reg_coef, self._g_est = self._seeds.unbind()
        self._perm = None
        self._graphs = None
        self._eager_updates = 0
        # bumped whenever captured state is dropped (invalidate_graphs): the runner's rollout
        # graphs record the act kernel's buffers (S8Act) and drop themselves when it changes
        self.graph_generation = 0
        self.graph_mode = None  # "whole" | "phased" once captured
        self.phased_graphs = None  # None: phased iff world_size > 1 (tests force it on one GPU)
        self.use_s8 = USE_S8 and self.on_gpu
        # reduce the gradients over the process group even at world size 1 (tests of the
        # distributed path's graph capture on one GPU)
        self.allreduce_always = False
        self._s8 = None  # S8Minibatch, built at the first update (static buffers for the graphs)
        self.use_fused_act = USE_FUSED_ACT and self.on_gpu
        self._s8act = None  # S8Act, built at the first (eager) act
        self._dagger_graph = None  # update_dagger's hipGraph (world size 1) or phased graphs (> 1)
        self.dagger_path = None  # "fused" | "autograd" | "cpu": the DAgger update that ran
        self.dagger_graph_mode = None  # "whole" | "phased" once captured
        self._dagger_sum = torch.zeros((), device=device)

    # ------------------------------------------------------------------ flat Adam (HIP)
    def _flatten_params_and_moments(self):
        """Parameters, Adam exp_avg and exp_avg_sq as views into flat buffers with the
        gradient buffer's layout, so one lgx_adam_step per optimizer updates a whole
        segment. The torch Adam objects stay the containers (param groups, state_dict)."""
        g = self.grads
        self.params_buf = torch.zeros_like(g.buf)
        self.exp_avg = torch.zeros_like(g.buf)
        self.exp_avg_sq = torch.zeros_like(g.buf)
        for p in self._main_params + self._est_params + self._adapt_params:
            off = (p.grad.data_ptr() - g.buf.data_ptr()) // 4
            n = p.numel()
            self.params_buf[off:off + n].copy_(p.data.reshape(-1))
            p.data = self.params_buf[off:off + n].view_as(p)
        self._opt_step = {name: torch.zeros((), device=self.device) for name in self._segment_of}
        for name in self._segment_of:
            self._bind_adam_state(name)

    def _range_of(self, p):
        off = (p.data_ptr() - self.params_buf.data_ptr()) // 4
        return off, off + p.numel()

    def _bind_adam_state(self, name):
        opt = getattr(self, name)
        step = self._opt_step[name]
        for grp in opt.param_groups:
            for p in grp["params"]:
                a, b = self._range_of(p)
                opt.state[p] = {"step": step, "exp_avg": self.exp_avg[a:b].view_as(p),
                                "exp_avg_sq": self.exp_avg_sq[a:b].view_as(p)}

    def _adam(self, name, lr, grad_scale=None):
        """torch Adam(fused) arithmetic over this optimizer's whole flat segment."""
        opt = getattr(self, name)
        b1, b2 = opt.param_groups[0]["betas"]
        eps = opt.param_groups[0]["eps"]
        a, b = self.grads.slices[self._segment_of[name]]
        step = self._opt_step[name]
        step.add_(1)
        hip_mlp.adam_step(self.params_buf[a:b], self.grads.buf[a:b], self.exp_avg[a:b], self.exp_avg_sq[a:b], step,
                          lr, b1, b2, eps, grad_scale)

    # ------------------------------------------------------------------ storage / rollout
    def init_storage(self, num_envs, num_transitions_per_env, total_obs_shape, privileged_obs_shape, critic_obs_shape,
                     estimated_obs_shape, scan_obs_shape, action_shape):
        self.storage = RolloutStorage(num_envs, num_transitions_per_env, total_obs_shape, privileged_obs_shape,
                                      critic_obs_shape, estimated_obs_shape, scan_obs_shape, action_shape, self.device)
        self._perm = torch.zeros(num_envs * num_transitions_per_env, dtype=torch.long, device=self.device)
        self._graphs = None

    def test_mode(self):
        self.actor_critic.test()

    def train_mode(self):
        self.actor_critic.train()

    def act(self, obs, privileged_obs, critic_obs, true_estimated_obs, scan_obs, adaptation_mode=False):
        """ppo.py:129-153: the rollout actor sees the ESTIMATOR's output (Q12). The
        observations are stored at act time (RolloutStorage.record_observations): the env
        overwrites its buffers in place during the step that follows.

        Aliasing (GPU rollout with `act_dst` set by the runner): the returned tensor IS the
        env's action input buffer (`env.actions_in`), which the act head writes together with
        this step's storage row, bit-identical to it (tests/test_gpu_rollout.py). It is
        overwritten by the next act(); a caller that keeps actions across steps must clone()
        them. Without `act_dst` (or on the CPU) the storage row / transition tensor is returned."""
        t = self.transition
        ac = self.actor_critic
        if self._gpu_rollout():
            # the estimator, privileged/scan encoders and critic read only observations: one
            # grouped launch per depth (hip_mlp.forward_group), then the actor — or all of them
            # in one launch (s8_act.py), which also writes this step's observation rows and runs
            # the act head; otherwise one HIP kernel samples a = mu + std * eps and writes actions, mu, sigma and the Normal
            # log-prob straight into this step's storage rows (lgx_act_head)
            s, k = self.storage, self.storage.step
            fused = self._fused_act(adaptation_mode)
            if fused is None:
                slots = self.storage.record_observations(obs, privileged_obs, critic_obs, true_estimated_obs,
                                                         scan_obs)
            else:
                if k >= s.num_transitions_per_env:
                    raise AssertionError("Rollout buffer overflow")
                slots = self.storage.observation_slots()
            (t.observations, t.privileged_observations, t.critic_observations, t.true_estimated_observations,
             t.scan_observations) = slots
            with torch.no_grad():
                if fused is not None:
                    # its S8 weights are refreshed at the rollout's first step (the update changed them)
                    if k == 0:
                        fused.refresh_weights()
                    noise = self.act_noise
                    dst = self.act_dst if self.act_dst is not None and self.act_dst.shape == s.actions[k].shape else None
                    head = dict(std=ac.std.detach(), eps=torch.randn_like(s.mu[k]) if noise is None else None,
                                noise=noise, actions=s.actions[k], mu=s.mu[k], sigma=s.sigma[k],
                                logp=s.actions_log_prob[k], actions_copy=dst)
                    _, t.values = fused.run(obs, privileged_obs, critic_obs, scan_obs, est=true_estimated_obs,
                                            rows=slots, head=head, adaptation_mode=adaptation_mode)
                else:
                    items = [self.estimator.group_item(obs), ac.scan_encoder.group_item(scan_obs)]
                    if not adaptation_mode:
                        items.append(ac.privileged_encoder_.group_item(privileged_obs))
                    outs = hip_mlp.forward_group(items)
                    estimated_obs, scan_latent = outs[:2]
                    latent = ac.adaptation_encoder(obs) if adaptation_mode else outs[2]
                    mean, t.values = hip_mlp.forward_group([(ac.actor, (obs, latent, scan_latent, estimated_obs)),
                                                            (ac.critic, critic_obs)])
                if fused is None:
                    noise = self.act_noise
                    eps = torch.randn_like(mean) if noise is None else None
                    dst = self.act_dst if self.act_dst is not None and self.act_dst.shape == mean.shape else None
                    hip_mlp.act_head(mean, ac.std.detach(), eps, s.actions[k], s.mu[k], s.sigma[k],
                                     s.actions_log_prob[k], actions_copy=dst, noise=noise)
            t.actions, t.action_mean, t.action_sigma = s.actions[k], s.mu[k], s.sigma[k]
            t.actions_log_prob = s.actions_log_prob[k].view(-1)
            return t.actions if dst is None else dst
        estimated_obs = self.estimator(obs)
        (t.observations, t.privileged_observations, t.critic_observations, t.true_estimated_observations,
         t.scan_observations) = self.storage.record_observations(obs, privileged_obs, critic_obs, true_estimated_obs,
                                                                 scan_obs)
        t.actions = ac.act(obs, privileged_obs, estimated_obs, scan_obs, adaptation_mode).detach()
        t.values = ac.evaluate(critic_obs).detach()
        t.actions_log_prob = ac.get_actions_log_prob(t.actions).detach()
        t.action_mean = ac.action_mean.detach()
        t.action_sigma = ac.action_std.detach()
        return t.actions

    def _fused_act(self, adaptation_mode):
        """The one-launch act networks (S8Act) for this rollout step (PPO and DAgger iterations),
        or None: shapes it does not cover, or disabled. Built outside graph capture."""
        if not self.use_fused_act:
            return None
        n = self.storage.num_envs
        if self._s8act is not None and self._s8act.B == n:
            return self._s8act
        if torch.cuda.is_current_stream_capturing() or not S8Act.supported(self):
            return None
        self._s8act = S8Act(self, n)
        return self._s8act

    def _gpu_rollout(self):
        return str(self.device).startswith("cuda")

    def post_step_fusable(self):
        """process_env_step takes the runner's episode-tracking arguments (one launch for both)."""
        return self._gpu_rollout() and POST_STEP_FUSED

    def process_env_step(self, rewards, dones, infos, track=None):
        """ppo.py:156-171: time-out bootstrap r += γ V(s) on timed-out envs. track: the runner's
        lgx_track_episodes arguments (GPU), launched with the transition row as one kernel."""
        t = self.transition
        if track is not None and not self._gpu_rollout():
            raise ValueError("process_env_step: fused tracking needs the GPU rollout")
        if self._gpu_rollout():
            # bootstrap + rewards/dones/values rows in one HIP kernel (lgx_store_transition)
            s, k = self.storage, self.storage.step
            if k >= s.num_transitions_per_env:
                raise AssertionError("Rollout buffer overflow")
            to = infos.get("time_outs")
            b = lambda x: x.view(torch.uint8) if x.dtype == torch.bool else x.to(torch.uint8)  # noqa: E731
            hip_mlp.store_transition(rewards.contiguous(), b(dones), None if to is None else b(to),
                                     t.values.reshape(-1), s.rewards[k].view(-1), s.dones[k].view(-1),
                                     s.values[k].view(-1), self.gamma, track=track)
            s.step += 1
            t.clear()
            self.actor_critic.reset(dones)
            return
        t.rewards = rewards.clone()
        t.dones = dones
        if "time_outs" in infos:
            t.rewards += self.gamma * torch.squeeze(t.values * infos["time_outs"].unsqueeze(1).to(self.device), 1)
        self.storage.add_transitions(t)
        t.clear()
        self.actor_critic.reset(dones)

    def compute_returns(self, last_critic_obs):
        last_values = self.actor_critic.evaluate(last_critic_obs).detach()
        self.storage.compute_returns(last_values, self.gamma, self.lam)

    def reg_coef(self):
        stage = min(max((self.total_updates - self.start_step) / self.duration, 0.0), 1.0)
        return self.start_val + stage * (self.end_val - self.start_val)

    # ------------------------------------------------------------------ one minibatch
    def _minibatch_grads(self, idx):
        """Phase A of one minibatch (ppo.py:186-265 minus the optimizer steps): both
        backwards into the flat gradient buffer, the local KL into its slot, losses.
        `idx` is the minibatch's slice of the permutation (GPU: a slice of the storage
        permuted once per update)."""
        ac = self.actor_critic
        g = self.grads
        s = self.storage
        if self.on_gpu and self._s8 is not None:
            # the pre-split GEMM core: forward, loss heads, backward and every gradient of the
            # minibatch as a fixed kernel sequence (s8_update.py); gradients assigned, not added
            adaptive = self.desired_kl is not None and self.schedule == "adaptive"
            mb = self._perm.numel() // self.num_mini_batches
            self._s8.run(idx.start // mb, [None if t is None else t[idx] for t in self._shuf], self._adapt_all[idx],
                         self._head_out, self._aux_out, g.segment("kl") if adaptive else None)
            ac.distribution = None
            return
        if self.on_gpu:
            (obs_b, priv_b, critic_b, est_b, scan_b, actions_b, target_values_b, adv_b, returns_b, old_logp_b,
             old_mu_b, old_sigma_b) = [t[idx] for t in self._shuf]
        else:
            (obs_b, priv_b, critic_b, est_b, scan_b, actions_b, target_values_b, adv_b, returns_b, old_logp_b,
             old_mu_b, old_sigma_b) = s.gather(idx)
        if self.on_gpu:
            # fused loss head: Normal log-prob/entropy, ratio, clipped surrogate, clipped value
            # loss and KL in one HIP kernel each way (hip_mlp.ppo_head); the KL goes straight
            # into its slot of the flat gradient buffer (it rides the all-reduce). The
            # privileged latent is computed once and feeds both the actor and the ROA
            # regulariser (the reference evaluates the same encoder on the same input twice,
            # ppo.py:190,204)
            adaptive = self.desired_kl is not None and self.schedule == "adaptive"
            # the privileged/scan encoders and the estimator read only the minibatch, then the
            # actor (on their latents) and the critic: two autograd nodes, one grouped launch
            # per depth each way (hip_mlp.forward_group)
            # the encoders' last layers write their latents straight into this minibatch's rows
            # of the actor-input buffer [obs | priv latent | scan latent | est]
            ain = self._actor_in[idx]
            nobs, nest = obs_b.shape[1], est_b.shape[1]
            nlat = ain.shape[1] - nobs - nest - self._scan_latent_dim
            priv_latent, scan_latent, pred = hip_mlp.forward_group(
                [(*ac.privileged_encoder_.group_item(priv_b), None, ain[:, nobs:nobs + nlat]),
                 (*ac.scan_encoder.group_item(scan_b), None, ain[:, nobs + nlat:ain.shape[1] - nest]),
                 self.estimator.group_item(obs_b)])
            mu_b, value_b = hip_mlp.forward_group(
                [(ac.actor, (ain[:, :nobs], priv_latent, scan_latent, ain[:, ain.shape[1] - nest:]), ain),  # TRUE est
                 (ac.critic, critic_b)])
            # sg(z_adapt): the adaptation encoder only trains in DAgger iterations, so over a
            # PPO update its latents are fixed — computed once per update (_adapt_all). Both
            # loss heads (PPO terms; ROA regulariser + estimator loss) in one launch each way
            adapt_latent = self._adapt_all[idx]  # (shuffled order, like the rows)
            (surrogate_loss, value_loss, entropy_mean, _kl, regularization_loss,
             estimator_loss) = hip_mlp.loss_heads(
                mu_b, value_b, ac.std, actions_b, old_logp_b, adv_b, target_values_b, returns_b, old_mu_b, old_sigma_b,
                self.clip_param, self.use_clipped_value_loss, priv_latent, adapt_latent, pred, est_b,
                kl_dst=g.segment("kl") if adaptive else None, out=self._head_out, out_aux=self._aux_out)
            # zero_grad of `optimizer` and `estimator_optimizer` (adaptation grads stay), then
            # both backwards (ppo.py:207, :262) as one pass seeded with the loss coefficients
            # (loss = surr + c_v vloss - c_e entropy + c_reg reg; the estimator loss on its own
            # parameters), every weight-gradient reduction in one launch
            g.span("main", "estimator").zero_()
            with hip_mlp.deferred_weight_grads():
                torch.autograd.backward([surrogate_loss, value_loss, entropy_mean, regularization_loss, estimator_loss],
                                        [self._g_one, self._g_value, self._g_ent, self._reg_coef, self._g_est])
            ac.distribution = None
            return
        (surrogate_loss, value_loss, entropy_mean, regularization_loss,
         estimator_loss) = self._losses_torch(obs_b, priv_b, critic_b, est_b, scan_b, actions_b, target_values_b,
                                              adv_b, returns_b, old_logp_b, old_mu_b, old_sigma_b)
        loss = surrogate_loss + self.value_loss_coef * value_loss - self.entropy_coef * entropy_mean + \
            self._reg_coef * regularization_loss
        # zero_grad of `optimizer` and `estimator_optimizer` (adaptation grads stay)
        g.span("main", "estimator").zero_()
        estimator_loss.backward()
        loss.backward()
        with torch.no_grad():
            self._losses.copy_(torch.stack([value_loss, surrogate_loss, regularization_loss, estimator_loss]))
        ac.distribution = None

    def _losses_torch(self, obs_b, priv_b, critic_b, est_b, scan_b, actions_b, target_values_b, adv_b, returns_b,
                      old_logp_b, old_mu_b, old_sigma_b):
        """The reference's loss terms in torch ops (CPU learner): ppo.py:186-260."""
        ac = self.actor_critic
        # the sample drawn by act() in the reference's update is unused: build the distribution only
        ac.update_distribution(obs_b, priv_b, est_b, scan_b, adaptation_mode=False)  # TRUE est obs (Q12)
        logp_b = ac.get_actions_log_prob(actions_b)
        value_b = ac.evaluate(critic_b)
        mu_b, sigma_b, entropy_b = ac.action_mean, ac.action_std, ac.entropy
        priv_latent = ac.privileged_encoder(priv_b)
        with torch.no_grad():
            adapt_latent = ac.adaptation_encoder(obs_b)
        regularization_loss = (priv_latent - adapt_latent).norm(p=2, dim=1).mean()
        pred = self.estimator(obs_b)
        estimator_loss = (pred - est_b).norm(p=2, dim=1).pow(2).mean()
        if self.desired_kl is not None and self.schedule == "adaptive":
            with torch.no_grad():
                kl = torch.sum(torch.log(sigma_b / old_sigma_b + 1.0e-5) +
                               (torch.square(old_sigma_b) + torch.square(old_mu_b - mu_b)) /
                               (2.0 * torch.square(sigma_b)) - 0.5, axis=-1)
                self.grads.segment("kl").copy_(kl.mean().reshape(1))
        ratio = torch.exp(logp_b - torch.squeeze(old_logp_b))
        surrogate = -torch.squeeze(adv_b) * ratio
        surrogate_clipped = -torch.squeeze(adv_b) * torch.clamp(ratio, 1.0 - self.clip_param, 1.0 + self.clip_param)
        surrogate_loss = torch.max(surrogate, surrogate_clipped).mean()
        if self.use_clipped_value_loss:
            value_clipped = target_values_b + (value_b - target_values_b).clamp(-self.clip_param, self.clip_param)
            value_loss = torch.max((value_b - returns_b).pow(2), (value_clipped - returns_b).pow(2)).mean()
        else:
            value_loss = (returns_b - value_b).pow(2).mean()
        return surrogate_loss, value_loss, entropy_b.mean(), regularization_loss, estimator_loss

    def _minibatch_step(self):
        """Phase B: (ranks averaged) clip + estimator step, KL schedule, clip + main step.
        GPU: one lgx_ppo_tail (two launches) for all of it."""
        g = self.grads
        if self.on_gpu:
            adaptive = self.desired_kl is not None and self.schedule == "adaptive"
            o, eo = self.optimizer.param_groups[0], self.estimator_optimizer.param_groups[0]
            hip_mlp.ppo_tail(g.buf, self.params_buf, self.exp_avg, self.exp_avg_sq, g.slices["main"],
                             g.slices["estimator"], g.slices["adaptation"],
                             g.slices["kl"][0] if adaptive else -1, self.max_grad_norm, o["betas"], o["eps"],
                             eo["betas"], eo["eps"], self.estimator_learning_rate,
                             self.desired_kl if adaptive else 0.0, self._lr64, self._lr32,
                             self._opt_step["optimizer"], self._opt_step["estimator_optimizer"],
                             [self._head_out[1], self._head_out[0], self._aux_out[0], self._aux_out[1]], self._sums,
                             self._tail_ws, self._tail_counter,
                             s8=self._s8.tail_table() if self._s8 is not None else None)
            return
        with torch.no_grad():
            _clip_([g.segment("estimator")], self.max_grad_norm)
            self.estimator_optimizer.step()
        if self.desired_kl is not None and self.schedule == "adaptive":
            with torch.no_grad():
                kl_mean = g.segment("kl")[0].double()
                lr = self._lr64
                up = torch.clamp(lr * 1.5, max=1e-2)
                down = torch.clamp(lr / 1.5, min=1e-5)
                lr_new = torch.where(kl_mean > self.desired_kl * 2.0, down,
                                     torch.where((kl_mean < self.desired_kl / 2.0) & (kl_mean > 0.0), up, lr))
                self._lr64.copy_(lr_new)
            for grp in self.optimizer.param_groups:  # host Adam (CPU): the schedule value goes to the param groups
                grp["lr"] = float(self._lr64)
        with torch.no_grad():
            _clip_([g.segment("main"), g.segment("adaptation")], self.max_grad_norm)
            self.optimizer.step()
            self._sums.add_(self._losses)

    def _reducing(self):
        return _distributed() or (self.allreduce_always and dist.is_available() and dist.is_initialized())

    @staticmethod
    def capture_mode():
        """hipGraph capture mode. Under a process group the capture is thread-local: RCCL's
        watchdog thread polls the events of earlier eager collectives while this thread
        captures, which a global-mode capture rejects (hipErrorStreamCaptureUnsupported)."""
        return "thread_local" if dist.is_available() and dist.is_initialized() else "global"

    def _captures_allreduce(self):
        """RCCL collectives can be recorded in a hipGraph (gloo's host-side ones cannot)."""
        return GRAPH_ALLREDUCE and dist.is_initialized() and dist.get_backend() == "nccl"

    def _allreduce_minibatch(self):
        if self._reducing():
            span = self.grads.span("main", "kl")
            dist.all_reduce(span)
            span.div_(dist.get_world_size())
            # the stale adaptation grads are identical on every rank (averaged at DAgger time)

    def _perm_slices(self):
        mb = self._perm.numel() // self.num_mini_batches
        return [self._perm[i * mb:(i + 1) * mb] for i in range(self.num_mini_batches)]

    def _minibatches(self):
        mb = self._perm.numel() // self.num_mini_batches
        if self.on_gpu:  # slices of the once-permuted storage (_precompute)
            return [slice(i * mb, (i + 1) * mb) for i in range(self.num_mini_batches)]
        return [self._perm[i * mb:(i + 1) * mb] for i in range(self.num_mini_batches)]

    def _precompute(self):
        """Per-update constants read by every minibatch (GPU): the storage rows permuted
        once (the permutation is shared by all epochs, rollout_storage.py:142, so minibatch
        i is the same rows every epoch — a contiguous slice here instead of 12 gathers per
        minibatch), and sg(adaptation_encoder(obs)) for all samples (its weights change only
        in update_dagger)."""
        if self.on_gpu and self._s8_plan() is not None:
            with torch.no_grad():
                flat = self.storage._flat()
                self._s8.prepare(self._perm, flat)  # the network inputs, permuted, in S8
                # the loss heads' fields (true est, actions, values, advantages, returns, log-probs,
                # mu, sigma), permuted, fp32
                sel = (3, 5, 6, 7, 8, 9, 10, 11)
                got = hip_mlp.gather_rows([flat[k] for k in sel], self._perm)
                self._shuf = [None] * 12
                for k, t in zip(sel, got):
                    self._shuf[k] = t
                self._adapt_all = hip_mlp.gather_rows([self.actor_critic.adaptation_encoder(flat[0])], self._perm)[0]
            return
        if self.on_gpu:
            with torch.no_grad():
                # the actor input [obs | priv latent | scan latent | est] per row: the gather
                # writes the permuted obs and est rows straight into their columns (the latents
                # follow per minibatch), so obs_b is a column span of it; row pitch padded to
                # 128 B (whole cache lines per row: the strided gather ran 3 % faster than at a
                # 16-B pitch, tools/gather_timing.py). est is also gathered contiguous (loss head)
                flat = self.storage._flat()
                obs_w, est_w = flat[0].shape[1], flat[3].shape[1]
                width = self.actor_critic.actor[0].in_features
                rows = self._perm.numel()
                pitch = (width + 31) // 32 * 32
                buf = getattr(self, "_actor_in_buf", None)
                if buf is None or buf.shape != (rows, pitch) or buf.device != flat[0].device:
                    buf = self._actor_in_buf = torch.empty(rows, pitch, device=flat[0].device, dtype=flat[0].dtype)
                self._actor_in = buf[:, :width]
                dsts = [self._actor_in[:, :obs_w]] + [None] * (len(flat) - 1) + [self._actor_in[:, width - est_w:]]
                shuf = hip_mlp.gather_rows(flat + [flat[3]], self._perm, dsts)  # one launch
                self._shuf = shuf[:-1]
                self._scan_latent_dim = self.actor_critic.scan_encoder.output_dim
                # on the storage's own (contiguous) obs rows, then permuted: rows are
                # independent, and the strided obs span would need a copy for the per-step view
                self._adapt_all = hip_mlp.gather_rows([self.actor_critic.adaptation_encoder(flat[0])], self._perm)[0]

    def _s8_plan(self):
        """The S8 minibatch executor for the current storage shape (built outside graph capture,
        at the first eager update), or None where its layout does not apply (legacy path)."""
        if not self.use_s8:
            return None
        rows = self._perm.numel()
        mb = rows // self.num_mini_batches
        if self._s8 is not None and (self._s8.rows, self._s8.mb) == (rows, mb):
            return self._s8
        self._s8 = None
        if torch.cuda.is_current_stream_capturing() or not S8Minibatch.supported(self, mb):
            return None
        self._s8 = S8Minibatch(self, rows, mb)
        return self._s8

    def _update_body_eager(self):
        self._precompute()
        slices = self._minibatches()
        for _ in range(self.num_learning_epochs):
            for idx in slices:
                self._minibatch_grads(idx)
                self._allreduce_minibatch()
                self._minibatch_step()

    # ------------------------------------------------------------------ graphs
    def _capture(self):
        torch.cuda.synchronize(self.device)
        slices = self._minibatches()
        pool = torch.cuda.graph_pool_handle()
        mode = self.capture_mode()
        reducing = self._reducing()
        phased = (reducing and not self._captures_allreduce()) if self.phased_graphs is None else self.phased_graphs
        if not phased:
            # one graph for the whole update; at world size > 1 under RCCL the per-minibatch
            # all-reduce of [main | estimator | kl] is recorded in it (ppo.py:273-276: the
            # global-norm clip after the reduce)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, pool=pool, capture_error_mode=mode):
                self._precompute()
                for _ in range(self.num_learning_epochs):
                    for idx in slices:
                        self._minibatch_grads(idx)
                        if reducing:
                            self._allreduce_minibatch()
                        self._minibatch_step()
            self._graphs = {"whole": g}
            self.graph_mode = "whole"
        else:
            gp = torch.cuda.CUDAGraph()
            with torch.cuda.graph(gp, pool=pool, capture_error_mode=mode):
                self._precompute()
            ga = []
            for idx in slices:
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g, pool=pool, capture_error_mode=mode):
                    self._minibatch_grads(idx)
                ga.append(g)
            gb = torch.cuda.CUDAGraph()
            with torch.cuda.graph(gb, pool=pool, capture_error_mode=mode):
                self._minibatch_step()
            self._graphs = {"P": gp, "A": ga, "B": gb}
            self.graph_mode = "phased"

    def invalidate_graphs(self):
        """Drop every captured graph and the executors whose argument lists hold parameter /
        gradient addresses (S8Minibatch, S8Act). The runner's rollout graphs replay S8Act's
        buffers: they check `graph_generation` before every replay and re-capture."""
        self._graphs = None
        self._eager_updates = 0
        self.graph_mode = None
        self._s8 = None
        self._s8act = None
        self._dagger_graph = None
        self.graph_generation += 1

    def _run_update(self):
        if not self.use_graphs:
            self._update_body_eager()
            return
        if self._graphs is None:
            # the first update runs eagerly on a side stream (lazy optimizer state, autograd
            # and GEMM workspaces), then the graph is captured right away — capture only
            # records, so the next update is already a replay
            cur = torch.cuda.current_stream(self.device)
            side = torch.cuda.Stream(self.device)
            side.wait_stream(cur)
            with torch.cuda.stream(side):
                self._update_body_eager()
            cur.wait_stream(side)
            self._eager_updates += 1
            snap = [p.detach().clone() for p in self._main_params + self._est_params]
            self._capture()
            for p, v in zip(self._main_params + self._est_params, snap):
                assert torch.equal(p.detach(), v), "graph capture must not execute the update"
            return
        if self.graph_mode == "whole":
            self._graphs["whole"].replay()
        else:
            self._graphs["P"].replay()
            for _ in range(self.num_learning_epochs):
                for ga in self._graphs["A"]:
                    ga.replay()
                    self._allreduce_minibatch()
                    self._graphs["B"].replay()

    # ------------------------------------------------------------------ update
    def update(self):
        """ppo.py:182-293 (num_learning_epochs x num_mini_batches minibatches)."""
        if not self.grads.check():
            self.grads.rebind()
            self.invalidate_graphs()
        regularization_coef = self.reg_coef()
        self._reg_coef.fill_(regularization_coef)
        self._sums.zero_()
        # one permutation shared by all epochs (rollout_storage.py:142, Appendix B Q24)
        self._perm.copy_(self._next_perm(self._perm.numel()))
        self._run_update()
        num_updates = self.num_learning_epochs * self.num_mini_batches
        mv, ms, mr, me, self.learning_rate = torch.cat([(self._sums / num_updates).double(),
                                                        self._lr64.reshape(1)]).tolist()
        for grp in self.optimizer.param_groups:  # the containers show the scheduled lr
            grp["lr"] = self.learning_rate
        self.storage.clear()
        self.increase_update_count()
        self.enforce_max_std(1.0)
        return mv, ms, mr, regularization_coef, me

    def _next_perm(self, n):
        """The epoch-shared minibatch permutation (rollout_storage.py:142)."""
        return torch.randperm(n, device=self.device)

    def increase_update_count(self):
        self.total_updates += 1

    def enforce_max_std(self, max_action_std=1.0):
        """ppo.py:299-303 (std = min(std, max)); in place so captured graphs keep the address."""
        with torch.no_grad():
            self.actor_critic.std.clamp_(max=max_action_std)

    def update_dagger(self):
        """ppo.py:309-349: adaptation-encoder-only imitation of the privileged latent
        (same epoch-shared permutation and minibatch slices as update()).

        GPU: the privileged latents and the observation rows of every sample are formed once per
        update in the epoch-shared permutation (the privileged encoder does not train here, and
        minibatch i is the same rows every epoch), and the 20 minibatches (adaptation encoder
        forward + backward, L2 loss, clip, Adam) are one hipGraph: the first call runs eagerly on
        a side stream and records the graph, later calls replay it. The loss sum stays on the
        device until the one .item() of the return value (ppo.py:347)."""
        if not self.grads.check():
            self.grads.rebind()
            self.invalidate_graphs()
        self._perm.copy_(self._next_perm(self._perm.numel()))
        n = self.num_learning_epochs * self.num_mini_batches
        if not self.on_gpu:
            self.dagger_path = "cpu"
            total = self._dagger_body_cpu()
        elif not self.use_graphs:
            self._dagger_body()
            total = self._dagger_sum
        elif _distributed():
            # world size > 1: phased graphs around the host-issued all-reduce of the adaptation
            # gradient (per minibatch: graph A = forward + backward + the block-row reduce, the
            # all-reduce, graph B = clip + Adam), as update() does with its phased graphs
            self._dagger_phased()
            total = self._dagger_sum
        else:
            if self._dagger_graph is None:
                cur = torch.cuda.current_stream(self.device)
                side = torch.cuda.Stream(self.device)
                side.wait_stream(cur)
                with torch.cuda.stream(side):
                    self._dagger_body()
                cur.wait_stream(side)
                torch.cuda.synchronize(self.device)
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g, pool=torch.cuda.graph_pool_handle(), capture_error_mode=self.capture_mode()):
                    self._dagger_body()
                self._dagger_graph = g
                self.dagger_graph_mode = "whole"
            else:
                self._dagger_graph.replay()
            total = self._dagger_sum
        mean_adaptation_loss = (total / n).item()
        self.storage.clear()
        self.increase_update_count()
        return mean_adaptation_loss

    def _dagger_body(self):
        """The GPU DAgger update's kernels (fixed addresses: captured by the graph)."""
        ac = self.actor_critic
        adapt = self.grads.segment("adaptation")
        s = self.storage
        rows = self._perm.numel()
        mb = rows // self.num_mini_batches
        with torch.no_grad():
            obs = s.observations.flatten(0, 1)
            obs_p, priv_p = hip_mlp.gather_rows([obs, s.privileged_observations.flatten(0, 1)], self._perm)
            priv_lat = ac.privileged_encoder(priv_p)
        self._dagger_sum.zero_()
        if DAGGER_FUSED and self._dagger_fused_ok(adapt):
            self.dagger_path = "fused"
            self._dagger_fused(obs_p, priv_lat, mb, adapt)
            return
        self.dagger_path = "autograd"
        for _ in range(self.num_learning_epochs):
            for i in range(self.num_mini_batches):
                adapt_latent = ac.adaptation_encoder(obs_p[i * mb:(i + 1) * mb])
                adaptation_loss = (priv_lat[i * mb:(i + 1) * mb] - adapt_latent).norm(p=2, dim=1).mean()
                adapt.zero_()
                adaptation_loss.backward()
                if _distributed():
                    dist.all_reduce(adapt)
                    adapt.div_(dist.get_world_size())
                with torch.no_grad():
                    _clip_([adapt], self.max_grad_norm)
                    self._adam("adaptation_optimizer", self._adapt_lr)
                    self._dagger_sum.add_(adaptation_loss.detach())

    def _dagger_fused_ok(self, adapt):
        """lgx_adaptation_train writes the gradient in the flat order of hip_mlp.adaptation_param_order:
        the adaptation segment must hold exactly those parameters' gradients, in that order."""
        ac = self.actor_critic
        mod = ac.adaptation_encoder_
        if not hip_mlp.adaptation_train_supported(mod, ac.num_proprio):
            return False  # outside lgx_adaptation_train's tiling
        why = None
        if adapt.numel() > 65536:
            why = "the adaptation segment exceeds lgx_clip_adam's one-block limit (65536)"
        else:
            off = adapt.data_ptr()
            for p in hip_mlp.adaptation_param_order(mod):
                if p.grad is None or p.grad.data_ptr() != off or not p.grad.is_contiguous():
                    why = "the adaptation gradients are not views of the flat segment in lgx_adaptation_train's order"
                    break
                off += 4 * p.numel()
            if why is None and off != adapt.data_ptr() + 4 * adapt.numel():
                why = "the adaptation segment holds more than the encoder's parameters"
        if why is not None and not getattr(self, "_dagger_warned", False):
            self._dagger_warned = True
            print(f"[ppo] update_dagger: fused path not used ({why}); running the autograd path", flush=True)
        return why is None

    def _dagger_fused(self, obs_p, priv_lat, mb, adapt):
        """The DAgger minibatches with the adaptation encoder's forward, loss and backward in ONE
        launch each (lgx_adaptation_train: per-block gradient rows), the rows summed into the flat
        gradient segment and the loss into the running sum by one reduce launch, then the clip and
        Adam of _dagger_body (ppo.py:336-345) as one lgx_clip_adam launch: 3 launches per minibatch."""
        for _ in range(self.num_learning_epochs):
            for i in range(self.num_mini_batches):
                self._dagger_fused_grads(obs_p, priv_lat, mb, adapt, i)
                if _distributed():
                    dist.all_reduce(adapt)
                    adapt.div_(dist.get_world_size())
                self._clip_adam("adaptation_optimizer", self._adapt_lr)

    def _dagger_fused_grads(self, obs_p, priv_lat, mb, adapt, i):
        """Minibatch i's adaptation gradient (lgx_adaptation_train block rows, one reduce launch
        into the flat segment) and its loss into the running sum."""
        from legged_gym_custom_amd.rsl_rl.modules import hip_s8 as S
        ac = self.actor_critic
        hist_cols = ac.num_proprio * ac.history_buffer_length
        grid = hip_mlp.adapt_train_grid(mb, DAGGER_BLOCKS)
        NP = adapt.numel()
        ws = getattr(self, "_dagger_ws", None)
        if ws is None or ws[0].numel() != grid * NP:
            ws = (torch.empty(grid * NP, device=self.device), torch.empty(grid, device=self.device))
            self._dagger_ws = ws
        gws, lws = ws
        jobs = [S.flat_reduce(gws.data_ptr(), NP, adapt.data_ptr(), NP, grid),
                S.flat_reduce(lws.data_ptr(), 1, self._dagger_sum.data_ptr(), 1, grid, accumulate=1)]
        keep = hip_mlp.adaptation_train(ac.adaptation_encoder_, obs_p[i * mb:(i + 1) * mb], hist_cols,
                                        priv_lat[i * mb:(i + 1) * mb], gws, lws, DAGGER_BLOCKS)
        S.reduce(jobs)
        del keep

    def _dagger_phased(self):
        """update_dagger at world size > 1 (GPU, fused path): graph P (gathers, privileged latents),
        per minibatch graph A_i (the fused forward + backward + reduce), the host-issued all-reduce
        of the 5,040-entry adaptation segment, graph B (mean, clip, Adam). The first call runs the
        body eagerly and captures; the autograd fallback stays eager."""
        adapt = self.grads.segment("adaptation")
        if not (DAGGER_FUSED and self._dagger_fused_ok(adapt)):
            self._dagger_body()
            return
        rows = self._perm.numel()
        mb = rows // self.num_mini_batches
        if self._dagger_graph is None:
            cur = torch.cuda.current_stream(self.device)
            side = torch.cuda.Stream(self.device)
            side.wait_stream(cur)
            with torch.cuda.stream(side):
                self._dagger_body()
            cur.wait_stream(side)
            torch.cuda.synchronize(self.device)
            pool, mode = torch.cuda.graph_pool_handle(), self.capture_mode()
            keep = {}

            def prep():
                ac, s = self.actor_critic, self.storage
                with torch.no_grad():
                    obs = s.observations.flatten(0, 1)
                    keep["obs_p"], priv_p = hip_mlp.gather_rows([obs, s.privileged_observations.flatten(0, 1)],
                                                                self._perm)
                    keep["priv_lat"] = ac.privileged_encoder(priv_p)
                self._dagger_sum.zero_()
            gp = torch.cuda.CUDAGraph()
            with torch.cuda.graph(gp, pool=pool, capture_error_mode=mode):
                prep()
            ga = []
            for i in range(self.num_mini_batches):
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g, pool=pool, capture_error_mode=mode):
                    self._dagger_fused_grads(keep["obs_p"], keep["priv_lat"], mb, adapt, i)
                ga.append(g)
            gb = torch.cuda.CUDAGraph()
            with torch.cuda.graph(gb, pool=pool, capture_error_mode=mode):
                adapt.div_(dist.get_world_size())
                self._clip_adam("adaptation_optimizer", self._adapt_lr)
            self._dagger_graph = {"P": gp, "A": ga, "B": gb, "keep": keep}
            self.dagger_graph_mode = "phased"
            return
        gr = self._dagger_graph
        gr["P"].replay()
        for _ in range(self.num_learning_epochs):
            for g in gr["A"]:
                g.replay()
                dist.all_reduce(adapt)
                gr["B"].replay()

    def _clip_adam(self, name, lr):
        """clip_grad_norm_ of this optimizer's segment (in place) + its Adam step in one launch
        (lgx_clip_adam; the segment is small: the adaptation encoder)."""
        opt = getattr(self, name)
        b1, b2 = opt.param_groups[0]["betas"]
        a, b = self.grads.slices[self._segment_of[name]]
        hip_mlp.clip_adam(self.params_buf[a:b], self.grads.buf[a:b], self.exp_avg[a:b], self.exp_avg_sq[a:b],
                          self._opt_step[name], lr, b1, b2, opt.param_groups[0]["eps"], self.max_grad_norm)

    def _dagger_body_cpu(self):
        """The CPU learner's DAgger update (the reference's statement order, per-minibatch
        gathers)."""
        total = torch.zeros((), device=self.device)
        ac = self.actor_critic
        adapt = self.grads.segment("adaptation")
        for _ in range(self.num_learning_epochs):
            for idx in self._perm_slices():
                obs_b, priv_b = self.storage.gather_fields(idx, ("observations", "privileged_observations"))
                with torch.no_grad():
                    priv_latent = ac.privileged_encoder(priv_b)
                adapt_latent = ac.adaptation_encoder(obs_b)
                adaptation_loss = (priv_latent - adapt_latent).norm(p=2, dim=1).mean()
                adapt.zero_()
                adaptation_loss.backward()
                if _distributed():
                    dist.all_reduce(adapt)
                    adapt.div_(dist.get_world_size())
                with torch.no_grad():
                    _clip_([adapt], self.max_grad_norm)
                self.adaptation_optimizer.step()
                total += adaptation_loss.detach()
        return total

    # ------------------------------------------------------------------ checkpoints
    def optimizer_state_dicts(self):
        """{'optimizer_state_dict', 'estimator_optimizer_state_dict',
        'adaptation_optimizer_state_dict'} in the reference's (plain Adam) format."""
        return {"optimizer_state_dict": export_adam_state(self.optimizer),
                "estimator_optimizer_state_dict": export_adam_state(self.estimator_optimizer),
                "adaptation_optimizer_state_dict": export_adam_state(self.adaptation_optimizer)}

    def load_optimizer_state(self, name, state_dict):
        """Load a (reference-format) Adam state into `name`; on the GPU the moments are
        copied into the flat buffers and the state re-bound to views. Drops graphs."""
        opt = getattr(self, name)
        opt.load_state_dict(state_dict)
        for grp in opt.param_groups:
            grp["lr"] = float(grp["lr"])
            grp["fused"], grp["capturable"] = None, False
        if name == "optimizer":
            lr = float(opt.param_groups[0]["lr"])
            self._lr64.fill_(lr)
            if self._lr32 is not None:
                self._lr32.fill_(lr)
            self.learning_rate = lr
        elif name == "adaptation_optimizer":
            self._adapt_lr = float(opt.param_groups[0]["lr"])
        if self.on_gpu:
            step = None
            with torch.no_grad():
                for grp in opt.param_groups:
                    for p in grp["params"]:
                        st = opt.state.get(p, {})
                        a, b = self._range_of(p)
                        if "exp_avg" in st:
                            self.exp_avg[a:b].copy_(st["exp_avg"].reshape(-1))
                            self.exp_avg_sq[a:b].copy_(st["exp_avg_sq"].reshape(-1))
                            step = float(st["step"])
            self._opt_step[name].fill_(step or 0.0)
            self._bind_adam_state(name)
        self.invalidate_graphs()

    def after_model_load(self):
        self.invalidate_graphs()
