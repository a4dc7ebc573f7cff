"""PPO + ROA (regularised online adaptation) — drop-in for rsl_rl/algorithms/ppo.py:10-349.

Same hyper-parameters, losses, schedules, optimizers and param groups:
  optimizer            Adam([actor, critic, privileged_encoder_, std, scan_encoder]) lr
  adaptation_optimizer Adam(adaptation_encoder_) lr
  estimator_optimizer  Adam(estimator) estimator_learning_rate
MI355X-side changes that keep the math: no per-minibatch host syncs (loss sums stay on
device, one transfer per update instead of 80 .item() calls), and — when
torch.distributed is initialised — one flattened-gradient all-reduce (mean over ranks)
per backward before the global-norm clip.
"""
import torch
import torch.distributed as dist
import torch.nn as nn
import torch.optim as optim

from legged_gym_custom_amd.rsl_rl.modules import ActorCritic
from legged_gym_custom_amd.rsl_rl.modules.support_networks import MlpEstimator
from legged_gym_custom_amd.rsl_rl.storage import RolloutStorage


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


class PPO:
    actor_critic: ActorCritic
    estimator: MlpEstimator

    def __init__(self, actor_critic, estimator, num_learning_epochs=1, num_mini_batches=1, clip_param=0.2,
                 gamma=0.998, lam=0.95, value_loss_coef=1.0, entropy_coef=0.0, learning_rate=1e-3,
                 estimator_learning_rate=1e-3, max_grad_norm=1.0, use_clipped_value_loss=True, schedule="fixed",
                 desired_kl=0.01, resume=False, device="cpu"):
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
        self.estimator = estimator.to(self.device)
        ac = self.actor_critic
        self.optimizer = optim.Adam([
            {"params": ac.actor.parameters()},
            {"params": ac.critic.parameters()},
            {"params": ac.privileged_encoder_.parameters()},
            {"params": ac.std},
            {"params": ac.scan_encoder.parameters()},
        ], lr=self.learning_rate)
        self.adaptation_optimizer = optim.Adam(ac.adaptation_encoder_.parameters(), lr=self.learning_rate)
        self.estimator_optimizer = optim.Adam(self.estimator.parameters(), lr=self.estimator_learning_rate)
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

    def init_storage(self, num_envs, num_transitions_per_env, total_obs_shape, privileged_obs_shape, critic_obs_shape,
                     estimated_obs_shape, scan_obs_shape, action_shape):
        self.storage = RolloutStorage(num_envs, num_transitions_per_env, total_obs_shape, privileged_obs_shape,
                                      critic_obs_shape, estimated_obs_shape, scan_obs_shape, action_shape, self.device)

    def test_mode(self):
        self.actor_critic.test()

    def train_mode(self):
        self.actor_critic.train()

    def act(self, obs, privileged_obs, critic_obs, true_estimated_obs, scan_obs, adaptation_mode=False):
        """ppo.py:129-153: the rollout actor sees the ESTIMATOR's output (Q12)."""
        estimated_obs = self.estimator(obs)
        t = self.transition
        t.actions = self.actor_critic.act(obs, privileged_obs, estimated_obs, scan_obs, adaptation_mode).detach()
        t.values = self.actor_critic.evaluate(critic_obs).detach()
        t.actions_log_prob = self.actor_critic.get_actions_log_prob(t.actions).detach()
        t.action_mean = self.actor_critic.action_mean.detach()
        t.action_sigma = self.actor_critic.action_std.detach()
        t.observations = obs
        t.privileged_observations = privileged_obs
        t.critic_observations = critic_obs
        t.true_estimated_observations = true_estimated_obs
        t.scan_observations = scan_obs
        return t.actions

    def process_env_step(self, rewards, dones, infos):
        """ppo.py:156-171: time-out bootstrap r += γ V(s) on timed-out envs."""
        t = self.transition
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

    def update(self):
        """ppo.py:182-293 (5 epochs x 4 minibatches)."""
        sums = torch.zeros(4, device=self.device)  # value, surrogate, regularisation, estimator
        ac = self.actor_critic
        regularization_coef = self.reg_coef()
        generator = self.storage.mini_batch_generator(self.num_mini_batches, self.num_learning_epochs)
        for (obs_b, priv_b, critic_b, est_b, scan_b, actions_b, target_values_b, adv_b, returns_b, old_logp_b,
             old_mu_b, old_sigma_b, _, _) in generator:
            ac.act(obs_b, priv_b, est_b, scan_b, adaptation_mode=False)  # TRUE estimated obs here (Q12)
            logp_b = ac.get_actions_log_prob(actions_b)
            value_b = ac.evaluate(critic_b)
            mu_b, sigma_b, entropy_b = ac.action_mean, ac.action_std, ac.entropy
            priv_latent = ac.privileged_encoder(priv_b)
            with torch.inference_mode():
                adapt_latent = ac.adaptation_encoder(obs_b)
            regularization_loss = (priv_latent - adapt_latent.detach()).norm(p=2, dim=1).mean()
            # estimator (own optimizer, own clip)
            pred = self.estimator(obs_b)
            estimator_loss = (pred - est_b).norm(p=2, dim=1).pow(2).mean()
            self.estimator_optimizer.zero_grad()
            estimator_loss.backward()
            allreduce_grads(list(self.estimator.parameters()))
            nn.utils.clip_grad_norm_(self.estimator.parameters(), self.max_grad_norm)
            self.estimator_optimizer.step()
            if self.desired_kl is not None and self.schedule == "adaptive":
                with torch.inference_mode():
                    kl = torch.sum(torch.log(sigma_b / old_sigma_b + 1.0e-5) +
                                   (torch.square(old_sigma_b) + torch.square(old_mu_b - mu_b)) /
                                   (2.0 * torch.square(sigma_b)) - 0.5, axis=-1)
                    kl_mean = torch.mean(kl)
                    if _distributed():
                        dist.all_reduce(kl_mean)
                        kl_mean /= dist.get_world_size()
                    kl_mean = kl_mean.item()  # the schedule needs the value on the host
                    if kl_mean > self.desired_kl * 2.0:
                        self.learning_rate = max(1e-5, self.learning_rate / 1.5)
                    elif self.desired_kl / 2.0 > kl_mean > 0.0:
                        self.learning_rate = min(1e-2, self.learning_rate * 1.5)
                    for g in self.optimizer.param_groups:
                        g["lr"] = self.learning_rate
            ratio = torch.exp(logp_b - torch.squeeze(old_logp_b))
            surrogate = -torch.squeeze(adv_b) * ratio
            surrogate_clipped = -torch.squeeze(adv_b) * torch.clamp(ratio, 1.0 - self.clip_param, 1.0 + self.clip_param)
            surrogate_loss = torch.max(surrogate, surrogate_clipped).mean()
            if self.use_clipped_value_loss:
                value_clipped = target_values_b + (value_b - target_values_b).clamp(-self.clip_param, self.clip_param)
                value_loss = torch.max((value_b - returns_b).pow(2), (value_clipped - returns_b).pow(2)).mean()
            else:
                value_loss = (returns_b - value_b).pow(2).mean()
            loss = surrogate_loss + self.value_loss_coef * value_loss - self.entropy_coef * entropy_b.mean() + \
                regularization_coef * regularization_loss
            self.optimizer.zero_grad()
            loss.backward()
            allreduce_grads(list(ac.parameters()))
            nn.utils.clip_grad_norm_(ac.parameters(), self.max_grad_norm)
            self.optimizer.step()
            sums += torch.stack([value_loss.detach(), surrogate_loss.detach(), regularization_loss.detach(),
                                 estimator_loss.detach()])
        num_updates = self.num_learning_epochs * self.num_mini_batches
        mv, ms, mr, me = (sums / num_updates).tolist()
        self.storage.clear()
        self.increase_update_count()
        self.enforce_max_std(1.0)
        return mv, ms, mr, regularization_coef, me

    def increase_update_count(self):
        self.total_updates += 1

    def enforce_max_std(self, max_action_std=1.0):
        cur = self.actor_critic.std.detach()
        self.actor_critic.std.data = torch.min(cur, torch.tensor(max_action_std, device=cur.device, dtype=cur.dtype))

    def update_dagger(self):
        """ppo.py:309-349: adaptation-encoder-only imitation of the privileged latent."""
        total = torch.zeros((), device=self.device)
        ac = self.actor_critic
        generator = self.storage.mini_batch_generator(self.num_mini_batches, self.num_learning_epochs)
        for obs_b, priv_b, critic_b, est_b, scan_b, actions_b, *_ in generator:
            with torch.inference_mode():
                ac.act(obs_b, priv_b, est_b, scan_b, adaptation_mode=True)
                priv_latent = ac.privileged_encoder(priv_b)
            adapt_latent = ac.adaptation_encoder(obs_b)
            adaptation_loss = (priv_latent.detach() - adapt_latent).norm(p=2, dim=1).mean()
            self.adaptation_optimizer.zero_grad()
            adaptation_loss.backward()
            allreduce_grads(list(ac.adaptation_encoder_.parameters()))
            nn.utils.clip_grad_norm_(ac.adaptation_encoder_.parameters(), self.max_grad_norm)
            self.adaptation_optimizer.step()
            total += adaptation_loss.detach()
        mean_adaptation_loss = (total / (self.num_learning_epochs * self.num_mini_batches)).item()
        self.storage.clear()
        self.increase_update_count()
        return mean_adaptation_loss
