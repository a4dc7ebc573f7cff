"""OnPolicyRunner — drop-in for rsl_rl/runners/on_policy_runner.py:16-309.

Same construction (ActorCritic + MlpEstimator + PPO from the train-cfg dict), same
rollout/learn loop, DAgger iterations at it % dagger_update_freq == 0 (incl. 0, Q14),
same timers and `Perf/total_fps = steps*envs/(collection+learn)`, same checkpoint keys
{'model_state_dict','optimizer_state_dict','iter','infos'} (+ 'estimator_state_dict',
additive: the reference's load() ignores unknown keys).

Deliberate fix: policy/algorithm keys the go2 / anymal configs lack
fall back to the reference constructors' own defaults instead of raising KeyError.
Multi-GPU: one process per GPU; rank 0 logs and saves; PPO all-reduces gradients.
"""
import os
import statistics
import time
from collections import deque

import torch
import torch.distributed as dist

from legged_gym_custom_amd.rsl_rl.algorithms import PPO
from legged_gym_custom_amd.rsl_rl.modules import ActorCritic
from legged_gym_custom_amd.rsl_rl.modules.support_networks import MlpEstimator

_POLICY_DEFAULTS = {"priv_encoder_hidden_dims": [64, 20], "scan_encoder_hidden_dims": [128, 64],
                    "estimator_hidden_dims": [128, 64], "use_history": True}
_ALG_DEFAULTS = {"estimator_learning_rate": 1e-3}


class _CsvWriter:
    """Minimal SummaryWriter stand-in when tensorboard is not installed."""

    def __init__(self, log_dir, flush_secs=10):
        os.makedirs(log_dir, exist_ok=True)
        self._f = open(os.path.join(log_dir, "scalars.csv"), "a")

    def add_scalar(self, tag, value, step):
        self._f.write(f"{tag},{step},{float(value)}\n")

    def flush(self):
        self._f.flush()


def _make_writer(log_dir):
    try:
        from torch.utils.tensorboard import SummaryWriter
        return SummaryWriter(log_dir=log_dir, flush_secs=10)
    except Exception:
        return _CsvWriter(log_dir)


class OnPolicyRunner:
    def __init__(self, env, train_cfg, log_dir=None, device="cpu"):
        self.cfg = train_cfg["runner"]
        self.alg_cfg = dict(_ALG_DEFAULTS, **train_cfg["algorithm"])
        self.policy_cfg = dict(_POLICY_DEFAULTS, **train_cfg["policy"])
        self.device = device
        self.env = env
        self.rank = dist.get_rank() if dist.is_available() and dist.is_initialized() else 0
        pc = self.policy_cfg
        actor_critic = ActorCritic(num_proprio=env.num_proprio, num_privileged_obs=env.num_privileged_obs,
                                   num_critic_obs=env.num_critic_obs, num_estimated_obs=env.num_estimated_obs,
                                   num_scan_obs=env.num_scan_obs, num_actions=env.num_actions,
                                   history_buffer_length=env.history_buffer_length,
                                   actor_hidden_dims=pc["actor_hidden_dims"], critic_hidden_dims=pc["critic_hidden_dims"],
                                   priv_encoder_hidden_dims=pc["priv_encoder_hidden_dims"],
                                   scan_encoder_hidden_dims=pc["scan_encoder_hidden_dims"],
                                   latent_encoder_output_dim=pc["latent_encoder_output_dim"],
                                   scan_encoder_output_dim=pc["scan_encoder_output_dim"],
                                   activation=pc["activation"], init_noise_std=pc["init_noise_std"])
        estimator = MlpEstimator(num_proprio=env.num_proprio, history_buffer_length=env.history_buffer_length,
                                 output_dim=env.num_estimated_obs, hidden_dims=pc["estimator_hidden_dims"],
                                 activation=pc["activation"], use_history=pc["use_history"])
        if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
            # identical initial weights on every rank
            for p in list(actor_critic.parameters()) + list(estimator.parameters()):
                p.data = p.data.to(device)
                dist.broadcast(p.data, 0)
        a = self.alg_cfg
        self.alg = PPO(actor_critic=actor_critic, estimator=estimator, num_learning_epochs=a["num_learning_epochs"],
                       num_mini_batches=a["num_mini_batches"], clip_param=a["clip_param"], gamma=a["gamma"],
                       lam=a["lam"], value_loss_coef=a["value_loss_coef"], entropy_coef=a["entropy_coef"],
                       learning_rate=a["learning_rate"], estimator_learning_rate=a["estimator_learning_rate"],
                       max_grad_norm=a["max_grad_norm"], use_clipped_value_loss=a["use_clipped_value_loss"],
                       schedule=a["schedule"], desired_kl=a["desired_kl"], resume=self.cfg["resume"], device=device)
        self.dagger_update_freq = a["dagger_update_freq"]
        self.num_steps_per_env = self.cfg["num_steps_per_env"]
        self.save_interval = self.cfg["save_interval"]
        self.alg.init_storage(num_envs=env.num_envs, num_transitions_per_env=self.num_steps_per_env,
                              total_obs_shape=[env.num_obs], privileged_obs_shape=[env.num_privileged_obs],
                              critic_obs_shape=[env.num_critic_obs], estimated_obs_shape=[env.num_estimated_obs],
                              scan_obs_shape=[env.num_scan_obs], action_shape=[env.num_actions])
        self.log_dir = log_dir if self.rank == 0 else None
        self.writer = None
        self.tot_timesteps = 0
        self.tot_time = 0
        self.current_learning_iteration = 0
        self.last_perf = {}
        _ = self.env.reset()

    def learn(self, num_learning_iterations, init_at_random_ep_len=False):
        mean_value_loss = mean_surrogate_loss = mean_regularization_loss = 0.0
        mean_adaptation_loss = mean_estimator_loss = reg_coef = 0.0
        if self.log_dir is not None and self.writer is None:
            self.writer = _make_writer(self.log_dir)
        if init_at_random_ep_len:
            self.env.episode_length_buf = torch.randint_like(self.env.episode_length_buf,
                                                             high=int(self.env.max_episode_length))
        env = self.env
        obs = env.get_observations().to(self.device)
        privileged_obs = env.get_privileged_observations().to(self.device)
        critic_obs = env.get_critic_observations().to(self.device)
        true_estimated_obs = env.get_estimated_observations().to(self.device)
        scan_obs = env.get_scan_observations().to(self.device)
        self.alg.actor_critic.train()
        ep_infos = []
        rewbuffer, lenbuffer = deque(maxlen=100), deque(maxlen=100)
        cur_reward_sum = torch.zeros(env.num_envs, dtype=torch.float, device=self.device)
        cur_episode_length = torch.zeros(env.num_envs, dtype=torch.float, device=self.device)
        tot_iter = self.current_learning_iteration + num_learning_iterations
        for it in range(self.current_learning_iteration, tot_iter):
            start = time.time()
            use_adaptation_mode = it % self.dagger_update_freq == 0
            with torch.inference_mode():
                for _ in range(self.num_steps_per_env):
                    actions = self.alg.act(obs, privileged_obs, critic_obs, true_estimated_obs, scan_obs,
                                           adaptation_mode=use_adaptation_mode)
                    obs, privileged_obs, critic_obs, true_estimated_obs, scan_obs, rewards, dones, infos = env.step(actions)
                    self.alg.process_env_step(rewards, dones, infos)
                    if self.log_dir is not None:
                        if "episode" in infos:
                            ep_infos.append(infos["episode"])
                        cur_reward_sum += rewards
                        cur_episode_length += 1
                        new_ids = (dones > 0).nonzero(as_tuple=False)
                        rewbuffer.extend(cur_reward_sum[new_ids][:, 0].cpu().numpy().tolist())
                        lenbuffer.extend(cur_episode_length[new_ids][:, 0].cpu().numpy().tolist())
                        cur_reward_sum[new_ids] = 0
                        cur_episode_length[new_ids] = 0
                if self.device.startswith("cuda"):
                    torch.cuda.synchronize(self.device)
                stop = time.time()
                collection_time = stop - start
                start = stop
                self.alg.compute_returns(critic_obs)
            if use_adaptation_mode:
                mean_adaptation_loss = self.alg.update_dagger()
            else:
                mean_value_loss, mean_surrogate_loss, mean_regularization_loss, reg_coef, mean_estimator_loss = \
                    self.alg.update()
            if self.device.startswith("cuda"):
                torch.cuda.synchronize(self.device)
            stop = time.time()
            learn_time = stop - start
            self.last_perf = {"collection_time": collection_time, "learn_time": learn_time,
                              "fps": self.num_steps_per_env * env.num_envs / (collection_time + learn_time)}
            if self.log_dir is not None:
                self.log(locals())
                if it % self.save_interval == 0:
                    self.save(os.path.join(self.log_dir, "model_{}.pt".format(it)))
            ep_infos.clear()
        self.current_learning_iteration += num_learning_iterations
        if self.log_dir is not None:
            self.save(os.path.join(self.log_dir, "model_{}.pt".format(self.current_learning_iteration)))

    def log(self, locs, width=80, pad=35):
        self.tot_timesteps += self.num_steps_per_env * self.env.num_envs
        self.tot_time += locs["collection_time"] + locs["learn_time"]
        iteration_time = locs["collection_time"] + locs["learn_time"]
        ep_string = ""
        if locs["ep_infos"]:
            for key in locs["ep_infos"][0]:
                vals = []
                for ep_info in locs["ep_infos"]:
                    v = ep_info[key]
                    if not isinstance(v, torch.Tensor):
                        v = torch.Tensor([v])
                    vals.append(v.reshape(-1).to(self.device))
                value = torch.mean(torch.cat(vals))
                self.writer.add_scalar("Episode/" + key, value, locs["it"])
                ep_string += f"""{f'Mean episode {key}:':>{pad}} {value:.4f}\n"""
        mean_std = self.alg.actor_critic.std.mean()
        fps = int(self.num_steps_per_env * self.env.num_envs / (locs["collection_time"] + locs["learn_time"]))
        w = self.writer
        w.add_scalar("Loss/value_function", locs["mean_value_loss"], locs["it"])
        w.add_scalar("Loss/surrogate", locs["mean_surrogate_loss"], locs["it"])
        w.add_scalar("Loss/regularization", locs["mean_regularization_loss"], locs["it"])
        w.add_scalar("Loss/regularization coef", locs["reg_coef"], locs["it"])
        w.add_scalar("Loss/adaptation", locs["mean_adaptation_loss"], locs["it"])
        w.add_scalar("Loss/estimator", locs["mean_estimator_loss"], locs["it"])
        w.add_scalar("Loss/learning_rate", self.alg.learning_rate, locs["it"])
        w.add_scalar("Policy/mean_noise_std", mean_std.item(), locs["it"])
        w.add_scalar("Perf/total_fps", fps, locs["it"])
        w.add_scalar("Perf/collection time", locs["collection_time"], locs["it"])
        w.add_scalar("Perf/learning_time", locs["learn_time"], locs["it"])
        if len(locs["rewbuffer"]) > 0:
            w.add_scalar("Train/mean_reward", statistics.mean(locs["rewbuffer"]), locs["it"])
            w.add_scalar("Train/mean_episode_length", statistics.mean(locs["lenbuffer"]), locs["it"])
        title = f" \033[1m Learning iteration {locs['it']}/{self.current_learning_iteration + locs['num_learning_iterations']} \033[0m "
        s = (f"{'#' * width}\n{title.center(width, ' ')}\n\n"
             f"{'Computation:':>{pad}} {fps:.0f} steps/s (collection: {locs['collection_time']:.3f}s, "
             f"learning {locs['learn_time']:.3f}s)\n"
             f"{'Value function loss:':>{pad}} {locs['mean_value_loss']:.4f}\n"
             f"{'Surrogate loss:':>{pad}} {locs['mean_surrogate_loss']:.4f}\n"
             f"{'Adaptation loss:':>{pad}} {locs['mean_adaptation_loss']:.4f}\n"
             f"{'Regularization loss:':>{pad}} {locs['mean_regularization_loss']:.4f}\n"
             f"{'Regularization coef:':>{pad}} {locs['reg_coef']:.4f}\n"
             f"{'Estimator loss:':>{pad}} {locs['mean_estimator_loss']:.4f}\n"
             f"{'Mean action noise std:':>{pad}} {mean_std.item():.2f}\n")
        if len(locs["rewbuffer"]) > 0:
            s += (f"{'Mean reward:':>{pad}} {statistics.mean(locs['rewbuffer']):.2f}\n"
                  f"{'Mean episode length:':>{pad}} {statistics.mean(locs['lenbuffer']):.2f}\n")
        s += ep_string
        s += (f"{'-' * width}\n{'Total timesteps:':>{pad}} {self.tot_timesteps}\n"
              f"{'Iteration time:':>{pad}} {iteration_time:.2f}s\n{'Total time:':>{pad}} {self.tot_time:.2f}s\n"
              f"{'ETA:':>{pad}} {self.tot_time / (locs['it'] + 1) * (locs['num_learning_iterations'] - locs['it']):.1f}s\n")
        print(s)

    def save(self, path, infos=None):
        opt = self.alg.optimizer_state_dicts()
        torch.save({"model_state_dict": self.alg.actor_critic.state_dict(),
                    "optimizer_state_dict": opt["optimizer_state_dict"],
                    "iter": self.current_learning_iteration, "infos": infos,
                    "estimator_state_dict": self.alg.estimator.state_dict(),
                    "estimator_optimizer_state_dict": opt["estimator_optimizer_state_dict"],
                    "adaptation_optimizer_state_dict": opt["adaptation_optimizer_state_dict"]}, path)

    def load(self, path, load_optimizer=True):
        loaded = torch.load(path, map_location=self.device, weights_only=True)
        self.alg.actor_critic.load_state_dict(loaded["model_state_dict"])
        if load_optimizer:
            self.alg.load_optimizer_state("optimizer", loaded["optimizer_state_dict"])
        if "estimator_state_dict" in loaded:
            self.alg.estimator.load_state_dict(loaded["estimator_state_dict"])
            if load_optimizer and "estimator_optimizer_state_dict" in loaded:
                self.alg.load_optimizer_state("estimator_optimizer", loaded["estimator_optimizer_state_dict"])
                self.alg.load_optimizer_state("adaptation_optimizer", loaded["adaptation_optimizer_state_dict"])
        self.alg.after_model_load()
        self.current_learning_iteration = loaded["iter"]
        return loaded["infos"]

    def get_inference_policy(self, device=None, stochastic=False):
        self.alg.actor_critic.eval()
        if device is not None:
            self.alg.actor_critic.to(device)
        return self.alg.actor_critic.act if stochastic else self.alg.actor_critic.act_inference
