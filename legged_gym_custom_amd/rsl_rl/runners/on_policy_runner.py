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


def reseed_for_rank(seed, rank):
    """torch CPU and device generators keyed by (seed, rank), after the weight broadcast."""
    s = (int(seed) if int(seed) >= 0 else 0) * 1000003 + int(rank)
    torch.manual_seed(s)
    if torch.cuda.is_available():
        torch.cuda.manual_seed_all(s)


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
            # ...but independent draws per rank from here on (policy noise, the episode-length
            # randomisation, minibatch permutations): rank r's envs must not replay rank 0's
            # exploration noise, so the shards behave like one GPU with world x num_envs envs
            reseed_for_rank(int(train_cfg.get("seed", 1)), self.rank)
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
        # the act head writes the actions straight into the env's input buffer as well, so
        # env.step has nothing to copy
        dst = getattr(env, "actions_in", None)
        if torch.is_tensor(dst) and dst.is_cuda and dst.device == torch.device(device) and dst.is_contiguous():
            self.alg.act_dst = dst
            step_dev = getattr(env, "_step_dev", None)
            if torch.is_tensor(step_dev) and step_dev.device == dst.device and hasattr(env, "env_id_offset"):
                # exploration noise per (global env, env step), drawn in the act head
                self.alg.act_noise = (int(env.seed), step_dev, int(env.env_id_offset))
        self.log_dir = log_dir if self.rank == 0 else None
        # per-step episode bookkeeping (on_policy_runner.py:160-170) runs whenever there is a
        # log dir, as in the reference; bench.py also switches it on without one
        self.track_episodes = False
        self.writer = None
        self.tot_timesteps = 0
        self.tot_time = 0
        self.current_learning_iteration = 0
        self.last_perf = {}
        self.use_graphs = str(device).startswith("cuda")
        self._graphs = {}
        self._eager_rollouts = {}  # per adaptation mode
        self._graphs_gen = getattr(self.alg, "graph_generation", 0)
        self._stats = None
        self._obs = None
        _ = self.env.reset()

    # ------------------------------------------------------------------ rollout
    def _track_episodes(self, rewards, dones, infos):
        """Device-side form of on_policy_runner.py:160-170 (no host sync, graph-capturable):
        rewbuffer/lenbuffer are 100-slot rings with the deque's keep-the-last-100 rule,
        and ep_infos are kept as per-step sums of infos['episode']."""
        if not self._track_native(rewards, dones, infos):
            self._track_episodes_torch(self._stats, rewards, dones, infos)

    def _track_episodes_torch(self, st, rewards, dones, infos):
        st["cur_rew"] += rewards
        st["cur_len"] += 1
        d = dones > 0
        k = d.sum()
        rank = torch.cumsum(d.long(), 0) - 1
        keep = d & (rank >= k - 100)
        pos = torch.where(keep, (st["ptr"] + rank) % 100, torch.full_like(rank, 100))  # slot 100 = discard
        st["rew_ring"].scatter_(0, pos, st["cur_rew"])
        st["len_ring"].scatter_(0, pos, st["cur_len"])
        st["ptr"].copy_((st["ptr"] + k) % 100)
        st["n"].copy_(torch.clamp(st["n"] + k, max=100))
        st["cur_rew"].masked_fill_(d, 0.0)
        st["cur_len"].masked_fill_(d, 0.0)
        if "episode" in infos:
            ep = infos["episode"]
            if st["ep_keys"] is None:
                st["ep_keys"] = list(ep.keys())
                with torch.inference_mode(False):  # a normal tensor: a later capture updates it in place
                    st["ep_sum"] = torch.zeros(len(st["ep_keys"]), device=self.device)
            st["ep_sum"] += torch.stack([ep[key].reshape(()).to(self.device).float() for key in st["ep_keys"]])
            st["ep_cnt"] += 1

    def _track_native(self, rewards, dones, infos, launch=True):
        """One lgx_track_episodes launch for the whole bookkeeping when the buffers allow it
        (HIP device, fp32 rewards, bool/uint8 dones, infos['episode'] values laid out as at most
        two contiguous fp32 runs, e.g. the env's episode means and its terrain-level mean).
        launch=False: its arguments (the post-step launch's), or False."""
        st = self._stats
        if not (rewards.is_cuda and rewards.dtype == torch.float32 and dones.dtype in (torch.bool, torch.uint8)
                and rewards.is_contiguous() and dones.is_contiguous()):
            return False
        runs = None
        if "episode" in infos:
            ep = infos["episode"]
            if st["ep_keys"] is None:
                st["ep_keys"] = list(ep.keys())
                with torch.inference_mode(False):
                    st["ep_sum"] = torch.zeros(len(st["ep_keys"]), device=self.device)
            runs = st.get("ep_runs")
            if runs is None:
                runs = self._ep_runs([ep[k] for k in st["ep_keys"]])
                st["ep_runs"] = runs
            if runs is False:
                return False
        from legged_gym_custom_amd.rsl_rl.modules import hip_mlp as H
        a, b = (runs + [None, None])[:2] if runs else (None, None)
        args = H.track_episodes(rewards, dones.view(torch.uint8), st, a, b, launch=launch)
        return args if not launch else True

    @staticmethod
    def _ep_runs(vals):
        """Group 0-dim fp32 device tensors into <= 2 runs of consecutive storage (as tensors
        over those runs), or False."""
        runs, cur = [], None
        for v in vals:
            if not (torch.is_tensor(v) and v.is_cuda and v.dtype == torch.float32 and v.numel() == 1):
                return False
            if cur is not None and v.data_ptr() == cur[0].data_ptr() + 4 * cur[1]:
                cur[1] += 1
            else:
                cur = [v, 1]
                runs.append(cur)
        if len(runs) > 2:
            return False
        return [torch.as_strided(t.reshape(-1), (n,), (1,)) for t, n in runs]

    def _rollout_step(self, adaptation_mode, track):
        """One env step of the rollout loop (on_policy_runner.py:147-170)."""
        o = self._obs
        actions = self.alg.act(o[0], o[1], o[2], o[3], o[4], adaptation_mode=adaptation_mode)
        obs, priv, critic, est, scan, rewards, dones, infos = self.env.step(actions)
        new = (obs.to(self.device), priv.to(self.device), critic.to(self.device), est.to(self.device),
               scan.to(self.device))
        for dst, src in zip(o, new):  # the env hands back its own static buffers; keep them
            if dst.data_ptr() != src.data_ptr():
                dst.copy_(src)
        rewards, dones = rewards.to(self.device), dones.to(self.device)
        # the transition row and the episode bookkeeping as one launch where both are native
        targs = None
        if track and getattr(self.alg, "post_step_fusable", lambda: False)():
            targs = self._track_native(rewards, dones, infos, launch=False) or None
        self.alg.process_env_step(rewards, dones, infos, track=targs)
        if track and targs is None:
            self._track_episodes(rewards, dones, infos)

    def _graphable(self, adaptation_mode):
        return (self.use_graphs and self.device.startswith("cuda")
                and hasattr(self.env, "advance_step_counter") and getattr(self.env, "graph_capturable", True))

    @staticmethod
    def _rollout_key(adaptation_mode, track):
        # one graph per (DAgger iteration's adaptation-mode rollout, PPO rollout) x tracking
        return ("rollout", track) if not adaptation_mode else ("rollout", track, "adaptation")

    def _check_generation(self):
        """Drop the rollout graphs when the algorithm has dropped the state they replay
        (PPO.invalidate_graphs frees the act kernel's buffers: a stale replay would read and
        write freed memory)."""
        gen = getattr(self.alg, "graph_generation", 0)
        if gen != self._graphs_gen:
            self._graphs = {}
            self._eager_rollouts = {}
            self._graphs_gen = gen

    def _rollout(self, adaptation_mode, track):
        self._check_generation()
        key = self._rollout_key(adaptation_mode, track)
        if self._graphable(adaptation_mode) and key in self._graphs:
            self._graphs[key].replay()
            self.alg.storage.step = self.num_steps_per_env
            self.env.advance_step_counter(self.num_steps_per_env)
            return
        for _ in range(self.num_steps_per_env):
            self._rollout_step(adaptation_mode, track)
        mode = bool(adaptation_mode)
        self._eager_rollouts[mode] = self._eager_rollouts.get(mode, 0) + 1

    def _capture_rollout(self, track, adaptation_mode=False):
        """Record the 24-step rollout of this mode once (after one eager rollout of it has
        warmed every kernel and the storage is empty). Capture does not execute anything. The
        DAgger iterations' rollout (adaptation mode: the latent from the adaptation encoder over
        the observation history, ppo.py:135-141) gets its own graph."""
        self._check_generation()
        key = self._rollout_key(adaptation_mode, track)
        if (key in self._graphs or not self._graphable(adaptation_mode)
                or self._eager_rollouts.get(bool(adaptation_mode), 0) < 1):
            return
        torch.cuda.synchronize(self.device)
        csc, st0 = self.env.common_step_counter, self.alg.storage.step
        g = torch.cuda.CUDAGraph()
        # no_grad, not inference_mode: capture registers the CUDA generator's graph-safe
        # state, which must stay a normal tensor for the update graph's capture
        with torch.inference_mode(False), torch.no_grad(), \
                torch.cuda.graph(g, capture_error_mode=self.alg.capture_mode()):
            for _ in range(self.num_steps_per_env):
                self._rollout_step(adaptation_mode, track)
        self.env.common_step_counter = csc  # host mirror (capture advanced it, the device did not)
        self.alg.storage.step = st0
        self._graphs[key] = g

    def learn(self, num_learning_iterations, init_at_random_ep_len=False):
        mean_value_loss = mean_surrogate_loss = mean_regularization_loss = 0.0
        mean_adaptation_loss = mean_estimator_loss = reg_coef = 0.0
        if self.log_dir is not None and self.writer is None:
            self.writer = _make_writer(self.log_dir)
        if init_at_random_ep_len:
            self.env.episode_length_buf = self._random_episode_lengths()
        env = self.env
        self._obs = [env.get_observations().to(self.device), env.get_privileged_observations().to(self.device),
                     env.get_critic_observations().to(self.device), env.get_estimated_observations().to(self.device),
                     env.get_scan_observations().to(self.device)]
        self.alg.actor_critic.train()
        track = self.log_dir is not None or self.track_episodes
        if track and self._stats is None:
            z = lambda *sh: torch.zeros(*sh, device=self.device)  # noqa: E731
            self._stats = {"cur_rew": z(env.num_envs), "cur_len": z(env.num_envs), "rew_ring": z(101),
                           "len_ring": z(101), "ptr": torch.zeros((), dtype=torch.long, device=self.device),
                           "n": torch.zeros((), dtype=torch.long, device=self.device), "ep_keys": None,
                           "ep_sum": None, "ep_cnt": z(())}
        tot_iter = self.current_learning_iteration + num_learning_iterations
        on_gpu = self.device.startswith("cuda")
        for it in range(self.current_learning_iteration, tot_iter):
            start = time.time()
            use_adaptation_mode = it % self.dagger_update_freq == 0
            if on_gpu:  # split collection/learning by device events: no host sync in between
                evs = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
                evs[0].record()
            with torch.inference_mode():
                self._rollout(use_adaptation_mode, track)
                if on_gpu:
                    evs[1].record()
                mid = time.time()
                self.alg.compute_returns(self._obs[2])
            if use_adaptation_mode:
                mean_adaptation_loss = self.alg.update_dagger()
            else:
                mean_value_loss, mean_surrogate_loss, mean_regularization_loss, reg_coef, mean_estimator_loss = \
                    self.alg.update()
            if on_gpu:
                evs[2].record()
                torch.cuda.synchronize(self.device)
            stop = time.time()
            if on_gpu:  # wall time of the iteration, split at the rollout's end on the device
                host_lead = max(0.0, stop - start - evs[0].elapsed_time(evs[2]) * 1e-3)
                collection_time = evs[0].elapsed_time(evs[1]) * 1e-3 + host_lead
                learn_time = stop - start - collection_time
            else:
                collection_time, learn_time = mid - start, stop - mid
            self.last_perf = {"collection_time": collection_time, "learn_time": learn_time,
                              "fps": self.num_steps_per_env * env.num_envs / (collection_time + learn_time)}
            self._capture_rollout(track, use_adaptation_mode)
            if self.log_dir is not None:
                rewbuffer, lenbuffer, ep_means = self._host_stats()
                self.log(locals())
                if it % self.save_interval == 0:
                    self.save(os.path.join(self.log_dir, "model_{}.pt".format(it)))
        self.current_learning_iteration += num_learning_iterations
        if self.log_dir is not None:
            self.save(os.path.join(self.log_dir, "model_{}.pt".format(self.current_learning_iteration)))

    def _random_episode_lengths(self):
        """on_policy_runner.py:121-122 (uniform in [0, max_episode_length)). An env shard
        (env_id_offset / num_envs_total) takes its slice of one draw over all global envs from a
        generator keyed by the env seed, so ranks start the episodes one GPU would."""
        env = self.env
        buf = env.episode_length_buf
        total = getattr(env, "num_envs_total", None)
        off = getattr(env, "env_id_offset", None)
        seed = getattr(env, "seed", None)
        if total is None or off is None or seed is None:
            return torch.randint_like(buf, high=int(env.max_episode_length))
        g = torch.Generator().manual_seed(int(seed) & 0x7FFFFFFFFFFFFFFF)
        full = torch.randint(int(env.max_episode_length), (int(total),), generator=g, dtype=buf.dtype)
        return full[int(off):int(off) + env.num_envs].to(buf.device)

    def _host_stats(self):
        """One transfer per iteration: the rings (last <=100 completed episodes, oldest
        first as a deque would iterate) and the mean of each infos['episode'] key over the
        steps since the last log (then reset)."""
        with torch.inference_mode():  # the accumulators are touched inside the rollout's inference mode
            return self._host_stats_impl()

    def _host_stats_impl(self):
        st = self._stats
        n, ptr = int(st["n"]), int(st["ptr"])
        idx = [(ptr - n + i) % 100 for i in range(n)]
        rew = st["rew_ring"][idx].tolist() if n else []
        ln = st["len_ring"][idx].tolist() if n else []
        ep = {}
        cnt = float(st["ep_cnt"])
        if st["ep_keys"] is not None and cnt > 0:
            ep = dict(zip(st["ep_keys"], (st["ep_sum"] / cnt).tolist()))
            st["ep_sum"].zero_()
            st["ep_cnt"].zero_()
        return rew, ln, ep

    def log(self, locs, width=80, pad=35):
        self.tot_timesteps += self.num_steps_per_env * self.env.num_envs
        self.tot_time += locs["collection_time"] + locs["learn_time"]
        iteration_time = locs["collection_time"] + locs["learn_time"]
        ep_string = ""
        for key, value in locs["ep_means"].items():
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
        self._graphs = {}
        self._eager_rollouts = {}
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
