"""RolloutStorage — drop-in for rsl_rl/storage/rollout_storage.py:7-181.

[T, N, ·] buffers on the learner device; GAE backward scan (rollout_storage.py:110-124);
advantage normalisation by the mean and UNBIASED std (+1e-8) — over all ranks when
torch.distributed is initialised (one all-reduce of {Σa, Σa², n}, fp64).
"""
import torch
import torch.distributed as dist


class RolloutStorage:
    class Transition:
        def __init__(self):
            self.observations = None
            self.privileged_observations = None
            self.critic_observations = None
            self.true_estimated_observations = None
            self.scan_observations = None
            self.actions = None
            self.rewards = None
            self.dones = None
            self.values = None
            self.actions_log_prob = None
            self.action_mean = None
            self.action_sigma = None
            self.hidden_states = None

        def clear(self):
            self.__init__()

    def __init__(self, num_envs, num_transitions_per_env, obs_shape, privileged_obs_shape, critic_obs_shape,
                 estimated_obs_shape, scan_obs_shape, actions_shape, device="cpu"):
        self.device = device
        self.obs_shape = obs_shape
        self.privileged_obs_shape = privileged_obs_shape
        self.critic_obs_shape = critic_obs_shape
        self.estimated_obs_shape = estimated_obs_shape
        self.actions_shape = actions_shape
        T, N = num_transitions_per_env, num_envs
        z = lambda *s: torch.zeros(T, N, *s, device=device)  # noqa: E731
        self.observations = z(*obs_shape)
        self.privileged_observations = z(*privileged_obs_shape)
        self.critic_observations = z(*critic_obs_shape)
        self.true_estimated_observations = z(*estimated_obs_shape)
        self.scan_observations = z(*scan_obs_shape)
        self.rewards = z(1)
        self.actions = z(*actions_shape)
        self.dones = z(1).byte()
        self.actions_log_prob = z(1)
        self.values = z(1)
        self.returns = z(1)
        self.advantages = z(1)
        self.mu = z(*actions_shape)
        self.sigma = z(*actions_shape)
        self.num_transitions_per_env = T
        self.num_envs = N
        self.saved_hidden_states_a = None
        self.saved_hidden_states_c = None
        self.step = 0

    def observation_slots(self):
        """This step's [obs, priv, critic, true est, scan] rows of the storage."""
        s = self.step
        return [self.observations[s], self.privileged_observations[s], self.critic_observations[s],
                self.true_estimated_observations[s], self.scan_observations[s]]

    def record_observations(self, obs, privileged_obs, critic_obs, true_estimated_obs, scan_obs):
        """Copy the observations an action is taken on into this step's rows, at act time.
        The env here writes its observation buffers in place, so by add_transitions time
        (after env.step) they already hold the next observations; the reference keeps the
        pre-step tensors because its env rebinds new ones (legged_robot.py:93-98)."""
        if self.step >= self.num_transitions_per_env:
            raise AssertionError("Rollout buffer overflow")
        dst = self.observation_slots()
        src = [obs, privileged_obs, critic_obs, true_estimated_obs, scan_obs]
        if str(self.device).startswith("cuda"):
            from legged_gym_custom_amd.rsl_rl.modules import hip_mlp
            hip_mlp.copy_batch(dst, [x.contiguous() for x in src])  # one launch for the five rows
        else:
            for d, x in zip(dst, src):
                d.copy_(x)
        return dst

    def add_transitions(self, transition):
        """rollout_storage.py:87-105. Observation fields that already alias this step's rows
        (record_observations) are not copied again."""
        if self.step >= self.num_transitions_per_env:
            raise AssertionError("Rollout buffer overflow")
        s = self.step
        dst = [self.actions[s], self.rewards[s], self.dones[s], self.values[s], self.actions_log_prob[s], self.mu[s],
               self.sigma[s]]
        src = [transition.actions, transition.rewards.view(-1, 1), transition.dones.view(-1, 1).to(self.dones.dtype),
               transition.values, transition.actions_log_prob.view(-1, 1), transition.action_mean,
               transition.action_sigma]
        obs_src = [transition.observations, transition.privileged_observations, transition.critic_observations,
                   transition.true_estimated_observations, transition.scan_observations]
        for d, x in zip(self.observation_slots(), obs_src):
            if x is not None and d.data_ptr() != x.data_ptr():
                dst.append(d)
                src.append(x)
        if str(self.device).startswith("cuda"):
            torch._foreach_copy_(dst, src)  # one multi-tensor call instead of 12 copies
        else:
            for d, x in zip(dst, src):
                d.copy_(x)
        self.step += 1

    def clear(self):
        self.step = 0

    def compute_returns(self, last_values, gamma, lam):
        if str(self.device).startswith("cuda"):
            self._compute_returns_hip(last_values, gamma, lam)
            return
        advantage = 0
        for step in reversed(range(self.num_transitions_per_env)):
            next_values = last_values if step == self.num_transitions_per_env - 1 else self.values[step + 1]
            not_terminal = 1.0 - self.dones[step].float()
            delta = self.rewards[step] + not_terminal * gamma * next_values - self.values[step]
            advantage = delta + not_terminal * gamma * lam * advantage
            self.returns[step] = advantage + self.values[step]
        # in place: the captured update graph reads this buffer's address
        torch.sub(self.returns, self.values, out=self.advantages)
        mean, std = self._global_mean(self.advantages)
        self.advantages.sub_(mean).div_(std + 1e-8)

    def _compute_returns_hip(self, last_values, gamma, lam):
        """The same scan and normalisation as two HIP launches (lgx_gae, lgx_normalize_advantages)
        instead of ~150 small kernels; the moments are all-reduced across ranks in between."""
        from legged_gym_custom_amd.rsl_rl.modules import hip_mlp
        if getattr(self, "_gae_ws", None) is None:
            self._gae_moments = torch.zeros(2, dtype=torch.float64, device=self.device)
            self._gae_ws = torch.empty(2 * ((self.num_envs + 255) // 256), dtype=torch.float64, device=self.device)
            self._gae_counter = torch.zeros(1, dtype=torch.int32, device=self.device)
        m = self._gae_moments
        hip_mlp.gae(self.rewards, self.dones, self.values, last_values.reshape(-1).contiguous(), self.returns,
                    self.advantages, gamma, lam, m, self._gae_ws, self._gae_counter)
        count = float(self.advantages.numel())
        if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
            dist.all_reduce(m)
            count *= dist.get_world_size()
        hip_mlp.normalize_advantages(self.advantages, m, count)

    def _global_mean(self, a):
        """(mean, unbiased std) of `a` over every rank's shard."""
        if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
            return a.mean(), a.std()
        a64 = a.double()
        m = torch.stack([a64.sum(), (a64 * a64).sum(), torch.tensor(float(a.numel()), device=a.device, dtype=torch.float64)])
        dist.all_reduce(m)
        n = m[2]
        mean = m[0] / n
        var = (m[1] - n * mean * mean) / (n - 1)
        return mean.float(), var.clamp(min=0).sqrt().float()

    def get_statistics(self):
        done = self.dones
        done[-1] = 1
        flat_dones = done.permute(1, 0, 2).reshape(-1, 1)
        done_indices = torch.cat((flat_dones.new_tensor([-1], dtype=torch.int64), flat_dones.nonzero(as_tuple=False)[:, 0]))
        trajectory_lengths = done_indices[1:] - done_indices[:-1]
        return trajectory_lengths.float().mean(), self.rewards.mean()

    def _flat(self):
        return [t.flatten(0, 1) for t in (self.observations, self.privileged_observations, self.critic_observations,
                                          self.true_estimated_observations, self.scan_observations, self.actions,
                                          self.values, self.advantages, self.returns, self.actions_log_prob,
                                          self.mu, self.sigma)]

    def gather(self, idx):
        """The minibatch rows `idx` of every flattened [T*N, .] buffer (same tuple order
        as mini_batch_generator's first 12 fields)."""
        return tuple(t[idx] for t in self._flat())

    def gather_fields(self, idx, names):
        """Minibatch rows `idx` of the named [T, N, .] buffers only."""
        return tuple(getattr(self, n).flatten(0, 1)[idx] for n in names)

    def mini_batch_generator(self, num_mini_batches, num_epochs=8):
        batch_size = self.num_envs * self.num_transitions_per_env
        mini_batch_size = batch_size // num_mini_batches
        # one permutation shared by all epochs (rollout_storage.py:142, Appendix B Q24)
        indices = torch.randperm(num_mini_batches * mini_batch_size, requires_grad=False, device=self.device)
        flat = self._flat()
        for _ in range(num_epochs):
            for i in range(num_mini_batches):
                idx = indices[i * mini_batch_size:(i + 1) * mini_batch_size]
                (obs, priv, critic, est, scan, act, val, adv, ret, logp, mu, sigma) = [t[idx] for t in flat]
                yield obs, priv, critic, est, scan, act, val, adv, ret, logp, mu, sigma, (None, None), None
