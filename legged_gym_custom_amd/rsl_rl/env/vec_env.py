"""VecEnv ABC (rsl_rl/env/vec_env.py:7-38) — documentation of the env surface."""
from abc import ABC, abstractmethod


class VecEnv(ABC):
    num_envs: int
    num_obs: int
    num_proprio: int
    num_privileged_obs: int
    num_critic_obs: int
    history_buffer_length: int
    num_actions: int
    max_episode_length: int

    @abstractmethod
    def step(self, actions):
        pass

    @abstractmethod
    def reset(self, env_ids):
        pass

    @abstractmethod
    def get_observations(self):
        pass

    @abstractmethod
    def get_privileged_observations(self):
        pass
