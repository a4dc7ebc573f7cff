"""ActorCritic with privileged/adaptation/scan encoders (rsl_rl/modules/actor_critic.py:10-251).

actor input = [obs ‖ latent(20) ‖ scan latent(32) ‖ estimated(3)], latent from the
privileged encoder, or from the adaptation encoder over the obs history in adaptation
mode; Gaussian policy with a learnable state-independent std.
"""
import torch
import torch.nn as nn
from torch.distributions import Normal

from .support_networks import AdaptationEncoder, PrivilegedEncoder, ScanEncoder, _mlp
from .support_networks import get_activation as _get_activation


class ActorCritic(nn.Module):
    is_recurrent = False

    def __init__(self, num_proprio, num_privileged_obs, num_critic_obs, num_estimated_obs, num_scan_obs, num_actions,
                 history_buffer_length, actor_hidden_dims=[256, 256, 256], critic_hidden_dims=[256, 256, 256],
                 priv_encoder_hidden_dims=[64, 20], scan_encoder_hidden_dims=[128, 64], latent_encoder_output_dim=20,
                 scan_encoder_output_dim=32, activation="elu", init_noise_std=1.0, **kwargs):
        if kwargs:
            print("ActorCritic.__init__ got unexpected arguments, which will be ignored: " + str(list(kwargs.keys())))
        super().__init__()
        self.num_proprio = num_proprio
        self.num_privileged_obs = num_privileged_obs
        self.history_buffer_length = history_buffer_length
        self.num_critic_obs = num_critic_obs
        self.num_estimated_obs = num_estimated_obs
        self.num_scan_obs = num_scan_obs
        self.num_actions = num_actions
        act = get_activation(activation)
        in_a = num_proprio * (1 + history_buffer_length) + latent_encoder_output_dim + scan_encoder_output_dim + \
            num_estimated_obs
        self.actor = _mlp(in_a, actor_hidden_dims, num_actions, act)
        self.critic = _mlp(num_critic_obs, critic_hidden_dims, 1, act)
        self.adaptation_encoder_ = AdaptationEncoder(num_proprio=num_proprio, history_buffer_length=history_buffer_length,
                                                     output_dim=latent_encoder_output_dim, activation="elu")
        self.privileged_encoder_ = PrivilegedEncoder(num_privileged_obs=num_privileged_obs,
                                                     output_dim=latent_encoder_output_dim,
                                                     hidden_dims=priv_encoder_hidden_dims, activation="elu")
        self.scan_encoder = ScanEncoder(num_scan_obs=num_scan_obs, output_dim=scan_encoder_output_dim,
                                        hidden_dims=scan_encoder_hidden_dims, activation="elu")
        self.std = nn.Parameter(init_noise_std * torch.ones(num_actions))
        self.distribution = None
        # the reference ASSIGNS False to Normal.set_default_validate_args (actor_critic.py:135),
        # which leaves argument validation on; nothing to do here (the HIP paths never build a
        # Normal: lgx_act_head / the fused loss heads)

    def reset(self, dones=None):
        pass

    def forward(self):
        raise NotImplementedError

    @property
    def action_mean(self):
        return self.distribution.mean

    @property
    def action_std(self):
        return self.distribution.stddev

    @property
    def entropy(self):
        return self.distribution.entropy().sum(dim=-1)

    def privileged_encoder(self, privileged_obs_buf):
        return self.privileged_encoder_(privileged_obs_buf)

    def adaptation_encoder(self, obs_buf):
        hist = obs_buf[:, :-self.num_proprio]
        return self.adaptation_encoder_(hist.reshape(-1, self.history_buffer_length, self.num_proprio))

    def get_latent(self, obs_buf, privileged_obs_buf, adaptation_mode=False):
        return self.adaptation_encoder(obs_buf) if adaptation_mode else self.privileged_encoder(privileged_obs_buf)

    def _actor_mean(self, obs_buf, privileged_obs_buf, estimated_obs_buf, scan_obs_buf, adaptation_mode):
        latent = self.get_latent(obs_buf, privileged_obs_buf, adaptation_mode)
        scan_latent = self.scan_encoder(scan_obs_buf)
        return self.actor_forward(obs_buf, latent, scan_latent, estimated_obs_buf)

    def actor_forward(self, obs_buf, latent, scan_latent, estimated_obs_buf):
        """actor(cat(obs, latent, scan latent, est)) (actor_critic.py:79); on the HIP device
        the input gradient covers only the latent columns (obs/est carry none)."""
        parts = (obs_buf, latent, scan_latent, estimated_obs_buf)
        fp = getattr(self.actor, "forward_parts", None)
        return fp(parts) if fp is not None else self.actor(torch.cat(parts, dim=-1))

    def update_distribution(self, obs_buf, privileged_obs_buf, estimated_obs_buf, scan_obs_buf, adaptation_mode=False):
        mean = self._actor_mean(obs_buf, privileged_obs_buf, estimated_obs_buf, scan_obs_buf, adaptation_mode)
        self.distribution = Normal(mean, mean * 0.0 + self.std)

    def act(self, obs_buf, privileged_obs_buf, estimated_obs_buf, scan_obs_buf, adaptation_mode=False):
        """actor_critic.py:205-207: a ~ N(mean, std). Drawn as mean + std * eps with
        eps = randn_like(mean) (the same law as Normal.sample(); torch.normal(loc, scale)
        checks scale >= 0 on the host, which a captured hipGraph rollout cannot do)."""
        self.update_distribution(obs_buf, privileged_obs_buf, estimated_obs_buf, scan_obs_buf, adaptation_mode)
        d = self.distribution
        with torch.no_grad():
            return d.loc + d.scale * torch.randn_like(d.loc)

    def act_inference(self, obs_buf, privileged_obs_buf, estimated_obs_buf, scan_obs_buf, adaptation_mode=False):
        return self._actor_mean(obs_buf, privileged_obs_buf, estimated_obs_buf, scan_obs_buf, adaptation_mode)

    def get_actions_log_prob(self, actions):
        return self.distribution.log_prob(actions).sum(dim=-1)

    def evaluate(self, critic_observations, **kwargs):
        return self.critic(critic_observations)


def get_activation(act_name):
    return _get_activation(act_name)
