"""Encoders and estimator (rsl_rl/modules/support_networks.py:9-199). Module attribute
names (scan_encoder, estimator, priv_encoder, fc_encoder, conv_layers, fc_final) are
kept so state_dict keys match reference checkpoints and TorchScript exports."""
import torch.nn as nn

from .hip_mlp import HipMLP


def get_activation(act_name):
    table = {"elu": nn.ELU, "selu": nn.SELU, "relu": nn.ReLU, "crelu": nn.ReLU, "lrelu": nn.LeakyReLU,
             "tanh": nn.Tanh, "sigmoid": nn.Sigmoid}
    if act_name not in table:
        print("invalid activation function!")
        return None
    return table[act_name]()


def _mlp(in_dim, hidden, out_dim, activation):
    """[Linear, act] per hidden layer, last Linear -> out_dim (same layout as the reference);
    a HipMLP, i.e. fused HIP GEMMs on the GPU."""
    layers = [nn.Linear(in_dim, hidden[0]), activation]
    for i in range(len(hidden)):
        if i == len(hidden) - 1:
            layers.append(nn.Linear(hidden[i], out_dim))
        else:
            layers += [nn.Linear(hidden[i], hidden[i + 1]), activation]
    return HipMLP(*layers)


class ScanEncoder(nn.Module):
    def __init__(self, num_scan_obs, output_dim, hidden_dims=[128, 64], activation="elu"):
        super().__init__()
        self.input_dim = num_scan_obs
        self.output_dim = output_dim
        self.scan_encoder = _mlp(num_scan_obs, hidden_dims, output_dim, get_activation(activation))

    def forward(self, scan_obs):
        return self.scan_encoder(scan_obs)

    def group_item(self, scan_obs):
        """(chain, input) of forward() for hip_mlp.forward_group."""
        return self.scan_encoder, scan_obs


class MlpEstimator(nn.Module):
    def __init__(self, num_proprio, history_buffer_length, output_dim, hidden_dims=[128, 64], activation="elu",
                 use_history=True):
        super().__init__()
        self.use_history = use_history
        self.num_proprio = num_proprio
        self.history_buffer_length = history_buffer_length
        self.input_dim = num_proprio * (1 + history_buffer_length) if use_history else num_proprio
        self.output_dim = output_dim
        self.estimator = _mlp(self.input_dim, hidden_dims, output_dim, get_activation(activation))

    def forward(self, obs_with_history):
        if self.use_history:
            return self.estimator(obs_with_history)
        return self.estimator(obs_with_history[:, -self.num_proprio:])

    def group_item(self, obs_with_history):
        """(chain, input) of forward() for hip_mlp.forward_group."""
        return self.estimator, obs_with_history if self.use_history else obs_with_history[:, -self.num_proprio:]


class PrivilegedEncoder(nn.Module):
    def __init__(self, num_privileged_obs, output_dim=20, hidden_dims=[64, 20], activation="elu"):
        super().__init__()
        self.activation = get_activation(activation)
        self.num_privileged = num_privileged_obs
        self.output_dim = output_dim
        self.encoder_hidden_dims = hidden_dims
        self.priv_encoder = _mlp(num_privileged_obs, hidden_dims, output_dim, self.activation)

    def forward(self, privileged_obs):
        return self.priv_encoder(privileged_obs)

    def group_item(self, privileged_obs):
        """(chain, input) of forward() for hip_mlp.forward_group."""
        return self.priv_encoder, privileged_obs


class AdaptationEncoder(nn.Module):
    """Per-step Linear(P->30) + Conv1d(30->20,k4,s2) + Conv1d(20->10,k2) + Linear(30->out).
    As in the reference the flatten size (10 x 3 = 30) assumes a history of 10 (Q17)."""

    def __init__(self, num_proprio, history_buffer_length, output_dim=20, activation="elu"):
        super().__init__()
        self.activation = get_activation(activation)
        self.history_buffer_length = history_buffer_length
        self.num_proprio = num_proprio
        self.output_dim = output_dim
        ch = 10
        self.fc_encoder = nn.Sequential(nn.Linear(num_proprio, 3 * ch), self.activation)
        self.conv_layers = nn.Sequential(
            nn.Conv1d(in_channels=3 * ch, out_channels=2 * ch, kernel_size=4, stride=2), self.activation,
            nn.Conv1d(in_channels=2 * ch, out_channels=ch, kernel_size=2, stride=1), self.activation,
            nn.Flatten())
        self.fc_final = nn.Sequential(nn.Linear(3 * ch, output_dim), self.activation)

    def forward(self, unflattened_obs_history):
        if unflattened_obs_history.device.type == "cuda" and isinstance(self.activation, nn.ELU):
            from .hip_mlp import adaptation_forward  # channels-last conv1d as HIP GEMMs
            return adaptation_forward(self, unflattened_obs_history)
        x = self.fc_encoder(unflattened_obs_history)
        x = self.conv_layers(x.permute(0, 2, 1))
        return self.fc_final(x)


class AdaptationEncoderTS(AdaptationEncoder):
    """The adaptation encoder's plain forward only (TorchScript export, helpers.py:196-200)."""

    def forward(self, unflattened_obs_history):
        x = self.fc_encoder(unflattened_obs_history)
        x = self.conv_layers(x.permute(0, 2, 1))
        return self.fc_final(x)
