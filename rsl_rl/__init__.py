"""`rsl_rl` — the reference's learner package path (rsl_rl/rsl_rl), served by
legged_gym_custom_amd.rsl_rl: rsl_rl.runners.OnPolicyRunner, rsl_rl.algorithms.PPO,
rsl_rl.modules.ActorCritic, rsl_rl.storage.RolloutStorage, rsl_rl.env.VecEnv."""
from legged_gym_custom_amd import _alias

_alias.install("rsl_rl", "legged_gym_custom_amd.rsl_rl")
