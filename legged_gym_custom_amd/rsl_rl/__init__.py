"""rsl_rl drop-in (PPO + ROA fork, rsl_rl/rsl_rl/*): same class names, constructor
arguments, state_dict keys and optimizer param groups; PyTorch-ROCm learner."""
