"""legged_gym_custom_amd — MI355X-native env step + PPO/ROA rollout engine, drop-in for
the `legged_gym` / `rsl_rl` APIs of JustinMLu/legged_gym_custom.

The env step (physics + post-physics) runs as hand-written HIP kernels (liblgx.so, C ABI
in include/lgx.h); the learner is PyTorch-ROCm. `import legged_gym` / `import rsl_rl`
resolve to this package through the thin alias packages at the repository root.
"""
import os

LEGGED_GYM_ROOT_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LEGGED_GYM_ENVS_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "envs")
