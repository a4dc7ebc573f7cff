"""`legged_gym` — the reference's package path (legged_gym/__init__.py), served by
legged_gym_custom_amd: `legged_gym.envs`, `legged_gym.utils`, `legged_gym.envs.base.
legged_robot_config`, ... are the implementation's own modules (see _alias.py)."""
import os
import sys

_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if _ROOT not in sys.path:
    sys.path.insert(0, _ROOT)

from legged_gym_custom_amd import LEGGED_GYM_ENVS_DIR, LEGGED_GYM_ROOT_DIR  # noqa: E402,F401
from legged_gym_custom_amd import _alias  # noqa: E402

_alias.install("legged_gym", "legged_gym_custom_amd")
