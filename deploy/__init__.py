"""`deploy` — the reference's deploy package path (deploy/base/*), served by
legged_gym_custom_amd.deploy (see legged_gym_custom_amd/_alias.py)."""
import os
import sys

_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if _ROOT not in sys.path:
    sys.path.insert(0, _ROOT)

from legged_gym_custom_amd import _alias  # noqa: E402

_alias.install("deploy", "legged_gym_custom_amd.deploy")
