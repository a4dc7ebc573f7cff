"""`python legged_gym/scripts/train.py --task=go2` — the reference's entry point
(legged_gym/scripts/train.py), running legged_gym_custom_amd.scripts.train."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from legged_gym_custom_amd.scripts.train import main  # noqa: E402

if __name__ == "__main__":
    main()
