"""`python legged_gym/scripts/play.py --task=go2` — the reference's entry point
(legged_gym/scripts/play.py), running legged_gym_custom_amd.scripts.play."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from legged_gym_custom_amd.scripts.play import main  # noqa: E402

if __name__ == "__main__":
    main()
