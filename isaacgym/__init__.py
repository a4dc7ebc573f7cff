"""Placeholder for the `import isaacgym` line of reference scripts (legged_gym/scripts/
train.py:34). This build has no Isaac Gym: the simulator is liblgx.so (HIP, include/lgx.h)
behind the same env API. Only `isaacgym.torch_utils` (tensor math helpers user task code
imports) is provided; gymapi / gymutil / gymtorch are not."""
