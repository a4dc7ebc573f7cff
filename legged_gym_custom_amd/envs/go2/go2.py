"""Go2Robot — drop-in for legged_gym/envs/go2/go2.py:34-831.

Go2's post_physics_step (feet states, gait phase, IMU roll/pitch, modular obs/priv/
critic/est/scan buffers, Go2 reward terms, parkour jump flags) is the LGX_TASK_GO2
branch of the fused env-step kernel; this class only selects it and exposes the
Go2-specific index tables (go2.py:40-77) and feet views.
"""
import torch

from legged_gym_custom_amd import _abi
from legged_gym_custom_amd.envs.base.legged_robot import LeggedRobot


def quaternion_to_euler(quat_angle):
    """go2.py:11-31 (xyzw -> roll, pitch, yaw); host helper for user code."""
    x, y, z, w = quat_angle[:, 0], quat_angle[:, 1], quat_angle[:, 2], quat_angle[:, 3]
    roll = torch.atan2(2.0 * (w * x + y * z), 1.0 - 2.0 * (x * x + y * y))
    pitch = torch.asin(torch.clip(2.0 * (w * y - z * x), -1, 1))
    yaw = torch.atan2(2.0 * (w * z + x * y), 1.0 - 2.0 * (y * y + z * z))
    return roll, pitch, yaw


class Go2Robot(LeggedRobot):
    TASK_KIND = _abi.TASK_GO2

    def __init__(self, cfg, sim_params, physics_engine, sim_device, headless):
        super().__init__(cfg, sim_params, physics_engine, sim_device, headless)
        self.debug_viz = True

    def _create_envs(self):
        super()._create_envs()
        names = self.body_names
        t = lambda lst: torch.tensor(lst, dtype=torch.long, device=self.device)  # noqa: E731
        self.hip_indices = t([i for i, s in enumerate(names) if "hip" in s])
        self.thigh_indices = t([i for i, s in enumerate(names) if "thigh" in s])
        self.calf_indices = t([i for i, s in enumerate(names) if "calf" in s])
        legs = ("FL", "FR", "RL", "RR")
        self.hip_joint_indices = t([self.dof_names.index(f"{l}_hip_joint") for l in legs])
        self.thigh_joint_indices = t([self.dof_names.index(f"{l}_thigh_joint") for l in legs])
        self.calf_joint_indices = t([self.dof_names.index(f"{l}_calf_joint") for l in legs])

    @property
    def feet_pos(self):
        return self.rigid_body_states_view[:, self.feet_indices, 0:3]

    @property
    def feet_vel(self):
        return self.rigid_body_states_view[:, self.feet_indices, 7:10]
