"""Go2 parkour task config (task `go2_parkour`) — drop-in restatement of
legged_gym/envs/go2/go2_parkour_config.py:4-267: same class/attribute names and values
(checked against the reference's class_to_dict in tests/test_configs.py).

Like the reference, this derives from LeggedRobotCfg (not Go2Cfg): everything not set
here is the base default. Terrain: trimesh parkour curriculum, 12 difficulty rows x 20
columns of 28 m x 10 m gap courses (terrain.py:103-115, 194-243)."""
import numpy as np

from legged_gym_custom_amd.envs.base.legged_robot_config import LeggedRobotCfg, LeggedRobotCfgPPO
from legged_gym_custom_amd.envs.go2.go2_config import _GO2_DEFAULT_ANGLES, _SCAN_X, _SCAN_Y


def _gap_course(x_start, dx, n, heights, lengths):
    xs = list(np.arange(x_start, x_start + n * dx, dx))
    return xs, {"start_platform_length": 3., "start_platform_height": 0., "x_positions": xs,
                "y_positions": [0.0] * n, "obstacle_heights": heights, "obstacle_lengths": lengths,
                "half_valid_width": 5.0, "border_width": 0.50, "border_height": -2.0}


class Go2ParkourCfg(LeggedRobotCfg):
    class env(LeggedRobotCfg.env):
        num_envs = 4096
        num_proprio = 52
        num_scan_obs = 132
        num_estimated_obs = 3
        num_privileged_obs = 4 + 1 + 12 + 12
        history_buffer_length = 10
        num_actions = 12
        num_critic_obs = num_proprio + num_proprio * history_buffer_length + num_privileged_obs + num_estimated_obs + num_scan_obs
        num_observations = num_proprio + num_proprio * history_buffer_length
        period = 0.40                  # bound: front pair in phase, rear pair half a period later
        fr_offset = 0.0
        bl_offset = 0.5
        fl_offset = 0.0
        br_offset = 0.5

    class terrain(LeggedRobotCfg.terrain):
        measured_points_x = list(_SCAN_X)
        measured_points_y = list(_SCAN_Y)
        mesh_type = "trimesh"
        measure_heights = True
        add_roughness_to_selected_terrain = False
        num_rows = 12
        num_cols = 20
        terrain_length = 28.
        terrain_width = 10.
        selected = False
        parkour = True
        curriculum = True
        promote_threshold = 0.60
        demote_threshold = 0.40
        terrain_proportions = [1.0, 0.0]   # [gap courses, hurdle courses]
        max_init_terrain_level = 2
        x_start = 5.0
        dx = 3.5
        n = 7
        gap_heights = [-2.0] * n
        gap_lengths = [0.2, 0.4, 0.6, 0.8, 1.0, 1.1, 1.2]
        obstacle_x_positions, parkour_kwargs = _gap_course(x_start, dx, n, gap_heights, gap_lengths)
        obstacle_y_positions = [0.0] * n

    class domain_rand:
        randomize_friction = True
        friction_range = [0.1, 1.0]
        randomize_base_mass = True
        added_mass_range = [0.0, 3.0]
        randomize_center_of_mass = True
        added_com_range = [-0.15, 0.15]
        randomize_kp_kd = True
        kp_kd_range = [0.8, 1.2]
        push_robots = True
        push_interval_s = 8
        max_push_vel_xy = 0.5

    class init_state(LeggedRobotCfg.init_state):
        pos = [2.0, 0.0, 0.50]         # 2 m into the start platform
        default_joint_angles = dict(_GO2_DEFAULT_ANGLES)

    class control(LeggedRobotCfg.control):
        control_type = "P"
        stiffness = {"joint": 40.}
        damping = {"joint": 1.}
        action_scale = 0.25
        decimation = 4

    class asset(LeggedRobotCfg.asset):
        file = "{LEGGED_GYM_ROOT_DIR}/resources/robots/go2/urdf/go2.urdf"
        name = "go2"
        foot_name = "foot"
        penalize_contacts_on = ["base", "hip", "thigh", "calf", "Head"]
        terminate_after_contacts_on = ["base", "Head"]
        self_collisions = 0

    class commands(LeggedRobotCfg.commands):
        resampling_time = 10.
        zero_command = True
        zero_command_prob = 0.10
        curriculum = False
        max_forward_vel = 1.75
        max_reverse_vel = 0.5
        vel_increment = 0.10
        heading_command = True
        heading_error_gain = 0.5

        class ranges:
            lin_vel_x = [0.75, 1.5]
            lin_vel_y = [0.0, 0.0]
            ang_vel_yaw = [-0.0, 0.0]
            heading = [-0.2, 0.2]

    class normalization(LeggedRobotCfg.normalization):
        clip_observations = 100.
        clip_actions = 3.14

        class obs_scales(LeggedRobotCfg.normalization.obs_scales):
            lin_vel = 2.0
            ang_vel = 0.25
            dof_pos = 1.0
            dof_vel = 0.05
            height_measurements = 5.0

    class noise(LeggedRobotCfg.noise):
        add_noise = True
        noise_level = 1.0

        class noise_scales(LeggedRobotCfg.noise.noise_scales):
            lin_vel = 0.1
            dof_pos = 0.01
            dof_vel = 0.05
            ang_vel = 0.05
            gravity = 0.02
            imu = 0.02
            height_measurements = 0.02

    class rewards(LeggedRobotCfg.rewards):
        only_positive_rewards = True
        soft_dof_pos_limit = 0.9
        base_height_target = 0.27
        pitch_deg_target = 0.0
        roll_deg_target = 0.0
        max_foot_height = 0.08
        percent_time_on_ground = 0.50
        max_contact_force = 75.0

        class scales(LeggedRobotCfg.rewards.scales):
            tracking_lin_vel = 2.25
            tracking_ang_vel = 2.25
            phase_contact_match = 1.0
            phase_foot_lifting = 1.0
            action_rate = -0.1
            lin_vel_z = -1.0
            ang_vel_xy = -0.01
            torques = -0.00001
            dof_acc = -2.5e-7
            delta_torques = -1.0e-7
            collision = -10.0
            orientation = -1.0
            stumble_feet = -1.0
            dof_error = -0.04
            hip_pos = -0.5
            thigh_pos = -0.5
            thigh_symmetry = -0.2
            calf_symmetry = -0.2
            heading_alignment = -4.5
            reverse_penalty = -1.0
            jump_zone_forward_vel = 1.75
            jump_zone_upward_vel = 3.75
            zero_cmd_dof_error = -1.0


class Go2ParkourCfgPPO(LeggedRobotCfgPPO):
    class policy(LeggedRobotCfgPPO.policy):
        actor_hidden_dims = [512, 256, 128]
        critic_hidden_dims = [512, 256, 128]
        init_noise_std = 1.0
        priv_encoder_hidden_dims = [64, 20]
        latent_encoder_output_dim = 20
        scan_encoder_hidden_dims = [128, 64]
        scan_encoder_output_dim = 32
        estimator_hidden_dims = [256, 128]
        use_history = True
        activation = "elu"

    class algorithm(LeggedRobotCfgPPO.algorithm):
        value_loss_coef = 1.0
        use_clipped_value_loss = True
        clip_param = 0.2
        entropy_coef = 0.01
        num_learning_epochs = 5
        num_mini_batches = 4
        estimator_learning_rate = 1e-4
        learning_rate = 2e-4
        schedule = "fixed"
        gamma = 0.99
        lam = 0.95
        desired_kl = 0.01
        max_grad_norm = 1.
        dagger_update_freq = 20

    class runner(LeggedRobotCfgPPO.runner):
        policy_class_name = "ActorCritic"
        algorithm_class_name = "PPO"
        num_steps_per_env = 24
        max_iterations = 5000
        save_interval = 50
        run_name = "parkour_v15_ft"
        experiment_name = "go2_parkour"
        resume = False
        load_run = -1
        checkpoint = -1
        resume_path = None
