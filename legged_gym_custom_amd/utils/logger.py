"""Logger — drop-in for legged_gym/utils/logger.py:36-138: per-step state traces and
per-episode reward sums collected by play.py, printed as average rewards per second and
plotted as a 3x3 panel. Headless boxes get the panel saved as a PNG instead of a window."""
import os
from collections import defaultdict

import numpy as np


class Logger:
    def __init__(self, dt):
        self.state_log = defaultdict(list)
        self.rew_log = defaultdict(list)
        self.dt = dt
        self.num_episodes = 0
        self.plot_process = None

    def log_state(self, key, value):
        self.state_log[key].append(value)

    def log_states(self, dict):
        for key, value in dict.items():
            self.log_state(key, value)

    def log_rewards(self, dict, num_episodes):
        """logger.py:51-55: episode means (per second) x number of finished episodes."""
        for key, value in dict.items():
            if "rew" in key:
                self.rew_log[key].append(float(value) * num_episodes)
        self.num_episodes += num_episodes

    def reset(self):
        self.state_log.clear()
        self.rew_log.clear()

    def plot_states(self, path=None):
        """The reference's 3x3 state panel (logger.py:65-126), written to `path` (default
        ./logger_states.png) — this build runs headless."""
        import matplotlib
        matplotlib.use("Agg")
        import matplotlib.pyplot as plt
        log = self.state_log
        n = len(next(iter(log.values()))) if log else 0
        t = np.arange(n) * self.dt
        fig, axs = plt.subplots(3, 3, figsize=(15, 10))
        panels = [
            (0, 0, [("dof_pos", "measured"), ("dof_pos_target", "target")], "Joint position [rad]"),
            (0, 1, [("dof_vel", "measured"), ("dof_vel_target", "target")], "Joint velocity [rad/s]"),
            (0, 2, [("base_vel_x", "measured"), ("command_x", "commanded")], "Base lin vel x [m/s]"),
            (1, 0, [("base_vel_y", "measured"), ("command_y", "commanded")], "Base lin vel y [m/s]"),
            (1, 1, [("base_vel_yaw", "measured"), ("command_yaw", "commanded")], "Base ang vel yaw [rad/s]"),
            (1, 2, [("base_vel_z", "measured")], "Base lin vel z [m/s]"),
            (2, 0, [("contact_forces_z", None)], "Vertical contact forces [N]"),
            (2, 1, [("dof_torque", "measured")], "Joint torque [Nm]"),
        ]
        for r, c, series, title in panels:
            a = axs[r, c]
            for key, label in series:
                if log.get(key):
                    a.plot(t, np.array(log[key]), label=label)
            a.set(xlabel="time [s]", title=title)
            if any(lbl for _, lbl in series):
                a.legend()
        if log.get("dof_vel") and log.get("dof_torque"):
            axs[2, 2].plot(log["dof_vel"], log["dof_torque"], "x")
            axs[2, 2].set(xlabel="Joint vel [rad/s]", ylabel="Joint Torque [Nm]", title="Torque/velocity curves")
        path = path or os.path.join(os.getcwd(), "logger_states.png")
        fig.savefig(path)
        plt.close(fig)
        return path

    def print_rewards(self):
        print("Average rewards per second:")
        for key, values in self.rew_log.items():
            mean = np.sum(np.array(values)) / self.num_episodes
            print(f" - {key}: {mean}")
        print(f"Total number of episodes: {self.num_episodes}")
