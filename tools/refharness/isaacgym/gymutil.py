"""No-op stand-in for isaacgym.gymutil (fixture generation only)."""


def parse_device_str(s):
    if s.startswith("cuda"):
        return "cuda", int(s.split(":")[1]) if ":" in s else 0
    return "cpu", 0


def parse_sim_config(cfg, sim_params):
    pass
