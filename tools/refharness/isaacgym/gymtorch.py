"""Identity stand-in for isaacgym.gymtorch (fixture generation only)."""


def wrap_tensor(t):
    return t


def unwrap_tensor(t):
    return t
