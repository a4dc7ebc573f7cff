"""Permissive no-op stand-in for isaacgym.gymapi (fixture generation only)."""
SIM_PHYSX = 1
SIM_FLEX = 0


class _Dummy:
    def __init__(self, *a, **k):
        pass

    def __getattr__(self, name):
        return _Dummy()

    def __call__(self, *a, **k):
        return _Dummy()


def __getattr__(name):
    return _Dummy


class Vec3:
    def __init__(self, x=0.0, y=0.0, z=0.0):
        self.x, self.y, self.z = float(x), float(y), float(z)

    def __add__(self, o):
        return Vec3(self.x + o.x, self.y + o.y, self.z + o.z)


class SimParams:
    def __init__(self):
        self.dt = 0.005
        self.use_gpu_pipeline = False
        self.physx = _Dummy()
