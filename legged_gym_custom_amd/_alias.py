"""Module-path aliases for drop-in use: `legged_gym.X` / `rsl_rl.X` resolve to the SAME
module objects as `legged_gym_custom_amd.X` / `legged_gym_custom_amd.rsl_rl.X` (one
task registry, one set of classes), so reference scripts and user code that import the
reference's module paths (legged_gym/scripts/train.py:34-36, envs/__init__.py,
rsl_rl/runners/on_policy_runner.py imports) run on this build unchanged."""
import importlib
import importlib.abc
import importlib.util
import sys


class _AliasFinder(importlib.abc.MetaPathFinder, importlib.abc.Loader):
    def __init__(self, prefix, target):
        self.prefix, self.target = prefix, target

    def _real(self, fullname):
        return self.target + fullname[len(self.prefix):]

    def find_spec(self, fullname, path=None, target=None):
        if not fullname.startswith(self.prefix + "."):
            return None
        real = self._real(fullname)
        try:
            if importlib.util.find_spec(real) is None:
                return None
        except ModuleNotFoundError:
            return None
        return importlib.util.spec_from_loader(fullname, self)

    def create_module(self, spec):
        # hand back the real module: its __name__/__spec__ stay those of the implementation
        return importlib.import_module(self._real(spec.name))

    def exec_module(self, module):
        pass


def install(prefix, target):
    for f in sys.meta_path:
        if isinstance(f, _AliasFinder) and f.prefix == prefix:
            return
    sys.meta_path.insert(0, _AliasFinder(prefix, target))
