from .helpers import class_to_dict, get_load_path, get_args, export_policy_as_jit, set_seed, update_class_from_dict  # noqa: F401
from .task_registry import task_registry  # noqa: F401
from .math import *  # noqa: F401,F403
from .logger import Logger  # noqa: F401
