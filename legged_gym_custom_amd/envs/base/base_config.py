"""Nested-class configuration base (drop-in for legged_gym/envs/base/base_config.py:33-55).

Instantiating a config instantiates every nested class recursively, so a config object
is a tree of plain attribute holders. Attribute discovery uses dir(), i.e. alphabetical
order — the reward term order depends on it.
"""
import inspect


class BaseConfig:
    def __init__(self) -> None:
        BaseConfig.init_member_classes(self)

    @staticmethod
    def init_member_classes(obj):
        for name in dir(obj):
            if name == "__class__":
                continue
            member = getattr(obj, name)
            if inspect.isclass(member):
                instance = member()
                setattr(obj, name, instance)
                BaseConfig.init_member_classes(instance)
