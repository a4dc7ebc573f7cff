#!/usr/bin/env python3
"""Regenerate legged_gym_custom_amd/resources/robots/*.json from the reference URDFs
(only where /root/reference exists; the JSON is committed so the GPU box needs no URDF)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from legged_gym_custom_amd import model  # noqa: E402

REF = "/root/reference/resources/robots"
for name, rel, foot in [("go2", "go2/urdf/go2.urdf", "foot"), ("anymal_c", "anymal_c/urdf/anymal_c.urdf", "FOOT")]:
    path = os.path.join(REF, rel)
    if not os.path.exists(path):
        print("skip", path)
        continue
    m = model.build_from_urdf(path, foot)
    model.save_json(m, name)
    print(name, len(m["body_names"]), "bodies", len(m["dof_names"]), "dofs", len(m["candidates"]), "candidates")
