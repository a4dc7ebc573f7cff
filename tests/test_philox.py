"""The counter RNG every per-env draw uses (oracle/philox.py restatement; the HIP kernels'
philox4x32_10 in csrc/lgx_device.h): Random123 known answers, and the act head's standard
normals (act_noise) as a distribution and as a function of the global env id only."""
import numpy as np

import philox


def test_philox_known_answers():
    kat = [
        ((0, 0, 0, 0), (0, 0), (0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8)),
        ((0xffffffff,) * 4, (0xffffffff, 0xffffffff), (0x408f276d, 0x41c83b0e, 0xa20bc7c6, 0x6d5451fd)),
        ((0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344), (0xa4093822, 0x299f31d0),
         (0xd16cfe09, 0x94fdcceb, 0x5001e420, 0x24126ea1)),
    ]
    for ctr, key, want in kat:
        got = tuple(int(g) for g in philox.philox4x32_10(*[np.uint32(c) for c in ctr], *key))
        assert got == want


def test_act_noise_is_standard_normal():
    z = philox.act_noise(1, np.arange(20000), 5, 12)
    assert abs(z.mean()) < 0.01 and abs(z.std() - 1.0) < 0.01
    # every action column is its own N(0, 1); neighbouring columns (one Box-Muller pair) uncorrelated
    assert np.all(np.abs(z.mean(0)) < 0.03) and np.all(np.abs(z.std(0) - 1.0) < 0.03)
    c = np.corrcoef(z.T)
    assert np.abs(c - np.eye(12)).max() < 0.04
    assert abs(np.mean(np.abs(z) > 1.96) - 0.05) < 0.005


def test_act_noise_depends_on_global_env_and_step_only():
    full = philox.act_noise(3, np.arange(64), 17, 12)
    assert np.array_equal(philox.act_noise(3, np.arange(32, 64), 17, 12), full[32:])
    assert not np.allclose(philox.act_noise(3, np.arange(64), 18, 12), full)
    assert not np.allclose(philox.act_noise(4, np.arange(64), 17, 12), full)
