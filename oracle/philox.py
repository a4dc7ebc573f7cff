"""Philox4x32-10 counter RNG, numpy restatement (TEST INFRASTRUCTURE ONLY).

This is the one RNG definition shared by:
  * the HIP env kernel   (legged_gym_custom_amd/csrc/lgx_rng.h, device code),
  * the C oracle         (oracle/lgx_oracle.c, philox4x32_10),
  * the golden-vector generator (tools/gen_golden.py), which routes every random
    draw of the reference's tensor code (torch_rand_float / torch.rand /
    torch.rand_like at legged_robot.py:491,520,526,539 and go2.py:428-456,519)
    through the same per-env uniform table ("masked-RNG mode").

Counter layout (one 128-bit counter per (env, step, block)):
    c0 = global env id, c1 = step counter (low 32 bits),
    c2 = block | (stream << 16), c3 = step counter (high 32 bits)
Key = (seed_lo, seed_hi). Uniform = (x >> 8) * 2**-24 in [0, 1).
"""
import numpy as np

M0 = np.uint64(0xD2511F53)
M1 = np.uint64(0xCD9E8D57)
W0 = np.uint32(0x9E3779B9)
W1 = np.uint32(0xBB67AE85)
MASK32 = np.uint64(0xFFFFFFFF)

# ---- slot layout: must match lgx_rng.h / lgx_oracle.c --------------------------
SLOT_CMD = 0          # block 0: cmd x, cmd y, cmd yaw/heading, zero-mask   (step callback)
SLOT_PUSH = 4         # block 1: push vx, push vy, terrain level, (unused)
SLOT_TERR = 6         # block 1, 3rd: solved-terrain random level (legged_robot.py:571-573)
SLOT_DOF = 8          # blocks 2-4: 12 dof reset draws
SLOT_ROOT_XY = 20     # block 5: root x, root y
SLOT_ROOT_VEL = 24    # blocks 6-7: 6 root velocity draws
SLOT_RCMD = 32        # block 8: cmd resample inside reset_idx
SLOT_NOISE = 36       # blocks 9-21: 52 observation-noise draws
NUM_BLOCKS = 22       # Go2 (52 noise draws); see num_blocks
NUM_SLOTS = NUM_BLOCKS * 4


def num_blocks(num_proprio):
    """Blocks per env per step: 9 fixed + one per 4 noise draws (ANYmal 235 -> 68)."""
    return SLOT_NOISE // 4 + (num_proprio + 3) // 4

STREAM_STEP = 0       # draws inside env.step()
STREAM_RESET = 1      # draws inside an external reset_idx() call (BaseTask.reset)
STREAM_ACT = 2        # the PPO act head's exploration noise (lgx_mlp.h LGX_ACT_NOISE_STREAM)


def philox4x32_10(c0, c1, c2, c3, k0, k1):
    """Vectorised Philox4x32-10 over uint32 arrays. Returns 4 uint32 arrays."""
    c0 = np.asarray(c0, dtype=np.uint32)
    c1 = np.asarray(c1, dtype=np.uint32)
    c2 = np.asarray(c2, dtype=np.uint32)
    c3 = np.asarray(c3, dtype=np.uint32)
    k0 = np.uint32(k0)
    k1 = np.uint32(k1)
    c0, c1, c2, c3 = np.broadcast_arrays(c0, c1, c2, c3)
    c0 = c0.copy(); c1 = c1.copy(); c2 = c2.copy(); c3 = c3.copy()
    with np.errstate(over="ignore"):
        for r in range(10):
            p0 = M0 * c0.astype(np.uint64)
            p1 = M1 * c2.astype(np.uint64)
            hi0 = (p0 >> np.uint64(32)).astype(np.uint32)
            lo0 = (p0 & MASK32).astype(np.uint32)
            hi1 = (p1 >> np.uint64(32)).astype(np.uint32)
            lo1 = (p1 & MASK32).astype(np.uint32)
            n0 = hi1 ^ c1 ^ k0
            n2 = hi0 ^ c3 ^ k1
            c0, c1, c2, c3 = n0, lo1, n2, lo0
            k0 = np.uint32(k0 + W0)
            k1 = np.uint32(k1 + W1)
    return c0, c1, c2, c3


def to_uniform(x):
    return (np.asarray(x, dtype=np.uint32) >> np.uint32(8)).astype(np.float32) * np.float32(1.0 / 16777216.0)


def uniform_table(seed, env_ids, step, stream=STREAM_STEP, num_blocks=NUM_BLOCKS):
    """[len(env_ids), num_blocks*4] float32 uniforms for one step."""
    env_ids = np.asarray(env_ids, dtype=np.uint32)
    seed = int(seed)
    k0 = seed & 0xFFFFFFFF
    k1 = (seed >> 32) & 0xFFFFFFFF
    step = int(step)
    s_lo = np.uint32(step & 0xFFFFFFFF)
    s_hi = np.uint32((step >> 32) & 0xFFFFFFFF)
    out = np.empty((env_ids.shape[0], num_blocks * 4), dtype=np.float32)
    for b in range(num_blocks):
        x0, x1, x2, x3 = philox4x32_10(env_ids, s_lo, np.uint32(b | (stream << 16)), s_hi, k0, k1)
        out[:, 4 * b + 0] = to_uniform(x0)
        out[:, 4 * b + 1] = to_uniform(x1)
        out[:, 4 * b + 2] = to_uniform(x2)
        out[:, 4 * b + 3] = to_uniform(x3)
    return out


def act_noise(seed, env_ids, step, num_actions):
    """[len(env_ids), num_actions] standard normals the act head draws when it is given no
    eps (lgx_mlp.hip act_noise): block j // 4 of stream STREAM_ACT, Box-Muller on uniforms
    (u[p], u[p + 1]), p = j & 2, with u1 = 1 - u[p]; cos for even j, sin for odd j (float64 here)."""
    u = uniform_table(seed, env_ids, step, STREAM_ACT, (num_actions + 3) // 4).astype(np.float64)
    out = np.empty((u.shape[0], num_actions))
    for j in range(num_actions):
        b, p = j >> 2, j & 2
        r = np.sqrt(-2.0 * np.log(1.0 - u[:, 4 * b + p]))
        th = 2.0 * np.pi * u[:, 4 * b + p + 1]
        out[:, j] = r * (np.sin(th) if j & 1 else np.cos(th))
    return out


if __name__ == "__main__":
    # Random123 known-answer test vectors for philox4x32_10
    kat = [
        ((0, 0, 0, 0), (0, 0), (0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8)),
        ((0xffffffff,) * 4, (0xffffffff, 0xffffffff), (0x408f276d, 0x41c83b0e, 0xa20bc7c6, 0x6d5451fd)),
        ((0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344), (0xa4093822, 0x299f31d0),
         (0xd16cfe09, 0x94fdcceb, 0x5001e420, 0x24126ea1)),
    ]
    for ctr, key, want in kat:
        got = philox4x32_10(*[np.uint32(c) for c in ctr], *key)
        got = tuple(int(g) for g in got)
        assert got == want, (hex(got[0]), want)
    print("philox KAT ok")
