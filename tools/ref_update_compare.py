#!/usr/bin/env python3
"""Diff two tools/ref_update_probe.py outputs minibatch by minibatch: the worst per-tensor
gradient difference (max|dg| / max|g|), the largest parameter difference at the minibatch's
start, the number of per-sample torch.max decisions (surrogate ppo.py:254, value ppo.py:261)
that differ, and the decisions' margins.

  python tools/ref_update_compare.py a.npz b.npz
"""
import sys

import numpy as np


def main():
    a, b = np.load(sys.argv[1]), np.load(sys.argv[2])
    nmb = len(a["norm_main"])
    names = sorted({k.split(".", 1)[1] for k in a.files if k.startswith("g0.")})
    print(f"{'mb':>3} {'grad worst':>11} {'(tensor)':28s} {'param max':>10} {'surr flips':>10} {'value flips':>11} "
          f"{'norm main a/b':>24}")
    for i in range(nmb):
        worst, wn = 0.0, ""
        for n in names:
            ga, gb = a[f"g{i}.{n}"], b[f"g{i}.{n}"]
            e = float(np.abs(ga - gb).max()) / (float(np.abs(ga).max()) + 1e-30)
            if e > worst:
                worst, wn = e, n
        pmax = max(float(np.abs(a[f"p{i}.{n}"] - b[f"p{i}.{n}"]).max()) for n in names)
        flips = []
        for j in (2 * i, 2 * i + 1):
            ma = np.unpackbits(a[f"mask{j}"])[:a[f"maxa{j}"].size].astype(bool)
            mb = np.unpackbits(b[f"mask{j}"])[:b[f"maxa{j}"].size].astype(bool)
            flips.append(np.flatnonzero(ma != mb))
        print(f"{i:3d} {worst:11.3e} {wn:28s} {pmax:10.3e} {flips[0].size:10d} {flips[1].size:11d} "
              f"{a['norm_main'][i]:12.6f}/{b['norm_main'][i]:.6f}")
        for j, fl in zip((2 * i, 2 * i + 1), flips):
            for s in fl[:4]:
                xa, ya = a[f"maxa{j}"][s], a[f"maxb{j}"][s]
                xb, yb = b[f"maxa{j}"][s], b[f"maxb{j}"][s]
                print(f"      {'surrogate' if j % 2 == 0 else 'value'} sample {s}: a ({xa:.9g}, {ya:.9g}) "
                      f"b ({xb:.9g}, {yb:.9g})")


if __name__ == "__main__":
    main()
