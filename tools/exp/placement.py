"""Which blocks of a 512-block launch (64 KB LDS each: 2 per CU) share a CU (dev tool)."""
import ctypes as C
import collections
import os
import torch
L = C.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "placement.so"))
for n, lds in ((512, 65536), (512, 65536), (384, 65536)):
    out = torch.zeros(n * 4, dtype=torch.int32, device="cuda:0")
    assert L.run_probe(C.c_void_p(out.data_ptr()), n, lds, 2000) == 0  # 20 us resident (100 MHz ticks)
    o = out.view(n, 4).cpu().numpy().astype("int64") & 0xffffffff
    cu = {}
    for b in range(n):
        hw = int(o[b, 1])
        key = (int(o[b, 0]), (hw >> 13) & 7, (hw >> 12) & 1, (hw >> 8) & 15)  # xcc, se, sh, cu
        cu.setdefault(key, []).append(b)
    sizes = collections.Counter(len(v) for v in cu.values())
    pairs = [tuple(v) for v in cu.values() if len(v) == 2]
    diffs = collections.Counter(b - a for a, b in pairs)
    print(f"n={n}: CUs used {len(cu)}, blocks per CU {dict(sizes)}, pair index differences {diffs.most_common(6)}")
    print("  first pairs:", sorted(pairs)[:12])
    xb = collections.Counter((b % 8, k[0]) for k, v in cu.items() for b in v)
    print("  (b % 8 -> xcc) map:", sorted(set((a, x) for (a, x) in xb)))
