"""Run C4 x 16 once on the stamp lab build (scripts/lab_dec_stamp.py) and
summarise the per-wave phase times (cycles, median over iterations 2..60 of
the first four workgroups).  Stamps: 0 iteration start, 1 after phase 2,
2 after the Y barrier, 3 after phase 3, 4 after slot 0 (early phase 1),
5 after slot 1 (late phase 1), 6 image-free barrier, 7 end barrier."""
import ctypes as C
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
NWG, NIT, NPT = 4, 80, 8


def main():
    import torch

    import reedsolomon16_amd as rs
    from reedsolomon16_amd import _capi

    k, p, S, ns = 128, 32, 1 << 20, 16
    c = rs.ReedSolomon(k, p, 16)
    slab = torch.randint(0, 256, (ns, k + p, S), dtype=torch.uint8, device="cuda")
    present = np.ones(k + p, bool)
    present[np.random.default_rng(0x5EED).choice(k + p, p, replace=False)] = False
    for _ in range(3):
        c.reconstruct_dev_batch(slab, present)
    torch.cuda.synchronize()
    buf = np.zeros(NWG * NIT * 12 * NPT, np.uint32)
    L = _capi.lib()
    L.rs_debug_dec_stamps.argtypes = [C.c_void_p, C.c_size_t]
    assert L.rs_debug_dec_stamps(buf.ctypes.data, buf.size) == 0
    st = buf.reshape(NWG, NIT, 12, NPT).astype(np.int64)
    # per wave: segment durations relative to the iteration start (stamp 0)
    out = {}
    for w in range(12):
        rows = []
        for g in range(NWG):
            for i in range(2, 60):
                s = st[g, i, w]
                if s[0] == 0 or s[7] == 0:
                    continue
                rows.append([int(x - s[0]) & 0xFFFFFFFF for x in s])
        a = np.median(np.array(rows), axis=0) if rows else []
        out[w] = [int(x) for x in a]
    it_len = []
    for g in range(NWG):
        for i in range(2, 59):
            it_len.append((int(st[g, i + 1, 0, 0]) - int(st[g, i, 0, 0])) & 0xFFFFFFFF)
    print(json.dumps({"iter_cycles_median": int(np.median(it_len)), "per_wave": out}))


if __name__ == "__main__":
    main()
