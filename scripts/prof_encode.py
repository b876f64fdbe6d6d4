"""Profiling driver: run one codec operation N times on synthetic HBM-resident
data (no checks).  Used under rocprofv3: `rocprofv3 ... -- python3 scripts/prof_encode.py ...`."""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--k", type=int, default=128)
    ap.add_argument("--p", type=int, default=32)
    ap.add_argument("--S", type=int, default=1 << 20)
    ap.add_argument("--bits", type=int, default=16)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--op", default="encode", choices=["encode", "verify", "reconstruct"])
    a = ap.parse_args()
    import numpy as np
    import torch

    import reedsolomon16_amd as rs

    c = rs.ReedSolomon(a.k, a.p, a.bits)
    slab = torch.randint(0, 256, (a.k + a.p, a.S), dtype=torch.uint8, device="cuda")
    c.encode_dev(slab)
    present = np.ones(a.k + a.p, bool)
    present[np.random.default_rng(0x5EED).choice(a.k + a.p, a.p, replace=False)] = False
    for _ in range(a.iters):
        if a.op == "encode":
            c.encode_dev(slab)
        elif a.op == "verify":
            c.verify_dev(slab)
        else:
            c.reconstruct_dev(slab, present)
    torch.cuda.synchronize()
    print("done", c.encode_path)


if __name__ == "__main__":
    main()
