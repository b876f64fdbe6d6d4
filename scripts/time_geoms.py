"""Kernel time and HBM-roofline fraction of the device-resident encode for a
list of geometries (k:p), B stripes x (k+p) rows x S bytes per launch.
usage: python scripts/time_geoms.py [--stripes B] [--shard S] k:p [k:p ...]"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("geoms", nargs="+")
    ap.add_argument("--stripes", type=int, default=16)
    ap.add_argument("--shard", type=int, default=1 << 20)
    ap.add_argument("--steps", type=int, default=50)
    args = ap.parse_args()
    import torch

    import reedsolomon16_amd as rs
    s = torch.cuda.current_stream()
    for gk in args.geoms:
        k, p = (int(x) for x in gk.split(":"))
        c = rs.New16(k, p)
        B, S = args.stripes, args.shard
        slab = torch.randint(0, 256, (B, k + p, S), dtype=torch.uint8, device="cuda")
        for _ in range(5):
            c.encode_dev_batch(slab, s)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record(s)
        for _ in range(args.steps):
            c.encode_dev_batch(slab, s)
        e1.record(s)
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / args.steps
        alg = B * (k + p) * S
        print(json.dumps({"k": k, "p": p, "path": c.encode_path, "stripes": B, "shard": S, "kernel_ms": round(ms, 4),
                          "frac": round(alg / (ms * 1e-3) / 8e12, 4)}), flush=True)
        del slab


if __name__ == "__main__":
    main()
