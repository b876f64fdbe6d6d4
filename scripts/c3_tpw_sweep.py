"""C3 encode (k_encode_hp) tiles per workgroup, swept through the test-only
rs_debug_set_path("hp_tiles", n) knob (0 = the launcher's automatic choice):
HIP-event kernel time per launch on resident stripes, rows 1 MiB + 3.5 KiB
apart (bench.py's layout), for full rows and for the per-rank row slices of
2-, 4- and 8-rank byte-range splits.  Prints one JSON line per point."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--stripes", default="256,64,16")
    ap.add_argument("--slices", default="1,2,8")
    ap.add_argument("--tiles", default="0,1,2,4,8")
    ap.add_argument("--steps", default="0", help="hp_step values (tile distance; 0 = the grid size)")
    ap.add_argument("--tails", default="-1", help="hp_tail values of a lab build (single-tile tail; -1 = the product, no knob)")
    ap.add_argument("--alloc", type=int, default=0, help="stripes to allocate (0: the largest launched)")
    ap.add_argument("--geom", default="128,32")
    ap.add_argument("--pad", default="3584", help="bytes between rows beyond the row (0: rows back to back); a comma list sweeps")
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    import torch

    import reedsolomon16_amd as rs
    from reedsolomon16_amd import _capi
    from reedsolomon16_amd import dist as rsd

    K, P = (int(x) for x in a.geom.split(","))
    S = 1 << 20
    pads = [int(x) for x in a.pad.split(",")]
    codec = rs.New16(K, P)
    bmax = a.alloc or max(int(x) for x in a.stripes.split(","))
    for nsl in (int(x) for x in a.slices.split(",")):
        lo, hi = rsd.byte_range(S, 0, nsl)
        W = hi - lo
        buf = torch.randint(0, 256, (bmax * (K + P) * (W + max(pads)),), dtype=torch.uint8, device="cuda")
        for B, pad in [(int(x), pd) for x in a.stripes.split(",") for pd in pads]:
            RS = W + pad
            slab = buf[: B * (K + P) * RS].as_strided((B, K + P, W), ((K + P) * RS, RS, 1))
            for t, stp, tl in [(int(x), int(y), int(z)) for x in a.tiles.split(",") for y in a.steps.split(",") for z in a.tails.split(",")]:
                if t == 1 and (stp or tl > 0):
                    continue
                _capi.set_path("hp_tiles", t)
                _capi.set_path("hp_step", stp)
                if tl != -1:  # lab builds with the hp_tail knob only (profiles/r05_c3_tail_sweep.txt)
                    _capi.set_path("hp_tail", tl)
                st = torch.cuda.current_stream()
                for _ in range(3):
                    codec.encode_dev_batch(slab, st)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                torch.cuda.synchronize()
                e0.record(st)
                for _ in range(a.iters):
                    codec.encode_dev_batch(slab, st)
                e1.record(st)
                torch.cuda.synchronize()
                ms = e0.elapsed_time(e1) / a.iters
                alg = B * (K + P) * W
                print(json.dumps({"geom": f"{K}+{P}", "stripes": B, "ranks": nsl, "row_bytes": W, "tiles": t, "step": stp, "tail": tl, "pad": pad, "alloc": bmax,
                                  "ms": round(ms, 5), "frac": round(alg / (ms * 1e-3) / 8e12, 4)}), flush=True)
        del buf
        torch.cuda.empty_cache()
    _capi.reset_paths()


if __name__ == "__main__":
    main()
