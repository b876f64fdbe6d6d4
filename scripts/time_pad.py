"""Layout experiment: C3 encode (rs_encode_dev_batch, 16 stripes per launch)
with the shard rows placed at a padded row stride (S + pad) and stripes at a
padded stripe stride.  Rows exactly 1 MiB apart put every row's column tile
at the same low 20 address bits; this measures what that aliasing costs the
HBM channels.  HIP events on the launch stream; parity of every layout is
checked against the unpadded layout's output.  Diagnostic only."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pads", default="0,256,4096,65536")
    ap.add_argument("--stripe-pads", default="0")
    ap.add_argument("--stripes", type=int, default=16)
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--k", type=int, default=128)
    ap.add_argument("--p", type=int, default=32)
    ap.add_argument("--S", type=int, default=1 << 20)
    a = ap.parse_args()
    import torch

    import reedsolomon16_amd as rs

    k, p, S, B = a.k, a.p, a.S, a.stripes
    c = rs.ReedSolomon(k, p, 16)
    g = torch.Generator(device="cuda")
    g.manual_seed(0x5EED)
    ref_par = None
    st = torch.cuda.current_stream()
    for spad in [int(x) for x in a.stripe_pads.split(",")]:
        for pad in [int(x) for x in a.pads.split(",")]:
            RS = S + pad
            SS = (k + p) * RS + spad
            buf = torch.empty(B * SS, dtype=torch.uint8, device="cuda")
            view = buf.as_strided((B, k + p, S), (SS, RS, 1))
            g.manual_seed(0x5EED)
            view.copy_(torch.randint(0, 256, (B, k + p, S), dtype=torch.uint8, device="cuda", generator=g))
            for _ in range(20):
                c.encode_dev_batch(view, st)
            torch.cuda.synchronize()
            par = view[:, k:].contiguous()
            if ref_par is None:
                ref_par = par
            ok = bool(torch.equal(par, ref_par))
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.iters):
                c.encode_dev_batch(view, st)
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) * 1e3 / a.iters
            alg = B * (k + p) * S
            print(json.dumps({"row_pad": pad, "stripe_pad": spad, "us": round(us, 1),
                              "frac": round(alg / us / 1e3 / 8000, 4), "parity_same": ok}), flush=True)
            del buf, view, par
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
