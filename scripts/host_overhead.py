"""Per-call host time vs GPU time of the device-resident entry points, calls
issued back to back on one caller stream: if the host time per call is close
to the GPU time per call, something in the call blocks on earlier work."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import numpy as np
    import torch

    import reedsolomon16_amd as rs
    st = torch.cuda.current_stream()
    cases = []
    c5 = rs.New16(1024, 256)
    s5 = torch.randint(0, 256, (1, 1280, 256 << 10), dtype=torch.uint8, device="cuda")
    cases.append(("C5 encode_dev_batch", lambda: c5.encode_dev_batch(s5, st)))
    c4 = rs.New16(128, 32)
    r4 = torch.randint(0, 256, (160, 1 << 20), dtype=torch.uint8, device="cuda")
    pr = np.ones(160, bool)
    pr[np.random.default_rng(1).choice(160, 32, replace=False)] = False
    cases.append(("C4 reconstruct_dev", lambda: c4.reconstruct_dev(r4, pr, stream=st)))
    cases.append(("C3x1 encode_dev_batch", lambda: c4.encode_dev_batch(r4.view(1, 160, 1 << 20), st)))
    for name, fn in cases:
        for _ in range(5):
            fn()
        torch.cuda.synchronize()
        n = 50
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        t0 = time.perf_counter()
        for _ in range(n):
            fn()
        t1 = time.perf_counter()
        e1.record(st)
        torch.cuda.synchronize()
        print(json.dumps({"case": name, "host_us_per_call": round((t1 - t0) / n * 1e6, 1),
                          "gpu_us_per_call": round(e0.elapsed_time(e1) * 1e3 / n, 1),
                          "stream": "torch default (RS_NULL_STREAM)"}), flush=True)


if __name__ == "__main__":
    main()
