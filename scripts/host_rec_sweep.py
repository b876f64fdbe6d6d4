"""Host-resident C4 reconstruct (128+32 x 1 MiB, 32 random erasures) into the
caller's pinned rows (EmptyShard), by host-pipeline segment width, and the
same for encode: how much of the reconstruct's extra time is per-copy cost
(scattered rows -> many small copies per segment).  Diagnostic only."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np

import reedsolomon16_amd as rs


def main():
    k, p, S = 128, 32, 1 << 20
    c = rs.New16(k, p)
    sh = c.alloc_aligned(S, pinned=True)
    rng = np.random.default_rng(1)
    for i in range(k):
        sh[i][:] = rng.integers(0, 256, S, dtype=np.uint8)
    c.encode(sh)
    er = set(rng.choice(k + p, p, replace=False).tolist())
    for seg in (0, 131072, 524288, 1048576):
        c.set_host_segment(seg)
        for op in ("encode", "reconstruct"):
            def run():
                if op == "encode":
                    c.encode(sh)
                else:
                    c.reconstruct([rs.EmptyShard(sh[i]) if i in er else sh[i] for i in range(k + p)])
            for _ in range(3):
                run()
            t0 = time.perf_counter()
            n = 20
            for _ in range(n):
                run()
            us = (time.perf_counter() - t0) / n * 1e6
            print(json.dumps({"seg": seg, "op": op, "us": round(us, 1), "pcie_GBps": round((k + p) * S / us / 1e3, 1)}), flush=True)


if __name__ == "__main__":
    main()
