"""Host-resident pipeline: wall time per call vs column-segment width
(rs_set_host_segment), 128+32 x 1 MiB, pinned input slab.  Reconstruct is
timed with 32 random erasures whose outputs are fresh pageable arrays (the
Go caller's make([]byte, S))."""
import json
import sys
import time

import numpy as np

sys.path.insert(0, ".")
import reedsolomon16_amd as rs  # noqa: E402

k, p, S = 128, 32, 1 << 20
c = rs.ReedSolomon(k, p, 16)
shards = c.alloc_aligned(S, pinned=True)
rng = np.random.default_rng(1)
for i in range(k):
    shards[i][:] = rng.integers(0, 256, S, dtype=np.uint8)
c.encode(shards)
er = sorted(rng.choice(k + p, p, replace=False).tolist())


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    return (time.perf_counter() - t0) / iters * 1e6


def rec_pageable():
    c.reconstruct([np.zeros(0, np.uint8) if i in er else shards[i] for i in range(k + p)])


for seg in [0, 32 << 10, 64 << 10, 128 << 10, 256 << 10, 512 << 10]:
    c.set_host_segment(seg)
    enc = timeit(lambda: c.encode(shards))
    rec = timeit(rec_pageable)
    print(json.dumps({"seg": seg, "encode_us": round(enc, 1), "reconstruct_pageable_us": round(rec, 1),
                      "encode_pcie_GBps": round((k + p) * S / enc / 1e3, 1),
                      "reconstruct_pcie_GBps": round((k + p) * S / rec / 1e3, 1)}), flush=True)
t = timeit(lambda: np.zeros((p, S), np.uint8).fill(1))
print(json.dumps({"alloc_and_touch_32MiB_us": round(t, 1)}), flush=True)
