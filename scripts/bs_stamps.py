"""Per-phase time split of the bit-sliced C3 encode (diagnostic build with
-DRS_BS_STAMP=1, see scripts/build_bs_stamp.sh): fraction of each wave's run
spent waiting for its prefetched rows at chunk starts, in LDS barriers, and in
the final FFT + parity stores.  Run with RS_MI355X_LIB pointing at that build."""
import ctypes as C
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import reedsolomon16_amd as rs  # noqa: E402
from reedsolomon16_amd import _capi  # noqa: E402

stripes = int(sys.argv[1]) if len(sys.argv) > 1 else 16
c = rs.New16(128, 32)
slab = torch.randint(0, 256, (stripes, 160, 1 << 20), dtype=torch.uint8, device="cuda")
for _ in range(5):
    c.encode_dev_batch(slab)
torch.cuda.synchronize()
L = _capi.lib()
n = 1024 * 8 * 4
buf = (C.c_ulonglong * n)()
assert L.rs_debug_bs_stamps(buf, C.c_size_t(n)) == 0
st = np.frombuffer(buf, dtype=np.uint64).reshape(1024, 8, 4).astype(np.float64)
live = st[:, :, 3] > 0
st = st[live]
tot = st[:, 3]
res = {"stripes": stripes, "waves": int(live.sum()), "total_ticks_mean": round(float(tot.mean()), 1)}
for i, name in enumerate(["load_wait", "lds_barrier", "fft_and_stores"]):
    res[name + "_frac"] = round(float((st[:, i] / tot).mean()), 4)
res["by_wave_load_wait_frac"] = [round(float((st[:, 0] / tot)[np.arange(len(st)) % 8 == w].mean()), 4) for w in range(8)]
res["by_wave_barrier_frac"] = [round(float((st[:, 1] / tot)[np.arange(len(st)) % 8 == w].mean()), 4) for w in range(8)]
print(json.dumps(res), flush=True)
