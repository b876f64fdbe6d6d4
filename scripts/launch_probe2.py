"""Which HIP runtime does a torch process use for this library, and do our
launches return before their kernels finish?  Loads the library first when
argv[1] == 'lib-first' (the process then runs on /opt/rocm's runtime)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
if len(sys.argv) > 1 and sys.argv[1] == "lib-first":
    from reedsolomon16_amd import _capi
    _capi.lib()
import torch  # noqa: E402

import reedsolomon16_amd as rs  # noqa: E402

maps = open("/proc/self/maps").read()
print("runtimes:", sorted({l.split()[-1] for l in maps.splitlines() if "libamdhip64" in l}))
c = rs.New16(1024, 256)
s5 = torch.randint(0, 256, (1, 1280, 256 << 10), dtype=torch.uint8, device="cuda")
st = torch.cuda.current_stream()
for _ in range(5):
    c.encode_dev_batch(s5, st)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(50):
    c.encode_dev_batch(s5, st)
t1 = time.perf_counter()
torch.cuda.synchronize()
t2 = time.perf_counter()
print(sys.argv[1:], {"host_us_per_call": round((t1 - t0) / 50 * 1e6, 1), "wall_us_per_call": round((t2 - t0) / 50 * 1e6, 1)})
