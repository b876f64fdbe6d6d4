"""Does the host run ahead of the GPU on this box?  50 back-to-back torch
elementwise kernels (~100 us each) after warmup: host time per launch vs GPU
time per launch."""
import time

import torch

x = torch.randn(64 << 20, device="cuda")
for _ in range(5):
    x.mul_(1.0001)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(50):
    x.mul_(1.0001)
t1 = time.perf_counter()
torch.cuda.synchronize()
t2 = time.perf_counter()
print({"host_us_per_launch": round((t1 - t0) / 50 * 1e6, 1), "wall_us_per_launch": round((t2 - t0) / 50 * 1e6, 1)})
