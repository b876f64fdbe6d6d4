"""Do kernels from a hipcc-built library block the host when launched from a
torch process (torch's bundled HIP runtime)?  spin: plain kernel; lds64: 64 KB
static LDS."""
import ctypes as C
import os
import time

import torch

L = C.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "micro", "libspin.so"))
x = torch.randn(64 << 20, device="cuda")
st = torch.cuda.current_stream()
for name, fn in [("spin", lambda: L.spin_launch(C.c_void_p(x.data_ptr()), 64 << 20, 20, C.c_void_p(st.cuda_stream))),
                 ("lds64", lambda: L.lds64_launch(C.c_void_p(x.data_ptr()), 64 << 20, C.c_void_p(st.cuda_stream)))]:
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(50):
        fn()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(name, {"host_us": round((t1 - t0) / 50 * 1e6, 1), "wall_us": round((t2 - t0) / 50 * 1e6, 1)})
