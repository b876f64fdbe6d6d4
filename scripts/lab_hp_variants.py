"""Lab builds of the C3 kernel (bitslice.hip k_encode_hp) with alternative
tile-to-workgroup mappings, for same-box A/B timing only (not product code).
Writes labbuild/<name>/librs_mi355x.so, linking the product's other objects."""
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "reedsolomon16_amd", "csrc")
B = os.path.join(ROOT, "reedsolomon16_amd", "build")
HIPCC = "/opt/rocm/bin/hipcc"

MAPS = {
    # consecutive workgroups -> the 8 XCDs round-robin; give XCD x a contiguous range of tiles
    "xcd": "const int nx = gridDim.x >> 3; const int bid = ((int)blockIdx.x & 7) * nx + ((int)blockIdx.x >> 3);",
    # concurrently running workgroups spread over stripes (same column tile of many stripes)
    "stripe": "const int ns = a.ntiles / a.tiles_per_stripe; const int bid = ((int)blockIdx.x % ns) * a.tiles_per_stripe + (int)blockIdx.x / ns;",
    # pairs of adjacent column tiles on one XCD
    "xcd2": "const int b0 = (int)blockIdx.x; const int bid = ((b0 >> 4) << 4) | ((b0 & 1) << 3) | ((b0 >> 1) & 7);",
}


def build(name, mapping):
    d = os.path.join(ROOT, "labbuild", name)
    os.makedirs(d, exist_ok=True)
    s = open(os.path.join(SRC, "bitslice.hip")).read()
    old = "const Loc cur = locate(blockIdx.x);"
    assert old in s
    s = s.replace(old, mapping + " const Loc cur = locate(bid);")
    open(os.path.join(d, "bitslice.hip"), "w").write(s)
    obj = os.path.join(d, "bitslice.o")
    subprocess.check_call([HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-I" + B, "-I" + SRC,
                           "-c", os.path.join(d, "bitslice.hip"), "-o", obj])
    subprocess.check_call([HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", "-o", os.path.join(d, "librs_mi355x.so"),
                           os.path.join(B, "kernels.o"), obj, os.path.join(B, "bitslice_dec.o"),
                           os.path.join(B, "gf_host.o"), os.path.join(B, "codec.o")])


if __name__ == "__main__":
    names = sys.argv[1:] or list(MAPS)
    for n in names:
        build(n, MAPS[n])
        print("built", n)
