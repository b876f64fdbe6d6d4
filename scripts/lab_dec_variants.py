"""Lab builds of the C4 decoder (bitslice_dec.hip) for same-box A/B timing
(not product code): where the early waves pass phase 2's barriers, wave
priority of the late phase-1 units, and a SIMD-aware phase-3 placement.
Writes labbuild/<name>/librs_mi355x.so."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "reedsolomon16_amd", "csrc")
B = os.path.join(ROOT, "reedsolomon16_amd", "build")
HIPCC = "/opt/rocm/bin/hipcc"

BAR_IFFT0 = ("        ifft0_bytes(u);\n        for (int b = 0; b < nbar; b++) lds_barrier();\n")


def bar_scale(s):
    assert BAR_IFFT0 in s
    s = s.replace(BAR_IFFT0, "        ifft0_bytes(u);\n")
    return s.replace("        scale(u);\n        ifft0_bytes(u);\n",
                     "        scale(u);\n        for (int b = 0; b < nbar; b++) lds_barrier();\n        ifft0_bytes(u);\n")


def bar_load(s):
    assert BAR_IFFT0 in s
    s = s.replace(BAR_IFFT0, "        ifft0_bytes(u);\n")
    return s.replace("        load_rows(u);\n        scale(u);\n",
                     "        load_rows(u);\n        for (int b = 0; b < nbar; b++) lds_barrier();\n        scale(u);\n")


def late_prio(s):
    old = "                if (slot == 0) __builtin_amdgcn_s_setprio(3);\n"
    assert old in s
    return s.replace(old, "                if (slot == 0) __builtin_amdgcn_s_setprio(3);\n                else __builtin_amdgcn_s_setprio(2);\n")


def p3simd(s):
    old = "                if (t3[w][1] < 0 && (bw < 0 || cost[w] < cost[bw])) bw = w;\n"
    assert old in s
    new = ("                if (t3[w][1] < 0 && (bw < 0 || cost[w] + pen[w & 3] < cost[bw] + pen[bw & 3])) bw = w;\n")
    s = s.replace(old, new)
    old2 = "        bool ok = true;\n        for (int g = 0; g < G && ok; g++) {\n"
    assert old2 in s
    new2 = ("        int pen[4] = {0, 0, 0, 0};  // SIMDs running a late phase-1 unit\n"
            "        for (int w = 0; w < 8; w++) if (t1[w][0] >= 0) pen[w & 3] += 10;\n" + old2)
    return s.replace(old2, new2)


VARIANTS = {
    "bar_scale": [bar_scale],
    "bar_load": [bar_load],
    "late_prio": [late_prio],
    "p3simd": [p3simd],
    "bar_scale_p3simd": [bar_scale, p3simd],
    "bar_scale_late_prio": [bar_scale, late_prio],
}


def build(name, fns):
    d = os.path.join(ROOT, "labbuild", name)
    os.makedirs(d, exist_ok=True)
    s = open(os.path.join(SRC, "bitslice_dec.hip")).read()
    for f in fns:
        s = f(s)
    open(os.path.join(d, "bitslice_dec.hip"), "w").write(s)
    obj = os.path.join(d, "bitslice_dec.o")
    subprocess.check_call([HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-I" + B, "-I" + SRC,
                           "-c", os.path.join(d, "bitslice_dec.hip"), "-o", obj])
    subprocess.check_call([HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", "-o", os.path.join(d, "librs_mi355x.so"),
                           os.path.join(B, "kernels.o"), os.path.join(B, "bitslice.o"), obj,
                           os.path.join(B, "gf_host.o"), os.path.join(B, "codec.o")])
    os.remove(obj)


if __name__ == "__main__":
    for n in (sys.argv[1:] or VARIANTS):
        build(n, VARIANTS[n])
