"""Lab build of the C4 decoder (bitslice_dec.hip k_rec_bs256) with per-wave
s_memtime stamps at the phase boundaries of every iteration, for the first
four workgroups (timing study only, not product code).  Writes
labbuild/stamp/librs_mi355x.so with an extra rs_debug_dec_stamps(out, n)."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "reedsolomon16_amd", "csrc")
B = os.path.join(ROOT, "reedsolomon16_amd", "build")
HIPCC = "/opt/rocm/bin/hipcc"
NWG, NIT, NPT = 4, 80, 8


def patch(s):
    decl = ("__device__ uint32_t g_stamp[%d * %d * 12 * %d];\n"
            "#define STAMP(k) do { if (blockIdx.x < %d && it < %d && (threadIdx.x & 63) == 0) "
            "g_stamp[((blockIdx.x * %d + it) * 12 + w) * %d + (k)] = (uint32_t)__builtin_amdgcn_s_memtime(); } while (0)\n"
            % (NWG, NIT, NPT, NWG, NIT, NIT, NPT))
    anchor = "template <bool STRIDED>\n__global__ void __launch_bounds__(64 * kWaves, kWaves / 4) k_rec_bs256"
    assert anchor in s
    s = s.replace(anchor, decl + anchor)
    reps = [
        ("    int t = -1, tn = blockIdx.x;  // tile in phases 2-3, tile in phase 1\n    if (tn >= pl.ntiles) return;\n    for (;;) {\n",
         "    int t = -1, tn = blockIdx.x;  // tile in phases 2-3, tile in phase 1\n    if (tn >= pl.ntiles) return;\n    int it = 0;\n    for (;; it++) {\n        STAMP(0);\n"),
        ("                if (!early)\n                    d.phase2();\n",
         "                if (!early)\n                    d.phase2();\n                STAMP(1);\n"),
        ("                if (!early_p1) lds_barrier();  // Y is in the image\n",
         "                if (!early_p1) lds_barrier();  // Y is in the image\n                STAMP(2);\n"),
        ("                        d.phase3(u);\n                    }\n                }\n",
         "                        d.phase3(u);\n                    }\n                }\n                STAMP(3);\n"),
        ("                __builtin_amdgcn_s_setprio(0);\n            }\n        }\n",
         "                __builtin_amdgcn_s_setprio(0);\n            }\n            STAMP(4 + slot);\n        }\n"),
        ("        lds_barrier();  // the image is free for phase 1 of tile tn\n",
         "        lds_barrier();  // the image is free for phase 1 of tile tn\n        STAMP(6);\n"),
        ("        lds_barrier();  // u of tile tn is in the image\n",
         "        lds_barrier();  // u of tile tn is in the image\n        STAMP(7);\n"),
    ]
    for a, b in reps:
        assert a in s, a
        s = s.replace(a, b)
    s += ("\nextern \"C\" int rs_debug_dec_stamps(uint32_t *out, size_t n) {\n"
          "    return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(rs::g_stamp), n * 4, 0, hipMemcpyDeviceToHost);\n}\n")
    # g_stamp lives in the anonymous namespace: expose it
    s = s.replace("__device__ uint32_t g_stamp", "}  // namespace\n__device__ uint32_t g_stamp", 1)
    s = s.replace("#define STAMP(k)", "namespace {\n#define STAMP(k)", 1)
    return s


def main():
    d = os.path.join(ROOT, "labbuild", "stamp")
    os.makedirs(d, exist_ok=True)
    s = patch(open(os.path.join(SRC, "bitslice_dec.hip")).read())
    open(os.path.join(d, "bitslice_dec.hip"), "w").write(s)
    obj = os.path.join(d, "bitslice_dec.o")
    subprocess.check_call([HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-I" + B, "-I" + SRC,
                           "-c", os.path.join(d, "bitslice_dec.hip"), "-o", obj])
    subprocess.check_call([HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", "-o", os.path.join(d, "librs_mi355x.so"),
                           os.path.join(B, "kernels.o"), os.path.join(B, "bitslice.o"), obj,
                           os.path.join(B, "gf_host.o"), os.path.join(B, "codec.o")])


if __name__ == "__main__":
    main()
