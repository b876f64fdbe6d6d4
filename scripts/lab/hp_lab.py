"""Rewrite a copy of bitslice.hip with RS_HP_ABL hooks (scripts/ablate_hp.sh)."""
import sys

p = sys.argv[1]
s = open(p).read()


def rep(old, new):
    global s
    assert old in s, old
    s = s.replace(old, new)


rep("namespace rs {\nnamespace {\nusing namespace bs;",
    "#ifndef RS_HP_ABL\n#define RS_HP_ABL 0\n#endif\nnamespace rs {\nnamespace {\nusing namespace bs;\n"
    "__device__ __forceinline__ void abl_t8(Half &v) { if constexpr (!(RS_HP_ABL & 2)) bs_transpose8(v); "
    "else { _Pragma(\"unroll\") for (int q = 0; q < 8; q++) asm volatile(\"\" : \"+v\"(v[q])); } }")
# networks
rep("    for (int i = 0; i < 8; i++) xor_net8(x[i], y, C < 0 ? TW::fft8[SLOT][i] : TW::ifft8[C < 0 ? 0 : C][SLOT][i]);",
    "    for (int i = 0; i < 8; i++) { if constexpr (RS_HP_ABL & 1) x[i] ^= y[i]; else xor_net8(x[i], y, C < 0 ? TW::fft8[SLOT][i] : TW::ifft8[C < 0 ? 0 : C][SLOT][i]); }")
rep("    for (int r = 0; r < 8; r++) xor_net8(lo[r], hi, TW::dmat[r]);",
    "    for (int r = 0; r < 8; r++) { if constexpr (RS_HP_ABL & 1) lo[r] ^= hi[r]; else xor_net8(lo[r], hi, TW::dmat[r]); }")
# transposes and half swaps
s = s.replace("bs_transpose8(R[", "abl_t8(R[")
rep("__device__ __forceinline__ void hp_swap_halves(Half (&R)[2 * HR]) {\n",
    "__device__ __forceinline__ void hp_swap_halves(Half (&R)[2 * HR]) {\n    if constexpr (RS_HP_ABL & 2) return;\n")
# LDS exchanges
rep("__device__ __forceinline__ void hp_put(uint32_t lbase, int row, const Half &v) {\n",
    "__device__ __forceinline__ void hp_put(uint32_t lbase, int row, const Half &v) {\n    if constexpr (RS_HP_ABL & 4) { _Pragma(\"unroll\") for (int q = 0; q < 8; q++) asm volatile(\"\" :: \"v\"(v[q])); return; }\n")
rep("__device__ __forceinline__ void hp_get(uint32_t lbase, int row, Half &v) {\n",
    "__device__ __forceinline__ void hp_get(uint32_t lbase, int row, Half &v) {\n    if constexpr (RS_HP_ABL & 4) { _Pragma(\"unroll\") for (int q = 0; q < 8; q++) asm volatile(\"\" : \"=v\"(v[q])); return; }\n")
s = s.replace("lds_barrier();", "if constexpr (!(RS_HP_ABL & 4)) lds_barrier();")
# 8: lane-contiguous load addressing (each instruction 512 contiguous bytes
# per lane half; the data lands in the wrong lanes), 16: the same for stores
rep("                const u32x4 x = __builtin_amdgcn_raw_buffer_load_b128(rs, voff + q * QS, soff, 0);",
    "                const uint32_t vo = (RS_HP_ABL & 8) ? voff - (uint32_t)blk * 48 + (uint32_t)q * 512 : voff + q * QS;\n"
    "                const u32x4 x = __builtin_amdgcn_raw_buffer_load_b128(rs, vo, soff, 0);")
rep("                            __builtin_amdgcn_raw_buffer_store_b128(v, ps, voff + k * QS, soff, 0);",
    "                            __builtin_amdgcn_raw_buffer_store_b128(v, ps, (RS_HP_ABL & 16) ? voff - (uint32_t)blk * 48 + (uint32_t)k * 512 : voff + k * QS, soff, 0);")
# 32 / 64: PF1 = 1 / 3 rows of the next chunk before phase 1 (m = 32)
rep("    static constexpr int PF1 = LOGM == 5 ? 2 : HR / 2;",
    "    static constexpr int PF1 = LOGM == 5 ? ((RS_HP_ABL & 32) ? 1 : (RS_HP_ABL & 64) ? 3 : 2) : HR / 2;")
# 128: the first prefetch part right after the staged rows are copied, before the transposes
rep("""        for (int i = 0; i < HR; i++) {
            abl_t8(R[i]);""", """        for (int i = 0; i < HR; i++) {
            if constexpr (RS_HP_ABL & 128) if (i == 0) {
                _Pragma("unroll") for (int i2 = 0; i2 < RW; i2++) _Pragma("unroll") for (int q = 0; q < 8; q++) asm volatile("" : "+v"(R[i2][q])::"memory");
                __builtin_amdgcn_sched_barrier(0);
                prefetch<C, 0, PF1>(cur, nxt);
                __builtin_amdgcn_sched_barrier(0);
            }
            abl_t8(R[i]);""")
rep("""        __builtin_amdgcn_sched_barrier(0);
        prefetch<C, 0, PF1>(cur, nxt);
        __builtin_amdgcn_sched_barrier(0);
        dispatch<4>""", """        __builtin_amdgcn_sched_barrier(0);
        if constexpr (!(RS_HP_ABL & 128)) prefetch<C, 0, PF1>(cur, nxt);
        __builtin_amdgcn_sched_barrier(0);
        dispatch<4>""")
open(p, "w").write(s)
