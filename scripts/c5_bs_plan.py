"""Cost plan of a bit-sliced C5 encode (m = 256, 4 chunks) from the engine's own
field tables (C-ABI host diagnostics, no GPU): VERDICT round 5, item 3, "First,
commit the static code size and VALU count of the plan against k_enc_lds".

The plan: every chunk twiddle is the FFT's twiddle of the same
(layer, group) XOR one constant per (chunk, layer) -- fftSkew[j + 2^(i+1)] =
fftSkew[j] ^ temp_L[i] in FFTInitialize (leopard16.go:986-1031) -- so
x * tw(c, L, r) = x * a(L, r) ^ x * delta(c, L), where a(L, r) lies in GF(2^8)
(one 8x8 GF(2) network on both byte halves in subfield coordinates, shared by
the FFT and every chunk) and delta(c, L) needs one 16x16 network per
(chunk, layer), shared by every group of the layer.  This script checks that
decomposition on every butterfly of the m = 256, k = 1024 encode and counts:

  - distinct networks (code), with their op counts;
  - VALU ops per 32-symbol column (one lane's 16 plane dwords) for the whole
    encode (4 chunk IFFTs + the FFT), naive network cost (an output plane that
    XORs n input planes into an accumulator: ceil(n / 2) v_bitop3_b32);
  - the same for the byte-permute form k_enc_lds runs today (per 32 symbols:
    full-field product 12 v_perm + 10 index ops + 6 XOR3 per dword pair, 8
    pairs; subfield product 6 + 10 + 4; butterfly XOR 2 per pair).

usage: python scripts/c5_bs_plan.py   (prints the table DESIGN §4.6 cites)
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from reedsolomon16_amd import _capi  # noqa: E402

M, NCH, MOD = 256, 4, 65535


def tables():
    L = _capi.lib()
    log = np.zeros(65536, np.uint16)
    exp = np.zeros(65536, np.uint16)
    skew = np.zeros(65536, np.uint16)
    walsh = np.zeros(65536, np.uint16)
    assert L.rs_debug_field_tables(16, log.ctypes.data, exp.ctypes.data, skew.ctypes.data, walsh.ctypes.data) == 0
    return L, log.astype(np.int64), exp.astype(np.int64), skew.astype(np.int64)


def main():
    L, log, exp, skew = tables()

    def val(lg):  # element from its log (MOD = the zero element)
        return 0 if lg == MOD else int(exp[lg])

    def mul(a, v):  # a * v in the table basis
        if a == 0 or v == 0:
            return 0
        return int(exp[(log[a] + log[v]) % MOD])

    def sub(x):
        return int(L.rs_debug_sub_swap(x))

    def matrix(v):  # 16x16 GF(2) rows (bit j of row i: input bit j feeds output bit i), subfield coordinates
        cols = [sub(mul(sub(1 << j), v)) for j in range(16)]
        return [sum(((cols[j] >> i) & 1) << j for j in range(16)) for i in range(16)]

    def net_ops(rows):  # naive accumulate cost of x ^= M y
        return sum((bin(r).count("1") + 1) // 2 for r in rows)

    def is_sub(rows):  # one 8x8 map on both halves
        return all((rows[i] >> 8) == 0 for i in range(8)) and all(rows[i] & 0xFF == 0 for i in range(8, 16)) and \
            all(rows[i] == rows[i + 8] >> 8 for i in range(8))

    # butterflies: (transform, layer, group base r) -> twiddle value
    def tw_fft(Lr, r):
        return val(int(skew[r + (1 << Lr) - 1]))

    def tw_chunk(c, Lr, r):
        return val(int(skew[(c + 1) * M - 1 + r + (1 << Lr)]))

    groups = [(Lr, r) for Lr in range(8) for r in range(0, M, 2 << Lr)]
    sub_nets, delta_nets, bad = {}, {}, 0
    bs_ops = bp_ops = 0
    full_bf = sub_bf = zero_bf = 0
    for c in list(range(NCH)) + [-1]:
        for Lr, r in groups:
            nb = 1 << Lr  # butterflies of the group (pairs (i, i + 2^L), r <= i < r + 2^L)
            t = tw_fft(Lr, r) if c < 0 else tw_chunk(c, Lr, r)
            a = tw_fft(Lr, r)
            d = t ^ a
            bs_ops += 16 * nb  # butterfly XOR (y ^= x or x ^= y), one op per plane
            bp_ops += 16 * nb
            if t == 0:
                zero_bf += nb
                continue
            ma = matrix(a) if a else [0] * 16
            if a and not is_sub(ma):
                bad += 1
            if a:
                sub_nets.setdefault(a, net_ops(ma[:8]))
                bs_ops += 2 * sub_nets[a] * nb
            if d:
                key = (c, Lr)
                md = matrix(d)
                if delta_nets.setdefault(key, (d, net_ops(md)))[0] != d:
                    bad += 1  # delta must be one constant per (chunk, layer)
                bs_ops += (delta_nets[key][1] + 16) * nb  # the delta product, then its XOR into x
            if is_sub(matrix(t)):
                sub_bf += nb
                bp_ops += 8 * (6 + 10 + 4) * nb
            else:
                full_bf += nb
                bp_ops += 8 * (12 + 10 + 6) * nb
    rows_io = NCH * M + M  # rows transposed in (data) and out (parity) per column
    transposes = rows_io * 2 * 16  # byte <-> plane: ~2 ops per plane dword per row
    coords = rows_io * 16  # lo ^= D(hi) per row (8 output planes, ~2 ops each)
    sub_code = sum(2 * v for v in sub_nets.values())
    delta_code = sum(v[1] for v in delta_nets.values())
    meas = 2.31e9 / 32 * 64 / (256 * 1024 // 64)  # k_enc_lds SQ_INSTS_VALU x lanes per 32-symbol column
    print(f"decomposition tw(c, L, r) = a(L, r) ^ delta(c, L) with a in GF(2^8): "
          f"{'holds on every butterfly' if bad == 0 else f'FAILS on {bad}'}")
    print(f"butterflies per column: {full_bf} full-field, {sub_bf} subfield, {zero_bf} zero twiddle")
    print(f"code: {len(sub_nets)} subfield networks ({sub_code} ops on both halves), "
          f"{len(delta_nets)} delta networks ({delta_code} ops); "
          f"~{(sub_code + delta_code) * 8 / 1024:.0f} KB at 8 bytes per v_bitop3_b32, unrolled once")
    print(f"VALU per 32-symbol column, bit-sliced plan: networks+XORs {bs_ops}, transposes {transposes}, "
          f"coordinates {coords}: total {bs_ops + transposes + coords}")
    print(f"VALU per 32-symbol column, byte-permute model (k_enc_lds): {bp_ops}; measured "
          f"(SQ_INSTS_VALU 2.31e9 per 32 stripes, r05_sq_counters.txt): {meas:.0f}")
    print(f"plan / measured: {(bs_ops + transposes + coords) / meas:.2f}  (LDS exchange, address and load/store "
          f"instructions not counted in the plan)")


if __name__ == "__main__":
    main()
