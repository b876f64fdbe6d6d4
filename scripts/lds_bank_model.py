"""LDS bank-conflict model of the LDS-resident transforms (k_rec_lds /
k_enc_lds, 128-byte GF(2^16) tiles: 4 units of 16 low + 16 high bytes, 256
threads, 4 lanes per row).  Lane groups and bank functions are
MI355X_MICROARCH.md §LDS: ds_read_b128 = 4 groups of 16 lanes
{0-3,12-15,20-27}, {4-11,16-19,28-31} (+32), banks (a/4) % 64; ds_write_b128 =
8 groups of 8 contiguous lanes, banks (a/4) % 32.  Prints the LDS-array cycles
of every access of an n = 256 reconstruct (IFFT passes at dist 1 (stores
only), 4, 16, 64; the fused derivative + first FFT pass; FFT passes at dist
16, 4, 1 (loads only)) for the padded layout and for the swizzled layout the
kernels use (LTile::SWZ), against the conflict-free count.  Design aid only."""
N, U = 256, 4
G128 = [list(range(0, 4)) + list(range(12, 16)) + list(range(20, 28)),
        list(range(4, 12)) + list(range(16, 20)) + list(range(28, 32))]
G128 += [[l + 32 for l in g] for g in G128]


def cyc_read(A):
    tot = 0
    for g in G128:
        cnt = {}
        for l in g:
            if A[l] is None:
                continue
            for d in range(4):
                cnt.setdefault((A[l] // 4 + d) % 64, set()).add(A[l] // 4 + d)
        tot += max([len(v) for v in cnt.values()] or [0])
    return tot


def cyc_write(A):
    tot = 0
    for g0 in range(0, 64, 8):
        cnt = {}
        for l in range(g0, g0 + 8):
            if A[l] is None:
                continue
            for d in range(4):
                cnt.setdefault((A[l] // 4 + d) % 32, set()).add(A[l] // 4 + d)
        tot += max([len(v) for v in cnt.values()] or [0])
    return tot


PASSES = [(1, "W"), (4, "RW"), (16, "RW"), (64, "RW"), (64, "D"), (16, "RW"), (4, "RW"), (1, "R")]


def wave_accesses(dist, kind, w):
    """(kind, [(row, unit) per lane]) per wave instruction; items as lds_pass
    numbers them (unit fastest, then j < dist, then group)."""
    items = (N // (4 * dist)) * dist * U
    insts = []
    for k in range((items + 255) // 256):
        lanes = []
        for l in range(64):
            it = 256 * k + 64 * w + l
            if it >= items:
                lanes.append(None)
                continue
            q, u = it // U, it % U
            lanes.append(((q // dist) * 4 * dist + (q & (dist - 1)), u))
        for a in range(4):
            rows = [None if x is None else (x[0] + a * dist, x[1]) for x in lanes]
            if kind in ("R", "RW", "D"):
                insts.append(("R", rows))
            if kind in ("W", "RW", "D"):
                insts.append(("W", rows))
        if kind == "D":  # derivative terms of the low row bits
            for a in range(4):
                b = 1
                while b < dist:
                    insts.append(("R", [None if x is None or x[0] & b else ((x[0] | b) + a * dist, x[1]) for x in lanes]))
                    b <<= 1
    return insts


def cost(addr):
    tr = tw = nr = nw = 0
    for dist, kind in PASSES:
        for w in range(4):
            for t, rows in wave_accesses(dist, kind, w):
                for hi in (0, 1):
                    A = [None if x is None else addr(x[0], x[1], hi) for x in rows]
                    if t == "R":
                        tr += cyc_read(A)
                        nr += 1
                    else:
                        tw += cyc_write(A)
                        nw += 1
    return tr, tw, 4 * nr, 8 * nw


def padded(r, u, hi):  # rows of 128 + 16 B, units in global order (lo at (u/2)*64 + (u%2)*16)
    return r * 144 + (u // 2) * 64 + (u % 2) * 16 + 32 * hi


def swizzled(r, u, hi):  # LTile<F16<4>>::loff
    h = (4 if r & 1 else 0) ^ (7 if r & 4 else 0) ^ (14 if r & 8 else 0) ^ (10 if r & 16 else 0)
    return (r * 128 + u * 16 + 64 * hi) ^ (h << 4)


if __name__ == "__main__":
    seen = set()
    for r in range(N):
        for u in range(U):
            for hi in (0, 1):
                a = swizzled(r, u, hi)
                assert a not in seen and 0 <= a < N * 128
                seen.add(a)
    for name, fn in (("padded 144 B", padded), ("swizzled 128 B", swizzled)):
        tr, tw, ir, iw = cost(fn)
        print(f"{name:16s} read cycles {tr:5d} (conflict-free {ir})  write cycles {tw:5d} (conflict-free {iw})")
