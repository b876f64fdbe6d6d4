// Compile-time butterfly schedules shared by the kernels (kernels.hip) and the
// host codec (codec.cpp), so that the twiddle images the host lays out are
// exactly the ones the kernels consume.
//
// A transform over M = 2^LOGM rows is a list of radix-2 butterfly ops.  Kinds:
// IFFT (y ^= x; x ^= y*t), FFT (x ^= y*t; y ^= x) and FFT-XOR (y ^= x, zero
// twiddle).  Orders and twiddle slots follow
//   ifftDITEncoder leopard16.go:694-741: radix-4 pairs at dist 1,4,16 (m01 on
//     (i,i+d), m23 on (i+2d,i+3d), then m02 on (i,i+2d),(i+d,i+3d)), and a
//     radix-2 layer at M/2 when log2(M) is odd;
//   fftDIT leopard16.go:618-657: radix-4 pairs at dist M/4, M/16, ... (m02
//     first, then m01 / m23), and a radix-2 layer at dist 1 when log2(M) is odd.
// The reference skips IFFT groups with r >= mtrunc: those rows are zero here,
// and any twiddle maps zero rows to zero rows, so computing them is equivalent.
// In the FFT, the r = 0 group's m01 = fftSkew[dist-1] and m02 = fftSkew[2*dist-1]
// (and the radix-2 fftSkew[0]) are fftSkew[2^j - 1] = log(0) (initFFTSkew
// leopard16.go:997), so they are XOR-only by construction (checked on the host
// in encode_schedule).  FFT rows >= p are computed but never stored.
#pragma once

namespace rs {

// Twiddle slot of one butterfly of the reference schedule (gf_host.cpp
// ifft_passes / fft_passes order), by layer and the lower row of its pair.
constexpr int ilog2c(int x) { return x <= 1 ? 0 : 1 + ilog2c(x >> 1); }
// IFFT: radix-4 passes at dist 1, 4, 16, ... then a radix-2 pass if logm is
// odd.  A radix-4 group's slots are (m01, m02, m23): layer log2(dist) pairs
// rows with m01 (second bit of row/dist clear) or m23, layer log2(dist)+1
// pairs them with m02.
constexpr int ifft_slot(int logm, int layer, int row) {
    int off = 0;
    for (int dist = 1; dist * 4 <= (1 << logm); dist *= 4) {
        const int l0 = ilog2c(dist), g = row / (4 * dist);
        if (layer == l0 + 1) return off + 3 * g + 1;
        if (layer == l0) return off + 3 * g + (((row / dist) & 2) ? 2 : 0);
        off += 3 * ((1 << logm) / (4 * dist));
    }
    return off;
}
// FFT: radix-4 passes at dist m/4, m/16, ... (layer log2(dist)+1 first, with
// m02), then a radix-2 pass over layer 0 if logm is odd (slot per row pair).
constexpr int fft_slot(int logm, int layer, int row) {
    const int M = 1 << logm;
    int off = 0, dist4 = M;
    for (int dist = M >> 2; dist != 0; dist4 = dist, dist >>= 2) {
        const int l0 = ilog2c(dist), g = row / dist4;
        if (layer == l0 + 1) return off + 3 * g + 1;
        if (layer == l0) return off + 3 * g + (((row / dist) & 2) ? 2 : 0);
        off += 3 * (M / dist4);
    }
    return off + row / 2;
}

enum : int { OP_IFFT = 0, OP_FFT = 1, OP_FFTX = 2 };
struct BOp {
    int x, y, slot, kind;
};

// Within a radix-4 group the ops are ordered by twiddle (all m01 butterflies,
// then all m23, then all m02 for the IFFT; m02, m01, m23 for the FFT) so
// consecutive ops share a table; this is legal because butterflies of one
// layer over different i are independent.
template <int LOGM>
struct IfftOps {
    static constexpr int M = 1 << LOGM, N = (M / 2) * LOGM;
    BOp op[N > 0 ? N : 1];
    constexpr IfftOps() : op() {
        int n = 0, slot = 0, dist = 1;
        for (; dist * 4 <= M; dist *= 4)
            for (int r = 0; r < M; r += 4 * dist, slot += 3) {
                for (int i = r; i < r + dist; i++) op[n++] = BOp{i, i + dist, slot, OP_IFFT};                   // m01
                for (int i = r; i < r + dist; i++) op[n++] = BOp{i + 2 * dist, i + 3 * dist, slot + 2, OP_IFFT};  // m23
                for (int i = r; i < r + dist; i++) {                                                             // m02
                    op[n++] = BOp{i, i + 2 * dist, slot + 1, OP_IFFT};
                    op[n++] = BOp{i + dist, i + 3 * dist, slot + 1, OP_IFFT};
                }
            }
        if (dist < M)
            for (int i = 0; i < M / 2; i++) op[n++] = BOp{i, i + M / 2, slot, OP_IFFT};
    }
};
template <int LOGM>
struct FftOps {
    static constexpr int M = 1 << LOGM, N = (M / 2) * LOGM;
    BOp op[N > 0 ? N : 1];
    constexpr FftOps() : op() {
        int n = 0, slot = 0, dist = M / 4;
        for (; dist != 0; dist /= 4)
            for (int r = 0; r < M; r += 4 * dist, slot += 3) {
                const int k0 = r == 0 ? OP_FFTX : OP_FFT;
                for (int i = r; i < r + dist; i++) {  // m02
                    op[n++] = BOp{i, i + 2 * dist, slot + 1, k0};
                    op[n++] = BOp{i + dist, i + 3 * dist, slot + 1, k0};
                }
                for (int i = r; i < r + dist; i++) op[n++] = BOp{i, i + dist, slot, k0};                          // m01
                for (int i = r; i < r + dist; i++) op[n++] = BOp{i + 2 * dist, i + 3 * dist, slot + 2, OP_FFT};  // m23
            }
        if (LOGM & 1)
            for (int r = 0; r < M; r += 2) op[n++] = BOp{r, r + 1, slot + r / 2, r == 0 ? OP_FFTX : OP_FFT};
    }
};

// ---------------------------------------------------------------- half-wave split schedules
// The split encode kernel holds the M rows of a column unit in two lanes
// (lane L and L+32): lanes of half h hold the rows whose bit H equals h, in
// M/2 registers, so that register k holds, in its two half-waves, two rows
// that differ only in bit H.  A butterfly whose rows do not differ in bit H
// then runs in both halves at once as a pair of ops (the op on the rows with
// bit H = 0 in the lower half, its twin with bit H = 1 in the upper half);
// the pair may need different twiddles (when H is above the layer's bits),
// so each half reads its own table.  Before a layer that pairs rows across
// bit H, the split bit moves to H' with one v_permlane32_swap per register
// pair: for rows R00, R01, R10, R11 (bits H, H'), registers [R00|R10] and
// [R01|R11] become [R00|R01] and [R10|R11].  The ops are taken radix-2
// sub-layer by sub-layer (see the constructor); ops of one sub-layer are
// mutually independent and an op's twin sits in the same sub-layer, so running
// each op together with its twin keeps every dependency.
enum : int { ST_OP = 0, ST_SWAP = 1 };
struct SStep {
    int type, a, b, kind, tab;  // OP: registers a (x), b (y), kind, table index (-1: none); SWAP: vdst a, src b
};

constexpr int sched_bit_of(int v) {
    int b = 0;
    while ((1 << b) < v) b++;
    return b;
}
constexpr int sched_remove_bit(int r, int h) { return (r & ((1 << h) - 1)) | ((r >> (h + 1)) << h); }

// Best split bit for an op list from op index i on: the bit that no op
// touches for the longest prefix (ties: the lowest bit); `avoid` excluded.
template <class OPS, int LOGM>
constexpr int sched_best_bit(const OPS &ops, const bool *done, int i, int avoid) {
    int best = -1, best_run = -1;
    for (int c = 0; c < LOGM; c++) {
        if (c == avoid) continue;
        int run = 0;
        for (int j = i; j < OPS::N; j++) {
            if (done && done[j]) continue;
            if (sched_bit_of(ops.op[j].x ^ ops.op[j].y) == c) break;
            run++;
        }
        if (run > best_run) {
            best_run = run;
            best = c;
        }
    }
    return best;
}

template <class OPS, int LOGM>
struct SplitSched {
    static constexpr int M = 1 << LOGM, HM = M / 2;
    static constexpr int MAXS = OPS::N / 2 + LOGM * (HM / 2 + 1) + 4;
    SStep step[MAXS];
    int nsteps;
    int tab_lo[OPS::N], tab_hi[OPS::N];  // twiddle slot per table load and half (-1: zero table)
    int ntab;
    int h0, hend;
    int row0[HM];        // initial layout: register k holds rows row0[k] (lower) and row0[k] | 1 << h0 (upper)
    int fin_row[2][HM];  // final layout: register k, half h holds row fin_row[h][k]
    int fin_phys[M], fin_half[M];  // final layout per row

    // hstart < 0: pick the best start bit; hfinal < 0: leave the final bit free.
    // init_phys / init_half: start from this layout (split bit hstart) instead
    // of the canonical one (row r in register remove_bit(r, hstart)), e.g. the
    // final layout of the transform that produced the rows.
    constexpr SplitSched(int hstart, int hfinal, const int *init_phys = nullptr, const int *init_half = nullptr)
        : step(), nsteps(0), tab_lo(), tab_hi(), ntab(0), h0(0), hend(0), row0(), fin_row(), fin_phys(), fin_half() {
        // Layer-major order: the op lists interleave a radix-4 group's two
        // radix-2 sub-layers group by group; a twin across a group bit may sit
        // in a group whose first sub-layer has not run yet.  Each sub-layer
        // touches exactly one row bit, so sorting (stably) by the first
        // appearance of the touched bit makes every sub-layer contiguous.
        constexpr OPS src{};
        OPS ops{};
        {
            int first[LOGM > 0 ? LOGM : 1] = {}, n = 0;
            for (int b = 0; b < LOGM; b++) first[b] = OPS::N;
            for (int i = 0; i < OPS::N; i++) {
                const int b = sched_bit_of(src.op[i].x ^ src.op[i].y);
                if (first[b] > i) first[b] = i;
            }
            for (int pass = 0; pass < LOGM; pass++) {
                int bb = -1;
                for (int b = 0; b < LOGM; b++)
                    if (first[b] < OPS::N && (bb < 0 || first[b] < first[bb])) bb = b;
                if (bb < 0) break;
                for (int i = 0; i < OPS::N; i++)
                    if (sched_bit_of(src.op[i].x ^ src.op[i].y) == bb) ops.op[n++] = src.op[i];
                first[bb] = OPS::N;
            }
        }
        bool done[OPS::N > 0 ? OPS::N : 1] = {};
        int phys[M] = {}, half[M] = {};
        int H = hstart >= 0 ? hstart : sched_best_bit<OPS, LOGM>(ops, nullptr, 0, -1);
        h0 = H;
        for (int r = 0; r < M; r++) {
            phys[r] = init_phys ? init_phys[r] : sched_remove_bit(r, H);
            half[r] = init_half ? init_half[r] : (r >> H) & 1;
            if (!half[r]) row0[phys[r]] = r;
        }
        int last_lo = -2, last_hi = -2;
        for (int i = 0; i < OPS::N; i++) {
            if (done[i]) continue;
            const BOp o = ops.op[i];
            if (sched_bit_of(o.x ^ o.y) == H) {
                const int H2 = sched_best_bit<OPS, LOGM>(ops, done, i, H);
                move_split(phys, half, H, H2);
                H = H2;
            }
            const int xl = o.x & ~(1 << H), yl = o.y & ~(1 << H);
            const int xh = xl | (1 << H), yh = yl | (1 << H);
            int jl = -1, jh = -1;
            for (int j = 0; j < OPS::N; j++) {
                if (done[j]) continue;
                if (ops.op[j].x == xl && ops.op[j].y == yl) jl = j;
                if (ops.op[j].x == xh && ops.op[j].y == yh) jh = j;
            }
            // jl, jh >= 0 by the symmetry of the op lists (checked in tests)
            done[jl] = true;
            done[jh] = true;
            const BOp lo = ops.op[jl], hi = ops.op[jh];
            SStep s{ST_OP, phys[xl], phys[yl], OP_FFTX, -1};
            if (lo.kind != OP_FFTX || hi.kind != OP_FFTX) {
                s.kind = lo.kind == OP_IFFT ? OP_IFFT : OP_FFT;
                const int slo = lo.kind == OP_FFTX ? -1 : lo.slot, shi = hi.kind == OP_FFTX ? -1 : hi.slot;
                if (slo != last_lo || shi != last_hi) {
                    tab_lo[ntab] = slo;
                    tab_hi[ntab] = shi;
                    ntab++;
                    last_lo = slo;
                    last_hi = shi;
                }
                s.tab = ntab - 1;
            }
            step[nsteps++] = s;
        }
        if (hfinal >= 0 && H != hfinal) {
            move_split(phys, half, H, hfinal);
            H = hfinal;
        }
        hend = H;
        for (int r = 0; r < M; r++) {
            fin_row[half[r]][phys[r]] = r;
            fin_phys[r] = phys[r];
            fin_half[r] = half[r];
        }
    }

   private:
    constexpr void move_split(int *phys, int *half, int H, int H2) {
        for (int r = 0; r < M; r++) {
            if ((r >> H) & 1 || (r >> H2) & 1) continue;
            const int r01 = r | (1 << H2), r10 = r | (1 << H);
            const int pa = phys[r], pb = phys[r01];
            step[nsteps++] = SStep{ST_SWAP, pa, pb, 0, -1};
            phys[r01] = pa;
            half[r01] = 1;
            phys[r10] = pb;
            half[r10] = 0;
        }
    }
};

// The encode pair: chunk IFFTs end in the split bit the FFT starts from, so
// the accumulator needs no re-layout between them.
template <int LOGM>
struct EncodeSplit {
    static constexpr SplitSched<FftOps<LOGM>, LOGM> fft_probe{-1, -1};
    static constexpr int HF = fft_probe.h0;
    static constexpr SplitSched<IfftOps<LOGM>, LOGM> ifft{-1, HF};
    // the FFT consumes the accumulator in the chunk IFFT's final layout
    static constexpr SplitSched<FftOps<LOGM>, LOGM> fft{HF, -1, ifft.fin_phys, ifft.fin_half};
};

}  // namespace rs
