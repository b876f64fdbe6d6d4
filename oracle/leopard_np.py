"""ORACLE — TEST INFRASTRUCTURE ONLY.  Not part of the product.

Independent numpy restatement of the reference Leopard-FFT Reed-Solomon path
(bpfs/reedsolomon16 leopard16.go / leopard8.go).  It deliberately uses a
different formulation from oracle/leopard_ref.c so the two cross-check each
other:

* shards are decoded into SYMBOL arrays (GF(2^16): each 64-byte block holds 32
  symbols, lo bytes in [0:32), hi bytes in [32:64) — leopard16.go:778-792);
* multiplication is ``exp[addMod(log[x], log_m)]`` evaluated elementwise
  (mulLog, leopard16.go:828-838) instead of the Lo/Hi byte tables;
* the formal derivative uses its closed form
  ``out[r] = in[r] ^ XOR_{b: bit b of r == 0} in[r | 2^b]`` instead of the
  sequential loop at leopard16.go:527-530 (the two are equal because the loop
  only ever reads rows it has not yet written).

"Parity unpinned": the reference holds no golden vectors; this
module and the C oracle agree bit-for-bit and satisfy the reference tests'
round-trip properties.
"""
from __future__ import annotations

import numpy as np


class _Field:
    """Log/exp tables and FFT skew for GF(2^w), w in {8, 16}.

    Table construction follows initLUTs / initFFTSkew:
    GF(2^16) leopard16.go:940-1031, GF(2^8) leopard8.go:1034-1122.
    """

    def __init__(self, bits: int):
        self.bits = bits
        self.order = 1 << bits
        self.mod = self.order - 1
        if bits == 16:
            poly = 0x1002D
            cantor = [0x0001, 0xACCA, 0x3C0E, 0x163E, 0xC582, 0xED2E, 0x914C, 0x4012,
                      0x6C98, 0x10D8, 0x6A72, 0xB900, 0xFDB8, 0xFB34, 0xFF38, 0x991E]
        elif bits == 8:
            poly = 0x11D
            cantor = [1, 214, 152, 146, 86, 200, 88, 230]
        else:
            raise ValueError(bits)
        order, mod = self.order, self.mod
        dt = np.uint16 if bits == 16 else np.uint8
        # LFSR: lfsr_log[state] = i
        lfsr_log = np.zeros(order, dtype=np.int64)
        state = 1
        for i in range(mod):
            lfsr_log[state] = i
            state <<= 1
            if state >= order:
                state ^= poly
        lfsr_log[0] = mod
        # Cantor basis span: span[j] = XOR of basis[b] for set bits b of j
        span = np.zeros(order, dtype=np.int64)
        for i, b in enumerate(cantor):
            w = 1 << i
            span[w:2 * w] = span[:w] ^ b
        log = lfsr_log[span]
        exp = np.zeros(order, dtype=np.int64)
        exp[log] = np.arange(order)
        exp[mod] = exp[0]
        self.log = log.astype(dt)
        self.exp = exp.astype(dt)
        self._log = log
        self._exp = exp
        self._build_skew()

    # addMod / subMod with the partial reduction (leopard16.go:840-850)
    def add_mod(self, a, b):
        s = np.asarray(a, dtype=np.int64) + np.asarray(b, dtype=np.int64)
        return (s + (s >> self.bits)) & (self.order - 1)

    def sub_mod(self, a, b):
        # Go computes in uint (64-bit): for a < b the high part is all ones.
        a = np.asarray(a, dtype=np.int64)
        b = np.asarray(b, dtype=np.int64)
        d = a - b
        hi = np.where(d < 0, (1 << (64 - self.bits)) - 1, 0)  # (d mod 2^64) >> bits, low part irrelevant
        return (d + hi) & (self.order - 1)

    def mul_log(self, a, log_b):
        a = np.asarray(a, dtype=np.int64)
        r = self._exp[self.add_mod(self._log[a], log_b)]
        return np.where(a == 0, 0, r)

    def _fwht(self, data: np.ndarray, mtrunc: int) -> None:
        order = self.order
        dist, dist4 = 1, 4
        while dist4 <= order:
            # all groups r = 0, dist4, ... < mtrunc at once: view as (G, 4, dist)
            G = (mtrunc + dist4 - 1) // dist4
            v = data[:G * dist4].reshape(G, 4, dist)
            t0, t1, t2, t3 = v[:, 0].copy(), v[:, 1].copy(), v[:, 2].copy(), v[:, 3].copy()
            t0, t1 = self.add_mod(t0, t1), self.sub_mod(t0, t1)
            t2, t3 = self.add_mod(t2, t3), self.sub_mod(t2, t3)
            t0, t2 = self.add_mod(t0, t2), self.sub_mod(t0, t2)
            t1, t3 = self.add_mod(t1, t3), self.sub_mod(t1, t3)
            v[:, 0], v[:, 1], v[:, 2], v[:, 3] = t0, t1, t2, t3
            dist, dist4 = dist4, dist4 << 2

    def fwht(self, data: np.ndarray, mtrunc: int) -> None:
        self._fwht(data, mtrunc)

    def _build_skew(self):
        bits, mod = self.bits, self.mod
        temp = [1 << i for i in range(1, bits)]
        skew = np.zeros(mod, dtype=np.int64)
        for m in range(bits - 1):
            step = 1 << (m + 1)
            skew[(1 << m) - 1] = 0
            for i in range(m, bits - 1):
                s = 1 << (i + 1)
                j = np.arange((1 << m) - 1, s, step)
                skew[j + s] = skew[j] ^ temp[i]
            temp[m] = (mod - int(self._log[int(self.mul_log(temp[m], self._log[temp[m] ^ 1]))])) & mod
            for i in range(m + 1, bits - 1):
                ssum = int(self.add_mod(self._log[temp[i] ^ 1], temp[m]))
                temp[i] = int(self.mul_log(temp[i], ssum))
        self._skew = self._log[skew]
        walsh = self._log.copy()
        walsh[0] = 0
        self._fwht(walsh, self.order)
        self._walsh = walsh
        dt = np.uint16 if bits == 16 else np.uint8
        self.skew = self._skew.astype(dt)
        self.walsh = walsh.astype(dt)


_FIELDS: dict[int, _Field] = {}


def field(bits: int) -> _Field:
    if bits not in _FIELDS:
        _FIELDS[bits] = _Field(bits)
    return _FIELDS[bits]


def ceil_pow2(n: int) -> int:
    return 1 if n <= 1 else 1 << (n - 1).bit_length()


# ---------------------------------------------------------------------------
# Shard bytes <-> symbols
# ---------------------------------------------------------------------------
def to_symbols(rows: np.ndarray, bits: int) -> np.ndarray:
    """rows: (R, S) uint8 -> (R, S/2) int64 symbols for GF(2^16), (R, S) for GF(2^8)."""
    rows = np.asarray(rows, dtype=np.uint8)
    if bits == 8:
        return rows.astype(np.int64)
    R, S = rows.shape
    blk = rows.reshape(R, S // 64, 2, 32).astype(np.int64)
    return (blk[:, :, 0, :] | (blk[:, :, 1, :] << 8)).reshape(R, S // 2)


def from_symbols(sym: np.ndarray, bits: int) -> np.ndarray:
    if bits == 8:
        return sym.astype(np.uint8)
    R, n = sym.shape
    s = sym.reshape(R, n // 32, 32)
    out = np.empty((R, n // 32, 2, 32), dtype=np.uint8)
    out[:, :, 0, :] = s & 0xFF
    out[:, :, 1, :] = s >> 8
    return out.reshape(R, n * 2)


# ---------------------------------------------------------------------------
# Transforms over a symbol matrix W (rows x symbols)
# ---------------------------------------------------------------------------
def _ifft2(F, W, x, y, log_m):
    # ifftDIT2: y ^= x; x ^= y*m  (galois_noasm.go:72-76); log_m == mod: XOR only
    W[y] ^= W[x]
    if log_m != F.mod:
        W[x] ^= F.mul_log(W[y], log_m)


def _fft2(F, W, x, y, log_m):
    # fftDIT2: x ^= y*m; y ^= x (galois_noasm.go:58-62)
    if log_m != F.mod:
        W[x] ^= F.mul_log(W[y], log_m)
    W[y] ^= W[x]


def _ifft4(F, W, i, d, m01, m23, m02):
    # ifftDIT4Ref: leopard16.go:750-772
    _ifft2(F, W, i, i + d, m01)
    _ifft2(F, W, i + 2 * d, i + 3 * d, m23)
    _ifft2(F, W, i, i + 2 * d, m02)
    _ifft2(F, W, i + d, i + 3 * d, m02)


def _fft4(F, W, i, d, m01, m23, m02):
    # fftDIT4Ref: leopard16.go:660-682
    _fft2(F, W, i, i + 2 * d, m02)
    _fft2(F, W, i + d, i + 3 * d, m02)
    _fft2(F, W, i, i + d, m01)
    _fft2(F, W, i + 2 * d, i + 3 * d, m23)


def ifft_encoder(F, W, mtrunc, m, skew_off):
    """ifftDITEncoder transform part (leopard16.go:694-741); skew index = skew_off + j."""
    sk = F._skew
    dist, dist4 = 1, 4
    while dist4 <= m:
        for r in range(0, mtrunc, dist4):
            iend = r + dist
            m01, m02, m23 = (int(sk[skew_off + iend]), int(sk[skew_off + iend + dist]),
                             int(sk[skew_off + iend + 2 * dist]))
            for i in range(r, iend):
                _ifft4(F, W, i, dist, m01, m23, m02)
        dist, dist4 = dist4, dist4 << 2
    if dist < m:
        logm = int(sk[skew_off + dist])
        for i in range(dist):
            _ifft2(F, W, i, i + dist, logm)


def ifft_decoder(F, W, mtrunc, m):
    """ifftDITDecoder (leopard16.go:573-615)."""
    sk = F._skew
    dist, dist4 = 1, 4
    while dist4 <= m:
        for r in range(0, mtrunc, dist4):
            iend = r + dist
            m01, m02, m23 = int(sk[iend - 1]), int(sk[iend + dist - 1]), int(sk[iend + 2 * dist - 1])
            for i in range(r, iend):
                _ifft4(F, W, i, dist, m01, m23, m02)
        dist, dist4 = dist4, dist4 << 2
    if dist < m:
        logm = int(sk[dist - 1])
        for i in range(dist):
            _ifft2(F, W, i, i + dist, logm)


def fft(F, W, mtrunc, m):
    """fftDIT (leopard16.go:618-657)."""
    sk = F._skew
    dist4, dist = m, m >> 2
    while dist != 0:
        for r in range(0, mtrunc, dist4):
            iend = r + dist
            m01, m02, m23 = int(sk[iend - 1]), int(sk[iend + dist - 1]), int(sk[iend + 2 * dist - 1])
            for i in range(r, iend):
                _fft4(F, W, i, dist, m01, m23, m02)
        dist4, dist = dist, dist >> 2
    if dist4 == 2:
        for r in range(0, mtrunc, 2):
            _fft2(F, W, r, r + 1, int(sk[r]))


def encode(bits: int, k: int, p: int, data: np.ndarray) -> np.ndarray:
    """Systematic parity for data (k, S) uint8 -> (p, S) uint8 (leopard16.go:128-224)."""
    F = field(bits)
    D = to_symbols(data, bits)
    m = ceil_pow2(p)
    acc = np.zeros((m, D.shape[1]), dtype=np.int64)
    off = 0
    base = m - 1
    first = True
    while off < k:
        cnt = min(m, k - off)
        W = np.zeros((m, D.shape[1]), dtype=np.int64)
        W[:cnt] = D[off:off + cnt]
        ifft_encoder(F, W, cnt, m, base)
        if first:
            acc = W
            first = False
        else:
            acc ^= W
        off += m
        base += m
    fft(F, acc, p, m)
    return from_symbols(acc[:p], bits)


def formal_derivative(W, n):
    out = W.copy()
    for r in range(n):
        b = 0
        while (1 << b) < n:
            if not (r >> b) & 1:
                out[r] ^= W[r | (1 << b)]
            b += 1
    return out


def error_locators(bits: int, k: int, p: int, erased: np.ndarray) -> np.ndarray:
    """errLocs after the two FWHTs (leopard16.go:433-470). erased: bool (k+p,), data first."""
    F = field(bits)
    m = ceil_pow2(p)
    e = np.zeros(F.order, dtype=np.int64)
    for i in range(p):
        if erased[k + i]:
            e[i] = 1
    e[p:m] = 1
    for i in range(k):
        if erased[i]:
            e[i + m] = 1
    F.fwht(e, m + k)
    e = (e * F._walsh) % F.mod
    F.fwht(e, F.order)
    return e


def reconstruct(bits: int, k: int, p: int, shards: list, recover_all: bool = True) -> dict:
    """Return {index: recovered bytes} for missing shards (None entries), leopard16.go:390-570."""
    F = field(bits)
    total = k + p
    erased = np.array([s is None for s in shards])
    S = next(len(s) for s in shards if s is not None)
    m = ceil_pow2(p)
    n = ceil_pow2(m + k)
    el = error_locators(bits, k, p, erased)
    nsym = S // 2 if bits == 16 else S
    W = np.zeros((n, nsym), dtype=np.int64)
    for i in range(p):
        if not erased[k + i]:
            W[i] = F.mul_log(to_symbols(np.asarray(shards[k + i])[None], bits)[0], int(el[i]))
    for i in range(k):
        if not erased[i]:
            W[m + i] = F.mul_log(to_symbols(np.asarray(shards[i])[None], bits)[0], int(el[m + i]))
    ifft_decoder(F, W, m + k, n)
    W = formal_derivative(W, n)
    fft(F, W, m + k, n)
    out = {}
    end = total if recover_all else k
    for i in range(end):
        if not erased[i]:
            continue
        if i >= k:
            sym = F.mul_log(W[i - k], F.mod - int(el[i - k]))
        else:
            sym = F.mul_log(W[i + m], F.mod - int(el[i + m]))
        out[i] = from_symbols(sym[None], bits)[0]
    return out
