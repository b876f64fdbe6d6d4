"""Generate the golden fixtures in tests/golden/ (run from the repo root:
``python tests/golden/make_golden.py``).

The reference (Go) cannot be run here and holds no golden vectors of its own
(SURVEY.md §8c), so these vectors come from the oracle: the C restatement
(oracle/leopard_ref.c), each one cross-checked bit-for-bit against the
independent numpy restatement (oracle/leopard_np.py) before it is written.
They pin the GPU engine and any future change of either restatement.

Inputs follow the reference tests' own patterns where they exist
(``data[i] = i % 256``: simple_test.go:23-26, hybrid_test.go:23-26) plus
seeded random data (numpy default_rng) and the BASELINE.md special inputs.
Each .npz holds plain uint8/int arrays (no pickles); MANIFEST.sha256 lists
their digests.
"""
import hashlib
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from oracle import leopard_np as lnp  # noqa: E402
from oracle import orc  # noqa: E402

# (name, bits, k, p, S, data kind, erasure patterns)
CASES = [
    ("gf16_simple_4p2_mod256", 16, 4, 2, 256, "mod256", [[0, 5], [1], [4, 5]]),
    ("gf16_2p1", 16, 2, 1, 64, "rand", [[0], [2]]),
    ("gf16_10p4", 16, 10, 4, 256, "rand", [[0, 2, 10, 11], [3, 7, 9, 13]]),
    ("gf16_3p7_k_lt_m", 16, 3, 7, 64, "rand", [[0, 1, 2, 3, 4, 5, 6]]),
    ("gf16_37p9_tail_chunk", 16, 37, 9, 64, "rand", [[0, 8, 16, 24, 36, 37, 40, 45, 44]]),
    ("gf16_128p32", 16, 128, 32, 128, "rand", [list(range(0, 128, 4)), list(range(32))]),
    ("gf16_128p32_ff", 16, 128, 32, 64, "ones", [[5, 130]]),
    ("gf16_200p100", 16, 200, 100, 64, "rand", [list(range(0, 200, 2))]),
    ("gf16_1024p256", 16, 1024, 256, 64, "rand", [list(range(0, 1280, 5))]),
    ("gf8_10p4", 8, 10, 4, 256, "rand", [[0, 2, 10, 11], [1, 12]]),
    ("gf8_simple_4p2_mod256", 8, 4, 2, 256, "mod256", [[0, 5]]),
    ("gf8_100p28", 8, 100, 28, 64, "rand", [list(range(0, 100, 4))[:28]]),
    ("gf8_128p128", 8, 128, 128, 64, "rand", [list(range(0, 256, 2))]),
]


def make_data(kind, k, S, seed):
    if kind == "mod256":
        return (np.arange(k * S) % 256).astype(np.uint8).reshape(k, S)
    if kind == "ones":
        return np.full((k, S), 0xFF, np.uint8)
    return np.random.default_rng(seed).integers(0, 256, (k, S), dtype=np.uint8)


def build(write=True):
    out = {}
    for idx, (name, bits, k, p, S, kind, erasures) in enumerate(CASES):
        data = make_data(kind, k, S, 0x5EED + idx)
        parity = orc.encode(bits, k, p, data)
        ref = lnp.encode(bits, k, p, data)
        assert np.array_equal(parity, ref), f"{name}: C and numpy oracles disagree"
        full = [data[i] for i in range(k)] + [parity[i] for i in range(p)]
        er_mask = np.zeros((len(erasures), k + p), np.uint8)
        for j, er in enumerate(erasures):
            er_mask[j, er] = 1
            sh = [None if i in er else full[i].copy() for i in range(k + p)]
            e, got = orc.Oracle(bits, k, p).reconstruct(sh, True)
            assert e == 0 and all(np.array_equal(got[i], full[i]) for i in range(k + p)), f"{name}: reconstruct"
        out[name] = dict(bits=np.array([bits]), k=np.array([k]), p=np.array([p]), data=data, parity=parity,
                         erasures=er_mask)
        if write:
            np.savez_compressed(os.path.join(HERE, name + ".npz"), **out[name])
    if write:
        lines = []
        for name in sorted(out):
            h = hashlib.sha256(open(os.path.join(HERE, name + ".npz"), "rb").read()).hexdigest()
            lines.append(f"{h}  {name}.npz")
        open(os.path.join(HERE, "MANIFEST.sha256"), "w").write("\n".join(lines) + "\n")
    return out


if __name__ == "__main__":
    build()
    print("wrote", len(CASES), "fixtures")
