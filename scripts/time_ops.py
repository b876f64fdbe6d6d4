"""Time device-resident codec operations with HIP events (kernel-side time,
launches back to back).  Prints one line per config."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

CONFIGS = {
    "C2": (8, 10, 4, 1 << 20, "encode"),
    "C3": (16, 128, 32, 1 << 20, "encode"),
    "C3v": (16, 128, 32, 1 << 20, "verify"),
    "C4": (16, 128, 32, 1 << 20, "reconstruct"),
    # few-erasure repair (the reference prunes its FFT below p/4 erasures): C4 geometry, e erased shards
    "C4e1": (16, 128, 32, 1 << 20, "reconstruct", 1, 1),
    "C4e2": (16, 128, 32, 1 << 20, "reconstruct", 1, 2),
    "C4e4": (16, 128, 32, 1 << 20, "reconstruct", 1, 4),
    "C4e8": (16, 128, 32, 1 << 20, "reconstruct", 1, 8),
    "C5": (16, 1024, 256, 256 << 10, "encode"),
    "C5x8": (16, 1024, 256, 32 << 10, "encode"),
    # C5 batched: 32 stripes per launch, whole rows and the 8-rank 32 KiB slice
    "C5b32": (16, 1024, 256, 256 << 10, "encode", 32),
    "C5x8b32": (16, 1024, 256, 32 << 10, "encode", 32),
    "C5vb32": (16, 1024, 256, 256 << 10, "verify", 32),
    # encode batches: stripes per launch (rs_encode_dev_batch), so a small
    # stripe's kernel time is not hidden behind the per-call host cost
    "C2x16": (8, 10, 4, 1 << 20, "encode", 16),
    "C3x16": (16, 128, 32, 1 << 20, "encode", 16),
    # one erasure pattern over 16 stripes in one launch (rs_reconstruct_dev_batch)
    "C4x16": (16, 128, 32, 1 << 20, "reconstruct", 16),
    "C3vx16": (16, 128, 32, 1 << 20, "verify", 16),
    # failing verify (every stripe corrupt): the flag path
    "C3vbadx16": (16, 128, 32, 1 << 20, "verify_bad", 16),
    # the C5-geometry repair (n = 2048 work rows: the multi-pass reconstruct),
    # 256 erasures, one stripe and one pattern over 8 stripes per launch
    "C5r": (16, 1024, 256, 256 << 10, "reconstruct"),
    "C5rb8": (16, 1024, 256, 256 << 10, "reconstruct", 8),
    # m = 512 / 1024 encodes (the reference's 1000- and 5000-shard tests' geometries, larger rows)
    "L512": (16, 700, 300, 256 << 10, "encode"),
    "L1024": (16, 4000, 1000, 64 << 10, "encode"),
    "L1024b4": (16, 4000, 1000, 64 << 10, "encode", 4),
    "L1024v": (16, 4000, 1000, 64 << 10, "verify"),
    "L2048": (16, 3000, 1500, 64 << 10, "encode"),
    "L4096": (16, 3000, 3000, 64 << 10, "encode"),
    "L512v": (16, 700, 300, 256 << 10, "verify"),
    "L2048v": (16, 3000, 1500, 64 << 10, "verify"),
    # n = 4096 reconstruct (3000 + 1000: 1000 erasures; 2100 + 10: 10 erasures)
    "R4096": (16, 3000, 1000, 64 << 10, "reconstruct"),
    "R4096e10": (16, 2100, 10, 256 << 10, "reconstruct"),
    # n = 8192 reconstruct (the reference's 4000 + 1000 at 64 KiB rows)
    "R8192": (16, 4000, 1000, 64 << 10, "reconstruct"),
}
# Host-resident (PCIe-inclusive) variants: shards in host memory, rs_encode /
# rs_reconstruct stream them through the GPU.  "p" = pinned rows (rs_host_alloc).
HOST_CONFIGS = {
    "H3": (16, 128, 32, 1 << 20, "encode", False),
    "H3p": (16, 128, 32, 1 << 20, "encode", True),
    "H4p": (16, 128, 32, 1 << 20, "reconstruct", True),
    # outputs rebuilt into the caller's pinned rows (EmptyShard, Go's shards[i][:0])
    "H4pc": (16, 128, 32, 1 << 20, "reconstruct_cap", True),
    "H3vp": (16, 128, 32, 1 << 20, "verify", True),
    # a stream of 8 stripes (pinned), encoded one call at a time (sync) or
    # queued with rs_encode_async and waited at the end (async)
    "H3s_sync": (16, 128, 32, 1 << 20, "stream_sync", True),
    "H3s_async": (16, 128, 32, 1 << 20, "stream_async", True),
    # the same stream verified (parity already written) or repaired (32 erasures
    # per block, rebuilt into the caller's pinned rows), sync vs tickets
    "H3vs_sync": (16, 128, 32, 1 << 20, "stream_verify_sync", True),
    "H3vs_async": (16, 128, 32, 1 << 20, "stream_verify_async", True),
    "H4s_sync": (16, 128, 32, 1 << 20, "stream_rec_sync", True),
    "H4s_async": (16, 128, 32, 1 << 20, "stream_rec_async", True),
}


def time_host(name, iters, tag):
    import time

    import numpy as np

    import reedsolomon16_amd as rs

    bits, k, p, S, op, pinned = HOST_CONFIGS[name]
    c = rs.ReedSolomon(k, p, bits)
    if op.startswith("stream"):
        nblk = 8
        blocks = []
        rng = np.random.default_rng(1)
        for _ in range(nblk):
            sh = c.alloc_aligned(S, pinned=True)
            for i in range(k):
                sh[i][:] = rng.integers(0, 256, S, dtype=np.uint8)
            blocks.append(sh)

        if op != "stream_sync" and op != "stream_async":
            for sh in blocks:
                c.encode(sh)
        erased = [set(rng.choice(k + p, p, replace=False).tolist()) for _ in range(nblk)]

        def rec_view(j):
            return [rs.EmptyShard(blocks[j][i]) if i in erased[j] else blocks[j][i] for i in range(k + p)]

        def run_stream():
            if op == "stream_sync":
                for sh in blocks:
                    c.encode(sh)
            elif op == "stream_async":
                ts = [c.encode_async(sh) for sh in blocks]
                for t in ts:
                    t.wait()
            elif op == "stream_verify_sync":
                for sh in blocks:
                    assert c.verify(sh)
            elif op == "stream_verify_async":
                ts = [c.verify_async(sh) for sh in blocks]
                assert all(t.result() for t in ts)
            elif op == "stream_rec_sync":
                for j in range(nblk):
                    c.reconstruct(rec_view(j))
            else:
                ts = [c.reconstruct_async(rec_view(j)) for j in range(nblk)]
                for t in ts:
                    t.wait()

        run_stream()
        t0 = time.perf_counter()
        for _ in range(iters):
            run_stream()
        us = (time.perf_counter() - t0) / iters / nblk * 1e6
        print(json.dumps({"tag": tag, "config": name, "op": op, "pinned": True, "us_per_stripe": round(us, 1),
                          "data_GiBps": round(k * S / us * 1e6 / 2**30, 2),
                          "pcie_GBps": round((k + p) * S / us / 1e3, 1)}), flush=True)
        return
    shards = c.alloc_aligned(S, pinned=pinned)
    rng = np.random.default_rng(1)
    for i in range(k):
        shards[i][:] = rng.integers(0, 256, S, dtype=np.uint8)
    c.encode(shards)
    er = set(rng.choice(k + p, p, replace=False).tolist())

    def run():
        if op == "encode":
            c.encode(shards)
        elif op == "verify":
            assert c.verify(shards)
        elif op == "reconstruct_cap":
            c.reconstruct([rs.EmptyShard(shards[i]) if i in er else shards[i] for i in range(k + p)])
        else:
            c.reconstruct([np.zeros(0, np.uint8) if i in er else shards[i] for i in range(k + p)])

    for _ in range(3):
        run()
    t0 = time.perf_counter()
    for _ in range(iters):
        run()
    us = (time.perf_counter() - t0) / iters * 1e6
    moved = (k + p) * S
    print(json.dumps({"tag": tag, "config": name, "op": op, "pinned": pinned, "us": round(us, 1),
                      "data_GiBps": round(k * S / us * 1e6 / 2**30, 2),
                      "pcie_GBps": round(moved / us / 1e3, 1)}), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="C3")
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--tag", default="")
    ap.add_argument("--knobs", default="", help="rs_debug_set_path knobs, e.g. rec_half=1,hp_tiles=4")
    a = ap.parse_args()
    import numpy as np
    import torch

    import reedsolomon16_amd as rs
    from reedsolomon16_amd import _capi

    for kv in filter(None, a.knobs.split(",")):
        kn, val = kv.split("=")
        _capi.set_path(kn, int(val))

    for name in a.configs.split(","):
        if name in HOST_CONFIGS:
            time_host(name, max(5, a.iters // 5), a.tag)
            continue
        bits, k, p, S, op = CONFIGS[name][:5]
        ns = CONFIGS[name][5] if len(CONFIGS[name]) > 5 else 1
        ne = CONFIGS[name][6] if len(CONFIGS[name]) > 6 else p
        c = rs.ReedSolomon(k, p, bits)
        slab = torch.randint(0, 256, (ns, k + p, S), dtype=torch.uint8, device="cuda")
        if op == "verify":  # the passing case; verify_bad times random (failing) stripes
            c.encode_dev_batch(slab)
        if op == "verify_bad":
            op = "verify"
        rows = slab[0]
        present = np.ones(k + p, bool)
        present[np.random.default_rng(0x5EED).choice(k + p, ne, replace=False)] = False

        st = torch.cuda.current_stream()

        def run():  # stream-ordered on the timing stream (verify reads its flag back)
            if op == "encode":
                c.encode_dev_batch(slab, st)
            elif op == "verify":
                c.verify_dev_batch(slab, st) if ns > 1 else c.verify_dev(rows, st)
            elif ns > 1:
                c.reconstruct_dev_batch(slab, present, stream=st)
            else:
                c.reconstruct_dev(rows, present, stream=st)

        for _ in range(5):
            run()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.iters):
            run()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / a.iters
        alg = ns * (k + p) * S
        print(json.dumps({"tag": a.tag, "knobs": a.knobs, "config": name, "op": op, "path": c.encode_path, "erased": int(ne) if op == "reconstruct" else 0,
                          "prune": os.environ.get("RS_NO_PRUNE", "0") != "1", "us": round(us, 2),
                          "GBps_alg": round(alg / us / 1e3, 1), "frac": round(alg / us / 1e3 / 8000, 4)}), flush=True)


if __name__ == "__main__":
    main()
