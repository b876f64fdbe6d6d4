"""world_size-2 gloo tests of the byte-range sharded layout (CPU).

Each rank encodes / verifies / reconstructs only its 64-byte-aligned byte
range of every shard; the per-rank codec here is the oracle (test
infrastructure) so the partition and reassembly logic run without a GPU.
The assembled result must equal the whole-stripe oracle result."""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from reedsolomon16_amd import dist as rsd


def test_byte_range_partition():
    for S in (64, 128, 1 << 20, 256 << 10, 64 * 1001):
        for world in (1, 2, 3, 4, 8):
            spans = [rsd.byte_range(S, r, world) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == S
            for (a, b), (c, d) in zip(spans, spans[1:]):
                assert b == c and (b - a) % 64 == 0
            sizes = [b - a for a, b in spans]
            assert max(sizes) - min(sizes) <= 64
    with pytest.raises(ValueError):
        rsd.byte_range(100, 0, 2)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, bits, k, p, S, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import sys

    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from oracle import orc

    rng = np.random.default_rng(123)  # same stripe on every rank
    data = rng.integers(0, 256, (k, S), dtype=np.uint8)
    rows = np.zeros((k + p, S), np.uint8)
    rows[:k] = data

    def enc(loc):
        shards = [np.ascontiguousarray(loc[i]) for i in range(k + p)]
        assert orc.Oracle(bits, k, p).encode(shards) == 0
        loc[k:] = np.stack(shards[k:])

    def ver(loc):
        ok, e = orc.Oracle(bits, k, p).verify([np.ascontiguousarray(loc[i]) for i in range(k + p)])
        assert e == 0
        return ok

    def rec(loc, present):
        sh = [np.ascontiguousarray(loc[i]) if present[i] else None for i in range(k + p)]
        e, out = orc.Oracle(bits, k, p).reconstruct(sh, True)
        assert e == 0
        for i in range(k + p):
            loc[i] = out[i]

    rsd.encode_sharded(rows, rank, world, enc)
    lo, hi = rsd.byte_range(S, rank, world)
    # gather the parity slices on every rank (test-side assembly only)
    import torch

    mine = torch.from_numpy(np.ascontiguousarray(rows[k:, lo:hi]))
    parts = [None] * world
    dist.all_gather_object(parts, (lo, hi, mine.numpy()))
    full = np.zeros((p, S), np.uint8)
    for a, b, arr in parts:
        full[:, a:b] = arr
    ref = orc.encode(bits, k, p, data)
    good = bool(np.array_equal(full, ref))
    rows[k:] = full
    ok_all = rsd.verify_sharded(rows, rank, world, ver)
    tampered = rows.copy()
    if rank == world - 1:
        tampered[0, hi - 1] ^= 1  # a byte only the last rank owns
    bad_all = rsd.verify_sharded(tampered, rank, world, ver)
    # reconstruct p erased shards in every slice
    er = rng.choice(k + p, p, replace=False)
    present = np.ones(k + p, bool)
    present[er] = False
    broken = rows.copy()
    broken[er] = 0
    rsd.reconstruct_sharded(broken, present, rank, world, rec)
    rec_ok = bool(np.array_equal(broken[:, lo:hi], rows[:, lo:hi]))

    # batched layout: 2 stripes in one [n, k+p, S] slab, each rank's column
    # slice handed to the codec's batch entry points (a CPU stand-in here)
    class _CpuBatch:
        def encode_dev_batch(self, loc, stream=None):
            for z in range(loc.shape[0]):
                enc(loc[z].numpy())

        def reconstruct_dev_batch(self, loc, present, recover_all=True, stream=None):
            for z in range(loc.shape[0]):
                rec(loc[z].numpy(), present)

    datas = [np.random.default_rng(500 + z).integers(0, 256, (k, S), dtype=np.uint8) for z in range(2)]
    slab = torch.zeros((2, k + p, S), dtype=torch.uint8)
    for z in range(2):
        slab[z, :k] = torch.from_numpy(datas[z])
    rsd.encode_sharded_batch(slab, rank, world, _CpuBatch())
    refs = [orc.encode(bits, k, p, datas[z]) for z in range(2)]
    benc_ok = all(np.array_equal(slab[z, k:, lo:hi].numpy(), refs[z][:, lo:hi]) for z in range(2))
    full_b = slab.clone()
    for z in range(2):
        full_b[z, k:] = torch.from_numpy(refs[z])
    broken_b = full_b.clone()
    broken_b[:, torch.from_numpy(er)] = 0
    rsd.reconstruct_sharded_batch(broken_b, present, rank, world, _CpuBatch())
    brec_ok = bool(torch.equal(broken_b[:, :, lo:hi], full_b[:, :, lo:hi]))
    q.put((rank, good, ok_all, bad_all, rec_ok and benc_ok and brec_ok))
    dist.destroy_process_group()


@pytest.mark.parametrize("bits,k,p,S", [(16, 12, 4, 64 * 9), (8, 10, 4, 64 * 5), (16, 40, 20, 64 * 3)])
def test_two_rank_byte_range(bits, k, p, S):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, bits, k, p, S, q)) for r in range(2)]
    for pr in procs:
        pr.start()
    res = [q.get(timeout=120) for _ in procs]
    for pr in procs:
        pr.join(timeout=60)
        assert pr.exitcode == 0
    for rank, good, ok_all, bad_all, rec_ok in res:
        assert good, f"rank {rank}: assembled parity differs from the whole-stripe oracle"
        assert ok_all and not bad_all and rec_ok


@pytest.mark.parametrize("gpus,workload", [(2, "C3"), (4, "C5")])
def test_bench_launcher_starts_n_ranks(gpus, workload):
    """`bench.py --gpus N` without WORLD_SIZE starts N ranks itself (a
    torch.distributed.run child) and each rank asserts WORLD_SIZE == N; the
    gloo dry run reports every rank and their complementary byte ranges."""
    import json
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    out = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", str(gpus), "--dry-run",
                          "--workload", workload, "--cpu-seconds", "0.4", "--cpu-threads", "2"],
                         capture_output=True, text=True, timeout=240, env=env, cwd=root)
    assert out.returncode == 0, out.stderr[-2000:]
    line = [ln for ln in out.stdout.splitlines() if ln.startswith("{")][-1]
    res = json.loads(line)
    assert res["n_gpus"] == gpus and len(res["ranks"]) == gpus
    assert sorted(r["rank"] for r in res["ranks"]) == list(range(gpus))
    assert all(r["world"] == gpus for r in res["ranks"])
    spans = sorted(tuple(r["byte_range"]) for r in res["ranks"])
    S = {"C3": 1 << 20, "C5": 256 << 10}[workload]
    assert spans[0][0] == 0 and spans[-1][1] == S
    assert all(b == c for (_, b), (c, _) in zip(spans, spans[1:]))
    # the N-rank line carries the 1-rank line's evidence: traffic keyed by each
    # rank's launch shape, a per-rank roofline fraction, and the CPU baseline
    assert "traffic" in res["roofline"] and len(res["roofline"]["per_rank_traffic"]) == gpus
    for r in res["ranks"]:
        assert r["traffic_key"].endswith("x%d" % (r["byte_range"][1] - r["byte_range"][0]))
        # the default layout keeps the per-GPU work fixed: each rank's launch
        # covers its byte range of N x 256 stripes
        assert r["stripes_per_launch"] == 256 * gpus
    assert res["split"] == "bytes-weak" and res["scaling"] == "weak"
    assert len(res["per_rank_frac"]) == gpus
    cb = res["cpu_baseline"]
    assert cb["unit"] == "GiB/s" and cb["value"] > 0 and cb["kind"] == "port"
    # and a mismatched WORLD_SIZE is refused
    bad = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "3", "--dry-run"],
                         capture_output=True, text=True, timeout=120, env=dict(env, WORLD_SIZE="2", RANK="0"), cwd=root)
    assert bad.returncode != 0 and "WORLD_SIZE=2" in (bad.stderr + bad.stdout)
