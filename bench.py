"""Headline benchmark: device-resident GF(2^16) encode (BASELINE.json metric),
128 data + 32 parity x 1 MiB shards (configs[2] / C3) by default, or
1024 + 256 x 256 KiB (configs[4] / C5) with --workload C5.

A step encodes B synthetic stripes (--stripes, default 256: 40 GiB of C3
stripes resident, a small fraction of the 288 GB HBM) already resident in HBM,
in one kernel launch per rank (rs_encode_dev_batch).  Larger batches amortise
the grid's fill and drain, which weighs most on the small per-rank slices of
a byte-range split: on one box the 8-rank slice (128 KiB of every row) ran at
0.608 / 0.624 / 0.627 of the HBM roofline for 128 / 256 / 512 stripes per
launch, the 2-rank slice at 0.640 for 128 and 256, full rows at 0.652 / 0.650
for 128 / 256 (profiles/r04_batch_slices.txt).

Multi-GPU (one process per GPU).  Under torch.distributed.run (WORLD_SIZE set)
every rank checks WORLD_SIZE == --gpus.  Started directly with --gpus N > 1,
the parent launches `python -m torch.distributed.run --nproc-per-node N` on
this same command line before it imports torch or touches a GPU, and exits
with the child's return code.  --dry-run runs the rank layout with gloo on the
CPU (no GPU): each rank reports its byte range.  Every layout runs without a
collective on the data path (column independence, leopard16.go:778-792):
  --split bytes-weak  (default, round 6) the north-star layout with the
                  per-GPU work fixed: the job is N*B stripes and rank r owns
                  the byte range dist.byte_range(S, r, N) of every shard of
                  all of them, so each rank's launch moves the bytes of B
                  whole stripes (N*B stripes x S/N bytes) as N grows ->
                  "scaling": "weak"; value = N*B*k*S data bytes / max-over-
                  ranks wall time.  At N = 1 it is the one-GPU line.
  --split bytes   the same byte ranges of a fixed B stripes: total work fixed
                  as N grows -> "strong" (each rank's launch shrinks N-fold;
                  the 8-rank slice of 256 stripes runs 0.60-0.66 of the
                  roofline against 0.67-0.69 at 2048 stripes).
  --split stripes each rank encodes B whole stripes of its own -> "weak".

Prints one JSON line (rank 0).  `roofline` is for the dominant (only) kernel:
achieved = algorithmic bytes per launch ((k+p)*bytes-per-row: read k rows,
write p rows) / its mean duration (one HIP event pair on the launch stream
around the timed launches, divided by their count).  `single_stripe` repeats
the kernel timing with one stripe per launch (the reference's Encode
granularity).  Resident rows sit at a stride of row bytes + --row-pad (3.5 KiB
by default); `unpadded_rows` times the same launch on rows
packed exactly one row length apart.  `other_workloads` (one GPU) reports the
kernel time and roofline fraction of the C2 encode, the C4 reconstruct and
the C5 encode and repair beside the headline; `host_resident` the
PCIe-inclusive rates with the shards in host memory (the engine's tickets and
the rsStream16 mirror at 4 MiB blocks).  `cpu_baseline` times the reference-equivalent AVX2 and AVX-512 ports of the
encode (oracle/leopard_ref.c, test/bench infrastructure) on a bounded sample:
1 thread (the reference is single-threaded per call) and N threads over byte
ranges.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

WORKLOADS = {"C3": (128, 32, 1 << 20), "C5": (1024, 256, 256 << 10)}
PEAK_HBM_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md)


def cpu_baseline(K, P, S, seconds: float, threads: int):
    """Reference-equivalent SIMD ports (oracle/leopard_ref.c orc16_encode_simd_isa:
    AVX2 like ifftDIT4_avx2, AVX-512 like ifftDIT4_avx512_*), same geometry,
    one stripe per call, each ISA the CPU runs at 1 thread and N threads;
    `value` is the widest ISA at N threads (the reference picks the widest,
    galois_amd64.go:192).  Scalar Ref oracle if AVX2 is absent."""
    import numpy as np

    from oracle import orc

    rng = np.random.default_rng(0x5EED)
    data = rng.integers(0, 256, (K, S), dtype=np.uint8)
    par = np.zeros((P, S), np.uint8)
    isas = orc.simd_isas()

    def rate(isa, th, budget):
        def run():
            if isa:
                orc.encode_simd(K, P, data, th, par, isa=isa)
            else:
                orc.encode(16, K, P, data)

        run()  # warm (tables, page faults)
        n, t0 = 0, time.perf_counter()
        while True:
            run()
            n += 1
            el = time.perf_counter() - t0
            if el >= budget:
                return n, el

    if not isas:
        n1, el1 = rate(None, 1, seconds)
        v = round(n1 * K * S / el1 / 2**30, 4)
        return {"value": v, "unit": "GiB/s", "cores": 1, "kind": "port", "isa": "scalar", "single_thread": v,
                "sample": f"{K}+{P} x {S >> 10} KiB stripe, scalar Ref oracle, {n1} encodes on 1 thread in {el1:.1f} s"}
    budget = seconds / (2 * len(isas))
    by_isa, notes = {}, []
    for isa in isas:
        n1, el1 = rate(isa, 1, budget)
        e = {"kind": "port", "isa": isa, "single_thread": round(n1 * K * S / el1 / 2**30, 4)}
        note = f"{isa}: {n1} encodes on 1 thread in {el1:.1f} s"
        if threads > 1:
            nN, elN = rate(isa, threads, budget)
            e["threads"] = threads
            e["value"] = round(nN * K * S / elN / 2**30, 4)
            note += f", {nN} on {threads} threads (byte ranges) in {elN:.1f} s"
        else:
            e["value"] = e["single_thread"]
        by_isa[isa] = e
        notes.append(note)
    top = by_isa[isas[-1]]
    return {"value": top["value"], "unit": "GiB/s", "cores": threads if threads > 1 else 1, "kind": "port",
            "isa": top["isa"], "single_thread": top["single_thread"], "by_isa": by_isa,
            "sample": (f"{K}+{P} x {S >> 10} KiB stripe, nibble-table ports of the reference encode "
                       f"(oracle/leopard_ref.c, -O3; AVX-512 = VL + VPTERNLOGD like ifftDIT4_avx512_*): "
                       + "; ".join(notes))}


def traffic_key(workload: str, kernel_name: str, stripes: int, row_bytes: int) -> str:
    """profiles/pmc_traffic.json key: the launch shape one rank runs (its
    stripes per launch and bytes of every row, i.e. its byte-range slice)."""
    return f"{workload}:{kernel_name}:{stripes}x{row_bytes}"


def load_traffic(kernel_name: str, workload: str, stripes: int, row_bytes: int, shard_bytes: int):
    """HBM bytes per launch from the committed rocprofv3 PMC summary
    (profiles/pmc_traffic.json, scripts/collect_profiles.py), if it was taken
    for this workload, batch size and per-rank row slice."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            d = json.load(f)
    except Exception:
        return None
    e = d.get(traffic_key(workload, kernel_name, stripes, row_bytes))
    if e is None and row_bytes == shard_bytes:  # entries written before the per-slice keys
        e = d.get(f"{workload}:{kernel_name}") or (d.get(kernel_name) if workload == "C3" else None)
        if e and e.get("stripes", 16) != stripes:
            e = None
    return e.get("hbm_bytes_per_launch") if e else None


def device_info(torch, dev) -> dict:
    """What the runtime reports about the GPU the line was measured on (C3's
    rate differs by up to 0.08 of the roofline between boxes with the same
    code)."""
    p = torch.cuda.get_device_properties(dev)
    out = {"name": p.name, "cus": p.multi_processor_count, "hbm_bytes": p.total_memory}
    for a in ("gcnArchName", "L2_cache_size", "pci_bus_id", "uuid"):
        v = getattr(p, a, None)
        if v is not None:
            out[a] = str(v) if a == "uuid" else v
    return out


def copy_rate(torch, dev, stream) -> float:
    """This box's torch device-to-device copy rate (GB/s of bytes read +
    written, 2 GiB tensor copies on the launch stream): a reference for
    comparing C3 lines from different boxes.  torch's copy
    kernel does not reach the HBM peak, so this is not a ceiling."""
    n = 1 << 31
    a = torch.empty(n, dtype=torch.uint8, device=dev)
    b = torch.empty(n, dtype=torch.uint8, device=dev)
    a.fill_(1)
    with torch.cuda.stream(stream):
        for _ in range(3):
            b.copy_(a)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(10):
            b.copy_(a)
        e1.record(stream)
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 10
    del a, b
    torch.cuda.empty_cache()
    return 2 * n / (ms * 1e-3) / 1e9


def other_workloads(torch, rs, dev, stream) -> dict:
    """Kernel time of the other BASELINE configs on this GPU, beside the
    headline (reported, not the metric): C4 = reconstruct of 128+32 x 1 MiB
    with 32 erased shards, 16 stripes per launch (rs_reconstruct_dev_batch);
    C5 = encode of 1024+256 x 256 KiB, 32 stripes per launch, and its repair
    with 256 erased shards, 8 stripes per launch.  Algorithmic bytes: rows
    read + rows written per stripe (C4: 128 + 32, C5: 1024 + 256)."""
    import numpy as np

    out = {}
    g = torch.Generator(device=dev)
    g.manual_seed(0xC4C5)

    def kernel_ms(fn, n):
        for _ in range(3):
            fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record(stream)
        for _ in range(n):
            fn()
        e1.record(stream)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / n

    k, p, S, ns = 128, 32, 1 << 20, 16
    c4 = rs.New16(k, p, device=dev.index)
    slab = torch.randint(0, 256, (ns, k + p, S), dtype=torch.uint8, device=dev, generator=g)
    c4.encode_dev_batch(slab, stream)
    present = np.ones(k + p, bool)
    present[np.random.default_rng(0x5EED).choice(k + p, p, replace=False)] = False
    ms = kernel_ms(lambda: c4.reconstruct_dev_batch(slab, present, stream=stream), 20)
    alg = ns * (k + p) * S
    out["C4_reconstruct"] = {"config": "128+32 x 1024 KiB, 32 erased shards, 16 stripes per launch",
                             "kernel_ms": round(ms, 5), "us_per_stripe": round(ms * 1e3 / ns, 2),
                             "alg_bytes_per_launch": alg, "frac": round(alg / (ms * 1e-3) / 1e9 / PEAK_HBM_GBS, 4)}
    del slab
    k, p, S, ns = 1024, 256, 256 << 10, 32
    c5 = rs.New16(k, p, device=dev.index)
    slab = torch.randint(0, 256, (ns, k + p, S), dtype=torch.uint8, device=dev, generator=g)
    ms = kernel_ms(lambda: c5.encode_dev_batch(slab, stream), 10)
    alg = ns * (k + p) * S
    out["C5_encode"] = {"config": "1024+256 x 256 KiB, 32 stripes per launch", "kernel_path": c5.encode_path,
                        "kernel_ms": round(ms, 5), "us_per_stripe": round(ms * 1e3 / ns, 2),
                        "alg_bytes_per_launch": alg, "frac": round(alg / (ms * 1e-3) / 1e9 / PEAK_HBM_GBS, 4)}
    # C5 is the north star's 8-GPU byte-range config: one rank's launch holds
    # its 32 KiB slice of every row (dist.byte_range), 32 stripes
    from reedsolomon16_amd import dist as rsd

    lo, hi = rsd.byte_range(S, 0, 8)
    sl = torch.randint(0, 256, (ns, k + p, hi - lo), dtype=torch.uint8, device=dev, generator=g)
    ms = kernel_ms(lambda: c5.encode_dev_batch(sl, stream), 20)
    alg = ns * (k + p) * (hi - lo)
    out["C5_encode_rank_of_8"] = {"config": f"1024+256 x 256 KiB split over 8 ranks: rank 0's {hi - lo} bytes of every row, "
                                            f"{ns} stripes per launch", "kernel_ms": round(ms, 5),
                                  "us_per_stripe": round(ms * 1e3 / ns, 2), "alg_bytes_per_launch": alg,
                                  "frac": round(alg / (ms * 1e-3) / 1e9 / PEAK_HBM_GBS, 4)}
    del sl
    # the C5 repair: 256 erased shards (n = 2048 work rows), 8 stripes of the slab
    ns = 8
    c5.encode_dev_batch(slab[:ns], stream)
    present = np.ones(k + p, bool)
    present[np.random.default_rng(0xC5).choice(k + p, p, replace=False)] = False
    ms = kernel_ms(lambda: c5.reconstruct_dev_batch(slab[:ns], present, stream=stream), 5)
    alg = ns * (k + p) * S
    out["C5_reconstruct"] = {"config": "1024+256 x 256 KiB, 256 erased shards, 8 stripes per launch",
                             "kernel_ms": round(ms, 5), "us_per_stripe": round(ms * 1e3 / ns, 2),
                             "alg_bytes_per_launch": alg, "frac": round(alg / (ms * 1e-3) / 1e9 / PEAK_HBM_GBS, 4)}
    del slab
    torch.cuda.empty_cache()
    return out


def c2_encode(torch, rs, dev, stream) -> dict:
    """C2 (BASELINE configs[1]): GF(2^8) encode of 10 + 4 x 1 MiB
    (leopard8.go:153-277), one stripe per launch and 16 stripes per launch
    (rs_encode_dev_batch), HIP-event kernel time on the launch stream.
    Algorithmic bytes (k + p) * S per stripe."""
    k, p, S = 10, 4, 1 << 20
    g = torch.Generator(device=dev)
    g.manual_seed(0xC2)
    import time

    from reedsolomon16_amd.codec import _stream_handle

    c2 = rs.New8(k, p, device=dev.index)
    slab = torch.randint(0, 256, (16, k + p, S), dtype=torch.uint8, device=dev, generator=g)
    out = {"config": "10+4 x 1024 KiB, GF(2^8)", "kernel_path": c2.encode_path,
           "caller": "rs_encode_dev_batch through ctypes with prebuilt arguments (a C or cgo caller's "
                     "per-call cost; the Python wrapper's own argument checks are not timed)"}
    fn = rs.lib().rs_encode_dev_batch
    for ns, reps in ((1, 400), (16, 100)):
        view = slab[:ns]
        args = (c2._h, view.data_ptr(), view.stride(1), view.stride(0), ns, S, _stream_handle(stream))
        for _ in range(10):
            assert fn(*args) == 0
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record(stream)
        t0 = time.perf_counter()
        for _ in range(reps):
            fn(*args)
        t1 = time.perf_counter()
        e1.record(stream)
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / reps
        alg = ns * (k + p) * S
        out[f"stripes_{ns}"] = {"kernel_ms": round(ms, 5), "us_per_stripe": round(ms * 1e3 / ns, 3),
                                "host_us_per_call": round((t1 - t0) * 1e6 / reps, 3),
                                "alg_bytes_per_launch": alg,
                                "frac": round(alg / (ms * 1e-3) / 1e9 / PEAK_HBM_GBS, 4)}
    del slab
    return out


class _ArrayReader:
    """io.Reader over a numpy byte array (readinto copies, as io.ReadFull does)."""

    def __init__(self, a):
        self.a, self.off = a, 0

    def readinto(self, b):
        n = min(len(b), len(self.a) - self.off)
        if n <= 0:
            return 0
        import numpy as np

        # a numpy copy, which drops the GIL like a file's readinto does
        np.copyto(np.frombuffer(b, np.uint8, n), self.a[self.off:self.off + n])
        self.off += n
        return n


class _ArrayWriter:
    """io.Writer into a preallocated numpy byte array."""

    def __init__(self, a):
        self.a, self.off = a, 0

    def write(self, b):
        import numpy as np

        n = len(b)
        np.copyto(self.a[self.off:self.off + n], np.frombuffer(b, np.uint8, n))
        self.off += n
        return n


def host_resident(rs, blocks: int = 2, block: int = 4 << 20) -> dict:
    """The north star's host-resident rate (PCIe-inclusive; never `value`):
    128 + 32 shards in host memory, rsStream16's 4 MiB blocks.
      tickets: the engine's async host entry points on pinned blocks
               (rs_encode_async / rs_verify_async / rs_reconstruct_async,
               32 erasures into pinned EmptyShard rows), `blocks` stripes
               queued back to back -- the codec side of the stream loop;
      stream:  the rsStream16 mirror (reedsolomon16_amd/stream.py
               StreamEncoder16, streaming16.go:200-468,1229-1318) over
               in-memory readers and writers, so io.ReadFull's copy into the
               block buffer and the output writes are inside the time.
    data GiB/s = k * bytes per shard / time; PCIe GB/s = bytes crossing the
    link / time (encode: k in + p out, verify: k + p in, reconstruct:
    present in + rebuilt out)."""
    import numpy as np

    from reedsolomon16_amd.stream import StreamEncoder16

    K, P = 128, 32
    L = blocks * block
    codec = rs.New16(K, P)
    rng = np.random.default_rng(0x5EED)
    data = rs.alloc_pinned(K * L).reshape(K, L)
    data[:] = rng.integers(0, 256, data.shape, dtype=np.uint8)
    par = rs.alloc_pinned(P * L).reshape(P, L)
    erased = sorted(np.random.default_rng(0xC4).choice(K + P, P, replace=False).tolist())
    out = {"config": f"{K}+{P} shards, {blocks} blocks of {block >> 20} MiB per shard, {len(erased)} erasures"}

    def rate(op, t, read_rows, write_rows):
        return {"ms": round(t * 1e3, 3), "data_gib_s": round(K * L / t / 2**30, 3),
                "pcie_gb_s": round((read_rows + write_rows) * L / t / 1e9, 3)}

    # ---- tickets on pinned blocks
    rows = [[data[i, b * block:(b + 1) * block] for i in range(K)] +
            [par[j, b * block:(b + 1) * block] for j in range(P)] for b in range(blocks)]

    def enc():
        ts = [codec.encode_async(r) for r in rows]
        for t in ts:
            t.wait()

    def ver():
        ts = [codec.verify_async(r) for r in rows]
        assert all(t.result() for t in ts)

    rebuilt = rs.alloc_pinned(len(erased) * block * blocks).reshape(blocks, len(erased), block)

    def rec():
        ts = []
        for b, r in enumerate(rows):
            sh = list(r)
            for j, i in enumerate(erased):
                sh[i] = rs.EmptyShard(rebuilt[b, j])
            ts.append(codec.reconstruct_async(sh, True))
        for t in ts:
            t.wait()

    def tickets():
        tick = {}
        for name, fn, rd, wr in (("encode", enc, K, P), ("verify", ver, K + P, 0),
                                 ("reconstruct", rec, K + P - len(erased), len(erased))):
            fn()  # warm: plans, staging buffers
            t0 = time.perf_counter()
            fn()
            tick[name] = rate(name, time.perf_counter() - t0, rd, wr)
        for j, i in enumerate(erased):
            src = data[i] if i < K else par[i - K]
            assert all(np.array_equal(rebuilt[b, j], src[b * block:(b + 1) * block]) for b in range(blocks))
        return tick

    out["tickets"] = tickets()
    # the same tickets on a multi-device codec of four parts on this one GPU
    # (rs_new_multi, devices = [d, d, d, d]): the cost of the byte-range
    # fan-out over per-part host threads and streams, sharing one PCIe link
    # (an 8-GPU node's parts each own a link; not measurable on this box)
    one = codec
    codec = rs.New16(K, P, devices=[one.device] * 4)
    out["tickets_parts4_one_gpu"] = tickets()
    codec.close()
    codec = one

    # ---- the rsStream16 mirror over readers / writers: the reference's
    # sequential loops, and the same loops with a block's readers and writers
    # on 8 threads (StreamEncoder16(threads=8); same bytes, stream.py)
    sink = np.empty((P, L), np.uint8)
    rsink = np.empty((len(erased), L), np.uint8)
    for threads in (1, 8):
        out["stream" if threads == 1 else f"stream_threads{threads}"] = _stream_rates(
            StreamEncoder16(K, P, block_size=block, codec=codec, threads=threads), data, par, sink, rsink, erased, K, P,
            rate)
    assert np.array_equal(sink, par)
    return out


def _stream_rates(st, data, par, sink, rsink, erased, K, P, rate) -> dict:
    stream_rates = {}

    def s_enc():
        st.encode([_ArrayReader(data[i]) for i in range(K)], [_ArrayWriter(sink[j]) for j in range(P)])

    def s_ver():
        assert st.verify([_ArrayReader(data[i]) for i in range(K)] + [_ArrayReader(par[j]) for j in range(P)])

    def s_rec():
        ins = [None if i in erased else _ArrayReader(data[i] if i < K else par[i - K]) for i in range(K + P)]
        outs = [None] * (K + P)
        for j, i in enumerate(erased):
            outs[i] = _ArrayWriter(rsink[j])
        st.reconstruct(ins, outs)

    for name, fn, rd, wr in (("encode", s_enc, K, P), ("verify", s_ver, K + P, 0),
                             ("reconstruct", s_rec, K + P - len(erased), len(erased))):
        fn()
        t0 = time.perf_counter()
        fn()
        stream_rates[name] = rate(name, time.perf_counter() - t0, rd, wr)
    return stream_rates


def free_port() -> int:
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n: int) -> int:
    """Start n ranks of this command under torch.distributed.run (a child
    process: nothing in this process has touched the GPU) and return its rc."""
    import subprocess

    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={free_port()}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


def rank_stripes(args, world: int) -> int:
    """Stripes in one rank's launch: the byte range of N*B stripes (bytes-weak,
    and --slice-of N: the launch shape of one of its ranks), else B."""
    n = args.slice_of if args.slice_of > 1 else world
    return args.stripes * n if args.split == "bytes-weak" else args.stripes


def scaling_of(args) -> str:
    return "strong" if args.split == "bytes" else "weak"


def dry_run(args, rank: int, world: int) -> None:
    """The rank layout without a GPU: gloo process group, each rank's byte
    range of the workload's shards, gathered on rank 0 and printed as JSON."""
    import torch.distributed as dist

    from reedsolomon16_amd import dist as rsd

    if "WORLD_SIZE" in os.environ:
        dist.init_process_group("gloo")
    else:
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{free_port()}", rank=0, world_size=1)
    K, P, S = WORKLOADS[args.workload]
    lo, hi = rsd.byte_range(S, rank, world) if args.split != "stripes" else (0, S)
    br = rank_stripes(args, world)
    kname = "bs16-m32" if args.workload == "C3" else "lds-m256"  # the engine's path for the workload (rs_encode_path)
    got = [None] * world
    dist.all_gather_object(got, {"rank": rank, "byte_range": [lo, hi], "world": dist.get_world_size(),
                                 "stripes_per_launch": br,
                                 "traffic_key": traffic_key(args.workload, kname, br, hi - lo),
                                 "traffic": load_traffic(kname, args.workload, br, hi - lo, S)})
    if rank == 0:
        threads = args.cpu_threads or min(16, os.cpu_count() or 1)
        print(json.dumps({"dry_run": True, "n_gpus": world, "gpus_requested": args.gpus, "workload": args.workload,
                          "split": args.split, "scaling": scaling_of(args), "ranks": got,
                          # the evidence keys of a real N-rank line (kernel times need a GPU)
                          "roofline": {"traffic": got[0]["traffic"], "traffic_key": got[0]["traffic_key"],
                                       "per_rank_traffic": [r["traffic"] for r in got]},
                          "per_rank_frac": [None] * world,
                          "cpu_baseline": None if args.no_cpu else cpu_baseline(K, P, S, args.cpu_seconds, threads)}),
              flush=True)
    dist.barrier()
    dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--workload", choices=sorted(WORKLOADS), default="C3")
    ap.add_argument("--split", choices=["bytes-weak", "bytes", "stripes"], default="bytes-weak",
                    help="multi-GPU layout: byte ranges of N x --stripes stripes (weak, default), byte ranges of "
                         "--stripes stripes (strong), or whole stripes per rank (weak)")
    ap.add_argument("--stripes", type=int, default=256, help="stripes encoded per step (one launch per rank)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--cpu-threads", type=int, default=0, help="0: min(16, os.cpu_count())")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-single", action="store_true", help="skip the one-stripe-per-launch figure")
    ap.add_argument("--row-pad", type=int, default=3584,
                    help="bytes between consecutive resident rows (HBM layout: row stride = row bytes + pad; "
                         "64-byte multiple); the unpadded layout is timed too and reported beside it")
    ap.add_argument("--no-unpadded", action="store_true", help="skip timing the unpadded layout")
    ap.add_argument("--dry-run", action="store_true", help="rank layout only: gloo on the CPU, no GPU")
    ap.add_argument("--no-other", action="store_true", help="skip the C4 / C5 kernel figures (one GPU only)")
    ap.add_argument("--no-host", action="store_true", help="skip the host-resident (PCIe-inclusive) figures")
    ap.add_argument("--backend", choices=["nccl", "gloo"], default="nccl",
                    help="process group of an N-rank run: nccl (RCCL, one GPU per rank, the product) or gloo "
                         "(a rehearsal of the same rank code on fewer GPUs than ranks: rank r uses GPU r %% count)")
    ap.add_argument("--slice-of", type=int, default=0,
                    help="one GPU: encode rank 0's byte range of an N-rank split (the launch shape each rank of an "
                         "N-GPU run has, for its rocprofv3 PMC passes); not a job-throughput figure")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus))  # before any GPU call in this process
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: WORLD_SIZE={world} but --gpus {args.gpus}")
    if args.dry_run:
        dry_run(args, rank, world)
        return

    import torch
    import torch.distributed as dist

    import reedsolomon16_amd as rs
    from reedsolomon16_amd import dist as rsd

    if world > 1 and args.backend == "gloo":
        torch.cuda.set_device(local % max(1, torch.cuda.device_count()))
        dist.init_process_group("gloo")
    elif world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", torch.cuda.current_device())

    K, P, S = WORKLOADS[args.workload]
    B = rank_stripes(args, world)  # stripes in this rank's launch
    if args.slice_of > 1:
        if world != 1:
            raise SystemExit("--slice-of is a one-GPU measurement")
        lo, hi = rsd.byte_range(S, 0, args.slice_of)
    elif args.split != "stripes":
        lo, hi = rsd.byte_range(S, rank, world)
    else:
        lo, hi = 0, S
    W = hi - lo  # bytes of each row this rank holds and encodes
    codec = rs.New16(K, P, device=dev.index)
    g = torch.Generator(device=dev)
    g.manual_seed(0x5EED + rank)
    # this rank's resident bytes: B stripes x (k+p) rows x W bytes (its byte
    # range), rows at a stride of W + row_pad bytes (rows exactly
    # a power of two apart put every row's column tile on the same low address
    # bits; a 3.5 KiB stagger measured the fastest of 27 at C3, 3.4 % over 3 KiB,
    # profiles/r04_row_pad_sweep.txt).  `flat` is the same
    # memory as an unpadded [B, k+p, W] slab, timed for comparison.
    pad = args.row_pad
    if pad % 64:
        raise SystemExit("--row-pad must be a multiple of 64")
    RS = W + pad
    buf = torch.randint(0, 256, (B * (K + P) * RS,), dtype=torch.uint8, device=dev, generator=g)
    slab = buf.as_strided((B, K + P, W), ((K + P) * RS, RS, 1))
    flat = buf[: B * (K + P) * W].view(B, K + P, W)
    stream = torch.cuda.current_stream()

    def rank_barrier():
        if args.backend == "gloo":
            dist.barrier()
        else:
            dist.barrier(device_ids=[dev.index])

    def barrier():
        if world > 1:
            rank_barrier()
        torch.cuda.synchronize()

    def timed(view, steps):
        """Wall time of `steps` launches and their mean kernel time from HIP
        events on the launch stream (one pair around all of them)."""
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        barrier()
        t0 = time.perf_counter()
        e0.record(stream)
        for _ in range(steps):
            codec.encode_dev_batch(view, stream)
        e1.record(stream)
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        barrier()
        return el, e0.elapsed_time(e1) / steps

    for _ in range(args.warmup):
        codec.encode_dev_batch(slab, stream)
    el, kern_ms = timed(slab, args.steps)
    flat_ms = None
    if pad and not args.no_unpadded:
        for _ in range(args.warmup):
            codec.encode_dev_batch(flat, stream)
        _, flat_ms = timed(flat, max(20, args.steps // 2))
    one_ms = None
    if not args.no_single:
        for _ in range(10):
            codec.encode_dev_batch(slab[:1], stream)
        _, one_ms = timed(slab[:1], max(50, args.steps))

    t = torch.tensor([el, kern_ms, one_ms or 0.0, flat_ms or 0.0], dtype=torch.float64, device=dev)
    per_rank, per_rank_w = [kern_ms], [W]
    if world > 1:
        mine = torch.tensor([kern_ms, float(W)], dtype=torch.float64, device=dev)
        allk = [torch.zeros(2, dtype=torch.float64, device=dev) for _ in range(world)]
        dist.all_gather(allk, mine)
        per_rank = [float(x[0]) for x in allk]
        per_rank_w = [int(x[1]) for x in allk]
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    el, kern_ms, one_ms, flat_ms = float(t[0]), float(t[1]), float(t[2]) or None, float(t[3]) or None

    other = host = calib = None
    if world == 1 and not args.no_other:
        del buf, slab, flat
        torch.cuda.empty_cache()
        calib = copy_rate(torch, dev, stream)
        other = other_workloads(torch, rs, dev, stream)
        other["C2_encode"] = c2_encode(torch, rs, dev, stream)
        torch.cuda.empty_cache()
    if world == 1 and not args.no_host:
        host = host_resident(rs)

    ms_per_step = el / args.steps * 1e3
    job_stripes = B if args.split != "stripes" else world * B  # stripes the whole job encodes per step
    data_bytes = args.steps * job_stripes * K * S
    value = data_bytes / el / 2**30
    alg_bytes = B * (K + P) * W  # per launch on one rank
    achieved = alg_bytes / (kern_ms * 1e-3) / 1e9
    kname = codec.encode_path
    # each rank's algorithmic bytes over its own kernel time
    per_rank_frac = [B * (K + P) * w_r / (k_ms * 1e-3) / 1e9 / PEAK_HBM_GBS for k_ms, w_r in zip(per_rank, per_rank_w)]

    if rank == 0:
        threads = args.cpu_threads or min(16, os.cpu_count() or 1)
        res = {
            "metric": "encode GiB/s (device-resident), %d+%d x %d KiB shards" % (K, P, S >> 10),
            "value": round(value, 2),
            "unit": "GiB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 5),
            "higher_is_better": True,
            "scaling": scaling_of(args),
            "vs_baseline": None,
            "dtype": "u8 (GF(2^16) symbols)",
            "data": "synthetic (uniform random bytes, torch.randint seed 0x5EED+rank)",
            "config": {
                "workload": f"{args.workload}: GF(2^16) Leopard encode, {K} data + {P} parity shards x {S >> 10} KiB, "
                            f"{job_stripes} stripes per step (one launch per rank)",
                "stripes_per_step": job_stripes,
                "stripes_per_rank_launch": B,
                "data_shards": K,
                "parity_shards": P,
                "shard_bytes": S,
                "parallelism": (f"one GPU running rank 0's slice of a {args.slice_of}-rank byte-range split: {W} bytes of every row"
                                if args.slice_of > 1 else
                                f"byte-range split over {world} rank(s): {W} bytes of every row per rank"
                                + (" (per-rank work fixed: the job grows with N)" if args.split == "bytes-weak" and world > 1 else "")
                                if args.split != "stripes" else f"independent stripes, {world} rank(s)"),
                "row_bytes_per_rank": W,
                "kernel_path": kname,
                "layout": f"rows at a stride of {W} + {pad} bytes, stripes back to back",
            },
            "hbm_gib_s": round(world * args.steps * alg_bytes / el / 2**30, 2),
            "per_rank_kernel_ms": [round(x, 5) for x in per_rank],
            "world_size": dist.get_world_size() if world > 1 else 1,
            "backend": dist.get_backend() if world > 1 else None,
            "device": device_info(torch, dev),
            "calibration": None if calib is None else {
                "torch_copy_gb_s": round(calib, 1),
                "note": "2 GiB tensor copy_ on the launch stream, bytes read + written: a box-speed reference "
                        "for comparing lines from different boxes, not a ceiling (the engine's kernels beat it)"},
            "roofline": {
                "bound": "hbm",
                "achieved": round(achieved, 1),
                "peak": PEAK_HBM_GBS,
                "unit": "GB/s",
                "frac": round(achieved / PEAK_HBM_GBS, 4),
                # HBM bytes of one launch of this rank's shape (its stripes x
                # its row slice), from the committed PMC passes of that shape
                "traffic": load_traffic(kname, args.workload, B, W, S),
                "traffic_key": traffic_key(args.workload, kname, B, W),
                "kernel_ms": round(kern_ms, 5),
                "alg_bytes_per_launch": alg_bytes,
            },
            "per_rank_frac": [round(f, 4) for f in per_rank_frac],
            "per_rank_row_bytes": per_rank_w,
            "unpadded_rows": None if flat_ms is None else {
                "kernel_ms": round(flat_ms, 5),
                "frac": round(alg_bytes / (flat_ms * 1e-3) / 1e9 / PEAK_HBM_GBS, 4),
            },
            "single_stripe": None if one_ms is None else {
                "kernel_ms": round(one_ms, 5),
                "frac": round((K + P) * W / (one_ms * 1e-3) / 1e9 / PEAK_HBM_GBS, 4),
            },
            # rank 0 of a one-GPU run only, after the timed region
            "cpu_baseline": None if args.no_cpu or world > 1 else cpu_baseline(K, P, S, args.cpu_seconds, threads),
            "other_workloads": other,
            "host_resident": host,
        }
        print(json.dumps(res), flush=True)
    if world > 1:
        rank_barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
