"""Headline benchmark: device-resident GF(2^16) encode, 128 data + 32 parity x 1 MiB
shards (BASELINE.json configs[2] / C3), --stripes stripes (default 16) per rank per step.

A step is one encode of B synthetic C3 stripes already resident in HBM, all in
one kernel launch (rs_encode_dev_batch; the stripes are independent objects,
as a storage server encodes many at once).  Multi-GPU: one process per GPU, each rank encodes its own
stripe (independent objects, no collective on the data path) -> weak scaling;
value = data bytes encoded by all ranks / max-over-ranks wall time.

Prints one JSON line (rank 0).  `roofline` is for the dominant (only) kernel:
achieved = algorithmic bytes per launch ((k+p)*S: read k rows, write p rows)
/ its mean duration: one HIP event pair on the launch stream around the K
back-to-back launches of the timed region, divided by K.  `cpu_baseline` times the oracle's scalar C
restatement of the reference path (single thread) on a bounded sample.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

K, P, S = 128, 32, 1 << 20
PEAK_HBM_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md)


def cpu_baseline(seconds: float):
    """Oracle (scalar C restatement of the reference Ref path), 1 thread, same config."""
    import numpy as np

    from oracle import orc

    rng = np.random.default_rng(0x5EED)
    data = rng.integers(0, 256, (K, S), dtype=np.uint8)
    orc.encode(16, K, P, data)  # warm (table init)
    n, t0 = 0, time.perf_counter()
    while True:
        orc.encode(16, K, P, data)
        n += 1
        el = time.perf_counter() - t0
        if el >= seconds:
            break
    return {
        "value": round(n * K * S / el / 2**30, 4),
        "unit": "GiB/s",
        "cores": 1,
        "kind": "port",
        "sample": f"{n} encodes of one 128+32 x 1 MiB stripe (oracle/leopard_ref.c scalar Ref path, -O2), {el:.1f} s",
    }


def load_traffic(kernel_name: str):
    """HBM bytes per launch from the committed rocprofv3 PMC summary, if present."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            d = json.load(f)
        return d.get(kernel_name, {}).get("hbm_bytes_per_launch")
    except Exception:
        return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--stripes", type=int, default=16,
                    help="stripes encoded per step (one launch); each is 128+32 x 1 MiB")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    import reedsolomon16_amd as rs

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", torch.cuda.current_device())

    codec = rs.New16(K, P, device=dev.index)
    g = torch.Generator(device=dev)
    g.manual_seed(0x5EED + rank)
    B = args.stripes
    slab = torch.randint(0, 256, (B, K + P, S), dtype=torch.uint8, device=dev, generator=g)
    stream = torch.cuda.current_stream()

    def barrier():
        if world > 1:
            dist.barrier(device_ids=[dev.index])
        torch.cuda.synchronize()

    for _ in range(args.warmup):
        codec.encode_dev_batch(slab, stream)
    barrier()

    # One HIP event pair on the launch stream brackets the K back-to-back
    # launches: per-launch event pairs would insert their own gaps.
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    barrier()
    t0 = time.perf_counter()
    e0.record(stream)
    for _ in range(args.steps):
        codec.encode_dev_batch(slab, stream)
    e1.record(stream)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    barrier()
    kern_ms = e0.elapsed_time(e1) / args.steps

    t = torch.tensor([el, kern_ms], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    el, kern_ms = float(t[0]), float(t[1])

    ms_per_step = el / args.steps * 1e3
    data_bytes = world * args.steps * B * K * S
    value = data_bytes / el / 2**30
    alg_bytes = B * (K + P) * S
    achieved = alg_bytes / (kern_ms * 1e-3) / 1e9
    kname = codec.encode_path

    if rank == 0:
        res = {
            "metric": "encode GiB/s (device-resident), 128+32 x 1 MiB shards",
            "value": round(value, 2),
            "unit": "GiB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 5),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8 (GF(2^16) symbols)",
            "data": "synthetic (uniform random bytes, torch.randint seed 0x5EED+rank)",
            "config": {
                "workload": f"GF(2^16) Leopard encode, 128 data + 32 parity shards x 1 MiB, {B} stripes per rank per step (one launch)",
                "stripes_per_step": B,
                "data_shards": K,
                "parity_shards": P,
                "shard_bytes": S,
                "parallelism": f"independent stripes, {world} rank(s)",
                "kernel_path": kname,
            },
            "hbm_gib_s": round(world * args.steps * alg_bytes / el / 2**30, 2),
            "roofline": {
                "bound": "hbm",
                "achieved": round(achieved, 1),
                "peak": PEAK_HBM_GBS,
                "unit": "GB/s",
                "frac": round(achieved / PEAK_HBM_GBS, 4),
                "traffic": load_traffic(kname),
                "kernel_ms": round(kern_ms, 5),
                "alg_bytes_per_launch": alg_bytes,
            },
            "cpu_baseline": None if (args.no_cpu or world > 1) else cpu_baseline(args.cpu_seconds),
        }
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
