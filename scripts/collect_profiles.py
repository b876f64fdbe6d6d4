"""Copy the round's GPU evidence from gpurun_out/round into profiles/.

Writes profiles/rNN_bench.json, rNN_kernel_stats.csv (rocprofv3 --stats,
kernel names shortened), rNN_pmc.txt and profiles/pmc_traffic.json, which
bench.py reads for roofline.traffic.  HBM bytes per launch =
2 * FETCH_SIZE + WRITE_SIZE (rocprofv3 reports KiB; gfx950 FETCH_SIZE counts
half of a wide coalesced streaming read, MI355X_MICROARCH.md "HBM")."""
import argparse
import collections
import csv
import glob
import json
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def short(name: str) -> str:
    if "rs::" not in name:
        return re.split(r"[<(]", name.replace("void ", ""), 1)[0][:80]
    name = name.replace("void ", "").replace("rs::(anonymous namespace)::", "")
    return re.sub(r"\(rs::\w+\)$", "", name)


def path_of(name: str):
    """Kernel symbol -> the engine's path name (codec.cpp plan_encode_host)."""
    def v(flag):
        return "-verify" if flag == "true" else ""
    m = re.search(r"k_encode_hp<(\d+), (false|true)>", name)
    if m:
        return f"bs16-m{1 << int(m.group(1))}" + v(m.group(2))
    m = re.search(r"k_encode_split<(\d+), (false|true)>", name)
    if m:
        return f"split16-m{1 << int(m.group(1))}" + v(m.group(2))
    m = re.search(r"k_enc_lds<rs::\(anonymous namespace\)::F(16|8)<\d+>, (\d+), (false|true)[,>]", name)
    if m:
        return f"lds-m{1 << int(m.group(2))}" + v(m.group(3))
    m = re.search(r"k_encode_reg<rs::\(anonymous namespace\)::F(16|8)<\d+>, (\d+), (false|true)", name)
    if m:
        return f"reg{m.group(1)}-m{1 << int(m.group(2))}" + v(m.group(3))
    return None


def rank_slices(src: str, out: str, bench: dict) -> None:
    """Per-rank launch shapes (bench.py --slice-of N, gpu_round.sh slice_N.json
    and slice_8_strong.json) beside the one-GPU line: kernel time, roofline
    fraction and the job value an N-rank run would report if every rank ran at
    that rate.  Written only when the round script produced the slices."""
    lines = []

    def one(label, d, n):
        c, r = d["config"], d["roofline"]
        job = d["value"]  # a --slice-of line already counts the whole job's shard bytes (k * S per stripe)
        lines.append(f"{label:<28} W={c['row_bytes_per_rank']:>8}  stripes/launch {c['stripes_per_rank_launch']:>5}  "
                     f"kernel {r['kernel_ms']:.4f} ms  frac {r['frac']:.4f}  projected job GiB/s {job:.1f}  "
                     f"efficiency {r['frac'] / bench['roofline']['frac']:.3f}")

    one("1 rank (the bench line)", bench, 1)
    found = False
    for n in (2, 4, 8):
        p = os.path.join(src, f"slice_{n}.json")
        if os.path.exists(p):
            with open(p) as f:
                one(f"{n}-rank slice (bytes-weak)", json.loads([l for l in f if l.startswith("{")][-1]), n)
            found = True
    p = os.path.join(src, "slice_8_strong.json")
    if os.path.exists(p):
        with open(p) as f:
            one("8-rank slice (strong)", json.loads([l for l in f if l.startswith("{")][-1]), 8)
    if not found:
        return
    with open(out, "w") as f:
        f.write("# Per-rank launch shapes of an N-GPU byte-range run on one GPU (bench.py --slice-of N, "
                "scripts/gpu_round.sh), HIP events.\n# bytes-weak (the default): rank 0's byte range of N x "
                f"{bench['config']['stripes_per_rank_launch']} stripes; strong: of {bench['config']['stripes_per_rank_launch']} stripes.\n"
                "# efficiency = the slice's roofline fraction over the one-GPU line's (the kernel-only scaling "
                "efficiency an N-GPU run would show if each GPU ran like this one).\n")
        f.write("\n".join(lines) + "\n")
    print("\n".join(lines))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--round", type=int, required=True)
    ap.add_argument("--src", default=os.path.join(ROOT, "gpurun_out", "round"))
    ap.add_argument("--suffix", default="", help="file-name suffix (a second evidence set of the same round)")
    a = ap.parse_args()
    tag = f"r{a.round:02d}{a.suffix}"
    prof = os.path.join(ROOT, "profiles")
    os.makedirs(prof, exist_ok=True)

    with open(os.path.join(a.src, "bench.json")) as f:
        bench = json.loads([l for l in f if l.startswith("{")][-1])
    with open(os.path.join(prof, f"{tag}_bench.json"), "w") as f:
        json.dump(bench, f, indent=1)

    rank_slices(a.src, os.path.join(prof, f"{tag}_rank_slices.txt"), bench)

    rows = list(csv.DictReader(open(os.path.join(a.src, "trace", "run_kernel_stats.csv"))))
    with open(os.path.join(prof, f"{tag}_kernel_stats.csv"), "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=list(rows[0].keys()))
        w.writeheader()
        for r in rows:
            r = dict(r)
            r["Name"] = short(r["Name"])
            w.writerow(r)

    # PMC passes: pmc_<COUNTER> (the bench's own shape) and pmc_<COUNTER>_s<N>
    # (bench.py --slice-of N: rank 0's byte range of an N-rank split)
    import sys
    sys.path.insert(0, ROOT)
    from reedsolomon16_amd.dist import byte_range

    S = bench["config"]["shard_bytes"]
    stripes = bench["config"].get("stripes_per_step", 16)
    workload = bench["config"]["workload"].split(":")[0]
    agg = collections.defaultdict(list)
    nstr = {}  # row slice -> stripes per launch of that pass (its bench line, when it has one)
    for c in ("FETCH_SIZE", "WRITE_SIZE"):
        for d in glob.glob(os.path.join(a.src, f"pmc_{c}*")):
            if not os.path.isdir(d):
                continue
            m = re.search(r"_s(\d+)$", d)
            W = byte_range(S, 0, int(m.group(1)))[1] if m else bench["config"].get("row_bytes_per_rank", S)
            try:  # bench.py --slice-of N in the bytes-weak layout launches N x stripes
                with open(d + ".json") as f:
                    cfg = json.loads([l for l in f if l.startswith("{")][-1])["config"]
                nstr[W] = cfg.get("stripes_per_rank_launch", cfg.get("stripes_per_step", stripes))
            except (OSError, IndexError, ValueError, KeyError):
                nstr.setdefault(W, stripes)
            for fn in glob.glob(os.path.join(d, "run_counter_collection.csv")):
                for r in csv.DictReader(open(fn)):
                    p = path_of(r["Kernel_Name"])
                    if p:
                        agg[(p, W, r["Counter_Name"])].append(float(r["Counter_Value"]))
    traffic, lines = {}, []
    for p, W in sorted({k[:2] for k in agg}):
        stripes_w = nstr.get(W, stripes)
        fk = agg.get((p, W, "FETCH_SIZE"), [])
        wk = agg.get((p, W, "WRITE_SIZE"), [])
        if not fk or not wk:
            continue
        fetch = sum(fk) / len(fk) * 1024
        write = sum(wk) / len(wk) * 1024
        hbm = 2 * fetch + write
        alg = stripes_w * (bench["config"]["data_shards"] + bench["config"]["parity_shards"]) * W
        traffic[f"{workload}:{p}:{stripes_w}x{W}"] = {
            "hbm_bytes_per_launch": round(hbm), "fetch_size_bytes": round(fetch),
            "write_size_bytes": round(write), "launches": len(fk), "stripes": stripes_w, "row_bytes": W,
            "alg_bytes_per_launch": alg, "traffic_over_alg": round(hbm / alg, 4),
            "correction": "2*FETCH_SIZE + WRITE_SIZE (gfx950 FETCH_SIZE = half of streamed reads)",
            "round": tag}
        lines.append(f"{p} {stripes_w}x{W}: FETCH_SIZE {fetch/1e6:.2f} MB (x2 = {2*fetch/1e6:.2f}), WRITE_SIZE "
                     f"{write/1e6:.2f} MB, HBM {hbm/1e6:.2f} MB/launch ({hbm/alg:.4f} x algorithmic) over {len(fk)} launches")
    kern = [r for r in rows if "k_enc" in r["Name"] or "k_rec" in r["Name"]]
    for r in kern:
        lines.append(f"trace {short(r['Name'])}: calls {r['Calls']} avg {float(r['AverageNs'])/1e3:.2f} us "
                     f"min {float(r['MinNs'])/1e3:.2f} max {float(r['MaxNs'])/1e3:.2f}")
    lines.append(f"bench kernel_ms (HIP events) {bench['roofline']['kernel_ms']*1e3:.2f} us, "
                 f"achieved {bench['roofline']['achieved']} GB/s, frac {bench['roofline']['frac']}")
    with open(os.path.join(prof, f"{tag}_pmc.txt"), "w") as f:
        f.write("\n".join(lines) + "\n")
    tpath = os.path.join(prof, "pmc_traffic.json")
    old = json.load(open(tpath)) if os.path.exists(tpath) else {}
    old.update(traffic)
    with open(tpath, "w") as f:
        json.dump(old, f, indent=1)
    print("\n".join(lines))


if __name__ == "__main__":
    main()
