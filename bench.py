"""Headline benchmark: device-resident encode+decode GiB/s, vandrs RS(10,4,8),
1 MiB objects (BASELINE.json metric / configs[1..2]).

One step = encode every object of this rank's batch (10 data blocks read, 4
coding blocks written per object) + in-place decode of the same batch with
data blocks {0,1,2,3} erased (6 data + 4 coding read, 4 data written).
Objects are independent, so N GPUs = N processes with their own batches and
no collectives on the data path (weak scaling); a barrier and a max-reduce of
the elapsed time bracket the timed region.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W]
       (N > 1: launched by torch.distributed.run, one rank per GPU)
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "GiB/s device-resident encode+decode, vandrs RS(10,4,w=8) 1 MiB objects"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
K, M, W = 10, 4, 8
ERASED = [0, 1, 2, 3]


def shard_range(rank, world, total):
    """Objects [lo, hi) owned by `rank` when `total` objects split evenly."""
    lo = total * rank // world
    hi = total * (rank + 1) // world
    return lo, hi


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=200)
    p.add_argument("--warmup", type=int, default=100)
    p.add_argument("--objects", type=int, default=2048, help="1 MiB objects per GPU (one launch)")
    p.add_argument("--size", type=int, default=1048576)
    p.add_argument("--cpu-seconds", type=float, default=12.0,
                   help="target CPU time of the bounded cpu_baseline sample")
    p.add_argument("--no-cpu", action="store_true", help="skip the cpu_baseline leg")
    p.add_argument("--traffic", default=os.path.join(ROOT, "profiles", "pmc_traffic.json"),
                   help="PMC-derived HBM bytes per launch (written by tools/pmc_traffic.py)")
    return p.parse_args(argv)


def cpu_baseline(size, target_s, threads, sample_objs=2048):
    """The CPU restatement with ISA-L's split-table (PSHUFB) technique, timed on
    this host's cores over a bounded sample of the same workload: a 2 GiB
    batch (beyond any host LLC) encoded + decoded in repeated passes until
    about `target_s` seconds of wall time have been spent."""
    import numpy as np

    from oracle import oracle as O

    bs = O.block_size(K, W, size)
    n = sample_objs
    rng = np.random.Generator(np.random.PCG64(0x1E0E))
    objs = rng.integers(0, 256, (n, size), dtype=np.uint8)
    parity = np.zeros((n, M * bs), dtype=np.uint8)
    te = td = 0.0
    passes = 0
    while te + td < target_s or passes == 0:
        t0 = time.perf_counter()
        O.bench_rs8(0, K, M, objs, size, size, n, parity, threads=threads)
        t1 = time.perf_counter()
        O.bench_rs8(1, K, M, objs, size, size, n, parity, erased=ERASED, threads=threads)
        t2 = time.perf_counter()
        te += t1 - t0
        td += t2 - t1
        passes += 1
    gib = 2 * n * passes * size / (te + td) / 2**30
    return {
        "value": round(gib, 3), "unit": "GiB/s", "cores": threads, "kind": "port",
        "simd": {0: "scalar", 2: "avx2-pshufb (ISA-L split tables)",
                 3: "avx512-gfni (ISA-L gf2p8affine)"}.get(O.simd_level(), "scalar"),
        "sample": f"{passes} passes over {n} x {size} B objects: vandrs RS({K},{M},8) encode "
                  f"{te:.2f} s + in-place decode of data blocks {ERASED} {td:.2f} s, "
                  f"{threads} threads",
    }


def main(argv=None):
    args = parse(argv)
    import torch
    import torch.distributed as dist

    import leo_erasure_amd as le

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl")
    else:
        torch.cuda.set_device(0)
    assert le.gf_init() == "ok", le.gf_init()
    dev = torch.device("cuda", torch.cuda.current_device())

    size, n = args.size, args.objects
    bs, _ = le.layout("vandrs", (K, M, W), size)
    gen = torch.Generator(device=dev).manual_seed(0x1E0E + rank)
    objs = torch.randint(0, 256, (n, size), dtype=torch.uint8, device=dev, generator=gen)
    parity = torch.empty((n, M * bs), dtype=torch.uint8, device=dev)
    ref = objs.clone()
    stream = torch.cuda.current_stream()

    def step(ev=None):
        if ev is not None:
            ev[0].record(stream)
        le.device.encode("vandrs", (K, M, W), objs, size, parity)
        if ev is not None:
            ev[1].record(stream)
        le.device.decode("vandrs", (K, M, W), objs, size, parity, ERASED)
        if ev is not None:
            ev[2].record(stream)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    events = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(args.steps)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(events[i])
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = t.item()

    enc_t = [e[0].elapsed_time(e[1]) for e in events]
    dec_t = [e[1].elapsed_time(e[2]) for e in events]
    enc_ms = sum(enc_t) / args.steps
    dec_ms = sum(dec_t) / args.steps
    # decode rebuilt blocks 0..3 in place every step: the batch must be intact
    intact = bool(torch.equal(objs, ref))
    if world > 1:
        f = torch.tensor([0 if intact else 1], device=dev)
        dist.all_reduce(f, op=dist.ReduceOp.MAX)
        intact = f.item() == 0

    if rank == 0:
        total_objs = n * world
        value = 2.0 * total_objs * size * args.steps / elapsed / 2**30
        enc_bytes = (K + M) * bs * n              # algorithmic bytes per encode launch
        dec_bytes = (K + len(ERASED)) * bs * n    # per decode launch
        enc_gbs = enc_bytes / (enc_ms * 1e-3) / 1e9
        dec_gbs = dec_bytes / (dec_ms * 1e-3) / 1e9
        traffic = None
        if os.path.exists(args.traffic):
            try:
                with open(args.traffic) as fh:
                    tr = json.load(fh)
                if tr.get("objects") == n and tr.get("object_bytes") == size:
                    traffic = tr.get("encode_bytes_per_launch")
            except (OSError, ValueError):
                traffic = None
        rec = {
            "metric": METRIC,
            "value": round(value, 3),
            "unit": "GiB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (uniform random bytes, torch Philox seed 0x1E0E+rank)",
            "config": {
                "workload": "vandrs RS(k=10,m=4,w=8) encode + in-place decode of data blocks "
                            "{0,1,2,3}, 1 MiB objects, device-resident batch",
                "objects_per_gpu": n, "object_bytes": size, "block_size": bs,
                "parallelism": f"object-sharded x{world}, no collectives",
            },
            "roofline": {
                "bound": "hbm", "kernel": "gf8_apply<10,4> (encode)",
                "achieved": round(enc_gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(enc_gbs / HBM_PEAK_GBS, 4), "traffic": traffic,
                "alg_bytes_per_launch": enc_bytes, "avg_launch_ms": round(enc_ms, 4),
                "decode": {"achieved": round(dec_gbs, 1), "frac": round(dec_gbs / HBM_PEAK_GBS, 4),
                           "alg_bytes_per_launch": dec_bytes, "avg_launch_ms": round(dec_ms, 4)},
            },
            "kernel_ms": {"encode_min_med_max": [round(x, 4) for x in (min(enc_t), sorted(enc_t)[len(enc_t) // 2], max(enc_t))],
                          "decode_min_med_max": [round(x, 4) for x in (min(dec_t), sorted(dec_t)[len(dec_t) // 2], max(dec_t))]},
            "verified": intact,
        }
        if world == 1 and not args.no_cpu:
            try:
                threads = min(16, len(os.sched_getaffinity(0)))
            except AttributeError:
                threads = min(16, os.cpu_count() or 1)
            rec["cpu_baseline"] = cpu_baseline(size, args.cpu_seconds, threads)
        else:
            rec["cpu_baseline"] = None
        print(json.dumps(rec), flush=True)
    if world > 1:
        dist.destroy_process_group()
    if not intact:
        sys.exit(1)


if __name__ == "__main__":
    main()
