#!/usr/bin/env python3
"""Benchmark of the kfec hot path: device-resident Reed-Solomon encode + decode on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config 20:3|10:3dec|200:55]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N ...

Metric (BASELINE.json): "FEC encode+decode GiB/s (device-resident), fec=20:3 kcp_mtu=1440".
One step = encode every group of the batch (K data -> R parity shards) and decode every group with R
data shards erased (selection, per-group m x m inverse, recovery MAC), all on the device with inputs
already resident in HBM.  value = payload bytes (G * K * B per GPU, summed over GPUs) per step / step
time, in GiB/s.  Shard groups are independent, so each rank owns its own contiguous group range
(weak scaling, no collective on the data path; gloo only for the timing barrier and the max-reduce).

Also reported: the roofline of the dominant kernel (the encode MAC launch, HIP events on its stream),
the decode kernels' figures, and the reference CPU coder (oracle/_ref, compiled from the reference's
own sources) timed on the host cores on a bounded sample (rank 0, N = 1 only).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "FEC encode+decode GiB/s (device-resident), fec=20:3 kcp_mtu=1440, 1/2/4/8 GPU"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)

CONFIGS = {
    # name: K, N, B, groups per GPU, erasure pool, erasures, random count, encode?, workload text
    "20:3": (20, 23, 1440, 1 << 20, 20, 3, False, True,
             "fec=20:3 kcp_mtu=1440, 1M shard groups per GPU, encode + decode with 3 data shards erased"),
    "10:3dec": (10, 13, 1400, 1 << 20, 13, 3, True, False,
                "fec=10:3 kcp_mtu=1400, 1M groups, decode-only, random 1-3 erasures over all 13 shards"),
    "200:55": (200, 255, 1440, 1 << 18, 200, 55, False, True,
               "fec=200:55 kcp_mtu=1440, 256k groups, encode + decode with 55 data shards erased"),
}


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--config", default="20:3", choices=sorted(CONFIGS))
    p.add_argument("--groups", type=int, default=0, help="override groups per GPU")
    p.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline leg")
    p.add_argument("--cpu-seconds", type=float, default=16.0, help="target CPU-seconds of the baseline sample")
    return p.parse_args()


def cpu_baseline(K, N, B, pool, erase, rnd, target_cpu_s, decode_only=False):
    """Reference coder on the host cores, bounded sample.  Test infrastructure (oracle/), used here
    only for the reported CPU baseline -- never for the GPU number."""
    import oracle as orc
    threads = max(1, min(16, len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()))
    G = 1 << 15 if K <= 32 else 1 << 9
    if orc.RefCoder.available():
        ref = orc.RefCoder()
        kind = "reference"
        run = lambda passes: ref.bench_roundtrip(K, N, B, G, pool, erase, rnd, threads, passes, 0x5EED0001,
                                                 decode_only)[:2]
    else:
        o = orc.Oracle()
        kind = "port"
        run = lambda passes: o.bench_roundtrip(K, N, B, G, erase, threads, passes, 0x5EED0001)
    bps, secs = run(1)  # calibration pass (also warms the pages)
    passes = max(1, int(target_cpu_s / max(secs * threads, 1e-3)))
    bps, secs = run(passes)
    # one core, same groups: about a tenth of the CPU time above
    if kind == "reference":
        g1 = max(64, G // 8)
        bps1 = ref.bench_roundtrip(K, N, B, g1, pool, erase, rnd, 1, 1, 0x5EED0001, decode_only)[0]
    else:
        g1 = G
        bps1 = None
    import platform
    model = platform.processor() or ""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    what = "decode-only" if decode_only else "encode + decode"
    return {"value": round(bps / 2**30, 4), "unit": "GiB/s", "cores": threads, "kind": kind,
            "value_1core": round(bps1 / 2**30, 4) if bps1 else None,
            "sample": f"{G} distinct groups x {passes} passes of fec={K}:{N-K} B={B} {what} "
                      f"({'random 1-%d of all %d' % (erase, N) if rnd else '%d data' % erase} shards erased), "
                      f"{secs:.1f} s wall on {threads} threads, {model}; value_1core: {g1} groups x 1 pass "
                      f"on 1 thread"}


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        dist.init_process_group("gloo")
    # one rank per GPU; local % count only matters for a multi-rank rehearsal on a smaller box
    local_dev = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local_dev)
    dev = torch.device("cuda", local_dev)

    from kcptube_amd import FecCode

    K, N, B, G, pool, erase, rnd, do_enc, workload = CONFIGS[args.config]
    if args.groups and args.groups != G:
        G = args.groups
        workload += f" (--groups override: {G} groups per GPU)"
    R = N - K
    c = FecCode(K, N)
    g0 = rank * G  # this rank's contiguous range of the global group space
    seed = 0x5EED0001
    data = torch.empty((G, K, B), dtype=torch.uint8, device=dev)
    par = torch.empty((G, R, B), dtype=torch.uint8, device=dev)
    masks = torch.empty((G, 4), dtype=torch.int64, device=dev)
    out = torch.empty((G, R, B), dtype=torch.uint8, device=dev)
    idx = torch.empty((G, R), dtype=torch.uint8, device=dev)
    st = torch.empty((G,), dtype=torch.uint8, device=dev)
    ws = c.decode_workspace(G, device=dev)
    c.synth(data, seed, g0=g0)
    c.erasure_masks(masks, seed, pool, erase, rnd, g0=g0)
    c.encode_batch(data, par)  # parity exists before a decode-only step
    torch.cuda.synchronize()

    stream = torch.cuda.current_stream()
    n_ev = args.steps
    ev = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(n_ev)]

    def step(i=None):
        if i is not None:
            ev[i][0].record(stream)
        if do_enc:
            c.encode_batch(data, par)
        if i is not None:
            ev[i][1].record(stream)
        c.decode_batch(data, par, masks, out, idx, st, ws)
        if i is not None:
            ev[i][2].record(stream)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(i)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    elapsed = t1 - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    enc_ms = sum(ev[i][0].elapsed_time(ev[i][1]) for i in range(n_ev)) / n_ev
    dec_ms = sum(ev[i][1].elapsed_time(ev[i][2]) for i in range(n_ev)) / n_ev

    # correctness of what was timed (untimed): every erased data shard recovered bit-exact
    mism = torch.zeros(1, dtype=torch.int64, device=dev)
    c.verify_recovered(data, out, idx, mism)
    torch.cuda.synchronize()
    n_rec = int((idx != 0xFF).sum().item())
    n_dec = int((idx[:, 0] != 0xFF).sum().item()) if R > 0 else 0  # groups with m > 0 (m = 0 reads nothing)
    ok = int(mism.item()) == 0 and int(st.max().item()) == 0 and n_rec > 0
    if world > 1:
        t = torch.tensor([0 if ok else 1], dtype=torch.int64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        ok = int(t.item()) == 0

    payload = K * B * G * world * args.steps
    value = payload / elapsed / 2**30
    ms_per_step = elapsed / args.steps * 1e3

    # roofline: algorithmic HBM bytes per launch / measured launch duration
    enc_bytes = G * (K + R) * B                    # read K*B, write R*B per group
    dec_bytes = n_dec * K * B + n_rec * B          # read the K selected shares, write the m recovered
    enc_read = G * K * B
    dec_read = n_dec * K * B
    if do_enc:
        dom_bytes, dom_read, dom_ms = enc_bytes, enc_read, enc_ms
        dom_name = "mac_kernel<VEC,MT,encode> (kfec_encode_batch)"
    else:
        dom_bytes, dom_read, dom_ms = dec_bytes, dec_read, dec_ms
        dom_name = "decode_prep_* + mac_kernel<VEC,MT,decode> (kfec_decode_batch)"
    achieved = dom_bytes / (dom_ms * 1e-3) / 1e9
    achieved_read = dom_read / (dom_ms * 1e-3) / 1e9
    traffic = None
    pmc = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if os.path.exists(pmc):
        try:
            with open(pmc) as f:
                tr = json.load(f).get(args.config)
            if tr and tr.get("groups") == G:
                traffic = tr.get("hbm_bytes_per_launch")
        except (OSError, ValueError):
            traffic = None
    result = {
        "metric": METRIC,
        "value": round(value, 2),
        "unit": "GiB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic: splitmix64 counter bytes generated on device (SURVEY 8d); erasure patterns per-group PRNG",
        "config": {"workload": workload, "fec": f"{K}:{R}", "kcp_mtu": B, "groups_per_gpu": G,
                   "global_groups": G * world, "parallelism": f"{world} independent group ranges (no collective)"},
        "roofline": {"bound": "hbm", "kernel": dom_name, "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                     "algorithmic_bytes_per_launch": dom_bytes, "avg_launch_ms": round(dom_ms, 4),
                     "achieved_read": round(achieved_read, 1), "frac_read": round(achieved_read / HBM_PEAK_GBS, 4)},
        "encode_ms": round(enc_ms, 4) if do_enc else None,
        "decode_ms": round(dec_ms, 4),
        "decode_hbm_GBps": round(dec_bytes / (dec_ms * 1e-3) / 1e9, 1),
        "roundtrip_hbm_GBps": round(((enc_bytes if do_enc else 0) + dec_bytes) / ((enc_ms if do_enc else 0) + dec_ms) / 1e6, 1),
        "recovered_shards_per_step": n_rec * world,
        "decoded_groups_per_step": n_dec * world,
        "verified_bit_exact": ok,
        "cpu_baseline": None,
    }
    if rank == 0 and world == 1 and not args.no_cpu:
        try:
            result["cpu_baseline"] = cpu_baseline(K, N, B, pool, erase, rnd, args.cpu_seconds,
                                                  decode_only=not do_enc)
        except Exception as e:  # the GPU number stands on its own
            result["cpu_baseline"] = {"error": repr(e)}
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()
    if not ok:
        sys.exit(3)


if __name__ == "__main__":
    main()
