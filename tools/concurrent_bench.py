#!/usr/bin/env python3
"""Batched throughput with the per-call worker resident beside it.

The bench.py step (fec=20:3, B=1440, 1M groups: encode every group, decode every group with 3 data shards
erased) is timed three ways in one process: alone, while a second thread calls the single-group
``FecCode.encode`` back to back (the resident worker then holds its 8 workgroups on 8 CUs and polls), and alone
again.  Prints one JSON line: step ms of each phase (HIP events on the batch stream, mean of --steps), the
per-call thread's calls and mean us per call, and the relative cost of the resident worker.

    python tools/concurrent_bench.py [--groups 1048576] [--steps 10]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--groups", type=int, default=1 << 20)
    ap.add_argument("--steps", type=int, default=10)
    args = ap.parse_args()
    import numpy as np
    import torch

    from kcptube_amd import FecCode
    from kcptube_amd.fec import worker_requests

    K, N, B, G = 20, 23, 1440, args.groups
    R = N - K
    dev = torch.device("cuda:0")
    c = FecCode(K, N)
    data = torch.empty((G, K, B), dtype=torch.uint8, device=dev)
    par = torch.empty((G, R, B), dtype=torch.uint8, device=dev)
    masks = torch.empty((G, 4), dtype=torch.int64, device=dev)
    out = torch.empty((G, R, B), dtype=torch.uint8, device=dev)
    idx = torch.empty((G, R), dtype=torch.uint8, device=dev)
    st = torch.empty((G,), dtype=torch.uint8, device=dev)
    ws = c.decode_workspace(G, device=dev)
    c.synth(data, 0x5EED0001)
    c.erasure_masks(masks, 0x5EED0001, K, R)
    stream = torch.cuda.current_stream()

    def phase(steps):
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
        c.encode_batch(data, par)
        c.decode_batch(data, par, masks, out, idx, st, ws)
        stream.synchronize()
        t0 = time.perf_counter()
        for a, b in ev:
            a.record(stream)
            c.encode_batch(data, par)
            c.decode_batch(data, par, masks, out, idx, st, ws)
            b.record(stream)
        stream.synchronize()
        wall = (time.perf_counter() - t0) / steps * 1e3
        return sum(a.elapsed_time(b) for a, b in ev) / steps, wall

    alone1, wall1 = phase(args.steps)
    # the per-call thread: one 20:3 group per call, its own coder, checked against its first answer
    stop = threading.Event()
    stats = {"calls": 0, "bad": 0, "secs": 0.0}
    rng = np.random.default_rng(1)
    group = rng.integers(0, 256, K * B, dtype=np.uint8).tobytes()
    c2 = FecCode(K, N)
    want = c2.encode(group, len(group), B)

    def caller():
        t0 = time.perf_counter()
        n = bad = 0
        while not stop.is_set():
            bad += c2.encode(group, len(group), B) != want
            n += 1
        stats.update(calls=n, bad=bad, secs=time.perf_counter() - t0)

    req0 = worker_requests()
    th = threading.Thread(target=caller)
    th.start()
    time.sleep(0.05)
    busy, wall_busy = phase(args.steps)
    stop.set()
    th.join()
    served = worker_requests() - req0
    alone2, wall2 = phase(args.steps)
    base = (alone1 + alone2) / 2
    print(json.dumps({
        "workload": f"fec=20:3 B=1440, {G} groups: encode + decode (3 data shards erased) per step, HIP events on the "
                    f"batch stream; a second thread calls FecCode.encode (one group from host memory) back to back "
                    f"during the middle phase",
        "step_ms_alone_before": round(alone1, 4), "step_ms_with_percall": round(busy, 4),
        "step_ms_alone_after": round(alone2, 4),
        "wall_ms_alone_before": round(wall1, 4), "wall_ms_with_percall": round(wall_busy, 4),
        "wall_ms_alone_after": round(wall2, 4),
        "batched_slowdown": round(busy / base - 1, 4),
        "percall_calls": stats["calls"], "percall_bad": stats["bad"],
        "percall_us": round(stats["secs"] * 1e6 / max(stats["calls"], 1), 2),
        "percall_served_by_worker": served,
    }), flush=True)
    if stats["bad"] or served == 0:
        sys.exit(3)


if __name__ == "__main__":
    main()
