#!/usr/bin/env python3
"""End-to-end rate from pinned host memory (the path starts and ends in UDP socket buffers).

Encode: data groups in pinned host memory -> hipMemcpyAsync H2D -> kfec_encode_batch -> parity D2H.
Decode: surviving shards (K per group: the data minus the erased ones, plus parity) H2D -> decode ->
recovered shards D2H.  Chunks of C groups are pipelined over NS streams (copy of chunk i+1 overlaps the
kernel of chunk i).  Prints one JSON line with GiB/s of payload (G*K*B) for encode, decode and the round
trip, next to the PCIe bytes moved.

    python tools/e2e.py [--groups 262144] [--chunk 16384] [--streams 3]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from kcptube_amd import FecCode  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--groups", type=int, default=1 << 18)
ap.add_argument("--chunk", type=int, default=1 << 14)
ap.add_argument("--streams", type=int, default=3)
ap.add_argument("--K", type=int, default=20)
ap.add_argument("--R", type=int, default=3)
ap.add_argument("--B", type=int, default=1440)
ap.add_argument("--iters", type=int, default=3)
args = ap.parse_args()
K, R, B, G, C = args.K, args.R, args.B, args.groups, args.chunk
N = K + R
dev = torch.device("cuda:0")
c = FecCode(K, N)

# host side: pinned buffers standing in for socket buffers
h_data = torch.empty((G, K, B), dtype=torch.uint8).pin_memory()
h_par = torch.empty((G, R, B), dtype=torch.uint8).pin_memory()
h_out = torch.empty((G, R, B), dtype=torch.uint8).pin_memory()
tmp = torch.empty((C, K, B), dtype=torch.uint8, device=dev)
for g0 in range(0, G, C):  # fill host data with the synthetic generator (device), untimed
    n = min(C, G - g0)
    c.synth(tmp[:n], 0x5EED0001, g0=g0)
    h_data[g0:g0 + n].copy_(tmp[:n].cpu())
masks_all = torch.empty((G, 4), dtype=torch.int64, device=dev)
c.erasure_masks(masks_all, 0x5EED0001, K, R)
torch.cuda.synchronize()

NS = args.streams
streams = [torch.cuda.Stream() for _ in range(NS)]
d_data = [torch.empty((C, K, B), dtype=torch.uint8, device=dev) for _ in range(NS)]
d_par = [torch.empty((C, R, B), dtype=torch.uint8, device=dev) for _ in range(NS)]
d_out = [torch.empty((C, R, B), dtype=torch.uint8, device=dev) for _ in range(NS)]
d_idx = [torch.empty((C, R), dtype=torch.uint8, device=dev) for _ in range(NS)]
d_st = [torch.empty((C,), dtype=torch.uint8, device=dev) for _ in range(NS)]
d_ws = [c.decode_workspace(C) for _ in range(NS)]


def run_encode():
    for i, g0 in enumerate(range(0, G, C)):
        n = min(C, G - g0)
        k = i % NS
        with torch.cuda.stream(streams[k]):
            d_data[k][:n].copy_(h_data[g0:g0 + n], non_blocking=True)
            c.encode_batch(d_data[k][:n], d_par[k][:n], stream=streams[k])
            h_par[g0:g0 + n].copy_(d_par[k][:n], non_blocking=True)
    torch.cuda.synchronize()


def run_decode():
    # the surviving shards travel: K of the N per group (data slots + parity slots; absent slots are not
    # copied in a real receiver -- here whole slots are copied but only K*B bytes/group are counted as
    # needed, and the copy volume reported below is what was actually moved)
    for i, g0 in enumerate(range(0, G, C)):
        n = min(C, G - g0)
        k = i % NS
        with torch.cuda.stream(streams[k]):
            d_data[k][:n].copy_(h_data[g0:g0 + n], non_blocking=True)
            d_par[k][:n].copy_(h_par[g0:g0 + n], non_blocking=True)
            c.decode_batch(d_data[k][:n], d_par[k][:n], masks_all[g0:g0 + n], d_out[k][:n], d_idx[k][:n],
                           d_st[k][:n], d_ws[k], stream=streams[k])
            h_out[g0:g0 + n].copy_(d_out[k][:n], non_blocking=True)
    torch.cuda.synchronize()


def timeit(fn):
    fn()
    best = 1e9
    for _ in range(args.iters):
        t0 = time.perf_counter()
        fn()
        best = min(best, time.perf_counter() - t0)
    return best


te = timeit(run_encode)
td = timeit(run_decode)
payload = G * K * B
res = {
    "what": "end-to-end from pinned host memory (H2D + kernel + D2H, %d streams, %d-group chunks)" % (NS, C),
    "config": f"fec={K}:{R} B={B} groups={G}",
    "encode_GiBps": round(payload / te / 2**30, 2),
    "decode_GiBps": round(payload / td / 2**30, 2),
    "roundtrip_GiBps": round(payload / (te + td) / 2**30, 2),
    "encode_pcie_GBps": round(G * (K + R) * B / te / 1e9, 2),
    "decode_pcie_GBps": round(G * (K + R + R) * B / td / 1e9, 2),
}
print(json.dumps(res), flush=True)
