#!/usr/bin/env python3
"""End-to-end rate from pinned host memory: the path starts and ends in UDP socket buffers (SURVEY 8(d)
"End-to-end"; north_star: "the end-to-end rate including pinned hipMemcpyAsync to and from the GPU").

Encode (the sender, fec_maker): the K framed data slots of each group in pinned host memory -> hipMemcpyAsync
H2D -> kfec_encode_batch -> the R parity shards D2H.  K + R shards cross the link per group.

Decode (the receiver, fec_find_missings -> decode): what a receiver holds is the packets that ARRIVED, nothing
else.  With R data packets lost per group (the bench's worst case) that is K packets per group -- K - R data
packets (9-byte header + datagram) and R redundant packets (13-byte header + parity shard) -- back to back in a
pinned receive arena of 1456-byte packet slots, as the socket reads left them, plus the receiver's bookkeeping
(kfec_rx: per shard the payload offset and length, per group the presence bits).  Those go H2D; the fused
kfec_decode_framed_batch (the kfec_rxq flush's kernel) selects each group's K shares from the presence bits,
frames the data shards on the fly and recovers the missing ones; the R recovered slots (+ their ids and the
group status) come back D2H.  K + R shards cross the link per group; the erased slots never do.

Chunks of C groups are pipelined over NS streams (the copies of chunk i+1 overlap the kernel of chunk i).  Both
directions are verified on the device after the timed runs (parity against the device-resident encode of the
same groups, recovered slots against the framed originals).  The reference coder on the host's cores runs in the
same process afterwards (bench.py's cpu_baseline: the compiled reference, all usable cores and one core) unless
--no-cpu.  Prints one JSON line: GiB/s of payload (G*K*B) per direction and for the round trip, the bytes that
actually crossed the link per group and their rate, and the GPU/CPU ratios at this host-memory boundary.

    python tools/e2e.py [--groups 262144] [--chunk 16384] [--streams 3] [--K 20 --R 3 --B 1440] [--no-cpu]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from kcptube_amd import FecCode  # noqa: E402
from kcptube_amd.frame import FecFrame, PKT_DATA_HEADER, PKT_REDUNDANT_HEADER  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--groups", type=int, default=1 << 18)
ap.add_argument("--chunk", type=int, default=1 << 14)
ap.add_argument("--streams", type=int, default=3)
ap.add_argument("--K", type=int, default=20)
ap.add_argument("--R", type=int, default=3)
ap.add_argument("--B", type=int, default=1440)
ap.add_argument("--iters", type=int, default=3)
ap.add_argument("--no-cpu", action="store_true")
ap.add_argument("--cpu-seconds", type=float, default=16.0)
args = ap.parse_args()
K, R, B, G, C = args.K, args.R, args.B, args.groups, args.chunk
N = K + R
assert G % C == 0 and R <= K
SEED = 0x5EED0001
SLOT = (max(PKT_REDUNDANT_HEADER + B, PKT_DATA_HEADER + B - 2) + 15) // 16 * 16  # one received packet per slot
dev = torch.device("cuda:0")
c = FecCode(K, N)
fr = FecFrame(c)
NS = args.streams
nchunks = G // C

# ---- untimed set-up: datagrams, their framed slots and parity (device), the host buffers ----------------------
# datagram j of group g = B - 2 synthetic bytes (full-size KCP segments: kcp_mtu = B - 2 + the 2-byte length)
h_data = torch.empty((G, K, B), dtype=torch.uint8).pin_memory()   # sender: framed data slots [len][datagram]
h_par = torch.empty((G, R, B), dtype=torch.uint8).pin_memory()    # sender output: parity shards
h_arena = torch.empty((G, K, SLOT), dtype=torch.uint8).pin_memory()  # receiver: the K packets that arrived
h_off = torch.empty((G, N), dtype=torch.int64).pin_memory()       # receiver bookkeeping (kfec_rx)
h_len = torch.empty((G, N), dtype=torch.int16).pin_memory()
h_present = torch.empty((G, 4), dtype=torch.int64).pin_memory()
h_out = torch.empty((G, R, B), dtype=torch.uint8).pin_memory()    # recovered slots
h_oidx = torch.empty((G, R), dtype=torch.uint8).pin_memory()
h_st = torch.empty((G,), dtype=torch.uint8).pin_memory()

gen = torch.empty((C, K, B), dtype=torch.uint8, device=dev)
slots = torch.empty((C, K, B), dtype=torch.uint8, device=dev)
par = torch.empty((C, R, B), dtype=torch.uint8, device=dev)
masks = torch.empty((C, 4), dtype=torch.int64, device=dev)
src_off = (torch.arange(C * K, dtype=torch.int64, device=dev) * B + 2)
src_len = torch.full((C * K,), B - 2, dtype=torch.int16, device=dev)
align = torch.empty((C,), dtype=torch.int16, device=dev)
kk = torch.arange(K, device=dev)
for ci in range(nchunks):
    g0 = ci * C
    c.synth(gen, SEED, g0=g0)                       # bytes [2, B) of each slot are the datagram
    fr.frame_data(gen.reshape(-1), src_off, src_len, slots, align, B)  # [BE16 B-2][datagram]
    c.encode_batch(slots, par)
    c.erasure_masks(masks, SEED, K, R, 0, g0=g0)    # R data packets lost per group
    # the arrived packets, ascending shard id: present data j (9-byte header + datagram), then the parity shards
    pm = masks[:, 0]
    bits = ((pm.unsqueeze(1) >> kk) & 1).bool()     # [C][K] data present
    ids = torch.cat([kk.expand(C, K)[bits].view(C, K - R), torch.arange(K, N, device=dev).expand(C, R)], 1)
    arena = torch.zeros((C, K, SLOT), dtype=torch.uint8, device=dev)
    dsel = ids[:, :K - R]
    arena[:, :K - R, PKT_DATA_HEADER:PKT_DATA_HEADER + B - 2] = torch.gather(
        slots[:, :, 2:], 1, dsel.unsqueeze(-1).expand(C, K - R, B - 2))
    arena[:, K - R:, PKT_REDUNDANT_HEADER:PKT_REDUNDANT_HEADER + B] = par
    arena[:, :K - R, 8] = dsel.to(torch.uint8)      # sub_sn bytes of the headers (the rest: zeros)
    arena[:, K - R:, 8] = torch.arange(K, N, device=dev, dtype=torch.uint8)
    # the receiver's table: payload offset (relative to the chunk's arena) and length per present shard
    off = torch.zeros((C, N), dtype=torch.int64, device=dev)
    ln = torch.zeros((C, N), dtype=torch.int16, device=dev)
    rank = torch.arange(K, device=dev).expand(C, K)
    base = (torch.arange(C, device=dev).unsqueeze(1) * K + rank) * SLOT
    hdr = torch.where(ids < K, PKT_DATA_HEADER, PKT_REDUNDANT_HEADER)
    off.scatter_(1, ids, base + hdr)
    ln.scatter_(1, ids, torch.where(ids < K, B - 2, B).to(torch.int16))
    h_data[g0:g0 + C].copy_(slots)
    h_par[g0:g0 + C].copy_(par)
    h_arena[g0:g0 + C].copy_(arena)
    h_off[g0:g0 + C].copy_(off)
    h_len[g0:g0 + C].copy_(ln)
    h_present[g0:g0 + C].copy_(masks)
torch.cuda.synchronize()
del arena, off, ln

streams = [torch.cuda.Stream() for _ in range(NS)]
d_data = [torch.empty((C, K, B), dtype=torch.uint8, device=dev) for _ in range(NS)]
d_par = [torch.empty((C, R, B), dtype=torch.uint8, device=dev) for _ in range(NS)]
d_arena = [torch.empty((C * K * SLOT,), dtype=torch.uint8, device=dev) for _ in range(NS)]
d_off = [torch.empty((C, N), dtype=torch.int64, device=dev) for _ in range(NS)]
d_len = [torch.empty((C, N), dtype=torch.int16, device=dev) for _ in range(NS)]
d_pres = [torch.empty((C, 4), dtype=torch.int64, device=dev) for _ in range(NS)]
d_out = [torch.empty((C, R, B), dtype=torch.uint8, device=dev) for _ in range(NS)]
d_idx = [torch.empty((C, R), dtype=torch.uint8, device=dev) for _ in range(NS)]
d_st = [torch.empty((C,), dtype=torch.uint8, device=dev) for _ in range(NS)]
d_al = [torch.empty((C,), dtype=torch.int16, device=dev) for _ in range(NS)]
d_ws = [c.decode_workspace(C) for _ in range(NS)]
h_par_out = torch.empty_like(h_par).pin_memory()


def run_encode():
    for ci in range(nchunks):
        g0, k = ci * C, ci % NS
        with torch.cuda.stream(streams[k]):
            d_data[k].copy_(h_data[g0:g0 + C], non_blocking=True)
            c.encode_batch(d_data[k], d_par[k], stream=streams[k])
            h_par_out[g0:g0 + C].copy_(d_par[k], non_blocking=True)
    torch.cuda.synchronize()


def run_decode():
    for ci in range(nchunks):
        g0, k = ci * C, ci % NS
        s = streams[k]
        with torch.cuda.stream(s):
            d_arena[k].copy_(h_arena[g0:g0 + C].view(-1), non_blocking=True)
            d_off[k].copy_(h_off[g0:g0 + C], non_blocking=True)
            d_len[k].copy_(h_len[g0:g0 + C], non_blocking=True)
            d_pres[k].copy_(h_present[g0:g0 + C], non_blocking=True)
            fr.decode_framed(d_arena[k], d_off[k], d_len[k], d_pres[k], d_out[k], d_idx[k], d_st[k], d_al[k],
                             d_ws[k], B, stream=s)
            h_out[g0:g0 + C].copy_(d_out[k], non_blocking=True)
            h_oidx[g0:g0 + C].copy_(d_idx[k], non_blocking=True)
            h_st[g0:g0 + C].copy_(d_st[k], non_blocking=True)
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

# ---- verification (untimed): parity and every recovered slot against the sender's framed slots --------------
ok = bool(torch.equal(h_par_out, h_par))
mism = torch.zeros(1, dtype=torch.int64, device=dev)
for ci in range(nchunks):
    g0 = ci * C
    d_data[0].copy_(h_data[g0:g0 + C])
    d_out[0].copy_(h_out[g0:g0 + C])
    d_idx[0].copy_(h_oidx[g0:g0 + C])
    c.verify_recovered(d_data[0], d_out[0], d_idx[0], mism)
torch.cuda.synchronize()
n_rec = int((h_oidx != 0xFF).sum())
ok = ok and int(mism.item()) == 0 and n_rec == G * R and int(h_st.max()) == 0

payload = G * K * B
enc_link = G * (K + R) * B                                   # K slots in, R parity out
dec_in = G * (K * SLOT + N * 10 + 32)                        # the K arrived packets + the receiver's tables
dec_out = G * (R * B + R + 1)                                # recovered slots + ids + status
res = {
    "what": "end-to-end from pinned host memory (H2D + kernel + D2H, %d streams, %d-group chunks); decode moves only "
            "the K packets that arrived per group (receive arena + kfec_rx tables) and the R recovered slots" % (NS, C),
    "config": f"fec={K}:{R} B={B} groups={G}, {R} data packets lost per group",
    "encode_GiBps": round(payload / te / 2**30, 2),
    "decode_GiBps": round(payload / td / 2**30, 2),
    "roundtrip_GiBps": round(payload / (te + td) / 2**30, 2),
    "encode_link_bytes_per_group": enc_link // G,
    "decode_link_bytes_per_group": (dec_in + dec_out) // G,
    "decode_link_shards_per_group": {"in": K, "out": R},
    "encode_pcie_GBps": round(enc_link / te / 1e9, 2),
    "decode_pcie_GBps": round((dec_in + dec_out) / td / 1e9, 2),
    "decode_h2d_GBps": round(dec_in / td / 1e9, 2),
    "verified_bit_exact": ok,
}
if not args.no_cpu:
    import bench
    cb = bench.cpu_baseline(K, N, B, K, R, 0, args.cpu_seconds, 1 << 16)
    res["cpu_baseline"] = cb
    if cb.get("value"):
        res["gpu_vs_cpu_all_cores"] = round(res["roundtrip_GiBps"] / cb["value"], 3)
        res["gpu_vs_cpu_one_core"] = round(res["roundtrip_GiBps"] / cb["value_1core"], 2)
print(json.dumps(res), flush=True)
sys.exit(0 if ok else 3)
