#!/usr/bin/env python3
"""Shard-row pitch A/B at fec=20:3, B=1440, 1M groups: encode / decode kernel time for rows of 1440 bytes
back to back versus rows padded to 64- or 128-byte boundaries (the shard bytes and the algorithmic traffic
are the same; only the row alignment in HBM changes).  Interleaved rounds; prints one JSON line per pitch
per round, with the device-side check that every recovered shard equals its original.

    python tools/pitch_ab.py [rounds] [pitch ...]
    PITCH_AB_CFG=10:13:1400:random python tools/pitch_ab.py 3 1400 1408   # other configs (K:N:B[:random])
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from kcptube_amd import FecCode  # noqa: E402

rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
pitches = [int(x) for x in sys.argv[2:]] or [1440, 1472, 1536]
cfg = os.environ.get("PITCH_AB_CFG", "20:23:1440").split(":")
K, N, B, G = int(cfg[0]), int(cfg[1]), int(cfg[2]), 1 << 20
rnd = len(cfg) > 3 and cfg[3] == "random"
R = N - K
dev = torch.device("cuda:0")
c = FecCode(K, N)
st = torch.empty((G,), dtype=torch.uint8, device=dev)
idx = torch.empty((G, R), dtype=torch.uint8, device=dev)
masks = torch.empty((G, 4), dtype=torch.int64, device=dev)
ws = c.decode_workspace(G, device=dev)
if rnd:  # bench config 10:3dec: 1..R erasures anywhere in the N shards
    c.erasure_masks(masks, 0x5EED0001, N, R, True)
else:
    c.erasure_masks(masks, 1, K, R)
mism = torch.zeros(1, dtype=torch.int64, device=dev)
s = torch.cuda.current_stream()
for r in range(rounds):
    for pitch in pitches:
        data = torch.empty((G, K, pitch), dtype=torch.uint8, device=dev)
        par = torch.empty((G, R, pitch), dtype=torch.uint8, device=dev)
        out = torch.empty((G, R, pitch), dtype=torch.uint8, device=dev)
        c.synth(data, 1, B=B)
        e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
        enc, dec = [], []
        for i in range(8):
            e[0].record(s)
            c.encode_batch(data, par, B=B)
            e[1].record(s)
            c.decode_batch(data, par, masks, out, idx, st, ws, B=B)
            e[2].record(s)
            torch.cuda.synchronize()
            if i >= 2:
                enc.append(e[0].elapsed_time(e[1]))
                dec.append(e[1].elapsed_time(e[2]))
        mism.zero_()
        c.verify_recovered(data, out, idx, mism, B=B)
        torch.cuda.synchronize()
        enc.sort()
        dec.sort()
        print(json.dumps({"pitch": pitch, "enc_ms": round(enc[len(enc) // 2], 4), "dec_ms": round(dec[len(dec) // 2], 4),
                          "mismatched_shards": int(mism.item())}), flush=True)
        del data, par, out
        torch.cuda.empty_cache()
