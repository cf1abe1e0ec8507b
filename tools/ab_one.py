#!/usr/bin/env python3
"""Time encode / decode of one library build (KFEC_LIB env) on fec=K:R groups; prints one JSON line."""
import json, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from kcptube_amd import FecCode

K, N, B, G = (int(x) for x in (sys.argv[1:5] if len(sys.argv) > 4 else (20, 23, 1440, 1 << 20)))
iters = int(os.environ.get("AB_ITERS", "10"))
P = max(B, int(os.environ.get("AB_PITCH", "0")))  # shard slot pitch (default B: rows back to back)
R = N - K
dev = torch.device("cuda:0")
c = FecCode(K, N)
data = torch.empty((G, K, P), dtype=torch.uint8, device=dev)
par = torch.empty((G, R, P), dtype=torch.uint8, device=dev)
masks = torch.empty((G, 4), dtype=torch.int64, device=dev)
out = torch.empty((G, R, P), dtype=torch.uint8, device=dev)
idx = torch.empty((G, R), dtype=torch.uint8, device=dev)
st = torch.empty((G,), dtype=torch.uint8, device=dev)
ws = c.decode_workspace(G)
c.synth(data, 1, B=B)
mode = os.environ.get("AB_ERASE", "random" if os.environ.get("AB_RANDOM") else "data")
if mode == "random":  # bench config 10:3dec: random 1..R erasures over all N shards
    c.erasure_masks(masks, 0x5EED0001, N, R, 1)
elif mode == "none":  # nothing lost
    c.erasure_masks(masks, 1, K, 0, 0)
elif mode.startswith("iid:"):  # i.i.d. loss, ppm per shard
    c.erasure_masks(masks, 0x5EED0001, N, int(mode[4:]), 2)
elif mode == "data":  # the first min(R, K) data shards of every group lost
    c.erasure_masks(masks, 1, K, min(R, K))
else:
    sys.exit(f"AB_ERASE={mode!r}: expected data, random, none or iid:<ppm>")
s = torch.cuda.current_stream()
e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
enc, dec = [], []
for i in range(iters + 2):
    e[0].record(s); c.encode_batch(data, par, B=B); e[1].record(s)
    c.decode_batch(data, par, masks, out, idx, st, ws, B=B); e[2].record(s)
    torch.cuda.synchronize()
    if i >= 2:
        enc.append(e[0].elapsed_time(e[1])); dec.append(e[1].elapsed_time(e[2]))
enc.sort(); dec.sort()
eb = G * (K + R) * B
db = G * (K + min(R, K)) * B
print(json.dumps({"lib": os.path.basename(os.environ.get("KFEC_LIB", "libkfec.so")), "erase": mode, "enc_ms": enc[len(enc)//2],
                  "dec_ms": dec[len(dec)//2], "enc_GBps": round(eb / enc[len(enc)//2] / 1e6, 1),
                  "dec_GBps": round(db / dec[len(dec)//2] / 1e6, 1)}), flush=True)
