#!/usr/bin/env python3
"""Small driver for counter runs: N encodes (and decodes) of G groups at fec=K:R, block B."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from kcptube_amd import FecCode
K, N, B, G, it = (int(x) for x in sys.argv[1:6])
dec = len(sys.argv) > 6 and sys.argv[6] == "dec"
R = N - K
c = FecCode(K, N)
dev = torch.device("cuda:0")
data = torch.empty((G, K, B), dtype=torch.uint8, device=dev)
par = torch.empty((G, R, B), dtype=torch.uint8, device=dev)
c.synth(data, 1)
for _ in range(it):
    c.encode_batch(data, par)
if dec:
    masks = torch.empty((G, 4), dtype=torch.int64, device=dev)
    c.erasure_masks(masks, 1, K, min(R, K))
    out = torch.empty((G, R, B), dtype=torch.uint8, device=dev)
    idx = torch.empty((G, R), dtype=torch.uint8, device=dev)
    st = torch.empty((G,), dtype=torch.uint8, device=dev)
    ws = c.decode_workspace(G)
    for _ in range(it):
        c.decode_batch(data, par, masks, out, idx, st, ws)
torch.cuda.synchronize()
