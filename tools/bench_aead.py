#!/usr/bin/env python3
"""Throughput of the AEAD packet kernels (kfec_aead_seal_batch / kfec_aead_open_batch).

    python tools/bench_aead.py [--packets P] [--len L] [--steps K] [--cpu-threads T]

P packets of L bytes (default 4M x 1449 B: the 20:3 wire's data packets at kcp_mtu 1440) sealed and opened
in chacha20 and xchacha20 modes.  Prints one JSON line: per mode, kernel ms (HIP events on the launch stream,
median) and plaintext GB/s; opened packets are checked (every tag verifies, bytes equal).  With
--cpu-threads, tools/cpu_aead (OpenSSL ChaCha20-Poly1305, 1 and T threads) is timed beside it.
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def cpu_baseline(L, threads):
    exe = os.path.join(ROOT, "tools", "cpu_aead")
    if not os.path.exists(exe):
        return None
    res = {}
    for cipher in ("chacha", "gcm"):
        for t, packets in ((1, 400000), (threads, 400000 * threads)):
            out = subprocess.run([exe, str(packets), str(L), str(t)] + (["gcm"] if cipher == "gcm" else []),
                                 capture_output=True, text=True, timeout=300)
            if out.returncode == 0:
                res[f"{cipher}_threads_{t}"] = json.loads(out.stdout)
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--packets", type=int, default=1 << 22)
    ap.add_argument("--len", type=int, default=1449)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--cpu-threads", type=int, default=0)
    ap.add_argument("--no-verify", action="store_true", help="timing ablations (KFEC_LIB) whose output is wrong")
    args = ap.parse_args()
    import torch
    from kcptube_amd.aead import AeadCipher

    dev = torch.device("cuda:0")
    P, L = args.packets, args.len
    pitch = (L + 18 + 3) // 4 * 4
    src = torch.randint(0, 256, (P * pitch,), dtype=torch.uint8, device=dev)
    off = torch.arange(P, dtype=torch.int64, device=dev) * pitch
    ln = torch.full((P,), L, dtype=torch.int32, device=dev)
    ivs = torch.randint(-32768, 32768, (P,), dtype=torch.int16, device=dev)
    sealed = torch.empty((P, pitch), dtype=torch.uint8, device=dev)
    slen = torch.empty(P, dtype=torch.int32, device=dev)
    plain = torch.empty((P, pitch), dtype=torch.uint8, device=dev)
    plen = torch.empty(P, dtype=torch.int32, device=dev)
    ok = torch.empty(P, dtype=torch.uint8, device=dev)
    s = torch.cuda.current_stream()
    e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    res = {"metric": "AEAD packet seal/open GB/s of plaintext (chacha20 / xchacha20 / aes_gcm / aes_ocb modes, device-resident)",
           "packets": P, "len": L}
    good = True
    for name in ("chacha20", "xchacha20", "aes_gcm", "aes_ocb"):
        c = AeadCipher(name, b"kcptube bench password")
        ts, to = [], []
        for i in range(args.steps + 2):
            e[0].record(s)
            c.seal(src, off, ln, ivs, sealed, slen)
            e[1].record(s)
            c.open_(sealed.view(-1), off, slen, plain, plen, ok)
            e[2].record(s)
            torch.cuda.synchronize()
            if i >= 2:
                ts.append(e[0].elapsed_time(e[1]))
                to.append(e[1].elapsed_time(e[2]))
        good = good and bool(ok.all().item()) and bool((plen == L).all().item())
        good = good and torch.equal(plain.view(P, pitch)[:, :L], src.view(P, pitch)[:, :L])
        byt = P * L
        res[name] = {"seal_ms": round(float(np.median(ts)), 4), "open_ms": round(float(np.median(to)), 4),
                     "seal_GBps": round(byt / (np.median(ts) * 1e-3) / 1e9, 1),
                     "open_GBps": round(byt / (np.median(to) * 1e-3) / 1e9, 1)}
    res["verified"] = good
    if args.no_verify:
        good = True
    if args.cpu_threads:
        res["cpu_openssl"] = cpu_baseline(L, args.cpu_threads)
    print(json.dumps(res), flush=True)
    if not good:
        sys.exit(3)


if __name__ == "__main__":
    main()
