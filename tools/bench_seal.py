#!/usr/bin/env python3
"""Throughput of the per-packet integrity kernels (kfec_seal_batch / kfec_open_batch).

    python tools/bench_seal.py [--packets P] [--len L] [--steps K]

P packets of L bytes (default 4M x 1449 B = the 20:3 wire's data packets at kcp_mtu 1440) sealed and opened
in both non-AEAD modes, and in place in checksum mode.  Prints one JSON line: per mode, kernel ms (HIP
events, median) and algorithmic HBM GB/s (read L + write L + 2 per packet; in place: read L, write the
trailer dword).  Opened packets are checked (all checksums good, bytes equal).
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--packets", type=int, default=1 << 22)
    ap.add_argument("--len", type=int, default=1449)
    ap.add_argument("--steps", type=int, default=10)
    args = ap.parse_args()
    import torch
    from kcptube_amd.frame import SEAL_CHECKSUM, SEAL_PLAIN_XOR, open_, seal

    dev = torch.device("cuda:0")
    P, L = args.packets, args.len
    pitch = (L + 2 + 3) // 4 * 4
    src = torch.randint(0, 256, (P * pitch,), dtype=torch.uint8, device=dev)
    off = torch.arange(P, dtype=torch.int64, device=dev) * pitch
    ln = torch.full((P,), L, dtype=torch.int32, device=dev)
    sealed = torch.empty((P, pitch), dtype=torch.uint8, device=dev)
    slen = torch.empty(P, dtype=torch.int32, device=dev)
    plain = torch.empty((P, pitch), dtype=torch.uint8, device=dev)
    plen = torch.empty(P, dtype=torch.int32, device=dev)
    ok = torch.empty(P, dtype=torch.uint8, device=dev)
    s = torch.cuda.current_stream()
    e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    res = {"metric": "packet seal/open GB/s (checksum16 + xor modes, device-resident)", "packets": P, "len": L}
    good = True
    for mode, name in ((SEAL_CHECKSUM, "none"), (SEAL_PLAIN_XOR, "plain_xor")):
        ts, to = [], []
        for i in range(args.steps + 2):
            e[0].record(s)
            seal(mode, src, off, ln, sealed, slen)
            e[1].record(s)
            open_(mode, sealed.view(-1), off, slen, plain, plen, ok)
            e[2].record(s)
            torch.cuda.synchronize()
            if i >= 2:
                ts.append(e[0].elapsed_time(e[1]))
                to.append(e[1].elapsed_time(e[2]))
        good = good and bool(ok.all().item()) and bool((plen == L).all().item())
        good = good and torch.equal(plain.view(P, pitch)[:, :L], src.view(P, pitch)[:, :L])
        byt = P * (2 * L + 2)
        res[name] = {"seal_ms": round(float(np.median(ts)), 4), "open_ms": round(float(np.median(to)), 4),
                     "seal_GBps": round(byt / (np.median(ts) * 1e-3) / 1e9, 1),
                     "open_GBps": round(byt / (np.median(to) * 1e-3) / 1e9, 1)}
    # in place, checksum mode (d_dst NULL, as after kfec_pack_batch): the CRC reads the packet, seal writes the
    # 2 trailer bytes, open writes nothing (algorithmic bytes: read L + 2 per packet, write 2 on seal)
    work = src.clone()
    wflat = work.view(-1)
    ti, tio = [], []
    for i in range(args.steps + 2):
        e[0].record(s)
        seal(SEAL_CHECKSUM, wflat, off, ln, None, slen, slot=pitch)
        e[1].record(s)
        open_(SEAL_CHECKSUM, wflat, off, slen, None, plen, ok)
        e[2].record(s)
        torch.cuda.synchronize()
        if i >= 2:
            ti.append(e[0].elapsed_time(e[1]))
            tio.append(e[1].elapsed_time(e[2]))
    good = good and bool(ok.all().item()) and bool((plen == L).all().item())
    good = good and torch.equal(work.view(P, pitch)[:, :L], src.view(P, pitch)[:, :L])
    res["none_in_place"] = {"seal_ms": round(float(np.median(ti)), 4), "open_ms": round(float(np.median(tio)), 4),
                            "seal_GBps": round(P * (L + 2) / (np.median(ti) * 1e-3) / 1e9, 1),
                            "open_GBps": round(P * (L + 2) / (np.median(tio) * 1e-3) / 1e9, 1)}
    res["verified"] = good
    print(json.dumps(res), flush=True)
    if not good:
        sys.exit(3)


if __name__ == "__main__":
    main()
