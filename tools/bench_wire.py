#!/usr/bin/env python3
"""Device-resident packet-in / packet-out throughput of the whole FEC wire path (include/kfec_frame.h).

    python tools/bench_wire.py [--groups G] [--steps K] [--ragged]

fec=20:3, kcp_mtu=1440.  Send step: frame_data -> encode_batch -> pack (data + redundant packets), and the
fused form encode_framed (frame + encode in one kernel, checked equal) -> pack, and encode_pack (the encoder
also writes the data packets; then the redundant ones: two launches, checked equal).
Receive step (every group lost 3 data packets, worst case): unpack -> scatter -> frame_shards -> decode_batch
-> unframe, and the fused form unpack -> scatter -> decode_framed (frame_shards + decode in one kernel, checked
equal) -> unframe.  Datagrams are 1440 B (bulk traffic) or, with --ragged, uniform 0..1440 B.  Prints one JSON line:
payload GiB/s of each direction and per-kernel times / HBM GB/s (algorithmic bytes per launch / HIP-event
time on the launch stream).
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
    ap.add_argument("--groups", type=int, default=1 << 18)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--ragged", action="store_true")
    args = ap.parse_args()
    import torch
    from kcptube_amd import FecCode
    from kcptube_amd.frame import FecFrame

    K, N, mtu = 20, 23, 1440
    R = N - K
    B = mtu + 2
    pitch = (B + 3) // 4 * 4
    G = args.groups
    dev = torch.device("cuda:0")
    c = FecCode(K, N)
    fr = FecFrame(c)
    gen = torch.Generator(device=dev).manual_seed(1)
    # datagram arena: slot i at i * mtu_pad (offsets need not be aligned; these are, as a socket batch's)
    mtu_pad = (mtu + 3) // 4 * 4
    arena = torch.randint(0, 256, (G * K * mtu_pad,), dtype=torch.uint8, device=dev, generator=gen)
    off = torch.arange(G * K, dtype=torch.int64, device=dev) * mtu_pad
    if args.ragged:
        lens = torch.randint(0, mtu + 1, (G * K,), dtype=torch.int32, device=dev, generator=gen)
    else:
        lens = torch.full((G * K,), mtu, dtype=torch.int32, device=dev)
    d_len = lens.to(torch.int16)
    data = torch.empty((G, K, pitch), dtype=torch.uint8, device=dev)
    align = torch.empty(G, dtype=torch.int16, device=dev)
    parity = torch.empty((G, R, pitch), dtype=torch.uint8, device=dev)
    pkt_pitch = (13 + B + 3) // 4 * 4
    pkt = torch.empty((G, N, pkt_pitch), dtype=torch.uint8, device=dev)
    plen = torch.empty((G, N), dtype=torch.int16, device=dev)
    sn = torch.arange(G, dtype=torch.int32, device=dev)
    conv = torch.full((G,), 0x1234, dtype=torch.int32, device=dev)

    # receive side: the packets of every group except data packets 0, 7, 13 (3 lost per group)
    lost = {0, 7, 13}
    keep_s = torch.tensor([s for s in range(N) if s not in lost], dtype=torch.int64, device=dev)
    P = G * keep_s.numel()
    r_off = ((torch.arange(G, dtype=torch.int64, device=dev)[:, None] * N + keep_s[None, :]) * pkt_pitch).reshape(-1)
    hdr = torch.empty((P, 24), dtype=torch.uint8, device=dev)
    present = torch.empty((G, 4), dtype=torch.int64, device=dev)
    toff = torch.empty(G * N, dtype=torch.int64, device=dev)
    tlen = torch.empty(G * N, dtype=torch.int16, device=dev)
    rdata = torch.empty((G, K, pitch), dtype=torch.uint8, device=dev)
    rpar = torch.empty((G, R, pitch), dtype=torch.uint8, device=dev)
    ralign = torch.empty(G, dtype=torch.int16, device=dev)
    out = torch.empty((G, R, pitch), dtype=torch.uint8, device=dev)
    idx = torch.empty((G, R), dtype=torch.uint8, device=dev)
    st = torch.empty(G, dtype=torch.uint8, device=dev)
    ws = c.decode_workspace(G)
    rec_len = torch.empty((G, R), dtype=torch.int16, device=dev)
    dst = torch.empty((G, R, pitch), dtype=torch.uint8, device=dev)
    flat = pkt.view(-1)
    parity2 = torch.empty_like(parity)
    align2 = torch.empty_like(align)
    out2, idx2, st2, ralign2 = torch.empty_like(out), torch.empty_like(idx), torch.empty_like(st), torch.empty_like(ralign)
    ws2 = c.decode_workspace(G)
    parity3, align3 = torch.empty_like(parity), torch.empty_like(align)
    pkt3, plen3 = torch.empty_like(pkt), torch.empty_like(plen)

    s = torch.cuda.current_stream()
    names = ["frame_data", "encode", "pack", "unpack", "scatter", "frame_shards", "decode", "unframe", "encode_framed",
             "decode_framed", "encode_pack"]
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(len(names) + 1)]
    times = {n: [] for n in names}

    def step(timed):
        if timed:
            ev[0].record(s)
        fr.frame_data(arena, off, d_len, data, align, B)
        if timed:
            ev[1].record(s)
        c.encode_batch(data, parity, B=B)
        if timed:
            ev[2].record(s)
        fr.pack(arena, off, d_len, parity, align, sn, conv, 77, pkt, plen)
        if timed:
            ev[3].record(s)
        fr.unpack(flat, r_off, r_len, hdr)
        if timed:
            ev[4].record(s)
        present.zero_()
        fr.scatter(hdr, present, toff, tlen, G, sn_base=0)
        if timed:
            ev[5].record(s)
        fr.frame_shards(flat, toff, tlen, present, rdata, rpar, ralign, B)
        if timed:
            ev[6].record(s)
        c.decode_batch(rdata, rpar, present, out, idx, st, ws, B=B)
        if timed:
            ev[7].record(s)
        fr.unframe(out, idx, rec_len, B, dst=dst)
        if timed:
            ev[8].record(s)
        fr.encode_framed(arena, off, d_len, parity2, align2, B)  # fused frame_data + encode (same parity)
        if timed:
            ev[9].record(s)
        fr.decode_framed(flat, toff, tlen, present, out2, idx2, st2, ralign2, ws2, B)  # fused frame_shards + decode
        if timed:
            ev[10].record(s)
        # the whole send side in two launches: framed encode writing the data packets, then the redundant ones
        fr.encode_pack(arena, off, d_len, parity3, align3, sn, conv, 77, pkt3, plen3, B)
        if timed:
            ev[11].record(s)

    # received packet lengths (what recvmmsg reports) -- identical every step, so taken once up front
    fr.frame_data(arena, off, d_len, data, align, B)
    c.encode_batch(data, parity, B=B)
    fr.pack(arena, off, d_len, parity, align, sn, conv, 77, pkt, plen)
    r_len = plen.view(-1).to(torch.int32).view(G, N)[:, keep_s].reshape(-1).contiguous()
    for _ in range(2):
        step(False)
    torch.cuda.synchronize()
    for _ in range(args.steps):
        step(True)
        torch.cuda.synchronize()
        for i, n in enumerate(names):
            times[n].append(ev[i].elapsed_time(ev[i + 1]))
    med = {n: float(np.median(v)) for n, v in times.items()}

    # correctness of what was timed: every lost datagram recovered bit-exact
    torch.cuda.synchronize()
    rl = rec_len.cpu().numpy().view(np.uint16)
    ln = lens.cpu().numpy().reshape(G, K)
    lost_sorted = sorted(lost)
    ok = bool((st.cpu().numpy() == 0).all()) and all((rl[:, t] == ln[:, i]).all() for t, i in enumerate(lost_sorted))
    chk = min(G, 512)
    a_np = arena[: chk * K * mtu_pad].cpu().numpy().reshape(chk, K, mtu_pad)
    d_np = dst[:chk].cpu().numpy()
    for g in range(chk):
        for t, i in enumerate(lost_sorted):
            n = int(ln[g, i])
            ok = ok and np.array_equal(d_np[g, t, :n], a_np[g, i, :n])

    payload = float(lens.sum().item())  # datagram bytes per step
    lost_bytes = float(ln[:, lost_sorted].sum())
    pk = plen.cpu().numpy().view(np.uint16).astype(np.int64)
    pkt_bytes = float(pk.sum())
    kept_pkt_bytes = float(pk[:, [s_ for s_ in range(N) if s_ not in lost]].sum())
    slot_bytes = G * K * B
    # algorithmic HBM bytes per launch
    alg = {
        "frame_data": payload + slot_bytes,
        "encode": G * (K + R) * B,
        "pack": payload + G * R * B + pkt_bytes,
        "unpack": P * 13 + P * 24,
        "scatter": 3 * P * 24 + P * 10,
        "frame_shards": (kept_pkt_bytes - P * 9) + G * K * B,
        "decode": G * K * B + G * R * B,
        "unframe": lost_bytes * 2,
        "encode_framed": payload + G * R * B,
        "decode_framed": (kept_pkt_bytes - P * 9 - G * R * 4) + G * R * B,
        "encode_pack": payload + G * R * B * 2 + pkt_bytes,
    }
    send_ms = med["frame_data"] + med["encode"] + med["pack"]
    send_fused_ms = med["encode_framed"] + med["pack"]
    recv_ms = sum(med[n] for n in names[3:8])
    recv_fused_ms = med["unpack"] + med["scatter"] + med["decode_framed"] + med["unframe"]
    send_fused2_ms = med["encode_pack"]
    ok = ok and torch.equal(parity2, parity) and torch.equal(align2, align)
    ok = ok and torch.equal(idx2, idx) and torch.equal(st2, st) and torch.equal(ralign2, ralign)
    B4 = (B + 3) // 4 * 4
    ok = ok and torch.equal(out2[:, :, :B4], out[:, :, :B4])
    ok = ok and torch.equal(plen3, plen) and torch.equal(align3, align)
    pk_np, pk3_np, pl_np = pkt.cpu().numpy(), pkt3.cpu().numpy(), plen.cpu().numpy().view(np.uint16)
    for g in range(min(G, 256)):  # packet bytes below each packet's length (the rest of the row is scratch)
        for s_ in range(N):
            n_ = int(pl_np[g, s_])
            ok = ok and np.array_equal(pk_np[g, s_, :n_], pk3_np[g, s_, :n_])
    res = {
        "metric": "FEC wire path payload GiB/s (device-resident, packet-in/packet-out), fec=20:3 kcp_mtu=1440",
        "groups": G, "ragged": args.ragged, "steps": args.steps,
        "send_GiBps": round(payload / (send_ms * 1e-3) / 2**30, 2),
        "recv_GiBps": round(payload / (recv_ms * 1e-3) / 2**30, 2),
        "send_fused_GiBps": round(payload / (send_fused_ms * 1e-3) / 2**30, 2),
        "recv_fused_GiBps": round(payload / (recv_fused_ms * 1e-3) / 2**30, 2),
        "send_encode_pack_GiBps": round(payload / (send_fused2_ms * 1e-3) / 2**30, 2),
        "send_encode_pack_ms": round(send_fused2_ms, 4),
        "recv_fused_ms": round(recv_fused_ms, 4),
        "send_ms": round(send_ms, 4), "send_fused_ms": round(send_fused_ms, 4), "recv_ms": round(recv_ms, 4),
        "kernels": {n: {"ms": round(med[n], 4), "alg_GBps": round(alg[n] / (med[n] * 1e-3) / 1e9, 1)} for n in names},
        "verified_bit_exact": ok,
    }
    print(json.dumps(res), flush=True)
    if not ok:
        sys.exit(3)


if __name__ == "__main__":
    main()
