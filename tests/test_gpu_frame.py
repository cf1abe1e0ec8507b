"""GPU parity tests of the framing and wire layer (include/kfec_frame.h) against oracle/frame_oracle.py.

Bar: bit-exact.  Every kernel is compared byte for byte with the CPU restatement on ragged inputs
(zero-length datagrams, datagrams of exactly B - 2 bytes, too-long datagrams, absent shards, malformed
packets), output slots are pre-filled with a sentinel so that writes outside the documented extent show
up, and the whole send -> lossy channel -> receive path runs on the device and is checked against both the
original datagrams and the oracle's fec_maker / fec_find_missings pipeline.
"""
from __future__ import annotations

import random

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

from oracle import frame_oracle as fo  # noqa: E402

SENT = 0xA5


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from kcptube_amd import load_library
    load_library()
    return torch.device("cuda:0")


def _arena(chunks: list[bytes], dev, pad_to=4):
    """Concatenate byte strings at odd offsets (a 1-3 byte gap after each) into a device arena."""
    rng = random.Random(len(chunks))
    buf = bytearray()
    offs, lens = [], []
    for c in chunks:
        buf += bytes(rng.randint(0, 3))
        offs.append(len(buf))
        lens.append(len(c))
        buf += c
    buf += bytes((-len(buf)) % pad_to + 4)
    a = torch.tensor(np.frombuffer(bytes(buf), np.uint8).copy(), device=dev)
    return a, torch.tensor(offs, dtype=torch.int64, device=dev), lens


def _u16(t):
    return t.cpu().numpy().view(np.uint16)


def _i16(vals, dev):
    return torch.tensor(np.asarray(vals, np.uint16).view(np.int16), device=dev)


def _coder(K, N):
    from kcptube_amd import FecCode
    from kcptube_amd.frame import FecFrame
    c = FecCode(K, N)
    return c, FecFrame(c)


@pytest.mark.parametrize("K,N,B,pitch", [(20, 23, 1442, 1444), (10, 13, 1402, 1408), (3, 5, 7, 8), (1, 2, 2, 4)])
def test_frame_data_matches_oracle(dev, K, N, B, pitch):
    c, fr = _coder(K, N)
    rng = random.Random(B)
    G = 37
    dgs = []
    for g in range(G):
        for i in range(K):
            n = rng.choice([0, 1, B - 2, rng.randint(0, B - 2)])
            if g == 5 and i == K - 1:
                n = B - 1  # too long: the group is flagged
            dgs.append(rng.randbytes(n))
    src, off, lens = _arena(dgs, dev)
    data = torch.full((G, K, pitch), SENT, dtype=torch.uint8, device=dev)
    align = torch.zeros(G, dtype=torch.int16, device=dev)
    fr.frame_data(src, off, _i16(lens, dev), data, align, B)
    torch.cuda.synchronize()
    got, al = data.cpu().numpy(), _u16(align)
    Bp = (B + 3) // 4 * 4
    for g in range(G):
        grp = dgs[g * K:(g + 1) * K]
        cont, a, _ = fo.compact_send(grp)
        if a > B:
            assert al[g] == 0
            assert not got[g, :, :Bp].any()
            continue
        assert al[g] == a
        for i in range(K):
            exp = cont[i * a:(i + 1) * a] + bytes(Bp - a)
            assert got[g, i, :Bp].tobytes() == exp, (g, i)
            assert (got[g, i, Bp:] == SENT).all()


def test_frame_shards_matches_oracle(dev):
    K, N, B, pitch = 20, 23, 1442, 1444
    R = N - K
    c, fr = _coder(K, N)
    rng = random.Random(7)
    G = 41
    chunks, present = [], np.zeros((G, 4), np.uint64)
    cache = []
    for g in range(G):
        pal = rng.randint(2, B)
        have = sorted(rng.sample(range(N), rng.randint(0, N)))
        d = {}
        for s in range(N):
            n = rng.randint(0, B - 2) if s < K else pal
            if g == 3 and s == 0:
                n = B - 1  # a data shard that cannot be framed in B
            d[s] = rng.randbytes(n)
        for s in have:
            present[g, s >> 6] |= np.uint64(1 << (s & 63))
        cache.append({s: d[s] for s in have})
        chunks += [d[s] for s in range(N)]
    src, off, lens = _arena(chunks, dev)
    data = torch.full((G, K, pitch), SENT, dtype=torch.uint8, device=dev)
    par = torch.full((G, R, pitch), SENT, dtype=torch.uint8, device=dev)
    align = torch.zeros(G, dtype=torch.int16, device=dev)
    pres = torch.tensor(present.view(np.int64), device=dev)
    fr.frame_shards(src, off, _i16(lens, dev), pres, data, par, align, B)
    torch.cuda.synchronize()
    gd, gp, al = data.cpu().numpy(), par.cpu().numpy(), _u16(align)
    Bp = (B + 3) // 4 * 4
    for g in range(G):
        slots, a = fo.compact_recv(cache[g], K)
        if a > B:
            assert al[g] == 0
            continue
        assert al[g] == a
        for s in range(N):
            row = gd[g, s] if s < K else gp[g, s - K]
            if s in slots:
                assert row[:Bp].tobytes() == slots[s] + bytes(Bp - a), (g, s)
                assert (row[Bp:] == SENT).all()
            else:
                assert (row == SENT).all(), (g, s)


def test_unframe_matches_oracle(dev):
    K, N, B, pitch = 10, 13, 1402, 1404
    R = N - K
    c, fr = _coder(K, N)
    rng = np.random.default_rng(3)
    G = 53
    out = rng.integers(0, 256, (G, R, pitch), dtype=np.uint8)
    idx = np.full((G, R), 0xFF, np.uint8)
    for g in range(G):
        m = g % (R + 1)
        idx[g, :m] = np.sort(rng.choice(K, m, replace=False))
        for t in range(m):
            n = [0, 1, B - 2, B - 1, 0xFFFF, int(rng.integers(0, B - 1))][(g + t) % 6]
            out[g, t, 0:2] = [n >> 8, n & 0xFF]
    d_out = torch.tensor(out, device=dev)
    d_idx = torch.tensor(idx, device=dev)
    rec_len = torch.zeros((G, R), dtype=torch.int16, device=dev)
    dst_pitch = 1400
    dst = torch.full((G, R, dst_pitch), SENT, dtype=torch.uint8, device=dev)
    fr.unframe(d_out, d_idx, rec_len, B, dst=dst)
    torch.cuda.synchronize()
    rl, gd = _u16(rec_len), dst.cpu().numpy()
    for g in range(G):
        for t in range(R):
            if idx[g, t] == 0xFF:
                assert rl[g, t] == 0xFFFF
                assert (gd[g, t] == SENT).all()
                continue
            exp = fo.extract(out[g, t, :B].tobytes())
            if exp is None:
                assert rl[g, t] == 0xFFFF
                assert (gd[g, t] == SENT).all()
            else:
                n = len(exp)
                assert rl[g, t] == n
                np4 = (n + 3) // 4 * 4
                assert gd[g, t, :n].tobytes() == exp
                assert not gd[g, t, n:np4].any()
                assert (gd[g, t, np4:] == SENT).all()


def test_pack_matches_oracle(dev):
    K, N, B, pitch = 6, 9, 202, 204
    R = N - K
    c, fr = _coder(K, N)
    rng = random.Random(11)
    G = 29
    dgs = [rng.randbytes(rng.choice([0, 3, 200, rng.randint(0, 200)])) for _ in range(G * K)]
    src, off, lens = _arena(dgs, dev)
    parity = np.frombuffer(rng.randbytes(G * R * pitch), np.uint8).reshape(G, R, pitch)
    al = [max(len(d) for d in dgs[g * K:(g + 1) * K]) + 2 for g in range(G)]
    al[4] = 0  # a group whose framing overflowed
    sn = [rng.getrandbits(32) for _ in range(G)]
    conv = [rng.getrandbits(32) for _ in range(G)]
    pkt_pitch = (13 + B + 3) // 4 * 4
    pkt = torch.full((G, N, pkt_pitch), SENT, dtype=torch.uint8, device=dev)
    plen = torch.zeros((G, N), dtype=torch.int16, device=dev)
    ts = 0x89ABCDEF
    fr.pack(src, off, _i16(lens, dev), torch.tensor(parity, device=dev), _i16(al, dev),
            torch.tensor(np.asarray(sn, np.uint32).view(np.int32), device=dev),
            torch.tensor(np.asarray(conv, np.uint32).view(np.int32), device=dev), ts, pkt, plen)
    torch.cuda.synchronize()
    gp, pl = pkt.cpu().numpy(), _u16(plen)
    for g in range(G):
        for s in range(N):
            if s < K:
                exp = fo.data_packet(dgs[g * K + s], sn[g], s, ts)
            elif al[g] == 0:
                assert pl[g, s] == 0
                continue
            else:
                exp = fo.redundant_packet(parity[g, s - K, :al[g]].tobytes(), sn[g], s, conv[g], ts)
            n = len(exp)
            assert pl[g, s] == n
            assert gp[g, s, :n].tobytes() == exp, (g, s)
            n4 = (n + 3) // 4 * 4
            assert not gp[g, s, n:n4].any()
            assert (gp[g, s, n4:] == SENT).all()


def test_pack_which_flags(dev):
    K, N, B = 2, 4, 10
    c, fr = _coder(K, N)
    src, off, lens = _arena([b"ab", b"cde"], dev)
    par = torch.zeros((1, 2, 12), dtype=torch.uint8, device=dev)
    pkt = torch.full((1, N, 28), SENT, dtype=torch.uint8, device=dev)
    plen = torch.full((1, N), -1, dtype=torch.int16, device=dev)
    one = torch.ones(1, dtype=torch.int32, device=dev)
    fr.pack(src, off, _i16(lens, dev), par, _i16([5], dev), one, one, 0, pkt, plen, which=1)
    torch.cuda.synchronize()
    assert list(_u16(plen)[0]) == [11, 12, 0xFFFF, 0xFFFF]
    assert (pkt.cpu().numpy()[0, 2:] == SENT).all()


def test_unpack_and_scatter_match_oracle(dev):
    K, N = 20, 23
    c, fr = _coder(K, N)
    rng = random.Random(13)
    pkts = []
    for p in range(300):
        sub = rng.randrange(N)
        sn = rng.choice([1000, 1001, 1002, rng.getrandbits(32)])
        payload = rng.randbytes(rng.choice([0, 2, 3, 4, 5, rng.randint(0, 1400)]))
        if sub < K:
            pkts.append(fo.data_packet(payload, sn, sub, rng.getrandbits(32)))
        else:
            pkts.append(fo.redundant_packet(payload, sn, sub, rng.getrandbits(32), rng.getrandbits(32)))
        if p % 37 == 0:
            pkts[-1] = pkts[-1][:rng.randint(0, 12)]  # malformed (shorter than its header)
    src, off, lens = _arena(pkts, dev)
    P = len(pkts)
    hdr = torch.zeros((P, 24), dtype=torch.uint8, device=dev)
    fr.unpack(src, off, torch.tensor(lens, dtype=torch.int32, device=dev), hdr)
    torch.cuda.synchronize()
    from kcptube_amd.frame import KIND_DATA, KIND_MALFORMED, KIND_REDUNDANT, pkt_headers
    h = pkt_headers(hdr)
    offs = off.cpu().numpy()
    arena = src.cpu().numpy()
    for p, pk in enumerate(pkts):
        e = fo.parse_packet(pk, K)
        if e is None:
            assert h[p]["kind"] == KIND_MALFORMED
            continue
        assert h[p]["kind"] == (KIND_REDUNDANT if e["redundant"] else KIND_DATA)
        assert (h[p]["timestamp"], h[p]["sn"], h[p]["sub_sn"], h[p]["conv"]) == (
            e["timestamp"], e["sn"], e["sub_sn"], e["conv"])
        n = int(h[p]["payload_len"])
        o = int(h[p]["payload_off"])
        assert n == len(e["payload"]) and arena[o:o + n].tobytes() == e["payload"]
        assert o == offs[p] + (13 if e["redundant"] else 9)
    # scatter into 3 group slots: sn 1000..1002
    G = 3
    present = torch.zeros((G, 4), dtype=torch.int64, device=dev)
    toff = torch.full((G * N,), -1, dtype=torch.int64, device=dev)
    tlen = torch.zeros(G * N, dtype=torch.int16, device=dev)
    fr.scatter(hdr, present, toff, tlen, G, sn_base=1000)
    torch.cuda.synchronize()
    pm = present.cpu().numpy().view(np.uint64)
    to, tl = toff.cpu().numpy(), _u16(tlen)
    expect = {}  # the last packet of each (sn, sub_sn) wins, as the reference cache's assignment
    for p, pk in enumerate(pkts):
        e = fo.parse_packet(pk, K)
        if e and 1000 <= e["sn"] <= 1002:
            expect[(e["sn"] - 1000, e["sub_sn"])] = (e["payload"], int(offs[p]) + (13 if e["redundant"] else 9))
    for g in range(G):
        for s in range(N):
            bit = int(pm[g, s >> 6]) >> (s & 63) & 1
            assert bit == ((g, s) in expect)
            if bit:
                got = arena[to[g * N + s]:to[g * N + s] + tl[g * N + s]].tobytes()
                assert (got, int(to[g * N + s])) == expect[(g, s)]


def test_device_pipeline_end_to_end(dev, oracle):
    """fec_maker -> packets -> loss -> fec_unpack / cache / compact / decode / extract, all on the device, for
    fec=20:3 at kcp_mtu 1440; compared with the original datagrams and with the oracle pipeline."""
    K, N, mtu = 20, 23, 1440
    R = N - K
    B = mtu + 2
    pitch = (B + 3) // 4 * 4
    c, fr = _coder(K, N)
    rng = random.Random(17)
    G = 96
    dgs = [rng.randbytes(rng.choice([0, 24, mtu, rng.randint(0, mtu)])) for _ in range(G * K)]
    src, off, lens = _arena(dgs, dev)
    d_len = _i16(lens, dev)
    data = torch.empty((G, K, pitch), dtype=torch.uint8, device=dev)
    align = torch.zeros(G, dtype=torch.int16, device=dev)
    fr.frame_data(src, off, d_len, data, align, B)
    parity = torch.empty((G, R, pitch), dtype=torch.uint8, device=dev)
    c.encode_batch(data, parity, B=B)
    sn0 = 0xFFFFFFF0  # sn wraps inside the batch
    sns = np.array([(sn0 + g) & 0xFFFFFFFF for g in range(G)], np.uint32)
    conv = np.full(G, 0x4B435054, np.uint32)
    pkt_pitch = (13 + B + 3) // 4 * 4
    pkt = torch.empty((G, N, pkt_pitch), dtype=torch.uint8, device=dev)
    plen = torch.zeros((G, N), dtype=torch.int16, device=dev)
    fr.pack(src, off, d_len, parity, align, torch.tensor(sns.view(np.int32), device=dev),
            torch.tensor(conv.view(np.int32), device=dev), 12345, pkt, plen)
    torch.cuda.synchronize()
    # channel: each group loses 0..R packets, every 8th group loses R + 1 (unrecoverable)
    keep = []
    for g in range(G):
        lost = set(rng.sample(range(N), R + 1 if g % 8 == 7 else rng.randint(0, R)))
        keep += [(g, s) for s in range(N) if s not in lost]
    rng.shuffle(keep)
    pl = _u16(plen)
    k_off = torch.tensor([(g * N + s) * pkt_pitch for g, s in keep], dtype=torch.int64, device=dev)
    k_len = torch.tensor([int(pl[g, s]) for g, s in keep], dtype=torch.int32, device=dev)
    arena = pkt.view(-1)
    P = len(keep)
    hdr = torch.zeros((P, 24), dtype=torch.uint8, device=dev)
    fr.unpack(arena, k_off, k_len, hdr)
    present = torch.zeros((G, 4), dtype=torch.int64, device=dev)
    toff = torch.zeros(G * N, dtype=torch.int64, device=dev)
    tlen = torch.zeros(G * N, dtype=torch.int16, device=dev)
    fr.scatter(hdr, present, toff, tlen, G, sn_base=sn0)
    rdata = torch.full((G, K, pitch), SENT, dtype=torch.uint8, device=dev)
    rpar = torch.full((G, R, pitch), SENT, dtype=torch.uint8, device=dev)
    ralign = torch.zeros(G, dtype=torch.int16, device=dev)
    fr.frame_shards(arena, toff, tlen, present, rdata, rpar, ralign, B)
    out = torch.empty((G, R, pitch), dtype=torch.uint8, device=dev)
    idx = torch.empty((G, R), dtype=torch.uint8, device=dev)
    st = torch.empty(G, dtype=torch.uint8, device=dev)
    c.decode_batch(rdata, rpar, present, out, idx, st, c.decode_workspace(G), B=B)
    rec_len = torch.zeros((G, R), dtype=torch.int16, device=dev)
    dst = torch.zeros((G, R, pitch), dtype=torch.uint8, device=dev)
    fr.unframe(out, idx, rec_len, B, dst=dst)
    torch.cuda.synchronize()
    ix, rl, gd, stn = idx.cpu().numpy(), _u16(rec_len), dst.cpu().numpy(), st.cpu().numpy()
    kept = {}
    for g, s in keep:
        kept.setdefault(g, set()).add(s)
    n_rec = 0
    for g in range(G):
        have = kept.get(g, set())
        if len(have) < K:
            assert stn[g] == 1 and (ix[g] == 0xFF).all()
            continue
        assert stn[g] == 0
        missing = [i for i in range(K) if i not in have]
        assert [int(x) for x in ix[g] if x != 0xFF] == missing
        for t, i in enumerate(missing):
            assert gd[g, t, :rl[g, t]].tobytes() == dgs[g * K + i], (g, i)
            n_rec += 1
    assert n_rec > 50
    # the same packets through the oracle's fec_unpack / fec_find_missings deliver the same datagrams
    host_pkts = pkt.cpu().numpy()
    rx = fo.FecRx(K, N, lambda s, a: oracle.decode(K, N, s, a))
    got = []
    for g, s in sorted(keep):  # in send order: the oracle cache expires groups older than fec_sn - 3
        got += rx.push(host_pkts[g, s, :pl[g, s]].tobytes())
    exp = [dgs[g * K + s] for g, s in keep if s < K]
    exp += [gd[g, t, :rl[g, t]].tobytes() for g in range(G) for t in range(R) if ix[g, t] != 0xFF]
    assert sorted(got) == sorted(exp)


@pytest.mark.parametrize("mode", [fo.SEAL_CHECKSUM, fo.SEAL_PLAIN_XOR])
def test_seal_open_match_oracle(dev, mode):
    """encrypt_data / decrypt_data (none, plain_xor) on the device vs the restatement: ragged lengths at odd
    offsets, empty / 1-3 byte packets, corrupted packets (checksum must fail), and a full round trip."""
    from kcptube_amd.frame import open_, seal
    rng = random.Random(100 + mode)
    # register rows up to 2 KiB sealed (both sides of every 512-byte round edge), streaming rows past it
    edges = [e + d for e in (512, 1024, 1536, 2048) for d in range(-4, 3)]
    pk = [b"", b"\x01", b"ab", b"abc", b"1234", b"12345"] + [rng.randbytes(n) for n in edges + [3000, 4094, 4096]]
    pk += [rng.randbytes(rng.choice([5, 1440, 1442, rng.randint(1, 1500), rng.randint(1, 4100)])) for _ in range(400)]
    src, off, lens = _arena(pk, dev)
    P = len(pk)
    pitch = 4096
    d_len = torch.tensor(lens, dtype=torch.int32, device=dev)
    dst = torch.full((P, pitch), SENT, dtype=torch.uint8, device=dev)
    olen = torch.full((P,), -1, dtype=torch.int32, device=dev)
    seal(mode, src, off, d_len, dst, olen)
    torch.cuda.synchronize()
    gd, ol = dst.cpu().numpy(), olen.cpu().numpy()
    sealed = []
    for p, d in enumerate(pk):
        exp = fo.seal(d, mode)
        if exp is None or len(exp) > pitch:
            assert ol[p] == 0
            sealed.append(b"")
            continue
        n = len(exp)
        assert ol[p] == n
        assert gd[p, :n].tobytes() == exp, p
        n4 = (n + 3) // 4 * 4
        assert not gd[p, n:n4].any() and (gd[p, n4:] == SENT).all()
        sealed.append(exp)
    # open: the sealed packets, a third of them with one flipped byte, plus short ones
    rx = []
    for p, s in enumerate(sealed):
        if s and p % 3 == 0:
            b = bytearray(s)
            b[rng.randrange(len(b))] ^= 1 << rng.randrange(8)
            s = bytes(b)
        rx.append(s)
    rx += [b"\x00", b"\x00\x00", b"\x00\x00\x01"]
    src2, off2, lens2 = _arena(rx, dev)
    Q = len(rx)
    dst2 = torch.full((Q, pitch), SENT, dtype=torch.uint8, device=dev)
    olen2 = torch.full((Q,), -1, dtype=torch.int32, device=dev)
    ok = torch.full((Q,), 7, dtype=torch.uint8, device=dev)
    open_(mode, src2, off2, torch.tensor(lens2, dtype=torch.int32, device=dev), dst2, olen2, ok)
    torch.cuda.synchronize()
    g2, l2, k2 = dst2.cpu().numpy(), olen2.cpu().numpy(), ok.cpu().numpy()
    n_bad = 0
    for p, s in enumerate(rx):
        exp = fo.open_(s, mode)
        if exp is None:
            assert l2[p] == 0 and k2[p] == 0
            continue
        body, good = exp
        assert l2[p] == len(body) and k2[p] == int(good), p
        assert g2[p, :len(body)].tobytes() == body, p
        n4 = (len(body) + 3) // 4 * 4
        assert not g2[p, len(body):n4].any() and (g2[p, n4:] == SENT).all()
        n_bad += not good
        if p < len(pk) and p % 3 != 0 and pk[p]:
            assert good and body == pk[p]
    assert n_bad > 100


@pytest.mark.parametrize("K,N,B,pitch", [(20, 23, 1442, 1444), (10, 13, 1402, 1404), (200, 255, 1442, 1444),
                                         (3, 5, 7, 8), (1, 2, 2, 4), (4, 6, 40, 64)])
def test_encode_framed_matches_two_step_and_oracle(dev, oracle, K, N, B, pitch):
    """kfec_encode_framed_batch == kfec_frame_data_batch + kfec_encode_batch, byte for byte, and == the oracle's
    compact_into_container + fec_code::encode on the zero-padded slots (incl. an overflowing group)."""
    c, fr = _coder(K, N)
    R = N - K
    rng = random.Random(K * 7 + B)
    G = 23 if K < 100 else 5
    dgs = []
    for g in range(G):
        for i in range(K):
            n = rng.choice([0, 1, B - 2, rng.randint(0, B - 2)])
            if g == 2 and i == 0:
                n = B - 1  # too long: align 0 and zero parity
            dgs.append(rng.randbytes(n))
    src, off, lens = _arena(dgs, dev)
    d_len = _i16(lens, dev)
    par = torch.full((G, R, pitch), SENT, dtype=torch.uint8, device=dev)
    al = torch.zeros(G, dtype=torch.int16, device=dev)
    fr.encode_framed(src, off, d_len, par, al, B)
    data = torch.empty((G, K, pitch), dtype=torch.uint8, device=dev)
    al2 = torch.zeros(G, dtype=torch.int16, device=dev)
    par2 = torch.full((G, R, pitch), SENT, dtype=torch.uint8, device=dev)
    fr.frame_data(src, off, d_len, data, al2, B)
    c.encode_batch(data, par2, B=B)
    torch.cuda.synchronize()
    gp, gp2 = par.cpu().numpy(), par2.cpu().numpy()
    assert np.array_equal(_u16(al), _u16(al2))
    Bp = (B + 3) // 4 * 4
    assert np.array_equal(gp[:, :, :Bp], gp2[:, :, :Bp])
    assert (gp[:, :, Bp:] == SENT).all()
    for g in range(G):
        cont, a, total = fo.compact_send(dgs[g * K:(g + 1) * K])
        if a > B:
            assert not gp[g, :, :Bp].any()
            continue
        exp = oracle.encode(K, N, cont, a)
        for r in range(R):
            assert gp[g, r, :a].tobytes() == exp[r], (g, r)
            assert not gp[g, r, a:Bp].any()


def _ws(c, G, dev):
    return c.decode_workspace(G, device=dev)


@pytest.mark.parametrize("K,N,B,pitch", [(20, 23, 1442, 1444), (10, 13, 1402, 1404), (3, 5, 7, 8), (1, 2, 2, 4),
                                         (4, 6, 40, 64), (200, 255, 1442, 1444)])
def test_decode_framed_matches_two_step(dev, K, N, B, pitch):
    """kfec_decode_framed_batch == kfec_frame_shards_batch + kfec_decode_batch, byte for byte, on arbitrary
    shard bytes: random present sets (some below K), ragged lengths, a group whose data shard does not fit."""
    c, fr = _coder(K, N)
    R = N - K
    rng = random.Random(K * 31 + B)
    G = 37 if K < 100 else 4
    chunks, present = [], np.zeros((G, 4), np.uint64)
    for g in range(G):
        pal = rng.randint(0, B)
        nh = N if g == 0 else rng.choice([K, K, N - 1, rng.randint(max(0, K - 1), N)])
        have = rng.sample(range(N), nh)
        for s in range(N):
            n = rng.choice([0, B - 2, rng.randint(0, B - 2)]) if s < K else pal
            if g == 1 and s == 0 and B > 2:
                n = B - 1  # cannot be framed in B: the group reads as zeros on both paths
            chunks.append(rng.randbytes(n))
        for s in have:
            present[g, s >> 6] |= np.uint64(1 << (s & 63))
    src, off, lens = _arena(chunks, dev)
    d_len = _i16(lens, dev)
    pres = torch.tensor(present.view(np.int64), device=dev)
    out = torch.full((G, R, pitch), SENT, dtype=torch.uint8, device=dev)
    idx = torch.full((G, R), 0x5A, dtype=torch.uint8, device=dev)
    st = torch.full((G,), 0x5A, dtype=torch.uint8, device=dev)
    al = torch.zeros(G, dtype=torch.int16, device=dev)
    fr.decode_framed(src, off, d_len, pres, out, idx, st, al, _ws(c, G, dev), B)
    data = torch.full((G, K, pitch), SENT, dtype=torch.uint8, device=dev)
    par = torch.full((G, R, pitch), SENT, dtype=torch.uint8, device=dev)
    al2 = torch.zeros(G, dtype=torch.int16, device=dev)
    fr.frame_shards(src, off, d_len, pres, data, par, al2, B)
    out2 = torch.full((G, R, pitch), SENT, dtype=torch.uint8, device=dev)
    idx2 = torch.full((G, R), 0x5A, dtype=torch.uint8, device=dev)
    st2 = torch.full((G,), 0x5A, dtype=torch.uint8, device=dev)
    c.decode_batch(data, par, pres, out2, idx2, st2, _ws(c, G, dev), B=B)
    torch.cuda.synchronize()
    assert np.array_equal(_u16(al), _u16(al2))
    assert np.array_equal(st.cpu().numpy(), st2.cpu().numpy())
    assert np.array_equal(idx.cpu().numpy(), idx2.cpu().numpy())
    assert np.array_equal(out.cpu().numpy(), out2.cpu().numpy())
    assert (st.cpu().numpy() == 0).sum() >= G // 3


@pytest.mark.parametrize("K,N,B", [(20, 23, 1442), (10, 13, 1402), (5, 8, 300)])
def test_decode_framed_recovers_datagrams(dev, oracle, K, N, B):
    """Real groups (oracle compact_into_container + fec_code::encode), up to N-K packets lost per group:
    decode_framed + unframe hand back exactly the lost datagrams."""
    c, fr = _coder(K, N)
    R = N - K
    pitch = (B + 3) // 4 * 4
    rng = random.Random(K + N)
    G = 29
    chunks, present, lost = [], np.zeros((G, 4), np.uint64), []
    for g in range(G):
        dgs = [rng.randbytes(rng.choice([0, 1, B - 2, rng.randint(0, B - 2)])) for _ in range(K)]
        cont, a, _ = fo.compact_send(dgs)
        par = oracle.encode(K, N, cont, a)
        chunks += dgs + list(par)
        gone = set(rng.sample(range(N), rng.randint(0, R)))
        for s in range(N):
            if s not in gone:
                present[g, s >> 6] |= np.uint64(1 << (s & 63))
        lost.append({s: dgs[s] for s in gone if s < K})
    src, off, lens = _arena(chunks, dev)
    pres = torch.tensor(present.view(np.int64), device=dev)
    out = torch.zeros((G, R, pitch), dtype=torch.uint8, device=dev)
    idx = torch.zeros((G, R), dtype=torch.uint8, device=dev)
    st = torch.zeros((G,), dtype=torch.uint8, device=dev)
    al = torch.zeros(G, dtype=torch.int16, device=dev)
    fr.decode_framed(src, off, _i16(lens, dev), pres, out, idx, st, al, _ws(c, G, dev), B)
    rec_len = torch.zeros((G, R), dtype=torch.int16, device=dev)
    dst = torch.zeros((G, R, pitch), dtype=torch.uint8, device=dev)
    fr.unframe(out, idx, rec_len, B, dst=dst)
    torch.cuda.synchronize()
    gi, gl, gd = idx.cpu().numpy(), _u16(rec_len), dst.cpu().numpy()
    assert (st.cpu().numpy() == 0).all()
    n = 0
    for g in range(G):
        got = {int(gi[g, t]): gd[g, t, :gl[g, t]].tobytes() for t in range(R) if gi[g, t] != 0xFF}
        assert got == lost[g], g
        n += len(got)
    assert n > G // 3


@pytest.mark.parametrize("K,N,B,pitch,pkt_pitch", [(20, 23, 1442, 1444, 1456), (10, 13, 1402, 1404, 1416),
                                                   (4, 6, 40, 64, 44), (3, 5, 7, 8, 24), (200, 255, 1442, 1444, 1456),
                                                   (3, 3, 40, 40, 52)])
def test_encode_pack_matches_two_step(dev, K, N, B, pitch, pkt_pitch):
    """kfec_encode_pack_batch (data packets written by the encoder) == kfec_encode_framed_batch +
    kfec_pack_batch(DATA | REDUNDANT), byte for byte over the whole packet array: ragged datagrams, a group
    with a datagram too long for B (its data packets still go out, longer than the framed columns), packets
    that do not fit pkt_pitch (length 0, nothing written)."""
    c, fr = _coder(K, N)
    R = N - K
    rng = random.Random(K * 13 + B + pkt_pitch)
    G = 19 if K < 100 else 3
    dgs = []
    for g in range(G):
        for i in range(K):
            n = rng.choice([0, 1, B - 2, rng.randint(0, B - 2)])
            if g == 1 and i == 2 and B > 3:
                n = B - 1 if K < 100 else B + 5  # too long: align 0 (and, at 200:255, past the framed columns)
            dgs.append(rng.randbytes(n))
    src, off, lens = _arena(dgs, dev)
    d_len = _i16(lens, dev)
    sn = torch.tensor(np.asarray([rng.getrandbits(32) for _ in range(G)], np.uint32).view(np.int32), device=dev)
    conv = torch.tensor(np.asarray([rng.getrandbits(32) for _ in range(G)], np.uint32).view(np.int32), device=dev)
    ts = 0x01234567

    def run(fused):
        par = torch.full((G, R, pitch), SENT, dtype=torch.uint8, device=dev)
        al = torch.zeros(G, dtype=torch.int16, device=dev)
        pkt = torch.full((G, N, pkt_pitch), SENT, dtype=torch.uint8, device=dev)
        pl = torch.full((G, N), -1, dtype=torch.int16, device=dev)
        if fused:
            fr.encode_pack(src, off, d_len, par, al, sn, conv, ts, pkt, pl, B)
        else:
            fr.encode_framed(src, off, d_len, par, al, B)
            fr.pack(src, off, d_len, par, al, sn, conv, ts, pkt, pl)
        torch.cuda.synchronize()
        return par.cpu().numpy(), _u16(al), pkt.cpu().numpy(), _u16(pl)

    p1, a1, k1, l1 = run(True)
    p2, a2, k2, l2 = run(False)
    assert np.array_equal(a1, a2)
    assert np.array_equal(l1, l2)
    assert np.array_equal(k1, k2)
    B4 = (B + 3) // 4 * 4
    assert np.array_equal(p1[:, :, :B4], p2[:, :, :B4])
    assert (l1[:, :K] > 0).sum() > G * K // 2 and ((l1 == 0).sum() > 0 or N == K)


@pytest.mark.parametrize("mode", [0, 1])
def test_seal_open_in_place(dev, mode):
    """Checksum mode in place (d_dst NULL, e.g. straight after kfec_pack_batch): the 2 checksum bytes land right
    after each packet and nothing else changes, with the lengths of the out-of-place call; opening in place
    gives its lengths and verdicts.  plain_xor in place is refused (KFEC_EINVAL)."""
    from kcptube_amd.fec import KfecError
    from kcptube_amd.frame import open_, seal
    rng = random.Random(300 + mode)
    pitch = 2600
    lens = [1, 2, 3, 4, 5, 1449, 1450, 1451, 1452, 2046, 2047, 2048, 2049, 2050, 2051, 2590, 2598]
    lens += [rng.randint(1, 1460) for _ in range(300)] + [rng.randint(1, 2598) for _ in range(100)]
    P = len(lens)
    rows = np.zeros((P, pitch), np.uint8)
    for p, n in enumerate(lens):
        rows[p, :n] = np.frombuffer(rng.randbytes(n), np.uint8)
    buf = torch.tensor(rows, device=dev)
    # packets at odd offsets inside the rows (in place needs no alignment)
    off = torch.arange(P, dtype=torch.int64, device=dev) * pitch
    d_len = torch.tensor(lens, dtype=torch.int32, device=dev)
    flat = buf.view(-1)
    if mode == 1:
        with pytest.raises(KfecError):
            seal(mode, flat, off, d_len, None, torch.empty(P, dtype=torch.int32, device=dev), slot=pitch)
        return
    ref = torch.full((P, pitch), SENT, dtype=torch.uint8, device=dev)
    rl = torch.full((P,), -1, dtype=torch.int32, device=dev)
    seal(mode, flat, off, d_len, ref, rl)
    il = torch.full((P,), -1, dtype=torch.int32, device=dev)
    seal(mode, flat, off, d_len, None, il, slot=pitch)  # in place
    torch.cuda.synchronize()
    assert torch.equal(rl, il)
    r_np, b_np, n_np = ref.cpu().numpy(), buf.cpu().numpy(), rl.cpu().numpy()
    for p in range(P):
        n = int(n_np[p])
        assert np.array_equal(r_np[p, :n], b_np[p, :n]), p
        assert not b_np[p, n:].any()  # nothing beyond the trailer was written
    # open in place, a quarter of the packets corrupted first
    for p in range(0, P, 4):
        b_np[p, rng.randrange(int(n_np[p]))] ^= 0x10
    buf2 = torch.tensor(b_np, device=dev)
    flat2 = buf2.view(-1)
    sl = torch.tensor(n_np, dtype=torch.int32, device=dev)
    ref2 = torch.full((P, pitch), SENT, dtype=torch.uint8, device=dev)
    ol, ok = torch.full((P,), -1, dtype=torch.int32, device=dev), torch.full((P,), 7, dtype=torch.uint8, device=dev)
    open_(mode, flat2, off, sl, ref2, ol, ok)
    ol2, ok2 = torch.full((P,), -1, dtype=torch.int32, device=dev), torch.full((P,), 7, dtype=torch.uint8, device=dev)
    open_(mode, flat2, off, sl, None, ol2, ok2)  # in place
    torch.cuda.synchronize()
    assert torch.equal(ol, ol2) and torch.equal(ok, ok2)
    assert int((ok.cpu().numpy() == 0).sum()) >= P // 4 - 2
    assert np.array_equal(buf2.cpu().numpy(), b_np)  # opening in place writes nothing into the packets


def test_seal_in_place_respects_slots_and_buffer_end(dev):
    """In place, a packet whose trailer would not fit its slot (a full-pitch packet from kfec_pack_batch) or
    would pass the end of the buffer is refused (out_len 0) and nothing is written -- its neighbour's bytes
    and the bytes past the buffer stay as they were; slot 0 is rejected."""
    from kcptube_amd.fec import KfecError
    from kcptube_amd.frame import seal
    pitch, P = 64, 6
    lens = [62, 63, 64, 10, 61, 62]  # 62 + 2 == pitch fits; 63 / 64 fill the slot; the last row ends the buffer
    rows = np.frombuffer(random.Random(9).randbytes(P * pitch + 16), np.uint8).copy()
    buf = torch.tensor(rows, device=dev)
    flat = buf[: P * pitch - 1]  # the buffer ends one byte short of the last slot: its trailer cannot fit
    off = torch.arange(P, dtype=torch.int64, device=dev) * pitch
    d_len = torch.tensor(lens, dtype=torch.int32, device=dev)
    ol = torch.full((P,), -1, dtype=torch.int32, device=dev)
    seal(0, flat, off, d_len, None, ol, slot=pitch)
    torch.cuda.synchronize()
    got = buf.cpu().numpy()
    assert ol.cpu().tolist() == [64, 0, 0, 12, 63, 0]
    changed = np.nonzero(got != rows)[0].tolist()
    allowed = set(range(62, 64)) | set(range(3 * pitch + 10, 3 * pitch + 12)) | set(range(4 * pitch + 61, 4 * pitch + 63))
    assert set(changed) <= allowed  # only trailers of the packets that fit
    with pytest.raises(KfecError):
        seal(0, flat, off, d_len, None, ol, slot=0)
    # open in place: the sealed packets verify; a length that runs past the buffer end is a bad length (out_len 0,
    # ok 0) and its trailer is not read
    from kcptube_amd.frame import open_
    o_len = torch.tensor([64, 12, 63, 64, pitch + 2], dtype=torch.int32, device=dev)
    o_off = torch.tensor([0, 3 * pitch, 4 * pitch, 5 * pitch, 5 * pitch - 2], dtype=torch.int64, device=dev)
    ol2 = torch.full((5,), -1, dtype=torch.int32, device=dev)
    ok2 = torch.full((5,), 7, dtype=torch.uint8, device=dev)
    open_(0, flat, o_off, o_len, None, ol2, ok2)
    torch.cuda.synchronize()
    assert ol2.cpu().tolist()[:3] == [62, 10, 61] and ok2.cpu().tolist()[:3] == [1, 1, 1]
    assert ol2.cpu().tolist()[3:] == [0, 0] and ok2.cpu().tolist()[3:] == [0, 0]


@pytest.mark.parametrize("mode", [fo.SEAL_CHECKSUM, fo.SEAL_PLAIN_XOR])
def test_seal_open_packet_at_buffer_end(dev, mode):
    """A packet that ends exactly at the end of src (whose 16-byte windows would run past the buffer) takes the
    streaming rows; its neighbours take the register rows: all byte-exact vs the oracle, at every alignment."""
    from kcptube_amd.frame import open_, seal
    rng = random.Random(700 + mode)
    for L in (1, 3, 4, 5, 17, 100, 511, 513, 1449, 2046, 2047):
        for lead in range(4):
            pk = [rng.randbytes(rng.randint(1, 1500)) for _ in range(5)] + [rng.randbytes(L)]
            src, off, lens = _arena(pk, dev)
            end = int(off[-1].item()) + L + lead  # the buffer ends `lead` bytes after the last packet
            src = src[:end]
            pitch = 2056
            d_len = torch.tensor(lens, dtype=torch.int32, device=dev)
            dst = torch.full((len(pk), pitch), SENT, dtype=torch.uint8, device=dev)
            olen = torch.full((len(pk),), -1, dtype=torch.int32, device=dev)
            seal(mode, src, off, d_len, dst, olen)
            torch.cuda.synchronize()
            sealed = []
            for p, d in enumerate(pk):
                exp = fo.seal(d, mode)
                assert int(olen[p]) == len(exp), (L, lead, p)
                assert dst[p, :len(exp)].cpu().numpy().tobytes() == exp, (L, lead, p)
                sealed.append(exp)
            # open, with the last sealed packet ending at the end of its buffer
            src2, off2, lens2 = _arena(sealed, dev)
            src2 = src2[:int(off2[-1].item()) + len(sealed[-1]) + lead]
            dst2 = torch.full((len(pk), pitch), SENT, dtype=torch.uint8, device=dev)
            olen2 = torch.full((len(pk),), -1, dtype=torch.int32, device=dev)
            ok = torch.full((len(pk),), 7, dtype=torch.uint8, device=dev)
            open_(mode, src2, off2, torch.tensor(lens2, dtype=torch.int32, device=dev), dst2, olen2, ok)
            torch.cuda.synchronize()
            for p, d in enumerate(pk):
                assert int(ok[p]) == 1 and int(olen2[p]) == len(d), (L, lead, p)
                assert dst2[p, :len(d)].cpu().numpy().tobytes() == d, (L, lead, p)
