"""CPU tests of the framing / wire-packet / group-cache oracle (oracle/frame_oracle.py).

The reference's data_operations.cpp / connections.cpp need asio and cannot be built here, and the reference
holds no tests for them, so these tests pin the restatement by (1) byte layouts written out by hand from
the packed structs (connections.hpp:88-111, share_defines.hpp:186-192), and (2) end-to-end behaviour
through the PINNED coder oracle: fec_maker -> lossy channel -> fec_unpack/fec_find_missings delivers every
datagram of every group that lost at most R packets.
"""
from __future__ import annotations

import random

import pytest

from oracle import frame_oracle as fo


def test_data_packet_layout():
    p = fo.data_packet(b"\xAA\xBB", sn=0x01020304, sub_sn=7, timestamp=0x11223344)
    assert p == bytes([0x44, 0x33, 0x22, 0x11, 0x01, 0x02, 0x03, 0x04, 0x07, 0xAA, 0xBB])
    assert fo.unpack_fec(p) == (0x11223344, 0x01020304, 7, b"\xAA\xBB")


def test_redundant_packet_layout():
    p = fo.redundant_packet(b"\x01", sn=5, sub_sn=20, conv=0xDEADBEEF, timestamp=1)
    assert p == bytes([1, 0, 0, 0, 0, 0, 0, 5, 20, 0xDE, 0xAD, 0xBE, 0xEF, 0x01])
    assert fo.unpack_redundant(p) == (1, 5, 20, 0xDEADBEEF, b"\x01")
    assert fo.parse_packet(p, K=20)["redundant"] and not fo.parse_packet(p, K=21)["redundant"]


def test_short_packets_rejected():
    assert fo.unpack_fec(b"\0" * 8) is None
    assert fo.unpack_redundant(b"\0" * 12) is None
    assert fo.parse_packet(b"\0" * 8 + b"\x05" + b"\0" * 3, K=3) is None  # redundant id, 12 bytes


def test_compact_send_layout():
    c, align, total = fo.compact_send([b"abc", b"", b"hello"])
    assert align == 7 and total == 21
    assert c == b"\x00\x03abc\x00\x00" + b"\x00\x00" + b"\x00" * 5 + b"\x00\x05hello"
    assert [fo.extract(c[i * 7:(i + 1) * 7]) for i in range(3)] == [b"abc", b"", b"hello"]


def test_compact_recv_layout():
    slots, align = fo.compact_recv({0: b"ab", 2: b"xyz", 3: b"PPPPPP"}, data_max_count=3)
    assert align == 6  # max(2 + 2, 3 + 2, 6)
    assert slots == {0: b"\x00\x02ab\x00\x00", 2: b"\x00\x03xyz\x00", 3: b"PPPPPP"}


def test_extract_rejects_overrun():
    assert fo.extract(b"\x00\x09abc") is None


def test_kcp_conv_little_endian():
    assert fo.kcp_conv(b"\x01\x02\x03\x04rest") == 0x04030201
    assert fo.kcp_conv(b"\x01") == 0


def _channel(oracle, K, N, datagrams, loss, seed):
    rng = random.Random(seed)
    enc = lambda data, total, align: oracle.encode(K, N, data, align, total)
    dec = lambda slots, align: oracle.decode(K, N, slots, align)
    tx = fo.FecTx(K, N, enc, conv=0x1234)
    rx = fo.FecRx(K, N, dec)
    delivered = []
    for d in datagrams:
        for pkt in tx.send(d, timestamp=99):
            if rng.random() >= loss:
                delivered += rx.push(pkt)
    return tx, rx, delivered


@pytest.mark.parametrize("K,N", [(20, 23), (10, 13), (4, 6)])
def test_roundtrip_through_pinned_coder(oracle, K, N):
    rng = random.Random(K * 1000 + N)
    groups = 40
    datagrams = [bytes(rng.getrandbits(8) for _ in range(rng.randint(0, 300))) for _ in range(groups * K)]
    # lose exactly R of the N packets of every group (worst case), alternating data / parity choices
    R = N - K
    tx = fo.FecTx(K, N, lambda d, t, a: oracle.encode(K, N, d, a, t), conv=7)
    rx = fo.FecRx(K, N, lambda s, a: oracle.decode(K, N, s, a))
    got = []
    for g in range(groups):
        pkts = []
        for d in datagrams[g * K:(g + 1) * K]:
            pkts += tx.send(d)
        assert len(pkts) == N
        drop = set(rng.sample(range(N), R))
        for i, p in enumerate(pkts):
            if i not in drop:
                got += rx.push(p)
    assert sorted(got) == sorted(datagrams)
    assert tx.sn == groups


def test_random_loss_delivers_what_fec_can(oracle):
    K, N = 6, 9
    rng = random.Random(5)
    datagrams = [rng.randbytes(rng.randint(1, 200)) for _ in range(60 * K)]
    _, rx, got = _channel(oracle, K, N, datagrams, loss=0.1, seed=3)
    assert set(got) <= set(datagrams)
    assert rx.recovered > 0


def test_zero_padding_fixes_reference_garbage_padding(oracle):
    """with the reference's uninitialised padding (different garbage on each side) a long
    datagram recovered from shorter ones is corrupted; with zero padding it is exact."""
    K, N = 3, 4
    dg = [b"S" * 10, b"L" * 200, b"s" * 20]
    rng = random.Random(1)

    def frame(datagrams, garbage, align=None):
        align = align or max(len(d) for d in datagrams) + 2
        out = bytearray()
        for d in datagrams:
            slot = bytearray(rng.randbytes(align) if garbage else bytes(align))
            slot[0:2] = len(d).to_bytes(2, "big")
            slot[2:2 + len(d)] = d
            out += slot
        return bytes(out), align

    for garbage in (True, False):
        c, align = frame(dg, garbage)
        par = oracle.encode(K, N, c, align)[0]
        # the receiver frames its own copies of shards 0 and 2 to the parity's length (data_operations.cpp:638-646)
        recv, _ = frame([dg[0], dg[2]], garbage, align=len(par))
        shares = {0: recv[:align], 2: recv[align:], 3: par}
        rec = fo.extract(oracle.decode(K, N, shares, align)[1])
        assert (rec == dg[1]) is (not garbage)


def test_stale_groups_expire():
    rx = fo.FecRx(4, 6, decode=lambda s, a: {})
    rx.push(fo.data_packet(b"x", 0, 0, 0))
    assert 0 in rx.cache
    rx.push(fo.data_packet(b"y", 3, 0, 0))  # fec_sn - sn = 3: kept (> gbv_fec_waits drops)
    assert 0 in rx.cache
    rx.push(fo.data_packet(b"z", 4, 0, 0))
    assert 0 not in rx.cache and 3 in rx.cache


def test_restored_group_decoded_once():
    calls = []
    rx = fo.FecRx(2, 3, decode=lambda s, a: calls.append(sorted(s)) or {})
    for sub in range(3):
        rx.push(fo.data_packet(b"d", 0, sub, 0) if sub < 2 else fo.redundant_packet(b"\0\0\0", 0, sub, 1, 0))
    assert calls == [[0, 1]]  # decoded when the 2nd share arrived, never again
    assert 0 in rx.restored


# ---- rank 4: checksum16 and the non-AEAD encryption modes --------------------------------------------------
def test_checksum16_known_answer():
    # CRC-32 check value: crc32("123456789") = 0xCBF43926, stored big-endian CB F4 39 26 -> [CB^39, F4^26]
    assert fo.checksum16(b"123456789") == bytes([0xCB ^ 0x39, 0xF4 ^ 0x26])
    assert fo.checksum16(b"") == b"\x00\x00"  # crc32("") = 0


def test_xor_forward_backward_inverse():
    rng = random.Random(3)
    for n in (1, 2, 3, 7, 64, 1443):
        d = rng.randbytes(n)
        assert fo.xor_backward(fo.xor_forward(d)) == d
    assert fo.xor_forward(b"\x01\x02\x04") == b"\x03\x06\x04"
    assert fo.xor_backward(b"\x03\x06\x04") == b"\x01\x02\x04"


@pytest.mark.parametrize("mode", [fo.SEAL_CHECKSUM, fo.SEAL_PLAIN_XOR])
def test_seal_open_roundtrip_and_corruption(mode):
    rng = random.Random(mode)
    for n in (1, 2, 3, 4, 5, 100, 1440):
        d = rng.randbytes(n)
        s = fo.seal(d, mode)
        assert len(s) == n + 2
        assert fo.open_(s, mode) == (d, True)
        bad = bytearray(s)
        bad[rng.randrange(len(bad))] ^= 0x10
        body, ok = fo.open_(bytes(bad), mode)
        assert not ok
    assert fo.seal(b"", mode) is None
    assert fo.open_(b"\x00\x00", mode) is None
