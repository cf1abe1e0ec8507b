"""GPU tests of the batched fec_maker / fec_find_missings pipeline (include/kfec_pipeline.h) against the
oracle's restatement of the same reference functions (oracle/frame_oracle.py FecTx / FecRx).

Bar: the data packets are byte-identical to create_fec_data_packet's, the redundant packets to
create_fec_redundant_packet's over the oracle encoder's parity, and through a lossy multi-connection channel
the receiver hands KCP exactly the datagrams the oracle's fec_unpack / fec_find_missings hands it (same set,
same per-group recovered datagrams), with the same cache expiry.
"""
from __future__ import annotations

import random

import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

from oracle import frame_oracle as fo  # noqa: E402


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from kcptube_amd import load_library
    load_library()
    return torch.device("cuda:0")


def _coder(K, N):
    from kcptube_amd import FecCode
    return FecCode(K, N)


@pytest.mark.parametrize("K,N,mtu", [(20, 23, 1440), (10, 13, 1400), (4, 6, 100)])
def test_sender_packets_match_oracle(dev, oracle, K, N, mtu):
    from kcptube_amd.pipeline import FecSender, TxQueue
    c = _coder(K, N)
    q = TxQueue(c, max_groups=64, max_datagram=mtu)
    rng = random.Random(K)
    conns = [(FecSender(q, conv=0x1000 + i, tag=i), fo.FecTx(K, N, lambda d, t, a: oracle.encode(K, N, d, a, t),
                                                             conv=0x1000 + i)) for i in range(3)]
    exp_red = []
    for step in range(K * 7 + 3):
        for tag, (tx, ref) in enumerate(conns):
            d = rng.randbytes(rng.choice([0, 1, mtu, rng.randint(0, mtu)]))
            pkt = tx.send(d, timestamp=1234)
            ref_pkts = ref.send(d, timestamp=1234)
            assert pkt == ref_pkts[0]
            exp_red += [(tag, p) for p in ref_pkts[1:]]
    assert q.pending() == 3 * 7
    got = q.flush(timestamp=1234)
    assert q.pending() == 0
    assert sorted((t, p) for t, _, _, p in got) == sorted(exp_red)
    for t, sn, sub, p in got:
        assert p[8] == sub and int.from_bytes(p[4:8], "big") == sn


@pytest.mark.parametrize("max_groups,senders", [(8, 4), (1, 9)])
def test_sender_flushes_between_partial_groups(dev, oracle, max_groups, senders):
    """Flushes at random points: the partial groups of every sender survive each flush (their datagrams are
    moved to the front of the staging arena) and complete later with the right bytes.  With 9 senders and a
    one-group queue the partial groups alone outgrow the arena, which then grows."""
    from kcptube_amd.fec import KfecError
    from kcptube_amd.pipeline import FecSender, TxQueue
    K, N, mtu = 5, 7, 200
    c = _coder(K, N)
    q = TxQueue(c, max_groups=max_groups, max_datagram=mtu)
    rng = random.Random(99)
    conns = [(FecSender(q, conv=0x2000 + i, tag=i), fo.FecTx(K, N, lambda d, t, a: oracle.encode(K, N, d, a, t),
                                                             conv=0x2000 + i)) for i in range(senders)]
    exp_red, got = [], []
    for step in range(400):
        tag = rng.randrange(len(conns))
        tx, ref = conns[tag]
        d = rng.randbytes(rng.choice([0, 3, mtu, rng.randint(0, mtu)]))
        if q.pending() == max_groups or rng.random() < 0.05:
            got += q.flush(timestamp=7)
        try:
            pkt = tx.send(d, timestamp=7)
        except KfecError:  # arena full while groups are queued: flush, then retry
            got += q.flush(timestamp=7)
            pkt = tx.send(d, timestamp=7)
        assert pkt == (ref_pkts := ref.send(d, timestamp=7))[0]
        exp_red += [(tag, p) for p in ref_pkts[1:]]
    got += q.flush(timestamp=7)
    assert len(exp_red) > 100
    assert sorted((t, p) for t, _, _, p in got) == sorted(exp_red)


def test_sender_conv_zero_builds_no_groups(dev):
    from kcptube_amd.pipeline import FecSender, TxQueue
    c = _coder(3, 5)
    q = TxQueue(c, 4, 64)
    tx = FecSender(q, conv=0)
    for i in range(10):
        p = tx.send(b"x" * i)
        assert p[8] == 0 and int.from_bytes(p[4:8], "big") == 0  # sub_sn reset, sn never advances
    assert q.pending() == 0


def test_queue_full_is_reported_without_side_effects(dev):
    from kcptube_amd.fec import KfecError
    from kcptube_amd.pipeline import FecSender, TxQueue
    c = _coder(2, 3)
    q = TxQueue(c, 1, 16)
    tx = FecSender(q, conv=5)
    tx.send(b"a"), tx.send(b"b")
    tx.send(b"c")
    with pytest.raises(KfecError):
        tx.send(b"d")  # would complete a second group
    assert q.pending() == 1
    assert len(q.flush()) == 1
    assert tx.send(b"d")[8] == 1  # the refused datagram was not counted


def _data_pkt(sn: int, sub: int, payload: bytes) -> bytes:
    # create_fec_data_packet (connections.cpp:395-411): [LE32 ts][BE32 sn][u8 sub_sn][payload]
    return (0).to_bytes(4, "little") + sn.to_bytes(4, "big") + bytes([sub]) + payload


def test_receiver_stale_traffic_keeps_arena_bounded(dev):
    """Groups that never reach K shares, and duplicates that overwrite cached shards, leave dead bytes in
    the staging arena; with nothing queued a full arena is compacted before it may grow, so a lossy peer
    cannot grow host + device memory without bound (the reference frees those bytes on erase)."""
    from kcptube_amd.pipeline import FecReceiver, RxQueue
    K, N, mtu = 20, 23, 1440
    rq = RxQueue(_coder(K, N), max_groups=8, max_shard=mtu + 2)
    rx = FecReceiver(rq)
    cap0 = rq.capacity()
    payload = bytes(range(256)) * 5 + bytes(160)  # 1440 bytes
    for sn in range(400):  # 400 x 19 x 1444 B = 11 MB through a 266 KB arena
        for sub in range(K - 1):
            rx.push(_data_pkt(sn, sub, payload))
        rx.push(_data_pkt(sn, 0, payload))  # a duplicate: overwrites, its old bytes are dead
        assert rx.cached() <= 5
    assert rq.pending() == 0
    assert rq.capacity() == cap0


def test_sender_destroyed_partial_groups_keep_arena_bounded(dev):
    """The bytes of a sender destroyed with a partial group are reclaimed before the arena grows."""
    from kcptube_amd.pipeline import FecSender, TxQueue
    K, N, mtu = 20, 23, 1440
    q = TxQueue(_coder(K, N), max_groups=2, max_datagram=mtu)
    cap0 = q.capacity()
    for i in range(200):
        tx = FecSender(q, conv=9 + i)
        for _ in range(K - 1):
            tx.send(b"\xab" * mtu)
        del tx  # kfec_tx_destroy with K - 1 datagrams cached
    assert q.pending() == 0
    assert q.capacity() == cap0


def test_queues_refuse_work_after_the_coder_is_reset(dev):
    """A queue is sized for its coder's K / N: after reset_martix its flush / push / send return
    KFEC_EINVAL instead of running the kernels past its buffers."""
    from kcptube_amd.fec import KfecError
    from kcptube_amd.pipeline import FecReceiver, FecSender, RxQueue, TxQueue
    c = _coder(4, 6)
    tq, rq = TxQueue(c, 4, 64), RxQueue(c, 4, 66)
    tx, rx = FecSender(tq, conv=3), FecReceiver(rq)
    for _ in range(4):
        tx.send(b"q" * 10)
    for sub in range(4):
        rx.push(_data_pkt(0, sub, b"r" * 10))
    assert tq.pending() == 1 and rq.pending() == 1
    c.reset_martix(20, 23)
    with pytest.raises(KfecError):
        tq.flush()
    with pytest.raises(KfecError):
        rq.flush()
    with pytest.raises(KfecError):
        tx.send(b"x")
    with pytest.raises(KfecError):
        rx.push(_data_pkt(1, 0, b"y"))
    c.reset_martix(4, 6)  # back to the queue's shape: usable again
    assert len(tq.flush()) == 2 and len(rq.flush()) == 0


@pytest.mark.parametrize("K,N,mtu", [(20, 23, 1440), (6, 9, 300)])
def test_receiver_matches_oracle_through_lossy_channel(dev, oracle, K, N, mtu):
    from kcptube_amd.pipeline import FecReceiver, RxQueue
    c = _coder(K, N)
    rq = RxQueue(c, max_groups=256, max_shard=mtu + 2)
    rng = random.Random(N)
    conns = 3
    streams = []
    for i in range(conns):
        tx = fo.FecTx(K, N, lambda d, t, a: oracle.encode(K, N, d, a, t), conv=77 + i)
        pkts = []
        for _ in range(K * 25):
            pkts += tx.send(rng.randbytes(rng.randint(0, mtu)))
        streams.append(pkts)
    # per connection: drop ~8% of packets, interleave the connections, reorder slightly within a connection
    rx = [FecReceiver(rq, tag=i) for i in range(conns)]
    ref = [fo.FecRx(K, N, lambda s, a: oracle.decode(K, N, s, a)) for _ in range(conns)]
    got = [[] for _ in range(conns)]
    exp = [[] for _ in range(conns)]
    order = []
    for i, pkts in enumerate(streams):
        kept = [p for p in pkts if rng.random() >= 0.08]
        for j in range(0, len(kept) - 1, 7):
            kept[j], kept[j + 1] = kept[j + 1], kept[j]
        order.append(kept)
    pos = [0] * conns
    while any(pos[i] < len(order[i]) for i in range(conns)):
        i = rng.randrange(conns)
        if pos[i] >= len(order[i]):
            continue
        p = order[i][pos[i]]
        pos[i] += 1
        own, _ = rx[i].push(p)
        if own is not None:
            got[i].append(own)
        exp[i] += ref[i].push(p)
        if rq.pending() > 200:
            for tag, sn, idx, d in rq.flush():
                got[tag].append(d)
    for tag, sn, idx, d in rq.flush():
        got[tag].append(d)
    n_rec = 0
    for i in range(conns):
        assert sorted(got[i]) == sorted(exp[i]), i
        assert rx[i].cached() == len(ref[i].cache)
        n_rec += ref[i].recovered
    assert n_rec > 20


@pytest.mark.parametrize("K,N,mtu,max_groups", [(20, 23, 1440, 4), (6, 9, 300, 2)])
def test_receiver_frequent_flushes_and_duplicates(dev, oracle, K, N, mtu, max_groups):
    """Flushes at random points (groups still waiting for K shares keep their shards across each flush, moved
    to the front of the staging arena), a tiny queue (KFEC_ENOMEM -> flush and retry), duplicated packets
    (the later copy wins, as the reference's map assignment): same datagrams as the oracle."""
    from kcptube_amd.fec import KfecError
    from kcptube_amd.pipeline import FecReceiver, RxQueue
    c = _coder(K, N)
    rq = RxQueue(c, max_groups=max_groups, max_shard=mtu + 2)
    rng = random.Random(K * 1000 + N)
    conns = 3
    streams = []
    for i in range(conns):
        tx = fo.FecTx(K, N, lambda d, t, a: oracle.encode(K, N, d, a, t), conv=900 + i)
        pkts = []
        for _ in range(K * 12):
            pkts += tx.send(rng.randbytes(rng.randint(0, mtu)))
        kept = []
        for p in pkts:
            r = rng.random()
            if r < 0.10:
                continue  # lost
            kept.append(p)
            if r > 0.95:
                kept.append(p)  # duplicated on the wire
        for j in range(0, len(kept) - 2, 5):
            kept[j], kept[j + 2] = kept[j + 2], kept[j]
        streams.append(kept)
    rx = [FecReceiver(rq, tag=i) for i in range(conns)]
    ref = [fo.FecRx(K, N, lambda s, a: oracle.decode(K, N, s, a)) for _ in range(conns)]
    got = [[] for _ in range(conns)]
    exp = [[] for _ in range(conns)]
    pos = [0] * conns
    n_full = 0
    while any(pos[i] < len(streams[i]) for i in range(conns)):
        i = rng.randrange(conns)
        if pos[i] >= len(streams[i]):
            continue
        p = streams[i][pos[i]]
        try:
            own, _ = rx[i].push(p)
        except KfecError:
            n_full += 1
            for tag, sn, idx, d in rq.flush():
                got[tag].append(d)
            own, _ = rx[i].push(p)
        pos[i] += 1
        if own is not None:
            got[i].append(own)
        exp[i] += ref[i].push(p)
        if rng.random() < 0.1:
            for tag, sn, idx, d in rq.flush():
                got[tag].append(d)
    for tag, sn, idx, d in rq.flush():
        got[tag].append(d)
    n_rec = 0
    for i in range(conns):
        assert sorted(got[i]) == sorted(exp[i]), i
        assert rx[i].cached() == len(ref[i].cache)
        n_rec += ref[i].recovered
    assert n_rec > 5
    if max_groups <= 2:
        assert n_full > 0  # the KFEC_ENOMEM -> flush -> retry path ran


def test_cpp_program_over_the_pipeline_header(dev):
    """tools/pipeline_bench.cpp: a C++ program over include/kfec_pipeline.h (what a kcptube build links),
    two host threads each with their own queues and stream on one shared context, every group losing 3 data
    packets; it exits 0 only when every lost datagram came back bit-exact."""
    import json
    import os
    import subprocess
    exe = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools", "pipeline_bench")
    if not os.path.exists(exe):
        pytest.skip("tools/pipeline_bench not built (kcptube_amd.build.build_tools)")
    p = subprocess.run([exe, "10", "13", "1400", "512", "3", "3", "2"], capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stdout + p.stderr
    r = json.loads(p.stdout.strip().splitlines()[-1])
    assert r["bad"] == 0 and r["recovered"] == r["recovered_expected"] == 2 * 512 * 3 * 3


@pytest.mark.parametrize("seal", ["none", "chacha20"])
def test_cpp_program_sealed_deferred_pipeline(dev, seal):
    """tools/pipeline_bench.cpp with PB_SEAL: the sealed queue from C++ as the header documents it -- kfec_tx_send
    with pkt = NULL and pkt_len = NULL under KFEC_TXQ_DEFER_DATA, every packet sealed by the flush, opened on the
    device by kfec_opener and pushed into kfec_rx -- 4096 groups per flush, every lost datagram back bit-exact.
    The host cost of a deferred send stays flat with the flush size (it was quadratic: the staged-packet table
    grew by one element per send)."""
    import json
    import os
    import subprocess
    exe = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools", "pipeline_bench")
    if not os.path.exists(exe):
        pytest.skip("tools/pipeline_bench not built (kcptube_amd.build.build_tools)")
    p = subprocess.run([exe, "20", "23", "1440", "4096", "3", "3", "1"], capture_output=True, text=True, timeout=120,
                       env=dict(os.environ, PB_SEAL=seal))
    assert p.returncode == 0, p.stdout + p.stderr
    r = json.loads(p.stdout.strip().splitlines()[-1])
    assert r["seal"] == seal and r["bad"] == 0 and r["recovered"] == r["recovered_expected"] == 4096 * 3 * 3
    assert r["tx_host_ns_per_packet"] < 2000, r  # ~150 ns measured; 15 us per packet when it was quadratic
    assert 0 < r["data_pkt_delay_us_p50"] <= r["data_pkt_delay_us_p99"]


_SEAL_MODES = {"none": 0, "plain_xor": 1}


def _ref_seal(enc: str, password: bytes, pkt: bytes, iv: int) -> bytes:
    from oracle import aead_oracle as ao
    if enc in _SEAL_MODES:
        return fo.seal(pkt, _SEAL_MODES[enc])
    return ao.aead_seal(enc, password, pkt, iv)


def _ref_open(enc: str, password: bytes, pkt: bytes):
    from oracle import aead_oracle as ao
    if enc in _SEAL_MODES:
        r = fo.open_(pkt, _SEAL_MODES[enc])
        return (b"", False) if r is None else r
    return ao.aead_open(enc, password, pkt)


@pytest.mark.parametrize("enc", ["none", "plain_xor", "chacha20", "aes_gcm"])
def test_sealed_pipeline_through_lossy_channel(dev, oracle, enc):
    """data_sender's encrypt_data on every packet fec_maker emits (client.cpp:780-840), on the device: the
    queue stages the data packets (KFEC_TXQ_DEFER_DATA), and each flush emits every packet sealed, in the order
    the reference sends them -- byte-exact against FecTx + encrypt_data with the queue's iv draws replayed.  The
    receiver opens the sealed packets in device batches (kfec_opener, decrypt_data) and feeds kfec_rx_push: same
    recovered datagrams as the oracle's fec_unpack / fec_find_missings over the oracle-opened packets; a
    tampered packet fails to open and is dropped, as the reference drops it."""
    from kcptube_amd.aead import AeadCipher
    from kcptube_amd.pipeline import FecReceiver, FecSender, Opener, RxQueue, TxQueue, iv_draw
    K, N, mtu = 6, 9, 300
    password, seed = b"kcptube-test-password", 0x1234_5678_9ABC_DEF0
    c = _coder(K, N)
    q = TxQueue(c, max_groups=16, max_datagram=mtu)
    cipher = None if enc in _SEAL_MODES else AeadCipher(enc, password)
    q.seal(_SEAL_MODES.get(enc, 0), aead=cipher, iv_seed=seed)
    rng = random.Random(sum(enc.encode()))
    conns = 3
    txs = [FecSender(q, conv=0x300 + i, tag=i) for i in range(conns)]
    refs = [fo.FecTx(K, N, lambda d, t, a: oracle.encode(K, N, d, a, t), conv=0x300 + i) for i in range(conns)]
    got, exp_plain = [], []
    for step in range(K * 8 * conns + 5):
        i = rng.randrange(conns)
        d = rng.randbytes(rng.choice([0, 1, mtu, rng.randint(0, mtu)]))
        assert txs[i].send(d, timestamp=99) == b""  # deferred: nothing leaves before the flush
        exp_plain += [(i, p) for p in refs[i].send(d, timestamp=99)]
        if q.pending() == 16 or rng.random() < 0.04:
            got += q.flush(timestamp=99)
    got += q.flush(timestamp=99)
    assert q.staged() == 0 and q.pending() == 0
    # the sealed stream equals the reference's plain stream sealed with the replayed iv draws
    exp = [(t, _ref_seal(enc, password, p, iv_draw(seed, k))) for k, (t, p) in enumerate(exp_plain)]
    assert len(got) == len(exp) > 100
    assert [(t, p) for t, _, _, p in got] == exp
    # receive: lossy, reordered channel; one tampered packet
    kept = [(t, p) for t, p in exp if rng.random() >= 0.08]
    for j in range(0, len(kept) - 1, 7):
        kept[j], kept[j + 1] = kept[j + 1], kept[j]
    bad = len(kept) // 2
    t_bad, p_bad = kept[bad]
    kept[bad] = (t_bad, p_bad[:3] + bytes([p_bad[3] ^ 0x40]) + p_bad[4:])
    op = Opener(_SEAL_MODES.get(enc, 0), aead=cipher, max_packets=64, max_packet=mtu + 64)
    rq = RxQueue(c, max_groups=64, max_shard=mtu + 2)
    rx = [FecReceiver(rq, tag=i) for i in range(conns)]
    ref_rx = [fo.FecRx(K, N, lambda s, a: oracle.decode(K, N, s, a)) for _ in range(conns)]
    out, exp_out = [[] for _ in range(conns)], [[] for _ in range(conns)]
    n_bad = 0

    def drain():
        nonlocal n_bad
        for tag, plain, ok in op.flush():
            if not ok:
                n_bad += 1
                continue
            own, _ = rx[tag].push(plain)
            if own is not None:
                out[tag].append(own)
        for tag, sn, idx, d in rq.flush():
            out[tag].append(d)

    for t, p in kept:
        plain, ok = _ref_open(enc, password, p)
        if ok:
            exp_out[t] += ref_rx[t].push(plain)
        op.add(p, tag=t)
        if op.pending() == 64:
            drain()
    drain()
    assert n_bad == 1
    for i in range(conns):
        assert sorted(out[i]) == sorted(exp_out[i]), i
    assert sum(r.recovered for r in ref_rx) > 3


def test_txq_seal_arguments(dev):
    """kfec_txq_seal refuses an unknown mode, an AEAD mode without its cipher, a cipher with a checksum mode,
    and a change while packets are staged."""
    from kcptube_amd.aead import AeadCipher
    from kcptube_amd.fec import KfecError
    from kcptube_amd.pipeline import FecSender, TxQueue
    c = _coder(4, 6)
    q = TxQueue(c, 4, 64)
    with pytest.raises(KfecError):
        q.seal(9)
    with pytest.raises(KfecError):
        q.seal(6)  # chacha20 without a cipher
    cipher = AeadCipher("chacha20", b"pw")
    assert c._lib.kfec_txq_seal(q._q, 0, cipher._h, 0, 1) == -1  # a cipher with a checksum mode
    assert c._lib.kfec_txq_seal(q._q, 4, cipher._h, 0, 1) == -1  # a cipher of another mode
    q.seal(0, defer_data=True)
    tx = FecSender(q, conv=1)
    assert tx.send(b"abc") == b""
    with pytest.raises(KfecError):
        q.seal(1)  # a packet is staged
    pk = q.flush()
    assert [p for _, _, _, p in pk] == [fo.seal(fo.data_packet(b"abc", 0, 0, 0), 0)]
    q.seal(-1, defer_data=False)  # back to plain, immediate data packets
    assert tx.send(b"d") == fo.data_packet(b"d", 0, 1, 0)
