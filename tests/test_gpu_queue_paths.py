"""GPU tests of the batched queues' two flush paths (kfec_pipeline.cpp) against the oracle's restatement of
fec_maker / fec_find_missings (oracle/frame_oracle.py FecTx / FecRx, client.cpp:797-938):

* small flushes go to the resident worker as one batch request (shards read in place from the BAR-written
  staging arena), large ones and sealed queues to kernel launches -- both must give the oracle's bytes;
* a flush whose n-th HIP step fails (the KFEC_TEST_FAIL_FLUSH knob) leaves the queue as it was, and the retried
  flush emits exactly the packets / datagrams the oracle does, with the queue filled past 0.8 of its groups
  (where the round-4 in-place table packing overlapped its own source) and in sealed mode (the iv counter is
  committed only by a flush that succeeds).
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
    yield torch.device("cuda:0")
    from kcptube_amd.pipeline import arm_flush_fault, set_queue_worker_max
    arm_flush_fault(0)
    set_queue_worker_max(-1)


@pytest.fixture(params=["worker", "launch"])
def path(request, dev):
    from kcptube_amd.pipeline import set_queue_worker_max
    set_queue_worker_max(64 if request.param == "worker" else 0)
    yield request.param
    set_queue_worker_max(-1)


def _coder(K, N):
    from kcptube_amd import FecCode
    return FecCode(K, N)


def _send_groups(oracle, q, K, N, mtu, groups, conns=3, seed=0, ts=4321):
    """Fill the queue with `groups` complete groups over `conns` senders (ragged datagrams, one empty);
    returns the oracle's redundant packets in queue order [(tag, pkt)] and the senders."""
    from kcptube_amd.pipeline import FecSender
    rng = random.Random(seed)
    txs = [(FecSender(q, conv=0x4000 + i, tag=i),
            fo.FecTx(K, N, lambda d, t, a: oracle.encode(K, N, d, a, t), conv=0x4000 + i)) for i in range(conns)]
    exp = []
    while q.pending() < groups:
        tag = rng.randrange(conns)
        tx, ref = txs[tag]
        d = rng.randbytes(rng.choice([0, 1, mtu, rng.randint(0, mtu)]))
        assert tx.send(d, timestamp=ts) == (r := ref.send(d, timestamp=ts))[0]
        exp += [(tag, p) for p in r[1:]]
    return exp, txs


@pytest.mark.parametrize("K,N,mtu", [(20, 23, 1440), (10, 13, 1400), (4, 6, 100), (8, 16, 200), (1, 2, 7), (30, 32, 333)])
def test_sender_flush_paths_match_oracle(dev, oracle, path, K, N, mtu):
    from kcptube_amd.pipeline import TxQueue, worker_batches
    q = TxQueue(_coder(K, N), max_groups=40, max_datagram=mtu)
    exp, _ = _send_groups(oracle, q, K, N, mtu, groups=33, seed=K * 7 + N)
    b0 = worker_batches()
    got = q.flush(timestamp=4321)
    took_worker = worker_batches() > b0
    assert took_worker == (path == "worker")
    assert [(t, p) for t, _, _, p in got] == exp  # queue order, byte for byte


@pytest.mark.parametrize("K,N,mtu,groups,worker", [
    (64, 72, 200, 31, True),    # K x R = 512: the matrix tables fill the worker's 16 KiB; 31 x 64 descriptors fit
    (64, 72, 200, 32, False),   # one group more: the request (128 + 32 x 64 x 8 bytes) exceeds 16 KiB
    (65, 73, 200, 4, False),    # K x R = 520: the tables do not fit
    (20, 29, 100, 8, False),    # R = 9: more parity rows than a batch request carries
    (100, 104, 64, 20, True),   # K > 64 (two present words), R = 4
])
def test_sender_worker_limits(dev, oracle, K, N, mtu, groups, worker):
    """At and just past the worker's shape limits (kfec_worker.hip: kTabMax, kBatchReqMax, kBatchMaxR) a small
    flush takes the worker exactly when the request fits, and either path gives the oracle's packets."""
    from kcptube_amd.pipeline import TxQueue, set_queue_worker_max, worker_batches
    set_queue_worker_max(64)
    try:
        q = TxQueue(_coder(K, N), max_groups=groups + 2, max_datagram=mtu)
        exp, _ = _send_groups(oracle, q, K, N, mtu, groups=groups, seed=K + N + groups)
        b0 = worker_batches()
        got = q.flush(timestamp=4321)
        assert (worker_batches() > b0) == worker
        assert [(t, p) for t, _, _, p in got] == exp
    finally:
        set_queue_worker_max(-1)


@pytest.mark.parametrize("K,N,mtu", [(20, 23, 1440), (10, 13, 1400), (6, 9, 300), (8, 16, 200), (1, 2, 7)])
def test_receiver_flush_paths_match_oracle(dev, oracle, path, K, N, mtu):
    """A lossy, duplicated, reordered three-connection channel; small flushes at random points."""
    from kcptube_amd.pipeline import FecReceiver, RxQueue, worker_batches
    rq = RxQueue(_coder(K, N), max_groups=48, max_shard=mtu + 2)
    rng = random.Random(K * 131 + N)
    conns = 3
    streams = []
    for i in range(conns):
        tx = fo.FecTx(K, N, lambda d, t, a: oracle.encode(K, N, d, a, t), conv=500 + i)
        pkts = []
        for _ in range(K * 14):
            pkts += tx.send(rng.randbytes(rng.randint(0, mtu)))
        kept = []
        for p in pkts:
            r = rng.random()
            if r < 0.12:
                continue
            kept.append(p)
            if r > 0.96:
                kept.append(p)
        for j in range(0, len(kept) - 1, 6):
            kept[j], kept[j + 1] = kept[j + 1], kept[j]
        streams.append(kept)
    rx = [FecReceiver(rq, tag=i) for i in range(conns)]
    ref = [fo.FecRx(K, N, lambda s, a: oracle.decode(K, N, s, a)) for _ in range(conns)]
    got = [[] for _ in range(conns)]
    exp = [[] for _ in range(conns)]
    pos = [0] * conns
    b0 = worker_batches()
    while any(pos[i] < len(streams[i]) for i in range(conns)):
        i = rng.randrange(conns)
        if pos[i] >= len(streams[i]):
            continue
        p = streams[i][pos[i]]
        pos[i] += 1
        own, _ = rx[i].push(p)
        if own is not None:
            got[i].append(own)
        exp[i] += ref[i].push(p)
        if rq.pending() >= 40 or rng.random() < 0.05:
            for tag, sn, idx, d in rq.flush():
                got[tag].append(d)
    for tag, sn, idx, d in rq.flush():
        got[tag].append(d)
    n_rec = 0
    for i in range(conns):
        assert sorted(got[i]) == sorted(exp[i]), i
        n_rec += ref[i].recovered
    assert n_rec > 5
    assert (worker_batches() > b0) == (path == "worker")


def _fill_rx(oracle, rq, K, N, mtu, groups, seed):
    """`groups` decodable groups (3 data packets lost in each) over two connections; returns the receivers,
    the oracles and the oracle's recovered datagrams per tag (a data packet's own datagram left out: kfec_rx_push
    hands that one back at once, the flush only the recovered ones)."""
    from kcptube_amd.pipeline import FecReceiver
    rng = random.Random(seed)
    rx = [FecReceiver(rq, tag=i) for i in range(2)]
    ref = [fo.FecRx(K, N, lambda s, a: oracle.decode(K, N, s, a)) for _ in range(2)]
    txs = [fo.FecTx(K, N, lambda d, t, a: oracle.encode(K, N, d, a, t), conv=60 + i) for i in range(2)]
    exp = [[] for _ in range(2)]
    g = 0
    while rq.pending() < groups:
        i = g % 2
        pkts = []
        for _ in range(K):
            pkts += txs[i].send(rng.randbytes(rng.randint(0, mtu)))
        lost = set(rng.sample(range(K), min(3, N - K)))
        for k, p in enumerate(pkts):
            if k in lost:
                continue
            rx[i].push(p)
            out = ref[i].push(p)
            exp[i] += out if p[8] >= K else out[:-1]
        g += 1
    return rx, ref, exp


@pytest.mark.parametrize("K,N,mtu,groups", [(64, 72, 200, 12), (100, 104, 64, 12), (20, 29, 100, 8), (65, 73, 200, 4)])
def test_receiver_worker_limits(dev, oracle, K, N, mtu, groups):
    """Receive flushes of shapes at and past the worker's limits (decode tables per workgroup, R > 8): whichever
    path a flush takes, the recovered datagrams are the oracle's."""
    from kcptube_amd.pipeline import RxQueue, set_queue_worker_max
    set_queue_worker_max(64)
    try:
        rq = RxQueue(_coder(K, N), max_groups=groups + 2, max_shard=mtu + 2)
        rx, ref, exp = _fill_rx(oracle, rq, K, N, mtu, groups=groups, seed=K * 3 + N)
        got = rq.flush()
        per_tag = [[], []]
        for tag, sn, idx, d in got:
            per_tag[tag].append(d)
        for i in range(2):
            assert sorted(per_tag[i]) == sorted(exp[i])
        assert sum(len(x) for x in per_tag) == groups * min(3, N - K)
    finally:
        set_queue_worker_max(-1)


@pytest.mark.parametrize("step", range(1, 9))
def test_sender_flush_retry_after_failure(dev, oracle, path, step):
    """The step-th HIP step of a flush fails once; the queue (filled to 14 of 16 groups, past the 0.8 G where the
    round-4 in-place table packing overlapped its source) keeps every group, and the retried flush emits the
    oracle's redundant packets byte for byte."""
    from kcptube_amd.fec import KfecError
    from kcptube_amd.pipeline import TxQueue, arm_flush_fault
    K, N, mtu = 20, 23, 1440
    q = TxQueue(_coder(K, N), max_groups=16, max_datagram=mtu)
    exp, _ = _send_groups(oracle, q, K, N, mtu, groups=14, seed=step)
    arm_flush_fault(step)
    try:
        got = q.flush(timestamp=4321)
        arm_flush_fault(0)  # the flush had fewer steps: it succeeded untouched
    except KfecError:
        assert q.pending() == 14
        got = q.flush(timestamp=4321)
    assert [(t, p) for t, _, _, p in got] == exp


@pytest.mark.parametrize("groups", [14, 3])
@pytest.mark.parametrize("enc", ["none", "chacha20", "aes_gcm"])
@pytest.mark.parametrize("step", range(1, 12))
def test_sealed_flush_retry_after_failure(dev, oracle, path, enc, step, groups):
    """Sealed deferred queue: a failed flush keeps the staged data packets, the groups and the iv counter; the
    retry emits every packet sealed with the same iv draws as an unfailed flush (replayed from the oracle).
    worker: the small sealed flush (worker parity rows + one seal launch); launch: pack + seal kernels.
    groups = 3 keeps the worker path's seal launch under kSealCountRows, so the flush waits for the kernel's
    completion count (a failure after the launch leaves that kernel counting ahead of the retry's)."""
    from kcptube_amd.aead import AeadCipher
    from kcptube_amd.fec import KfecError
    from kcptube_amd.pipeline import FecSender, TxQueue, arm_flush_fault, iv_draw
    from oracle import aead_oracle as ao
    K, N, mtu = 6, 9, 300
    password, seed = b"retry-pw", 0xC0FFEE + step
    q = TxQueue(_coder(K, N), max_groups=16, max_datagram=mtu)
    cipher = AeadCipher(enc, password) if enc != "none" else None
    q.seal(0, aead=cipher, iv_seed=seed)
    rng = random.Random(step)
    txs = [FecSender(q, conv=0x77 + i, tag=i) for i in range(2)]
    refs = [fo.FecTx(K, N, lambda d, t, a: oracle.encode(K, N, d, a, t), conv=0x77 + i) for i in range(2)]
    plain = []
    while q.pending() < groups:
        i = rng.randrange(2)
        d = rng.randbytes(rng.randint(0, mtu))
        txs[i].send(d, timestamp=5)
        plain += [(i, p) for p in refs[i].send(d, timestamp=5)]
    arm_flush_fault(step)
    try:
        got = q.flush(timestamp=5)
        arm_flush_fault(0)
    except KfecError:
        assert q.pending() == groups and q.staged() > 0
        # a failure after the counted launch re-baselines the count on the drained stream (advisor, round 5):
        # neither ahead (the next wait would return before its kernel wrote its rows) nor behind (it would spin)
        assert q.count_drift() == 0
        got = q.flush(timestamp=5)
    assert q.count_drift() == 0

    def sealed(p, iv):
        return fo.seal(p, 0) if enc == "none" else ao.aead_seal(enc, password, p, iv)
    assert [(t, p) for t, _, _, p in got] == [(t, sealed(p, iv_draw(seed, k))) for k, (t, p) in enumerate(plain)]
    # the flush after the retried one waits on the re-based count: its packets are the oracle's too
    k0 = len(plain)
    more = []
    while q.pending() < groups:
        i = rng.randrange(2)
        d = rng.randbytes(rng.randint(0, mtu))
        txs[i].send(d, timestamp=6)
        more += [(i, p) for p in refs[i].send(d, timestamp=6)]
    got2 = q.flush(timestamp=6)
    assert q.count_drift() == 0
    assert [(t, p) for t, _, _, p in got2] == [(t, sealed(p, iv_draw(seed, k0 + k))) for k, (t, p) in enumerate(more)]


@pytest.mark.parametrize("step", range(1, 8))
def test_receiver_flush_retry_after_failure(dev, oracle, path, step):
    from kcptube_amd.fec import KfecError
    from kcptube_amd.pipeline import RxQueue, arm_flush_fault
    K, N, mtu = 20, 23, 1440
    rq = RxQueue(_coder(K, N), max_groups=16, max_shard=mtu + 2)
    rx, ref, exp = _fill_rx(oracle, rq, K, N, mtu, groups=14, seed=step)
    arm_flush_fault(step)
    try:
        got = rq.flush()
        arm_flush_fault(0)
    except KfecError:
        assert rq.pending() == 14
        got = rq.flush()
    per_tag = [[], []]
    for tag, sn, idx, d in got:
        per_tag[tag].append(d)
    # the oracle recovered the lost datagrams at the K-th share of each group; own datagrams are not in exp
    for i in range(2):
        assert sorted(per_tag[i]) == sorted(exp[i])
    assert sum(len(x) for x in per_tag) == 14 * 3


def test_matrix_cache_stays_bounded(dev):
    """A coder re-targeted through many shapes (adaptive FEC, a K:N sweep) keeps the device's matrix cache
    bounded: shapes no coder uses are freed beyond 8 (least recently released first); shapes in use stay."""
    import ctypes
    from kcptube_amd import FecCode
    lib = FecCode(2, 3)._lib
    keep = FecCode(20, 23)  # holds its shape throughout
    c = FecCode(3, 4)
    nb = ctypes.c_size_t(0)
    for k in range(4, 44):
        c.reset_martix(k, k + 3)
    n = lib.kfec_cached_matrices(c._ctx, ctypes.byref(nb))
    assert n <= 1 + 1 + 8 + 1, n  # keep's, c's, the unused cache, the (2, 3) coder's if still alive
    assert nb.value < 8 << 20
    c.reset_martix(20, 23)  # a shape in use by another coder: a lookup
    assert lib.kfec_cached_matrices(c._ctx, None) <= n
    p = c.encode(bytes(range(20)) * 4, 80, 4)
    assert p == keep.encode(bytes(range(20)) * 4, 80, 4)
