"""Python mirror of include/kfec_pipeline.h: kcptube's fec_maker / fec_unpack + fec_find_missings bookkeeping
over batched GPU coding.

=========================================================================  ================================
reference (file:line)                                                      here
=========================================================================  ================================
client_mode::fec_maker (src/modes/client.cpp:797-840)                      ``FecSender.send`` + ``TxQueue.flush``
client_mode::fec_unpack + fec_find_missings (client.cpp:842-938)            ``FecReceiver.push`` + ``RxQueue.flush``
=========================================================================  ================================

Data packets leave at once (host), redundant packets and recovered datagrams come from the queue's flush,
which codes every queued group of every connection in one GPU batch.
"""
from __future__ import annotations

import ctypes as C

from .fec import FecCode, KfecError, _check

_u8p = C.POINTER(C.c_uint8)
PACKET_CB = C.CFUNCTYPE(None, C.c_void_p, C.c_uint64, C.c_uint32, C.c_uint8, _u8p, C.c_size_t)
DATAGRAM_CB = C.CFUNCTYPE(None, C.c_void_p, C.c_uint64, C.c_uint32, C.c_uint8, _u8p, C.c_size_t)
OPENED_CB = C.CFUNCTYPE(None, C.c_void_p, C.c_uint64, _u8p, C.c_size_t, C.c_int)

SEAL_OFF = -1        # KFEC_TXQ_SEAL_OFF
SEAL_CHECKSUM = 0    # KFEC_SEAL_CHECKSUM: encryption none (checksum16 trailer)
SEAL_PLAIN_XOR = 1   # KFEC_SEAL_PLAIN_XOR
DEFER_DATA = 1       # KFEC_TXQ_DEFER_DATA


def iv_draw(seed: int, i: int) -> int:
    """iv_raw of the i-th sealed packet of a queue (kfec_txq_seal): top 16 bits of splitmix64(seed + i)."""
    m = (1 << 64) - 1
    x = (seed + i + 0x9E3779B97F4A7C15) & m
    x = ((x ^ (x >> 30)) * 0xBF58476D1CE4E5B9) & m
    x = ((x ^ (x >> 27)) * 0x94D049BB133111EB) & m
    return (x ^ (x >> 31)) >> 48


def worker_batches() -> int:
    """Small queue flushes served by the resident worker so far (kfec_worker_batches; process-wide)."""
    from .fec import load_library
    return int(load_library().kfec_worker_batches())


def set_queue_worker_max(n: int) -> None:
    """Test hook: the largest flush (groups) the queues send to the resident worker (0: always the launch path;
    -1: back to KFEC_QUEUE_WORKER_MAX / the default)."""
    from .fec import load_library
    lib = load_library()
    lib.kfec_test_queue_worker_max.argtypes = [C.c_long]
    lib.kfec_test_queue_worker_max(n)


def arm_flush_fault(n: int) -> None:
    """Test hook: make the n-th HIP step (copy, launch, worker request, synchronisation) of the next queue flush
    fail once with KFEC_EHIP (0: off)."""
    from .fec import load_library
    lib = load_library()
    lib.kfec_test_fail_flush.argtypes = [C.c_int]
    lib.kfec_test_fail_flush(n)


def _mode_and_handle(mode, aead):
    if aead is not None:
        return aead.mode, aead._h
    return int(mode), None


class TxQueue:
    """kfec_txq: batched encode queue for up to max_groups complete groups of datagrams <= max_datagram."""

    def __init__(self, code: FecCode, max_groups: int, max_datagram: int):
        self.code = code
        self._lib = code._lib
        self._q = C.c_void_p()
        _check(self._lib.kfec_txq_create(code._ctx, max_groups, max_datagram, C.byref(self._q)), "kfec_txq_create")
        self.max_datagram = max_datagram
        self._defer = False

    def pending(self) -> int:
        return int(self._lib.kfec_txq_pending(self._q))

    def capacity(self) -> int:
        return int(self._lib.kfec_txq_capacity(self._q))

    def seal(self, mode: int = SEAL_CHECKSUM, aead=None, iv_seed: int = 0, defer_data: bool = True) -> None:
        """kfec_txq_seal: protect every emitted packet on the device (mode SEAL_CHECKSUM / SEAL_PLAIN_XOR, or an
        AeadCipher whose mode is used); defer_data stages the data packets for the flush as well."""
        m, h = _mode_and_handle(mode, aead)
        self._aead = aead  # the cipher must outlive the queue's use of it
        _check(self._lib.kfec_txq_seal(self._q, m, h, iv_seed & ((1 << 64) - 1), DEFER_DATA if defer_data else 0),
               "kfec_txq_seal")
        self._defer = bool(defer_data)

    def staged(self) -> int:
        return int(self._lib.kfec_txq_staged(self._q))

    def count_drift(self) -> int:
        """Test hook: the sealed small flush's completion count minus the baseline its next wait adds to (0 when
        no counted kernel is in flight -- after every flush, a failed one included)."""
        self._lib.kfec_test_txq_count_drift.restype = C.c_int32
        self._lib.kfec_test_txq_count_drift.argtypes = [C.c_void_p]
        return int(self._lib.kfec_test_txq_count_drift(self._q))

    def flush(self, timestamp: int = 0) -> list[tuple[int, int, int, bytes]]:
        """Encode every queued group; returns [(tag, sn, sub_sn, packet bytes)] in emission order: the redundant
        packets in queue order or, with deferred data packets, every packet in the order fec_maker sends it."""
        out = []

        def cb(_user, tag, sn, sub, ptr, n):
            out.append((int(tag), int(sn), int(sub), C.string_at(ptr, n)))

        fn = PACKET_CB(cb)  # kept alive for the call
        rc = self._lib.kfec_txq_flush(self._q, timestamp & 0xFFFFFFFF, C.cast(fn, C.c_void_p), None, None)
        _check(rc, "kfec_txq_flush")
        return out

    def __del__(self):
        try:
            if self._q.value:
                self._lib.kfec_txq_destroy(self._q)
        except Exception:
            pass


class FecSender:
    """kfec_tx: one connection direction's fec_maker state (conv 0: no FEC groups, as the reference)."""

    def __init__(self, q: TxQueue, conv: int, tag: int = 0):
        self.q = q
        self._lib = q._lib
        self._tx = C.c_void_p()
        _check(self._lib.kfec_tx_create(q._q, conv & 0xFFFFFFFF, tag, C.byref(self._tx)), "kfec_tx_create")

    def send(self, datagram: bytes, timestamp: int = 0) -> bytes:
        """fec_maker(datagram): the data packet (the group, once complete, is queued for the flush); b"" when
        the queue defers data packets to its flush."""
        d = (C.c_uint8 * max(len(datagram), 1)).from_buffer_copy(bytes(datagram) or b"\0")
        if self.q._defer:  # the header's contract: pkt and pkt_len may be NULL when data packets are deferred
            rc = self._lib.kfec_tx_send(self._tx, d, len(datagram), timestamp & 0xFFFFFFFF, None, None)
        else:
            pkt = (C.c_uint8 * (len(datagram) + 16))()
            n = C.c_size_t(0)
            rc = self._lib.kfec_tx_send(self._tx, d, len(datagram), timestamp & 0xFFFFFFFF, pkt, C.byref(n))
        if rc == -4:
            raise KfecError("kfec_tx_send: queue full, flush first")
        _check(rc, "kfec_tx_send")
        return b"" if self.q._defer else bytes(pkt)[:n.value]

    def __del__(self):
        try:
            if self._tx.value:
                self._lib.kfec_tx_destroy(self._tx)
        except Exception:
            pass


class RxQueue:
    """kfec_rxq: batched decode queue for up to max_groups decodable groups of shards <= max_shard bytes."""

    def __init__(self, code: FecCode, max_groups: int, max_shard: int):
        self.code = code
        self._lib = code._lib
        self._q = C.c_void_p()
        _check(self._lib.kfec_rxq_create(code._ctx, max_groups, max_shard, C.byref(self._q)), "kfec_rxq_create")

    def pending(self) -> int:
        return int(self._lib.kfec_rxq_pending(self._q))

    def capacity(self) -> int:
        return int(self._lib.kfec_rxq_capacity(self._q))

    def flush(self) -> list[tuple[int, int, int, bytes]]:
        """Decode every queued group; returns [(tag, sn, data index, recovered datagram)] in queue order."""
        out = []

        def cb(_user, tag, sn, idx, ptr, n):
            out.append((int(tag), int(sn), int(idx), C.string_at(ptr, n)))

        fn = DATAGRAM_CB(cb)  # kept alive for the call
        _check(self._lib.kfec_rxq_flush(self._q, C.cast(fn, C.c_void_p), None, None), "kfec_rxq_flush")
        return out

    def __del__(self):
        try:
            if self._q.value:
                self._lib.kfec_rxq_destroy(self._q)
        except Exception:
            pass


class FecReceiver:
    """kfec_rx: one connection direction's fec_rcv_cache / fec_rcv_restored."""

    def __init__(self, q: RxQueue, tag: int = 0):
        self.q = q
        self._lib = q._lib
        self._rx = C.c_void_p()
        _check(self._lib.kfec_rx_create(q._q, tag, C.byref(self._rx)), "kfec_rx_create")

    def cached(self) -> int:
        return int(self._lib.kfec_rx_cached(self._rx))

    def push(self, pkt: bytes) -> tuple[bytes | None, int]:
        """fec_unpack(pkt): (the data packet's own datagram or None, groups queued for decoding)."""
        buf = (C.c_uint8 * max(len(pkt), 1)).from_buffer_copy(bytes(pkt) or b"\0")
        dp = _u8p()
        dn = C.c_size_t(0)
        rc = self._lib.kfec_rx_push(self._rx, buf, len(pkt), C.byref(dp), C.byref(dn))
        if rc == -4:
            raise KfecError("kfec_rx_push: decode queue full, flush first")
        _check(rc, "kfec_rx_push")
        own = C.string_at(dp, dn.value) if dp else None
        return own, rc

    def __del__(self):
        try:
            if self._rx.value:
                self._lib.kfec_rx_destroy(self._rx)
        except Exception:
            pass


class Opener:
    """kfec_opener: decrypt_data for batches of received packets on the device, ahead of FecReceiver.push."""

    def __init__(self, mode: int = SEAL_CHECKSUM, aead=None, max_packets: int = 1024, max_packet: int = 1500):
        from .fec import load_library
        self._lib = load_library()
        self._aead = aead
        m, h = _mode_and_handle(mode, aead)
        self._o = C.c_void_p()
        _check(self._lib.kfec_opener_create(m, h, max_packets, max_packet, C.byref(self._o)), "kfec_opener_create")

    def pending(self) -> int:
        return int(self._lib.kfec_opener_pending(self._o))

    def count_drift(self) -> int:
        """Test hook: as TxQueue.count_drift, for the opener's counted flushes."""
        self._lib.kfec_test_opener_count_drift.restype = C.c_int32
        self._lib.kfec_test_opener_count_drift.argtypes = [C.c_void_p]
        return int(self._lib.kfec_test_opener_count_drift(self._o))

    def add(self, pkt: bytes, tag: int = 0) -> None:
        buf = (C.c_uint8 * max(len(pkt), 1)).from_buffer_copy(bytes(pkt) or b"\0")
        rc = self._lib.kfec_opener_add(self._o, buf, len(pkt), tag)
        if rc == -4:
            raise KfecError("kfec_opener_add: batch full, flush first")
        _check(rc, "kfec_opener_add")

    def flush(self) -> list[tuple[int, bytes, bool]]:
        """Open every staged packet; returns [(tag, plaintext, ok)] in staging order (plaintext b"" if not ok)."""
        out = []

        def cb(_user, tag, ptr, n, ok):
            out.append((int(tag), C.string_at(ptr, n) if n else b"", bool(ok)))

        fn = OPENED_CB(cb)
        _check(self._lib.kfec_opener_flush(self._o, C.cast(fn, C.c_void_p), None, None), "kfec_opener_flush")
        return out

    def __del__(self):
        try:
            if self._o.value:
                self._lib.kfec_opener_destroy(self._o)
        except Exception:
            pass
