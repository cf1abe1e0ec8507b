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


class TxQueue:
    """kfec_txq: batched encode queue for up to max_groups complete groups of datagrams <= max_datagram."""

    def __init__(self, code: FecCode, max_groups: int, max_datagram: int):
        self.code = code
        self._lib = code._lib
        self._q = C.c_void_p()
        _check(self._lib.kfec_txq_create(code._ctx, max_groups, max_datagram, C.byref(self._q)), "kfec_txq_create")
        self.max_datagram = max_datagram

    def pending(self) -> int:
        return int(self._lib.kfec_txq_pending(self._q))

    def capacity(self) -> int:
        return int(self._lib.kfec_txq_capacity(self._q))

    def flush(self, timestamp: int = 0) -> list[tuple[int, int, int, bytes]]:
        """Encode every queued group; returns [(tag, sn, sub_sn, redundant packet bytes)] in queue order."""
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
        """fec_maker(datagram): the data packet (the group, once complete, is queued for the flush)."""
        d = (C.c_uint8 * max(len(datagram), 1)).from_buffer_copy(bytes(datagram) or b"\0")
        pkt = (C.c_uint8 * (len(datagram) + 16))()
        n = C.c_size_t(0)
        rc = self._lib.kfec_tx_send(self._tx, d, len(datagram), timestamp & 0xFFFFFFFF, pkt, C.byref(n))
        if rc == -4:
            raise KfecError("kfec_tx_send: queue full, flush first")
        _check(rc, "kfec_tx_send")
        return bytes(pkt)[:n.value]

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
