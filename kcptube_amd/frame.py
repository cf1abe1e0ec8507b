"""Python host mirror of kcptube's FEC framing and wire layer on top of libkfec.so (include/kfec_frame.h).

The reference functions and their batched device counterparts here:

=====================================================================  ==========================================
reference (file:line)                                                  here
=====================================================================  ==========================================
compact_into_container, send (src/shares/data_operations.cpp:610-631)   ``FecFrame.frame_data``
compact_into_container, receive (data_operations.cpp:633-667)          ``FecFrame.frame_shards``
extract_from_container (data_operations.cpp:697-704)                   ``FecFrame.unframe``
create_fec_data_packet / create_fec_redundant_packet                   ``FecFrame.pack``
(src/networks/connections.cpp:395-430)
unpack_fec / unpack_fec_redundant (connections.cpp:488-511)            ``FecFrame.unpack``
fec_rcv_cache[sn][sub_sn] = payload (src/modes/client.cpp:851-892)      ``FecFrame.scatter``
encrypt_data / decrypt_data, modes none and plain_xor                  ``seal`` / ``open_``
(src/shares/data_operations.cpp:171-234, 373-435)
=====================================================================  ==========================================

Everything runs as gfx950 kernels on device-resident ``torch`` tensors; no CPU path.  Shard slot padding is
zero on both sides (include/kfec_frame.h explains why that is the one deliberate difference).
"""
from __future__ import annotations

import numpy as np

from .fec import FecCode, _check, _dptr, _stream_handle, load_library

FEC_CONTAINER_HEADER = 2
PKT_DATA_HEADER = 9
PKT_REDUNDANT_HEADER = 13
FEC_WAITS = 3
PACK_DATA, PACK_REDUNDANT = 1, 2
SEAL_TRAILER, SEAL_CHECKSUM, SEAL_PLAIN_XOR = 2, 0, 1
KIND_DATA, KIND_REDUNDANT, KIND_MALFORMED = 0, 1, 255

# struct kfec_pkt_hdr (include/kfec_frame.h), 24 bytes
PKT_HDR_DTYPE = np.dtype([("payload_off", "<u8"), ("timestamp", "<u4"), ("sn", "<u4"), ("conv", "<u4"),
                          ("payload_len", "<u2"), ("sub_sn", "u1"), ("kind", "u1")])
assert PKT_HDR_DTYPE.itemsize == 24


def pkt_headers(raw) -> np.ndarray:
    """View a uint8 [P][24] tensor/array filled by ``unpack`` as kfec_pkt_hdr records."""
    a = raw.cpu().numpy() if hasattr(raw, "cpu") else np.asarray(raw)
    return np.ascontiguousarray(a, dtype=np.uint8).reshape(-1).view(PKT_HDR_DTYPE)


class FecFrame:
    """Batched framing / packet kernels bound to a coder (its K and N)."""

    def __init__(self, code: FecCode):
        self.code = code
        self._lib = code._lib

    @property
    def K(self) -> int:
        return self.code.K

    @property
    def N(self) -> int:
        return self.code.N

    def frame_data(self, src, off, length, data, align, B: int, stream=None) -> None:
        """src: uint8 arena; off: int64 [G*K]; length: int16/uint16 [G*K]; data: uint8 [G][K][pitch] (written,
        bytes [0, B) of each slot); align: int16 [G] (written, max length + 2; 0 = a datagram too long)."""
        G, k, pitch = data.shape
        assert k == self.K and off.numel() == G * k and length.numel() == G * k and align.numel() == G
        _check(self._lib.kfec_frame_data_batch(self.code._ctx, G, _dptr(src), src.numel(), _dptr(off), _dptr(length),
                                               B, pitch, _dptr(data), _dptr(align), _stream_handle(stream)),
               "kfec_frame_data_batch")

    def encode_framed(self, src, off, length, parity, align, B: int, stream=None) -> None:
        """frame_data + encode_batch fused: parity [G][R][pitch] and align [G] of the framed groups, without
        materialising the framed data slots."""
        G, r, pitch = parity.shape
        assert off.numel() == G * self.K and align.numel() == G
        _check(self._lib.kfec_encode_framed_batch(self.code._ctx, G, _dptr(src), src.numel(), _dptr(off),
                                                  _dptr(length), B, pitch, _dptr(parity), _dptr(align),
                                                  _stream_handle(stream)), "kfec_encode_framed_batch")

    def encode_pack(self, src, off, length, parity, align, sn, conv, timestamp: int, pkt, pkt_len, B: int,
                    stream=None) -> None:
        """encode_framed + pack(DATA | REDUNDANT) with the data packets written by the encoder: pkt [G][N][pitch],
        pkt_len int16 [G][N], parity [G][R][pitch], align [G] (all written)."""
        G, r, pitch = parity.shape
        assert off.numel() == G * self.K and align.numel() == G and pkt.shape[:2] == (G, self.N)
        _check(self._lib.kfec_encode_pack_batch(self.code._ctx, G, _dptr(src), src.numel(), _dptr(off), _dptr(length),
                                                B, pitch, _dptr(parity), _dptr(align), _dptr(sn), _dptr(conv),
                                                timestamp & 0xFFFFFFFF, _dptr(pkt), pkt.shape[-1], _dptr(pkt_len),
                                                _stream_handle(stream)), "kfec_encode_pack_batch")

    def frame_shards(self, src, off, length, present, data, parity, align, B: int, stream=None) -> None:
        """Receive side: off/length [G*N] shard table, present int64 [G][4]; writes the present slots of
        data [G][K][pitch] / parity [G][R][pitch] and align [G]."""
        G, k, pitch = data.shape
        assert k == self.K and off.numel() == G * self.N and present.shape == (G, 4)
        _check(self._lib.kfec_frame_shards_batch(self.code._ctx, G, _dptr(src), src.numel(), _dptr(off),
                                                 _dptr(length), _dptr(present), B, pitch, _dptr(data), _dptr(parity),
                                                 _dptr(align), _stream_handle(stream)), "kfec_frame_shards_batch")

    def decode_framed(self, src, off, length, present, out, out_idx, status, align, workspace, B: int,
                      stream=None) -> None:
        """frame_shards + decode_batch fused: the missing data shards out [G][R][pitch] (+ out_idx, status,
        align) straight from the shard table, without materialising the framed shards."""
        G, r, pitch = out.shape
        assert off.numel() == G * self.N and present.shape == (G, 4) and align.numel() == G
        _check(self._lib.kfec_decode_framed_batch(self.code._ctx, G, _dptr(src), src.numel(), _dptr(off),
                                                  _dptr(length), _dptr(present), B, pitch, _dptr(out),
                                                  _dptr(out_idx), _dptr(status), _dptr(align), _dptr(workspace),
                                                  _stream_handle(stream)), "kfec_decode_framed_batch")

    def unframe(self, out, out_idx, rec_len, B: int, dst=None, stream=None) -> None:
        """out [G][R][pitch] from decode_batch; rec_len int16 [G][R] (written; 0xFFFF = no datagram);
        dst [G][R][dst_pitch] (optional) receives the datagram bytes."""
        G, r, pitch = out.shape
        dst_pitch = dst.shape[-1] if dst is not None else 0
        _check(self._lib.kfec_unframe_batch(self.code._ctx, G, B, pitch, _dptr(out), _dptr(out_idx), _dptr(rec_len),
                                            _dptr(dst), dst_pitch, _stream_handle(stream)), "kfec_unframe_batch")

    def pack(self, src, off, length, parity, align, sn, conv, timestamp: int, pkt, pkt_len,
             which: int = PACK_DATA | PACK_REDUNDANT, stream=None) -> None:
        """pkt: uint8 [G][N][pkt_pitch] (written); pkt_len int16 [G][N] (written); sn/conv int32 [G]."""
        G, n, pkt_pitch = pkt.shape
        assert n == self.N
        pitch = parity.shape[-1] if parity is not None else 0
        _check(self._lib.kfec_pack_batch(self.code._ctx, G, which, _dptr(src), src.numel() if src is not None else 0,
                                         _dptr(off), _dptr(length), pitch, _dptr(parity), _dptr(align), _dptr(sn),
                                         _dptr(conv), timestamp & 0xFFFFFFFF, _dptr(pkt), pkt_pitch, _dptr(pkt_len),
                                         _stream_handle(stream)), "kfec_pack_batch")

    def unpack(self, src, off, length, hdr, stream=None) -> None:
        """P packets [off[p], off[p] + length[p]) of src (length int32 [P]); hdr uint8 [P][24] (written)."""
        P = off.numel()
        assert hdr.numel() == 24 * P
        _check(self._lib.kfec_unpack_batch(self.code._ctx, P, _dptr(src), src.numel(), _dptr(off), _dptr(length),
                                           _dptr(hdr), _stream_handle(stream)), "kfec_unpack_batch")

    def scatter(self, hdr, present, off, length, G: int, slot=None, sn_base: int = 0, stream=None) -> None:
        """Insert P parsed packets into the [G][N] shard tables (present must be zeroed by the caller)."""
        P = hdr.numel() // 24
        _check(self._lib.kfec_group_scatter(self.code._ctx, P, _dptr(hdr), _dptr(slot), sn_base & 0xFFFFFFFF, G,
                                            _dptr(present), _dptr(off), _dptr(length), _stream_handle(stream)),
               "kfec_group_scatter")


def seal(mode: int, src, off, length, dst, out_len, stream=None, slot: int = 0) -> None:
    """encrypt_data (none / plain_xor) for P packets [off[p], off[p] + length[p]) of src (length int32 [P]):
    dst [P][dst_pitch] receives data || checksum16 (xor_forward'ed for plain_xor), out_len int32 [P].
    dst None: checksum mode in place (the 2 checksum bytes go right after each packet in src, when they fit
    its `slot` bytes from off[p])."""
    P = off.numel()
    _check(load_library().kfec_seal_batch(mode, P, _dptr(src), src.numel(), _dptr(off), _dptr(length), _dptr(dst),
                                          dst.shape[-1] if dst is not None else slot, _dptr(out_len),
                                          _stream_handle(stream)), "kfec_seal_batch")


def open_(mode: int, src, off, length, dst, out_len, ok, stream=None) -> None:
    """decrypt_data (none / plain_xor): plaintext to dst [P][dst_pitch], out_len int32 [P], ok uint8 [P].
    dst None: checksum mode in place (only out_len / ok are written)."""
    P = off.numel()
    _check(load_library().kfec_open_batch(mode, P, _dptr(src), src.numel(), _dptr(off), _dptr(length), _dptr(dst),
                                          dst.shape[-1] if dst is not None else 0, _dptr(out_len), _dptr(ok),
                                          _stream_handle(stream)), "kfec_open_batch")
