"""TEST INFRASTRUCTURE ONLY -- CPU restatement of kcptube's FEC framing, wire packets and group cache.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import this module;
it is the checker for ``libkfec.so``'s framing kernels (include/kfec_frame.h), never the thing measured.

Restated (pure Python byte work, small cases only), with the reference lines each function follows:

* ``compact_send``      compact_into_container, send variant   src/shares/data_operations.cpp:610-631
* ``compact_recv``      compact_into_container, receive variant src/shares/data_operations.cpp:633-667
* ``extract``           extract_from_container / copy_from_container  data_operations.cpp:682-704
* ``data_packet``       packet::create_fec_data_packet       src/networks/connections.cpp:395-411
* ``redundant_packet``  packet::create_fec_redundant_packet  src/networks/connections.cpp:413-430
* ``unpack_fec``        packet::unpack_fec                   src/networks/connections.cpp:488-498
* ``unpack_redundant``  packet::unpack_fec_redundant         src/networks/connections.cpp:500-511
* ``checksum16``        simple_hashing::checksum16           src/shares/simple_hashing.hpp:10-25
* ``xor_forward`` / ``xor_backward``                         src/shares/data_operations.cpp:120-148
* ``seal`` / ``open_``  encrypt_data / decrypt_data, modes none and plain_xor
                        src/shares/data_operations.cpp:171-234, 373-435
* ``FecTx``             client_mode::fec_maker               src/modes/client.cpp:797-840
* ``FecRx``             client_mode::fec_unpack + fec_find_missings  src/modes/client.cpp:842-938
                        (server.cpp:977-1020 and relay.cpp:1384-1428 are the same logic)

Struct layouts: packet_layer_data / packet_layer_fec are ``#pragma pack(1)`` (connections.hpp:88-111):
9- and 13-byte headers; timestamp little-endian (host_to_little_endian), sn and kcp_conv big-endian (htonl);
fec_container is a BE16 length in front of the datagram (share_defines.hpp:186-192, header size 2 at
share_defines.hpp:46).

Where the reference is undefined the restatement pins the contract the product implements: the padding of
a shard slot is ZERO (the reference leaves it uninitialised: make_unique_for_overwrite at
data_operations.cpp:618 and :651), and packets shorter than their header are rejected
(the reference's ``length - header`` would wrap).

checksum16 is Botan's "CRC32" (the standard reflected CRC-32, the one zlib.crc32 computes), written out
big-endian by Botan's CRC32::final_result, then ``*(uint16_t*)out = *(uint16_t*)crc ^ *(uint16_t*)(crc+2)``
on a little-endian host.  Botan is absent here, so that byte order is restated from Botan's source, not
run: parity unpinned for rank 4 as for the rest of this file.

Parity status: the framing and packet functions live in data_operations.cpp / connections.cpp, which need
asio (absent from this image), so the reference cannot be compiled here and its repository holds no tests
or fixtures for them: this restatement is **parity unpinned** against the reference binary.  It is
cross-checked in tests/test_frame_oracle.py against the byte layouts above and end to end through the
pinned coder oracle (framed groups encode -> erase -> decode -> extract back to the datagrams).
"""
from __future__ import annotations

import struct
import zlib

FEC_CONTAINER_HEADER = 2  # share_defines.hpp:46
DATA_HEADER = 9           # sizeof(packet_layer_data) - 1
REDUNDANT_HEADER = 13     # sizeof(packet_layer_fec) - 1
FEC_WAITS = 3             # gbv_fec_waits, connections.hpp:36


def compact_send(datagrams: list[bytes]) -> tuple[bytes, int, int]:
    """(container, align_length, total_size): slot i = [htons(len)][datagram][zeros to align]
    (data_operations.cpp:612-630; align = max len + fec_container_header)."""
    align = max((len(d) for d in datagrams), default=0) + FEC_CONTAINER_HEADER
    out = bytearray(len(datagrams) * align)
    for i, d in enumerate(datagrams):
        out[i * align:i * align + 2] = struct.pack(">H", len(d) & 0xFFFF)
        out[i * align + 2:i * align + 2 + len(d)] = d
    return bytes(out), align, len(out)


def compact_recv(cache: dict[int, bytes], data_max_count: int) -> tuple[dict[int, bytes], int]:
    """({sub_sn: slot}, align_length): data shards (id < K) framed like the send side, parity shards copied
    raw, every slot zero-padded to align = max(len + 2 for data, len for parity) (data_operations.cpp:636-667)."""
    align = 0
    for i, d in cache.items():
        align = max(align, len(d) + FEC_CONTAINER_HEADER if i < data_max_count else len(d))
    out = {}
    for i, d in sorted(cache.items()):
        slot = bytearray(align)
        if i < data_max_count:
            slot[0:2] = struct.pack(">H", len(d) & 0xFFFF)
            slot[2:2 + len(d)] = d
        else:
            slot[0:len(d)] = d
        out[i] = bytes(slot)
    return out, align


def extract(container: bytes) -> bytes | None:
    """Datagram of a recovered slot: ntohs length, then that many bytes (data_operations.cpp:697-704).
    None when the length overruns the slot (the reference would read past it)."""
    n = struct.unpack(">H", bytes(container[:2]))[0]
    if n + FEC_CONTAINER_HEADER > len(container):
        return None
    return bytes(container[2:2 + n])


def data_packet(data: bytes, sn: int, sub_sn: int, timestamp: int) -> bytes:
    """[LE32 timestamp][BE32 sn][u8 sub_sn][data] (connections.cpp:395-411)."""
    return struct.pack("<I", timestamp & 0xFFFFFFFF) + struct.pack(">IB", sn & 0xFFFFFFFF, sub_sn & 0xFF) + bytes(data)


def redundant_packet(data: bytes, sn: int, sub_sn: int, conv: int, timestamp: int) -> bytes:
    """[LE32 timestamp][BE32 sn][u8 sub_sn][BE32 kcp_conv][data] (connections.cpp:413-430)."""
    return (struct.pack("<I", timestamp & 0xFFFFFFFF) + struct.pack(">IBI", sn & 0xFFFFFFFF, sub_sn & 0xFF,
                                                                     conv & 0xFFFFFFFF) + bytes(data))


def unpack_fec(pkt: bytes):
    """(timestamp, sn, sub_sn, payload) of a packet_layer_data (connections.cpp:488-498); None if short."""
    if len(pkt) < DATA_HEADER:
        return None
    ts = struct.unpack("<I", pkt[0:4])[0]
    sn, sub = struct.unpack(">IB", pkt[4:9])
    return ts, sn, sub, bytes(pkt[DATA_HEADER:])


def unpack_redundant(pkt: bytes):
    """(timestamp, sn, sub_sn, kcp_conv, payload) of a packet_layer_fec (connections.cpp:500-511)."""
    if len(pkt) < REDUNDANT_HEADER:
        return None
    ts = struct.unpack("<I", pkt[0:4])[0]
    sn, sub, conv = struct.unpack(">IBI", pkt[4:13])
    return ts, sn, sub, conv, bytes(pkt[REDUNDANT_HEADER:])


def kcp_conv(segment: bytes) -> int:
    """KCP::GetConv (kcp.cpp:263-266 -> ikcp_decode32u, ikcp.cpp:146-158): little-endian u32."""
    return struct.unpack("<I", bytes(segment[:4]))[0] if len(segment) >= 4 else 0


def parse_packet(pkt: bytes, K: int) -> dict | None:
    """fec_unpack's dispatch (client.cpp:851-891): sub_sn >= fec_data -> redundant layout."""
    if len(pkt) < DATA_HEADER:
        return None
    sub = pkt[8]
    if sub >= K:
        r = unpack_redundant(pkt)
        if r is None:
            return None
        ts, sn, sub, conv, payload = r
        return {"timestamp": ts, "sn": sn, "sub_sn": sub, "conv": conv, "payload": payload, "redundant": True}
    ts, sn, sub, payload = unpack_fec(pkt)
    return {"timestamp": ts, "sn": sn, "sub_sn": sub, "conv": kcp_conv(payload), "payload": payload,
            "redundant": False}


SEAL_CHECKSUM, SEAL_PLAIN_XOR = 0, 1


def checksum16(data: bytes) -> bytes:
    """simple_hashing::checksum16 (simple_hashing.hpp:17-24): CRC-32 stored big-endian, halves XORed."""
    c = zlib.crc32(bytes(data)) & 0xFFFFFFFF
    be = c.to_bytes(4, "big")
    return bytes([be[0] ^ be[2], be[1] ^ be[3]])


def xor_forward(data: bytes) -> bytes:
    """data[i] ^= data[i + 1], i ascending (data_operations.cpp:120-128)."""
    b = bytearray(data)
    for i in range(len(b) - 1):
        b[i] ^= b[i + 1]
    return bytes(b)


def xor_backward(data: bytes) -> bytes:
    """data[i - 1] ^= data[i], i descending (data_operations.cpp:140-148)."""
    b = bytearray(data)
    for i in range(len(b) - 1, 0, -1):
        b[i - 1] ^= b[i]
    return bytes(b)


def seal(data: bytes, mode: int) -> bytes | None:
    """encrypt_data for encryption none / plain_xor (data_operations.cpp:171-234); None for empty data."""
    if len(data) <= 0:
        return None
    out = bytes(data) + checksum16(data)
    return xor_forward(out) if mode == SEAL_PLAIN_XOR else out


def open_(packet: bytes, mode: int) -> tuple[bytes, bool] | None:
    """decrypt_data for encryption none / plain_xor (data_operations.cpp:373-435): (plaintext, checksum ok);
    None for packets of <= 2 bytes ("incorrect data length")."""
    if len(packet) <= 2:
        return None
    b = xor_backward(packet) if mode == SEAL_PLAIN_XOR else bytes(packet)
    body, trailer = b[:-2], b[-2:]
    return body, checksum16(body) == trailer


class FecTx:
    """client_mode::fec_maker (client.cpp:797-840) for one connection: every datagram goes out at once as a
    data packet; after fec_data of them the group is framed, encoded and its redundant packets follow."""

    def __init__(self, K: int, N: int, encode, conv: int = 1):
        self.K, self.N, self.encode, self.conv = K, N, encode, conv
        self.sn = 0
        self.sub_sn = 0
        self.cache: list[bytes] = []

    def send(self, datagram: bytes, timestamp: int = 0) -> list[bytes]:
        out = [data_packet(datagram, self.sn, self.sub_sn, timestamp)]
        self.sub_sn += 1
        if self.conv == 0:  # client.cpp:811-815
            self.sub_sn = 0
            return out
        self.cache.append(bytes(datagram))
        if len(self.cache) == self.K:
            container, align, total = compact_send(self.cache)
            for par in self.encode(container, total, align):
                out.append(redundant_packet(par, self.sn, self.sub_sn, self.conv, timestamp))
                self.sub_sn += 1
            self.cache = []
            self.sub_sn = 0
            self.sn = (self.sn + 1) & 0xFFFFFFFF
        return out


class FecRx:
    """fec_unpack's cache insert + fec_find_missings (client.cpp:842-938) for one connection.

    ``push(packet)`` returns the datagrams handed to KCP::Input, in order: those recovered by the scan
    (fec_find_missings inputs them itself, client.cpp:928-933), then a data packet's own payload, which
    fec_unpack returns to its caller (client.cpp:876-891)."""

    def __init__(self, K: int, N: int, decode):
        self.K, self.N, self.decode = K, N, decode
        self.cache: dict[int, dict[int, bytes]] = {}
        self.restored: set[int] = set()
        self.recovered = 0

    def push(self, pkt: bytes) -> list[bytes]:
        p = parse_packet(pkt, self.K)
        if p is None:
            return []
        self.cache.setdefault(p["sn"], {})[p["sub_sn"]] = p["payload"]
        out = self.find_missings(p["sn"])
        return out if p["redundant"] else out + [p["payload"]]

    def find_missings(self, fec_sn: int) -> list[bytes]:
        out = []
        for sn in sorted(self.cache):  # std::map iterates in ascending sn
            mapped = self.cache[sn]
            stale = ((fec_sn - sn) & 0xFFFFFFFF) > FEC_WAITS
            if len(mapped) < self.K:
                if stale:
                    del self.cache[sn]
                    self.restored.discard(sn)
                continue
            if sn in self.restored:
                if stale:
                    del self.cache[sn]
                    self.restored.discard(sn)
                continue
            slots, align = compact_recv(mapped, self.K)
            for i, shard in sorted(self.decode(slots, align).items()):
                d = extract(shard)
                if d is not None:
                    out.append(d)
                    self.recovered += 1
            self.restored.add(sn)
        return out
