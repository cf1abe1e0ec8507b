/*
 * kfec_frame.h -- C ABI of the framing and wire layer around the coder (libkfec.so), SURVEY.md 8(f)
 * ranks 1-3: the steps kcptube runs either side of fecpp::fec_code, batched over many shard groups on the
 * device so that a batch of UDP payloads goes packet-in -> packet-out without leaving HBM.
 *
 *   send:    compact_into_container (send variant)  src/shares/data_operations.cpp:610-631
 *            fec_code::encode                         (kfec_encode_batch, include/kfec.h)
 *            create_fec_data_packet / create_fec_redundant_packet  src/networks/connections.cpp:395-430
 *   receive: unpack_fec / unpack_fec_redundant        src/networks/connections.cpp:488-511
 *            the per-sn shard cache                   src/modes/client.cpp:851-892 (fec_rcv_cache[sn][sub_sn])
 *            compact_into_container (recv variant)    src/shares/data_operations.cpp:633-667
 *            fec_code::decode                         (kfec_decode_batch)
 *            extract_from_container                   src/shares/data_operations.cpp:697-704
 *
 * One deliberate difference from the reference, where the reference is undefined: the padding of a
 * shard slot (bytes after [length][datagram]) is ZERO here on both sides.  The reference allocates the
 * slots with make_unique_for_overwrite (data_operations.cpp:618,651) and never writes the padding, so its
 * parity depends on heap garbage and a receiver's garbage differs from the sender's; recovering a long
 * datagram from shorter ones can then corrupt its tail.  With zero padding parity is a
 * pure function of the datagrams and recovery is exact.
 *
 * Conventions as include/kfec.h: device pointers are prefixed d_, streams are hipStream_t as void*, calls
 * are asynchronous on `stream` and return KFEC_OK or a negative KFEC_E* code.  Every byte is produced by
 * gfx950 kernels; there is no CPU path.  Byte arenas (d_src) must be 4-byte aligned and readable up to
 * src_bytes rounded up to a multiple of 4; shard slot arrays need pitch % 4 == 0 and 4-byte aligned bases.
 */
#ifndef KFEC_FRAME_H_
#define KFEC_FRAME_H_

#include <stddef.h>
#include <stdint.h>

#include "kfec.h"

#ifdef __cplusplus
extern "C" {
#endif

#define KFEC_FEC_CONTAINER_HEADER 2   /* constant_values::fec_container_header, share_defines.hpp:46 */
#define KFEC_PKT_DATA_HEADER 9        /* sizeof(packet_layer_data) - 1, connections.hpp:96-101 (packed) */
#define KFEC_PKT_REDUNDANT_HEADER 13  /* sizeof(packet_layer_fec) - 1, connections.hpp:103-110 (packed) */
#define KFEC_FEC_WAITS 3              /* gbv_fec_waits, connections.hpp:36 */

/* ---- framing (rank 1) -------------------------------------------------------------------------------- */

/* compact_into_container, send variant (data_operations.cpp:610-631), for G groups of K datagrams.
 * Datagram i of group g is bytes [d_off[g*K+i], d_off[g*K+i] + d_len[g*K+i]) of the arena d_src.
 *   d_data[g][i][0..B)  = [BE16 length][datagram][zeros]   (slot pitch `pitch`, as kfec_encode_batch reads it)
 *   d_align[g]          = max_i length + 2                 (the block size the reference encodes with)
 * A group holding a datagram longer than B - 2 gets d_align[g] = 0 and all-zero slots. */
int kfec_frame_data_batch(const kfec_ctx *ctx, size_t G, const void *d_src, size_t src_bytes,
                          const uint64_t *d_off, const uint16_t *d_len, size_t B, size_t pitch, void *d_data,
                          uint16_t *d_align, void *stream);

/* The fused form of kfec_frame_data_batch + kfec_encode_batch: the parity of G framed groups straight from
 * the datagram arena, without writing the framed data slots (the encoder assembles each slot's bytes on the
 * fly).  d_parity[g][r][0..B) and d_align[g] are exactly what the two-step path produces; the framed data
 * slots themselves are not needed on the wire (the data packets carry the datagrams unframed). */
int kfec_encode_framed_batch(const kfec_ctx *ctx, size_t G, const void *d_src, size_t src_bytes,
                             const uint64_t *d_off, const uint16_t *d_len, size_t B, size_t pitch, void *d_parity,
                             uint16_t *d_align, void *stream);

/* The whole send side in two launches: kfec_encode_framed_batch + kfec_pack_batch(KFEC_PACK_DATA |
 * KFEC_PACK_REDUNDANT), with the data packets written by the encoder itself while it reads each datagram
 * for the parity (so the datagrams are read once, not twice).  d_pkt[g][N][pkt_pitch] / d_pkt_len[g][N],
 * d_parity and d_align are byte-identical to the two-call path. */
int kfec_encode_pack_batch(const kfec_ctx *ctx, size_t G, const void *d_src, size_t src_bytes, const uint64_t *d_off,
                           const uint16_t *d_len, size_t B, size_t pitch, void *d_parity, uint16_t *d_align,
                           const uint32_t *d_sn, const uint32_t *d_conv, uint32_t timestamp, void *d_pkt,
                           size_t pkt_pitch, uint16_t *d_pkt_len, void *stream);

/* compact_into_container, receive variant (data_operations.cpp:633-667), for G cached groups.
 * Shard s < N of group g is present when bit s of d_present[g][4] is set; its bytes are
 * [d_off[g*N+s], +d_len[g*N+s]) of d_src.  Present data shards (s < K) are framed as on the send side into
 * d_data[g][s]; present parity shards are copied raw into d_parity[g][s-K]; every written slot is
 * zero-padded to B.  Absent slots are not written (kfec_decode_batch never reads them).
 *   d_align[g] = max over present shards of (length + 2 for data, length for parity);
 *   0 when a present shard does not fit in B (its group's slots are then zeroed). */
int kfec_frame_shards_batch(const kfec_ctx *ctx, size_t G, const void *d_src, size_t src_bytes,
                            const uint64_t *d_off, const uint16_t *d_len, const uint64_t *d_present, size_t B,
                            size_t pitch, void *d_data, void *d_parity, uint16_t *d_align, void *stream);

/* The fused form of kfec_frame_shards_batch + kfec_decode_batch: the missing data shards of G cached groups
 * straight from the packet arena, without writing the framed shards (the decoder assembles the columns of the
 * K shares it selected on the fly).  Inputs as kfec_frame_shards_batch; d_out / d_out_idx / d_status /
 * d_workspace as kfec_decode_batch (workspace of kfec_decode_workspace_size(ctx, G) bytes); d_align as
 * kfec_frame_shards_batch.  Every output is byte-identical to the two-step path. */
int kfec_decode_framed_batch(const kfec_ctx *ctx, size_t G, const void *d_src, size_t src_bytes,
                             const uint64_t *d_off, const uint16_t *d_len, const uint64_t *d_present, size_t B,
                             size_t pitch, void *d_out, uint8_t *d_out_idx, uint8_t *d_status, uint16_t *d_align,
                             void *d_workspace, void *stream);

/* extract_from_container (data_operations.cpp:697-704) on kfec_decode_batch's output.  For every used
 * recovered slot t of group g (d_out_idx[g][t] != 0xFF), d_rec_len[g*R+t] = the slot's BE16 length;
 * 0xFFFF when the slot is unused or the length does not fit in B - 2 (an inconsistent group: the reference
 * would copy past the shard).  When d_dst is non-NULL the datagram bytes [2, 2 + length) of each valid
 * slot are copied to d_dst + (g*R + t) * dst_pitch (dst_pitch % 4 == 0, >= B - 2). */
int kfec_unframe_batch(const kfec_ctx *ctx, size_t G, size_t B, size_t pitch, const void *d_out,
                       const uint8_t *d_out_idx, uint16_t *d_rec_len, void *d_dst, size_t dst_pitch,
                       void *stream);

/* ---- wire packets (rank 3) ----------------------------------------------------------------------------- */

#define KFEC_PACK_DATA 1u       /* emit the K data packets of each group */
#define KFEC_PACK_REDUNDANT 2u  /* emit the R redundant packets of each group */
#define KFEC_PACK_COMPACT 4u    /* lay out only the emitted kinds: [G][K] data, [G][R] redundant, or [G][N] */

/* create_fec_data_packet / create_fec_redundant_packet (connections.cpp:395-430) for G encoded groups.
 * Packet s of group g goes to d_pkt + (g*N + s) * pkt_pitch with its length in d_pkt_len[g*N + s]:
 *   s <  K: [LE32 timestamp][BE32 d_sn[g]][u8 s][datagram s]                                  9 + len bytes
 *   s >= K: [LE32 timestamp][BE32 d_sn[g]][u8 s][BE32 d_conv[g]][parity s-K, d_align[g] bytes] 13 + align
 * (sub_sn numbering as fec_maker, client.cpp:797-840: data 0..K-1, redundant K..N-1).  Bytes of the
 * packet slot past the packet's length, up to the next multiple of 4, are written as zero.  Groups with
 * d_align[g] == 0 get length-0 redundant packets.  With KFEC_PACK_COMPACT in `which`, slot (g, s) is
 * instead g * n_kinds + (s - first emitted s), e.g. [G][R] for the redundant packets alone. */
int kfec_pack_batch(const kfec_ctx *ctx, size_t G, unsigned which, const void *d_src, size_t src_bytes,
                    const uint64_t *d_off, const uint16_t *d_len, size_t pitch, const void *d_parity,
                    const uint16_t *d_align, const uint32_t *d_sn, const uint32_t *d_conv, uint32_t timestamp,
                    void *d_pkt, size_t pkt_pitch, uint16_t *d_pkt_len, void *stream);

/* Parsed FEC packet header (unpack_fec / unpack_fec_redundant, connections.cpp:488-511). */
typedef struct kfec_pkt_hdr {
    uint64_t payload_off;  /* byte offset of the payload in the arena */
    uint32_t timestamp;    /* little_endian_to_host(timestamp) */
    uint32_t sn;           /* ntohl(sn) */
    uint32_t conv;         /* redundant: ntohl(kcp_conv); data: the KCP segment's conversation id (LE32 of the
                              first payload bytes, KCP::GetConv / ikcp_decode32u) as fec_unpack verifies it,
                              0 when the payload is shorter than 4 bytes */
    uint16_t payload_len;  /* packet length - header length */
    uint8_t sub_sn;
    uint8_t kind;          /* KFEC_PKT_* below */
} kfec_pkt_hdr;

#define KFEC_PKT_KIND_DATA 0
#define KFEC_PKT_KIND_REDUNDANT 1   /* sub_sn >= K, as fec_unpack decides (client.cpp:851) */
#define KFEC_PKT_KIND_MALFORMED 255 /* shorter than its header (the reference's size_t would wrap) */

/* Parse P packets, packet p being bytes [d_off[p], d_off[p] + d_len[p]) of d_src. */
int kfec_unpack_batch(const kfec_ctx *ctx, size_t P, const void *d_src, size_t src_bytes, const uint64_t *d_off,
                      const uint32_t *d_len, kfec_pkt_hdr *d_hdr, void *stream);

/* ---- group assembly on the device (rank 2, the batched form of fec_rcv_cache[sn][sub_sn] = payload) ---
 * Scatter P parsed packets into the shard tables kfec_frame_shards_batch reads: packet p belongs to group
 * slot d_slot[p] (or, when d_slot is NULL, to slot sn - sn_base, uint32 wrap-around); packets whose slot is
 * outside [0, G), malformed packets and sub_sn >= N are skipped.  Sets bit sub_sn of d_present[slot] and
 * writes d_off[slot*N + sub_sn] / d_len[slot*N + sub_sn] (payload).  The caller zeroes d_present first.
 * A duplicated (sn, sub_sn) keeps the copy with the highest packet index -- the last to arrive, as the
 * reference's fec_rcv_cache[sn][sub_sn] assignment overwrites (client.cpp:869,887). */
int kfec_group_scatter(const kfec_ctx *ctx, size_t P, const kfec_pkt_hdr *d_hdr, const int32_t *d_slot,
                       uint32_t sn_base, size_t G, uint64_t *d_present, uint64_t *d_off, uint16_t *d_len,
                       void *stream);

/* ---- packet integrity for the non-AEAD encryption modes (rank 4) -----------------------------------------
 * encrypt_data / decrypt_data (data_operations.cpp:171-234, 373-435) for encryption=none and plain_xor:
 * a 2-byte checksum16 (simple_hashing.hpp:10-25: CRC-32 -- Botan "CRC32", stored big-endian -- with its two
 * 16-bit halves XORed) is appended to the packet, and plain_xor then runs xor_forward
 * (data_operations.cpp:120-128) over packet + checksum; opening runs xor_backward (:140-148) and compares.
 * The AEAD modes need Botan and are not provided.  These calls do not depend on a coder: they run on the
 * current HIP device. */
#define KFEC_SEAL_TRAILER 2     /* constant_values::iv_checksum_block_size, share_defines.hpp:41 */
#define KFEC_SEAL_CHECKSUM 0    /* encryption_mode none (encrypt_data's default branch) */
#define KFEC_SEAL_PLAIN_XOR 1   /* encryption_mode plain_xor */

/* Seal P packets [d_off[p], +d_len[p]) of d_src into d_dst + p * dst_pitch (dst_pitch % 4 == 0):
 * data || checksum16(data), xor_forward'ed for plain_xor.  d_out_len[p] = len + 2, or 0 for an empty packet
 * (encrypt_data returns "empty data") or one that does not fit in dst_pitch.  Bytes after the sealed packet
 * up to the next multiple of 4 are written as zero.
 * d_dst == NULL seals in place (checksum mode only): the two checksum bytes are written right after each
 * packet in d_src and nothing else is written -- the CRC reads each packet once.  dst_pitch is then the size
 * of each packet's slot from d_off[p] (e.g. pkt_pitch after kfec_pack_batch, whose packets may fill their
 * slot): a packet with len + 2 > dst_pitch, or whose trailer would pass src_bytes, gets d_out_len = 0 and
 * is left untouched, as one that does not fit dst_pitch out of place.  dst_pitch == 0 is KFEC_EINVAL. */
int kfec_seal_batch(int mode, size_t P, const void *d_src, size_t src_bytes, const uint64_t *d_off,
                    const uint32_t *d_len, void *d_dst, size_t dst_pitch, uint32_t *d_out_len, void *stream);

/* Open P sealed packets: (plain_xor: xor_backward, then) split off the 2-byte trailer and compare it with
 * checksum16 of the rest.  d_dst + p * dst_pitch receives the len - 2 plaintext bytes (zero-padded to a
 * multiple of 4), d_out_len[p] = len - 2 and d_ok[p] = 1 when the checksum matches, 0 when it does not
 * (decrypt_data's "checksum incorrect"); packets of <= 2 bytes get d_out_len = 0, d_ok = 0.
 * d_dst == NULL opens in place (checksum mode only): the plaintext is the packet's first len - 2 bytes where
 * it lies; only d_out_len and d_ok are written. */
int kfec_open_batch(int mode, size_t P, const void *d_src, size_t src_bytes, const uint64_t *d_off,
                    const uint32_t *d_len, void *d_dst, size_t dst_pitch, uint32_t *d_out_len, uint8_t *d_ok,
                    void *stream);

#ifdef __cplusplus
}
#endif

#endif /* KFEC_FRAME_H_ */
