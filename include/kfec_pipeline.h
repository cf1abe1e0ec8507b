/*
 * kfec_pipeline.h -- the per-connection FEC bookkeeping of kcptube over batched GPU coding (libkfec.so),
 * the callers of fec_code, restated so that many groups of many connections are
 * coded in one device batch instead of one CPU call per group.
 *
 *   kfec_tx  = client_mode::fec_maker          (src/modes/client.cpp:797-840; server.cpp:932-975 is the same)
 *   kfec_rx  = fec_unpack's cache insert + fec_find_missings
 *                                              (client.cpp:842-938; server.cpp:977-1020; relay.cpp:1384-1428)
 *   kfec_txq / kfec_rxq = the batched encode / decode queues shared by many kfec_tx / kfec_rx.
 *
 * What stays exactly as in the reference (host side, per packet, no GPU round trip on the latency path):
 *   - every datagram leaves at once as a data packet (create_fec_data_packet: [LE32 ts][BE32 sn][u8 sub_sn]);
 *   - sn / sub_sn numbering, including conv == 0 (no FEC group is built, sub_sn resets);
 *   - the receive cache fec_rcv_cache[sn][sub_sn] (a duplicate overwrites), the fec_rcv_restored set, the
 *     gbv_fec_waits = 3 expiry with uint32 wrap-around, and the rule that a group is decoded once, as soon
 *     as it holds >= K shares (even when nothing is missing).
 * What is batched: a group that becomes complete (send) or decodable (receive) is copied into the queue's
 * pinned staging; kfec_txq_flush / kfec_rxq_flush code every queued group in one GPU batch
 * (kfec_encode_framed_batch + kfec_pack_batch; kfec_decode_framed_batch, whose recovered shards come back
 * whole and have their BE16 length read at the callback) and hand back redundant packets / recovered
 * datagrams through a callback, in queue order.  The reference inputs a recovered datagram to KCP inside fec_find_missings; here that happens at the
 * flush, which the caller schedules (e.g. once per event-loop turn) -- the latency / throughput trade the
 * batching buys.  Shard padding is zero (include/kfec_frame.h).
 *
 * Threading: a kfec_tx / kfec_rx and its queue are used from one thread at a time (the reference serialises
 * with mutex_fec_snd / mutex_fec_rcv, connections.hpp:609-611).  Destroy the kfec_tx / kfec_rx of a queue
 * before the queue.  A queue is sized for its coder's K / N: after kfec_reset (reset_martix) of that coder
 * every push / send / flush of the queue returns KFEC_EINVAL -- recreate the queues.  That check is for resets
 * sequenced before the call; a reset concurrent with a queue call is not allowed (kfec.h, kfec_reset).
 * Staging: datagrams and shards are copied once, into the queue's pinned arena, when they arrive.  On a
 * large-BAR device (MI355X) and while the queue's flushes stay small (KFEC_QUEUE_BAR_MAX groups, default 2048)
 * each is also written straight into the arena's device image through the PCIe BAR, so a flush moves no bulk
 * bytes; otherwise finished 8 MiB stretches of the arena go H2D on the queue's own copy stream while the host
 * keeps filling it, so a flush waits only for the tail (KFEC_QUEUE_BAR=0: always the latter).
 * Flush paths: a flush of at most KFEC_QUEUE_WORKER_MAX groups (default 64) in BAR mode is one request to the
 * resident worker (kfec.h; no kernel launch, no stream synchronisation: ~10 us for one 20:3 group, ~16-21 us for
 * 16); a sealed one is a worker request plus one seal launch; larger flushes run kernel launches on `stream`.
 * Both give the same bytes.  `stream` NULL: the queue's own non-blocking stream (HIP's null stream would also
 * wait for every other stream of the device, a resident worker's included).  The callbacks of a send flush and
 * of kfec_opener_flush get rows the device has just written to pinned memory; the flush requests each a few
 * packets before its callback (KFEC_QUEUE_PREFETCH=0: not).
 * A flush that returns an error leaves the queue as it was -- queued groups, staged packets, the sealed iv
 * counter -- and can be retried.
 */
#ifndef KFEC_PIPELINE_H_
#define KFEC_PIPELINE_H_

#include <stddef.h>
#include <stdint.h>

#include "kfec_aead.h"
#include "kfec_frame.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct kfec_txq kfec_txq;
typedef struct kfec_tx kfec_tx;
typedef struct kfec_rxq kfec_rxq;
typedef struct kfec_rx kfec_rx;
typedef struct kfec_opener kfec_opener;

/* ---- send -------------------------------------------------------------------------------------------- */

/* A batched encode queue for the coder's fec=K:N-K: up to max_groups complete groups of datagrams of at most
 * max_datagram bytes (kcp_mtu) between flushes.  Pinned host and device buffers are allocated here. */
int kfec_txq_create(const kfec_ctx *ctx, size_t max_groups, size_t max_datagram, kfec_txq **out);
void kfec_txq_destroy(kfec_txq *q);
size_t kfec_txq_pending(const kfec_txq *q);
/* Bytes of the queue's datagram staging arena (it grows only when the live partial groups fill it). */
size_t kfec_txq_capacity(const kfec_txq *q);

/* One connection direction's fec_maker state: conv is the KCP conversation id written into redundant
 * packets (0: the reference builds no FEC groups for this connection). */
int kfec_tx_create(kfec_txq *q, uint32_t conv, uint64_t tag, kfec_tx **out);
void kfec_tx_destroy(kfec_tx *tx);

/* fec_maker(input_data, data_size): writes the data packet to pkt[9 + len] (*pkt_len) and, when this
 * datagram completes a group, queues the group (its redundant packets come from kfec_txq_flush).
 * The datagram is stored once, in the queue's staging arena (initially max_groups x K datagram slots, shared
 * by the complete groups and every sender's partial group; a flush keeps the partial groups, and the arena
 * doubles when the partial groups alone fill it).  KFEC_EINVAL for a datagram longer than max_datagram;
 * KFEC_ENOMEM, with nothing sent, when the datagram would complete a group and the queue is full, or the
 * arena is full while groups are queued (flush, then retry). */
int kfec_tx_send(kfec_tx *tx, const uint8_t *datagram, size_t len, uint32_t timestamp, uint8_t *pkt,
                 size_t *pkt_len);

/* Redundant packet callback: tag of the kfec_tx, the packet bytes (13-byte header + align bytes). */
typedef void (*kfec_packet_cb)(void *user, uint64_t tag, uint32_t sn, uint8_t sub_sn, const uint8_t *pkt,
                               size_t len);

/* Encode every queued group on the GPU and emit its N-K redundant packets (queue order).  Synchronous.
 * With KFEC_TXQ_DEFER_DATA (kfec_txq_seal) the staged data packets come out here too, in send order, each
 * group's redundant packets right after the data packet that completed it -- the order in which the
 * reference's fec_maker hands its packets to data_sender (client.cpp:797-840). */
int kfec_txq_flush(kfec_txq *q, uint32_t timestamp, kfec_packet_cb cb, void *user, void *stream);

/* Packet protection on the device, encrypt_data (data_operations.cpp:171-234) as data_sender applies it to
 * every packet it sends (client.cpp:780-795):
 *   mode KFEC_SEAL_CHECKSUM / KFEC_SEAL_PLAIN_XOR (kfec_frame.h; encryption none / plain_xor, aead NULL) or
 *   KFEC_AEAD_AES_GCM / _AES_OCB / _CHACHA20 / _XCHACHA20 with the matching cipher (kfec_aead.h, created on the
 *   coder's device); KFEC_TXQ_SEAL_OFF (the default) emits plain FEC packets.
 * Sealed, every packet the flush emits is ciphertext || tag || iv_raw (AEAD) or data || checksum16 (checksum
 * modes), computed after the pack on the device and copied back once.  The AEAD iv_raw of the i-th sealed
 * packet (emission order, counted over the queue's life) is the top 16 bits of splitmix64(iv_seed + i): the
 * reference draws it uniformly from a thread-local mt19937 (change_iv, aead.hpp:464-475); a counter-based
 * draw gives the same distribution and lets a test replay the sequence.
 * flags KFEC_TXQ_DEFER_DATA: kfec_tx_send no longer writes the data packet (pkt may be NULL, *pkt_len = 0): the
 * packet is staged in the queue's arena and emitted -- sealed, if a mode is set -- by the next flush, so no
 * packet is sealed on the host.  KFEC_EINVAL for an unknown mode, a missing / mismatched cipher, or a change
 * while packets are staged or groups queued. */
#define KFEC_TXQ_SEAL_OFF (-1)
#define KFEC_TXQ_DEFER_DATA 1u
int kfec_txq_seal(kfec_txq *q, int mode, const kfec_aead *aead, uint64_t iv_seed, unsigned flags);
/* Data packets staged by KFEC_TXQ_DEFER_DATA senders since the last flush. */
size_t kfec_txq_staged(const kfec_txq *q);

/* ---- receive ----------------------------------------------------------------------------------------- */

/* A batched decode queue: up to max_groups decodable groups whose shards are at most max_shard bytes
 * (kcp_mtu + 2, the parity length) between flushes.  Pinned host and device buffers are allocated here. */
int kfec_rxq_create(const kfec_ctx *ctx, size_t max_groups, size_t max_shard, kfec_rxq **out);
void kfec_rxq_destroy(kfec_rxq *q);
size_t kfec_rxq_pending(const kfec_rxq *q);
/* Bytes of the queue's shard staging arena: when it is full the bytes of restored, evicted and overwritten
 * shards are reclaimed first, and it doubles only when the groups still waiting for K shares fill it. */
size_t kfec_rxq_capacity(const kfec_rxq *q);

int kfec_rx_create(kfec_rxq *q, uint64_t tag, kfec_rx **out);
void kfec_rx_destroy(kfec_rx *rx);
/* Groups currently held in the receive cache (fec_rcv_cache.size()). */
size_t kfec_rx_cached(const kfec_rx *rx);

/* fec_unpack for one received FEC packet: caches its payload under (sn, sub_sn), runs the fec_find_missings
 * scan (expiry relative to this packet's sn; every group holding >= K shares and not yet restored is queued
 * for decoding and marked restored).  For a data packet *datagram / *datagram_len point at its payload inside
 * pkt (what fec_unpack returns to its caller for KCP::Input); NULL / 0 otherwise.  Returns the number of
 * groups queued by this call (0 or 1: only the packet's own group can reach K shares), KFEC_EINVAL for a
 * packet shorter than its header or a shard longer than max_shard, KFEC_ENOMEM when that group would be
 * queued and the queue is full, or the staging arena is full while groups are queued (flush, then retry; the
 * packet is then not cached).  The payload is stored once, in that arena (initially max_groups x N shard
 * slots, also holding the shards of groups still waiting for K shares: a flush keeps them, and the arena
 * doubles when they alone fill it). */
int kfec_rx_push(kfec_rx *rx, const uint8_t *pkt, size_t len, const uint8_t **datagram, size_t *datagram_len);

/* Recovered datagram callback: tag of the kfec_rx, group sn, data index, bytes (what KCP::Input gets). */
typedef void (*kfec_datagram_cb)(void *user, uint64_t tag, uint32_t sn, uint8_t index, const uint8_t *data,
                                 size_t len);

/* Decode every queued group on the GPU and emit the recovered datagrams (queue order, ascending index within
 * a group), as fec_find_missings' extract_from_container + KCP::Input loop.  Synchronous. */
int kfec_rxq_flush(kfec_rxq *q, kfec_datagram_cb cb, void *user, void *stream);

/* ---- receive-side packet opening ---------------------------------------------------------------------- */

/* decrypt_data (data_operations.cpp:373-435) for batches of received packets on the device, ahead of
 * kfec_rx_push: the packets of many connections are staged (one host copy into pinned memory), opened by one
 * kernel launch per flush and handed back in staging order.  mode / aead as kfec_txq_seal (KFEC_TXQ_SEAL_OFF is
 * refused); the cipher, if any, must live on the current device.  Up to max_packets packets of at most
 * max_packet bytes between flushes. */
int kfec_opener_create(int mode, const kfec_aead *aead, size_t max_packets, size_t max_packet, kfec_opener **out);
void kfec_opener_destroy(kfec_opener *o);
size_t kfec_opener_pending(const kfec_opener *o);
/* Stage one received packet: KFEC_EINVAL for a packet longer than max_packet, KFEC_ENOMEM when max_packets
 * are staged (flush, then retry). */
int kfec_opener_add(kfec_opener *o, const uint8_t *pkt, size_t len, uint64_t tag);
/* Opened packet callback: tag given to kfec_opener_add, the plaintext (what decrypt_data returns), ok = 0
 * when the tag / checksum did not verify or the length was invalid (the reference drops such a packet). */
typedef void (*kfec_opened_cb)(void *user, uint64_t tag, const uint8_t *plain, size_t len, int ok);
/* Open every staged packet on the device (synchronous) and call cb for each, in staging order. */
int kfec_opener_flush(kfec_opener *o, kfec_opened_cb cb, void *user, void *stream);

#ifdef __cplusplus
}
#endif

#endif /* KFEC_PIPELINE_H_ */
