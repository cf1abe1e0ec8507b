/*
 * kfec.h -- C ABI of the MI355X-native GF(2^8) Reed-Solomon coder (libkfec.so).
 *
 * Drop-in target: kcptube's vendored coder `fecpp::fec_code` (/root/reference/src/3rd_party/fecpp.hpp:36-81),
 * used as `fec_control_data::fecc` (src/networks/connections.hpp:614).  include/fecpp_compat.hpp rebuilds
 * that class, with identical signatures and error behaviour, on top of these entry points.
 *
 * Arithmetic: GF(2^8), polynomial 0x11D, alpha = 2, systematic Vandermonde code (fecpp.cpp:39-165,368-490).
 * Every byte of parity / recovered data is computed by hand-written gfx950 HIP kernels; there is no CPU
 * compute path.  A call returns KFEC_ENODEV when no MI355X (or no HIP runtime) is available.
 *
 * Conventions: plain pointers and sizes; no HIP or C++ types.  `stream` arguments are hipStream_t passed
 * as void* (NULL = the null stream).  Pointers prefixed d_ are device pointers (hipMalloc / torch tensors);
 * all others are host pointers.  Return value: KFEC_OK (0) or a negative KFEC_E* code; KFEC_EMPTY (1) is
 * the "reference returns an empty container" outcome, not an error.
 */
#ifndef KFEC_H_
#define KFEC_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define KFEC_OK 0
#define KFEC_EMPTY 1        /* fec_code::encode/decode would return {} (fecpp.cpp:497-498, 520-521, 550-551) */
#define KFEC_EINVAL (-1)    /* fec_code ctor/reset_martix would throw std::invalid_argument (fecpp.cpp:431,439) */
#define KFEC_ENODEV (-2)    /* no usable gfx950 device / HIP runtime: the coder never falls back to the CPU */
#define KFEC_EHIP (-3)      /* a HIP runtime call failed */
#define KFEC_ENOMEM (-4)    /* device or pinned-host allocation failed */
#define KFEC_ESINGULAR (-5) /* decode matrix singular: the reference throws from invert_matrix (fecpp.cpp:261,303) */

/* Per-group decode status written by kfec_decode_batch (d_status[g]). */
#define KFEC_GROUP_OK 0
#define KFEC_GROUP_EMPTY 1     /* fewer than K shares present: reference decode returns {} (fecpp.cpp:520-521) */
#define KFEC_GROUP_SINGULAR 2  /* unreachable for an MDS code with distinct ids; reported, never silently wrong */

typedef struct kfec_ctx kfec_ctx;

/* ---- construction: fec_code(K, N) / reset_martix(K, N) / get_K / get_N (fecpp.hpp:39-56, fecpp.cpp:428-490) */

/* Create a coder for K data shares out of N (1 <= K <= N <= 256).  Builds the N x K systematic encoding
 * matrix on the device.  KFEC_EINVAL on a K/N violation, KFEC_ENODEV without a GPU. */
int kfec_create(size_t K, size_t N, kfec_ctx **out);
/* reset_martix(K, N) (fecpp.cpp:437-451): re-targets an existing coder.  On any error (KFEC_EINVAL, or a
 * failed allocation / launch) the coder is unchanged: the new matrix is committed only once built.
 * Batch queues (kfec_pipeline.h) created on the coder must be recreated after a reset.
 * A reset must not run concurrently with any other call that uses the same coder (its queues included):
 * it re-points the coder's K, N and matrix without a lock on the per-call path.  fecpp::fec_code has no
 * locking either; kcptube re-targets a coder from the thread that uses it (client.cpp:1755, relay.cpp:947).
 * Matrices are shared per (device, K, N) and immutable: create and reset build one on the first use of a shape
 * and are a lookup afterwards (no allocation, launch or synchronisation); the old matrix stays valid for
 * batched launches still in flight.  Matrices no coder uses stay cached up to 8 shapes / 4 MiB per device (the
 * least recently released beyond that are freed; that free waits for the device's in-flight work).  Worst case:
 * the reset (or destroy) that pushes the cache past its bound blocks its own thread until the longest batched
 * launch in flight on the device ends (~150 ms at fec=200:55, 256k groups); the free runs outside the cache's
 * lock, so other threads' create / reset / kfec_cached_matrices do not wait for it.  The rest are released with
 * the device's last coder. */
int kfec_reset(kfec_ctx *ctx, size_t K, size_t N);
void kfec_destroy(kfec_ctx *ctx);
size_t kfec_get_K(const kfec_ctx *ctx);
size_t kfec_get_N(const kfec_ctx *ctx);
/* Copy the N x K row-major encoding matrix (rows 0..K-1 are the identity) to host memory enc[N*K]. */
int kfec_enc_matrix(const kfec_ctx *ctx, uint8_t *enc);

/* ---- single group from host memory: fec_code::encode / fec_code::decode semantics ------------------- */

/* fec_code::encode(input, data_length, block_size) (fecpp.cpp:495-513).  Reads the first K blocks of
 * `input`; writes the N-K parity blocks to parity_out[(N-K) * block_size].  KFEC_EMPTY when the reference
 * returns {}: input == NULL or (data_length / block_size) % K != 0; also for block_size == 0 and for
 * data_length < K * block_size, where the reference divides by zero / reads out of bounds. */
int kfec_encode(const kfec_ctx *ctx, const uint8_t *input, size_t data_length, size_t block_size,
                uint8_t *parity_out);

/* fec_code::decode(shares, share_size) (fecpp.cpp:518-587).  share_ids[n] must be strictly ascending
 * (a std::map's iteration order); share_ptrs[i] points at share_size bytes.  Selects K shares exactly as
 * the reference (data share i fills row i; each missing row takes the highest unused id), then writes the
 * recovered missing DATA shares in ascending index order: out_ids[*n_out] and out[*n_out * share_size]
 * (capacity: K entries).  KFEC_EMPTY (with *n_out = 0) when the reference returns {}: fewer than K shares,
 * or a chosen share id >= N.  No data share missing -> KFEC_OK with *n_out = 0 (the reference's empty map).
 * share_size == 0 -> KFEC_OK with the missing data ids in out_ids and no bytes (the reference's map of
 * empty vectors, fecpp.cpp:572-583). */
int kfec_decode(const kfec_ctx *ctx, const size_t *share_ids, const uint8_t *const *share_ptrs,
                size_t n_shares, size_t share_size, size_t *out_ids, uint8_t *out, size_t *n_out);

/* ---- batched, device-resident (the GPU path; asynchronous on `stream`) -------------------------------
 * Layout (R = N - K, every slot `pitch` bytes apart, block size B <= pitch):
 *   d_data    [G][K][pitch]   data shards of group g
 *   d_parity  [G][R][pitch]   parity shards
 * The code is byte-column independent, so any pitch works.  When pitch and every base pointer are
 * multiples of 4 the kernels move 32-byte granules (the last one of a row ending at ceil(B/4)*4) and may
 * read and write bytes [B, ceil(B/4)*4) of a slot, which lie inside the slot's pitch; otherwise they move
 * bytes and touch only [0, B).  Bytes [0, B) are bit-exact with the reference. */

/* Parity of G groups: d_parity[g][r] = XOR_j enc[K+r][j] * d_data[g][j]. */
int kfec_encode_batch(const kfec_ctx *ctx, size_t G, size_t B, size_t pitch, const void *d_data,
                      void *d_parity, void *stream);

/* Device workspace (bytes) kfec_decode_batch needs for G groups; allocate once, reuse. */
size_t kfec_decode_workspace_size(const kfec_ctx *ctx, size_t G);

/* Recover missing data shards of G groups in place-free fashion.
 *   d_present [G][4] uint64: bit s of group g set <=> shard s (data s < K, parity s - K) is present.
 *     Absent slots of d_data / d_parity are never read.  Bits >= N are ignored: the batch layout has no
 *     slot for a share id >= N, so the reference's "a chosen id >= N returns {}" (fecpp.cpp:550-551) cannot
 *     arise here; callers holding such ids (kcptube never sends them: sub_sn < N) use kfec_decode.
 *   d_out     [G][R][pitch]: recovered shard t of group g (ascending data index) in slot t.
 *   d_out_idx [G][R] uint8:  data index of recovered slot t, 0xFF for unused slots.
 *   d_status  [G] uint8:     KFEC_GROUP_OK / KFEC_GROUP_EMPTY / KFEC_GROUP_SINGULAR.
 * Share selection per group follows fecpp.cpp:528-548 exactly (matters for inconsistent shares). */
int kfec_decode_batch(const kfec_ctx *ctx, size_t G, size_t B, size_t pitch, const void *d_data,
                      const void *d_parity, const uint64_t *d_present, void *d_out, uint8_t *d_out_idx,
                      uint8_t *d_status, void *d_workspace, void *stream);

/* ---- synthetic inputs and checks for benchmarks / tests -------------------- */

/* Fill shard slots [s0, s0+ns) of groups [g0, g0+G) into d_out[G][ns][pitch] with the counter bytes
 * splitmix64(seed ^ ((g*N + s) * ceil(B/8) + w)) (little-endian words). */
int kfec_synth(const kfec_ctx *ctx, uint64_t seed, size_t g0, size_t G, size_t s0, size_t ns, size_t B,
               size_t pitch, void *d_out, void *stream);
/* Per-group erasure masks: erase `count` distinct ids drawn from [0, pool) (count = count_max, or
 * 1 + draw % count_max when random_count == 1), every other id in [0, N) present; random_count == 2:
 * i.i.d. loss, every id in [0, N) lost independently with probability count_max / 1e6 (pool ignored).
 * Same draws as the CPU harness (oracle/rs_oracle.c). */
int kfec_erasure_masks(const kfec_ctx *ctx, uint64_t seed, size_t g0, size_t G, size_t pool,
                       size_t count_max, int random_count, uint64_t *d_present, void *stream);
/* Compare recovered shards with the original data: d_mismatch[0] += number of (g, t) slots whose bytes
 * [0, B) differ from d_data[g][d_out_idx[g][t]].  d_mismatch is a device uint64 (caller zeroes it). */
int kfec_verify_recovered(const kfec_ctx *ctx, size_t G, size_t B, size_t pitch, const void *d_data,
                          const void *d_out, const uint8_t *d_out_idx, uint64_t *d_mismatch, void *stream);

/* Library version string and the device the context runs on (-1 if none). */
const char *kfec_version(void);
int kfec_device(const kfec_ctx *ctx);
/* Single-group calls served so far by the resident per-call workers (process-wide; diagnostics).
 * kfec_encode / kfec_decode run on a resident worker (KFEC_WORKER_WGS workgroups, default 8, per slot: no
 * launch or stream synchronisation per call) for groups with N - K <= 16, N * round16(B) <= 36 KiB and
 * (N - K) * K <= 512; other shapes take a kernel launch.  A worker leaves the GPU after KFEC_WORKER_IDLE_US
 * (default 20000) without a request, between requests once it has been resident KFEC_WORKER_LEASE_US
 * (default 2000: the bound on how long a device-wide synchronisation -- hipFree, hipHostFree,
 * hipDeviceSynchronize -- in another thread waits for it while calls continue), and when the last coder of
 * its device is destroyed; it is relaunched on demand.  KFEC_WORKER=0 turns the workers off; KFEC_WORKER=1 makes a worker failure an error instead of a
 * switch to the launch path; KFEC_WORKER_SLOTS (1-8, default 2) sets the workers per device. */
uint64_t kfec_worker_requests(void);
/* Batch requests served so far by the resident workers (process-wide; diagnostics): the small flushes of the
 * batched queues (kfec_pipeline.h) that took the worker instead of kernel launches. */
uint64_t kfec_worker_batches(void);
/* Matrices cached on the coder's device (diagnostics): their count, and in *bytes (if not NULL) their device
 * allocation.  Bounded by the coders' distinct shapes plus the unused-shape cache of kfec_reset. */
size_t kfec_cached_matrices(const kfec_ctx *ctx, size_t *bytes);
/* One empty request through a resident worker of the coder's device (diagnostics: the communication floor of
 * the per-call path).  KFEC_OK, or KFEC_ENODEV when the workers are off. */
int kfec_worker_ping(const kfec_ctx *ctx);

#ifdef __cplusplus
}
#endif

#endif /* KFEC_H_ */
