// kfec_internal.hpp -- launch interface between the C ABI (kfec_api.cpp) and the kernels (kfec_kernels.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "../../include/kfec.h"
#include "../../include/kfec_frame.h"
#include "../../include/kfec_aead.h"

namespace kfec {

// Per-group decode record written by the prep kernels and read by the MAC kernels (group-major, so the
// few records a workgroup needs are a couple of contiguous cache lines).  Coefficient form:
//   [0] status (KFEC_GROUP_*), [1] m = missing data shards, [2..3] 0,
//   [4, 4+K4)              src[j]     share id used as column j of the selected K x K system,
//   [4+K4, 4+K4+R*K4)      coef[u][j] row u (u < m) of the inverse decode matrix for missing shard u,
// with K4 = K rounded up to 4 so that the prep kernel writes whole dwords.  Syndrome form (R <= 8, see
// write_syn in kfec_kernels.hip): [0] status, [1] m, [2] used-parity bits, [8, 40) present data bits,
// [40, 40 + 8 RT) the RT rows of the C matrix (RT = R up to 4, else 8; kfec_kernels.hip syn_record_stride).
inline size_t rec_k4(size_t K) { return (K + 3) & ~size_t(3); }
inline size_t record_stride(size_t K, size_t R)
{
    const size_t coef = (4 + rec_k4(K) + R * rec_k4(K) + 15) & ~size_t(15);
    return coef > 112 ? coef : 112;
}
// after the G records (256-aligned): the syndrome decode's active-group list -- a count (+ 252 bytes of
// padding), per-1024-group chunk counts / offsets, then the list of up to G group ids (uint32 each)
inline size_t decode_list_offset(size_t G, size_t K, size_t R) { return (G * record_stride(K, R) + 255) & ~size_t(255); }
inline size_t decode_list_chunks(size_t G) { return (G + 1023) / 1024; }
// Hybrid decode (R in [KFEC_DEC_HYBRID_MIN_R, 8]): both record forms are prepared, the syndrome records after the
// list (at most 112 bytes per group, RT <= 8), and the device picks the listed syndrome kernel for sparse loss or the
// coefficient-form MAC for dense loss
#ifndef KFEC_DEC_HYBRID_MIN_R
#define KFEC_DEC_HYBRID_MIN_R 4  // R = 7, 8: dense decode 14-22% faster, sparse unchanged (profiles/r06_dec_hybrid_ab.txt);
                                 // R = 5, 6 with R-row coefficient tiles (KFEC_DEC_MT_MID): 2-16% (r06_dec_mt_mid_ab.txt);
                                 // R = 4 (KFEC_DEC_MT_SMALL): 6%; R = 3 slower (r06_dec_mt_small_ab.txt)
#endif
inline bool decode_hybrid_r(size_t R) { return R >= KFEC_DEC_HYBRID_MIN_R && R <= 8; }
inline size_t decode_hybrid_syn_offset(size_t G, size_t K, size_t R)
{
    return (decode_list_offset(G, K, R) + 256 + 4 * decode_list_chunks(G) + 4 * G + 255) & ~size_t(255);
}
inline size_t decode_workspace_bytes(size_t G, size_t K, size_t R)
{
    if (decode_hybrid_r(R)) return decode_hybrid_syn_offset(G, K, R) + 112 * G;
    return decode_list_offset(G, K, R) + 256 + 4 * decode_list_chunks(G) + 4 * G;
}

// The encoding matrix allocation also holds the perm-MAC tables of its parity rows (gf_perm_tables, 5 dwords
// per coefficient) for the encode kernel, laid out [K][R + 8][5]: shard-major so that the rows of one shard
// are contiguous (scalar loads), with 8 zero rows of slack for any row tile's overshoot.
__host__ __device__ inline size_t enc_tab_rows(size_t R) { return R + 8; }
__host__ __device__ inline size_t enc_tab_offset(size_t K, size_t N) { return (N * K + 255) & ~size_t(255); }
inline size_t enc_alloc_bytes(size_t K, size_t N) { return enc_tab_offset(K, N) + K * enc_tab_rows(N - K) * 5 * 4; }

struct DeviceInfo {
    int device = -1;
    int cus = 0;
};

// multiprocessor count of the current device, cached per device id (grids of the persistent kernels)
int current_device_cus();

// the coder's shared matrix (kfec_api.cpp): device allocation, host copy, worker table-cache id
const uint8_t *ctx_enc(const kfec_ctx *c);
const uint8_t *ctx_h_enc(const kfec_ctx *c);
uint64_t ctx_mat_id(const kfec_ctx *c);

// every launcher returns 0 or a negative KFEC_E* code
int launch_build_matrix(uint8_t *d_enc, int K, int N, hipStream_t s);
int launch_encode(const DeviceInfo &di, const uint8_t *d_enc, int K, int N, size_t G, size_t B, size_t pitch,
                  const void *d_data, void *d_parity, hipStream_t s);
int launch_decode(const DeviceInfo &di, const uint8_t *d_enc, int K, int N, size_t G, size_t B, size_t pitch,
                  const void *d_data, const void *d_parity, const uint64_t *d_present, void *d_out,
                  uint8_t *d_out_idx, uint8_t *d_status, void *d_workspace, hipStream_t s);
int launch_decode_prep(const DeviceInfo &di, const uint8_t *d_enc, int K, int N, size_t G, const uint64_t *d_present,
                       uint8_t *d_out_idx, uint8_t *d_status, void *d_workspace, hipStream_t s, bool syn = false,
                       bool factored = false, const uint32_t *skip_listed = nullptr, uint32_t cols = 0,
                       uint32_t cols_pad = 0);
int launch_synth(uint64_t seed, int N, size_t g0, size_t G, size_t s0, size_t ns, size_t B, size_t pitch,
                 void *d_out, hipStream_t s);
int launch_erasure_masks(uint64_t seed, int N, size_t g0, size_t G, size_t pool, size_t count_max,
                         int random_count, uint64_t *d_present, hipStream_t s);
int launch_verify(int K, int N, size_t G, size_t B, size_t pitch, const void *d_data, const void *d_out,
                  const uint8_t *d_out_idx, uint64_t *d_mismatch, hipStream_t s);

// resident per-call worker (kfec_worker.hip): 0 done, 1 shape not taken (use the launch path), < 0 KFEC_E*
bool worker_enabled();
uint64_t worker_served();  // requests the workers completed (process-wide)
int worker_encode(int device, const uint8_t *d_enc, uint64_t mat_id, int K, int N, size_t B, const uint8_t *input,
                  uint8_t *parity_out);
int worker_decode(int device, const uint8_t *d_enc, const uint8_t *h_enc, uint64_t mat_id, int K, int N, size_t B,
                  const uint8_t *const *row_ptr, int m, const uint8_t *M, const uint8_t *P, uint8_t *out);
void worker_stop(int device);
int worker_ping(int device);  // 0, 1 workers off, < 0 KFEC_E*

// Batch requests through the resident worker (the queues' small flushes, kfec_pipeline.cpp): n groups whose
// shards sit in a device staging arena.  kBatchEncode: the R parity rows of each group's K framed data
// shards; kBatchDecode: the m recovered rows of each group from its K selected shares and the host-solved
// coefficients.  Output row (g, r) at out + (g * R + r) * opitch + ooff (host memory, coherent pinned).
enum { kBatchEncode = 1, kBatchDecode = 2 };
struct BatchSpec {
    int op = kBatchEncode;
    const uint8_t *enc = nullptr;  // encode: the coder's matrix allocation
    uint64_t mat_id = 0;
    const void *arena = nullptr;   // device address (64 bytes of readable headroom before and after)
    uint8_t *out = nullptr;
    size_t opitch = 0, ooff = 0;
    int n = 0, K = 0, N = 0, B = 0;
    const uint64_t *desc = nullptr;  // [n][K] shard descriptors (kfec_worker.hip bdesc_pack)
    const uint8_t *rec = nullptr;    // decode: [n] records of rec_stride bytes: [0] m, [16 + u * K + j] D[u][j]
    size_t rec_stride = 0;
};
// shard descriptor: byte offset in the arena, payload length, raw (parity share) or framed (data shard)
inline uint64_t batch_desc(uint64_t off, uint32_t len, bool raw)
{
    return (off & 0xFFFFFFFFFFull) | ((uint64_t)(len & 0xFFFFu) << 40) | ((uint64_t)raw << 56);
}
bool worker_batch_ok(const BatchSpec &b);
int worker_batch(int device, const BatchSpec &b);  // 0 done, 1 not taken (launch path), < 0 KFEC_E*
uint64_t worker_batches();                          // batch requests served (process-wide)
// the single-group decode's host solve: D[u][j] (m x K) for shares selected as rows M_t <- parity P_t
bool worker_solve(const uint8_t *h_enc, int K, int m, const uint8_t *M, const uint8_t *P, uint8_t *D);
// large-BAR staging: whether the host may write this device's memory directly, the write-combined copy, and
// the fence that orders those writes before a later doorbell / launch
bool bar_writable(int device);
void copy_to_bar(void *dst, const void *src, size_t n);
void bar_fence();

// framing and wire layer (kfec_frame.hip)
int launch_frame(int K, int N, bool recv, size_t G, const void *src, size_t src_bytes, const uint64_t *off,
                 const uint16_t *len, const uint64_t *present, size_t B, size_t pitch, void *data, void *parity,
                 uint16_t *align, hipStream_t s);
// frame_shards + decode fused: 1 when the shape is not taken (the caller falls back to the two-step path)
int launch_framed_decode(const DeviceInfo &di, const uint8_t *d_enc, int K, int N, size_t G, const void *src,
                         size_t src_bytes, const uint64_t *off, const uint16_t *len, const uint64_t *present, size_t B,
                         size_t pitch, void *out, uint8_t *out_idx, uint8_t *status, uint16_t *align,
                         void *workspace, hipStream_t s);
int launch_unframe(int K, int N, size_t G, size_t B, size_t pitch, const void *out, const uint8_t *out_idx,
                   uint16_t *rec_len, void *dst, size_t dst_pitch, hipStream_t s);
int launch_pack(int K, int N, size_t G, unsigned which, const void *src, size_t src_bytes, const uint64_t *off,
                const uint16_t *len, size_t pitch, const void *parity, const uint16_t *align, const uint32_t *sn,
                const uint32_t *conv, uint32_t timestamp, void *pkt, size_t pkt_pitch, uint16_t *pkt_len,
                hipStream_t s);
int launch_unpack(int K, size_t P, const void *src, const uint64_t *off, const uint32_t *len, kfec_pkt_hdr *hdr,
                  hipStream_t s);
int launch_scatter(int N, size_t P, const kfec_pkt_hdr *hdr, const int32_t *slot, uint32_t sn_base, size_t G,
                   uint64_t *present, uint64_t *off, uint16_t *len, hipStream_t s);
// data packets written by the fused encode (kfec_encode_pack_batch): [G][N][pkt_pitch] as kfec_pack_batch
struct DataPackets {
    void *pkt;
    uint16_t *pkt_len;
    const uint32_t *sn;
    size_t pkt_pitch;
    uint32_t timestamp;
};
int launch_framed_encode(const uint8_t *d_enc, int K, int N, size_t G, const void *src, size_t src_bytes,
                         const uint64_t *off, const uint16_t *len, size_t B, size_t pitch, void *parity,
                         uint16_t *align, hipStream_t s, const DataPackets *dp = nullptr);
// off[i] = i * pitch, len32[i] = len16[i] for i < P: descriptors of a packet array for the seal / open calls
int launch_pkt_desc(size_t P, size_t pitch, const uint16_t *len16, uint64_t *off, uint32_t *len32, hipStream_t s);
// packet integrity (kfec_seal.hip)
// done (optional, out-of-place only): coherent pinned u32 that each workgroup adds 1 to when its rows are stored
// and visible to the host; *blocks = the count to wait for (0: nothing launched / no count).  The queues count
// launches of at most kSealCountRows rows (8 workgroups) only: measured faster there, slower with 23 workgroups.
constexpr size_t kSealCountRows = 128;
int launch_seal(bool open, int mode, size_t P, const void *src, size_t src_bytes, const uint64_t *off,
                const uint32_t *len, void *dst, size_t dst_pitch, uint32_t *out_len, uint8_t *ok, hipStream_t s,
                uint32_t *done = nullptr, uint32_t *blocks = nullptr);

}  // namespace kfec

// a per-connection AEAD cipher (include/kfec_aead.h): the derived key and its per-iv device tables
struct kfec_aead {
    int mode = 0;
    int device = 0;
    uint32_t key[8] = {};
    uint32_t *d_tab = nullptr;   // chacha modes: per-iv polykey (xchacha20: subkey first), kfec_aead.hip
    uint8_t *d_rk = nullptr;     // aes_gcm (kfec_gcm.hip): AES-256 round keys
    uint8_t *d_h = nullptr;      //   H = E_K(0)
    uint8_t *d_gh = nullptr;     //   Shoup tables of H^1..H^4
    uint8_t *d_ivt = nullptr;    //   per iv: J0, E_K(J0)
    uint8_t *d_ks = nullptr;     //   per iv: the first ks_bytes of CTR keystream
    uint32_t ks_bytes = 0;
    uint8_t *d_ocb = nullptr;    // aes_ocb (kfec_ocb.hip): round keys, L values, AD hash, T-tables; d_ivt: Offset_0
};

namespace kfec {
int gcm_setup(kfec_aead *k, const uint32_t *d_key, hipStream_t s);
void gcm_free(kfec_aead *k);  // every AES-mode table (gcm and ocb)
int ocb_setup(kfec_aead *k, const uint32_t *d_key, hipStream_t s);
// done / blocks: a counted launch, as launch_seal's (kfec_count.hpp)
int launch_ocb(const kfec_aead *k, bool open, size_t P, const void *src, size_t src_bytes, const uint64_t *off,
               const uint32_t *len, const uint16_t *iv, void *dst, size_t dst_pitch, uint32_t *out_len, uint8_t *ok,
               hipStream_t s, uint32_t *done = nullptr, uint32_t *blocks = nullptr);
int launch_gcm(const kfec_aead *k, bool open, size_t P, const void *src, size_t src_bytes, const uint64_t *off,
               const uint32_t *len, const uint16_t *iv, void *dst, size_t dst_pitch, uint32_t *out_len, uint8_t *ok,
               hipStream_t s, uint32_t *done = nullptr, uint32_t *blocks = nullptr);
// every AEAD mode (chacha20 / xchacha20 here, aes_gcm / aes_ocb through the two above)
int launch_aead(const kfec_aead *k, bool open, size_t P, const void *src, size_t src_bytes, const uint64_t *off,
                const uint32_t *len, const uint16_t *iv, void *dst, size_t dst_pitch, uint32_t *out_len, uint8_t *ok,
                hipStream_t s, uint32_t *done = nullptr, uint32_t *blocks = nullptr);
}  // namespace kfec
