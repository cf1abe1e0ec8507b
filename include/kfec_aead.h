/*
 * kfec_aead.h -- kcptube's AEAD packet modes on the device (the AEAD half).
 *
 * encrypt_data / decrypt_data (/root/reference/src/shares/data_operations.cpp:171-234, 373-435) for
 * encryption = aes_gcm, aes_ocb, chacha20 and xchacha20, with the key and nonce handling of the reference's
 * aead.hpp:
 *   key    = SHA-3(256)(password)                                          (aead.hpp:405-437, 488-515)
 *   nonce  = the 16-bit iv_raw repeated: 16 bytes (aes_gcm), 12 (aes_ocb), 8 (chacha20), 24 (xchacha20)
 *            (aead.hpp:291-311, 379-400, 464-483, 542-562)
 *   packet = ciphertext || 16-byte tag || iv_raw (2 bytes, little-endian)    (data_operations.cpp:214-219);
 *            the tag is Poly1305 (chacha20, xchacha20), GHASH (aes_gcm) or the OCB tag (aes_ocb)
 *   associated data "KCP PortHopping"                                      (aead.hpp:16)
 * Botan's AES-256/GCM takes the 16-byte nonce through GHASH into J0 (SP 800-38D); AES-256/OCB is RFC 7253
 * with a 128-bit tag.
 * Botan's ChaCha20Poly1305 (the reference's library) runs the 8-byte nonce as the original construction
 * (64-bit block counter; MAC over AD || le64(|AD|) || C || le64(|C|)) and the 24-byte nonce as
 * XChaCha20-Poly1305 (HChaCha20 subkey, RFC 8439 MAC layout).  oracle/aead_oracle.py restates both and
 * tests/test_aead_oracle.py pins them against OpenSSL's libcrypto.
 *
 * The nonce depends only on iv_raw, so everything the key and the nonce alone determine -- the Poly1305 key
 * (ChaCha20 block 0), for xchacha20 the HChaCha20 subkey, and the first 2 KiB of keystream; for aes_gcm J0,
 * E_K(J0) and the first 2 KiB of CTR keystream; for aes_ocb Offset_0 -- is computed once per key for all
 * 65536 iv values (kfec_aead_create, on the device: 130 / 132 / 130 / 1 MiB for chacha20 / xchacha20 /
 * aes_gcm / aes_ocb) and looked up per packet.
 *
 * Conventions as include/kfec.h: d_ pointers are device pointers, the stream is a hipStream_t as void*.
 */
#ifndef KFEC_AEAD_H_
#define KFEC_AEAD_H_

#include <stddef.h>
#include <stdint.h>

#include "kfec.h"

#ifdef __cplusplus
extern "C" {
#endif

/* encryption_mode values (share_defines.hpp:29) this header implements */
#define KFEC_AEAD_AES_GCM 4    /* encryption_mode::aes_gcm: AES-256-GCM, 16-byte nonce */
#define KFEC_AEAD_AES_OCB 5    /* encryption_mode::aes_ocb: AES-256-OCB (RFC 7253), 12-byte nonce */
#define KFEC_AEAD_CHACHA20 6   /* encryption_mode::chacha20: ChaCha20-Poly1305, 8-byte nonce */
#define KFEC_AEAD_XCHACHA20 7  /* encryption_mode::xchacha20: XChaCha20-Poly1305, 24-byte nonce */
#define KFEC_AEAD_TAG 16
#define KFEC_AEAD_OVERHEAD 18  /* tag + iv_raw trailer (constant_values::iv_checksum_block_size) */

typedef struct kfec_aead kfec_aead;

/* The per-connection cipher object (encrypt_decrypt<chacha20 / xchacha20>(password), aead.hpp): derives the
 * key on the current HIP device and builds the per-iv tables there.  KFEC_EINVAL for another mode or an
 * empty password (the reference leaves its Botan objects unset then, aead.hpp:408-413, and the first packet
 * dereferences them); KFEC_ENODEV without a GPU; KFEC_ENOMEM.
 *
 * Device memory: EVERY object holds its own tables on its device -- about 130 MiB (chacha20, aes_gcm: 128 MiB
 * of per-iv keystream), 132 MiB (xchacha20) or 1 MiB (aes_ocb).  Objects are not shared between connections
 * with the same password and mode, so create one per password and device (kcptube derives everything from
 * the password) and hand it to every connection that uses it; the object is read-only after creation and
 * may be used from several threads and streams at once.  Creation runs on a private stream and blocks the
 * calling thread for ~2 ms; the seal / open calls switch to the object's device before launching. */
int kfec_aead_create(int mode, const void *password, size_t password_len, kfec_aead **out);
void kfec_aead_destroy(kfec_aead *a);
int kfec_aead_mode(const kfec_aead *a);
/* The derived 32-byte key, copied to host memory (tests). */
int kfec_aead_key(const kfec_aead *a, uint8_t key[32]);

/* encrypt_data for P packets [d_off[p], +d_len[p]) of d_src (dword-aligned base, src_bytes long) with the
 * 16-bit iv_raw d_iv[p] (the caller's uniformly random draw -- change_iv(), aead.hpp:464-475): writes
 * ciphertext || tag || iv_raw to d_dst + p * dst_pitch (dst_pitch % 4 == 0, d_dst dword-aligned) and
 * d_out_len[p] = len + 18; bytes after it up to the next multiple of 4 are written as zero.  An empty packet
 * ("empty data", data_operations.cpp:173-174) or one whose len + 18 exceeds dst_pitch gets d_out_len = 0. */
int kfec_aead_seal_batch(const kfec_aead *a, size_t P, const void *d_src, size_t src_bytes, const uint64_t *d_off,
                         const uint32_t *d_len, const uint16_t *d_iv, void *d_dst, size_t dst_pitch,
                         uint32_t *d_out_len, void *stream);

/* decrypt_data for P sealed packets: iv_raw from each packet's last two bytes, the tag verified over the
 * ciphertext.  d_ok[p] = 1 and d_out_len[p] = len - 18 with the plaintext at d_dst + p * dst_pitch (zero
 * padded to a multiple of 4) when the tag verifies; otherwise d_ok[p] = 0 and d_out_len[p] = 0.  A packet
 * whose tag fails has its dst bytes zeroed; packets rejected on length -- shorter than 18 bytes (decrypt_data:
 * "incorrect data length" for <= 2 bytes, Botan's too-short-for-the-tag exception for the rest) or with a
 * plaintext longer than dst_pitch -- leave their dst bytes untouched. */
int kfec_aead_open_batch(const kfec_aead *a, size_t P, const void *d_src, size_t src_bytes, const uint64_t *d_off,
                         const uint32_t *d_len, void *d_dst, size_t dst_pitch, uint32_t *d_out_len, uint8_t *d_ok,
                         void *stream);

#ifdef __cplusplus
}
#endif

#endif /* KFEC_AEAD_H_ */
