/* cpu_aead.c -- CPU baseline for the AEAD packet kernels: OpenSSL's ChaCha20-Poly1305 or AES-256-GCM (its
 * AVX-512 / VAES assembly) over P packets of L bytes with kcptube's associated data and per-packet nonces,
 * on T threads.
 * Botan (the reference's library) is absent from the image; OpenSSL's implementation of the same cipher
 * stands in for it.  The draft 8-byte-nonce construction costs the same (one more 16-byte MAC block), and
 * xchacha20 adds one HChaCha20 per packet (not counted here: a lower bound on CPU time).
 *
 *   tools/cpu_aead <packets> <len> <threads>     -> one JSON line: GB/s of plaintext sealed
 *
 *   tools/cpu_aead <packets> <len> <threads> gcm -> the same with AES-256-GCM (16-byte nonce, as kcptube's)
 *
 * Build: gcc -O2 -pthread -o tools/cpu_aead tools/cpu_aead.c -lcrypto
 */
#include <openssl/evp.h>
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

static size_t g_packets, g_len;
static int g_gcm;
static uint8_t g_key[32];

typedef struct {
    size_t p0, p1;
    uint8_t *buf;
    int fail;
} job;

static void *worker(void *arg)
{
    job *j = (job *)arg;
    EVP_CIPHER_CTX *ctx = EVP_CIPHER_CTX_new();
    static const unsigned char ad[] = "KCP PortHopping";
    uint8_t out[65536 + 32], tag[16], nonce[16];
    int n = 0;
    const int nlen = g_gcm ? 16 : 12;
    if (!ctx || EVP_EncryptInit_ex(ctx, g_gcm ? EVP_aes_256_gcm() : EVP_chacha20_poly1305(), NULL, NULL, NULL) != 1 ||
        EVP_CIPHER_CTX_ctrl(ctx, EVP_CTRL_AEAD_SET_IVLEN, nlen, NULL) != 1 ||
        EVP_EncryptInit_ex(ctx, NULL, NULL, g_key, NULL) != 1)
        j->fail = 1;
    for (size_t p = j->p0; p < j->p1 && !j->fail; ++p) {
        const uint16_t iv = (uint16_t)(p * 40503u);
        for (int i = 0; i < nlen; i += 2) memcpy(nonce + i, &iv, 2);
        if (EVP_EncryptInit_ex(ctx, NULL, NULL, NULL, nonce) != 1 ||
            EVP_EncryptUpdate(ctx, NULL, &n, ad, 15) != 1 ||
            EVP_EncryptUpdate(ctx, out, &n, j->buf + (p % 64) * g_len, (int)g_len) != 1 ||
            EVP_EncryptFinal_ex(ctx, out + n, &n) != 1 ||
            EVP_CIPHER_CTX_ctrl(ctx, EVP_CTRL_AEAD_GET_TAG, 16, tag) != 1)
            j->fail = 1;
        j->buf[(p % 64) * g_len] ^= tag[0];  /* keep the work observable */
    }
    EVP_CIPHER_CTX_free(ctx);
    return NULL;
}

int main(int argc, char **argv)
{
    if (argc < 4) {
        fprintf(stderr, "usage: %s packets len threads [gcm]\n", argv[0]);
        return 2;
    }
    g_gcm = argc > 4 && strcmp(argv[4], "gcm") == 0;
    g_packets = strtoull(argv[1], NULL, 10);
    g_len = strtoull(argv[2], NULL, 10);
    int T = atoi(argv[3]);
    if (g_len == 0 || g_len > 65536 || T < 1 || T > 1024) return 2;
    for (int i = 0; i < 32; ++i) g_key[i] = (uint8_t)(i * 7 + 1);
    pthread_t *th = calloc(T, sizeof(pthread_t));
    job *jobs = calloc(T, sizeof(job));
    for (int t = 0; t < T; ++t) {
        jobs[t].buf = malloc(64 * g_len);
        for (size_t i = 0; i < 64 * g_len; ++i) jobs[t].buf[i] = (uint8_t)(i * 31 + t);
        jobs[t].p0 = g_packets * t / T;
        jobs[t].p1 = g_packets * (t + 1) / T;
    }
    struct timespec a, b;
    clock_gettime(CLOCK_MONOTONIC, &a);
    for (int t = 0; t < T; ++t) pthread_create(&th[t], NULL, worker, &jobs[t]);
    int fail = 0;
    for (int t = 0; t < T; ++t) {
        pthread_join(th[t], NULL);
        fail |= jobs[t].fail;
    }
    clock_gettime(CLOCK_MONOTONIC, &b);
    const double s = (b.tv_sec - a.tv_sec) + 1e-9 * (b.tv_nsec - a.tv_nsec);
    printf("{\"cipher\": \"%s\", \"packets\": %zu, \"len\": %zu, \"threads\": %d, \"seconds\": %.4f, \"GBps\": %.3f, "
           "\"ok\": %s}\n", g_gcm ? "AES-256-GCM" : "ChaCha20-Poly1305", g_packets, g_len, T, s,
           g_packets * (double)g_len / s / 1e9, fail ? "false" : "true");
    return fail ? 1 : 0;
}
