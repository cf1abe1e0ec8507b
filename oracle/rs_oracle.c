/*
 * rs_oracle.c -- TEST INFRASTRUCTURE ONLY (parity checker, never shipped, never measured as the product).
 *
 * A plain-C restatement of the Reed-Solomon coder that kcptube vendors as `fecpp::fec_code`
 * (/root/reference/src/3rd_party/fecpp.{hpp,cpp}).  Only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py may load this file's shared object (oracle/liboracle.so).
 *
 * What is restated, with the reference lines it follows:
 *   - GF(2^8) with polynomial 0x11D and generator alpha = 2:         fecpp.cpp:39-165 (GF_EXP/GF_LOG/
 *     GF_INVERSE/GF_MUL_TABLE).  Here the tables are generated, not transcribed.
 *   - the systematic encoding matrix enc = [I_K ; Vbot * Vtop^-1]:  fecpp.cpp:368-415 (create_inverted_vdm)
 *     and fecpp.cpp:453-490 (setup_matrix).  Here Vtop^-1 is obtained by a generic Gauss-Jordan solve
 *     of the same Vandermonde matrix (V[0][j] = delta_j0, V[r][j] = alpha^((r*j) mod 255)), which is
 *     the unique inverse the reference's synthetic-division formula produces.
 *   - encode: parity r = XOR_j enc[K+r][j] * D_j, with the reference's argument checks:
 *     fecpp.cpp:495-513.
 *   - decode: the share-selection rule (data share i fills row i, each missing row takes the highest
 *     unused id), the `< K shares` and `id >= N` rejections, the K x K inversion and the m output rows:
 *     fecpp.cpp:518-587, invert_matrix fecpp.cpp:229-354 (singular -> error, like the throw at :261/:303).
 *   - synthetic inputs of SURVEY.md section 8(d): splitmix64 counter bytes and per-group erasure draws
 *     (shared definition with the HIP generator in kcptube_amd/csrc/kfec_kernels.hip).
 *
 * Parity is pinned: tests/test_oracle.py checks every function here against tests/golden/ fixtures
 * generated from the reference coder compiled from /root/reference sources (oracle/Makefile,
 * tests/golden/make_golden.py), and against oracle/_ref/libfecpp_ref.so directly when it is present.
 */
#include <stdint.h>
#include <stddef.h>
#include <stdlib.h>
#include <string.h>
#include <pthread.h>
#include <time.h>

#define ORC_OK 0
#define ORC_EMPTY 1      /* reference returns an empty container */
#define ORC_EINVAL -1    /* reference throws std::invalid_argument */

static uint8_t g_exp[512];
static uint8_t g_log[256];
static uint8_t g_mul[256][256];
static pthread_once_t g_once = PTHREAD_ONCE_INIT;

static void gf_build(void)
{
    unsigned v = 1;
    for (int i = 0; i < 255; ++i) {
        g_exp[i] = (uint8_t)v;
        g_log[v] = (uint8_t)i;
        v <<= 1;
        if (v & 0x100) v ^= 0x11D;
    }
    for (int i = 255; i < 512; ++i) g_exp[i] = g_exp[i - 255];
    g_log[0] = 0xFF; /* sentinel, as the reference table */
    for (int a = 0; a < 256; ++a)
        for (int b = 0; b < 256; ++b)
            g_mul[a][b] = (a && b) ? g_exp[g_log[a] + g_log[b]] : 0;
}

static void gf_init(void) { pthread_once(&g_once, gf_build); }

static inline uint8_t gmul(uint8_t a, uint8_t b) { return g_mul[a][b]; }
static inline uint8_t ginv(uint8_t a) { return a ? g_exp[255 - g_log[a]] : 0; }

/* exported table access for the known-answer tests */
void orc_gf_tables(uint8_t exp_out[510], uint8_t log_out[256], uint8_t inv_out[256], uint8_t *mul_out /*65536*/)
{
    gf_init();
    if (exp_out) memcpy(exp_out, g_exp, 510);
    if (log_out) memcpy(log_out, g_log, 256);
    if (inv_out) for (int a = 0; a < 256; ++a) inv_out[a] = ginv((uint8_t)a);
    if (mul_out) memcpy(mul_out, g_mul, 65536);
}

/* z ^= c * x over n bytes (the reference's addmul, fecpp.cpp:170-223, without the SIMD split) */
static void addmul(uint8_t *z, const uint8_t *x, uint8_t c, size_t n)
{
    if (!c) return;
    const uint8_t *row = g_mul[c];
    for (size_t i = 0; i < n; ++i) z[i] ^= row[x[i]];
}

/* In-place Gauss-Jordan inverse of an n x n matrix with full pivot search.
 * Returns 0 on success, -1 if singular (reference: invert_matrix throws, fecpp.cpp:261,303). */
static int gj_invert(uint8_t *a, size_t n)
{
    uint8_t *aug = (uint8_t *)calloc(n * 2 * n, 1);
    if (!aug) return -1;
    const size_t w = 2 * n;
    for (size_t r = 0; r < n; ++r) {
        memcpy(aug + r * w, a + r * n, n);
        aug[r * w + n + r] = 1;
    }
    for (size_t col = 0; col < n; ++col) {
        size_t piv = n;
        for (size_t r = col; r < n; ++r)
            if (aug[r * w + col]) { piv = r; break; }
        if (piv == n) { free(aug); return -1; }
        if (piv != col)
            for (size_t k = 0; k < w; ++k) {
                uint8_t t = aug[piv * w + k]; aug[piv * w + k] = aug[col * w + k]; aug[col * w + k] = t;
            }
        uint8_t inv = ginv(aug[col * w + col]);
        for (size_t k = 0; k < w; ++k) aug[col * w + k] = gmul(aug[col * w + k], inv);
        for (size_t r = 0; r < n; ++r) {
            if (r == col) continue;
            uint8_t f = aug[r * w + col];
            if (f) addmul(aug + r * w, aug + col * w, f, w);
        }
    }
    for (size_t r = 0; r < n; ++r) memcpy(a + r * n, aug + r * w + n, n);
    free(aug);
    return 0;
}

/* Systematic encoding matrix, N x K row-major (fecpp.cpp:453-490 semantics).
 * Returns ORC_EINVAL on a K/N violation (fecpp.cpp:431-432). */
int orc_enc_matrix(size_t K, size_t N, uint8_t *enc)
{
    gf_init();
    if (K == 0 || N == 0 || K > 256 || N > 256 || K > N) return ORC_EINVAL;
    uint8_t *vtop = (uint8_t *)malloc(K * K);
    if (!vtop) return ORC_EINVAL;
    /* evaluation points: row 0 -> 0 (so V[0] = e_0), row r>=1 -> alpha^r */
    for (size_t r = 0; r < K; ++r)
        for (size_t j = 0; j < K; ++j)
            vtop[r * K + j] = (r == 0) ? (j == 0) : g_exp[(r * j) % 255];
    if (gj_invert(vtop, K) != 0) { free(vtop); return ORC_EINVAL; }
    memset(enc, 0, N * K);
    for (size_t i = 0; i < K; ++i) enc[i * K + i] = 1;
    for (size_t r = K; r < N; ++r)
        for (size_t c = 0; c < K; ++c) {
            uint8_t acc = 0;
            for (size_t t = 0; t < K; ++t)
                acc ^= gmul(g_exp[(r * t) % 255], vtop[t * K + c]);
            enc[r * K + c] = acc;
        }
    free(vtop);
    return ORC_OK;
}

/* encode (fecpp.cpp:495-513): reads the first K blocks of `input`, writes N-K parity blocks to
 * parity_out ((N-K) * block_size bytes).  ORC_EMPTY mirrors `return {}`.  block_size == 0 and
 * data_length < K*block_size (an out-of-bounds read in the reference) are rejected as ORC_EMPTY. */
int orc_encode(size_t K, size_t N, const uint8_t *input, size_t data_length, size_t block_size,
               uint8_t *parity_out)
{
    gf_init();
    if (K == 0 || N == 0 || K > 256 || N > 256 || K > N) return ORC_EINVAL;
    if (input == NULL || block_size == 0) return ORC_EMPTY;
    if ((data_length / block_size) % K != 0) return ORC_EMPTY;
    if (data_length < K * block_size) return ORC_EMPTY;
    uint8_t *enc = (uint8_t *)malloc(N * K);
    orc_enc_matrix(K, N, enc);
    memset(parity_out, 0, (N - K) * block_size);
    for (size_t r = K; r < N; ++r)
        for (size_t j = 0; j < K; ++j)
            addmul(parity_out + (r - K) * block_size, input + j * block_size, enc[r * K + j], block_size);
    free(enc);
    return ORC_OK;
}

/* Share selection of fecpp.cpp:528-566.  ids must be strictly ascending (a std::map's order).
 * Fills sel_ids[K] (share id used for row i) and sel_pos[K] (index into ids).
 * Returns ORC_OK, or ORC_EMPTY for `< K shares` / `chosen id >= N`. */
int orc_select(size_t K, size_t N, const size_t *ids, size_t n, size_t *sel_ids, size_t *sel_pos)
{
    if (n < K) return ORC_EMPTY;
    size_t fwd = 0, bwd = n; /* bwd: one past the next highest unused */
    for (size_t i = 0; i < K; ++i) {
        size_t pos;
        if (fwd < n && ids[fwd] == i) pos = fwd++;
        else pos = --bwd;
        if (ids[pos] >= N) return ORC_EMPTY;
        sel_ids[i] = ids[pos];
        sel_pos[i] = pos;
    }
    return ORC_OK;
}

/* decode (fecpp.cpp:518-587).  Shares are given as ascending ids + pointers.  Writes the recovered
 * missing data shards, in ascending row order, to out (n_out * share_size) and their row indices to
 * out_ids.  Returns ORC_OK, ORC_EMPTY (empty map) or ORC_EINVAL (singular: the reference throws). */
int orc_decode(size_t K, size_t N, const size_t *ids, const uint8_t *const *ptrs, size_t n,
               size_t share_size, size_t *out_ids, uint8_t *out, size_t *n_out)
{
    gf_init();
    *n_out = 0;
    if (K == 0 || N == 0 || K > 256 || N > 256 || K > N) return ORC_EINVAL;
    size_t *sel_ids = (size_t *)malloc(K * sizeof(size_t));
    size_t *sel_pos = (size_t *)malloc(K * sizeof(size_t));
    int rc = orc_select(K, N, ids, n, sel_ids, sel_pos);
    if (rc != ORC_OK) { free(sel_ids); free(sel_pos); return rc; }
    uint8_t *enc = (uint8_t *)malloc(N * K);
    uint8_t *mdec = (uint8_t *)calloc(K * K, 1);
    orc_enc_matrix(K, N, enc);
    for (size_t i = 0; i < K; ++i) {
        if (sel_ids[i] < K) mdec[i * K + sel_ids[i]] = 1;   /* data share i sits in row i */
        else memcpy(mdec + i * K, enc + sel_ids[i] * K, K);
    }
    if (gj_invert(mdec, K) != 0) {
        free(sel_ids); free(sel_pos); free(enc); free(mdec);
        return ORC_EINVAL;
    }
    size_t m = 0;
    for (size_t i = 0; i < K; ++i) {
        if (sel_ids[i] < K) continue;
        uint8_t *dst = out + m * share_size;
        memset(dst, 0, share_size);
        for (size_t c = 0; c < K; ++c)
            addmul(dst, ptrs[sel_pos[c]], mdec[i * K + c], share_size);
        out_ids[m++] = i;
    }
    *n_out = m;
    free(sel_ids); free(sel_pos); free(enc); free(mdec);
    return ORC_OK;
}

/* ---------------------------------------------------------------------------------------------
 * Synthetic inputs; the HIP generator in kfec_kernels.hip must agree.
 * Byte b of shard slot s (0 <= s < N) in group g is byte (b % 8) (little-endian) of
 *     splitmix64(seed ^ ((g * N + s) * W + b / 8)),  W = ceil(B / 8).
 * -------------------------------------------------------------------------------------------*/
static inline uint64_t splitmix64(uint64_t x)
{
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

uint64_t orc_splitmix64(uint64_t x) { return splitmix64(x); }

/* fill shards [s0, s0+ns) of groups [g0, g0+ng) into out laid out [ng][ns][pitch] */
void orc_synth(uint64_t seed, size_t N, size_t B, size_t g0, size_t ng, size_t s0, size_t ns,
               uint8_t *out, size_t pitch)
{
    const size_t W = (B + 7) / 8;
    for (size_t g = 0; g < ng; ++g)
        for (size_t s = 0; s < ns; ++s) {
            uint8_t *dst = out + (g * ns + s) * pitch;
            const uint64_t base = ((g0 + g) * N + (s0 + s)) * W;
            for (size_t w = 0; w < W; ++w) {
                uint64_t v = splitmix64(seed ^ (base + w));
                for (size_t k = 0; k < 8 && w * 8 + k < B; ++k) dst[w * 8 + k] = (uint8_t)(v >> (8 * k));
            }
        }
}

/* Per-group erasure draw.  Pool = shard ids [0, pool); erase `cnt` distinct ids by a partial
 * Fisher-Yates shuffle driven by splitmix64(seed ^ (g * 0x100 + t)).  Writes a 256-bit present
 * mask (4 x u64, bit s set = shard s present) with every id in [0, N) present except the erased. */
void orc_erasure_mask(uint64_t seed, size_t g, size_t N, size_t pool, size_t cnt, uint64_t mask[4])
{
    uint8_t perm[256];
    for (size_t i = 0; i < 256; ++i) perm[i] = (uint8_t)i;
    mask[0] = mask[1] = mask[2] = mask[3] = 0;
    for (size_t s = 0; s < N; ++s) mask[s >> 6] |= 1ull << (s & 63);
    for (size_t t = 0; t < cnt && t < pool; ++t) {
        uint64_t r = splitmix64(seed ^ ((uint64_t)g * 0x100u + t));
        size_t k = t + (size_t)(r % (uint64_t)(pool - t));
        uint8_t tmp = perm[t]; perm[t] = perm[k]; perm[k] = tmp;
        mask[perm[t] >> 6] &= ~(1ull << (perm[t] & 63));
    }
}

/* i.i.d. loss (random_count == 2 in kfec_erasure_masks): shard s of group g is lost when
 * splitmix64(seed ^ 0xC2B2AE3D27D4EB4F ^ (g * 0x100 + s)) % 1000000 < ppm, independently for every s < N. */
void orc_erasure_mask_iid(uint64_t seed, size_t g, size_t N, size_t ppm, uint64_t mask[4])
{
    mask[0] = mask[1] = mask[2] = mask[3] = 0;
    for (size_t s = 0; s < N; ++s) {
        uint64_t r = splitmix64(seed ^ 0xC2B2AE3D27D4EB4Full ^ ((uint64_t)g * 0x100u + s));
        if (r % 1000000u >= ppm) mask[s >> 6] |= 1ull << (s & 63);
    }
}

/* erasure count for "random 1..maxc over all N" configs: 1 + splitmix64(seed ^ ~g) % maxc */
size_t orc_erasure_count(uint64_t seed, size_t g, size_t maxc)
{
    return 1 + (size_t)(splitmix64(seed ^ ~(uint64_t)g) % (uint64_t)maxc);
}

/* ---------------------------------------------------------------------------------------------
 * Batched helpers so the Python tests stay fast.  Layout: data [G][K][pitch], parity [G][R][pitch],
 * present masks [G][4] (u64).  Decode outputs: out [G][R][pitch], out_idx [G][R] (0xFF unused),
 * status [G] (0 ok, 1 empty).  These are loops over the single-group functions above.
 * -------------------------------------------------------------------------------------------*/
int orc_encode_batch(size_t K, size_t N, size_t G, size_t B, size_t pitch, const uint8_t *data,
                     uint8_t *parity)
{
    gf_init();
    const size_t R = N - K;
    uint8_t *enc = (uint8_t *)malloc(N * K);
    int rc = orc_enc_matrix(K, N, enc);
    if (rc != ORC_OK) { free(enc); return rc; }
    for (size_t g = 0; g < G; ++g)
        for (size_t r = 0; r < R; ++r) {
            uint8_t *dst = parity + (g * R + r) * pitch;
            memset(dst, 0, B);
            for (size_t j = 0; j < K; ++j)
                addmul(dst, data + (g * K + j) * pitch, enc[(K + r) * K + j], B);
        }
    free(enc);
    return ORC_OK;
}

int orc_decode_batch(size_t K, size_t N, size_t G, size_t B, size_t pitch, const uint8_t *data,
                     const uint8_t *parity, const uint64_t *present, uint8_t *out, uint8_t *out_idx,
                     uint8_t *status)
{
    gf_init();
    const size_t R = N - K;
    size_t ids[256];
    const uint8_t *ptrs[256];
    size_t oids[256];
    uint8_t *tmp = (uint8_t *)malloc(K * B + 1);
    for (size_t g = 0; g < G; ++g) {
        size_t n = 0;
        for (size_t s = 0; s < N; ++s)
            if (present[g * 4 + (s >> 6)] >> (s & 63) & 1) {
                ids[n] = s;
                ptrs[n] = s < K ? data + (g * K + s) * pitch : parity + (g * R + (s - K)) * pitch;
                ++n;
            }
        size_t n_out = 0;
        int rc = orc_decode(K, N, ids, ptrs, n, B, oids, tmp, &n_out);
        if (R) memset(out_idx + g * R, 0xFF, R);
        status[g] = (rc == ORC_OK) ? 0 : 1;
        for (size_t t = 0; t < n_out; ++t) {
            memcpy(out + (g * R + t) * pitch, tmp + t * B, B);
            out_idx[g * R + t] = (uint8_t)oids[t];
        }
    }
    free(tmp);
    return ORC_OK;
}

/* ---------------------------------------------------------------------------------------------
 * CPU timing harness used by bench.py's cpu_baseline leg when oracle/_ref is absent ("port").
 * Runs encode + (erase `erase` data shards) + decode over G groups of synthetic data with T threads
 * for at least min_seconds; returns payload bytes per second (G*K*B per pass / time).
 * -------------------------------------------------------------------------------------------*/
typedef struct {
    size_t K, N, B, g0, ng, erase, passes;
    uint64_t seed;
    const uint8_t *data;
    double ok;
} orc_job;

static void *orc_worker(void *arg)
{
    orc_job *j = (orc_job *)arg;
    const size_t K = j->K, N = j->N, B = j->B, R = N - K;
    uint8_t *par = (uint8_t *)malloc(R * B + 1), *rec = (uint8_t *)malloc(K * B + 1);
    size_t ids[256], oids[256];
    const uint8_t *ptrs[256];
    size_t good = 0;
    for (size_t p = 0; p < j->passes; ++p)
        for (size_t g = 0; g < j->ng; ++g) {
            const uint8_t *d = j->data + (j->g0 + g) * K * B;
            orc_encode(K, N, d, K * B, B, par);
            uint64_t mask[4];
            orc_erasure_mask(j->seed, j->g0 + g, N, K, j->erase, mask);
            size_t n = 0;
            for (size_t s = 0; s < N; ++s)
                if (mask[s >> 6] >> (s & 63) & 1) {
                    ids[n] = s;
                    ptrs[n] = s < K ? d + s * B : par + (s - K) * B;
                    ++n;
                }
            size_t n_out = 0;
            orc_decode(K, N, ids, ptrs, n, B, oids, rec, &n_out);
            good += (n_out == j->erase);
        }
    j->ok = (double)good;
    free(par); free(rec);
    return NULL;
}

double orc_bench_roundtrip(size_t K, size_t N, size_t B, size_t G, size_t erase, size_t threads,
                           size_t passes, uint64_t seed, double *seconds_out)
{
    gf_init();
    uint8_t *data = (uint8_t *)malloc(G * K * B);
    orc_synth(seed, N, B, 0, G, 0, K, data, B); /* note: synth over K slots laid out [G][K][B] */
    /* orc_synth with ns=K writes [G][K][B] directly */
    pthread_t th[256];
    orc_job jobs[256];
    if (threads > 256) threads = 256;
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    for (size_t t = 0; t < threads; ++t) {
        size_t a = G * t / threads, b = G * (t + 1) / threads;
        jobs[t] = (orc_job){K, N, B, a, b - a, erase, passes, seed, data, 0};
        pthread_create(&th[t], NULL, orc_worker, &jobs[t]);
    }
    for (size_t t = 0; t < threads; ++t) pthread_join(th[t], NULL);
    clock_gettime(CLOCK_MONOTONIC, &t1);
    double secs = (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
    if (seconds_out) *seconds_out = secs;
    free(data);
    return (double)(G * passes) * (double)(K * B) / secs;
}
