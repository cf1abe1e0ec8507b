// kfec_api.cpp -- C ABI of libkfec.so (include/kfec.h): coder contexts, argument checking with the
// reference's error conventions, single-group staging for the fecpp::fec_code drop-in, and the
// batched device-resident entry points.  Every output byte (parity, recovered shards) is computed by the HIP
// kernels (kfec_kernels.hip, kfec_worker.hip).  The host does bookkeeping and coefficients only: the
// single-group decode selects its shares here (fecpp.cpp:528-548), and for small losses through the resident
// worker the m x K decode coefficients are solved on the host (host_solve, kfec_worker.hip).
#include "../../include/kfec.h"
#include "../../include/kfec_frame.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <new>
#include <string>
#include <vector>

#include "kfec_internal.hpp"

namespace {

// The encoding matrix depends on (K, N) alone, so every coder of one device with the same (K, N) shares ONE
// immutable device allocation (the N x K matrix, then its perm tables) and its host copy.  kcptube builds a
// coder per connection and direction and re-targets it with reset_martix (client.cpp:1755, relay.cpp:947,
// server.cpp:438): after the first coder of a shape, create / reset are a table lookup -- no allocation, no
// launch, no synchronisation.  Each matrix counts the coders pointing at it.  A matrix no coder points at stays
// cached (a reset back to its shape is a lookup again, and a batched launch still reading it stays valid) until
// more than kKeepUnused such matrices -- or more than kKeepUnusedBytes of them -- exist on the device: then the
// least recently released ones are freed.  hipFree waits for every stream of the device (in-flight launches that
// still read the matrix finish first; the resident worker's lease bounds that wait), so eviction only runs on
// the rare reset that leaves the cache over its bound, never on the common lookup.  What is left goes with the
// device's last coder, after its workers have stopped.  Matrix ids are never reused, so the worker's LDS table
// cache (keyed by id) cannot mistake a new matrix at a freed address for the old one.
constexpr size_t kKeepUnused = 8;
constexpr size_t kKeepUnusedBytes = size_t(4) << 20;
struct Matrix {
    size_t K = 0, N = 0;
    uint8_t *d = nullptr;     // N x K matrix, then the perm tables (enc_alloc_bytes)
    std::vector<uint8_t> h;   // host copy of the N x K matrix
    uint64_t id = 0;          // unique per built matrix: the resident worker's LDS table-cache key
    size_t refs = 0;          // coders whose d_enc is this matrix
    uint64_t released = 0;    // release clock when refs last dropped to 0 (eviction order)
};
struct DevMatrices {
    std::mutex mu;
    hipStream_t stream = nullptr;  // builds run here
    std::vector<Matrix *> all;
    uint64_t clock = 0;
};
DevMatrices g_mats[64];
std::atomic<uint64_t> g_mat_ids{0};

}  // namespace

struct kfec_ctx {
    size_t K = 0, N = 0;
    kfec::DeviceInfo di;
    const uint8_t *d_enc = nullptr;  // the shared matrix of (K, N) on the device (Matrix::d)
    const uint8_t *h_enc = nullptr;  // its host copy (Matrix::h)
    uint64_t mat_id = 0;             // Matrix::id
    Matrix *mat = nullptr;           // the shared matrix this coder holds a reference on
    hipStream_t stream = nullptr;    // private stream of the single-group launch path (created on first use)
    std::mutex mu;                   // single-group staging is shared by encode and decode callers
    uint8_t *d_stage = nullptr;
    size_t stage_cap = 0;
    uint8_t *h_stage = nullptr;  // fine-grained pinned host staging the kernels read and write in place
    size_t h_stage_cap = 0;
    bool counted = false;        // kfec_create returned it (counted in g_live)
};

const uint8_t *kfec::ctx_enc(const kfec_ctx *c) { return c->d_enc; }
const uint8_t *kfec::ctx_h_enc(const kfec_ctx *c) { return c->h_enc; }
uint64_t kfec::ctx_mat_id(const kfec_ctx *c) { return c->mat_id; }

int kfec::current_device_cus()
{
    static std::atomic<int> cache[64];
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess) return 256;
    if (dev < 0 || dev >= 64) {
        return hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && n > 0 ? n : 256;
    }
    n = cache[dev].load(std::memory_order_relaxed);
    if (n > 0) return n;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) return 256;
    cache[dev].store(n, std::memory_order_relaxed);
    return n;
}

namespace {

bool kn_valid(size_t K, size_t N) { return !(K == 0 || N == 0 || K > 256 || N > 256 || K > N); }

std::mutex g_live_mu;
int g_live[64];  // coders per device: the resident workers and the cached matrices of a device go with its last coder

int probe_device(kfec::DeviceInfo &di)
{
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return KFEC_ENODEV;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return KFEC_ENODEV;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, dev) != hipSuccess) return KFEC_ENODEV;
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) return KFEC_ENODEV;  // code objects are gfx950-only
    if (dev < 0 || dev >= 64) return KFEC_ENODEV;
    di.device = dev;
    di.cus = prop.multiProcessorCount;
    return KFEC_OK;
}

// Unlink the least recently released unreferenced matrices while more than kKeepUnused (or kKeepUnusedBytes) of
// them are cached.  Called with dm.mu held; the caller frees what it returns after releasing the lock.
std::vector<Matrix *> evict_unused(DevMatrices &dm)
{
    std::vector<Matrix *> gone;
    for (;;) {
        size_t n = 0, bytes = 0;
        Matrix *oldest = nullptr;
        for (Matrix *m : dm.all) {
            if (m->refs) continue;
            ++n;
            bytes += kfec::enc_alloc_bytes(m->K, m->N);
            if (!oldest || m->released < oldest->released) oldest = m;
        }
        if (!oldest || (n <= kKeepUnused && bytes <= kKeepUnusedBytes)) return gone;
        dm.all.erase(std::remove(dm.all.begin(), dm.all.end(), oldest), dm.all.end());
        try {
            gone.push_back(oldest);
        } catch (...) {
            (void)hipFree(oldest->d);  // (out of host memory: free it here, under the lock, as before)
            delete oldest;
        }
    }
}

void unref_matrix(int dev, Matrix *m)
{
    if (!m) return;
    DevMatrices &dm = g_mats[dev];
    std::vector<Matrix *> gone;
    {
        std::lock_guard<std::mutex> lk(dm.mu);
        if (m->refs && --m->refs == 0) {
            m->released = ++dm.clock;
            gone = evict_unused(dm);
        }
    }
    // hipFree waits for the device's in-flight work (which may still read the matrix) -- up to the longest
    // batched launch, ~150 ms at fec=200:55 -- so it runs without the lock: kfec_create / kfec_reset /
    // kfec_cached_matrices of other threads on this device do not queue behind it
    for (Matrix *g : gone) {
        (void)hipFree(g->d);
        delete g;
    }
}

// The shared matrix of (K, N) on the current device, built on first use, with one more reference counted on
// it.  nullptr + rc on failure.
Matrix *get_matrix(int dev, size_t K, size_t N, int &rc)
{
    DevMatrices &dm = g_mats[dev];
    std::lock_guard<std::mutex> lk(dm.mu);
    for (Matrix *m : dm.all)
        if (m->K == K && m->N == N) {
            ++m->refs;
            rc = KFEC_OK;
            return m;
        }
    rc = KFEC_EHIP;
    if (!dm.stream && hipStreamCreateWithFlags(&dm.stream, hipStreamNonBlocking) != hipSuccess) {
        dm.stream = nullptr;
        return nullptr;
    }
    Matrix *m = new (std::nothrow) Matrix;
    if (!m) {
        rc = KFEC_ENOMEM;
        return nullptr;
    }
    try {
        m->h.assign(N * K, 0);
        dm.all.reserve(dm.all.size() + 1);
    } catch (...) {
        delete m;
        rc = KFEC_ENOMEM;
        return nullptr;
    }
    void *d = nullptr;
    if (hipMalloc(&d, kfec::enc_alloc_bytes(K, N)) != hipSuccess) {
        delete m;
        rc = KFEC_ENOMEM;
        return nullptr;
    }
    m->d = static_cast<uint8_t *>(d);
    if (kfec::launch_build_matrix(m->d, (int)K, (int)N, dm.stream) ||
        hipMemcpyAsync(m->h.data(), m->d, N * K, hipMemcpyDeviceToHost, dm.stream) != hipSuccess ||
        hipStreamSynchronize(dm.stream) != hipSuccess) {
        (void)hipStreamSynchronize(dm.stream);
        (void)hipFree(m->d);  // (first use of a shape only, and only on failure)
        delete m;
        return nullptr;
    }
    m->K = K;
    m->N = N;
    m->id = g_mat_ids.fetch_add(1) + 1;
    m->refs = 1;
    dm.all.push_back(m);
    rc = KFEC_OK;
    return m;
}

// Re-target the context to (K, N); commits only once the matrix exists (a failed reset leaves it unchanged).
int set_matrix(kfec_ctx *c, size_t K, size_t N)
{
    int rc = KFEC_OK;
    Matrix *m = get_matrix(c->di.device, K, N, rc);
    if (!m) return rc;
    Matrix *old = c->mat;
    c->mat = m;
    c->d_enc = m->d;
    c->h_enc = m->h.data();
    c->K = K;
    c->N = N;
    c->mat_id = m->id;
    unref_matrix(c->di.device, old);  // (after the new one is referenced: a reset to the same shape keeps it)
    return KFEC_OK;
}

// The device's last coder is gone and its workers have stopped: release the cached matrices.
void release_matrices(int dev)
{
    DevMatrices &dm = g_mats[dev];
    std::lock_guard<std::mutex> lk(dm.mu);
    for (Matrix *m : dm.all) {
        (void)hipFree(m->d);
        delete m;
    }
    dm.all.clear();
}

int ensure_stream(kfec_ctx *c)
{
    if (c->stream) return KFEC_OK;
    if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
        c->stream = nullptr;
        return KFEC_EHIP;
    }
    return KFEC_OK;
}

int ensure_stage(kfec_ctx *c, size_t bytes)
{
    if (bytes <= c->stage_cap) return KFEC_OK;
    if (c->d_stage) (void)hipFree(c->d_stage);
    c->d_stage = nullptr;
    c->stage_cap = 0;
    const size_t cap = std::max<size_t>(bytes, 64 * 1024);
    if (hipMalloc(&c->d_stage, cap) != hipSuccess) return KFEC_ENOMEM;
    c->stage_cap = cap;
    return KFEC_OK;
}

inline size_t al256(size_t x) { return (x + 255) & ~size_t(255); }

// Single-group calls (the drop-in's per-call path) are latency-bound: a DMA copy costs ~10 us to set up, more
// than a 29 KB group's whole encode.  So the shares are gathered on the host into fine-grained (coherent)
// pinned memory, and the kernels read the shares and write the recovered / parity blocks there directly over
// PCIe; the decode records stay in device memory.  KFEC_ZERO_COPY=0 restores the copy-based path (A/B).
bool zero_copy()
{
    static const bool on = [] {
        const char *e = getenv("KFEC_ZERO_COPY");
        return !(e && std::string(e) == "0");
    }();
    return on;
}

int ensure_host_stage(kfec_ctx *c, size_t bytes)
{
    if (bytes <= c->h_stage_cap) return KFEC_OK;
    if (c->h_stage) (void)hipHostFree(c->h_stage);
    c->h_stage = nullptr;
    c->h_stage_cap = 0;
    const size_t cap = std::max<size_t>(bytes, 64 * 1024);
    void *p = nullptr;
    if (hipHostMalloc(&p, cap, hipHostMallocCoherent) != hipSuccess) return KFEC_ENOMEM;
    c->h_stage = static_cast<uint8_t *>(p);
    c->h_stage_cap = cap;
    return KFEC_OK;
}

inline hipStream_t as_stream(void *s) { return static_cast<hipStream_t>(s); }

inline int set_dev(const kfec_ctx *c) { return hipSetDevice(c->di.device) == hipSuccess ? KFEC_OK : KFEC_EHIP; }

}  // namespace

extern "C" {

const char *kfec_version(void) { return "kfec 0.3 (gfx950 perm-MAC, flattened column kernel)"; }

int kfec_device(const kfec_ctx *ctx) { return ctx ? ctx->di.device : -1; }

uint64_t kfec_worker_requests(void) { return kfec::worker_served(); }

uint64_t kfec_worker_batches(void) { return kfec::worker_batches(); }

size_t kfec_cached_matrices(const kfec_ctx *ctx, size_t *bytes)
{
    if (bytes) *bytes = 0;
    if (!ctx) return 0;
    DevMatrices &dm = g_mats[ctx->di.device];
    std::lock_guard<std::mutex> lk(dm.mu);
    size_t b = 0;
    for (const Matrix *m : dm.all) b += kfec::enc_alloc_bytes(m->K, m->N);
    if (bytes) *bytes = b;
    return dm.all.size();
}

int kfec_worker_ping(const kfec_ctx *ctx)
{
    if (!ctx) return KFEC_EINVAL;
    if (set_dev(ctx)) return KFEC_EHIP;
    const int rc = kfec::worker_ping(ctx->di.device);
    return rc == 1 ? KFEC_ENODEV : rc;
}

int kfec_create(size_t K, size_t N, kfec_ctx **out)
{
    if (!out) return KFEC_EINVAL;
    *out = nullptr;
    if (!kn_valid(K, N)) return KFEC_EINVAL;
    kfec::DeviceInfo di;
    int rc = probe_device(di);
    if (rc) return rc;
    kfec_ctx *c = new (std::nothrow) kfec_ctx;
    if (!c) return KFEC_ENOMEM;
    c->di = di;
    {
        // counted before the matrix exists, so that a concurrent destroy of the device's last other coder does
        // not release the cached matrices under this one
        std::lock_guard<std::mutex> lk(g_live_mu);
        ++g_live[di.device];
        c->counted = true;
    }
    rc = set_matrix(c, K, N);
    if (rc) {
        kfec_destroy(c);
        return rc;
    }
    *out = c;
    return KFEC_OK;
}

int kfec_reset(kfec_ctx *ctx, size_t K, size_t N)
{
    if (!ctx || !kn_valid(K, N)) return KFEC_EINVAL;  // reference throws before touching its state
    std::lock_guard<std::mutex> lk(ctx->mu);
    if (set_dev(ctx)) return KFEC_EHIP;
    return set_matrix(ctx, K, N);
}

void kfec_destroy(kfec_ctx *ctx)
{
    if (!ctx) return;
    const int dev = ctx->di.device;
    (void)hipSetDevice(dev);
    // The frees below (launch-path staging only) wait for every stream of the device, so the device's last
    // coder stops the resident workers first; otherwise a worker's lease (kfec_worker.hip) bounds the wait.
    bool last = false;
    if (ctx->counted) {
        std::lock_guard<std::mutex> lk(g_live_mu);
        last = --g_live[dev] == 0;
        if (last) kfec::worker_stop(dev);
    }
    if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
    if (ctx->d_stage) (void)hipFree(ctx->d_stage);
    if (ctx->h_stage) (void)hipHostFree(ctx->h_stage);
    if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
    unref_matrix(dev, ctx->mat);  // (the device's last coder then releases every cached matrix below)
    delete ctx;
    if (last) {
        std::lock_guard<std::mutex> lk(g_live_mu);
        if (g_live[dev] == 0) release_matrices(dev);  // (unless a coder was created meanwhile)
    }
}

size_t kfec_get_K(const kfec_ctx *ctx) { return ctx ? ctx->K : 0; }
size_t kfec_get_N(const kfec_ctx *ctx) { return ctx ? ctx->N : 0; }

int kfec_enc_matrix(const kfec_ctx *ctx, uint8_t *enc)
{
    if (!ctx || !enc) return KFEC_EINVAL;
    std::memcpy(enc, ctx->h_enc, ctx->N * ctx->K);
    return KFEC_OK;
}

int kfec_encode(const kfec_ctx *cctx, const uint8_t *input, size_t data_length, size_t block_size,
                uint8_t *parity_out)
{
    kfec_ctx *ctx = const_cast<kfec_ctx *>(cctx);
    if (!ctx) return KFEC_EINVAL;
    const size_t K = ctx->K, N = ctx->N, R = N - K, B = block_size;
    // fecpp.cpp:497-498; plus the cases where the reference is undefined (B = 0, short input)
    if (input == nullptr || B == 0 || (data_length / B) % K != 0 || data_length < K * B) return KFEC_EMPTY;
    if (R == 0) return KFEC_OK;
    if (!parity_out) return KFEC_EINVAL;
    if (kfec::worker_enabled()) {
        // resident worker: no launch and no stream synchronisation per call (kfec_worker.hip)
        if (set_dev(ctx)) return KFEC_EHIP;
        const int wr = kfec::worker_encode(ctx->di.device, ctx->d_enc, ctx->mat_id, (int)K, (int)N, B, input, parity_out);
        if (wr <= 0) return wr;  // 1: shape the worker does not take
    }
    std::lock_guard<std::mutex> lk(ctx->mu);
    if (set_dev(ctx)) return KFEC_EHIP;
    const size_t off_par = al256(K * B);
    if (ensure_stream(ctx)) return KFEC_EHIP;
    int rc = ensure_stage(ctx, off_par + al256(R * B));
    if (rc) return rc;
    if (zero_copy()) {
        rc = ensure_host_stage(ctx, off_par + al256(R * B));
        if (rc) return rc;
        uint8_t *h_data = ctx->h_stage, *h_par = ctx->h_stage + off_par;
        std::memcpy(h_data, input, K * B);
        if (kfec::launch_encode(ctx->di, ctx->d_enc, (int)K, (int)N, 1, B, B, h_data, h_par, ctx->stream))
            return KFEC_EHIP;
        if (hipStreamSynchronize(ctx->stream) != hipSuccess) return KFEC_EHIP;
        std::memcpy(parity_out, h_par, R * B);
        return KFEC_OK;
    }
    uint8_t *d_data = ctx->d_stage, *d_par = ctx->d_stage + off_par;
    if (hipMemcpyAsync(d_data, input, K * B, hipMemcpyHostToDevice, ctx->stream) != hipSuccess) return KFEC_EHIP;
    rc = kfec::launch_encode(ctx->di, ctx->d_enc, (int)K, (int)N, 1, B, B, d_data, d_par, ctx->stream);
    if (rc) return KFEC_EHIP;
    if (hipMemcpyAsync(parity_out, d_par, R * B, hipMemcpyDeviceToHost, ctx->stream) != hipSuccess) return KFEC_EHIP;
    if (hipStreamSynchronize(ctx->stream) != hipSuccess) return KFEC_EHIP;
    return KFEC_OK;
}

int kfec_decode(const kfec_ctx *cctx, const size_t *share_ids, const uint8_t *const *share_ptrs, size_t n_shares,
                size_t share_size, size_t *out_ids, uint8_t *out, size_t *n_out)
{
    kfec_ctx *ctx = const_cast<kfec_ctx *>(cctx);
    if (!ctx || !n_out) return KFEC_EINVAL;
    *n_out = 0;
    const size_t K = ctx->K, N = ctx->N, R = N - K, B = share_size;
    if (n_shares < K) return KFEC_EMPTY;  // fecpp.cpp:520-521
    if (!share_ids || !share_ptrs) return KFEC_EINVAL;
    for (size_t i = 1; i < n_shares; ++i)
        if (share_ids[i] <= share_ids[i - 1]) return KFEC_EINVAL;  // must be a std::map's key order
    // fecpp.cpp:550-551: a chosen id >= N returns {}.  Ids >= N are the highest ids, so they are chosen
    // first whenever a data share is missing; with none missing the reference returns {} anyway.
    if (n_shares && share_ids[n_shares - 1] >= N) return KFEC_EMPTY;
    if (B == 0) {
        // nothing to compute, but the reference still returns one (empty) block per missing data row
        // (fecpp.cpp:572-583): the data ids below K that are not among the shares, ascending
        size_t m = 0, i = 0;
        for (size_t d = 0; d < K; ++d) {
            while (i < n_shares && share_ids[i] < d) ++i;
            if (i < n_shares && share_ids[i] == d) continue;
            if (!out_ids) return KFEC_EINVAL;
            out_ids[m++] = d;
        }
        *n_out = m;
        return KFEC_OK;
    }
    if (kfec::worker_enabled()) {
        // The reference's share selection (fecpp.cpp:528-548) as bookkeeping on the ids: row i takes data
        // share i when present, otherwise the highest id not used yet; the worker does all the arithmetic.
        const uint8_t *row_ptr[256];
        uint8_t M[256], P[256];
        size_t m = 0, lo = 0, hi = n_shares;
        for (size_t i = 0; i < K; ++i) {
            if (lo < n_shares && share_ids[lo] == i) {
                row_ptr[i] = share_ptrs[lo++];
            } else {
                --hi;
                row_ptr[i] = share_ptrs[hi];
                M[m] = (uint8_t)i;
                P[m] = (uint8_t)share_ids[hi];
                ++m;
            }
        }
        if (m == 0) return KFEC_OK;  // every data share present: the reference's empty map
        if (!out || !out_ids) return KFEC_EINVAL;
        if (set_dev(ctx)) return KFEC_EHIP;
        const int wr = kfec::worker_decode(ctx->di.device, ctx->d_enc, ctx->h_enc, ctx->mat_id, (int)K, (int)N, B, row_ptr, (int)m,
                                           M, P, out);
        if (wr == 0) {
            for (size_t t = 0; t < m; ++t) out_ids[t] = M[t];
            *n_out = m;
            return KFEC_OK;
        }
        if (wr < 0) return wr;
    }
    std::lock_guard<std::mutex> lk(ctx->mu);
    if (set_dev(ctx)) return KFEC_EHIP;
    const size_t o_data = 0, o_par = al256(K * B), o_out = o_par + al256(R * B), o_mask = o_out + al256(R * B);
    const size_t o_idx = o_mask + 256, o_st = o_idx + al256(R + 1), o_rec = o_st + 256,
                 total = o_rec + al256(kfec::decode_workspace_bytes(1, K, R));
    if (ensure_stream(ctx)) return KFEC_EHIP;
    int rc = ensure_stage(ctx, total);
    if (rc) return rc;
    if (zero_copy()) {
        rc = ensure_host_stage(ctx, o_rec);
        if (rc) return rc;
        uint8_t *h = ctx->h_stage;
        uint64_t *mask = reinterpret_cast<uint64_t *>(h + o_mask);
        mask[0] = mask[1] = mask[2] = mask[3] = 0;
        for (size_t i = 0; i < n_shares; ++i) {
            const size_t s = share_ids[i];
            mask[s >> 6] |= 1ull << (s & 63);
            std::memcpy((s < K) ? h + o_data + s * B : h + o_par + (s - K) * B, share_ptrs[i], B);
        }
        rc = kfec::launch_decode(ctx->di, ctx->d_enc, (int)K, (int)N, 1, B, B, h + o_data, h + o_par, mask, h + o_out,
                                 h + o_idx, h + o_st, ctx->d_stage + o_rec, ctx->stream);
        if (rc) return KFEC_EHIP;
        if (hipStreamSynchronize(ctx->stream) != hipSuccess) return KFEC_EHIP;
        const uint8_t st = h[o_st];
        if (st == KFEC_GROUP_EMPTY) return KFEC_EMPTY;
        if (st == KFEC_GROUP_SINGULAR) return KFEC_ESINGULAR;
        size_t m = 0;
        while (m < R && h[o_idx + m] != 0xFF) ++m;
        if (m) {
            if (!out || !out_ids) return KFEC_EINVAL;
            std::memcpy(out, h + o_out, m * B);
            for (size_t t = 0; t < m; ++t) out_ids[t] = h[o_idx + t];
        }
        *n_out = m;
        return KFEC_OK;
    }
    uint8_t *base = ctx->d_stage;
    uint64_t mask[4] = {0, 0, 0, 0};
    for (size_t i = 0; i < n_shares; ++i) {
        const size_t s = share_ids[i];
        mask[s >> 6] |= 1ull << (s & 63);
        uint8_t *dst = (s < K) ? base + o_data + s * B : base + o_par + (s - K) * B;
        if (hipMemcpyAsync(dst, share_ptrs[i], B, hipMemcpyHostToDevice, ctx->stream) != hipSuccess) return KFEC_EHIP;
    }
    if (hipMemcpyAsync(base + o_mask, mask, sizeof(mask), hipMemcpyHostToDevice, ctx->stream) != hipSuccess)
        return KFEC_EHIP;
    rc = kfec::launch_decode(ctx->di, ctx->d_enc, (int)K, (int)N, 1, B, B, base + o_data, base + o_par,
                             reinterpret_cast<const uint64_t *>(base + o_mask), base + o_out, base + o_idx,
                             base + o_st, base + o_rec, ctx->stream);
    if (rc) return KFEC_EHIP;
    uint8_t idx[256], st = 0;
    if (R && hipMemcpyAsync(idx, base + o_idx, R, hipMemcpyDeviceToHost, ctx->stream) != hipSuccess) return KFEC_EHIP;
    if (hipMemcpyAsync(&st, base + o_st, 1, hipMemcpyDeviceToHost, ctx->stream) != hipSuccess) return KFEC_EHIP;
    if (hipStreamSynchronize(ctx->stream) != hipSuccess) return KFEC_EHIP;
    if (st == KFEC_GROUP_EMPTY) return KFEC_EMPTY;
    if (st == KFEC_GROUP_SINGULAR) return KFEC_ESINGULAR;
    size_t m = 0;
    while (m < R && idx[m] != 0xFF) ++m;
    if (m) {
        if (!out || !out_ids) return KFEC_EINVAL;
        if (hipMemcpyAsync(out, base + o_out, m * B, hipMemcpyDeviceToHost, ctx->stream) != hipSuccess)
            return KFEC_EHIP;
        if (hipStreamSynchronize(ctx->stream) != hipSuccess) return KFEC_EHIP;
        for (size_t t = 0; t < m; ++t) out_ids[t] = idx[t];
    }
    *n_out = m;
    return KFEC_OK;
}

int kfec_encode_batch(const kfec_ctx *ctx, size_t G, size_t B, size_t pitch, const void *d_data, void *d_parity,
                      void *stream)
{
    if (!ctx || pitch < B || (G && (!d_data || (!d_parity && ctx->N > ctx->K)))) return KFEC_EINVAL;
    if (set_dev(ctx)) return KFEC_EHIP;
    return kfec::launch_encode(ctx->di, ctx->d_enc, (int)ctx->K, (int)ctx->N, G, B, pitch, d_data, d_parity,
                               as_stream(stream))
               ? KFEC_EHIP
               : KFEC_OK;
}

size_t kfec_decode_workspace_size(const kfec_ctx *ctx, size_t G)
{
    return ctx ? kfec::decode_workspace_bytes(G, ctx->K, ctx->N - ctx->K) : 0;
}

int kfec_decode_batch(const kfec_ctx *ctx, size_t G, size_t B, size_t pitch, const void *d_data,
                      const void *d_parity, const uint64_t *d_present, void *d_out, uint8_t *d_out_idx,
                      uint8_t *d_status, void *d_workspace, void *stream)
{
    if (!ctx || pitch < B) return KFEC_EINVAL;
    if (G && (!d_present || !d_status || !d_workspace || !d_data)) return KFEC_EINVAL;
    if (G && ctx->N > ctx->K && (!d_parity || !d_out || !d_out_idx)) return KFEC_EINVAL;
    if (set_dev(ctx)) return KFEC_EHIP;
    return kfec::launch_decode(ctx->di, ctx->d_enc, (int)ctx->K, (int)ctx->N, G, B, pitch, d_data, d_parity,
                               d_present, d_out, d_out_idx, d_status, d_workspace, as_stream(stream))
               ? KFEC_EHIP
               : KFEC_OK;
}

int kfec_synth(const kfec_ctx *ctx, uint64_t seed, size_t g0, size_t G, size_t s0, size_t ns, size_t B, size_t pitch,
               void *d_out, void *stream)
{
    if (!ctx || pitch < B || (G && ns && !d_out)) return KFEC_EINVAL;
    if (set_dev(ctx)) return KFEC_EHIP;
    return kfec::launch_synth(seed, (int)ctx->N, g0, G, s0, ns, B, pitch, d_out, as_stream(stream)) ? KFEC_EHIP
                                                                                                     : KFEC_OK;
}

int kfec_erasure_masks(const kfec_ctx *ctx, uint64_t seed, size_t g0, size_t G, size_t pool, size_t count_max,
                       int random_count, uint64_t *d_present, void *stream)
{
    if (!ctx || pool > ctx->N || (G && !d_present)) return KFEC_EINVAL;
    if (set_dev(ctx)) return KFEC_EHIP;
    return kfec::launch_erasure_masks(seed, (int)ctx->N, g0, G, pool, count_max, random_count, d_present,
                                      as_stream(stream))
               ? KFEC_EHIP
               : KFEC_OK;
}

int kfec_verify_recovered(const kfec_ctx *ctx, size_t G, size_t B, size_t pitch, const void *d_data,
                          const void *d_out, const uint8_t *d_out_idx, uint64_t *d_mismatch, void *stream)
{
    if (!ctx || pitch < B || !d_mismatch) return KFEC_EINVAL;
    if (set_dev(ctx)) return KFEC_EHIP;
    return kfec::launch_verify((int)ctx->K, (int)ctx->N, G, B, pitch, d_data, d_out, d_out_idx, d_mismatch,
                               as_stream(stream))
               ? KFEC_EHIP
               : KFEC_OK;
}


// ---- framing and wire layer (include/kfec_frame.h) ---------------------------------------------------
static bool al4(const void *p) { return (reinterpret_cast<uintptr_t>(p) & 3u) == 0; }

int kfec_frame_data_batch(const kfec_ctx *ctx, size_t G, const void *d_src, size_t src_bytes, const uint64_t *d_off,
                          const uint16_t *d_len, size_t B, size_t pitch, void *d_data, uint16_t *d_align, void *stream)
{
    if (!ctx || pitch < B || pitch % 4 || B > 0xFFFF) return KFEC_EINVAL;
    if (G && (!d_src || !al4(d_src) || !d_off || !d_len || !d_data || !al4(d_data) || !d_align)) return KFEC_EINVAL;
    if (set_dev(ctx)) return KFEC_EHIP;
    return kfec::launch_frame((int)ctx->K, (int)ctx->N, false, G, d_src, src_bytes, d_off, d_len, nullptr, B, pitch,
                              d_data, nullptr, d_align, as_stream(stream))
               ? KFEC_EHIP
               : KFEC_OK;
}

int kfec_encode_framed_batch(const kfec_ctx *ctx, size_t G, const void *d_src, size_t src_bytes,
                             const uint64_t *d_off, const uint16_t *d_len, size_t B, size_t pitch, void *d_parity,
                             uint16_t *d_align, void *stream)
{
    if (!ctx || pitch < B || pitch % 4 || B > 0xFFFF) return KFEC_EINVAL;
    if (G && (!d_src || !al4(d_src) || !d_off || !d_len || !d_align)) return KFEC_EINVAL;
    if (G && ctx->N > ctx->K && (!d_parity || !al4(d_parity))) return KFEC_EINVAL;
    if (set_dev(ctx)) return KFEC_EHIP;
    const int rc = kfec::launch_framed_encode(ctx->d_enc, (int)ctx->K, (int)ctx->N, G, d_src, src_bytes, d_off, d_len,
                                              B, pitch, d_parity, d_align, as_stream(stream));
    if (rc < 0) return KFEC_EHIP;
    if (rc == 0) return KFEC_OK;
    // shapes the fused kernel does not take (tiny slots with many groups per workgroup, R = 0, huge batches):
    // frame into a scratch slot array, then encode
    if (ctx->N == ctx->K) {
        return kfec::launch_frame((int)ctx->K, (int)ctx->N, false, G, d_src, src_bytes, d_off, d_len, nullptr, B, pitch,
                                  nullptr, nullptr, d_align, as_stream(stream)) == 0 ? KFEC_OK : KFEC_EHIP;
    }
    void *slots = nullptr;
    if (hipMallocAsync(&slots, G * ctx->K * pitch, as_stream(stream)) != hipSuccess) return KFEC_ENOMEM;
    int r = kfec::launch_frame((int)ctx->K, (int)ctx->N, false, G, d_src, src_bytes, d_off, d_len, nullptr, B, pitch,
                               slots, nullptr, d_align, as_stream(stream));
    if (!r) r = kfec::launch_encode(ctx->di, ctx->d_enc, (int)ctx->K, (int)ctx->N, G, B, pitch, slots, d_parity,
                                    as_stream(stream));
    (void)hipFreeAsync(slots, as_stream(stream));
    return r ? KFEC_EHIP : KFEC_OK;
}

int kfec_frame_shards_batch(const kfec_ctx *ctx, size_t G, const void *d_src, size_t src_bytes,
                            const uint64_t *d_off, const uint16_t *d_len, const uint64_t *d_present, size_t B,
                            size_t pitch, void *d_data, void *d_parity, uint16_t *d_align, void *stream)
{
    if (!ctx || pitch < B || pitch % 4 || B > 0xFFFF) return KFEC_EINVAL;
    if (G && (!d_src || !al4(d_src) || !d_off || !d_len || !d_present || !d_data || !al4(d_data) || !d_align))
        return KFEC_EINVAL;
    if (G && ctx->N > ctx->K && (!d_parity || !al4(d_parity))) return KFEC_EINVAL;
    if (set_dev(ctx)) return KFEC_EHIP;
    return kfec::launch_frame((int)ctx->K, (int)ctx->N, true, G, d_src, src_bytes, d_off, d_len, d_present, B, pitch,
                              d_data, d_parity, d_align, as_stream(stream))
               ? KFEC_EHIP
               : KFEC_OK;
}

int kfec_decode_framed_batch(const kfec_ctx *ctx, size_t G, const void *d_src, size_t src_bytes,
                             const uint64_t *d_off, const uint16_t *d_len, const uint64_t *d_present, size_t B,
                             size_t pitch, void *d_out, uint8_t *d_out_idx, uint8_t *d_status, uint16_t *d_align,
                             void *d_workspace, void *stream)
{
    if (!ctx || pitch < B || pitch % 4 || B > 0xFFFF) return KFEC_EINVAL;
    if (G && (!d_src || !al4(d_src) || !d_off || !d_len || !d_present || !d_status || !d_workspace || !d_align))
        return KFEC_EINVAL;
    if (G && ctx->N > ctx->K && (!d_out || !al4(d_out) || !d_out_idx)) return KFEC_EINVAL;
    if (set_dev(ctx)) return KFEC_EHIP;
    const hipStream_t s = as_stream(stream);
    const int rc = kfec::launch_framed_decode(ctx->di, ctx->d_enc, (int)ctx->K, (int)ctx->N, G, d_src, src_bytes, d_off,
                                              d_len, d_present, B, pitch, d_out, d_out_idx, d_status, d_align,
                                              d_workspace, s);
    if (rc < 0) return KFEC_EHIP;
    if (rc == 0) return KFEC_OK;
    // shapes the fused kernel does not take (R = 0, K x row tile too large for its LDS staging, huge batches):
    // frame into scratch shard arrays, then decode
    const size_t R = ctx->N - ctx->K;
    void *data = nullptr, *par = nullptr;
    if (hipMallocAsync(&data, std::max<size_t>(G * ctx->K * pitch, 4), s) != hipSuccess) return KFEC_ENOMEM;
    if (hipMallocAsync(&par, std::max<size_t>(G * R * pitch, 4), s) != hipSuccess) {
        (void)hipFreeAsync(data, s);
        return KFEC_ENOMEM;
    }
    int r = kfec::launch_frame((int)ctx->K, (int)ctx->N, true, G, d_src, src_bytes, d_off, d_len, d_present, B, pitch,
                               data, par, d_align, s);
    if (!r) r = kfec::launch_decode(ctx->di, ctx->d_enc, (int)ctx->K, (int)ctx->N, G, B, pitch, data, par, d_present,
                                    d_out, d_out_idx, d_status, d_workspace, s);
    (void)hipFreeAsync(data, s);
    (void)hipFreeAsync(par, s);
    return r ? KFEC_EHIP : KFEC_OK;
}

int kfec_unframe_batch(const kfec_ctx *ctx, size_t G, size_t B, size_t pitch, const void *d_out,
                       const uint8_t *d_out_idx, uint16_t *d_rec_len, void *d_dst, size_t dst_pitch, void *stream)
{
    if (!ctx || pitch < B || pitch % 4 || B < KFEC_FEC_CONTAINER_HEADER || B > 0xFFFF) return KFEC_EINVAL;
    if (d_dst && (dst_pitch % 4 || dst_pitch + KFEC_FEC_CONTAINER_HEADER < B || !al4(d_dst))) return KFEC_EINVAL;
    if (G && ctx->N > ctx->K && (!d_out || !al4(d_out) || !d_out_idx || !d_rec_len)) return KFEC_EINVAL;
    if (set_dev(ctx)) return KFEC_EHIP;
    return kfec::launch_unframe((int)ctx->K, (int)ctx->N, G, B, pitch, d_out, d_out_idx, d_rec_len, d_dst, dst_pitch,
                                as_stream(stream))
               ? KFEC_EHIP
               : KFEC_OK;
}

int kfec_pack_batch(const kfec_ctx *ctx, size_t G, unsigned which, const void *d_src, size_t src_bytes,
                    const uint64_t *d_off, const uint16_t *d_len, size_t pitch, const void *d_parity,
                    const uint16_t *d_align, const uint32_t *d_sn, const uint32_t *d_conv, uint32_t timestamp,
                    void *d_pkt, size_t pkt_pitch, uint16_t *d_pkt_len, void *stream)
{
    if (!ctx || pkt_pitch % 4 || (which & ~(KFEC_PACK_DATA | KFEC_PACK_REDUNDANT | KFEC_PACK_COMPACT))) return KFEC_EINVAL;
    if (G && (!d_sn || !d_pkt || !al4(d_pkt) || !d_pkt_len)) return KFEC_EINVAL;
    if (G && (which & KFEC_PACK_DATA) && (!d_src || !al4(d_src) || !d_off || !d_len)) return KFEC_EINVAL;
    if (G && (which & KFEC_PACK_REDUNDANT) && ctx->N > ctx->K &&
        (!d_parity || !al4(d_parity) || pitch % 4 || !d_align || !d_conv))
        return KFEC_EINVAL;
    if (set_dev(ctx)) return KFEC_EHIP;
    return kfec::launch_pack((int)ctx->K, (int)ctx->N, G, which, d_src, src_bytes, d_off, d_len, pitch, d_parity,
                             d_align, d_sn, d_conv, timestamp, d_pkt, pkt_pitch, d_pkt_len, as_stream(stream))
               ? KFEC_EHIP
               : KFEC_OK;
}

int kfec_encode_pack_batch(const kfec_ctx *ctx, size_t G, const void *d_src, size_t src_bytes, const uint64_t *d_off,
                           const uint16_t *d_len, size_t B, size_t pitch, void *d_parity, uint16_t *d_align,
                           const uint32_t *d_sn, const uint32_t *d_conv, uint32_t timestamp, void *d_pkt,
                           size_t pkt_pitch, uint16_t *d_pkt_len, void *stream)
{
    if (!ctx || pitch < B || pitch % 4 || B > 0xFFFF || pkt_pitch % 4) return KFEC_EINVAL;
    if (G && (!d_src || !al4(d_src) || !d_off || !d_len || !d_align || !d_sn || !d_pkt || !al4(d_pkt) || !d_pkt_len))
        return KFEC_EINVAL;
    if (G && ctx->N > ctx->K && (!d_parity || !al4(d_parity) || !d_conv)) return KFEC_EINVAL;
    if (set_dev(ctx)) return KFEC_EHIP;
    const hipStream_t s = as_stream(stream);
    const kfec::DataPackets dp{d_pkt, d_pkt_len, d_sn, pkt_pitch, timestamp};
    const int rc = kfec::launch_framed_encode(ctx->d_enc, (int)ctx->K, (int)ctx->N, G, d_src, src_bytes, d_off, d_len,
                                              B, pitch, d_parity, d_align, s, &dp);
    if (rc < 0) return KFEC_EHIP;
    if (rc == 0)  // data packets came out of the encoder; the redundant ones from the parity it wrote
        return kfec::launch_pack((int)ctx->K, (int)ctx->N, G, KFEC_PACK_REDUNDANT, d_src, src_bytes, d_off, d_len, pitch,
                                 d_parity, d_align, d_sn, d_conv, timestamp, d_pkt, pkt_pitch, d_pkt_len, s)
                   ? KFEC_EHIP
                   : KFEC_OK;
    // shapes the fused kernel does not take: the framed encode (with its own fallback), then both packet kinds
    const int r = kfec_encode_framed_batch(ctx, G, d_src, src_bytes, d_off, d_len, B, pitch, d_parity, d_align, stream);
    if (r) return r;
    return kfec::launch_pack((int)ctx->K, (int)ctx->N, G, KFEC_PACK_DATA | KFEC_PACK_REDUNDANT, d_src, src_bytes, d_off,
                             d_len, pitch, d_parity, d_align, d_sn, d_conv, timestamp, d_pkt, pkt_pitch, d_pkt_len, s)
               ? KFEC_EHIP
               : KFEC_OK;
}

int kfec_unpack_batch(const kfec_ctx *ctx, size_t P, const void *d_src, size_t src_bytes, const uint64_t *d_off,
                      const uint32_t *d_len, kfec_pkt_hdr *d_hdr, void *stream)
{
    (void)src_bytes;
    if (!ctx || (P && (!d_src || !d_off || !d_len || !d_hdr))) return KFEC_EINVAL;
    if (set_dev(ctx)) return KFEC_EHIP;
    return kfec::launch_unpack((int)ctx->K, P, d_src, d_off, d_len, d_hdr, as_stream(stream)) ? KFEC_EHIP : KFEC_OK;
}

int kfec_group_scatter(const kfec_ctx *ctx, size_t P, const kfec_pkt_hdr *d_hdr, const int32_t *d_slot,
                       uint32_t sn_base, size_t G, uint64_t *d_present, uint64_t *d_off, uint16_t *d_len,
                       void *stream)
{
    if (!ctx || (P && (!d_hdr || !d_present || !d_off || !d_len))) return KFEC_EINVAL;
    if (set_dev(ctx)) return KFEC_EHIP;
    return kfec::launch_scatter((int)ctx->N, P, d_hdr, d_slot, sn_base, G, d_present, d_off, d_len,
                                as_stream(stream))
               ? KFEC_EHIP
               : KFEC_OK;
}

int kfec_seal_batch(int mode, size_t P, const void *d_src, size_t src_bytes, const uint64_t *d_off,
                    const uint32_t *d_len, void *d_dst, size_t dst_pitch, uint32_t *d_out_len, void *stream)
{
    if (mode != KFEC_SEAL_CHECKSUM && mode != KFEC_SEAL_PLAIN_XOR) return KFEC_EINVAL;
    if (d_dst ? dst_pitch % 4 != 0 : dst_pitch == 0) return KFEC_EINVAL;  // in place: dst_pitch = slot size
    if (!d_dst && mode != KFEC_SEAL_CHECKSUM) return KFEC_EINVAL;  // in place: checksum mode only
    if (P && (!d_src || !al4(d_src) || !d_off || !d_len || (d_dst && !al4(d_dst)) || !d_out_len)) return KFEC_EINVAL;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return KFEC_ENODEV;
    return kfec::launch_seal(false, mode, P, d_src, src_bytes, d_off, d_len, d_dst, dst_pitch, d_out_len, nullptr,
                             as_stream(stream))
               ? KFEC_EHIP
               : KFEC_OK;
}

int kfec_open_batch(int mode, size_t P, const void *d_src, size_t src_bytes, const uint64_t *d_off,
                    const uint32_t *d_len, void *d_dst, size_t dst_pitch, uint32_t *d_out_len, uint8_t *d_ok,
                    void *stream)
{
    if ((mode != KFEC_SEAL_CHECKSUM && mode != KFEC_SEAL_PLAIN_XOR) || dst_pitch % 4) return KFEC_EINVAL;
    if (!d_dst && mode != KFEC_SEAL_CHECKSUM) return KFEC_EINVAL;  // in place: checksum mode only
    if (P && (!d_src || !al4(d_src) || !d_off || !d_len || (d_dst && !al4(d_dst)) || !d_out_len || !d_ok))
        return KFEC_EINVAL;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return KFEC_ENODEV;
    return kfec::launch_seal(true, mode, P, d_src, src_bytes, d_off, d_len, d_dst, dst_pitch, d_out_len, d_ok,
                             as_stream(stream))
               ? KFEC_EHIP
               : KFEC_OK;
}

}  // extern "C"
