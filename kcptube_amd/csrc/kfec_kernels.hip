// kfec_kernels.hip -- hand-written gfx950 (CDNA4) kernels of the kfec Reed-Solomon coder.
//
// Reference semantics (all /root/reference/src/3rd_party/):
//   matrix   fecpp.cpp:368-415, 453-490   enc = [I_K ; Vbot * Vtop^-1]  (build_matrix_kernel)
//   encode   fecpp.cpp:495-513            parity_r = XOR_j enc[K+r][j] * D_j   (mac_kernel<.., false>)
//   decode   fecpp.cpp:518-587            share selection + K x K inverse + m output rows
//                                           (decode_prep_* + mac_kernel<.., true>)
//   addmul   fecpp.cpp:170-223, fecpp_ssse3.cpp:541-575   z ^= c * x  (the "perm MAC" below)
//
// Design (DESIGN.md has the numbers):
// * perm MAC.  c * x for a constant c is linear over GF(2), so c*x = c*(x & 7) ^ c*(x & 0x38) ^ c*(x & 0xC0).
//   Each term is an 8- or 4-entry table lookup, and v_perm_b32 does 4 such byte lookups (one per byte of a
//   dword) in one VALU op.  Per data dword and coefficient: 3 v_perm_b32 + XORs; the 3 selector extractions
//   are shared by all coefficients of a data dword.  No LDS traffic per data byte and no bank conflicts:
//   the ~5 table dwords per coefficient are read once per shard per lane (LDS broadcast reads).
// * Flattened work: one lane = one (group, V-byte column) item; consecutive lanes take consecutive columns
//   (coalesced 1 KiB per wave-instruction at V = 16), wrapping into the next group.  Persistent grid-stride
//   over items.  A workgroup iteration touches <= GMAX groups, whose per-group decode tables are expanded
//   into LDS at the start of the iteration.
// * Decode coefficients: per group only the m x m sub-system of the missing rows is inverted (Gauss-Jordan
//   with LDS log/antilog tables); the rest of the K x K inverse follows by one product.  The inverse is
//   unique, so the coefficients equal the reference's K x K Gauss-Jordan result bit for bit.
#include "kfec_gf.hpp"
#include "kfec_internal.hpp"

#include <algorithm>
#include <cstdlib>
#include <string>

namespace kfec {

__constant__ GfTables c_gf = make_gf_tables();

// set by the stream engine if a bounded spin ever times out (read by kfec_engine_error)
__device__ uint32_t g_engine_err;

static uint32_t *g_err_word()
{
    static uint32_t *p[64] = {};
    int dev = 0;
    (void)hipGetDevice(&dev);
    dev &= 63;
    if (!p[dev]) (void)hipGetSymbolAddress(reinterpret_cast<void **>(&p[dev]), HIP_SYMBOL(g_engine_err));
    return p[dev];
}

uint32_t engine_error_word()
{
    uint32_t v = 0;
    (void)hipMemcpyFromSymbol(&v, HIP_SYMBOL(g_engine_err), sizeof(v));
    return v;
}

static constexpr int kBlock = 256;
#ifndef KFEC_MAC_BLOCK
#define KFEC_MAC_BLOCK 256
#endif
static constexpr int kMacBlock = KFEC_MAC_BLOCK;  // workgroup of the flattened MAC kernel

// build-time tuning knobs (tools/ab.py builds variants; the shipped library uses the defaults)
#ifndef KFEC_PD
#define KFEC_PD 4
#endif
#ifndef KFEC_ABLATE
#define KFEC_ABLATE 0
#endif
#ifndef KFEC_VEC32
#define KFEC_VEC32 1  // 32-byte lane granules in the flattened kernel (2 KiB per wave-instruction pair)
#endif
#ifndef KFEC_MINW
#define KFEC_MINW 1  // __launch_bounds__ minimum waves per SIMD of the flattened kernel
#endif
#ifndef KFEC_SGPR_TABLES
#define KFEC_SGPR_TABLES 0  // encode reads its perm tables with scalar loads instead of LDS (KFEC_SGPR_TABLES env)
#endif
#ifndef KFEC_XCD_REMAP
#define KFEC_XCD_REMAP 0  // XCD-contiguous workgroup numbering in the flattened kernel (A/B knob)
#endif
#ifndef KFEC_NTSTORE
#define KFEC_NTSTORE 1  // nontemporal output stores in the flattened kernel (+2.5% encode, measured)
#endif

// ---------------------------------------------------------------------------------------------------
// small device helpers
// ---------------------------------------------------------------------------------------------------
__device__ __forceinline__ void stage_gf(uint8_t *s_exp, uint8_t *s_log)
{
    for (int i = threadIdx.x; i < 512; i += blockDim.x) s_exp[i] = c_gf.exp[i];
    for (int i = threadIdx.x; i < 256; i += blockDim.x) s_log[i] = c_gf.log[i];
}

__device__ __forceinline__ uint32_t gmul(const uint8_t *e, const uint8_t *l, uint32_t a, uint32_t b)
{
    return (a && b) ? e[l[a] + l[b]] : 0u;
}

__device__ __forceinline__ uint32_t ginv(const uint8_t *e, const uint8_t *l, uint32_t a)
{
    return a ? e[255 - l[a]] : 0u;
}

__device__ __forceinline__ uint64_t splitmix64(uint64_t x)
{
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

// mask word q of a present bitmap to ids < n
__device__ __forceinline__ uint64_t bits_below(int n, int q)
{
    const int v = n - 64 * q;
    return v <= 0 ? 0ull : (v >= 64 ? ~0ull : ((1ull << v) - 1ull));
}

// ---------------------------------------------------------------------------------------------------
// (A6) encoding matrix: Lagrange closed form of Vbot * Vtop^-1.
// Evaluation points x_0 = 0, x_i = alpha^i (i >= 1) -- the rows of the reference's Vandermonde matrix
// (fecpp.cpp:401 uses p_0 = 0, p_row = GF_EXP[row]; fecpp.cpp:467 alpha^(row*col)).  Systematic row r >= K,
// column j:  enc[r][j] = L_j(x_r) = prod_{i<K, i!=j} (x_r ^ x_i) / (x_j ^ x_i), summed in the log domain.
// ---------------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(kBlock) build_matrix_kernel(uint8_t *enc, int K, int N)
{
    __shared__ uint8_t s_exp[512], s_log[256];
    stage_gf(s_exp, s_log);
    __syncthreads();
    const int idx = blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= N * K) return;
    const int r = idx / K, j = idx - r * K;
    if (r < K) {
        enc[idx] = (r == j) ? 1 : 0;
        return;
    }
    const uint32_t xr = s_exp[r], xj = (j == 0) ? 0u : s_exp[j];  // r >= 1 here; s_exp[255] == 1
    uint32_t ln = 0, ld = 0;
    for (int i = 0; i < K; ++i) {
        if (i == j) continue;
        const uint32_t xi = (i == 0) ? 0u : s_exp[i];
        ln += s_log[xr ^ xi];
        ld += s_log[xj ^ xi];
    }
    int e = (int)(ln % 255u) - (int)(ld % 255u);
    if (e < 0) e += 255;
    enc[idx] = s_exp[e];
}

// perm-MAC tables of the parity rows for the encode kernel: etab[j][r][0..5) = gf_perm_tables(enc[K + r][j])
// (zero for the slack rows r >= R)
__global__ void __launch_bounds__(kBlock) build_enc_tables_kernel(const uint8_t *enc, int K, int N, uint32_t *etab)
{
    const int R = N - K, rows = (int)enc_tab_rows(R);
    const int idx = blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= K * rows) return;
    const int j = idx / rows, r = idx - j * rows;
    uint32_t t[5];
    gf_perm_tables(r < R ? enc[(K + r) * K + j] : 0u, t);
#pragma unroll
    for (int i = 0; i < 5; ++i) etab[(size_t)idx * 5 + i] = t[i];
}

int launch_build_matrix(uint8_t *d_enc, int K, int N, hipStream_t s)
{
    const int total = N * K;
    hipLaunchKernelGGL(build_matrix_kernel, dim3((total + kBlock - 1) / kBlock), dim3(kBlock), 0, s, d_enc, K, N);
    if (hipGetLastError() != hipSuccess) return -3;
    const int nt = K * (int)enc_tab_rows(N - K);
    uint32_t *etab = reinterpret_cast<uint32_t *>(d_enc + enc_tab_offset(K, N));
    hipLaunchKernelGGL(build_enc_tables_kernel, dim3((nt + kBlock - 1) / kBlock), dim3(kBlock), 0, s, d_enc, K, N, etab);
    return hipGetLastError() == hipSuccess ? 0 : -3;
}

// ---------------------------------------------------------------------------------------------------
// (A11/A12) decode preparation: share selection (fecpp.cpp:528-548), the m x m inverse and the
// coefficient rows of the missing data shards.  One thread per group, for m <= MAXM.
//   Selection: data share i fills row i; the missing rows, ascending, take the highest present ids,
//   descending.  With >= K shares present those are always parity ids (present parity >= m).
//   With S[t][u] = enc[P_t][M_u] (t,u < m; P_t the parity used for missing row M_t):
//     coef[u][M_t] = Sinv[u][t]                                  (the parity share in column M_t)
//     coef[u][k]   = XOR_t Sinv[u][t] * enc[P_t][k],  k present    (data shares)
//   S is a square submatrix of the parity part of a systematic MDS generator, so every leading minor is
//   non-singular and elimination needs no pivot search; a zero pivot is still detected and reported.
// ---------------------------------------------------------------------------------------------------
struct PrepArgs {
    const uint64_t *present;
    const uint8_t *enc;  // N x K
    uint8_t *rec;
    uint8_t *out_idx;
    uint8_t *status;
    uint64_t G;
    int K, N, R;
    uint32_t rec_stride;
};

// (no early return: the unrolled q index stays a constant, so w[] lives in registers, not scratch)
__device__ __forceinline__ int pop_lowest(uint64_t (&w)[4])
{
    int res = -1;
#pragma unroll
    for (int q = 0; q < 4; ++q)
        if (res < 0 && w[q]) {
            res = q * 64 + __ffsll((unsigned long long)w[q]) - 1;
            w[q] &= w[q] - 1;
        }
    return res;
}

__device__ __forceinline__ int pop_highest(uint64_t (&w)[4])
{
    int res = -1;
#pragma unroll
    for (int q = 3; q >= 0; --q)
        if (res < 0 && w[q]) {
            const int b = 63 - __clzll((unsigned long long)w[q]);
            w[q] &= ~(1ull << b);
            res = q * 64 + b;
        }
    return res;
}

__device__ __forceinline__ void write_empty(const PrepArgs &a, uint64_t g, uint8_t st)
{
    uint8_t *rec = a.rec + g * a.rec_stride;
    rec[0] = st;
    rec[1] = 0;
    for (int t = 0; t < a.R; ++t) a.out_idx[g * a.R + t] = 0xFF;
    a.status[g] = st;
}

template <int MAXM>
__global__ void __launch_bounds__(kBlock) decode_prep_small(PrepArgs a)
{
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    uint8_t *s_exp = smem, *s_log = smem + 512, *s_E = smem + 768;  // s_E: parity rows, R x K
    stage_gf(s_exp, s_log);
    const int K = a.K, N = a.N, R = a.R;
    for (int i = threadIdx.x; i < R * K; i += blockDim.x) s_E[i] = a.enc[K * K + i];
    __syncthreads();

    for (uint64_t g = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; g < a.G;
         g += (uint64_t)gridDim.x * blockDim.x) {
        uint64_t w[4], dm[4];
        int cnt = 0, m = 0;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            w[q] = a.present[g * 4 + q] & bits_below(N, q);
            dm[q] = ~w[q] & bits_below(K, q);
            cnt += __popcll(w[q]);
            m += __popcll(dm[q]);
        }
        if (cnt < K) {
            write_empty(a, g, 1);
            continue;
        }
        uint8_t *rec = a.rec + g * a.rec_stride;
        int M[MAXM], P[MAXM];
        uint64_t dmw[4] = {dm[0], dm[1], dm[2], dm[3]};
        uint64_t pw[4] = {w[0], w[1], w[2], w[3]};
#pragma unroll
        for (int t = 0; t < MAXM; ++t) {
            M[t] = (t < m) ? pop_lowest(dmw) : 0;
            P[t] = (t < m) ? pop_highest(pw) : K;
        }
        // A = S extended by the identity to MAXM x MAXM; Iv accumulates the inverse
        uint32_t A[MAXM][MAXM], Iv[MAXM][MAXM];
#pragma unroll
        for (int t = 0; t < MAXM; ++t)
#pragma unroll
            for (int u = 0; u < MAXM; ++u) {
                A[t][u] = (t < m && u < m) ? s_E[(P[t] - K) * K + M[u]] : (uint32_t)(t == u);
                Iv[t][u] = (uint32_t)(t == u);
            }
        bool singular = false;
#pragma unroll
        for (int c = 0; c < MAXM; ++c) {
            if (c < m) {
                const uint32_t piv = A[c][c];
                singular |= (piv == 0);
                const uint32_t inv = ginv(s_exp, s_log, piv);
#pragma unroll
                for (int u = 0; u < MAXM; ++u) {
                    A[c][u] = gmul(s_exp, s_log, A[c][u], inv);
                    Iv[c][u] = gmul(s_exp, s_log, Iv[c][u], inv);
                }
#pragma unroll
                for (int r = 0; r < MAXM; ++r) {
                    if (r == c) continue;
                    const uint32_t f = A[r][c];
                    if (f) {
#pragma unroll
                        for (int u = 0; u < MAXM; ++u) {
                            A[r][u] ^= gmul(s_exp, s_log, f, A[c][u]);
                            Iv[r][u] ^= gmul(s_exp, s_log, f, Iv[c][u]);
                        }
                    }
                }
            }
        }
        if (singular) {
            write_empty(a, g, 2);
            continue;
        }
        rec[0] = 0;
        rec[1] = (uint8_t)m;
        rec[2] = rec[3] = 0;
        // log of the inverse, so each product below is one antilog lookup
        uint32_t lS[MAXM][MAXM];
#pragma unroll
        for (int u = 0; u < MAXM; ++u)
#pragma unroll
            for (int t = 0; t < MAXM; ++t) lS[u][t] = Iv[u][t] ? s_log[Iv[u][t]] : 0x1FFu;
        // columns in groups of 4 so that src and every coefficient row are written as whole dwords
        const int K4 = (K + 3) & ~3;
        uint32_t *srcw = reinterpret_cast<uint32_t *>(rec + 4);
        uint32_t *coefw = reinterpret_cast<uint32_t *>(rec + 4 + K4);
        for (int j0 = 0; j0 < K4; j0 += 4) {
            uint32_t sw = 0, cw[MAXM];
#pragma unroll
            for (int u = 0; u < MAXM; ++u) cw[u] = 0;
#pragma unroll
            for (int b = 0; b < 4; ++b) {
                const int j = j0 + b;
                if (j >= K) break;
                const bool miss = (dm[j >> 6] >> (j & 63)) & 1ull;
                if (miss) {
                    int t = 0;  // rank of j among the missing ids
#pragma unroll
                    for (int q = 0; q < 4; ++q)
                        t += (q < (j >> 6)) ? __popcll(dm[q])
                                            : (q == (j >> 6) ? __popcll(dm[q] & ((1ull << (j & 63)) - 1ull)) : 0);
                    uint32_t pt = 0;
#pragma unroll
                    for (int tt = 0; tt < MAXM; ++tt) pt = (tt == t) ? (uint32_t)P[tt] : pt;
                    sw |= pt << (8 * b);
#pragma unroll
                    for (int u = 0; u < MAXM; ++u) {
                        uint32_t v = 0;
#pragma unroll
                        for (int tt = 0; tt < MAXM; ++tt) v = (tt == t) ? Iv[u][tt] : v;
                        cw[u] |= v << (8 * b);
                    }
                } else {
                    sw |= (uint32_t)j << (8 * b);
                    uint32_t le[MAXM];
#pragma unroll
                    for (int t = 0; t < MAXM; ++t) {
                        const uint32_t e = (t < m) ? s_E[(P[t] - K) * K + j] : 0u;
                        le[t] = e ? s_log[e] : 0x1FFu;
                    }
#pragma unroll
                    for (int u = 0; u < MAXM; ++u) {
                        uint32_t v = 0;
#pragma unroll
                        for (int t = 0; t < MAXM; ++t)
                            if (t < m && lS[u][t] != 0x1FFu && le[t] != 0x1FFu) v ^= s_exp[lS[u][t] + le[t]];
                        cw[u] |= v << (8 * b);
                    }
                }
            }
            srcw[j0 >> 2] = sw;
#pragma unroll
            for (int u = 0; u < MAXM; ++u)
                if (u < m) coefw[u * (K4 >> 2) + (j0 >> 2)] = cw[u];
        }
#pragma unroll
        for (int t = 0; t < MAXM; ++t)
            if (t < R) a.out_idx[g * R + t] = (t < m) ? (uint8_t)M[t] : (uint8_t)0xFF;
        for (int t = MAXM; t < R; ++t) a.out_idx[g * R + t] = 0xFF;
        a.status[g] = 0;
    }
}

// acc ^ c * x for the 4 bytes of x (c given by its permute tables)
__device__ __forceinline__ uint32_t pm_apply(uint32_t acc, const uint32_t *t, uint32_t x)
{
    return perm_mac(acc, t, x & 0x07070707u, (x >> 3) & 0x07070707u, (x >> 6) & 0x03030303u);
}

// m <= MAXM <= 4 (fec=20:3, 10:3, ...): one thread per group, all GF arithmetic on packed bytes with the
// perm MAC instead of log/antilog lookups.  A row of [S | I] is one dword each for S and I (MAXM <= 4
// bytes); Gauss-Jordan normalises and eliminates whole rows with one perm MAC per dword; the coefficient
// product runs over dwords of the parity rows with the MAXM^2 tables of Sinv held in VGPRs.
template <int MAXM>
__global__ void __launch_bounds__(kBlock) decode_prep_perm(PrepArgs a)
{
    static_assert(MAXM >= 1 && MAXM <= 4, "rows are packed into one dword");
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    uint8_t *s_exp = smem, *s_log = smem + 512, *s_E = smem + 768;  // s_E: parity rows, R x K4 (zero padded)
    stage_gf(s_exp, s_log);
    const int K = a.K, N = a.N, R = a.R, K4 = (K + 3) & ~3, kd = K4 / 4;
    for (int i = threadIdx.x; i < R * K4; i += blockDim.x) {
        const int r = i / K4, j = i - r * K4;
        s_E[i] = j < K ? a.enc[(K + r) * K + j] : 0;
    }
    __syncthreads();
    const uint32_t *s_E32 = reinterpret_cast<const uint32_t *>(s_E);

    for (uint64_t g = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; g < a.G;
         g += (uint64_t)gridDim.x * blockDim.x) {
        uint64_t w[4], dm[4];
        int cnt = 0, m = 0;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            w[q] = a.present[g * 4 + q] & bits_below(N, q);
            dm[q] = ~w[q] & bits_below(K, q);
            cnt += __popcll(w[q]);
            m += __popcll(dm[q]);
        }
        if (cnt < K || m > MAXM) {
            write_empty(a, g, 1);
            continue;
        }
        uint8_t *rec = a.rec + g * a.rec_stride;
        int M[MAXM], P[MAXM];
        uint64_t dmw[4] = {dm[0], dm[1], dm[2], dm[3]};
        uint64_t pw[4] = {w[0], w[1], w[2], w[3]};
#pragma unroll
        for (int t = 0; t < MAXM; ++t) {
            M[t] = (t < m) ? pop_lowest(dmw) : 0;
            P[t] = (t < m) ? pop_highest(pw) : K;
        }
        // A[t] = row t of S (byte u = S[t][u]); identity beyond m.  Iv[t] = row t of the inverse.
        uint32_t A[MAXM], Iv[MAXM];
#pragma unroll
        for (int t = 0; t < MAXM; ++t) {
            uint32_t v = 0;
#pragma unroll
            for (int u = 0; u < MAXM; ++u) {
                const uint32_t x = (t < m && u < m) ? s_E[(P[t] - K) * K4 + M[u]] : (uint32_t)(t == u);
                v |= x << (8 * u);
            }
            A[t] = v;
            Iv[t] = 1u << (8 * t);
        }
        bool singular = false;
#pragma unroll
        for (int c = 0; c < MAXM; ++c) {
            if (c < m) {
                const uint32_t piv = (A[c] >> (8 * c)) & 0xFFu;
                singular |= (piv == 0);
                uint32_t tb[5];
                gf_perm_tables(ginv(s_exp, s_log, piv), tb);
                A[c] = pm_apply(0u, tb, A[c]);
                Iv[c] = pm_apply(0u, tb, Iv[c]);
#pragma unroll
                for (int r = 0; r < MAXM; ++r) {
                    if (r == c || r >= m) continue;
                    gf_perm_tables((A[r] >> (8 * c)) & 0xFFu, tb);
                    A[r] = pm_apply(A[r], tb, A[c]);
                    Iv[r] = pm_apply(Iv[r], tb, Iv[c]);
                }
            }
        }
        if (singular) {
            write_empty(a, g, 2);
            continue;
        }
        rec[0] = 0;
        rec[1] = (uint8_t)m;
        rec[2] = rec[3] = 0;
        // tables of Sinv[u][t] (zero beyond m, so those terms vanish)
        uint32_t T[MAXM][MAXM][5];
#pragma unroll
        for (int u = 0; u < MAXM; ++u)
#pragma unroll
            for (int t = 0; t < MAXM; ++t) gf_perm_tables((u < m && t < m) ? (Iv[u] >> (8 * t)) & 0xFFu : 0u, T[u][t]);
        uint32_t *srcw = reinterpret_cast<uint32_t *>(rec + 4);
        uint32_t *coefw = reinterpret_cast<uint32_t *>(rec + 4 + K4);
        for (int d = 0; d < kd; ++d) {
            uint32_t x[MAXM];
#pragma unroll
            for (int t = 0; t < MAXM; ++t) x[t] = (t < m) ? s_E32[(P[t] - K) * kd + d] : 0u;
            uint32_t cw[MAXM];
#pragma unroll
            for (int u = 0; u < MAXM; ++u) {
                uint32_t v = 0;
#pragma unroll
                for (int t = 0; t < MAXM; ++t) v = pm_apply(v, T[u][t], x[t]);
                cw[u] = v;
            }
            // columns of missing shards: source = the parity share P_rank, coefficient Sinv[u][rank]
            uint32_t sw = 0;
#pragma unroll
            for (int b = 0; b < 4; ++b) {
                const int j = 4 * d + b;
                uint32_t src = (uint32_t)j;
#pragma unroll
                for (int t = 0; t < MAXM; ++t)
                    if (t < m && M[t] == j) {
                        src = (uint32_t)P[t];
#pragma unroll
                        for (int u = 0; u < MAXM; ++u)
                            cw[u] = (cw[u] & ~(0xFFu << (8 * b))) | (((Iv[u] >> (8 * t)) & 0xFFu) << (8 * b));
                    }
                sw |= (j < K ? src : 0u) << (8 * b);
            }
            srcw[d] = sw;
#pragma unroll
            for (int u = 0; u < MAXM; ++u)
                if (u < m) coefw[u * kd + d] = cw[u];
        }
#pragma unroll
        for (int t = 0; t < MAXM; ++t)
            if (t < R) a.out_idx[g * R + t] = (t < m) ? (uint8_t)M[t] : (uint8_t)0xFF;
        for (int t = MAXM; t < R; ++t) a.out_idx[g * R + t] = 0xFF;
        a.status[g] = 0;
    }
}

// number of set bits of a 256-bit id map below id s
__device__ __forceinline__ int rank_below(const uint64_t (&b)[4], int s)
{
    int r = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int lo = 64 * q;
        if (s >= lo + 64) r += __popcll(b[q]);
        else if (s > lo) r += __popcll(b[q] & ((1ull << (s - lo)) - 1ull));
    }
    return r;
}

// General m (fec=200:55 and any m > 8): Lagrange (barycentric) form, one 256-thread workgroup per group.
//   Every share s is an evaluation of the data polynomial f (deg < K) at the point x_s (x_0 = 0,
//   x_s = alpha^s: the rows of the reference's Vandermonde matrix, fecpp.cpp:401,467), and the K selected
//   shares S (fecpp.cpp:528-548) determine f.  So the missing data shard M_u is
//     D_{M_u} = XOR_{i in S} share_i * prod_{k in S, k != i} (x_{M_u} ^ x_k) / (x_i ^ x_k).
//   The decoding map from the K selected shares is unique, so these coefficients are byte for byte the rows
//   of the reference's K x K inverse (fecpp.cpp:550-585) -- no elimination, nothing can be singular.
//   With FULL_s = sum_{k < N, k != s} log(x_s ^ x_k) (once per workgroup) and C = the R ids outside S:
//     log den_i = FULL_i - sum_{k in C} log(x_i ^ x_k)
//     log num_u = FULL_{M_u} - sum_{k in C, k != M_u} log(x_{M_u} ^ x_k)          (M_u is in C)
//     coef[u][i] = exp(log num_u - log(x_{M_u} ^ x_i) - log den_i)
//   That is O(K*R + m*R + m*K) table lookups per group, against O(m^3 + m^2*K) byte MACs for Gauss-Jordan
//   followed by the product with the parity rows (measured at 200:55: 63.8 ms -> see DESIGN.md 5).
constexpr int kPrepThreads = 256;

__global__ void __launch_bounds__(kPrepThreads) decode_prep_lagrange(PrepArgs a)
{
    __shared__ uint8_t s_exp[512], s_log[256];
    __shared__ uint16_t s_full[256];  // FULL_s mod 255
    __shared__ uint8_t s_C[256];      // ids outside S, ascending
    __shared__ uint8_t s_xC[256];     // their points
    __shared__ uint8_t s_M[256];      // missing data ids, ascending
    __shared__ uint8_t s_P[256];      // parity share used for missing rank t: the highest present ids, descending
    __shared__ uint8_t s_src[256];    // source share of column j
    __shared__ uint16_t s_lden[256];  // log den of the source of column j
    __shared__ uint16_t s_lnum[256];  // log num_u without the (x_{M_u} ^ x_i) factor
    const int K = a.K, N = a.N, R = a.R, tid = threadIdx.x;
    const int K4 = (K + 3) & ~3, kd = K4 / 4;
    stage_gf(s_exp, s_log);
    __syncthreads();
    auto xpt = [&](int sid) -> uint32_t { return sid ? (uint32_t)s_exp[sid] : 0u; };  // s_exp[255] = 1
    for (int sid = tid; sid < N; sid += kPrepThreads) {
        const uint32_t xs = xpt(sid);
        uint32_t acc = 0;
        for (int k = 0; k < N; ++k)
            if (k != sid) acc += s_log[xs ^ xpt(k)];
        s_full[sid] = (uint16_t)(acc % 255u);
    }
    __syncthreads();

    for (uint64_t g = blockIdx.x; g < a.G; g += gridDim.x) {
        uint64_t w[4], dm[4];
        int cnt = 0, m = 0;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            w[q] = a.present[g * 4 + q] & bits_below(N, q);
            dm[q] = ~w[q] & bits_below(K, q);
            cnt += __popcll(w[q]);
            m += __popcll(dm[q]);
        }
        uint8_t *rec = a.rec + g * a.rec_stride;
        if (cnt < K) {  // uniform over the workgroup
            if (tid == 0) {
                rec[0] = 1;
                rec[1] = 0;
                a.status[g] = 1;
            }
            for (int t = tid; t < R; t += kPrepThreads) a.out_idx[g * R + t] = 0xFF;
            continue;
        }
        // P_t = the present id with exactly t present ids above it (t < m; all parity since cnt >= K);
        // the lowest of them, P_{m-1}, bounds the used-parity set from below
        for (int sid = tid; sid < N; sid += kPrepThreads) {
            if ((w[sid >> 6] >> (sid & 63)) & 1ull) {
                const int above = cnt - 1 - rank_below(w, sid);
                if (above < m) s_P[above] = (uint8_t)sid;
            }
        }
        __syncthreads();
        const int thr = m > 0 ? (int)s_P[m - 1] : 256;
        uint64_t Cb[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const uint64_t used_par = w[q] & ~bits_below(thr, q);
            const uint64_t S = (w[q] & bits_below(K, q)) | used_par;
            Cb[q] = ~S & bits_below(N, q);
        }
        for (int sid = tid; sid < N; sid += kPrepThreads) {
            const int q = sid >> 6, b = sid & 63;
            if ((Cb[q] >> b) & 1ull) {
                const int r = rank_below(Cb, sid);
                s_C[r] = (uint8_t)sid;
                s_xC[r] = (uint8_t)xpt(sid);
            }
            if (sid < K && ((dm[q] >> b) & 1ull)) s_M[rank_below(dm, sid)] = (uint8_t)sid;
        }
        __syncthreads();
        for (int j = tid; j < K; j += kPrepThreads) {
            const bool miss = (dm[j >> 6] >> (j & 63)) & 1ull;
            const int i = miss ? (int)s_P[rank_below(dm, j)] : j;
            s_src[j] = (uint8_t)i;
            const uint32_t xi = xpt(i);
            uint32_t acc = 0;
            for (int c = 0; c < R; ++c) acc += s_log[xi ^ s_xC[c]];
            s_lden[j] = (uint16_t)((s_full[i] + 255u - acc % 255u) % 255u);
        }
        for (int u = tid; u < m; u += kPrepThreads) {
            const int mu = s_M[u];
            const uint32_t xm = xpt(mu);
            uint32_t acc = 0;
            for (int c = 0; c < R; ++c)
                if (s_C[c] != mu) acc += s_log[xm ^ s_xC[c]];
            s_lnum[u] = (uint16_t)((s_full[mu] + 255u - acc % 255u) % 255u);
        }
        __syncthreads();
        uint32_t *srcw = reinterpret_cast<uint32_t *>(rec + 4);
        uint32_t *coefw = reinterpret_cast<uint32_t *>(rec + 4 + K4);
        for (int d = tid; d < kd; d += kPrepThreads) {
            uint32_t v = 0;
#pragma unroll
            for (int b = 0; b < 4; ++b)
                if (4 * d + b < K) v |= (uint32_t)s_src[4 * d + b] << (8 * b);
            srcw[d] = v;
        }
        for (int e = tid; e < m * kd; e += kPrepThreads) {
            const int u = e / kd, d = e - u * kd;
            const uint32_t xm = xpt(s_M[u]);
            const int ln = s_lnum[u];
            uint32_t v = 0;
#pragma unroll
            for (int b = 0; b < 4; ++b) {
                const int j = 4 * d + b;
                if (j < K) {
                    const int ex = (ln + 510 - (int)s_log[xm ^ xpt(s_src[j])] - (int)s_lden[j]) % 255;
                    v |= (uint32_t)s_exp[ex] << (8 * b);
                }
            }
            coefw[u * kd + d] = v;
        }
        for (int t = tid; t < R; t += kPrepThreads) a.out_idx[g * R + t] = (t < m) ? s_M[t] : (uint8_t)0xFF;
        if (tid == 0) {
            rec[0] = 0;
            rec[1] = (uint8_t)m;
            rec[2] = rec[3] = 0;
            a.status[g] = 0;
        }
        __syncthreads();  // the lists are rewritten for the next group
    }
}

// ---------------------------------------------------------------------------------------------------
// (A4/A5/A8/A11) perm-MAC kernel: out[g][row] = XOR_j coef[row][j] * share_j[g]  over V-byte columns.
// ---------------------------------------------------------------------------------------------------
struct MacArgs {
    const uint8_t *data;    // [G][K][pitch]
    const uint8_t *parity;  // [G][R][pitch]
    uint8_t *out;           // encode: parity, decode: recovered [G][R][pitch]
    const uint8_t *enc;     // N x K encoding matrix (encode)
    const uint8_t *rec;     // per-group records (decode)
    uint64_t pitch;
    uint32_t total;         // G * cpad work items
    uint32_t cols;          // granules per shard
    uint32_t cpad;          // items per group (>= cols; lanes with col >= cols idle)
    uint32_t G, K, R, B;
    uint32_t rec_stride;
    uint32_t JC;            // shards per LDS chunk
    uint32_t gmax;          // group slots per chunk
    const uint32_t *etab;   // encode: perm tables [K][etab_rows][5] read with scalar loads (null: LDS path)
    uint32_t etab_rows;
    const uint32_t *list;   // decode: the groups with work (m > 0), ascending per wave; null = every group
    const uint32_t *list_count;
};

template <int VEC>
struct Gran {
    static constexpr int W = VEC >= 4 ? VEC / 4 : 1;
    uint32_t d[W];
};

template <int VEC>
__device__ __forceinline__ Gran<VEC> load_gran(const uint8_t *p, uint32_t col, uint32_t B)
{
    Gran<VEC> v;
    if constexpr (VEC == 32) {
        const uint4 x = reinterpret_cast<const uint4 *>(p)[0], y = reinterpret_cast<const uint4 *>(p)[1];
        v.d[0] = x.x; v.d[1] = x.y; v.d[2] = x.z; v.d[3] = x.w;
        v.d[4] = y.x; v.d[5] = y.y; v.d[6] = y.z; v.d[7] = y.w;
    } else if constexpr (VEC == 16) {
        const uint4 x = *reinterpret_cast<const uint4 *>(p);
        v.d[0] = x.x; v.d[1] = x.y; v.d[2] = x.z; v.d[3] = x.w;
    } else if constexpr (VEC == 8) {
        const uint2 x = *reinterpret_cast<const uint2 *>(p);
        v.d[0] = x.x; v.d[1] = x.y;
    } else if constexpr (VEC == 4) {
        v.d[0] = *reinterpret_cast<const uint32_t *>(p);
    } else {  // bytewise: 4 bytes at p, only those below B
        uint32_t x = 0;
        const uint32_t b0 = col * 4;
#pragma unroll
        for (int b = 0; b < 4; ++b)
            if (b0 + b < B) x |= (uint32_t)p[b] << (8 * b);
        v.d[0] = x;
    }
    return v;
}

template <int VEC>
__device__ __forceinline__ void store_gran(uint8_t *p, const uint32_t *d, uint32_t col, uint32_t B)
{
    if constexpr (VEC == 32) {
        store_gran<16>(p, d, col, B);
        store_gran<16>(p + 16, d + 4, col, B);
    } else if constexpr (VEC == 16) {
#if KFEC_NTSTORE
        typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));
        __builtin_nontemporal_store(u32x4_t{d[0], d[1], d[2], d[3]}, reinterpret_cast<u32x4_t *>(p));
#else
        *reinterpret_cast<uint4 *>(p) = make_uint4(d[0], d[1], d[2], d[3]);
#endif
    } else if constexpr (VEC == 8) {
        *reinterpret_cast<uint2 *>(p) = make_uint2(d[0], d[1]);
    } else if constexpr (VEC == 4) {
        *reinterpret_cast<uint32_t *>(p) = d[0];
    } else {
        const uint32_t b0 = col * 4;
#pragma unroll
        for (int b = 0; b < 4; ++b)
            if (b0 + b < B) p[b] = (uint8_t)(d[0] >> (8 * b));
    }
}

// Last granule of a shard row when B is not a multiple of VEC (e.g. B = 1400 at VEC = 32): only the nd
// dwords that hold bytes below B are loaded / stored (bytes [B, 4*ceil(B/4)) lie inside the pitch), so no
// lane reads or writes past its own slot -- pitch only needs to be a multiple of 4.
template <int VEC>
__device__ __forceinline__ Gran<VEC> load_gran_tail(const uint8_t *p, uint32_t nd)
{
    Gran<VEC> v;
#pragma unroll
    for (int w = 0; w < Gran<VEC>::W; ++w) v.d[w] = (uint32_t)w < nd ? reinterpret_cast<const uint32_t *>(p)[w] : 0u;
    return v;
}

template <int VEC>
__device__ __forceinline__ void store_gran_tail(uint8_t *p, const uint32_t *d, uint32_t nd)
{
#pragma unroll
    for (int w = 0; w < Gran<VEC>::W; ++w)
        if ((uint32_t)w < nd) reinterpret_cast<uint32_t *>(p)[w] = d[w];
}

template <int MT>
struct MacLayout {
    static_assert(MT >= 1 && MT <= 8, "row tile");
    static constexpr int TBL_DW = ((5 * MT + 3) / 4) * 4;  // table dwords per (group, shard): 5 per row
    static constexpr int ENTRY = 16 + 4 * TBL_DW;          // + 8-byte share pointer, 8 pad
};

// expand coefficients of shards [c0, c0+nj) for group slots [0, ng) into LDS entries
template <int MT, bool DEC>
__device__ __forceinline__ void mac_expand(const MacArgs &a, uint8_t *s_ent, uint32_t gfirst, uint32_t ng,
                                           uint32_t c0, uint32_t nj, uint32_t row0)
{
    using L = MacLayout<MT>;
    const uint32_t items = ng * nj * MT;
    for (uint32_t e = threadIdx.x; e < items; e += blockDim.x) {
        const uint32_t r = e % MT, q = e / MT;
        const uint32_t jj = q % nj, gs = q / nj;
        const uint32_t j = c0 + jj, u = row0 + r;
        uint8_t *ent = s_ent + (gs * a.JC + jj) * L::ENTRY;
        uint32_t c = 0;
        if constexpr (DEC) {
            const uint32_t K4 = (a.K + 3) & ~3u;
            const uint32_t g = a.list ? a.list[gfirst + gs] : gfirst + gs;
            const uint8_t *rec = a.rec + (uint64_t)g * a.rec_stride;
            const uint32_t st = rec[0], m = rec[1];
            if (st == 0 && u < m) c = rec[4 + K4 + u * K4 + j];
            if (r == 0) {
                const uint32_t src = rec[4 + j];
                const uint8_t *p = (src < a.K) ? a.data + ((uint64_t)g * a.K + src) * a.pitch
                                               : a.parity + ((uint64_t)g * a.R + (src - a.K)) * a.pitch;
                *reinterpret_cast<const uint8_t **>(ent) = p;
            }
        } else {
            if (u < a.R) c = a.enc[(uint64_t)(a.K + u) * a.K + j];
        }
        uint32_t t[5];
#if KFEC_ABLATE == 4  // timing-only: no table construction in the per-workgroup expansion
        t[0] = t[1] = t[2] = t[3] = t[4] = c;
#else
        gf_perm_tables(c, t);
#endif
        uint32_t *tp = reinterpret_cast<uint32_t *>(ent + 16) + 5 * r;
#pragma unroll
        for (int i = 0; i < 5; ++i) tp[i] = t[i];
    }
}

template <int VEC, int MT, bool DEC, int PDX = 0>
__global__ void __launch_bounds__(kMacBlock, KFEC_MINW) mac_kernel(MacArgs a)
{
    using L = MacLayout<MT>;
    constexpr int W = Gran<VEC>::W;
    // shards in flight per lane (~64 B per lane); PDX: the latency shape (a handful of groups, often read
    // straight from pinned host memory) keeps many more loads in flight so the PCIe round trips overlap
    constexpr int PD = PDX ? PDX : (VEC >= 32 ? KFEC_PD / 2 : KFEC_PD);
    constexpr int VB = VEC >= 4 ? VEC : 4;  // bytes per granule
    extern __shared__ __attribute__((aligned(16))) uint8_t s_ent[];

    const uint32_t row0 = blockIdx.y * MT;
    const uint32_t K = a.K, cols = a.cpad;
    const bool gtab = !DEC && a.etab != nullptr;  // encode: wave-uniform tables straight from memory
    const bool enc_once = !DEC && (gtab || K <= a.JC);
    if (enc_once && !gtab) {
        mac_expand<MT, false>(a, s_ent, 0, 1, 0, K, row0);
        __syncthreads();
    }
    const uint32_t stride = gridDim.x * kMacBlock;
    // XCD-aware order: the dispatcher deals workgroups round-robin over the 8 XCDs, so workgroup b would run
    // next to b+8, not b+1.  Re-numbering (bijective, MI355X guide T1) gives each XCD a contiguous run of
    // items, so the 128-B lines that straddle two workgroups' columns are fetched by one L2, not two.
    uint32_t wg = blockIdx.x;
#if KFEC_XCD_REMAP
    {
        const uint32_t n = gridDim.x, q = n / 8, r = n % 8, x = wg % 8, i = wg / 8;
        wg = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + i;
    }
#endif
    // decode with a work list: only the groups that lost data shards are visited (list index space)
    const uint32_t total = (DEC && a.list) ? min(*a.list_count, a.G) * cols : a.total;
    for (uint32_t base = wg * kMacBlock; base < total; base += stride) {
        const uint32_t item = base + threadIdx.x;
        const uint32_t gi = item < total ? item / cols : 0;  // list index (= group without a list)
        const uint32_t col = item < total ? item - gi * cols : 0;
        const bool in = item < total && col < a.cols;
        const uint32_t g = (DEC && a.list) ? (item < total ? a.list[gi] : 0u) : gi;
        // dwords of this lane's granule below B: W except in the last granule of a row when VEC does not
        // divide B (VEC >= 4 only; the bytewise VEC = 1 path checks every byte itself)
        const uint32_t nd = (VEC >= 4 && (col + 1) * VB > a.B) ? (a.B - col * VB + 3) / 4 : (uint32_t)W;
        const uint32_t gfirst = base / cols;
        const uint32_t glast = min(base + kMacBlock - 1, total - 1) / cols;
        const uint32_t ng = glast - gfirst + 1;
        const uint32_t gs = DEC ? gi - gfirst : 0;

        uint32_t rows = 0;
        if (in) {
            if constexpr (DEC) {
                const uint8_t *rec = a.rec + (uint64_t)g * a.rec_stride;
                const uint32_t st = rec[0], m = rec[1];
                rows = (st == 0 && m > row0) ? min((uint32_t)MT, m - row0) : 0u;
            } else {
                rows = a.R > row0 ? min((uint32_t)MT, a.R - row0) : 0u;
            }
        }
        uint32_t acc[MT][W];
#pragma unroll
        for (int r = 0; r < MT; ++r)
#pragma unroll
            for (int w = 0; w < W; ++w) acc[r][w] = 0;

        const uint8_t *enc_base = a.data + ((uint64_t)g * K) * a.pitch + (uint64_t)col * VB;
        for (uint32_t c0 = 0; c0 < K; c0 += a.JC) {
            const uint32_t nj = min(a.JC, K - c0);
            if (!enc_once) {
                __syncthreads();
                mac_expand<MT, DEC>(a, s_ent, gfirst, DEC ? ng : 1u, c0, nj, row0);
                __syncthreads();
            }
            if (rows == 0) continue;
            const uint8_t *ent0 = s_ent + (gs * a.JC) * L::ENTRY;
            // (a shard visiting order that puts the two readers of a line straddling shards j and j+1 >= PD
            // loads apart, or lags odd waves, was measured: no gain at 20:3, -15% at 10:3 -- DESIGN.md 4.5)
            auto sj = [](uint32_t jj) -> uint32_t { return jj; };
            auto share_ptr = [&](uint32_t jj) -> const uint8_t * {
                const uint32_t j = sj(jj);
                if constexpr (DEC) {
#if KFEC_ABLATE == 2  // timing-only: decode reads shards like encode (data buffer, no pointer indirection)
                    return enc_base + (uint64_t)(c0 + j) * a.pitch;
#endif
                    return *reinterpret_cast<const uint8_t *const *>(ent0 + j * L::ENTRY) + (uint64_t)col * VB;
                } else {
                    return enc_base + (uint64_t)(c0 + j) * a.pitch;
                }
            };
            Gran<VEC> x[PD];
#pragma unroll
            for (int u = 0; u < PD; ++u)
                if ((uint32_t)u < nj)
                    x[u] = nd < (uint32_t)W ? load_gran_tail<VEC>(share_ptr(u), nd) : load_gran<VEC>(share_ptr(u), col, a.B);
            for (uint32_t jb = 0; jb < nj; jb += PD) {
#pragma unroll
                for (int u = 0; u < PD; ++u) {
                    const uint32_t jj = jb + u;
                    if (jj < nj) {
                        const Gran<VEC> cur = x[u];
                        if (jj + PD < nj)
                            x[u] = nd < (uint32_t)W ? load_gran_tail<VEC>(share_ptr(jj + PD), nd)
                                                    : load_gran<VEC>(share_ptr(jj + PD), col, a.B);
                        const uint8_t *ent = ent0 + sj(jj) * L::ENTRY;
                        uint32_t t[L::TBL_DW];
                        if (gtab) {
                            // uniform address in the constant address space: scalar loads into SGPRs, no LDS
                            typedef const __attribute__((address_space(4))) uint32_t cu32;
                            const cu32 *tg = (const cu32 *)(a.etab + ((size_t)(c0 + jj) * a.etab_rows + row0) * 5);
#pragma unroll
                            for (int i = 0; i < 5 * MT; ++i) t[i] = tg[i];
                        } else {
                            const uint4 *tv = reinterpret_cast<const uint4 *>(ent + 16);
#pragma unroll
                            for (int i = 0; i < L::TBL_DW / 4; ++i) {
                                const uint4 q = tv[i];
                                t[4 * i] = q.x; t[4 * i + 1] = q.y; t[4 * i + 2] = q.z; t[4 * i + 3] = q.w;
                            }
                        }
#pragma unroll
                        for (int w = 0; w < W; ++w) {
                            const uint32_t xv = cur.d[w];
                            const uint32_t s0 = xv & 0x07070707u;
                            const uint32_t s1 = (xv >> 3) & 0x07070707u;
                            const uint32_t s2 = (xv >> 6) & 0x03030303u;
#pragma unroll
                            for (int r = 0; r < MT; ++r) {
#if KFEC_ABLATE == 1  // timing-only build: memory traffic of the real kernel, XOR instead of the GF MAC
                                acc[r][w] ^= xv ^ t[5 * r];
                                (void)s0; (void)s1; (void)s2;
#else
                                acc[r][w] = perm_mac(acc[r][w], t + 5 * r, s0, s1, s2);
#endif
                            }
                        }
                    }
                }
            }
        }
        if (rows) {
            const uint64_t obase = ((uint64_t)g * a.R + row0) * a.pitch + (uint64_t)col * VB;
#pragma unroll
            for (int r = 0; r < MT; ++r)
                if ((uint32_t)r < rows) {
                    uint8_t *o = a.out + obase + (uint64_t)r * a.pitch;
                    if (nd < (uint32_t)W) store_gran_tail<VEC>(o, acc[r], nd);
                    else store_gran<VEC>(o, acc[r], col, a.B);
                }
        }
    }
}

// ---------------------------------------------------------------------------------------------------
// (A4/A5/A8/A11) group-tile perm-MAC kernel: the primary path for shards up to 8 KiB.
// One workgroup owns one shard group at a time.  It stages the group's K selected shards (or a chunk of
// JS of them) into LDS with linear, coalesced 16-B loads -- a whole group of 20 x 1440 B is 225 complete
// 128-B lines, so no line is fetched twice, unlike per-lane strided column reads whose 1-KiB wave
// chunks straddle shard boundaries -- then every lane computes one 8-byte column of the MT output rows
// from LDS.  The coefficient tables of the chunk are expanded into LDS once per group (decode) or once
// per kernel (encode) and read back with broadcast ds_read_b128.
// ---------------------------------------------------------------------------------------------------
struct LdsArgs {
    const uint8_t *data;    // [G][K][pitch]
    const uint8_t *parity;  // [G][R][pitch]
    uint8_t *out;           // encode: parity, decode: recovered [G][R][pitch]
    const uint8_t *enc;     // N x K (encode)
    const uint8_t *rec;     // per-group records (decode)
    uint64_t pitch;
    uint32_t G, K, R, B;
    uint32_t rec_stride;
    uint32_t JS;            // shards staged per chunk
    uint32_t Bs;            // LDS row stride of a staged shard (multiple of 16, >= B)
    uint32_t cols;          // 8-byte columns = ceil(B / 8)
    uint64_t bs_inv;        // ceil(2^32 / Bs): o / Bs for staged offsets o < 2^16 without a divide
    uint32_t tbl_all;       // encode: tables of all K shards stay in LDS for the whole kernel
};

template <int MT>
struct TileLayout {
    static constexpr int T4 = (MT + 3) / 4 * 4;
    static constexpr int TBL = MT * 16 + T4 * 4;  // per shard: [MT][t0..t3] then t4[MT] (padded to 16 B)
};

// expand coefficient tables of shards [c0, c0+nj) for rows [row0, row0+MT) of group g into LDS
template <int MT, bool DEC>
__device__ __forceinline__ void tile_expand(const LdsArgs &a, uint8_t *s_tbl, uint32_t g, uint32_t c0, uint32_t nj,
                                            uint32_t row0, uint32_t m)
{
    using L = TileLayout<MT>;
    for (uint32_t e = threadIdx.x; e < nj * MT; e += blockDim.x) {
        const uint32_t r = e % MT, jj = e / MT, j = c0 + jj, u = row0 + r;
        uint32_t c = 0;
        if constexpr (DEC) {
            if (u < m) c = a.rec[(uint64_t)g * a.rec_stride + 4 + ((a.K + 3) & ~3u) * (1 + u) + j];
        } else {
            if (u < a.R) c = a.enc[(uint64_t)(a.K + u) * a.K + j];
        }
        uint32_t t[5];
        gf_perm_tables(c, t);
        uint8_t *base = s_tbl + jj * L::TBL;
        *reinterpret_cast<uint4 *>(base + r * 16) = make_uint4(t[0], t[1], t[2], t[3]);
        reinterpret_cast<uint32_t *>(base + MT * 16)[r] = t[4];
    }
}

template <int SV>
__device__ __forceinline__ void stage_copy(uint8_t *dst, const uint8_t *src)
{
    if constexpr (SV == 16) *reinterpret_cast<uint4 *>(dst) = *reinterpret_cast<const uint4 *>(src);
    else if constexpr (SV == 8) *reinterpret_cast<uint2 *>(dst) = *reinterpret_cast<const uint2 *>(src);
    else if constexpr (SV == 4) *reinterpret_cast<uint32_t *>(dst) = *reinterpret_cast<const uint32_t *>(src);
    else *dst = *src;
}

typedef unsigned int u32x2_t __attribute__((ext_vector_type(2)));

// One work unit = (group g, chunk of shards [c0, c0+nj)).  Stage a unit into an LDS buffer of JS rows of
// Bs bytes.  SV == 16: LDS-DMA (global_load_lds_dwordx4): each wave-instruction fills 1 KiB of LDS
// contiguously while every lane names its own 16-B source -- a gather of shard rows; asynchronous, no
// VGPRs, completion awaited by the next s_waitcnt vmcnt(0) + barrier.  Other SV (pitch not 16-aligned):
// synchronous register staging.
template <int SV, bool DEC>
__device__ __forceinline__ void tile_stage(const LdsArgs &a, uint8_t *buf, uint32_t g, uint32_t c0, uint32_t nj)
{
    const uint32_t K = a.K;
    auto shard_src = [&](uint32_t jj) -> const uint8_t * {
        if constexpr (DEC) {
            const uint32_t sid = a.rec[(uint64_t)g * a.rec_stride + 4 + c0 + jj];
            return (sid < K) ? a.data + ((uint64_t)g * K + sid) * a.pitch
                             : a.parity + ((uint64_t)g * a.R + (sid - K)) * a.pitch;
        } else {
            return a.data + ((uint64_t)g * K + c0 + jj) * a.pitch;
        }
    };
    if constexpr (SV == 16) {
        const uint32_t bytes = nj * a.Bs;
        const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63, nw = blockDim.x >> 6;
        for (uint32_t ch = wave; ch * 1024 < bytes; ch += nw) {
            const uint32_t o = ch * 1024 + lane * 16;
            const uint32_t jj = (uint32_t)(((uint64_t)o * a.bs_inv) >> 32), off = o - jj * a.Bs;  // o / Bs
            (void)off;  // read only in the device pass
            if (o < bytes) {
#if defined(__HIP_DEVICE_COMPILE__)  // the builtin exists only in the device pass of this single-source file
                __builtin_amdgcn_global_load_lds(shard_src(jj) + off,
                                                 (__attribute__((address_space(3))) void *)(buf + ch * 1024), 16, 0, 0);
#endif
            }
        }
    } else {
        const uint32_t gps = a.Bs / SV;  // granules per staged row (rows padded to 16 B)
        const uint32_t total = nj * gps;
        constexpr int NB = 8;
        for (uint32_t base = threadIdx.x; base < total; base += NB * blockDim.x) {
            uint8_t v[NB][SV];
#pragma unroll
            for (int k = 0; k < NB; ++k) {
                const uint32_t gi = base + k * blockDim.x;
                if (gi < total) {
                    const uint32_t jj = gi / gps, off = (gi - jj * gps) * SV;
                    if (off < a.B) {
                        const uint8_t *src = shard_src(jj) + off;
                        if constexpr (SV == 8) *reinterpret_cast<uint2 *>(v[k]) = *reinterpret_cast<const uint2 *>(src);
                        else if constexpr (SV == 4) *reinterpret_cast<uint32_t *>(v[k]) = *reinterpret_cast<const uint32_t *>(src);
                        else v[k][0] = *src;
                    }
                }
            }
#pragma unroll
            for (int k = 0; k < NB; ++k) {
                const uint32_t gi = base + k * blockDim.x;
                if (gi < total) {
                    const uint32_t jj = gi / gps, off = (gi - jj * gps) * SV;
                    uint8_t *dst = buf + jj * a.Bs + off;
                    if constexpr (SV == 8) *reinterpret_cast<uint2 *>(dst) = *reinterpret_cast<uint2 *>(v[k]);
                    else if constexpr (SV == 4) *reinterpret_cast<uint32_t *>(dst) = *reinterpret_cast<uint32_t *>(v[k]);
                    else *dst = v[k][0];
                }
            }
        }
    }
}

// acc[r] ^= coef(r, jj) * x over one 8-byte column, tables at tb (TileLayout)
template <int MT>
__device__ __forceinline__ void tile_mac(u32x2_t (&acc)[MT], u32x2_t x, const uint8_t *tb)
{
    using L = TileLayout<MT>;
    uint32_t t4[L::T4];
#pragma unroll
    for (int q = 0; q < L::T4 / 4; ++q) {
        const uint4 v = reinterpret_cast<const uint4 *>(tb + MT * 16)[q];
        t4[4 * q] = v.x; t4[4 * q + 1] = v.y; t4[4 * q + 2] = v.z; t4[4 * q + 3] = v.w;
    }
    uint32_t s0[2], s1[2], s2[2];
#pragma unroll
    for (int w = 0; w < 2; ++w) {
        s0[w] = x[w] & 0x07070707u;
        s1[w] = (x[w] >> 3) & 0x07070707u;
        s2[w] = (x[w] >> 6) & 0x03030303u;
    }
#pragma unroll
    for (int r = 0; r < MT; ++r) {
        const uint4 v = reinterpret_cast<const uint4 *>(tb)[r];
        const uint32_t t[5] = {v.x, v.y, v.z, v.w, t4[r]};
#if KFEC_ABLATE == 1
        acc[r][0] ^= x[0] ^ t[0];
        acc[r][1] ^= x[1] ^ t[4];
#else
#pragma unroll
        for (int w = 0; w < 2; ++w) acc[r][w] = perm_mac(acc[r][w], t, s0[w], s1[w], s2[w]);
#endif
    }
}

// as tile_mac, with the shard's tables already in registers (TileLayout order)
template <int MT>
__device__ __forceinline__ void tile_mac_regs(u32x2_t (&acc)[MT], u32x2_t x, const uint4 *tv)
{
    using L = TileLayout<MT>;
    const uint32_t *t4 = reinterpret_cast<const uint32_t *>(tv + MT);
    uint32_t s0[2], s1[2], s2[2];
#pragma unroll
    for (int w = 0; w < 2; ++w) {
        s0[w] = x[w] & 0x07070707u;
        s1[w] = (x[w] >> 3) & 0x07070707u;
        s2[w] = (x[w] >> 6) & 0x03030303u;
    }
#pragma unroll
    for (int r = 0; r < MT; ++r) {
        const uint32_t t[5] = {tv[r].x, tv[r].y, tv[r].z, tv[r].w, t4[r]};
#if KFEC_ABLATE == 1
        acc[r][0] ^= x[0] ^ t[0];
        acc[r][1] ^= x[1] ^ t[4];
#else
#pragma unroll
        for (int w = 0; w < 2; ++w) acc[r][w] = perm_mac(acc[r][w], t, s0[w], s1[w], s2[w]);
#endif
    }
    (void)sizeof(L);
}

// Persistent workgroup walking its (group, chunk) units through a 2-deep LDS ring: the DMA of unit u+1
// is in flight while unit u is computed.  Tables (and, for encode with few shards, the whole table set)
// live beside the ring.
template <int MT, bool DEC, int SV>
__global__ void __launch_bounds__(256) mac_tile_kernel(LdsArgs a)
{
    using L = TileLayout<MT>;
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const uint32_t K = a.K, JS = a.JS, row0 = blockIdx.y * MT;
    const uint32_t nch = (K + JS - 1) / JS;  // chunks per group
    // LDS carve-up as integer offsets from smem: selecting between two pointers at run time makes hipcc
    // lose the LDS address space and emit flat loads for the whole compute loop
    const uint32_t ring_sz = JS * a.Bs, tbl0 = 2 * ring_sz, tring_sz = JS * L::TBL;
    uint8_t *tbl_base = smem + tbl0;
    // encode tables for all K shards fit once (enc_all) or are expanded per unit into a 2-deep ring
    const bool enc_all = !DEC && a.tbl_all;

    // rows of this workgroup's tile for group g; 0 = nothing to do for g
    auto rows_of = [&](uint32_t g) -> uint32_t {
        if constexpr (DEC) {
            const uint8_t *rec = a.rec + (uint64_t)g * a.rec_stride;
            const uint32_t st = rec[0], m = rec[1];
            return (st == 0 && m > row0) ? min((uint32_t)MT, m - row0) : 0u;
        } else {
            return a.R > row0 ? min((uint32_t)MT, a.R - row0) : 0u;
        }
    };
    auto m_of = [&](uint32_t g) -> uint32_t {
        if constexpr (DEC) return a.rec[(uint64_t)g * a.rec_stride + 1];
        else return 0u;
    };
    // first group at or after g with work for this tile
    auto next_group = [&](uint32_t g) -> uint32_t {
        while (g < a.G && rows_of(g) == 0) g += gridDim.x;
        return g;
    };

    if (enc_all) tile_expand<MT, false>(a, tbl_base, 0, 0, K, row0, 0);

    uint32_t g = next_group(blockIdx.x), c = 0;
    if (g >= a.G) return;
    // prologue: unit (g, 0) into slot 0
    if (!enc_all) tile_expand<MT, DEC>(a, smem + tbl0, g, 0, min(JS, K), row0, m_of(g));
    tile_stage<SV, DEC>(a, smem, g, 0, min(JS, K));
    uint32_t slot = 0, rows = rows_of(g);
    u32x2_t acc[MT];
#pragma unroll
    for (int r = 0; r < MT; ++r) acc[r] = u32x2_t{0u, 0u};
    const uint32_t col = threadIdx.x;
    while (true) {
        // the unit after (g, c)
        uint32_t gn = g, cn = c + 1;
        if (cn == nch) {
            cn = 0;
            gn = next_group(g + gridDim.x);
        }
        if constexpr (SV == 16) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();  // unit (g, c) has landed in ring[slot]; everyone is done with ring[slot ^ 1]
        if (gn < a.G) {
            const uint32_t njn = min(JS, K - cn * JS);
            if (!enc_all) tile_expand<MT, DEC>(a, smem + tbl0 + (slot ^ 1) * tring_sz, gn, cn * JS, njn, row0, m_of(gn));
            tile_stage<SV, DEC>(a, smem + (slot ^ 1) * ring_sz, gn, cn * JS, njn);
        }
        const uint32_t nj = min(JS, K - c * JS);
        const uint32_t tb_off = enc_all ? tbl0 + c * JS * L::TBL : tbl0 + slot * tring_sz;
        if (col < a.cols) {
            const uint8_t *tb = smem + tb_off;
            const uint8_t *xs = smem + slot * ring_sz + col * 8;
            for (uint32_t jj = 0; jj < nj; ++jj)
                tile_mac<MT>(acc, *reinterpret_cast<const u32x2_t *>(xs + jj * a.Bs), tb + jj * L::TBL);
        }
        if (c + 1 == nch) {  // group finished: store its rows
            if (col < a.cols) {
                const uint64_t obase = ((uint64_t)g * a.R + row0) * a.pitch + (uint64_t)col * 8;
#pragma unroll
                for (int r = 0; r < MT; ++r) {
                    if ((uint32_t)r < rows) {
                        uint8_t *o = a.out + obase + (uint64_t)r * a.pitch;
                        if constexpr (SV >= 8) {
                            *reinterpret_cast<u32x2_t *>(o) = acc[r];
                        } else if constexpr (SV == 4) {
                            // pitch is only 4-aligned: the second dword may lie past the slot's pitch
                            *reinterpret_cast<uint32_t *>(o) = acc[r][0];
                            if (col * 8 + 4 < a.B) *reinterpret_cast<uint32_t *>(o + 4) = acc[r][1];
                        } else {
#pragma unroll
                            for (int b = 0; b < 8; ++b)
                                if (col * 8 + b < a.B) o[b] = (uint8_t)(acc[r][b >> 2] >> (8 * (b & 3)));
                        }
                    }
                }
            }
#pragma unroll
            for (int r = 0; r < MT; ++r) acc[r] = u32x2_t{0u, 0u};
            if (gn >= a.G) break;
            rows = rows_of(gn);
        }
        g = gn;
        c = cn;
        slot ^= 1;
    }
}

// ---------------------------------------------------------------------------------------------------
// (A4/A5/A8/A11) wave-tile kernel: the primary path for 16-B aligned layouts, B <= 2 KiB, R <= 8.
// One workgroup = one wave, persistent over its groups.  A group is streamed in chunks of JS shards
// (20 x 1440 B -> chunks of 8, 8, 4 shards = 90, 90, 45 whole 128-B lines): every wave-instruction
// loads 1 KiB of consecutive bytes, so each line is requested exactly once (per-lane column loads make
// the L2 fetch the lines that straddle two shards twice: +12% DRAM reads, measured).  The chunk lands
// in VGPRs (up to 12 x 16 B per lane), is written to the wave's private LDS tile, and the next chunk's
// loads are issued before the current one is computed, so ~12 chunks (~135 KiB) are in flight per CU.
// Each lane computes 16-byte columns l and l + 64 of the MT output rows from LDS.  No barriers: the
// only LDS hazards are inside one wave (s_waitcnt lgkmcnt + wave barrier).
// ---------------------------------------------------------------------------------------------------
static constexpr int kWtLoads = 12;  // max 16-B loads per lane per chunk (12 KiB chunks)
typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));  // native vector: stays in VGPRs

struct WtArgs {
    const uint8_t *data, *parity;
    uint8_t *out;
    const uint8_t *enc, *rec;
    uint64_t pitch;
    uint32_t G, K, R, B;
    uint32_t rec_stride;
    uint32_t JS, nch;       // shards per chunk, chunks per group
    uint32_t Bs;            // staged row stride in LDS (B rounded up to 16)
    uint32_t cols;          // 16-B columns = ceil(B / 16) (<= 128)
    uint64_t bs_inv;        // ceil(2^32 / Bs)
};

// issue the loads of chunk c of group g into pf; `base` = this lane's shard base address for g (lane j
// holds shard j's), shuffled to the lanes that need it
template <bool DEC>
__device__ __forceinline__ void wt_issue(const WtArgs &a, u32x4_t (&pf)[kWtLoads], uint32_t g, uint32_t c, uint64_t base)
{
    const uint32_t K = a.K, lane = threadIdx.x;
    const uint32_t c0 = c * a.JS, nj = min(a.JS, K - c0), bytes = nj * a.Bs;
#pragma unroll
    for (int i = 0; i < kWtLoads; ++i) {
        const uint32_t o = i * 1024 + lane * 16;
        const uint32_t oc = min(o, bytes - 1);
        const uint32_t jj = (uint32_t)(((uint64_t)oc * a.bs_inv) >> 32), off = oc - jj * a.Bs;
        uint64_t sb;
        if (K <= 64) {
            sb = __shfl(base, (int)(c0 + jj));
        } else {
            uint32_t sid = c0 + jj;
            if constexpr (DEC) sid = a.rec[(uint64_t)g * a.rec_stride + 4 + c0 + jj];
            sb = reinterpret_cast<uint64_t>((sid < K) ? a.data + ((uint64_t)g * K + sid) * a.pitch
                                                      : a.parity + ((uint64_t)g * a.R + (sid - K)) * a.pitch);
        }
        if (o < bytes) pf[i] = *reinterpret_cast<const u32x4_t *>(reinterpret_cast<const uint8_t *>(sb) + off);
    }
}

template <int MT, bool DEC>
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(1, 4))) mac_wave_kernel(WtArgs a)
{
    using L = TileLayout<MT>;
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const uint32_t K = a.K, JS = a.JS, nch = a.nch, lane = threadIdx.x;
    uint8_t *tile = smem;                              // JS rows of Bs bytes
    uint8_t *tbl = smem + ((JS * a.Bs + 15) & ~15u);   // K x TBL coefficient tables
    const uint32_t K4 = (K + 3) & ~3u;

    auto rows_of = [&](uint32_t g) -> uint32_t {
        if constexpr (DEC) {
            const uint8_t *rec = a.rec + (uint64_t)g * a.rec_stride;
            return rec[0] == 0 ? min((uint32_t)MT, (uint32_t)rec[1]) : 0u;
        } else {
            return min((uint32_t)MT, a.R);
        }
    };
    auto next_group = [&](uint32_t g) -> uint32_t {
        if constexpr (DEC)
            while (g < a.G && rows_of(g) == 0) g += gridDim.x;
        return g;
    };
    // shard base addresses of group g, lane j holds shard j's (decode: the selected share)
    auto shard_base = [&](uint32_t g) -> uint64_t {
        uint64_t p = 0;
        if (lane < K) {
            uint32_t sid = lane;
            if constexpr (DEC) sid = a.rec[(uint64_t)g * a.rec_stride + 4 + lane];
            p = reinterpret_cast<uint64_t>((sid < K) ? a.data + ((uint64_t)g * K + sid) * a.pitch
                                                     : a.parity + ((uint64_t)g * a.R + (sid - K)) * a.pitch);
        }
        return p;
    };
    u32x4_t pf[kWtLoads];
    auto expand = [&](uint32_t g) {
        uint32_t m = a.R;
        const uint8_t *rec = nullptr;
        if constexpr (DEC) {
            rec = a.rec + (uint64_t)g * a.rec_stride;
            m = rec[1];
        }
        for (uint32_t e = lane; e < K * MT; e += 64) {
            const uint32_t r = e % MT, j = e / MT;
            uint32_t cf = 0;
            if constexpr (DEC) {
                if (r < m) cf = rec[4 + K4 * (1 + r) + j];
            } else {
                if (r < a.R) cf = a.enc[(uint64_t)(K + r) * K + j];
            }
            uint32_t t[5];
            gf_perm_tables(cf, t);
            *reinterpret_cast<uint4 *>(tbl + j * L::TBL + r * 16) = make_uint4(t[0], t[1], t[2], t[3]);
            reinterpret_cast<uint32_t *>(tbl + j * L::TBL + MT * 16)[r] = t[4];
        }
    };

    uint32_t g = next_group(blockIdx.x);
    if (g >= a.G) return;
    if constexpr (!DEC) expand(0);
    uint64_t base = shard_base(g);
    wt_issue<DEC>(a, pf, g, 0, base);
    uint32_t c = 0, rows = rows_of(g);
    uint32_t accw[2][MT][4];
#pragma unroll
    for (int p = 0; p < 2; ++p)
#pragma unroll
        for (int r = 0; r < MT; ++r)
#pragma unroll
            for (int w = 0; w < 4; ++w) accw[p][r][w] = 0;
    bool need_tables = DEC;
    while (true) {
        // the chunk in pf has landed (the compiler waits on first use): stage it into the LDS tile
        const uint32_t c0 = c * JS, nj = min(JS, K - c0), bytes = nj * a.Bs;
        __builtin_amdgcn_wave_barrier();
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // previous chunk's tile reads are done
#pragma unroll
        for (int i = 0; i < kWtLoads; ++i) {
            const uint32_t o = i * 1024 + lane * 16;
            if (o < bytes) *reinterpret_cast<u32x4_t *>(tile + o) = pf[i];
        }
        if (need_tables) {
            expand(g);
            need_tables = false;
        }
        // next unit, and its loads, before computing this one
        uint32_t gn = g, cn = c + 1;
        if (cn == nch) {
            cn = 0;
            gn = next_group(g + gridDim.x);
        }
        uint64_t nbase = base;
        if (gn < a.G) {
            if (gn != g) nbase = shard_base(gn);
            wt_issue<DEC>(a, pf, gn, cn, nbase);
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_wave_barrier();
        // compute chunk (g, c) from the tile
        for (uint32_t jj = 0; jj < nj; ++jj) {
            const uint8_t *tb = tbl + (c0 + jj) * L::TBL;
            uint4 tv[L::TBL / 16];
#pragma unroll
            for (int q = 0; q < L::TBL / 16; ++q) tv[q] = reinterpret_cast<const uint4 *>(tb)[q];
            const uint32_t *t4 = reinterpret_cast<const uint32_t *>(tv + MT);
#pragma unroll
            for (int p = 0; p < 2; ++p) {
                const uint32_t col = lane + 64 * p;
                if (p == 1 && col >= a.cols) break;
                const uint4 xv = *reinterpret_cast<const uint4 *>(tile + jj * a.Bs + col * 16);
                const uint32_t x[4] = {xv.x, xv.y, xv.z, xv.w};
#pragma unroll
                for (int w = 0; w < 4; ++w) {
                    const uint32_t s0 = x[w] & 0x07070707u, s1 = (x[w] >> 3) & 0x07070707u, s2 = (x[w] >> 6) & 0x03030303u;
#pragma unroll
                    for (int r = 0; r < MT; ++r) {
                        const uint32_t t[5] = {tv[r].x, tv[r].y, tv[r].z, tv[r].w, t4[r]};
#if KFEC_ABLATE == 1
                        accw[p][r][w] ^= x[w] ^ t[0];
                        (void)s0; (void)s1; (void)s2;
#else
                        accw[p][r][w] = perm_mac(accw[p][r][w], t, s0, s1, s2);
#endif
                    }
                }
            }
        }
        if (c + 1 == nch) {  // group done: store its rows, 16 B per lane and column
            const uint64_t obase = (uint64_t)g * a.R * a.pitch;
#pragma unroll
            for (int p = 0; p < 2; ++p) {
                const uint32_t col = lane + 64 * p;
                if (col < a.cols) {
#pragma unroll
                    for (int r = 0; r < MT; ++r)
                        if ((uint32_t)r < rows) {
                            __builtin_nontemporal_store(u32x4_t{accw[p][r][0], accw[p][r][1], accw[p][r][2], accw[p][r][3]},
                                                        reinterpret_cast<u32x4_t *>(a.out + obase + (uint64_t)r * a.pitch + col * 16));
                        }
                }
#pragma unroll
                for (int r = 0; r < MT; ++r)
#pragma unroll
                    for (int w = 0; w < 4; ++w) accw[p][r][w] = 0;
            }
            if (gn >= a.G) break;
            rows = rows_of(gn);
            need_tables = DEC;
        }
        g = gn;
        c = cn;
        base = nbase;
    }
}

// ---------------------------------------------------------------------------------------------------
// (A4/A5/A8/A11) stream engine: one persistent workgroup per CU, role-split waves.
//   loader waves (kEngNL) gather whole groups (or chunks of JS shards) into a kEngS-slot LDS ring with
//     LDS-DMA (global_load_lds_dwordx4, per-lane 16-B sources, 1 KiB of LDS per wave-instruction).
//     A group of 20 x 1440 B is 225 complete 128-B lines, so no line is fetched twice.  Each loader owns
//     units u = w, w + NL, ...: waits for the slot to be free, issues all its DMAs, waits vmcnt(0),
//     publishes the slot.  Several units are in flight per CU at any time.
//   consumer teams (2 x kEngTW waves) take alternate groups; each lane owns one 8-byte column and
//     accumulates its MT output rows over the group's chunks, then stores them (non-temporal).
//   Hand-off: LDS counters filled[s] (fill generation) and consumed[s] (consumer waves done), workgroup-
//   scope release/acquire.  Every spin is bounded: on timeout the wave sets a flag and leaves, so a bug
//   can never hang the GPU (outputs would then fail verification).
// ---------------------------------------------------------------------------------------------------
static constexpr int kEngS = 5;     // ring slots
static constexpr int kEngNL = 3;    // loader waves
static constexpr int kEngTW = 4;    // waves per consumer team (256 lanes: one 8-byte column each)
static constexpr int kEngThreads = (kEngNL + 2 * kEngTW) * 64;
static constexpr uint32_t kSpinMax = 1u << 22;

struct StreamArgs {
    const uint8_t *data, *parity;
    uint8_t *out;
    const uint8_t *enc, *rec;
    uint32_t *err;          // device word: set non-zero if a spin timed out
    uint64_t pitch;
    uint32_t G, K, R, B;
    uint32_t rec_stride;
    uint32_t JS, nch;       // shards per unit, units per group
    uint32_t Bs;            // LDS row stride (B rounded up to 16)
    uint32_t slot_bytes;    // JS * Bs rounded up to 1 KiB
    uint32_t cols;          // 8-byte columns = ceil(B / 8)
    uint64_t bs_inv;        // ceil(2^32 / Bs)
};

__device__ __forceinline__ uint32_t lds_load_acq(uint32_t *p)
{
    return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// wait until *p >= target; false on timeout
__device__ __forceinline__ bool spin_ge(uint32_t *p, uint32_t target)
{
    for (uint32_t i = 0; i < kSpinMax; ++i) {
        if (lds_load_acq(p) >= target) return true;
        __builtin_amdgcn_s_sleep(1);
    }
    return false;
}

template <int MT, bool DEC>
__global__ void __launch_bounds__(kEngThreads) mac_stream_kernel(StreamArgs a)
{
    using L = TileLayout<MT>;
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const uint32_t K = a.K, JS = a.JS, nch = a.nch;
    // LDS: [S slots][tables: encode K*TBL once | decode S*JS*TBL][filled[S], consumed[S]]
    const uint32_t tbl0 = kEngS * a.slot_bytes;
    const uint32_t tbl_bytes = DEC ? kEngS * JS * L::TBL : K * L::TBL;
    uint32_t *filled = reinterpret_cast<uint32_t *>(smem + tbl0 + tbl_bytes);
    uint32_t *consumed = filled + kEngS;

    if (threadIdx.x < kEngS) {
        filled[threadIdx.x] = 0;
        consumed[threadIdx.x] = 0;
    }
    if constexpr (!DEC) {  // encode tables of all K shards, once
        for (uint32_t e = threadIdx.x; e < K * MT; e += blockDim.x) {
            const uint32_t r = e % MT, j = e / MT;
            const uint32_t cf = (r < a.R) ? a.enc[(uint64_t)(K + r) * K + j] : 0u;
            uint32_t t[5];
            gf_perm_tables(cf, t);
            uint8_t *tb = smem + tbl0 + j * L::TBL;
            *reinterpret_cast<uint4 *>(tb + r * 16) = make_uint4(t[0], t[1], t[2], t[3]);
            reinterpret_cast<uint32_t *>(tb + MT * 16)[r] = t[4];
        }
    }
    __syncthreads();

    const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const uint32_t my_groups = a.G > blockIdx.x ? (a.G - blockIdx.x + gridDim.x - 1) / gridDim.x : 0;
    const uint32_t n_units = my_groups * nch;

    if (wave < kEngNL) {
        // ---------------- loader ----------------
        for (uint32_t u = wave; u < n_units; u += kEngNL) {
            const uint32_t k = u / nch, c = u - k * nch, g = blockIdx.x + k * gridDim.x;
            const uint32_t s = u % kEngS, f = u / kEngS;
            if (!spin_ge(&consumed[s], kEngTW * f)) {
                if (lane == 0) atomicOr(a.err, 1u);
                return;
            }
            const uint32_t c0 = c * JS, nj = min(JS, K - c0);
            [[maybe_unused]] uint8_t *slot = smem + s * a.slot_bytes;  // read only in the device pass
            bool work = true;
            const uint8_t *rec = nullptr;
            if constexpr (DEC) {
                rec = a.rec + (uint64_t)g * a.rec_stride;
                const uint32_t st = rec[0], m = rec[1];
                work = (st == 0 && m > 0);
                if (work) {
                    uint8_t *tb = smem + tbl0 + s * JS * L::TBL;
                    for (uint32_t e = lane; e < nj * MT; e += 64) {
                        const uint32_t r = e % MT, jj = e / MT;
                        const uint32_t cf = (r < m) ? rec[4 + ((K + 3) & ~3u) * (1 + r) + c0 + jj] : 0u;
                        uint32_t t[5];
                        gf_perm_tables(cf, t);
                        *reinterpret_cast<uint4 *>(tb + jj * L::TBL + r * 16) = make_uint4(t[0], t[1], t[2], t[3]);
                        reinterpret_cast<uint32_t *>(tb + jj * L::TBL + MT * 16)[r] = t[4];
                    }
                }
            }
            if (work) {
                // shard base addresses of this unit, one per lane (nj <= 64 is not required: lanes
                // beyond 64 shards fall back to a direct lookup), fetched with one coalesced load
                uint64_t my_base = 0;
                if constexpr (DEC) {
                    if (lane < nj) {
                        const uint32_t sid = rec[4 + c0 + lane];
                        my_base = reinterpret_cast<uint64_t>((sid < K) ? a.data + ((uint64_t)g * K + sid) * a.pitch
                                                                       : a.parity + ((uint64_t)g * a.R + (sid - K)) * a.pitch);
                    }
                }
                const uint32_t bytes = nj * a.Bs;
                for (uint32_t ch = 0; ch * 1024 < bytes; ++ch) {
                    const uint32_t o = ch * 1024 + lane * 16;
                    const uint32_t jj = (uint32_t)(((uint64_t)min(o, bytes - 1) * a.bs_inv) >> 32), off = o - jj * a.Bs;
                    (void)off;  // read only in the device pass
                    [[maybe_unused]] const uint8_t *src;
                    if constexpr (DEC) {
                        if (nj <= 64) {
                            src = reinterpret_cast<const uint8_t *>(__shfl(my_base, (int)jj));
                        } else {
                            const uint32_t sid = rec[4 + c0 + jj];
                            src = (sid < K) ? a.data + ((uint64_t)g * K + sid) * a.pitch
                                            : a.parity + ((uint64_t)g * a.R + (sid - K)) * a.pitch;
                        }
                    } else {
                        src = a.data + ((uint64_t)g * K + c0 + jj) * a.pitch;
                    }
                    if (o < bytes) {
#if defined(__HIP_DEVICE_COMPILE__)
                        __builtin_amdgcn_global_load_lds(src + off, (__attribute__((address_space(3))) void *)(slot + ch * 1024),
                                                         16, 0, 0);
#endif
                    }
                }
            }
            asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
            if (lane == 0) __hip_atomic_store(&filled[s], f + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        return;
    }
    // ---------------- consumer ----------------
    const uint32_t team = (wave - kEngNL) / kEngTW, tw = (wave - kEngNL) % kEngTW;
    const uint32_t col = tw * 64 + lane;
    for (uint32_t k = team; k < my_groups; k += 2) {
        const uint32_t g = blockIdx.x + k * gridDim.x;
        uint32_t rows;
        if constexpr (DEC) {
            const uint8_t *rec = a.rec + (uint64_t)g * a.rec_stride;
            const uint32_t st = rec[0], m = rec[1];
            rows = (st == 0) ? min((uint32_t)MT, m) : 0u;
        } else {
            rows = min((uint32_t)MT, a.R);
        }
        u32x2_t acc[MT];
#pragma unroll
        for (int r = 0; r < MT; ++r) acc[r] = u32x2_t{0u, 0u};
        for (uint32_t c = 0; c < nch; ++c) {
            const uint32_t u = k * nch + c, s = u % kEngS, f = u / kEngS;
            if (!spin_ge(&filled[s], f + 1)) {
                if (lane == 0) atomicOr(a.err, 2u);
                return;
            }
            const uint32_t c0 = c * JS, nj = min(JS, K - c0);
            if (rows && col < a.cols) {
                const uint8_t *xs = smem + s * a.slot_bytes + col * 8;
                const uint8_t *tb = DEC ? smem + tbl0 + s * JS * L::TBL : smem + tbl0 + c0 * L::TBL;
                // software pipeline: shard jj+1's data and tables are read while shard jj is computed
                // (2 waves per SIMD cannot hide LDS latency by themselves)
                u32x2_t xn = *reinterpret_cast<const u32x2_t *>(xs);
                uint4 tn[L::TBL / 16];
#pragma unroll
                for (int q = 0; q < L::TBL / 16; ++q) tn[q] = reinterpret_cast<const uint4 *>(tb)[q];
                for (uint32_t jj = 0; jj < nj; ++jj) {
                    const u32x2_t x = xn;
                    uint4 tc[L::TBL / 16];
#pragma unroll
                    for (int q = 0; q < L::TBL / 16; ++q) tc[q] = tn[q];
                    if (jj + 1 < nj) {
                        xn = *reinterpret_cast<const u32x2_t *>(xs + (jj + 1) * a.Bs);
#pragma unroll
                        for (int q = 0; q < L::TBL / 16; ++q)
                            tn[q] = reinterpret_cast<const uint4 *>(tb + (jj + 1) * L::TBL)[q];
                    }
                    tile_mac_regs<MT>(acc, x, tc);
                }
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            if (lane == 0) __hip_atomic_fetch_add(&consumed[s], 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        if (rows && col < a.cols) {
            uint8_t *o = a.out + ((uint64_t)g * a.R) * a.pitch + (uint64_t)col * 8;
#pragma unroll
            for (int r = 0; r < MT; ++r)
                if ((uint32_t)r < rows) __builtin_nontemporal_store(acc[r], reinterpret_cast<u32x2_t *>(o + (uint64_t)r * a.pitch));
        }
    }
}

// ---------------------------------------------------------------------------------------------------
// host-side launch helpers
// ---------------------------------------------------------------------------------------------------
static int pick_vec(size_t pitch, std::initializer_list<const void *> ptrs)
{
#if KFEC_VEC32
    {
        bool ok = (pitch % 32) == 0;
        for (const void *p : ptrs) ok = ok && (reinterpret_cast<uintptr_t>(p) % 16) == 0;
        if (ok) return 32;
    }
#endif
    for (int v : {16, 8, 4}) {
        bool ok = (pitch % v) == 0;
        for (const void *p : ptrs) ok = ok && (reinterpret_cast<uintptr_t>(p) % v) == 0;
        if (ok) return v;
    }
    return 1;
}

// granule of the flattened kernel: 32 B whenever the pitch and every base pointer are dword aligned (the
// tail granule of a row is loaded / stored dword by dword), bytewise otherwise
static int pick_vec_mac(size_t pitch, std::initializer_list<const void *> ptrs)
{
    bool ok = (pitch % 4) == 0;
    for (const void *p : ptrs) ok = ok && (reinterpret_cast<uintptr_t>(p) % 4) == 0;
#if KFEC_VEC32
    return ok ? 32 : 1;
#else
    return ok ? 16 : 1;
#endif
}

// resident 256-thread blocks per CU for a kernel (occupancy API, capped at 8: MI355X_MICROARCH.md
// "Residency": the API can over-report by one for SGPR-heavy kernels; ours stay below 80 SGPRs)
static int env_int(const char *name, int dflt)
{
    const char *e = getenv(name);
    return e && *e ? atoi(e) : dflt;
}

static int resident_blocks(const void *kernel, size_t lds)
{
    static const int cap = std::max(1, std::min(8, env_int("KFEC_BLOCKS", 8)));
    int n = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, kernel, kBlock, lds) != hipSuccess || n <= 0) n = 1;
    return std::min(n, cap);
}

static int pick_mt(int R) { return R <= 4 ? std::max(R, 1) : 8; }

// (granule bytes, output rows per tile) of the flattened kernel: the widest granule and MT = min(R, 8)
// rows.  Measured at 200:55: taller tiles on narrower granules (16 x 16 B, 32 x 8 B) read each
// input byte fewer times but are no faster -- the re-reads hit L2 and the kernel is VALU-bound there,
// where 32-B granules amortise each table read over the most bytes.  KFEC_MT / KFEC_VEC override.
static void mac_shape(int R, int vec_max, int &vec, int &mt)
{
    static const int mt_env = env_int("KFEC_MT", 0), vec_env = env_int("KFEC_VEC", 0);
    vec = vec_max;
    mt = pick_mt(R);
    if (mt_env == 1 || mt_env == 2 || mt_env == 3 || mt_env == 4 || mt_env == 8) mt = mt_env;
    if (vec_env > 0 && vec_env <= vec_max && (vec_env & (vec_env - 1)) == 0) vec = vec_env;
}

// KFEC_PAD=1: pad a group's items to whole waves, so one wave-instruction reads a whole shard row and
// both halves of every 128-B line that straddles two shards are read by consecutive instructions
static size_t pad_cols(size_t cols)
{
    static const bool on = [] {
        const char *e = getenv("KFEC_PAD");
        return e && std::string(e) == "1";
    }();
    return on ? (cols + 63) / 64 * 64 : cols;
}

template <int VEC, int MT, bool DEC, int PDX = 0>
static int run_mac(const DeviceInfo &di, MacArgs a, int tiles, hipStream_t s)
{
    using L = MacLayout<MT>;
    const size_t lds = a.etab ? 0 : (size_t)a.gmax * a.JC * L::ENTRY;
    // one workgroup per 256 items (non-persistent): the dispatcher refills each CU as workgroups retire.
    // Measured against a persistent grid sized to the resident workgroups (KFEC_GRID_PERSIST=1): encode
    // 6.90 -> 6.08 ms and decode 7.39 -> 6.75 ms at 20:3 B=1440 1M groups, 205 -> 173 ms encode at 200:55
    // (DESIGN.md 5).  With several row tiles the grid's x extent stays a multiple of the 8 XCDs, so
    // workgroups (x, y) and (x, y') share an XCD and the tiles' re-reads of the same shard bytes hit its L2.
    const uint32_t want = (a.total + kMacBlock - 1) / kMacBlock;
    static const int persist = env_int("KFEC_GRID_PERSIST", 0);
    uint32_t gx = want;
    if (persist) {
        uint32_t cap = (uint32_t)(std::max(1, di.cus) * resident_blocks((const void *)mac_kernel<VEC, MT, DEC, PDX>, lds))
                       / (uint32_t)std::max(1, tiles);
        if (tiles > 1 && cap >= 8) cap &= ~7u;
        gx = std::min(want, std::max(cap, 1u));
    } else if (tiles > 1) {
        gx = (want + 7) & ~7u;
    }
    gx = std::max(1u, gx);
    hipLaunchKernelGGL((mac_kernel<VEC, MT, DEC, PDX>), dim3(gx, tiles), dim3(kMacBlock), lds, s, a);
    return hipGetLastError() == hipSuccess ? 0 : -3;
}

// Batches of at most kLatencyGroups groups (the single-group drop-in calls, whose shares sit in pinned host
// memory) run the MAC with 4-byte granules and 16 shards in flight per lane: ~8x more lanes and loads in
// flight than the streaming shape, so the PCIe round trips of a 29 KB group overlap instead of queueing.
constexpr int kLatencyVec = -4;
constexpr size_t kLatencyGroups = 4;

template <bool DEC>
static int dispatch_mac(const DeviceInfo &di, int vec, int mt, MacArgs a, int tiles, hipStream_t s)
{
#define KFEC_MT_CASES(V)                                                     \
    switch (mt) {                                                            \
    case 1: return run_mac<V, 1, DEC>(di, a, tiles, s);                      \
    case 2: return run_mac<V, 2, DEC>(di, a, tiles, s);                      \
    case 3: return run_mac<V, 3, DEC>(di, a, tiles, s);                      \
    case 4: return run_mac<V, 4, DEC>(di, a, tiles, s);                      \
    default: return run_mac<V, 8, DEC>(di, a, tiles, s);                     \
    }
    if (vec == kLatencyVec) {  // the latency shape: dword granules, 16 shards in flight per lane
        switch (mt) {
        case 1: return run_mac<4, 1, DEC, 16>(di, a, tiles, s);
        case 2: return run_mac<4, 2, DEC, 16>(di, a, tiles, s);
        case 3: return run_mac<4, 3, DEC, 16>(di, a, tiles, s);
        case 4: return run_mac<4, 4, DEC, 16>(di, a, tiles, s);
        default: return run_mac<4, 8, DEC, 16>(di, a, tiles, s);
        }
    }
    switch (vec) {
#if KFEC_VEC32
    case 32: KFEC_MT_CASES(32)
#endif
    case 16: KFEC_MT_CASES(16)
    case 8: KFEC_MT_CASES(8)
    case 4: KFEC_MT_CASES(4)
    default: KFEC_MT_CASES(1)
    }
#undef KFEC_MT_CASES
}

static int entry_bytes(int mt)
{
    switch (mt) {
    case 1: return MacLayout<1>::ENTRY;
    case 2: return MacLayout<2>::ENTRY;
    case 3: return MacLayout<3>::ENTRY;
    case 4: return MacLayout<4>::ENTRY;
    default: return MacLayout<8>::ENTRY;
    }
}

static constexpr size_t kLdsBudget = 32 * 1024;
static constexpr size_t kTileLdsBudget = 31 * 1024;  // 5 workgroups per CU (160 KiB of LDS)

// group-tile kernel for shards up to 2 KiB (one 8-byte column per lane of a 256-lane workgroup) and
// < 2^32 groups; larger shards take the flattened kernel
// Measured slower than the flattened kernel on MI355X once the GF math is in (DESIGN.md "kernel
// architecture"), so it is opt-in: KFEC_KERNEL=tile.
static bool use_tile_path(size_t G, size_t B)
{
    static const bool on = [] {
        const char *e = getenv("KFEC_KERNEL");
        return e && std::string(e) == "tile";
    }();
    return on && B <= 2048 && G < 0xFFFFFFFFull;
}

template <int MT, bool DEC, int SV>
static int run_tile(const DeviceInfo &di, LdsArgs a, int tiles, hipStream_t s)
{
    using L = TileLayout<MT>;
    a.Bs = (a.B + 15) & ~15u;
    a.cols = (a.B + 7) / 8;
    a.bs_inv = ((1ull << 32) + a.Bs - 1) / a.Bs;
    // 2-deep ring of JS-shard chunks (+ their tables) within the per-workgroup LDS budget; encode keeps
    // all K shards' tables resident when they are small
    const size_t all_tbl = (size_t)a.K * L::TBL;
    a.tbl_all = (!DEC && all_tbl <= 4096) ? 1u : 0u;
    const size_t per_row = 2 * (size_t)a.Bs + (a.tbl_all ? 0 : 2 * (size_t)L::TBL);
    const size_t budget = kTileLdsBudget - (a.tbl_all ? all_tbl : 0);
    const size_t nch = std::max<size_t>(1, (a.K * per_row + budget - 1) / budget);
    a.JS = (uint32_t)((a.K + nch - 1) / nch);
    const size_t lds = (size_t)a.JS * per_row + (a.tbl_all ? all_tbl : 0);
    const uint32_t threads = 256;
    int occ = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, (const void *)mac_tile_kernel<MT, DEC, SV>, threads, lds) !=
            hipSuccess || occ <= 0)
        occ = 1;
    const uint32_t cap = (uint32_t)std::max(1, di.cus * std::min(occ, 8) / std::max(1, tiles));
    const uint32_t gx = std::max(1u, std::min<uint32_t>(a.G, cap));
    hipLaunchKernelGGL((mac_tile_kernel<MT, DEC, SV>), dim3(gx, tiles), dim3(threads), lds, s, a);
    return hipGetLastError() == hipSuccess ? 0 : -3;
}

// ---- wave-tile launch ----
[[maybe_unused]] static constexpr size_t kWtLdsMax = 13 * 1024;  // 12 waves (workgroups) per CU fit in 160 KiB

struct WtPlan {
    bool ok = false;
    uint32_t JS = 0, nch = 0, Bs = 0;
    size_t lds = 0;
};

static WtPlan plan_wave(uint32_t K, uint32_t R, uint32_t B, int mt)
{
    WtPlan p;
    if (B == 0 || B > 2048 || R == 0 || R > (uint32_t)mt) return p;
    const uint32_t tbl = (uint32_t)(mt * 16 + (mt + 3) / 4 * 16);
    p.Bs = (B + 15) & ~15u;
    const uint32_t cap = (uint32_t)std::min<size_t>(K, (size_t)kWtLoads * 1024 / p.Bs);
    if (cap == 0) return p;
    // prefer chunks that are whole 128-B lines (e.g. 8 x 1440 B = 90 lines), else the largest
    uint32_t js = cap;
    for (uint32_t j = cap; j >= 1; --j)
        if ((j * p.Bs) % 128 == 0 && 2 * j >= cap) {
            js = j;
            break;
        }
    p.JS = js;
    p.nch = (K + js - 1) / js;
    p.lds = ((size_t)js * p.Bs + 15) / 16 * 16 + (size_t)K * tbl;
    p.ok = p.lds <= 64 * 1024;
    return p;
}

template <int MT, bool DEC>
static int run_wave(const DeviceInfo &di, WtArgs a, const WtPlan &p, hipStream_t s)
{
    a.JS = p.JS;
    a.nch = p.nch;
    a.Bs = p.Bs;
    a.cols = (a.B + 15) / 16;
    a.bs_inv = ((1ull << 32) + a.Bs - 1) / a.Bs;
    int occ = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, (const void *)mac_wave_kernel<MT, DEC>, 64, p.lds) !=
            hipSuccess || occ <= 0)
        occ = 1;
    const uint32_t gx = std::max(1u, std::min<uint32_t>(a.G, (uint32_t)std::max(1, di.cus * std::min(occ, 32))));
    hipLaunchKernelGGL((mac_wave_kernel<MT, DEC>), dim3(gx), dim3(64), p.lds, s, a);
    return hipGetLastError() == hipSuccess ? 0 : -3;
}

template <bool DEC>
static int dispatch_wave(const DeviceInfo &di, WtArgs a, const WtPlan &p, int mt, hipStream_t s)
{
    switch (mt) {
    case 1: return run_wave<1, DEC>(di, a, p, s);
    case 2: return run_wave<2, DEC>(di, a, p, s);
    case 3: return run_wave<3, DEC>(di, a, p, s);
    case 4: return run_wave<4, DEC>(di, a, p, s);
    default: return run_wave<8, DEC>(di, a, p, s);
    }
}

static bool wave_enabled()
{
    static const bool on = [] {
        const char *e = getenv("KFEC_KERNEL");
        return e && std::string(e) == "wave";
    }();
    return on;
}

// ---- stream engine launch ----
static constexpr size_t kEngLdsMax = 160 * 1024 - 1024;

struct EngPlan {
    bool ok = false;
    uint32_t JS = 0, nch = 0, Bs = 0, slot_bytes = 0;
    size_t lds = 0;
};

static EngPlan plan_stream(uint32_t K, uint32_t R, uint32_t B, int mt, bool dec)
{
    EngPlan p;
    if (B == 0 || B > 2048 || R == 0 || R > (uint32_t)mt) return p;
    const uint32_t tbl = (uint32_t)(mt * 16 + (mt + 3) / 4 * 16);
    p.Bs = (B + 15) & ~15u;
    const size_t enc_tbl = dec ? 0 : (size_t)K * tbl;
    if (enc_tbl + 64 >= kEngLdsMax) return p;
    for (uint32_t js = std::min<uint32_t>(K, (32 * 1024) / p.Bs); js >= 1; --js) {
        const uint32_t slot = ((js * p.Bs + 1023) / 1024) * 1024;
        const size_t lds = (size_t)kEngS * (slot + (dec ? (size_t)js * tbl : 0)) + enc_tbl + 64;
        if (lds <= kEngLdsMax) {
            p.ok = true;
            p.JS = js;
            p.nch = (K + js - 1) / js;
            p.slot_bytes = slot;
            p.lds = lds;
            return p;
        }
    }
    return p;
}

template <int MT, bool DEC>
static int run_stream(const DeviceInfo &di, StreamArgs a, const EngPlan &p, hipStream_t s)
{
    static bool attr_set = false;  // per instantiation: allow > 64 KiB of dynamic LDS
    if (!attr_set) {
        if (hipFuncSetAttribute((const void *)mac_stream_kernel<MT, DEC>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)kEngLdsMax) != hipSuccess)
            return -3;
        attr_set = true;
    }
    a.JS = p.JS;
    a.nch = p.nch;
    a.Bs = p.Bs;
    a.slot_bytes = p.slot_bytes;
    a.cols = (a.B + 7) / 8;
    a.bs_inv = ((1ull << 32) + a.Bs - 1) / a.Bs;
    const uint32_t gx = std::max(1u, std::min<uint32_t>(a.G, (uint32_t)std::max(1, di.cus)));
    hipLaunchKernelGGL((mac_stream_kernel<MT, DEC>), dim3(gx), dim3(kEngThreads), p.lds, s, a);
    return hipGetLastError() == hipSuccess ? 0 : -3;
}

template <bool DEC>
static int dispatch_stream(const DeviceInfo &di, StreamArgs a, const EngPlan &p, int mt, hipStream_t s)
{
    switch (mt) {
    case 1: return run_stream<1, DEC>(di, a, p, s);
    case 2: return run_stream<2, DEC>(di, a, p, s);
    case 3: return run_stream<3, DEC>(di, a, p, s);
    case 4: return run_stream<4, DEC>(di, a, p, s);
    default: return run_stream<8, DEC>(di, a, p, s);
    }
}

// the stream engine serves layouts with 16-B aligned slots, B <= 2 KiB and R <= 8 (one row tile).
// Measured slower than the flattened kernel (its LDS ring holds ~3 groups in flight per CU, the
// flattened kernel's VGPRs ~4x that), so it is opt-in: KFEC_KERNEL=engine.
static bool stream_enabled()
{
    static const bool on = [] {
        const char *e = getenv("KFEC_KERNEL");
        return e && std::string(e) == "engine";
    }();
    return on;
}

template <bool DEC>
static int dispatch_tile(const DeviceInfo &di, int sv, LdsArgs a, hipStream_t g_stream)
{
    const int mt = a.R <= 4 ? std::max<int>(a.R, 1) : 8;
    const int tiles = ((int)a.R + mt - 1) / mt;
    if (sv > 16) sv = 16;
#define KFEC_TILE_MT(SV)                                                           \
    switch (mt) {                                                                  \
    case 1: return run_tile<1, DEC, SV>(di, a, tiles, g_stream);                   \
    case 2: return run_tile<2, DEC, SV>(di, a, tiles, g_stream);                   \
    case 3: return run_tile<3, DEC, SV>(di, a, tiles, g_stream);                   \
    case 4: return run_tile<4, DEC, SV>(di, a, tiles, g_stream);                   \
    default: return run_tile<8, DEC, SV>(di, a, tiles, g_stream);                  \
    }
    switch (sv) {
    case 16: KFEC_TILE_MT(16)
    case 8: KFEC_TILE_MT(8)
    case 4: KFEC_TILE_MT(4)
    default: KFEC_TILE_MT(1)
    }
#undef KFEC_TILE_MT
}
static constexpr size_t kMaxItemsPerLaunch = 0x7FFFFFFFu;

// split G into launches whose item count fits 32-bit indexing
template <typename F>
static int for_group_ranges(size_t G, size_t cols, F &&f)
{
    const size_t gmax_launch = std::max<size_t>(1, kMaxItemsPerLaunch / std::max<size_t>(cols, 1));
    for (size_t g0 = 0; g0 < G; g0 += gmax_launch) {
        const int rc = f(g0, std::min(gmax_launch, G - g0));
        if (rc) return rc;
    }
    return 0;
}

int launch_encode(const DeviceInfo &di, const uint8_t *d_enc, int K, int N, size_t G, size_t B, size_t pitch,
                  const void *d_data, void *d_parity, hipStream_t s)
{
    const int R = N - K;
    if (R == 0 || G == 0 || B == 0) return 0;
    if (use_tile_path(G, B)) {
        LdsArgs a{};
        a.data = static_cast<const uint8_t *>(d_data);
        a.out = static_cast<uint8_t *>(d_parity);
        a.enc = d_enc;
        a.pitch = pitch;
        a.G = (uint32_t)G; a.K = K; a.R = R; a.B = (uint32_t)B;
        return dispatch_tile<false>(di, pick_vec(pitch, {d_data, d_parity}), a, s);
    }
    if (wave_enabled() && G < 0xFFFFFFFFull && pick_vec(pitch, {d_data, d_parity}) >= 16) {
        const int mt = pick_mt(R);
        const WtPlan p = plan_wave(K, R, (uint32_t)B, mt);
        if (p.ok) {
            WtArgs a{};
            a.data = static_cast<const uint8_t *>(d_data);
            a.out = static_cast<uint8_t *>(d_parity);
            a.enc = d_enc;
            a.pitch = pitch;
            a.G = (uint32_t)G; a.K = K; a.R = R; a.B = (uint32_t)B;
            return dispatch_wave<false>(di, a, p, mt, s);
        }
    }
    if (stream_enabled() && G < 0xFFFFFFFFull && pick_vec(pitch, {d_data, d_parity}) >= 16) {
        const int mt = pick_mt(R);
        const EngPlan p = plan_stream(K, R, (uint32_t)B, mt, false);
        if (p.ok) {
            StreamArgs a{};
            a.data = static_cast<const uint8_t *>(d_data);
            a.out = static_cast<uint8_t *>(d_parity);
            a.enc = d_enc;
            a.err = g_err_word();
            a.pitch = pitch;
            a.G = (uint32_t)G; a.K = K; a.R = R; a.B = (uint32_t)B;
            return dispatch_stream<false>(di, a, p, mt, s);
        }
    }
    int vec = 0, mt = 0;
    mac_shape(R, pick_vec_mac(pitch, {d_data, d_parity}), vec, mt);
    if (G <= kLatencyGroups && vec >= 4) vec = kLatencyVec;
    const int vb = vec >= 4 ? vec : 4;
    const size_t cols = (B + vb - 1) / vb, cpad = pad_cols(cols);
    const int tiles = (R + mt - 1) / mt;
    const size_t ent = entry_bytes(mt);
    const uint32_t JC = (uint32_t)std::max<size_t>(1, std::min<size_t>(K, kLdsBudget / ent));
    return for_group_ranges(G, cpad, [&](size_t g0, size_t gn) {
        MacArgs a{};
        a.data = static_cast<const uint8_t *>(d_data) + g0 * K * pitch;
        a.parity = nullptr;
        a.out = static_cast<uint8_t *>(d_parity) + g0 * R * pitch;
        a.enc = d_enc;
        a.rec = nullptr;
        a.pitch = pitch;
        a.total = (uint32_t)(gn * cpad);
        a.cols = (uint32_t)cols;
        a.cpad = (uint32_t)cpad;
        a.G = (uint32_t)gn;
        a.K = K; a.R = R; a.B = (uint32_t)B;
        a.rec_stride = 0;
        a.JC = JC;
        a.gmax = 1;
        static const int stab = env_int("KFEC_SGPR_TABLES", KFEC_SGPR_TABLES);
        if (stab) {
            a.etab = reinterpret_cast<const uint32_t *>(d_enc + enc_tab_offset(K, K + R));
            a.etab_rows = (uint32_t)enc_tab_rows(R);
            a.JC = K;
        }
        return dispatch_mac<false>(di, vec, mt, a, tiles, s);
    });
}

// Work list of the decode MAC: the groups whose decode has work (status OK and at least one data shard
// missing).  A group with nothing lost -- the common case on a live link, where fec_find_missings decodes
// every group that reached K shares (client.cpp:924-925) -- then costs the MAC kernel nothing.  Ballot per
// wave, one atomic per wave: groups are ascending within a wave, waves land in any order.
__global__ void __launch_bounds__(kBlock) compact_kernel(uint64_t G, uint32_t R, const uint8_t *status,
                                                         const uint8_t *out_idx, uint32_t *count, uint32_t *list)
{
    const uint64_t g = blockIdx.x * (uint64_t)kBlock + threadIdx.x;
    const bool active = g < G && status[g] == 0 && out_idx[g * R] != 0xFF;
    const uint64_t mask = __ballot(active);
    const uint32_t lane = threadIdx.x & 63u;
    uint32_t base = 0;
    if (lane == 0 && mask) base = atomicAdd(count, (uint32_t)__popcll(mask));
    base = __shfl(base, 0);
    if (active) list[base + __popcll(mask & ((1ull << lane) - 1ull))] = (uint32_t)g;
}

// decode_prep_*: share selection, the m x m solve and the coefficient rows of every group into the decode
// records of d_workspace (+ d_out_idx, d_status).  The MAC kernels (here and kfec_frame.hip) consume them.
int launch_decode_prep(const DeviceInfo &di, const uint8_t *d_enc, int K, int N, size_t G, const uint64_t *d_present,
                       uint8_t *d_out_idx, uint8_t *d_status, void *d_workspace, hipStream_t s)
{
    const int R = N - K;
    if (G == 0) return 0;
    uint8_t *rec = static_cast<uint8_t *>(d_workspace);
    const size_t rs = record_stride(K, R);
    PrepArgs p{};
    p.present = d_present;
    p.enc = d_enc;
    p.rec = rec;
    p.out_idx = d_out_idx;
    p.status = d_status;
    p.G = G;
    p.K = K; p.N = N; p.R = R;
    p.rec_stride = (uint32_t)rs;
    const int mmax = std::min(K, R);
    if (mmax <= 8) {
        const size_t lds = 768 + (size_t)R * K;
        // one thread per group: the per-group work is a chain of dependent LDS lookups, so latency is hidden
        // by having many groups in flight, not by looping
        const uint32_t blocks = (uint32_t)std::max<size_t>(1, std::min<size_t>((G + kBlock - 1) / kBlock,
                                                                                (size_t)std::max(di.cus, 1) * 64));
        const size_t lds4 = 768 + (size_t)R * (((size_t)K + 3) & ~size_t(3));
        if (mmax == 1) hipLaunchKernelGGL((decode_prep_perm<1>), dim3(blocks), dim3(kBlock), lds4, s, p);
        else if (mmax == 2) hipLaunchKernelGGL((decode_prep_perm<2>), dim3(blocks), dim3(kBlock), lds4, s, p);
        else if (mmax == 3) hipLaunchKernelGGL((decode_prep_perm<3>), dim3(blocks), dim3(kBlock), lds4, s, p);
        else if (mmax == 4) hipLaunchKernelGGL((decode_prep_perm<4>), dim3(blocks), dim3(kBlock), lds4, s, p);
        else hipLaunchKernelGGL((decode_prep_small<8>), dim3(blocks), dim3(kBlock), lds, s, p);
    } else {
        int occ = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, (const void *)decode_prep_lagrange, kPrepThreads, 0) !=
                hipSuccess || occ <= 0)
            occ = 1;
        const uint32_t blocks = (uint32_t)std::max<size_t>(1, std::min<size_t>(G, (size_t)std::max(di.cus, 1) * occ));
        hipLaunchKernelGGL(decode_prep_lagrange, dim3(blocks), dim3(kPrepThreads), 0, s, p);
    }
    return hipGetLastError() == hipSuccess ? 0 : -3;
}

int launch_decode(const DeviceInfo &di, const uint8_t *d_enc, int K, int N, size_t G, size_t B, size_t pitch,
                  const void *d_data, const void *d_parity, const uint64_t *d_present, void *d_out,
                  uint8_t *d_out_idx, uint8_t *d_status, void *d_workspace, hipStream_t s)
{
    const int R = N - K;
    if (G == 0) return 0;
    uint8_t *rec = static_cast<uint8_t *>(d_workspace);
    const size_t rs = record_stride(K, R);
    if (launch_decode_prep(di, d_enc, K, N, G, d_present, d_out_idx, d_status, d_workspace, s)) return -3;
    if (R == 0 || B == 0) return 0;
    if (use_tile_path(G, B)) {
        LdsArgs a{};
        a.data = static_cast<const uint8_t *>(d_data);
        a.parity = static_cast<const uint8_t *>(d_parity);
        a.out = static_cast<uint8_t *>(d_out);
        a.enc = d_enc;
        a.rec = rec;
        a.pitch = pitch;
        a.G = (uint32_t)G; a.K = K; a.R = R; a.B = (uint32_t)B;
        a.rec_stride = (uint32_t)rs;
        return dispatch_tile<true>(di, pick_vec(pitch, {d_data, d_parity, d_out}), a, s);
    }
    if (wave_enabled() && G < 0xFFFFFFFFull && pick_vec(pitch, {d_data, d_parity, d_out}) >= 16) {
        const int mt = pick_mt(R);
        const WtPlan p = plan_wave(K, R, (uint32_t)B, mt);
        if (p.ok) {
            WtArgs a{};
            a.data = static_cast<const uint8_t *>(d_data);
            a.parity = static_cast<const uint8_t *>(d_parity);
            a.out = static_cast<uint8_t *>(d_out);
            a.enc = d_enc;
            a.rec = rec;
            a.pitch = pitch;
            a.G = (uint32_t)G; a.K = K; a.R = R; a.B = (uint32_t)B;
            a.rec_stride = (uint32_t)rs;
            return dispatch_wave<true>(di, a, p, mt, s);
        }
    }
    if (stream_enabled() && G < 0xFFFFFFFFull && pick_vec(pitch, {d_data, d_parity, d_out}) >= 16) {
        const int mt = pick_mt(R);
        const EngPlan p = plan_stream(K, R, (uint32_t)B, mt, true);
        if (p.ok) {
            StreamArgs a{};
            a.data = static_cast<const uint8_t *>(d_data);
            a.parity = static_cast<const uint8_t *>(d_parity);
            a.out = static_cast<uint8_t *>(d_out);
            a.enc = d_enc;
            a.rec = rec;
            a.err = g_err_word();
            a.pitch = pitch;
            a.G = (uint32_t)G; a.K = K; a.R = R; a.B = (uint32_t)B;
            a.rec_stride = (uint32_t)rs;
            return dispatch_stream<true>(di, a, p, mt, s);
        }
    }

    int vec = 0, mt = 0;
    mac_shape(R, pick_vec_mac(pitch, {d_data, d_parity, d_out}), vec, mt);
    if (G <= kLatencyGroups && vec >= 4) vec = kLatencyVec;
    const int vb = vec >= 4 ? vec : 4;
    const size_t cols = (B + vb - 1) / vb, cpad = pad_cols(cols);
    const int tiles = (R + mt - 1) / mt;
    const size_t ent = entry_bytes(mt);
    // Work-list mode (KFEC_DECODE_LIST=1) measured slower on the benchmark configs, where >= 91% of the groups
    // lost data: 20:3 decode 6.84 -> 7.35 ms, 10:3 random 3.59 -> 3.75 ms (the list lookup is one more
    // dependent load at the head of every workgroup, and wave-order compaction scatters neighbouring groups).
    // It is kept for batches where most groups lost nothing.
    static const int use_list = env_int("KFEC_DECODE_LIST", 0);
    if (use_list && G * cpad <= kMaxItemsPerLaunch) {
        uint32_t *count = reinterpret_cast<uint32_t *>(rec + decode_list_offset(G, K, R));
        uint32_t *list = count + 16;
        if (hipMemsetAsync(count, 0, sizeof(uint32_t), s) != hipSuccess) return -3;
        hipLaunchKernelGGL(compact_kernel, dim3((uint32_t)((G + kBlock - 1) / kBlock)), dim3(kBlock), 0, s, (uint64_t)G,
                           (uint32_t)R, d_status, d_out_idx, count, list);
        if (hipGetLastError() != hipSuccess) return -3;
        const uint32_t gmax = (uint32_t)std::min<size_t>(G, (kMacBlock - 1) / cpad + 2);
        const uint32_t JC = (uint32_t)std::max<size_t>(1, std::min<size_t>(K, kLdsBudget / (ent * gmax)));
        MacArgs a{};
        a.data = static_cast<const uint8_t *>(d_data);
        a.parity = static_cast<const uint8_t *>(d_parity);
        a.out = static_cast<uint8_t *>(d_out);
        a.enc = d_enc;
        a.rec = rec;
        a.pitch = pitch;
        a.total = (uint32_t)(G * cpad);  // grid size: every group could have work
        a.cols = (uint32_t)cols;
        a.cpad = (uint32_t)cpad;
        a.G = (uint32_t)G;
        a.K = K; a.R = R; a.B = (uint32_t)B;
        a.rec_stride = (uint32_t)rs;
        a.JC = JC;
        a.gmax = gmax;
        a.list = list;
        a.list_count = count;
        return dispatch_mac<true>(di, vec, mt, a, tiles, s);
    }
    return for_group_ranges(G, cpad, [&](size_t g0, size_t gn) {
        const uint32_t gmax = (uint32_t)std::min<size_t>(gn, (kMacBlock - 1) / cpad + 2);
        const uint32_t JC = (uint32_t)std::max<size_t>(1, std::min<size_t>(K, kLdsBudget / (ent * gmax)));
        MacArgs a{};
        a.data = static_cast<const uint8_t *>(d_data) + g0 * K * pitch;
        a.parity = static_cast<const uint8_t *>(d_parity) + g0 * R * pitch;
        a.out = static_cast<uint8_t *>(d_out) + g0 * R * pitch;
        a.enc = d_enc;
        a.rec = rec + g0 * rs;
        a.pitch = pitch;
        a.total = (uint32_t)(gn * cpad);
        a.cols = (uint32_t)cols;
        a.cpad = (uint32_t)cpad;
        a.G = (uint32_t)gn;
        a.K = K; a.R = R; a.B = (uint32_t)B;
        a.rec_stride = (uint32_t)rs;
        a.JC = JC;
        a.gmax = gmax;
        return dispatch_mac<true>(di, vec, mt, a, tiles, s);
    });
}

// ---------------------------------------------------------------------------------------------------
// synthetic inputs / checks; the CPU definitions are in oracle/rs_oracle.c
// ---------------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(kBlock) synth_kernel(uint64_t seed, uint32_t N, uint64_t g0, uint64_t G, uint32_t s0,
                                                       uint32_t ns, uint32_t B, uint64_t pitch, uint8_t *out)
{
    const uint64_t Wd = (B + 7) / 8;
    const uint64_t total = G * ns * Wd;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < total; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t w = i % Wd, q = i / Wd;
        const uint64_t s = q % ns, gl = q / ns;
        const uint64_t v = splitmix64(seed ^ (((g0 + gl) * N + s0 + s) * Wd + w));
        uint8_t *dst = out + (gl * ns + s) * pitch + w * 8;
        if (w * 8 + 8 <= B && (reinterpret_cast<uintptr_t>(dst) & 7) == 0) {
            *reinterpret_cast<uint64_t *>(dst) = v;
        } else {
            for (uint32_t k = 0; k < 8 && w * 8 + k < B; ++k) dst[k] = (uint8_t)(v >> (8 * k));
        }
    }
}

int launch_synth(uint64_t seed, int N, size_t g0, size_t G, size_t s0, size_t ns, size_t B, size_t pitch,
                 void *d_out, hipStream_t s)
{
    if (G == 0 || ns == 0 || B == 0) return 0;
    hipLaunchKernelGGL(synth_kernel, dim3(4096), dim3(kBlock), 0, s, seed, (uint32_t)N, (uint64_t)g0, (uint64_t)G,
                       (uint32_t)s0, (uint32_t)ns, (uint32_t)B, (uint64_t)pitch, static_cast<uint8_t *>(d_out));
    return hipGetLastError() == hipSuccess ? 0 : -3;
}

__global__ void __launch_bounds__(kBlock) erasure_kernel(uint64_t seed, uint32_t N, uint64_t g0, uint64_t G, uint32_t pool,
                                                         uint32_t count_max, int random_count, uint64_t *present)
{
    const uint64_t g = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (g >= G) return;
    const uint64_t gg = g0 + g;
    uint32_t cnt = count_max;
    if (random_count) cnt = 1 + (uint32_t)(splitmix64(seed ^ ~gg) % count_max);
    uint64_t m[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) m[q] = bits_below((int)N, q);
    uint8_t perm[256];
    for (int i = 0; i < 256; ++i) perm[i] = (uint8_t)i;
    for (uint32_t t = 0; t < cnt && t < pool; ++t) {
        const uint64_t r = splitmix64(seed ^ (gg * 0x100u + t));
        const uint32_t k = t + (uint32_t)(r % (uint64_t)(pool - t));
        const uint8_t tmp = perm[t];
        perm[t] = perm[k];
        perm[k] = tmp;
        m[perm[t] >> 6] &= ~(1ull << (perm[t] & 63));
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) present[g * 4 + q] = m[q];
}

int launch_erasure_masks(uint64_t seed, int N, size_t g0, size_t G, size_t pool, size_t count_max, int random_count,
                         uint64_t *d_present, hipStream_t s)
{
    if (G == 0) return 0;
    hipLaunchKernelGGL(erasure_kernel, dim3((uint32_t)((G + kBlock - 1) / kBlock)), dim3(kBlock), 0, s, seed,
                       (uint32_t)N, (uint64_t)g0, (uint64_t)G, (uint32_t)pool, (uint32_t)std::max<size_t>(count_max, 1),
                       random_count, d_present);
    return hipGetLastError() == hipSuccess ? 0 : -3;
}

__global__ void __launch_bounds__(kBlock) verify_kernel(uint32_t K, uint32_t R, uint64_t G, uint32_t B, uint64_t pitch,
                                                        const uint8_t *data, const uint8_t *out, const uint8_t *out_idx,
                                                        unsigned long long *mismatch)
{
    const uint64_t cols = (B + 3) / 4;
    const uint64_t total = G * R * cols;
    unsigned long long bad = 0;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < total; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t c = i % cols, slot = i / cols;  // slot = g * R + t
        const uint32_t idx = out_idx[slot];
        if (idx == 0xFF) continue;
        const uint64_t g = slot / R;
        const uint8_t *o = out + slot * pitch + c * 4;
        const uint8_t *d = data + (g * K + idx) * pitch + c * 4;
        bool diff = false;
        for (uint32_t b = 0; b < 4 && c * 4 + b < B; ++b) diff |= (o[b] != d[b]);
        bad += diff;
    }
    if (bad) atomicAdd(mismatch, bad);
}

int launch_verify(int K, int N, size_t G, size_t B, size_t pitch, const void *d_data, const void *d_out,
                  const uint8_t *d_out_idx, uint64_t *d_mismatch, hipStream_t s)
{
    const int R = N - K;
    if (G == 0 || R == 0 || B == 0) return 0;
    hipLaunchKernelGGL(verify_kernel, dim3(4096), dim3(kBlock), 0, s, (uint32_t)K, (uint32_t)R, (uint64_t)G,
                       (uint32_t)B, (uint64_t)pitch, static_cast<const uint8_t *>(d_data),
                       static_cast<const uint8_t *>(d_out), d_out_idx,
                       reinterpret_cast<unsigned long long *>(d_mismatch));
    return hipGetLastError() == hipSuccess ? 0 : -3;
}

}  // namespace kfec
