// kfec_kernels.hip -- hand-written gfx950 (CDNA4) kernels of the kfec Reed-Solomon coder.
//
// Reference semantics (all /root/reference/src/3rd_party/):
//   matrix   fecpp.cpp:368-415, 453-490   enc = [I_K ; Vbot * Vtop^-1]  (build_matrix_kernel)
//   encode   fecpp.cpp:495-513            parity_r = XOR_j enc[K+r][j] * D_j   (mac_kernel<.., false>)
//   decode   fecpp.cpp:518-587            share selection + K x K inverse + m output rows
//                                           (decode_prep_* + syn_kernel / syn_list_kernel for R <= 8,
//                                            mac_kernel<.., true> for R > 8)
//   addmul   fecpp.cpp:170-223, fecpp_ssse3.cpp:541-575   z ^= c * x  (the "perm MAC" below)
//
// Design (DESIGN.md section 4 has the numbers):
// * perm MAC.  c * x for a constant c is linear over GF(2), so c*x = c*(x & 7) ^ c*(x & 0x38) ^ c*(x & 0xC0).
//   Each term is an 8- or 4-entry table lookup, and v_perm_b32 does 4 such byte lookups (one per byte of a
//   dword) in one VALU op.  Per data dword and coefficient: 3 v_perm_b32 + v_bitop3_b32 + v_xor_b32; the 3
//   selector extractions are shared by all coefficients of a data dword.  No LDS traffic per data byte.
// * Flattened work: one lane = one (group, 32-byte column) item; consecutive lanes take consecutive columns
//   (2 KiB per wave-instruction), wrapping into the next group.  One workgroup per 256 items (non-persistent);
//   R > 8 runs MT = 8 row tiles numbered so that the tiles of one chunk share an XCD (block_chunk_tile).
//   A row's last granule is end-aligned (gran_off), loads run consume-then-refill PD granules ahead.
// * Decode for R <= 8 in syndrome form: y = parity ^ E * D_present with the encode's wave-uniform tables,
//   then out = C * y with the per-group m x m inverse in C (syn_kernel); sparse loss takes a listed shape
//   over the groups that lost data (syn_list_kernel), chosen on the device.  The coefficients equal the
//   reference's K x K Gauss-Jordan result bit for bit (the inverse is unique).
#include "kfec_gf.hpp"
#include "kfec_internal.hpp"
#include "kfec_xcd.hpp"

#include <algorithm>
#include <cstdlib>
#include <string>

namespace kfec {

__constant__ GfTables c_gf = make_gf_tables();

static constexpr int kBlock = 256;
#ifndef KFEC_MAC_BLOCK
#define KFEC_MAC_BLOCK 256
#endif
static constexpr int kMacBlock = KFEC_MAC_BLOCK;  // workgroup of the flattened MAC kernel

// build-time tuning knobs (tools/ab.py builds variants; the shipped library uses the defaults)
#ifndef KFEC_MAC_BURST
#define KFEC_MAC_BURST 2  // encode MAC (MT 3..4): 2 = tables, MACs, next loads as bursts; 1 = loads only; 0 = interleaved
#endif
#ifndef KFEC_MAC_PD
#define KFEC_MAC_PD KFEC_PD  // the same for the MAC kernel's 32-byte shape with MT < 8
#endif
#ifndef KFEC_PD
#define KFEC_PD 4  // granules per lane in the load pipeline of the 32-byte shape (PD - 1 in flight during a MAC)
#endif
#ifndef KFEC_SYN_MAX_R
#define KFEC_SYN_MAX_R 8  // decode in syndrome form up to this R (0: coefficient form always; A/B builds)
#endif
#ifndef KFEC_SYN_SMALLK_PD
#define KFEC_SYN_SMALLK_PD 0  // > 0: granules in flight per lane of the syndrome decode for K <= 12 (A/B knob)
#endif
#ifndef KFEC_SYN_MINW
#define KFEC_SYN_MINW 1  // __launch_bounds__ minimum waves per SIMD of the syndrome-form decode kernel
#endif
#ifndef KFEC_EXPAND_EB
#define KFEC_EXPAND_EB 8  // mac_expand: items per thread whose loads are issued together (1: load-use per item)
#endif
#ifndef KFEC_SYN_EARLY
#define KFEC_SYN_EARLY 1  // syn_kernel: C-table bytes loaded with the record header, expanded after the shard loop
#endif
#ifndef KFEC_SYN_XORONLY
#define KFEC_SYN_XORONLY 0  // ablation (timing only, wrong results): the syndrome MACs as plain XORs, same loads / stores
                            // (1: the E / C table reads kept; 2: no table reads -- the arithmetic-free ceiling build)
#endif
#ifndef KFEC_MAC_XORONLY
#define KFEC_MAC_XORONLY 0  // ablation (timing only, wrong results): mac_kernel's MACs as plain XORs of the shard granules,
                            // no table reads -- same grid, loads and stores (tools/libkfec_arithfree.so: bench.py's ceiling)
#endif
#ifndef KFEC_SYN_TPRE
#define KFEC_SYN_TPRE 1  // syn_loop: the next shard's E tables loaded into SGPRs one shard ahead (0: at use; A/B knob)
#endif
#ifndef KFEC_SYN_PAIR
#define KFEC_SYN_PAIR 0  // syn_loop: two shards per row step, as KFEC_MAC_PAIR (RT <= 4): bit 0 syn_kernel, bit 1
                         // syn_list_kernel (A/B knob)
#endif
#ifndef KFEC_PREP_FUSED
#define KFEC_PREP_FUSED 1  // decode_prep_lagrange: denominators and numerators in one pass (0: two loops; A/B knob)
#endif
#ifndef KFEC_PREP_COEF2
#define KFEC_PREP_COEF2 1  // decode_prep_lagrange coefficients from stored column points, no modulo (A/B knob)
#endif
#if KFEC_PREP_COEF2 && !KFEC_PREP_FUSED
#error "KFEC_PREP_COEF2 reads the column points the fused pass (KFEC_PREP_FUSED) stores"
#endif
#ifndef KFEC_PREP_PREFETCH
#define KFEC_PREP_PREFETCH 1  // decode_prep_lagrange loads the next group's present bits one group ahead (A/B knob)
#endif
#ifndef KFEC_PREP_WAVE
#define KFEC_PREP_WAVE 1  // decode_prep_lagrange: one wave per group, four groups per workgroup (0: the workgroup; A/B)
#endif
#ifndef KFEC_PREP_WAVE_MINW
#define KFEC_PREP_WAVE_MINW 4  // the same for one wave per group (4: 128 VGPRs, 16 groups in flight per CU)
#endif
#ifndef KFEC_PREP_MINW
#define KFEC_PREP_MINW 8  // decode_prep_lagrange: minimum waves per SIMD (8: 64 VGPRs, 12 spilled, 3% faster than uncapped)
#endif
#ifndef KFEC_SYN_REC_COMPACT
#define KFEC_SYN_REC_COMPACT 1  // syndrome records of 40 + 8 RT bytes (64 at R = 3: one full line per group)
#endif
#ifndef KFEC_SYN_ROWMASK
#define KFEC_SYN_ROWMASK 1  // listed syndrome decode: 0 every parity row, 1 only the rows the group uses,
                            // 2 as 1 but single-row groups run a two-row variant (A/B knob)
#endif
#ifndef KFEC_MAC_PAIR
#define KFEC_MAC_PAIR 1  // encode MAC, 8-row tiles (R > 8): two shards per row step, acc ^= c_a x_a ^ c_b x_b as three
                         // 3-input XORs over the six permutes (instead of 2 x (v_bitop3 + v_xor)), rows outer;
                         // 200:55 encode 151.1 -> 133.8 ms, 40:20 13.24 -> 11.98 ms (profiles/r06_mac_pair_ab.txt)
#endif
#ifndef KFEC_ENC_MT_MID
#define KFEC_ENC_MT_MID 1  // encode R = 5..7 (32-byte granules): 0 an 8-row tile, 1 an R-row tile with the paired MAC, 2 an
                           // R-row tile in the plain loop. 1: 20:5 9.30 -> 7.49 ms, 20:6 9.56 -> 8.50, 16:7 8.10 -> 7.86,
                           // 10:6 5.33 -> 4.94 (2: 4.85 there, slower elsewhere) (profiles/r06_mt_mid_ab.txt)
#endif
#ifndef KFEC_MAC_PAIR_SMALL
#define KFEC_MAC_PAIR_SMALL 1  // the pairing in the encode burst loop (3..4-row tiles): 8:4 encode 3.39 -> 3.33 ms,
                               // 20:3 and 10:3 unchanged (HBM-bound) (profiles/r06_pair_small_ab.txt)
#endif
#ifndef KFEC_DEC_PAIR
#define KFEC_DEC_PAIR 1  // the same pairing in the T-table decode MAC (8-row tiles): 200:55 decode 151.4 -> 137.5 ms,
                         // 40:20 14.09 -> 13.30 ms, 20:20 15.50 -> 15.07 ms (profiles/r06_dec_pair_ab.txt)
#endif
#ifndef KFEC_PREP_SYN_T
#define KFEC_PREP_SYN_T 1  // decode_prep_perm's syndrome-record form as its own instantiation (0: runtime flag; A/B knob)
#endif
#ifndef KFEC_MINW
#define KFEC_MINW 1  // __launch_bounds__ minimum waves per SIMD of the MAC kernels
#endif
#ifndef KFEC_DEC_FACTORED
#define KFEC_DEC_FACTORED 1  // R > 8 decode records carry the Lagrange factors, not the m x K coefficients (A/B knob)
#endif
#ifndef KFEC_DEC_TTAB
#define KFEC_DEC_TTAB 1  // coefficient-form decode (R > 8): LDS entries point into one table of all 256 coefficients'
                         // perm tables (1) instead of holding each coefficient's expanded tables (0; A/B knob)
#endif
#ifndef KFEC_DEC_EXPAND2
#define KFEC_DEC_EXPAND2 1  // factored-record entries by dec_expand_fac (0: the flat-index dec_expand; A/B knob)
#endif
#ifndef KFEC_DEC_OFS16
#define KFEC_DEC_OFS16 1  // T-table decode: each row's table offset read by its own 2-byte LDS read (A/B knob)
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
    int syn;       // write syndrome-form records (R <= 8) instead of the coefficient form
    int factored;  // decode_prep_lagrange: write the factored form (dec_expand rebuilds each coefficient)
    // hybrid decode: the coefficient-form prep exits when the listed syndrome shape takes the launch (syn_listed)
    const uint32_t *skip_listed;
    uint32_t cols, cols_pad;
};

__device__ __forceinline__ bool prep_skip(const PrepArgs &a)
{
    return a.skip_listed && (uint64_t)*a.skip_listed * a.cols_pad < a.G * a.cols;
}

// Factored coefficient-form record (decode_prep_lagrange for the mac_kernel decode, KFEC_DEC_FACTORED): the
// m x K coefficients of a group are coef[u][j] = exp(lnum_u - log(xm_u ^ xs_j) - lden_j) (see the prep), so the
// record keeps the factors -- src[j] (and with it the point xs_j), lden_j, lnum_u and the missing points xm_u --
// 2 K + 2 R bytes instead of m K: at fec=200:55, 528 bytes per group instead of 11 KB, which the prep no longer
// writes and the MAC's row tiles no longer read (2.9 GB each way per 256k groups).
//   [0] status, [1] m, [4, 4 + K4) src, [4 + K4, 4 + 2 K4) lden, [L0, L0 + R8) lnum, [L0 + R8, L0 + 2 R8) xm,
//   L0 = round16(4 + 2 K4), R8 = round8(R)
__host__ __device__ inline uint32_t fac_lnum_off(uint32_t K) { return (4 + 2 * ((K + 3) & ~3u) + 15) & ~15u; }
__host__ __device__ inline uint32_t fac_r8(uint32_t R) { return (R + 7) & ~7u; }
__host__ __device__ inline size_t fac_record_stride(size_t K, size_t R)
{
    return (fac_lnum_off((uint32_t)K) + 2 * fac_r8((uint32_t)R) + 15) & ~size_t(15);
}

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

// Syndrome-form record (syn_kernel, R <= 8): [0] status 0, [1] m, [2] bit r set = parity row K + r is one
// of the m shares used, [3..7] 0, [8, 40) the present DATA shard bits (4 x u64, so the MAC kernel gets
// its header and the first 64 bits in one 16-byte load), [40 + 8u + r] = C[u][r] = Sinv[u][t] for the rank
// t with P_t = K + r (0 for unused rows and for u >= m): rows u < RT are written (the ones the syn kernels
// read), so the kernels read zeros beyond m.
// Row tile of the syndrome form (the C rows a syn kernel reads: RT x RT bytes) and the record stride: the
// header, the present bits and RT rows of C -- 64 bytes at R = 3, one whole line per group
#ifndef KFEC_SYN_FINAL_ROWS
#define KFEC_SYN_FINAL_ROWS 1  // syn_list_kernel's final mix at RT 5, 6, 8 with the syndromes outer (260 -> 176 VGPRs at RT
                               // 8): 1%-loss decode 20:8 3.89 -> 3.44 ms, 20:5 2.18 -> 2.13, 20:6 2.49 -> 2.46; RT 7 measured
                               // 6% slower and keeps the row order (profiles/r06_syn_final_rows_ab.txt)
#endif
#ifndef KFEC_DEC_MT_MID
#define KFEC_DEC_MT_MID 1  // the hybrid decode's coefficient-form MAC for R = 5..7 as an R-row tile (129-149 VGPRs):
                           // with the hybrid from R = 5, dense 20:6 11.05 -> 9.87 ms, 10:6 random 5.99 -> 5.00, 16:7
                           // 9.63 -> 9.19, 20:5 9.06 -> 8.88; sparse unchanged (profiles/r06_dec_mt_mid_ab.txt)
#endif
#ifndef KFEC_DEC_MT_SMALL
#define KFEC_DEC_MT_SMALL 1  // the hybrid decode's coefficient-form MAC for R = 4 as a 4-row tile: dense 8:4 decode 3.97 ->
                             // 3.72 ms; for R = 3 it was slower than the syndrome kernel (20:3 6.2-6.6 -> 6.7, 10:3 random
                             // 3.11 -> 3.28), so R = 3 stays syndrome-only (profiles/r06_dec_mt_small_ab.txt)
#endif
// the coefficient-form decode MAC reads its tables from T (KFEC_DEC_TTAB) for these row tiles
__host__ __device__ constexpr bool dec_ttab(int MT)
{
    return KFEC_DEC_TTAB && (MT == 8 || (KFEC_DEC_MT_MID && MT >= 5 && MT < 8) || (KFEC_DEC_MT_SMALL && MT == 4));
}
#ifndef KFEC_DEC_MT4_WIDE
#define KFEC_DEC_MT4_WIDE 1  // R > 8 coefficient-form decode in 4-row tiles where they compute fewer rows: 40:20 13.40 ->
                             // 12.62 ms, 30:20 random 6.97 -> 6.38, 30:12 14.57 -> 12.72, 40:20 at 1% loss 4.58 -> 3.23;
                             // 200:55 keeps 8-row tiles (profiles/r06_dec_mt4_ab.txt)
#endif
#ifndef KFEC_SYN_RT_MID
#define KFEC_SYN_RT_MID 1  // syndrome decode for R = 5..7: RT = R instead of 8 (166 VGPRs at RT 5, 3 waves per SIMD, against
                           // RT 8's 256): 20:5 decode 12.83 -> 9.18 ms, 20:6 13.40 -> 11.05, 16:7 11.87 -> 10.90, 10:6
                           // random 7.31 -> 5.89, 20:6 at 1% loss 3.93 -> 2.53 (profiles/r06_syn_rt_mid_ab.txt)
#endif
__host__ __device__ constexpr int syn_rt(int R) { return R <= 4 ? (R > 0 ? R : 1) : (KFEC_SYN_RT_MID && R <= 7 ? R : 8); }
__host__ __device__ inline size_t syn_record_stride(size_t K, size_t R)
{
    return KFEC_SYN_REC_COMPACT ? (size_t)((40 + 8 * syn_rt((int)R) + 15) & ~15) : record_stride(K, R);
}

template <int MAXM, typename F>
__device__ __forceinline__ void write_syn(const PrepArgs &a, uint64_t g, int m, const int (&M)[MAXM],
                                          const int (&P)[MAXM], const uint64_t (&w)[4], F sinv)
{
    uint64_t *rw = reinterpret_cast<uint64_t *>(a.rec + g * a.rec_stride);
    uint32_t used = 0;
    uint64_t row[MAXM];
#pragma unroll
    for (int u = 0; u < MAXM; ++u) row[u] = 0;
#pragma unroll
    for (int t = 0; t < MAXM; ++t) {
        if (t < m) {
            const uint32_t r = (uint32_t)(P[t] - a.K);
            used |= 1u << r;
#pragma unroll
            for (int u = 0; u < MAXM; ++u)
                if (u < m) row[u] |= (uint64_t)sinv(u, t) << (8 * r);
        }
    }
    rw[0] = (uint64_t)(((uint32_t)m << 8) | (used << 16));
#pragma unroll
    for (int q = 0; q < 4; ++q) rw[1 + q] = w[q] & bits_below(a.K, q);
    // rows u < RT only (the record ends there); rows past m are zero
    const int rt = syn_rt((int)a.R);
#pragma unroll
    for (int u = 0; u < 8; ++u)
        if (u < rt) rw[5 + u] = u < MAXM ? row[u] : 0ull;
#pragma unroll
    for (int t = 0; t < MAXM; ++t)
        if (t < a.R) a.out_idx[g * a.R + t] = (t < m) ? (uint8_t)M[t] : (uint8_t)0xFF;
    for (int t = MAXM; t < a.R; ++t) a.out_idx[g * a.R + t] = 0xFF;
    a.status[g] = 0;
}

template <int MAXM>
__global__ void __launch_bounds__(kBlock) decode_prep_small(PrepArgs a)
{
    if (prep_skip(a)) return;  // (whole grid)
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
        if (a.syn) {
            write_syn<MAXM>(a, g, m, M, P, w, [&](int u, int t) { return Iv[u][t]; });
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
// SYN: the syndrome-form records only (a compile-time branch: without the coefficient-form path's tables the
// kernel needs far fewer registers -- 145 -> fewer VGPRs at MAXM = 3 -- and more groups are in flight per SIMD)
template <int MAXM, bool SYN = false>
__global__ void __launch_bounds__(kBlock) decode_prep_perm(PrepArgs a)
{
    static_assert(MAXM >= 1 && MAXM <= 4, "rows are packed into one dword");
    if (prep_skip(a)) return;  // (whole grid)
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
        if (SYN || a.syn) {
            write_syn<MAXM>(a, g, m, M, P, w, [&](int u, int t) { return (Iv[u] >> (8 * t)) & 0xFFu; });
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

// The fused pass (KFEC_PREP_FUSED) drops a numerator's excluded term (x_s ^ x_c = 0) by reading log[0], which
// must therefore be 0 mod 255; and its coefficient exponents index exp[] up to 509 without a modulo, which
// needs exp[] periodic with period 255 over the doubled table.
constexpr bool gf_exp_periodic()
{
    constexpr GfTables t = make_gf_tables();
    for (int i = 255; i < 510; ++i)
        if (t.exp[i] != t.exp[i - 255]) return false;
    return true;
}
static_assert(make_gf_tables().log[0] % 255 == 0, "decode_prep_lagrange relies on log[0] == 255 (0 mod 255)");
static_assert(gf_exp_periodic(), "decode_prep_lagrange indexes exp[] up to 509 without reduction");

// TEAM threads solve one group: the whole workgroup (256, barriers between the steps) or one wave (64:
// four groups per workgroup at once, each wave with its own lists and no workgroup barrier inside the group loop --
// a wave's LDS operations complete in order, the fences only keep the compiler from reordering them).
template <int TEAM>
__global__ void __launch_bounds__(kPrepThreads, TEAM == 64 ? KFEC_PREP_WAVE_MINW : KFEC_PREP_MINW) decode_prep_lagrange(PrepArgs a)
{
    static_assert(TEAM == kPrepThreads || TEAM == 64, "a team is the workgroup or one wave");
    constexpr int NT = kPrepThreads / TEAM;  // teams (groups in flight) per workgroup
    __shared__ uint8_t s_exp[512], s_log[256];
    __shared__ uint16_t s_full[256];  // FULL_s mod 255
    __shared__ uint8_t s_C_all[NT][256];      // ids outside S, ascending
    __shared__ uint8_t s_xC_all[NT][256];     // their points
    __shared__ uint8_t s_M_all[NT][256];      // missing data ids, ascending
    __shared__ uint8_t s_P_all[NT][256];      // parity share used for missing rank t: the highest present ids, descending
    __shared__ uint8_t s_src_all[NT][256];    // source share of column j
    __shared__ uint16_t s_lden_all[NT][256];  // log den of the source of column j
    __shared__ uint16_t s_lnum_all[NT][256];  // log num_u without the (x_{M_u} ^ x_i) factor
    __shared__ uint8_t s_xs_all[NT][256];     // KFEC_PREP_COEF2: the point of column j's source
    const int K = a.K, N = a.N, R = a.R;
    const int team = threadIdx.x / TEAM, tid = threadIdx.x % TEAM;  // (tid: the thread's index in its team)
    uint8_t *s_C = s_C_all[team], *s_xC = s_xC_all[team], *s_M = s_M_all[team], *s_P = s_P_all[team];
    uint8_t *s_src = s_src_all[team], *s_xs = s_xs_all[team];
    uint16_t *s_lden = s_lden_all[team], *s_lnum = s_lnum_all[team];
    auto team_sync = [&]() {
        if constexpr (TEAM == kPrepThreads) __syncthreads();
        else __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    };
    const int K4 = (K + 3) & ~3, kd = K4 / 4;
    stage_gf(s_exp, s_log);
    __syncthreads();
    auto xpt = [&](int sid) -> uint32_t { return sid ? (uint32_t)s_exp[sid] : 0u; };  // s_exp[255] = 1
    for (int sid = threadIdx.x; sid < N; sid += kPrepThreads) {
        const uint32_t xs = xpt(sid);
        uint32_t acc = 0;
        for (int k = 0; k < N; ++k)
            if (k != sid) acc += s_log[xs ^ xpt(k)];
        s_full[sid] = (uint16_t)(acc % 255u);
    }
    __syncthreads();

    // KFEC_PREP_PREFETCH: the next group's present bits are loaded while this group is solved
    const uint64_t g0 = (uint64_t)blockIdx.x * NT + team, gstride = (uint64_t)gridDim.x * NT;
    uint64_t pn[4] = {0, 0, 0, 0};
    if (KFEC_PREP_PREFETCH && g0 < a.G) {
#pragma unroll
        for (int q = 0; q < 4; ++q) pn[q] = a.present[g0 * 4 + q];
    }
    for (uint64_t g = g0; g < a.G; g += gstride) {
        uint64_t w[4], dm[4], pc[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) pc[q] = KFEC_PREP_PREFETCH ? pn[q] : a.present[g * 4 + q];
        if (KFEC_PREP_PREFETCH && g + gstride < a.G) {
#pragma unroll
            for (int q = 0; q < 4; ++q) pn[q] = a.present[(g + gstride) * 4 + q];
        }
        int cnt = 0, m = 0;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            w[q] = pc[q] & bits_below(N, q);
            dm[q] = ~w[q] & bits_below(K, q);
            cnt += __popcll(w[q]);
            m += __popcll(dm[q]);
        }
        uint8_t *rec = a.rec + g * a.rec_stride;
        if (cnt < K) {  // uniform over the team
            if (tid == 0) {
                rec[0] = 1;
                rec[1] = 0;
                a.status[g] = 1;
            }
            for (int t = tid; t < R; t += TEAM) a.out_idx[g * R + t] = 0xFF;
            continue;
        }
        // P_t = the present id with exactly t present ids above it (t < m; all parity since cnt >= K);
        // the lowest of them, P_{m-1}, bounds the used-parity set from below
        for (int sid = tid; sid < N; sid += TEAM) {
            if ((w[sid >> 6] >> (sid & 63)) & 1ull) {
                const int above = cnt - 1 - rank_below(w, sid);
                if (above < m) s_P[above] = (uint8_t)sid;
            }
        }
        team_sync();
        const int thr = m > 0 ? (int)s_P[m - 1] : 256;
        uint64_t Cb[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const uint64_t used_par = w[q] & ~bits_below(thr, q);
            const uint64_t S = (w[q] & bits_below(K, q)) | used_par;
            Cb[q] = ~S & bits_below(N, q);
        }
        for (int sid = tid; sid < N; sid += TEAM) {
            const int q = sid >> 6, b = sid & 63;
            if ((Cb[q] >> b) & 1ull) {
                const int r = rank_below(Cb, sid);
                s_C[r] = (uint8_t)sid;
                s_xC[r] = (uint8_t)xpt(sid);
            }
            if (sid < K && ((dm[q] >> b) & 1ull)) s_M[rank_below(dm, sid)] = (uint8_t)sid;
        }
        team_sync();
#if KFEC_PREP_FUSED
        // the K column denominators and the m numerators are one kind of sum, log FULL_s - sum_c log(x_s ^ x_c),
        // so they are one pass of K + m <= N <= 256 items (one per thread) instead of two loops that wave 0
        // ran back to back; a numerator's excluded term c = M_u has x_s ^ x_c = 0, and log[0] = 255 = 0 mod 255
        for (int it = tid; it < K + m; it += TEAM) {
            int sid;
            if (it < K) {
                const bool miss = (dm[it >> 6] >> (it & 63)) & 1ull;
                sid = miss ? (int)s_P[rank_below(dm, it)] : it;
                s_src[it] = (uint8_t)sid;
            } else {
                sid = s_M[it - K];
            }
            const uint32_t xs = xpt(sid);
            if (KFEC_PREP_COEF2 && it < K) s_xs[it] = (uint8_t)xs;
            uint32_t acc = 0;
#pragma unroll 8
            for (int c = 0; c < R; ++c) acc += s_log[xs ^ s_xC[c]];
            const uint16_t v = (uint16_t)((s_full[sid] + 255u - acc % 255u) % 255u);
            if (it < K) s_lden[it] = v;
            else s_lnum[it - K] = v;
        }
#else
        for (int j = tid; j < K; j += TEAM) {
            const bool miss = (dm[j >> 6] >> (j & 63)) & 1ull;
            const int i = miss ? (int)s_P[rank_below(dm, j)] : j;
            s_src[j] = (uint8_t)i;
            const uint32_t xi = xpt(i);
            uint32_t acc = 0;
            for (int c = 0; c < R; ++c) acc += s_log[xi ^ s_xC[c]];
            s_lden[j] = (uint16_t)((s_full[i] + 255u - acc % 255u) % 255u);
        }
        for (int u = tid; u < m; u += TEAM) {
            const int mu = s_M[u];
            const uint32_t xm = xpt(mu);
            uint32_t acc = 0;
            for (int c = 0; c < R; ++c)
                if (s_C[c] != mu) acc += s_log[xm ^ s_xC[c]];
            s_lnum[u] = (uint16_t)((s_full[mu] + 255u - acc % 255u) % 255u);
        }
#endif
        team_sync();
        uint32_t *srcw = reinterpret_cast<uint32_t *>(rec + 4);
        if (a.factored) {
            // the factors only (see fac_record_stride): src and lden as dwords of 4 columns, lnum and xm per row
            const uint32_t L0 = fac_lnum_off((uint32_t)K), R8 = fac_r8((uint32_t)R);
            uint32_t *ldw = reinterpret_cast<uint32_t *>(rec + 4 + K4);
            for (int d = tid; d < kd; d += TEAM) {
                uint32_t v = 0, l = 0;
#pragma unroll
                for (int b = 0; b < 4; ++b)
                    if (4 * d + b < K) {
                        v |= (uint32_t)s_src[4 * d + b] << (8 * b);
                        l |= (uint32_t)s_lden[4 * d + b] << (8 * b);
                    }
                srcw[d] = v;
                ldw[d] = l;
            }
            for (int u = tid; u < m; u += TEAM) {
                rec[L0 + u] = (uint8_t)s_lnum[u];
                rec[L0 + R8 + u] = (uint8_t)xpt(s_M[u]);
            }
            for (int t = tid; t < R; t += TEAM) a.out_idx[g * R + t] = (t < m) ? s_M[t] : (uint8_t)0xFF;
            if (tid == 0) {
                rec[0] = 0;
                rec[1] = (uint8_t)m;
                rec[2] = rec[3] = 0;
                a.status[g] = 0;
            }
            team_sync();  // the lists are rewritten for the next group
            continue;
        }
        uint32_t *coefw = reinterpret_cast<uint32_t *>(rec + 4 + K4);
        for (int d = tid; d < kd; d += TEAM) {
            uint32_t v = 0;
#pragma unroll
            for (int b = 0; b < 4; ++b)
                if (4 * d + b < K) v |= (uint32_t)s_src[4 * d + b] << (8 * b);
            srcw[d] = v;
        }
        for (int e = tid; e < m * kd; e += TEAM) {
            const int u = e / kd, d = e - u * kd;
            const uint32_t xm = xpt(s_M[u]);
            const int ln = s_lnum[u];
            uint32_t v = 0;
#pragma unroll
            for (int b = 0; b < 4; ++b) {
                const int j = 4 * d + b;
                if (j < K) {
                    int ex;
                    if (KFEC_PREP_COEF2) {
                        // one LDS level less (the column's point is stored), and the exponent in [2, 764] brought
                        // under the 510-entry antilog table by one compare instead of a modulo
                        ex = ln + 510 - (int)s_log[xm ^ s_xs[j]] - (int)s_lden[j];
                        ex = ex >= 510 ? ex - 255 : ex;
                    } else {
                        ex = (ln + 510 - (int)s_log[xm ^ xpt(s_src[j])] - (int)s_lden[j]) % 255;
                    }
                    v |= (uint32_t)s_exp[ex] << (8 * b);
                }
            }
            coefw[u * kd + d] = v;
        }
        for (int t = tid; t < R; t += TEAM) a.out_idx[g * R + t] = (t < m) ? s_M[t] : (uint8_t)0xFF;
        if (tid == 0) {
            rec[0] = 0;
            rec[1] = (uint8_t)m;
            rec[2] = rec[3] = 0;
            a.status[g] = 0;
        }
        team_sync();  // the lists are rewritten for the next group
    }
}

// ---------------------------------------------------------------------------------------------------
// (A4/A5/A8/A11) perm-MAC kernels over V-byte columns.
//   mac_kernel (coefficient form): out[g][row] = XOR_j coef[row][j] * share_j[g]
//     encode: coef = the parity rows of the encoding matrix (fecpp.cpp:495-513);
//     decode for R > 8: coef = the K x K inverse rows of the missing shards, shares gathered through the
//     record's source ids (fecpp.cpp:550-585).
//   syn_kernel (syndrome form, decode with R <= 8): see below.
// ---------------------------------------------------------------------------------------------------
struct MacArgs {
    const uint8_t *data;    // [G][K][pitch]
    const uint8_t *parity;  // [G][R][pitch]
    uint8_t *out;           // encode: parity, decode: recovered [G][R][pitch]
    const uint8_t *enc;     // N x K encoding matrix (encode)
    const uint8_t *rec;     // per-group records (decode)
    uint64_t pitch;
    uint32_t total;         // G * cols work items
    uint32_t cols;          // granules per shard
    uint32_t G, K, R, B;
    uint32_t rec_stride;
    uint32_t JC;            // shards per LDS chunk
    uint32_t gmax;          // group slots per chunk
    uint32_t tiles;         // row tiles of MT output rows
    uint32_t factored;      // decode: factored records (fac_record_stride), coefficients rebuilt by dec_expand
    const uint32_t *list_count;  // hybrid decode: the listed groups' count; the kernel exits when the listed shape runs
    uint32_t cols_pad;
};

template <int VEC>
struct Gran {
    static constexpr int W = VEC >= 4 ? VEC / 4 : 1;
    uint32_t d[W];
};

// Shares are always in global memory (HBM, or pinned host memory mapped into the device's address space), so
// the loads go through global-address-space pointers: a share pointer read back from LDS (the decode's
// entries) would otherwise become a flat load, which also counts on lgkmcnt -- every wait for an LDS read
// (the next shard's tables) then also waited for the shard loads in flight.
typedef unsigned int gx4_t __attribute__((ext_vector_type(4)));
typedef const __attribute__((address_space(1))) gx4_t gu4;
typedef const __attribute__((address_space(1))) uint32_t gu32;

template <int VEC>
__device__ __forceinline__ Gran<VEC> load_gran(const uint8_t *p, uint32_t col, uint32_t B)
{
    Gran<VEC> v;
    if constexpr (VEC == 32) {
        const gx4_t x = ((gu4 *)p)[0], y = ((gu4 *)p)[1];
        v.d[0] = x.x; v.d[1] = x.y; v.d[2] = x.z; v.d[3] = x.w;
        v.d[4] = y.x; v.d[5] = y.y; v.d[6] = y.z; v.d[7] = y.w;
    } else if constexpr (VEC == 4) {
        v.d[0] = *(gu32 *)p;
    } else {  // bytewise: 4 bytes at p, only those below B
        static_assert(VEC == 1, "granule");
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
        // nontemporal: the outputs are not re-read by this launch (+2.5% encode, measured)
        typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));
        __builtin_nontemporal_store(u32x4_t{d[0], d[1], d[2], d[3]}, reinterpret_cast<u32x4_t *>(p));
        __builtin_nontemporal_store(u32x4_t{d[4], d[5], d[6], d[7]}, reinterpret_cast<u32x4_t *>(p + 16));
    } else if constexpr (VEC == 4) {
        *reinterpret_cast<uint32_t *>(p) = d[0];
    } else {
        const uint32_t b0 = col * 4;
#pragma unroll
        for (int b = 0; b < 4; ++b)
            if (b0 + b < B) p[b] = (uint8_t)(d[0] >> (8 * b));
    }
}

// Byte offset of a lane's granule in a shard row: VB * col, except that the last granule of a row whose B
// is not a multiple of VB is moved back to end at round4(B).  It then overlaps the previous granule, whose
// output bytes it recomputes identically (the MAC is column-wise: output byte i depends only on byte i of
// every share), so every lane loads and stores one whole granule and the shard loop has no per-lane branch.
// (A per-lane "tail" branch around the loads made hipcc wait for every load right where it was issued --
// the two paths define the granule registers differently -- so nothing was in flight across shards.)
// Bytes in [B, round4(B)) are read and written, inside the slot (pitch % 4 == 0); the host only takes
// VB > 4 when B >= VB.
template <int VEC>
__device__ __forceinline__ uint32_t gran_off(uint32_t col, uint32_t B)
{
    constexpr uint32_t VB = VEC >= 4 ? VEC : 4;
    if constexpr (VEC >= 4) return min(col * VB, ((B + 3) & ~3u) - VB);
    return col * 4;
}

template <int MT>
struct MacLayout {
    static_assert(MT >= 1 && MT <= 16, "row tile");
    static constexpr int TBL_DW = ((5 * MT + 3) / 4) * 4;  // table dwords per (group, shard): 5 per row
    static constexpr int ENTRY = 16 + 4 * TBL_DW;          // + 8-byte share pointer, 8 pad
};

// Coefficient-form decode entries (KFEC_DEC_TTAB): the workgroup's LDS starts with T, the perm tables of all 256
// coefficient values (8-dword stride, built once per workgroup); an entry per (group slot, shard) is the share
// pointer and, per output row of the tile, the byte offset of its coefficient's table in T (u16).  An entry is
// 24 bytes instead of 16 + 40 * 4, so every shard of a workgroup's groups fits one expansion (fec=200:55,
// B=1440: 7 groups x 200 shards, 33.6 KB): one global-load round trip and one barrier per workgroup instead of
// one per 26-shard chunk, and no per-entry table construction.
constexpr int kDecEntry = 24;
constexpr uint32_t kTBytes = 256 * 32;
// after T (factored records): the GF exp (512) / log (256) tables, then the T-address table of dec_expand_fac
// (768 u16: tbase + 32 exp(e mod 255) for every exponent e the coefficient form produces, [2, 764])
constexpr uint32_t kDecGfBytes = 768 + 768 * 2;

// Workgroup b -> (column chunk, row tile).  With R > MT the tiles of one column chunk are numbered
// b, b+8, b+16, ...: the dispatcher deals workgroups round-robin over the 8 XCDs, so those run back to back
// on ONE XCD and all but the first read the chunk's shard bytes from that XCD's L2 (speed only: any
// placement gives the same bytes).  The previous (chunk = x, tile = y) grid ran every chunk of tile 0 before
// tile 1, so each of the 7 tiles of fec=200:55 re-read the 75.5 GB of data from HBM.
__device__ __forceinline__ void block_chunk_tile(uint32_t b, uint32_t tiles, uint32_t &chunk, uint32_t &tile)
{
    if (tiles <= 1) {
        chunk = xcd_chunk(b);
        tile = 0;
        return;
    }
    const uint32_t k = b >> 3;
    tile = k % tiles;
    chunk = xcd_tile_chunk(k / tiles, b & 7, gridDim.x / tiles);
}

// expand coefficients of shards [c0, c0+nj) for group slots [0, ng) into LDS entries
template <int MT, bool DEC>
__device__ __forceinline__ void mac_expand(const MacArgs &a, uint8_t *s_ent, uint32_t gfirst, uint32_t ng,
                                           uint32_t c0, uint32_t nj, uint32_t row0)
{
    using L = MacLayout<MT>;
    const uint32_t items = ng * nj * MT;
    // In batches of EB items per thread whose global loads (coefficient byte, record header, source id) are
    // all issued before the first is used: one memory latency per batch instead of one per item (the
    // per-item loop waited for each byte in turn, ~6 round trips per chunk at fec=200:55).
    constexpr int EB = KFEC_EXPAND_EB;
    for (uint32_t e0 = 0; e0 < items; e0 += EB * blockDim.x) {
        uint32_t cv[EB], sv[EB];
#pragma unroll
        for (int b = 0; b < EB; ++b) {
            const uint32_t e = min(e0 + b * blockDim.x + threadIdx.x, items - 1);  // clamped: loads unconditional
            const uint32_t r = e % MT, q = e / MT;
            const uint32_t jj = q % nj, gs = q / nj;
            const uint32_t j = c0 + jj, u = row0 + r;
            if constexpr (DEC) {
                const uint32_t K4 = (a.K + 3) & ~3u;
                const uint8_t *rec = a.rec + (uint64_t)(gfirst + gs) * a.rec_stride;
                const uint32_t hd = *reinterpret_cast<const uint16_t *>(rec);  // status | m << 8
                const uint32_t c = rec[4 + K4 + min(u, a.R - 1) * K4 + j];
                cv[b] = ((hd & 0xFFu) == 0 && u < (hd >> 8)) ? c : 0u;
                sv[b] = rec[4 + j];
            } else {
                cv[b] = u < a.R ? a.enc[(uint64_t)(a.K + u) * a.K + j] : 0u;
                sv[b] = 0;
            }
        }
#pragma unroll
        for (int b = 0; b < EB; ++b) {
            const uint32_t e = e0 + b * blockDim.x + threadIdx.x;
            if (e >= items) break;
            const uint32_t r = e % MT, q = e / MT;
            const uint32_t jj = q % nj, gs = q / nj;
            uint8_t *ent = s_ent + (gs * a.JC + jj) * L::ENTRY;
            if constexpr (DEC) {
                if (r == 0) {
                    const uint32_t src = sv[b];
                    const uint64_t g = gfirst + gs;
                    const uint8_t *p = (src < a.K) ? a.data + (g * a.K + src) * a.pitch
                                                   : a.parity + (g * a.R + (src - a.K)) * a.pitch;
                    *reinterpret_cast<const uint8_t **>(ent) = p;
                }
            }
            uint32_t t[5];
            gf_perm_tables(cv[b], t);
            uint32_t *tp = reinterpret_cast<uint32_t *>(ent + 16) + 5 * r;
#pragma unroll
            for (int i = 0; i < 5; ++i) tp[i] = t[i];
        }
    }
}

// T: gf_perm_tables(c) at s_T + 32 c for every byte c (no barrier: the caller's follows)
__device__ __forceinline__ void dec_build_t(uint8_t *s_T)
{
    for (uint32_t c = threadIdx.x; c < 256; c += blockDim.x) {
        uint32_t t[5];
        gf_perm_tables(c, t);
        uint32_t *d = reinterpret_cast<uint32_t *>(s_T + c * 32);
        *reinterpret_cast<uint4 *>(d) = uint4{t[0], t[1], t[2], t[3]};
        d[4] = t[4];
    }
}

// the LDS address of a pointer into the workgroup's shared memory
__device__ __forceinline__ uint32_t lds_addr(const uint8_t *p)
{
    return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) uint8_t *)p;
}

// entries of shards [c0, c0 + nj) for group slots [0, ng): share pointer + MT u16 offsets into T (KFEC_DEC_OFS16:
// T's LDS address tbase added, so each is the address its table is read at)
template <int MT>
__device__ __forceinline__ void dec_expand(const MacArgs &a, uint8_t *s_ent, uint32_t gfirst, uint32_t ng, uint32_t c0,
                                           uint32_t nj, uint32_t row0, const uint8_t *s_exp, const uint8_t *s_log,
                                           uint32_t tbase)
{
    static_assert(MT >= 1 && MT <= 8, "entry: 8 offsets (rows past MT take the zero table)");
    const uint32_t items = ng * nj, K4 = (a.K + 3) & ~3u;
    constexpr int EB = 4;  // entries per thread whose loads are issued together
    for (uint32_t e0 = 0; e0 < items; e0 += EB * blockDim.x) {
        uint32_t hd[EB], sv[EB], cv[EB][MT];
#pragma unroll
        for (int b = 0; b < EB; ++b) {
            const uint32_t e = min(e0 + b * blockDim.x + threadIdx.x, items - 1);  // clamped: loads unconditional
            const uint32_t jj = e % nj, gs = e / nj, j = c0 + jj;
            const uint8_t *rec = a.rec + (uint64_t)(gfirst + gs) * a.rec_stride;
            hd[b] = *reinterpret_cast<const uint16_t *>(rec);  // status | m << 8
            sv[b] = rec[4 + j];
            if (a.factored) {
                const uint32_t L0 = fac_lnum_off(a.K), R8 = fac_r8(a.R);
                const uint2 ln = *reinterpret_cast<const uint2 *>(rec + L0 + row0);  // (row0 % 8 == 0, rows < R8)
                const uint2 xm = *reinterpret_cast<const uint2 *>(rec + L0 + R8 + row0);
                const uint32_t ld = rec[4 + K4 + j];
#pragma unroll
                for (int r = 0; r < MT; ++r) {
                    const uint32_t lnr = ((r < 4 ? ln.x : ln.y) >> (8 * (r & 3))) & 0xFFu;
                    const uint32_t xmr = ((r < 4 ? xm.x : xm.y) >> (8 * (r & 3))) & 0xFFu;
                    cv[b][r] = lnr | (xmr << 8) | (ld << 16);  // (combined below, after every load is issued)
                }
            } else {
#pragma unroll
                for (int r = 0; r < MT; ++r) cv[b][r] = rec[4 + K4 + min(row0 + r, a.R - 1) * K4 + j];
            }
        }
#pragma unroll
        for (int b = 0; b < EB; ++b) {
            const uint32_t e = e0 + b * blockDim.x + threadIdx.x;
            if (e >= items) break;
            const uint32_t jj = e % nj, gs = e / nj;
            const uint64_t g = gfirst + gs;
            const uint32_t src = sv[b];
            const uint8_t *p = (src < a.K) ? a.data + (g * a.K + src) * a.pitch : a.parity + (g * a.R + (src - a.K)) * a.pitch;
            uint8_t *ent = s_ent + (gs * a.JC + jj) * kDecEntry;
            *reinterpret_cast<const uint8_t **>(ent) = p;
            const bool ok = (hd[b] & 0xFFu) == 0;
            const uint32_t m = hd[b] >> 8;
            // the tile's coefficients of (group, column j) from the record's factors: exp(lnum_u - log(xm_u ^ xs_j)
            // - lden_j), two lookups each in the workgroup's GF tables; the exponent in [1, 764] is brought under the
            // doubled antilog table by one compare (as the prep does)
            if (a.factored) {
                const uint32_t xs = src ? (uint32_t)s_exp[src] : 0u;  // the point of the column's share (x_0 = 0)
#pragma unroll
                for (int r = 0; r < MT; ++r) {
                    const uint32_t v = cv[b][r];
                    int ex = (int)(v & 0xFFu) + 510 - (int)s_log[((v >> 8) & 0xFFu) ^ xs] - (int)(v >> 16);
                    ex = ex >= 510 ? ex - 255 : ex;
                    cv[b][r] = s_exp[ex];
                }
            }
            uint32_t o[8];
#pragma unroll
            for (int r = 0; r < 8; ++r) o[r] = tbase + ((r < MT && ok && row0 + r < m) ? cv[b][r < MT ? r : 0] * 32u : 0u);  // T[0] = zero tables
            uint32_t *ow = reinterpret_cast<uint32_t *>(ent + 8);
#pragma unroll
            for (int r = 0; r < 8; r += 2) ow[r / 2] = o[r] | (o[r + 1] << 16);
        }
    }
}

// dec_expand for factored records (KFEC_DEC_EXPAND2): one column per thread (nj <= K < 256 = the workgroup),
// groups in batches of four whose two per-column bytes (src, lden) are loaded together; a group's header and the
// tile's 8 lnum / xm bytes are uniform (scalar loads), and each coefficient's T address is one lookup of its
// exponent in s_taddr -- no division of the flat entry index, no per-entry header loads, no exponent fold.
// staged_sync: the first chunk's barrier for the tables the workgroup staged (after the loads are issued).
template <int MT>
__device__ __forceinline__ void dec_expand_fac(const MacArgs &a, uint8_t *s_ent, uint32_t gfirst, uint32_t ng, uint32_t c0,
                                               uint32_t nj, uint32_t row0, const uint8_t *s_exp, const uint8_t *s_log,
                                               const uint16_t *s_taddr, uint32_t tbase, bool staged_sync)
{
    static_assert(MT >= 1 && MT <= 8, "entry: 8 offsets (rows past MT take the zero table)");
    typedef const __attribute__((address_space(4))) uint32_t cu32;
    const uint32_t K = a.K, K4 = (K + 3) & ~3u, L0 = fac_lnum_off(K), R8 = fac_r8(a.R);
    const bool has = threadIdx.x < nj;
    const uint32_t jj = has ? threadIdx.x : nj - 1, j = c0 + jj;
    constexpr uint32_t GB = 4;
    for (uint32_t gs0 = 0; gs0 < ng; gs0 += GB) {  // (uniform)
        uint32_t sv[GB], lv[GB];
#pragma unroll
        for (uint32_t b = 0; b < GB; ++b) {
            const uint8_t *rec = a.rec + (uint64_t)(gfirst + min(gs0 + b, ng - 1)) * a.rec_stride;
            sv[b] = rec[4 + j];
            lv[b] = rec[4 + K4 + j];
        }
        if (gs0 == 0 && staged_sync) __syncthreads();
#pragma unroll
        for (uint32_t b = 0; b < GB; ++b) {
            const uint32_t gs = gs0 + b;
            if (gs >= ng) break;
            const uint64_t g = __builtin_amdgcn_readfirstlane(gfirst + gs);  // (uniform: the record by scalar loads)
            const cu32 *rq = (const cu32 *)(a.rec + g * a.rec_stride);
            const uint32_t hd = rq[0];  // status | m << 8
            const uint32_t ln0 = rq[(L0 + row0) / 4], ln1 = rq[(L0 + row0) / 4 + 1];
            const uint32_t xm0 = rq[(L0 + R8 + row0) / 4], xm1 = rq[(L0 + R8 + row0) / 4 + 1];
            const uint32_t m = (hd >> 8) & 0xFFu;
            const uint32_t nrow = ((hd & 0xFFu) == 0 && m > row0) ? min(m - row0, (uint32_t)MT) : 0u;
            const uint32_t src = sv[b];
            const uint32_t xs = src ? (uint32_t)s_exp[src] : 0u;  // the point of the column's share (x_0 = 0)
            const uint32_t base = 510u - lv[b];
            uint32_t o[8];
#pragma unroll
            for (int r = 0; r < 8; ++r) {
                // coef = exp(lnum_u - log(xm_u ^ xs_j) - lden_j); rows past the group's m take T[0] (zero tables)
                const uint32_t lnr = ((r < 4 ? ln0 : ln1) >> (8 * (r & 3))) & 0xFFu;
                const uint32_t xmr = ((r < 4 ? xm0 : xm1) >> (8 * (r & 3))) & 0xFFu;
                o[r] = (r < MT && (uint32_t)r < nrow) ? (uint32_t)s_taddr[lnr + base - s_log[xmr ^ xs]] : tbase;
            }
            if (has) {
                const uint8_t *p = (src < K) ? a.data + (g * K + src) * a.pitch : a.parity + (g * a.R + (src - K)) * a.pitch;
                uint8_t *ent = s_ent + (gs * a.JC + jj) * kDecEntry;
                *reinterpret_cast<const uint8_t **>(ent) = p;
                uint32_t *ow = reinterpret_cast<uint32_t *>(ent + 8);
#pragma unroll
                for (int r = 0; r < 8; r += 2) ow[r / 2] = o[r] | (o[r + 1] << 16);
            }
        }
    }
}

// One lane = one (group, V-byte column) item; consecutive lanes take consecutive columns and wrap into the
// next group, so a wave-instruction reads 2 KiB of one shard row (V = 32).  One workgroup per 256 items
// (non-persistent grid: the dispatcher refills each CU as workgroups retire).  Per lane: K loads of V bytes
// (PD in flight), MT accumulator rows, MT stores.
template <int VEC, int MT, bool DEC, int PDX = 0>
__global__ void __launch_bounds__(kMacBlock, KFEC_MINW) mac_kernel(MacArgs a)
{
    using L = MacLayout<MT>;
    constexpr int W = Gran<VEC>::W;
    // shards in flight per lane (~64 B per lane); PDX: the latency shape (a handful of groups, often read
    // straight from pinned host memory) keeps many more loads in flight so the PCIe round trips overlap
    // (MT = 8, the VALU-bound tall tiles: 2, to keep 3 waves per SIMD)
    constexpr bool PAIRED = !DEC && (MT >= 8 || (KFEC_ENC_MT_MID == 1 && MT >= 5));
    constexpr int PD = PDX ? PDX : (VEC >= 32 ? (MT >= 8 || PAIRED || (DEC && dec_ttab(MT)) ? 2 : KFEC_MAC_PD)
                                               : 2 * KFEC_PD);
    constexpr int VB = VEC >= 4 ? VEC : 4;  // bytes per granule
    extern __shared__ __attribute__((aligned(16))) uint8_t s_ent[];

    if constexpr (DEC) {  // hybrid decode: the listed syndrome kernel has it (same rule as syn_listed)
        if (a.list_count && (uint64_t)*a.list_count * a.cols_pad < (uint64_t)a.G * a.cols) return;
    }
    uint32_t chunk, tile;
    block_chunk_tile(blockIdx.x, a.tiles, chunk, tile);
    const uint32_t base = chunk * kMacBlock;
    if (base >= a.total) return;  // padding chunk of the XCD-ordered tile grid (whole workgroup)
    const uint32_t row0 = tile * MT;
    const uint32_t K = a.K, cols = a.cols;
    const bool enc_once = !DEC && K <= a.JC;
    constexpr bool ttab = DEC && dec_ttab(MT);
    uint8_t *s_T = s_ent;
    // ttab: T, then (factored records) the GF exp / log tables, then the entries
    constexpr uint32_t kGfBytes = ttab ? kDecGfBytes : 0u;
    uint8_t *s_gexp = s_ent + kTBytes, *s_glog = s_gexp + 512;
    uint16_t *s_taddr = reinterpret_cast<uint16_t *>(s_gexp + 768);
    uint8_t *s_E = ttab ? s_ent + kTBytes + kGfBytes : s_ent;  // entries (after T)
    if (enc_once) {
        mac_expand<MT, false>(a, s_ent, 0, 1, 0, K, row0);
        __syncthreads();
    }
    if constexpr (ttab) {
        dec_build_t(s_T);  // (ordered by the first chunk's barrier below)
        if (a.factored) {
            stage_gf(s_gexp, s_glog);
            if (KFEC_DEC_EXPAND2) {
                const uint32_t tb = KFEC_DEC_OFS16 ? lds_addr(s_T) : 0u;
                for (uint32_t i = threadIdx.x; i < 768; i += blockDim.x) s_taddr[i] = (uint16_t)(tb + 32u * c_gf.exp[i % 255u]);
            }
        }
    }
    const uint32_t item = base + threadIdx.x;
    const bool in = item < a.total;
    const uint32_t g = in ? item / cols : 0;
    const uint32_t col = in ? item - g * cols : 0;
    const uint32_t off = gran_off<VEC>(col, a.B);
    const uint32_t gfirst = base / cols;
    const uint32_t glast = min(base + kMacBlock - 1, a.total - 1) / cols;
    const uint32_t ng = glast - gfirst + 1;
    const uint32_t gs = DEC ? g - gfirst : 0;

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

    const uint8_t *enc_base = a.data + ((uint64_t)g * K) * a.pitch + off;
    for (uint32_t c0 = 0; c0 < K; c0 += a.JC) {
        const uint32_t nj = min(a.JC, K - c0);
        if (!enc_once) {
            // (ttab: T is read only after the expansion's barrier; the factored form's GF tables are read by the
            // expansion itself -- dec_expand_fac waits for them after issuing its loads, dec_expand here)
            if (!ttab || c0 > 0 || (a.factored && !KFEC_DEC_EXPAND2)) __syncthreads();
            if constexpr (ttab) {
                const uint32_t tb = KFEC_DEC_OFS16 ? lds_addr(s_T) : 0u;
                if (KFEC_DEC_EXPAND2 && a.factored) dec_expand_fac<MT>(a, s_E, gfirst, ng, c0, nj, row0, s_gexp, s_glog, s_taddr, tb, c0 == 0);
                else dec_expand<MT>(a, s_E, gfirst, ng, c0, nj, row0, s_gexp, s_glog, tb);
            }
            else mac_expand<MT, DEC>(a, s_ent, gfirst, DEC ? ng : 1u, c0, nj, row0);
            __syncthreads();
        }
        if (rows == 0) continue;
        constexpr uint32_t ENT = ttab ? kDecEntry : L::ENTRY;
        const uint8_t *ent0 = s_E + (gs * a.JC) * ENT;
        auto share_ptr = [&](uint32_t jj) -> const uint8_t * {
            if constexpr (DEC) {
                return *reinterpret_cast<const uint8_t *const *>(ent0 + jj * ENT) + off;
            } else {
                return enc_base + (uint64_t)(c0 + jj) * a.pitch;
            }
        };
        // ttab: the T offsets of a shard are read one shard ahead, so the table reads of the shard being
        // multiplied depend on no LDS read still in flight.  KFEC_DEC_OFS16: one ds_read_u16 per row straight
        // into the register that addresses its table (no extraction op per row and shard: 8 of ~370 VALU ops)
        // instead of two 8-byte reads and a word-select add per row
        uint64_t ofs_lo = 0, ofs_hi = 0;
        uint32_t ofs16[MT];
        auto read_ofs = [&](uint32_t jj) {
            if constexpr (ttab) {
                if constexpr (KFEC_DEC_OFS16) {
                    // (volatile: kept as separate 2-byte reads, not merged into one wide read and split by VALU)
                    typedef const volatile __attribute__((address_space(3))) uint16_t lds_u16;
                    const lds_u16 *q = (const lds_u16 *)(ent0 + min(jj, nj - 1) * ENT + 8);
#pragma unroll
                    for (int r = 0; r < MT; ++r) ofs16[r] = q[r];
                } else {
                    const uint64_t *q = reinterpret_cast<const uint64_t *>(ent0 + min(jj, nj - 1) * ENT + 8);
                    ofs_lo = q[0];
                    ofs_hi = q[1];
                }
            }
        };
        auto mac = [&](const Gran<VEC> &cur, uint32_t jj) {
            uint32_t t[L::TBL_DW];
            if constexpr (ttab) {
                const uint64_t lo = ofs_lo, hi = ofs_hi;
                uint32_t oc[MT];
#pragma unroll
                for (int r = 0; r < MT; ++r) oc[r] = KFEC_DEC_OFS16 ? ofs16[r] : 0u;
                read_ofs(jj + 1);
#pragma unroll
                for (int r = 0; r < MT; ++r) {
                    const uint32_t o = KFEC_DEC_OFS16 ? oc[r] : (uint32_t)((r < 4 ? lo : hi) >> (16 * (r & 3))) & 0xFFFFu;
                    if constexpr (KFEC_DEC_OFS16) {  // o: the table's LDS address (dec_expand added T's base)
                        typedef unsigned int v4u __attribute__((ext_vector_type(4)));
                        typedef const __attribute__((address_space(3))) v4u lds_u4;
                        typedef const __attribute__((address_space(3))) uint32_t lds_u32;
                        const v4u q = *(const lds_u4 *)(uintptr_t)o;
                        t[5 * r] = q.x; t[5 * r + 1] = q.y; t[5 * r + 2] = q.z; t[5 * r + 3] = q.w;
                        t[5 * r + 4] = *(const lds_u32 *)(uintptr_t)(o + 16);
                    } else {
                        const uint8_t *te = s_T + o;
                        const uint4 q = *reinterpret_cast<const uint4 *>(te);
                        t[5 * r] = q.x; t[5 * r + 1] = q.y; t[5 * r + 2] = q.z; t[5 * r + 3] = q.w;
                        t[5 * r + 4] = *reinterpret_cast<const uint32_t *>(te + 16);
                    }
                }
            } else {
                const uint4 *tv = reinterpret_cast<const uint4 *>(ent0 + jj * ENT + 16);
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
                for (int r = 0; r < MT; ++r) acc[r][w] = KFEC_MAC_XORONLY ? acc[r][w] ^ xv : perm_mac(acc[r][w], t + 5 * r, s0, s1, s2);
            }
        };
        // PD shards in flight.  Every load is unconditional (past the end it re-reads the last shard, a
        // cache hit): a load under a branch makes hipcc wait for it at the branch's join, i.e. at issue.
        Gran<VEC> x[PD];
#pragma unroll
        for (int u = 0; u < PD; ++u) x[u] = load_gran<VEC>(share_ptr(min((uint32_t)u, nj - 1)), col, a.B);
        read_ofs(0);
        uint32_t jb = 0;
        for (; jb + PD <= nj; jb += PD) {
            if constexpr (!DEC && MT >= 3 && MT <= 4 && VEC >= 32 && KFEC_MAC_BURST == 2) {
                // every table of the PD granules first (one LDS burst), the PD MACs, then the next PD
                // granules' loads as one burst: 129 VGPRs at MT = 3 (3 waves per SIMD, from 98 and 5); encode
                // 20:3 2.2% and 8:4 4% faster, 10:3 within 1%, in an interleaved A/B (profiles/r05_enc_burst_ab.txt;
                // 20:1 was 0.9% slower, so MT < 3 keeps the interleaved loop); 4 waves per SIMD (launch bounds)
                // and the loads alone as a burst measured slower
                uint32_t tt[PD][L::TBL_DW];
#pragma unroll
                for (int u = 0; u < PD; ++u) {
                    const uint4 *tv = reinterpret_cast<const uint4 *>(ent0 + (jb + u) * ENT + 16);
#pragma unroll
                    for (int i = 0; i < L::TBL_DW / 4; ++i) {
                        const uint4 q = tv[i];
                        tt[u][4 * i] = q.x; tt[u][4 * i + 1] = q.y; tt[u][4 * i + 2] = q.z; tt[u][4 * i + 3] = q.w;
                    }
                }
                if constexpr (KFEC_MAC_PAIR_SMALL && !KFEC_MAC_XORONLY && PD % 2 == 0) {
#pragma unroll
                    for (int u = 0; u < PD; u += 2) {
#pragma unroll
                        for (int w = 0; w < W; ++w) {
                            const uint32_t xa = x[u].d[w], xb = x[u + 1].d[w];
                            const uint32_t sa0 = xa & 0x07070707u, sa1 = (xa >> 3) & 0x07070707u, sa2 = (xa >> 6) & 0x03030303u;
                            const uint32_t sb0 = xb & 0x07070707u, sb1 = (xb >> 3) & 0x07070707u, sb2 = (xb >> 6) & 0x03030303u;
#pragma unroll
                            for (int r = 0; r < MT; ++r) {
                                const uint32_t *ta = tt[u] + 5 * r, *tb = tt[u + 1] + 5 * r;
                                const uint32_t a0 = __builtin_amdgcn_perm(ta[1], ta[0], sa0);
                                const uint32_t a1 = __builtin_amdgcn_perm(ta[3], ta[2], sa1);
                                const uint32_t a2 = __builtin_amdgcn_perm(ta[4], ta[4], sa2);
                                const uint32_t b0 = __builtin_amdgcn_perm(tb[1], tb[0], sb0);
                                const uint32_t b1 = __builtin_amdgcn_perm(tb[3], tb[2], sb1);
                                const uint32_t b2 = __builtin_amdgcn_perm(tb[4], tb[4], sb2);
                                acc[r][w] = xor3(xor3(xor3(acc[r][w], a0, a1), a2, b0), b1, b2);
                            }
                        }
                    }
                } else {
#pragma unroll
                for (int u = 0; u < PD; ++u) {
#pragma unroll
                    for (int w = 0; w < W; ++w) {
                        const uint32_t xv = x[u].d[w];
                        const uint32_t s0 = xv & 0x07070707u;
                        const uint32_t s1 = (xv >> 3) & 0x07070707u;
                        const uint32_t s2 = (xv >> 6) & 0x03030303u;
#pragma unroll
                        for (int r = 0; r < MT; ++r)
                            acc[r][w] = KFEC_MAC_XORONLY ? acc[r][w] ^ xv : perm_mac(acc[r][w], tt[u] + 5 * r, s0, s1, s2);
                    }
                }
                }
#pragma unroll
                for (int u = 0; u < PD; ++u) x[u] = load_gran<VEC>(share_ptr(min(jb + u + PD, nj - 1)), col, a.B);
            } else if constexpr (PAIRED && VEC >= 32 && PD == 2 && KFEC_MAC_PAIR && !KFEC_MAC_XORONLY) {
                // the two shards of the trip together, row by row: 6 permutes and three 3-input XORs per row and dword
                // (one VALU op fewer than two separate MACs); the selectors of both granules stay live across the
                // rows, each row's two tables are read from LDS just before use (not all 8 rows' at once)
                uint32_t sa[W][3], sb[W][3];
#pragma unroll
                for (int w = 0; w < W; ++w) {
                    const uint32_t xa = x[0].d[w], xb = x[1].d[w];
                    sa[w][0] = xa & 0x07070707u; sa[w][1] = (xa >> 3) & 0x07070707u; sa[w][2] = (xa >> 6) & 0x03030303u;
                    sb[w][0] = xb & 0x07070707u; sb[w][1] = (xb >> 3) & 0x07070707u; sb[w][2] = (xb >> 6) & 0x03030303u;
                }
                const uint32_t *tA = reinterpret_cast<const uint32_t *>(ent0 + jb * ENT + 16);
                const uint32_t *tB = reinterpret_cast<const uint32_t *>(ent0 + (jb + 1) * ENT + 16);
#pragma unroll
                for (int r = 0; r < MT; ++r) {
                    uint32_t ta[5], tb[5];
#pragma unroll
                    for (int i = 0; i < 5; ++i) {
                        ta[i] = tA[5 * r + i];
                        tb[i] = tB[5 * r + i];
                    }
#pragma unroll
                    for (int w = 0; w < W; ++w) {
                        const uint32_t a0 = __builtin_amdgcn_perm(ta[1], ta[0], sa[w][0]);
                        const uint32_t a1 = __builtin_amdgcn_perm(ta[3], ta[2], sa[w][1]);
                        const uint32_t a2 = __builtin_amdgcn_perm(ta[4], ta[4], sa[w][2]);
                        const uint32_t b0 = __builtin_amdgcn_perm(tb[1], tb[0], sb[w][0]);
                        const uint32_t b1 = __builtin_amdgcn_perm(tb[3], tb[2], sb[w][1]);
                        const uint32_t b2 = __builtin_amdgcn_perm(tb[4], tb[4], sb[w][2]);
                        acc[r][w] = xor3(xor3(xor3(acc[r][w], a0, a1), a2, b0), b1, b2);
                    }
                }
#pragma unroll
                for (int u = 0; u < PD; ++u) x[u] = load_gran<VEC>(share_ptr(min(jb + u + PD, nj - 1)), col, a.B);
            } else if constexpr (DEC && ttab && KFEC_DEC_OFS16 && VEC >= 32 && PD == 2 && KFEC_DEC_PAIR && !KFEC_MAC_XORONLY) {
                // the decode's form of the same pairing: each row's two tables are read from T at the addresses the
                // two entries hold (dec_expand added T's base)
                typedef const volatile __attribute__((address_space(3))) uint16_t lds_u16;
                typedef unsigned int v4u __attribute__((ext_vector_type(4)));
                typedef const __attribute__((address_space(3))) v4u lds_u4;
                typedef const __attribute__((address_space(3))) uint32_t lds_u32;
                const lds_u16 *qa = (const lds_u16 *)(ent0 + jb * ENT + 8);
                const lds_u16 *qb = (const lds_u16 *)(ent0 + (jb + 1) * ENT + 8);
                uint32_t oa[MT], ob[MT];
#pragma unroll
                for (int r = 0; r < MT; ++r) {
                    oa[r] = qa[r];
                    ob[r] = qb[r];
                }
                uint32_t sa[W][3], sb[W][3];
#pragma unroll
                for (int w = 0; w < W; ++w) {
                    const uint32_t xa = x[0].d[w], xb = x[1].d[w];
                    sa[w][0] = xa & 0x07070707u; sa[w][1] = (xa >> 3) & 0x07070707u; sa[w][2] = (xa >> 6) & 0x03030303u;
                    sb[w][0] = xb & 0x07070707u; sb[w][1] = (xb >> 3) & 0x07070707u; sb[w][2] = (xb >> 6) & 0x03030303u;
                }
#pragma unroll
                for (int r = 0; r < MT; ++r) {
                    const v4u qa4 = *(const lds_u4 *)(uintptr_t)oa[r];
                    const v4u qb4 = *(const lds_u4 *)(uintptr_t)ob[r];
                    const uint32_t ta4 = *(const lds_u32 *)(uintptr_t)(oa[r] + 16);
                    const uint32_t tb4 = *(const lds_u32 *)(uintptr_t)(ob[r] + 16);
#pragma unroll
                    for (int w = 0; w < W; ++w) {
                        const uint32_t a0 = __builtin_amdgcn_perm(qa4.y, qa4.x, sa[w][0]);
                        const uint32_t a1 = __builtin_amdgcn_perm(qa4.w, qa4.z, sa[w][1]);
                        const uint32_t a2 = __builtin_amdgcn_perm(ta4, ta4, sa[w][2]);
                        const uint32_t b0 = __builtin_amdgcn_perm(qb4.y, qb4.x, sb[w][0]);
                        const uint32_t b1 = __builtin_amdgcn_perm(qb4.w, qb4.z, sb[w][1]);
                        const uint32_t b2 = __builtin_amdgcn_perm(tb4, tb4, sb[w][2]);
                        acc[r][w] = xor3(xor3(xor3(acc[r][w], a0, a1), a2, b0), b1, b2);
                    }
                }
#pragma unroll
                for (int u = 0; u < PD; ++u) x[u] = load_gran<VEC>(share_ptr(min(jb + u + PD, nj - 1)), col, a.B);
            } else if constexpr (!DEC && KFEC_MAC_BURST == 1) {
                // the PD granules' MACs, then the next PD granules' loads as one burst
#pragma unroll
                for (int u = 0; u < PD; ++u) mac(x[u], jb + u);
#pragma unroll
                for (int u = 0; u < PD; ++u) x[u] = load_gran<VEC>(share_ptr(min(jb + u + PD, nj - 1)), col, a.B);
            } else {
#pragma unroll
                for (int u = 0; u < PD; ++u) {
                    // consume, then refill the same registers: PD - 1 granules stay in flight during the MAC
                    // (loading first would need a fresh register set and a copy -- and a wait -- per iteration)
                    mac(x[u], jb + u);
                    x[u] = load_gran<VEC>(share_ptr(min(jb + u + PD, nj - 1)), col, a.B);
                }
            }
        }
        if constexpr (DEC && ttab && KFEC_DEC_OFS16 && VEC >= 32 && PD == 2 && KFEC_DEC_PAIR && !KFEC_MAC_XORONLY)
            read_ofs(jb);  // (the paired loop read its offsets itself: the tail's MAC takes shard jb's)
#pragma unroll
        for (int u = 0; u < PD; ++u)
            if (jb + u < nj) mac(x[u], jb + u);
    }
    if (rows) {
        const uint64_t obase = ((uint64_t)g * a.R + row0) * a.pitch + off;
#pragma unroll
        for (int r = 0; r < MT; ++r)
            if ((uint32_t)r < rows) store_gran<VEC>(a.out + obase + (uint64_t)r * a.pitch, acc[r], col, a.B);
    }
}

// ---------------------------------------------------------------------------------------------------
// (A11) syndrome-form decode MAC for R <= 8.
// The selected shares are every present data shard plus the m parity shares P_t (fecpp.cpp:528-548), and
// the recovered shards are D_M = Sinv * (P - E_P,present * D_present), where E is the parity part of the
// encoding matrix and Sinv the m x m inverse computed by the prep kernel.  Per column:
//   y_r = parity_r ^ XOR_{j present} E[r][j] * D_j     for every parity row r < RT  (the encode loop, with
//         the SAME wave-uniform tables for every group: scalar loads, no LDS, no pointer gather; a missing
//         data shard is simply not loaded, a parity row that is not used is not loaded)
//   out_u = XOR_r C[u][r] * y_r                         C[u][P_t - K] = Sinv[u][t], 0 for unused rows
// so the only per-group coefficients are the RT x RT bytes of C (LDS, built per workgroup).  Expanding the
// coefficient form instead (K x m per-group tables and share pointers in LDS before the first load) kept
// decode ~5-10% behind encode.  A group with nothing to recover (m = 0, the zero-loss case of
// fec_find_missings, client.cpp:923-925) issues no loads and no stores; a wave of such groups skips the loop.
// The product is the same linear map of the same shares as the reference's K x K inverse, so the bytes are
// the reference's.
// ---------------------------------------------------------------------------------------------------
struct SynArgs {
    const uint8_t *data;      // [G][K][pitch]
    const uint8_t *parity;    // [G][R][pitch]
    uint8_t *out;             // [G][R][pitch] recovered data shards, ascending index
    const uint8_t *rec;       // syndrome-form records (kfec_internal.hpp)
    const uint32_t *etab;     // [K][etab_rows][5] perm tables of the parity rows (zero slack rows)
    const uint32_t *list;     // ascending ids of the groups with data to recover (active_* kernels)
    const uint32_t *list_count;
    uint64_t pitch;
    uint32_t total, cols, cols_pad, G, K, R, B, rec_stride, etab_rows;
    uint32_t no_dense;        // hybrid decode: the coefficient-form MAC takes the dense shape (no syn_kernel launch)
};

template <int RT>
struct SynLayout {
    static constexpr int TD = ((5 * RT + 3) / 4) * 4;  // table dwords per (group, output row u): RT tables
};

typedef unsigned int u32x4v __attribute__((ext_vector_type(4)));

// One granule at byte offset o of a buffer resource.  An offset beyond the resource returns zeros and
// touches no memory: that is how an absent share is "not loaded" without a per-lane branch.
template <int VEC>
__device__ __forceinline__ Gran<VEC> bload(__amdgpu_buffer_rsrc_t r, uint32_t o)
{
    static_assert(VEC == 32 || VEC == 4, "dword granules");
    Gran<VEC> v;
    if constexpr (VEC == 32) {
        const u32x4v x = __builtin_amdgcn_raw_buffer_load_b128(r, o, 0, 0);
        const u32x4v y = __builtin_amdgcn_raw_buffer_load_b128(r, o + 16u, 0, 0);
        v.d[0] = x.x; v.d[1] = x.y; v.d[2] = x.z; v.d[3] = x.w;
        v.d[4] = y.x; v.d[5] = y.y; v.d[6] = y.z; v.d[7] = y.w;
    } else {
        v.d[0] = __builtin_amdgcn_raw_buffer_load_b32(r, o, 0, 0);
    }
    return v;
}

constexpr uint32_t kAbsent = 0x80000000u;  // beyond every resource (the host keeps them below 2^31 bytes)

// C tables of one group into LDS: tp[u * TD + 5 r + i] (zero for a group that recovers nothing)
template <int RT>
__device__ __forceinline__ void syn_expand_put(uint32_t c, uint32_t ur, uint32_t *tp)
{
    constexpr int TD = SynLayout<RT>::TD;
    const uint32_t u = ur / RT, r = ur - u * RT;
    uint32_t t[5];
    gf_perm_tables(c, t);
#pragma unroll
    for (int i = 0; i < 5; ++i) tp[u * TD + 5 * r + i] = t[i];
}

// C[u][r] of entry ur = u * RT + r of a record (0 unless status 0); both bytes are loaded unconditionally, so
// the two loads are in flight together
template <int RT>
__device__ __forceinline__ uint32_t syn_coef(const uint8_t *rec, uint32_t ur)
{
    const uint32_t u = ur / RT, r = ur - u * RT;
    const uint32_t st = rec[0], c = rec[40 + 8 * u + r];
    return st == 0 ? c : 0u;
}

template <int RT>
__device__ __forceinline__ void syn_expand_one(const uint8_t *rec, uint32_t ur, uint32_t *tp)
{
    syn_expand_put<RT>(syn_coef<RT>(rec, ur), ur, tp);
}

// y_r = parity_r ^ XOR_{j present} E[r][j] * D_j for one lane's column (rd / rp: resources over its group's
// data / parity rows, drow / prow: byte offsets of the lane's granule in the group's first data / parity row)
// ROWS: the parity rows computed (bit r = row r; a compile-time mask, so each variant is the plain unrolled loop).
// A group that lost m data shards uses m parity rows: syn_list_kernel (one group per task, so the mask is
// uniform) leaves out the rows its group does not use -- at ~1% loss mostly 2 of 3 (fec=20:3 listed decode
// 1.41 -> 1.23 ms, profiles/r04_rowmask_ab.txt).
template <int VEC, int RT, int PD, uint32_t ROWS = (1u << RT) - 1u, bool PAIR = (KFEC_SYN_PAIR & 1) != 0>
__device__ __forceinline__ void syn_loop(const SynArgs &a, uint32_t (&acc)[RT][Gran<VEC>::W], __amdgpu_buffer_rsrc_t rd,
                                         __amdgpu_buffer_rsrc_t rp, uint32_t drow, uint32_t prow, uint32_t used,
                                         uint64_t p0, const uint8_t *rec)
{
    constexpr int W = Gran<VEC>::W;
    const uint32_t K = a.K, pitch = (uint32_t)a.pitch;
    // the parity shares of the rows in use start the accumulators (issued with the first data loads)
#pragma unroll
    for (int r = 0; r < RT; ++r) {
        const Gran<VEC> y = bload<VEC>(rp, ((used >> r) & 1u) ? prow + r * pitch : kAbsent);
#pragma unroll
        for (int w = 0; w < W; ++w) acc[r][w] = y.d[w];
    }
    const uint64_t *pr = reinterpret_cast<const uint64_t *>(rec + 8);
    const uint64_t p1 = K > 64 ? pr[1] : 0ull, p2 = K > 128 ? pr[2] : 0ull, p3 = K > 192 ? pr[3] : 0ull;
    auto dofs = [&](uint32_t j) -> uint32_t {
        const uint64_t wq = j < 64 ? p0 : (j < 128 ? p1 : (j < 192 ? p2 : p3));
        return ((wq >> (j & 63u)) & 1ull) ? drow + j * pitch : kAbsent;
    };
    typedef const __attribute__((address_space(4))) uint32_t cu32;  // uniform: scalar loads into SGPRs
    uint32_t tn[5 * RT];  // KFEC_SYN_TPRE: shard j's tables, loaded while shard j - 1 is multiplied
    auto tload = [&](uint32_t j) {
        const cu32 *tg = (const cu32 *)(a.etab + (size_t)min(j, K - 1) * a.etab_rows * 5);
#pragma unroll
        for (int i = 0; i < 5 * RT; ++i) tn[i] = tg[i];
    };
    if (KFEC_SYN_TPRE) tload(0);
    auto mac = [&](const Gran<VEC> &cur, uint32_t j) {
        uint32_t t[5 * RT];
        if (KFEC_SYN_TPRE) {
#pragma unroll
            for (int i = 0; i < 5 * RT; ++i) t[i] = tn[i];
            tload(j + 1);
        } else {
            const cu32 *tg = (const cu32 *)(a.etab + (size_t)j * a.etab_rows * 5);
#pragma unroll
            for (int i = 0; i < 5 * RT; ++i) t[i] = tg[i];
        }
#pragma unroll
        for (int w = 0; w < W; ++w) {
            const uint32_t xv = cur.d[w];
            const uint32_t s0 = xv & 0x07070707u;
            const uint32_t s1 = (xv >> 3) & 0x07070707u;
            const uint32_t s2 = (xv >> 6) & 0x03030303u;
#pragma unroll
            for (int r = 0; r < RT; ++r)
                if ((ROWS >> r) & 1u)
                    acc[r][w] = KFEC_SYN_XORONLY == 2 ? acc[r][w] ^ xv
                                : KFEC_SYN_XORONLY ? acc[r][w] ^ xv ^ t[5 * r] : perm_mac(acc[r][w], t + 5 * r, s0, s1, s2);
        }
    };
    // PD shards in flight, every load unconditional (see mac_kernel)
    Gran<VEC> x[PD];
#pragma unroll
    for (int u = 0; u < PD; ++u) x[u] = bload<VEC>(rd, dofs(min((uint32_t)u, K - 1)));
    uint32_t jb = 0;
    if constexpr (PAIR && KFEC_SYN_TPRE && !KFEC_SYN_XORONLY && PD % 2 == 0 && RT <= 4) {
        // two shards per row step (mac_kernel's KFEC_MAC_PAIR): both shards' tables prefetched one pair ahead
        uint32_t tm[5 * RT];
        auto tload2 = [&](uint32_t j) {
            tload(j);
            const cu32 *tg = (const cu32 *)(a.etab + (size_t)min(j + 1, K - 1) * a.etab_rows * 5);
#pragma unroll
            for (int i = 0; i < 5 * RT; ++i) tm[i] = tg[i];
        };
        tload2(0);
        for (; jb + PD <= K; jb += PD) {
#pragma unroll
            for (int u = 0; u < PD; u += 2) {
                uint32_t ta[5 * RT], tb[5 * RT];
#pragma unroll
                for (int i = 0; i < 5 * RT; ++i) {
                    ta[i] = tn[i];
                    tb[i] = tm[i];
                }
                tload2(jb + u + 2);
#pragma unroll
                for (int w = 0; w < W; ++w) {
                    const uint32_t xa = x[u].d[w], xb = x[u + 1].d[w];
                    const uint32_t sa0 = xa & 0x07070707u, sa1 = (xa >> 3) & 0x07070707u, sa2 = (xa >> 6) & 0x03030303u;
                    const uint32_t sb0 = xb & 0x07070707u, sb1 = (xb >> 3) & 0x07070707u, sb2 = (xb >> 6) & 0x03030303u;
#pragma unroll
                    for (int r = 0; r < RT; ++r) {
                        if (!((ROWS >> r) & 1u)) continue;
                        const uint32_t *pa = ta + 5 * r, *pb = tb + 5 * r;
                        const uint32_t a0 = __builtin_amdgcn_perm(pa[1], pa[0], sa0);
                        const uint32_t a1 = __builtin_amdgcn_perm(pa[3], pa[2], sa1);
                        const uint32_t a2 = __builtin_amdgcn_perm(pa[4], pa[4], sa2);
                        const uint32_t b0 = __builtin_amdgcn_perm(pb[1], pb[0], sb0);
                        const uint32_t b1 = __builtin_amdgcn_perm(pb[3], pb[2], sb1);
                        const uint32_t b2 = __builtin_amdgcn_perm(pb[4], pb[4], sb2);
                        acc[r][w] = xor3(xor3(xor3(acc[r][w], a0, a1), a2, b0), b1, b2);
                    }
                }
                x[u] = bload<VEC>(rd, dofs(min(jb + u + PD, K - 1)));
                x[u + 1] = bload<VEC>(rd, dofs(min(jb + u + 1 + PD, K - 1)));
            }
        }
        tload(jb);  // the tail's single MACs take their tables through tn, shard jb first
    } else
    for (; jb + PD <= K; jb += PD) {
        // (the encode's burst order, KFEC_MAC_BURST, measured slower here, also at 3 or 2 waves per SIMD:
        // profiles/r05_syn_burst_ab.txt)
#pragma unroll
        for (int u = 0; u < PD; ++u) {
            mac(x[u], jb + u);
            x[u] = bload<VEC>(rd, dofs(min(jb + u + PD, K - 1)));
        }
    }
#pragma unroll
    for (int u = 0; u < PD; ++u)
        if (jb + u < K) mac(x[u], jb + u);
}

// out_u = XOR_r C[u][r] * y_r for u < m, stored to recovered slot u of group g
template <int VEC, int RT, uint32_t ROWS = (1u << RT) - 1u, bool OUTER = false>
__device__ __forceinline__ void syn_final(const SynArgs &a, const uint32_t (&acc)[RT][Gran<VEC>::W], const uint32_t *ct,
                                          uint32_t m, uint32_t g, uint32_t off, uint32_t col)
{
    constexpr int W = Gran<VEC>::W;
    constexpr int TD = SynLayout<RT>::TD;
    const uint64_t obase = ((uint64_t)g * a.R) * a.pitch + off;
    if constexpr (OUTER && RT >= 5 && RT != 7 && !KFEC_SYN_XORONLY) {
        // syndromes outer: y_r's selectors once per r, its contribution to every output row, then y_r is dead --
        // the output-row order below keeps all RT x W x 3 selectors live (192 VGPRs at RT 8)
        uint32_t o[RT][W];
#pragma unroll
        for (int u = 0; u < RT; ++u)
#pragma unroll
            for (int w = 0; w < W; ++w) o[u][w] = 0;
#pragma unroll
        for (int r = 0; r < RT; ++r) {
            if (!((ROWS >> r) & 1u)) continue;
            uint32_t sl[W][3];
#pragma unroll
            for (int w = 0; w < W; ++w) {
                const uint32_t yv = acc[r][w];
                sl[w][0] = yv & 0x07070707u; sl[w][1] = (yv >> 3) & 0x07070707u; sl[w][2] = (yv >> 6) & 0x03030303u;
            }
#pragma unroll
            for (int u = 0; u < RT; ++u) {
                if ((uint32_t)u < m) {
                    const uint32_t *tp = ct + u * TD + 5 * r;
                    uint32_t t[5];
#pragma unroll
                    for (int i = 0; i < 5; ++i) t[i] = tp[i];
#pragma unroll
                    for (int w = 0; w < W; ++w) o[u][w] = perm_mac(o[u][w], t, sl[w][0], sl[w][1], sl[w][2]);
                }
            }
        }
#pragma unroll
        for (int u = 0; u < RT; ++u)
            if ((uint32_t)u < m) store_gran<VEC>(a.out + obase + (uint64_t)u * a.pitch, o[u], col, a.B);
        return;
    }
#pragma unroll
    for (int u = 0; u < RT; ++u) {
        if ((uint32_t)u < m) {
            uint32_t t[TD];
            const uint4 *tv = reinterpret_cast<const uint4 *>(ct + u * TD);
#pragma unroll
            for (int i = 0; i < TD / 4; ++i) {
                const uint4 q = tv[i];
                t[4 * i] = q.x; t[4 * i + 1] = q.y; t[4 * i + 2] = q.z; t[4 * i + 3] = q.w;
            }
            uint32_t o[W];
#pragma unroll
            for (int w = 0; w < W; ++w) {
                uint32_t v = 0;
#pragma unroll
                for (int r = 0; r < RT; ++r) {
                    if (!((ROWS >> r) & 1u)) continue;  // (C[u][r] = 0 for a row no lane of the wave uses)
                    const uint32_t yv = acc[r][w];
                    v = KFEC_SYN_XORONLY == 2 ? v ^ yv : KFEC_SYN_XORONLY ? v ^ yv ^ t[5 * r]
                                         : perm_mac(v, t + 5 * r, yv & 0x07070707u, (yv >> 3) & 0x07070707u, (yv >> 6) & 0x03030303u);
                }
                o[w] = v;
            }
            store_gran<VEC>(a.out + obase + (uint64_t)u * a.pitch, o, col, a.B);
        }
    }
}

// f(std::integral_constant<uint32_t, ROWS>) for the wave-uniform row mask `rows` (RT <= 3: one variant per
// non-empty mask; wider tiles always compute every row)
template <int RT, typename F>
__device__ __forceinline__ void by_row_mask(uint32_t rows, F &&f)
{
    // KFEC_SYN_ROWMASK 2: single-row waves take a two-row variant (fewer registers)
    constexpr uint32_t one0 = KFEC_SYN_ROWMASK == 1 ? 1u : 3u, one1 = KFEC_SYN_ROWMASK == 1 ? 2u : 3u,
                       one2 = KFEC_SYN_ROWMASK == 1 ? 4u : 5u;
    if constexpr (RT == 2 && KFEC_SYN_ROWMASK != 0) {
        if (rows == 1) return f(std::integral_constant<uint32_t, one0>());
        if (rows == 2) return f(std::integral_constant<uint32_t, one1>());
    } else if constexpr (RT == 3 && KFEC_SYN_ROWMASK != 0) {
        switch (rows) {
        case 1: return f(std::integral_constant<uint32_t, one0>());
        case 2: return f(std::integral_constant<uint32_t, one1>());
        case 3: return f(std::integral_constant<uint32_t, 3>());
        case 4: return f(std::integral_constant<uint32_t, one2>());
        case 5: return f(std::integral_constant<uint32_t, 5>());
        case 6: return f(std::integral_constant<uint32_t, 6>());
        default: break;
        }
    }
    f(std::integral_constant<uint32_t, (1u << RT) - 1u>());
}

// Two launch shapes, chosen per launch ON THE DEVICE from the number of groups with data to recover (the
// prep's list count; no host round trip).  Both kernels are launched; the one not chosen exits at once.
//  * dense (syn_kernel: most groups lost a data shard, e.g. the m = R benchmark configs): lane = (group,
//    column) over all groups, exactly the encode's item order; groups with nothing to recover issue no loads;
//  * listed (syn_list_kernel: few groups lost data, e.g. a live link at ~1% loss, where fec_find_missings
//    decodes every group that reached K shares, client.cpp:923-925): one wave per (listed group, 64 columns),
//    persistent over the ascending list of active groups only, so the work is proportional to the groups that
//    lost data instead of to the waves that hold one of them.
// Listed is taken when it needs fewer lanes: cnt * cols_pad < G * cols.
__device__ __forceinline__ bool syn_listed(const SynArgs &a, uint32_t cnt)
{
    return (uint64_t)cnt * a.cols_pad < (uint64_t)a.G * a.cols;
}

template <int VEC, int RT, int PDX = 0>
__global__ void __launch_bounds__(kMacBlock) syn_list_kernel(SynArgs a)
{
    constexpr int W = Gran<VEC>::W;
    constexpr int PD = PDX ? PDX : (VEC >= 32 ? KFEC_PD : 2 * KFEC_PD);
    constexpr int TD = SynLayout<RT>::TD;
    __shared__ __attribute__((aligned(16))) uint32_t s_ct[kMacBlock / 64][RT * TD];
    const uint32_t cnt = *a.list_count;
    if (!syn_listed(a, cnt)) return;
    const uint32_t wpg = a.cols_pad / 64;  // waves per group
    const uint32_t lane = threadIdx.x & 63u;
    uint32_t *ct = s_ct[threadIdx.x / 64];  // this wave's C tables (written and read by this wave only)
    const uint32_t tasks = cnt * wpg;
    for (uint32_t t = blockIdx.x * (kMacBlock / 64) + threadIdx.x / 64; t < tasks; t += gridDim.x * (kMacBlock / 64)) {
        const uint32_t li = __builtin_amdgcn_readfirstlane(t / wpg);
        const uint32_t col = (t - li * wpg) * 64 + lane;
        const uint32_t g = __builtin_amdgcn_readfirstlane(a.list[li]);
        const uint8_t *rec = a.rec + (uint64_t)g * a.rec_stride;
        if (lane < RT * RT) syn_expand_one<RT>(rec, lane, ct);
        const bool in = col < a.cols;
        const uint32_t off = gran_off<VEC>(in ? col : 0u, a.B);
        const uint4 h = *reinterpret_cast<const uint4 *>(rec);  // header + present data bits 0..63
        const uint32_t m = (h.x >> 8) & 0xFFu;  // listed groups have status 0 and m > 0
        const uint32_t used = (h.x >> 16) & 0xFFu;
        const uint64_t p0 = (uint64_t)h.z | ((uint64_t)h.w << 32);
        const uint32_t wrows = __builtin_amdgcn_readfirstlane(used);  // (one group per task: uniform)
        by_row_mask<RT>(wrows, [&](auto rows_c) {
            constexpr uint32_t ROWS = decltype(rows_c)::value;
            uint32_t acc[RT][W];
            if (in) {
                const __amdgpu_buffer_rsrc_t rd = __builtin_amdgcn_make_buffer_rsrc(
                    (void *)(a.data + (uint64_t)g * a.K * a.pitch), (short)0, (int)(a.K * a.pitch), 0x00020000);
                const __amdgpu_buffer_rsrc_t rp = __builtin_amdgcn_make_buffer_rsrc(
                    (void *)(a.parity + (uint64_t)g * a.R * a.pitch), (short)0, (int)(a.R * a.pitch), 0x00020000);
                syn_loop<VEC, RT, PD, ROWS, (KFEC_SYN_PAIR & 2) != 0>(a, acc, rd, rp, off, off, used, p0, rec);
            }
            // the tables were written by lanes of this wave: LDS operations of one wave complete in order, the
            // fence keeps the compiler from moving the reads above the writes
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
            if (in) syn_final<VEC, RT, ROWS, KFEC_SYN_FINAL_ROWS != 0>(a, acc, ct, m, g, off, col);
        });
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");  // the next task rewrites the tables
    }
}

#ifndef KFEC_SYN_WAVE_CT
#define KFEC_SYN_WAVE_CT 1  // 0: one set of C tables per workgroup behind a workgroup barrier (A/B knob)
#endif
// groups one wave of 64 consecutive items can touch
__host__ __device__ constexpr uint32_t syn_wave_groups(size_t cols) { return (uint32_t)(63 / (cols ? cols : 1) + 2); }

template <int VEC, int RT, int PDX = 0>
__global__ void __launch_bounds__(kMacBlock, KFEC_SYN_MINW) syn_kernel(SynArgs a)
{
    constexpr int W = Gran<VEC>::W;
    constexpr int PD = PDX ? PDX : (VEC >= 32 ? KFEC_PD : 2 * KFEC_PD);
    constexpr int TD = SynLayout<RT>::TD;
    extern __shared__ __attribute__((aligned(16))) uint32_t s_ct[];  // [wave][group slot][RT][TD] or [group slot][RT][TD]
    if (a.list_count && syn_listed(a, *a.list_count)) return;  // the listed kernel has it (whole workgroup)
    const uint32_t base = xcd_chunk(blockIdx.x) * kMacBlock;
    if (base >= a.total) return;  // padding chunk of the XCD-ordered grid (whole workgroup)
    const uint32_t cols = a.cols, K = a.K;
    const uint32_t gfirst = base / cols;
#if KFEC_SYN_WAVE_CT
    // C tables of the groups this wave touches, built and read by this wave only: no workgroup barrier, so a
    // wave that finishes its shards does not wait for the slowest wave of the workgroup
    const uint32_t wbase = min(base + (threadIdx.x & ~63u), a.total - 1);
    const uint32_t wfirst = wbase / cols, wlast = min(wbase + 63, a.total - 1) / cols;
    uint32_t *ctw = s_ct + (threadIdx.x / 64) * syn_wave_groups(cols) * RT * TD;
    const uint32_t ne = (wlast - wfirst + 1) * RT * RT;
#if KFEC_SYN_EARLY
    // the first 64 entries' coefficient bytes are loaded now, with the record header below, and expanded into
    // LDS after the shard loop: the shard loads wait for one dependent load (the header), not three
    const uint32_t e0 = threadIdx.x & 63u;
    const uint32_t e0g = min(e0, ne - 1) / (RT * RT);
    const uint32_t c_e0 = syn_coef<RT>(a.rec + (uint64_t)(wfirst + e0g) * a.rec_stride, min(e0, ne - 1) - e0g * (RT * RT));
#else
    for (uint32_t e = threadIdx.x & 63u; e < ne; e += 64) {
        const uint32_t gs = e / (RT * RT);
        syn_expand_one<RT>(a.rec + (uint64_t)(wfirst + gs) * a.rec_stride, e - gs * (RT * RT), ctw + gs * RT * TD);
    }
#endif
#else
    const uint32_t glast = min(base + kMacBlock - 1, a.total - 1) / cols;
    const uint32_t ng = glast - gfirst + 1;
    // C tables of the workgroup's groups
    for (uint32_t e = threadIdx.x; e < ng * RT * RT; e += kMacBlock) {
        const uint32_t gs = e / (RT * RT);
        syn_expand_one<RT>(a.rec + (uint64_t)(gfirst + gs) * a.rec_stride, e - gs * (RT * RT), s_ct + gs * RT * TD);
    }
#endif
    const uint32_t item = base + threadIdx.x;
    const bool in = item < a.total;
    const uint32_t g = in ? item / cols : gfirst;
    const uint32_t col = in ? item - g * cols : 0;
    const uint32_t off = gran_off<VEC>(col, a.B);
    const uint32_t gs = g - gfirst;
    uint32_t m = 0, used = 0;
    uint64_t p0 = 0;
    const uint8_t *rec = a.rec + (uint64_t)g * a.rec_stride;
    if (in) {
        const uint4 h = *reinterpret_cast<const uint4 *>(rec);  // header + present data bits 0..63
        if ((h.x & 0xFFu) == 0) {
            m = (h.x >> 8) & 0xFFu;
            used = (h.x >> 16) & 0xFFu;
        }
        p0 = (uint64_t)h.z | ((uint64_t)h.w << 32);
    }
    const bool active = m > 0;
    // (every parity row: the row-mask variants of syn_list_kernel cost this shape a register budget of 143
    // VGPRs and 3% at m = R, and gain nothing with random 1-3 erasures of 13; profiles/r04_rowmask_ab.txt)
    uint32_t acc[RT][W];
    if (active) {
        // resources over this workgroup's groups (wave-uniform: blockIdx and kernel arguments only)
        const uint32_t ngr = min(base + kMacBlock - 1, a.total - 1) / cols - gfirst + 1;
        const __amdgpu_buffer_rsrc_t rd = __builtin_amdgcn_make_buffer_rsrc(
            (void *)(a.data + (uint64_t)gfirst * K * a.pitch), (short)0, (int)(ngr * K * a.pitch), 0x00020000);
        const __amdgpu_buffer_rsrc_t rp = __builtin_amdgcn_make_buffer_rsrc(
            (void *)(a.parity + (uint64_t)gfirst * a.R * a.pitch), (short)0, (int)(ngr * a.R * a.pitch), 0x00020000);
        syn_loop<VEC, RT, PD>(a, acc, rd, rp, gs * K * (uint32_t)a.pitch + off, gs * a.R * (uint32_t)a.pitch + off, used,
                              p0, rec);
    }
#if KFEC_SYN_WAVE_CT
#if KFEC_SYN_EARLY
    if (e0 < ne) syn_expand_put<RT>(c_e0, e0 - e0g * (RT * RT), ctw + e0g * RT * TD);
    for (uint32_t e = e0 + 64; e < ne; e += 64) {  // (more than 64 entries: pitch < 64 bytes per group)
        const uint32_t gs = e / (RT * RT);
        syn_expand_one<RT>(a.rec + (uint64_t)(wfirst + gs) * a.rec_stride, e - gs * (RT * RT), ctw + gs * RT * TD);
    }
#endif
    // written by lanes of this wave: LDS operations of one wave complete in order; the fence keeps the
    // compiler from moving the reads above the writes
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    if (active) syn_final<VEC, RT>(a, acc, ctw + (g - wfirst) * RT * TD, m, g, off, col);
#else
    __syncthreads();  // C tables
    if (active) syn_final<VEC, RT>(a, acc, s_ct + gs * RT * TD, m, g, off, col);
#endif
}

// ---- ordered list of the groups with data to recover (out_idx[g * R] != 0xFF), for syn_kernel's listed
// shape: per-chunk counts, one exclusive scan, a scatter that keeps group order.  kActChunk groups per
// 256-thread workgroup, 4 per thread.
constexpr uint32_t kActChunk = 1024;

__device__ __forceinline__ uint32_t act_flags(uint64_t G, uint32_t R, const uint8_t *out_idx, uint64_t g0)
{
    uint32_t f = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const uint64_t g = g0 + k;
        if (g < G && out_idx[g * R] != 0xFF) f |= 1u << k;
    }
    return f;
}

// exclusive prefix of v over the 256 threads of the workgroup (and the total)
__device__ __forceinline__ uint32_t block_exclusive(uint32_t v, uint32_t *s_w, uint32_t &total)
{
    const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
    uint32_t x = v;  // inclusive scan within the wave
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(x, d);
        if (lane >= (uint32_t)d) x += y;
    }
    if (lane == 63) s_w[wv] = x;
    __syncthreads();
    uint32_t before = 0;
    total = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const uint32_t t = s_w[k];
        if ((uint32_t)k < wv) before += t;
        total += t;
    }
    return before + x - v;
}

__global__ void __launch_bounds__(kBlock) active_count_kernel(uint64_t G, uint32_t R, const uint8_t *out_idx,
                                                              uint32_t *chunk_cnt)
{
    __shared__ uint32_t s_w[4];
    const uint64_t g0 = (uint64_t)blockIdx.x * kActChunk + threadIdx.x * 4u;
    uint32_t total = 0;
    (void)block_exclusive(__popc(act_flags(G, R, out_idx, g0)), s_w, total);
    if (threadIdx.x == 0) chunk_cnt[blockIdx.x] = total;
}

// one workgroup: chunk counts -> exclusive chunk offsets (in place), total -> *count
__global__ void __launch_bounds__(kBlock) active_scan_kernel(uint32_t nchunks, uint32_t *chunk_cnt, uint32_t *count)
{
    __shared__ uint32_t s_w[4];
    uint32_t carry = 0;
    for (uint32_t c0 = 0; c0 < nchunks; c0 += kBlock) {
        const uint32_t c = c0 + threadIdx.x;
        const uint32_t v = c < nchunks ? chunk_cnt[c] : 0u;
        uint32_t total = 0;
        const uint32_t ex = block_exclusive(v, s_w, total);
        if (c < nchunks) chunk_cnt[c] = carry + ex;
        carry += total;
        __syncthreads();  // s_w is reused by the next round
    }
    if (threadIdx.x == 0) *count = carry;
}

__global__ void __launch_bounds__(kBlock) active_scatter_kernel(uint64_t G, uint32_t R, const uint8_t *out_idx,
                                                                const uint32_t *chunk_off, uint32_t *list)
{
    __shared__ uint32_t s_w[4];
    const uint64_t g0 = (uint64_t)blockIdx.x * kActChunk + threadIdx.x * 4u;
    const uint32_t f = act_flags(G, R, out_idx, g0);
    uint32_t total = 0;
    uint32_t at = chunk_off[blockIdx.x] + block_exclusive(__popc(f), s_w, total);
#pragma unroll
    for (int k = 0; k < 4; ++k)
        if ((f >> k) & 1u) list[at++] = (uint32_t)(g0 + k);
}

// ---------------------------------------------------------------------------------------------------
// host-side launch helpers
// ---------------------------------------------------------------------------------------------------
// Batches of at most kLatencyGroups groups (the single-group drop-in calls, whose shares sit in pinned host
// memory) run the MAC with 4-byte granules and 16 shards in flight per lane: ~8x more lanes and loads in
// flight than the streaming shape, so the PCIe round trips of a 29 KB group overlap instead of queueing.
constexpr int kLatencyVec = -4;
constexpr size_t kLatencyGroups = 4;

// granule of the MAC kernels: 32 B whenever the pitch and every base pointer are dword aligned (the tail
// granule of a row is loaded / stored dword by dword), bytewise otherwise
static int pick_vec_mac(size_t pitch, size_t B, std::initializer_list<const void *> ptrs)
{
    bool ok = (pitch % 4) == 0;
    for (const void *p : ptrs) ok = ok && (reinterpret_cast<uintptr_t>(p) % 4) == 0;
    if (!ok) return 1;
    return B >= 32 ? 32 : kLatencyVec;  // (B < 32: the dword shape, one granule per dword)
}

// output rows per tile: MT = R up to 4, else 8-row tiles.  Measured at 200:55: taller tiles on
// narrower granules read each input byte fewer times but are no faster (VALU-bound there, and 32-B
// granules amortise each table read over the most bytes).
static int pick_mt(int R) { return R <= 4 ? std::max(R, 1) : 8; }

// The encode's row tile for 32-byte granules.  R <= 8: one tile of R rows (R = 5..7 with the paired MAC, KFEC_ENC_MT_MID).
// R > 8: the height among 5..8 and 10 of least modelled VALU per (shard, dword) -- tiles x (4.5 per row for the paired
// MAC + 5 for the selector extractions every tile repeats), ties to the taller tile.  All of them run at 3 or more
// waves per SIMD (127-167 VGPRs) at about the same cost per row, so the rows a partial last tile wastes decide:
// 40:20 and 30:20 two 10-row tiles instead of three 8-row ones (11.86 -> 9.98 ms, 9.03 -> 7.78), 30:12 two of 6
// (26.05 -> 22.54 ms), 20:13 two of 7 (18.7 -> 17.7), 25:25 five of 5 (19.9 -> 18.8); 200:55 keeps 7 x 8 (10-row tiles
// compute 60 rows: 140.4 against 132.2 ms); 11-row tiles need 175 VGPRs, 2 waves (profiles/r06_mt_tall_ab.txt,
// profiles/r06_mt_model_ab.txt)
static int pick_mt_enc(int R)
{
    if (R <= 8) return KFEC_ENC_MT_MID != 0 && R >= 5 ? R : pick_mt(R);
    int best = 8, best_cost = 1 << 30;
    for (int mt : {10, 8, 7, 6, 5}) {
        if (KFEC_ENC_MT_MID == 0 && mt < 8) continue;
        const int cost = (R + mt - 1) / mt * (9 * mt + 10);
        if (cost < best_cost) best = mt, best_cost = cost;
    }
    return best;
}


#if KFEC_MAC_XORONLY || KFEC_SYN_XORONLY
// The arithmetic-free ceiling build only (tools/libkfec_arithfree.so): KFEC_AF_WAVES = n caps a launch at n 256-lane
// workgroups (n waves) per SIMD by padding its LDS, so bench.py can time the access pattern at the product's own
// occupancy too -- without its GF arithmetic the kernel needs fewer registers and would otherwise run more waves
// than the product (20:3 encode: 74 VGPRs against 129), which measured slower than the product itself.
static size_t af_lds(size_t lds)
{
    const char *e = std::getenv("KFEC_AF_WAVES");
    const long n = e ? std::strtol(e, nullptr, 10) : 0;
    if (n < 2) return lds;
    const size_t need = (size_t)160 * 1024 / (size_t)(n + 1) + 64;  // > 1/(n+1) of the CU's 160 KiB
    return std::max(lds, std::min<size_t>(need, 64 * 1024));
}
#else
static size_t af_lds(size_t lds) { return lds; }
#endif

template <int VEC, int MT, bool DEC, int PDX = 0>
static int run_mac(MacArgs a, hipStream_t s)
{
    using L = MacLayout<MT>;
    const size_t lds = af_lds((DEC && dec_ttab(MT)) ? kTBytes + kDecGfBytes + (size_t)a.gmax * a.JC * kDecEntry
                                                                : (size_t)a.gmax * a.JC * L::ENTRY);
    const uint32_t chunks = (a.total + kMacBlock - 1) / kMacBlock;
    const uint32_t nb = a.tiles > 1 ? xcd_tile_chunks(chunks) * a.tiles : xcd_grid(chunks);
    hipLaunchKernelGGL((mac_kernel<VEC, MT, DEC, PDX>), dim3(std::max(1u, nb)), dim3(kMacBlock), lds, s, a);
    return hipGetLastError() == hipSuccess ? 0 : -3;
}

template <bool DEC>
static int dispatch_mac(int vec, int mt, MacArgs a, hipStream_t s)
{
#if KFEC_SYN_MAX_R > 0
    if constexpr (DEC) {  // coefficient-form decode: R > 8, 8-row tiles only
        (void)mt;
        if (vec == kLatencyVec) return run_mac<4, 8, true, 16>(a, s);
        if constexpr (KFEC_DEC_MT_SMALL != 0)
            if (vec == 32 && mt == 4) return run_mac<32, 4, true>(a, s);
        if constexpr (KFEC_DEC_MT_MID != 0) {
            if (vec == 32 && mt == 5) return run_mac<32, 5, true>(a, s);
            if (vec == 32 && mt == 6) return run_mac<32, 6, true>(a, s);
            if (vec == 32 && mt == 7) return run_mac<32, 7, true>(a, s);
        }
        if (vec == 32) return run_mac<32, 8, true>(a, s);
        return run_mac<1, 8, true>(a, s);
    }
#endif
    if (vec == kLatencyVec) {  // the latency shape: dword granules, 16 shards in flight per lane
        switch (mt) {
        case 1: return run_mac<4, 1, DEC, 16>(a, s);
        case 2: return run_mac<4, 2, DEC, 16>(a, s);
        case 3: return run_mac<4, 3, DEC, 16>(a, s);
        case 4: return run_mac<4, 4, DEC, 16>(a, s);
        default: return run_mac<4, 8, DEC, 16>(a, s);
        }
    }
    if (vec == 32) {
        if constexpr (!DEC) {
            if (mt == 10) return run_mac<32, 10, false>(a, s);
            if constexpr (KFEC_ENC_MT_MID != 0) {
                if (mt == 5) return run_mac<32, 5, false>(a, s);
                if (mt == 6) return run_mac<32, 6, false>(a, s);
                if (mt == 7) return run_mac<32, 7, false>(a, s);
            }
        }
        switch (mt) {
        case 1: return run_mac<32, 1, DEC>(a, s);
        case 2: return run_mac<32, 2, DEC>(a, s);
        case 3: return run_mac<32, 3, DEC>(a, s);
        case 4: return run_mac<32, 4, DEC>(a, s);
        default: return run_mac<32, 8, DEC>(a, s);
        }
    }
    switch (mt) {
    case 1: return run_mac<1, 1, DEC>(a, s);
    case 2: return run_mac<1, 2, DEC>(a, s);
    case 3: return run_mac<1, 3, DEC>(a, s);
    case 4: return run_mac<1, 4, DEC>(a, s);
    default: return run_mac<1, 8, DEC>(a, s);
    }
}

static int entry_bytes(int mt)
{
    switch (mt) {
    case 1: return MacLayout<1>::ENTRY;
    case 2: return MacLayout<2>::ENTRY;
    case 3: return MacLayout<3>::ENTRY;
    case 4: return MacLayout<4>::ENTRY;
    case 5: return MacLayout<5>::ENTRY;
    case 6: return MacLayout<6>::ENTRY;
    case 7: return MacLayout<7>::ENTRY;
    case 10: return MacLayout<10>::ENTRY;
    default: return MacLayout<8>::ENTRY;
    }
}


static size_t syn_td(int rt)
{
    switch (rt) {
    case 1: return SynLayout<1>::TD;
    case 2: return SynLayout<2>::TD;
    case 3: return SynLayout<3>::TD;
    case 4: return SynLayout<4>::TD;
    case 5: return SynLayout<5>::TD;
    case 6: return SynLayout<6>::TD;
    case 7: return SynLayout<7>::TD;
    default: return SynLayout<8>::TD;
    }
}

#ifndef KFEC_SYN_WAVES
#define KFEC_SYN_WAVES 0  // syn_kernel capped at this many workgroups (= waves) per SIMD by padding its LDS (0: no cap)
#endif
static size_t syn_cap(size_t lds)
{
    if (KFEC_SYN_WAVES < 2) return lds;
    return std::max(lds, std::min<size_t>((size_t)160 * 1024 / (KFEC_SYN_WAVES + 1) + 64, 64 * 1024));
}

template <int VEC, int RT, int PDX = 0>
static int run_syn(SynArgs a, size_t lds, int cus, hipStream_t s)
{
    const uint32_t nb = xcd_grid((a.total + kMacBlock - 1) / kMacBlock);
    if (!a.no_dense)
        hipLaunchKernelGGL((syn_kernel<VEC, RT, PDX>), dim3(std::max(1u, nb)), dim3(kMacBlock), af_lds(syn_cap(lds)), s, a);
    if (!a.list_count) return hipGetLastError() == hipSuccess ? 0 : -3;  // dense only
    // the listed shape: persistent, ~8 workgroups per CU, at most one wave per (group, 64 columns) task
    const uint64_t tasks = (uint64_t)a.G * (a.cols_pad / 64);
    const uint32_t nl = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>((tasks + 3) / 4, (uint64_t)std::max(cus, 1) * 8));
    hipLaunchKernelGGL((syn_list_kernel<VEC, RT, PDX>), dim3(nl), dim3(kMacBlock), 0, s, a);
    return hipGetLastError() == hipSuccess ? 0 : -3;
}

static int dispatch_syn(int vec, int rt, SynArgs a, size_t lds, int cus, hipStream_t s)
{
#define KFEC_RT_CASES(V, P)                                                          \
    do {                                                                             \
        switch (rt) {                                                                \
        case 1: return run_syn<V, 1, P>(a, lds, cus, s);                             \
        case 2: return run_syn<V, 2, P>(a, lds, cus, s);                             \
        case 3: return run_syn<V, 3, P>(a, lds, cus, s);                             \
        case 4: return run_syn<V, 4, P>(a, lds, cus, s);                             \
        case 5: if constexpr (KFEC_SYN_RT_MID != 0) return run_syn<V, 5, P>(a, lds, cus, s); break; \
        case 6: if constexpr (KFEC_SYN_RT_MID != 0) return run_syn<V, 6, P>(a, lds, cus, s); break; \
        case 7: if constexpr (KFEC_SYN_RT_MID != 0) return run_syn<V, 7, P>(a, lds, cus, s); break; \
        default: break;                                                              \
        }                                                                            \
        return run_syn<V, 8, P>(a, lds, cus, s);                                     \
    } while (0)
    if (vec == kLatencyVec) KFEC_RT_CASES(4, 16);
#if KFEC_SYN_SMALLK_PD > 0
    if (a.K <= 12) KFEC_RT_CASES(32, KFEC_SYN_SMALLK_PD);
#endif
    KFEC_RT_CASES(32, 0);
#undef KFEC_RT_CASES
}

static constexpr size_t kLdsBudget = 32 * 1024;
static constexpr size_t kDecLdsBudget = 40 * 1024;  // T-table decode entries (+ 8 KiB of T): 3 workgroups per CU
static constexpr size_t kSynLdsMax = 64 * 1024;
static constexpr size_t kMaxItemsPerLaunch = 0x7FFFFFFFu;

// split G into launches whose item count (x row tiles) fits 32-bit indexing
template <typename F>
static int for_group_ranges(size_t G, size_t cols, size_t tiles, F &&f)
{
    const size_t cap = kMaxItemsPerLaunch / std::max<size_t>(tiles, 1) / std::max<size_t>(cols, 1);
    const size_t gmax_launch = std::max<size_t>(1, cap);
    for (size_t g0 = 0; g0 < G; g0 += gmax_launch) {
        const int rc = f(g0, std::min(gmax_launch, G - g0));
        if (rc) return rc;
    }
    return 0;
}

int launch_encode(const DeviceInfo &di, const uint8_t *d_enc, int K, int N, size_t G, size_t B, size_t pitch,
                  const void *d_data, void *d_parity, hipStream_t s)
{
    (void)di;
    const int R = N - K;
    if (R == 0 || G == 0 || B == 0) return 0;
    int vec = pick_vec_mac(pitch, B, {d_data, d_parity});
    if (G <= kLatencyGroups && vec >= 4) vec = kLatencyVec;
    const int mt = vec == 32 ? pick_mt_enc(R) : pick_mt(R);
    const int vb = vec >= 4 ? vec : 4;
    const size_t cols = (B + vb - 1) / vb;
    const int tiles = (R + mt - 1) / mt;
    const size_t ent = entry_bytes(mt);
    const uint32_t JC = (uint32_t)std::max<size_t>(1, std::min<size_t>(K, kLdsBudget / ent));
    return for_group_ranges(G, cols, tiles, [&](size_t g0, size_t gn) {
        MacArgs a{};
        a.data = static_cast<const uint8_t *>(d_data) + g0 * K * pitch;
        a.parity = nullptr;
        a.out = static_cast<uint8_t *>(d_parity) + g0 * R * pitch;
        a.enc = d_enc;
        a.rec = nullptr;
        a.pitch = pitch;
        a.total = (uint32_t)(gn * cols);
        a.cols = (uint32_t)cols;
        a.G = (uint32_t)gn;
        a.K = K; a.R = R; a.B = (uint32_t)B;
        a.rec_stride = 0;
        a.JC = JC;
        a.gmax = 1;
        a.tiles = (uint32_t)tiles;
        return dispatch_mac<false>(vec, mt, a, s);
    });
}

// decode_prep_*: share selection, the m x m solve and the coefficient rows (or, syn = true, the syndrome-form
// records) of every group into d_workspace (+ d_out_idx, d_status).  The MAC kernels here and in
// kfec_frame.hip consume them.
int launch_decode_prep(const DeviceInfo &di, const uint8_t *d_enc, int K, int N, size_t G, const uint64_t *d_present,
                       uint8_t *d_out_idx, uint8_t *d_status, void *d_workspace, hipStream_t s, bool syn, bool factored,
                       const uint32_t *skip_listed, uint32_t cols, uint32_t cols_pad)
{
    const int R = N - K;
    if (G == 0) return 0;
    uint8_t *rec = static_cast<uint8_t *>(d_workspace);
    factored = factored && !syn && std::min(K, R) > 8;  // (only decode_prep_lagrange writes the factored form)
    const size_t rs = syn ? syn_record_stride(K, R) : factored ? fac_record_stride(K, R) : record_stride(K, R);
    PrepArgs p{};
    p.present = d_present;
    p.enc = d_enc;
    p.rec = rec;
    p.out_idx = d_out_idx;
    p.status = d_status;
    p.G = G;
    p.K = K; p.N = N; p.R = R;
    p.rec_stride = (uint32_t)rs;
    p.syn = syn ? 1 : 0;
    p.factored = factored ? 1 : 0;
    p.skip_listed = skip_listed;
    p.cols = cols;
    p.cols_pad = cols_pad;
    const int mmax = std::min(K, R);
    if (mmax <= 8) {
        const size_t lds = 768 + (size_t)R * K;
        // one thread per group: the per-group work is a chain of dependent LDS lookups, so latency is hidden
        // by having many groups in flight, not by looping
        const uint32_t blocks = (uint32_t)std::max<size_t>(1, std::min<size_t>((G + kBlock - 1) / kBlock,
                                                                                (size_t)std::max(di.cus, 1) * 64));
        const size_t lds4 = 768 + (size_t)R * (((size_t)K + 3) & ~size_t(3));
        if (syn && KFEC_PREP_SYN_T) {
            if (mmax == 1) hipLaunchKernelGGL((decode_prep_perm<1, true>), dim3(blocks), dim3(kBlock), lds4, s, p);
            else if (mmax == 2) hipLaunchKernelGGL((decode_prep_perm<2, true>), dim3(blocks), dim3(kBlock), lds4, s, p);
            else if (mmax == 3) hipLaunchKernelGGL((decode_prep_perm<3, true>), dim3(blocks), dim3(kBlock), lds4, s, p);
            else if (mmax == 4) hipLaunchKernelGGL((decode_prep_perm<4, true>), dim3(blocks), dim3(kBlock), lds4, s, p);
            else hipLaunchKernelGGL((decode_prep_small<8>), dim3(blocks), dim3(kBlock), lds, s, p);
        }
        else if (mmax == 1) hipLaunchKernelGGL((decode_prep_perm<1>), dim3(blocks), dim3(kBlock), lds4, s, p);
        else if (mmax == 2) hipLaunchKernelGGL((decode_prep_perm<2>), dim3(blocks), dim3(kBlock), lds4, s, p);
        else if (mmax == 3) hipLaunchKernelGGL((decode_prep_perm<3>), dim3(blocks), dim3(kBlock), lds4, s, p);
        else if (mmax == 4) hipLaunchKernelGGL((decode_prep_perm<4>), dim3(blocks), dim3(kBlock), lds4, s, p);
        else hipLaunchKernelGGL((decode_prep_small<8>), dim3(blocks), dim3(kBlock), lds, s, p);
    } else {
        constexpr int kTeam = KFEC_PREP_WAVE ? 64 : kPrepThreads;
        const void *fn = reinterpret_cast<const void *>(&decode_prep_lagrange<kTeam>);
        int occ = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, fn, kPrepThreads, 0) != hipSuccess || occ <= 0) occ = 1;
        const size_t teams = kPrepThreads / kTeam;
        const uint32_t blocks =
            (uint32_t)std::max<size_t>(1, std::min<size_t>((G + teams - 1) / teams, (size_t)std::max(di.cus, 1) * occ));
        hipLaunchKernelGGL((decode_prep_lagrange<kTeam>), dim3(blocks), dim3(kPrepThreads), 0, s, p);
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
    int vec = pick_vec_mac(pitch, B, {d_data, d_parity, d_out});
    if (G <= kLatencyGroups && vec >= 4) vec = kLatencyVec;
    const int vb = vec >= 4 ? vec : 4;
    const size_t cols = (B + vb - 1) / vb;
    // syndrome form for R <= 8 unless its per-workgroup C tables outgrow LDS (tiny B: hundreds of groups
    // per workgroup)
    const int rt = syn_rt(R);
    const size_t gmax_syn = std::min<size_t>(G, (kMacBlock - 1) / std::max<size_t>(cols, 1) + 2);
    const size_t lds_syn = (KFEC_SYN_WAVE_CT ? (size_t)(kMacBlock / 64) * syn_wave_groups(cols) : gmax_syn) *
                           (size_t)rt * syn_td(rt) * 4;
    // (syndrome form: whole-dword granules, and each workgroup's groups must fit one buffer resource)
    const bool syn = R > 0 && R <= KFEC_SYN_MAX_R && lds_syn <= kSynLdsMax && vec != 1 &&
                     gmax_syn * (size_t)K * pitch < (size_t(1) << 31) && gmax_syn * (size_t)R * pitch < (size_t(1) << 31) &&
                     G * (size_t)R < (size_t(1) << 32);
    // (the mac_kernel decode rebuilds the coefficients of factored records; the prep writes them for K, R > 8)
    const bool factored = !syn && KFEC_DEC_FACTORED && KFEC_DEC_TTAB && std::min(K, R) > 8;
    // hybrid (decode_hybrid_r): the listed syndrome kernel for sparse loss, the coefficient-form MAC (3 waves per
    // SIMD against the RT >= 6 syndrome kernel's 2) for dense loss, chosen on the device by the same rule
    const bool hybrid = syn && decode_hybrid_r(R) && vec == 32 && G > kLatencyGroups && B > 0 &&
                        G * cols <= kMaxItemsPerLaunch && KFEC_DEC_TTAB;
    if (hybrid) {
        // syndrome records and the list first; the coefficient records only when the dense shape will run (the
        // prep exits at once otherwise)
        uint8_t *rec_syn = rec + decode_hybrid_syn_offset(G, K, R);
        if (launch_decode_prep(di, d_enc, K, N, G, d_present, d_out_idx, d_status, rec_syn, s, true, false)) return -3;
        uint32_t *count = reinterpret_cast<uint32_t *>(rec + decode_list_offset(G, K, R));
        uint32_t *chunk_cnt = count + 64;
        uint32_t *list = chunk_cnt + decode_list_chunks(G);
        const size_t cols_pad = (cols + 63) / 64 * 64;
        const uint32_t nch = (uint32_t)((G + kActChunk - 1) / kActChunk);
        hipLaunchKernelGGL(active_count_kernel, dim3(nch), dim3(kBlock), 0, s, (uint64_t)G, (uint32_t)R, d_out_idx, chunk_cnt);
        hipLaunchKernelGGL(active_scan_kernel, dim3(1), dim3(kBlock), 0, s, nch, chunk_cnt, count);
        hipLaunchKernelGGL(active_scatter_kernel, dim3(nch), dim3(kBlock), 0, s, (uint64_t)G, (uint32_t)R, d_out_idx,
                           (const uint32_t *)chunk_cnt, list);
        if (hipGetLastError() != hipSuccess) return -3;
        if (launch_decode_prep(di, d_enc, K, N, G, d_present, d_out_idx, d_status, d_workspace, s, false, false, count,
                               (uint32_t)cols, (uint32_t)cols_pad))
            return -3;
        SynArgs sa{};
        sa.data = static_cast<const uint8_t *>(d_data);
        sa.parity = static_cast<const uint8_t *>(d_parity);
        sa.out = static_cast<uint8_t *>(d_out);
        sa.rec = rec_syn;
        sa.etab = reinterpret_cast<const uint32_t *>(d_enc + enc_tab_offset(K, N));
        sa.list = list;
        sa.list_count = count;
        sa.etab_rows = (uint32_t)enc_tab_rows(R);
        sa.pitch = pitch;
        sa.total = (uint32_t)(G * cols);
        sa.cols = (uint32_t)cols;
        sa.cols_pad = (uint32_t)cols_pad;
        sa.G = (uint32_t)G;
        sa.K = K; sa.R = R; sa.B = (uint32_t)B;
        sa.rec_stride = (uint32_t)syn_record_stride(K, R);
        sa.no_dense = 1;
        if (dispatch_syn(vec, rt, sa, lds_syn, di.cus, s)) return -3;
        const uint32_t gmax = (uint32_t)std::min<size_t>(G, (kMacBlock - 1) / cols + 2);
        MacArgs a{};
        a.data = static_cast<const uint8_t *>(d_data);
        a.parity = static_cast<const uint8_t *>(d_parity);
        a.out = static_cast<uint8_t *>(d_out);
        a.enc = d_enc;
        a.rec = rec;
        a.pitch = pitch;
        a.total = (uint32_t)(G * cols);
        a.cols = (uint32_t)cols;
        a.G = (uint32_t)G;
        a.K = K; a.R = R; a.B = (uint32_t)B;
        a.rec_stride = (uint32_t)rs;
        a.factored = 0;
        a.JC = (uint32_t)std::max<size_t>(1, std::min<size_t>(K, kDecLdsBudget / (kDecEntry * gmax)));
        a.gmax = gmax;
        a.tiles = 1;
        a.list_count = count;
        a.cols_pad = (uint32_t)cols_pad;
        return dispatch_mac<true>(vec, (KFEC_DEC_MT_MID && R >= 5 && R < 8) || (KFEC_DEC_MT_SMALL && R == 4) ? R : 8, a, s);
    }
    if (launch_decode_prep(di, d_enc, K, N, G, d_present, d_out_idx, d_status, d_workspace, s, syn, factored)) return -3;
    if (R == 0 || B == 0) return 0;
    if (syn) {
        const size_t rs_syn = syn_record_stride(K, R);  // (the prep wrote syndrome records)
        uint32_t *count = reinterpret_cast<uint32_t *>(rec + decode_list_offset(G, K, R));
        uint32_t *chunk_cnt = count + 64;
        uint32_t *list = chunk_cnt + decode_list_chunks(G);
        const size_t cols_pad = (cols + 63) / 64 * 64;
        const size_t lds = lds_syn;
        return for_group_ranges(G, cols, 1, [&](size_t g0, size_t gn) {
            // the ordered list of this launch's groups with data to recover, and its length, on the device
            // (not for the latency shape's few groups: there the dense kernel alone runs, two launches fewer
            // per decode call plus the listed kernel's)
            const bool small = gn <= kLatencyGroups;
            const uint32_t nch = (uint32_t)((gn + kActChunk - 1) / kActChunk);
            const uint8_t *oi = d_out_idx + g0 * R;
            if (!small) {
                hipLaunchKernelGGL(active_count_kernel, dim3(nch), dim3(kBlock), 0, s, (uint64_t)gn, (uint32_t)R, oi, chunk_cnt);
                hipLaunchKernelGGL(active_scan_kernel, dim3(1), dim3(kBlock), 0, s, nch, chunk_cnt, count);
                hipLaunchKernelGGL(active_scatter_kernel, dim3(nch), dim3(kBlock), 0, s, (uint64_t)gn, (uint32_t)R, oi,
                                   (const uint32_t *)chunk_cnt, list);
                if (hipGetLastError() != hipSuccess) return -3;
            }
            SynArgs a{};
            a.data = static_cast<const uint8_t *>(d_data) + g0 * K * pitch;
            a.parity = static_cast<const uint8_t *>(d_parity) + g0 * R * pitch;
            a.out = static_cast<uint8_t *>(d_out) + g0 * R * pitch;
            a.rec = rec + g0 * rs_syn;
            a.etab = reinterpret_cast<const uint32_t *>(d_enc + enc_tab_offset(K, N));
            a.list = list;
            a.list_count = small ? nullptr : count;  // nullptr: dense only (syn_kernel runs, no listed launch)
            a.etab_rows = (uint32_t)enc_tab_rows(R);
            a.pitch = pitch;
            a.total = (uint32_t)(gn * cols);
            a.cols = (uint32_t)cols;
            a.cols_pad = (uint32_t)cols_pad;
            a.G = (uint32_t)gn;
            a.K = K; a.R = R; a.B = (uint32_t)B;
            a.rec_stride = (uint32_t)rs_syn;
            return dispatch_syn(vec, rt, a, lds, di.cus, s);
        });
    }
#if KFEC_SYN_MAX_R > 0
    // coefficient form: R > 8 (or tiny shards), 8-row tiles; KFEC_DEC_MT4_WIDE: 4-row tiles where they compute fewer
    // rows (the factored records' scalar loads need row0 % 4 == 0)
    const int mt = (KFEC_DEC_MT4_WIDE && KFEC_DEC_MT_SMALL && vec == 32 && (R + 3) / 4 * 4 < (R + 7) / 8 * 8) ? 4 : 8;
#else
    const int mt = pick_mt(R);  // A/B build: coefficient form for every R
#endif
    const int tiles = (R + mt - 1) / mt;
    const size_t ent = entry_bytes(mt);
    return for_group_ranges(G, cols, tiles, [&](size_t g0, size_t gn) {
        const uint32_t gmax = (uint32_t)std::min<size_t>(gn, (kMacBlock - 1) / cols + 2);
        const uint32_t JC = dec_ttab(mt) ? (uint32_t)std::max<size_t>(1, std::min<size_t>(K, kDecLdsBudget / (kDecEntry * gmax)))
                                          : (uint32_t)std::max<size_t>(1, std::min<size_t>(K, kLdsBudget / (ent * gmax)));
        MacArgs a{};
        a.data = static_cast<const uint8_t *>(d_data) + g0 * K * pitch;
        a.parity = static_cast<const uint8_t *>(d_parity) + g0 * R * pitch;
        a.out = static_cast<uint8_t *>(d_out) + g0 * R * pitch;
        a.enc = d_enc;
        a.rec = rec + g0 * rs;
        a.pitch = pitch;
        a.total = (uint32_t)(gn * cols);
        a.cols = (uint32_t)cols;
        a.G = (uint32_t)gn;
        a.K = K; a.R = R; a.B = (uint32_t)B;
        a.rec_stride = (uint32_t)(factored ? fac_record_stride(K, R) : rs);
        a.factored = factored ? 1u : 0u;
        a.JC = JC;
        a.gmax = gmax;
        a.tiles = (uint32_t)tiles;
        return dispatch_mac<true>(vec, mt, a, s);
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
    if (random_count == 2) {  // i.i.d. loss with probability count_max / 1e6 per shard (orc_erasure_mask_iid)
        uint64_t m[4] = {0, 0, 0, 0};
        for (uint32_t s = 0; s < N; ++s)
            if (splitmix64(seed ^ 0xC2B2AE3D27D4EB4Full ^ (gg * 0x100u + s)) % 1000000u >= count_max)
                m[s >> 6] |= 1ull << (s & 63);
#pragma unroll
        for (int q = 0; q < 4; ++q) present[g * 4 + q] = m[q];
        return;
    }
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
                       (uint32_t)N, (uint64_t)g0, (uint64_t)G, (uint32_t)pool,
                       (uint32_t)(random_count == 1 ? std::max<size_t>(count_max, 1) : count_max),
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
