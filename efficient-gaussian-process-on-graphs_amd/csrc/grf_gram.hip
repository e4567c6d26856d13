// grf_gram.hip -- K = Phi Phi^T on gfx950.
//
// Replaces `Phi @ Phi.T`:
//   efficient_graph_gp_sparse/graph_kernels_sparse/fast_grf_kernel_general.py:55 (scipy SpGEMM)
//   efficient_graph_gp/graph_kernels/fast_grf_kernel_general.py:39 (dense BLAS)
//
// Sparse path (Gustavson, output-stationary in LDS): one workgroup owns the
// tile K[row, j0 : j0 + W] (W = one band of the banded transpose, 8192 columns =
// 64 KB of int64 accumulator, 2 workgroups per CU).  For every nonzero
// Phi[row, k] it streams bucket (band, k) -- the entries Phi[j, k] with j in the
// band, stored as (uint16 j - j0, float32 value) -- and adds the exact product
// Phi[row,k]*Phi[j,k] in int64 fixed point with ds_add_u64.  Measured on gfx950
// (tools/lds_bench.hip): ds_add_f32 serialises per lane (~170 cycles per wave
// instruction per CU) while ds_add_u64 takes ~12, so fixed point is both ~14x
// cheaper and exactly order-independent (bit-reproducible K).  The finished tile is
// written once, coalesced, with non-temporal stores (K is write-once; keep L2
// for the transpose).  Bound: HBM write of K (4 N^2 bytes).
//
// Dense path: LDS-tiled fp32 MFMA (v_mfma_f32_32x32x2f32, exact f32 FMA chain),
// 128x128 tile per 256-thread workgroup, 2x2 waves of 64x64.
#include "grf_block.h"

namespace grf {

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kGramThreads = 256;  // 4 waves share one tile
constexpr int kChunk = 1024;       // stream positions covered by one marker chunk
constexpr int kGramUnroll = 4;     // windows of 64 tuples in flight per wave

// inclusive max-scan over the 64 lanes with DPP (VALU only, no LDS traffic)
__device__ inline int wave_incl_max(int v) {
    v = max(v, __builtin_amdgcn_update_dpp(-1, v, 0x111, 0xf, 0xf, false));  // row_shr:1
    v = max(v, __builtin_amdgcn_update_dpp(-1, v, 0x112, 0xf, 0xf, false));  // row_shr:2
    v = max(v, __builtin_amdgcn_update_dpp(-1, v, 0x114, 0xf, 0xf, false));  // row_shr:4
    v = max(v, __builtin_amdgcn_update_dpp(-1, v, 0x118, 0xf, 0xf, false));  // row_shr:8
    v = max(v, __builtin_amdgcn_update_dpp(-1, v, 0x142, 0xa, 0xf, false));  // row_bcast:15
    v = max(v, __builtin_amdgcn_update_dpp(-1, v, 0x143, 0xc, 0xf, false));  // row_bcast:31
    return v;
}

// |x| < 2^51 -> round-to-nearest int64 with one f64 add and one integer subtract
__device__ inline long long fx_round(double x) {
    const double magic = 6755399441055744.0;  // 1.5 * 2^52
    return (long long)(__double_as_longlong(x + magic) - __double_as_longlong(magic));
}

// One workgroup = one tile K[row, j0 : j0 + W] (W = a band of the banded
// transpose).  Accumulation is exact int64 fixed point with a per-row power-of-two
// scale S = 2^(50 - ceil(log2(sum_k |Phi[row,k]| * max|Phi|))), so every partial sum
// stays below 2^51: the result is the exactly rounded fixed-point sum, independent of
// the order of the adds (ds_add_u64) and therefore of scheduling, GPU count, row split.
// The 4 waves pull batches of 64 nonzeros of the row from an LDS counter; each batch's
// buckets are flattened into one lane-dense stream whose bucket index per position is
// recovered from bucket-start markers (one u8 LDS read) and a DPP max-scan.
// Grid is band-major so the Phi^T slice in use stays resident in the Infinity Cache.
__global__ __launch_bounds__(kGramThreads, 2) void gram_sparse_kernel(
    int64_t n_total, int64_t row_begin, int64_t n_rows, int64_t W, const int64_t *__restrict__ ptr,
    const int32_t *__restrict__ idx, const float *__restrict__ val, const int64_t *__restrict__ t_ptr,
    const uint16_t *__restrict__ t_col, const float *__restrict__ t_val, const float *__restrict__ maxabs,
    float *__restrict__ K, int64_t ldk) {
    extern __shared__ __attribute__((aligned(16))) unsigned long long acc[];  // [W]
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    unsigned char *mark_all = reinterpret_cast<unsigned char *>(acc + W);       // [4][kChunk]
    int64_t *tb_all = reinterpret_cast<int64_t *>(mark_all + 4 * kChunk);       // [4][64]
    double *as_all = reinterpret_cast<double *>(tb_all + 4 * 64);              // [4][64]
    double *red = as_all + 4 * 64;                                             // [8]
    int *next_batch = reinterpret_cast<int *>(red + 8);                        // [1]
    unsigned char *mark = mark_all + wave * kChunk;
    int64_t *tbase = tb_all + wave * 64;
    double *ascale = as_all + wave * 64;

    const int64_t bid = blockIdx.x;
    const int64_t band = bid / n_rows, r = bid - band * n_rows, row = row_begin + r;
    const int64_t j0 = band * W;
    const int64_t wlen = (n_total - j0) < W ? (n_total - j0) : W;
    const int64_t e0 = ptr[row], e1 = ptr[row + 1];

    // zero the accumulator, sum |Phi[row, :]| for the scale
    typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));
    u64x2 *acc2 = reinterpret_cast<u64x2 *>(acc);
    const u64x2 z2 = {0ull, 0ull};
    for (int64_t i = tid; i < (wlen + 1) / 2; i += kGramThreads) acc2[i] = z2;
    // scale: every term |Phi[row,k] Phi[j,k]| S < 2^51 (exact magic-number rounding) and
    // the sum of all |terms| S < 2^62 (no int64 overflow)
    double sa = 0.0;
    float ma = 0.f;
    for (int64_t e = e0 + tid; e < e1; e += kGramThreads) {
        const float a = fabsf(val[e]);
        sa += (double)a;
        ma = fmaxf(ma, a);
    }
    sa = wave_sum<double>(sa);
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) ma = fmaxf(ma, __shfl_xor(ma, off, 64));
    if (lane == 0) { red[wave] = sa; red[4 + wave] = (double)ma; }
    if (tid == 0) *next_batch = 0;
    __syncthreads();
    const double mx = (double)maxabs[0];
    const double B = (red[0] + red[1] + red[2] + red[3]) * mx;
    const double T = fmax(fmax(red[4], red[5]), fmax(red[6], red[7])) * mx;
    const int eB = B > 0.0 ? ilogb(B) + 1 : 0;  // B < 2^eB
    const int eT = T > 0.0 ? ilogb(T) + 1 : 0;  // every term < 2^eT
    const int sh = min(51 - eT, 62 - eB);
    const double S = ldexp(1.0, sh), inv_S = ldexp(1.0, -sh);

    const int64_t boff = band * n_total;
    for (;;) {
        int bi = 0;
        if (lane == 0) bi = atomicAdd(next_batch, 1);
        bi = __builtin_amdgcn_readfirstlane(bi);
        const int64_t g0 = e0 + (int64_t)bi * 64;
        if (g0 >= e1) break;
        const int64_t e = g0 + lane;
        int32_t cnt = 0;
        int64_t t0 = 0;
        double as = 0.0;
        if (e < e1) {
            const int32_t k = idx[e];
            as = (double)val[e] * S;
            t0 = t_ptr[boff + k];
            cnt = (int32_t)(t_ptr[boff + k + 1] - t0);
        }
        const int32_t incl = wave_inclusive_scan<int32_t>(cnt);
        const int32_t excl = incl - cnt;
        const int32_t total = __shfl(incl, 63, 64);
        tbase[lane] = t0 - excl;
        ascale[lane] = as;
        int carry = -1;
        for (int32_t c0 = 0; c0 < total; c0 += kChunk) {
            reinterpret_cast<uint4 *>(mark)[lane] = make_uint4(~0u, ~0u, ~0u, ~0u);  // 64 x 16 B = kChunk
            if (cnt > 0 && excl >= c0 && excl < c0 + kChunk) mark[excl - c0] = (unsigned char)lane;
            __builtin_amdgcn_wave_barrier();
            const int32_t cend = (total - c0) < kChunk ? total : c0 + kChunk;
            for (int32_t w0 = c0; w0 < cend; w0 += 64 * kGramUnroll) {
                int bk[kGramUnroll];
#pragma unroll
                for (int u = 0; u < kGramUnroll; ++u) {
                    const int32_t p = w0 + u * 64 + lane;
                    int m = p < cend ? (int)mark[p - c0] : 255;
                    m = m == 255 ? -1 : m;
                    if (lane == 0) m = max(m, carry);
                    m = wave_incl_max(m);
                    carry = __builtin_amdgcn_readlane(m, 63);
                    bk[u] = m;
                }
                int64_t pos[kGramUnroll];
                double sc[kGramUnroll];
#pragma unroll
                for (int u = 0; u < kGramUnroll; ++u) {
                    const int32_t p = w0 + u * 64 + lane;
                    const bool ok = p < cend;
                    const int b = bk[u] < 0 ? 0 : bk[u];
                    pos[u] = ok ? tbase[b] + p : 0;  // tuple 0 always exists when total > 0
                    sc[u] = ok ? ascale[b] : 0.0;
                }
                uint32_t jj[kGramUnroll];
                float v[kGramUnroll];
#pragma unroll
                for (int u = 0; u < kGramUnroll; ++u) jj[u] = t_col[pos[u]];
#pragma unroll
                for (int u = 0; u < kGramUnroll; ++u) v[u] = t_val[pos[u]];
#pragma unroll
                for (int u = 0; u < kGramUnroll; ++u) {
                    const long long q = fx_round(sc[u] * (double)v[u]);  // exact product, one rounding
                    __hip_atomic_fetch_add(&acc[jj[u]], (unsigned long long)q, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_WORKGROUP);
                }
            }
            __builtin_amdgcn_wave_barrier();
        }
    }
    __syncthreads();

    float *krow = K + r * ldk + j0;
    if ((ldk & 3) == 0 && (j0 & 3) == 0) {
        const int64_t n4 = wlen / 4;
        f32x4 *k4 = reinterpret_cast<f32x4 *>(krow);
        for (int64_t i = tid; i < n4; i += kGramThreads) {
            const u64x2 a = acc2[2 * i], b = acc2[2 * i + 1];
            f32x4 o;
            o[0] = (float)((double)(long long)a[0] * inv_S);
            o[1] = (float)((double)(long long)a[1] * inv_S);
            o[2] = (float)((double)(long long)b[0] * inv_S);
            o[3] = (float)((double)(long long)b[1] * inv_S);
            __builtin_nontemporal_store(o, &k4[i]);
        }
        for (int64_t i = n4 * 4 + tid; i < wlen; i += kGramThreads)
            krow[i] = (float)((double)(long long)acc[i] * inv_S);
    } else {
        for (int64_t i = tid; i < wlen; i += kGramThreads) krow[i] = (float)((double)(long long)acc[i] * inv_S);
    }
}

__global__ void absmax_reset_kernel(float *m) { *m = 0.f; }

// ------------------------------------------------------------------ dense MFMA
constexpr int kBM = 128, kBK = 16, kPad = 4;
typedef float f32x16 __attribute__((ext_vector_type(16)));

__global__ __launch_bounds__(256) void gram_dense_kernel(int64_t n, int64_t k_dim, const float *__restrict__ A,
                                                         int64_t lda, float *__restrict__ K, int64_t ldk) {
    __shared__ __attribute__((aligned(16))) float As[kBK][kBM + kPad];
    __shared__ __attribute__((aligned(16))) float Bs[kBK][kBM + kPad];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave >> 1, wn = wave & 1;
    const int64_t m0 = (int64_t)blockIdx.y * kBM, n0 = (int64_t)blockIdx.x * kBM;
    f32x16 c[2][2];
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b)
#pragma unroll
            for (int q = 0; q < 16; ++q) c[a][b][q] = 0.f;

    for (int64_t k0 = 0; k0 < k_dim; k0 += kBK) {
        // stage: 128 rows x 16 k of A (M tile) and of A (N tile), transposed to [k][row]
#pragma unroll
        for (int it = 0; it < 2; ++it) {
            const int idx = tid + it * 256;        // 0..511 float4 slots
            const int row = idx >> 2, kq = (idx & 3) * 4;
            float4 va = make_float4(0.f, 0.f, 0.f, 0.f), vb = va;
            if (m0 + row < n) va = *reinterpret_cast<const float4 *>(A + (m0 + row) * lda + k0 + kq);
            if (n0 + row < n) vb = *reinterpret_cast<const float4 *>(A + (n0 + row) * lda + k0 + kq);
            As[kq + 0][row] = va.x; As[kq + 1][row] = va.y; As[kq + 2][row] = va.z; As[kq + 3][row] = va.w;
            Bs[kq + 0][row] = vb.x; Bs[kq + 1][row] = vb.y; Bs[kq + 2][row] = vb.z; Bs[kq + 3][row] = vb.w;
        }
        __syncthreads();
#pragma unroll
        for (int kk = 0; kk < kBK; kk += 2) {
            const int kr = kk + (lane >> 5), rc = lane & 31;
            float a0 = As[kr][wm * 64 + rc], a1 = As[kr][wm * 64 + 32 + rc];
            float b0 = Bs[kr][wn * 64 + rc], b1 = Bs[kr][wn * 64 + 32 + rc];
            c[0][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b0, c[0][0], 0, 0, 0);
            c[0][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b1, c[0][1], 0, 0, 0);
            c[1][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b0, c[1][0], 0, 0, 0);
            c[1][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b1, c[1][1], 0, 0, 0);
        }
        __syncthreads();
    }
    // C/D map (32x32): col = lane & 31, row = (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5)
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b)
#pragma unroll
            for (int q = 0; q < 16; ++q) {
                const int64_t row = m0 + wm * 64 + a * 32 + (q & 3) + 8 * (q >> 2) + 4 * (lane >> 5);
                const int64_t col = n0 + wn * 64 + b * 32 + (lane & 31);
                if (row < n && col < n) K[row * ldk + col] = c[a][b][q];
            }
}

__global__ __launch_bounds__(256) void densify_kernel(int64_t n_rows, const int64_t *__restrict__ ptr,
                                                      const int32_t *__restrict__ idx, const float *__restrict__ val,
                                                      float *__restrict__ out, int64_t lda) {
    const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= n_rows) return;
    const int lane = threadIdx.x & 63;
    for (int64_t e = ptr[row] + lane; e < ptr[row + 1]; e += 64) out[row * lda + idx[e]] = val[e];
}

}  // namespace grf

using namespace grf;

extern "C" {
#pragma GCC visibility push(default)

int32_t grf_gram_sparse(int64_t n_total, int64_t row_begin, int64_t row_end, const int64_t *ptr, const int32_t *idx,
                        const float *val, int64_t band_width, const int64_t *t_ptr, const uint16_t *t_col,
                        const float *t_val, const float *t_maxabs, float *K, int64_t ldk, grf_stream_t stream) {
    GRF_REQUIRE(n_total >= 0 && 0 <= row_begin && row_begin <= row_end && row_end <= n_total && ptr && t_ptr && K &&
                    t_maxabs,
                GRF_EINVAL, "grf_gram_sparse: bad arguments");
    GRF_REQUIRE(ldk >= n_total, GRF_EINVAL, "grf_gram_sparse: ldk < n");
    GRF_REQUIRE(band_width >= 64 && band_width % 64 == 0 && band_width <= 8192, GRF_EUNSUPPORTED,
                "grf_gram_sparse: band_width must be a multiple of 64 in [64, 8192]");
    const int64_t rows = row_end - row_begin;
    if (rows == 0 || n_total == 0) return GRF_OK;
    const int64_t nb = cdiv<int64_t>(n_total, band_width);
    const int64_t tiles = rows * nb;
    GRF_REQUIRE(tiles < (1ll << 31), GRF_EUNSUPPORTED, "grf_gram_sparse: too many tiles; split the row range");
    const size_t lds = (size_t)band_width * 8 + 4 * kChunk + 4 * 64 * 8 + 4 * 64 * 8 + 8 * 8 + 16;
    gram_sparse_kernel<<<(unsigned)tiles, kGramThreads, lds, S(stream)>>>(
        n_total, row_begin, rows, band_width, ptr, idx, val, t_ptr, t_col, t_val, t_maxabs, K, ldk);
    GRF_CHECK_LAUNCH("gram_sparse_kernel");
    return GRF_OK;
}

int32_t grf_gram_dense(int64_t n, int64_t k_dim, const float *A, int64_t lda, float *K, int64_t ldk,
                       grf_stream_t stream) {
    GRF_REQUIRE(n >= 0 && k_dim >= 0 && A && K && ldk >= n && lda >= k_dim, GRF_EINVAL,
                "grf_gram_dense: bad arguments");
    GRF_REQUIRE(lda % 16 == 0 && ((uintptr_t)A & 15) == 0, GRF_EINVAL,
                "grf_gram_dense: lda must be a multiple of 16 and A 16-byte aligned");
    if (n == 0) return GRF_OK;
    const int64_t kpad = cdiv<int64_t>(k_dim, kBK) * kBK;
    GRF_REQUIRE(kpad <= lda, GRF_EINVAL, "grf_gram_dense: lda must cover k_dim rounded up to 16");
    const int64_t tiles = cdiv<int64_t>(n, kBM);
    dim3 grid((unsigned)tiles, (unsigned)tiles);
    gram_dense_kernel<<<grid, 256, 0, S(stream)>>>(n, kpad, A, lda, K, ldk);
    GRF_CHECK_LAUNCH("gram_dense_kernel");
    return GRF_OK;
}

int32_t grf_densify(int64_t n_rows, const int64_t *ptr, const int32_t *idx, const float *val, float *out,
                    int64_t lda, grf_stream_t stream) {
    GRF_REQUIRE(n_rows >= 0 && ptr && out && lda >= 0, GRF_EINVAL, "grf_densify: bad arguments");
    if (n_rows == 0) return GRF_OK;
    GRF_CHECK_HIP(hipMemsetAsync(out, 0, (size_t)n_rows * (size_t)lda * sizeof(float), S(stream)));
    densify_kernel<<<(unsigned)cdiv<int64_t>(n_rows, 4), 256, 0, S(stream)>>>(n_rows, ptr, idx, val, out, lda);
    GRF_CHECK_LAUNCH("densify_kernel");
    return GRF_OK;
}

}  // extern "C"
