// grf_gram.hip -- K = Phi Phi^T on gfx950.
//
// Replaces `Phi @ Phi.T`:
//   efficient_graph_gp_sparse/graph_kernels_sparse/fast_grf_kernel_general.py:55 (scipy SpGEMM)
//   efficient_graph_gp/graph_kernels/fast_grf_kernel_general.py:39 (dense BLAS)
//
// Sparse path (Gustavson, output-stationary in LDS): one workgroup owns the
// tile K[row, c0 : c0 + 4W] as a float32 accumulator in LDS; wave v owns the
// columns [c0 + vW, c0 + (v+1)W) (one band of the banded transpose).  For every
// nonzero Phi[row, k] the wave streams bucket (band, k) -- the entries Phi[j, k]
// with j in its band -- and adds Phi[row,k]*Phi[j,k] into acc[j] with LDS
// float atomics.  Waves never share an accumulator word, so the order of the
// adds into every K entry is fixed (k order of the row): K is bit-reproducible.
// Each wave flattens the buckets of 64 nonzeros into one lane-dense stream
// (4 iterations in flight per lane), so short buckets do not idle lanes.  The finished tile is
// written once, coalesced, with non-temporal stores (K is write-once; keep L2
// for the transpose).  Bound: HBM write of K (4 N^2 bytes).
//
// Dense path: LDS-tiled fp32 MFMA (v_mfma_f32_32x32x2f32, exact f32 FMA chain),
// 128x128 tile per 256-thread workgroup, 2x2 waves of 64x64.
#include "grf_block.h"

namespace grf {

constexpr int kGramThreads = 256;
typedef float f32x4 __attribute__((ext_vector_type(4)));
constexpr int kGramUnroll = 4;

__global__ __launch_bounds__(kGramThreads, 2) void gram_sparse_kernel(
    int64_t n_total, int64_t row_begin, int64_t nb, int64_t ww, const int64_t *__restrict__ ptr,
    const int32_t *__restrict__ idx, const float *__restrict__ val, const int64_t *__restrict__ t_ptr,
    const int32_t *__restrict__ t_row, const float *__restrict__ t_val, float *__restrict__ K, int64_t ldk) {
    // tile = (row, band of 4 sub-bands of ww columns); wave v owns sub-band 4*band + v,
    // so no two waves ever add to the same accumulator word: the summation order of
    // every K entry is fixed (row order of k), independent of scheduling.
    extern __shared__ __attribute__((aligned(16))) float acc[];
    const int64_t tw = 4 * ww;
    int32_t *tab_incl = reinterpret_cast<int32_t *>(acc + tw);         // [4][66]
    int64_t *tab_t0 = reinterpret_cast<int64_t *>(tab_incl + 4 * 66);  // [4][64]
    float *tab_a = reinterpret_cast<float *>(tab_t0 + 4 * 64);         // [4][64]

    const int64_t tile = blockIdx.x;
    const int64_t band = tile % nb, r = tile / nb, row = row_begin + r;
    const int64_t w0 = band * tw;
    const int64_t wlen = (n_total - w0) < tw ? (n_total - w0) : tw;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;

    float4 *acc4 = reinterpret_cast<float4 *>(acc);
    for (int64_t i = tid; i < (wlen + 3) / 4; i += kGramThreads) acc4[i] = make_float4(0.f, 0.f, 0.f, 0.f);
    __syncthreads();

    const int64_t sub = 4 * band + wave;         // this wave's sub-band
    const int64_t j0 = sub * ww;                 // its first column
    if (j0 < n_total) {
        int32_t *incl_w = tab_incl + wave * 66;
        int64_t *t0_w = tab_t0 + wave * 64;
        float *a_w = tab_a + wave * 64;
        const int64_t e0 = ptr[row], e1 = ptr[row + 1];
        const int64_t boff = sub * n_total;
        float *accw = acc - w0;                  // absolute column index -> LDS word
        for (int64_t g0 = e0; g0 < e1; g0 += 64) {
            const int64_t e = g0 + lane;
            int32_t cnt = 0;
            int64_t t0 = 0;
            float a = 0.f;
            if (e < e1) {
                const int32_t k = idx[e];
                a = val[e];
                t0 = t_ptr[boff + k];
                cnt = (int32_t)(t_ptr[boff + k + 1] - t0);
            }
            const int32_t incl = wave_inclusive_scan<int32_t>(cnt);
            const int32_t total = __shfl(incl, 63, 64);
            incl_w[lane] = incl;
            t0_w[lane] = t0 - (incl - cnt);  // pos = t0' + q for q inside this bucket
            a_w[lane] = a;
            if (lane == 0) incl_w[64] = 0x7fffffff;
            __builtin_amdgcn_wave_barrier();
            int cur = 0;
            for (int32_t q0 = 0; q0 < total; q0 += 64 * kGramUnroll) {
                int32_t j[kGramUnroll];
                float v[kGramUnroll], sc[kGramUnroll];
#pragma unroll
                for (int u = 0; u < kGramUnroll; ++u) {
                    const int32_t q = q0 + u * 64 + lane;
                    j[u] = -1;
                    if (q < total) {
                        while (incl_w[cur] <= q) ++cur;
                        const int64_t pos = t0_w[cur] + q;
                        j[u] = t_row[pos];
                        v[u] = t_val[pos];
                        sc[u] = a_w[cur];
                    }
                }
#pragma unroll
                for (int u = 0; u < kGramUnroll; ++u)
                    if (j[u] >= 0)
                        __hip_atomic_fetch_add(&accw[j[u]], sc[u] * v[u], __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_WORKGROUP);
            }
            __builtin_amdgcn_wave_barrier();
        }
    }
    __syncthreads();

    float *krow = K + r * ldk + w0;
    if ((ldk & 3) == 0 && (w0 & 3) == 0) {
        const int64_t n4 = wlen / 4;
        f32x4 *k4 = reinterpret_cast<f32x4 *>(krow);
        const f32x4 *a4 = reinterpret_cast<const f32x4 *>(acc);
        for (int64_t i = tid; i < n4; i += kGramThreads) __builtin_nontemporal_store(a4[i], &k4[i]);
        for (int64_t i = n4 * 4 + tid; i < wlen; i += kGramThreads) __builtin_nontemporal_store(acc[i], &krow[i]);
    } else {
        for (int64_t i = tid; i < wlen; i += kGramThreads) krow[i] = acc[i];
    }
}

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
                        const float *val, int64_t band_width, const int64_t *t_ptr, const int32_t *t_row,
                        const float *t_val, float *K, int64_t ldk, grf_stream_t stream) {
    GRF_REQUIRE(n_total >= 0 && 0 <= row_begin && row_begin <= row_end && row_end <= n_total && ptr && t_ptr && K,
                GRF_EINVAL, "grf_gram_sparse: bad arguments");
    GRF_REQUIRE(ldk >= n_total, GRF_EINVAL, "grf_gram_sparse: ldk < n");
    GRF_REQUIRE(band_width >= 16 && band_width % 16 == 0 && band_width <= 8192, GRF_EUNSUPPORTED,
                "grf_gram_sparse: band_width must be a multiple of 16 in [16, 8192]");
    const int64_t rows = row_end - row_begin;
    if (rows == 0 || n_total == 0) return GRF_OK;
    const int64_t nb = cdiv<int64_t>(n_total, 4 * band_width);  // a tile spans 4 transpose bands
    const int64_t tiles = rows * nb;
    GRF_REQUIRE(tiles < (1ll << 31), GRF_EUNSUPPORTED, "grf_gram_sparse: too many tiles; split the row range");
    const size_t lds = (size_t)band_width * 16 + 4 * 66 * 4 + 4 * 64 * 8 + 4 * 64 * 4;
    gram_sparse_kernel<<<(unsigned)tiles, kGramThreads, lds, S(stream)>>>(n_total, row_begin, nb, band_width, ptr, idx,
                                                                         val, t_ptr, t_row, t_val, K, ldk);
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
