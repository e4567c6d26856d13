// grf_dense_steps.hip -- the GPflow surface's per-call algebra on a dense (N, N, L) step tensor.
//
// Replaces, for GraphGeneralFastGRFKernel / GraphDiffusionFastGRFKernel:
//   Phi = tf.linalg.matmul(feature_matrices_tf, modulator[:, None])[:, :, 0]
//       efficient_graph_gp/gpflow_kernels/general_kernel_fast_grf.py:76, diffusion_kernel_fast_grf.py:58
// and the modulator gradient TensorFlow's autodiff takes through K = Phi Phi^T (:77 / :60):
//   dL/df_l = sum_ij G_ij dK_ij/df_l = <F_l, (G + G^T) Phi>       (F_l = F[:, :, l])
//
// dense_steps_phi_kernel: one thread per (i, j), Phi[i, j] = sum_l F[i, j, l] f_l in fp64 (l ascending), written
//   as fp64 (the backward's operand) and as the zero-padded fp32 image the MFMA Gram (grf_gram_dense) reads.
//   HBM-bound: N^2 L 8 B read, N^2 12 B written.
// dense_steps_grad_kernel: H = (G + G^T) Phi on v_mfma_f64_16x16x4_f64 (64 x 64 tile per 4-wave workgroup,
//   16-deep k-tiles through LDS, S = G + G^T formed while staging), with the reduction fused into the
//   epilogue: each workgroup's partial sum_{(i,j) in tile} F[i, j, l] H[i, j] per l, so H never reaches
//   HBM; dense_steps_grad_reduce_kernel sums the partials in workgroup order (deterministic).
//   2 N^3 fp64 flops on the matrix cores + one read of F.
#include "grf_block.h"

namespace grf {

__global__ __launch_bounds__(256) void dense_steps_phi_kernel(int64_t n, int32_t L, const double *__restrict__ F,
                                                              const double *__restrict__ f, double *__restrict__ phi64,
                                                              float *__restrict__ phi32, int64_t lda32) {
    const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int64_t i = t / lda32, j = t - i * lda32;
    if (i >= n) return;
    if (j >= n) {  // the fp32 image's zero padding (the Gram's k range is padded to lda32)
        phi32[t] = 0.f;
        return;
    }
    const double *src = F + (i * n + j) * (int64_t)L;
    double acc = 0.0;
    for (int l = 0; l < L; ++l) acc = acc + src[l] * f[l];  // (-ffp-contract=off: one rounding each)
    if (phi64) phi64[i * n + j] = acc;
    phi32[t] = (float)acc;
}

typedef double f64x4 __attribute__((ext_vector_type(4)));

constexpr int kGT = 64;         // output tile (rows and columns)
constexpr int kGK = 16;         // k-tile depth
constexpr int kGPitch = 64 + 16; // LDS row pitch (doubles): k-rows k and k + 1 fall on disjoint bank halves

// H[i0 : i0 + 64, j0 : j0 + 64] = sum_k S[i, k] Phi[k, j], S = G + G^T; then partial[blk][l] =
// sum over the tile of F[i, j, l] H[i, j].  Waves 2 x 2, each 32 x 32 = 2 x 2 MFMA blocks of 16 x 16.
__global__ __launch_bounds__(256) void dense_steps_grad_kernel(int64_t n, int32_t L, const double *__restrict__ F,
                                                               const double *__restrict__ phi,
                                                               const double *__restrict__ G, int64_t ldg,
                                                               double *__restrict__ partial) {
    __shared__ __attribute__((aligned(16))) double As[kGK][kGPitch];  // As[k][i] = S[i0 + i, k0 + k]
    __shared__ __attribute__((aligned(16))) double Bs[kGK][kGPitch];  // Bs[k][j] = Phi[k0 + k, j0 + j]
    __shared__ double red[4][8];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave >> 1, wn = wave & 1;
    const int64_t nt = cdiv<int64_t>(n, kGT);
    const int64_t bi = blockIdx.x / nt, bj = blockIdx.x - bi * nt;
    const int64_t i0 = bi * kGT, j0 = bj * kGT;
    f64x4 acc[2][2];
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b) acc[a][b] = f64x4{0.0, 0.0, 0.0, 0.0};
    for (int64_t k0 = 0; k0 < n; k0 += kGK) {
        // stage: 64 x 16 of S (G[i, k] + G[k, i]) and 16 x 64 of Phi, 4 elements per thread each
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int e = tid + 256 * q;
            // S: element (i = e / 16, k = e % 16) -> G[i0 + i, k0 + k]; (k = e / 64, i = e % 64) -> G[k0 + k, i0 + i]
            const int si = e >> 4, sk = e & 15;
            const int64_t gi = i0 + si, gk = k0 + sk;
            const double g1 = (gi < n && gk < n) ? G[gi * ldg + gk] : 0.0;
            As[sk][si] = g1;
        }
        __syncthreads();
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int e = tid + 256 * q;
            const int tk = e >> 6, ti = e & 63;
            const int64_t gi = i0 + ti, gk = k0 + tk;
            const double g2 = (gi < n && gk < n) ? G[gk * ldg + gi] : 0.0;
            As[tk][ti] += g2;
            const int64_t gj = j0 + ti;
            Bs[tk][ti] = (gk < n && gj < n) ? phi[gk * n + gj] : 0.0;
        }
        __syncthreads();
#pragma unroll
        for (int ks = 0; ks < kGK; ks += 4) {
            const int kk = ks + (lane >> 4);
            double a[2], b[2];
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                a[u] = As[kk][wm * 32 + u * 16 + (lane & 15)];
                b[u] = Bs[kk][wn * 32 + u * 16 + (lane & 15)];
            }
#pragma unroll
            for (int u = 0; u < 2; ++u)
#pragma unroll
                for (int v = 0; v < 2; ++v) acc[u][v] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[u], b[v], acc[u][v], 0, 0, 0);
        }
        __syncthreads();
    }
    // epilogue: C/D map of v_mfma_f64_16x16x4_f64 -- col = lane & 15, row = (lane >> 4) + 4 r.  The
    // steps l are taken 8 at a time, so an entry's F[i, j, l0 : l0 + 8] (one 64-byte run) is read once.
    for (int l0 = 0; l0 < L; l0 += 8) {
        double p[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) p[q] = 0.0;
#pragma unroll
        for (int u = 0; u < 2; ++u)
#pragma unroll
            for (int v = 0; v < 2; ++v)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int64_t i = i0 + wm * 32 + u * 16 + (lane >> 4) + 4 * r;
                    const int64_t j = j0 + wn * 32 + v * 16 + (lane & 15);
                    if (i < n && j < n) {
                        const double *src = F + (i * n + j) * (int64_t)L + l0;
                        const double h = acc[u][v][r];
#pragma unroll
                        for (int q = 0; q < 8; ++q)
                            if (l0 + q < L) p[q] += src[q] * h;
                    }
                }
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            const double s = wave_sum<double>(p[q]);
            if (lane == 0) red[wave][q] = s;
        }
        __syncthreads();
        if (tid < 8 && l0 + tid < L)  // the four waves in fixed order
            partial[(int64_t)blockIdx.x * L + l0 + tid] = ((red[0][tid] + red[1][tid]) + red[2][tid]) + red[3][tid];
        __syncthreads();
    }
}

// grad[l] = sum over the workgroups' partials in workgroup order (one wave per l)
__global__ __launch_bounds__(64) void dense_steps_grad_reduce_kernel(int64_t n_blk, int32_t L,
                                                                     const double *__restrict__ partial,
                                                                     double *__restrict__ grad) {
    const int l = blockIdx.x, lane = threadIdx.x;
    double s = 0.0;
    for (int64_t b = lane; b < n_blk; b += 64) s += partial[b * L + l];
    s = wave_sum<double>(s);
    if (lane == 0) grad[l] = s;
}

}  // namespace grf

using namespace grf;

extern "C" {
#pragma GCC visibility push(default)

int32_t grf_dense_steps_phi(int64_t n, int32_t L, const double *F, const double *f, double *phi64, float *phi32,
                            int64_t lda32, grf_stream_t stream) {
    GRF_REQUIRE(n >= 0 && L >= 1 && lda32 >= n && (n == 0 || (F && f && phi32)), GRF_EINVAL,
                "grf_dense_steps_phi: bad arguments");
    if (n == 0) return GRF_OK;
    const int64_t work = n * lda32;
    GRF_REQUIRE_GRID(cdiv<int64_t>(work, 256), 256, "dense_steps_phi_kernel");
    dense_steps_phi_kernel<<<(unsigned)cdiv<int64_t>(work, 256), 256, 0, S(stream)>>>(n, L, F, f, phi64, phi32,
                                                                                      lda32);
    GRF_CHECK_LAUNCH("dense_steps_phi_kernel");
    return GRF_OK;
}

size_t grf_dense_steps_grad_workspace_bytes(int64_t n, int32_t L) {
    const int64_t nt = cdiv<int64_t>(n > 0 ? n : 1, (int64_t)kGT);
    return (size_t)(nt * nt) * (size_t)(L > 0 ? L : 1) * sizeof(double);
}

int32_t grf_dense_steps_grad(int64_t n, int32_t L, const double *F, const double *phi64, const double *G, int64_t ldg,
                             double *grad, void *workspace, size_t workspace_bytes, grf_stream_t stream) {
    GRF_REQUIRE(n >= 0 && L >= 1 && ldg >= n && grad && (n == 0 || (F && phi64 && G && workspace)), GRF_EINVAL,
                "grf_dense_steps_grad: bad arguments");
    hipStream_t st = S(stream);
    if (n == 0) {
        GRF_CHECK_HIP(hipMemsetAsync(grad, 0, (size_t)L * sizeof(double), st));
        return GRF_OK;
    }
    GRF_REQUIRE(workspace_bytes >= grf_dense_steps_grad_workspace_bytes(n, L), GRF_EINVAL,
                "grf_dense_steps_grad: workspace needs %zu bytes", grf_dense_steps_grad_workspace_bytes(n, L));
    const int64_t nt = cdiv<int64_t>(n, (int64_t)kGT), nblk = nt * nt;
    GRF_REQUIRE_GRID(nblk, 256, "dense_steps_grad_kernel");
    dense_steps_grad_kernel<<<(unsigned)nblk, 256, 0, st>>>(n, L, F, phi64, G, ldg, (double *)workspace);
    GRF_CHECK_LAUNCH("dense_steps_grad_kernel");
    dense_steps_grad_reduce_kernel<<<(unsigned)L, 64, 0, st>>>(nblk, L, (const double *)workspace, grad);
    GRF_CHECK_LAUNCH("dense_steps_grad_reduce_kernel");
    return GRF_OK;
}

}  // extern "C"
