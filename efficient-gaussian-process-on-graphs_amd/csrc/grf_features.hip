// grf_features.hip -- the GPyTorch surface's feature algebra on device-resident step matrices.
//
// Replaces, for efficient_graph_gp_sparse/gptorch_kernels_sparse/sparse_grf_kernel.py:24-61 and
// sparse_diffusion_kernel.py:74-96:
//   phi = sum(mod_vec * mat for mod_vec, mat in zip(modulator_vector, step_matrices))   (:54-60)
//   phi[x1_idx], phi[x2_idx]                                                              (:33-41)
//   (phi_x1 * phi_x2).sum(dim=-1)                                                         (:43-45)
// and the pieces of the modulator gradient dK/df_l = M_l[x1] Phi[x2]^T + Phi[x1] M_l[x2]^T that
// the autograd Function (grf_amd/features.py) contracts with the upstream gradient.
// K[x1, x2] = Phi[x1] Phi[x2]^T itself runs on the sparse Gram kernels (grf_gram.hip).
//
// Step matrices arrive in the layout the preprocessor hands to the kernels (one CSR per step,
// int64 row pointers, sorted int32 columns, float32 values: the reference's torch CSR values).
#include "grf_common.h"

namespace grf {

constexpr int kMaxSteps = 64;

struct StepPtrs {  // L <= 64 step matrices (device pointers), passed by value
    const int64_t *ptr[kMaxSteps];
    const int32_t *idx[kMaxSteps];
    const float *val[kMaxSteps];
};

// One wave per row: L-way merge of the row's sorted step rows (lane l follows step l).
// Phi[row, k] = sum over the steps l holding k, in step order, of f_l * M_l[row, k] (fp64,
// 0.0 + first term, then left to right: scipy's `Phi += f_l * M_l`); exact zeros dropped.
// kFill = false: count the row's entries into cnt[row]; true: write them at out_ptr[row].
template <bool kFill>
__global__ __launch_bounds__(256) void phi_steps_csr_kernel(int64_t n_rows, int32_t Lf, StepPtrs sp,
                                                            const double *__restrict__ f, int32_t *__restrict__ cnt,
                                                            const int64_t *__restrict__ out_ptr,
                                                            int32_t *__restrict__ out_idx,
                                                            double *__restrict__ out_val,
                                                            float *__restrict__ out_val32) {
    const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= n_rows) return;
    const int lane = threadIdx.x & 63;
    int64_t pos = 0, end = 0;
    double fl = 0.0;
    const int32_t *ix = nullptr;
    const float *vx = nullptr;
    if (lane < Lf) {
        pos = sp.ptr[lane][row];
        end = sp.ptr[lane][row + 1];
        ix = sp.idx[lane];
        vx = sp.val[lane];
        fl = f[lane];
    }
    int32_t head = pos < end ? ix[pos] : INT32_MAX;
    int64_t out = kFill ? out_ptr[row] : 0;
    for (;;) {
        int32_t mn = head;
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) mn = min(mn, __shfl_xor(mn, off, 64));
        if (mn == INT32_MAX) break;
        const bool match = head == mn;
        const double t = match ? fl * (double)vx[pos] : 0.0;
        uint64_t mask = __ballot(match);
        double acc = 0.0;
        bool first = true;
        while (mask) {
            const int b = __ffsll((long long)mask) - 1;
            mask &= mask - 1;
            const double tb = __shfl(t, b, 64);
            acc = first ? 0.0 + tb : acc + tb;
            first = false;
        }
        if (acc != 0.0) {
            if (kFill && lane == 0) {
                out_idx[out] = mn;
                if (out_val) out_val[out] = acc;
                if (out_val32) out_val32[out] = (float)acc;
            }
            ++out;
        }
        if (match) {
            ++pos;
            head = pos < end ? ix[pos] : INT32_MAX;
        }
    }
    if (!kFill && lane == 0) cnt[row] = (int32_t)out;
}

__global__ __launch_bounds__(256) void csr_row_lengths_kernel(int64_t n_sel, const int64_t *__restrict__ ptr,
                                                              const int32_t *__restrict__ row_map,
                                                              int32_t *__restrict__ len) {
    const int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (r >= n_sel) return;
    const int64_t row = row_map ? row_map[r] : r;
    len[r] = (int32_t)(ptr[row + 1] - ptr[row]);
}

// one wave per selected row: a contiguous copy of the row's entries
__global__ __launch_bounds__(256) void csr_gather_rows_kernel(int64_t n_sel, const int64_t *__restrict__ ptr,
                                                              const int32_t *__restrict__ idx,
                                                              const float *__restrict__ val,
                                                              const int32_t *__restrict__ row_map,
                                                              const int64_t *__restrict__ out_ptr,
                                                              int32_t *__restrict__ out_idx,
                                                              float *__restrict__ out_val) {
    const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (r >= n_sel) return;
    const int lane = threadIdx.x & 63;
    const int64_t row = row_map[r];
    const int64_t e0 = ptr[row], e1 = ptr[row + 1], o = out_ptr[r];
    for (int64_t e = e0 + lane; e < e1; e += 64) {
        out_idx[o + (e - e0)] = idx[e];
        out_val[o + (e - e0)] = val[e];
    }
}

// first position in [lo, hi) of sorted idx[] holding a value >= key
__device__ inline int64_t lower_bound_i32(const int32_t *__restrict__ idx, int64_t lo, int64_t hi, int32_t key) {
    while (lo < hi) {
        const int64_t mid = lo + ((hi - lo) >> 1);
        if (idx[mid] < key) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

// out[r] = A[rows_a[r], :] . B[rows_b[r], :] for sorted CSR rows: one wave per r, each lane takes
// entries of row A and binary-searches row B; the 64 lane sums are added by a fixed xor tree
// (deterministic).  fp64 accumulation of the exact products of the fp32 values.
__global__ __launch_bounds__(256) void csr_rowdot_kernel(int64_t n_pairs, const int64_t *__restrict__ a_ptr,
                                                         const int32_t *__restrict__ a_idx,
                                                         const float *__restrict__ a_val,
                                                         const int32_t *__restrict__ rows_a,
                                                         const int64_t *__restrict__ b_ptr,
                                                         const int32_t *__restrict__ b_idx,
                                                         const float *__restrict__ b_val,
                                                         const int32_t *__restrict__ rows_b, double *__restrict__ out) {
    const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (r >= n_pairs) return;
    const int lane = threadIdx.x & 63;
    const int64_t ra = rows_a ? rows_a[r] : r, rb = rows_b ? rows_b[r] : r;
    const int64_t a0 = a_ptr[ra], a1 = a_ptr[ra + 1], b0 = b_ptr[rb], b1 = b_ptr[rb + 1];
    double acc = 0.0;
    for (int64_t e = a0 + lane; e < a1; e += 64) {
        const int32_t k = a_idx[e];
        const int64_t p = lower_bound_i32(b_idx, b0, b1, k);
        if (p < b1 && b_idx[p] == k) acc += (double)a_val[e] * (double)b_val[p];
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off, 64);
    if (lane == 0) out[r] = acc;
}

// out[r] = sum over the entries e of row row_map[r]: val[e] * Z[idx[e] * ldz + r]
// (the contraction of one step matrix's rows with the columns of Z = Phi[x2]^T G^T); one wave
// per r, xor-tree lane sum (deterministic).
__global__ __launch_bounds__(256) void csr_rows_dot_cols_kernel(int64_t n_sel, const int64_t *__restrict__ ptr,
                                                                const int32_t *__restrict__ idx,
                                                                const float *__restrict__ val,
                                                                const int32_t *__restrict__ row_map,
                                                                const float *__restrict__ Z, int64_t ldz,
                                                                double *__restrict__ out) {
    const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (r >= n_sel) return;
    const int lane = threadIdx.x & 63;
    const int64_t row = row_map ? row_map[r] : r;
    const int64_t e0 = ptr[row], e1 = ptr[row + 1];
    double acc = 0.0;
    for (int64_t e = e0 + lane; e < e1; e += 64) acc += (double)val[e] * (double)Z[(int64_t)idx[e] * ldz + r];
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off, 64);
    if (lane == 0) out[r] = acc;
}

// K (dense fp32 on the device) -> the scipy CSR the reference's sparse entry point returns
// (graph_kernels_sparse/fast_grf_kernel_general.py:55: `Phi @ Phi.T` is a scipy CSR: float64 values,
// sorted columns, exact zeros absent).  One wave per row, 64 columns per step: the nonzero lanes'
// positions from a ballot (mbcnt prefix), kFill = false counts the row's entries, true writes them
// (int32 column, the fp32 value widened) at out_ptr[row].
template <bool kFill>
__global__ __launch_bounds__(256) void dense_to_csr_kernel(int64_t n_rows, int64_t n_cols,
                                                           const float *__restrict__ K, int64_t ldk,
                                                           int32_t *__restrict__ cnt,
                                                           const int64_t *__restrict__ out_ptr,
                                                           int32_t *__restrict__ out_idx,
                                                           double *__restrict__ out_val) {
    const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= n_rows) return;
    const int lane = threadIdx.x & 63;
    const float *krow = K + row * ldk;
    int64_t o = kFill ? out_ptr[row] : 0;
    for (int64_t c0 = 0; c0 < n_cols; c0 += 64) {
        const int64_t c = c0 + lane;
        const float v = c < n_cols ? krow[c] : 0.f;
        const bool nz = v != 0.f;  // (-0.0 counts as zero, like scipy's dense -> CSR)
        const unsigned long long m = __ballot(nz);
        if (kFill && nz) {
            const int64_t at = o + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0));
            out_idx[at] = (int32_t)c;
            out_val[at] = (double)v;
        }
        o += __popcll(m);
    }
    if (!kFill && lane == 0) cnt[row] = (int32_t)o;
}

}  // namespace grf

using namespace grf;

namespace {
int32_t phi_steps_check(int64_t n_rows, int32_t L, const int64_t *const *step_ptr,
                               const int32_t *const *step_idx, const float *const *step_val, const double *f,
                               int32_t n_f) {
    GRF_REQUIRE(n_rows >= 0 && L >= 1 && step_ptr && step_idx && step_val, GRF_EINVAL,
                "grf_phi_steps_csr: bad arguments");
    GRF_REQUIRE(L <= kMaxSteps, GRF_EUNSUPPORTED, "grf_phi_steps_csr: more than %d step matrices", kMaxSteps);
    GRF_REQUIRE(n_f >= 0 && (n_f == 0 || f), GRF_EINVAL, "grf_phi_steps_csr: bad modulator");
    for (int l = 0; l < L; ++l)
        GRF_REQUIRE(step_ptr[l], GRF_EINVAL, "grf_phi_steps_csr: step %d has no row pointers", l);
    return GRF_OK;
}

StepPtrs pack_steps(int32_t Lf, const int64_t *const *step_ptr, const int32_t *const *step_idx,
                           const float *const *step_val) {
    StepPtrs sp{};
    for (int l = 0; l < Lf; ++l) {
        sp.ptr[l] = step_ptr[l];
        sp.idx[l] = step_idx[l];
        sp.val[l] = step_val[l];
    }
    return sp;
}
}  // namespace

extern "C" {
#pragma GCC visibility push(default)

int32_t grf_phi_steps_csr_count(int64_t n_rows, int32_t L, const int64_t *const *step_ptr,
                                const int32_t *const *step_idx, const float *const *step_val, const double *f,
                                int32_t n_f, int32_t *phi_cnt, grf_stream_t stream) {
    int32_t rc = phi_steps_check(n_rows, L, step_ptr, step_idx, step_val, f, n_f);
    if (rc != GRF_OK) return rc;
    GRF_REQUIRE(phi_cnt || n_rows == 0, GRF_EINVAL, "grf_phi_steps_csr_count: phi_cnt is NULL");
    if (n_rows == 0) return GRF_OK;
    const int32_t Lf = n_f < L ? n_f : L;
    GRF_REQUIRE_GRID(cdiv<int64_t>(n_rows, 4), 256, "phi_steps_csr_kernel");
    phi_steps_csr_kernel<false><<<(unsigned)cdiv<int64_t>(n_rows, 4), 256, 0, S(stream)>>>(
        n_rows, Lf, pack_steps(Lf, step_ptr, step_idx, step_val), f, phi_cnt, nullptr, nullptr, nullptr, nullptr);
    GRF_CHECK_LAUNCH("phi_steps_csr_kernel");
    return GRF_OK;
}

int32_t grf_phi_steps_csr_fill(int64_t n_rows, int32_t L, const int64_t *const *step_ptr,
                               const int32_t *const *step_idx, const float *const *step_val, const double *f,
                               int32_t n_f, const int64_t *phi_ptr, int32_t *phi_idx, double *phi_val,
                               float *phi_val32, grf_stream_t stream) {
    int32_t rc = phi_steps_check(n_rows, L, step_ptr, step_idx, step_val, f, n_f);
    if (rc != GRF_OK) return rc;
    GRF_REQUIRE(n_rows == 0 || (phi_ptr && phi_idx && (phi_val || phi_val32)), GRF_EINVAL,
                "grf_phi_steps_csr_fill: bad outputs");
    if (n_rows == 0) return GRF_OK;
    const int32_t Lf = n_f < L ? n_f : L;
    GRF_REQUIRE_GRID(cdiv<int64_t>(n_rows, 4), 256, "phi_steps_csr_kernel");
    phi_steps_csr_kernel<true><<<(unsigned)cdiv<int64_t>(n_rows, 4), 256, 0, S(stream)>>>(
        n_rows, Lf, pack_steps(Lf, step_ptr, step_idx, step_val), f, nullptr, phi_ptr, phi_idx, phi_val, phi_val32);
    GRF_CHECK_LAUNCH("phi_steps_csr_kernel");
    return GRF_OK;
}

int32_t grf_csr_row_lengths(int64_t n_sel, const int64_t *ptr, const int32_t *row_map, int32_t *len,
                            grf_stream_t stream) {
    GRF_REQUIRE(n_sel >= 0 && ptr && (len || n_sel == 0), GRF_EINVAL, "grf_csr_row_lengths: bad arguments");
    if (n_sel == 0) return GRF_OK;
    csr_row_lengths_kernel<<<(unsigned)cdiv<int64_t>(n_sel, 256), 256, 0, S(stream)>>>(n_sel, ptr, row_map, len);
    GRF_CHECK_LAUNCH("csr_row_lengths_kernel");
    return GRF_OK;
}

int32_t grf_csr_gather_rows(int64_t n_sel, const int64_t *ptr, const int32_t *idx, const float *val,
                            const int32_t *row_map, const int64_t *out_ptr, int32_t *out_idx, float *out_val,
                            grf_stream_t stream) {
    GRF_REQUIRE(n_sel >= 0 && ptr && row_map && out_ptr, GRF_EINVAL, "grf_csr_gather_rows: bad arguments");
    if (n_sel == 0) return GRF_OK;
    GRF_REQUIRE_GRID(cdiv<int64_t>(n_sel, 4), 256, "csr_gather_rows_kernel");
    csr_gather_rows_kernel<<<(unsigned)cdiv<int64_t>(n_sel, 4), 256, 0, S(stream)>>>(n_sel, ptr, idx, val, row_map,
                                                                                    out_ptr, out_idx, out_val);
    GRF_CHECK_LAUNCH("csr_gather_rows_kernel");
    return GRF_OK;
}

int32_t grf_csr_rowdot(int64_t n_pairs, const int64_t *a_ptr, const int32_t *a_idx, const float *a_val,
                       const int32_t *rows_a, const int64_t *b_ptr, const int32_t *b_idx, const float *b_val,
                       const int32_t *rows_b, double *out, grf_stream_t stream) {
    GRF_REQUIRE(n_pairs >= 0 && a_ptr && b_ptr && (out || n_pairs == 0), GRF_EINVAL, "grf_csr_rowdot: bad arguments");
    if (n_pairs == 0) return GRF_OK;
    GRF_REQUIRE_GRID(cdiv<int64_t>(n_pairs, 4), 256, "csr_rowdot_kernel");
    csr_rowdot_kernel<<<(unsigned)cdiv<int64_t>(n_pairs, 4), 256, 0, S(stream)>>>(
        n_pairs, a_ptr, a_idx, a_val, rows_a, b_ptr, b_idx, b_val, rows_b, out);
    GRF_CHECK_LAUNCH("csr_rowdot_kernel");
    return GRF_OK;
}

int32_t grf_csr_rows_dot_cols(int64_t n_sel, const int64_t *ptr, const int32_t *idx, const float *val,
                              const int32_t *row_map, const float *Z, int64_t ldz, double *out, grf_stream_t stream) {
    GRF_REQUIRE(n_sel >= 0 && ptr && (n_sel == 0 || (Z && out)) && ldz >= n_sel, GRF_EINVAL,
                "grf_csr_rows_dot_cols: bad arguments");
    if (n_sel == 0) return GRF_OK;
    GRF_REQUIRE_GRID(cdiv<int64_t>(n_sel, 4), 256, "csr_rows_dot_cols_kernel");
    csr_rows_dot_cols_kernel<<<(unsigned)cdiv<int64_t>(n_sel, 4), 256, 0, S(stream)>>>(n_sel, ptr, idx, val, row_map,
                                                                                      Z, ldz, out);
    GRF_CHECK_LAUNCH("csr_rows_dot_cols_kernel");
    return GRF_OK;
}

int32_t grf_dense_to_csr_count(int64_t n_rows, int64_t n_cols, const float *K, int64_t ldk, int32_t *cnt,
                               grf_stream_t stream) {
    GRF_REQUIRE(n_rows >= 0 && n_cols >= 0 && n_cols < ((int64_t)1 << 31) && ldk >= n_cols &&
                    (n_rows == 0 || (K && cnt)),
                GRF_EINVAL, "grf_dense_to_csr_count: bad arguments");
    if (n_rows == 0) return GRF_OK;
    GRF_REQUIRE_GRID(cdiv<int64_t>(n_rows, 4), 256, "dense_to_csr_kernel");
    dense_to_csr_kernel<false><<<(unsigned)cdiv<int64_t>(n_rows, 4), 256, 0, S(stream)>>>(n_rows, n_cols, K, ldk, cnt,
                                                                                        nullptr, nullptr, nullptr);
    GRF_CHECK_LAUNCH("dense_to_csr_kernel");
    return GRF_OK;
}

int32_t grf_dense_to_csr_fill(int64_t n_rows, int64_t n_cols, const float *K, int64_t ldk, const int64_t *out_ptr,
                              int32_t *out_idx, double *out_val, grf_stream_t stream) {
    GRF_REQUIRE(n_rows >= 0 && n_cols >= 0 && n_cols < ((int64_t)1 << 31) && ldk >= n_cols &&
                    (n_rows == 0 || (K && out_ptr && out_idx && out_val)),
                GRF_EINVAL, "grf_dense_to_csr_fill: bad arguments");
    if (n_rows == 0) return GRF_OK;
    GRF_REQUIRE_GRID(cdiv<int64_t>(n_rows, 4), 256, "dense_to_csr_kernel");
    dense_to_csr_kernel<true><<<(unsigned)cdiv<int64_t>(n_rows, 4), 256, 0, S(stream)>>>(
        n_rows, n_cols, K, ldk, nullptr, out_ptr, out_idx, out_val);
    GRF_CHECK_LAUNCH("dense_to_csr_kernel");
    return GRF_OK;
}

#pragma GCC visibility pop
}  // extern "C"
