// grf_sparse.hip -- device scans, padded-row compaction and the banded
// transpose of Phi that feeds the Gram kernel.
//
// Replaces the host-side CSR assembly of the reference
// (sparse_sampler.py:117-130 np.fromiter + csr_matrix, and scipy's internal
// csc->csr conversion of Phi.T inside `Phi @ Phi.T`,
// graph_kernels_sparse/fast_grf_kernel_general.py:55).
#include "grf_block.h"

namespace grf {

constexpr int kScanThreads = 256;
constexpr int kScanItems = 16;
constexpr int64_t kScanTile = (int64_t)kScanThreads * kScanItems;

template <typename TIn>
__global__ __launch_bounds__(kScanThreads) void scan_reduce_kernel(int64_t n, const TIn *in, int64_t *part) {
    __shared__ int64_t scratch[kScanThreads / 64 + 1];
    const int64_t base = (int64_t)blockIdx.x * kScanTile + (int64_t)threadIdx.x * kScanItems;
    int64_t s = 0;
#pragma unroll
    for (int k = 0; k < kScanItems; ++k)
        if (base + k < n) s += (int64_t)in[base + k];
    int64_t tot;
    block_exclusive_scan<int64_t>(s, scratch, &tot);
    if (threadIdx.x == 0) part[blockIdx.x] = tot;
}

// out[i] = offset[blockIdx] + exclusive prefix; out[n] = total (written by the last tile)
template <typename TIn>
__global__ __launch_bounds__(kScanThreads) void scan_apply_kernel(int64_t n, const TIn *in, const int64_t *offset,
                                                                  int64_t *out) {
    __shared__ int64_t scratch[kScanThreads / 64 + 1];
    const int64_t base = (int64_t)blockIdx.x * kScanTile + (int64_t)threadIdx.x * kScanItems;
    int64_t v[kScanItems];
    int64_t s = 0;
#pragma unroll
    for (int k = 0; k < kScanItems; ++k) {
        v[k] = base + k < n ? (int64_t)in[base + k] : 0;
        s += v[k];
    }
    int64_t tot;
    int64_t run = block_exclusive_scan<int64_t>(s, scratch, &tot) + (offset ? offset[blockIdx.x] : 0);
#pragma unroll
    for (int k = 0; k < kScanItems; ++k) {
        if (base + k < n) out[base + k] = run;
        run += v[k];
    }
    if (blockIdx.x == gridDim.x - 1 && threadIdx.x == blockDim.x - 1) out[n] = run;
}

static size_t scan_ws_elems(int64_t n) {
    int64_t nb = cdiv<int64_t>(n, kScanTile);
    if (nb <= 1) return 0;
    return (size_t)(nb + nb + 1) + scan_ws_elems(nb);
}

template <typename TIn>
static int32_t scan_exclusive(int64_t n, const TIn *in, int64_t *out, int64_t *ws, hipStream_t st) {
    int64_t nb = cdiv<int64_t>(n, kScanTile);
    if (n == 0) {
        GRF_CHECK_HIP(hipMemsetAsync(out, 0, sizeof(int64_t), st));
        return GRF_OK;
    }
    if (nb == 1) {
        scan_apply_kernel<TIn><<<1, kScanThreads, 0, st>>>(n, in, nullptr, out);
        GRF_CHECK_LAUNCH("scan_apply_kernel");
        return GRF_OK;
    }
    int64_t *part = ws, *part_ex = ws + nb, *rest = ws + nb + nb + 1;
    scan_reduce_kernel<TIn><<<(unsigned)nb, kScanThreads, 0, st>>>(n, in, part);
    GRF_CHECK_LAUNCH("scan_reduce_kernel");
    int32_t rc = scan_exclusive<int64_t>(nb, part, part_ex, rest, st);
    if (rc != GRF_OK) return rc;
    scan_apply_kernel<TIn><<<(unsigned)nb, kScanThreads, 0, st>>>(n, in, part_ex, out);
    GRF_CHECK_LAUNCH("scan_apply_kernel");
    return GRF_OK;
}

// exported for the other translation units
int32_t scan_counts_i32(int64_t n, const int32_t *cnt, int64_t *out, void *ws, size_t ws_bytes, hipStream_t st) {
    GRF_REQUIRE(ws_bytes >= scan_ws_elems(n) * sizeof(int64_t), GRF_EINVAL, "scan workspace too small (%zu < %zu)",
                ws_bytes, scan_ws_elems(n) * sizeof(int64_t));
    return scan_exclusive<int32_t>(n, cnt, out, (int64_t *)ws, st);
}
int32_t scan_counts_i64(int64_t n, const int64_t *cnt, int64_t *out, void *ws, size_t ws_bytes, hipStream_t st) {
    GRF_REQUIRE(ws_bytes >= scan_ws_elems(n) * sizeof(int64_t), GRF_EINVAL, "scan workspace too small");
    return scan_exclusive<int64_t>(n, cnt, out, (int64_t *)ws, st);
}
size_t scan_ws_bytes(int64_t n) { return scan_ws_elems(n) * sizeof(int64_t); }

// ----------------------------------------------------------------- compaction
// one wave per padded row
__global__ __launch_bounds__(256) void compact_rows_kernel(int64_t n_rows, int64_t cap, const int32_t *cnt,
                                                           const int64_t *out_ptr, const int32_t *in_idx,
                                                           const double *in_val, const float *in_val32,
                                                           int32_t *out_idx, double *out_val, float *out_val32) {
    const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= n_rows) return;
    const int lane = threadIdx.x & 63;
    const int64_t c = cnt[row], src = row * cap, dst = out_ptr[row];
    for (int64_t e = lane; e < c; e += 64) {
        out_idx[dst + e] = in_idx[src + e];
        if (out_val) out_val[dst + e] = in_val[src + e];
        if (out_val32) out_val32[dst + e] = in_val32[src + e];
    }
}

// ------------------------------------------------------------ banded transpose
__global__ __launch_bounds__(256) void tr_count_kernel(int64_t n_rows, int64_t n_cols, int64_t bw,
                                                       const int64_t *ptr, const int32_t *idx, int32_t *cnt) {
    const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= n_rows) return;
    const int lane = threadIdx.x & 63;
    const int64_t band_off = (row / bw) * n_cols;
    for (int64_t e = ptr[row] + lane; e < ptr[row + 1]; e += 64) atomicAdd(&cnt[band_off + idx[e]], 1);
}

__global__ void tr_pad_counts_kernel(int64_t n, int32_t *cnt) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) cnt[i] += cnt[i] & 1;  // every bucket holds an even number of records
}

__global__ __launch_bounds__(256) void tr_fill_kernel(int64_t n_rows, int64_t n_cols, int64_t bw, const int64_t *ptr,
                                                      const int32_t *idx, const float *val, const int64_t *t_ptr,
                                                      int32_t *cursor, uint2 *t_rec, unsigned int *maxabs_bits) {
    const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= n_rows) return;
    const int lane = threadIdx.x & 63;
    const int64_t band = row / bw, band_off = band * n_cols;
    const uint32_t jr = (uint32_t)(row - band * bw);
    float mx = 0.f;
    for (int64_t e = ptr[row] + lane; e < ptr[row + 1]; e += 64) {
        const int64_t b = band_off + idx[e];
        const int64_t pos = t_ptr[b] + atomicAdd(&cursor[b], 1);
        t_rec[pos] = make_uint2(jr, __float_as_uint(val[e]));
        mx = fmaxf(mx, fabsf(val[e]));
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) mx = fmaxf(mx, __shfl_xor(mx, off, 64));
    // non-negative floats order like their bit patterns
    if (lane == 0 && mx > 0.f) atomicMax(maxabs_bits, __float_as_uint(mx));
}

// odd buckets get a (col 0, +0.0) pad record: adds exactly 0 in the Gram kernel
__global__ void tr_pad_fill_kernel(int64_t n, const int64_t *t_ptr, const int32_t *cursor, uint2 *t_rec) {
    const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (b < n && (cursor[b] & 1)) t_rec[t_ptr[b] + cursor[b]] = make_uint2(0u, 0u);
}

}  // namespace grf

using namespace grf;

extern "C" {
#pragma GCC visibility push(default)

size_t grf_scan_workspace_bytes(int64_t n) { return scan_ws_bytes(n); }

int32_t grf_scan_counts(int64_t n, const int32_t *cnt, int64_t *out_ptr, void *workspace, size_t workspace_bytes,
                        grf_stream_t stream) {
    GRF_REQUIRE(n >= 0 && cnt && out_ptr, GRF_EINVAL, "grf_scan_counts: bad arguments");
    return scan_counts_i32(n, cnt, out_ptr, workspace, workspace_bytes, S(stream));
}

int32_t grf_compact_rows(int64_t n_rows, int64_t cap, const int32_t *cnt, const int64_t *out_ptr,
                         const int32_t *in_idx, const double *in_val, const float *in_val32, int32_t *out_idx,
                         double *out_val, float *out_val32, grf_stream_t stream) {
    GRF_REQUIRE(n_rows >= 0 && cap >= 0 && cnt && out_ptr && in_idx && out_idx, GRF_EINVAL,
                "grf_compact_rows: bad arguments");
    GRF_REQUIRE(!out_val || in_val, GRF_EINVAL, "grf_compact_rows: out_val needs in_val");
    GRF_REQUIRE(!out_val32 || in_val32, GRF_EINVAL, "grf_compact_rows: out_val32 needs in_val32");
    if (n_rows == 0) return GRF_OK;
    compact_rows_kernel<<<(unsigned)cdiv<int64_t>(n_rows, 4), 256, 0, S(stream)>>>(
        n_rows, cap, cnt, out_ptr, in_idx, in_val, in_val32, out_idx, out_val, out_val32);
    GRF_CHECK_LAUNCH("compact_rows_kernel");
    return GRF_OK;
}

size_t grf_transpose_workspace_bytes(int64_t n_buckets) {
    size_t a = ((size_t)n_buckets * sizeof(int32_t) + 255) & ~(size_t)255;
    return a + scan_ws_bytes(n_buckets);
}

int32_t grf_transpose_banded(int64_t n_rows, int64_t n_cols, int64_t band_width, const int64_t *ptr,
                             const int32_t *idx, const float *val, int64_t *t_ptr, uint32_t *t_rec, float *t_maxabs,
                             void *workspace, size_t workspace_bytes, grf_stream_t stream) {
    GRF_REQUIRE(n_rows >= 0 && n_cols > 0 && band_width > 0 && ptr && idx && val && t_ptr && t_rec && t_maxabs,
                GRF_EINVAL, "grf_transpose_banded: bad arguments");
    GRF_REQUIRE(((uintptr_t)t_rec & 15) == 0, GRF_EINVAL, "grf_transpose_banded: t_rec must be 16-byte aligned");
    const int64_t nb = cdiv<int64_t>(n_rows, band_width), nbk = nb * n_cols;
    GRF_REQUIRE(workspace_bytes >= grf_transpose_workspace_bytes(nbk), GRF_EINVAL,
                "grf_transpose_banded: workspace too small (%zu < %zu)", workspace_bytes,
                grf_transpose_workspace_bytes(nbk));
    hipStream_t st = S(stream);
    int32_t *cnt = (int32_t *)workspace;
    size_t a = ((size_t)nbk * sizeof(int32_t) + 255) & ~(size_t)255;
    void *scan_ws = (char *)workspace + a;
    GRF_CHECK_HIP(hipMemsetAsync(cnt, 0, (size_t)nbk * sizeof(int32_t), st));
    GRF_CHECK_HIP(hipMemsetAsync(t_maxabs, 0, sizeof(float), st));
    if (n_rows > 0) {
        tr_count_kernel<<<(unsigned)cdiv<int64_t>(n_rows, 4), 256, 0, st>>>(n_rows, n_cols, band_width, ptr, idx,
                                                                          cnt);
        GRF_CHECK_LAUNCH("tr_count_kernel");
    }
    tr_pad_counts_kernel<<<(unsigned)cdiv<int64_t>(nbk, 256), 256, 0, st>>>(nbk, cnt);
    GRF_CHECK_LAUNCH("tr_pad_counts_kernel");
    int32_t rc = scan_counts_i32(nbk, cnt, t_ptr, scan_ws, workspace_bytes - a, st);
    if (rc != GRF_OK) return rc;
    GRF_CHECK_HIP(hipMemsetAsync(cnt, 0, (size_t)nbk * sizeof(int32_t), st));
    if (n_rows > 0) {
        tr_fill_kernel<<<(unsigned)cdiv<int64_t>(n_rows, 4), 256, 0, st>>>(
            n_rows, n_cols, band_width, ptr, idx, val, t_ptr, cnt, reinterpret_cast<uint2 *>(t_rec),
            reinterpret_cast<unsigned int *>(t_maxabs));
        GRF_CHECK_LAUNCH("tr_fill_kernel");
    }
    tr_pad_fill_kernel<<<(unsigned)cdiv<int64_t>(nbk, 256), 256, 0, st>>>(nbk, t_ptr, cnt,
                                                                          reinterpret_cast<uint2 *>(t_rec));
    GRF_CHECK_LAUNCH("tr_pad_fill_kernel");
    return GRF_OK;
}

}  // extern "C"
