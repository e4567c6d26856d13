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

// Exclusive scans of n values map(in[i]) (int64 sums).  A tile of kScanTile values is loaded
// lane-striped (consecutive lanes, consecutive elements), transposed through LDS to per-thread
// runs of kScanItems for the scan, and handed to the output functor lane-striped again, so both
// global sides are coalesced (a per-lane run layout gives every lane its own 64-byte input and
// 128-byte output run: C5's 123 M-bucket scans ran at ~2 TB/s that way).  One padding slot per
// 16 keeps the per-thread runs on distinct LDS banks.
__device__ __forceinline__ int scan_pad(int i) { return i + (i >> 4); }
constexpr int kScanLds = (int)kScanTile + (int)(kScanTile >> 4);

struct ScanIdentity {
    template <typename T>
    __device__ int64_t operator()(T v) const { return (int64_t)v; }
};
struct ScanStore {  // out[i] = prefix, out[n] = total
    int64_t *out;
    __device__ void operator()(int64_t i, int64_t prefix) const { out[i] = prefix; }
    __device__ void total(int64_t n, int64_t t) const { out[n] = t; }
};

template <typename TIn, typename Map>
__global__ __launch_bounds__(kScanThreads) void scan_reduce_kernel(int64_t n, const TIn *in, Map map, int64_t *part) {
    __shared__ int64_t scratch[kScanThreads / 64 + 1];
    const int64_t blk = (int64_t)blockIdx.x * kScanTile;
    int64_t s = 0;
#pragma unroll
    for (int k = 0; k < kScanItems; ++k) {
        const int64_t g = blk + k * kScanThreads + threadIdx.x;
        if (g < n) s += map(in[g]);  // (an integer sum: any order gives the same total)
    }
    int64_t tot;
    block_exclusive_scan<int64_t>(s, scratch, &tot);
    if (threadIdx.x == 0) part[blockIdx.x] = tot;
}

template <typename TIn, typename Map, typename Out>
__global__ __launch_bounds__(kScanThreads) void scan_apply_kernel(int64_t n, const TIn *in, Map map,
                                                                  const int64_t *offset, Out out) {
    __shared__ int64_t sh[kScanLds];
    __shared__ int64_t scratch[kScanThreads / 64 + 1];
    const int tid = threadIdx.x;
    const int64_t blk = (int64_t)blockIdx.x * kScanTile;
#pragma unroll
    for (int k = 0; k < kScanItems; ++k) {
        const int i = k * kScanThreads + tid;
        sh[scan_pad(i)] = blk + i < n ? map(in[blk + i]) : 0;
    }
    __syncthreads();
    int64_t v[kScanItems];
    int64_t s = 0;
#pragma unroll
    for (int k = 0; k < kScanItems; ++k) {
        v[k] = sh[scan_pad(tid * kScanItems + k)];
        s += v[k];
    }
    int64_t tot;
    int64_t run = block_exclusive_scan<int64_t>(s, scratch, &tot) + (offset ? offset[blockIdx.x] : 0);
#pragma unroll
    for (int k = 0; k < kScanItems; ++k) {
        sh[scan_pad(tid * kScanItems + k)] = run;
        run += v[k];
    }
    if (blockIdx.x == gridDim.x - 1 && tid == kScanThreads - 1) out.total(n, run);
    __syncthreads();
#pragma unroll
    for (int k = 0; k < kScanItems; ++k) {
        const int i = k * kScanThreads + tid;
        if (blk + i < n) out(blk + i, sh[scan_pad(i)]);
    }
}

static size_t scan_ws_elems(int64_t n) {
    int64_t nb = cdiv<int64_t>(n, kScanTile);
    if (nb <= 1) return 0;
    return (size_t)(nb + nb + 1) + scan_ws_elems(nb);
}

template <typename TIn, typename Map, typename Out>
static int32_t scan_exclusive(int64_t n, const TIn *in, Map map, Out out, int64_t *ws, hipStream_t st) {
    const int64_t nb = cdiv<int64_t>(n, kScanTile);
    if (n == 0) {
        scan_apply_kernel<TIn, Map, Out><<<1, kScanThreads, 0, st>>>(0, in, map, nullptr, out);  // (the total, 0)
        GRF_CHECK_LAUNCH("scan_apply_kernel");
        return GRF_OK;
    }
    if (nb == 1) {
        scan_apply_kernel<TIn, Map, Out><<<1, kScanThreads, 0, st>>>(n, in, map, nullptr, out);
        GRF_CHECK_LAUNCH("scan_apply_kernel");
        return GRF_OK;
    }
    int64_t *part = ws, *part_ex = ws + nb, *rest = ws + nb + nb + 1;
    GRF_REQUIRE_GRID(nb, kScanThreads, "scan_reduce_kernel");
    scan_reduce_kernel<TIn, Map><<<(unsigned)nb, kScanThreads, 0, st>>>(n, in, map, part);
    GRF_CHECK_LAUNCH("scan_reduce_kernel");
    int32_t rc = scan_exclusive<int64_t>(nb, part, ScanIdentity{}, ScanStore{part_ex}, rest, st);
    if (rc != GRF_OK) return rc;
    scan_apply_kernel<TIn, Map, Out><<<(unsigned)nb, kScanThreads, 0, st>>>(n, in, map, part_ex, out);
    GRF_CHECK_LAUNCH("scan_apply_kernel");
    return GRF_OK;
}

// exported for the other translation units
int32_t scan_counts_i32(int64_t n, const int32_t *cnt, int64_t *out, void *ws, size_t ws_bytes, hipStream_t st) {
    GRF_REQUIRE(ws_bytes >= scan_ws_elems(n) * sizeof(int64_t), GRF_EINVAL, "scan workspace too small (%zu < %zu)",
                ws_bytes, scan_ws_elems(n) * sizeof(int64_t));
    return scan_exclusive<int32_t>(n, cnt, ScanIdentity{}, ScanStore{out}, (int64_t *)ws, st);
}
int32_t scan_counts_i64(int64_t n, const int64_t *cnt, int64_t *out, void *ws, size_t ws_bytes, hipStream_t st) {
    GRF_REQUIRE(ws_bytes >= scan_ws_elems(n) * sizeof(int64_t), GRF_EINVAL, "scan workspace too small");
    return scan_exclusive<int64_t>(n, cnt, ScanIdentity{}, ScanStore{out}, (int64_t *)ws, st);
}
size_t scan_ws_bytes(int64_t n) { return scan_ws_elems(n) * sizeof(int64_t); }

// ----------------------------------------------------------------- compaction
// Padded rows (row r at r * cap, cnt[r] entries) -> the CSR at out_ptr.  A wave takes kCompactRows
// consecutive rows and issues the loads of all of them, kCompactU entries per lane and row, before
// its stores: one row per wave kept ~2 loads per lane in flight (C5: ~176 entries per row), 3.1 TB/s.
constexpr int kCompactRows = 4, kCompactU = 2;
static_assert(kCompactRows == 4, "wg_max holds one max per 4 rows (grf_phi_row_shifts_stats reads cdiv(n, 4))");

// kStats: also the Gram row-shift statistics of the compact rows (row max / fp64 sum of |value| and
// the max of every kCompactRows rows): the entries of a row are summed in the order
// phi_row_stats_kernel reads them (lane + 64 i, then the wave sum), so grf_phi_row_shifts_stats gives
// grf_phi_row_shifts' bits without another pass over the values
template <bool kStats>
__global__ __launch_bounds__(256) void compact_rows_kernel(int64_t n_rows, int64_t cap, const int32_t *__restrict__ cnt,
                                                           const int64_t *__restrict__ out_ptr,
                                                           const int32_t *__restrict__ in_idx,
                                                           const double *__restrict__ in_val,
                                                           const float *__restrict__ in_val32,
                                                           int32_t *__restrict__ out_idx, double *__restrict__ out_val,
                                                           float *__restrict__ out_val32, float *__restrict__ row_max,
                                                           double *__restrict__ row_sum, float *__restrict__ wg_max) {
    const int lane = threadIdx.x & 63;
    const int64_t gw = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);  // the wave's group of rows
    const int64_t row0 = gw * kCompactRows;
    if (row0 >= n_rows) return;
    int64_t c[kCompactRows], src[kCompactRows], dst[kCompactRows];
    int64_t cmax = 0;
#pragma unroll
    for (int r = 0; r < kCompactRows; ++r) {
        const bool in = row0 + r < n_rows;
        c[r] = in ? cnt[row0 + r] : 0;
        dst[r] = in ? out_ptr[row0 + r] : 0;
        src[r] = (row0 + r) * cap;
        cmax = c[r] > cmax ? c[r] : cmax;
    }
    float mx[kCompactRows];
    double sm[kCompactRows];
#pragma unroll
    for (int r = 0; r < kCompactRows; ++r) {
        mx[r] = 0.f;
        sm[r] = 0.0;
    }
    for (int64_t base = lane; base < cmax; base += 64 * kCompactU) {
        int32_t ix[kCompactRows][kCompactU];
        float v32[kCompactRows][kCompactU];
        double v64[kCompactRows][kCompactU];
#pragma unroll
        for (int r = 0; r < kCompactRows; ++r)
#pragma unroll
            for (int u = 0; u < kCompactU; ++u) {
                const int64_t e = base + 64 * u;
                const bool in = e < c[r];
                ix[r][u] = in ? in_idx[src[r] + e] : 0;
                v32[r][u] = in && out_val32 ? in_val32[src[r] + e] : 0.f;
                v64[r][u] = in && out_val ? in_val[src[r] + e] : 0.0;
            }
#pragma unroll
        for (int r = 0; r < kCompactRows; ++r)
#pragma unroll
            for (int u = 0; u < kCompactU; ++u) {
                const int64_t e = base + 64 * u;
                if (e >= c[r]) continue;
                out_idx[dst[r] + e] = ix[r][u];
                if (out_val) out_val[dst[r] + e] = v64[r][u];
                if (out_val32) out_val32[dst[r] + e] = v32[r][u];
                if (kStats) {
                    const float a = fabsf(v32[r][u]);
                    mx[r] = fmaxf(mx[r], a);
                    sm[r] += (double)a;
                }
            }
    }
    if (!kStats) return;
    float gmx = 0.f;
#pragma unroll
    for (int r = 0; r < kCompactRows; ++r) {
        float m = mx[r];
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) m = fmaxf(m, __shfl_xor(m, off, 64));
        const double s = wave_sum<double>(sm[r]);
        if (lane == 0 && row0 + r < n_rows) {
            row_max[row0 + r] = m;
            row_sum[row0 + r] = s;
        }
        gmx = fmaxf(gmx, m);
    }
    if (lane == 0) wg_max[gw] = gmx;
}

// ------------------------------------------------------------ banded transpose
// Bucket b = band * n_cols + k holds the entries Phi[j, k], j in the band, as PAIRS of
// records packed in 12 bytes: {u16 8 (j0 - band start), u16 8 (j1 - band start), f32 v0, f32 v1}
// (the row is stored as the byte offset of its int64 counter in the Gram tile).
// Record unit u (bytes): GRF_REC_LINE (128) starts every bucket on a 128-byte line (the Gram
// kernel reads a bucket as one short segment; aligned, a segment of <= 10 pairs is one line
// instead of two) -- for the dense-bucket regime (C4: ~9 pairs per bucket); GRF_REC_PACKED (12)
// packs the buckets pair after pair -- for sparse buckets (C5: ~0.7 pairs per bucket, where a
// line per bucket is ~15x the records' bytes).  Descriptors count units of u bytes.
constexpr int kPairBytes = 12;

__global__ __launch_bounds__(256) void tr_count_kernel(int64_t n_rows, int64_t n_cols, int64_t bw,
                                                       const int64_t *ptr, const int32_t *idx, int32_t *cnt) {
    const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= n_rows) return;
    const int lane = threadIdx.x & 63;
    const int64_t band_off = (row / bw) * n_cols;
    for (int64_t e = ptr[row] + lane; e < ptr[row + 1]; e += 64) atomicAdd(&cnt[band_off + idx[e]], 1);
}

// the transpose plan as one scan: units per bucket (map) -> descriptors {first unit, pairs} (output);
// desc[n] = the total units as {low, high} 32-bit words
struct TrUnitsMap {
    int32_t unit;
    __device__ int64_t operator()(int32_t c) const { return (kPairBytes * ((c + 1) >> 1) + unit - 1) / unit; }
};
struct TrDescOut {
    const int32_t *cnt;
    uint2 *desc;
    __device__ void operator()(int64_t i, int64_t first) const {
        desc[i] = make_uint2((uint32_t)first, (uint32_t)((cnt[i] + 1) >> 1));
    }
    __device__ void total(int64_t n, int64_t t) const { desc[n] = make_uint2((uint32_t)t, (uint32_t)(t >> 32)); }
};

__global__ __launch_bounds__(256) void tr_fill_kernel(int64_t n_rows, int64_t n_cols, int64_t bw, const int64_t *ptr,
                                                      const int32_t *idx, const float *val, const uint2 *desc,
                                                      int32_t *cursor, unsigned char *t_rec, int32_t unit,
                                                      unsigned int *maxabs_bits, float *row_max, double *row_sum) {
    const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= n_rows) return;
    const int lane = threadIdx.x & 63;
    const int64_t band = row / bw, band_off = band * n_cols;
    const uint16_t jr = (uint16_t)(row - band * bw);
    float mx = 0.f;
    double sm = 0.0;
    for (int64_t e = ptr[row] + lane; e < ptr[row + 1]; e += 64) {
        const int64_t b = band_off + idx[e];
        const int32_t s = atomicAdd(&cursor[b], 1);
        unsigned char *pair = t_rec + (int64_t)desc[b].x * unit + (int64_t)kPairBytes * (s >> 1);
        reinterpret_cast<uint16_t *>(pair)[s & 1] = (uint16_t)(jr * 8u);  // byte offset of the int64 counter
        reinterpret_cast<float *>(pair + 4)[s & 1] = val[e];
        mx = fmaxf(mx, fabsf(val[e]));
        sm += (double)fabsf(val[e]);
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) mx = fmaxf(mx, __shfl_xor(mx, off, 64));
    sm = wave_sum<double>(sm);
    if (lane == 0) { row_max[row] = mx; row_sum[row] = sm; }
    // non-negative floats order like their bit patterns
    if (lane == 0 && mx > 0.f) atomicMax(maxabs_bits, __float_as_uint(mx));
}

// Gram fixed-point shift of every row r: the largest power of two S = 2^sh with every
// term |Phi[r,k] Phi[j,k]| S <= T S < 2^51 (exact magic-number rounding) and the sum of all
// |terms| S <= B S < 2^62 (no int64 overflow); T = max_k |Phi[r,k]| max|Phi|, B = sum_k |Phi[r,k]| max|Phi|.
__global__ void tr_rowshift_kernel(int64_t n_rows, const float *row_max, const double *row_sum,
                                   const float *maxabs, int32_t *shift) {
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n_rows) return;
    const double mx = (double)maxabs[0];
    const double B = row_sum[r] * mx * (1.0 + 1e-12), T = (double)row_max[r] * mx;
    const int eB = B > 0.0 ? ilogb(B) + 1 : 0;  // B < 2^eB
    const int eT = T > 0.0 ? ilogb(T) + 1 : 0;  // every term < 2^eT
    shift[r] = min(51 - eT, 62 - eB);
}

// odd buckets: the second record of the last pair is (col 0, +0.0) -- adds exactly 0
__global__ void tr_pad_fill_kernel(int64_t n, const uint2 *desc, const int32_t *cursor, unsigned char *t_rec,
                                   int32_t unit) {
    const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (b < n && (cursor[b] & 1)) {
        unsigned char *pair = t_rec + (int64_t)desc[b].x * unit + (int64_t)kPairBytes * (cursor[b] >> 1);
        reinterpret_cast<uint16_t *>(pair)[1] = 0;
        reinterpret_cast<float *>(pair + 4)[1] = 0.f;
    }
}


// ---------------------------------------------------- staged (binned) transpose fill
// tr_fill_kernel places every record with a global atomic on its bucket's cursor and two
// scattered sub-line stores (43.5 M atomics and partially written lines at C4).  The staged
// fill moves the entries in two passes whose global writes are whole lines:
//   1. tr_bin_kernel: a workgroup takes kBinRows rows of one band, counting-sorts their
//      entries by region = (band, cr-column range) in LDS and writes them back over its own
//      CSR range of the staging buffer as {u16 8 * row-in-band, u16 column-in-region, f32
//      value}, plus its per-region offsets (table row of nreg + 1 ints).
//   2. tr_place_kernel: a workgroup per region gathers the region's sub-runs from the band's
//      binning workgroups, builds the region's records (a contiguous range of lines: buckets
//      are ordered by (band, column)) in LDS with LDS cursors -- the odd buckets' padding is
//      the zero fill -- and writes the image with 16-byte stores.  A region whose image
//      exceeds the LDS cap falls back to global cursors.
constexpr int kRegionCols = 128;          // columns per region (at least; see tr_region_cols)
constexpr int kPlaceCap = 48 * 1024;      // LDS image cap of one region
constexpr int kBinRows = 16;              // rows per binning workgroup (divides every band: band_width % 64 == 0)
constexpr int kBinCap = 8192;             // entries of one binning workgroup sorted in LDS (64 KiB)

__global__ __launch_bounds__(256) void tr_bin_kernel(int64_t n_rows, int64_t n_cols, int64_t bw, int32_t cr,
                                                     int32_t nreg, const int64_t *ptr, const int32_t *idx,
                                                     const float *val, uint2 *staging, int32_t *tab,
                                                     float *wg_max, float *row_max, double *row_sum) {
    extern __shared__ __attribute__((aligned(16))) unsigned char tb_smem[];
    uint2 *img = reinterpret_cast<uint2 *>(tb_smem);                        // [kBinCap]
    uint32_t *cnt = reinterpret_cast<uint32_t *>(img + kBinCap);            // [nreg] counts, then cursors
    int32_t *rp = reinterpret_cast<int32_t *>(cnt + nreg);                  // [kBinRows + 1]
    int32_t *scratch = rp + kBinRows + 1;                                   // [8]
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int64_t r0 = (int64_t)blockIdx.x * kBinRows, r1 = min<int64_t>(n_rows, r0 + kBinRows);
    const int nr = (int)(r1 - r0);
    const int64_t band = r0 / bw;
    const int64_t E0 = ptr[r0];
    const int32_t nE = (int32_t)(ptr[r1] - E0);
    for (int g = tid; g < nreg; g += 256) cnt[g] = 0u;
    for (int i = tid; i <= nr; i += 256) rp[i] = (int32_t)(ptr[r0 + i] - E0);
    __syncthreads();
    // the workgroup's entries: in registers (all loads in flight at once) when they fit
    constexpr int kPerT = kBinCap / 256;
    const bool in_lds = nE <= kBinCap;
    int32_t kr[kPerT];
    float vr[kPerT];
    if (in_lds) {
#pragma unroll
        for (int q = 0; q < kPerT; ++q) {
            const int32_t e = tid + q * 256;
            kr[q] = e < nE ? idx[E0 + e] : -1;
            vr[q] = e < nE ? val[E0 + e] : 0.f;
        }
#pragma unroll
        for (int q = 0; q < kPerT; ++q)
            if (kr[q] >= 0) atomicAdd(&cnt[kr[q] / cr], 1u);
    } else {
        for (int32_t e = tid; e < nE; e += 256) atomicAdd(&cnt[idx[E0 + e] / cr], 1u);
    }
    // per-row max / sum of |values| (one wave per row, fixed order: deterministic shifts)
    float wmx = 0.f;
    for (int i = wave; i < nr; i += 4) {
        float mx = 0.f;
        double sm = 0.0;
        for (int32_t e = rp[i] + lane; e < rp[i + 1]; e += 64) {
            const float a = fabsf(val[E0 + e]);
            mx = fmaxf(mx, a);
            sm += (double)a;
        }
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) mx = fmaxf(mx, __shfl_xor(mx, off, 64));
        sm = wave_sum<double>(sm);
        if (lane == 0) {
            row_max[r0 + i] = mx;
            row_sum[r0 + i] = sm;
        }
        wmx = fmaxf(wmx, mx);
    }
    // the workgroup's max |value| (one store; reduced by tr_maxabs_kernel -- one global atomic per
    // row on a single word serialised the old fill)
    if (lane == 0) scratch[wave] = (int32_t)__float_as_uint(wmx);
    __syncthreads();
    if (tid == 0) {
        float m = 0.f;
        for (int q = 0; q < 4; ++q) m = fmaxf(m, __uint_as_float((uint32_t)scratch[q]));
        wg_max[blockIdx.x] = m;
    }
    __syncthreads();
    // exclusive offsets of the regions (thread t owns regions [t * per, (t + 1) * per))
    const int per = (nreg + 255) / 256;
    int32_t sum = 0;
    for (int q = 0; q < per; ++q) {
        const int g = tid * per + q;
        if (g < nreg) sum += (int32_t)cnt[g];
    }
    int32_t total;
    int32_t run = block_exclusive_scan<int32_t>(sum, scratch, &total);
    int32_t *trow = tab + (int64_t)blockIdx.x * (nreg + 1);
    for (int q = 0; q < per; ++q) {
        const int g = tid * per + q;
        if (g < nreg) {
            const int32_t c = (int32_t)cnt[g];
            trow[g] = run;
            cnt[g] = (uint32_t)run;  // cursor
            run += c;
        }
    }
    if (tid == 0) trow[nreg] = total;
    __syncthreads();
    const uint32_t jr0 = (uint32_t)(r0 - band * bw);
    uint2 *out = staging + E0;
    auto row_of = [&](int32_t e) {  // the entry's row: the last i with rp[i] <= e
        int lo = 0, hi = nr;
        while (hi - lo > 1) {
            const int mid = (lo + hi) >> 1;
            if (rp[mid] <= e) lo = mid;
            else hi = mid;
        }
        return lo;
    };
    if (in_lds) {
#pragma unroll
        for (int q = 0; q < kPerT; ++q) {
            const int32_t e = tid + q * 256, k = kr[q];
            if (k >= 0) {
                const int g = k / cr;
                const uint32_t s = atomicAdd(&cnt[g], 1u);
                img[s] = make_uint2(((jr0 + (uint32_t)row_of(e)) * 8u) | ((uint32_t)(k - g * cr) << 16),
                                    __float_as_uint(vr[q]));
            }
        }
    } else {
        for (int32_t e = tid; e < nE; e += 256) {
            const int32_t k = idx[E0 + e];
            const int g = k / cr;
            const uint32_t s = atomicAdd(&cnt[g], 1u);
            out[s] = make_uint2(((jr0 + (uint32_t)row_of(e)) * 8u) | ((uint32_t)(k - g * cr) << 16),
                                __float_as_uint(val[E0 + e]));
        }
    }
    if (in_lds) {
        __syncthreads();
        for (int32_t e = tid; e < nE; e += 256) out[e] = img[e];
    }
}

// max over the binning workgroups' maxima (one workgroup)
__global__ __launch_bounds__(1024) void tr_maxabs_kernel(int64_t n, const float *wg_max, float *maxabs) {
    __shared__ float red[16];
    float m = 0.f;
    for (int64_t i = threadIdx.x; i < n; i += 1024) m = fmaxf(m, wg_max[i]);
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) m = fmaxf(m, __shfl_xor(m, off, 64));
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int q = 1; q < 16; ++q) m = fmaxf(m, red[q]);
        *maxabs = fmaxf(m, red[0]);
    }
}

// Per-row max / sum of |values| over a whole CSR (one wave per row, the loop order of the
// transpose's binning kernel) and each workgroup's max: the Gram row shifts of rows that are not
// in the transpose (the column-block Gram of the multi-GPU path).
// (cap > 0: padded rows instead -- row r's cnt[r] entries at r cap, ptr unused; the same sums)
__global__ __launch_bounds__(256) void phi_row_stats_kernel(int64_t n_rows, const int64_t *ptr, const float *val,
                                                            float *wg_max, float *row_max, double *row_sum,
                                                            int64_t cap = 0, const int32_t *cnt = nullptr) {
    __shared__ float red[4];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int64_t r = (int64_t)blockIdx.x * 4 + wave;
    float mx = 0.f;
    if (r < n_rows) {
        double sm = 0.0;
        const int64_t e0 = cap > 0 ? r * cap : ptr[r], e1 = cap > 0 ? r * cap + cnt[r] : ptr[r + 1];
        for (int64_t e = e0 + lane; e < e1; e += 256) {  // (up to four loads in flight, summed in e order)
            float a[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) a[q] = e + 64 * q < e1 ? fabsf(val[e + 64 * q]) : 0.f;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                if (e + 64 * q < e1) {
                    mx = fmaxf(mx, a[q]);
                    sm += (double)a[q];
                }
            }
        }
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) mx = fmaxf(mx, __shfl_xor(mx, off, 64));
        sm = wave_sum<double>(sm);
        if (lane == 0) {
            row_max[r] = mx;
            row_sum[r] = sm;
        }
    }
    if (lane == 0) red[wave] = mx;
    __syncthreads();
    if (threadIdx.x == 0) wg_max[blockIdx.x] = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
}

__global__ __launch_bounds__(256) void tr_place_kernel(int64_t n_rows, int64_t n_cols, int64_t bw, int32_t cr,
                                                       int32_t nreg, const int64_t *ptr, const uint2 *desc,
                                                       const int64_t *ent_off, const uint2 *staging,
                                                       const int32_t *tab, int32_t *gcur, unsigned char *t_rec,
                                                       int32_t unit) {
    extern __shared__ __attribute__((aligned(16))) unsigned char tp_smem[];
    const int tid = threadIdx.x;
    const int64_t band = blockIdx.x / nreg, g = blockIdx.x - band * nreg;
    const int64_t c0 = g * cr, c1 = min<int64_t>(n_cols, c0 + cr);
    const int64_t b0 = band * n_cols + c0, b1 = band * n_cols + c1;
    const int64_t L0 = desc[b0].x, L1 = desc[b1].x;  // (desc[nbk].x = total lines, low word)
    const int64_t img = (L1 - L0) * unit;
    if (ent_off[b1] == ent_off[b0]) return;
    // the band's binning workgroups
    const int64_t w0 = band * bw / kBinRows, w1 = cdiv<int64_t>(min<int64_t>(n_rows, (band + 1) * bw), kBinRows);
    const bool lds = (img + 15) / 16 * 16 <= kPlaceCap;
    uint32_t *lcur = reinterpret_cast<uint32_t *>(tp_smem);   // [cr]
    uint32_t *lline = lcur + cr;                               // [cr] first byte of each bucket in the image
    unsigned char *image = tp_smem + 8 * cr;                   // [img]
    if (lds) {
        for (int i = tid; i < c1 - c0; i += 256) {
            lcur[i] = 0u;
            lline[i] = (uint32_t)((desc[b0 + i].x - L0) * unit);
        }
        for (int64_t i = tid; i < (img + 15) / 16; i += 256) reinterpret_cast<uint4 *>(image)[i] = make_uint4(0u, 0u, 0u, 0u);
        __syncthreads();
    }
    for (int64_t w = w0 + tid; w < w1; w += 256) {
        const int32_t *trow = tab + w * (nreg + 1);
        const int32_t o0 = trow[g], o1 = trow[g + 1];
        const uint2 *run = staging + ptr[w * kBinRows];
        for (int32_t o = o0; o < o1; ++o) {
            const uint2 x = run[o];
            const uint32_t kk = x.x >> 16;
            if (lds) {
                const uint32_t s = atomicAdd(&lcur[kk], 1u);
                unsigned char *pair = image + lline[kk] + kPairBytes * (s >> 1);
                reinterpret_cast<uint16_t *>(pair)[s & 1] = (uint16_t)(x.x & 0xffffu);
                reinterpret_cast<uint32_t *>(pair + 4)[s & 1] = x.y;
            } else {  // oversized region: global cursors (zeroed by the caller)
                const int64_t b = b0 + kk;
                const int32_t s = atomicAdd(&gcur[b], 1);
                unsigned char *pair = t_rec + (int64_t)desc[b].x * unit + (int64_t)kPairBytes * (s >> 1);
                reinterpret_cast<uint16_t *>(pair)[s & 1] = (uint16_t)(x.x & 0xffffu);
                reinterpret_cast<uint32_t *>(pair + 4)[s & 1] = x.y;
            }
        }
    }
    if (lds) {
        __syncthreads();
        if ((L0 * unit) % 16 == 0 && img % 16 == 0) {  // whole lines: 16-byte stores
            uint4 *dst = reinterpret_cast<uint4 *>(t_rec + L0 * unit);
            for (int64_t i = tid; i < img / 16; i += 256) dst[i] = reinterpret_cast<const uint4 *>(image)[i];
        } else {  // packed records: the region's exact byte range (a multiple of 4 at a 4-byte offset)
            uint32_t *dst = reinterpret_cast<uint32_t *>(t_rec + L0 * unit);
            for (int64_t i = tid; i < img / 4; i += 256) dst[i] = reinterpret_cast<const uint32_t *>(image)[i];
        }
        return;
    }
    for (int64_t b = b0 + tid; b < b1; b += 256) {  // pad the odd buckets
        const int32_t c = (int32_t)(ent_off[b + 1] - ent_off[b]);
        if (c & 1) {
            unsigned char *pair = t_rec + (int64_t)desc[b].x * unit + (int64_t)kPairBytes * (c >> 1);
            reinterpret_cast<uint16_t *>(pair)[1] = 0;
            reinterpret_cast<float *>(pair + 4)[1] = 0.f;
        }
    }
}

// ---- the plan-free (self-counting) staged transpose: no bucket counts from the walk, no scan over
// every bucket.  After tr_bin, (1) tr_region_units bounds each (band, region)'s record units from
// its entry count E and bucket count nb (units of its buckets <= 6 (E + nb) / unit + nb + 1, packed:
// (E + nb + 1) / 2), (2) one scan over the regions gives every region a slab of that size, and
// (3) tr_place_self counts the region's buckets in LDS, lays them out inside the slab (the unused
// tail of a slab is never read: the Gram reads through the descriptors), writes their descriptors
// and places the records as tr_place does.
__global__ __launch_bounds__(256) void tr_region_units_kernel(int64_t n_rows, int64_t n_cols, int64_t bw, int32_t cr,
                                                              int32_t nreg, int64_t n_regions, const int32_t *tab,
                                                              int32_t unit, int64_t *region_units) {
    const int64_t rg = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (rg >= n_regions) return;
    const int lane = threadIdx.x & 63;
    const int64_t band = rg / nreg, g = rg - band * nreg;
    const int64_t w0 = band * bw / kBinRows, w1 = cdiv<int64_t>(min<int64_t>(n_rows, (band + 1) * bw), kBinRows);
    int64_t E = 0;
    for (int64_t w = w0 + lane; w < w1; w += 64) {
        const int32_t *trow = tab + w * (nreg + 1);
        E += trow[g + 1] - trow[g];
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) E += __shfl_xor(E, off, 64);
    const int64_t nb = min<int64_t>(n_cols, (g + 1) * (int64_t)cr) - g * (int64_t)cr;
    if (lane == 0)
        region_units[rg] = E == 0 ? 0 : unit == kPairBytes ? (E + nb + 1) / 2 : (6 * (E + nb)) / unit + nb + 1;
}

struct RegionBaseOut {  // region_base[i] = first unit of region i; the total also as desc[nbk] (lo, hi)
    int64_t *base;
    uint2 *desc_total;
    __device__ void operator()(int64_t i, int64_t prefix) const { base[i] = prefix; }
    __device__ void total(int64_t n, int64_t t) const {
        base[n] = t;
        *desc_total = make_uint2((uint32_t)t, (uint32_t)(t >> 32));
    }
};

// kSplit: every bucket's entries are laid out by sub-band -- the eight row ranges of W / 8 rows
// of the band, in order -- and t_split[b] holds 8 u16 entry offsets, the entries of bucket b before
// each sub-band.  A symmetric-mode Gram tile on its own (diagonal) band needs only the columns j >= its
// row, i.e. the sub-bands from its row's on: it starts its bucket streams there.
// Oversized regions (global cursors) keep arbitrary order and report no split (all offsets 0).
constexpr int kSub = 8;

template <bool kSplit>
__global__ __launch_bounds__(256) void tr_place_self_kernel(int64_t n_rows, int64_t n_cols, int64_t bw, int32_t cr,
                                                            int32_t nreg, const int64_t *ptr,
                                                            const int64_t *region_base, const uint2 *staging,
                                                            const int32_t *tab, int32_t *gcur, uint2 *desc,
                                                            uint4 *t_split, unsigned char *t_rec, int32_t unit) {
    extern __shared__ __attribute__((aligned(16))) unsigned char tps_smem[];
    constexpr int kS = kSplit ? kSub : 1;  // counters per bucket
    const int tid = threadIdx.x;
    // dispatch group x = blockIdx % 8 (one XCD) takes a contiguous run of regions: neighbouring
    // regions read neighbouring words of the same table lines, which then come from one L2
    const int64_t nblk = gridDim.x, per8 = nblk / 8, rem8 = nblk % 8;
    const int64_t x8 = blockIdx.x % 8, k8 = blockIdx.x / 8;
    const int64_t rg = x8 * per8 + (x8 < rem8 ? x8 : rem8) + k8, band = rg / nreg, g = rg - band * nreg;
    const int64_t c0 = g * cr, c1 = min<int64_t>(n_cols, c0 + cr);
    const int nbk_r = (int)(c1 - c0);
    const int64_t b0 = band * n_cols + c0;
    const int64_t U0 = region_base[rg];
    uint32_t *lcur = reinterpret_cast<uint32_t *>(tps_smem);   // [cr * kS] counts, then cursors
    uint32_t *lline = lcur + cr * kS;                           // [cr] first byte of each bucket in the image
    int32_t *scratch = reinterpret_cast<int32_t *>(lline + cr); // [8]
    unsigned char *image = reinterpret_cast<unsigned char *>(scratch + 8);
    const int64_t w0 = band * bw / kBinRows, w1 = cdiv<int64_t>(min<int64_t>(n_rows, (band + 1) * bw), kBinRows);
    // (the staged entry's low half is 8 * its row in the band: 8 sub-bands of bw / 8 rows -> x / bw)
    auto slot = [&](uint32_t x) -> uint32_t {
        return kSplit ? (x >> 16) * kSub + (x & 0xffffu) / (uint32_t)bw : (x >> 16);
    };
    for (int i = tid; i < nbk_r * kS; i += 256) lcur[i] = 0u;
    __syncthreads();
    // pass 1: the region's bucket (and sub-band) counts (four loads in flight per thread)
    for (int64_t w = w0 + tid; w < w1; w += 256) {
        const int32_t *trow = tab + w * (nreg + 1);
        const int32_t o0 = trow[g], o1 = trow[g + 1];
        const uint2 *run = staging + ptr[w * kBinRows];
        int32_t o = o0;
        for (; o + 4 <= o1; o += 4) {
            uint32_t x[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) x[r] = run[o + r].x;
#pragma unroll
            for (int r = 0; r < 4; ++r) atomicAdd(&lcur[slot(x[r])], 1u);
        }
        for (; o < o1; ++o) atomicAdd(&lcur[slot(run[o].x)], 1u);
    }
    __syncthreads();
    auto bucket_count = [&](int i) -> uint32_t {
        uint32_t c = 0;
#pragma unroll
        for (int q = 0; q < kS; ++q) c += lcur[i * kS + q];
        return c;
    };
    // bucket units -> local offsets (thread t owns buckets [t * per, (t + 1) * per)), descriptors
    const int per = (nbk_r + 255) / 256;
    int32_t sum = 0;
    for (int q = 0; q < per; ++q) {
        const int i = tid * per + q;
        if (i < nbk_r) sum += (int32_t)((kPairBytes * ((bucket_count(i) + 1) >> 1) + unit - 1) / unit);
    }
    int32_t total;
    int32_t run_u = block_exclusive_scan<int32_t>(sum, scratch, &total);
    const bool lds = ((int64_t)total * unit + 15) / 16 * 16 <= kPlaceCap;
    for (int q = 0; q < per; ++q) {
        const int i = tid * per + q;
        if (i < nbk_r) {
            const uint32_t c = bucket_count(i);
            desc[b0 + i] = make_uint2((uint32_t)(U0 + run_u), (c + 1) >> 1);
            lline[i] = (uint32_t)run_u * (uint32_t)unit;
            run_u += (int32_t)((kPairBytes * ((c + 1) >> 1) + unit - 1) / unit);
            if (kSplit) {
                // entry offsets of the sub-bands; the counters become the sub-band cursors (an oversized
                // region keeps its counts for the padding below and reports no split)
                uint32_t off[kSub], o = 0;
#pragma unroll
                for (int sb = 0; sb < kSub; ++sb) {
                    off[sb] = lds ? o : 0u;
                    o += lcur[i * kSub + sb];
                    if (lds) lcur[i * kSub + sb] = off[sb];
                }
                t_split[b0 + i] = make_uint4(off[0] | (off[1] << 16), off[2] | (off[3] << 16), off[4] | (off[5] << 16),
                                             off[6] | (off[7] << 16));
            }
        }
    }
    __syncthreads();
    const int64_t img = (int64_t)total * unit;
    if (img == 0) return;
    if (!lds && !kSplit) {
        // oversized region (hub columns: 12 % of Enron's regions exceed the LDS image cap, up to ~500 KB):
        // the bucket cursors stay in LDS and every record is stored straight to its place in t_rec --
        // one global atomic per entry in a dependent chain per thread took ~1 ms per launch on Enron
        for (int i = tid; i < nbk_r; i += 256) {  // the odd buckets' padding record (0, +0.0)
            const uint32_t c = lcur[i];
            if (c & 1) {
                unsigned char *pair = t_rec + (U0 * unit + lline[i]) + (int64_t)kPairBytes * (c >> 1);
                reinterpret_cast<uint16_t *>(pair)[1] = 0;
                reinterpret_cast<float *>(pair + 4)[1] = 0.f;
            }
        }
        __syncthreads();
        for (int i = tid; i < nbk_r; i += 256) lcur[i] = 0u;
        __syncthreads();
        unsigned char *region = t_rec + U0 * unit;
        for (int64_t w = w0 + tid; w < w1; w += 256) {
            const int32_t *trow = tab + w * (nreg + 1);
            const int32_t o0 = trow[g], o1 = trow[g + 1];
            const uint2 *run = staging + ptr[w * kBinRows];
            int32_t o = o0;
            for (; o + 4 <= o1; o += 4) {  // (four loads in flight per thread)
                uint2 x[4];
#pragma unroll
                for (int r = 0; r < 4; ++r) x[r] = run[o + r];
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const uint32_t kk = x[r].x >> 16;
                    const uint32_t sl = atomicAdd(&lcur[kk], 1u);
                    unsigned char *pair = region + lline[kk] + kPairBytes * (sl >> 1);
                    reinterpret_cast<uint16_t *>(pair)[sl & 1] = (uint16_t)(x[r].x & 0xffffu);
                    reinterpret_cast<uint32_t *>(pair + 4)[sl & 1] = x[r].y;
                }
            }
            for (; o < o1; ++o) {
                const uint2 x = run[o];
                const uint32_t kk = x.x >> 16;
                const uint32_t sl = atomicAdd(&lcur[kk], 1u);
                unsigned char *pair = region + lline[kk] + kPairBytes * (sl >> 1);
                reinterpret_cast<uint16_t *>(pair)[sl & 1] = (uint16_t)(x.x & 0xffffu);
                reinterpret_cast<uint32_t *>(pair + 4)[sl & 1] = x.y;
            }
        }
        return;
    }
    if (lds) {
        for (int64_t i = tid; i < (img + 15) / 16; i += 256) reinterpret_cast<uint4 *>(image)[i] = make_uint4(0u, 0u, 0u, 0u);
    } else {  // oversized region: global cursors of its own buckets, odd buckets padded below
        for (int i = tid; i < nbk_r; i += 256) {
            gcur[b0 + i] = 0;
            const uint32_t c = bucket_count(i);
            if (c & 1) {
                unsigned char *pair = t_rec + (U0 * unit + lline[i]) + (int64_t)kPairBytes * (c >> 1);
                reinterpret_cast<uint16_t *>(pair)[1] = 0;
                reinterpret_cast<float *>(pair + 4)[1] = 0.f;
            }
        }
    }
    if (!kSplit) {
        for (int i = tid; i < nbk_r; i += 256) lcur[i] = 0u;
    }
    __syncthreads();
    // pass 2: place the records (the region's entries come from L2: pass 1 just read them)
    for (int64_t w = w0 + tid; w < w1; w += 256) {
        const int32_t *trow = tab + w * (nreg + 1);
        const int32_t o0 = trow[g], o1 = trow[g + 1];
        const uint2 *run = staging + ptr[w * kBinRows];
        int32_t o = o0;
        if (lds) {
            for (; o + 4 <= o1; o += 4) {  // (four loads in flight per thread)
                uint2 x[4];
#pragma unroll
                for (int r = 0; r < 4; ++r) x[r] = run[o + r];
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const uint32_t s = atomicAdd(&lcur[slot(x[r].x)], 1u);
                    unsigned char *pair = image + lline[x[r].x >> 16] + kPairBytes * (s >> 1);
                    reinterpret_cast<uint16_t *>(pair)[s & 1] = (uint16_t)(x[r].x & 0xffffu);
                    reinterpret_cast<uint32_t *>(pair + 4)[s & 1] = x[r].y;
                }
            }
        }
        for (; o < o1; ++o) {
            const uint2 x = run[o];
            const uint32_t kk = x.x >> 16;
            if (lds) {
                const uint32_t s = atomicAdd(&lcur[slot(x.x)], 1u);
                unsigned char *pair = image + lline[kk] + kPairBytes * (s >> 1);
                reinterpret_cast<uint16_t *>(pair)[s & 1] = (uint16_t)(x.x & 0xffffu);
                reinterpret_cast<uint32_t *>(pair + 4)[s & 1] = x.y;
            } else {
                const int32_t s = atomicAdd(&gcur[b0 + kk], 1);
                unsigned char *pair = t_rec + (U0 * unit + lline[kk]) + (int64_t)kPairBytes * (s >> 1);
                reinterpret_cast<uint16_t *>(pair)[s & 1] = (uint16_t)(x.x & 0xffffu);
                reinterpret_cast<uint32_t *>(pair + 4)[s & 1] = x.y;
            }
        }
    }
    if (!lds) return;
    __syncthreads();
    if ((U0 * unit) % 16 == 0 && img % 16 == 0) {
        uint4 *dst = reinterpret_cast<uint4 *>(t_rec + U0 * unit);
        for (int64_t i = tid; i < img / 16; i += 256) dst[i] = reinterpret_cast<const uint4 *>(image)[i];
    } else {
        uint32_t *dst = reinterpret_cast<uint32_t *>(t_rec + U0 * unit);
        for (int64_t i = tid; i < img / 4; i += 256) dst[i] = reinterpret_cast<const uint32_t *>(image)[i];
    }
}

// GRF_REC_SLOT: bucket b owns the 32-byte slot t_rec + 32 b = {u32 pairs, u32 first overflow pair,
// pair 0, pair 1}: its first four entries inline, the rest as packed pairs in the overflow area after
// all nbk slots (t_rec + 32 nbk + 12 * pair).  The Gram reads a bucket of <= 2 pairs -- almost every
// bucket of a column block over a power-law Phi (C5: ~1.4 entries) -- with its header in one line,
// instead of a descriptor line and a record line.  Same staging and region bases as the packed
// placement (the region's units bound its overflow pairs); one workgroup per region, slots written
// whole (header + zeroed payload) before the entries land in them.
__global__ __launch_bounds__(256) void tr_place_slots_kernel(int64_t n_rows, int64_t n_cols, int64_t bw, int32_t cr,
                                                             int32_t nreg, int64_t nbk, const int64_t *ptr,
                                                             const int64_t *region_base, const uint2 *staging,
                                                             const int32_t *tab, int32_t *gcur,
                                                             unsigned char *t_rec) {
    extern __shared__ __attribute__((aligned(16))) unsigned char tps_smem[];
    const int tid = threadIdx.x;
    const int64_t nblk = gridDim.x, per8 = nblk / 8, rem8 = nblk % 8;
    const int64_t x8 = blockIdx.x % 8, k8 = blockIdx.x / 8;
    const int64_t rg = x8 * per8 + (x8 < rem8 ? x8 : rem8) + k8, band = rg / nreg, g = rg - band * nreg;
    const int64_t c0 = g * cr, c1 = min<int64_t>(n_cols, c0 + cr);
    const int nbk_r = (int)(c1 - c0);
    const int64_t b0 = band * n_cols + c0;
    const int64_t U0 = region_base[rg];                          // the region's first overflow pair
    uint32_t *lcur = reinterpret_cast<uint32_t *>(tps_smem);     // [cr] counts, then cursors
    uint32_t *lovf = lcur + cr;                                  // [cr] first overflow pair (local)
    int32_t *scratch = reinterpret_cast<int32_t *>(lovf + cr);   // [8]
    unsigned char *image = reinterpret_cast<unsigned char *>(scratch + 8);
    unsigned char *slots = t_rec + 32 * b0, *ovf = t_rec + 32 * nbk + (int64_t)kPairBytes * U0;
    const int64_t w0 = band * bw / kBinRows, w1 = cdiv<int64_t>(min<int64_t>(n_rows, (band + 1) * bw), kBinRows);
    for (int i = tid; i < nbk_r; i += 256) lcur[i] = 0u;
    __syncthreads();
    for (int64_t w = w0 + tid; w < w1; w += 256) {  // pass 1: the region's bucket counts
        const int32_t *trow = tab + w * (nreg + 1);
        const int32_t o0 = trow[g], o1 = trow[g + 1];
        const uint2 *run = staging + ptr[w * kBinRows];
        for (int32_t o = o0; o < o1; ++o) atomicAdd(&lcur[run[o].x >> 16], 1u);
    }
    __syncthreads();
    const int per = (nbk_r + 255) / 256;
    int32_t sum = 0;
    for (int q = 0; q < per; ++q) {
        const int i = tid * per + q;
        if (i < nbk_r) sum += max(0, (int32_t)((lcur[i] + 1) >> 1) - 2);
    }
    int32_t total;
    int32_t run_p = block_exclusive_scan<int32_t>(sum, scratch, &total);
    const bool lds = ((int64_t)total * kPairBytes + 15) / 16 * 16 <= kPlaceCap;
    for (int q = 0; q < per; ++q) {
        const int i = tid * per + q;
        if (i < nbk_r) {
            const uint32_t c = lcur[i], pairs = (c + 1) >> 1;
            lovf[i] = (uint32_t)run_p;
            uint4 *sl = reinterpret_cast<uint4 *>(slots + 32 * (int64_t)i);
            sl[0] = make_uint4(pairs, (uint32_t)(U0 + run_p), 0u, 0u);
            sl[1] = make_uint4(0u, 0u, 0u, 0u);
            run_p += max(0, (int32_t)pairs - 2);
            lcur[i] = 0u;  // (the counts become cursors)
        }
    }
    const int64_t img = (int64_t)total * kPairBytes;
    if (lds) {
        for (int64_t i = tid; i < (img + 15) / 16; i += 256) reinterpret_cast<uint4 *>(image)[i] = make_uint4(0u, 0u, 0u, 0u);
    } else {  // oversized region: overflow pairs straight to global, zeroed first
        for (int64_t i = tid; i < img / 4; i += 256) reinterpret_cast<uint32_t *>(ovf)[i] = 0u;
    }
    __threadfence_block();
    __syncthreads();
    for (int64_t w = w0 + tid; w < w1; w += 256) {  // pass 2: place the entries
        const int32_t *trow = tab + w * (nreg + 1);
        const int32_t o0 = trow[g], o1 = trow[g + 1];
        const uint2 *run = staging + ptr[w * kBinRows];
        for (int32_t o = o0; o < o1; ++o) {
            const uint2 x = run[o];
            const uint32_t kk = x.x >> 16;
            const uint32_t s = atomicAdd(&lcur[kk], 1u);
            unsigned char *pair;
            uint32_t half;
            if (s < 4) {
                pair = slots + 32 * (int64_t)kk + 8 + kPairBytes * (s >> 1);
                half = s & 1;
            } else {
                const uint32_t q = s - 4;
                pair = (lds ? image : ovf) + kPairBytes * (int64_t)(lovf[kk] + (q >> 1));
                half = q & 1;
            }
            reinterpret_cast<uint16_t *>(pair)[half] = (uint16_t)(x.x & 0xffffu);
            reinterpret_cast<uint32_t *>(pair + 4)[half] = x.y;
        }
    }
    if (!lds || img == 0) return;
    __syncthreads();
    uint32_t *dst = reinterpret_cast<uint32_t *>(ovf);
    for (int64_t i = tid; i < img / 4; i += 256) dst[i] = reinterpret_cast<const uint32_t *>(image)[i];
    (void)gcur;
}

// Region width: at most 4096 regions per band, and every placing workgroup reads one table
// entry per binning workgroup of its band, n_rows * n_cols / (16 cr) scattered reads in all --
// kept <= 32 M (C4: cr = 128, 4.9 M; C5, N = 1M: cr = 2048 instead of 256, where 244 M reads
// took 4.9 ms of the placing pass).
static int32_t tr_region_cols(int64_t n_rows, int64_t n_cols) {
    int64_t cr = kRegionCols;
    while (cr < 65536 && (cdiv<int64_t>(n_cols, cr) > 4096 ||
                          (double)std::max<int64_t>(n_rows, 1) * (double)n_cols / (16.0 * (double)cr) > 32e6))
        cr *= 2;
    return (int32_t)cr;
}

// Segment r (src[r * stride .. r * stride + len[r])) -> dst[dst_off[r] ..]: the multi-GPU Phi
// all-gather's compaction, with every length and offset on the device (no host round trip).
__global__ __launch_bounds__(256) void concat_segments_kernel(int64_t stride, const uint32_t *__restrict__ src,
                                                              const int64_t *__restrict__ len,
                                                              const int64_t *__restrict__ dst_off,
                                                              uint32_t *__restrict__ dst) {
    const int64_t seg = blockIdx.y;
    const int64_t l = len[seg], o = dst_off[seg];
    const uint32_t *s = src + seg * stride;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < l; i += (int64_t)gridDim.x * 256) dst[o + i] = s[i];
}

}  // namespace grf

using namespace grf;

extern "C" {
#pragma GCC visibility push(default)

int32_t grf_concat_segments(int32_t n_seg, int64_t stride, const void *src, const int64_t *seg_len,
                            const int64_t *dst_off, void *dst, grf_stream_t stream) {
    GRF_REQUIRE(n_seg >= 0 && n_seg <= 65535 && stride >= 0 && (n_seg == 0 || (src && seg_len && dst_off && dst)),
                GRF_EINVAL, "grf_concat_segments: bad arguments");
    if (n_seg == 0 || stride == 0) return GRF_OK;
    const int64_t bx = std::min<int64_t>(cdiv<int64_t>(stride, 256), 2048);
    concat_segments_kernel<<<dim3((unsigned)bx, (unsigned)n_seg), 256, 0, S(stream)>>>(
        stride, (const uint32_t *)src, seg_len, dst_off, (uint32_t *)dst);
    GRF_CHECK_LAUNCH("concat_segments_kernel");
    return GRF_OK;
}

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
    const int64_t nwg = cdiv<int64_t>(n_rows, 4 * kCompactRows);
    GRF_REQUIRE_GRID(nwg, 256, "compact_rows_kernel");
    compact_rows_kernel<false><<<(unsigned)nwg, 256, 0, S(stream)>>>(n_rows, cap, cnt, out_ptr, in_idx, in_val, in_val32,
                                                                    out_idx, out_val, out_val32, nullptr, nullptr,
                                                                    nullptr);
    GRF_CHECK_LAUNCH("compact_rows_kernel");
    return GRF_OK;
}

static size_t tr_align(size_t x) { return (x + 255) & ~(size_t)255; }

size_t grf_transpose_workspace_bytes(int64_t n_buckets) {
    return 2 * tr_align((size_t)n_buckets * sizeof(int32_t)) + tr_align((size_t)(n_buckets + 1) * sizeof(int64_t)) +
           scan_ws_bytes(n_buckets);
}

int32_t grf_transpose_banded_plan(int64_t n_rows, int64_t n_cols, int64_t band_width, int32_t rec_unit,
                                  const int64_t *ptr, const int32_t *idx, uint32_t *t_desc, int32_t counted,
                                  void *workspace, size_t workspace_bytes, grf_stream_t stream) {
    GRF_REQUIRE(n_rows >= 0 && n_cols > 0 && band_width > 0 && band_width <= 8192 && ptr && idx && t_desc,
                GRF_EINVAL, "grf_transpose_banded_plan: bad arguments");
    GRF_REQUIRE(rec_unit == GRF_REC_LINE || rec_unit == GRF_REC_PACKED, GRF_EINVAL,
                "grf_transpose_banded_plan: rec_unit must be GRF_REC_LINE or GRF_REC_PACKED");
    const int64_t nb = cdiv<int64_t>(n_rows, band_width), nbk = nb * n_cols;
    GRF_REQUIRE(workspace_bytes >= grf_transpose_workspace_bytes(nbk), GRF_EINVAL,
                "grf_transpose_banded_plan: workspace too small (%zu < %zu)", workspace_bytes,
                grf_transpose_workspace_bytes(nbk));
    hipStream_t st = S(stream);
    char *w = (char *)workspace;
    int32_t *cnt = (int32_t *)w;
    // (the workspace layout is shared with the fills: [cnt | row_max | ent_off | scan scratch])
    void *scan_ws = w + 2 * tr_align((size_t)nbk * 4) + tr_align((size_t)(nbk + 1) * 8);
    if (!counted) GRF_CHECK_HIP(hipMemsetAsync(cnt, 0, (size_t)nbk * sizeof(int32_t), st));
    if (n_rows > 0 && !counted) {
        GRF_REQUIRE_GRID(cdiv<int64_t>(n_rows, 4), 256, "tr_count_kernel");
        tr_count_kernel<<<(unsigned)cdiv<int64_t>(n_rows, 4), 256, 0, st>>>(n_rows, n_cols, band_width, ptr, idx,
                                                                          cnt);
        GRF_CHECK_LAUNCH("tr_count_kernel");
    }
    // units per bucket -> exclusive scan -> descriptors, in one scan (no units / offsets arrays)
    return scan_exclusive<int32_t>(nbk, cnt, TrUnitsMap{rec_unit}, TrDescOut{cnt, reinterpret_cast<uint2 *>(t_desc)},
                                   (int64_t *)scan_ws, st);
}

int32_t grf_transpose_banded_fill(int64_t n_rows, int64_t n_cols, int64_t band_width, int32_t rec_unit,
                                  const int64_t *ptr, const int32_t *idx, const float *val, const uint32_t *t_desc,
                                  void *t_rec, int64_t t_rec_bytes, float *t_maxabs, int32_t *t_rowshift,
                                  void *workspace, size_t workspace_bytes, grf_stream_t stream) {
    GRF_REQUIRE(n_rows >= 0 && n_cols > 0 && band_width > 0 && band_width <= 8192 && ptr && idx && val && t_desc &&
                    t_rec && t_maxabs && t_rowshift && t_rec_bytes >= 0,
                GRF_EINVAL, "grf_transpose_banded_fill: bad arguments");
    GRF_REQUIRE(rec_unit == GRF_REC_LINE || rec_unit == GRF_REC_PACKED, GRF_EINVAL,
                "grf_transpose_banded_fill: rec_unit must be GRF_REC_LINE or GRF_REC_PACKED");
    GRF_REQUIRE(((uintptr_t)t_rec & 127) == 0, GRF_EINVAL, "grf_transpose_banded_fill: t_rec must be 128-byte aligned");
    const int64_t nb = cdiv<int64_t>(n_rows, band_width), nbk = nb * n_cols;
    GRF_REQUIRE(workspace_bytes >= grf_transpose_workspace_bytes(nbk), GRF_EINVAL,
                "grf_transpose_banded_fill: workspace too small");
    hipStream_t st = S(stream);
    char *w = (char *)workspace;
    int32_t *cursor = (int32_t *)w;
    float *row_max = (float *)(w + tr_align((size_t)nbk * 4));                                // n_rows <= nbk
    double *row_sum = (double *)(w + 2 * tr_align((size_t)nbk * 4));                         // n_rows <= nbk + 1
    const uint2 *desc = reinterpret_cast<const uint2 *>(t_desc);
    GRF_CHECK_HIP(hipMemsetAsync(cursor, 0, (size_t)nbk * sizeof(int32_t), st));
    GRF_CHECK_HIP(hipMemsetAsync(t_maxabs, 0, sizeof(float), st));
    if (n_rows > 0) {
        GRF_REQUIRE_GRID(cdiv<int64_t>(n_rows, 4), 256, "tr_fill_kernel");
        tr_fill_kernel<<<(unsigned)cdiv<int64_t>(n_rows, 4), 256, 0, st>>>(
            n_rows, n_cols, band_width, ptr, idx, val, desc, cursor, (unsigned char *)t_rec, rec_unit,
            reinterpret_cast<unsigned int *>(t_maxabs), row_max, row_sum);
        GRF_CHECK_LAUNCH("tr_fill_kernel");
        GRF_REQUIRE_GRID(cdiv<int64_t>(n_rows, 256), 256, "tr_rowshift_kernel");
        tr_rowshift_kernel<<<(unsigned)cdiv<int64_t>(n_rows, 256), 256, 0, st>>>(n_rows, row_max, row_sum, t_maxabs,
                                                                                t_rowshift);
        GRF_CHECK_LAUNCH("tr_rowshift_kernel");
    }
    GRF_REQUIRE_GRID(cdiv<int64_t>(nbk, 256), 256, "tr_pad_fill_kernel");
    tr_pad_fill_kernel<<<(unsigned)cdiv<int64_t>(nbk, 256), 256, 0, st>>>(nbk, desc, cursor, (unsigned char *)t_rec,
                                                                          rec_unit);
    GRF_CHECK_LAUNCH("tr_pad_fill_kernel");
    return GRF_OK;
}


size_t grf_transpose_staging_bytes(int64_t n_rows, int64_t n_cols, int64_t band_width, int64_t nnz) {
    if (n_cols <= 0 || band_width <= 0) return 0;
    const int64_t nreg = cdiv<int64_t>(n_cols, tr_region_cols(n_rows, n_cols)), nwg = cdiv<int64_t>(n_rows, kBinRows);
    return tr_align((size_t)nnz * 8) + tr_align((size_t)std::max<int64_t>(n_rows, 1) * 8) +
           tr_align((size_t)std::max<int64_t>(nwg, 1) * (nreg + 1) * 4) + tr_align((size_t)std::max<int64_t>(nwg, 1) * 4);
}

int32_t grf_transpose_banded_fill_staged(int64_t n_rows, int64_t n_cols, int64_t band_width, int32_t rec_unit,
                                         const int64_t *ptr, const int32_t *idx, const float *val,
                                         const uint32_t *t_desc, void *t_rec, int64_t t_rec_bytes, float *t_maxabs,
                                         int32_t *t_rowshift, void *workspace, size_t workspace_bytes, int64_t nnz,
                                         void *staging, size_t staging_bytes, grf_stream_t stream) {
    GRF_REQUIRE(n_rows >= 0 && n_cols > 0 && band_width > 0 && band_width <= 8192 && ptr && idx && val && t_desc &&
                    t_rec && t_maxabs && t_rowshift && t_rec_bytes >= 0 && staging,
                GRF_EINVAL, "grf_transpose_banded_fill_staged: bad arguments");
    GRF_REQUIRE(rec_unit == GRF_REC_LINE || rec_unit == GRF_REC_PACKED, GRF_EINVAL,
                "grf_transpose_banded_fill_staged: rec_unit must be GRF_REC_LINE or GRF_REC_PACKED");
    GRF_REQUIRE(band_width % 64 == 0, GRF_EUNSUPPORTED,
                "grf_transpose_banded_fill_staged: band_width must be a multiple of 64");
    GRF_REQUIRE(((uintptr_t)t_rec & 127) == 0, GRF_EINVAL,
                "grf_transpose_banded_fill_staged: t_rec must be 128-byte aligned");
    const int64_t nb = cdiv<int64_t>(n_rows, band_width), nbk = nb * n_cols;
    const int32_t cr = tr_region_cols(n_rows, n_cols);
    GRF_REQUIRE(cr <= 65536, GRF_EUNSUPPORTED, "grf_transpose_banded_fill_staged: too many columns");
    const int32_t nreg = (int32_t)cdiv<int64_t>(n_cols, cr);
    GRF_REQUIRE(workspace_bytes >= grf_transpose_workspace_bytes(nbk), GRF_EINVAL,
                "grf_transpose_banded_fill_staged: workspace too small");
    GRF_REQUIRE(nnz >= 0 && staging_bytes >= grf_transpose_staging_bytes(n_rows, n_cols, band_width, nnz), GRF_EINVAL,
                "grf_transpose_banded_fill_staged: staging too small (%zu < %zu)", staging_bytes,
                grf_transpose_staging_bytes(n_rows, n_cols, band_width, nnz));
    hipStream_t st = S(stream);
    // workspace: [cnt: bucket counts from the plan | row_max | ent_off (nbk + 1) | scan scratch]
    char *w = (char *)workspace;
    int32_t *cnt = (int32_t *)w;
    float *row_max = (float *)(w + tr_align((size_t)nbk * 4));
    int64_t *ent_off = (int64_t *)(w + 2 * tr_align((size_t)nbk * 4));
    void *scan_ws = w + 2 * tr_align((size_t)nbk * 4) + tr_align((size_t)(nbk + 1) * 8);
    char *sg = (char *)staging;
    uint2 *ent = (uint2 *)sg;
    double *row_sum = (double *)(sg + tr_align((size_t)nnz * 8));
    int32_t *tab = (int32_t *)(sg + tr_align((size_t)nnz * 8) + tr_align((size_t)std::max<int64_t>(n_rows, 1) * 8));
    const int64_t nwg = cdiv<int64_t>(n_rows, kBinRows);
    float *wg_max = (float *)((char *)tab + tr_align((size_t)std::max<int64_t>(nwg, 1) * (nreg + 1) * 4));
    const uint2 *desc = reinterpret_cast<const uint2 *>(t_desc);
    int32_t rc = scan_counts_i32(nbk, cnt, ent_off, scan_ws, scan_ws_bytes(nbk), st);  // entries before each bucket
    if (rc != GRF_OK) return rc;
    GRF_CHECK_HIP(hipMemsetAsync(t_maxabs, 0, sizeof(float), st));
    if (n_rows == 0) return GRF_OK;
    const size_t lds1 = (size_t)kBinCap * 8 + (size_t)nreg * 4 + (kBinRows + 1 + 8) * 4;
    GRF_REQUIRE_GRID(nwg, 256, "tr_bin_kernel");
    tr_bin_kernel<<<(unsigned)nwg, 256, lds1, st>>>(n_rows, n_cols, band_width, cr, nreg, ptr, idx, val, ent, tab,
                                                    wg_max, row_max, row_sum);
    GRF_CHECK_LAUNCH("tr_bin_kernel");
    tr_maxabs_kernel<<<1, 1024, 0, st>>>(nwg, wg_max, t_maxabs);
    GRF_CHECK_LAUNCH("tr_maxabs_kernel");
    GRF_REQUIRE_GRID(cdiv<int64_t>(n_rows, 256), 256, "tr_rowshift_kernel");
    tr_rowshift_kernel<<<(unsigned)cdiv<int64_t>(n_rows, 256), 256, 0, st>>>(n_rows, row_max, row_sum, t_maxabs,
                                                                            t_rowshift);
    GRF_CHECK_LAUNCH("tr_rowshift_kernel");
    GRF_CHECK_HIP(hipMemsetAsync(cnt, 0, (size_t)nbk * sizeof(int32_t), st));  // fallback cursors
    const int64_t n_regions = nb * nreg;
    const size_t lds2 = (size_t)8 * cr + kPlaceCap;
    GRF_REQUIRE_GRID(n_regions, 256, "tr_place_kernel");
    tr_place_kernel<<<(unsigned)n_regions, 256, lds2, st>>>(n_rows, n_cols, band_width, cr, nreg, ptr, desc, ent_off,
                                                            ent, tab, cnt, (unsigned char *)t_rec, rec_unit);
    GRF_CHECK_LAUNCH("tr_place_kernel");
    return GRF_OK;
}

size_t grf_transpose_self_workspace_bytes(int64_t n_rows, int64_t n_cols, int64_t band_width) {
    if (n_cols <= 0 || band_width <= 0) return 16;
    const int64_t nb = cdiv<int64_t>(std::max<int64_t>(n_rows, 1), band_width);
    const int64_t n_regions = nb * cdiv<int64_t>(n_cols, tr_region_cols(n_rows, n_cols));
    return tr_align((size_t)std::max<int64_t>(n_rows, 1) * 4) + 2 * tr_align((size_t)(n_regions + 1) * 8) +
           tr_align((size_t)nb * n_cols * 4) + scan_ws_bytes(n_regions);
}

int64_t grf_transpose_self_units_bound(int64_t n_rows, int64_t n_cols, int64_t band_width, int32_t rec_unit,
                                       int64_t nnz) {
    if (n_cols <= 0 || band_width <= 0) return 1;
    const int64_t nb = cdiv<int64_t>(std::max<int64_t>(n_rows, 1), band_width), nbk = nb * n_cols;
    const int64_t n_regions = nb * cdiv<int64_t>(n_cols, tr_region_cols(n_rows, n_cols));
    // the sum of tr_region_units over the regions, for any split of nnz entries
    if (rec_unit == GRF_REC_PACKED) return (nnz + nbk) / 2 + n_regions + 1;
    // GRF_REC_SLOT: 32-byte units covering the slots and the overflow pairs (at most the packed bound)
    if (rec_unit == GRF_REC_SLOT) return nbk + cdiv<int64_t>(kPairBytes * ((nnz + nbk) / 2 + n_regions + 1), 32);
    return (6 * (nnz + nbk)) / rec_unit + nbk + 2 * n_regions + 1;
}

int32_t grf_transpose_banded_self(int64_t n_rows, int64_t n_cols, int64_t band_width, int32_t rec_unit,
                                  const int64_t *ptr, const int32_t *idx, const float *val, uint32_t *t_desc,
                                  void *t_split, void *t_rec, int64_t t_rec_bytes, float *t_maxabs, int32_t *t_rowshift,
                                  void *workspace, size_t workspace_bytes, int64_t nnz, void *staging,
                                  size_t staging_bytes, grf_stream_t stream) {
    GRF_REQUIRE(n_rows >= 0 && n_cols > 0 && band_width > 0 && band_width <= 8192 && ptr && idx && val && t_desc &&
                    t_rec && t_maxabs && t_rowshift && t_rec_bytes >= 0 && staging && workspace,
                GRF_EINVAL, "grf_transpose_banded_self: bad arguments");
    GRF_REQUIRE(rec_unit == GRF_REC_LINE || rec_unit == GRF_REC_PACKED || rec_unit == GRF_REC_SLOT, GRF_EINVAL,
                "grf_transpose_banded_self: rec_unit must be GRF_REC_LINE, GRF_REC_PACKED or GRF_REC_SLOT");
    GRF_REQUIRE(rec_unit != GRF_REC_SLOT || !t_split, GRF_EUNSUPPORTED,
                "grf_transpose_banded_self: GRF_REC_SLOT has no sub-band split");
    GRF_REQUIRE(band_width % 64 == 0, GRF_EUNSUPPORTED, "grf_transpose_banded_self: band_width must be a multiple of 64");
    GRF_REQUIRE(((uintptr_t)t_rec & 127) == 0, GRF_EINVAL, "grf_transpose_banded_self: t_rec must be 128-byte aligned");
    const int64_t nb = cdiv<int64_t>(n_rows, band_width), nbk = nb * n_cols;
    const int32_t cr = tr_region_cols(n_rows, n_cols);
    GRF_REQUIRE(cr <= 65536, GRF_EUNSUPPORTED, "grf_transpose_banded_self: too many columns");
    const int32_t nreg = (int32_t)cdiv<int64_t>(n_cols, cr);
    GRF_REQUIRE(workspace_bytes >= grf_transpose_self_workspace_bytes(n_rows, n_cols, band_width), GRF_EINVAL,
                "grf_transpose_banded_self: workspace too small");
    GRF_REQUIRE(nnz >= 0 && staging_bytes >= grf_transpose_staging_bytes(n_rows, n_cols, band_width, nnz), GRF_EINVAL,
                "grf_transpose_banded_self: staging too small");
    GRF_REQUIRE(t_rec_bytes >= grf_transpose_self_units_bound(n_rows, n_cols, band_width, rec_unit, nnz) * rec_unit,
                GRF_ECAPACITY, "grf_transpose_banded_self: t_rec too small for the region slabs");
    hipStream_t st = S(stream);
    const int64_t n_regions = nb * nreg;
    char *w = (char *)workspace;
    float *row_max = (float *)w;
    w += tr_align((size_t)std::max<int64_t>(n_rows, 1) * 4);
    int64_t *region_units = (int64_t *)w;
    w += tr_align((size_t)(n_regions + 1) * 8);
    int64_t *region_base = (int64_t *)w;
    w += tr_align((size_t)(n_regions + 1) * 8);
    int32_t *gcur = (int32_t *)w;  // (fallback cursors of oversized regions; zeroed by their owners)
    w += tr_align((size_t)nbk * 4);
    void *scan_ws = w;
    char *sg = (char *)staging;
    uint2 *ent = (uint2 *)sg;
    double *row_sum = (double *)(sg + tr_align((size_t)nnz * 8));
    int32_t *tab = (int32_t *)(sg + tr_align((size_t)nnz * 8) + tr_align((size_t)std::max<int64_t>(n_rows, 1) * 8));
    const int64_t nwg = cdiv<int64_t>(n_rows, kBinRows);
    float *wg_max = (float *)((char *)tab + tr_align((size_t)std::max<int64_t>(nwg, 1) * (nreg + 1) * 4));
    uint2 *desc = reinterpret_cast<uint2 *>(t_desc);
    GRF_CHECK_HIP(hipMemsetAsync(t_maxabs, 0, sizeof(float), st));
    if (n_rows == 0) {
        GRF_CHECK_HIP(hipMemsetAsync(t_desc, 0, (size_t)(nbk + 1) * 8, st));
        return GRF_OK;
    }
    GRF_REQUIRE(!t_split || band_width <= 8192, GRF_EUNSUPPORTED,
                "grf_transpose_banded_self: the sub-band split needs band_width <= 8192 (u16 offsets)");
    GRF_REQUIRE(((uintptr_t)t_split & 15) == 0, GRF_EINVAL, "grf_transpose_banded_self: t_split must be 16-byte aligned");
    const size_t lds1 = (size_t)kBinCap * 8 + (size_t)nreg * 4 + (kBinRows + 1 + 8) * 4;
    GRF_REQUIRE_GRID(nwg, 256, "tr_bin_kernel");
    tr_bin_kernel<<<(unsigned)nwg, 256, lds1, st>>>(n_rows, n_cols, band_width, cr, nreg, ptr, idx, val, ent, tab,
                                                    wg_max, row_max, row_sum);
    GRF_CHECK_LAUNCH("tr_bin_kernel");
    tr_maxabs_kernel<<<1, 1024, 0, st>>>(nwg, wg_max, t_maxabs);
    GRF_CHECK_LAUNCH("tr_maxabs_kernel");
    GRF_REQUIRE_GRID(cdiv<int64_t>(n_rows, 256), 256, "tr_rowshift_kernel");
    tr_rowshift_kernel<<<(unsigned)cdiv<int64_t>(n_rows, 256), 256, 0, st>>>(n_rows, row_max, row_sum, t_maxabs,
                                                                            t_rowshift);
    GRF_CHECK_LAUNCH("tr_rowshift_kernel");
    GRF_REQUIRE_GRID(cdiv<int64_t>(n_regions, 4), 256, "tr_region_units_kernel");
    tr_region_units_kernel<<<(unsigned)cdiv<int64_t>(n_regions, 4), 256, 0, st>>>(n_rows, n_cols, band_width, cr, nreg,
                                                                                 n_regions, tab,
                                                                                 rec_unit == GRF_REC_SLOT ? kPairBytes : rec_unit,
                                                                                 region_units);
    GRF_CHECK_LAUNCH("tr_region_units_kernel");
    int32_t rc = scan_exclusive<int64_t>(n_regions, region_units, ScanIdentity{},
                                         RegionBaseOut{region_base, desc + nbk}, (int64_t *)scan_ws, st);
    if (rc != GRF_OK) return rc;
    GRF_REQUIRE_GRID(n_regions, 256, "tr_place_self_kernel");
    if (rec_unit == GRF_REC_SLOT) {
        const size_t lds2 = (size_t)8 * cr + 32 + kPlaceCap;
        tr_place_slots_kernel<<<(unsigned)n_regions, 256, lds2, st>>>(n_rows, n_cols, band_width, cr, nreg, nbk, ptr,
                                                                       region_base, ent, tab, gcur,
                                                                       (unsigned char *)t_rec);
        GRF_CHECK_LAUNCH("tr_place_slots_kernel");
        return GRF_OK;
    }
    if (t_split) {
        const size_t lds2 = (size_t)4 * cr * (kSub + 1) + 32 + kPlaceCap;
        tr_place_self_kernel<true><<<(unsigned)n_regions, 256, lds2, st>>>(
            n_rows, n_cols, band_width, cr, nreg, ptr, region_base, ent, tab, gcur, desc, (uint4 *)t_split,
            (unsigned char *)t_rec, rec_unit);
    } else {
        const size_t lds2 = (size_t)8 * cr + 32 + kPlaceCap;
        tr_place_self_kernel<false><<<(unsigned)n_regions, 256, lds2, st>>>(
            n_rows, n_cols, band_width, cr, nreg, ptr, region_base, ent, tab, gcur, desc, nullptr,
            (unsigned char *)t_rec, rec_unit);
    }
    GRF_CHECK_LAUNCH("tr_place_self_kernel");
    return GRF_OK;
}

size_t grf_phi_row_shifts_workspace_bytes(int64_t n_rows) {
    const int64_t n = std::max<int64_t>(n_rows, 1);
    return tr_align((size_t)n * 4) + tr_align((size_t)n * 8) + tr_align((size_t)cdiv<int64_t>(n, 4) * 4);
}

static void row_stats_layout(void *workspace, int64_t n_rows, float *&row_max, double *&row_sum, float *&wg_max) {
    char *w = (char *)workspace;
    row_max = (float *)w;
    row_sum = (double *)(w + tr_align((size_t)n_rows * 4));
    wg_max = (float *)(w + tr_align((size_t)n_rows * 4) + tr_align((size_t)n_rows * 8));
}

int32_t grf_compact_rows_stats(int64_t n_rows, int64_t cap, const int32_t *cnt, const int64_t *out_ptr,
                               const int32_t *in_idx, const double *in_val, const float *in_val32, int32_t *out_idx,
                               double *out_val, float *out_val32, void *stats, size_t stats_bytes,
                               grf_stream_t stream) {
    GRF_REQUIRE(n_rows >= 0 && cap >= 0 && cnt && out_ptr && in_idx && out_idx && in_val32 && out_val32 && stats,
                GRF_EINVAL, "grf_compact_rows_stats: bad arguments");
    GRF_REQUIRE(!out_val || in_val, GRF_EINVAL, "grf_compact_rows_stats: out_val needs in_val");
    GRF_REQUIRE(stats_bytes >= grf_phi_row_shifts_workspace_bytes(n_rows), GRF_EINVAL,
                "grf_compact_rows_stats: stats buffer too small");
    if (n_rows == 0) return GRF_OK;
    float *row_max, *wg_max;
    double *row_sum;
    row_stats_layout(stats, n_rows, row_max, row_sum, wg_max);
    const int64_t nwg = cdiv<int64_t>(n_rows, 4 * kCompactRows);
    GRF_REQUIRE_GRID(nwg, 256, "compact_rows_kernel<stats>");
    compact_rows_kernel<true><<<(unsigned)nwg, 256, 0, S(stream)>>>(n_rows, cap, cnt, out_ptr, in_idx, in_val, in_val32,
                                                                   out_idx, out_val, out_val32, row_max, row_sum, wg_max);
    GRF_CHECK_LAUNCH("compact_rows_kernel<stats>");
    return GRF_OK;
}

int32_t grf_phi_row_shifts_stats(int64_t n_rows, const void *stats, float *maxabs, int32_t *row_shift,
                                 grf_stream_t stream) {
    GRF_REQUIRE(n_rows >= 0 && stats && maxabs && row_shift, GRF_EINVAL, "grf_phi_row_shifts_stats: bad arguments");
    hipStream_t st = S(stream);
    GRF_CHECK_HIP(hipMemsetAsync(maxabs, 0, sizeof(float), st));
    if (n_rows == 0) return GRF_OK;
    float *row_max, *wg_max;
    double *row_sum;
    row_stats_layout(const_cast<void *>(stats), n_rows, row_max, row_sum, wg_max);
    const int64_t nwg = cdiv<int64_t>(n_rows, 4);
    tr_maxabs_kernel<<<1, 1024, 0, st>>>(nwg, wg_max, maxabs);
    GRF_CHECK_LAUNCH("tr_maxabs_kernel");
    tr_rowshift_kernel<<<(unsigned)cdiv<int64_t>(n_rows, 256), 256, 0, st>>>(n_rows, row_max, row_sum, maxabs,
                                                                            row_shift);
    GRF_CHECK_LAUNCH("tr_rowshift_kernel");
    return GRF_OK;
}

int32_t grf_phi_row_shifts_padded(int64_t n_rows, int64_t cap, const int32_t *cnt, const float *val, float *maxabs,
                                  int32_t *row_shift, void *workspace, size_t workspace_bytes, grf_stream_t stream) {
    GRF_REQUIRE(n_rows >= 0 && cap >= 1 && cnt && val && maxabs && row_shift && workspace, GRF_EINVAL,
                "grf_phi_row_shifts_padded: bad arguments");
    GRF_REQUIRE(workspace_bytes >= grf_phi_row_shifts_workspace_bytes(n_rows), GRF_EINVAL,
                "grf_phi_row_shifts_padded: workspace too small");
    hipStream_t st = S(stream);
    GRF_CHECK_HIP(hipMemsetAsync(maxabs, 0, sizeof(float), st));
    if (n_rows == 0) return GRF_OK;
    float *row_max, *wg_max;
    double *row_sum;
    row_stats_layout(workspace, n_rows, row_max, row_sum, wg_max);
    const int64_t nwg = cdiv<int64_t>(n_rows, 4);
    GRF_REQUIRE_GRID(nwg, 256, "phi_row_stats_kernel");
    phi_row_stats_kernel<<<(unsigned)nwg, 256, 0, st>>>(n_rows, nullptr, val, wg_max, row_max, row_sum, cap, cnt);
    GRF_CHECK_LAUNCH("phi_row_stats_kernel");
    tr_maxabs_kernel<<<1, 1024, 0, st>>>(nwg, wg_max, maxabs);
    GRF_CHECK_LAUNCH("tr_maxabs_kernel");
    tr_rowshift_kernel<<<(unsigned)cdiv<int64_t>(n_rows, 256), 256, 0, st>>>(n_rows, row_max, row_sum, maxabs,
                                                                            row_shift);
    GRF_CHECK_LAUNCH("tr_rowshift_kernel");
    return GRF_OK;
}

int32_t grf_phi_row_shifts(int64_t n_rows, const int64_t *ptr, const float *val, float *maxabs, int32_t *row_shift,
                           void *workspace, size_t workspace_bytes, grf_stream_t stream) {
    GRF_REQUIRE(n_rows >= 0 && ptr && val && maxabs && row_shift && workspace, GRF_EINVAL,
                "grf_phi_row_shifts: bad arguments");
    GRF_REQUIRE(workspace_bytes >= grf_phi_row_shifts_workspace_bytes(n_rows), GRF_EINVAL,
                "grf_phi_row_shifts: workspace too small");
    hipStream_t st = S(stream);
    GRF_CHECK_HIP(hipMemsetAsync(maxabs, 0, sizeof(float), st));
    if (n_rows == 0) return GRF_OK;
    char *w = (char *)workspace;
    float *row_max = (float *)w;
    double *row_sum = (double *)(w + tr_align((size_t)n_rows * 4));
    float *wg_max = (float *)(w + tr_align((size_t)n_rows * 4) + tr_align((size_t)n_rows * 8));
    const int64_t nwg = cdiv<int64_t>(n_rows, 4);
    GRF_REQUIRE_GRID(nwg, 256, "phi_row_stats_kernel");
    phi_row_stats_kernel<<<(unsigned)nwg, 256, 0, st>>>(n_rows, ptr, val, wg_max, row_max, row_sum);
    GRF_CHECK_LAUNCH("phi_row_stats_kernel");
    tr_maxabs_kernel<<<1, 1024, 0, st>>>(nwg, wg_max, maxabs);
    GRF_CHECK_LAUNCH("tr_maxabs_kernel");
    tr_rowshift_kernel<<<(unsigned)cdiv<int64_t>(n_rows, 256), 256, 0, st>>>(n_rows, row_max, row_sum, maxabs,
                                                                            row_shift);
    GRF_CHECK_LAUNCH("tr_rowshift_kernel");
    return GRF_OK;
}

}  // extern "C"
