// grf_cg.hip -- K.v = Phi (Phi^T V) and the pathwise-conditioning CG solve on gfx950.
//
// The step after the GRF path: the reference's
// SparseGraphGP.predict (models/sparse_grf_model.py:21-45) solves
// (K_tt + s2 I) V = B with linear_operator's linear_cg (gpytorch 1.11 ->
// linear_operator 0.5, utils/linear_cg.py, no preconditioner) for a batch of
// right-hand sides.  Here K is never formed: every matvec is two CSR SpMMs,
//   W = Phi_t^T P   (n_cols x S, over the transposed training rows)
//   Y = Phi_t  W + s2 P
// with S = n_samples columns laid out row-major (one 4*S-byte row per node), so
// a wavefront gathers whole rows: lane c owns column c (S = 64 fills the wave).
//
// Kernels
//   csr_tr_gather / unpack      deterministic CSR transpose of a row subset: the
//                               entries laid out in row order, a stable rocPRIM
//                               radix sort by column -> every column lists its
//                               rows in ascending order.
//   spmm_kernel<SG>             Y = A[row_map] X (+ zc Z); one wave per row, 64/SG
//                               lane groups split the nonzeros, fixed-order sums.
//   cg_* kernels                column reductions (fp64, fixed order, last block
//                               finalises) and the vector updates of linear_cg.
// All CG kernels read a device `done` flag first: once the stopping rule fires
// the rest of the enqueued iterations are no-ops, so the host only polls the
// flag and never serialises the stream per iteration.
#include <rocprim/device/device_radix_sort.hpp>
#include <hip/hip_runtime.h>
#include <math.h>

#include <algorithm>

#include "grf_common.h"

namespace grf {

int32_t scan_counts_i32(int64_t n, const int32_t *cnt, int64_t *out, void *ws, size_t ws_bytes, hipStream_t st);
size_t scan_ws_bytes(int64_t n);

static size_t al256(size_t x) { return (x + 255) & ~(size_t)255; }

// ------------------------------------------------------------ CSR transpose
// (Phi[row_map])^T by a stable radix sort: the selected rows' entries are laid out in row order as
// (key = column, value = {position r, value bits}); a stable LSD sort by column keeps every column's
// positions ascending -- the same CSR the chunked cursor fill gives, without its n_cols x chunks
// count / cursor tables (1.6 GB at C4) and their random atomics.
__global__ __launch_bounds__(256) void csr_tr_len_kernel(int64_t n_sel, const int64_t *ptr, const int32_t *row_map,
                                                         int32_t *len) {
    const int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (r < n_sel) {
        const int64_t row = row_map ? row_map[r] : r;
        len[r] = (int32_t)(ptr[row + 1] - ptr[row]);
    }
}

__global__ __launch_bounds__(256) void csr_tr_gather_kernel(int64_t n_sel, const int64_t *ptr, const int32_t *idx,
                                                            const float *val, const int32_t *row_map,
                                                            const int64_t *off, uint32_t *keys, uint64_t *vals) {
    const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);  // one wave per selected row
    if (r >= n_sel) return;
    const int lane = threadIdx.x & 63;
    const int64_t row = row_map ? row_map[r] : r, b = ptr[row], e = ptr[row + 1], o = off[r];
    for (int64_t q = lane; q < e - b; q += 64) {
        keys[o + q] = (uint32_t)idx[b + q];
        vals[o + q] = ((uint64_t)(uint32_t)r << 32) | __float_as_uint(val[b + q]);
    }
}

// nnz given as an upper bound (no host read of the gathered count): the positions past the gathered
// entries get the key n_cols, so they sort after every column and t_ptr[n_cols] ends at the real count
__global__ __launch_bounds__(256) void csr_tr_pad_kernel(int64_t nnz, int64_t n_sel, const int64_t *off,
                                                         int64_t n_cols, uint32_t *keys) {
    const int64_t total = n_sel > 0 ? off[n_sel] : 0;
    for (int64_t i = total + (int64_t)blockIdx.x * 256 + threadIdx.x; i < nnz; i += (int64_t)gridDim.x * 256)
        keys[i] = (uint32_t)n_cols;
}

// sorted keys -> t_ptr (first position of every column, n_cols + 1 entries) and t_idx / t_val
__global__ __launch_bounds__(256) void csr_tr_unpack_kernel(int64_t nnz, int64_t n_cols, const uint32_t *keys,
                                                            const uint64_t *vals, int64_t *t_ptr, int32_t *t_idx,
                                                            float *t_val) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i > nnz) return;
    const int64_t k = i < nnz ? (int64_t)keys[i] : n_cols;             // (past the end: column n_cols)
    const int64_t kp = i > 0 ? (int64_t)keys[i - 1] : -1;
    for (int64_t c = kp + 1; c <= k; ++c) t_ptr[c] = i;                 // columns (kp, k] start at i
    if (i < nnz) {
        const uint64_t v = vals[i];
        t_idx[i] = (int32_t)(v >> 32);
        t_val[i] = __uint_as_float((uint32_t)v);
    }
}

static unsigned key_bits(int64_t n_cols) {
    unsigned b = 1;
    while (b < 32 && (int64_t(1) << b) <= n_cols) ++b;
    return b;
}

static size_t csr_tr_sort_temp_bytes(int64_t nnz, int64_t n_cols) {
    size_t bytes = 0;
    (void)rocprim::radix_sort_pairs(nullptr, bytes, (const uint32_t *)nullptr, (uint32_t *)nullptr,
                                    (const uint64_t *)nullptr, (uint64_t *)nullptr, (size_t)std::max<int64_t>(nnz, 1),
                                    0u, key_bits(n_cols));
    return bytes;
}


// ------------------------------------------------------------------- SpMM
// Y[r, c] = sum_e val[e] X[idx[e], c] (+ zc Z[r, c]) over row row_map[r] of A.
// SG lanes per column group; the 64/SG groups take the nonzeros j = g, g + G, ...
// of each 64-batch and are summed by a fixed xor tree.  T = type of the dense blocks and
// of the accumulation (float: the reference's precision; double: A's fp32 values widened).
//
// Column tiles: a gathered X row comes from the Infinity Cache at ~8.6 TB/s chip-wide but
// from the XCD's L2 at ~17 TB/s (MI355X_MICROARCH.md, "Indexed rows").  With `seg` the
// launch covers only the entries whose column lies in tile `tile` (X rows
// [tile * tw, (tile + 1) * tw), a slice that fits every XCD's L2): row r's entries of that
// tile are the contiguous range [seg[tile][r], seg[tile + 1][r]) of its (column-sorted) CSR
// row.  Tiles run as successive launches; `accumulate` adds to the Y of the tiles before.
template <int SG, typename T>
__global__ __launch_bounds__(256) void spmm_kernel(int64_t n_out, const int64_t *ptr, const int32_t *idx,
                                                   const float *val, const int32_t *row_map, const T *X,
                                                   int64_t ldx, int32_t S, T *Y, int64_t ldy, const T *Z,
                                                   int64_t ldz, T zc, const int32_t *done, const int64_t *seg,
                                                   int32_t tile, int32_t accumulate) {
    if (done && __builtin_nontemporal_load(done)) return;
    constexpr int G = 64 / SG;
    const int lane = threadIdx.x & 63;
    const int g = lane / SG, cl = lane % SG;
    const int64_t n_waves = (int64_t)gridDim.x * 4;
    for (int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); r < n_out; r += n_waves) {
        int64_t e0, e1;
        if (seg) {
            e0 = uniform(seg[(int64_t)tile * n_out + r]);
            e1 = uniform(seg[(int64_t)(tile + 1) * n_out + r]);
        } else {
            const int64_t row = uniform(row_map ? (int64_t)row_map[r] : r);
            e0 = uniform(ptr[row]);
            e1 = uniform(ptr[row + 1]);
        }
        for (int c0 = 0; c0 < S; c0 += SG) {
            const int c = c0 + cl;
            const bool cok = c < S;
            const T *Xc = X + (cok ? c : 0);
            T acc = T(0);
            for (int64_t eb = e0; eb < e1; eb += 64) {
                const int64_t e = eb + lane;
                const int32_t k_l = e < e1 ? __builtin_nontemporal_load(&idx[e]) : 0;
                const float v_l = e < e1 ? __builtin_nontemporal_load(&val[e]) : 0.f;
                const int cnt = (int)min<int64_t>(64, e1 - eb);
                if constexpr (SG == 64) {
                    int j = 0;
                    for (; j + 8 <= cnt; j += 8) {
                        T x[8], v[8];
#pragma unroll
                        for (int u = 0; u < 8; ++u) {
                            const int32_t k = __builtin_amdgcn_readlane(k_l, j + u);
                            v[u] = (T)__builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int32_t, v_l), j + u));
                            x[u] = cok ? Xc[(int64_t)k * ldx] : T(0);
                        }
#pragma unroll
                        for (int u = 0; u < 8; ++u) acc = fma(v[u], x[u], acc);
                    }
                    for (; j < cnt; ++j) {
                        const int32_t k = __builtin_amdgcn_readlane(k_l, j);
                        const T v = (T)__builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int32_t, v_l), j));
                        acc = fma(v, cok ? Xc[(int64_t)k * ldx] : T(0), acc);
                    }
                } else {
                    // every lane runs the same trip count (ceil(cnt / G)) so all lanes take part
                    // in the shuffles; lanes j >= cnt hold v = 0 and add nothing
                    const int n_u = (cnt + G - 1) / G;
                    int u = 0;
                    for (; u + 4 <= n_u; u += 4) {
                        T x[4], v[4];
#pragma unroll
                        for (int uu = 0; uu < 4; ++uu) {
                            const int j = g + (u + uu) * G;
                            const int32_t k = __shfl(k_l, j);
                            v[uu] = (T)__shfl(v_l, j);
                            x[uu] = (cok && j < cnt) ? Xc[(int64_t)k * ldx] : T(0);
                        }
#pragma unroll
                        for (int uu = 0; uu < 4; ++uu) acc = fma(v[uu], x[uu], acc);
                    }
                    for (; u < n_u; ++u) {
                        const int j = g + u * G;
                        const int32_t k = __shfl(k_l, j);
                        const T v = (T)__shfl(v_l, j);
                        acc = fma(v, (cok && j < cnt) ? Xc[(int64_t)k * ldx] : T(0), acc);
                    }
                }
            }
#pragma unroll
            for (int off = SG; off < 64; off <<= 1) acc += __shfl_xor(acc, off);
            if (g == 0 && cok) {
                T y = acc;
                if (accumulate) y = Y[r * ldy + c] + y;
                if (Z) y += zc * Z[r * ldz + c];
                Y[r * ldy + c] = y;
            }
        }
    }
}

template <int SG, typename T>
static int32_t spmm_launch(int64_t n_out, const int64_t *ptr, const int32_t *idx, const float *val,
                           const int32_t *row_map, const T *X, int64_t ldx, int32_t S, T *Y, int64_t ldy,
                           const T *Z, int64_t ldz, T zc, const int32_t *done, const int64_t *seg,
                           int32_t n_tiles, hipStream_t st) {
    const int64_t blocks = std::min<int64_t>(cdiv<int64_t>(n_out, 4), 1 << 16);
    if (!seg) {
        spmm_kernel<SG, T><<<(unsigned)blocks, 256, 0, st>>>(n_out, ptr, idx, val, row_map, X, ldx, S, Y, ldy, Z,
                                                             ldz, zc, done, nullptr, 0, 0);
        GRF_CHECK_LAUNCH("spmm_kernel");
        return GRF_OK;
    }
    for (int32_t t = 0; t < n_tiles; ++t) {
        const bool last = t == n_tiles - 1;
        spmm_kernel<SG, T><<<(unsigned)blocks, 256, 0, st>>>(n_out, ptr, idx, val, row_map, X, ldx, S, Y, ldy,
                                                             last ? Z : nullptr, ldz, zc, done, seg, t, t > 0);
        GRF_CHECK_LAUNCH("spmm_kernel");
    }
    return GRF_OK;
}

template <typename T>
static int32_t spmm_dispatch(int64_t n_out, const int64_t *ptr, const int32_t *idx, const float *val,
                             const int32_t *row_map, const T *X, int64_t ldx, int32_t S, T *Y, int64_t ldy,
                             const T *Z, int64_t ldz, T zc, const int32_t *done, hipStream_t st,
                             const int64_t *seg = nullptr, int32_t n_tiles = 1) {
    if (n_out == 0 || S == 0) return GRF_OK;
    if (n_tiles <= 1) seg = nullptr;
#define GRF_SPMM(SGV) spmm_launch<SGV, T>(n_out, ptr, idx, val, row_map, X, ldx, S, Y, ldy, Z, ldz, zc, done, seg, n_tiles, st)
    if (S >= 48) return GRF_SPMM(64);
    if (S >= 12) return GRF_SPMM(16);
    if (S >= 3) return GRF_SPMM(4);
    return GRF_SPMM(1);
#undef GRF_SPMM
}

// ---- column-tile plan: seg[t * n_out + r] = first entry of row r with column >= t * tw
// (t = 0..n_tiles; seg[n_tiles][r] = row end).  One wave per output row, no atomics.
__global__ __launch_bounds__(256) void spmm_plan_kernel(int64_t n_out, const int64_t *ptr, const int32_t *idx,
                                                        const int32_t *row_map, int32_t tw, int32_t n_tiles,
                                                        int64_t *seg) {
    const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (r >= n_out) return;
    const int lane = threadIdx.x & 63;
    const int64_t row = row_map ? (int64_t)row_map[r] : r;
    const int64_t s = ptr[row], e = ptr[row + 1];
    for (int64_t i = s + lane; i < e; i += 64) {
        const int32_t tc = idx[i] / tw;
        const int32_t tp = i > s ? idx[i - 1] / tw : -1;
        for (int32_t t = tp + 1; t <= tc; ++t) seg[(int64_t)t * n_out + r] = i;
    }
    const int32_t last = e > s ? idx[e - 1] / tw : -1;
    for (int32_t t = last + 1 + lane; t <= n_tiles; t += 64) seg[(int64_t)t * n_out + r] = e;
}

static int64_t spmm_tile_bytes() {
    static int64_t v = [] {
        const char *e = getenv("GRF_SPMM_TILE_BYTES");
        return e ? std::max<int64_t>(0, atoll(e)) : (int64_t)(8 << 20);
    }();
    return v;
}

// tile width (X rows per tile) for S columns of elem bytes: a power of two, 0 = untiled.
// Budget 8 MiB -> X tiles of <= 4 MiB (one XCD L2).  Measured at C4 (CG iteration, S = 64):
// fp32 1.63 ms untiled -> 1.36 ms; fp64 3.39 -> 2.25 ms (2 MiB tiles: 1.45 / 2.18 ms;
// 1 MiB: 1.72 / 2.82 ms -- per-tile overheads; 8 MiB: 1.51 / 2.89 ms -- spills past L2).
// At most 16 tiles: every tile launch visits every output row, so with many tiles a sparse row
// has ~1 entry per tile (C5, N = 1M, S = 64 fp64: 123 L2-sized tiles took 40.9 ms per CG
// iteration, 8 tiles of 64 MiB 19.8 ms, untiled 20.1 ms).
static int32_t spmm_tile_rows(int64_t n_in, int32_t S, size_t elem) {
    const int64_t tb = spmm_tile_bytes();
    if (tb <= 0) return 0;
    int64_t tw = 64;
    while (tw * 2 * S * (int64_t)elem <= tb) tw *= 2;
    while (cdiv<int64_t>(n_in, tw) > 16) tw *= 2;
    return tw >= n_in ? 0 : (int32_t)tw;
}

static int32_t spmm_plan(int64_t n_out, const int64_t *ptr, const int32_t *idx, const int32_t *row_map, int32_t tw,
                         int32_t n_tiles, int64_t *seg, hipStream_t st) {
    if (n_out == 0) return GRF_OK;
    GRF_REQUIRE_GRID(cdiv<int64_t>(n_out, 4), 256, "spmm_plan_kernel");
    spmm_plan_kernel<<<(unsigned)cdiv<int64_t>(n_out, 4), 256, 0, st>>>(n_out, ptr, idx, row_map, tw, n_tiles, seg);
    GRF_CHECK_LAUNCH("spmm_plan_kernel");
    return GRF_OK;
}

// --------------------------------------------------------------------- CG
constexpr int kMaxRhs = 256;        // columns per solve (4 per lane)
constexpr int kRedBlocks = 256;     // blocks of the reduction kernels
constexpr double kCgEps = 1e-10;    // linear_cg(eps=1e-10)
constexpr double kStopAfter = 1e-10;  // linear_cg(stop_updating_after=1e-10)

struct CgState {
    double *rhs_norm, *rr, *alpha, *beta, *rnorm, *part;
    int32_t *rhs_zero, *conv;
    uint32_t *ticket;
    int32_t *iters, *done;
};

enum CgFinal { kFinNorm = 0, kFinInit = 1, kFinAlpha = 2, kFinUpdate = 3 };

// Per-column sums of f(row, c) over the rows: wave-per-row partials -> LDS -> one fp64
// partial per (block, column); the last block to finish sums the partials in block order
// and finalises the column state.  f is folded into the callers below.
struct ColReduce {
    double acc[4];
    __device__ void zero() {
#pragma unroll
        for (int i = 0; i < 4; ++i) acc[i] = 0.0;
    }
};

// finalisation of one column (called by one thread per column in the last block); the
// scalars are rounded to T like linear_cg's (float for the reference's precision)
template <typename T>
__device__ inline void cg_final_column(int fin, int c, double s, const CgState &st, double *lds_norm, int *lds_conv) {
    if (fin == kFinNorm) {
        double nrm = (double)(T)sqrt(s);  // rhs.norm(2, dim=-2)
        const int zero = nrm < kCgEps;
        st.rhs_zero[c] = zero;
        st.rhs_norm[c] = zero ? 1.0 : nrm;
    } else if (fin == kFinInit) {
        st.rr[c] = s;
        const double nrm = st.rhs_zero[c] ? 0.0 : sqrt(s);
        st.rnorm[c] = nrm;
        const int cv = sqrt(s) < kStopAfter;  // (the initial check does not mask zero rhs)
        st.conv[c] = cv;
        lds_conv[c] = cv;
    } else if (fin == kFinAlpha) {
        double a;
        if (s < kCgEps) a = 0.0;
        else a = st.rr[c] / s;
        if (st.conv[c]) a = 0.0;
        st.alpha[c] = (double)(T)a;
    } else {
        const double old = st.rr[c];
        const double b = old < kCgEps ? 0.0 : s / old;
        st.beta[c] = (double)(T)b;
        st.rr[c] = s;
        const double nrm = st.rhs_zero[c] ? 0.0 : sqrt(s);
        st.rnorm[c] = nrm;
        st.conv[c] = nrm < kStopAfter;
        lds_norm[c] = nrm;
    }
}

template <int kOp, typename T>
__device__ inline void cg_row_op(int64_t r, int c, int32_t S, T *R, T *P, T *Y, T *X, const T *B, int64_t ldb,
                                 const CgState &st, double &acc) {
    const int64_t o = r * S + c;
    if constexpr (kOp == kFinNorm) {
        const double b = B[r * ldb + c];
        acc += b * b;
    } else if constexpr (kOp == kFinInit) {
        const T b = B[r * ldb + c] / (T)st.rhs_norm[c];
        R[o] = b;
        P[o] = b;
        X[o] = 0.f;
        acc += (double)b * b;
    } else if constexpr (kOp == kFinAlpha) {
        acc += (double)P[o] * Y[o];
    } else {
        const T a = (T)st.alpha[c];
        const T rn = R[o] - a * Y[o];
        R[o] = rn;
        X[o] = X[o] + a * P[o];
        acc += (double)rn * rn;
    }
}

template <int kOp, typename T>
__global__ __launch_bounds__(256) void cg_reduce_kernel(int64_t n, int32_t S, T *R, T *P, T *Y, T *X, const T *B,
                                                        int64_t ldb, CgState st, int32_t k_check, double tol) {
    if (kOp >= kFinAlpha && __builtin_nontemporal_load(st.done)) return;
    __shared__ double red[4][kMaxRhs];
    __shared__ double fin_norm[kMaxRhs];
    __shared__ int fin_conv[kMaxRhs];
    __shared__ uint32_t last;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    double acc[4] = {0.0, 0.0, 0.0, 0.0};
    const int64_t n_waves = (int64_t)gridDim.x * 4;
    for (int64_t r = (int64_t)blockIdx.x * 4 + w; r < n; r += n_waves) {
#pragma unroll
        for (int ci = 0; ci < 4; ++ci) {
            const int c = lane + 64 * ci;
            if (c < S) cg_row_op<kOp, T>(r, c, S, R, P, Y, X, B, ldb, st, acc[ci]);
        }
    }
#pragma unroll
    for (int ci = 0; ci < 4; ++ci) red[w][lane + 64 * ci] = acc[ci];
    __syncthreads();
    for (int c = threadIdx.x; c < S; c += 256)
        st.part[(int64_t)blockIdx.x * S + c] = ((red[0][c] + red[1][c]) + red[2][c]) + red[3][c];
    __threadfence();
    __syncthreads();
    if (threadIdx.x == 0) last = atomicAdd(st.ticket, 1u) == gridDim.x - 1;
    __syncthreads();
    if (!last) return;
    __threadfence();
    // the last block: column c summed over blocks in order; tpc threads per column split the
    // blocks into contiguous ranges, combined in range order
    const int tpc = max(1, 256 / S);
    double *sum = &red[0][0];  // reuse: [tpc][S] <= 1024 doubles
    const int nb = gridDim.x;
    if ((int)threadIdx.x < tpc * S) {
        const int c = threadIdx.x % S, q = threadIdx.x / S;
        const int b0 = (int)((int64_t)nb * q / tpc), b1 = (int)((int64_t)nb * (q + 1) / tpc);
        double s = 0.0;
        for (int b = b0; b < b1; ++b) s += __builtin_nontemporal_load(&st.part[(int64_t)b * S + c]);
        sum[q * S + c] = s;
    }
    __syncthreads();
    for (int c = threadIdx.x; c < S; c += 256) {
        double s = 0.0;
        for (int q = 0; q < tpc; ++q) s += sum[q * S + c];
        cg_final_column<T>(kOp, c, s, st, fin_norm, fin_conv);
    }
    if (threadIdx.x == 0) *st.ticket = 0u;
    if constexpr (kOp == kFinInit || kOp == kFinUpdate) {
        __syncthreads();
        if (threadIdx.x == 0) {
            if constexpr (kOp == kFinInit) {
                int all = 1;  // (from LDS: the block's own global stores may not be visible to its loads yet)
                for (int c = 0; c < S; ++c) all &= fin_conv[c];
                *st.iters = 0;
                *st.done = all;  // has_converged.all() -> n_iter = 0
            } else {
                const int k = (*st.iters)++;
                double mean = 0.0;
                for (int c = 0; c < S; ++c) mean += fin_norm[c];
                mean /= S;
                if (k >= k_check && mean < tol) *st.done = 1;
            }
        }
    }
}

// P = R + beta P  (curr_conjugate_vec.mul_(beta).add_(precond_residual))
template <typename T>
__global__ __launch_bounds__(256) void cg_dir_kernel(int64_t n, int32_t S, const T *R, T *P, CgState st) {
    if (__builtin_nontemporal_load(st.done)) return;
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n * S) return;
    const T b = (T)st.beta[i % S];
    P[i] = P[i] * b + R[i];
}

// result.mul(rhs_norm) into the caller's layout
template <typename T>
__global__ __launch_bounds__(256) void cg_out_kernel(int64_t n, int32_t S, const T *X, T *out, int64_t ldo,
                                                     CgState st) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n * S) return;
    const int64_t r = i / S;
    const int c = (int)(i % S);
    out[r * ldo + c] = X[i] * (T)st.rhs_norm[c];
}

struct CgLayout {
    size_t R, P, Y, X, W, part, dbl, i32, seg1, seg2, total;
    int32_t tw1, nt1, tw2, nt2;  // column tiles of Phi_t^T (over the n_sys rows of P) and Phi_t (over W)
};

static CgLayout cg_layout(int64_t n_sys, int64_t n_cols, int32_t S, size_t elem) {
    CgLayout l{};
    size_t o = 0;
    const size_t vec = al256((size_t)n_sys * S * elem);
    l.R = o; o += vec;
    l.P = o; o += vec;
    l.Y = o; o += vec;
    l.X = o; o += vec;
    l.W = o; o += al256((size_t)n_cols * S * elem);
    l.part = o; o += al256((size_t)kRedBlocks * S * sizeof(double));
    l.dbl = o; o += al256((size_t)5 * S * sizeof(double));
    l.i32 = o; o += al256((size_t)(2 * S + 8) * sizeof(int32_t));
    l.tw1 = spmm_tile_rows(n_sys, S, elem);
    l.nt1 = l.tw1 ? (int32_t)cdiv<int64_t>(n_sys, l.tw1) : 1;
    l.tw2 = spmm_tile_rows(n_cols, S, elem);
    l.nt2 = l.tw2 ? (int32_t)cdiv<int64_t>(n_cols, l.tw2) : 1;
    l.seg1 = o; o += l.tw1 ? al256((size_t)(l.nt1 + 1) * n_cols * sizeof(int64_t)) : 0;
    l.seg2 = o; o += l.tw2 ? al256((size_t)(l.nt2 + 1) * n_sys * sizeof(int64_t)) : 0;
    l.total = o;
    return l;
}

template <typename T>
static int32_t cg_solve_impl(int64_t n_sys, const int64_t *ptr, const int32_t *idx, const float *val,
                             const int32_t *row_map, int64_t n_cols, const int64_t *t_ptr, const int32_t *t_idx,
                             const float *t_val, double noise, const T *rhs, int64_t ld_rhs, int32_t n_rhs,
                             double tolerance, int32_t max_iter, T *x, int64_t ldx, void *workspace,
                             size_t workspace_bytes, int32_t *iters_out, double *resid_out, grf_stream_t stream) {
    GRF_REQUIRE(n_sys > 0 && n_cols > 0 && ptr && t_ptr && rhs && x, GRF_EINVAL, "grf_cg_gram_solve: bad arguments");
    GRF_REQUIRE(n_rhs >= 1 && n_rhs <= kMaxRhs, GRF_EUNSUPPORTED, "grf_cg_gram_solve: n_rhs must be in [1, %d]",
                kMaxRhs);
    GRF_REQUIRE(ld_rhs >= n_rhs && ldx >= n_rhs && max_iter >= 0, GRF_EINVAL, "grf_cg_gram_solve: bad strides");
    const CgLayout l = cg_layout(n_sys, n_cols, n_rhs, sizeof(T));
    GRF_REQUIRE(workspace && workspace_bytes >= l.total, GRF_EINVAL, "grf_cg_gram_solve: workspace too small (%zu < %zu)",
                workspace_bytes, l.total);
    hipStream_t sm = S(stream);
    char *w = (char *)workspace;
    T *R = (T *)(w + l.R), *P = (T *)(w + l.P), *Y = (T *)(w + l.Y), *X = (T *)(w + l.X), *W = (T *)(w + l.W);
    const int32_t Sn = n_rhs;
    CgState st;
    double *d = (double *)(w + l.dbl);
    st.rhs_norm = d; st.rr = d + Sn; st.alpha = d + 2 * Sn; st.beta = d + 3 * Sn; st.rnorm = d + 4 * Sn;
    st.part = (double *)(w + l.part);
    int32_t *q = (int32_t *)(w + l.i32);
    st.rhs_zero = q; st.conv = q + Sn;
    st.ticket = (uint32_t *)(q + 2 * Sn); st.iters = q + 2 * Sn + 1; st.done = q + 2 * Sn + 2;
    GRF_CHECK_HIP(hipMemsetAsync(q, 0, (size_t)(2 * Sn + 8) * sizeof(int32_t), sm));

    const unsigned rb = (unsigned)std::min<int64_t>(cdiv<int64_t>(n_sys, 4), kRedBlocks);
    const int64_t nel = n_sys * Sn;
    GRF_REQUIRE_GRID(cdiv<int64_t>(nel, 256), 256, "cg_dir_kernel");
    const unsigned eb = (unsigned)cdiv<int64_t>(nel, 256);
    const int32_t k_check = std::min(10, max_iter - 1);
    int32_t rc0;

    int64_t *seg1 = l.tw1 ? (int64_t *)(w + l.seg1) : nullptr, *seg2 = l.tw2 ? (int64_t *)(w + l.seg2) : nullptr;
    if (seg1 && (rc0 = spmm_plan(n_cols, t_ptr, t_idx, nullptr, l.tw1, l.nt1, seg1, sm)) != GRF_OK) return rc0;
    if (seg2 && (rc0 = spmm_plan(n_sys, ptr, idx, row_map, l.tw2, l.nt2, seg2, sm)) != GRF_OK) return rc0;
    cg_reduce_kernel<kFinNorm, T><<<rb, 256, 0, sm>>>(n_sys, Sn, R, P, Y, X, rhs, ld_rhs, st, k_check, tolerance);
    GRF_CHECK_LAUNCH("cg_reduce_kernel<norm>");
    cg_reduce_kernel<kFinInit, T><<<rb, 256, 0, sm>>>(n_sys, Sn, R, P, Y, X, rhs, ld_rhs, st, k_check, tolerance);
    GRF_CHECK_LAUNCH("cg_reduce_kernel<init>");

    int32_t *h = nullptr;  // pinned: [done of even iterations, done of odd iterations, iters]
    GRF_CHECK_HIP(hipHostMalloc((void **)&h, 4 * sizeof(int32_t), hipHostMallocDefault));
    hipEvent_t ev[2];
    GRF_CHECK_HIP(hipEventCreateWithFlags(&ev[0], hipEventDisableTiming));
    GRF_CHECK_HIP(hipEventCreateWithFlags(&ev[1], hipEventDisableTiming));
    int32_t rc = GRF_OK;
    for (int32_t k = 0; k < max_iter && rc == GRF_OK; ++k) {
        // mvms = (K + s2 I) p = Phi_t (Phi_t^T p) + s2 p
        rc = spmm_dispatch<T>(n_cols, t_ptr, t_idx, t_val, nullptr, P, Sn, Sn, W, Sn, nullptr, 0, T(0), st.done, sm,
                              seg1, l.nt1);
        if (rc != GRF_OK) break;
        rc = spmm_dispatch<T>(n_sys, ptr, idx, val, row_map, W, Sn, Sn, Y, Sn, P, Sn, (T)noise, st.done, sm, seg2,
                              l.nt2);
        if (rc != GRF_OK) break;
        cg_reduce_kernel<kFinAlpha, T><<<rb, 256, 0, sm>>>(n_sys, Sn, R, P, Y, X, rhs, ld_rhs, st, k_check, tolerance);
        cg_reduce_kernel<kFinUpdate, T><<<rb, 256, 0, sm>>>(n_sys, Sn, R, P, Y, X, rhs, ld_rhs, st, k_check, tolerance);
        cg_dir_kernel<T><<<eb, 256, 0, sm>>>(n_sys, Sn, R, P, st);
        if (hipGetLastError() != hipSuccess) {
            set_error("grf_cg_gram_solve: launch failed");
            rc = GRF_EHIP;
            break;
        }
        if (k < k_check) continue;
        // poll: copy this iteration's flag, then look at the previous one's (one iteration in flight)
        if (hipMemcpyAsync(&h[k & 1], st.done, sizeof(int32_t), hipMemcpyDeviceToHost, sm) != hipSuccess ||
            hipEventRecord(ev[k & 1], sm) != hipSuccess) {
            set_error("grf_cg_gram_solve: poll failed");
            rc = GRF_EHIP;
            break;
        }
        if (k > k_check) {
            if (hipEventSynchronize(ev[(k - 1) & 1]) != hipSuccess) {
                set_error("grf_cg_gram_solve: event wait failed");
                rc = GRF_EHIP;
                break;
            }
            if (h[(k - 1) & 1]) break;
        }
    }
    if (rc == GRF_OK) {
        cg_out_kernel<T><<<eb, 256, 0, sm>>>(n_sys, Sn, X, x, ldx, st);
        if (hipGetLastError() != hipSuccess) {
            set_error("grf_cg_gram_solve: launch of cg_out_kernel failed");
            rc = GRF_EHIP;
        }
    }
    if (rc == GRF_OK && (iters_out || resid_out)) {
        if (hipMemcpyAsync(&h[2], st.iters, sizeof(int32_t), hipMemcpyDeviceToHost, sm) != hipSuccess ||
            (resid_out && hipMemcpyAsync(resid_out, st.rnorm, Sn * sizeof(double), hipMemcpyDeviceToHost, sm) !=
                              hipSuccess) ||
            hipStreamSynchronize(sm) != hipSuccess) {
            set_error("grf_cg_gram_solve: reading the iteration count failed");
            rc = GRF_EHIP;
        } else {
            if (iters_out) *iters_out = h[2];
        }
    } else {
        (void)hipStreamSynchronize(sm);  // the pinned buffer is freed below
    }
    (void)hipEventDestroy(ev[0]);
    (void)hipEventDestroy(ev[1]);
    (void)hipHostFree(h);
    return rc;
}

}  // namespace grf

using namespace grf;

extern "C" {
#pragma GCC visibility push(default)

size_t grf_csr_transpose_workspace_bytes(int64_t n_sel, int64_t n_cols, int64_t nnz) {
    const int64_t z = std::max<int64_t>(nnz, 1);
    return al256((size_t)(n_sel + 1) * 4) + al256((size_t)(n_sel + 1) * 8) + scan_ws_bytes(n_sel + 1) +
           2 * al256((size_t)z * 4) + 2 * al256((size_t)z * 8) + al256(csr_tr_sort_temp_bytes(nnz, n_cols));
}

int32_t grf_csr_transpose(int64_t n_sel, const int64_t *ptr, const int32_t *idx, const float *val,
                          const int32_t *row_map, int64_t n_cols, int64_t nnz, int64_t *t_ptr, int32_t *t_idx,
                          float *t_val, void *workspace, size_t workspace_bytes, grf_stream_t stream) {
    // (idx / val / t_idx / t_val may be NULL when there are no entries)
    GRF_REQUIRE(n_sel >= 0 && n_cols > 0 && nnz >= 0 && ptr && t_ptr, GRF_EINVAL, "grf_csr_transpose: bad arguments");
    const size_t need = grf_csr_transpose_workspace_bytes(n_sel, n_cols, nnz);
    GRF_REQUIRE(workspace && workspace_bytes >= need, GRF_EINVAL, "grf_csr_transpose: workspace too small (%zu < %zu)",
                workspace_bytes, need);
    GRF_REQUIRE(n_sel < (1ll << 31) && n_cols < (1ll << 31), GRF_EUNSUPPORTED, "grf_csr_transpose: more than 2^31 rows");
    hipStream_t st = S(stream);
    const int64_t z = std::max<int64_t>(nnz, 1);
    char *w = (char *)workspace;
    int32_t *len = (int32_t *)w;
    w += al256((size_t)(n_sel + 1) * 4);
    int64_t *off = (int64_t *)w;
    w += al256((size_t)(n_sel + 1) * 8);
    void *scan_ws = w;
    w += scan_ws_bytes(n_sel + 1);
    uint32_t *k0 = (uint32_t *)w, *k1 = (uint32_t *)(w + al256((size_t)z * 4));
    w += 2 * al256((size_t)z * 4);
    uint64_t *v0 = (uint64_t *)w, *v1 = (uint64_t *)(w + al256((size_t)z * 8));
    w += 2 * al256((size_t)z * 8);
    size_t temp_bytes = csr_tr_sort_temp_bytes(nnz, n_cols);
    if (n_sel > 0) {
        csr_tr_len_kernel<<<(unsigned)cdiv<int64_t>(n_sel, 256), 256, 0, st>>>(n_sel, ptr, row_map, len);
        GRF_CHECK_LAUNCH("csr_tr_len_kernel");
        int32_t rc = scan_counts_i32(n_sel, len, off, scan_ws, scan_ws_bytes(n_sel + 1), st);
        if (rc != GRF_OK) return rc;
        GRF_REQUIRE_GRID(cdiv<int64_t>(n_sel, 4), 256, "csr_tr_gather_kernel");
        csr_tr_gather_kernel<<<(unsigned)cdiv<int64_t>(n_sel, 4), 256, 0, st>>>(n_sel, ptr, idx, val, row_map, off, k0,
                                                                               v0);
        GRF_CHECK_LAUNCH("csr_tr_gather_kernel");
    }
    if (nnz > 0) {
        // (nnz may bound the gathered entries from above: pad the tail with the key n_cols)
        csr_tr_pad_kernel<<<(unsigned)std::min<int64_t>(cdiv<int64_t>(nnz, 256), 1024), 256, 0, st>>>(nnz, n_sel, off,
                                                                                                    n_cols, k0);
        GRF_CHECK_LAUNCH("csr_tr_pad_kernel");
    }
    if (nnz > 0) {
        GRF_CHECK_HIP(rocprim::radix_sort_pairs(w, temp_bytes, (const uint32_t *)k0, k1, (const uint64_t *)v0, v1,
                                                (size_t)nnz, 0u, key_bits(n_cols), st));
    }
    GRF_REQUIRE_GRID(cdiv<int64_t>(nnz + 1, 256), 256, "csr_tr_unpack_kernel");
    csr_tr_unpack_kernel<<<(unsigned)cdiv<int64_t>(nnz + 1, 256), 256, 0, st>>>(nnz, n_cols, k1, v1, t_ptr, t_idx,
                                                                                t_val);
    GRF_CHECK_LAUNCH("csr_tr_unpack_kernel");
    return GRF_OK;
}

int32_t grf_spmm_csr(int64_t n_out, const int64_t *ptr, const int32_t *idx, const float *val, const int32_t *row_map,
                     const float *X, int64_t ldx, int32_t n_rhs, float *Y, int64_t ldy, grf_stream_t stream) {
    GRF_REQUIRE(n_out >= 0 && n_rhs >= 0 && ptr && X && Y && ldx >= n_rhs && ldy >= n_rhs, GRF_EINVAL,
                "grf_spmm_csr: bad arguments");
    return spmm_dispatch<float>(n_out, ptr, idx, val, row_map, X, ldx, n_rhs, Y, ldy, nullptr, 0, 0.f, nullptr,
                                S(stream));
}

int32_t grf_spmm_csr_f64(int64_t n_out, const int64_t *ptr, const int32_t *idx, const float *val,
                         const int32_t *row_map, const double *X, int64_t ldx, int32_t n_rhs, double *Y, int64_t ldy,
                         grf_stream_t stream) {
    GRF_REQUIRE(n_out >= 0 && n_rhs >= 0 && ptr && X && Y && ldx >= n_rhs && ldy >= n_rhs, GRF_EINVAL,
                "grf_spmm_csr_f64: bad arguments");
    return spmm_dispatch<double>(n_out, ptr, idx, val, row_map, X, ldx, n_rhs, Y, ldy, nullptr, 0, 0.0, nullptr,
                                 S(stream));
}

size_t grf_cg_workspace_bytes(int64_t n_sys, int64_t n_cols, int32_t n_rhs) {
    return std::max(cg_layout(n_sys, n_cols, n_rhs, sizeof(float)).total,
                    cg_layout(n_sys, n_cols, n_rhs, sizeof(double)).total);
}

int32_t grf_cg_gram_solve(int64_t n_sys, const int64_t *ptr, const int32_t *idx, const float *val,
                          const int32_t *row_map, int64_t n_cols, const int64_t *t_ptr, const int32_t *t_idx,
                          const float *t_val, double noise, const float *rhs, int64_t ld_rhs, int32_t n_rhs,
                          double tolerance, int32_t max_iter, float *x, int64_t ldx, void *workspace,
                          size_t workspace_bytes, int32_t *iters_out, double *resid_out, grf_stream_t stream) {
    return cg_solve_impl<float>(n_sys, ptr, idx, val, row_map, n_cols, t_ptr, t_idx, t_val, noise, rhs, ld_rhs, n_rhs,
                                tolerance, max_iter, x, ldx, workspace, workspace_bytes, iters_out, resid_out, stream);
}

int32_t grf_cg_gram_solve_f64(int64_t n_sys, const int64_t *ptr, const int32_t *idx, const float *val,
                              const int32_t *row_map, int64_t n_cols, const int64_t *t_ptr, const int32_t *t_idx,
                              const float *t_val, double noise, const double *rhs, int64_t ld_rhs, int32_t n_rhs,
                              double tolerance, int32_t max_iter, double *x, int64_t ldx, void *workspace,
                              size_t workspace_bytes, int32_t *iters_out, double *resid_out, grf_stream_t stream) {
    return cg_solve_impl<double>(n_sys, ptr, idx, val, row_map, n_cols, t_ptr, t_idx, t_val, noise, rhs, ld_rhs,
                                 n_rhs, tolerance, max_iter, x, ldx, workspace, workspace_bytes, iters_out, resid_out,
                                 stream);
}

#pragma GCC visibility pop
}  // extern "C"
