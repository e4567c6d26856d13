// grf_laplacian.hip -- normalised graph Laplacians on the device, with the
// exact floating-point semantics of the reference's numpy / scipy code so that
// the walk matrix (and therefore every walk) is bit-identical.
//
//   GRF_LAP_SCIPY : efficient_graph_gp_sparse/utils_sparse/graph_utils.py:16-30
//     deg  = A.sum(axis=1)  -> np.add.reduceat per row = a0 + pairwise(rest)
//     dinv = 1/sqrt(deg), inf -> 0
//     L    = (D_inv_sqrt @ (D - A)) @ D_inv_sqrt, exact zeros dropped at every
//            scipy op, columns ascending, diagonal stored.
//   GRF_LAP_NUMPY / _SAFE / _COMBINATORIAL / _NONE (dense input):
//     efficient_graph_gp/graph_kernels/utils.py:21-26 and
//     efficient_graph_gp/preprocessing/laplacian_np.py:13-34; deg = np.sum(W, 1)
//     (numpy pairwise summation over the full dense row); the walk matrix is the
//     CSR of the nonzeros in ascending column order (np.flatnonzero,
//     random_walk_samplers/sampler.py:22-28).
#include "grf_block.h"

namespace grf {

int32_t scan_counts_i32(int64_t n, const int32_t *cnt, int64_t *out, void *ws, size_t ws_bytes, hipStream_t st);
size_t scan_ws_bytes(int64_t n);

// numpy pairwise_sum_DOUBLE leaf (n <= 128)
__device__ inline double pw_leaf(const double *a, int64_t n) {
    if (n < 8) {
        double r = 0.0;
        for (int64_t i = 0; i < n; ++i) r += a[i];
        return r;
    }
    double r0 = a[0], r1 = a[1], r2 = a[2], r3 = a[3], r4 = a[4], r5 = a[5], r6 = a[6], r7 = a[7];
    int64_t i;
    for (i = 8; i < n - (n % 8); i += 8) {
        r0 += a[i + 0]; r1 += a[i + 1]; r2 += a[i + 2]; r3 += a[i + 3];
        r4 += a[i + 4]; r5 += a[i + 5]; r6 += a[i + 6]; r7 += a[i + 7];
    }
    double res = ((r0 + r1) + (r2 + r3)) + ((r4 + r5) + (r6 + r7));
    for (; i < n; ++i) res += a[i];
    return res;
}

// The recursion's explicit stack lives in LDS (one per wave, used by lane 0 only): a per-lane array in
// registers would be dynamically indexed, i.e. private (scratch) memory -- 2.5 KB per lane, which the runtime
// must back for every wave the device can hold at each launch of every kernel reaching this code.
// Depth: a frame of m > 128 values splits into halves of <= m / 2 + 8, so 64 frames cover any int64 n.
constexpr int kPwDepth = 64;
struct PwFrame { int64_t off, n; double left; int32_t state; };

// numpy pairwise_sum_DOUBLE, recursion unrolled onto the explicit stack `st`
__device__ double np_pairwise(const double *a, int64_t n, PwFrame *st) {
    if (n <= 128) return pw_leaf(a, n);
    int sp = 0;
    st[0] = {0, n, 0.0, 0};
    double ret = 0.0;
    while (sp >= 0) {
        PwFrame &f = st[sp];
        if (f.n <= 128) {
            ret = pw_leaf(a + f.off, f.n);
            --sp;
            continue;
        }
        int64_t n2 = f.n / 2;
        n2 -= n2 % 8;
        if (f.state == 0) {
            f.state = 1;
            st[sp + 1] = {f.off, n2, 0.0, 0};
            ++sp;
        } else if (f.state == 1) {
            f.left = ret;
            f.state = 2;
            st[sp + 1] = {f.off + n2, f.n - n2, 0.0, 0};
            ++sp;
        } else {
            ret = f.left + ret;
            --sp;
        }
    }
    return ret;
}

// numpy pairwise_sum_DOUBLE of a[0 .. n) by one wave, bit for bit: the recursion's leaves (runs
// of <= 128 values, split points n2 = n/2 - (n/2) % 8) are listed by lane 0, summed by the 64 lanes
// in parallel with the leaf's own 8-accumulator order, and combined by lane 0 in the recursion's
// order.  `ws` is the wave's LDS: kPwLeaves leaves and the stack; longer inputs fall back to lane 0.
// Every lane returns the sum.  (A hub row of thousands of entries, or a dense row, no longer
// costs one lane thousands of dependent adds.)
constexpr int kPwLeaves = 128;
struct PwLeaf { int64_t off; int64_t n; double sum; };
struct PwScratch {
    PwLeaf leaf[kPwLeaves];
    PwFrame st[kPwDepth];
};

__device__ double wave_np_pairwise(const double *a, int64_t n, PwScratch *ws) {
    const int lane = threadIdx.x & 63;
    PwLeaf *leaf = ws->leaf;
    PwFrame *st = ws->st;
    if (n <= 128) {
        // one leaf: lanes 0..7 own the accumulators r_j (a[j], a[j + 8], ...), then the fixed tree
        double r = 0.0;
        if (n < 8) {
            double t = 0.0;
            if (lane == 0)
                for (int64_t i = 0; i < n; ++i) t += a[i];
            return __shfl(t, 0, 64);
        }
        const int64_t nb = n - (n % 8);
        if (lane < 8) {
            r = a[lane];
            for (int64_t i = 8 + lane; i < nb; i += 8) r += a[i];
        }
        const double r0 = __shfl(r, 0, 64), r1 = __shfl(r, 1, 64), r2 = __shfl(r, 2, 64), r3 = __shfl(r, 3, 64);
        const double r4 = __shfl(r, 4, 64), r5 = __shfl(r, 5, 64), r6 = __shfl(r, 6, 64), r7 = __shfl(r, 7, 64);
        double res = ((r0 + r1) + (r2 + r3)) + ((r4 + r5) + (r6 + r7));
        for (int64_t i = nb; i < n; ++i) res += a[i];
        return res;
    }
    // Integer rows (unit or small integer weights: every graph the benches run): when every value is an
    // integer of magnitude <= 2^20 and one is nonzero, every partial sum of any order is an exact integer
    // (< 2^51), so the numpy recursion's result is the exact sum -- taken here in one strided pass and a
    // wave reduction (bit-identical; a zero total is +0.0 either way).  Otherwise the recursion below.
    {
        bool integral = true, nonzero = false;
        double s = 0.0;
        for (int64_t i = lane; i < n; i += 64) {
            const double v = a[i];
            integral = integral && v == rint(v) && fabs(v) <= 1048576.0;
            nonzero = nonzero || v != 0.0;
            s += v;
        }
        if (__all(integral) && __any(nonzero)) {
#pragma unroll
            for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
            return s;
        }
    }
    // list the leaves (lane 0, the recursion's explicit stack), left to right
    int32_t nl = 0;
    if (lane == 0) {
        int sp = 0;
        st[0].off = 0;
        st[0].n = n;
        while (sp >= 0) {
            const int64_t o = st[sp].off, m = st[sp].n;
            --sp;
            if (m <= 128) {
                if (nl < kPwLeaves) leaf[nl] = PwLeaf{o, m, 0.0};
                ++nl;
                continue;
            }
            int64_t n2 = m / 2;
            n2 -= n2 % 8;
            // push right then left: the left subtree's leaves come first
            ++sp;
            st[sp].off = o + n2;
            st[sp].n = m - n2;
            ++sp;
            st[sp].off = o;
            st[sp].n = n2;
        }
    }
    nl = __shfl(nl, 0, 64);
    __builtin_amdgcn_wave_barrier();
    if (nl > kPwLeaves) {
        const double t = lane == 0 ? np_pairwise(a, n, st) : 0.0;
        return __shfl(t, 0, 64);
    }
    for (int l = lane; l < nl; l += 64) leaf[l].sum = pw_leaf(a + leaf[l].off, leaf[l].n);
    __builtin_amdgcn_wave_barrier();
    // combine in the recursion's order (lane 0): the same stack machine with leaf sums in order
    double total = 0.0;
    if (lane == 0) {
        int sp = 0, next = 0;
        st[0] = {0, n, 0.0, 0};
        double ret = 0.0;
        while (sp >= 0) {
            PwFrame &f = st[sp];
            if (f.n <= 128) {
                ret = leaf[next++].sum;
                --sp;
                continue;
            }
            int64_t n2 = f.n / 2;
            n2 -= n2 % 8;
            if (f.state == 0) {
                f.state = 1;
                st[sp + 1] = {0, n2, 0.0, 0};
                ++sp;
            } else if (f.state == 1) {
                f.left = ret;
                f.state = 2;
                st[sp + 1] = {0, f.n - n2, 0.0, 0};
                ++sp;
            } else {
                ret = f.left + ret;
                --sp;
            }
        }
        total = ret;
    }
    __builtin_amdgcn_wave_barrier();
    return __shfl(total, 0, 64);
}

// ------------------------------------------------------------------- scipy
// degrees a_ii... : deg = a0 + pairwise(rest) per row (np.add.reduceat), one wave per row
__global__ __launch_bounds__(256) void lap_deg_kernel(int64_t n, const int64_t *ptr, const double *val, double *deg,
                                                      double *dinv) {
    __shared__ PwScratch leaves[4];
    const int64_t i = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (i >= n) return;
    const int64_t b = ptr[i], e = ptr[i + 1];
    const double rest = e - b > 1 ? wave_np_pairwise(val + b + 1, e - b - 1, &leaves[threadIdx.x >> 6]) : 0.0;
    if ((threadIdx.x & 63) == 0) {
        const double d = e > b ? val[b] + rest : 0.0;
        deg[i] = d;
        const double v = 1.0 / sqrt(d);
        dinv[i] = isinf(v) ? 0.0 : v;
    }
}

// One row of D^-1/2 (D - A) D^-1/2 in scipy order, one wave per row (a power-law hub row of
// thousands of entries is spread over the 64 lanes instead of serialising one thread).
// The row's virtual sequence is A's entries in column order with the diagonal merged into an
// explicit (i, i) entry (value d - a_ii) or inserted before the first column > i (value d);
// sp.diags drops a zero diagonal, so d == 0 inserts nothing and an explicit a_ii stays -a_ii.
// Every element is computed independently with the serial code's exact arithmetic
// (u = (dinv_i v) dinv_j, exact zeros dropped), then compacted in order by ballot counts.
// EMIT=false counts.
template <bool EMIT>
__global__ __launch_bounds__(256) void lap_row_kernel(int64_t n, const int64_t *ptr, const int32_t *idx,
                                                      const double *val, const double *deg, const double *dinv,
                                                      int32_t *cnt, const int64_t *l_ptr, int32_t *l_idx,
                                                      double *l_val, int64_t l_cap) {
    const int64_t i = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (i >= n) return;
    const int lane = threadIdx.x & 63;
    const double d = deg[i], di = dinv[i];
    const int64_t b = ptr[i], e = ptr[i + 1];
    // first entry with column >= i (columns ascending)
    int64_t lo = b, hi = e;
    while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if (idx[mid] < i) lo = mid + 1;
        else hi = mid;
    }
    const int64_t pd = lo - b;  // position of the diagonal in the virtual sequence
    const bool has_diag = d != 0.0;
    const bool expl = lo < e && idx[lo] == i;
    const bool insert = has_diag && !expl;
    const int64_t total = (e - b) + (insert ? 1 : 0);
    int64_t out = EMIT ? l_ptr[i] : 0;
    int32_t c = 0;
    for (int64_t base = 0; base < total; base += 64) {
        const int64_t k = base + lane;
        bool keep = false;
        int64_t col = 0;
        double u = 0.0;
        if (k < total) {
            double v;
            if (insert && k == pd) {
                col = i;
                v = d;
            } else {
                const int64_t a = b + ((insert && k > pd) ? k - 1 : k);
                col = idx[a];
                v = (has_diag && col == i) ? d - val[a] : 0.0 - val[a];
            }
            if (v != 0.0 && di != 0.0) {
                const double t = di * v;
                if (t != 0.0) {
                    const double dj = dinv[col];
                    if (dj != 0.0) {
                        u = t * dj;
                        keep = u != 0.0;
                    }
                }
            }
        }
        const uint64_t m = __ballot(keep);
        if (EMIT) {
            const int64_t o = out + __popcll(m & ((1ull << lane) - 1ull));
            if (keep && o < l_cap) {
                l_idx[o] = (int32_t)col;
                l_val[o] = u;
            }
            out += __popcll(m);
        } else {
            c += __popcll(m);
        }
    }
    if (!EMIT && lane == 0) cnt[i] = c;
}

// ---------------------------------------------- scipy, eight rows per wave
// Most rows of a sparse graph are short (C5: mean degree ~10): a wave per row leaves 50+ lanes
// idle.  These kernels give each row a group of 8 lanes (8 rows per wave); rows too long for a
// group (degree sums over more than one numpy leaf, or 64 entries and more) are done afterwards by
// the whole wave.  Same arithmetic, same bits.  Each lane issues ALL its loads of a row at once
// (then the neighbours' D^-1/2 at once): a row costs three dependent round trips (row bounds,
// entries, neighbour scales) instead of one per entry tail element and per binary-search step
// (C5, 1M rows: 627 us for the three launches, latency-bound at ~0.1 TB/s).
constexpr int kGroupRowMax = 64;
constexpr int kLeafPer = 16;  // 128 (one numpy leaf) / 8 lanes

__global__ __launch_bounds__(256) void lap_deg_group_kernel(int64_t n, const int64_t *__restrict__ ptr,
                                                            const double *__restrict__ val, double *__restrict__ deg,
                                                            double *__restrict__ dinv) {
    __shared__ PwScratch leaves[4];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, g = lane >> 3, j = lane & 7;
    const int64_t r0 = ((int64_t)blockIdx.x * 4 + wave) * 8;
    if (r0 >= n) return;
    const int64_t i = r0 + g;
    int64_t b = 0, e = 0;
    if (i < n) {
        b = ptr[i];
        e = ptr[i + 1];
    }
    const int64_t m = e - b > 1 ? e - b - 1 : 0;  // deg = a0 + pairwise(a[1 ..])
    const bool lng = m > 128;
    const int64_t mm = lng ? 0 : m;
    const double *a = val + b + 1;
    // numpy's leaf: accumulator r_j = a[j] + a[j + 8] + ... over the first nb = mm - mm % 8 values,
    // the fixed tree over r_0..r_7, then the tail a[nb ..) added in order (mm < 8: the tail alone from 0)
    // (loads past the wave's longest row are skipped by a scalar branch: ER rows of ~20 entries issue 3)
    int64_t mw = mm;
#pragma unroll
    for (int off = 8; off < 64; off <<= 1) mw = max(mw, (int64_t)__shfl_xor(mw, off, 64));
    const int qmax = __builtin_amdgcn_readfirstlane((int)((mw + 7) >> 3));
    double x[kLeafPer];
#pragma unroll
    for (int q = 0; q < kLeafPer; ++q) {
        x[q] = 0.0;
        if (q < qmax && 8 * q + j < mm) x[q] = a[8 * q + j];
    }
    const double a0 = (j == 0 && e > b) ? val[b] : 0.0;
    const int64_t nb = mm >= 8 ? mm - (mm % 8) : 0;
    double r = x[0];
#pragma unroll
    for (int q = 1; q < kLeafPer; ++q)
        if (q < qmax && 8 * q + j < nb) r += x[q];
    const double r1 = __shfl_xor(r, 1, 64);
    const double p01 = (j & 1) ? r1 + r : r + r1;
    const double p23 = __shfl_xor(p01, 2, 64);
    const double qq = (j & 2) ? p23 + p01 : p01 + p23;
    const double q4 = __shfl_xor(qq, 4, 64);
    double res = (j & 4) ? q4 + qq : qq + q4;
    if (mm < 8) res = 0.0;  // (numpy: res = 0; res += a[i] for short inputs)
    // the tail value a[nb + j] is this lane's x[nb / 8]
    const int qt = (int)(nb >> 3);
    double tv = 0.0;
#pragma unroll
    for (int q = 0; q < kLeafPer; ++q)
        if (q < qmax && q == qt) tv = x[q];
    const int64_t ntail = mm - nb;  // <= 7
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const double t = __shfl(tv, (lane & ~7) + k, 64);
        if (k < ntail) res += t;
    }
    if (j == 0 && i < n && !lng) {
        const double d = e > b ? a0 + res : 0.0;
        deg[i] = d;
        const double v = 1.0 / sqrt(d);
        dinv[i] = isinf(v) ? 0.0 : v;
    }
    uint64_t todo = __ballot(lng && j == 0 && i < n);
    while (todo) {  // long rows: the whole wave, one at a time
        const int gg = (__ffsll((long long)todo) - 1) >> 3;
        todo &= todo - 1;
        const int64_t ii = r0 + gg, bb = ptr[ii], ee = ptr[ii + 1];
        const double rr = wave_np_pairwise(val + bb + 1, ee - bb - 1, &leaves[wave]);
        if (lane == 0) {
            const double d = val[bb] + rr;
            deg[ii] = d;
            const double v = 1.0 / sqrt(d);
            dinv[ii] = isinf(v) ? 0.0 : v;
        }
    }
}

// One element of row i of D^-1/2 (D - A) D^-1/2 with the serial code's exact arithmetic, in two
// halves so that the neighbour's D^-1/2 loads of several elements are in flight together:
// lap_pre gives the scaled value t = di v and whether D^-1/2[col] is needed (else dropped),
// lap_post the element u = t dj and whether it is kept (u != 0).  v = d - a_ii for an explicit
// diagonal when d != 0, else 0 - a (sp.diags drops a zero diagonal); the inserted diagonal has v = d.
__device__ __forceinline__ bool lap_pre(double v, double di, double &t) {
    if (v != 0.0 && di != 0.0) {
        t = di * v;
        return t != 0.0;
    }
    return false;
}
__device__ __forceinline__ bool lap_post(bool need, double t, double dj, double &u) {
    u = 0.0;
    if (need && dj != 0.0) {
        u = t * dj;
        return u != 0.0;
    }
    return false;
}

// the row's virtual sequence (long rows, the whole wave): element k -> (column, scaled value, kept)
struct LapRow {
    int64_t i, b, e, pd, total;
    double d, di;
    bool has_diag, insert;
    __device__ void init(int64_t row, const int64_t *ptr, const int32_t *idx, const double *deg, const double *dinv) {
        i = row;
        d = deg[i];
        di = dinv[i];
        b = ptr[i];
        e = ptr[i + 1];
        int64_t lo = b, hi = e;
        while (lo < hi) {
            const int64_t mid = (lo + hi) >> 1;
            if (idx[mid] < i) lo = mid + 1;
            else hi = mid;
        }
        pd = lo - b;
        has_diag = d != 0.0;
        const bool expl = lo < e && idx[lo] == i;
        insert = has_diag && !expl;
        total = (e - b) + (insert ? 1 : 0);
    }
    // element k's column and value before the neighbour scale (k < total)
    __device__ void raw(int64_t k, const int32_t *idx, const double *val, int32_t &col, double &v) const {
        if (insert && k == pd) {
            col = (int32_t)i;
            v = d;
        } else {
            const int64_t a = b + ((insert && k > pd) ? k - 1 : k);
            col = idx[a];
            const double w = val[a];
            v = (has_diag && col == i) ? d - w : 0.0 - w;
        }
    }
};

template <bool EMIT>
__global__ __launch_bounds__(256) void lap_row_group_kernel(int64_t n, const int64_t *__restrict__ ptr,
                                                            const int32_t *__restrict__ idx,
                                                            const double *__restrict__ val,
                                                            const double *__restrict__ deg,
                                                            const double *__restrict__ dinv, int32_t *__restrict__ cnt,
                                                            const int64_t *__restrict__ l_ptr,
                                                            int32_t *__restrict__ l_idx, double *__restrict__ l_val,
                                                            int64_t l_cap) {
    constexpr int kQ = kGroupRowMax / 8;  // entries per lane of a group row
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, g = lane >> 3, j = lane & 7;
    const int64_t r0 = ((int64_t)blockIdx.x * 4 + wave) * 8;
    if (r0 >= n) return;
    const int64_t i = r0 + g;
    const bool valid = i < n;
    int64_t b = 0, e = 0, out = 0;
    double d = 0.0, di = 0.0;
    if (valid) {
        b = ptr[i];
        e = ptr[i + 1];
        d = deg[i];
        di = dinv[i];
        if (EMIT) out = l_ptr[i];
    }
    const bool lng = e - b >= kGroupRowMax;  // (with an inserted diagonal: more than kGroupRowMax elements)
    const int64_t len = lng ? 0 : e - b;
    const int sh = 8 * g;
    // round trip 2: the row's entries, all at once (entry 8 q + j in lane j; rounds past the wave's
    // longest group row are skipped by a scalar branch)
    int64_t lw = len;
#pragma unroll
    for (int off = 8; off < 64; off <<= 1) lw = max(lw, (int64_t)__shfl_xor(lw, off, 64));
    const int qmax = __builtin_amdgcn_readfirstlane((int)((lw + 7) >> 3));
    int32_t col[kQ];
    double w[kQ];
#pragma unroll
    for (int q = 0; q < kQ; ++q) {
        col[q] = -1;
        w[q] = 0.0;
        if (q < qmax && 8 * q + j < len) {
            col[q] = idx[b + 8 * q + j];
            w[q] = val[b + 8 * q + j];
        }
    }
    const bool has_diag = d != 0.0;
    bool expl = false;
#pragma unroll
    for (int q = 0; q < kQ; ++q)
        if (q < qmax) expl = expl || ((__ballot(col[q] == i) >> sh) & 0xffu) != 0;
    const bool insert = has_diag && !expl;
    // round trip 3: the neighbours' D^-1/2 (a dropped element reads its own row's, a valid address)
    double t[kQ], dj[kQ];
    bool need[kQ];
#pragma unroll
    for (int q = 0; q < kQ; ++q) {
        need[q] = false;
        t[q] = 0.0;
        dj[q] = 0.0;
        if (q < qmax) {
            const bool in = 8 * q + j < len;
            const double v = (has_diag && col[q] == i) ? d - w[q] : 0.0 - w[q];
            need[q] = in && lap_pre(v, di, t[q]);
            dj[q] = dinv[need[q] ? col[q] : (valid ? i : 0)];
        }
    }
    double ti = 0.0;
    const bool need_i = insert && lap_pre(d, di, ti);
    double ui;
    const bool keep_i = lap_post(need_i, ti, di, ui);  // (dinv[i] is di)
    int64_t run = out;  // EMIT: the next place; else the count
    int32_t klt = 0;    // kept entries with columns < i: the inserted diagonal goes after them
#pragma unroll
    for (int q = 0; q < kQ; ++q) {
        if (q >= qmax) break;
        double u;
        const bool keep = lap_post(need[q], t[q], dj[q], u);
        const uint32_t gm = (uint32_t)(__ballot(keep) >> sh) & 0xffu;
        klt += __popc((uint32_t)(__ballot(keep && col[q] < i) >> sh) & 0xffu);
        if (EMIT) {
            const int64_t o = run + __popc(gm & ((1u << j) - 1u)) + ((keep_i && col[q] > i) ? 1 : 0);
            if (keep && o < l_cap) {
                l_idx[o] = col[q];
                l_val[o] = u;
            }
        }
        run += __popc(gm);
    }
    if (j == 0 && valid && !lng) {
        if (EMIT) {
            const int64_t o = out + klt;
            if (keep_i && o < l_cap) {
                l_idx[o] = (int32_t)i;
                l_val[o] = ui;
            }
        } else {
            cnt[i] = (int32_t)(run + (keep_i ? 1 : 0));
        }
    }
    uint64_t todo = __ballot(lng && j == 0 && valid);
    while (todo) {  // long rows: the whole wave, 4 x 64 elements in flight per round
        const int gg = (__ffsll((long long)todo) - 1) >> 3;
        todo &= todo - 1;
        LapRow W;
        W.init(r0 + gg, ptr, idx, deg, dinv);
        int64_t o0 = EMIT ? l_ptr[W.i] : 0;
        for (int64_t base = 0; base < W.total; base += 256) {
            int32_t c4[4];
            double t4[4], dj4[4];
            bool n4[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int64_t k = base + 64 * u + lane;
                double v = 0.0;
                c4[u] = (int32_t)W.i;
                if (k < W.total) W.raw(k, idx, val, c4[u], v);
                n4[u] = k < W.total && lap_pre(v, W.di, t4[u]);
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) dj4[u] = dinv[n4[u] ? c4[u] : (int32_t)W.i];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                double uu;
                const bool keep = lap_post(n4[u], t4[u], dj4[u], uu);
                const uint64_t m = __ballot(keep);
                if (EMIT) {
                    const int64_t o = o0 + __popcll(m & ((1ull << lane) - 1ull));
                    if (keep && o < l_cap) {
                        l_idx[o] = c4[u];
                        l_val[o] = uu;
                    }
                }
                o0 += __popcll(m);
            }
        }
        if (!EMIT && lane == 0) cnt[W.i] = (int32_t)o0;
    }
}

// ------------------------------------------------------------------- dense
// Two launches, one HBM read of W (was three full passes: degrees, counts, fill).
//
//  lapd_stage_kernel -- one wave per row, 16-B loads with 8 per lane in flight: the degree (numpy's
//    pairwise sum: rows of integer values take the exact strided sum, any other row the recursion's
//    plan below), D^-1/2, and the row's structural nonzeros (w != 0) in column order, the first
//    kLapdCap of them staged as (column, w) pairs.  It also zeroes the next launch's look-back words.
//  lapd_emit_kernel -- tiles of 256 rows in ticket order: each row's Laplacian nonzeros from its staged
//    pairs and the diagonal (one thread per row; a row with more than kLapdCap structural nonzeros is
//    re-read from W by the whole workgroup), a block scan, and the tile's count published for a
//    decoupled look-back over the tiles (CUB-style: wave 0 sums its predecessors' aggregates until an
//    inclusive prefix), so the row pointer and the CSR come out of the one launch with no scan pass.
//    Workgroups take tiles by an atomic ticket, so every tile a workgroup waits on is already running.
//    (One wave per row with the look-back over rows took 124 us at C3: the chain of inclusive prefixes
//    advanced 64 rows per round trip.)
//
// Values: lapd_value below, the reference's elementwise arithmetic; an entry with w = 0 off the
// diagonal is exactly zero in every mode (D^-1/2 is finite), so only the structural nonzeros and the
// diagonal can be stored -- the CSR is the np.flatnonzero order of the dense L (sampler.py:22-28).
constexpr int kLapdCap = 127;  // staged structural nonzeros per row (+ the diagonal: two 64-lane rounds)

// numpy's pairwise sum of a dense row, leaves and combine order from the host-built plan (all rows
// have the same length): the 8 lanes of group l % 8 sum leaf l with numpy's accumulators r_j = a[j],
// a[j + 8], ..., folded ((r0 + r1) + (r2 + r3)) + ((r4 + r5) + (r6 + r7)) plus the leaf's tail; lane 0
// combines the leaf sums with the recorded post-order program.  Every lane returns the sum.
constexpr int kPwPlanLeaves = 64;  // rows of up to 64 leaves: n <= 8192
struct PwPlan {
    int32_t nl;                      // leaves
    int32_t nprog;                   // program tokens
    int32_t off[kPwPlanLeaves];      // leaf l: a[off, off + len)
    int32_t len[kPwPlanLeaves];
    int8_t prog[2 * kPwPlanLeaves];  // post-order: >= 0 push leaf sum, -1 pop two, push (left + right)
};

static bool pw_plan_build(int64_t n, PwPlan &p) {
    p.nl = 0;
    p.nprog = 0;
    if (n <= 128) return false;  // (one leaf: wave_np_pairwise's own path)
    struct F { int64_t o, m; int state; };
    F st[64];
    int sp = 0;
    st[0] = {0, n, 0};
    while (sp >= 0) {
        F &f = st[sp];
        if (f.m <= 128) {
            if (p.nl >= kPwPlanLeaves) return false;
            p.off[p.nl] = (int32_t)f.o;
            p.len[p.nl] = (int32_t)f.m;
            p.prog[p.nprog++] = (int8_t)p.nl;
            ++p.nl;
            --sp;
            continue;
        }
        int64_t n2 = f.m / 2;
        n2 -= n2 % 8;
        if (f.state == 0) {
            f.state = 1;
            st[sp + 1] = {f.o, n2, 0};
            ++sp;
        } else if (f.state == 1) {
            f.state = 2;
            st[sp + 1] = {f.o + n2, f.m - n2, 0};
            ++sp;
        } else {
            p.prog[p.nprog++] = -1;
            --sp;
        }
    }
    return true;
}

// (stk: the wave's LDS stack of the combine, kPwPlanLeaves doubles -- not a per-lane array, which would be
// private memory)
__device__ double plan_row_sum(const double *a, const PwPlan &plan, double *sums, double *stk, int lane) {
    const int g = lane >> 3, j = lane & 7;
    for (int l0 = 0; l0 < plan.nl; l0 += 8) {
        const int l = l0 + g;
        double r = 0.0;
        int32_t off = 0, len = 0, nb = 0;
        if (l < plan.nl) {
            off = plan.off[l];
            len = plan.len[l];
            nb = len - (len % 8);  // (leaves of a split row hold >= 64 values)
            r = a[off + j];
            for (int32_t q = 8 + j; q < nb; q += 8) r += a[off + q];
        }
        const double r1 = __shfl_xor(r, 1, 64);
        const double p01 = (j & 1) ? r1 + r : r + r1;       // (r0 + r1), (r2 + r3), ...
        const double p23 = __shfl_xor(p01, 2, 64);
        const double q = (j & 2) ? p23 + p01 : p01 + p23;  // ((r0 + r1) + (r2 + r3)), ...
        const double q4 = __shfl_xor(q, 4, 64);
        double res = (j & 4) ? q4 + q : q + q4;
        if (j == 0 && l < plan.nl) {
            for (int32_t t = nb; t < len; ++t) res += a[off + t];
            sums[l] = res;
        }
    }
    __builtin_amdgcn_wave_barrier();
    double d = 0.0;
    if (lane == 0) {
        int sp = -1;
        for (int t = 0; t < plan.nprog; ++t) {
            const int tok = plan.prog[t];
            if (tok >= 0) {
                stk[++sp] = sums[tok];
            } else {
                const double rgt = stk[sp--];
                stk[sp] = stk[sp] + rgt;
            }
        }
        d = stk[0];
    }
    __builtin_amdgcn_wave_barrier();
    return __shfl(d, 0, 64);
}

__device__ inline double lapd_value(int32_t mode, int64_t i, int64_t j, double w, const double *deg,
                                    const double *dinv) {
    switch (mode) {
        case GRF_LAP_COMBINATORIAL: return (i == j ? deg[i] : 0.0) - w;
        case GRF_LAP_NONE: return w;
        default: return (i == j ? 1.0 : 0.0) - (dinv[i] * w) * dinv[j];
    }
}

// the row's elements in column order, up to two per lane per round: lane-ordered positions by ballots
struct RowStager {
    int32_t *col;
    double *val;
    int32_t cnt;  // wave-uniform running count
    __device__ void put(bool nz0, int64_t c0, double v0, bool nz1, int64_t c1, double v1, int lane) {
        const uint64_t m0 = __ballot(nz0), m1 = __ballot(nz1);
        const uint64_t lt = (1ull << lane) - 1ull;
        int32_t p = cnt + __popcll(m0 & lt) + __popcll(m1 & lt);
        if (nz0) {
            if (p < kLapdCap) { col[p] = (int32_t)c0; val[p] = v0; }
            ++p;
        }
        if (nz1 && p < kLapdCap) { col[p] = (int32_t)c1; val[p] = v1; }
        cnt += __popcll(m0) + __popcll(m1);
    }
};

struct IntSum {  // per-lane exact-integer-sum state of numpy's shortcut (wave_np_pairwise)
    bool integral = true, nonzero = false;
    double s = 0.0;
    __device__ void add(double v) {
        integral = integral && v == rint(v) && fabs(v) <= 1048576.0;
        nonzero = nonzero || v != 0.0;
        s += v;
    }
};

__global__ __launch_bounds__(256) void lapd_stage_kernel(int64_t n, const double *W, int32_t mode, PwPlan plan,
                                                         double *deg, double *dinv, int32_t *scnt, int32_t *scol,
                                                         double *sval, uint64_t *flags, uint32_t *ticket) {
    __shared__ double sums[4][kPwPlanLeaves], stk[4][kPwPlanLeaves];
    __shared__ PwScratch leaves[4];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int64_t i = (int64_t)blockIdx.x * 4 + wave;  // one wave per row
    if (i >= n) return;
    const double *a = W + i * n;
    const int h = (int)(((uintptr_t)a >> 3) & 1);  // the row starts mid-16-B: element 0 alone
    const int64_t npair = (n - h) >> 1;
    const bool tail = ((n - h) & 1) != 0;
    const double2 *pa = reinterpret_cast<const double2 *>(a + h);
    RowStager st{scol + i * kLapdCap, sval + i * kLapdCap, 0};
    IntSum is;
    if (h) {
        const double v = lane == 0 ? a[0] : 0.0;
        if (lane == 0) is.add(v);
        st.put(lane == 0 && v != 0.0, 0, v, false, 0, 0.0, lane);
    }
    constexpr int kU = 16;  // 16-B loads in flight per lane (C3: a row in two rounds)
    for (int64_t p0 = 0; p0 < npair; p0 += 64 * kU) {
        double2 v[kU];
#pragma unroll
        for (int u = 0; u < kU; ++u) {
            const int64_t p = p0 + u * 64 + lane;
            v[u] = p < npair ? pa[p] : double2{0.0, 0.0};
        }
#pragma unroll
        for (int u = 0; u < kU; ++u) {
            if (p0 + u * 64 >= npair) break;  // (uniform)
            const int64_t c0 = h + 2 * (p0 + u * 64 + lane);
            is.add(v[u].x);
            is.add(v[u].y);
            st.put(v[u].x != 0.0, c0, v[u].x, v[u].y != 0.0, c0 + 1, v[u].y, lane);
        }
    }
    if (tail) {
        const double v = lane == 0 ? a[n - 1] : 0.0;
        if (lane == 0) is.add(v);
        st.put(lane == 0 && v != 0.0, n - 1, v, false, 0, 0.0, lane);
    }
    double d;
    if (__all(is.integral) && __any(is.nonzero)) {
        // every partial sum of any order is an exact integer (< 2^53): the recursion's result, bit for bit
        d = wave_sum(is.s);
    } else {
        d = plan.nl > 0 ? plan_row_sum(a, plan, sums[wave], stk[wave], lane) : wave_np_pairwise(a, n, &leaves[wave]);
    }
    if (lane == 0) {
        deg[i] = d;
        if (mode == GRF_LAP_NUMPY) dinv[i] = d > 0.0 ? 1.0 / sqrt(d) : 0.0;
        else dinv[i] = 1.0 / sqrt(d > 0.0 ? d : 1.0);
        scnt[i] = st.cnt;
        flags[i] = 0;
        if (i == 0) *ticket = 0u;
    }
}

typedef __attribute__((address_space(1))) uint64_t gu64_t;
constexpr uint64_t kLbAgg = 1ull << 62, kLbIncl = 2ull << 62, kLbVal = (1ull << 62) - 1ull;

// Decoupled look-back (R2 granules: the 8-byte word {status, value} is the whole hand-off, written and
// polled by relaxed agent-scope atomics; cdna_hip_programming.md Guideline 16).  Publishes this row's
// count, returns the exclusive prefix of the counts before it.  The spin on an unpublished word has no
// bound: tiles take their tickets when they start, so every predecessor of a polling tile is resident (or
// done) and publishes without waiting on anything later -- a bounded spin could only turn a slow
// predecessor (preempted, or starved beside another queue) into a silently wrong row pointer.
__device__ int64_t lookback(uint64_t *flags, int64_t i, int64_t c, int lane) {
    gu64_t *f = (gu64_t *)flags;
    if (lane == 0) __hip_atomic_store(f + i, (i == 0 ? kLbIncl : kLbAgg) | (uint64_t)c, __ATOMIC_RELAXED,
                                      __HIP_MEMORY_SCOPE_AGENT);
    if (i == 0) return 0;
    int64_t excl = 0, pos = i - 1;
    for (;;) {
        const int64_t idx = pos - lane;
        uint64_t w = kLbIncl;  // (before row 0: an inclusive zero)
        if (idx >= 0) {
            for (;;) {
                w = __hip_atomic_load(f + idx, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if ((w >> 62) != 0) break;
                __builtin_amdgcn_s_sleep(1);
            }
        }
        const uint64_t incl = __ballot((w >> 62) == 2);
        const int64_t v = (int64_t)(w & kLbVal);
        if (incl) {
            const int k = __ffsll((long long)incl) - 1;
            excl += wave_sum<int64_t>(lane <= k ? v : 0);
            break;
        }
        excl += wave_sum<int64_t>(v);
        pos -= 64;
    }
    if (lane == 0) __hip_atomic_store(f + i, kLbIncl | (uint64_t)(excl + c), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return excl;
}

// A row with more structural nonzeros than the stage holds, by the whole workgroup (256 threads) over W's
// row: counts (EMIT = false, the total in every thread) or writes from `o` in column order.  A pass takes
// 2048 columns, 8 consecutive ones per thread (four 16-B loads in flight), places by a block scan of the
// threads' counts: Cora's 168-neighbour rows are 2 passes (were 11 chunks of 256 with two barriers each).
constexpr int kLapdRowPer = 8;

template <bool EMIT>
__device__ int64_t lapd_dense_row(int64_t i, int64_t n, int32_t mode, const double *W, const double *deg,
                                  const double *dinv, int64_t o, int32_t *l_idx, double *l_val, int64_t l_cap,
                                  int64_t *scan) {
    const int tid = threadIdx.x;
    const double *a = W + i * n;
    int64_t total = 0;
    for (int64_t j0 = 0; j0 < n; j0 += 256 * kLapdRowPer) {
        const int64_t jb = j0 + (int64_t)tid * kLapdRowPer;
        double v[kLapdRowPer];
#pragma unroll
        for (int q = 0; q < kLapdRowPer; ++q) {
            const int64_t j = jb + q;
            const double w = j < n ? a[j] : 0.0;
            v[q] = j < n && (w != 0.0 || j == i) ? lapd_value(mode, i, j, w, deg, dinv) : 0.0;
        }
        int64_t c = 0;
#pragma unroll
        for (int q = 0; q < kLapdRowPer; ++q) c += v[q] != 0.0 ? 1 : 0;
        int64_t chunk;
        int64_t pos = o + total + block_exclusive_scan<int64_t>(c, scan, &chunk);
        if (EMIT) {
#pragma unroll
            for (int q = 0; q < kLapdRowPer; ++q) {
                if (v[q] != 0.0) {
                    if (pos < l_cap) {
                        l_idx[pos] = (int32_t)(jb + q);
                        l_val[pos] = v[q];
                    }
                    ++pos;
                }
            }
        }
        total += chunk;
    }
    return total;
}

// Tiles of 64 rows in ticket order, 256 threads: every staged pair of the tile's rows is one work item
// (rows laid end to end, each followed by one item for its diagonal), so the items' dependent loads
// (pair -> D^-1/2 of its column) run side by side instead of row after row.  Pass 1: values, per-row
// counts (LDS adds of integers), rows past the stage by the whole workgroup; a block scan of the counts;
// the tile total published for the look-back over tiles (wave 0); pass 2: the items again, their places
// from a running scan of the nonzero flags in item order.  An inserted diagonal (no explicit w_ii) goes
// after the row's pairs with columns < i, which is where the items of columns > i are shifted by one.
// (Measured: one wave per row with the look-back over rows took 124 us at C3, the chain of inclusive
// prefixes advancing 64 rows per round trip; one thread per row of a 256-row tile 169 us, a hub row's
// pairs walked by one thread.)
constexpr int kLapdTileRows = 64;

__global__ __launch_bounds__(256) void lapd_emit_kernel(int64_t n, const double *W, int32_t mode, const double *deg,
                                                        const double *dinv, const int32_t *scnt, const int32_t *scol,
                                                        const double *sval, uint64_t *flags, uint32_t *ticket,
                                                        int64_t *l_ptr, int32_t *l_idx, double *l_val, int64_t l_cap) {
    constexpr int R = kLapdTileRows;
    __shared__ int32_t s_seg[R + 1];  // items before row r (pairs + 1 diagonal item per staged row)
    __shared__ int32_t s_cnt[R];      // nonzeros of row r
    __shared__ int32_t s_expl[R];     // row r has an explicit diagonal pair
    __shared__ int32_t s_dnz[R];      // row r's inserted diagonal is a nonzero
    __shared__ int32_t s_off[R + 1];  // nonzeros of the tile before row r
    __shared__ int32_t s_lt[R];       // nonzero pairs of row r with columns < r0 + r
    __shared__ int32_t s_nzp[R + 1];  // nonzero pairs (diagonal items excluded) of the tile before row r
    __shared__ int32_t s_wsum[4];
    __shared__ int64_t s_rscan[5];
    __shared__ int64_t s_excl;
    __shared__ uint32_t s_tile;
    __shared__ uint64_t s_long;  // rows past the stage (bit r)
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    if (tid == 0) s_tile = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (tid < R) {
        s_cnt[tid] = 0;
        s_expl[tid] = 0;
        s_lt[tid] = 0;
    }
    __syncthreads();
    const int64_t tile = s_tile, r0 = tile * R;
    if (r0 >= n) return;
    // rows -> item segments (wave 0, one lane per row)
    if (wave == 0) {
        const int64_t i = r0 + lane;
        const int32_t c = i < n ? scnt[i] : 0;
        const bool lng = i < n && c > kLapdCap;
        const int32_t seg = (i < n && !lng) ? c + 1 : 0;
        const int32_t inc = wave_inclusive_scan<int32_t>(seg);
        s_seg[lane + 1] = inc;
        if (lane == 0) s_seg[0] = 0;
        const uint64_t lm = __ballot(lng);
        if (lane == 0) s_long = lm;
    }
    __syncthreads();
    const int32_t E = s_seg[R];
    // the item e -> (row r, position k in the row's segment): upper bound in s_seg
    auto locate = [&](int32_t e, int &r, int32_t &k) {
        int lo = 0, hi = R;  // s_seg[lo] <= e < s_seg[hi]
#pragma unroll
        for (int st = 0; st < 6; ++st) {
            const int mid = (lo + hi) >> 1;
            if (s_seg[mid] <= e) lo = mid;
            else hi = mid;
        }
        r = lo;
        k = e - s_seg[lo];
    };
    // pass 1a: the pairs (explicit diagonals flagged, nonzeros counted)
    for (int32_t e = tid; e < E; e += 256) {
        int r;
        int32_t k;
        locate(e, r, k);
        const int64_t i = r0 + r;
        const int32_t c = s_seg[r + 1] - s_seg[r] - 1;
        if (k < c) {
            const int64_t col = scol[i * kLapdCap + k];
            const double u = lapd_value(mode, i, col, sval[i * kLapdCap + k], deg, dinv);
            if (col == i) s_expl[r] = 1;
            if (u != 0.0) {
                atomicAdd(&s_cnt[r], 1);
                if (col < i) atomicAdd(&s_lt[r], 1);
            }
        }
    }
    __syncthreads();
    // pass 1b: the inserted diagonals (w_ii = 0) of rows with no explicit one
    if (tid < R) {
        const int64_t i = r0 + tid;
        const bool staged = s_seg[tid + 1] > s_seg[tid];
        const bool dnz = staged && !s_expl[tid] && lapd_value(mode, i, i, 0.0, deg, dinv) != 0.0;
        s_dnz[tid] = dnz ? 1 : 0;
        if (dnz) s_cnt[tid] += 1;
    }
    // rows past the stage: the whole workgroup over W's row (uniform loop)
    for (uint64_t m = s_long; m; m &= m - 1) {
        const int r = __ffsll((long long)m) - 1;
        const int64_t t = lapd_dense_row<false>(r0 + r, n, mode, W, deg, dinv, 0, nullptr, nullptr, 0, s_rscan);
        if (tid == 0) s_cnt[r] = (int32_t)t;
    }
    __syncthreads();
    if (wave == 0) {
        const int32_t cr = s_cnt[lane];
        const int32_t inc = wave_inclusive_scan<int32_t>(cr);
        s_off[lane + 1] = inc;
        if (lane == 0) s_off[0] = 0;
        const bool lng = (s_long >> lane) & 1;
        const int32_t pz = wave_inclusive_scan<int32_t>(lng ? 0 : cr - s_dnz[lane]);
        s_nzp[lane + 1] = pz;
        if (lane == 0) s_nzp[0] = 0;
        const int64_t total = __shfl(inc, 63, 64);
        const int64_t ex = lookback(flags, tile, total, lane);
        if (lane == 0) s_excl = ex;
    }
    __syncthreads();
    const int64_t base = s_excl;
    if (tid < R && r0 + tid < n) {
        const int64_t i = r0 + tid;
        l_ptr[i] = base + s_off[tid];
        if (i == n - 1) l_ptr[n] = base + s_off[tid + 1];
    }
    // pass 2: places by a running scan of the pairs' nonzero flags in item order (diagonal items: 0)
    int32_t run = 0;  // nonzero pairs before this chunk
    for (int32_t e0 = 0; e0 < E; e0 += 256) {
        const int32_t e = e0 + tid;
        int r = 0;
        int32_t k = 0;
        bool nz = false;
        int64_t col = 0;
        double u = 0.0;
        if (e < E) {
            locate(e, r, k);
            const int32_t c = s_seg[r + 1] - s_seg[r] - 1;
            if (k < c) {
                const int64_t i = r0 + r;
                col = scol[i * kLapdCap + k];
                u = lapd_value(mode, i, col, sval[i * kLapdCap + k], deg, dinv);
                nz = u != 0.0;
            }
        }
        const uint64_t m = __ballot(nz);
        __syncthreads();  // (the previous chunk's wave sums are read)
        if (lane == 0) s_wsum[wave] = __popcll(m);
        __syncthreads();
        int32_t before = run, chunk = 0;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            before += q < wave ? s_wsum[q] : 0;
            chunk += s_wsum[q];
        }
        if (nz) {
            const int64_t i = r0 + r;
            // this pair's rank among the tile's nonzero pairs, made row-local, placed after the row's own
            // offset and after the inserted diagonal when its column is past i
            const int32_t rank = before + __popcll(m & ((1ull << lane) - 1ull));
            const int64_t pos = base + s_off[r] + (rank - s_nzp[r]) + ((s_dnz[r] && col > i) ? 1 : 0);
            if (pos < l_cap) {
                l_idx[pos] = (int32_t)col;
                l_val[pos] = u;
            }
        }
        run += chunk;
    }
    // the inserted diagonals: after the row's nonzero pairs with columns < i
    if (tid < R && s_dnz[tid]) {
        const int64_t i = r0 + tid;
        const int64_t pos = base + s_off[tid] + s_lt[tid];
        if (pos < l_cap) {
            l_idx[pos] = (int32_t)i;
            l_val[pos] = lapd_value(mode, i, i, 0.0, deg, dinv);
        }
    }
    // rows past the stage: the whole workgroup fills from the row's offset
    for (uint64_t m = s_long; m; m &= m - 1) {
        const int r = __ffsll((long long)m) - 1;
        lapd_dense_row<true>(r0 + r, n, mode, W, deg, dinv, base + s_off[r], l_idx, l_val, l_cap, s_rscan);
    }
}

}  // namespace grf

using namespace grf;

extern "C" {
#pragma GCC visibility push(default)

size_t grf_laplacian_csr_workspace_bytes(int64_t n) {
    const size_t cnt_bytes = ((size_t)(n > 0 ? n : 1) * sizeof(int32_t) + 255) & ~(size_t)255;
    return cnt_bytes + scan_ws_bytes(n);
}

// dense workspace: dinv [n] f64 | staged counts [n] i32 | staged columns [n x cap] i32 | staged values
// [n x cap] f64 | look-back words [n] u64 | ticket (256 B)
static size_t al256(size_t b) { return (b + 255) & ~(size_t)255; }
size_t grf_laplacian_dense_workspace_bytes(int64_t n) {
    const size_t nn = (size_t)(n > 0 ? n : 1);
    return al256(nn * sizeof(double)) + al256(nn * sizeof(int32_t)) + al256(nn * kLapdCap * sizeof(int32_t)) +
           al256(nn * kLapdCap * sizeof(double)) + al256(nn * sizeof(uint64_t)) + 256;
}

int32_t grf_laplacian_csr(int64_t n, const int64_t *a_ptr, const int32_t *a_idx, const double *a_val, int32_t mode,
                          int64_t *l_ptr, int32_t *l_idx, double *l_val, int64_t l_cap, double *deg, double *dinv,
                          void *workspace, size_t workspace_bytes, grf_stream_t stream) {
    GRF_REQUIRE(n >= 0 && a_ptr && l_ptr && deg && dinv, GRF_EINVAL, "grf_laplacian_csr: bad arguments");
    GRF_REQUIRE(mode == GRF_LAP_SCIPY, GRF_EUNSUPPORTED,
                "grf_laplacian_csr: only GRF_LAP_SCIPY is defined for CSR input (got %d)", mode);
    const size_t cnt_bytes = ((size_t)(n > 0 ? n : 1) * sizeof(int32_t) + 255) & ~(size_t)255;
    GRF_REQUIRE(workspace_bytes >= cnt_bytes + scan_ws_bytes(n), GRF_EINVAL,
                "grf_laplacian_csr: workspace too small (%zu < %zu)", workspace_bytes, cnt_bytes + scan_ws_bytes(n));
    hipStream_t st = S(stream);
    int32_t *cnt = (int32_t *)workspace;
    if (n == 0) {
        GRF_CHECK_HIP(hipMemsetAsync(l_ptr, 0, sizeof(int64_t), st));
        return GRF_OK;
    }
    // eight rows per wave (GRF_LAP_WAVE_ROWS=1: one row per wave, for A/B runs)
    static const bool wave_rows = [] {
        const char *e = getenv("GRF_LAP_WAVE_ROWS");
        return e && atoi(e) != 0;
    }();
    const unsigned gw = (unsigned)cdiv<int64_t>(n, wave_rows ? 4 : 32);
    GRF_REQUIRE_GRID(gw, 256, "lap_deg_kernel");
    if (wave_rows) lap_deg_kernel<<<gw, 256, 0, st>>>(n, a_ptr, a_val, deg, dinv);
    else lap_deg_group_kernel<<<gw, 256, 0, st>>>(n, a_ptr, a_val, deg, dinv);
    GRF_CHECK_LAUNCH("lap_deg_kernel");
    if (wave_rows)
        lap_row_kernel<false><<<gw, 256, 0, st>>>(n, a_ptr, a_idx, a_val, deg, dinv, cnt, nullptr, nullptr, nullptr, 0);
    else
        lap_row_group_kernel<false><<<gw, 256, 0, st>>>(n, a_ptr, a_idx, a_val, deg, dinv, cnt, nullptr, nullptr,
                                                        nullptr, 0);
    GRF_CHECK_LAUNCH("lap_row_kernel<count>");
    int32_t rc = scan_counts_i32(n, cnt, l_ptr, (char *)workspace + cnt_bytes, workspace_bytes - cnt_bytes, st);
    if (rc != GRF_OK) return rc;
    if (wave_rows)
        lap_row_kernel<true><<<gw, 256, 0, st>>>(n, a_ptr, a_idx, a_val, deg, dinv, nullptr, l_ptr, l_idx, l_val, l_cap);
    else
        lap_row_group_kernel<true><<<gw, 256, 0, st>>>(n, a_ptr, a_idx, a_val, deg, dinv, nullptr, l_ptr, l_idx, l_val,
                                                       l_cap);
    GRF_CHECK_LAUNCH("lap_row_kernel<fill>");
    return GRF_OK;
}

int32_t grf_laplacian_dense(int64_t n, const double *W, int32_t mode, int64_t *l_ptr, int32_t *l_idx, double *l_val,
                            int64_t l_cap, double *deg, void *workspace, size_t workspace_bytes, grf_stream_t stream) {
    GRF_REQUIRE(n >= 0 && W && l_ptr && deg, GRF_EINVAL, "grf_laplacian_dense: bad arguments");
    GRF_REQUIRE(mode == GRF_LAP_NUMPY || mode == GRF_LAP_NUMPY_SAFE || mode == GRF_LAP_COMBINATORIAL ||
                    mode == GRF_LAP_NONE,
                GRF_EINVAL, "grf_laplacian_dense: bad mode %d", mode);
    GRF_REQUIRE(((uintptr_t)W & 7) == 0, GRF_EINVAL, "grf_laplacian_dense: W must be 8-byte aligned");
    GRF_REQUIRE(n < INT32_MAX, GRF_EINVAL, "grf_laplacian_dense: n must fit int32 column indices");
    GRF_REQUIRE(workspace_bytes >= grf_laplacian_dense_workspace_bytes(n) && ((uintptr_t)workspace & 255) == 0,
                GRF_EINVAL, "grf_laplacian_dense: workspace too small or not 256-byte aligned");
    hipStream_t st = S(stream);
    if (n == 0) {
        GRF_CHECK_HIP(hipMemsetAsync(l_ptr, 0, sizeof(int64_t), st));
        return GRF_OK;
    }
    const size_t nn = (size_t)n;
    char *w = (char *)workspace;
    double *dinv = (double *)w;
    w += al256(nn * sizeof(double));
    int32_t *scnt = (int32_t *)w;
    w += al256(nn * sizeof(int32_t));
    int32_t *scol = (int32_t *)w;
    w += al256(nn * kLapdCap * sizeof(int32_t));
    double *sval = (double *)w;
    w += al256(nn * kLapdCap * sizeof(double));
    uint64_t *flags = (uint64_t *)w;
    w += al256(nn * sizeof(uint64_t));
    uint32_t *ticket = (uint32_t *)w;
    PwPlan plan;
    if (!pw_plan_build(n, plan)) plan.nl = 0;
    const unsigned g = (unsigned)cdiv<int64_t>(n, 4);
    GRF_REQUIRE_GRID(g, 256, "lapd_stage_kernel");
    lapd_stage_kernel<<<g, 256, 0, st>>>(n, W, mode, plan, deg, dinv, scnt, scol, sval, flags, ticket);
    GRF_CHECK_LAUNCH("lapd_stage_kernel");
    const unsigned gt = (unsigned)cdiv<int64_t>(n, kLapdTileRows);
    lapd_emit_kernel<<<gt, 256, 0, st>>>(n, W, mode, deg, dinv, scnt, scol, sval, flags, ticket, l_ptr, l_idx, l_val,
                                        l_cap);
    GRF_CHECK_LAUNCH("lapd_emit_kernel");
    return GRF_OK;
}

}  // extern "C"
