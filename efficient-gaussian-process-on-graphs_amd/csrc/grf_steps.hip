// grf_steps.hip -- visit slots -> per-step occupancy rows -> feature rows Phi.
//
// Reference behaviour replaced (paths under the reference checkout):
//   step_accumulators[step][(start, cur)] += load, merged and normalised:
//     efficient_graph_gp_sparse/random_walk_samplers_sparse/sparse_sampler.py:47,107-130
//     efficient_graph_gp/random_walk_samplers/sampler.py:47,137-146,188-203
//   Phi = sum_l f_l M_l (scipy CSR adds drop exact zeros):
//     efficient_graph_gp_sparse/graph_kernels_sparse/fast_grf_kernel_general.py:47-52
//
// Bit-exactness: every (source, step, node) value is the left-to-right sum of
// the loads in walk order starting from 0.0 (dict `+=`), then divided by m
// (dense sampler) or multiplied by 1/m (scipy), and Phi entries are summed in
// step order starting from 0.0 -- the orders the reference uses.  Sorting
// (node, walk) keys in LDS gives those orders without atomics.
#include <algorithm>

#include <stdlib.h>

#include "grf_block.h"
#include "grf_philox.h"

namespace grf {

__device__ inline double normalise(double acc, int32_t norm, int64_t m) {
    return norm == GRF_NORM_DIV ? acc / (double)m : acc * (1.0 / (double)m);
}
// The same with 1 / m computed once per workgroup: NORM_DIV divides through Divisor (grf_philox.h: the
// correctly rounded quotient, same bits as acc / m), NORM_MUL_RECIP multiplies by the rounded reciprocal
struct Norm {
    Divisor d;
    double inv;
    int32_t norm;
    __device__ Norm(int32_t norm_, int64_t m_) : d((double)m_), inv(1.0 / (double)m_), norm(norm_) {}
    __device__ double operator()(double acc) const { return norm == GRF_NORM_DIV ? d(acc) : acc * inv; }
};

// --------------------------------------------------------------- grf_steps
// one workgroup per (source, step) group of m slots; P = next_pow2(m) keys in LDS
__global__ __launch_bounds__(256) void steps_kernel(int64_t m, int32_t norm, int32_t P,
                                                    const int32_t *__restrict__ slot_node,
                                                    const double *__restrict__ slot_load,
                                                    int32_t *__restrict__ step_cnt, int32_t *__restrict__ step_idx,
                                                    double *__restrict__ step_val) {
    extern __shared__ __attribute__((aligned(16))) uint64_t key[];
    int32_t *scratch = reinterpret_cast<int32_t *>(key + P);  // 17 ints after the keys
    const int64_t g = blockIdx.x;
    const int32_t *nd = slot_node + g * m;
    const double *ld = slot_load + g * m;
    for (int t = threadIdx.x; t < P; t += blockDim.x) {
        uint64_t k = ~0ull;
        if (t < m) {
            const int32_t v = nd[t];
            if (v >= 0) k = ((uint64_t)(uint32_t)v << 32) | (uint32_t)t;
        }
        key[t] = k;
    }
    __syncthreads();
    block_bitonic_sort<uint64_t>(key, P);
    // contiguous chunk per thread
    const int T = blockDim.x;
    const int per = P >= T ? P / T : 1;
    const int i0 = threadIdx.x * per;
    int c = 0;
    for (int i = i0; i < i0 + per && i < P; ++i) {
        const uint64_t k = key[i];
        if (k != ~0ull && (i == 0 || (key[i - 1] >> 32) != (k >> 32))) ++c;
    }
    int32_t total;
    int32_t rank = block_exclusive_scan<int32_t>(c, scratch, &total);
    for (int i = i0; i < i0 + per && i < P; ++i) {
        const uint64_t k = key[i];
        if (k == ~0ull || (i > 0 && (key[i - 1] >> 32) == (k >> 32))) continue;
        double acc = 0.0;
        int j = i;
        do {
            acc += ld[(uint32_t)key[j]];
            ++j;
        } while (j < P && (key[j] >> 32) == (k >> 32));
        step_idx[g * m + rank] = (int32_t)(k >> 32);
        step_val[g * m + rank] = normalise(acc, norm, m);
        ++rank;
    }
    if (threadIdx.x == 0) step_cnt[g] = total;
}

// ------------------------------------------------------------------ grf_phi
// one wave per source: L-way merge of the sorted step rows (L <= 64)
__global__ __launch_bounds__(256) void phi_merge_kernel(int64_t n_src, int64_t m, int32_t L, int32_t Lf,
                                                        const int32_t *__restrict__ step_cnt,
                                                        const int32_t *__restrict__ step_idx,
                                                        const double *__restrict__ step_val,
                                                        const double *__restrict__ f, int64_t cap,
                                                        int32_t *__restrict__ phi_cnt, int32_t *__restrict__ phi_idx,
                                                        double *__restrict__ phi_val, float *__restrict__ phi_val32) {
    const int64_t s = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (s >= n_src) return;
    const int lane = threadIdx.x & 63;
    int64_t pos = 0, end = 0;
    double fl = 0.0;
    if (lane < Lf) {
        pos = (s * L + lane) * m;
        end = pos + step_cnt[s * L + lane];
        fl = f[lane];
    }
    int32_t head = pos < end ? step_idx[pos] : INT32_MAX;
    int64_t out = 0;
    const int64_t obase = s * cap;
    for (;;) {
        int32_t mn = head;
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) mn = min(mn, __shfl_xor(mn, off, 64));
        if (mn == INT32_MAX) break;
        const bool match = (head == mn);
        const double t = match ? fl * step_val[pos] : 0.0;
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
            if (lane == 0 && out < cap) {
                phi_idx[obase + out] = mn;
                phi_val[obase + out] = acc;
                if (phi_val32) phi_val32[obase + out] = (float)acc;
            }
            ++out;
        }
        if (match) {
            ++pos;
            head = pos < end ? step_idx[pos] : INT32_MAX;
        }
    }
    if (lane == 0) phi_cnt[s] = (int32_t)(out < cap ? out : cap);
}

// ------------------------------------------------------------ grf_phi_fused
// One workgroup per source: the (node, step, walk) keys of all m*L visit slots are sorted
// in LDS; runs of (node, step) are the step entries (loads summed in walk order), runs of
// node the Phi entries (f_l * step value summed in step order).  The slots come from HBM
// (kWalk = false, grf_phi_fused) or from the source's own Philox walks run by the
// workgroup (kWalk = true, grf_walk_phi: no slot round trip through HBM).
constexpr int kPhiMaxPer = 16;  // sorted positions per thread (P <= 4096, 256 threads)

// kPer = P / blockDim.x sorted positions per thread; kT > 0: blockDim.x == kT, known at compile time
// (the sort network then unrolls into straight-line code)
template <bool kWalk, int kPer, typename KT, int kT = 0>
__global__ __launch_bounds__(256) void phi_fused_kernel(int64_t m, int32_t L, int32_t norm, int32_t P, int32_t wbits,
                                                        int32_t lbits, const int32_t *__restrict__ slot_node,
                                                        const double *__restrict__ slot_load,
                                                        const int64_t *__restrict__ g_ptr,
                                                        const int32_t *__restrict__ g_idx,
                                                        const double *__restrict__ g_val,
                                                        const unsigned char *__restrict__ g_aug, double p_halt, int32_t rule,
                                                        uint32_t k0, uint32_t k1, int64_t src_begin,
                                                        const double *__restrict__ f, int32_t Lf, int64_t cap,
                                                        int32_t *__restrict__ phi_cnt, int32_t *__restrict__ phi_idx,
                                                        double *__restrict__ phi_val, float *__restrict__ phi_val32,
                                                        int32_t *__restrict__ t_count, int64_t band_width,
                                                        int64_t n_cols, int64_t count_row0, int32_t sort_lds) {
    // LDS: ld [E] loads by slot (later the compacted step values), fl [Lf] the modulator,
    // scratch (2 x 16 ints), key [P] the sorted keys (later the compacted step keys).  32-bit
    // keys when (node, step, walk) fits 32 bits (C4 / C5): half the sort's LDS traffic and a
    // third of the footprint of the 64-bit layout with its separate head-value array.
    extern __shared__ __attribute__((aligned(16))) uint64_t smem[];
    const int E = (int)(m * L), T = kT > 0 ? kT : (int)blockDim.x, tid = (int)threadIdx.x;
    double *ld = reinterpret_cast<double *>(smem);             // [E]
    double *fl = ld + E;                                        // [Lf rounded up to even]
    int32_t *scratch = reinterpret_cast<int32_t *>(fl + ((Lf + 1) & ~1));  // [32]
    KT *key = reinterpret_cast<KT *>(scratch + 32);             // [P]
    const KT kNone = (KT)~(KT)0;
    const int64_t s = blockIdx.x;
    const Norm nrm(norm, m);
    const int sh = wbits + lbits;
    const KT wmask = (KT)(((KT)1 << wbits) - 1), lmask = (KT)(((KT)1 << lbits) - 1);
    auto make_key = [&](int32_t node, int l, int64_t w) {
        return (KT)(((KT)(uint32_t)node << sh) | ((KT)l << wbits) | (KT)w);
    };
    // the load slot l m + w of a key, in 32-bit arithmetic (m L <= 4096)
    const uint32_t mu = (uint32_t)m;
    auto slot_of = [&](KT k) -> uint32_t {
        return __umul24((uint32_t)((k >> wbits) & lmask), mu) + (uint32_t)(k & wmask);
    };

    for (int l = tid; l < Lf; l += T) fl[l] = f[l];
    // ---- slots -> keys
    if (kWalk) {
        for (int t = tid; t < P; t += T) key[t] = kNone;
        __syncthreads();
        const int64_t src = src_begin + s;
        for (int64_t w = tid; w < m; w += T) {
            auto visit = [&](int32_t l, int32_t node, double load) {
                if (l == 0) {
                    // every walk records (source, step 0) with load 1.0, a run of m equal slots whose
                    // sum is exactly m: one slot carries it (the same bits as the m-term sum) and the
                    // head thread no longer walks an m-long run
                    if (w == 0) {
                        key[0] = make_key(node, 0, 0);
                        ld[0] = (double)m;
                    }
                    return;
                }
                const uint32_t t = __umul24((uint32_t)l, mu) + (uint32_t)w;
                key[t] = make_key(node, l, w);
                ld[t] = load;
            };
            if (g_aug) philox_walk_aug(g_ptr, g_aug, src, (uint32_t)w, p_halt, L, rule, k0, k1, visit);
            else philox_walk(g_ptr, g_idx, g_val, src, (uint32_t)w, p_halt, L, rule, k0, k1, visit);
        }
    } else {
        const int32_t *nd = slot_node + s * E;
        const double *sl = slot_load + s * E;
        for (int t = tid; t < P; t += T) {
            KT k = kNone;
            if (t < E) {
                const int32_t v = nd[t];
                if (v >= 0) {
                    const int l = t / (int)m;
                    k = make_key(v, l, t - l * (int)m);
                    ld[t] = sl[t];
                }
            }
            key[t] = k;
        }
    }
    __syncthreads();
    if (sort_lds == 1) block_bitonic_sort<KT>(key, P);
    else if (sort_lds == 0) block_bitonic_sort_regs<KT, kPer, kT * kPer>(key, P);  // (P == kPer * blockDim.x)
    // (sort_lds == 2: no sort -- a TIMING-ONLY ablation, GRF_PHI_SORT_LDS=2; Phi is then wrong)

    // ---- step values of the (node, step) runs, kept in registers: loads in walk order from 0.0.
    //      Thread t owns the sorted positions [t kPer, (t + 1) kPer) and the runs whose first visit
    //      is among them; it scans its positions once, left to right, and records each run's value
    //      at the run's last position in the block (so the runs stay in sorted order).  Only a run
    //      still open at the block's end reads on into the next threads' positions (8 keys / loads
    //      per LDS round trip) -- one such loop per thread instead of one per head: the wave no
    //      longer runs the loop body once per position whenever any lane has a longer run there.
    //      (The source's step-0 run is one slot of load m, see the walk above.)
    const int i0 = tid * kPer;
    KT kq[kPer];
#pragma unroll
    for (int q = 0; q < kPer; ++q) kq[q] = key[i0 + q];
    const KT kprev = i0 > 0 ? key[i0 - 1] : kNone;
    KT hk_[kPer];  // the key of the run recorded at position q (kNone: none), its step value
    double hv_[kPer];
    int c = 0;
    KT run_k = kNone;
    double acc = 0.0;
    bool owned = false;  // the open run started in this block
#pragma unroll
    for (int q = 0; q < kPer; ++q) {
        const KT k = kq[q];
        const KT before = q == 0 ? kprev : kq[q - 1];
        hk_[q] = kNone;
        hv_[q] = 0.0;
        if (k == kNone) {
            owned = false;  // (sorted: only sentinels from here on)
            continue;
        }
        if ((before >> wbits) != (k >> wbits)) {  // a run's first visit: this thread owns it
            run_k = k;
            acc = 0.0 + ld[slot_of(k)];
            owned = true;
        } else if (owned) {
            acc += ld[slot_of(k)];
        }
        if (!owned) continue;  // (a run owned by an earlier thread)
        if (q < kPer - 1) {
            if ((kq[q + 1] >> wbits) == (k >> wbits)) continue;  // the run goes on in this block
        } else {
            // the block's last position: read on while the run continues
            const KT hk = k >> wbits;
            for (int j = i0 + kPer;; j += 8) {
                KT kk[8];
                double lv[8];
#pragma unroll
                for (int r = 0; r < 8; ++r) kk[r] = j + r < P ? key[j + r] : kNone;
#pragma unroll
                for (int r = 0; r < 8; ++r) lv[r] = (kk[r] >> wbits) == hk ? ld[slot_of(kk[r])] : 0.0;
                bool more = true;
#pragma unroll
                for (int r = 0; r < 8; ++r) {
                    if ((kk[r] >> wbits) == hk) acc += lv[r];  // keys are sorted: the run is contiguous
                    else more = false;
                }
                if (!more) break;
            }
        }
        hk_[q] = run_k;  // (static register indexing: q is the unrolled position)
        hv_[q] = nrm(acc);
        owned = false;
        ++c;
    }
    // ---- compact the step heads (sorted order): key -> key[rank], value -> ld[rank]
    int32_t n_heads;
    const int32_t rank0 = block_exclusive_scan_fast<int32_t>(c, scratch, &n_heads);  // (barrier: reads done)
    int32_t r0 = rank0;
#pragma unroll
    for (int q = 0; q < kPer; ++q) {
        if (hk_[q] != kNone) {
            key[r0] = hk_[q];
            ld[r0] = hv_[q];
            ++r0;
        }
    }
    __syncthreads();

    // ---- Phi entries at node run heads of the compacted list: f_l * value in step order
    const int per2 = (n_heads + T - 1) / T;  // <= kPer
    const int q0 = tid * per2;
    int emit = 0;
    double pv_[kPer];   // position qq's Phi value, its node (-1: no entry)
    int32_t pn_[kPer];
#pragma unroll
    for (int qq = 0; qq < kPer; ++qq) {
        pn_[qq] = -1;
        pv_[qq] = 0.0;
        const int q = q0 + qq;
        if (qq >= per2 || q >= n_heads) continue;
        const KT k = key[q];
        if (q > 0 && (key[q - 1] >> sh) == (k >> sh)) continue;  // not a node head
        double acc = 0.0;
        bool present = false;
        for (int j = q; j < n_heads && (key[j] >> sh) == (k >> sh); ++j) {
            const int l = (int)((key[j] >> wbits) & lmask);
            if (l < Lf) {
                const double t = fl[l] * ld[j];
                acc = present ? acc + t : 0.0 + t;
                present = true;
            }
        }
        if (present && acc != 0.0) {
            pv_[qq] = acc;  // (static register indexing)
            pn_[qq] = (int32_t)(k >> sh);
            ++emit;
        }
    }
    int32_t total;
    int32_t rank = block_exclusive_scan_fast<int32_t>(emit, scratch + 16, &total);
    const int64_t obase = s * cap;
#pragma unroll
    for (int qq = 0; qq < kPer; ++qq) {
        if (pn_[qq] >= 0) {
            if (rank < cap) {
                phi_idx[obase + rank] = pn_[qq];
                if (phi_val) phi_val[obase + rank] = pv_[qq];  // (NULL: the caller keeps the f32 copy only)
                if (phi_val32) phi_val32[obase + rank] = (float)pv_[qq];
                // the banded transpose's bucket counts of this row's entries (grf_transpose_banded_plan)
                if (t_count) atomicAdd(&t_count[((src_begin + s - count_row0) / band_width) * n_cols + pn_[qq]], 1);
            }
            ++rank;
        }
    }
    if (tid == 0) phi_cnt[s] = total < cap ? total : (int32_t)cap;
}

// ---------------------------------------------- augmented walk matrix (philox_walk_aug)
// The header and one record per entry e of the walk matrix (grf_philox.h).  The compact 16-byte
// format when tb + rb + lb <= 64 (tb: bits of the largest node id, lb: bits of a row length <= n, rb:
// bits of a row start <= nnz); every thread derives the same choice from nnz = g_ptr[n].
// A record needs only its entry (target v, weight) and v's row bounds, not the entry's own row: the
// entries are taken flat, grid-stride, kAugPer per thread with their loads in flight (was one wave per
// row: C5's ~11 entries per row left 53 of 64 lanes idle, 0.50 ms for 176 MB of records).
constexpr int kAugPer = 4;
__global__ __launch_bounds__(256) void walk_aug_kernel(int64_t n, int32_t tb, int32_t lb, int32_t allow16,
                                                       const int64_t *__restrict__ g_ptr,
                                                       const int32_t *__restrict__ g_idx,
                                                       const double *__restrict__ g_val, unsigned char *__restrict__ aug) {
    const int64_t nnz = g_ptr[n];
    const int rb = ceil_log2((uint64_t)nnz + 1) > 0 ? ceil_log2((uint64_t)nnz + 1) : 1;
    const bool compact = allow16 && tb + rb + lb <= 64;
    if (blockIdx.x == 0 && threadIdx.x == 0)
        *reinterpret_cast<int4 *>(aug) = make_int4(compact ? 1 : 0, tb, rb, 0);
    unsigned char *recs = aug + kAugHeader;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t e0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e0 < nnz; e0 += stride * kAugPer) {
        int32_t v[kAugPer];
        double w[kAugPer];
        int64_t rs[kAugPer], re[kAugPer];
#pragma unroll
        for (int u = 0; u < kAugPer; ++u) {
            const int64_t e = e0 + u * stride;
            v[u] = e < nnz ? g_idx[e] : 0;
            w[u] = e < nnz ? g_val[e] : 0.0;
        }
#pragma unroll
        for (int u = 0; u < kAugPer; ++u) {
            rs[u] = g_ptr[v[u]];
            re[u] = g_ptr[v[u] + 1];
        }
#pragma unroll
        for (int u = 0; u < kAugPer; ++u) {
            const int64_t e = e0 + u * stride;
            if (e >= nnz) break;
            const int64_t len = re[u] - rs[u];
            if (compact) {
                AugRec16 r;
                r.packed = (uint64_t)(uint32_t)v[u] | ((uint64_t)rs[u] << tb) | ((uint64_t)len << (tb + rb));
                r.w = w[u];
                reinterpret_cast<AugRec16 *>(recs)[e] = r;
            } else {
                AugRec r;
                r.v = v[u];
                r.rs = (int32_t)(uint32_t)rs[u];
                r.len = (int32_t)len;
                r.pad = 0;
                r.w = w[u];
                r.pad2 = 0.0;
                reinterpret_cast<AugRec *>(recs)[e] = r;
            }
        }
    }
}

__global__ __launch_bounds__(256) void steps_densify_kernel(int64_t n_src, int64_t m, int32_t L, int64_t n_cols,
                                                            const int32_t *__restrict__ step_cnt,
                                                            const int32_t *__restrict__ step_idx,
                                                            const double *__restrict__ step_val,
                                                            double *__restrict__ out) {
    const int64_t g = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (g >= n_src * L) return;
    const int lane = threadIdx.x & 63;
    const int64_t s = g / L;
    const int l = (int)(g - s * L);
    for (int64_t r = lane; r < step_cnt[g]; r += 64)
        out[(s * n_cols + step_idx[g * m + r]) * L + l] = step_val[g * m + r];
}

}  // namespace grf

using namespace grf;

extern "C" {
#pragma GCC visibility push(default)

int32_t grf_steps(int64_t n_src, int64_t m, int32_t L, int32_t norm, const int32_t *slot_node,
                  const double *slot_load, int32_t *step_cnt, int32_t *step_idx, double *step_val,
                  grf_stream_t stream) {
    GRF_REQUIRE(n_src >= 0 && m >= 1 && L >= 1 && slot_node && slot_load && step_cnt && step_idx && step_val,
                GRF_EINVAL, "grf_steps: bad arguments");
    GRF_REQUIRE(norm == GRF_NORM_DIV || norm == GRF_NORM_MUL_RECIP, GRF_EINVAL, "grf_steps: bad norm");
    GRF_REQUIRE(m <= 16384, GRF_EUNSUPPORTED, "grf_steps: walks_per_node > 16384 not supported by this build");
    if (n_src == 0) return GRF_OK;
    const int P = (int)next_pow2_u32((uint32_t)m);
    // threads per source: P / 4 up to 256, and at most one per walk -- measured (tools/walkphi_ab.py)
    // with the 12.9 KB LDS layout: m = 128 (C4) 128 threads 2.85 ms vs 256 3.28; m = 64 (C5) 64
    // threads 11.2 ms vs 128 13.0 (idle waves hold the source's slot while its walks run, and LDS
    // no longer caps the sources per CU); GRF_PHI_THREADS caps it for experiments
    static const int t_env = [] {
        const char *e = getenv("GRF_PHI_THREADS");
        const int v = e ? atoi(e) : 0;
        return (v == 64 || v == 128 || v == 256) ? v : 0;
    }();
    const int t_cap = t_env ? t_env : (int)std::min<int64_t>(256, std::max<int64_t>(64, ((m + 63) / 64) * 64));
    int T = P >= 512 ? 256 : (P >= 128 ? P / 2 : 64);
    while (T > t_cap && P / (T / 2) <= kPhiMaxPer) T /= 2;
    const size_t lds = (size_t)P * sizeof(uint64_t) + 128;
    GRF_REQUIRE_GRID((n_src * L), T, "steps_kernel");
    steps_kernel<<<(unsigned)(n_src * L), T, lds, S(stream)>>>(m, norm, P, slot_node, slot_load, step_cnt, step_idx,
                                                              step_val);
    GRF_CHECK_LAUNCH("steps_kernel");
    return GRF_OK;
}

int32_t grf_phi(int64_t n_src, int64_t m, int32_t L, const int32_t *step_cnt, const int32_t *step_idx,
                const double *step_val, const double *f, int32_t n_f, int64_t phi_cap, int32_t *phi_cnt,
                int32_t *phi_idx, double *phi_val, float *phi_val32, grf_stream_t stream) {
    GRF_REQUIRE(n_src >= 0 && m >= 1 && L >= 1 && step_cnt && step_idx && step_val && phi_cnt && phi_idx && phi_val,
                GRF_EINVAL, "grf_phi: bad arguments");
    GRF_REQUIRE(n_f >= 0 && (n_f == 0 || f), GRF_EINVAL, "grf_phi: bad modulator");
    GRF_REQUIRE(L <= 64, GRF_EUNSUPPORTED, "grf_phi: max_walk_length > 64 not supported by this build");
    GRF_REQUIRE(phi_cap >= 1, GRF_EINVAL, "grf_phi: phi_cap must be >= 1");
    if (n_src == 0) return GRF_OK;
    const int32_t Lf = n_f < L ? n_f : L;
    GRF_REQUIRE_GRID(cdiv<int64_t>(n_src, 4), 256, "phi_merge_kernel");
    phi_merge_kernel<<<(unsigned)cdiv<int64_t>(n_src, 4), 256, 0, S(stream)>>>(
        n_src, m, L, Lf, step_cnt, step_idx, step_val, f, phi_cap, phi_cnt, phi_idx, phi_val, phi_val32);
    GRF_CHECK_LAUNCH("phi_merge_kernel");
    return GRF_OK;
}

static int32_t phi_fused_launch(bool walk, int64_t n_src, int64_t m, int32_t L, int32_t norm,
                                const int32_t *slot_node, const double *slot_load, const int64_t *g_ptr,
                                const int32_t *g_idx, const double *g_val, const void *g_aug, double p_halt,
                                int32_t rule, uint64_t seed,
                                int64_t src_begin, const double *f, int32_t n_f, int64_t phi_cap, int32_t *phi_cnt,
                                int32_t *phi_idx, double *phi_val, float *phi_val32, int32_t *t_count,
                                int64_t band_width, int64_t n_cols, hipStream_t st, int64_t count_row0 = 0) {
    GRF_REQUIRE(norm == GRF_NORM_DIV || norm == GRF_NORM_MUL_RECIP, GRF_EINVAL, "grf_phi_fused: bad norm");
    GRF_REQUIRE(n_f >= 0 && (n_f == 0 || f), GRF_EINVAL, "grf_phi_fused: bad modulator");
    GRF_REQUIRE(m * (int64_t)L <= 4096, GRF_EUNSUPPORTED, "grf_phi_fused: needs walks_per_node * L <= 4096");
    GRF_REQUIRE(phi_cap >= 1, GRF_EINVAL, "grf_phi_fused: phi_cap must be >= 1");
    if (n_src == 0) return GRF_OK;
    const int E = (int)(m * L);
    const int P = std::max(64, (int)next_pow2_u32((uint32_t)E));
    const int wbits = ceil_log2((uint64_t)m), lbits = ceil_log2((uint64_t)L) > 0 ? ceil_log2((uint64_t)L) : 1;
    GRF_REQUIRE(wbits + lbits <= 32, GRF_EUNSUPPORTED, "grf_phi_fused: key overflow");
    // 32-bit keys when every key (node << (wbits + lbits) | step | walk) < the sentinel 2^32 - 1:
    // needs the node-id bound n_cols, known for the walking kernel (the slots path stays 64-bit)
    const bool key32 = walk && n_cols > 0 && ((uint64_t)n_cols << (wbits + lbits)) <= 0xffffffffull;
    const int32_t Lf_ = n_f < L ? n_f : L;
    static const int32_t sort_lds = [] {  // (experiments: GRF_PHI_SORT_LDS=1, the all-LDS bitonic sort;
        const char *e = getenv("GRF_PHI_SORT_LDS");  //  2, no sort at all: timing-only)
        return (int32_t)(e ? atoi(e) : 0);
    }();
    static const size_t lds_pad = [] {  // (experiments: extra LDS per source, GRF_PHI_LDS_PAD bytes)
        const char *e = getenv("GRF_PHI_LDS_PAD");
        return e ? (size_t)atoll(e) : (size_t)0;
    }();
    const size_t lds = (size_t)E * 8 + (size_t)((Lf_ + 1) & ~1) * 8 + 32 * 4 + (size_t)P * (key32 ? 4 : 8) + lds_pad;
    // threads per source: P / 4 up to 256, and at most one per walk -- measured (tools/walkphi_ab.py)
    // with the 12.9 KB LDS layout: m = 128 (C4) 128 threads 2.85 ms vs 256 3.28; m = 64 (C5) 64
    // threads 11.2 ms vs 128 13.0 (idle waves hold the source's slot while its walks run, and LDS
    // no longer caps the sources per CU); GRF_PHI_THREADS caps it for experiments
    static const int t_env = [] {
        const char *e = getenv("GRF_PHI_THREADS");
        const int v = e ? atoi(e) : 0;
        return (v == 64 || v == 128 || v == 256) ? v : 0;
    }();
    const int t_cap = t_env ? t_env : (int)std::min<int64_t>(256, std::max<int64_t>(64, ((m + 63) / 64) * 64));
    int T = P >= 512 ? 256 : (P >= 128 ? P / 2 : 64);
    while (T > t_cap && P / (T / 2) <= kPhiMaxPer) T /= 2;
    GRF_REQUIRE(n_f <= 64 || L <= 64, GRF_EUNSUPPORTED, "grf_phi_fused: max_walk_length > 64");
    GRF_REQUIRE(P / T <= kPhiMaxPer, GRF_EUNSUPPORTED, "grf_phi_fused: too many positions per thread");
    const int32_t Lf = n_f < L ? n_f : L;
    GRF_REQUIRE_GRID(n_src, T, "phi_fused_kernel");
#define GRF_PHI_LAUNCH_KTT(W, K, KT, TT)                                                                           \
    phi_fused_kernel<W, K, KT, TT><<<(unsigned)n_src, T, lds, st>>>(                                              \
        m, L, norm, P, wbits, lbits, slot_node, slot_load, g_ptr, g_idx, g_val,                                   \
        reinterpret_cast<const unsigned char *>(g_aug), p_halt, rule, (uint32_t)seed,                               \
        (uint32_t)(seed >> 32), src_begin, f, Lf, phi_cap, phi_cnt, phi_idx, phi_val, phi_val32, t_count, band_width, \
        n_cols, count_row0, sort_lds)
#define GRF_PHI_LAUNCH_KT(W, K, KT) GRF_PHI_LAUNCH_KTT(W, K, KT, 0)
#define GRF_PHI_LAUNCH(W, K)                                                                                      \
    do {                                                                                                          \
        if (key32) GRF_PHI_LAUNCH_KT(W, K, uint32_t);                                                             \
        else GRF_PHI_LAUNCH_KT(W, K, uint64_t);                                                                   \
    } while (0)
#define GRF_PHI_PER(W)                                                                                            \
    switch (P / T) {                                                                                              \
        case 1: GRF_PHI_LAUNCH(W, 1); break;                                                                      \
        case 2: GRF_PHI_LAUNCH(W, 2); break;                                                                      \
        case 4: GRF_PHI_LAUNCH(W, 4); break;                                                                      \
        case 8: GRF_PHI_LAUNCH(W, 8); break;                                                                      \
        default: GRF_PHI_LAUNCH(W, 16); break;                                                                    \
    }
    // the walking configurations of C4 (m = 128, L = 8: 128 threads) and C5 (m = 64: 64 threads),
    // 8 positions per thread, 32-bit keys: the sort fully unrolled
    if (walk && key32 && P / T == 8 && T == 128) GRF_PHI_LAUNCH_KTT(true, 8, uint32_t, 128);
    else if (walk && key32 && P / T == 8 && T == 64) GRF_PHI_LAUNCH_KTT(true, 8, uint32_t, 64);
    else if (walk) { GRF_PHI_PER(true) } else { GRF_PHI_PER(false) }
#undef GRF_PHI_PER
#undef GRF_PHI_LAUNCH
#undef GRF_PHI_LAUNCH_KT
#undef GRF_PHI_LAUNCH_KTT
    GRF_CHECK_LAUNCH("phi_fused_kernel");
    return GRF_OK;
}

int32_t grf_phi_fused(int64_t n_src, int64_t m, int32_t L, int32_t norm, const int32_t *slot_node,
                      const double *slot_load, const double *f, int32_t n_f, int64_t phi_cap, int32_t *phi_cnt,
                      int32_t *phi_idx, double *phi_val, float *phi_val32, grf_stream_t stream) {
    GRF_REQUIRE(n_src >= 0 && m >= 1 && L >= 1 && slot_node && slot_load && phi_cnt && phi_idx && phi_val,
                GRF_EINVAL, "grf_phi_fused: bad arguments");
    return phi_fused_launch(false, n_src, m, L, norm, slot_node, slot_load, nullptr, nullptr, nullptr, nullptr, 0.0, 0,
                            0, 0, f,
                            n_f, phi_cap, phi_cnt, phi_idx, phi_val, phi_val32, nullptr, 1, 0, S(stream));
}

int32_t grf_walk_phi(int64_t n, const int64_t *g_ptr, const int32_t *g_idx, const double *g_val, const void *g_aug,
                     const grf_walk_params *params, int64_t src_begin, int64_t src_end, int32_t norm, const double *f,
                     int32_t n_f, int64_t phi_cap, int32_t *phi_cnt, int32_t *phi_idx, double *phi_val,
                     float *phi_val32, int32_t *t_count, int64_t band_width, int64_t count_row0,
                     grf_stream_t stream) {
    GRF_REQUIRE(params != nullptr, GRF_EINVAL, "grf_walk_phi: params is NULL");
    const grf_walk_params P = *params;
    GRF_REQUIRE(n >= 0 && g_ptr && phi_cnt && phi_idx && (phi_val || phi_val32), GRF_EINVAL,
                "grf_walk_phi: bad arguments");
    GRF_REQUIRE(P.rng == GRF_RNG_PHILOX, GRF_EUNSUPPORTED, "grf_walk_phi: Philox walks only (use grf_walk for PCG64)");
    GRF_REQUIRE(P.walks_per_node >= 1 && P.walks_per_node <= 0x7fffffff, GRF_EINVAL,
                "grf_walk_phi: walks_per_node must be in [1, 2^31)");
    GRF_REQUIRE(P.max_walk_length >= 1, GRF_EINVAL, "grf_walk_phi: max_walk_length must be >= 1");
    GRF_REQUIRE(P.p_halt >= 0.0 && P.p_halt < 1.0, GRF_EINVAL, "grf_walk_phi: p_halt must be in [0, 1)");
    GRF_REQUIRE(P.load_rule >= 0 && P.load_rule <= 2, GRF_EINVAL, "grf_walk_phi: bad load_rule %d", P.load_rule);
    GRF_REQUIRE(0 <= src_begin && src_begin <= src_end && src_end <= n, GRF_EINVAL, "grf_walk_phi: bad source range");
    GRF_REQUIRE(n <= 0x7fffffffLL, GRF_EUNSUPPORTED, "grf_walk_phi: n must fit int32 node ids");
    GRF_REQUIRE(!t_count || (band_width >= 1 &&
                             phi_cap >= std::min<int64_t>(P.walks_per_node * (int64_t)P.max_walk_length, n)),
                GRF_EINVAL, "grf_walk_phi: counting needs band_width >= 1 and phi_cap that never truncates a row");
    GRF_REQUIRE(!t_count || (0 <= count_row0 && count_row0 <= src_begin), GRF_EINVAL,
                "grf_walk_phi: count_row0 must be in [0, src_begin]");
    GRF_REQUIRE(!g_aug || ((uintptr_t)g_aug & 31) == 0, GRF_EINVAL, "grf_walk_phi: g_aug must be 32-byte aligned");
    return phi_fused_launch(true, src_end - src_begin, P.walks_per_node, P.max_walk_length, norm, nullptr, nullptr,
                            g_ptr, g_idx, g_val, g_aug, P.p_halt, P.load_rule, P.seed, src_begin, f, n_f, phi_cap, phi_cnt,
                            phi_idx, phi_val, phi_val32, t_count, band_width, n, S(stream), count_row0);
}

size_t grf_walk_aug_bytes(int64_t nnz) { return kAugHeader + (size_t)(nnz > 0 ? nnz : 0) * sizeof(AugRec); }

int32_t grf_walk_aug(int64_t n, const int64_t *g_ptr, const int32_t *g_idx, const double *g_val, void *g_aug,
                     grf_stream_t stream) {
    GRF_REQUIRE(n >= 0 && g_ptr && g_idx && g_val && g_aug, GRF_EINVAL, "grf_walk_aug: bad arguments");
    GRF_REQUIRE(((uintptr_t)g_aug & 31) == 0, GRF_EINVAL, "grf_walk_aug: g_aug must be 32-byte aligned");
    if (n == 0) return GRF_OK;
    // GRF_WALK_AUG16=0: always the 32-byte records (A/B; read per call so tests can cover both formats)
    const char *e16 = getenv("GRF_WALK_AUG16");
    const int allow16 = e16 ? atoi(e16) : 1;
    const int32_t tb = ceil_log2((uint64_t)n) > 0 ? ceil_log2((uint64_t)n) : 1;  // node ids < n
    const int32_t lb = ceil_log2((uint64_t)n + 1);                               // row lengths <= n
    // grid-stride over the entries (nnz stays on the device): ~32 rows per workgroup, at most 8 per CU
    const unsigned grid = (unsigned)std::min<int64_t>(2048, std::max<int64_t>(1, cdiv<int64_t>(n, 32)));
    walk_aug_kernel<<<grid, 256, 0, S(stream)>>>(n, tb, lb, allow16, g_ptr, g_idx, g_val,
                                                 reinterpret_cast<unsigned char *>(g_aug));
    GRF_CHECK_LAUNCH("walk_aug_kernel");
    return GRF_OK;
}

int32_t grf_steps_densify(int64_t n_src, int64_t m, int32_t L, int64_t n_cols, const int32_t *step_cnt,
                          const int32_t *step_idx, const double *step_val, double *out, grf_stream_t stream) {
    GRF_REQUIRE(n_src >= 0 && m >= 1 && L >= 1 && n_cols >= 0 && step_cnt && step_idx && step_val && out,
                GRF_EINVAL, "grf_steps_densify: bad arguments");
    if (n_src == 0) return GRF_OK;
    GRF_REQUIRE_GRID(cdiv<int64_t>(n_src * L, 4), 256, "steps_densify_kernel");
    steps_densify_kernel<<<(unsigned)cdiv<int64_t>(n_src * L, 4), 256, 0, S(stream)>>>(n_src, m, L, n_cols, step_cnt,
                                                                                      step_idx, step_val, out);
    GRF_CHECK_LAUNCH("steps_densify_kernel");
    return GRF_OK;
}

}  // extern "C"
