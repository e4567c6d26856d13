// grf_philox.h -- the Philox4x32-10 random walk shared by the walk kernel and the fused
// walk -> Phi kernel (one definition, so both produce the same visits bit for bit).
#pragma once
#include "grf_common.h"

namespace grf {

// ------------------------------------------------------------------ Philox
__device__ __forceinline__ void philox4x32_10(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0, uint32_t k1,
                                     uint32_t &o0, uint32_t &o1, uint32_t &o2, uint32_t &o3) {
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        // one 32 x 32 -> 64-bit product per multiplier (v_mad_u64_u32: both halves from one
        // instruction instead of a v_mul_lo_u32 + v_mul_hi_u32 pair)
        const uint64_t p0 = (uint64_t)0xD2511F53u * c0, p1 = (uint64_t)0xCD9E8D57u * c2;
        const uint32_t lo0 = (uint32_t)p0, hi0 = (uint32_t)(p0 >> 32);
        const uint32_t lo1 = (uint32_t)p1, hi1 = (uint32_t)(p1 >> 32);
        // (three-input XOR in one v_bitop3_b32, truth table 0x96, the key from its SGPR)
        const uint32_t n0 = __builtin_amdgcn_bitop3_b32(hi1, c1, k0, 0x96);
        const uint32_t n2 = __builtin_amdgcn_bitop3_b32(hi0, c3, k1, 0x96);
        c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
        k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
    }
    o0 = c0; o1 = c1; o2 = c2; o3 = c3;
}

// Lemire rejection tail of step l (probability < deg / 2^32): words from blocks 1, 2, ... of the step's own
// counter (l, w, s, blk) -- block 0 of (j, w, s) is the step pair's main draw (philox_walk).
__device__ __noinline__ uint64_t philox_lemire_retry(uint32_t d, uint32_t thr, uint32_t l, uint32_t w, uint32_t s,
                                                     uint32_t k0, uint32_t k1) {
    for (uint32_t blk = 1;; ++blk) {
        uint32_t y[4];
        philox4x32_10(l, w, s, blk, k0, k1, y[0], y[1], y[2], y[3]);
        for (int i = 0; i < 4; ++i) {
            const uint64_t mm = (uint64_t)y[i] * d;
            if ((uint32_t)mm >= thr) return mm;
        }
    }
}

// The halt test of one 32-bit word x: halt iff x < ceil(p 2^32) (p 2^32 is exact; P(halt) = ceil(p 2^32) / 2^32,
// within 2^-32 of p); 0 when p <= 0 or NaN (never halts), 2^32 when p >= 1 (always).
__device__ inline uint64_t halt_threshold(double p) {
    const double y = ceil(p * 4294967296.0);
    return y > 0.0 ? (y < 4294967296.0 ? (uint64_t)y : (1ull << 32)) : 0ull;
}
__device__ inline bool halts(uint32_t x, uint64_t thr) { return (uint64_t)x < thr; }

// The words of step l: one Philox4x32-10 block (l / 2, w, s, 0) serves the step pair -- the even step halts on
// x0 and picks its neighbour from x1, the odd step uses x2 and x3 -- so a walk of L recorded visits runs
// ceil((L - 1) / 2) blocks (the last recorded visit draws nothing).  The walks below take the steps in pairs,
// so the four words live in registers for one loop iteration (carried across iterations, with the block
// computed on every other step, they went to scratch memory).

// x / c correctly rounded without the IEEE divide sequence (v_div_scale x2, v_rcp_f64, 5 FMAs, v_div_fmas,
// v_div_fixup per call): with y = RN(1 / c) (loop-invariant: computed once per walk) the quotient
// q = RN(x y) is faithful, the remainder x - c q is exact in one FMA, and RN(q + (x - c q) y) is RN(x / c)
// (Markstein's theorem; it needs x, the quotient and the remainder normal and c q free of overflow).
// Divisor precomputes, once per walk, the window of x's biased exponent for which both |x| and |x / c|
// lie in [2^-959, 2^961): there the fast path is exact; anything else -- zero, subnormal, huge, inf or
// NaN operands or quotients, e.g. cumulative loads that overflowed -- takes the IEEE divide (a branch no
// lane takes on the benchmarked graphs), so the bits are x / c's everywhere (tools/div_check.c checks
// both ranges).  The window test is one bit-field extract and one unsigned compare on x's high word.
struct Divisor {
    double c, y;
    uint32_t lo, span;  // fast path iff (exponent(x) - lo) <= span, unsigned
    __device__ explicit Divisor(double c_) : c(c_), y(1.0 / c_) {
        const int32_t ec = (int32_t)((__double2hiint(c_) >> 20) & 0x7ff);
        const int32_t l = ec - 958 > 64 ? ec - 958 : 64, h = ec + 959 < 1983 ? ec + 959 : 1983;
        lo = (uint32_t)l;
        span = h >= l ? (uint32_t)(h - l) : 0u;
        if (h < l) lo = 0xffffffffu;  // (an empty window: always the IEEE divide)
    }
    __device__ double operator()(double x) const {
        const uint32_t ex = ((uint32_t)__double2hiint(x) >> 20) & 0x7ffu;
        if (ex - lo > span) return x / c;
        const double q = x * y;
        return __builtin_fma(__builtin_fma(-q, c, x), y, q);
    }
};

// The importance weight deg w / (1 - p) applied by the load rule; keep = the divisor 1 - p (once per walk).
struct LoadKeep {
    Divisor d;
    __device__ explicit LoadKeep(double p) : d(1.0 - p) {}
};
template <typename Deg>
__device__ inline double load_update(int rule, double load, Deg deg, double w, const LoadKeep &keep) {
    const double f = keep.d((double)deg * w);
    if (rule == GRF_LOAD_CUMULATIVE) return load * f;
    if (rule == GRF_LOAD_NONCUMULATIVE) return f;
    return w;
}

// One Philox walk (source s, walk w) of at most L recorded visits: visit(l, node, load) is
// called for the recorded steps l = 0, 1, ...; returns the number of recorded visits.
// Per step: record (current node, load); stop after the L-th visit, at a zero-degree node or with
// probability p_halt (StepWords: halt word < ceil(p 2^32)); otherwise move to neighbour Lemire(pick
// word, deg) and update the load by the importance weight deg * w / (1 - p).
template <typename Visit>
__device__ inline int32_t philox_walk(const int64_t *__restrict__ g_ptr, const int32_t *__restrict__ g_idx,
                                      const double *__restrict__ g_val, int64_t s, uint32_t w, double p, int32_t L,
                                      int32_t rule, uint32_t k0, uint32_t k1, Visit visit) {
    int64_t cur = s;
    double load = 1.0;
    const uint64_t hthr = halt_threshold(p);
    const LoadKeep keep(p);
    int64_t rs = g_ptr[s], deg = g_ptr[s + 1] - rs;
    // one move of step l with halt word hw and neighbour word pw; false: the walk halts here
    auto move = [&](int32_t l, uint32_t hw, uint32_t pw) -> bool {
        if (halts(hw, hthr)) return false;
        const uint32_t d = (uint32_t)deg;
        uint32_t k = 0;
        if (d > 1) {
            uint64_t mm = (uint64_t)pw * d;
            if ((uint32_t)mm < d) {
                const uint32_t thr = (0u - d) % d;
                if ((uint32_t)mm < thr) mm = philox_lemire_retry(d, thr, (uint32_t)l, w, (uint32_t)s, k0, k1);
            }
            k = (uint32_t)(mm >> 32);
        }
        const double wt = g_val[rs + k];
        load = load_update(rule, load, deg, wt, keep);
        cur = g_idx[rs + k];
        rs = g_ptr[cur];
        deg = g_ptr[cur + 1] - rs;
        return true;
    };
    for (int32_t l = 0; l < L; l += 2) {
        visit(l, (int32_t)cur, load);
        if (l == L - 1 || deg == 0) return l + 1;
        uint32_t x0, x1, x2, x3;
        philox4x32_10((uint32_t)l >> 1, w, (uint32_t)s, 0u, k0, k1, x0, x1, x2, x3);
        if (!move(l, x0, x1)) return l + 1;
        visit(l + 1, (int32_t)cur, load);
        if (l + 1 == L - 1 || deg == 0) return l + 2;
        if (!move(l + 1, x2, x3)) return l + 2;
    }
    return L;
}

// The same walk over the "augmented" walk matrix: a record per entry e holding {target node, its
// row start, its row length, the entry's weight}, so a step is ONE dependent round trip that touches
// ONE record (instead of two round trips -- the target, then its row bounds -- over three arrays).
// Same draws, same choices, same loads: bit-identical to philox_walk.
// Layout (grf_walk_aug): a 32-byte header {format, tb, rb, 0, ...} then the records.
//   format 0 (AugRec, 32 B): {int32 v, int32 row start (low 32 bits), int32 length, 0, f64 w, 0};
//   format 1 (AugRec16, 16 B; when tb + rb + lb <= 64: tb, lb, rb = bits of the largest node id,
//     of a row length <= n and of a row start <= nnz):
//     {u64 v | row start << tb | length << (tb + rb), f64 w} -- half the table (C5: 352 -> 176 MB,
//     inside the 256 MB Infinity Cache), still one record per step.
struct __attribute__((aligned(32))) AugRec {
    int32_t v, rs, len, pad;
    double w, pad2;
};
struct __attribute__((aligned(16))) AugRec16 {
    uint64_t packed;
    double w;
};
constexpr int kAugHeader = 32;  // bytes before the first record

template <typename Visit>
__device__ inline int32_t philox_walk_aug(const int64_t *__restrict__ g_ptr, const unsigned char *__restrict__ aug,
                                          int64_t s, uint32_t w, double p,
                                          int32_t L, int32_t rule, uint32_t k0, uint32_t k1, Visit visit) {
    // the header (uniform: the same 16 bytes for every lane)
    const int4 hd = *reinterpret_cast<const int4 *>(aug);
    const bool compact = hd.x == 1;
    const int tb = hd.y, rb = hd.z;
    const uint64_t tmask = (1ull << tb) - 1, rmask = (1ull << rb) - 1;
    const unsigned char *recs = aug + kAugHeader;
    int64_t cur = s;
    double load = 1.0;
    const uint64_t hthr = halt_threshold(p);
    const LoadKeep keep(p);
    int64_t rs = g_ptr[s];
    int64_t deg = g_ptr[s + 1] - rs;
    auto move = [&](int32_t l, uint32_t hw, uint32_t pw) -> bool {
        if (halts(hw, hthr)) return false;
        const uint32_t d = (uint32_t)deg;
        uint32_t k = 0;
        if (d > 1) {
            uint64_t mm = (uint64_t)pw * d;
            if ((uint32_t)mm < d) {
                const uint32_t thr = (0u - d) % d;
                if ((uint32_t)mm < thr) mm = philox_lemire_retry(d, thr, (uint32_t)l, w, (uint32_t)s, k0, k1);
            }
            k = (uint32_t)(mm >> 32);
        }
        if (compact) {
            const int4 a = *reinterpret_cast<const int4 *>(recs + (size_t)(rs + k) * sizeof(AugRec16));
            const uint64_t pk = ((uint64_t)(uint32_t)a.y << 32) | (uint32_t)a.x;
            const double wt = __hiloint2double(a.w, a.z);
            load = load_update(rule, load, (uint32_t)deg, wt, keep);  // (a row length < n < 2^31: exact either way)
            cur = (int64_t)(pk & tmask);
            rs = (int64_t)((pk >> tb) & rmask);
            deg = (int64_t)(pk >> (tb + rb));
        } else {
            const AugRec *rec = reinterpret_cast<const AugRec *>(recs) + rs + k;
            const int4 a = *reinterpret_cast<const int4 *>(rec);
            const double wt = rec->w;
            load = load_update(rule, load, (uint32_t)deg, wt, keep);
            cur = a.x;
            rs = (int64_t)(uint32_t)a.y;
            deg = a.z;
        }
        return true;
    };
    for (int32_t l = 0; l < L; l += 2) {
        visit(l, (int32_t)cur, load);
        if (l == L - 1 || deg == 0) return l + 1;
        uint32_t x0, x1, x2, x3;
        philox4x32_10((uint32_t)l >> 1, w, (uint32_t)s, 0u, k0, k1, x0, x1, x2, x3);
        if (!move(l, x0, x1)) return l + 1;
        visit(l + 1, (int32_t)cur, load);
        if (l + 1 == L - 1 || deg == 0) return l + 2;
        if (!move(l + 1, x2, x3)) return l + 2;
    }
    return L;
}

}  // namespace grf
