// grf_walk.hip -- random-walk kernels (the walk loop of the reference samplers).
//
// Reference loops replaced (paths under the reference checkout):
//   efficient_graph_gp_sparse/random_walk_samplers_sparse/sparse_sampler.py:36-54
//   efficient_graph_gp/random_walk_samplers/sampler.py:40-59 (pool) and :162-184 (sequential)
// Per step: record (current node, load); stop at a zero-degree node or with
// probability p_halt; otherwise move to a uniformly chosen CSR neighbour and
// update the load by the importance weight deg * w / (1 - p).
//
// Two RNG modes:
//   Philox4x32-10, one lane per walk, counter (step, walk, source, block), key = seed.
//     Result is independent of the launch geometry and of how sources are sharded
//     over GPUs.  Halt: 53-bit double from two words < p; neighbour: 32-bit Lemire.
//   PCG64 replay, one lane per chunk: numpy default_rng(seed + c) consumed exactly
//     as the reference consumes it (random() for the halt, integers(deg) through
//     the buffered 32-bit Lemire path, no draw for deg == 1).  Reference-exact,
//     sequential within a chunk (the reference's own parallel granularity).
#include "grf_philox.h"

namespace grf {

__global__ __launch_bounds__(256) void walk_philox_kernel(const int64_t *__restrict__ g_ptr,
                                                          const int32_t *__restrict__ g_idx,
                                                          const double *__restrict__ g_val,
                                                          const unsigned char *__restrict__ g_aug, int64_t m, double p,
                                                          int32_t L, int32_t rule, uint32_t k0, uint32_t k1,
                                                          int64_t src_begin, int64_t n_src,
                                                          int32_t *__restrict__ slot_node,
                                                          double *__restrict__ slot_load) {
    const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (gid >= n_src * m) return;
    const int64_t sl = gid / m, w = gid - sl * m, s = src_begin + sl;
    int32_t *nd = slot_node + sl * L * m + w;
    double *ld = slot_load + sl * L * m + w;
    auto visit = [&](int32_t l, int32_t node, double load) {
        nd[(int64_t)l * m] = node;
        ld[(int64_t)l * m] = load;
    };
    // (g_aug: one dependent round trip per step instead of two; the same draws and slots)
    const int32_t n_vis = g_aug ? philox_walk_aug(g_ptr, g_aug, s, (uint32_t)w, p, L, rule, k0, k1, visit)
                                : philox_walk(g_ptr, g_idx, g_val, s, (uint32_t)w, p, L, rule, k0, k1, visit);
    for (int32_t l = n_vis; l < L; ++l) nd[(int64_t)l * m] = -1;
}

// ------------------------------------------------------------------- PCG64
typedef unsigned __int128 u128;

struct Pcg64 {
    u128 state, inc;
    uint32_t has32, u32;
    __device__ inline uint64_t next64() {
        const u128 mult = (((u128)2549297995355413924ULL) << 64) | (u128)4865540595714422341ULL;
        state = state * mult + inc;
        const uint64_t hi = (uint64_t)(state >> 64), lo = (uint64_t)state;
        const unsigned rot = (unsigned)(state >> 122);
        const uint64_t x = hi ^ lo;
        return (x >> rot) | (x << ((64u - rot) & 63u));
    }
    __device__ inline uint32_t next32() {
        if (has32) { has32 = 0; return u32; }
        const uint64_t n = next64();
        has32 = 1;
        u32 = (uint32_t)(n >> 32);
        return (uint32_t)n;
    }
    __device__ inline double random() { return (double)(next64() >> 11) * (1.0 / 9007199254740992.0); }
    __device__ inline uint32_t integers(uint32_t d) {
        const uint32_t rng = d - 1u;
        if (rng == 0) return 0;
        uint64_t m = (uint64_t)next32() * d;
        uint32_t left = (uint32_t)m;
        if (left < d) {
            const uint32_t thr = (0xFFFFFFFFu - rng) % d;
            while (left < thr) {
                m = (uint64_t)next32() * d;
                left = (uint32_t)m;
            }
        }
        return (uint32_t)(m >> 32);
    }
};

// numpy SeedSequence(seed).generate_state(4, uint64) -> PCG64 seeding
__device__ inline void pcg64_seed(uint64_t seed, Pcg64 &g) {
    uint32_t ent[2];
    int n_ent = 0;
    if (seed == 0) ent[n_ent++] = 0;
    while (seed) { ent[n_ent++] = (uint32_t)seed; seed >>= 32; }
    uint32_t pool[4], hc = 0x43b0d7e5u;
    auto hashmix = [&](uint32_t v) {
        v ^= hc;
        hc *= 0x931e8875u;
        v *= hc;
        v ^= v >> 16;
        return v;
    };
    auto mix = [](uint32_t x, uint32_t y) {
        uint32_t r = 0xca01f9ddu * x - 0x4973f715u * y;
        r ^= r >> 16;
        return r;
    };
    for (int i = 0; i < 4; ++i) pool[i] = hashmix(i < n_ent ? ent[i] : 0u);
    for (int s = 0; s < 4; ++s)
        for (int d = 0; d < 4; ++d)
            if (s != d) pool[d] = mix(pool[d], hashmix(pool[s]));
    uint32_t hb = 0x8b51f9ddu, w[8];
    for (int i = 0; i < 8; ++i) {
        uint32_t v = pool[i & 3];
        v ^= hb;
        hb *= 0x58f38dedu;
        v *= hb;
        v ^= v >> 16;
        w[i] = v;
    }
    const uint64_t s0 = (uint64_t)w[0] | ((uint64_t)w[1] << 32), s1 = (uint64_t)w[2] | ((uint64_t)w[3] << 32);
    const uint64_t s2 = (uint64_t)w[4] | ((uint64_t)w[5] << 32), s3 = (uint64_t)w[6] | ((uint64_t)w[7] << 32);
    const u128 initstate = ((u128)s0 << 64) | s1, initseq = ((u128)s2 << 64) | s3;
    const u128 mult = (((u128)2549297995355413924ULL) << 64) | (u128)4865540595714422341ULL;
    g.inc = (initseq << 1) | 1u;
    g.state = g.inc;  // 0 * mult + inc
    g.state += initstate;
    g.state = g.state * mult + g.inc;
    g.has32 = 0;
    g.u32 = 0;
}

// kAug: the steps read the augmented walk matrix (grf_walk_aug: the chosen entry's target, the target's
// row start and length and the weight in one record), so each step is ONE dependent memory round trip
// instead of two (the row bounds of the new node, then its entry); the draws and slots are identical.
template <bool kAug>
__global__ __launch_bounds__(64) void walk_pcg64_kernel(int64_t n, const int64_t *__restrict__ g_ptr,
                                                        const int32_t *__restrict__ g_idx,
                                                        const double *__restrict__ g_val,
                                                        const unsigned char *__restrict__ g_aug, int64_t m, double p,
                                                        int32_t L, int32_t rule, int64_t n_chunks, uint64_t seed,
                                                        int64_t chunk_begin, int64_t chunk_end, int64_t src_begin,
                                                        int32_t *__restrict__ slot_node,
                                                        double *__restrict__ slot_load) {
    const int64_t c = chunk_begin + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= chunk_end) return;
    const int64_t base = n / n_chunks, extra = n % n_chunks;
    const int64_t b = c * base + (c < extra ? c : extra), e = b + base + (c < extra ? 1 : 0);
    Pcg64 g;
    pcg64_seed(seed + (uint64_t)c, g);
    bool compact = false;
    int tb = 0, rb = 0;
    const unsigned char *recs = nullptr;
    if (kAug) {
        const int4 hd = *reinterpret_cast<const int4 *>(g_aug);
        compact = hd.x == 1;
        tb = hd.y;
        rb = hd.z;
        recs = g_aug + kAugHeader;
    }
    const uint64_t tmask = (1ull << tb) - 1, rmask = (1ull << rb) - 1;
    const LoadKeep keep(p);
    for (int64_t s = b; s < e; ++s) {
        const int64_t sl = s - src_begin;
        const int64_t rs0 = g_ptr[s], deg0 = g_ptr[s + 1] - rs0;
        for (int64_t w = 0; w < m; ++w) {
            int32_t *nd = slot_node + sl * L * m + w;
            double *ld = slot_load + sl * L * m + w;
            int64_t cur = s, rs = rs0, deg = deg0;
            double load = 1.0;
            int32_t l = 0;
            for (; l < L; ++l) {
                nd[(int64_t)l * m] = (int32_t)cur;
                ld[(int64_t)l * m] = load;
                if (!kAug) {
                    rs = g_ptr[cur];
                    deg = g_ptr[cur + 1] - rs;
                }
                if (deg == 0 || g.random() < p) { ++l; break; }
                const uint32_t k = g.integers((uint32_t)deg);
                if (!kAug) {
                    const double wt = g_val[rs + k];
                    load = load_update(rule, load, deg, wt, keep);
                    cur = g_idx[rs + k];
                } else if (compact) {
                    const int4 a = *reinterpret_cast<const int4 *>(recs + (size_t)(rs + k) * sizeof(AugRec16));
                    const uint64_t pk = ((uint64_t)(uint32_t)a.y << 32) | (uint32_t)a.x;
                    load = load_update(rule, load, deg, __hiloint2double(a.w, a.z), keep);
                    cur = (int64_t)(pk & tmask);
                    rs = (int64_t)((pk >> tb) & rmask);
                    deg = (int64_t)(pk >> (tb + rb));
                } else {
                    const AugRec *rec = reinterpret_cast<const AugRec *>(recs) + rs + k;
                    const int4 a = *reinterpret_cast<const int4 *>(rec);
                    load = load_update(rule, load, deg, rec->w, keep);
                    cur = a.x;
                    rs = (int64_t)(uint32_t)a.y;
                    deg = a.z;
                }
            }
            for (; l < L; ++l) nd[(int64_t)l * m] = -1;
        }
    }
}

}  // namespace grf

using namespace grf;

static int32_t walk_impl(int64_t n, const int64_t *g_ptr, const int32_t *g_idx, const double *g_val,
                         const void *g_aug_v, const grf_walk_params *params, int64_t src_begin, int64_t src_end,
                         int32_t *slot_node, double *slot_load, grf_stream_t stream) {
    const unsigned char *g_aug = reinterpret_cast<const unsigned char *>(g_aug_v);
    GRF_REQUIRE(!g_aug || ((uintptr_t)g_aug & 31) == 0, GRF_EINVAL, "grf_walk: g_aug must be 32-byte aligned");
    GRF_REQUIRE(params != nullptr, GRF_EINVAL, "grf_walk: params is NULL");
    const grf_walk_params P = *params;
    GRF_REQUIRE(n >= 0 && g_ptr && slot_node && slot_load, GRF_EINVAL, "grf_walk: bad arguments");
    GRF_REQUIRE(P.walks_per_node >= 1 && P.walks_per_node <= 0x7fffffff, GRF_EINVAL,
                "grf_walk: walks_per_node must be in [1, 2^31)");
    GRF_REQUIRE(P.max_walk_length >= 1, GRF_EINVAL, "grf_walk: max_walk_length must be >= 1");
    GRF_REQUIRE(P.p_halt >= 0.0 && P.p_halt < 1.0, GRF_EINVAL, "grf_walk: p_halt must be in [0, 1)");
    GRF_REQUIRE(P.load_rule >= 0 && P.load_rule <= 2, GRF_EINVAL, "grf_walk: bad load_rule %d", P.load_rule);
    GRF_REQUIRE(0 <= src_begin && src_begin <= src_end && src_end <= n, GRF_EINVAL,
                "grf_walk: bad source range [%lld, %lld)", (long long)src_begin, (long long)src_end);
    GRF_REQUIRE(n <= 0x7fffffffLL, GRF_EUNSUPPORTED, "grf_walk: n must fit int32 node ids");
    hipStream_t st = S(stream);
    const int64_t n_src = src_end - src_begin;
    if (n_src == 0) return GRF_OK;
    if (P.rng == GRF_RNG_PHILOX) {
        const int64_t total = n_src * P.walks_per_node;
        GRF_REQUIRE_GRID(cdiv<int64_t>(total, 256), 256, "walk_philox_kernel");
        walk_philox_kernel<<<(unsigned)cdiv<int64_t>(total, 256), 256, 0, st>>>(
            g_ptr, g_idx, g_val, g_aug, P.walks_per_node, P.p_halt, P.max_walk_length, P.load_rule, (uint32_t)P.seed,
            (uint32_t)(P.seed >> 32), src_begin, n_src, slot_node, slot_load);
        GRF_CHECK_LAUNCH("walk_philox_kernel");
        return GRF_OK;
    }
    GRF_REQUIRE(P.rng == GRF_RNG_PCG64, GRF_EINVAL, "grf_walk: bad rng %d", P.rng);
    GRF_REQUIRE(P.n_chunks >= 1, GRF_EINVAL, "grf_walk: n_chunks must be >= 1");
    // [src_begin, src_end) must be whole chunks
    const int64_t base = n / P.n_chunks, extra = n % P.n_chunks;
    auto first = [&](int64_t c) { return c * base + (c < extra ? c : extra); };
    // locate chunk_begin / chunk_end by bisection on the monotone boundaries
    auto locate = [&](int64_t s) {
        int64_t lo = 0, hi = P.n_chunks;
        while (lo < hi) {
            int64_t mid = (lo + hi) / 2;
            if (first(mid) < s) lo = mid + 1; else hi = mid;
        }
        return lo;
    };
    const int64_t cb = locate(src_begin), ce = locate(src_end);
    GRF_REQUIRE(first(cb) == src_begin && (ce == P.n_chunks ? n : first(ce)) == src_end, GRF_EINVAL,
                "grf_walk: PCG64 source range must be a union of whole chunks");
    // empty chunks (n_chunks > n) have first(c) == first(c+1); cover [cb, ce) plus trailing empties is harmless
    const int64_t nch = ce - cb;
    if (nch <= 0) return GRF_OK;
    GRF_REQUIRE_GRID(cdiv<int64_t>(nch, 64), 64, "walk_pcg64_kernel");
    if (g_aug)
        walk_pcg64_kernel<true><<<(unsigned)cdiv<int64_t>(nch, 64), 64, 0, st>>>(
            n, g_ptr, g_idx, g_val, g_aug, P.walks_per_node, P.p_halt, P.max_walk_length, P.load_rule, P.n_chunks,
            P.seed, cb, ce, src_begin, slot_node, slot_load);
    else
        walk_pcg64_kernel<false><<<(unsigned)cdiv<int64_t>(nch, 64), 64, 0, st>>>(
            n, g_ptr, g_idx, g_val, nullptr, P.walks_per_node, P.p_halt, P.max_walk_length, P.load_rule, P.n_chunks,
            P.seed, cb, ce, src_begin, slot_node, slot_load);
    GRF_CHECK_LAUNCH("walk_pcg64_kernel");
    return GRF_OK;
}

extern "C" __attribute__((visibility("default"))) int32_t grf_walk(int64_t n, const int64_t *g_ptr, const int32_t *g_idx,
                                                                  const double *g_val, const grf_walk_params *params,
                                                                  int64_t src_begin, int64_t src_end, int32_t *slot_node,
                                                                  double *slot_load, grf_stream_t stream) {
    return walk_impl(n, g_ptr, g_idx, g_val, nullptr, params, src_begin, src_end, slot_node, slot_load, stream);
}

extern "C" __attribute__((visibility("default"))) int32_t grf_walk_ex(int64_t n, const int64_t *g_ptr, const int32_t *g_idx,
                                                                     const double *g_val, const void *g_aug,
                                                                     const grf_walk_params *params, int64_t src_begin,
                                                                     int64_t src_end, int32_t *slot_node,
                                                                     double *slot_load, grf_stream_t stream) {
    return walk_impl(n, g_ptr, g_idx, g_val, g_aug, params, src_begin, src_end, slot_node, slot_load, stream);
}
