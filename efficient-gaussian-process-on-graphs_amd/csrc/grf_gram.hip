// grf_gram.hip -- K = Phi Phi^T on gfx950.
//
// Replaces `Phi @ Phi.T`:
//   efficient_graph_gp_sparse/graph_kernels_sparse/fast_grf_kernel_general.py:55 (scipy SpGEMM)
//   efficient_graph_gp/graph_kernels/fast_grf_kernel_general.py:39 (dense BLAS)
//
// Sparse path (Gustavson, output-stationary in LDS): a workgroup of 4 waves owns the tile
// K[row, j0 : j0 + W] (W = one band of the banded transpose, 4096 columns = 32 KB of int64
// accumulators; 4 tiles per CU).  For every nonzero Phi[row, k] it streams bucket (band, k) --
// the entries Phi[j, k] with j in the band, stored as 12-byte record pairs (2 x u16 j - j0,
// 2 x f32 value) -- and adds the exact product Phi[row,k]*Phi[j,k] in int64 fixed point with
// ds_add_u64.  Measured on gfx950 (tools/lds_bench.hip): ds_add_f32 serialises per lane (~170
// cycles per wave instruction per CU) while ds_add_u64 takes ~12, so fixed point is both ~14x
// cheaper and exactly order-independent (bit-reproducible K).  Tiles are dispatched band-major,
// so the tiles in flight share one band's records in L2 / the Infinity Cache.  The finished tile
// is written once, coalesced, with non-temporal stores.  Bound: the gathers of bucket records
// that miss L2; the symmetric mode computes the tiles on and above the diagonal
// band and a mirror pass copies the upper triangle down.
//
// Dense path: grf_gram_dense.hip (fp32 MFMA, 128 x 128 tiles on and above the diagonal).
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>

#include "grf_block.h"

namespace grf {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t uint4_v __attribute__((ext_vector_type(4)));

// The Gram tiles' K stores and the swizzled mirror's K loads: non-temporal (K is write-once and
// larger than every cache).  -DGRF_GRAM_K_NT=0 builds them with the default policy (A/B build: the
// Infinity Cache keeps what default-policy stores wrote, profiles/r03_gram_persist_ab.txt).
#ifndef GRF_GRAM_K_NT
#define GRF_GRAM_K_NT 1
#endif
#if GRF_GRAM_K_NT
#define GRF_K_STORE(v, p) __builtin_nontemporal_store((v), (p))
#define GRF_K_LOAD(p) __builtin_nontemporal_load(p)
#else
#define GRF_K_STORE(v, p) (*(p) = (v))
#define GRF_K_LOAD(p) (*(p))
#endif

constexpr int kChunk = 1024;  // stream positions covered by one bucket-id chunk (16 per lane)
constexpr int kSub = 8;       // sub-bands of the transpose's split (grf_transpose_banded_self, t_split)
constexpr int kPairBytesG = 12;  // one record pair
// per wave: ids [kChunk], then tbase and aval for a batch of 64 * halves nonzeros
constexpr int wave_state_bytes(int halves) { return kChunk + halves * 64 * 8; }

// |x| < 2^51 -> round-to-nearest int64 with one f64 add and one integer subtract
// (the magic number's low word is 0: only the high word is corrected)
__device__ inline long long fx_round(double x) {
    const double magic = 6755399441055744.0;  // 1.5 * 2^52
    const unsigned long long b = (unsigned long long)__double_as_longlong(x + magic);
    const uint32_t hi = (uint32_t)(b >> 32) - 0x43380000u, lo = (uint32_t)b;
    return (long long)(((unsigned long long)hi << 32) | lo);
}

// round(a * v) for |a * v| < 2^51 in ONE fp64 operation: fma(a, v, 1.5 * 2^52) rounds the
// exact product plus the magic number once, i.e. to the nearest integer (ties to even), which
// is exactly fx_round(a * v) whenever a * v itself is exact in fp64 (a product of two f32
// scaled by a power of two is)
__device__ inline long long fx_fma_round(double a, double v) {
    const double magic = 6755399441055744.0;  // 1.5 * 2^52
    const unsigned long long b = (unsigned long long)__double_as_longlong(__builtin_fma(a, v, magic));
    const uint32_t hi = (uint32_t)(b >> 32) - 0x43380000u, lo = (uint32_t)b;
    return (long long)(((unsigned long long)hi << 32) | lo);
}


// inclusive max-scan of non-negative ints over the 64 lanes (DPP row shifts + row broadcasts)
__device__ inline int wave_incl_max(int v) {
    v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x111, 0xf, 0xf, false));  // row_shr:1
    v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x112, 0xf, 0xf, false));  // row_shr:2
    v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x114, 0xf, 0xf, false));  // row_shr:4
    v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x118, 0xf, 0xf, false));  // row_shr:8
    v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x142, 0xa, 0xf, false));  // row_bcast:15
    v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x143, 0xc, 0xf, false));  // row_bcast:31
    return v;
}

// Bucket ids of a chunk of 1024 stream positions from bucket-start markers: bid[p] holds
// (bucket + 1) at the first position of every non-empty bucket and 0 elsewhere; since the
// ids increase along the stream, the id of a position is the running maximum.  Lane l owns
// positions 16 l .. 16 l + 15 (one 16-byte LDS read and write); carry = the id running at
// the chunk start (0 for the first chunk).  Returns the id running at the chunk end.
__device__ inline int gram_propagate_ids(unsigned char *bid, int carry, int lane) {
    uint4 x = reinterpret_cast<uint4 *>(bid)[lane];
    uint32_t w[4] = {x.x, x.y, x.z, x.w};
    // in-lane running max over the 16 bytes (from 0), and the lane's maximum
    int run = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        uint32_t o = 0;
#pragma unroll
        for (int b = 0; b < 4; ++b) {
            run = max(run, (int)((w[i] >> (8 * b)) & 0xffu));
            o |= (uint32_t)run << (8 * b);
        }
        w[i] = o;
    }
    // ids running into this lane: the maximum over the previous lanes and the carry
    int before = __builtin_amdgcn_update_dpp(0, wave_incl_max(run), 0x138, 0xf, 0xf, false);  // wave_shr:1
    before = max(before, carry);
    const uint32_t rep = (uint32_t)before * 0x01010101u;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        // bytewise max(w, before): the bytes of w are non-decreasing, so only a leading run
        // of bytes below `before` changes
        uint32_t o = 0;
#pragma unroll
        for (int b = 0; b < 4; ++b) {
            const uint32_t v = (w[i] >> (8 * b)) & 0xffu;
            o |= (v > (uint32_t)before ? v : (uint32_t)before) << (8 * b);
        }
        w[i] = o;
    }
    (void)rep;
    reinterpret_cast<uint4 *>(bid)[lane] = make_uint4(w[0], w[1], w[2], w[3]);
    return __builtin_amdgcn_readlane(max(run, before), 63);
}

// gram_propagate_ids over a chunk of 64 * 4 * NW positions (NW = 1, 2: 4 or 8 per lane, one LDS read and write
// of 4 NW bytes): a short stream (C5's column-block tiles: ~235 pairs per wave) pays for the positions it has
// instead of 1024 (the 16-byte form is ~110 VALU per lane and batch)
template <int NW>
__device__ inline int gram_propagate_ids_n(unsigned char *bid, int carry, int lane) {
    uint32_t w[NW];
    if constexpr (NW == 1) {
        w[0] = reinterpret_cast<uint32_t *>(bid)[lane];
    } else {
        const uint2 x = reinterpret_cast<uint2 *>(bid)[lane];
        w[0] = x.x;
        w[1] = x.y;
    }
    int run = 0;
#pragma unroll
    for (int i = 0; i < NW; ++i) {
        uint32_t o = 0;
#pragma unroll
        for (int b = 0; b < 4; ++b) {
            run = max(run, (int)((w[i] >> (8 * b)) & 0xffu));
            o |= (uint32_t)run << (8 * b);
        }
        w[i] = o;
    }
    int before = __builtin_amdgcn_update_dpp(0, wave_incl_max(run), 0x138, 0xf, 0xf, false);  // wave_shr:1
    before = max(before, carry);
#pragma unroll
    for (int i = 0; i < NW; ++i) {
        uint32_t o = 0;
#pragma unroll
        for (int b = 0; b < 4; ++b) {
            const uint32_t v = (w[i] >> (8 * b)) & 0xffu;
            o |= (v > (uint32_t)before ? v : (uint32_t)before) << (8 * b);
        }
        w[i] = o;
    }
    if constexpr (NW == 1) reinterpret_cast<uint32_t *>(bid)[lane] = w[0];
    else reinterpret_cast<uint2 *>(bid)[lane] = make_uint2(w[0], w[1]);
    return __builtin_amdgcn_readlane(max(run, before), 63);
}

// Per-wave state of one flattened batch stream (see gram_sparse_kernel).
struct GramStream {
    const unsigned char *bid;   // bucket of every stream position of the current chunk (LDS)
    const int32_t *tbase;       // per bucket: byte offset of its first pair (from the band's
                                // first line) - 12 * stream position (LDS)
    const float *aval;          // per bucket: Phi[row,k] (LDS)
    __amdgpu_buffer_rsrc_t rec; // the band's record pairs, 12 bytes each (global, 32-bit offsets)
    unsigned char *acc;         // tile accumulator (LDS), addressed by byte offset
    double S;                   // the row's fixed-point scale 2^sh
    int32_t safe;               // byte offset of a pair with finite values (masked positions read it)
};

// one 12-byte record pair: {u16 col0 | u16 col1 << 16, f32 v0, f32 v1}
struct __attribute__((aligned(4))) RecPair {
    uint32_t cols;
    float v0, v1;
};

// NW windows of 64 pairs starting at stream position w0 (chunk base c0, chunk end cend).
// TAIL: positions >= cend are masked (they read pair 0 of the band and add exactly 0 to distinct
// entries) -- 0: no window, 1: the last window only (an exact tail group: NW = ceil((cend - w0) / 64),
// so every other window is full), 2: every window.
template <int NW, int TAIL>
__device__ __forceinline__ void gram_windows(const GramStream &g, int32_t w0, int32_t c0, int32_t cend, int lane) {
    int m[NW];
#pragma unroll
    for (int u = 0; u < NW; ++u) {
        const int32_t p = w0 + u * 64 + lane;
        const bool mk = TAIL == 2 || (TAIL == 1 && u == NW - 1);  // (compile-time per window)
        m[u] = (!mk || p < cend) ? (int)g.bid[p - c0] - 1 : 0;
    }
    int32_t pos[NW];
    double sc[NW];
#pragma unroll
    for (int u = 0; u < NW; ++u) {
        pos[u] = g.tbase[m[u]] + 12 * (w0 + u * 64 + lane);
        sc[u] = (double)g.aval[m[u]] * g.S;  // exact: a power-of-two scaling of an f32
    }
    if (TAIL) {
#pragma unroll
        for (int u = 0; u < NW; ++u) {
            if (TAIL == 1 && u != NW - 1) continue;
            const bool ok = w0 + u * 64 + lane < cend;
            pos[u] = ok ? pos[u] : g.safe;  // the band's first pair (slots: slot 0's first pair): finite
            sc[u] = ok ? sc[u] : 0.0;
        }
    }
    // phase order pinned: all descriptor reads, then all gathers in flight, then the adds
    __builtin_amdgcn_sched_barrier(0);
    RecPair rec[NW];
#pragma unroll
    for (int u = 0; u < NW; ++u) {
        const auto v = __builtin_amdgcn_raw_buffer_load_b96(g.rec, (uint32_t)pos[u], 0, 0);
        rec[u].cols = v[0];
        rec[u].v0 = __uint_as_float(v[1]);
        rec[u].v1 = __uint_as_float(v[2]);
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int u = 0; u < NW; ++u) {
        const long long q0 = fx_fma_round(sc[u], (double)rec[u].v0);
        const long long q1 = fx_fma_round(sc[u], (double)rec[u].v1);
        uint32_t c0 = rec[u].cols & 0xffffu, c1 = rec[u].cols >> 16;
        if (TAIL == 2 || (TAIL == 1 && u == NW - 1)) {
            const bool ok = w0 + u * 64 + lane < cend;
            c0 = ok ? c0 : (uint32_t)(lane & 15) * 8u;
            c1 = ok ? c1 : (uint32_t)(lane & 15) * 8u;
        }
        __hip_atomic_fetch_add(reinterpret_cast<unsigned long long *>(g.acc + c0), (unsigned long long)q0,
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        __hip_atomic_fetch_add(reinterpret_cast<unsigned long long *>(g.acc + c1), (unsigned long long)q1,
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
}

// int64 fixed point (scale 2^sh) -> float: two exact-width converts, one fma, one ldexp
// (|error| <= 1.5 ulp of the result; deterministic)
__device__ inline float fx_to_float(unsigned long long a, int sh) {
    const float hi = (float)(int)(a >> 32), lo = (float)(unsigned)(a & 0xffffffffull);
    return ldexpf(fmaf(hi, 4294967296.0f, lo), -sh);
}

// LDS bytes of one gram_sparse_kernel workgroup (W int64 counters + per-wave stream state):
// at W = 4096 and 4 waves exactly 40 KiB, i.e. four workgroups per CU.
constexpr size_t gram_lds_bytes(int64_t W, int waves, int halves) {
    return (size_t)W * 8 + (size_t)waves * wave_state_bytes(halves);
}

// Tiles of one Gram call in band-major order: band J holds count(J) tiles, the local rows
// 0 .. count(J)-1 (full mode: all rows; symmetric mode, whole K: the rows of bands <= J).
struct GramTiles {
    int64_t rows, W, nb;
    bool sym;
    int32_t k_begin, k_end;  // only the nonzeros Phi[i, k] with k in [k_begin, k_end) contribute
    int64_t J_off = 0;       // the launch's bands are the global bands J_off .. J_off + nb - 1
    int64_t t_rows = -1;     // rows of the transposed matrix (< 0: n_total, the square case)
    bool add_k = false;      // write-out adds to K (which holds the dense hub-column part: grf_gram_sparse_upper_add)
    __host__ __device__ int64_t count(int64_t J) const {
        if (!sym) return rows;
        const int64_t c = (J + 1) * W;
        return c < rows ? c : rows;
    }
    // tiles before band J
    __host__ __device__ int64_t before(int64_t J) const {
        if (!sym) return J * rows;
        const int64_t full = (rows + W - 1) / W - 1;  // bands J < full hold (J + 1) W rows
        return J <= full ? W * J * (J + 1) / 2 : W * full * (full + 1) / 2 + (J - full) * rows;
    }
    __host__ __device__ int64_t total() const { return before(nb); }
    // band and local row of tile t
    __device__ void locate(int64_t t, int64_t &J, int64_t &r) const {
        if (!sym) {
            J = t / rows;
        } else {
            J = (int64_t)((sqrt(8.0 * (double)(t / W) + 1.0) - 1.0) * 0.5);
            if (J > nb - 1) J = nb - 1;
            while (J > 0 && before(J) > t) --J;
            while (J < nb - 1 && before(J + 1) <= t) ++J;
        }
        r = t - before(J);
    }
};

// One workgroup of kWaves waves = one tile K[row, j0 : j0 + W] (W = a band of the banded
// transpose), accumulated in LDS in exact int64 fixed point with the per-row power-of-two
// scale S = 2^rowshift[row] (from the transpose) such that every term |Phi[row,k] Phi[j,k]| S
// < 2^51 and the sum of all terms < 2^62: each exact fp64 product is rounded once to an
// integer and the integer sum does not depend on the order of the adds (ds_add_u64) -- nor
// on scheduling, GPU count, row split or band width.
// Phi^T buckets hold 12-byte record pairs starting on 128-byte lines; wave w takes the
// batches w, w + kWaves, ... of 128 nonzeros of the row and flattens each batch's buckets
// into one stream of PAIRS.  The bucket of each pair comes from a per-position u8 bucket
// id (bucket-start markers propagated by a running maximum, one LDS read); the gathers of kGramUnroll
// windows of 64 pairs are in flight together.  Tiles are dispatched band-major, so the
// tiles in flight share one band's records (L2 / Infinity Cache).
// kSlot: the transpose is in the GRF_REC_SLOT layout -- bucket b's header {pairs, first overflow pair}
// and its first two pairs in the 32-byte slot t_rec + 32 b, the other pairs at t_rec + ovf_base + 12 p --
// so every nonzero contributes two virtual buckets (inline part, overflow part) to the wave's stream,
// and a small bucket costs one line (header and pairs) instead of a descriptor line and a record line.
template <int kWaves, int kHalves, int kGramUnroll, bool kTailExact, bool kSlot = false>
__global__ __launch_bounds__(64 * kWaves) void gram_sparse_kernel(
    int64_t n_total, int64_t row_begin, GramTiles tl, int64_t t_begin, const int64_t *__restrict__ ptr,
    const int32_t *__restrict__ idx, const float *__restrict__ val, const uint2 *__restrict__ t_desc,
    const unsigned char *__restrict__ t_rec, int32_t unit, const int32_t *__restrict__ rowshift,
    float *__restrict__ K, int64_t ldk, const uint16_t *__restrict__ t_split,
    int64_t ovf_base, int32_t balance, const int32_t *__restrict__ row_cuts) {
    extern __shared__ __attribute__((aligned(16))) unsigned long long acc[];  // [W]
    static_assert(!kSlot || kHalves == 1, "slot streams: 2 virtual buckets per nonzero, u8 ids <= 128");
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int64_t W = tl.W;
    constexpr int kB = 64 * kHalves;        // nonzeros per wave batch
    constexpr int kV = kSlot ? 2 * kHalves : kHalves;  // stream buckets per lane and batch
    unsigned char *st = reinterpret_cast<unsigned char *>(acc + W) + wave * wave_state_bytes(kV);
    unsigned char *bidv = st;                                          // [kChunk]
    int32_t *tbase = reinterpret_cast<int32_t *>(st + kChunk);         // [64 kV]
    float *aval = reinterpret_cast<float *>(st + kChunk + 64 * kV * 4);  // [64 kV]

    int64_t J, r;
    tl.locate(t_begin + (int64_t)blockIdx.x, J, r);
    const int64_t J_local = J;
    J += tl.J_off;  // global band
    const int64_t row = row_begin + r;
    const int64_t j0 = J * W;
    const int64_t t_rows = tl.t_rows < 0 ? n_total : tl.t_rows;  // (n_total: Phi's columns)
    const int64_t wlen = (t_rows - j0) < W ? (t_rows - j0) : W;
    const int64_t e0 = ptr[row], e1 = ptr[row + 1];
    const int64_t boff = J * n_total;
    const int sh = rowshift[row];
    const int32_t line0 = kSlot ? 0 : (int32_t)t_desc[boff].x;      // the band's first unit
    const unsigned char *brec = t_rec + (int64_t)line0 * unit;  // the band's records (slots: all of t_rec)
    // symmetric mode on the row's own band (a diagonal tile): only the columns j >= row are kept (the
    // mirror overwrites the rest), so with sub-band ordered buckets (t_split) every bucket stream starts
    // at the row's sub-band -- the pairs of the earlier sub-bands are never fetched -- and the write-out
    // starts at that sub-band's first column
    const int dsub = (t_split && tl.sym && r >= J_local * W) ? (int)(((r - J_local * W) * kSub) / W) : 0;

    typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));
    u64x2 *acc2 = reinterpret_cast<u64x2 *>(acc);
    const u64x2 z2 = {0ull, 0ull};
    for (int64_t i = tid; i < W / 2; i += 64 * kWaves) acc2[i] = z2;
    if (kWaves > 1) __syncthreads();
    else __builtin_amdgcn_wave_barrier();

    const GramStream gs{bidv, tbase, aval,
                        __builtin_amdgcn_make_buffer_rsrc(const_cast<unsigned char *>(brec), (short)0, 0x7fffffff,
                                                          0x00020000),
                        reinterpret_cast<unsigned char *>(acc), ldexp(1.0, sh), kSlot ? 8 : 0};
    // the row's nonzeros over the waves: balance = 1: wave w takes the w-th of kWaves equal contiguous
    // shares, in batches of kB (a tile ends with its slowest wave: C4's ~435 nonzeros as 109 per wave
    // instead of 128 / 128 / 128 / 51); 0: batches w, w + kWaves, ... of kB
    const int64_t nnz_row = e1 - e0, share = (nnz_row + kWaves - 1) / kWaves;
    int64_t ws0 = balance ? e0 + (wave * share < nnz_row ? wave * share : nnz_row) : e0 + (int64_t)wave * kB;
    int64_t ws1 = balance ? e0 + ((wave + 1) * share < nnz_row ? (wave + 1) * share : nnz_row) : e1;
    if (row_cuts) {
        // shares of about equal record pairs (grf_gram_row_cuts: 8 cuts per row from the columns'
        // pair counts over all bands; a kWaves-wave tile takes every (8 / kWaves)-th)
        static_assert(8 % kWaves == 0, "row cuts: 8 shares per row");
        constexpr int kStep = 8 / kWaves;
        ws0 = e0 + row_cuts[row * 8 + wave * kStep];
        ws1 = wave + 1 < kWaves ? e0 + row_cuts[row * 8 + (wave + 1) * kStep] : e1;
    }
    const int64_t gstep = (balance || row_cuts) ? kB : (int64_t)kB * kWaves;
    for (int64_t g0 = ws0; g0 < ws1; g0 += gstep) {
        const int64_t gend = (balance || row_cuts) ? ((g0 + kB) < ws1 ? g0 + kB : ws1) : e1;
        int32_t cnt[kV], excl[kV], t0[kV];
        float av[kV];
#pragma unroll
        for (int h = 0; h < kHalves; ++h) {
            const int64_t e = g0 + h * 64 + lane;
            int32_t k = e < gend ? idx[e] : -1;
            if (k < tl.k_begin || k >= tl.k_end) k = -1;  // (k-slice mode)
            const float a = k >= 0 ? val[e] : 0.f;
            if constexpr (kSlot) {
                // the slot's header and inline pairs share its line; the overflow pairs follow all slots
                const int64_t sb = 32 * (boff + (k >= 0 ? k : 0));
                const uint2 d = k >= 0 ? *reinterpret_cast<const uint2 *>(t_rec + sb) : make_uint2(0u, 0u);
                const int32_t inl = min((int32_t)d.x, 2);
                t0[2 * h] = (int32_t)sb + 8;
                cnt[2 * h] = inl;
                t0[2 * h + 1] = (int32_t)ovf_base + kPairBytesG * (int32_t)d.y;
                cnt[2 * h + 1] = (int32_t)d.x - inl;
                av[2 * h] = a;
                av[2 * h + 1] = a;
            } else {
                av[h] = a;
                const uint2 d = k >= 0 ? t_desc[boff + k] : make_uint2((uint32_t)line0, 0u);
                // pairs of the sub-bands before the row's (diagonal tiles; capped: a dropped hub bucket has 0)
                const int32_t skip = (dsub > 0 && k >= 0) ? min((int32_t)(t_split[(boff + k) * kSub + dsub] >> 1), (int32_t)d.y) : 0;
                t0[h] = ((int32_t)d.x - line0) * unit + kPairBytesG * skip;  // first fetched byte within the band
                cnt[h] = (int32_t)d.y - skip;                                   // pairs
            }
        }
        int32_t total = 0;
#pragma unroll
        for (int h = 0; h < kV; ++h) {
            const int32_t inc = wave_inclusive_scan<int32_t>(cnt[h]) + total;  // (DPP: grf_block.h)
            excl[h] = inc - cnt[h];
            total = __builtin_amdgcn_readlane(inc, 63);
        }
#pragma unroll
        for (int h = 0; h < kV; ++h) {
            tbase[h * 64 + lane] = t0[h] - 12 * excl[h];  // byte offset = tbase + 12 * position
            aval[h * 64 + lane] = av[h];
        }
        int carry = 0;
        // (chunks of 256 / 512 positions when the stream is that short: the propagation's VALU scales with it)
        const int32_t chunk = total <= 256 ? 256 : total <= 512 ? 512 : kChunk;
        for (int32_t c0 = 0; c0 < total; c0 += chunk) {
            const int32_t cend = (total - c0) < chunk ? total : c0 + chunk;
            // bucket ids of the chunk: clear, mark every non-empty bucket's first position, propagate
            if (chunk == 256) reinterpret_cast<uint32_t *>(bidv)[lane] = 0u;
            else if (chunk == 512) reinterpret_cast<uint2 *>(bidv)[lane] = make_uint2(0u, 0u);
            else reinterpret_cast<uint4 *>(bidv)[lane] = make_uint4(0u, 0u, 0u, 0u);
            __builtin_amdgcn_wave_barrier();
#pragma unroll
            for (int h = 0; h < kV; ++h)
                if (cnt[h] > 0 && excl[h] >= c0 && excl[h] < cend)
                    bidv[excl[h] - c0] = (unsigned char)(h * 64 + lane + 1);
            __builtin_amdgcn_wave_barrier();
            carry = chunk == 256   ? gram_propagate_ids_n<1>(bidv, carry, lane)
                    : chunk == 512 ? gram_propagate_ids_n<2>(bidv, carry, lane)
                                   : gram_propagate_ids(bidv, carry, lane);
            __builtin_amdgcn_wave_barrier();
            int32_t w0 = c0;
            for (; w0 + 64 * kGramUnroll <= cend; w0 += 64 * kGramUnroll)
                gram_windows<kGramUnroll, 0>(gs, w0, c0, cend, lane);
            if (w0 < cend) {
                // last group: exactly the windows left (a group of kGramUnroll would issue up to
                // kGramUnroll - 1 all-masked windows of loads and LDS adds per batch)
                if (kTailExact) {
                    switch ((cend - w0 + 63) >> 6) {
                        case 1: gram_windows<1, 1>(gs, w0, c0, cend, lane); break;
                        case 2: gram_windows<2, 1>(gs, w0, c0, cend, lane); break;
                        case 3: gram_windows<3, 1>(gs, w0, c0, cend, lane); break;
                        case 4: gram_windows<4, 1>(gs, w0, c0, cend, lane); break;
                        case 5: gram_windows<kGramUnroll < 5 ? kGramUnroll : 5, 1>(gs, w0, c0, cend, lane); break;
                        case 6: gram_windows<kGramUnroll < 6 ? kGramUnroll : 6, 1>(gs, w0, c0, cend, lane); break;
                        case 7: gram_windows<kGramUnroll < 7 ? kGramUnroll : 7, 1>(gs, w0, c0, cend, lane); break;
                        // (unroll <= 8: exactly kGramUnroll windows are left here; 16: 8 .. 16 are, so every window is masked)
                        default: gram_windows<kGramUnroll, (kGramUnroll <= 8 ? 1 : 2)>(gs, w0, c0, cend, lane); break;
                    }
                } else {
                    gram_windows<kGramUnroll, 2>(gs, w0, c0, cend, lane);  // masked last group
                }
            }
            __builtin_amdgcn_wave_barrier();
        }
    }
    if (kWaves > 1) __syncthreads();
    else __builtin_amdgcn_wave_barrier();

    // write the tile once (non-temporal: K is write-once); add_k: K already holds the dense
    // hub-column part of these entries, and the fixed-point sum is rounded once and added to it
    float *krow = K + r * ldk + j0;
    const bool addk = tl.add_k;
    const int64_t c_lo = (int64_t)dsub * (W / kSub);  // (a multiple of 8: W % 64 == 0)
    if ((ldk & 3) == 0 && (j0 & 3) == 0) {
        const int64_t n4 = wlen / 4;
        f32x4 *k4 = reinterpret_cast<f32x4 *>(krow);
        for (int64_t i = c_lo / 4 + tid; i < n4; i += 64 * kWaves) {
            const u64x2 a = acc2[2 * i], b = acc2[2 * i + 1];
            f32x4 o;
            o[0] = fx_to_float(a[0], sh);
            o[1] = fx_to_float(a[1], sh);
            o[2] = fx_to_float(b[0], sh);
            o[3] = fx_to_float(b[1], sh);
            if (addk) o += __builtin_nontemporal_load(&k4[i]);
            GRF_K_STORE(o, &k4[i]);
        }
        for (int64_t i = n4 * 4 + tid; i < wlen; i += 64 * kWaves)
            krow[i] = addk ? fx_to_float(acc[i], sh) + krow[i] : fx_to_float(acc[i], sh);
    } else {
        for (int64_t i = tid; i < wlen; i += 64 * kWaves)
            krow[i] = addk ? fx_to_float(acc[i], sh) + krow[i] : fx_to_float(acc[i], sh);
    }
}

// ------------------------------------------------- pipelined column-block tiles (GRF_REC_SLOT buckets)
// The column-block Gram of the slot layout (C5: 1M tiles K[i, 0:8192]) as a persistent kernel of two
// workgroups per CU (the LDS holds two 64 KB accumulators), each taking the tiles blockIdx.x + i gridDim.x in
// turn: tile i's gathers, a barrier, tile i's write-out and zeroing, a barrier.  A tile's dependent chain (row
// bounds -> the wave's nonzeros -> their slot headers -> record pairs) is software-pipelined over the tiles:
// the headers of tile i + 1, the nonzeros of tile i + 2 and the bounds of tile i + 3 are issued at the start of
// tile i, behind tile i - 1's K stores, so tile i's one wait covers the stores' completion, the prefetches and
// its own gathers (vmcnt counts loads and stores together in issue order) -- about one round trip per tile,
// against four dependent ones for gram_sparse_kernel -- while the CU's other workgroup overlaps it.  Same
// integer sums: identical bits.  Measured and removed (profiles/r06_c5_gram_ab.txt, AB_LOG round 6): gather and
// store waves split by role around double accumulators in one workgroup per CU; loader waves filling an LDS
// ring with each tile's nonzeros and headers; a wave prefetching the nonzeros into L2.
__device__ __forceinline__ void pipe_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

struct PipeNz {     // one tile's first batch of this wave's nonzeros (one per lane) and its bounds
    int32_t k;      // column (-1: none)
    float a;        // Phi[row, k]
    int32_t sh;     // the row's fixed-point shift
    int32_t nb;     // the wave's share of the row's nonzeros
    int64_t ws0;    // first nonzero of the share
};

template <int kWv>
__global__ __launch_bounds__(64 * kWv) void gram_slot_pipe_kernel(
    int64_t n_cols, int64_t row_begin, int64_t rows, int64_t W, int64_t t_rows, int64_t n_tiles,
    const int64_t *__restrict__ ptr, const int32_t *__restrict__ idx, const float *__restrict__ val,
    const unsigned char *__restrict__ t_rec, const int32_t *__restrict__ rowshift, float *__restrict__ K,
    int64_t ldk, int64_t ovf_base, int32_t ablate, int64_t pad_cap, const int32_t *__restrict__ pad_cnt) {
    extern __shared__ __attribute__((aligned(16))) unsigned long long acc[];  // [W], then the waves' stream state
    typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));
    constexpr int kV = 2;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int64_t G = gridDim.x;
    const int64_t n_mine = (int64_t)blockIdx.x < n_tiles ? (n_tiles - 1 - (int64_t)blockIdx.x) / G + 1 : 0;
    u64x2 *acc2 = reinterpret_cast<u64x2 *>(acc);
    const u64x2 z2 = {0ull, 0ull};
    for (int64_t q = tid; q < W / 2; q += 64 * kWv) acc2[q] = z2;
    unsigned char *st = reinterpret_cast<unsigned char *>(acc + W) + wave * wave_state_bytes(kV);
    unsigned char *bidv = st;                                             // [kChunk]
    int32_t *tbase = reinterpret_cast<int32_t *>(st + kChunk);            // [64 kV]
    float *aval = reinterpret_cast<float *>(st + kChunk + 64 * kV * 4);  // [64 kV]
    const __amdgpu_buffer_rsrc_t rec_rs =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<unsigned char *>(t_rec), (short)0, 0x7fffffff, 0x00020000);
    auto tile_row = [&](int64_t i, int64_t &J) -> int64_t {
        const int64_t t = (int64_t)blockIdx.x + i * G;
        J = t / rows;
        return row_begin + (t - J * rows);
    };
    // the row bounds: from the CSR row pointers (lanes 0 / 1: ptr[row], ptr[row + 1]), or with pad_cap > 0 from
    // padded rows (row r's pad_cnt[r] entries at r pad_cap: the walk's output, no compaction) -- the count kept
    // as loaded (pc) and combined only in load_nz, so no ALU op waits on the load here
    auto load_bounds = [&](int64_t i, int64_t &pv, int32_t &pc, int32_t &shv) {
        if (i >= n_mine) {
            pv = 0;
            pc = 0;
            shv = 0;
            return;
        }
        int64_t J;
        const int64_t row = tile_row(i, J);
        if (pad_cap > 0) {
            const __amdgpu_buffer_rsrc_t rc =
                __builtin_amdgcn_make_buffer_rsrc(const_cast<int32_t *>(pad_cnt + row), (short)0, 4, 0x00020000);
            pc = (int32_t)__builtin_amdgcn_raw_buffer_load_b32(rc, 0u, 0, 0);
        } else {
            const __amdgpu_buffer_rsrc_t rp =
                __builtin_amdgcn_make_buffer_rsrc(const_cast<int64_t *>(ptr + row), (short)0, 16, 0x00020000);
            const auto v = __builtin_amdgcn_raw_buffer_load_b64(rp, (uint32_t)(lane & 1) * 8u, 0, 0);
            pv = (int64_t)(((uint64_t)v[1] << 32) | v[0]);
        }
        const __amdgpu_buffer_rsrc_t rs =
            __builtin_amdgcn_make_buffer_rsrc(const_cast<int32_t *>(rowshift + row), (short)0, 4, 0x00020000);
        shv = (int32_t)__builtin_amdgcn_raw_buffer_load_b32(rs, 0u, 0, 0);
    };
    auto load_nz = [&](int64_t i, int64_t pv, int32_t pc, int32_t shv, PipeNz &z) {
        if (i >= n_mine) {
            z = PipeNz{-1, 0.f, 0, 0, 0};
            return;
        }
        auto lane_i64 = [&](int l) {
            const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)pv, l);
            const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)((uint64_t)pv >> 32), l);
            return (int64_t)(((uint64_t)hi << 32) | lo);
        };
        int64_t e0, e1;
        if (pad_cap > 0) {
            int64_t J;
            e0 = tile_row(i, J) * pad_cap;
            e1 = e0 + (int64_t)__builtin_amdgcn_readlane(pc, 0);
        } else {
            e0 = lane_i64(0);
            e1 = lane_i64(1);
        }
        const int64_t nnz = e1 - e0, share = (nnz + kWv - 1) / kWv;
        const int64_t s0 = wave * share < nnz ? wave * share : nnz, s1 = (wave + 1) * share < nnz ? (wave + 1) * share : nnz;
        const int64_t e = e0 + s0 + lane;
        const bool ok = s0 + lane < s1;
        z.k = ok ? idx[e] : -1;
        z.a = ok ? val[e] : 0.f;
        z.sh = shv;
        z.nb = (int32_t)(s1 - s0);
        z.ws0 = e0 + s0;
    };
    auto load_hdr = [&](int64_t i, int32_t k) -> uint2 {
        if (i >= n_mine || k < 0) return make_uint2(0u, 0u);
        int64_t J;
        tile_row(i, J);
        return *reinterpret_cast<const uint2 *>(t_rec + 32 * (J * n_cols + k));
    };
    auto run_batch = [&](const GramStream &gs, int64_t J, int32_t k, float a, uint2 d) {
        int32_t cnt[kV], excl[kV], t0[kV];
        const int32_t sb = (int32_t)(32 * (J * n_cols + (k >= 0 ? k : 0)));
        const int32_t inl = k >= 0 ? min((int32_t)d.x, 2) : 0;
        t0[0] = sb + 8;
        cnt[0] = inl;
        t0[1] = (int32_t)ovf_base + kPairBytesG * (int32_t)d.y;
        cnt[1] = k >= 0 ? (int32_t)d.x - inl : 0;
        int32_t total = 0;
#pragma unroll
        for (int h = 0; h < kV; ++h) {
            const int32_t inc = wave_inclusive_scan<int32_t>(cnt[h]) + total;
            excl[h] = inc - cnt[h];
            total = __builtin_amdgcn_readlane(inc, 63);
        }
#pragma unroll
        for (int h = 0; h < kV; ++h) {
            tbase[h * 64 + lane] = t0[h] - 12 * excl[h];
            aval[h * 64 + lane] = a;
        }
        int carry = 0;
        const int32_t chunk = total <= 256 ? 256 : total <= 512 ? 512 : kChunk;
        for (int32_t c0 = 0; c0 < total; c0 += chunk) {
            const int32_t cend = (total - c0) < chunk ? total : c0 + chunk;
            if (chunk == 256) reinterpret_cast<uint32_t *>(bidv)[lane] = 0u;
            else if (chunk == 512) reinterpret_cast<uint2 *>(bidv)[lane] = make_uint2(0u, 0u);
            else reinterpret_cast<uint4 *>(bidv)[lane] = make_uint4(0u, 0u, 0u, 0u);
            __builtin_amdgcn_wave_barrier();
#pragma unroll
            for (int h = 0; h < kV; ++h)
                if (cnt[h] > 0 && excl[h] >= c0 && excl[h] < cend) bidv[excl[h] - c0] = (unsigned char)(h * 64 + lane + 1);
            __builtin_amdgcn_wave_barrier();
            carry = chunk == 256   ? gram_propagate_ids_n<1>(bidv, carry, lane)
                    : chunk == 512 ? gram_propagate_ids_n<2>(bidv, carry, lane)
                                   : gram_propagate_ids(bidv, carry, lane);
            __builtin_amdgcn_wave_barrier();
            int32_t w0 = c0;
            for (; w0 + 64 * 8 <= cend; w0 += 64 * 8) gram_windows<8, 0>(gs, w0, c0, cend, lane);
            if (w0 < cend) {
                switch ((cend - w0 + 63) >> 6) {
                    case 1: gram_windows<1, 1>(gs, w0, c0, cend, lane); break;
                    case 2: gram_windows<2, 1>(gs, w0, c0, cend, lane); break;
                    case 3: gram_windows<3, 1>(gs, w0, c0, cend, lane); break;
                    case 4: gram_windows<4, 1>(gs, w0, c0, cend, lane); break;
                    case 5: gram_windows<5, 1>(gs, w0, c0, cend, lane); break;
                    case 6: gram_windows<6, 1>(gs, w0, c0, cend, lane); break;
                    case 7: gram_windows<7, 1>(gs, w0, c0, cend, lane); break;
                    default: gram_windows<8, 1>(gs, w0, c0, cend, lane); break;
                }
            }
            __builtin_amdgcn_wave_barrier();
        }
    };
    int64_t pv = 0;
    int32_t pc = 0, shv;
    PipeNz T0, T1;
    load_bounds(0, pv, pc, shv);
    load_nz(0, pv, pc, shv, T0);
    uint2 d0 = load_hdr(0, T0.k);
    load_bounds(1, pv, pc, shv);
    load_nz(1, pv, pc, shv, T1);
    load_bounds(2, pv, pc, shv);
    __builtin_amdgcn_s_waitcnt(0);
    pipe_barrier();
    for (int64_t i = 0; i < n_mine; ++i) {
        const uint2 d1 = load_hdr(i + 1, T1.k);
        PipeNz T2;
        load_nz(i + 2, pv, pc, shv, T2);
        load_bounds(i + 3, pv, pc, shv);
        int64_t J;
        const int64_t row = tile_row(i, J);
        if (ablate != 1) {
            const GramStream gs{bidv, tbase, aval, rec_rs, reinterpret_cast<unsigned char *>(acc), ldexp(1.0, T0.sh), 8};
            run_batch(gs, J, T0.k, T0.a, d0);
            for (int32_t g = 64; g < T0.nb; g += 64) {  // (a share past 64 nonzeros: batch by batch)
                const int64_t e = T0.ws0 + g + lane;
                const bool ok = g + lane < T0.nb;
                const int32_t k = ok ? idx[e] : -1;
                const float a = ok ? val[e] : 0.f;
                const uint2 d = k >= 0 ? *reinterpret_cast<const uint2 *>(t_rec + 32 * (J * n_cols + k)) : make_uint2(0u, 0u);
                run_batch(gs, J, k, a, d);
            }
        }
        // Every load of this tile and the prefetches issued at its start is complete here in practice (the
        // gathers' last window waited for them: vmcnt is in order), but the wait-count pass cannot see it through
        // the data-dependent batch loops, so it would guard the next tile's uses of the prefetched registers with a
        // vmcnt(0) behind this tile's K stores -- a store round trip per tile before the next one's loads issue.
        // Said explicitly here, before the stores, the stores stay in flight into the next tile.
        __builtin_amdgcn_s_waitcnt(0);
        pipe_barrier();
        // tile i out (non-temporal) and its accumulator zeroed
        const int64_t r = row - row_begin, j0 = J * W;
        const int64_t wlen = (t_rows - j0) < W ? (t_rows - j0) : W;
        const int sh = T0.sh;
        float *krow = K + r * ldk + j0;
        int64_t done = 0;
        if ((ldk & 3) == 0 && (j0 & 3) == 0) {
            const int64_t n4 = wlen / 4;
            f32x4 *k4 = reinterpret_cast<f32x4 *>(krow);
            for (int64_t q = tid; q < n4; q += 64 * kWv) {
                const u64x2 x = acc2[2 * q], y = acc2[2 * q + 1];
                f32x4 o;
                o[0] = fx_to_float(x[0], sh);
                o[1] = fx_to_float(x[1], sh);
                o[2] = fx_to_float(y[0], sh);
                o[3] = fx_to_float(y[1], sh);
                if (ablate != 2) GRF_K_STORE(o, &k4[q]);
                acc2[2 * q] = z2;
                acc2[2 * q + 1] = z2;
            }
            done = n4 * 4;
        }
        for (int64_t q = done + tid; q < wlen; q += 64 * kWv) {
            if (ablate != 2) krow[q] = fx_to_float(acc[q], sh);
            acc[q] = 0ull;
        }
        pipe_barrier();
        T0 = T1;
        d0 = d1;
        T1 = T2;
    }
}

// Hub columns (the densest columns of Phi): their entries as a dense fp32 panel
// P[r, hub_pos[k]] = Phi[r, k] (P zeroed by the caller; hub_pos[k] = -1 for the other columns),
// one wave per row.  The MFMA Gram of P carries those columns' share of K.
__global__ __launch_bounds__(256) void hub_panel_kernel(int64_t n_rows, const int64_t *__restrict__ ptr,
                                                        const int32_t *__restrict__ idx, const float *__restrict__ val,
                                                        const int32_t *__restrict__ hub_pos, float *__restrict__ P,
                                                        int64_t ldp) {
    const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= n_rows) return;
    const int lane = threadIdx.x & 63;
    const int64_t e1 = ptr[row + 1];
    for (int64_t e = ptr[row] + lane; e < e1; e += 64) {
        const int32_t q = hub_pos[idx[e]];
        if (q >= 0) P[row * ldp + q] = val[e];
    }
}

// the hub columns' buckets emptied in every band of a banded transpose (descriptor pair counts
// set to 0), so the sparse Gram skips the entries the panel carries
__global__ __launch_bounds__(256) void transpose_drop_kernel(int64_t n_bands, int64_t n_cols, uint2 *__restrict__ t_desc,
                                                             const int32_t *__restrict__ cols, int32_t n_drop) {
    const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (t >= n_bands * n_drop) return;
    const int64_t J = t / n_drop;
    t_desc[J * n_cols + cols[t - J * n_drop]].y = 0u;
}

// block b of the row-major upper triangle (bj >= bi) of an nt x nt block grid -> (bi, bj)
__device__ __forceinline__ void gram_mirror_tri_coords(int64_t nt, int64_t b, int64_t &bi_out, int64_t &bj_out) {
    int64_t bi = (int64_t)(((double)(2 * nt + 1) - sqrt((double)(2 * nt + 1) * (double)(2 * nt + 1) - 8.0 * (double)b)) * 0.5);
    auto first = [nt](int64_t i) { return i * nt - i * (i - 1) / 2; };  // first block of block-row i
    if (bi < 0) bi = 0;
    if (bi > nt - 1) bi = nt - 1;
    while (bi > 0 && first(bi) > b) --bi;
    while (bi < nt - 1 && first(bi + 1) <= b) ++bi;
    bi_out = bi;
    bj_out = bi + (b - first(bi));
}

// K[j, i] = K[i, j] for the 64 x 64 block (bi, bj), bj >= bi (diagonal: j > i inside the block)
__device__ __forceinline__ void gram_mirror_block_at(int64_t n, int64_t bi, int64_t bj, float *__restrict__ K,
                                                     int64_t ldk, float (*tile)[65]) {
    const int64_t i0 = bi * 64, j0 = bj * 64;
    const int t = threadIdx.x;
    const bool full = i0 + 64 <= n && j0 + 64 <= n && (ldk & 3) == 0;
    // load K[i0 + y, j0 .. j0 + 63]: 16 float4 per row, 4 rows per pass
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int y = (t >> 4) + 16 * q, x = (t & 15) * 4;
        const int64_t i = i0 + y;
        if (full) {
            const f32x4 v = __builtin_nontemporal_load(reinterpret_cast<const f32x4 *>(K + i * ldk + j0 + x));
            tile[y][x] = v[0]; tile[y][x + 1] = v[1]; tile[y][x + 2] = v[2]; tile[y][x + 3] = v[3];
        } else {
#pragma unroll
            for (int c = 0; c < 4; ++c) tile[y][x + c] = (i < n && j0 + x + c < n) ? K[i * ldk + j0 + x + c] : 0.f;
        }
    }
    __syncthreads();
    // store K[j0 + y, i0 .. i0 + 63] = column y of the tile (strictly below the diagonal)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int y = (t >> 4) + 16 * q, x = (t & 15) * 4;
        const int64_t j = j0 + y;
        if (full && bi != bj) {
            f32x4 v;
            v[0] = tile[x][y]; v[1] = tile[x + 1][y]; v[2] = tile[x + 2][y]; v[3] = tile[x + 3][y];
            __builtin_nontemporal_store(v, reinterpret_cast<f32x4 *>(K + j * ldk + i0 + x));
        } else {
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                const int64_t i = i0 + x + c;
                if (j < n && i < n && j > i) K[j * ldk + i] = tile[x + c][y];
            }
        }
    }
}

// The LDS block without bank conflicts: the 64 x 64 block is stored unpadded with its 16-byte chunks
// XOR-swizzled by row (element (r, c) at word r * 64 + (c ^ 4 ((r >> 2) & 15))).  Loads of K rows
// (256 B per row and wave-instruction) go in with ds_write_b128 (8 lanes per LDS cycle: 8 distinct
// chunks); each thread then reads two adjacent source columns of four source rows with ds_read_b64
// (64 banks; lanes {4k + c} x {y, y + 2} hit 32 distinct bank pairs) and stores two output rows of
// 16 B (256 B per row and wave-instruction).
__device__ __forceinline__ void gram_mirror_block_swz_at(int64_t n, int64_t bi, int64_t bj, float *__restrict__ K,
                                                         int64_t ldk, float *__restrict__ tile) {
    const int64_t i0 = bi * 64, j0 = bj * 64;
    const int t = threadIdx.x;
    const bool full = i0 + 64 <= n && j0 + 64 <= n && (ldk & 3) == 0 && bi != bj;
    if (!full) {  // diagonal / ragged blocks: the padded-tile path (same LDS)
        gram_mirror_block_at(n, bi, bj, K, ldk, reinterpret_cast<float(*)[65]>(tile));
        return;
    }
    auto swz = [](int r, int c) { return r * 64 + (c ^ (4 * ((r >> 2) & 15))); };
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int y = (t >> 4) + 16 * q, x = (t & 15) * 4;
        const f32x4 v = GRF_K_LOAD(reinterpret_cast<const f32x4 *>(K + (i0 + y) * ldk + j0 + x));
        *reinterpret_cast<f32x4 *>(tile + swz(y, x)) = v;
    }
    __syncthreads();
    const int k = t & 15, pr = t >> 4;
#pragma unroll
    for (int it = 0; it < 2; ++it) {
        const int y = 2 * pr + 32 * it;  // output rows y, y + 1 (source columns)
        typedef float f32x2 __attribute__((ext_vector_type(2)));
        typedef __attribute__((address_space(3))) float lds_float;
        uint32_t a[4];
#pragma unroll
        for (int c = 0; c < 4; ++c) a[c] = (uint32_t)(uintptr_t)(lds_float *)(tile + swz(4 * k + c, y));
        f32x2 v[4];
        // four single ds_read_b64 (the compiler would pair them into ds_read2_b64, whose 32-bank
        // halves conflict 2-way on this layout)
        asm volatile(
            "ds_read_b64 %0, %4\n\tds_read_b64 %1, %5\n\tds_read_b64 %2, %6\n\tds_read_b64 %3, %7\n\t"
            "s_waitcnt lgkmcnt(0)"
            : "=&v"(v[0]), "=&v"(v[1]), "=&v"(v[2]), "=&v"(v[3])
            : "v"(a[0]), "v"(a[1]), "v"(a[2]), "v"(a[3])
            : "memory");
        f32x4 o0, o1;
        o0[0] = v[0].x; o0[1] = v[1].x; o0[2] = v[2].x; o0[3] = v[3].x;
        o1[0] = v[0].y; o1[1] = v[1].y; o1[2] = v[2].y; o1[3] = v[3].y;
        __builtin_nontemporal_store(o0, reinterpret_cast<f32x4 *>(K + (j0 + y) * ldk + i0 + 4 * k));
        __builtin_nontemporal_store(o1, reinterpret_cast<f32x4 *>(K + (j0 + y + 1) * ldk + i0 + 4 * k));
    }
}

__device__ __forceinline__ void gram_mirror_block_swz(int64_t n, int64_t nt, int64_t b, float *__restrict__ K,
                                                      int64_t ldk, float *__restrict__ tile) {
    int64_t bi, bj;
    gram_mirror_tri_coords(nt, b, bi, bj);
    gram_mirror_block_swz_at(n, bi, bj, K, ldk, tile);
}

__global__ __launch_bounds__(256) void gram_mirror_swz_kernel(int64_t n, int64_t nt, int64_t nblocks,
                                                              float *__restrict__ K, int64_t ldk) {
    __shared__ __attribute__((aligned(16))) float tile[64 * 65];
    for (int64_t b = blockIdx.x; b < nblocks; b += gridDim.x) {
        gram_mirror_block_swz(n, nt, b, K, ldk, tile);
        __syncthreads();
    }
}

__global__ void absmax_reset_kernel(float *m) { *m = 0.f; }

__global__ __launch_bounds__(256) void densify_kernel(int64_t n_rows, const int64_t *__restrict__ ptr,
                                                      const int32_t *__restrict__ idx, const float *__restrict__ val,
                                                      float *__restrict__ out, int64_t lda) {
    const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= n_rows) return;
    const int lane = threadIdx.x & 63;
    for (int64_t e = ptr[row] + lane; e < ptr[row + 1]; e += 64) out[row * lda + idx[e]] = val[e];
}

// The dense path's Phi straight from the walk's padded rows (no compaction): one workgroup per row builds the
// zero-padded fp32 row in LDS (zero, scatter the row's entries, copy out with 16-B loads and stores), so the
// row is written once, whole, with no separate memset pass over the matrix.
__global__ __launch_bounds__(256) void densify_padded_kernel(int64_t cap, const int32_t *__restrict__ cnt,
                                                             const int32_t *__restrict__ idx,
                                                             const float *__restrict__ val, float *__restrict__ out,
                                                             int64_t lda) {
    extern __shared__ __attribute__((aligned(16))) float row[];  // [lda]
    const int64_t r = blockIdx.x;
    const int tid = threadIdx.x;
    const int q4 = (int)(lda >> 2);
    for (int t = tid; t < q4; t += 256) reinterpret_cast<float4 *>(row)[t] = float4{0.f, 0.f, 0.f, 0.f};
    __syncthreads();
    const int64_t b = r * cap;
    const int c = cnt[r];
    for (int e = tid; e < c; e += 256) row[idx[b + e]] = val[b + e];
    __syncthreads();
    float4 *o = reinterpret_cast<float4 *>(out + r * lda);
    for (int t = tid; t < q4; t += 256) o[t] = reinterpret_cast<const float4 *>(row)[t];
}

// grf_gram_dense.hip: the dense path's MFMA Gram
size_t dense_gram_workspace_bytes(int64_t n, int64_t k_dim);
size_t dense_gram_split_workspace_bytes(int64_t n, int64_t k_dim);
int32_t dense_gram_split(int64_t n, int64_t k_dim, const float *A, int64_t lda, float *K, int64_t ldk,
                         void *workspace, size_t workspace_bytes, bool upper_only, grf_stream_t stream);
int32_t dense_gram(int64_t n, int64_t k_dim, const float *A, int64_t lda, float *K, int64_t ldk, void *workspace,
                   size_t workspace_bytes, bool upper_only, grf_stream_t stream);
int64_t planes_row_bytes(int64_t k_dim);
int32_t split_planes(int64_t n, int64_t k_dim, const float *A, int64_t lda, void *P, int64_t ldp, grf_stream_t stream);
int32_t densify_padded_planes(int64_t n_rows, int64_t cap, int64_t n_cols, const int32_t *cnt, const int32_t *idx,
                              const float *val, void *P, int64_t ldp, grf_stream_t stream);
int32_t dense_gram_planes(int64_t n, int64_t k_dim, const void *P, int64_t ldp, float *K, int64_t ldk,
                          void *workspace, size_t workspace_bytes, grf_stream_t stream);

}  // namespace grf

using namespace grf;

extern "C" {
#pragma GCC visibility push(default)

size_t grf_gram_workspace_bytes(void) { return 256; }

// tiles [t_first, t_last) of one Gram call
// Equal contiguous shares of a row's nonzeros per wave (1) or round-robin batches (0): measured
// (profiles/r03_gram_balance_ab.txt) C5's slot tiles 19.2 -> 18.4 ms per step, Enron 9.4 -> 8.7 ms,
// C4's whole-K tiles -0.5 %; the N > 1 column blocks of line buckets (8-wave tiles, ~435 nonzeros:
// round-robin keeps 7 waves of 64) +2..5 %, so those keep round-robin batches.
// GRF_GRAM_BALANCE=0 / 1 forces either (A/B knob).
static int32_t gram_balance(const GramTiles &tl, int32_t unit) {
    static const int32_t force = [] {
        const char *e = getenv("GRF_GRAM_BALANCE");
        return e ? (int32_t)(atoi(e) != 0) : (int32_t)-1;
    }();
    if (force >= 0) return force;
    return (unit == GRF_REC_SLOT || tl.t_rows < 0) ? 1 : 0;
}

static int32_t gram_tiles_launch(int64_t n_total, int64_t row_begin, const GramTiles &tl, int64_t t_first,
                                 int64_t t_last, const int64_t *ptr, const int32_t *idx, const float *val,
                                 const uint32_t *t_desc, const void *t_rec, int32_t unit, const int32_t *t_rowshift,
                                 float *K, int64_t ldk, hipStream_t st, const void *t_split = nullptr,
                                 int64_t slot_buckets = 0, const int32_t *row_cuts = nullptr, int64_t pad_cap = 0,
                                 const int32_t *pad_cnt = nullptr) {
    if (unit == GRF_REC_SLOT) {
        // the slot layout: 8-wave tiles (one batch of 64 nonzeros per wave: two stream buckets each),
        // the default unroll and exact tails; the overflow pairs follow the slot_buckets slots
        GRF_REQUIRE(!t_split, GRF_EUNSUPPORTED, "gram: GRF_REC_SLOT has no split variant");
        GRF_REQUIRE(32 * slot_buckets < ((int64_t)1 << 30), GRF_EUNSUPPORTED,
                    "gram: GRF_REC_SLOT slots beyond 32-bit record offsets");
        // column blocks (a whole launch of non-symmetric tiles over all columns): the persistent software-pipelined
        // kernel, GRF_GRAM_PIPE=0: the tile-per-workgroup kernel below (read per call: the bit-identity test
        // switches it; GRF_GRAM_PIPE_ABLATE=1 / 2 are timing-only ablations -- no gathers / no K stores -- whose
        // K is wrong; profiles/r06_c5_gram_ab.txt)
        const bool pipe = [] {
            const char *e = getenv("GRF_GRAM_PIPE");
            return !e || atoi(e) != 0;
        }();
        const int32_t ablate = [] {
            const char *e = getenv("GRF_GRAM_PIPE_ABLATE");
            return e ? (int32_t)atoi(e) : 0;
        }();
        const bool pipe_ok = !tl.sym && tl.t_rows >= 0 && !tl.add_k && tl.k_begin == 0 &&
                             tl.k_end == (int32_t)n_total && t_first == 0 && t_last == tl.total() && tl.J_off == 0;
        GRF_REQUIRE(pad_cap == 0 || pipe_ok, GRF_EUNSUPPORTED,
                    "gram: padded rows need the pipelined column-block kernel (a whole non-symmetric launch)");
        if ((pipe || pad_cap > 0) && pipe_ok) {
            const size_t lds = gram_lds_bytes(tl.W, 8, 2);
            int dev = 0, n_cu = 0;
            GRF_CHECK_HIP(hipGetDevice(&dev));
            GRF_CHECK_HIP(hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev));
            const int per_cu = (int)std::max<int64_t>(1, (int64_t)(160 * 1024) / (int64_t)lds);
            const int64_t grid = std::min<int64_t>((int64_t)std::max(n_cu, 1) * per_cu, t_last);
            gram_slot_pipe_kernel<8><<<(unsigned)grid, 512, lds, st>>>(
                n_total, row_begin, tl.rows, tl.W, tl.t_rows, t_last, ptr, idx, val,
                reinterpret_cast<const unsigned char *>(t_rec), t_rowshift, K, ldk, 32 * slot_buckets, ablate, pad_cap,
                pad_cnt);
            GRF_CHECK_LAUNCH("gram_slot_pipe_kernel");
            return GRF_OK;
        }
        const size_t lds = gram_lds_bytes(tl.W, 8, 2);
        const int64_t max_tiles = ((1ll << 32) - 1) / (64 * 8);
        for (int64_t t0 = t_first; t0 < t_last; t0 += max_tiles) {
            const int64_t nt = (t_last - t0) < max_tiles ? (t_last - t0) : max_tiles;
            gram_sparse_kernel<8, 1, 8, true, true><<<(unsigned)nt, 512, lds, st>>>(
                n_total, row_begin, tl, t0, ptr, idx, val, reinterpret_cast<const uint2 *>(t_desc),
                reinterpret_cast<const unsigned char *>(t_rec), unit, t_rowshift, K, ldk, nullptr,
                32 * slot_buckets, gram_balance(tl, unit), nullptr);
            GRF_CHECK_LAUNCH("gram_sparse_kernel");
        }
        return GRF_OK;
    }
    // GRF_GRAM_SPLIT=0: ignore the sub-band split (A/B of the diagonal tiles' skip)
    static const bool use_split = [] {
        const char *e = getenv("GRF_GRAM_SPLIT");
        return !e || atoi(e) != 0;
    }();
    const uint16_t *split = (use_split && tl.sym) ? (const uint16_t *)t_split : nullptr;
    // waves per tile: 4 for W <= 4096 (4 tiles of 40 KiB per CU), 8 for wider bands (2 tiles of
    // 76 KiB per CU: 16 waves per CU either way); measured best at both widths (GRF_GRAM_WAVES=4/8
    // overrides); 8 windows of gathers in flight per wave and an exact-size last window group (the
    // round-1..3 sweeps of 4 / 16 windows and of masked tails: profiles/AB_LOG.md)
    static const int env_waves = [] {
        const char *w = getenv("GRF_GRAM_WAVES");
        const int ww = w ? atoi(w) : 0;
        return ww == 8 ? 8 : ww == 4 ? 4 : 0;
    }();
    const int waves = env_waves ? env_waves : (tl.W > 4096 ? 8 : 4);
    const size_t lds = gram_lds_bytes(tl.W, waves, waves == 8 ? 1 : 2);
    // one launch covers at most 2^32 - 1 work-items: split the tile range
    const int64_t max_tiles = ((1ll << 32) - 1) / (64 * waves);
    for (int64_t t0 = t_first; t0 < t_last; t0 += max_tiles) {
        const int64_t nt = (t_last - t0) < max_tiles ? (t_last - t0) : max_tiles;
#define GRF_GRAM_LAUNCH(WV, H)                                                                                    \
    gram_sparse_kernel<WV, H, 8, true><<<(unsigned)nt, 64 * WV, lds, st>>>(                                       \
        n_total, row_begin, tl, t0, ptr, idx, val, reinterpret_cast<const uint2 *>(t_desc),                       \
        reinterpret_cast<const unsigned char *>(t_rec), unit, t_rowshift, K, ldk, split, 0, gram_balance(tl, unit), \
        row_cuts)
        if (waves == 8) GRF_GRAM_LAUNCH(8, 1);
        else GRF_GRAM_LAUNCH(4, 2);
#undef GRF_GRAM_LAUNCH
        GRF_CHECK_LAUNCH("gram_sparse_kernel");
    }
    return GRF_OK;
}

static int32_t gram_sparse_launch(int64_t n_total, int64_t row_begin, int64_t rows, bool sym, int64_t k_begin,
                                  int64_t k_end, const int64_t *ptr, const int32_t *idx, const float *val,
                                  int64_t band_width, int32_t unit, const uint32_t *t_desc, const void *t_rec,
                                  const int32_t *t_rowshift, float *K, int64_t ldk, hipStream_t st,
                                  const void *t_split = nullptr) {
    const int64_t nb = cdiv<int64_t>(n_total, band_width);
    const GramTiles tl{rows, band_width, nb, sym, (int32_t)k_begin, (int32_t)k_end};
    const int64_t n_tiles = tl.total();
    if (n_tiles == 0) return GRF_OK;
    return gram_tiles_launch(n_total, row_begin, tl, 0, n_tiles, ptr, idx, val, t_desc, t_rec, unit, t_rowshift, K,
                             ldk, st, t_split, nb * n_total);
}

static int32_t gram_sparse_check(int64_t n_total, int64_t row_begin, int64_t row_end, const int64_t *ptr,
                                 int64_t band_width, int32_t unit, const uint32_t *t_desc, const void *t_rec,
                                 const int32_t *t_rowshift, float *K, int64_t ldk) {
    GRF_REQUIRE(unit == GRF_REC_LINE || unit == GRF_REC_PACKED || unit == GRF_REC_SLOT, GRF_EINVAL,
                "grf_gram_sparse: rec_unit must be GRF_REC_LINE, GRF_REC_PACKED or GRF_REC_SLOT");
    GRF_REQUIRE(n_total >= 0 && 0 <= row_begin && row_begin <= row_end && row_end <= n_total && ptr && t_desc && K &&
                    t_rowshift && t_rec,
                GRF_EINVAL, "grf_gram_sparse: bad arguments");
    GRF_REQUIRE(((uintptr_t)t_rec & 127) == 0, GRF_EINVAL, "grf_gram_sparse: t_rec must be 128-byte aligned");
    GRF_REQUIRE(ldk >= n_total, GRF_EINVAL, "grf_gram_sparse: ldk < n");
    GRF_REQUIRE(band_width >= 64 && band_width % 64 == 0 && band_width <= 8192, GRF_EUNSUPPORTED,
                "grf_gram_sparse: band_width must be a multiple of 64 in [64, 8192]");
    return GRF_OK;
}

int32_t grf_gram_sparse(int64_t n_total, int64_t row_begin, int64_t row_end, const int64_t *ptr, const int32_t *idx,
                        const float *val, int64_t band_width, int32_t rec_unit, const uint32_t *t_desc,
                        const void *t_rec, const int32_t *t_rowshift, float *K, int64_t ldk, void *workspace,
                        size_t workspace_bytes, grf_stream_t stream) {
    int32_t rc = gram_sparse_check(n_total, row_begin, row_end, ptr, band_width, rec_unit, t_desc, t_rec, t_rowshift,
                                   K, ldk);
    if (rc != GRF_OK) return rc;
    if (row_end == row_begin || n_total == 0) return GRF_OK;
    return gram_sparse_launch(n_total, row_begin, row_end - row_begin, false, 0, n_total, ptr, idx, val, band_width,
                              rec_unit, t_desc, t_rec, t_rowshift, K, ldk, S(stream));
}

int32_t grf_gram_sparse_sym(int64_t n_total, const int64_t *ptr, const int32_t *idx, const float *val,
                            int64_t band_width, int32_t rec_unit, const uint32_t *t_desc, const void *t_rec,
                            const void *t_split, const int32_t *t_rowshift, float *K, int64_t ldk, void *workspace, size_t workspace_bytes,
                            grf_stream_t stream) {
    int32_t rc = gram_sparse_check(n_total, 0, n_total, ptr, band_width, rec_unit, t_desc, t_rec, t_rowshift, K, ldk);
    if (rc != GRF_OK) return rc;
    if (n_total == 0) return GRF_OK;
    rc = gram_sparse_launch(n_total, 0, n_total, true, 0, n_total, ptr, idx, val, band_width, rec_unit, t_desc, t_rec,
                            t_rowshift, K, ldk, S(stream), t_split);
    if (rc != GRF_OK) return rc;
    return grf_gram_mirror(n_total, K, ldk, 0, stream);
}

static int32_t gram_sparse_upper_impl(int64_t n_total, const int64_t *ptr, const int32_t *idx, const float *val,
                                      int64_t band_width, int32_t rec_unit, const uint32_t *t_desc, const void *t_rec,
                                      const void *t_split, const int32_t *t_rowshift, float *K, int64_t ldk, int32_t part_begin,
                                      int32_t part_end, int32_t n_parts, bool add_k, grf_stream_t stream,
                                      const int32_t *row_cuts = nullptr) {
    int32_t rc = gram_sparse_check(n_total, 0, n_total, ptr, band_width, rec_unit, t_desc, t_rec, t_rowshift, K, ldk);
    if (rc != GRF_OK) return rc;
    GRF_REQUIRE(n_parts >= 1 && 0 <= part_begin && part_begin <= part_end && part_end <= n_parts, GRF_EINVAL,
                "grf_gram_sparse_upper: bad tile parts [%d, %d) of %d", part_begin, part_end, n_parts);
    if (n_total == 0 || part_begin == part_end) return GRF_OK;
    GramTiles tl{n_total, band_width, cdiv<int64_t>(n_total, band_width), true, 0, (int32_t)n_total};
    tl.add_k = add_k;
    const int64_t total = tl.total();
    const int64_t t0 = total * part_begin / n_parts, t1 = total * part_end / n_parts;
    if (t1 <= t0) return GRF_OK;
    GRF_REQUIRE(!row_cuts || rec_unit != GRF_REC_SLOT, GRF_EUNSUPPORTED, "grf_gram_sparse_upper: row cuts with slot buckets");
    return gram_tiles_launch(n_total, 0, tl, t0, t1, ptr, idx, val, t_desc, t_rec, rec_unit, t_rowshift, K, ldk,
                             S(stream), t_split, tl.nb * n_total, row_cuts);
}

int32_t grf_gram_sparse_upper_ex(int64_t n_total, const int64_t *ptr, const int32_t *idx, const float *val,
                                 int64_t band_width, int32_t rec_unit, const uint32_t *t_desc, const void *t_rec,
                                 const void *t_split, const int32_t *t_rowshift, const int32_t *row_cuts, float *K,
                                 int64_t ldk, int32_t part_begin, int32_t part_end, int32_t n_parts, int32_t add_k,
                                 grf_stream_t stream) {
    return gram_sparse_upper_impl(n_total, ptr, idx, val, band_width, rec_unit, t_desc, t_rec, t_split, t_rowshift,
                                  K, ldk, part_begin, part_end, n_parts, add_k != 0, stream, row_cuts);
}

// ---------------------------------------------------------------- wave shares by record pairs
// col_w[k] = the record pairs of column k over all bands of the transpose (after any hub drop)
__global__ __launch_bounds__(256) void col_pairs_kernel(int64_t n_bands, int64_t n_cols, const uint2 *__restrict__ t_desc,
                                                        int32_t *__restrict__ col_w) {
    const int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (k >= n_cols) return;
    int64_t s = 0;
    for (int64_t J = 0; J < n_bands; ++J) s += t_desc[J * n_cols + k].y;
    col_w[k] = (int32_t)(s < 0x7fffffff ? s : 0x7fffffff);
}

// One wave per row: cuts[8 row + s] = the first nonzero (offset in the row) whose exclusive prefix of
// column weights reaches s / 8 of the row's total (s = 1..7; s = 0 -> 0; none -> the row's length),
// i.e. 8 contiguous shares of about equal weight; weights from col_w (int64 sums)
__global__ __launch_bounds__(256) void row_cuts_kernel(int64_t n_rows, const int64_t *__restrict__ ptr,
                                                       const int32_t *__restrict__ idx, const int32_t *__restrict__ col_w,
                                                       int32_t *__restrict__ cuts) {
    const int lane = threadIdx.x & 63;
    const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= n_rows) return;
    const int64_t e0 = ptr[row], e1 = ptr[row + 1], nnz = e1 - e0;
    long long tot = 0;
    for (int64_t e = e0 + lane; e < e1; e += 64) tot += col_w[idx[e]];
    tot = wave_sum<long long>(tot);
    int32_t out = (int32_t)nnz;  // lane s (1..7) holds cut s
    long long run = 0;
    unsigned found = 1u;  // bit s: cut s set (cut 0 = 0)
    for (int64_t c = e0; c < e1 && found != 0xffu; c += 64) {
        const int64_t e = c + lane;
        const long long w = e < e1 ? (long long)col_w[idx[e]] : 0;
        const long long inc = wave_inclusive_scan<long long>(w) + run;
        const long long excl = inc - w;
#pragma unroll
        for (int sh = 1; sh < 8; ++sh) {
            if (found & (1u << sh)) continue;
            const unsigned long long m = __ballot(e < e1 && excl * 8 >= (long long)sh * tot);
            if (m) {
                found |= 1u << sh;
                if (lane == sh) out = (int32_t)(c - e0 + __builtin_ctzll(m));
            }
        }
        run = __shfl(inc, 63, 64);
    }
    if (lane == 0) out = 0;
    if (lane < 8) cuts[row * 8 + lane] = out;
}

int32_t grf_gram_row_cuts(int64_t n_rows, const int64_t *ptr, const int32_t *idx, int64_t n_bands, int64_t n_cols,
                          const uint32_t *t_desc, int32_t *col_w, int32_t *row_cuts, grf_stream_t stream) {
    GRF_REQUIRE(n_rows >= 0 && n_bands >= 0 && n_cols >= 0 &&
                    (n_rows == 0 || (ptr && idx && t_desc && col_w && row_cuts)),
                GRF_EINVAL, "grf_gram_row_cuts: bad arguments");
    if (n_rows == 0) return GRF_OK;
    if (n_cols > 0) {
        GRF_REQUIRE_GRID(cdiv<int64_t>(n_cols, 256), 256, "col_pairs_kernel");
        col_pairs_kernel<<<(unsigned)cdiv<int64_t>(n_cols, 256), 256, 0, S(stream)>>>(
            n_bands, n_cols, reinterpret_cast<const uint2 *>(t_desc), col_w);
        GRF_CHECK_LAUNCH("col_pairs_kernel");
    }
    GRF_REQUIRE_GRID(cdiv<int64_t>(n_rows, 4), 256, "row_cuts_kernel");
    row_cuts_kernel<<<(unsigned)cdiv<int64_t>(n_rows, 4), 256, 0, S(stream)>>>(n_rows, ptr, idx, col_w, row_cuts);
    GRF_CHECK_LAUNCH("row_cuts_kernel");
    return GRF_OK;
}

int32_t grf_gram_sparse_upper(int64_t n_total, const int64_t *ptr, const int32_t *idx, const float *val,
                              int64_t band_width, int32_t rec_unit, const uint32_t *t_desc, const void *t_rec,
                              const void *t_split, const int32_t *t_rowshift, float *K, int64_t ldk, int32_t part_begin,
                              int32_t part_end, int32_t n_parts, void *workspace, size_t workspace_bytes,
                              grf_stream_t stream) {
    return gram_sparse_upper_impl(n_total, ptr, idx, val, band_width, rec_unit, t_desc, t_rec, t_split, t_rowshift,
                                  K, ldk, part_begin, part_end, n_parts, false, stream);
}

int32_t grf_gram_sparse_upper_add(int64_t n_total, const int64_t *ptr, const int32_t *idx, const float *val,
                                  int64_t band_width, int32_t rec_unit, const uint32_t *t_desc, const void *t_rec,
                                  const void *t_split, const int32_t *t_rowshift, float *K, int64_t ldk,
                                  int32_t part_begin,
                                  int32_t part_end, int32_t n_parts, void *workspace, size_t workspace_bytes,
                                  grf_stream_t stream) {
    return gram_sparse_upper_impl(n_total, ptr, idx, val, band_width, rec_unit, t_desc, t_rec, t_split, t_rowshift,
                                  K, ldk, part_begin, part_end, n_parts, true, stream);
}

int32_t grf_hub_panel(int64_t n_rows, const int64_t *ptr, const int32_t *idx, const float *val,
                      const int32_t *hub_pos, float *P, int64_t ldp, grf_stream_t stream) {
    GRF_REQUIRE(n_rows >= 0 && ldp >= 0 && (n_rows == 0 || (ptr && idx && val && hub_pos && P)), GRF_EINVAL,
                "grf_hub_panel: bad arguments");
    if (n_rows == 0) return GRF_OK;
    GRF_REQUIRE_GRID(cdiv<int64_t>(n_rows, 4), 256, "hub_panel_kernel");
    hub_panel_kernel<<<(unsigned)cdiv<int64_t>(n_rows, 4), 256, 0, S(stream)>>>(n_rows, ptr, idx, val, hub_pos, P,
                                                                                 ldp);
    GRF_CHECK_LAUNCH("hub_panel_kernel");
    return GRF_OK;
}

int32_t grf_transpose_drop_columns(int64_t n_bands, int64_t n_cols, uint32_t *t_desc, const int32_t *cols,
                                   int32_t n_drop, grf_stream_t stream) {
    GRF_REQUIRE(n_bands >= 0 && n_cols >= 0 && n_drop >= 0 && (n_drop == 0 || (t_desc && cols)), GRF_EINVAL,
                "grf_transpose_drop_columns: bad arguments");
    const int64_t work = n_bands * (int64_t)n_drop;
    if (work == 0) return GRF_OK;
    GRF_REQUIRE_GRID(cdiv<int64_t>(work, 256), 256, "transpose_drop_kernel");
    transpose_drop_kernel<<<(unsigned)cdiv<int64_t>(work, 256), 256, 0, S(stream)>>>(
        n_bands, n_cols, reinterpret_cast<uint2 *>(t_desc), cols, n_drop);
    GRF_CHECK_LAUNCH("transpose_drop_kernel");
    return GRF_OK;
}

// Column block: K[r - row_begin, 0 : t_rows] = sum_k Phi[r, k] Phi_B[:, k] for the rows r of Phi
// against the t_rows rows of another matrix Phi_B (a rank's own rows) whose banded transpose is
// given; the row shifts come from grf_phi_row_shifts over all of Phi.  With Phi_B = Phi[b:e] this
// is K[:, b:e] -- entry for entry the row mode's K[r, b + j] -- so a rank transposes only its rows.
static int32_t gram_sparse_cols_impl(int64_t n_cols, int64_t row_begin, int64_t row_end, const int64_t *ptr,
                                     const int32_t *idx, const float *val, const int32_t *row_shift, int64_t t_rows,
                                     int64_t sym_row0, int64_t band_width, int32_t rec_unit, const uint32_t *t_desc,
                                     const void *t_rec, const void *t_split, float *K, int64_t ldk,
                                     grf_stream_t stream, int64_t pad_cap = 0, const int32_t *pad_cnt = nullptr) {
    GRF_REQUIRE(n_cols > 0 && 0 <= row_begin && row_begin <= row_end && (ptr || pad_cnt) && idx && val && row_shift &&
                    t_rows >= 0 && t_desc && t_rec && K && ldk >= t_rows,
                GRF_EINVAL, "grf_gram_sparse_cols: bad arguments");
    GRF_REQUIRE(band_width >= 64 && band_width % 64 == 0 && band_width <= 8192, GRF_EUNSUPPORTED,
                "grf_gram_sparse_cols: band_width must be a multiple of 64 in [64, 8192]");
    GRF_REQUIRE(((uintptr_t)t_rec & 127) == 0, GRF_EINVAL, "grf_gram_sparse_cols: t_rec must be 128-byte aligned");
    GRF_REQUIRE(rec_unit == GRF_REC_LINE || rec_unit == GRF_REC_PACKED || rec_unit == GRF_REC_SLOT, GRF_EINVAL,
                "grf_gram_sparse_cols: bad rec_unit");
    GRF_REQUIRE(sym_row0 < 0 || (row_begin <= sym_row0 && sym_row0 + t_rows <= row_end), GRF_EINVAL,
                "grf_gram_sparse_cols: the symmetric square [sym_row0, sym_row0 + t_rows) must lie in the rows");
    if (row_end == row_begin || t_rows == 0) return GRF_OK;
    const int64_t nb = cdiv<int64_t>(t_rows, band_width);
    hipStream_t st = S(stream);
    // (the kernel reads row_shift[row] for row = row_begin + r: the shifts of Phi's rows)
    auto launch = [&](int64_t r0, int64_t r1, bool sym) -> int32_t {
        if (r1 <= r0) return GRF_OK;
        GramTiles tl{r1 - r0, band_width, nb, sym, 0, (int32_t)n_cols};
        tl.t_rows = t_rows;
        return gram_tiles_launch(n_cols, r0, tl, 0, tl.total(), ptr, idx, val, t_desc, t_rec, rec_unit, row_shift,
                                 K + (r0 - row_begin) * ldk, ldk, st, sym ? t_split : nullptr, nb * n_cols, nullptr,
                                 pad_cap, pad_cnt);
    };
    if (sym_row0 < 0) return launch(row_begin, row_end, false);
    // Phi_B = Phi[sym_row0, sym_row0 + t_rows): the square K[B, B] is symmetric and its bands start at
    // sym_row0, so only its tiles on and above the diagonal run (symmetric enumeration), then a mirror
    int32_t rc = launch(sym_row0, sym_row0 + t_rows, true);
    if (rc == GRF_OK) rc = launch(row_begin, sym_row0, false);
    if (rc == GRF_OK) rc = launch(sym_row0 + t_rows, row_end, false);
    if (rc != GRF_OK) return rc;
    return grf_gram_mirror(t_rows, K + (sym_row0 - row_begin) * ldk, ldk, 0, stream);
}

int32_t grf_gram_sparse_cols(int64_t n_cols, int64_t row_begin, int64_t row_end, const int64_t *ptr,
                             const int32_t *idx, const float *val, const int32_t *row_shift, int64_t t_rows,
                             int64_t sym_row0, int64_t band_width, int32_t rec_unit, const uint32_t *t_desc,
                             const void *t_rec, const void *t_split, float *K, int64_t ldk, void *workspace,
                             size_t workspace_bytes, grf_stream_t stream) {
    (void)workspace;
    (void)workspace_bytes;
    return gram_sparse_cols_impl(n_cols, row_begin, row_end, ptr, idx, val, row_shift, t_rows, sym_row0, band_width,
                                 rec_unit, t_desc, t_rec, t_split, K, ldk, stream);
}

int32_t grf_gram_sparse_cols_padded(int64_t n_cols, int64_t row_begin, int64_t row_end, int64_t cap,
                                    const int32_t *cnt, const int32_t *idx, const float *val, const int32_t *row_shift,
                                    int64_t t_rows, int64_t band_width, const uint32_t *t_desc, const void *t_rec,
                                    float *K, int64_t ldk, grf_stream_t stream) {
    GRF_REQUIRE(cap >= 1 && cnt, GRF_EINVAL, "grf_gram_sparse_cols_padded: bad padded rows");
    return gram_sparse_cols_impl(n_cols, row_begin, row_end, nullptr, idx, val, row_shift, t_rows, -1, band_width,
                                 GRF_REC_SLOT, t_desc, t_rec, nullptr, K, ldk, stream, cap, cnt);
}

int32_t grf_gram_sparse_kslice(int64_t n_total, int64_t row_begin, int64_t row_end, int64_t k_begin, int64_t k_end,
                               const int64_t *ptr, const int32_t *idx, const float *val, int64_t band_width,
                               int32_t rec_unit, const uint32_t *t_desc, const void *t_rec,
                               const int32_t *t_rowshift, float *K, int64_t ldk, void *workspace,
                               size_t workspace_bytes, grf_stream_t stream) {
    int32_t rc = gram_sparse_check(n_total, row_begin, row_end, ptr, band_width, rec_unit, t_desc, t_rec, t_rowshift,
                                   K, ldk);
    if (rc != GRF_OK) return rc;
    GRF_REQUIRE(0 <= k_begin && k_begin <= k_end && k_end <= n_total, GRF_EINVAL,
                "grf_gram_sparse_kslice: bad column slice [%lld, %lld)", (long long)k_begin, (long long)k_end);
    if (row_end == row_begin || n_total == 0) return GRF_OK;
    (void)workspace;
    (void)workspace_bytes;
    return gram_sparse_launch(n_total, row_begin, row_end - row_begin, false, k_begin, k_end, ptr, idx, val,
                              band_width, rec_unit, t_desc, t_rec, t_rowshift, K, ldk, S(stream));
}

int32_t grf_gram_mirror(int64_t n, float *K, int64_t ldk, int64_t max_workgroups, grf_stream_t stream) {
    GRF_REQUIRE(n >= 0 && K && ldk >= n, GRF_EINVAL, "grf_gram_mirror: bad arguments");
    if (n == 0) return GRF_OK;
    const int64_t nt = cdiv<int64_t>(n, 64), blocks = nt * (nt + 1) / 2;
    // workgroups: one per block (max_workgroups <= 0), or a bounded grid-stride grid that leaves CU
    // slots to another stream (GRF_MIRROR_WGS overrides, for experiments)
    static const int64_t env_cap = [] {
        const char *e = getenv("GRF_MIRROR_WGS");
        return e ? (int64_t)atoll(e) : (int64_t)-1;
    }();
    const int64_t cap = env_cap >= 0 ? env_cap : max_workgroups;
    const int64_t grid = cap > 0 && cap < blocks ? cap : blocks;
    GRF_REQUIRE_GRID(grid, 256, "gram_mirror_swz_kernel");
    gram_mirror_swz_kernel<<<(unsigned)grid, 256, 0, S(stream)>>>(n, nt, blocks, K, ldk);
    GRF_CHECK_LAUNCH("gram_mirror_swz_kernel");
    return GRF_OK;
}

size_t grf_gram_dense_workspace_bytes(int64_t n, int64_t k_dim) { return grf::dense_gram_workspace_bytes(n, k_dim); }

// the MFMA Gram (grf_gram_dense.hip): tiles on and above the diagonal written to both triangles
// (upper_only: the tiles' K[row][col] only, the seed of the hub-column split's sparse tiles)
static int32_t gram_dense_impl(int64_t n, int64_t k_dim, const float *A, int64_t lda, float *K, int64_t ldk,
                               void *workspace, size_t workspace_bytes, bool upper_only, grf_stream_t stream) {
    return grf::dense_gram(n, k_dim, A, lda, K, ldk, workspace, workspace_bytes, upper_only, stream);
}

int32_t grf_gram_dense_ws(int64_t n, int64_t k_dim, const float *A, int64_t lda, float *K, int64_t ldk,
                          void *workspace, size_t workspace_bytes, grf_stream_t stream) {
    return gram_dense_impl(n, k_dim, A, lda, K, ldk, workspace, workspace_bytes, false, stream);
}

int32_t grf_gram_dense_upper(int64_t n, int64_t k_dim, const float *A, int64_t lda, float *K, int64_t ldk,
                             grf_stream_t stream) {
    return gram_dense_impl(n, k_dim, A, lda, K, ldk, nullptr, 0, true, stream);
}

int32_t grf_gram_dense(int64_t n, int64_t k_dim, const float *A, int64_t lda, float *K, int64_t ldk,
                       grf_stream_t stream) {
    return grf_gram_dense_ws(n, k_dim, A, lda, K, ldk, nullptr, 0, stream);
}

size_t grf_gram_dense_split_workspace_bytes(int64_t n, int64_t k_dim) {
    return grf::dense_gram_split_workspace_bytes(n, k_dim);
}

// the same K on the bf16 matrix cores: A split exactly into three bf16 planes, six products per term
int32_t grf_gram_dense_split(int64_t n, int64_t k_dim, const float *A, int64_t lda, float *K, int64_t ldk,
                             void *workspace, size_t workspace_bytes, grf_stream_t stream) {
    GRF_REQUIRE(workspace, GRF_EINVAL, "grf_gram_dense_split: workspace required");
    return grf::dense_gram_split(n, k_dim, A, lda, K, ldk, workspace, workspace_bytes, false, stream);
}

// grf_gram_dense_upper on the split products (the hub-column split's panel)
int32_t grf_gram_dense_split_upper(int64_t n, int64_t k_dim, const float *A, int64_t lda, float *K, int64_t ldk,
                                   grf_stream_t stream) {
    return grf::dense_gram_split(n, k_dim, A, lda, K, ldk, nullptr, 0, true, stream);
}

int64_t grf_planes_row_bytes(int64_t k_dim) { return grf::planes_row_bytes(k_dim); }

int32_t grf_split_planes(int64_t n, int64_t k_dim, const float *A, int64_t lda, void *P, int64_t ldp,
                         grf_stream_t stream) {
    return grf::split_planes(n, k_dim, A, lda, P, ldp, stream);
}

int32_t grf_densify_padded_planes(int64_t n_rows, int64_t cap, int64_t n_cols, const int32_t *cnt, const int32_t *idx,
                                  const float *val, void *P, int64_t ldp, grf_stream_t stream) {
    return grf::densify_padded_planes(n_rows, cap, n_cols, cnt, idx, val, P, ldp, stream);
}

int32_t grf_gram_dense_planes(int64_t n, int64_t k_dim, const void *P, int64_t ldp, float *K, int64_t ldk,
                              void *workspace, size_t workspace_bytes, grf_stream_t stream) {
    return grf::dense_gram_planes(n, k_dim, P, ldp, K, ldk, workspace, workspace_bytes, stream);
}

int32_t grf_densify_padded(int64_t n_rows, int64_t cap, int64_t n_cols, const int32_t *cnt, const int32_t *idx,
                           const float *val, float *out, int64_t lda, grf_stream_t stream) {
    GRF_REQUIRE(n_rows >= 0 && cap >= 1 && n_cols >= 0 && cnt && idx && val && out && lda >= n_cols, GRF_EINVAL,
                "grf_densify_padded: bad arguments");
    GRF_REQUIRE(lda % 4 == 0 && ((uintptr_t)out & 15) == 0, GRF_EINVAL,
                "grf_densify_padded: lda must be a multiple of 4 and out 16-byte aligned");
    GRF_REQUIRE(lda * (int64_t)sizeof(float) <= 160 * 1024, GRF_EUNSUPPORTED,
                "grf_densify_padded: a row of %lld floats does not fit one CU's LDS (use grf_densify)", (long long)lda);
    if (n_rows == 0) return GRF_OK;
    GRF_REQUIRE_GRID(n_rows, 256, "densify_padded_kernel");
    densify_padded_kernel<<<(unsigned)n_rows, 256, (size_t)lda * sizeof(float), S(stream)>>>(cap, cnt, idx, val, out,
                                                                                           lda);
    GRF_CHECK_LAUNCH("densify_padded_kernel");
    return GRF_OK;
}

int32_t grf_densify(int64_t n_rows, const int64_t *ptr, const int32_t *idx, const float *val, float *out,
                    int64_t lda, grf_stream_t stream) {
    GRF_REQUIRE(n_rows >= 0 && ptr && out && lda >= 0, GRF_EINVAL, "grf_densify: bad arguments");
    if (n_rows == 0) return GRF_OK;
    GRF_CHECK_HIP(hipMemsetAsync(out, 0, (size_t)n_rows * (size_t)lda * sizeof(float), S(stream)));
    GRF_REQUIRE_GRID(cdiv<int64_t>(n_rows, 4), 256, "densify_kernel");
    densify_kernel<<<(unsigned)cdiv<int64_t>(n_rows, 4), 256, 0, S(stream)>>>(n_rows, ptr, idx, val, out, lda);
    GRF_CHECK_LAUNCH("densify_kernel");
    return GRF_OK;
}

}  // extern "C"
