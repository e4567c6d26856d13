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
// Dense path: LDS-tiled fp32 MFMA (v_mfma_f32_32x32x2f32, exact f32 FMA chain),
// 128x128 tile per 256-thread workgroup, 2x2 waves of 64x64.
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>

#include "grf_block.h"

namespace grf {

typedef float f32x4 __attribute__((ext_vector_type(4)));

// The Gram tiles' K stores and the swizzled mirror's K loads: non-temporal (K is write-once and
// larger than every cache).  -DGRF_GRAM_K_NT=0 builds them with the default policy (an A/B build for
// the trailing mirror, tools/trail_exp.py: the Infinity Cache keeps what default-policy stores wrote).
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

// ---------------------------------------------------------------- fused symmetric completion
// grf_gram_sparse_sym_fused: the Gram tiles of the symmetric mode complete K themselves (no
// separate mirror pass re-reading the upper triangle from HBM).  The tiles of one band are
// dispatched row after row, so the 64 tiles of a row group g = rows [gs, gs + 64) of band J run
// together; each writes its row K[i, band J] write-through (sc1: visible to every XCD without a
// release fence), drains its stores and takes a ticket on the group's counter.  The last arriver
// (no waiting: the others exit) acquires and transposes the group's 64 x W block into
// K[band J, gs : gs + 64] (256-byte row segments, 4 x 4 register transposes).  Ownership keeps
// every lower entry single-writer and ordered after the upper one: on the diagonal band a tile
// writes only the columns >= its group's first row (the columns before it are lower entries that
// the earlier groups' last arrivers write), and inside the group's own diagonal block the last
// arriver overwrites the entries below the diagonal after all rows have been stored.  K is
// bit-identical to grf_gram_sparse_sym's.
// MEASURED SLOWER (profiles/r02_fused_ab.txt): 100-150 ms per K against 22.6 for tiles + mirror.
// The tiles with their tickets cost +0.8 ms and the block loads +5 ms (a timing-only decomposition,
// since removed), but the last arrivers' transposed stores (20 GB, one workgroup per 1 MB block)
// add ~100 ms: one workgroup cannot keep enough stores in flight, where the mirror pass spreads the
// same bytes over every CU.  Kept as a
// tested option (bench --fused); the default stays tiles + mirror.
#ifndef GRF_FUSE_GROUP
#define GRF_FUSE_GROUP 64
#endif
constexpr int kFuseGroup = GRF_FUSE_GROUP;         // rows per ticket group (64: 256-byte K row segments)

// The completion's edge cases, element by element: K[j, i] = K[i, j] for the K rows j = j0 + col
// .. j0 + col + 3 (< j0 + wlen) and i = gs + 4q .. gs + 4q + 3 (< ge, < j: the group's diagonal block)
__device__ __attribute__((noinline)) void gram_fused_edge(float *__restrict__ K, int64_t ldk, int64_t gs, int64_t ge,
                                                          int64_t j0, int64_t col, int64_t wlen, int q) {
    for (int u = 0; u < 4; ++u) {
        const int64_t i = gs + 4 * q + u;
        if (i >= ge) break;
        for (int e = 0; e < 4 && col + e < wlen; ++e) {
            const int64_t j = j0 + col + e;
            if (i < j) K[j * ldk + i] = __hip_atomic_load(K + i * ldk + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

template <int kWaves>
__device__ __forceinline__ void gram_fused_completion(const GramTiles &tl, int64_t J, int64_t r, int64_t j0,
                                                      int64_t wlen, int sh, unsigned long long *acc,
                                                      float *__restrict__ K, int64_t ldk,
                                                      int32_t *__restrict__ tickets) {
    typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    constexpr int kT = 64 * kWaves;
    const int tid = threadIdx.x;
    const int64_t gs = r & ~(int64_t)(kFuseGroup - 1);
    const int64_t rows_J = tl.count(J);
    const int64_t ge = (gs + kFuseGroup) < rows_J ? gs + kFuseGroup : rows_J;
    const int gn = (int)(ge - gs);
    const bool diag = gs >= j0;  // the group's rows lie in this band (j0 <= gs < j0 + W)
    // 1. the tile's row, write-through: on the diagonal band from the group's first row on
    const u64x2 *acc2 = reinterpret_cast<const u64x2 *>(acc);
    float *krow = K + r * ldk + j0;
    const int64_t c_lo = diag ? gs - j0 : 0;  // a multiple of 32
    const auto rs = __builtin_amdgcn_make_buffer_rsrc(krow, (short)0, 0x7fffffff, 0x00020000);
    const int64_t n4 = wlen / 4;
    for (int64_t i = c_lo / 4 + tid; i < n4; i += kT) {
        const u64x2 a = acc2[2 * i], b = acc2[2 * i + 1];
        u32x4 o;
        o[0] = __float_as_uint(fx_to_float(a[0], sh));
        o[1] = __float_as_uint(fx_to_float(a[1], sh));
        o[2] = __float_as_uint(fx_to_float(b[0], sh));
        o[3] = __float_as_uint(fx_to_float(b[1], sh));
        __builtin_amdgcn_raw_buffer_store_b128(o, rs, (int)(i * 16), 0, 16);  // aux 16: sc1 (write-through)
    }
    for (int64_t i = n4 * 4 + tid; i < wlen; i += kT)
        __hip_atomic_store(krow + i, fx_to_float(acc[i], sh), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    // 2. every storing wave drains, then one ticket for the workgroup
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    int *flag = reinterpret_cast<int *>(acc);
    if (tid == 0) {
        const int64_t ngroups = (tl.rows + kFuseGroup - 1) / kFuseGroup;
        const int old = __hip_atomic_fetch_add(tickets + J * ngroups + (r / kFuseGroup), 1, __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_AGENT);
        flag[0] = old == gn - 1;
    }
    __syncthreads();
    if (!flag[0]) return;  // (uniform) not the last of the group
    if (tid < 64) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
    // 3. the last arriver: K[j, gs : ge] = K[gs : ge, j] for the band's columns j (j > i), in 4 x 4
    // register transposes (no LDS, no barrier: the tiles still running on this CU keep the LDS
    // pipe).  Lane (q, g) = (lane % 8, lane / 8) of a wave loads rows 4q .. 4q + 3 of the group at
    // columns c + 4g .. c + 4g + 3 (8 lanes = one 128-byte segment of a row) and stores them as
    // rows c + 4g .. c + 4g + 3 of K at columns gs + 4q .. gs + 4q + 3 (8 lanes = one 128-byte
    // row segment); a wave covers 32 columns, kFuseUnroll column blocks in flight.
    constexpr int kQ = kFuseGroup / 4, kCols = 4 * (64 / kQ);  // lanes per row segment, columns per wave
    const int lane = tid & 63, wave = tid >> 6, q = lane % kQ, g = lane / kQ;
    const auto grs = __builtin_amdgcn_make_buffer_rsrc(K + gs * ldk + j0, (short)0, 0x7fffffff, 0x00020000);
    const int64_t cb0 = diag ? gs - j0 : 0;
    // compact code on purpose: this path runs once per 32 tiles, and its instructions share the
    // instruction cache with the tiles' loop (edge columns / rows go to a separate function)
    const int32_t row_off = (int32_t)(4 * q * ldk * 4);
    for (int64_t cb = cb0 + wave * kCols; cb < wlen; cb += kWaves * kCols) {
        const int64_t col = cb + 4 * g;
        const int64_t j = j0 + col;  // K rows j .. j + 3 are written
        if (gn == kFuseGroup && col + 4 <= wlen && j >= ge) {
            f32x4 x[4];
            const int32_t off = row_off + (int32_t)(col * 4);
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const auto y = __builtin_amdgcn_raw_buffer_load_b128(grs, off + (int32_t)(u * ldk * 4), 0, 16);
                x[u] = f32x4{__uint_as_float(y[0]), __uint_as_float(y[1]), __uint_as_float(y[2]), __uint_as_float(y[3])};
            }
            float *dst = K + j * ldk + gs + 4 * q;
#pragma unroll
            for (int e = 0; e < 4; ++e)
                __builtin_nontemporal_store(f32x4{x[0][e], x[1][e], x[2][e], x[3][e]}, reinterpret_cast<f32x4 *>(dst + e * ldk));
        } else {
            gram_fused_edge(K, ldk, gs, ge, j0, col, wlen, q);
        }
    }
}

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
template <int kWaves, int kHalves, int kGramUnroll, bool kTailExact, bool kFuse, bool kSlot = false>
__global__ __launch_bounds__(64 * kWaves) void gram_sparse_kernel(
    int64_t n_total, int64_t row_begin, GramTiles tl, int64_t t_begin, const int64_t *__restrict__ ptr,
    const int32_t *__restrict__ idx, const float *__restrict__ val, const uint2 *__restrict__ t_desc,
    const unsigned char *__restrict__ t_rec, int32_t unit, const int32_t *__restrict__ rowshift,
    float *__restrict__ K, int64_t ldk, int32_t *__restrict__ tickets, const uint16_t *__restrict__ t_split,
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
        for (int32_t c0 = 0; c0 < total; c0 += kChunk) {
            const int32_t cend = (total - c0) < kChunk ? total : c0 + kChunk;
            // bucket ids of the chunk: clear, mark every non-empty bucket's first position, propagate
            reinterpret_cast<uint4 *>(bidv)[lane] = make_uint4(0u, 0u, 0u, 0u);
            __builtin_amdgcn_wave_barrier();
#pragma unroll
            for (int h = 0; h < kV; ++h)
                if (cnt[h] > 0 && excl[h] >= c0 && excl[h] < cend)
                    bidv[excl[h] - c0] = (unsigned char)(h * 64 + lane + 1);
            __builtin_amdgcn_wave_barrier();
            carry = gram_propagate_ids(bidv, carry, lane);
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

    if constexpr (kFuse) {
        gram_fused_completion<kWaves>(tl, J_local, r, j0, wlen, sh, acc, K, ldk, tickets);
        return;
    }
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

__device__ __forceinline__ void gram_mirror_block(int64_t n, int64_t nt, int64_t b, float *__restrict__ K, int64_t ldk,
                                                  float (*tile)[65]) {
    int64_t bi, bj;
    gram_mirror_tri_coords(nt, b, bi, bj);
    gram_mirror_block_at(n, bi, bj, K, ldk, tile);
}

// Symmetric completion: K[j, i] = K[i, j] for every j > i (the Gram launch in symmetric
// mode wrote the tiles K[i, band >= band(i)], which cover the upper triangle; the lower
// parts of the diagonal band tiles are overwritten, so K is exactly symmetric).  One
// workgroup per upper-triangle 64 x 64 block (triangular grid: no idle workgroups) moves
// it through LDS with 16-byte loads and 16-byte non-temporal stores.  A bounded grid
// (grid-stride over the blocks) leaves CU slots to work on another stream.
__global__ __launch_bounds__(256) void gram_mirror_kernel(int64_t n, int64_t nt, int64_t nblocks,
                                                          float *__restrict__ K, int64_t ldk) {
    __shared__ float tile[64][65];
    for (int64_t b = blockIdx.x; b < nblocks; b += gridDim.x) {
        gram_mirror_block(n, nt, b, K, ldk, tile);
        __syncthreads();  // (the tile is reused by the next block)
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

// The mirror of one rectangle of 64-blocks: block rows [bi0, bi1) x block columns [bj0, bj1), the
// blocks with bj >= bi (the others are skipped).  A trailing mirror (grf_gram_mirror_rect) completes
// the tiles of one (row range, band) chunk right after the Gram wrote them, while they may still sit
// in the Infinity Cache.
__global__ __launch_bounds__(256) void gram_mirror_rect_kernel(int64_t n, int64_t bi0, int64_t bj0, int64_t nbj,
                                                               int64_t nblocks, float *__restrict__ K, int64_t ldk) {
    __shared__ __attribute__((aligned(16))) float tile[64 * 65];
    for (int64_t b = blockIdx.x; b < nblocks; b += gridDim.x) {
        const int64_t bi = bi0 + b / nbj, bj = bj0 + b % nbj;
        if (bj >= bi) gram_mirror_block_swz_at(n, bi, bj, K, ldk, tile);
        __syncthreads();
    }
}

// The bounded grid (grid-stride over the blocks: the pipelined bench gives the mirror 1024
// workgroups beside the next step's front), GRF_MIRROR_PIPE=1: a workgroup's loads of its next block
// are issued before the stores of the current one.  On gfx950 one vmcnt counter covers loads and stores, so a wait for
// loads issued after stores also waits for those stores' acknowledgements; issued before them, the
// next block's loads are in flight while the current block is written (profiles/r02_fused_ab.txt,
// where one workgroup per 1 MB block lost ~100 ms to that serialisation).  Measured beside the next
// front (profiles/r02_mirror_pipe_ab.txt): the K assembly ends at the same time but the front beside
// it is slowed (24.9 vs 24.0 ms per step, same box), so it is off by default.
// Strictly-upper full blocks only (the diagonal blocks and, for n % 64 != 0, the ragged last block
// column go to gram_mirror_edge_kernel): nf = nt - 1 (n % 64 == 0) or nt - 2 block columns are full,
// and the strictly-upper blocks of that nf x nf grid are enumerated row-major (bi < bj < nf).
__device__ __forceinline__ void gram_mirror_upper_coords(int64_t nf, int64_t b, int64_t &i0, int64_t &j0) {
    // row bi holds nf - 1 - bi blocks; first(bi) = bi (2 nf - bi - 1) / 2
    const double m = (double)(2 * nf - 1);
    int64_t bi = (int64_t)((m - sqrt(m * m - 8.0 * (double)b)) * 0.5);
    auto first = [nf](int64_t i) { return i * (2 * nf - i - 1) / 2; };
    if (bi < 0) bi = 0;
    if (bi > nf - 2) bi = nf - 2;
    while (bi > 0 && first(bi) > b) --bi;
    while (bi < nf - 2 && first(bi + 1) <= b) ++bi;
    i0 = bi * 64;
    j0 = (bi + 1 + (b - first(bi))) * 64;
}

__global__ __launch_bounds__(256) void gram_mirror_pipe_kernel(int64_t nf, int64_t nblocks, float *__restrict__ K,
                                                               int64_t ldk) {
    __shared__ __attribute__((aligned(16))) float tile[64 * 64];
    const int t = threadIdx.x;
    auto swz = [](int r, int c) { return r * 64 + (c ^ (4 * ((r >> 2) & 15))); };
    f32x4 v[4];
    int64_t i0 = 0, j0 = 0;
    auto load = [&](int64_t b) {
        gram_mirror_upper_coords(nf, b, i0, j0);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int y = (t >> 4) + 16 * q, x = (t & 15) * 4;
            v[q] = __builtin_nontemporal_load(reinterpret_cast<const f32x4 *>(K + (i0 + y) * ldk + j0 + x));
        }
    };
    auto to_lds = [&]() {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int y = (t >> 4) + 16 * q, x = (t & 15) * 4;
            *reinterpret_cast<f32x4 *>(tile + swz(y, x)) = v[q];
        }
    };
    int64_t b = blockIdx.x;
    if (b >= nblocks) return;
    load(b);
    to_lds();
    __syncthreads();
    for (; b < nblocks; b += gridDim.x) {
        const int64_t ci0 = i0, cj0 = j0;
        // the next block's loads, issued before this block's stores (unconditional, clamped: the wait
        // for them below is then vmcnt(4), the 4 stores behind them, on every path)
        load(b + gridDim.x < nblocks ? b + gridDim.x : nblocks - 1);
        const int k = t & 15, pr = t >> 4;
#pragma unroll
        for (int it = 0; it < 2; ++it) {
            const int y = 2 * pr + 32 * it;
            typedef float f32x2 __attribute__((ext_vector_type(2)));
            typedef __attribute__((address_space(3))) float lds_float;
            uint32_t a[4];
#pragma unroll
            for (int c = 0; c < 4; ++c) a[c] = (uint32_t)(uintptr_t)(lds_float *)(tile + swz(4 * k + c, y));
            f32x2 w[4];
            asm volatile(
                "ds_read_b64 %0, %4\n\tds_read_b64 %1, %5\n\tds_read_b64 %2, %6\n\tds_read_b64 %3, %7\n\t"
                "s_waitcnt lgkmcnt(0)"
                : "=&v"(w[0]), "=&v"(w[1]), "=&v"(w[2]), "=&v"(w[3])
                : "v"(a[0]), "v"(a[1]), "v"(a[2]), "v"(a[3])
                : "memory");
            f32x4 o0, o1;
            o0[0] = w[0].x; o0[1] = w[1].x; o0[2] = w[2].x; o0[3] = w[3].x;
            o1[0] = w[0].y; o1[1] = w[1].y; o1[2] = w[2].y; o1[3] = w[3].y;
            __builtin_nontemporal_store(o0, reinterpret_cast<f32x4 *>(K + (cj0 + y) * ldk + ci0 + 4 * k));
            __builtin_nontemporal_store(o1, reinterpret_cast<f32x4 *>(K + (cj0 + y + 1) * ldk + ci0 + 4 * k));
        }
        __syncthreads();  // (this block's LDS reads are done)
        to_lds();
        __syncthreads();
    }
}

// The blocks gram_mirror_pipe_kernel leaves: the nt diagonal blocks, then the blocks of the last
// (ragged) block column when n % 64 != 0, then the strictly-upper blocks of full block columns beyond
// the pipelined grid's enumeration (none: every full strictly-upper block is in it).
__global__ __launch_bounds__(256) void gram_mirror_edge_kernel(int64_t n, int64_t nt, float *__restrict__ K,
                                                               int64_t ldk) {
    __shared__ float tile[64][65];
    const int64_t e = blockIdx.x;
    // express the edge block as its index in the triangular enumeration of gram_mirror_block
    const int64_t bi = e < nt ? e : e - nt, bj = e < nt ? e : nt - 1;
    const int64_t b = bi * nt - bi * (bi - 1) / 2 + (bj - bi);
    gram_mirror_block(n, nt, b, K, ldk, tile);
}

__global__ void absmax_reset_kernel(float *m) { *m = 0.f; }

// ------------------------------------------------------------------ dense MFMA
// K = A A^T (A: n x k_dim fp32, row-major) on v_mfma_f32_32x32x2f32 (exact f32 FMA chains).
// Symmetric: only the tiles on and above the diagonal are computed (the mirror pass copies the
// upper triangle down), so a launch does n^2 k instead of 2 n^2 k flops.  A workgroup of 4 waves
// (2 x 2) owns a BM x BM tile, each wave (BM/2)^2 as (BM/64)^2 MFMA blocks of 32 x 32; the
// k-tiles (BK deep, staged k-major through LDS) are software-pipelined: the next tile's global
// loads are in flight in registers while the current one feeds the MFMAs.  BM = 64 for small n
// (more workgroups than CUs), 128 otherwise.
typedef float f32x16 __attribute__((ext_vector_type(16)));
// k-major LDS image, row pitch BM + 32 (the two k-rows one MFMA operand read spans fall on
// disjoint bank halves) and rows XOR-swizzled by the k group: the transposing stores (8 k-groups
// x 8 rows per wave) and the operand reads are both conflict-free
constexpr int kDensePad = 32;
__device__ __forceinline__ int dense_swz(int k) { return ((k >> 2) & 7) << 3; }

// Split-K (gridDim.y = S > 1, small n: too few tiles to fill the CUs): slice s of the k range,
// k_split wide, goes to the partial buffer K + s * part_stride; gram_dense_combine_kernel sums the
// S partials in slice order and writes both triangles.
template <int BM, int BK>
__global__ __launch_bounds__(256) void gram_dense_kernel(int64_t n, int64_t nt, int64_t k_dim,
                                                         const float *__restrict__ A, int64_t lda,
                                                         float *__restrict__ K, int64_t ldk, int64_t k_split,
                                                         int64_t part_stride, int32_t n_split) {
    constexpr int NB = BM / 64;          // 32 x 32 MFMA blocks per wave and dimension
    constexpr int F4 = BM * BK / 4 / 256;  // float4 loads per thread and operand per k-tile
    __shared__ __attribute__((aligned(16))) float As[BK][BM + kDensePad];
    __shared__ __attribute__((aligned(16))) float Bs[BK][BM + kDensePad];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave >> 1, wn = wave & 1;
    // workgroup -> (tile b, k slice): the slice is the fastest index, so with round-robin workgroup
    // placement over the 8 XCDs all tiles of one slice share an XCD (8 slices: one XCD's L2 holds its
    // slice of the operand; speed only, never correctness); tile b -> (bi, bj), bj >= bi, row-major
    // over the upper triangle of the nt x nt tile grid
    const int64_t b = (int64_t)blockIdx.x / n_split;
    const int32_t slice = (int32_t)((int64_t)blockIdx.x - b * n_split);
    int64_t bi = (int64_t)(((double)(2 * nt + 1) - sqrt((double)(2 * nt + 1) * (double)(2 * nt + 1) - 8.0 * (double)b)) * 0.5);
    auto first = [nt](int64_t i) { return i * nt - i * (i - 1) / 2; };
    if (bi < 0) bi = 0;
    if (bi > nt - 1) bi = nt - 1;
    while (bi > 0 && first(bi) > b) --bi;
    while (bi < nt - 1 && first(bi + 1) <= b) ++bi;
    const int64_t bj = bi + (b - first(bi));
    const int64_t m0 = bi * BM, n0 = bj * BM;

    f32x16 c[NB][NB];
#pragma unroll
    for (int x = 0; x < NB; ++x)
#pragma unroll
        for (int y = 0; y < NB; ++y)
#pragma unroll
            for (int q = 0; q < 16; ++q) c[x][y][q] = 0.f;

    const int64_t kb = (int64_t)slice * k_split;
    const int64_t ke = (kb + k_split) < k_dim ? kb + k_split : k_dim;
    K += (int64_t)slice * part_stride;
    float4 ra[F4], rb[F4];
    auto load = [&](int64_t k0) {
#pragma unroll
        for (int it = 0; it < F4; ++it) {
            const int idx = tid + it * 256;
            const int row = idx / (BK / 4), kq = (idx % (BK / 4)) * 4;
            ra[it] = make_float4(0.f, 0.f, 0.f, 0.f);
            rb[it] = ra[it];
            if (m0 + row < n) ra[it] = *reinterpret_cast<const float4 *>(A + (m0 + row) * lda + k0 + kq);
            if (n0 + row < n) rb[it] = *reinterpret_cast<const float4 *>(A + (n0 + row) * lda + k0 + kq);
        }
    };
    load(kb);
    for (int64_t k0 = kb; k0 < ke; k0 += BK) {
        __syncthreads();  // (the previous tile's MFMA reads are done)
#pragma unroll
        for (int it = 0; it < F4; ++it) {
            const int idx = tid + it * 256;
            const int row = idx / (BK / 4), kq = (idx % (BK / 4)) * 4;
            const int sr = row ^ dense_swz(kq);
            As[kq + 0][sr] = ra[it].x; As[kq + 1][sr] = ra[it].y; As[kq + 2][sr] = ra[it].z; As[kq + 3][sr] = ra[it].w;
            Bs[kq + 0][sr] = rb[it].x; Bs[kq + 1][sr] = rb[it].y; Bs[kq + 2][sr] = rb[it].z; Bs[kq + 3][sr] = rb[it].w;
        }
        __syncthreads();
        if (k0 + BK < ke) load(k0 + BK);  // in flight during the MFMAs below
#pragma unroll
        for (int kk = 0; kk < BK; kk += 2) {
            const int kr = kk + (lane >> 5), rc = lane & 31, sw = dense_swz(kr);
            float a[NB], bv[NB];
#pragma unroll
            for (int x = 0; x < NB; ++x) {
                a[x] = As[kr][(wm * (BM / 2) + x * 32 + rc) ^ sw];
                bv[x] = Bs[kr][(wn * (BM / 2) + x * 32 + rc) ^ sw];
            }
#pragma unroll
            for (int x = 0; x < NB; ++x)
#pragma unroll
                for (int y = 0; y < NB; ++y) c[x][y] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[x], bv[y], c[x][y], 0, 0, 0);
        }
    }
    // C/D map (32x32): col = lane & 31, row = (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5)
#pragma unroll
    for (int x = 0; x < NB; ++x)
#pragma unroll
        for (int y = 0; y < NB; ++y)
#pragma unroll
            for (int q = 0; q < 16; ++q) {
                const int64_t row = m0 + wm * (BM / 2) + x * 32 + (q & 3) + 8 * (q >> 2) + 4 * (lane >> 5);
                const int64_t col = n0 + wn * (BM / 2) + y * 32 + (lane & 31);
                if (row < n && col < n) K[row * ldk + col] = c[x][y][q];
            }
}

// Split-K epilogue: K[i, j] = sum_s P_s[i, j] (slices in order: deterministic) for the 64 x 64 blocks
// on and above the diagonal, written to the upper block and, transposed through LDS, to the lower one
// (the diagonal block: its upper half, mirrored), so K comes out exactly symmetric.
__global__ __launch_bounds__(256) void gram_dense_combine_kernel(int64_t n, int64_t nt, int n_parts,
                                                                 const float *__restrict__ P, int64_t ldp,
                                                                 int64_t part_stride, float *__restrict__ K,
                                                                 int64_t ldk) {
    __shared__ float tile[64][65];
    const int64_t b = blockIdx.x;
    int64_t bi = (int64_t)(((double)(2 * nt + 1) - sqrt((double)(2 * nt + 1) * (double)(2 * nt + 1) - 8.0 * (double)b)) * 0.5);
    auto first = [nt](int64_t i) { return i * nt - i * (i - 1) / 2; };
    if (bi < 0) bi = 0;
    if (bi > nt - 1) bi = nt - 1;
    while (bi > 0 && first(bi) > b) --bi;
    while (bi < nt - 1 && first(bi + 1) <= b) ++bi;
    const int64_t bj = bi + (b - first(bi));
    const int64_t i0 = bi * 64, j0 = bj * 64;
    const int t = threadIdx.x;
    const bool full = i0 + 64 <= n && j0 + 64 <= n && (ldk & 3) == 0 && (ldp & 3) == 0 && (part_stride & 3) == 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int y = (t >> 4) + 16 * q, x = (t & 15) * 4;
        const int64_t i = i0 + y;
        f32x4 acc = {0.f, 0.f, 0.f, 0.f};
        if (full) {
            for (int sl = 0; sl < n_parts; ++sl)
                acc += __builtin_nontemporal_load(reinterpret_cast<const f32x4 *>(P + sl * part_stride + i * ldp + j0 + x));
        } else {
            for (int sl = 0; sl < n_parts; ++sl)
#pragma unroll
                for (int c = 0; c < 4; ++c)
                    if (i < n && j0 + x + c < n) acc[c] += P[sl * part_stride + i * ldp + j0 + x + c];
        }
#pragma unroll
        for (int c = 0; c < 4; ++c) tile[y][x + c] = acc[c];
        if (full && bi != bj) {
            __builtin_nontemporal_store(acc, reinterpret_cast<f32x4 *>(K + i * ldk + j0 + x));
        } else {
#pragma unroll
            for (int c = 0; c < 4; ++c)
                if (i < n && j0 + x + c < n && j0 + x + c >= i) K[i * ldk + j0 + x + c] = acc[c];
        }
    }
    __syncthreads();
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

__global__ __launch_bounds__(256) void densify_kernel(int64_t n_rows, const int64_t *__restrict__ ptr,
                                                      const int32_t *__restrict__ idx, const float *__restrict__ val,
                                                      float *__restrict__ out, int64_t lda) {
    const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= n_rows) return;
    const int lane = threadIdx.x & 63;
    for (int64_t e = ptr[row] + lane; e < ptr[row + 1]; e += 64) out[row * lda + idx[e]] = val[e];
}

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
                                 float *K, int64_t ldk, hipStream_t st, int32_t *tickets = nullptr,
                                 const void *t_split = nullptr, int64_t slot_buckets = 0,
                                 const int32_t *row_cuts = nullptr) {
    if (unit == GRF_REC_SLOT) {
        // the slot layout: 8-wave tiles (one batch of 64 nonzeros per wave: two stream buckets each),
        // the default unroll and exact tails; the overflow pairs follow the slot_buckets slots
        GRF_REQUIRE(!tickets && !t_split, GRF_EUNSUPPORTED, "gram: GRF_REC_SLOT has no fused / split variant");
        GRF_REQUIRE(32 * slot_buckets < ((int64_t)1 << 30), GRF_EUNSUPPORTED,
                    "gram: GRF_REC_SLOT slots beyond 32-bit record offsets");
        const size_t lds = gram_lds_bytes(tl.W, 8, 2);
        const int64_t max_tiles = ((1ll << 32) - 1) / (64 * 8);
        for (int64_t t0 = t_first; t0 < t_last; t0 += max_tiles) {
            const int64_t nt = (t_last - t0) < max_tiles ? (t_last - t0) : max_tiles;
            gram_sparse_kernel<8, 1, 8, true, false, true><<<(unsigned)nt, 512, lds, st>>>(
                n_total, row_begin, tl, t0, ptr, idx, val, reinterpret_cast<const uint2 *>(t_desc),
                reinterpret_cast<const unsigned char *>(t_rec), unit, t_rowshift, K, ldk, nullptr, nullptr,
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
    const uint16_t *split = (use_split && tl.sym && !tickets) ? (const uint16_t *)t_split : nullptr;
    // tuning knobs (defaults = measured best on MI355X): gathers in flight per wave, waves per tile
    static const int knobs = [] {
        const char *e = getenv("GRF_GRAM_UNROLL"), *w = getenv("GRF_GRAM_WAVES"), *t = getenv("GRF_GRAM_TAIL");
        const int u = e ? atoi(e) : 8, ww = w ? atoi(w) : 0, tt = t ? atoi(t) : 1;
        return (tt ? 1000 : 0) + ((u == 4 || u == 8 || u == 16) ? u : 8) * 10 + (ww == 8 ? 8 : ww == 4 ? 4 : 0);
    }();
    const bool tail_exact = knobs >= 1000;
    // waves per tile: 4 for W <= 4096 (4 tiles of 40 KiB per CU), 8 for wider bands (2 tiles of
    // 76 KiB per CU: 16 waves per CU either way); measured best at both widths (GRF_GRAM_WAVES overrides)
    const int waves = knobs % 10 ? knobs % 10 : (tl.W > 4096 ? 8 : 4);
    const int unroll = (knobs % 1000) / 10, halves = waves == 8 ? 1 : 2;
    static const size_t lds_pad = [] {  // (experiments: GRF_GRAM_LDS_PAD bytes per tile -> fewer tiles per CU)
        const char *e = getenv("GRF_GRAM_LDS_PAD");
        return e ? (size_t)atoll(e) : (size_t)0;
    }();
    const size_t lds = gram_lds_bytes(tl.W, waves, halves) + lds_pad;
    // one launch covers at most 2^32 - 1 work-items: split the tile range
    const int64_t max_tiles = ((1ll << 32) - 1) / (64 * waves);
    for (int64_t t0 = t_first; t0 < t_last; t0 += max_tiles) {
        const int64_t nt = (t_last - t0) < max_tiles ? (t_last - t0) : max_tiles;
#define GRF_GRAM_LAUNCH_F(WV, H, U, T, F)                                                                         \
    gram_sparse_kernel<WV, H, U, T, F><<<(unsigned)nt, 64 * WV, lds, st>>>(n_total, row_begin, tl, t0, ptr, idx,   \
                                                                        val, reinterpret_cast<const uint2 *>(t_desc), \
                                                                        reinterpret_cast<const unsigned char *>(t_rec), \
                                                                        unit, t_rowshift, K, ldk, tickets, split, 0, \
                                                                        gram_balance(tl, unit), row_cuts)
#define GRF_GRAM_LAUNCH_T(WV, H, U, T) GRF_GRAM_LAUNCH_F(WV, H, U, T, false)
#define GRF_GRAM_LAUNCH(WV, H, U)                                                                                 \
    do {                                                                                                          \
        if (tail_exact) GRF_GRAM_LAUNCH_T(WV, H, U, true);                                                        \
        else GRF_GRAM_LAUNCH_T(WV, H, U, false);                                                                  \
    } while (0)
        if (tickets) {  // fused symmetric completion: the default unroll and exact tails only
            if (waves == 8) GRF_GRAM_LAUNCH_F(8, 1, 8, true, true);
            else GRF_GRAM_LAUNCH_F(4, 2, 8, true, true);
        } else if (waves == 8) {
            if (unroll == 4) GRF_GRAM_LAUNCH(8, 1, 4);
            else GRF_GRAM_LAUNCH(8, 1, 8);
        } else {
            if (unroll == 4) GRF_GRAM_LAUNCH(4, 2, 4);
            else if (unroll == 16) GRF_GRAM_LAUNCH(4, 2, 16);
            else GRF_GRAM_LAUNCH(4, 2, 8);
        }
#undef GRF_GRAM_LAUNCH
#undef GRF_GRAM_LAUNCH_T
#undef GRF_GRAM_LAUNCH_F
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
                             ldk, st, nullptr, t_split, nb * n_total);
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
                             S(stream), nullptr, t_split, tl.nb * n_total, row_cuts);
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

size_t grf_gram_sym_fused_workspace_bytes(int64_t n_total, int64_t band_width) {
    if (n_total <= 0 || band_width <= 0) return 16;
    const int64_t nb = cdiv<int64_t>(n_total, band_width), ng = cdiv<int64_t>(n_total, kFuseGroup);
    return (size_t)cdiv<int64_t>(nb * ng * 4, 16) * 16;
}

int32_t grf_gram_sparse_sym_fused(int64_t n_total, const int64_t *ptr, const int32_t *idx, const float *val,
                                  int64_t band_width, int32_t rec_unit, const uint32_t *t_desc, const void *t_rec,
                                  const int32_t *t_rowshift, float *K, int64_t ldk, int32_t part_begin,
                                  int32_t part_end, int32_t n_parts, void *workspace, size_t workspace_bytes,
                                  grf_stream_t stream) {
    int32_t rc = gram_sparse_check(n_total, 0, n_total, ptr, band_width, rec_unit, t_desc, t_rec, t_rowshift, K, ldk);
    if (rc != GRF_OK) return rc;
    GRF_REQUIRE(n_parts >= 1 && 0 <= part_begin && part_begin <= part_end && part_end <= n_parts, GRF_EINVAL,
                "grf_gram_sparse_sym_fused: bad tile parts [%d, %d) of %d", part_begin, part_end, n_parts);
    GRF_REQUIRE(ldk % 4 == 0 && ((uintptr_t)K & 15) == 0, GRF_EINVAL,
                "grf_gram_sparse_sym_fused: K must be 16-byte aligned with ldk a multiple of 4");
    const size_t need = grf_gram_sym_fused_workspace_bytes(n_total, band_width);
    GRF_REQUIRE(workspace && workspace_bytes >= need && ((uintptr_t)workspace & 15) == 0, GRF_EINVAL,
                "grf_gram_sparse_sym_fused: workspace needs %zu bytes (16-byte aligned), got %zu", need,
                workspace_bytes);
    if (n_total == 0 || part_begin == part_end) return GRF_OK;
    hipStream_t st = S(stream);
    // the group tickets are zeroed by the call that issues the first part
    if (part_begin == 0) GRF_CHECK_HIP(hipMemsetAsync(workspace, 0, need, st));
    const GramTiles tl{n_total, band_width, cdiv<int64_t>(n_total, band_width), true, 0, (int32_t)n_total};
    const int64_t total = tl.total();
    const int64_t t0 = total * part_begin / n_parts, t1 = total * part_end / n_parts;
    if (t1 <= t0) return GRF_OK;
    return gram_tiles_launch(n_total, 0, tl, t0, t1, ptr, idx, val, t_desc, t_rec, rec_unit, t_rowshift, K, ldk, st,
                             reinterpret_cast<int32_t *>(workspace));
}

// Column block: K[r - row_begin, 0 : t_rows] = sum_k Phi[r, k] Phi_B[:, k] for the rows r of Phi
// against the t_rows rows of another matrix Phi_B (a rank's own rows) whose banded transpose is
// given; the row shifts come from grf_phi_row_shifts over all of Phi.  With Phi_B = Phi[b:e] this
// is K[:, b:e] -- entry for entry the row mode's K[r, b + j] -- so a rank transposes only its rows.
static int32_t gram_sparse_cols_impl(int64_t n_cols, int64_t row_begin, int64_t row_end, const int64_t *ptr,
                                     const int32_t *idx, const float *val, const int32_t *row_shift, int64_t t_rows,
                                     int64_t sym_row0, int64_t band_width, int32_t rec_unit, const uint32_t *t_desc,
                                     const void *t_rec, const void *t_split, float *K, int64_t ldk, bool add_k,
                                     grf_stream_t stream) {
    GRF_REQUIRE(n_cols > 0 && 0 <= row_begin && row_begin <= row_end && ptr && idx && val && row_shift &&
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
        tl.add_k = add_k;
        return gram_tiles_launch(n_cols, r0, tl, 0, tl.total(), ptr, idx, val, t_desc, t_rec, rec_unit, row_shift,
                                 K + (r0 - row_begin) * ldk, ldk, st, nullptr, sym ? t_split : nullptr, nb * n_cols);
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
                                 rec_unit, t_desc, t_rec, t_split, K, ldk, false, stream);
}

// grf_gram_sparse_cols whose write-out ADDS the rounded fixed-point sums to the block (which holds the
// dense hub-column part first: the column-block hub-column split)
int32_t grf_gram_sparse_cols_add(int64_t n_cols, int64_t row_begin, int64_t row_end, const int64_t *ptr,
                                 const int32_t *idx, const float *val, const int32_t *row_shift, int64_t t_rows,
                                 int64_t sym_row0, int64_t band_width, int32_t rec_unit, const uint32_t *t_desc,
                                 const void *t_rec, const void *t_split, float *K, int64_t ldk, void *workspace,
                                 size_t workspace_bytes, grf_stream_t stream) {
    (void)workspace;
    (void)workspace_bytes;
    return gram_sparse_cols_impl(n_cols, row_begin, row_end, ptr, idx, val, row_shift, t_rows, sym_row0, band_width,
                                 rec_unit, t_desc, t_rec, t_split, K, ldk, true, stream);
}

// K rows [row_begin, row_end) of the whole K using the symmetry inside the row block: the bands
// that lie inside the block ("interior", rows [B0, B1)) are computed only on and above the
// diagonal for the block's interior rows and mirrored; everything else is the row mode.
int32_t grf_gram_sparse_block(int64_t n_total, int64_t row_begin, int64_t row_end, const int64_t *ptr,
                              const int32_t *idx, const float *val, int64_t band_width, int32_t rec_unit,
                              const uint32_t *t_desc, const void *t_rec, const void *t_split,
                              const int32_t *t_rowshift, float *K,
                              int64_t ldk, void *workspace, size_t workspace_bytes, grf_stream_t stream) {
    int32_t rc = gram_sparse_check(n_total, row_begin, row_end, ptr, band_width, rec_unit, t_desc, t_rec, t_rowshift,
                                   K, ldk);
    if (rc != GRF_OK) return rc;
    if (row_end == row_begin || n_total == 0) return GRF_OK;
    hipStream_t st = S(stream);
    const int64_t W = band_width, nb = cdiv<int64_t>(n_total, W);
    const int64_t J0 = cdiv<int64_t>(row_begin, W);
    const int64_t J1 = row_end == n_total ? nb : row_end / W;
    if (J1 <= J0) {
        return gram_sparse_launch(n_total, row_begin, row_end - row_begin, false, 0, n_total, ptr, idx, val, W,
                                  rec_unit, t_desc, t_rec, t_rowshift, K, ldk, st);
    }
    const int64_t B0 = J0 * W, B1 = std::min<int64_t>(J1 * W, n_total);
    auto launch = [&](int64_t r0, int64_t r1, int64_t ja, int64_t jb, bool sym) -> int32_t {
        if (r1 <= r0 || jb <= ja) return GRF_OK;
        GramTiles tl{r1 - r0, W, jb - ja, sym, 0, (int32_t)n_total};
        tl.J_off = ja;
        const int64_t n_tiles = tl.total();
        return gram_tiles_launch(n_total, r0, tl, 0, n_tiles, ptr, idx, val, t_desc, t_rec, rec_unit, t_rowshift,
                                 K + (r0 - row_begin) * ldk, ldk, st, nullptr, sym ? t_split : nullptr, nb * n_total);
    };
    if ((rc = launch(B0, B1, J0, J1, true)) != GRF_OK) return rc;            // interior, symmetric
    if ((rc = launch(row_begin, row_end, 0, J0, false)) != GRF_OK) return rc;  // bands before
    if ((rc = launch(row_begin, row_end, J1, nb, false)) != GRF_OK) return rc; // bands after
    if ((rc = launch(row_begin, B0, J0, J1, false)) != GRF_OK) return rc;     // edge rows x interior
    if ((rc = launch(B1, row_end, J0, J1, false)) != GRF_OK) return rc;
    return grf_gram_mirror(B1 - B0, K + (B0 - row_begin) * ldk + B0, ldk, 0, stream);
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
    GRF_REQUIRE_GRID(grid, 256, "gram_mirror_kernel");
    static const int padded = [] {  // GRF_MIRROR_PADDED=1: the padded 64 x 65 tile (A/B against the swizzle)
        const char *e = getenv("GRF_MIRROR_PADDED");
        return e ? atoi(e) : 0;
    }();
    static const int pipe = [] {  // GRF_MIRROR_PIPE=1: the bounded grid with the next block's loads in flight
        const char *e = getenv("GRF_MIRROR_PIPE");  // (measured slower beside the next front: off by default)
        return e ? atoi(e) : 0;
    }();
    if (padded) gram_mirror_kernel<<<(unsigned)grid, 256, 0, S(stream)>>>(n, nt, blocks, K, ldk);
    else if (pipe && grid < blocks && (ldk & 3) == 0 && nt >= 3) {
        // the full strictly-upper blocks, with the next block's loads in flight, then the edges
        const int64_t nf = n % 64 == 0 ? nt : nt - 1, nfull = nf * (nf - 1) / 2;
        const int64_t g = grid < nfull ? grid : nfull;
        if (nfull > 0) gram_mirror_pipe_kernel<<<(unsigned)g, 256, 0, S(stream)>>>(nf, nfull, K, ldk);
        const int64_t nedge = nt + (n % 64 == 0 ? 0 : nt - 1);
        gram_mirror_edge_kernel<<<(unsigned)nedge, 256, 0, S(stream)>>>(n, nt, K, ldk);
    } else gram_mirror_swz_kernel<<<(unsigned)grid, 256, 0, S(stream)>>>(n, nt, blocks, K, ldk);
    GRF_CHECK_LAUNCH("gram_mirror_kernel");
    return GRF_OK;
}

int32_t grf_gram_mirror_rect(int64_t n, float *K, int64_t ldk, int64_t row_begin, int64_t row_end, int64_t col_begin,
                             int64_t col_end, int64_t max_workgroups, grf_stream_t stream) {
    GRF_REQUIRE(n >= 0 && K && ldk >= n && 0 <= row_begin && row_begin <= row_end && row_end <= n && 0 <= col_begin &&
                    col_begin <= col_end && col_end <= n && row_begin % 64 == 0 && col_begin % 64 == 0,
                GRF_EINVAL, "grf_gram_mirror_rect: bad arguments (ranges inside [0, n), starts multiples of 64)");
    if (row_end == row_begin || col_end == col_begin) return GRF_OK;
    const int64_t bi0 = row_begin / 64, bj0 = col_begin / 64;
    const int64_t nbi = cdiv<int64_t>(row_end, 64) - bi0, nbj = cdiv<int64_t>(col_end, 64) - bj0;
    const int64_t blocks = nbi * nbj;
    const int64_t grid = max_workgroups > 0 && max_workgroups < blocks ? max_workgroups : blocks;
    GRF_REQUIRE_GRID(grid, 256, "gram_mirror_rect_kernel");
    gram_mirror_rect_kernel<<<(unsigned)grid, 256, 0, S(stream)>>>(n, bi0, bj0, nbj, blocks, K, ldk);
    GRF_CHECK_LAUNCH("gram_mirror_rect_kernel");
    return GRF_OK;
}

// split-K slices for a dense Gram of n rows (128-row tiles on and above the diagonal): measured on
// MI355X (tools/dense_sweep.py, profiles/r02_dense_splitk.txt) 2 slices below 384 tiles (n < 3.5 k:
// C3's 253 tiles, 0.209-0.214 ms vs 0.221 with 4), 4 below 1024 tiles (n < 5.8 k), 2 below 4096
// (n < 11.6 k), none above; every slice at least 256 deep
static int dense_splits(int64_t n, int64_t k_dim) {
    static const int env_split = [] {  // GRF_DENSE_SPLIT: A/B knob (1 = never split)
        const char *e = getenv("GRF_DENSE_SPLIT");
        return e ? atoi(e) : 0;
    }();
    if (env_split > 0) return env_split;
    const int64_t nt = cdiv<int64_t>(n, 128), tiles = nt * (nt + 1) / 2;
    const int64_t S = tiles < 384 ? 2 : tiles < 1024 ? 4 : tiles < 4096 ? 2 : 1;
    return (int)std::max<int64_t>(1, std::min<int64_t>(S, k_dim / 256));
}

size_t grf_gram_dense_workspace_bytes(int64_t n, int64_t k_dim) {
    const int S = n > 0 ? dense_splits(n, k_dim) : 1;
    if (S <= 1) return 16;
    const int64_t ldp = cdiv<int64_t>(n, 64) * 64;
    return (size_t)S * (size_t)n * (size_t)ldp * sizeof(float);
}

static int32_t gram_dense_impl(int64_t n, int64_t k_dim, const float *A, int64_t lda, float *K, int64_t ldk,
                               void *workspace, size_t workspace_bytes, bool upper_only, grf_stream_t stream) {
    GRF_REQUIRE(n >= 0 && k_dim >= 0 && A && K && ldk >= n && lda >= k_dim, GRF_EINVAL,
                "grf_gram_dense: bad arguments");
    GRF_REQUIRE(lda % 16 == 0 && ((uintptr_t)A & 15) == 0, GRF_EINVAL,
                "grf_gram_dense: lda must be a multiple of 16 and A 16-byte aligned");
    if (n == 0) return GRF_OK;
    // tile: 128 when the upper triangle of 128-tiles gives >= 2 workgroups per CU (n >= ~4.5 k), else
    // 64 -- or 128 with split-K slices when a workspace for the partials is given (small n)
    const int64_t nt128 = cdiv<int64_t>(n, 128);
    static const int env_tile = [] {  // GRF_DENSE_TILE=64/128, GRF_DENSE_BK=16/32: A/B knobs
        const char *e = getenv("GRF_DENSE_TILE");
        return e ? atoi(e) : 0;
    }();
    static const int env_bk = [] {
        const char *e = getenv("GRF_DENSE_BK");
        return e ? atoi(e) : 0;
    }();
    int ns = (workspace && !upper_only) ? dense_splits(n, k_dim) : 1;
    const int64_t ldp = cdiv<int64_t>(n, 64) * 64;
    if (ns > 1 && workspace_bytes < (size_t)ns * (size_t)n * (size_t)ldp * sizeof(float)) ns = 1;
    const bool big = ns > 1 || (env_tile ? env_tile == 128 : nt128 * (nt128 + 1) / 2 >= 512);
    int bk = (!big && lda % 32 == 0) ? 32 : 16;  // (zero padding up to lda covers the last k-tile)
    if (env_bk == 32 && lda % 32 == 0) bk = 32;
    if (env_bk == 16) bk = 16;
    const int64_t kpad = cdiv<int64_t>(k_dim, bk) * bk;
    GRF_REQUIRE(kpad <= lda, GRF_EINVAL, "grf_gram_dense: lda must cover k_dim rounded up to %d", bk);
    const int64_t nt = cdiv<int64_t>(n, big ? 128 : 64), tiles = nt * (nt + 1) / 2;
    GRF_REQUIRE_GRID(tiles, 256, "gram_dense_kernel");
    const int64_t k_split = ns > 1 ? cdiv<int64_t>(cdiv<int64_t>(kpad, ns), bk) * bk : kpad;
    if (ns > 1) ns = (int)cdiv<int64_t>(kpad, k_split);
    float *out = ns > 1 ? reinterpret_cast<float *>(workspace) : K;
    const int64_t ldo = ns > 1 ? ldp : ldk, pstride = ns > 1 ? n * ldp : 0;
    GRF_REQUIRE_GRID(tiles * ns, 256, "gram_dense_kernel");
    const unsigned grid = (unsigned)(tiles * ns);
    if (big && bk == 32) gram_dense_kernel<128, 32><<<grid, 256, 0, S(stream)>>>(n, nt, kpad, A, lda, out, ldo, k_split, pstride, ns);
    else if (big) gram_dense_kernel<128, 16><<<grid, 256, 0, S(stream)>>>(n, nt, kpad, A, lda, out, ldo, k_split, pstride, ns);
    else if (bk == 32) gram_dense_kernel<64, 32><<<grid, 256, 0, S(stream)>>>(n, nt, kpad, A, lda, out, ldo, k_split, pstride, ns);
    else gram_dense_kernel<64, 16><<<grid, 256, 0, S(stream)>>>(n, nt, kpad, A, lda, out, ldo, k_split, pstride, ns);
    GRF_CHECK_LAUNCH("gram_dense_kernel");
    if (ns == 1) return upper_only ? GRF_OK : grf_gram_mirror(n, K, ldk, 0, stream);  // the lower triangle
    const int64_t nt64 = cdiv<int64_t>(n, 64), blocks = nt64 * (nt64 + 1) / 2;
    GRF_REQUIRE_GRID(blocks, 256, "gram_dense_combine_kernel");
    gram_dense_combine_kernel<<<(unsigned)blocks, 256, 0, S(stream)>>>(n, nt64, ns, out, ldp, pstride, K, ldk);
    GRF_CHECK_LAUNCH("gram_dense_combine_kernel");
    return GRF_OK;
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
