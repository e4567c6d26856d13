// grf_gram_dense.hip -- the dense path's Gram K = A A^T on the MFMA: the fp32 instruction (grf_gram_dense_ws) and
// the same product on the bf16 matrix cores from an exact three-plane split of A (grf_gram_dense_split, below).
//
// Reference: efficient_graph_gp/graph_kernels/fast_grf_kernel_general.py:38-39 (Phi = F f; K = Phi Phi^T,
// a numpy dgemm); here A is the dense fp32 Phi (n x k_dim, row-major, zero-padded to lda).
//
// Tiles.  K is symmetric, so only the 128 x 128 tiles on and above the diagonal are computed
// (n^2 k flops instead of 2 n^2 k); every tile writes its entries to both triangles, so there is no
// mirror pass.  A workgroup of 4 waves (2 x 2) owns one tile, each wave a 64 x 64 quarter of 2 x 2 blocks
// of v_mfma_f32_32x32x2f32 (64 accumulator VGPRs).  A wave whose quarter lies wholly below the diagonal
// (diagonal tiles) or past n (edge tiles) issues no MFMAs.
//
// Staging.  Both operands are rows of A (k contiguous), so the k-tiles go global -> LDS by LDS-DMA
// (global_load_lds_dwordx4: no VGPR round trip, no transposing LDS writes) into a ring of NST = 4 stages
// with ONE barrier per k-tile and 2 k-tiles in flight behind a counted `s_waitcnt vmcnt` (never 0 in the
// loop).  The loop is software-pipelined across the k-tile boundary: each step's MFMAs go in four chunks,
// each preceded by a quarter of the NEXT fragments' reads and followed by a quarter of the boundary's DMA
// pieces; the boundary (retire k-tile t + 1, barrier, DMA of k-tile t + 3) sits before the MFMAs of tile
// t's last fragment group, so no MFMA waits on a read issued after a barrier.  WAR: the DMA issued at
// boundary t -> t + 1 refills the stage of tile t - 1, which every wave has consumed before that barrier.
// A diagonal tile stages one operand (B = A).  The LDS image of a k-tile is row-major, BK floats a row; one
// DMA piece (64 lanes x 16 B) is lane-linear, so the bank swizzle (16-B chunk c of row r stored at
// c ^ swz(r)) is applied on the per-lane SOURCE address and on the fragment read (conflict-free
// ds_read_b128).  Measured alternatives (16 x 16 x 4 blocks, 3 / 5 stages, MFMA-first chunks, wave
// priority, operands straight to registers, 3 workgroups per CU): profiles/r04_dense_ab.txt.
//
// k order.  Lane (r, h) holds k = h BK/2 + 4 g + s at step (g, s): one ds_read_b128 gives a lane the
// operands of four MFMA steps.  Each K entry is a fixed chain of exact f32 FMAs over that order (bitwise
// reproducible run to run); diagonal tiles write each entry computed at (i, j >= i) to both (i, j) and
// (j, i), so K is exactly symmetric.
//
// Work decomposition.  From 256 tiles on, stream-K (gram_dense_sk_kernel): 512 slots (2 workgroups per
// CU) take equal runs of k-tile units of the tiles laid end to end, so no slot idles in a last partial
// round and the hand-offs of the tiles cut by slot boundaries fall at different times.  Below that every
// tile is cut into 2-4 k-slices (gram_dense_mfma_kernel).  A cut tile's pieces write their partial tiles
// (16-B stores, register layout) to slabs, and the piece that draws the last ticket sums them in piece
// order (its own from registers) and writes the tile.  Hand-off (cdna_hip_programming.md, "Projection
// GEMM" item 2): slab stores -> every wave vmcnt(0) -> barrier -> agent release -> ticket fetch_add; the
// last arriver: agent acquire -> barrier -> plain loads.  The last arriver resets its ticket, so the
// ticket block stays zero between launches (it must be zero on first use).
// One wave per 128 x 128 tile (4 x 4 blocks, AccVGPR accumulators, one wave per SIMD) was built and measured in
// round 5: half the fragment reads, but the LDS-DMA pieces per MFMA unchanged and their issue cost exposed
// without a second wave per SIMD -- 0.645 vs 0.859 at C2 (profiles/r05_dense_w1_ab.txt); removed.
#include "grf_common.h"

namespace grf {
namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4v __attribute__((ext_vector_type(4)));

constexpr int kTile = 128;  // tile edge (rows and columns)

struct DenseArgs {
    const float *A;
    float *K;
    float *slabs;      // split pieces: [split tile][slice][4 waves][16 float4][64 lanes]
    int32_t *tickets;  // one per split tile (zero between launches)
    int64_t n, nt, lda, ldk;
    int64_t kpad;      // k range (multiple of BK, zero-padded up to lda)
    int64_t n_whole;   // work items [0, n_whole) are the whole tiles 0 .. n_whole - 1
    int64_t k_split;   // k-slice width of a split tile's piece (multiple of BK)
    int32_t n_split;   // pieces per split tile (the tiles from n_whole on)
    int32_t upper_only;  // write only K[row][col] of the computed tiles (the hub panel's seed)
    int64_t sk_units, sk_kt, sk_total;  // stream-K: k-tile units per slot, per tile, in all
    int64_t dp_rounds;  // wide kernels: rounds of whole items before the stream-K units [dp_rounds grid kt, total)
    int32_t xcd_slots;  // wide kernels: number the slots XCD-contiguously (grid a multiple of 8)
};

// Fragment layout of one wave's 64 x 64 quarter.
template <int MF, int BK>
struct Layout;

template <int BK>
struct Layout<32, BK> {  // 2 x 2 blocks of 32 x 32; lane (r = lane & 31, h = lane >> 5)
    static constexpr int NBLK = 2, GG = BK / 8;  // blocks per side; fragment groups per k-tile
    typedef f32x16 acc_t;
    static constexpr int C = BK / 4;  // 16-B chunks per LDS row
    static __device__ __forceinline__ int swz(int row) { return (row / (16 / C)) & (C - 1); }
    // LDS float offset of block x's fragment, group g, in an operand image whose quarter starts at row q0
    static __device__ __forceinline__ int off(int q0, int x, int g, int lane) {
        const int row = q0 + x * 32 + (lane & 31), chunk = ((lane >> 5) * (C / 2) + g) ^ swz(row);
        return (row * C + chunk) * 4;
    }
    static constexpr int XSTRIDE = 32 * C * 16;  // bytes between the blocks x and x + 1 of one group
    static __device__ __forceinline__ acc_t mfma(float a, float b, acc_t c) {
        return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
    }
    // float4 j (0..15) of the quarter: block (x, y) = (j >> 3, (j >> 2) & 1), rows
    // 32 x + 8 (j & 3) + 4 h + 0..3, column 32 y + (lane & 31)
    static __device__ __forceinline__ f32x4v get(const acc_t (&c)[2][2], int j) {
        const acc_t &b = c[j >> 3][(j >> 2) & 1];
        const int g = j & 3;
        return f32x4v{b[4 * g], b[4 * g + 1], b[4 * g + 2], b[4 * g + 3]};
    }
    static __device__ __forceinline__ void set(acc_t (&c)[2][2], int j, f32x4v v) {
        acc_t &b = c[j >> 3][(j >> 2) & 1];
        const int g = j & 3;
        b[4 * g] = v[0], b[4 * g + 1] = v[1], b[4 * g + 2] = v[2], b[4 * g + 3] = v[3];
    }
    static __device__ __forceinline__ int row0(int j, int lane) { return 32 * (j >> 3) + 8 * (j & 3) + 4 * (lane >> 5); }
    static __device__ __forceinline__ int col(int j, int lane) { return 32 * ((j >> 2) & 1) + (lane & 31); }
};

template <int BK>
struct Stage {
    static constexpr int F = kTile * BK;          // floats per operand per stage
    static constexpr int PW = kTile * BK / 1024;  // 1-KiB DMA pieces per wave per operand (4 waves)
};

__device__ __forceinline__ void dma16(const float *src, float *lds_piece) {
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)src,
                                     (__attribute__((address_space(3))) void *)lds_piece, 16, 0, 0);
}

template <int N>
__device__ __forceinline__ void wait_vm() {
    asm volatile("s_waitcnt vmcnt(%0)" ::"i"(N) : "memory");
}

// LDS fragment reads in inline asm: hipcc's own lgkmcnt bookkeeping waited for the NEXT fragments'
// reads before the current MFMAs (lgkmcnt(0) where the older reads alone were needed), so the reads are
// issued here and retired by lgkm_done(), a wait that names every destination register ("+v": no
// consumer or copy of them can move above it; cdna_hip_programming.md, inline-asm VGPR loads, form ii).
template <int OFF>
__device__ __forceinline__ f32x4v ds_read16(uint32_t addr) {
    f32x4v r;
    asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(r) : "v"(addr), "i"(OFF));
    return r;
}

__device__ __forceinline__ uint32_t lds_addr(const float *p) {
    return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) float *)p;
}

// tile b (row-major over the upper triangle of the nt x nt grid) -> (bi, bj), bj >= bi
__device__ __forceinline__ void tile_coords(int64_t b, int64_t nt, int64_t &bi, int64_t &bj) {
    const double t = (double)(2 * nt + 1);
    int64_t i = (int64_t)((t - sqrt(t * t - 8.0 * (double)b)) * 0.5);
    auto first = [nt](int64_t r) { return r * nt - r * (r - 1) / 2; };
    if (i < 0) i = 0;
    if (i > nt - 1) i = nt - 1;
    while (i > 0 && first(i) > b) --i;
    while (i < nt - 1 && first(i + 1) <= b) ++i;
    bi = i;
    bj = i + (b - first(i));
}

// The k-loop over [kb, ke) of one tile.  DIAG: B = A (one operand staged).  LIVE: this wave computes
// (a dead wave still stages its share of the DMA and joins the barriers).
template <int MF, int BK, int NST, bool DIAG, bool LIVE>
__device__ __forceinline__ void kloop(float *lds, const float *const *srcA, const float *const *srcB, int64_t kb,
                                      int64_t ke, int wave, const int *aoff, const int *boff,
                                      typename Layout<MF, BK>::acc_t (&c)[Layout<MF, BK>::NBLK][Layout<MF, BK>::NBLK]) {
    using L = Layout<MF, BK>;
    using St = Stage<BK>;
    constexpr int NB = L::NBLK, GG = L::GG;
    static_assert(NB == 2 && GG == 2, "the step sequence below is written for 2 x 2 blocks and 2 groups per k-tile");
    constexpr int D = NST - 2;  // k-tiles in flight behind the one being published
    static_assert(D >= 1 && D <= 3, "the pipelined k-loop needs 3 <= NST <= 5");
    constexpr int G = DIAG ? St::PW : 2 * St::PW;  // DMA instructions per wave per k-tile
    const int64_t nk = (ke - kb) / BK;
    const uint32_t lds0 = lds_addr(lds);
    // DMA pieces q, q + 4, ... of k-tile t (all of them: issue(t, -1))
    auto issue = [&](int64_t t, int q) {
        float *base = lds + (int)(t % NST) * 2 * St::F + wave * St::PW * 256;
        const int64_t k0 = kb + t * BK;
#pragma unroll
        for (int j = 0; j < G; ++j) {
            if (q >= 0 && (j & 3) != q) continue;
            if (j < St::PW) dma16(srcA[j] + k0, base + j * 256);
            else dma16(srcB[j - St::PW] + k0, base + St::F + (j - St::PW) * 256);
        }
    };
    // retire the oldest k-tile in flight (`ahead` younger ones may stay in flight) and publish it
    auto retire = [&](int64_t ahead) {  // (ahead <= D - 1)
        if constexpr (D == 3) {
            if (ahead >= 2) wait_vm<2 * G>();
            else if (ahead == 1) wait_vm<G>();
            else wait_vm<0>();
        } else if constexpr (D == 2) {
            if (ahead >= 1) wait_vm<G>();
            else wait_vm<0>();
        } else {
            wait_vm<0>();
        }
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
    };
    struct Frag { f32x4v a[NB], b[NB]; };
    // read q (0..3) of fragment group g of k-tile t: a0, b0, a1, b1
    auto read_q = [&](int64_t t, int g, int q, Frag &f) {
        const uint32_t As = lds0 + (uint32_t)(t % NST) * (2 * St::F * 4);
        const uint32_t Bs = DIAG ? As : As + St::F * 4;
        const uint32_t ab = As + (uint32_t)aoff[g] * 4, bb = Bs + (uint32_t)boff[g] * 4;
        switch (q) {
            case 0: f.a[0] = ds_read16<0>(ab); break;
            case 1: f.b[0] = ds_read16<0>(bb); break;
            case 2: f.a[1] = ds_read16<L::XSTRIDE>(ab); break;
            default: f.b[1] = ds_read16<L::XSTRIDE>(bb); break;
        }
    };
    // every read issued so far has landed; f's registers are redefined here (nothing reads them earlier)
    auto lgkm_done = [&](Frag &f) {
        asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(f.a[0]), "+v"(f.a[1]), "+v"(f.b[0]), "+v"(f.b[1])::"memory");
    };
    auto mfma_q = [&](const Frag &f, int s) {  // k-step s of the group: the 2 x 2 blocks
        if constexpr (LIVE) {
#pragma unroll
            for (int x = 0; x < NB; ++x)
#pragma unroll
                for (int y = 0; y < NB; ++y) c[x][y] = L::mfma(f.a[x][s], f.b[y][s], c[x][y]);
        }
    };
    if (nk <= 0) return;
#pragma unroll
    for (int t = 0; t < D; ++t)
        if (t < nk) issue(t, -1);
    retire(D - 1 < nk - 1 ? D - 1 : nk - 1);
    if (D < nk) issue(D, -1);
    // One step = the MFMAs of fragment group g of k-tile t in four chunks (one k-step each); ahead of chunk q
    // go read q of the NEXT group's fragments (so the last read still has 4 MFMAs behind it), after it a
    // quarter of the boundary's DMA pieces.  The two fragment sets alternate by name (no register copies).
    // Boundary t -> t + 1 (g = 1): k-tiles up to min(t + D, nk - 1) are issued; the DMA refills the stage of
    // tile t - 1, which every wave has consumed before this barrier.
    auto step = [&](int64_t t, int g, const Frag &cur, Frag &nxt) {
        const bool boundary = g + 1 == GG;
        const int64_t tn = boundary ? t + 1 : t;
        const int gn = boundary ? 0 : g + 1;
        const bool dma = boundary && t + 1 + D < nk;
        if (boundary) retire((t + D < nk - 1 ? t + D : nk - 1) - (t + 1));
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            __builtin_amdgcn_sched_barrier(0);
            read_q(tn, gn, q, nxt);
            __builtin_amdgcn_sched_barrier(0);
            mfma_q(cur, q);
            __builtin_amdgcn_sched_barrier(0);
            if (dma) issue(t + 1 + D, q);
        }
        __builtin_amdgcn_sched_barrier(0);
        lgkm_done(nxt);
    };
    Frag fa, fb;
#pragma unroll
    for (int q = 0; q < 4; ++q) read_q(0, 0, q, fa);
    lgkm_done(fa);
    for (int64_t t = 0; t + 1 < nk; ++t) {
        step(t, 0, fa, fb);
        step(t, 1, fb, fa);
    }
    step(nk - 1, 0, fa, fb);  // (g = 0 of the last k-tile reads g = 1: no boundary)
#pragma unroll
    for (int q = 0; q < 4; ++q) {  // the last step: no reads after it
        __builtin_amdgcn_sched_barrier(0);
        mfma_q(fb, q);
    }
    __builtin_amdgcn_sched_barrier(0);
}

// Writes the wave's 64 x 64 quarter (rows r0.., cols c0.. of K) to K[row][col] and, mirrored,
// K[col][row] (a lane's float4 j holds 4 consecutive rows of one column: one 16-B store mirrored).
// diag: the quarter straddles the diagonal (a diagonal tile): only entries with col >= row are written
// (each to both places).  upper: K[row][col] only (the whole quarter, nothing mirrored).
template <int MF, int BK>
__device__ __forceinline__ void write_quarter(const DenseArgs &a,
                                              const typename Layout<MF, BK>::acc_t (&c)[Layout<MF, BK>::NBLK]
                                                                                       [Layout<MF, BK>::NBLK],
                                              int64_t r0, int64_t c0, bool diag, bool upper, int lane) {
    using L = Layout<MF, BK>;
    const int64_t n = a.n, ldk = a.ldk;
    float *K = a.K;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
        const f32x4v v = L::get(c, j);
        const int64_t row = r0 + L::row0(j, lane), col = c0 + L::col(j, lane);
        if (col >= n) continue;
        if (upper) {
#pragma unroll
            for (int s = 0; s < 4; ++s)
                if (row + s < n) K[(row + s) * ldk + col] = v[s];
        } else if (!diag && row + 3 < n) {
#pragma unroll
            for (int s = 0; s < 4; ++s) K[(row + s) * ldk + col] = v[s];
            *reinterpret_cast<f32x4v *>(K + col * ldk + row) = v;  // the mirrored entries
        } else {
#pragma unroll
            for (int s = 0; s < 4; ++s) {
                const int64_t rr = row + s;
                if (rr < n && (!diag || col >= rr)) {
                    K[rr * ldk + col] = v[s];
                    K[col * ldk + rr] = v[s];
                }
            }
        }
    }
}

// One wave's part of tile `tile` over the k range [kb, ke): its quarter (rows qr.., cols qc..), whether it
// lies below the diagonal, and the accumulators (zeroed here).
struct Quarter {
    int64_t qr, qc;
    bool diag, below;
};

template <int MF, int BK, int NST>
__device__ __forceinline__ Quarter tile_compute(const DenseArgs &a, float *lds, int64_t tile, int64_t kb, int64_t ke,
                                                int wave, int lane,
                                                typename Layout<MF, BK>::acc_t (&c)[Layout<MF, BK>::NBLK]
                                                                                   [Layout<MF, BK>::NBLK]) {
    using L = Layout<MF, BK>;
    using St = Stage<BK>;
    constexpr int NB = L::NBLK;
    const int wm = wave >> 1, wn = wave & 1;
    int64_t bi, bj;
    tile_coords(tile, a.nt, bi, bj);
    const int64_t m0 = bi * kTile, n0 = bj * kTile;
    const bool diag = bi == bj;
    // per-lane DMA sources: piece j of this wave covers LDS chunks p = (wave * PW + j) * 64 + lane,
    // i.e. row p / C, stored chunk p % C, which holds logical chunk (p % C) ^ swz(row)
    const float *srcA[St::PW], *srcB[St::PW];
#pragma unroll
    for (int j = 0; j < St::PW; ++j) {
        const int p = (wave * St::PW + j) * 64 + lane;
        const int row = p / L::C, kc = (p % L::C) ^ L::swz(row);
        int64_t ra = m0 + row, rb = n0 + row;
        ra = ra < a.n ? ra : a.n - 1;  // (rows past n: a valid row, its products are never written)
        rb = rb < a.n ? rb : a.n - 1;
        srcA[j] = a.A + ra * a.lda + 4 * kc;
        srcB[j] = a.A + rb * a.lda + 4 * kc;
    }
    int aoff[L::GG], boff[L::GG];  // float offsets of block 0's fragment per group (block x: + x XSTRIDE bytes)
#pragma unroll
    for (int g = 0; g < L::GG; ++g) {
        aoff[g] = L::off(wm * 64, 0, g, lane);
        boff[g] = L::off(wn * 64, 0, g, lane);
    }
    // this wave's quarter: no MFMAs when it lies wholly below the diagonal or past n
    Quarter q{m0 + wm * 64, n0 + wn * 64, diag, diag && wn < wm};
    const bool live = !q.below && q.qr < a.n && q.qc < a.n;
#pragma unroll
    for (int x = 0; x < NB; ++x)
#pragma unroll
        for (int y = 0; y < NB; ++y) c[x][y] = typename L::acc_t{};
    if (diag) {
        if (live) kloop<MF, BK, NST, true, true>(lds, srcA, srcB, kb, ke, wave, aoff, boff, c);
        else kloop<MF, BK, NST, true, false>(lds, srcA, srcB, kb, ke, wave, aoff, boff, c);
    } else {
        if (live) kloop<MF, BK, NST, false, true>(lds, srcA, srcB, kb, ke, wave, aoff, boff, c);
        else kloop<MF, BK, NST, false, false>(lds, srcA, srcB, kb, ke, wave, aoff, boff, c);
    }
    return q;
}

// A piece of a split tile: its partial tile goes to slab slab_of(me) (16-B stores, register layout); the
// piece that draws the last of `pieces` tickets sums slab_of(0 .. pieces - 1) in that order (its own from
// registers) into c and returns true.  Hand-off: slab stores -> every wave vmcnt(0) -> barrier -> agent
// release -> ticket fetch_add; the last arriver resets the ticket, then agent acquire -> barrier -> loads.
// `flag` is LDS the ring no longer uses (every wave is past its k-loop).
template <int MF, int BK, int NW = 4, typename SlabOf>
__device__ __forceinline__ bool split_combine(const DenseArgs &a,
                                              typename Layout<MF, BK>::acc_t (&c)[Layout<MF, BK>::NBLK]
                                                                                 [Layout<MF, BK>::NBLK],
                                              int32_t *ticket, int64_t pieces, int64_t me, SlabOf slab_of,
                                              int32_t *flag, int wave, int lane) {
    using L = Layout<MF, BK>;
    constexpr int64_t kSlab = NW * 16 * 64;  // float4 per piece: [NW waves][16 float4][64 lanes]
    f32x4v *mine = reinterpret_cast<f32x4v *>(a.slabs) + slab_of(me) * kSlab + wave * 16 * 64 + lane;
#pragma unroll
    for (int j = 0; j < 16; ++j) mine[j * 64] = L::get(c, j);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const int32_t old = __hip_atomic_fetch_add(ticket, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const int32_t last = old == pieces - 1;
        if (last) {
            __hip_atomic_store(ticket, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        *flag = last;
    }
    __syncthreads();
    if (!*flag) return false;
    const f32x4v *slabs = reinterpret_cast<const f32x4v *>(a.slabs) + wave * 16 * 64 + lane;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
        const f32x4v own = L::get(c, j);
        f32x4v acc = me == 0 ? own : slabs[slab_of(0) * kSlab + j * 64];
        for (int64_t s = 1; s < pieces; ++s) acc += s == me ? own : slabs[slab_of(s) * kSlab + j * 64];
        L::set(c, j, acc);
    }
    return true;
}

template <int MF, int BK>
__device__ __forceinline__ void tile_write(const DenseArgs &a,
                                           const typename Layout<MF, BK>::acc_t (&c)[Layout<MF, BK>::NBLK]
                                                                                    [Layout<MF, BK>::NBLK],
                                           const Quarter &q, int wave, int lane) {
    if (q.qr >= a.n || q.qc >= a.n) return;
    if (a.upper_only) write_quarter<MF, BK>(a, c, q.qr, q.qc, false, true, lane);
    else if (!q.below) write_quarter<MF, BK>(a, c, q.qr, q.qc, q.diag && (wave >> 1) == (wave & 1), false, lane);
}

// One work item per workgroup: a whole tile, or a k-slice of one of the split tiles.
template <int MF, int BK, int NST, int WPE>
__global__ __launch_bounds__(256, WPE) void gram_dense_mfma_kernel(DenseArgs a) {
    using L = Layout<MF, BK>;
    using St = Stage<BK>;
    constexpr int NB = L::NBLK;
    __shared__ __attribute__((aligned(16))) float lds[NST * 2 * St::F];  // (one array: the DMA ring)
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const int64_t w = blockIdx.x;
    int64_t tile, slice = 0, pieces = 1;
    if (w < a.n_whole) {
        tile = w;
    } else {
        tile = a.n_whole + (w - a.n_whole) / a.n_split;
        slice = (w - a.n_whole) % a.n_split;
        pieces = a.n_split;
    }
    const int64_t kb = pieces > 1 ? slice * a.k_split : 0;
    const int64_t ke = pieces > 1 ? (kb + a.k_split < a.kpad ? kb + a.k_split : a.kpad) : a.kpad;
    typename L::acc_t c[NB][NB];
    const Quarter q = tile_compute<MF, BK, NST>(a, lds, tile, kb, ke, wave, lane, c);
    if (pieces > 1) {
        const int64_t u = tile - a.n_whole;
        if (!split_combine<MF, BK>(a, c, a.tickets + u, pieces, slice, [&](int64_t s) { return u * pieces + s; },
                                   reinterpret_cast<int32_t *>(lds), wave, lane))
            return;
    }
    tile_write<MF, BK>(a, c, q, wave, lane);
}

// Stream-K: slot (workgroup) s takes the k-tile units [s U, (s + 1) U) of the tiles laid end to end (tile t
// = units [t KT, (t + 1) KT)), so every slot does the same MFMA work and the split tiles' hand-offs fall at
// different times instead of in one burst at the end.  A tile wholly inside a slot is written directly; a
// tile cut by slot boundaries has pieces in slots s0 .. s1, piece j's slab being slot (s0 + j)'s first
// segment (j >= 1) -- slab 2 slot -- or, for j = 0, slot s0's last segment (slab 2 s0 + 1) unless the tile
// starts exactly at s0's start (slab 2 s0).  Each slot has at most one first and one last segment, so the
// slabs and the tickets (indexed by piece 0's slab) are private to one tile per launch.
template <int MF, int BK, int NST, int WPE>
__global__ __launch_bounds__(256, WPE) void gram_dense_sk_kernel(DenseArgs a) {
    using L = Layout<MF, BK>;
    using St = Stage<BK>;
    constexpr int NB = L::NBLK;
    __shared__ __attribute__((aligned(16))) float lds[NST * 2 * St::F];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const int64_t U = a.sk_units, KT = a.sk_kt;
    const int64_t u0 = (int64_t)blockIdx.x * U;
    const int64_t u1 = u0 + U < a.sk_total ? u0 + U : a.sk_total;
    for (int64_t u = u0; u < u1;) {
        const int64_t tile = u / KT, tb = tile * KT, te = tb + KT;
        const int64_t se = u1 < te ? u1 : te;
        __syncthreads();  // (the previous segment's ring reads and hand-off flag are done)
        typename L::acc_t c[NB][NB];
        const Quarter q =
            tile_compute<MF, BK, NST>(a, lds, tile, (u - tb) * BK, (se - tb) * BK, wave, lane, c);
        bool write = true;
        if (u != tb || se != te) {
            const int64_t s0 = tb / U, s1 = (te - 1) / U;
            const int64_t first = 2 * s0 + (tb == s0 * U ? 0 : 1);
            write = split_combine<MF, BK>(
                a, c, a.tickets + first, s1 - s0 + 1, blockIdx.x - s0,
                [&](int64_t j) { return j == 0 ? first : 2 * (s0 + j); }, reinterpret_cast<int32_t *>(lds), wave,
                lane);
        }
        if (write) tile_write<MF, BK>(a, c, q, wave, lane);
        u = se;
    }
}

// ------------------------------------------------------------ fp32 on the bf16 matrix cores
// The fp32 Gram by exact three-way bf16 splits (grf_gram_dense_split).  Every fp32 value a is the exact sum
// of three bf16 values: a0 = bf16(a), a1 = bf16(a - a0), a2 = a - a0 - a1 (round to nearest: a has 24
// significant bits, a0 and a1 take 8 each, so the last remainder has at most 8 and is a bf16 exactly;
// values below ~2^-100 lose their last plane to the bf16 subnormal range).  a b = sum over p, q of a_p b_q;
// the six products with p + q <= 2 are kept (the dropped three: at most (2u^3 + u^4) |a b| = (2^-23 + 2^-32)
// |a b| together, u = 2^-8), each exact
// in the MFMA's fp32 arithmetic, summed on v_mfma_f32_32x32x16_bf16 -- 16x the fp32 MFMA's rate per clock,
// so six of them cost 3/8 of the fp32 instruction's cycles per k.  The leading product a0 b0 is
// accumulated on its own (c0) and the five corrections together (c1, 2^-8 of the magnitude), c0 + c1 at
// the end: c0's rounding is the fp32 chain's, c1's 2^-8 of that, so the error bound stays the fp32 MFMA
// path's plus (2^-23 + 2^-32) sum |a_k b_k| for the dropped products.
//
// Staging is the fp32 path's (the same LDS-DMA pieces, swizzled k-tiles of BK = 16 floats, 4-stage ring,
// two workgroups per CU): the split is done in registers after the fragment reads, so the bytes staged
// per k are the fp32 kernel's.  (Staging three bf16 planes instead, 1.5x the bytes, measured slower:
// profiles/AB_LOG.md "split Gram".)  A lane's operand of one bf16 MFMA is 8 consecutive k of its row --
// the two 16-B chunks the fp32 kernel reads for fragment groups 0 and 1 (Layout<32, 16>::off).
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));  // a plane fragment as 4 packed bf16 pairs

// Two floats -> one dword of each of their three planes: v_cvt_pk_bf16_f32 (round to nearest), each plane
// unpacked from that pair (v_lshlrev / v_and; a per-element split converted every value twice), remainders
// exact.  This file is built with -fno-slp-vectorize (Makefile): hipcc otherwise packs the subtractions into
// v_pk_add_f32, which costs several issue slots beside MFMAs (MI355X_MICROARCH.md cycle constants) and
// needs s_nops.  11 VALU per pair; the split kernels run 7-8 % faster with the same bits
// (profiles/r05_split_gram_ab.txt, version 6).
typedef float f32x2v __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t cvt_pk(float x, float y) {
    return __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2v){x, y}, bf16x2v));
}
// plane 0 of one fragment (8 floats lo, hi): four v_cvt_pk_bf16_f32
__device__ __forceinline__ void plane0(const f32x4v &lo, const f32x4v &hi, u32x4 &p0) {
    p0[0] = cvt_pk(lo[0], lo[1]);
    p0[1] = cvt_pk(lo[2], lo[3]);
    p0[2] = cvt_pk(hi[0], hi[1]);
    p0[3] = cvt_pk(hi[2], hi[3]);
}

// pairs I, I + 1 of a fragment: the remainders after plane pq (exact; kept in place of the values) and their
// next plane pn -- called with (p0, p1), then (p1, p2)
template <int I>
__device__ __forceinline__ void next_plane2(f32x4v &lo, f32x4v &hi, const u32x4 &pq, u32x4 &pn) {
#pragma unroll
    for (int i = I; i < I + 2; ++i) {
        f32x4v &v = i < 2 ? lo : hi;
        const int e = 2 * (i & 1);
        const float rx = v[e] - __builtin_bit_cast(float, pq[i] << 16);
        const float ry = v[e + 1] - __builtin_bit_cast(float, pq[i] & 0xffff0000u);
        v[e] = rx;
        v[e + 1] = ry;
        pn[i] = cvt_pk(rx, ry);
    }
}

// One k-tile of a wave's 2 x 2 blocks: fragments ra[x] (A block x), rb[y] (B block y) -> 6 products per
// block.  Plane 0 of all four fragments first (16 conversions), so the four a0 b0 products start at once;
// planes 1 and 2 (two pairs of one fragment per gap) and the next k-tile's DMA pieces (issue(0 .. 3)) go
// between the MFMAs, each plane ready before the first product that reads it (sched_barrier fences).  Each
// block's c1 still takes its five products in the order s = 1 .. 5, so the sums are bitwise unchanged.
template <typename Issue>
__device__ __forceinline__ void split_ktile(f32x4v (&ra)[2][2], f32x4v (&rb)[2][2], f32x16 (&c0)[2][2],
                                            f32x16 (&c1)[2][2], Issue issue) {
    u32x4 a[2][3], b[2][3];
    plane0(ra[0][0], ra[0][1], a[0][0]);
    plane0(rb[0][0], rb[0][1], b[0][0]);
    plane0(ra[1][0], ra[1][1], a[1][0]);
    plane0(rb[1][0], rb[1][1], b[1][0]);
    __builtin_amdgcn_sched_barrier(0);
    auto mf = [&](int x, int y, int s) {
        if (s == 0) {
            c0[x][y] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a[x][0]),
                                                             __builtin_bit_cast(bf16x8, b[y][0]), c0[x][y], 0, 0, 0);
            return;
        }
        constexpr int P[6][2] = {{0, 0}, {0, 1}, {1, 0}, {0, 2}, {1, 1}, {2, 0}};
        c1[x][y] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a[x][P[s][0]]),
                                                         __builtin_bit_cast(bf16x8, b[y][P[s][1]]), c1[x][y], 0, 0, 0);
    };
    auto fence = [] { __builtin_amdgcn_sched_barrier(0); };
    // (each line: the product, then the work that fits behind it; comments name what the product reads)
    mf(0, 0, 0); next_plane2<0>(ra[0][0], ra[0][1], a[0][0], a[0][1]); fence();  // A0 p1
    mf(0, 1, 0); next_plane2<2>(ra[0][0], ra[0][1], a[0][0], a[0][1]); fence();
    mf(1, 0, 0); next_plane2<0>(rb[0][0], rb[0][1], b[0][0], b[0][1]); fence();  // B0 p1
    mf(1, 1, 0); next_plane2<2>(rb[0][0], rb[0][1], b[0][0], b[0][1]); fence();
    mf(0, 0, 1); next_plane2<0>(rb[1][0], rb[1][1], b[1][0], b[1][1]); fence();  // (A0 p0, B0 p1); B1 p1
    mf(0, 0, 2); next_plane2<2>(rb[1][0], rb[1][1], b[1][0], b[1][1]); fence();  // (A0 p1, B0 p0)
    mf(0, 1, 1); next_plane2<0>(ra[1][0], ra[1][1], a[1][0], a[1][1]); fence();  // (A0 p0, B1 p1); A1 p1
    mf(0, 1, 2); next_plane2<2>(ra[1][0], ra[1][1], a[1][0], a[1][1]); fence();
    mf(1, 0, 1); next_plane2<0>(ra[0][0], ra[0][1], a[0][1], a[0][2]); fence();  // (A1 p0, B0 p1); A0 p2
    mf(1, 0, 2); next_plane2<2>(ra[0][0], ra[0][1], a[0][1], a[0][2]); fence();  // (A1 p1, B0 p0)
    mf(1, 1, 1); next_plane2<0>(rb[0][0], rb[0][1], b[0][1], b[0][2]); fence();  // B0 p2
    mf(1, 1, 2); next_plane2<2>(rb[0][0], rb[0][1], b[0][1], b[0][2]); fence();
    mf(0, 0, 3); next_plane2<0>(rb[1][0], rb[1][1], b[1][1], b[1][2]); fence();  // (A0 p0, B0 p2); B1 p2
    mf(0, 0, 4); next_plane2<2>(rb[1][0], rb[1][1], b[1][1], b[1][2]); fence();
    mf(0, 0, 5); next_plane2<0>(ra[1][0], ra[1][1], a[1][1], a[1][2]); fence();  // (A0 p2, B0 p0); A1 p2
    mf(0, 1, 3); next_plane2<2>(ra[1][0], ra[1][1], a[1][1], a[1][2]); fence();  // (A0 p0, B1 p2)
    mf(0, 1, 4); issue(0); fence();
    mf(0, 1, 5); issue(1); fence();
    mf(1, 0, 3); issue(2); fence();
    mf(1, 0, 4); issue(3); fence();
    mf(1, 0, 5);
    mf(1, 1, 3);
    mf(1, 1, 4);
    mf(1, 1, 5);
}

// The k-loop of one tile over [kb, ke) with the split products.  The ring, the DMA pieces (issue: all of
// k-tile t's) and the retire/publish step are kloop's; per k-tile a wave reads its 2 + 2 blocks' two chunks,
// splits them and issues 4 blocks x 6 MFMAs.
template <int NST, bool DIAG, bool LIVE>
__device__ __forceinline__ void kloop_split(float *lds, const float *const *srcA, const float *const *srcB, int64_t kb,
                                            int64_t ke, int wave, const int *aoff, const int *boff,
                                            f32x16 (&c0)[2][2], f32x16 (&c1)[2][2]) {
    using L = Layout<32, 16>;
    using St = Stage<16>;
    constexpr int G = DIAG ? St::PW : 2 * St::PW;  // DMA pieces per wave per k-tile
    const int64_t nk = (ke - kb) / 16;
    // k-tile t's pieces into stage t % NST.  Issued unconditionally, the k-tiles past the last re-load the last
    // one into a stage nothing reads again (no branch in the MFMA region; every wait is the same count)
    auto issue = [&](int64_t t) {
        float *base = lds + (int)(t % NST) * 2 * St::F + wave * St::PW * 256;
        const int64_t k0 = kb + (t < nk ? t : nk - 1) * 16;
#pragma unroll
        for (int j = 0; j < G; ++j) {
            if (j < St::PW) dma16(srcA[j] + k0, base + j * 256);
            else dma16(srcB[j - St::PW] + k0, base + St::F + (j - St::PW) * 256);
        }
    };
    auto issue_part = [&](int64_t t, int q) {  // piece q of k-tile t's G (<= 4) pieces
        if (q >= G) return;
        float *base = lds + (int)(t % NST) * 2 * St::F + wave * St::PW * 256;
        const int64_t k0 = kb + (t < nk ? t : nk - 1) * 16;
        if (q < St::PW) dma16(srcA[q] + k0, base + q * 256);
        else dma16(srcB[q - St::PW] + k0, base + St::F + (q - St::PW) * 256);
    };
    if (nk <= 0) return;
#pragma unroll
    for (int t = 0; t < NST - 1; ++t) issue(t);
    for (int64_t t = 0; t < nk; ++t) {
        wait_vm<(NST - 2) * G>();  // k-tile t landed (the NST - 2 younger ones may stay in flight), then published
        __builtin_amdgcn_s_barrier();  // (also: every wave is done with k-tile t - 1, whose stage refills now)
        asm volatile("" ::: "memory");
        if constexpr (!LIVE) {
            issue(t + NST - 1);
        } else {
            const float *As = lds + (int)(t % NST) * 2 * St::F;
            const float *Bs = DIAG ? As : As + St::F;
            const char *pa = reinterpret_cast<const char *>(As), *pb = reinterpret_cast<const char *>(Bs);
            f32x4v ra[2][2], rb[2][2];
#pragma unroll
            for (int x = 0; x < 2; ++x)
#pragma unroll
                for (int g = 0; g < 2; ++g) {
                    ra[x][g] = *reinterpret_cast<const f32x4v *>(pa + aoff[g] * 4 + x * L::XSTRIDE);
                    rb[x][g] = *reinterpret_cast<const f32x4v *>(pb + boff[g] * 4 + x * L::XSTRIDE);
                }
            split_ktile(ra, rb, c0, c1, [&](int q) { issue_part(t + NST - 1, q); });
        }
    }
}

constexpr int kSplitNST = 4;

__device__ __forceinline__ Quarter tile_compute_split(const DenseArgs &a, float *lds, int64_t tile, int64_t kb,
                                                      int64_t ke, int wave, int lane, f32x16 (&c)[2][2]) {
    using L = Layout<32, 16>;
    using St = Stage<16>;
    const int wm = wave >> 1, wn = wave & 1;
    int64_t bi, bj;
    tile_coords(tile, a.nt, bi, bj);
    const int64_t m0 = bi * kTile, n0 = bj * kTile;
    const bool diag = bi == bj;
    // the fp32 path's DMA sources (tile_compute)
    const float *srcA[St::PW], *srcB[St::PW];
#pragma unroll
    for (int j = 0; j < St::PW; ++j) {
        const int p = (wave * St::PW + j) * 64 + lane;
        const int row = p / L::C, kc = (p % L::C) ^ L::swz(row);
        int64_t ra = m0 + row, rb = n0 + row;
        ra = ra < a.n ? ra : a.n - 1;
        rb = rb < a.n ? rb : a.n - 1;
        srcA[j] = a.A + ra * a.lda + 4 * kc;
        srcB[j] = a.A + rb * a.lda + 4 * kc;
    }
    int aoff[2], boff[2];
#pragma unroll
    for (int g = 0; g < 2; ++g) {
        aoff[g] = L::off(wm * 64, 0, g, lane);
        boff[g] = L::off(wn * 64, 0, g, lane);
    }
    Quarter q{m0 + wm * 64, n0 + wn * 64, diag, diag && wn < wm};
    const bool live = !q.below && q.qr < a.n && q.qc < a.n;
    f32x16 c0[2][2], c1[2][2];
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
        for (int y = 0; y < 2; ++y) {
            c0[x][y] = f32x16{};
            c1[x][y] = f32x16{};
        }
    if (diag) {
        if (live) kloop_split<kSplitNST, true, true>(lds, srcA, srcB, kb, ke, wave, aoff, boff, c0, c1);
        else kloop_split<kSplitNST, true, false>(lds, srcA, srcB, kb, ke, wave, aoff, boff, c0, c1);
    } else {
        if (live) kloop_split<kSplitNST, false, true>(lds, srcA, srcB, kb, ke, wave, aoff, boff, c0, c1);
        else kloop_split<kSplitNST, false, false>(lds, srcA, srcB, kb, ke, wave, aoff, boff, c0, c1);
    }
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
        for (int y = 0; y < 2; ++y) c[x][y] = c0[x][y] + c1[x][y];
    return q;
}

// the split path's kernels: the same work items as gram_dense_mfma_kernel / gram_dense_sk_kernel
__global__ __launch_bounds__(256, 2) void gram_split_mfma_kernel(DenseArgs a) {
    __shared__ __attribute__((aligned(16))) float lds[kSplitNST * 2 * Stage<16>::F];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const int64_t w = blockIdx.x;
    int64_t tile, slice = 0, pieces = 1;
    if (w < a.n_whole) {
        tile = w;
    } else {
        tile = a.n_whole + (w - a.n_whole) / a.n_split;
        slice = (w - a.n_whole) % a.n_split;
        pieces = a.n_split;
    }
    const int64_t kb = pieces > 1 ? slice * a.k_split : 0;
    const int64_t ke = pieces > 1 ? (kb + a.k_split < a.kpad ? kb + a.k_split : a.kpad) : a.kpad;
    f32x16 c[2][2];
    const Quarter q = tile_compute_split(a, lds, tile, kb, ke, wave, lane, c);
    if (pieces > 1) {
        const int64_t u = tile - a.n_whole;
        if (!split_combine<32, 16>(a, c, a.tickets + u, pieces, slice, [&](int64_t s) { return u * pieces + s; },
                                   reinterpret_cast<int32_t *>(lds), wave, lane))
            return;
    }
    tile_write<32, 16>(a, c, q, wave, lane);
}

__global__ __launch_bounds__(256, 2) void gram_split_sk_kernel(DenseArgs a) {
    __shared__ __attribute__((aligned(16))) float lds[kSplitNST * 2 * Stage<16>::F];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const int64_t U = a.sk_units, KT = a.sk_kt;
    const int64_t u0 = (int64_t)blockIdx.x * U;
    const int64_t u1 = u0 + U < a.sk_total ? u0 + U : a.sk_total;
    for (int64_t u = u0; u < u1;) {
        const int64_t tile = u / KT, tb = tile * KT, te = tb + KT;
        const int64_t se = u1 < te ? u1 : te;
        __syncthreads();  // (the previous segment's ring reads and hand-off flag are done)
        f32x16 c[2][2];
        const Quarter q = tile_compute_split(a, lds, tile, (u - tb) * 16, (se - tb) * 16, wave, lane, c);
        bool write = true;
        if (u != tb || se != te) {
            const int64_t s0 = tb / U, s1 = (te - 1) / U;
            const int64_t first = 2 * s0 + (tb == s0 * U ? 0 : 1);
            write = split_combine<32, 16>(
                a, c, a.tickets + first, s1 - s0 + 1, blockIdx.x - s0,
                [&](int64_t j) { return j == 0 ? first : 2 * (s0 + j); }, reinterpret_cast<int32_t *>(lds), wave,
                lane);
        }
        if (write) tile_write<32, 16>(a, c, q, wave, lane);
        u = se;
    }
}

// Wide workgroups for the split path (large n): 8 waves own a 256 x 128 item -- the row-block pair
// (2p, 2p + 1) against column block j >= 2p -- each wave the same 64 x 64 quarter (2 x 2 blocks, c0 / c1) as
// above.  A k-tile stages 256 + 128 rows (24 KiB) for 8 x 24 MFMAs instead of 256 rows for 4 x 24: 3 DMA
// pieces per wave and k-tile instead of 4, 3/4 of the staged bytes per flop (the 128-tile split kernel is
// bound by its LDS-DMA staging and its split VALU about equally: timing-only ablations in
// profiles/r05_split_gram_ab.txt).  One workgroup per CU (96 KiB ring; 3 or 5 stages measured slower), 2 waves
// per SIMD as before; stream-K over the items' k-tiles at every size.  A diagonal item (j = 2p or 2p + 1)
// stages its B rows again although they are A rows: ~2.5 % of the items at C2.
struct WideStage {
    static constexpr int FA = 2 * kTile * 16, FB = kTile * 16, F = FA + FB;  // floats per stage
    static constexpr int PW = F / 256 / 8;                                   // 1-KiB pieces per wave
};
static_assert(WideStage::PW * 256 * 8 == WideStage::F, "a stage is whole pieces over 8 waves");

// item b (row-major over (row pair p, column block j >= 2 p)) -> (p, j); row pair p has nt - 2 p items
__device__ __forceinline__ void item_coords(int64_t b, int64_t nt, int64_t &p, int64_t &j) {
    auto first = [nt](int64_t r) { return r * (nt + 1) - r * r; };
    const int64_t np = (nt + 1) / 2;
    const double t = (double)(nt + 1);
    int64_t i = (int64_t)((t - sqrt(t * t - 4.0 * (double)b)) * 0.5);
    if (i < 0) i = 0;
    if (i > np - 1) i = np - 1;
    while (i > 0 && first(i) > b) --i;
    while (i < np - 1 && first(i + 1) <= b) ++i;
    p = i;
    j = 2 * i + (b - first(i));
}

template <int NST, bool LIVE>
__device__ __forceinline__ void kloop_wide(float *lds, const float *const *src, const int *dst, int64_t kb, int64_t ke,
                                           const int *aoff, const int *boff, f32x16 (&c0)[2][2],
                                           f32x16 (&c1)[2][2]) {
    using L = Layout<32, 16>;
    constexpr int G = WideStage::PW;
    static_assert(G == 3, "the DMA placement below is written for 3 pieces per wave");
    const int64_t nk = (ke - kb) / 16;
    auto issue_part = [&](int64_t t, int q) {
        const int64_t k0 = kb + (t < nk ? t : nk - 1) * 16;
        dma16(src[q] + k0, lds + (int)(t % NST) * WideStage::F + dst[q]);
    };
    if (nk <= 0) return;
#pragma unroll
    for (int t = 0; t < NST - 1; ++t)
#pragma unroll
        for (int q = 0; q < G; ++q) issue_part(t, q);
    for (int64_t t = 0; t < nk; ++t) {
        wait_vm<(NST - 2) * G>();
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        if constexpr (!LIVE) {
#pragma unroll
            for (int q = 0; q < G; ++q) issue_part(t + NST - 1, q);
        } else {
            const float *As = lds + (int)(t % NST) * WideStage::F;
            const char *pa = reinterpret_cast<const char *>(As);
            const char *pb = reinterpret_cast<const char *>(As + WideStage::FA);
            f32x4v ra[2][2], rb[2][2];
#pragma unroll
            for (int x = 0; x < 2; ++x)
#pragma unroll
                for (int g = 0; g < 2; ++g) {
                    ra[x][g] = *reinterpret_cast<const f32x4v *>(pa + aoff[g] * 4 + x * L::XSTRIDE);
                    rb[x][g] = *reinterpret_cast<const f32x4v *>(pb + boff[g] * 4 + x * L::XSTRIDE);
                }
            split_ktile(ra, rb, c0, c1, [&](int q) { if (q < G) issue_part(t + NST - 1, q); });
        }
    }
}

template <int NST>
__device__ __forceinline__ Quarter item_compute_wide(const DenseArgs &a, float *lds, int64_t item, int64_t kb,
                                                     int64_t ke, int wave, int lane, f32x16 (&c)[2][2]) {
    using L = Layout<32, 16>;
    const int wm = wave >> 1, wn = wave & 1;
    int64_t p, j;
    item_coords(item, a.nt, p, j);
    const int64_t m0 = 2 * p * kTile, n0 = j * kTile;
    // piece P = wave PW + i of the stage: P < 16 the A image's (rows m0 ..), else the B image's (rows n0 ..)
    constexpr int PA = WideStage::FA / 256;
    const float *src[WideStage::PW];
    int dst[WideStage::PW];
#pragma unroll
    for (int i = 0; i < WideStage::PW; ++i) {
        const int P = wave * WideStage::PW + i;
        const bool isA = P < PA;
        const int pc = (isA ? P : P - PA) * 64 + lane;
        const int row = pc / L::C, kc = (pc % L::C) ^ L::swz(row);
        int64_t r = (isA ? m0 : n0) + row;
        r = r < a.n ? r : a.n - 1;
        src[i] = a.A + r * a.lda + 4 * kc;
        dst[i] = isA ? P * 256 : WideStage::FA + (P - PA) * 256;
    }
    int aoff[2], boff[2];
#pragma unroll
    for (int g = 0; g < 2; ++g) {
        aoff[g] = L::off(wm * 64, 0, g, lane);
        boff[g] = L::off(wn * 64, 0, g, lane);
    }
    const int64_t R = m0 + wm * 64, Cc = n0 + wn * 64;
    Quarter q{R, Cc, R == Cc, R > Cc};
    const bool live = !q.below && R < a.n && Cc < a.n;
    f32x16 c0[2][2], c1[2][2];
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
        for (int y = 0; y < 2; ++y) {
            c0[x][y] = f32x16{};
            c1[x][y] = f32x16{};
        }
    if (live) kloop_wide<NST, true>(lds, src, dst, kb, ke, aoff, boff, c0, c1);
    else kloop_wide<NST, false>(lds, src, dst, kb, ke, aoff, boff, c0, c1);
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
        for (int y = 0; y < 2; ++y) c[x][y] = c0[x][y] + c1[x][y];
    return q;
}

// The wide kernels' schedule.  Slot s of the grid G (one workgroup per CU) takes whole items in rounds -- round r's
// item r G + s -- then an equal share of the k-tile units of the items left, stream-K (split items summed in piece
// order by the last piece, as gram_split_sk_kernel over the tiles).  With xcd_slots the slots are numbered
// XCD-contiguously: workgroups are dealt round-robin over the 8 XCDs, so slot = (b mod 8) (G / 8) + b / 8 gives
// the 32 CUs of one XCD 32 consecutive items of a round -- mostly one row pair against consecutive column blocks --
// which start together and run the same k-loop, so each k-tile of the shared A rows comes from HBM once per XCD and
// hits that XCD's L2 for the other CUs (the items of a round also share their B column blocks across XCDs, in the
// Infinity Cache).  item(it, kb, ke, c) computes k range [kb, ke) of item `it` into c and returns its Quarter.
template <class ItemFn>
__device__ __forceinline__ void wide_schedule(const DenseArgs &a, int32_t *lds_scratch, int wave, int lane,
                                              ItemFn &&item_fn) {
    const int64_t G = gridDim.x, b = blockIdx.x;
    const int64_t slot = a.xcd_slots ? (b & 7) * (G >> 3) + (b >> 3) : b;
    const int64_t KT = a.sk_kt;
    for (int64_t r = 0; r < a.dp_rounds; ++r) {
        __syncthreads();
        f32x16 c[2][2];
        const Quarter q = item_fn(r * G + slot, (int64_t)0, KT * 16, c);
        if (!q.below && q.qr < a.n && q.qc < a.n) write_quarter<32, 16>(a, c, q.qr, q.qc, q.diag, false, lane);
    }
    const int64_t U = a.sk_units, base = a.dp_rounds * G * KT;
    const int64_t u0 = base + slot * U;
    const int64_t u1 = u0 + U < a.sk_total ? u0 + U : a.sk_total;
    for (int64_t u = u0; u < u1;) {
        const int64_t item = u / KT, tb = item * KT, te = tb + KT;
        const int64_t se = u1 < te ? u1 : te;
        __syncthreads();
        f32x16 c[2][2];
        const Quarter q = item_fn(item, (u - tb) * 16, (se - tb) * 16, c);
        bool write = true;
        if (u != tb || se != te) {
            const int64_t s0 = (tb - base) / U, s1 = (te - 1 - base) / U;
            const int64_t first = 2 * s0 + (tb - base == s0 * U ? 0 : 1);
            write = split_combine<32, 16, 8>(
                a, c, a.tickets + first, s1 - s0 + 1, slot - s0,
                [&](int64_t j) { return j == 0 ? first : 2 * (s0 + j); }, lds_scratch, wave, lane);
        }
        if (write && !q.below && q.qr < a.n && q.qc < a.n)
            write_quarter<32, 16>(a, c, q.qr, q.qc, q.diag, false, lane);
        u = se;
    }
}

template <int NST>
__global__ __launch_bounds__(512, 1) void gram_split_wide_kernel(DenseArgs a) {
    __shared__ __attribute__((aligned(16))) float lds[NST * WideStage::F];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    wide_schedule(a, reinterpret_cast<int32_t *>(lds), wave, lane,
                  [&](int64_t item, int64_t kb, int64_t ke, f32x16 (&c)[2][2]) {
                      return item_compute_wide<NST>(a, lds, item, kb, ke, wave, lane, c);
                  });
}

// ------------------------------------------------------------ the planes split once, by the producer
// The wide split kernel above splits every staged k-tile again in registers (184 VALU per wave and k-tile,
// ~2 ceil(n / 128) times per element).  Here A's three bf16 planes are written once (grf_split_planes, or the
// dense front's grf_densify_padded_planes) and staged as they are: the k-loop issues fragment reads and MFMAs
// only.  The planes are the in-register split's (the same cvt_pk / remainder sequence per element) and the
// MFMAs run in the same order per block, so K is bit-identical to gram_split_wide_kernel's.
// Plane layout P: row r, k-tile t (16 k) is 96 B at r ldp + 96 t: plane 0 of k = 16 t .. 16 t + 15 (bf16, k
// order), then plane 1, then plane 2 -- six 16-B chunks c = 2 p + h (h: the k half a lane's MFMA operand takes).
constexpr int kPlaneBytes = 96;  // one row's k-tile (3 planes x 16 bf16)

__device__ __forceinline__ void split_chunk(f32x4v lo, f32x4v hi, u32x4 &p0, u32x4 &p1, u32x4 &p2) {
    plane0(lo, hi, p0);
    next_plane2<0>(lo, hi, p0, p1);
    next_plane2<2>(lo, hi, p0, p1);
    next_plane2<0>(lo, hi, p1, p2);
    next_plane2<2>(lo, hi, p1, p2);
}

// one thread per (row, k-tile, half): 8 floats -> three 16-B plane chunks
__global__ __launch_bounds__(256) void split_planes_kernel(int64_t n, int64_t kt, const float *__restrict__ A,
                                                           int64_t lda, unsigned char *__restrict__ P, int64_t ldp) {
    const int64_t u = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (u >= n * kt * 2) return;
    const int64_t r = u / (kt * 2), rem = u - r * kt * 2, t = rem >> 1, h = rem & 1;
    const f32x4v *src = reinterpret_cast<const f32x4v *>(A + r * lda + 16 * t + 8 * h);
    u32x4 p0, p1, p2;
    split_chunk(src[0], src[1], p0, p1, p2);
    u32x4 *dst = reinterpret_cast<u32x4 *>(P + r * ldp + kPlaneBytes * t + 16 * h);
    dst[0] = p0;
    dst[2] = p1;
    dst[4] = p2;
}

// the dense front's producer: the walk's padded rows straight to the planes (densify_padded_kernel's LDS
// row, then the split of every 8-float chunk)
__global__ __launch_bounds__(256) void densify_padded_planes_kernel(int64_t cap, const int32_t *__restrict__ cnt,
                                                                    const int32_t *__restrict__ idx,
                                                                    const float *__restrict__ val, int64_t kt,
                                                                    unsigned char *__restrict__ P, int64_t ldp) {
    extern __shared__ __attribute__((aligned(16))) float prow[];  // [16 kt]
    const int64_t r = blockIdx.x;
    const int tid = threadIdx.x;
    const int q4 = (int)(4 * kt);
    for (int t = tid; t < q4; t += 256) reinterpret_cast<float4 *>(prow)[t] = float4{0.f, 0.f, 0.f, 0.f};
    __syncthreads();
    const int64_t b = r * cap;
    const int c = cnt[r];
    for (int e = tid; e < c; e += 256) prow[idx[b + e]] = val[b + e];
    __syncthreads();
    for (int u = tid; u < (int)(2 * kt); u += 256) {
        const f32x4v *src = reinterpret_cast<const f32x4v *>(prow + 8 * u);
        u32x4 p0, p1, p2;
        split_chunk(src[0], src[1], p0, p1, p2);
        u32x4 *dst = reinterpret_cast<u32x4 *>(P + r * ldp + kPlaneBytes * (u >> 1) + 16 * (u & 1));
        dst[0] = p0;
        dst[2] = p1;
        dst[4] = p2;
    }
}

// The wide items (256 x 128, 8 waves, stream-K) on the planes.  A stage is 256 + 128 rows of 96 B (36 KiB; 4
// stages = 144 KiB, one workgroup per CU as the fp32-staged wide kernel): 36 1-KiB DMA pieces, piece P of wave w
// for P = w + 8 i (i < 5; the four waves past piece 35 re-issue their first, the same bytes to the same place,
// so every wave's in-flight count is 5 per k-tile).  LDS row image: row R's chunk c at R 96 + 16 (c ^ ((R >> 3)
// & 1)) -- rows 8 apart differ in 96 B = 24 banks, so the swap of the halves of every 8th row's planes makes the
// 16 rows of a ds_read_b128 phase hit 16 distinct 4-bank groups.
struct PlaneStage {
    static constexpr int RA = 2 * kTile, RB = kTile;
    static constexpr int BA = RA * kPlaneBytes, BB = RB * kPlaneBytes, B = BA + BB;  // bytes
    static constexpr int NP = B / 1024, G = (NP + 7) / 8;  // pieces per stage, per wave
};
static_assert(PlaneStage::B % 1024 == 0, "whole pieces");
__device__ __forceinline__ uint32_t plane_lds_off(int row, int c) { return (uint32_t)(row * kPlaneBytes + 16 * (c ^ ((row >> 3) & 1))); }

__device__ __forceinline__ void dma16b(const unsigned char *src, unsigned char *lds_piece) {
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)src,
                                     (__attribute__((address_space(3))) void *)lds_piece, 16, 0, 0);
}

// one k-tile of a wave's 2 x 2 blocks from staged planes: a[x][p] / b[y][q] read from LDS, the six products
// per block in split_ktile's order (c0: a0 b0; c1: (0,1) (1,0) (0,2) (1,1) (2,0)), the DMA pieces between
// (a lane's chunk of block x, plane p sits at base + 32 rows x 96 B x + 32 p: rows 32 apart keep the swap bit,
// ((row >> 3) & 1) = ((lane >> 3) & 1), so one base per operand and immediate offsets address all six)
template <bool SIX = false, typename Issue>
__device__ __forceinline__ void planes_ktile(const unsigned char *As, const unsigned char *Bs, uint32_t abase,
                                             uint32_t bbase, f32x16 (&c0)[2][2], f32x16 (&c1)[2][2], Issue issue) {
    u32x4 a[2][3], b[2][3];
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
        for (int p = 0; p < 3; ++p) {
            a[x][p] = *reinterpret_cast<const u32x4 *>(As + abase + 32 * kPlaneBytes * x + 32 * p);
            b[x][p] = *reinterpret_cast<const u32x4 *>(Bs + bbase + 32 * kPlaneBytes * x + 32 * p);
        }
    auto mf = [&](int x, int y, int s) {
        if (s == 0) {
            c0[x][y] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a[x][0]),
                                                             __builtin_bit_cast(bf16x8, b[y][0]), c0[x][y], 0, 0, 0);
            return;
        }
        constexpr int PQ[6][2] = {{0, 0}, {0, 1}, {1, 0}, {0, 2}, {1, 1}, {2, 0}};
        c1[x][y] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a[x][PQ[s][0]]),
                                                         __builtin_bit_cast(bf16x8, b[y][PQ[s][1]]), c1[x][y], 0, 0, 0);
    };
    auto fence = [] { __builtin_amdgcn_sched_barrier(0); };
    mf(0, 0, 0); mf(0, 1, 0); mf(1, 0, 0); mf(1, 1, 0); fence();
    mf(0, 0, 1); issue(0); fence();
    mf(0, 0, 2); mf(0, 1, 1); fence();
    mf(0, 1, 2); issue(1); fence();
    mf(1, 0, 1); mf(1, 0, 2); fence();
    mf(1, 1, 1); issue(2); fence();
    mf(1, 1, 2); mf(0, 0, 3); fence();
    mf(0, 0, 4); issue(3); fence();
    mf(0, 0, 5); mf(0, 1, 3); fence();
    mf(0, 1, 4); issue(4); fence();
    mf(0, 1, 5);
    if constexpr (SIX) {  // (the 128-tile kernel's sixth piece)
        issue(5);
        fence();
    }
    mf(1, 0, 3);
    mf(1, 0, 4);
    mf(1, 0, 5);
    mf(1, 1, 3);
    mf(1, 1, 4);
    mf(1, 1, 5);
}

template <int NST, bool LIVE>
__device__ __forceinline__ void kloop_planes(unsigned char *lds, const unsigned char *const *src, const uint32_t *dst,
                                             int64_t kb, int64_t ke, uint32_t abase, uint32_t bbase,
                                             f32x16 (&c0)[2][2], f32x16 (&c1)[2][2]) {
    constexpr int G = PlaneStage::G;
    const int64_t nk = (ke - kb) / 16;
    auto issue_part = [&](int64_t t, int q) {
        const int64_t kt0 = kb / 16 + (t < nk ? t : nk - 1);
        dma16b(src[q] + kPlaneBytes * kt0, lds + (int)(t % NST) * PlaneStage::B + dst[q]);
    };
    if (nk <= 0) return;
#pragma unroll
    for (int t = 0; t < NST - 1; ++t)
#pragma unroll
        for (int q = 0; q < G; ++q) issue_part(t, q);
    for (int64_t t = 0; t < nk; ++t) {
        wait_vm<(NST - 2) * G>();
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        if constexpr (!LIVE) {
#pragma unroll
            for (int q = 0; q < G; ++q) issue_part(t + NST - 1, q);
        } else {
            const unsigned char *As = lds + (int)(t % NST) * PlaneStage::B;
            planes_ktile(As, As + PlaneStage::BA, abase, bbase, c0, c1,
                         [&](int q) { if (q < G) issue_part(t + NST - 1, q); });
        }
    }
}

template <int NST>
__device__ __forceinline__ Quarter item_compute_planes(const DenseArgs &a, const unsigned char *P, int64_t ldp,
                                                       unsigned char *lds, int64_t item, int64_t kb, int64_t ke,
                                                       int wave, int lane, f32x16 (&c)[2][2]) {
    const int wm = wave >> 1, wn = wave & 1;
    int64_t p, j;
    item_coords(item, a.nt, p, j);
    const int64_t m0 = 2 * p * kTile, n0 = j * kTile;
    const unsigned char *src[PlaneStage::G];
    uint32_t dst[PlaneStage::G];
#pragma unroll
    for (int i = 0; i < PlaneStage::G; ++i) {
        int Pc = wave + 8 * i;
        if (Pc >= PlaneStage::NP) Pc = wave;  // (the re-issued first piece)
        const uint32_t off = (uint32_t)Pc * 1024u + 16u * (uint32_t)lane;  // this lane's LDS bytes in the stage
        const bool isA = off < (uint32_t)PlaneStage::BA;
        const uint32_t o = isA ? off : off - PlaneStage::BA;
        const int R = (int)(o / kPlaneBytes), jj = (int)((o % kPlaneBytes) / 16);
        const int cc = jj ^ ((R >> 3) & 1);  // the global chunk that lands here
        int64_t r = (isA ? m0 : n0) + R;
        r = r < a.n ? r : a.n - 1;
        src[i] = P + r * ldp + 16 * cc;
        dst[i] = off;
    }
    const uint32_t abase = plane_lds_off(wm * 64 + (lane & 31), lane >> 5);
    const uint32_t bbase = plane_lds_off(wn * 64 + (lane & 31), lane >> 5);
    const int64_t R = m0 + wm * 64, Cc = n0 + wn * 64;
    Quarter q{R, Cc, R == Cc, R > Cc};
    const bool live = !q.below && R < a.n && Cc < a.n;
    f32x16 c0[2][2], c1[2][2];
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
        for (int y = 0; y < 2; ++y) {
            c0[x][y] = f32x16{};
            c1[x][y] = f32x16{};
        }
    if (live) kloop_planes<NST, true>(lds, src, dst, kb, ke, abase, bbase, c0, c1);
    else kloop_planes<NST, false>(lds, src, dst, kb, ke, abase, bbase, c0, c1);
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
        for (int y = 0; y < 2; ++y) c[x][y] = c0[x][y] + c1[x][y];
    return q;
}

template <int NST>
__global__ __launch_bounds__(512, 1) void gram_planes_wide_kernel(DenseArgs a, const unsigned char *P, int64_t ldp) {
    __shared__ __attribute__((aligned(16))) unsigned char lds[NST * PlaneStage::B];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    wide_schedule(a, reinterpret_cast<int32_t *>(lds), wave, lane,
                  [&](int64_t item, int64_t kb, int64_t ke, f32x16 (&c)[2][2]) {
                      return item_compute_planes<NST>(a, P, ldp, lds, item, kb, ke, wave, lane, c);
                  });
}

// The 128-tile kernel on the planes (n <= 8064, where the wide items leave CUs idle): the in-register split
// kernel's work items (gram_split_mfma_kernel: tiles cut into k-slices, pieces summed by the last) with stages of
// 128 + 128 rows of 96 B (24 KiB; 3 stages = 72 KiB, two workgroups per CU), 24 1-KiB DMA pieces per k-tile, piece
// P of wave w for P = w + 4 i (i < 6; a diagonal tile stages A alone: 12 pieces, 3 per wave), the fragment reads
// and MFMAs of planes_ktile.  Same products in the same order as the in-register kernel: the same K bits.
struct PlaneTileStage {
    static constexpr int BA = kTile * kPlaneBytes, B = 2 * BA;  // bytes: the A image, then the B image
    static constexpr int G = B / 1024 / 4, GD = BA / 1024 / 4;  // pieces per wave and k-tile (off / on the diagonal)
};
static_assert(PlaneTileStage::BA % 4096 == 0 && PlaneTileStage::G == 6, "whole pieces, six per wave");
constexpr int kPlaneTileNST = 3;

template <int NST, bool DIAG, bool LIVE>
__device__ __forceinline__ void kloop_planes_tile(unsigned char *lds, const unsigned char *const *src,
                                                  const uint32_t *dst, int64_t kb, int64_t ke, uint32_t abase,
                                                  uint32_t bbase, f32x16 (&c0)[2][2], f32x16 (&c1)[2][2]) {
    constexpr int G = DIAG ? PlaneTileStage::GD : PlaneTileStage::G;
    const int64_t nk = (ke - kb) / 16;
    auto issue_part = [&](int64_t t, int q) {
        const int64_t kt0 = kb / 16 + (t < nk ? t : nk - 1);
        dma16b(src[q] + kPlaneBytes * kt0, lds + (int)(t % NST) * PlaneTileStage::B + dst[q]);
    };
    if (nk <= 0) return;
#pragma unroll
    for (int t = 0; t < NST - 1; ++t)
#pragma unroll
        for (int q = 0; q < G; ++q) issue_part(t, q);
    for (int64_t t = 0; t < nk; ++t) {
        wait_vm<(NST - 2) * G>();
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        if constexpr (!LIVE) {
#pragma unroll
            for (int q = 0; q < G; ++q) issue_part(t + NST - 1, q);
        } else {
            const unsigned char *As = lds + (int)(t % NST) * PlaneTileStage::B;
            const unsigned char *Bs = DIAG ? As : As + PlaneTileStage::BA;
            planes_ktile<true>(As, Bs, abase, bbase, c0, c1, [&](int q) { if (q < G) issue_part(t + NST - 1, q); });
        }
    }
}

__device__ __forceinline__ Quarter tile_compute_planes(const DenseArgs &a, const unsigned char *P, int64_t ldp,
                                                       unsigned char *lds, int64_t tile, int64_t kb, int64_t ke,
                                                       int wave, int lane, f32x16 (&c)[2][2]) {
    const int wm = wave >> 1, wn = wave & 1;
    int64_t bi, bj;
    tile_coords(tile, a.nt, bi, bj);
    const int64_t m0 = bi * kTile, n0 = bj * kTile;
    const bool diag = bi == bj;
    const unsigned char *src[PlaneTileStage::G];
    uint32_t dst[PlaneTileStage::G];
#pragma unroll
    for (int i = 0; i < PlaneTileStage::G; ++i) {
        const uint32_t off = (uint32_t)(wave + 4 * i) * 1024u + 16u * (uint32_t)lane;  // this lane's stage bytes
        const bool isA = off < (uint32_t)PlaneTileStage::BA;
        const uint32_t o = isA ? off : off - PlaneTileStage::BA;
        const int R = (int)(o / kPlaneBytes), jj = (int)((o % kPlaneBytes) / 16);
        const int cc = jj ^ ((R >> 3) & 1);  // the global chunk that lands here
        int64_t r = (isA ? m0 : n0) + R;
        r = r < a.n ? r : a.n - 1;
        src[i] = P + r * ldp + 16 * cc;
        dst[i] = off;
    }
    const uint32_t abase = plane_lds_off(wm * 64 + (lane & 31), lane >> 5);
    const uint32_t bbase = plane_lds_off(wn * 64 + (lane & 31), lane >> 5);
    Quarter q{m0 + wm * 64, n0 + wn * 64, diag, diag && wn < wm};
    const bool live = !q.below && q.qr < a.n && q.qc < a.n;
    f32x16 c0[2][2], c1[2][2];
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
        for (int y = 0; y < 2; ++y) {
            c0[x][y] = f32x16{};
            c1[x][y] = f32x16{};
        }
    constexpr int NST = kPlaneTileNST;
    if (diag) {
        if (live) kloop_planes_tile<NST, true, true>(lds, src, dst, kb, ke, abase, bbase, c0, c1);
        else kloop_planes_tile<NST, true, false>(lds, src, dst, kb, ke, abase, bbase, c0, c1);
    } else {
        if (live) kloop_planes_tile<NST, false, true>(lds, src, dst, kb, ke, abase, bbase, c0, c1);
        else kloop_planes_tile<NST, false, false>(lds, src, dst, kb, ke, abase, bbase, c0, c1);
    }
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
        for (int y = 0; y < 2; ++y) c[x][y] = c0[x][y] + c1[x][y];
    return q;
}

__global__ __launch_bounds__(256, 2) void gram_planes_tile_kernel(DenseArgs a, const unsigned char *P, int64_t ldp) {
    __shared__ __attribute__((aligned(16))) unsigned char lds[kPlaneTileNST * PlaneTileStage::B];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const int64_t w = blockIdx.x;
    int64_t tile, slice = 0, pieces = 1;
    if (w < a.n_whole) {
        tile = w;
    } else {
        tile = a.n_whole + (w - a.n_whole) / a.n_split;
        slice = (w - a.n_whole) % a.n_split;
        pieces = a.n_split;
    }
    const int64_t kb = pieces > 1 ? slice * a.k_split : 0;
    const int64_t ke = pieces > 1 ? (kb + a.k_split < a.kpad ? kb + a.k_split : a.kpad) : a.kpad;
    f32x16 c[2][2];
    const Quarter q = tile_compute_planes(a, P, ldp, lds, tile, kb, ke, wave, lane, c);
    if (pieces > 1) {
        const int64_t u = tile - a.n_whole;
        if (!split_combine<32, 16>(a, c, a.tickets + u, pieces, slice, [&](int64_t s) { return u * pieces + s; },
                                   reinterpret_cast<int32_t *>(lds), wave, lane))
            return;
    }
    tile_write<32, 16>(a, c, q, wave, lane);
}

constexpr int kCUs = 256;

int env_int(const char *name, int dflt) {
    const char *e = getenv(name);
    return e ? atoi(e) : dflt;
}

// Workspace layout, the same for every (n, k): kMaxSplitTiles tickets at a fixed place, then the slabs.
// A ticket is zero between launches (the last arriver resets it) and slabs never overlap the ticket
// block, so one workspace, zeroed once, serves calls of any size in any order on its stream.
constexpr int64_t kMaxSplitTiles = 1024;  // (tiles < 512 when all split; the tail is < 1024)
constexpr size_t kTicketBytes = kMaxSplitTiles * sizeof(int32_t);

struct DensePlan {
    int64_t nt, tiles, n_whole, k_split, kpad;
    int32_t n_split;
    size_t ws_bytes;  // tickets + slabs
};

// Work plan: whole tiles, and split pieces where whole tiles would leave CUs idle -- every tile split
// when the tiles alone do not fill the GPU (small n), else the last `tail` tiles.
// A/B knobs (read once): GRF_DENSE_SPLIT (pieces per split tile), GRF_DENSE_TAIL (split tiles at the end)
DensePlan dense_plan(int64_t n, int64_t k_dim, int bk) {
    DensePlan p{};
    p.nt = cdiv<int64_t>(n, kTile);
    p.tiles = p.nt * (p.nt + 1) / 2;
    p.kpad = cdiv<int64_t>(k_dim, bk) * bk;
    static const int env_split = env_int("GRF_DENSE_SPLIT", -1);
    static const int env_tail = env_int("GRF_DENSE_TAIL", -1);
    constexpr int64_t slots = 2 * kCUs;  // workgroups resident at once (2 per CU: 64 KiB of LDS ring each)
    int64_t split = 1, tail = 0;
    if (p.tiles < slots) {  // small n: every tile split, ~2 pieces per CU slot
        split = std::max<int64_t>(1, std::min<int64_t>(4, slots / std::max<int64_t>(p.tiles, 1)));
        tail = p.tiles;
    } else if (p.tiles % slots != 0) {
        // large n: the last round of whole tiles would leave (slots - tiles % slots) slots idle; the
        // last slots + tiles % slots tiles go in thirds instead, so the final rounds are cut 3x finer
        split = 3;
        tail = std::min<int64_t>(p.tiles, slots + p.tiles % slots);
    }
    if (env_split >= 1) split = env_split;
    if (env_tail >= 0) tail = std::min<int64_t>(env_tail, p.tiles);
    tail = std::min<int64_t>(tail, kMaxSplitTiles);
    const int64_t ktiles = p.kpad / bk;
    split = std::max<int64_t>(1, std::min<int64_t>(split, ktiles));
    if (split == 1) tail = 0;
    p.n_split = (int32_t)split;
    p.n_whole = p.tiles - tail;
    p.k_split = cdiv<int64_t>(ktiles, split) * bk;
    if (tail > 0) p.n_split = (int32_t)cdiv<int64_t>(p.kpad, p.k_split);  // (no empty piece)
    if (p.n_split <= 1) {
        p.n_split = 1;
        p.n_whole = p.tiles;
    }
    const int64_t split_tiles = p.tiles - p.n_whole;
    p.ws_bytes = split_tiles > 0 ? kTicketBytes + (size_t)split_tiles * p.n_split * kTile * kTile * sizeof(float) : 0;
    return p;
}

// Stream-K plan (GRF_DENSE_SK=1): slots = 2 workgroups per CU, U k-tile units each.
struct SkPlan {
    int64_t kt, total, units, grid;
    size_t ws_bytes;
    int64_t dp_rounds;  // (wide plan) whole-item rounds before the stream-K units
    int32_t xcd_slots;  // (wide plan) XCD-contiguous slot numbering
};
SkPlan sk_plan(int64_t n, int64_t k_dim, int bk) {
    SkPlan p{};
    const int64_t nt = cdiv<int64_t>(n, kTile);
    p.kt = cdiv<int64_t>(k_dim, bk);
    p.total = nt * (nt + 1) / 2 * p.kt;
    const int64_t slots = std::min<int64_t>(2 * kCUs, std::max<int64_t>(p.total, 1));
    p.units = std::max<int64_t>(1, cdiv<int64_t>(p.total, slots));
    p.grid = cdiv<int64_t>(p.total, p.units);
    p.ws_bytes = kTicketBytes + (size_t)(2 * p.grid) * kTile * kTile * sizeof(float);
    return p;
}

// The wide kernels' plan: one 8-wave workgroup per CU, items of 256 x 128, slabs of 128 KiB.  From two items per
// slot on, whole-item rounds in XCD-contiguous slot order (wide_schedule) and stream-K over the rest; a rest below
// G / 4 items would cut each of its items into more than 4 pieces, so one round joins it.  GRF_DENSE_XCD=0 (read
// per call, A/B): stream-K over every item, slots in launch order (round 5's schedule).
SkPlan sk_plan_wide(int64_t n, int64_t k_dim) {
    SkPlan p{};
    const int64_t nt = cdiv<int64_t>(n, kTile), np = (nt + 1) / 2;
    const int64_t items = np * (nt + 1) - np * np;
    p.kt = cdiv<int64_t>(k_dim, 16);
    p.total = items * p.kt;
    const bool xcd = env_int("GRF_DENSE_XCD", 1) != 0;
    if (xcd && items >= 2 * kCUs) {
        p.grid = kCUs;
        p.dp_rounds = items / p.grid;
        const int64_t rest = items - p.dp_rounds * p.grid;
        if (rest > 0 && rest < p.grid / 4) --p.dp_rounds;
        p.units = std::max<int64_t>(1, cdiv<int64_t>(p.total - p.dp_rounds * p.grid * p.kt, p.grid));
        p.xcd_slots = 1;
    } else {
        const int64_t slots = std::min<int64_t>(kCUs, std::max<int64_t>(p.total, 1));
        p.units = std::max<int64_t>(1, cdiv<int64_t>(p.total, slots));
        p.grid = cdiv<int64_t>(p.total, p.units);
    }
    p.ws_bytes = kTicketBytes + (size_t)(2 * p.grid) * 2 * kTile * kTile * sizeof(float);
    return p;
}

}  // namespace

size_t dense_gram_workspace_bytes(int64_t n, int64_t k_dim) {
    if (n <= 0) return 16;
    const DensePlan p = dense_plan(n, k_dim, 16);
    return std::max<size_t>(16, std::max(p.ws_bytes, sk_plan(n, k_dim, 16).ws_bytes));
}

int32_t dense_gram(int64_t n, int64_t k_dim, const float *A, int64_t lda, float *K, int64_t ldk, void *workspace,
                   size_t workspace_bytes, bool upper_only, grf_stream_t stream) {
    GRF_REQUIRE(n >= 0 && k_dim >= 0 && A && K && ldk >= n && lda >= k_dim, GRF_EINVAL,
                "grf_gram_dense: bad arguments");
    GRF_REQUIRE(lda % 16 == 0 && ((uintptr_t)A & 15) == 0, GRF_EINVAL,
                "grf_gram_dense: lda must be a multiple of 16 and A 16-byte aligned");
    GRF_REQUIRE(upper_only || (ldk % 4 == 0 && ((uintptr_t)K & 15) == 0), GRF_EINVAL,
                "grf_gram_dense: ldk must be a multiple of 4 and K 16-byte aligned");
    if (n == 0) return GRF_OK;
    constexpr int BK = 16;
    DensePlan p = dense_plan(n, k_dim, BK);
    GRF_REQUIRE(p.kpad <= lda, GRF_EINVAL, "grf_gram_dense: lda must cover k_dim rounded up to %d", BK);
    DenseArgs a{};
    a.A = A;
    a.K = K;
    a.n = n;
    a.nt = p.nt;
    a.lda = lda;
    a.ldk = ldk;
    a.kpad = p.kpad;
    a.upper_only = upper_only ? 1 : 0;
    hipStream_t st = S(stream);
    // stream-K when the tiles fill at least half the slots (every slot then takes >= half a tile of k, so a
    // split tile has <= 3 pieces): n = 4096 0.68 -> 0.78, C2 0.83 -> 0.86 of the MFMA peak; at C3 (253 tiles)
    // even, below it the per-tile splits win (profiles/r04_dense_ab.txt).  GRF_DENSE_SK: 0 never, 1 always.
    static const int sk_env = env_int("GRF_DENSE_SK", -1);
    const bool sk = sk_env == 1 || (sk_env != 0 && p.tiles >= kCUs);
    if (sk) {
        const SkPlan q = sk_plan(n, k_dim, BK);
        if (workspace && workspace_bytes >= q.ws_bytes && ((uintptr_t)workspace & 255) == 0) {
            GRF_REQUIRE_GRID(q.grid, 256, "gram_dense_sk_kernel");
            a.tickets = reinterpret_cast<int32_t *>(workspace);
            a.slabs = reinterpret_cast<float *>(reinterpret_cast<char *>(workspace) + kTicketBytes);
            a.sk_units = q.units;
            a.sk_kt = q.kt;
            a.sk_total = q.total;
            gram_dense_sk_kernel<32, BK, 4, 2><<<(unsigned)q.grid, 256, 0, st>>>(a);
            GRF_CHECK_LAUNCH("gram_dense_sk_kernel");
            return GRF_OK;
        }
    }
    if (p.ws_bytes > 0 && (!workspace || workspace_bytes < p.ws_bytes || ((uintptr_t)workspace & 255))) {
        // no (or too small) workspace: whole tiles only
        p.n_split = 1;
        p.n_whole = p.tiles;
        p.ws_bytes = 0;
    }
    const int64_t split_tiles = p.tiles - p.n_whole;
    const int64_t items = p.n_whole + split_tiles * p.n_split;
    GRF_REQUIRE_GRID(items, 256, "gram_dense_mfma_kernel");
    a.tickets = split_tiles > 0 ? reinterpret_cast<int32_t *>(workspace) : nullptr;
    a.slabs = split_tiles > 0 ? reinterpret_cast<float *>(reinterpret_cast<char *>(workspace) + kTicketBytes) : nullptr;
    a.n_whole = p.n_whole;
    a.k_split = p.k_split;
    a.n_split = p.n_split;
    // the hub panel (upper_only, k of a few k-tiles): each tile is a short k-loop then a 64 KB write, so a
    // third workgroup per CU (3-stage ring, 48 KB) overlaps one tile's stores with the others' MFMAs: Enron's
    // panel 1.67 -> 1.49 ms, step 7.84-7.87 -> 7.62-7.71 ms (profiles/r04_hub_ring_ab.txt).
    // GRF_DENSE_HUB_NST: 3 (default) or 4 (the ring of the other launches).
    static const int hub_nst = env_int("GRF_DENSE_HUB_NST", 3);
    if (upper_only && split_tiles == 0 && hub_nst == 3) {
        gram_dense_mfma_kernel<32, BK, 3, 3><<<(unsigned)items, 256, 0, st>>>(a);
        GRF_CHECK_LAUNCH("gram_dense_mfma_kernel");
        return GRF_OK;
    }
    gram_dense_mfma_kernel<32, BK, 4, 2><<<(unsigned)items, 256, 0, st>>>(a);
    GRF_CHECK_LAUNCH("gram_dense_mfma_kernel");
    return GRF_OK;
}


// The split path: the fp32 path's workspace (tickets and slabs; the ticket block must be zero on first use)
size_t dense_gram_split_workspace_bytes(int64_t n, int64_t k_dim) {
    const size_t base = dense_gram_workspace_bytes(n, k_dim);
    return n <= 0 ? base : std::max(base, sk_plan_wide(n, k_dim).ws_bytes);
}

// workspace NULL (the hub panel's upper_only call): whole tiles only, as dense_gram without one
int32_t dense_gram_split(int64_t n, int64_t k_dim, const float *A, int64_t lda, float *K, int64_t ldk,
                         void *workspace, size_t workspace_bytes, bool upper_only, grf_stream_t stream) {
    GRF_REQUIRE(n >= 0 && k_dim >= 0 && A && K && ldk >= n && lda >= k_dim, GRF_EINVAL,
                "grf_gram_dense_split: bad arguments");
    GRF_REQUIRE(lda % 16 == 0 && ((uintptr_t)A & 15) == 0, GRF_EINVAL,
                "grf_gram_dense_split: lda must be a multiple of 16 and A 16-byte aligned");
    GRF_REQUIRE(upper_only || (ldk % 4 == 0 && ((uintptr_t)K & 15) == 0), GRF_EINVAL,
                "grf_gram_dense_split: ldk must be a multiple of 4 and K 16-byte aligned");
    if (n == 0) return GRF_OK;
    GRF_REQUIRE(!workspace || (((uintptr_t)workspace & 255) == 0 &&
                               workspace_bytes >= dense_gram_split_workspace_bytes(n, k_dim)),
                GRF_EINVAL, "grf_gram_dense_split: workspace too small or not 256-byte aligned");
    constexpr int BK = 16;
    DensePlan p = dense_plan(n, k_dim, BK);
    GRF_REQUIRE(p.kpad <= lda, GRF_EINVAL, "grf_gram_dense_split: lda must cover k_dim rounded up to %d", BK);
    hipStream_t st = S(stream);
    DenseArgs a{};
    a.A = A;
    a.K = K;
    a.n = n;
    a.nt = p.nt;
    a.lda = lda;
    a.ldk = ldk;
    a.kpad = p.kpad;
    a.upper_only = upper_only ? 1 : 0;
    // the wide workgroups (256 x 128 items) from 64 tile rows on (n > 8064): C2 (n = 10 000) 5.60 -> 5.12 ms,
    // n = 16384 24.5 -> 22.7; equal at n = 6144, slower at C3 (0.148 -> 0.164: 132 items on 256 CUs, every one
    // cut) -- profiles/r05_split_gram_ab.txt.  GRF_DENSE_WIDE (read per call, for A/B and tests): 0 never,
    // 1 always, unset / -1 by that rule.
    const int wide_env = env_int("GRF_DENSE_WIDE", -1);
    const bool wide = wide_env == 1 || (wide_env != 0 && p.nt >= 64);
    if (wide && workspace && !upper_only && p.kpad > 0) {
        const SkPlan q = sk_plan_wide(n, k_dim);
        GRF_REQUIRE_GRID(q.grid, 512, "gram_split_wide_kernel");
        a.tickets = reinterpret_cast<int32_t *>(workspace);
        a.slabs = reinterpret_cast<float *>(reinterpret_cast<char *>(workspace) + kTicketBytes);
        a.sk_units = q.units;
        a.sk_kt = q.kt;
        a.sk_total = q.total;
        a.dp_rounds = q.dp_rounds;
        a.xcd_slots = q.xcd_slots;
        gram_split_wide_kernel<kSplitNST><<<(unsigned)q.grid, 512, 0, st>>>(a);
        GRF_CHECK_LAUNCH("gram_split_wide_kernel");
        return GRF_OK;
    }
    static const int sk_env = env_int("GRF_DENSE_SK", -1);
    const bool sk = workspace && (sk_env == 1 || (sk_env != 0 && p.tiles >= kCUs));
    if (!workspace) {
        p.n_split = 1;
        p.n_whole = p.tiles;
    }
    if (sk) {
        const SkPlan q = sk_plan(n, k_dim, BK);
        GRF_REQUIRE_GRID(q.grid, 256, "gram_split_sk_kernel");
        a.tickets = reinterpret_cast<int32_t *>(workspace);
        a.slabs = reinterpret_cast<float *>(reinterpret_cast<char *>(workspace) + kTicketBytes);
        a.sk_units = q.units;
        a.sk_kt = q.kt;
        a.sk_total = q.total;
        gram_split_sk_kernel<<<(unsigned)q.grid, 256, 0, st>>>(a);
        GRF_CHECK_LAUNCH("gram_split_sk_kernel");
        return GRF_OK;
    }
    const int64_t split_tiles = p.tiles - p.n_whole;
    const int64_t items = p.n_whole + split_tiles * p.n_split;
    GRF_REQUIRE_GRID(items, 256, "gram_split_mfma_kernel");
    a.tickets = split_tiles > 0 ? reinterpret_cast<int32_t *>(workspace) : nullptr;
    a.slabs = split_tiles > 0 ? reinterpret_cast<float *>(reinterpret_cast<char *>(workspace) + kTicketBytes) : nullptr;
    a.n_whole = p.n_whole;
    a.k_split = p.k_split;
    a.n_split = p.n_split;
    gram_split_mfma_kernel<<<(unsigned)items, 256, 0, st>>>(a);
    GRF_CHECK_LAUNCH("gram_split_mfma_kernel");
    return GRF_OK;
}

// ---- the planes path
int64_t planes_row_bytes(int64_t k_dim) { return cdiv<int64_t>(k_dim, 16) * kPlaneBytes; }

int32_t split_planes(int64_t n, int64_t k_dim, const float *A, int64_t lda, void *P, int64_t ldp, grf_stream_t stream) {
    GRF_REQUIRE(n >= 0 && k_dim >= 0 && (n == 0 || (A && P)), GRF_EINVAL, "grf_split_planes: bad arguments");
    const int64_t kt = cdiv<int64_t>(k_dim, 16);
    GRF_REQUIRE(lda >= 16 * kt && lda % 4 == 0 && ((uintptr_t)A & 15) == 0, GRF_EINVAL,
                "grf_split_planes: lda must cover k_dim rounded up to 16 (zero-padded), A 16-byte aligned");
    GRF_REQUIRE(ldp >= kt * kPlaneBytes && ldp % 16 == 0 && ((uintptr_t)P & 15) == 0, GRF_EINVAL,
                "grf_split_planes: ldp must cover %lld bytes, a multiple of 16, P 16-byte aligned",
                (long long)(kt * kPlaneBytes));
    const int64_t work = n * kt * 2;
    if (work == 0) return GRF_OK;
    GRF_REQUIRE_GRID(cdiv<int64_t>(work, 256), 256, "split_planes_kernel");
    split_planes_kernel<<<(unsigned)cdiv<int64_t>(work, 256), 256, 0, S(stream)>>>(
        n, kt, A, lda, reinterpret_cast<unsigned char *>(P), ldp);
    GRF_CHECK_LAUNCH("split_planes_kernel");
    return GRF_OK;
}

int32_t densify_padded_planes(int64_t n_rows, int64_t cap, int64_t n_cols, const int32_t *cnt, const int32_t *idx,
                              const float *val, void *P, int64_t ldp, grf_stream_t stream) {
    GRF_REQUIRE(n_rows >= 0 && cap >= 1 && n_cols >= 0 && (n_rows == 0 || (cnt && idx && val && P)), GRF_EINVAL,
                "grf_densify_padded_planes: bad arguments");
    const int64_t kt = cdiv<int64_t>(n_cols, 16);
    GRF_REQUIRE(ldp >= kt * kPlaneBytes && ldp % 16 == 0 && ((uintptr_t)P & 15) == 0, GRF_EINVAL,
                "grf_densify_padded_planes: ldp must cover %lld bytes, a multiple of 16, P 16-byte aligned",
                (long long)(kt * kPlaneBytes));
    GRF_REQUIRE(16 * kt * (int64_t)sizeof(float) <= 160 * 1024, GRF_EUNSUPPORTED,
                "grf_densify_padded_planes: a row of %lld floats does not fit one CU's LDS", (long long)(16 * kt));
    if (n_rows == 0) return GRF_OK;
    GRF_REQUIRE_GRID(n_rows, 256, "densify_padded_planes_kernel");
    densify_padded_planes_kernel<<<(unsigned)n_rows, 256, (size_t)(16 * kt) * sizeof(float), S(stream)>>>(
        cap, cnt, idx, val, kt, reinterpret_cast<unsigned char *>(P), ldp);
    GRF_CHECK_LAUNCH("densify_padded_planes_kernel");
    return GRF_OK;
}

// K from the planes: the wide items from 64 tile rows on, else the 128-tile kernel; workspace as dense_gram_split's
int32_t dense_gram_planes(int64_t n, int64_t k_dim, const void *P, int64_t ldp, float *K, int64_t ldk,
                          void *workspace, size_t workspace_bytes, grf_stream_t stream) {
    GRF_REQUIRE(n >= 0 && k_dim >= 0 && K && ldk >= n && (n == 0 || P), GRF_EINVAL, "grf_gram_dense_planes: bad arguments");
    GRF_REQUIRE(ldp >= planes_row_bytes(k_dim) && ldp % 16 == 0 && ((uintptr_t)P & 15) == 0, GRF_EINVAL,
                "grf_gram_dense_planes: ldp must cover the k-tiles' planes, a multiple of 16, P 16-byte aligned");
    GRF_REQUIRE(ldk % 4 == 0 && ((uintptr_t)K & 15) == 0, GRF_EINVAL,
                "grf_gram_dense_planes: ldk must be a multiple of 4 and K 16-byte aligned");
    if (n == 0 || k_dim == 0) {
        if (n) GRF_CHECK_HIP(hipMemset2DAsync(K, (size_t)ldk * sizeof(float), 0, (size_t)n * sizeof(float), (size_t)n,
                                              S(stream)));
        return GRF_OK;
    }
    GRF_REQUIRE(workspace && ((uintptr_t)workspace & 255) == 0 &&
                    workspace_bytes >= dense_gram_split_workspace_bytes(n, k_dim),
                GRF_EINVAL, "grf_gram_dense_planes: workspace too small or not 256-byte aligned");
    DenseArgs a{};
    a.K = K;
    a.n = n;
    a.nt = cdiv<int64_t>(n, kTile);
    a.ldk = ldk;
    a.kpad = cdiv<int64_t>(k_dim, 16) * 16;
    // the wide items from 64 tile rows on (the split path's rule, GRF_DENSE_WIDE as there), else 128-tiles
    const int wide_env = env_int("GRF_DENSE_WIDE", -1);
    if (!(wide_env == 1 || (wide_env != 0 && a.nt >= 64))) {
        const DensePlan p = dense_plan(n, k_dim, 16);
        const int64_t split_tiles = p.tiles - p.n_whole;
        const int64_t items = p.n_whole + split_tiles * p.n_split;
        GRF_REQUIRE_GRID(items, 256, "gram_planes_tile_kernel");
        a.tickets = split_tiles > 0 ? reinterpret_cast<int32_t *>(workspace) : nullptr;
        a.slabs = split_tiles > 0 ? reinterpret_cast<float *>(reinterpret_cast<char *>(workspace) + kTicketBytes)
                                  : nullptr;
        a.n_whole = p.n_whole;
        a.k_split = p.k_split;
        a.n_split = p.n_split;
        gram_planes_tile_kernel<<<(unsigned)items, 256, 0, S(stream)>>>(a, reinterpret_cast<const unsigned char *>(P),
                                                                         ldp);
        GRF_CHECK_LAUNCH("gram_planes_tile_kernel");
        return GRF_OK;
    }
    const SkPlan q = sk_plan_wide(n, k_dim);
    GRF_REQUIRE_GRID(q.grid, 512, "gram_planes_wide_kernel");
    a.tickets = reinterpret_cast<int32_t *>(workspace);
    a.slabs = reinterpret_cast<float *>(reinterpret_cast<char *>(workspace) + kTicketBytes);
    a.sk_units = q.units;
    a.sk_kt = q.kt;
    a.sk_total = q.total;
    a.dp_rounds = q.dp_rounds;
    a.xcd_slots = q.xcd_slots;
    gram_planes_wide_kernel<kSplitNST><<<(unsigned)q.grid, 512, 0, S(stream)>>>(
        a, reinterpret_cast<const unsigned char *>(P), ldp);
    GRF_CHECK_LAUNCH("gram_planes_wide_kernel");
    return GRF_OK;
}

}  // namespace grf
