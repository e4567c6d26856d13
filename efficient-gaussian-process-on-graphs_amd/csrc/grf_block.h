// grf_block.h -- wave64 / workgroup primitives (scan, bitonic sort) for gfx950.
#pragma once
#include "grf_common.h"

namespace grf {

// inclusive scan across the 64 lanes of a wave
template <typename T>
__device__ inline T wave_inclusive_scan(T v) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        T o = __shfl_up(v, off, 64);
        if (lane >= off) v += o;
    }
    return v;
}

// int32: the same scan in DPP steps (row shifts within 16-lane rows, then the row broadcasts of
// lanes 15 and 31): no ds_bpermute round trips through the LDS pipe; identical sums
template <>
__device__ inline int32_t wave_inclusive_scan<int32_t>(int32_t v) {
    v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xf, 0xf, false);  // row_shr:1
    v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xf, 0xf, false);  // row_shr:2
    v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xf, 0xf, false);  // row_shr:4
    v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xf, 0xf, false);  // row_shr:8
    v += __builtin_amdgcn_update_dpp(0, v, 0x142, 0xa, 0xf, false);  // row_bcast:15
    v += __builtin_amdgcn_update_dpp(0, v, 0x143, 0xc, 0xf, false);  // row_bcast:31
    return v;
}

template <typename T>
__device__ inline T wave_sum(T v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    return v;
}

// Exclusive scan over the whole workgroup (blockDim.x multiple of 64, <= 1024).
// `scratch` must hold blockDim.x/64 + 1 elements of T.  Returns the exclusive
// prefix of this thread; *total receives the workgroup sum.  Contains barriers.
template <typename T>
__device__ inline T block_exclusive_scan(T v, T *scratch, T *total) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
    T inc = wave_inclusive_scan(v);
    __syncthreads();
    if (lane == 63) scratch[wid] = inc;
    __syncthreads();
    if (threadIdx.x == 0) {
        T run = 0;
        for (int w = 0; w < nw; ++w) {
            T t = scratch[w];
            scratch[w] = run;
            run += t;
        }
        scratch[nw] = run;
    }
    __syncthreads();
    T res = scratch[wid] + inc - v;
    *total = scratch[nw];
    return res;
}

// Exclusive scan over the whole workgroup with ONE barrier (blockDim.x multiple of 64,
// <= 1024): every wave publishes its total and every thread adds the totals of the waves
// before it.  `scratch` holds blockDim.x/64 elements of T and must not be reused by the
// caller before another barrier.
template <typename T>
__device__ inline T block_exclusive_scan_fast(T v, T *scratch, T *total) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
    const T inc = wave_inclusive_scan(v);
    if (lane == 63) scratch[wid] = inc;
    __syncthreads();
    T before = 0, all = 0;
    for (int w = 0; w < nw; ++w) {
        const T t = scratch[w];
        before += w < wid ? t : (T)0;
        all += t;
    }
    *total = all;
    return before + inc - v;
}

// In-LDS bitonic sort (ascending) of P = power-of-two 32- or 64-bit keys by the whole
// workgroup.  Caller must __syncthreads() before (keys written) and after.
template <typename KT>
__device__ inline void block_bitonic_sort(KT *key, int P) {
    for (int k = 2; k <= P; k <<= 1) {
        for (int j = k >> 1; j > 0; j >>= 1) {
            for (int i = threadIdx.x; i < (P >> 1); i += blockDim.x) {
                // i-th compare/exchange pair of this (k, j) stage
                int lo = ((i & ~(j - 1)) << 1) | (i & (j - 1));
                int hi = lo | j;
                bool asc = (lo & k) == 0;
                const KT a = key[lo], b = key[hi];
                if ((a > b) == asc) {
                    key[lo] = b;
                    key[hi] = a;
                }
            }
            __syncthreads();
        }
    }
}

// v from lane (lane ^ TJ) of the wave: DPP quad permutes for 1 and 2 (no LDS pipe), ds_swizzle in
// bitmask mode for 4..16 (within 32 lanes, no address operand), ds_bpermute for 32.
template <int TJ>
__device__ __forceinline__ uint32_t lane_xor_u32(uint32_t v) {
    // (mov_dpp with bound_ctrl: no `old` operand to zero first -- a quad permute never leaves the quad)
    if constexpr (TJ == 1) return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, true);
    else if constexpr (TJ == 2) return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xF, 0xF, true);
    else if constexpr (TJ < 32) return (uint32_t)__builtin_amdgcn_ds_swizzle((int)v, 0x1F | (TJ << 10));
    else return (uint32_t)__shfl_xor((int)v, TJ, 64);
}
template <int TJ, typename KT>
__device__ __forceinline__ KT lane_xor(KT v) {
    if constexpr (sizeof(KT) == 4) {
        return (KT)lane_xor_u32<TJ>((uint32_t)v);
    } else {
        const uint32_t lo = lane_xor_u32<TJ>((uint32_t)v), hi = lane_xor_u32<TJ>((uint32_t)((uint64_t)v >> 32));
        return (KT)(((uint64_t)hi << 32) | lo);
    }
}

// the compare-exchange of one key with its partner's: the minimum when take_min, else the maximum
// (u32 keys: v_min_u32 / v_max_u32 + one select)
template <typename KT>
__device__ __forceinline__ KT bitonic_keep(KT a, KT o, bool take_min) {
    const KT mn = o < a ? o : a, mx = o < a ? a : o;
    return take_min ? mn : mx;
}

// u32 keys: the same keep as ONE v_med3_u32 against a per-stage selector (0: the minimum, ~0: the
// maximum -- the median of {a, o, 0} is min(a, o), of {a, o, ~0} max(a, o)), instead of a min, a
// max and a select per key
// (written as min / max, which hipcc folds into v_med3_u32: an inline-asm v_med3_u32 left the scheduler
// blind to it -- no interleaving of a stage's DPP moves ahead of its medians, and an s_nop before every
// DPP move that read an asm result)
__device__ __forceinline__ uint32_t med3_u32(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_elementwise_min(__builtin_elementwise_max(a, b),
                                     __builtin_elementwise_max(__builtin_elementwise_min(a, b), c));
}
template <typename KT>
__device__ __forceinline__ KT bitonic_keep_sel(KT a, KT o, bool take_min, uint32_t sel) {
    if constexpr (sizeof(KT) == 4) return (KT)med3_u32((uint32_t)a, (uint32_t)o, sel);
    else return bitonic_keep(a, o, take_min);
}

template <int TJ, typename KT, int R>
__device__ __forceinline__ void bitonic_lane_stage(KT (&v)[R], int tid, int k) {
    if (TJ * R < k) {
        // k > TJ R >= R: bit k of the position tid R + r is bit k of tid R for every r (r < R), so
        // the direction is the thread's, computed once per stage
        const bool take_min = ((tid & TJ) == 0) == (((tid * R) & k) == 0);
        const uint32_t sel = take_min ? 0u : ~0u;
#pragma unroll
        for (int r = 0; r < R; ++r) v[r] = bitonic_keep_sel(v[r], lane_xor<TJ>(v[r]), take_min, sel);
    }
}

// One merge level k of block_bitonic_sort_regs (inlined with a compile-time k when the size is a
// template argument, so every stage's condition folds and the network is straight-line code: no
// register copies at the merge points of runtime-conditional stages).
template <typename KT, int R>
__device__ __forceinline__ void bitonic_regs_level(KT (&v)[R], KT *key, int tid, int k) {
    for (int j = k >> 1; j >= 64 * R; j >>= 1) {  // (a constant trip count of 0-2 when k is: unrolled by itself)  // partner thread tid ^ (j / R) in another wave
        const int tj = j / R;
        const bool lo = (tid & tj) == 0;
        __syncthreads();  // (key[] may still be read by a previous cross-wave stage)
#pragma unroll
        for (int r = 0; r < R; ++r) key[tid * R + r] = v[r];
        __syncthreads();
        const bool take_min = lo == (((tid * R) & k) == 0);  // (k > R: the thread's direction)
        const uint32_t sel = take_min ? 0u : ~0u;
#pragma unroll
        for (int r = 0; r < R; ++r) v[r] = bitonic_keep_sel(v[r], key[(tid ^ tj) * R + r], take_min, sel);
    }
    // partner lane tid ^ tj in this wave
    bitonic_lane_stage<32>(v, tid, k);
    bitonic_lane_stage<16>(v, tid, k);
    bitonic_lane_stage<8>(v, tid, k);
    bitonic_lane_stage<4>(v, tid, k);
    bitonic_lane_stage<2>(v, tid, k);
    bitonic_lane_stage<1>(v, tid, k);
#pragma unroll
    for (int jj = R / 2; jj >= 1; jj >>= 1) {  // partner in this thread's registers (static indices)
        if (jj < k) {
            if (k >= R) {  // one direction for the whole thread (bit k of tid R + r is tid R's)
                const bool asc = ((tid * R) & k) == 0;
                const uint32_t sel = asc ? 0u : ~0u;
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    const int p = r ^ jj;
                    if (p > r) {
                        const KT a = v[r], b = v[p];
                        if constexpr (sizeof(KT) == 4) {  // (two medians: the kept minimum / maximum)
                            v[r] = (KT)med3_u32((uint32_t)a, (uint32_t)b, sel);
                            v[p] = (KT)med3_u32((uint32_t)a, (uint32_t)b, ~sel);
                        } else {
                            const KT mn = b < a ? b : a, mx = b < a ? a : b;
                            v[r] = asc ? mn : mx;
                            v[p] = asc ? mx : mn;
                        }
                    }
                }
            } else {
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    const int p = r ^ jj;
                    if (p > r) {
                        const bool asc = ((tid * R + r) & k) == 0;
                        const KT a = v[r], b = v[p];
                        const bool sw = (a > b) == asc;
                        v[r] = sw ? b : a;
                        v[p] = sw ? a : b;
                    }
                }
            }
        }
    }
}

// Bitonic sort (ascending) of P = R * blockDim.x keys with each thread holding the R consecutive
// keys [tid R, (tid + 1) R) in registers: the stages whose partner is in the same thread (j < R)
// run in registers, the ones whose partner thread is in the same wave through lane shuffles, and
// only partners in another wave go through LDS -- against two LDS reads, up to two writes and a
// barrier per pair and stage for block_bitonic_sort.  Same result (a sorting network; keys equal
// only when interchangeable).  Reads its keys from key[] and writes the sorted keys back; the
// caller must __syncthreads() before (keys written); the sorted key[] is visible on return.
// kP > 0: the size P = kP is a compile-time constant (the network fully unrolled); kP = 0: P at
// run time (P == R * blockDim.x either way).
template <typename KT, int R, int kP = 0>
__device__ inline void block_bitonic_sort_regs(KT *key, int P) {
    const int tid = threadIdx.x;
    KT v[R];
#pragma unroll
    for (int r = 0; r < R; ++r) v[r] = key[tid * R + r];
    if constexpr (kP > 0) {
#pragma unroll
        for (int k = 2; k <= kP; k <<= 1) bitonic_regs_level<KT, R>(v, key, tid, k);
    } else {
        for (int k = 2; k <= P; k <<= 1) bitonic_regs_level<KT, R>(v, key, tid, k);
    }
    __syncthreads();  // (cross-wave stages: every read of key[] done)
#pragma unroll
    for (int r = 0; r < R; ++r) key[tid * R + r] = v[r];
    __syncthreads();
}

}  // namespace grf
