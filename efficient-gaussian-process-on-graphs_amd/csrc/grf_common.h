// grf_common.h -- shared device/host helpers for the gfx950 GRF engine.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "grf.h"

namespace grf {

void set_error(const char *fmt, ...) __attribute__((format(printf, 1, 2)));

inline hipStream_t S(grf_stream_t s) { return reinterpret_cast<hipStream_t>(s); }

constexpr int kWave = 64;

// ceil-div helpers
template <typename T>
__host__ __device__ inline T cdiv(T a, T b) { return (a + b - 1) / b; }

__host__ __device__ inline uint32_t next_pow2_u32(uint32_t v) {
    if (v <= 1) return 1;
    --v;
    v |= v >> 1; v |= v >> 2; v |= v >> 4; v |= v >> 8; v |= v >> 16;
    return v + 1;
}
__host__ __device__ inline int ceil_log2(uint64_t v) {
    int b = 0;
    while ((1ull << b) < v) ++b;
    return b;
}

// wave-uniform value (lets the compiler use SGPRs / scalar loads)
__device__ inline int64_t uniform(int64_t v) {
    int32_t lo = __builtin_amdgcn_readfirstlane((int32_t)(uint32_t)v);
    int32_t hi = __builtin_amdgcn_readfirstlane((int32_t)(uint32_t)((uint64_t)v >> 32));
    return (int64_t)(((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo);
}
__device__ inline int32_t uniform32(int32_t v) { return __builtin_amdgcn_readfirstlane(v); }

}  // namespace grf

#define GRF_CHECK_HIP(expr)                                                              \
    do {                                                                                 \
        hipError_t e_ = (expr);                                                          \
        if (e_ != hipSuccess) {                                                          \
            grf::set_error("%s failed: %s", #expr, hipGetErrorString(e_));               \
            return GRF_EHIP;                                                             \
        }                                                                                \
    } while (0)

#define GRF_CHECK_LAUNCH(name)                                                           \
    do {                                                                                 \
        hipError_t e_ = hipGetLastError();                                               \
        if (e_ != hipSuccess) {                                                          \
            grf::set_error("launch of %s failed: %s", name, hipGetErrorString(e_));      \
            return GRF_EHIP;                                                             \
        }                                                                                \
    } while (0)

#define GRF_REQUIRE(cond, code, ...)                                                     \
    do {                                                                                 \
        if (!(cond)) {                                                                   \
            grf::set_error(__VA_ARGS__);                                                 \
            return code;                                                                 \
        }                                                                                \
    } while (0)

// The dispatcher takes at most 2^32 - 1 work-items per launch (gridDim.x * blockDim.x):
// a larger grid is silently truncated on gfx950, so every variable-size launch checks it.
#define GRF_REQUIRE_GRID(blocks, threads, name)                                          \
    GRF_REQUIRE((int64_t)(blocks) * (int64_t)(threads) < (1ll << 32), GRF_EUNSUPPORTED,  \
                "%s: %lld work-items exceed one launch (2^32); split the input", name,   \
                (long long)((int64_t)(blocks) * (int64_t)(threads)))
