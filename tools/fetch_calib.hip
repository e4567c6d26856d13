// FETCH_SIZE calibration on known byte counts (MI355X_MICROARCH.md: "other access widths are
// uncalibrated: calibrate on a known byte count in your own access pattern").
//
// Three kernels read a 4 GiB buffer (far beyond the 256 MB Infinity Cache) exactly once each:
//   stream16   : 16 B per lane, coalesced (the guide's calibrated case: FETCH_SIZE = 1/2 of the bytes)
//   stream12   : 12 B per lane through buffer_load_dwordx3, 64 lanes = 768 contiguous bytes
//                (the Gram's record-pair loads when a bucket spans whole windows)
//   lines12    : the Gram's gather shape: each wave reads 8 random 128-byte lines (a bucket each),
//                10 of the 64 lanes per line reading one 12-byte pair (120 of 128 bytes) through
//                buffer_load_dwordx3; every line of the buffer is read exactly once (a permutation)
// Each kernel is launched on its own, so rocprofv3 --pmc FETCH_SIZE gives per-kernel KiB; the
// script tools/fetch_calib.sh divides by the known bytes (printed here).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
#include <numeric>
#include <random>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); return 1; } } while (0)

__global__ void stream16(const float4 *__restrict__ in, size_t n16, float *__restrict__ sink) {
    float acc = 0.f;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n16; i += (size_t)gridDim.x * blockDim.x) {
        float4 v = in[i];
        acc += v.x + v.y + v.z + v.w;
    }
    if (acc == 1.2345f) sink[0] = acc;  // (never true for the zero-filled input: keeps the loads)
}

__global__ void stream12(const unsigned char *__restrict__ in, size_t n_chunks, float *__restrict__ sink) {
    // chunk = 768 B = 64 lanes x 12 B
    const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<unsigned char *>(in), (short)0, 0x7fffffff, 0x00020000);
    float acc = 0.f;
    const int lane = threadIdx.x & 63;
    const size_t wave = (blockIdx.x * (size_t)blockDim.x + threadIdx.x) >> 6;
    const size_t waves = ((size_t)gridDim.x * blockDim.x) >> 6;
    for (size_t c = wave; c < n_chunks; c += waves) {
        // 32-bit buffer offsets: rebase the resource per 1 GiB window
        const size_t byte = c * 768 + lane * 12;
        const auto r = __builtin_amdgcn_make_buffer_rsrc(const_cast<unsigned char *>(in) + (byte & ~((size_t(1) << 30) - 1)),
                                                         (short)0, 0x7fffffff, 0x00020000);
        const auto v = __builtin_amdgcn_raw_buffer_load_b96(r, (uint32_t)(byte & ((size_t(1) << 30) - 1)), 0, 0);
        acc += __uint_as_float(v[0]) + __uint_as_float(v[1]) + __uint_as_float(v[2]);
    }
    (void)rsrc;
    if (acc == 1.2345f) sink[0] = acc;
}

__global__ void lines12(const unsigned char *__restrict__ in, const uint32_t *__restrict__ perm, size_t n_lines,
                        float *__restrict__ sink) {
    // a wave takes 8 lines per iteration: lane l -> line (l / 8), pair (l % 8); pairs 8, 9 of each
    // line by a second load of lanes 0..15 -> 10 pairs x 12 B = 120 B per line
    float acc = 0.f;
    const int lane = threadIdx.x & 63;
    const size_t wave = (blockIdx.x * (size_t)blockDim.x + threadIdx.x) >> 6;
    const size_t waves = ((size_t)gridDim.x * blockDim.x) >> 6;
    for (size_t g = wave * 8; g < n_lines; g += waves * 8) {
        const size_t li = g + (lane >> 3);
        if (li < n_lines) {
            const size_t line = perm[li];
            const size_t byte = line * 128 + (lane & 7) * 12;
            const auto r = __builtin_amdgcn_make_buffer_rsrc(
                const_cast<unsigned char *>(in) + (byte & ~((size_t(1) << 30) - 1)), (short)0, 0x7fffffff, 0x00020000);
            const auto v = __builtin_amdgcn_raw_buffer_load_b96(r, (uint32_t)(byte & ((size_t(1) << 30) - 1)), 0, 0);
            acc += __uint_as_float(v[0]) + __uint_as_float(v[1]) + __uint_as_float(v[2]);
        }
        const size_t lj = g + (lane >> 1);
        if (lane < 16 && lj < n_lines) {
            const size_t line = perm[lj];
            const size_t byte = line * 128 + (8 + (lane & 1)) * 12;
            const auto r = __builtin_amdgcn_make_buffer_rsrc(
                const_cast<unsigned char *>(in) + (byte & ~((size_t(1) << 30) - 1)), (short)0, 0x7fffffff, 0x00020000);
            const auto v = __builtin_amdgcn_raw_buffer_load_b96(r, (uint32_t)(byte & ((size_t(1) << 30) - 1)), 0, 0);
            acc += __uint_as_float(v[0]) + __uint_as_float(v[1]) + __uint_as_float(v[2]);
        }
    }
    if (acc == 1.2345f) sink[0] = acc;
}

int main() {
    const size_t bytes = size_t(4) << 30;
    unsigned char *buf;
    float *sink;
    uint32_t *perm_d;
    CHECK(hipMalloc(&buf, bytes));
    CHECK(hipMalloc(&sink, 64));
    CHECK(hipMemset(buf, 0, bytes));
    const size_t n_lines = bytes / 128;
    std::vector<uint32_t> perm(n_lines);
    std::iota(perm.begin(), perm.end(), 0u);
    std::mt19937_64 rng(7);
    std::shuffle(perm.begin(), perm.end(), rng);
    CHECK(hipMalloc(&perm_d, n_lines * 4));
    CHECK(hipMemcpy(perm_d, perm.data(), n_lines * 4, hipMemcpyHostToDevice));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    const int grid = 256 * 8, block = 256;
    float ms;
    // (each kernel once, after a flush-sized read of another region would be ideal; the 4 GiB
    // buffer already exceeds every cache level 16x)
    CHECK(hipEventRecord(e0));
    stream16<<<grid, block>>>((const float4 *)buf, bytes / 16, sink);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    printf("stream16 known_bytes %zu ms %.3f GBps %.1f\n", bytes, ms, bytes / (ms * 1e-3) / 1e9);
    const size_t n_chunks = bytes / 768;
    CHECK(hipEventRecord(e0));
    stream12<<<grid, block>>>(buf, n_chunks, sink);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    printf("stream12 known_bytes %zu ms %.3f GBps %.1f\n", n_chunks * 768, ms, n_chunks * 768 / (ms * 1e-3) / 1e9);
    CHECK(hipEventRecord(e0));
    lines12<<<grid, block>>>(buf, perm_d, n_lines, sink);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    printf("lines12 known_bytes %zu (lines x 128 + the 4-B permutation; 120 B used per line) ms %.3f GBps %.1f\n", n_lines * 132, ms,
           n_lines * 128 / (ms * 1e-3) / 1e9);
    CHECK(hipDeviceSynchronize());
    CHECK(hipFree(buf));
    CHECK(hipFree(sink));
    CHECK(hipFree(perm_d));
    return 0;
}
