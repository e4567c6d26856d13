// Microbenchmark: LDS instruction cost on gfx950 (cycles per wave-instruction per CU).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
template <int MODE>
__global__ __launch_bounds__(256) void k(float *out, int iters) {
    __shared__ __attribute__((aligned(16))) float s[8192];
    for (int i = threadIdx.x; i < 8192; i += 256) s[i] = 0.f;
    __syncthreads();
    uint32_t x = threadIdx.x * 2654435761u + blockIdx.x * 97u + 1u;
    float acc = 0.f;
    const int lane = threadIdx.x & 63;
    for (int it = 0; it < iters; ++it) {
        x ^= x << 13; x ^= x >> 17; x ^= x << 5;
        uint32_t a_rand = x & 8191u;
        uint32_t a_lin = ((it * 64u) + lane) & 8191u;
        if (MODE == 0) __hip_atomic_fetch_add(&s[a_rand], 1.0f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        if (MODE == 1) __hip_atomic_fetch_add(&s[a_lin], 1.0f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        if (MODE == 2) acc += s[a_rand];
        if (MODE == 3) acc += s[a_lin];
        if (MODE == 4) s[a_rand] = acc + 1.f;
        if (MODE == 5) s[a_lin] = acc + 1.f;
        if (MODE == 6) { float t = s[a_rand]; s[a_rand] = t + 1.f; }
        if (MODE == 8) __hip_atomic_fetch_add((uint32_t *)&s[a_rand], 3u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        if (MODE == 9) __hip_atomic_fetch_add((unsigned long long *)__builtin_assume_aligned(&s[a_rand & ~1u], 8), 3ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        if (MODE == 10) { if (lane == 0) __hip_atomic_fetch_add(&s[a_rand], 1.0f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP); }
        if (MODE == 11) { if (lane < 16) __hip_atomic_fetch_add(&s[a_rand], 1.0f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP); }
        if (MODE == 12) acc += __hip_atomic_fetch_add(&s[a_rand], 1.0f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        if (MODE == 13) __hip_atomic_fetch_max((uint32_t *)&s[a_rand], x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        if (MODE == 14) { double *sd = (double *)s; __hip_atomic_fetch_add(&sd[a_rand & 4095u], 1.0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP); }
        if (MODE == 7) {  // 4 groups of 16 lanes, same random base, contiguous within group
            uint32_t a = (x & ~15u) & 8191u;
            a = __shfl(a, lane & 48, 64) + (lane & 15);
            __hip_atomic_fetch_add(&s[a & 8191u], 1.0f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) out[blockIdx.x] = s[blockIdx.x & 8191] + acc;
}
template <int MODE>
void run(const char *name, float *d) {
    int iters = 4096, blocks = 256 * 8;
    hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
    k<MODE><<<blocks, 256>>>(d, 16); hipDeviceSynchronize();
    hipEventRecord(a); k<MODE><<<blocks, 256>>>(d, iters); hipEventRecord(b); hipEventSynchronize(b);
    float ms; hipEventElapsedTime(&ms, a, b);
    double instr_per_cu = (double)blocks * 4 * iters / 256.0;
    printf("%-34s %8.3f ms  %6.2f ns/wave-instr/CU  (~%5.1f cyc @2.1GHz)\n", name, ms, ms * 1e6 / instr_per_cu,
           ms * 1e6 / instr_per_cu * 2.1);
}
int main() {
    float *d; hipMalloc(&d, 1 << 20);
    run<0>("ds_add_f32 random", d); run<1>("ds_add_f32 contiguous", d);
    run<2>("ds_read_b32 random", d); run<3>("ds_read_b32 contiguous", d);
    run<4>("ds_write_b32 random", d); run<5>("ds_write_b32 contiguous", d);
    run<6>("read+write random (non-atomic RMW)", d); run<7>("ds_add_f32 4x16 contiguous groups", d);
    run<8>("ds_add_u32 random", d); run<9>("ds_add_u64 random", d); run<10>("ds_add_f32 1 lane", d);
    run<11>("ds_add_f32 16 lanes", d); run<12>("ds_add_rtn_f32 random", d); run<13>("ds_max_u32 random", d);
    run<14>("ds_add_f64 random", d);
    return 0;
}
