// fp32 MFMA issue ceiling on this box: back-to-back v_mfma_f32_32x32x2f32 / 16x16x4f32 on independent
// accumulators, operands in registers (no memory), 1..4 workgroups of 4 waves per CU; TF/s over HIP events.
// build: hipcc --offload-arch=gfx950 -O3 -o tools/mfma_ceiling tools/mfma_ceiling.hip
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int NACC>
__global__ __launch_bounds__(256) void mfma32(float *out, int iters, float seed) {
    f32x16 c[NACC];
    for (int i = 0; i < NACC; ++i)
        for (int q = 0; q < 16; ++q) c[i][q] = 0.f;
    float a = seed * (threadIdx.x + 1), b = seed * 0.5f + threadIdx.x;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int s = 0; s < 4; ++s)
#pragma unroll
            for (int i = 0; i < NACC; ++i) c[i] = __builtin_amdgcn_mfma_f32_32x32x2f32(a + s, b + i, c[i], 0, 0, 0);
    }
    float acc = 0.f;
    for (int i = 0; i < NACC; ++i)
        for (int q = 0; q < 16; ++q) acc += c[i][q];
    out[blockIdx.x * 256 + threadIdx.x] = acc;
}

template <int NACC>
__global__ __launch_bounds__(256) void mfma16(float *out, int iters, float seed) {
    f32x4 c[NACC];
    for (int i = 0; i < NACC; ++i)
        for (int q = 0; q < 4; ++q) c[i][q] = 0.f;
    float a = seed * (threadIdx.x + 1), b = seed * 0.5f + threadIdx.x;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int s = 0; s < 2; ++s)
#pragma unroll
            for (int i = 0; i < NACC; ++i) c[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(a + s, b + i, c[i], 0, 0, 0);
    }
    float acc = 0.f;
    for (int i = 0; i < NACC; ++i)
        for (int q = 0; q < 4; ++q) acc += c[i][q];
    out[blockIdx.x * 256 + threadIdx.x] = acc;
}

int main() {
    float *out;
    hipMalloc(&out, 256 * 4096 * sizeof(float));
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const int iters = 4000;
    for (int per_cu = 1; per_cu <= 4; ++per_cu) {
        const int grid = 256 * per_cu;
        for (int kind = 0; kind < 2; ++kind) {
            for (int rep = 0; rep < 2; ++rep) {
                hipEventRecord(e0);
                if (kind == 0) mfma32<4><<<grid, 256>>>(out, iters, 1e-3f);
                else mfma16<16><<<grid, 256>>>(out, iters, 1e-3f);
                hipEventRecord(e1);
                hipEventSynchronize(e1);
                float ms;
                hipEventElapsedTime(&ms, e0, e1);
                // flops per wave: iters x (4 x 4 x 32x32x2 x 2) = iters * 65536 (32x32); 16x16x4: iters x 2 x 16 x 2048
                const double flops = (double)grid * 4 * iters * (kind == 0 ? 4.0 * 4 * 32 * 32 * 2 * 2 : 2.0 * 16 * 16 * 16 * 4 * 2);
                if (rep == 1)
                    printf("{\"wg_per_cu\": %d, \"mfma\": \"%s\", \"ms\": %.3f, \"TFs\": %.1f, \"frac\": %.3f}\n", per_cu,
                           kind == 0 ? "32x32x2f32" : "16x16x4f32", ms, flops / ms / 1e9, flops / ms / 1e9 / 157.3);
            }
        }
    }
    return 0;
}
