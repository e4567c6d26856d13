// VALU issue ceiling on this box (the walk roofline's peak): back-to-back independent VALU
// instructions (inline asm, 8 chains, 128 per loop trip; the loop itself is SALU), one workgroup per CU of
// 64 * 4 * wps lanes, i.e. wps waves on every SIMD.  Every wave stamps s_memtime (shader clock) around its
// loop; cycles per instruction per SIMD = the workgroup's longest stamp / (instructions per wave * wps).
// The same launches also run under one rocprofv3 --pmc pass (SQ_INSTS_VALU, GRBM_GUI_ACTIVE) so the
// bench's PMC-derived rate (SQ_INSTS_VALU / (GRBM_GUI_ACTIVE / 8 * 1024)) is calibrated on a kernel whose
// rate is known.  build: hipcc --offload-arch=gfx950 -O3 -o tools/valu_ceiling tools/valu_ceiling.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

#define REP8(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)

template <int KIND>
__global__ void valu_kernel(unsigned long long *stamps, float *out, int iters, float seed) {
    float f[8];
    unsigned u[8];
    double d[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        f[i] = seed * (threadIdx.x + i);
        u[i] = threadIdx.x * 2654435761u + i;
        d[i] = (double)f[i];
    }
    const float a = seed * 0.5f, b = seed * 0.25f;
    const unsigned m = 0xD2511F53u;
    const double da = 0.5, db = 0.25;
    const unsigned long long t0 = __builtin_readcyclecounter();
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            if constexpr (KIND == 0) {  // v_fma_f32
#define OP(i) asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(f[i]) : "v"(a), "v"(b));
                REP8(OP)
#undef OP
            } else if constexpr (KIND == 1) {  // v_add_u32 / v_xor_b32 (the walk's integer glue)
#define OP(i) asm volatile("v_xad_u32 %0, %0, %1, %2" : "+v"(u[i]) : "v"(m), "v"(u[(i + 1) & 7]));
                REP8(OP)
#undef OP
            } else if constexpr (KIND == 2) {  // v_mul_hi_u32 (Philox)
#define OP(i) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(u[i]) : "v"(m));
                REP8(OP)
#undef OP
            } else if constexpr (KIND == 3) {  // v_fma_f64 (the walk's load update)
#define OP(i) asm volatile("v_fma_f64 %0, %1, %2, %0" : "+v"(d[i]) : "v"(da), "v"(db));
                REP8(OP)
#undef OP
            } else if constexpr (KIND == 5) {  // v_mad_u64_u32 (Philox's 32 x 32 -> 64 products)
#define OP(i) asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(d[i]) : "v"(u[i]), "v"(m) : "vcc");
                REP8(OP)
#undef OP
            } else if constexpr (KIND == 6) {  // v_med3_u32 (the sort network's keep)
#define OP(i) asm volatile("v_med3_u32 %0, %0, %1, %2" : "+v"(u[i]) : "v"(m), "v"(u[(i + 1) & 7]));
                REP8(OP)
#undef OP
            } else if constexpr (KIND == 4) {  // v_rcp_f64 (the fp64 divide's seed: transcendental rate)
#define OP(i) asm volatile("v_rcp_f64 %0, %0" : "+v"(d[i]));
                REP8(OP)
#undef OP
            }
        }
    }
    const unsigned long long t1 = __builtin_readcyclecounter();
    float acc = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) acc += f[i] + (float)u[i] + (float)d[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
    if ((threadIdx.x & 63) == 0) stamps[(blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64)] = t1 - t0;
}

int main() {
    const int cus = 256, iters = 2000;
    const char *names[] = {"v_fma_f32", "v_xad_u32", "v_mul_hi_u32", "v_fma_f64", "v_rcp_f64", "v_mad_u64_u32", "v_med3_u32"};
    float *out;
    unsigned long long *stamps;
    hipMalloc(&out, cus * 1024 * sizeof(float));
    hipMalloc(&stamps, cus * 16 * sizeof(unsigned long long));
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    std::vector<unsigned long long> h(cus * 16);
    printf("kind wps  cyc_per_inst_per_SIMD(median WG)  insts_per_SIMD_cycle  wall_ms  clock_GHz(from stamps)\n");
    for (int kind = 0; kind < 7; ++kind) {
        for (int wps = 1; wps <= 4; wps *= 2) {
            const int threads = 256 * wps;
            for (int rep = 0; rep < 2; ++rep) {
                hipEventRecord(e0);
                switch (kind) {
                    case 0: valu_kernel<0><<<cus, threads>>>(stamps, out, iters, 1e-3f); break;
                    case 1: valu_kernel<1><<<cus, threads>>>(stamps, out, iters, 1e-3f); break;
                    case 2: valu_kernel<2><<<cus, threads>>>(stamps, out, iters, 1e-3f); break;
                    case 3: valu_kernel<3><<<cus, threads>>>(stamps, out, iters, 1e-3f); break;
                    case 4: valu_kernel<4><<<cus, threads>>>(stamps, out, iters, 1e-3f); break;
                    case 5: valu_kernel<5><<<cus, threads>>>(stamps, out, iters, 1e-3f); break;
                    default: valu_kernel<6><<<cus, threads>>>(stamps, out, iters, 1e-3f); break;
                }
                hipEventRecord(e1);
                hipEventSynchronize(e1);
                if (rep == 0) continue;
                float ms = 0.f;
                hipEventElapsedTime(&ms, e0, e1);
                hipMemcpy(h.data(), stamps, cus * 4 * wps * sizeof(unsigned long long), hipMemcpyDeviceToHost);
                std::vector<double> per_wg(cus);
                for (int g = 0; g < cus; ++g) {
                    unsigned long long mx = 0;
                    for (int w = 0; w < 4 * wps; ++w) mx = std::max(mx, h[g * 4 * wps + w]);
                    per_wg[g] = (double)mx;
                }
                std::sort(per_wg.begin(), per_wg.end());
                const double insts = (double)iters * 128.0;
                const double cyc = per_wg[cus / 2] / (insts * wps);
                printf("%-13s %d  %8.3f  %8.4f  %8.3f  %6.3f\n", names[kind], wps, cyc, 1.0 / cyc, ms,
                       per_wg[cus - 1] / (ms * 1e6));
            }
        }
    }
    hipFree(out);
    hipFree(stamps);
    return 0;
}
