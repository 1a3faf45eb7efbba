// exec_half_probe.hip -- does an MI355X SIMD skip the idle 32-lane half of a wave64 VALU
// instruction?  16 independent v_fma_f32 chains run under EXEC = all 64 lanes, the low 32,
// the high 32, every other lane, and one lane; cycles per wave instruction per SIMD at
// 4 waves/SIMD.  If a half with EXEC = 0 were skipped, render loops could run their strip
// bodies under the strip's near mask and gain on half-empty strips.
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/bin/exec_half_probe tools/exec_half_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int ITERS = 2048;

#define FMA8(i0) "v_fma_f32 %0, %0, %8, %9\n v_fma_f32 %1, %1, %8, %9\n v_fma_f32 %2, %2, %8, %9\n v_fma_f32 %3, %3, %8, %9\n" \
                 "v_fma_f32 %4, %4, %8, %9\n v_fma_f32 %5, %5, %8, %9\n v_fma_f32 %6, %6, %8, %9\n v_fma_f32 %7, %7, %8, %9\n"

__global__ void __launch_bounds__(256) k_exec(float* out, unsigned long long mask) {
    float a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    float b = 0.999f + threadIdx.x * 1e-7f, c = 0.5f;
    if (__builtin_amdgcn_inverse_ballot_w64(mask)) {
        for (int it = 0; it < ITERS; ++it) {
            asm volatile(FMA8(0) FMA8(0)
                         : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
                         : "v"(b), "v"(c));
        }
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
}

int main() {
    hipDeviceProp_t p;
    if (hipGetDeviceProperties(&p, 0) != hipSuccess) return 1;
    const int cus = p.multiProcessorCount;
    const double clk = p.clockRate * 1e3;
    float* out;
    if (hipMalloc(&out, (size_t)cus * 16 * 256 * sizeof(float)) != hipSuccess) return 1;
    struct M { const char* name; unsigned long long m; };
    M ms[] = {{"all 64 lanes", ~0ull}, {"low 32 lanes", 0xFFFFFFFFull}, {"high 32 lanes", 0xFFFFFFFF00000000ull},
              {"every other lane", 0x5555555555555555ull}, {"lane 0 only", 1ull}, {"lanes 0 and 32", 0x100000001ull}};
    const int wps = 4, blocks = cus * wps;
    for (auto& m : ms) {
        hipLaunchKernelGGL(k_exec, dim3(blocks), dim3(256), 0, 0, out, m.m);
        hipEvent_t a, b;
        hipEventCreate(&a);
        hipEventCreate(&b);
        hipDeviceSynchronize();
        hipEventRecord(a);
        for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(k_exec, dim3(blocks), dim3(256), 0, 0, out, m.m);
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms_;
        hipEventElapsedTime(&ms_, a, b);
        ms_ /= 5;
        printf("EXEC %-18s %.2f cycles per wave instruction per SIMD\n", m.name, ms_ * 1e-3 * clk / (16.0 * ITERS * wps));
    }
    return 0;
}
