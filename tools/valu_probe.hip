// valu_probe.hip -- VALU issue-rate probe for the render kernels' design questions:
// how many cycles per SIMD does one wave64 instruction cost when several waves share a
// SIMD?  Kernels: independent v_fma_f32 chains, v_pk_fma_f32 chains, v_fma_f32 with
// SALU mask work interleaved (the render loops' ballot / s_and pattern), and v_fma_f32
// at 4 vs 8 waves per SIMD.  Also the HBM streaming-copy rate (read + write of 2 GiB).
// Build: hipcc -O3 -fno-slp-vectorize --offload-arch=gfx950 -o tools/bin/valu_probe tools/valu_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                   \
    do {                                                                        \
        hipError_t e_ = (x);                                                    \
        if (e_ != hipSuccess) {                                                 \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                            \
        }                                                                       \
    } while (0)

constexpr int ITERS = 4096;

// 8 independent fma chains per lane: 8 * ITERS wave instructions per wave.
__global__ void __launch_bounds__(256) k_fma(float* out, float s) {
    float a[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) a[i] = threadIdx.x * 1e-3f + i;
    for (int it = 0; it < ITERS; ++it) {
#pragma unroll
        for (int i = 0; i < 8; ++i) a[i] = __builtin_fmaf(a[i], s, 0.5f);
    }
    float r = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) r += a[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

typedef float f2 __attribute__((ext_vector_type(2)));
// 8 independent packed chains: 8 * ITERS v_pk_fma_f32 per wave (2 fma per lane each).
__global__ void __launch_bounds__(256) k_pkfma(float* out, float s) {
    f2 a[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) a[i] = f2{threadIdx.x * 1e-3f + i, threadIdx.x * 2e-3f + i};
    const f2 sv = f2{s, s}, h = f2{0.5f, 0.5f};
    for (int it = 0; it < ITERS; ++it) {
#pragma unroll
        for (int i = 0; i < 8; ++i) a[i] = __builtin_elementwise_fma(a[i], sv, h);
    }
    float r = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) r += a[i].x + a[i].y;
    out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

// fma chains with a compare + ballot + SALU and per 4 fmas (the render loops' pattern).
__global__ void __launch_bounds__(256) k_fma_salu(float* out, float s) {
    float a[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) a[i] = threadIdx.x * 1e-3f + i;
    uint64_t m = 0;
    for (int it = 0; it < ITERS; ++it) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            a[i] = __builtin_fmaf(a[i], s, 0.5f);
            if ((i & 3) == 3) m ^= __builtin_amdgcn_ballot_w64(a[i] > 1.f) & (m | 0x5555);
        }
    }
    float r = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) r += a[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = r + (float)(m & 1);
}

// one dependent chain per lane: latency-bound per wave, issue-bound across waves.
__global__ void __launch_bounds__(256) k_fma_dep(float* out, float s) {
    float a = threadIdx.x * 1e-3f;
    for (int it = 0; it < ITERS * 8; ++it) a = __builtin_fmaf(a, s, 0.5f);
    out[blockIdx.x * blockDim.x + threadIdx.x] = a;
}

typedef float f4 __attribute__((ext_vector_type(4)));
// packed / scalar fma with all three operands in VGPRs (per-lane values), 4 chains.
__global__ void __launch_bounds__(256) k_pkfma_vvv(float* out, float s) {
    f2 a[4], b[4], c[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        a[i] = f2{threadIdx.x * 1e-3f + i, threadIdx.x * 2e-3f + i};
        b[i] = f2{s + threadIdx.x * 1e-6f, s - threadIdx.x * 1e-6f};
        c[i] = f2{0.5f + i * threadIdx.x * 1e-7f, 0.25f};
    }
    for (int it = 0; it < ITERS * 2; ++it) {
#pragma unroll
        for (int i = 0; i < 4; ++i) a[i] = __builtin_elementwise_fma(a[i], b[i], c[i]);
    }
    float r = 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) r += a[i].x + a[i].y;
    out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}
__global__ void __launch_bounds__(256) k_fma_vvv(float* out, float s) {
    float a[4], b[4], c[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        a[i] = threadIdx.x * 1e-3f + i;
        b[i] = s + threadIdx.x * 1e-6f * i;
        c[i] = 0.5f + i * threadIdx.x * 1e-7f;
    }
    for (int it = 0; it < ITERS * 2; ++it) {
#pragma unroll
        for (int i = 0; i < 4; ++i) a[i] = __builtin_fmaf(a[i], b[i], c[i]);
    }
    float r = 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) r += a[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}
// packed mul with two VGPR-pair operands, 4 chains.
__global__ void __launch_bounds__(256) k_pkmul_vv(float* out, float s) {
    f2 a[4], b[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        a[i] = f2{threadIdx.x * 1e-3f + i, threadIdx.x * 2e-3f + i};
        b[i] = f2{s + threadIdx.x * 1e-6f, s - threadIdx.x * 1e-6f};
    }
    for (int it = 0; it < ITERS * 2; ++it) {
#pragma unroll
        for (int i = 0; i < 4; ++i) a[i] = a[i] * b[i];
    }
    float r = 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) r += a[i].x + a[i].y;
    out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

// one dependent packed chain per lane.
__global__ void __launch_bounds__(256) k_pkfma_dep(float* out, float s) {
    f2 a = f2{threadIdx.x * 1e-3f, threadIdx.x * 2e-3f};
    const f2 sv = f2{s, s}, h = f2{0.5f, 0.5f};
    for (int it = 0; it < ITERS * 8; ++it) a = __builtin_elementwise_fma(a, sv, h);
    out[blockIdx.x * blockDim.x + threadIdx.x] = a.x + a.y;
}
// two dependent packed chains per lane (the render loops' typical ILP).
__global__ void __launch_bounds__(256) k_pkfma_dep2(float* out, float s) {
    f2 a = f2{threadIdx.x * 1e-3f, threadIdx.x * 2e-3f}, b = a + f2{1.f, 1.f};
    const f2 sv = f2{s, s}, h = f2{0.5f, 0.5f};
    for (int it = 0; it < ITERS * 4; ++it) {
        a = __builtin_elementwise_fma(a, sv, h);
        b = __builtin_elementwise_fma(b, sv, h);
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a.x + a.y + b.x + b.y;
}
// two dependent scalar chains per lane.
__global__ void __launch_bounds__(256) k_fma_dep2(float* out, float s) {
    float a = threadIdx.x * 1e-3f, b = a + 1.f;
    for (int it = 0; it < ITERS * 4; ++it) {
        a = __builtin_fmaf(a, s, 0.5f);
        b = __builtin_fmaf(b, s, 0.5f);
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a + b;
}

__global__ void k_copy(const f4* __restrict__ src, f4* __restrict__ dst, size_t n) {
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (; i < n; i += stride) dst[i] = __builtin_nontemporal_load(src + i);
}

template <class F>
float time_ms(F f, int reps) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    f();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(a));
    for (int i = 0; i < reps; ++i) f();
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    return ms / reps;
}

int main() {
    hipDeviceProp_t p;
    CK(hipGetDeviceProperties(&p, 0));
    const int cus = p.multiProcessorCount;
    const double clk = p.clockRate * 1e3;  // Hz (peak)
    printf("device %s, %d CUs, peak clock %.2f GHz\n", p.name, cus, clk * 1e-9);
    float* out;
    CK(hipMalloc(&out, (size_t)cus * 64 * 256 * sizeof(float)));
    // waves per SIMD = blocks per CU * 4 waves per block / 4 SIMDs
    for (int wps : {1, 2, 4, 8}) {
        const int blocks = cus * wps;  // 256-thread blocks: 4 waves, one per SIMD
        const double winstr = 8.0 * ITERS;  // wave instructions per wave (inner loop)
        const double waves_per_simd = wps;
        auto rep = [&](const char* name, float ms, double per) {
            const double cyc = ms * 1e-3 * clk;
            printf("%-10s waves/SIMD %d: %.3f ms  -> %.2f cycles per wave instruction per SIMD (at peak clock)\n",
                   name, wps, ms, cyc / (waves_per_simd * per));
        };
        rep("fma", time_ms([&] { hipLaunchKernelGGL(k_fma, dim3(blocks), dim3(256), 0, 0, out, 0.999f); }, 5), winstr);
        rep("pk_fma", time_ms([&] { hipLaunchKernelGGL(k_pkfma, dim3(blocks), dim3(256), 0, 0, out, 0.999f); }, 5),
            winstr);
        rep("fma+salu", time_ms([&] { hipLaunchKernelGGL(k_fma_salu, dim3(blocks), dim3(256), 0, 0, out, 0.999f); }, 5),
            winstr);
        rep("fma_dep", time_ms([&] { hipLaunchKernelGGL(k_fma_dep, dim3(blocks), dim3(256), 0, 0, out, 0.999f); }, 5),
            winstr);
        rep("pk_vvv", time_ms([&] { hipLaunchKernelGGL(k_pkfma_vvv, dim3(blocks), dim3(256), 0, 0, out, 0.999f); }, 5),
            winstr);
        rep("fma_vvv", time_ms([&] { hipLaunchKernelGGL(k_fma_vvv, dim3(blocks), dim3(256), 0, 0, out, 0.999f); }, 5),
            winstr);
        rep("pkmul_vv", time_ms([&] { hipLaunchKernelGGL(k_pkmul_vv, dim3(blocks), dim3(256), 0, 0, out, 0.999f); }, 5),
            winstr);
        rep("pk_dep", time_ms([&] { hipLaunchKernelGGL(k_pkfma_dep, dim3(blocks), dim3(256), 0, 0, out, 0.999f); }, 5),
            winstr);
        rep("fma_dep2", time_ms([&] { hipLaunchKernelGGL(k_fma_dep2, dim3(blocks), dim3(256), 0, 0, out, 0.999f); }, 5),
            winstr);
        rep("pk_dep2", time_ms([&] { hipLaunchKernelGGL(k_pkfma_dep2, dim3(blocks), dim3(256), 0, 0, out, 0.999f); }, 5),
            winstr);
    }
    const size_t bytes = (size_t)2 << 30;
    f4 *s, *d;
    CK(hipMalloc(&s, bytes));
    CK(hipMalloc(&d, bytes));
    CK(hipMemset(s, 0, bytes));
    const size_t n = bytes / 16;
    for (int bpc : {4, 8, 16}) {
        const float ms = time_ms([&] { hipLaunchKernelGGL(k_copy, dim3(cus * bpc), dim3(256), 0, 0, s, d, n); }, 10);
        printf("copy kernel (%d blocks/CU): %.3f ms, %.1f GB/s (read + write)\n", bpc, ms, 2.0 * bytes / (ms * 1e-3) / 1e9);
    }
    const float ms = time_ms([&] { CK(hipMemcpyAsync(d, s, bytes, hipMemcpyDeviceToDevice, 0)); }, 10);
    printf("hipMemcpy D2D: %.3f ms, %.1f GB/s (read + write)\n", ms, 2.0 * bytes / (ms * 1e-3) / 1e9);
    return 0;
}
