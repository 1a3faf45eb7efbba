// exp_probe.hip -- is the hardware v_exp_f32 (2^y) correctly rounded on gfx950?
// Sweeps every fp32 y in [lo, 0] (all bit patterns), compares v_exp_f32(y) with
// exp2(y) evaluated in double and rounded to fp32, and histograms the ulp
// difference.  If it is correctly rounded on the blend range, a CPU oracle can
// reproduce it bit for bit (exp2 in double, round), which makes the hardware
// exp usable without giving up bit-parity.  Build: hipcc --offload-arch=gfx950 -O3.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cmath>
#include <cstring>
#include <cstdlib>

__global__ void k_probe(uint32_t b0, uint32_t n, unsigned long long* hist, uint32_t* worst, uint32_t* list,
                        uint32_t cap) {
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t stride = gridDim.x * blockDim.x;
    unsigned long long h[5] = {0, 0, 0, 0, 0};
    for (; i < n; i += stride) {
        const uint32_t bits = b0 + i;
        const float y = __uint_as_float(bits);
        const float hw = __builtin_amdgcn_exp2f(y);
        const float cr = (float)exp2((double)y);
        const int d = (int)__float_as_uint(hw) - (int)__float_as_uint(cr);
        const int ad = d < 0 ? -d : d;
        h[ad > 3 ? 4 : ad]++;
        if (ad > 0) atomicMax(worst, (uint32_t)ad);
        if (ad > 0) {
            // keep every mismatching input (up to cap) for the oracle's exception table
            unsigned int slot = atomicAdd(&worst[1], 1u);
            if (slot < cap) { list[2 * slot] = bits; list[2 * slot + 1] = __float_as_uint(hw); }
        }
    }
    for (int k = 0; k < 5; ++k)
        if (h[k]) atomicAdd(&hist[k], h[k]);
}

int main(int argc, char** argv) {
    // negative floats: 0x80000000 (-0) .. bits of lo (more negative = larger bits)
    const float lo = argc > 1 ? (float)atof(argv[1]) : -12.0f;
    uint32_t lob;
    memcpy(&lob, &lo, 4);
    const uint32_t b0 = 0x80000000u, n = lob - b0 + 1;
    unsigned long long* hist;
    uint32_t* worst;
    hipMalloc(&hist, 5 * sizeof(unsigned long long));
    hipMalloc(&worst, 18 * sizeof(uint32_t));
    hipMemset(hist, 0, 5 * sizeof(unsigned long long));
    hipMemset(worst, 0, 18 * sizeof(uint32_t));
    const uint32_t cap = 1u << 24;
    uint32_t* list;
    hipMalloc(&list, 2ull * cap * sizeof(uint32_t));
    hipLaunchKernelGGL(k_probe, dim3(8192), dim3(256), 0, 0, b0, n, hist, worst, list, cap);
    // positive side too (y in [0, 1]), small
    unsigned long long h[5];
    uint32_t w[18];
    hipMemcpy(h, hist, sizeof(h), hipMemcpyDeviceToHost);
    hipMemcpy(w, worst, sizeof(w), hipMemcpyDeviceToHost);
    printf("range [%g, -0]: %u inputs\n", lo, n);
    printf("ulp diff 0: %llu  1: %llu  2: %llu  3: %llu  >3: %llu  worst %u  mismatches %u\n", h[0], h[1], h[2],
           h[3], h[4], w[0], w[1]);
    const uint32_t m = w[1] < cap ? w[1] : cap;
    uint32_t* hl = (uint32_t*)malloc(2ull * m * sizeof(uint32_t) + 8);
    hipMemcpy(hl, list, 2ull * m * sizeof(uint32_t), hipMemcpyDeviceToHost);
    for (uint32_t k = 0; k < 16 && k < m; ++k) {
        float y, e;
        memcpy(&y, &hl[2 * k], 4);
        memcpy(&e, &hl[2 * k + 1], 4);
        printf("  mismatch y=%.9g (0x%08x) hw=%.9g cr=%.9g\n", y, hl[2 * k], e, (float)exp2((double)y));
    }
    if (argc > 2) {  // dump (input bits, hw bits) pairs
        FILE* f = fopen(argv[2], "wb");
        fwrite(hl, 8, m, f);
        fclose(f);
        printf("wrote %u pairs to %s\n", m, argv[2]);
    }
    return 0;
}
