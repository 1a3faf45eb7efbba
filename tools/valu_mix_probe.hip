// valu_mix_probe.hip -- issue cost per VALU instruction FORM on MI355X (cycles per wave
// instruction per SIMD, 4 waves/SIMD, 8 independent chains): which operand kinds (VGPR,
// SGPR, inline constant, literal), encodings and packed forms issue at the SIMD-32 rate
// (2 cycles per wave64 instruction) and which at half of it.
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/bin/valu_mix_probe tools/valu_mix_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

constexpr int ITERS = 2048;

#define BODY8(INS)                                                                           \
    asm volatile(INS(0) INS(1) INS(2) INS(3) INS(4) INS(5) INS(6) INS(7)                     \
                 : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) \
                 : "v"(b), "v"(c), "s"(sc), "s"(msk), "s"(msk2));

#define KERNEL(NAME, INS)                                                                    \
    __global__ void __launch_bounds__(256) NAME(float* out, float sc) {                      \
        float a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, \
              a6 = a0 + 6, a7 = a0 + 7;                                                      \
        float b = 0.999f + threadIdx.x * 1e-7f, c = 0.5f;                                    \
        uint64_t msk = 0x5555555555555555ull, msk2 = 0;                                      \
        for (int it = 0; it < ITERS; ++it) {                                                 \
            BODY8(INS) BODY8(INS)                                                            \
        }                                                                                    \
        out[blockIdx.x * blockDim.x + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;  \
    }

// dependent chains: ILP 1 / 2 / 4 over the 8 registers (chain i uses register i % ILP)
#define DEP1(i) "v_fma_f32 %0, %0, %8, %9\n"
#define DEP2(i) "v_fma_f32 %" #i ", %" #i ", %8, %9\n"
#define MINVV(i) "v_min_f32 %" #i ", %" #i ", %8\n"
#define MAXVV(i) "v_max_f32 %" #i ", %" #i ", %8\n"
#define CNDS(i) "v_cndmask_b32_e64 %" #i ", %" #i ", %8, %11\n"
#define CMPS(i) "v_cmp_ge_f32_e64 %12, %" #i ", %8\n"
#define LSHL2(i) "v_lshlrev_b32 %" #i ", 3, %" #i "\n"
#define ADDU(i) "v_add_u32 %" #i ", %" #i ", %9\n"
#define EXPF(i) "v_exp_f32 %" #i ", %" #i "\n"
#define PKFMA(i) "v_pk_fma_f32 %[p" #i "], %[p" #i "], %[pb], %[pc]\n"
#define FMA_VVV(i) "v_fma_f32 %" #i ", %" #i ", %8, %9\n"
#define FMA_VVS(i) "v_fma_f32 %" #i ", %" #i ", %8, %10\n"
#define FMA_VVI(i) "v_fma_f32 %" #i ", %" #i ", %8, 1.0\n"
#define FMAAK(i) "v_fmaak_f32 %" #i ", %" #i ", %8, 0x3e2aaa49\n"
#define FMAC(i) "v_fmac_f32 %" #i ", %8, %9\n"
#define MUL_VV(i) "v_mul_f32 %" #i ", %" #i ", %8\n"
#define MUL_SV(i) "v_mul_f32 %" #i ", %10, %" #i "\n"
#define ADD_VV(i) "v_add_f32 %" #i ", %" #i ", %8\n"
#define MIN_LIT(i) "v_min_f32 %" #i ", 0x3f7d70a4, %" #i "\n"
#define CND(i) "v_cndmask_b32 %" #i ", %" #i ", %8, vcc\n"
#define CMP(i) "v_cmp_ge_f32 vcc, %" #i ", %8\n"
#define LSHLADD(i) "v_lshl_add_u32 %" #i ", %" #i ", 3, %9\n"
#define RCP(i) "v_rcp_f32 %" #i ", %" #i "\n"
#define MOV(i) "v_mov_b32 %" #i ", %8\n"
#define SUB_VV(i) "v_sub_f32 %" #i ", %8, %" #i "\n"

KERNEL(k_dep1, DEP1)
KERNEL(k_min_vv, MINVV)
KERNEL(k_max_vv, MAXVV)
KERNEL(k_cnd_s, CNDS)
KERNEL(k_cmp_s, CMPS)
KERNEL(k_lshl2, LSHL2)
KERNEL(k_addu, ADDU)
KERNEL(k_exp, EXPF)
// 2 / 4 independent chains (ILP 2 / 4): registers 0..ILP-1 only
#define BODYN(INS, N)                                                                        \
    asm volatile(INS(0) INS(1) INS(0) INS(1) INS(0) INS(1) INS(0) INS(1)                     \
                 : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) \
                 : "v"(b), "v"(c), "s"(sc), "s"(msk), "s"(msk2));
#define BODYN4(INS)                                                                          \
    asm volatile(INS(0) INS(1) INS(2) INS(3) INS(0) INS(1) INS(2) INS(3)                     \
                 : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) \
                 : "v"(b), "v"(c), "s"(sc), "s"(msk), "s"(msk2));
#define KERNELX(NAME, BODY)                                                                  \
    __global__ void __launch_bounds__(256) NAME(float* out, float sc) {                      \
        float a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, \
              a6 = a0 + 6, a7 = a0 + 7;                                                      \
        float b = 0.999f + threadIdx.x * 1e-7f, c = 0.5f;                                    \
        uint64_t msk = 0x5555555555555555ull, msk2 = 0;                                      \
        for (int it = 0; it < ITERS; ++it) {                                                 \
            BODY BODY                                                                        \
        }                                                                                    \
        out[blockIdx.x * blockDim.x + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;  \
    }
KERNELX(k_dep2, BODYN(DEP2, 2))
KERNELX(k_dep4, BODYN4(DEP2))
typedef float f2 __attribute__((ext_vector_type(2)));
__global__ void __launch_bounds__(256) k_pk8(float* out, float sc) {
    f2 p0 = f2{threadIdx.x * 1.f, 1.f}, p1 = p0 + 1.f, p2 = p0 + 2.f, p3 = p0 + 3.f, p4 = p0 + 4.f, p5 = p0 + 5.f,
       p6 = p0 + 6.f, p7 = p0 + 7.f;
    f2 pb = f2{0.999f, 0.998f}, pc = f2{0.5f, 0.25f};
    for (int it = 0; it < ITERS * 2; ++it) {
        asm volatile(PKFMA(0) PKFMA(1) PKFMA(2) PKFMA(3) PKFMA(4) PKFMA(5) PKFMA(6) PKFMA(7)
                     : [p0] "+v"(p0), [p1] "+v"(p1), [p2] "+v"(p2), [p3] "+v"(p3), [p4] "+v"(p4), [p5] "+v"(p5),
                       [p6] "+v"(p6), [p7] "+v"(p7)
                     : [pb] "v"(pb), [pc] "v"(pc));
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = p0.x + p1.x + p2.x + p3.x + p4.y + p5.y + p6.y + p7.y;
}
KERNEL(k_fma_vvv, FMA_VVV)
KERNEL(k_fma_vvs, FMA_VVS)
KERNEL(k_fma_vvi, FMA_VVI)
KERNEL(k_fmaak, FMAAK)
KERNEL(k_fmac, FMAC)
KERNEL(k_mul_vv, MUL_VV)
KERNEL(k_mul_sv, MUL_SV)
KERNEL(k_add_vv, ADD_VV)
KERNEL(k_sub_vv, SUB_VV)
KERNEL(k_min_lit, MIN_LIT)
KERNEL(k_cndmask, CND)
KERNEL(k_cmp, CMP)
KERNEL(k_lshladd, LSHLADD)
KERNEL(k_rcp, RCP)
KERNEL(k_mov, MOV)

int main() {
    hipDeviceProp_t p;
    if (hipGetDeviceProperties(&p, 0) != hipSuccess) return 1;
    const int cus = p.multiProcessorCount;
    const double clk = p.clockRate * 1e3;
    float* out;
    if (hipMalloc(&out, (size_t)cus * 16 * 256 * sizeof(float)) != hipSuccess) return 1;
    struct K { const char* name; void (*f)(float*, float); };
    K ks[] = {{"dep chain ILP1 fma v,v,v", k_dep1}, {"dep chains ILP2", k_dep2}, {"dep chains ILP4", k_dep4},
              {"v_pk_fma_f32 v,v,v", k_pk8}, {"v_min_f32 v,v", k_min_vv}, {"v_max_f32 v,v", k_max_vv},
              {"v_cndmask_b32 s[mask]", k_cnd_s}, {"v_cmp_ge_f32 -> s[]", k_cmp_s}, {"v_lshlrev_b32 3,v", k_lshl2},
              {"v_add_u32 v,v", k_addu}, {"v_exp_f32", k_exp},{"v_fma_f32 v,v,v", k_fma_vvv}, {"v_fma_f32 v,v,s", k_fma_vvs}, {"v_fma_f32 v,v,1.0", k_fma_vvi},
              {"v_fmaak_f32 (literal)", k_fmaak}, {"v_fmac_f32 v,v", k_fmac}, {"v_mul_f32 v,v", k_mul_vv},
              {"v_mul_f32 s,v", k_mul_sv}, {"v_add_f32 v,v", k_add_vv}, {"v_sub_f32 v,v", k_sub_vv},
              {"v_min_f32 literal,v", k_min_lit}, {"v_cndmask_b32 vcc", k_cndmask}, {"v_cmp_ge_f32 vcc", k_cmp},
              {"v_lshl_add_u32 v,3,v", k_lshladd}, {"v_rcp_f32", k_rcp}, {"v_mov_b32 v", k_mov}};
    for (int wps : {2, 4, 8}) {
        for (auto& k : ks) {
            const int blocks = cus * wps;
            hipLaunchKernelGGL(k.f, dim3(blocks), dim3(256), 0, 0, out, 0.999f);
            hipEvent_t a, b;
            hipEventCreate(&a);
            hipEventCreate(&b);
            hipDeviceSynchronize();
            hipEventRecord(a);
            for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(k.f, dim3(blocks), dim3(256), 0, 0, out, 0.999f);
            hipEventRecord(b);
            hipEventSynchronize(b);
            float ms;
            hipEventElapsedTime(&ms, a, b);
            ms /= 5;
            const double instr = 16.0 * ITERS * wps;  // wave instructions per SIMD
            printf("waves/SIMD %d  %-24s %.2f cycles per wave instruction\n", wps, k.name, ms * 1e-3 * clk / instr);
        }
    }
    return 0;
}
