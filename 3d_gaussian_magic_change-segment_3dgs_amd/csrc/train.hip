// train.hip -- the training-step kernels of include/gsr_train.h:
// activations, activation backward, the fused Adam step and the densification
// statistics, all as single streaming passes over the Gaussian arena.
//
// Reference semantics:
//   activations        scene/gaussian_model.py:34-43 (exp, sigmoid, F.normalize) and
//                      the get_* properties :100-127
//   Adam               torch.optim.Adam(lr=0.0, eps=1e-15) built at :172, stepped at
//                      train.py:185; torch's _multi_tensor_adam arithmetic (lerp_,
//                      mul_/addcmul_, sqrt / bc2_sqrt + eps, addcdiv_)
//   densify statistics train.py:170-172 and gaussian_model.py:523-526
//
// Each kernel is HBM-bound; one thread owns one float4 of one arena block (every
// block starts 256-B aligned and is padded to a float4 multiple, include/
// gsr_train.h), so loads and stores are dwordx4 and fully coalesced.
#include <math.h>

#include "gsr_internal.h"
#include "../../include/gsr_train.h"

namespace gsr {
namespace {

constexpr int TR_THREADS = 256;
constexpr int TR_MAX_BLOCKS = 256 * 32;  // grid-stride beyond this (8192 workgroups)

// Adam launch shape (gsr_set_option "adam_items" / "adam_nt" / "adam_grid").
// Measured at P = 1M, SH3 (tools/adam_variants.py): 4 items + non-temporal + no cap
// = 0.289 ms (6.05 TB/s); 1 item, temporal, 8192-WG cap = 0.316 ms.
int g_adam_items = 4;        // float4 items per thread per grid-stride iteration
int g_adam_nt = 1;           // non-temporal loads/stores (every byte is touched once)
long long g_adam_grid = 0;   // workgroup cap (0 = no cap: each thread does `items` items)

inline long long arena_align(long long n) { return (n + GSR_ARENA_ALIGN - 1) / GSR_ARENA_ALIGN * GSR_ARENA_ALIGN; }

// Float4 work map of an arena: block b covers float4 items [c4[b], c4[b+1]).
struct ArenaMap {
    long long off[GSR_ARENA_BLOCKS];  // float offsets of the blocks
    long long aoff[GSR_ACT_BLOCKS];   // float offsets of the activated blocks (for b = 2..5)
    int c4[GSR_ARENA_BLOCKS + 1];     // float4 item prefix over the blocks
    int M3;                           // floats per Gaussian in the features block (3*M)
};

const int BLOCK_WIDTH[GSR_ARENA_BLOCKS] = {3, -1, 1, 3, 4, -2};  // -1: 3*M, -2: C

ArenaMap arena_map(int P, int M, int C) {
    ArenaMap am{};
    long long o = 0, a = 0;
    int c = 0;
    for (int b = 0; b < GSR_ARENA_BLOCKS; ++b) {
        const long long k = BLOCK_WIDTH[b] == -1 ? 3LL * M : BLOCK_WIDTH[b] == -2 ? (long long)C : BLOCK_WIDTH[b];
        const long long n = k * P;
        am.off[b] = o;
        o += arena_align(n);
        am.c4[b] = c;
        c += (int)((n + 3) / 4);
        if (b >= 2) {
            am.aoff[b - 2] = a;
            a += arena_align(n);
        }
    }
    am.c4[GSR_ARENA_BLOCKS] = c;
    am.M3 = 3 * M;
    return am;
}

__device__ __forceinline__ int block_of(const ArenaMap& am, int w) {
    int b = 0;
#pragma unroll
    for (int k = 1; k < GSR_ARENA_BLOCKS; ++k) b += (w >= am.c4[k]) ? 1 : 0;
    return b;
}

__device__ __forceinline__ float sigmoidf_(float x) { return 1.0f / (1.0f + expf(-x)); }  // torch sigmoid

// Activation of one float4 of block b (2..5) of the raw parameters.
__device__ __forceinline__ float4 activate4(int b, float4 x) {
    if (b == 3) return make_float4(expf(x.x), expf(x.y), expf(x.z), expf(x.w));
    if (b == 4) {  // F.normalize(dim=1, eps=1e-12): one quaternion per float4
        const float n = sqrtf(x.x * x.x + x.y * x.y + x.z * x.z + x.w * x.w);
        const float d = fmaxf(n, 1e-12f);
        return make_float4(x.x / d, x.y / d, x.z / d, x.w / d);
    }
    return make_float4(sigmoidf_(x.x), sigmoidf_(x.y), sigmoidf_(x.z), sigmoidf_(x.w));
}

__global__ void __launch_bounds__(TR_THREADS) k_activate(ArenaMap am, const float* __restrict__ param,
                                                         float* __restrict__ act) {
    const int lo = am.c4[2], hi = am.c4[GSR_ARENA_BLOCKS];
    for (int w = lo + blockIdx.x * TR_THREADS + threadIdx.x; w < hi; w += gridDim.x * TR_THREADS) {
        const int b = block_of(am, w);
        const int wl = w - am.c4[b];
        const float4 x = *reinterpret_cast<const float4*>(param + am.off[b] + 4LL * wl);
        *reinterpret_cast<float4*>(act + am.aoff[b - 2] + 4LL * wl) = activate4(b, x);
    }
}

// d(raw) from d(activated), in place (torch autograd formulas: exp -> g*result,
// sigmoid_backward -> g*(1-y)*y, F.normalize = x / clamp_min(norm(x), eps) through
// div / clamp_min / norm backward).
__global__ void __launch_bounds__(TR_THREADS) k_activation_backward(ArenaMap am, const float* __restrict__ param,
                                                                    const float* __restrict__ act,
                                                                    float* __restrict__ grad) {
    const int lo = am.c4[2], hi = am.c4[GSR_ARENA_BLOCKS];
    for (int w = lo + blockIdx.x * TR_THREADS + threadIdx.x; w < hi; w += gridDim.x * TR_THREADS) {
        const int b = block_of(am, w);
        const int wl = w - am.c4[b];
        float4* gp = reinterpret_cast<float4*>(grad + am.off[b] + 4LL * wl);
        const float4 g = *gp;
        float4 r;
        if (b == 4) {
            const float4 x = *reinterpret_cast<const float4*>(param + am.off[b] + 4LL * wl);
            const float n = sqrtf(x.x * x.x + x.y * x.y + x.z * x.z + x.w * x.w);
            const float d = fmaxf(n, 1e-12f);
            const float dd = d * d;
            float gd = (-g.x * x.x) / dd;
            gd += (-g.y * x.y) / dd;
            gd += (-g.z * x.z) / dd;
            gd += (-g.w * x.w) / dd;
            const float gn = (n >= 1e-12f && n > 0.0f) ? gd / n : 0.0f;
            r = make_float4(g.x / d + x.x * gn, g.y / d + x.y * gn, g.z / d + x.z * gn, g.w / d + x.w * gn);
        } else {
            const float4 y = *reinterpret_cast<const float4*>(act + am.aoff[b - 2] + 4LL * wl);
            if (b == 3) {
                r = make_float4(g.x * y.x, g.y * y.y, g.z * y.z, g.w * y.w);
            } else {
                r = make_float4((g.x * (1.0f - y.x)) * y.x, (g.y * (1.0f - y.y)) * y.y, (g.z * (1.0f - y.z)) * y.z,
                                (g.w * (1.0f - y.w)) * y.w);
            }
        }
        *gp = r;
    }
}

struct AdamArgs {
    float b1, b2, one_minus_b1, one_minus_b2, eps;
    float ss[GSR_ADAM_GROUPS];   // -step_size per group (0 for skipped groups)
    float bc2[GSR_ADAM_GROUPS];  // sqrt(1 - b2^t) per group
    int skip[GSR_ADAM_GROUPS];
};

// Reference param-group index (gaussian_model.py:162-170) of arena block b.
__device__ __forceinline__ int group_of_block(int b) {
    return b == 0 ? 0 : b == 2 ? 3 : b == 3 ? 5 : b == 4 ? 6 : b == 5 ? 4 : 1;
}

__device__ __forceinline__ void adam1(float& p, float& m, float& v, float g, float ss, float bc2, const AdamArgs& a) {
    m = m + a.one_minus_b1 * (g - m);      // exp_avg.lerp_(grad, 1 - beta1)  (weight < 0.5 branch)
    v = v * a.b2;                          // exp_avg_sq.mul_(beta2)
    v = v + a.one_minus_b2 * g * g;        //   .addcmul_(grad, grad, value=1 - beta2)
    const float den = sqrtf(v) / bc2 + a.eps;
    p = p + ss * (m / den);                // param.addcdiv_(exp_avg, denom, value=-step_size)
}

typedef float v4f __attribute__((ext_vector_type(4)));
template <bool NT>
__device__ __forceinline__ float4 ld4(const float* p) {
    if constexpr (NT) {
        const v4f r = __builtin_nontemporal_load(reinterpret_cast<const v4f*>(p));
        return make_float4(r.x, r.y, r.z, r.w);
    } else {
        return *reinterpret_cast<const float4*>(p);
    }
}
template <bool NT>
__device__ __forceinline__ void st4(float* p, float4 v) {
    if constexpr (NT) {
        const v4f r = {v.x, v.y, v.z, v.w};
        __builtin_nontemporal_store(r, reinterpret_cast<v4f*>(p));
    } else {
        *reinterpret_cast<float4*>(p) = v;
    }
}

template <bool NT>
__device__ __forceinline__ void adam_item(const ArenaMap& am, const AdamArgs& a, int w, float* __restrict__ param,
                                          const float* __restrict__ grad, float* __restrict__ exp_avg,
                                          float* __restrict__ exp_avg_sq, float* __restrict__ act) {
    const int b = block_of(am, w);
    const int wl = w - am.c4[b];
    const long long e = am.off[b] + 4LL * wl;
    float4 p = ld4<NT>(param + e);
    const float4 g = ld4<NT>(grad + e);
    const float4 m = ld4<NT>(exp_avg + e);
    const float4 v = ld4<NT>(exp_avg_sq + e);
    float pe[4] = {p.x, p.y, p.z, p.w}, me[4] = {m.x, m.y, m.z, m.w}, ve[4] = {v.x, v.y, v.z, v.w};
    const float ge[4] = {g.x, g.y, g.z, g.w};
    if (b == 1) {  // features: coefficient 0 of each Gaussian is f_dc, the rest f_rest
        int col = (4 * wl) % am.M3;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const bool dc = col < 3;
            const int grp = dc ? 1 : 2;
            if (!a.skip[grp]) adam1(pe[j], me[j], ve[j], ge[j], dc ? a.ss[1] : a.ss[2], dc ? a.bc2[1] : a.bc2[2], a);
            col = (col + 1 == am.M3) ? 0 : col + 1;
        }
    } else {
        const int grp = group_of_block(b);
        float ss = a.ss[0], bc2 = a.bc2[0];
        int sk = a.skip[0];
#pragma unroll
        for (int k = 3; k < GSR_ADAM_GROUPS; ++k) {  // select without dynamic kernarg indexing
            if (grp == k) {
                ss = a.ss[k];
                bc2 = a.bc2[k];
                sk = a.skip[k];
            }
        }
        if (!sk) {
#pragma unroll
            for (int j = 0; j < 4; ++j) adam1(pe[j], me[j], ve[j], ge[j], ss, bc2, a);
        }
    }
    p = make_float4(pe[0], pe[1], pe[2], pe[3]);
    st4<NT>(param + e, p);
    st4<NT>(exp_avg + e, make_float4(me[0], me[1], me[2], me[3]));
    st4<NT>(exp_avg_sq + e, make_float4(ve[0], ve[1], ve[2], ve[3]));
    if (act && b >= 2) st4<NT>(act + am.aoff[b - 2] + 4LL * wl, activate4(b, p));
}

template <int ITEMS, bool NT>
__global__ void __launch_bounds__(TR_THREADS) k_adam(ArenaMap am, AdamArgs a, float* __restrict__ param,
                                                     const float* __restrict__ grad, float* __restrict__ exp_avg,
                                                     float* __restrict__ exp_avg_sq, float* __restrict__ act) {
    const int hi = am.c4[GSR_ARENA_BLOCKS];
    const int nth = gridDim.x * TR_THREADS;
    for (int w = blockIdx.x * TR_THREADS + threadIdx.x; w < hi; w += ITEMS * nth) {
#pragma unroll
        for (int k = 0; k < ITEMS; ++k) {
            const int wk = w + k * nth;
            if (wk < hi) adam_item<NT>(am, a, wk, param, grad, exp_avg, exp_avg_sq, act);
        }
    }
}

__global__ void __launch_bounds__(TR_THREADS) k_densify_stats(int P, const uint8_t* __restrict__ filter,
                                                              const int* __restrict__ radii,
                                                              const float* __restrict__ dmeans2D,
                                                              float* __restrict__ max_radii2D,
                                                              float* __restrict__ accum, float* __restrict__ denom) {
    for (int i = blockIdx.x * TR_THREADS + threadIdx.x; i < P; i += gridDim.x * TR_THREADS) {
        const int r = radii ? radii[i] : 0;
        if (!(filter ? filter[i] != 0 : r > 0)) continue;
        if (max_radii2D) max_radii2D[i] = fmaxf(max_radii2D[i], (float)r);
        const float gx = dmeans2D[3LL * i], gy = dmeans2D[3LL * i + 1];
        accum[i] += sqrtf(gx * gx + gy * gy);  // torch.norm(grad[update_filter, :2], dim=-1)
        denom[i] += 1.0f;
    }
}

int grid_for(long long items) {
    const long long g = (items + TR_THREADS - 1) / TR_THREADS;
    return (int)(g < 1 ? 1 : g > TR_MAX_BLOCKS ? TR_MAX_BLOCKS : g);
}

int check_sizes(int P, int M, int C) {
    if (P < 0 || M < 0 || M > 16 || C < 0 || C > 64) return set_error("[gsr] arena: invalid P / M / C");
    // float4 item indices are int32
    if ((long long)P * (3LL * M + 11 + C) / 4 + 8 >= (1LL << 31)) return set_error("[gsr] arena: P too large");
    return 0;
}

int launched(const char* what) {
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return set_error(std::string("[gsr] ") + what + ": " + hipGetErrorString(e));
    return 0;
}

}  // namespace

int set_train_option(const std::string& name, long long v) {
    if (name == "adam_items") g_adam_items = (int)(v >= 4 ? 4 : v >= 2 ? 2 : 1);
    else if (name == "adam_nt") g_adam_nt = v != 0;
    else if (name == "adam_grid") g_adam_grid = v < 0 ? 0 : v;
    else return -1;
    return 0;
}
}  // namespace gsr

using namespace gsr;

extern "C" {

GSR_API long long gsr_arena_layout(int P, int M, int C, long long* off) {
    long long o = 0;
    for (int b = 0; b < GSR_ARENA_BLOCKS; ++b) {
        const long long k = BLOCK_WIDTH[b] == -1 ? 3LL * M : BLOCK_WIDTH[b] == -2 ? (long long)C : BLOCK_WIDTH[b];
        if (off) off[b] = o;
        o += arena_align(k * (P > 0 ? P : 0));
    }
    if (off) off[GSR_ARENA_BLOCKS] = o;
    return o;
}

GSR_API long long gsr_act_layout(int P, int C, long long* off) {
    const long long k[GSR_ACT_BLOCKS] = {1, 3, 4, C};
    long long o = 0;
    for (int b = 0; b < GSR_ACT_BLOCKS; ++b) {
        if (off) off[b] = o;
        o += arena_align(k[b] * (P > 0 ? P : 0));
    }
    if (off) off[GSR_ACT_BLOCKS] = o;
    return o;
}

GSR_API int gsr_activate(int P, int M, int C, const float* param, float* act, void* stream) {
    if (int rc = check_sizes(P, M, C)) return rc;
    if (P == 0) return 0;
    if (!param || !act) return set_error("[gsr] gsr_activate: null buffer");
    const ArenaMap am = arena_map(P, M, C);
    k_activate<<<grid_for(am.c4[GSR_ARENA_BLOCKS] - am.c4[2]), TR_THREADS, 0, (hipStream_t)stream>>>(am, param, act);
    return launched("activate");
}

GSR_API int gsr_activation_backward(int P, int M, int C, const float* param, const float* act, float* grad,
                                    void* stream) {
    if (int rc = check_sizes(P, M, C)) return rc;
    if (P == 0) return 0;
    if (!param || !act || !grad) return set_error("[gsr] gsr_activation_backward: null buffer");
    const ArenaMap am = arena_map(P, M, C);
    k_activation_backward<<<grid_for(am.c4[GSR_ARENA_BLOCKS] - am.c4[2]), TR_THREADS, 0, (hipStream_t)stream>>>(
        am, param, act, grad);
    return launched("activation_backward");
}

GSR_API int gsr_adam_step(int P, int M, int C, float* param, const float* grad, float* exp_avg,
                          float* exp_avg_sq, float* act, const gsr_adam_hyper* h, void* stream) {
    if (int rc = check_sizes(P, M, C)) return rc;
    if (!h) return set_error("[gsr] gsr_adam_step: null hyper-parameters");
    if (P == 0) return 0;
    if (!param || !grad || !exp_avg || !exp_avg_sq) return set_error("[gsr] gsr_adam_step: null buffer");
    AdamArgs a{};
    a.b1 = h->beta1;
    a.b2 = h->beta2;
    a.one_minus_b1 = h->one_minus_beta1;
    a.one_minus_b2 = h->one_minus_beta2;
    a.eps = h->eps;
    for (int g = 0; g < GSR_ADAM_GROUPS; ++g) {
        a.ss[g] = -h->step_size[g];
        a.bc2[g] = h->bc2_sqrt[g];
        a.skip[g] = h->skip[g];
    }
    const ArenaMap am = arena_map(P, M, C);
    const long long items = am.c4[GSR_ARENA_BLOCKS];
    long long blocks = (items + (long long)TR_THREADS * g_adam_items - 1) / ((long long)TR_THREADS * g_adam_items);
    if (g_adam_grid > 0 && blocks > g_adam_grid) blocks = g_adam_grid;
    if (blocks < 1) blocks = 1;
    hipStream_t st = (hipStream_t)stream;
    const dim3 grid((unsigned)blocks);
#define GSR_ADAM_LAUNCH(IT, NT) k_adam<IT, NT><<<grid, TR_THREADS, 0, st>>>(am, a, param, grad, exp_avg, exp_avg_sq, act)
    if (g_adam_nt) {
        if (g_adam_items >= 4) GSR_ADAM_LAUNCH(4, true);
        else if (g_adam_items == 2) GSR_ADAM_LAUNCH(2, true);
        else GSR_ADAM_LAUNCH(1, true);
    } else {
        if (g_adam_items >= 4) GSR_ADAM_LAUNCH(4, false);
        else if (g_adam_items == 2) GSR_ADAM_LAUNCH(2, false);
        else GSR_ADAM_LAUNCH(1, false);
    }
#undef GSR_ADAM_LAUNCH
    return launched("adam_step");
}

GSR_API int gsr_densify_stats(int P, const uint8_t* filter, const int* radii, const float* dmeans2D,
                              float* max_radii2D, float* grad_accum, float* denom, void* stream) {
    if (P < 0) return set_error("[gsr] gsr_densify_stats: P < 0");
    if (P == 0) return 0;
    if ((!filter && !radii) || (max_radii2D && !radii) || !dmeans2D || !grad_accum || !denom)
        return set_error("[gsr] gsr_densify_stats: null buffer");
    k_densify_stats<<<grid_for(P), TR_THREADS, 0, (hipStream_t)stream>>>(P, filter, radii, dmeans2D, max_radii2D,
                                                                         grad_accum, denom);
    return launched("densify_stats");
}

}  // extern "C"
