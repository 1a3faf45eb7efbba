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


// ---- densification / pruning (gaussian_model.py:386-521) ---------------------------
// Plan: one classification pass writes four 0/1 category arrays (kept original,
// kept clone, kept split child, split-selected), four inclusive scans turn them into
// stable output ranks, and the apply pass moves every Gaussian to its slot(s).

struct DensifyWs {
    uint32_t* cat;   // [4][P] category flags
    uint32_t* rank;  // [4][P] inclusive scans of cat
    void* scan[4];   // scan workspaces
    uint32_t* totals;  // [4]
};
inline size_t densify_cat_bytes(size_t P) { return align_up(4 * P * 4); }
inline size_t densify_ws_size(size_t P) {
    return 2 * densify_cat_bytes(P) + 4 * align_up(scan_ws_bytes(P)) + ALIGN;
}
inline DensifyWs densify_ws(size_t P, void* p) {
    char* c = static_cast<char*>(p);
    DensifyWs w;
    w.cat = reinterpret_cast<uint32_t*>(c);
    w.rank = reinterpret_cast<uint32_t*>(c + densify_cat_bytes(P));
    size_t o = 2 * densify_cat_bytes(P);
    for (int k = 0; k < 4; ++k) {
        w.scan[k] = c + o;
        o += align_up(scan_ws_bytes(P));
    }
    w.totals = reinterpret_cast<uint32_t*>(c + o);
    return w;
}

struct DensifyK {
    int mode, split_n;
    float max_grad, min_opacity, clone_max_scale, prune_max_scale, max_screen_size, inv_split_div;
};

__device__ __forceinline__ float max3(const float* s) { return fmaxf(fmaxf(s[0], s[1]), s[2]); }

__global__ void __launch_bounds__(TR_THREADS) k_densify_classify(ArenaMap am, int P, DensifyK d,
                                                                 const float* __restrict__ act,
                                                                 const float* __restrict__ accum,
                                                                 const float* __restrict__ denom,
                                                                 const uint8_t* __restrict__ mask,
                                                                 uint32_t* __restrict__ cat) {
    const int i = blockIdx.x * TR_THREADS + threadIdx.x;
    if (i >= P) return;
    uint32_t keep = 0, clone = 0, child = 0, split = 0;
    if (d.mode == GSR_PRUNE_MASK) {
        keep = mask[i] ? 0u : 1u;
    } else {
        float g = accum[i] / denom[i];  // grads = xyz_gradient_accum / denom; grads[isnan] = 0
        if (g != g) g = 0.0f;
        const float* s = act + am.aoff[1] + 3LL * i;  // get_scaling
        const float smax = max3(s);
        const bool sel = g >= d.max_grad;
        const bool c = sel && smax <= d.clone_max_scale;  // densify_and_clone (:441-444)
        const bool sp = sel && smax > d.clone_max_scale;  // densify_and_split (:408-411)
        if (d.mode == GSR_CLONE_ONLY) {
            keep = 1;
            clone = c;
        } else if (d.mode == GSR_SPLIT_ONLY) {
            keep = !sp;
            child = sp;
            split = sp;
        } else {
            // final prune (:510-516) on the grown set: opacity, world size, and the
            // screen size read from max_radii2D = 0 after densification_postfix
            const float op = act[am.aoff[0] + i];
            const bool mss = d.max_screen_size > 0.0f;
            const bool vs = mss && (0.0f > d.max_screen_size);
            const bool prune_o = op < d.min_opacity || vs || (mss && smax > d.prune_max_scale);
            // children: scaling = log(s / (0.8 N)); torch divides by a scalar as a
            // multiply by its float reciprocal
            float cmax = 0.0f;
            for (int k = 0; k < 3; ++k) cmax = fmaxf(cmax, expf(logf(s[k] * d.inv_split_div)));
            const bool prune_c = op < d.min_opacity || vs || (mss && cmax > d.prune_max_scale);
            keep = !sp && !prune_o;
            clone = c && !prune_o;
            child = sp && !prune_c;
            split = sp;
        }
    }
    cat[i] = keep;
    cat[(size_t)P + i] = clone;
    cat[2 * (size_t)P + i] = child;
    cat[3 * (size_t)P + i] = split;
}

__global__ void k_densify_totals(const uint32_t* __restrict__ rank, int P, uint32_t* __restrict__ totals) {
    const int k = threadIdx.x;
    if (k < 4) totals[k] = P > 0 ? rank[(size_t)k * P + (P - 1)] : 0u;
}

// Copy Gaussian i of (src, old layout) to slot j of (dst, new layout); moments too
// (zeroed when !keep_moments).
__device__ __forceinline__ void copy_gaussian(const ArenaMap& so, const ArenaMap& dn, int i, int j,
                                              const float* __restrict__ src, float* __restrict__ dst) {
    for (int k = 0; k < 3; ++k) dst[dn.off[0] + 3LL * j + k] = src[so.off[0] + 3LL * i + k];
    for (int k = 0; k < so.M3; ++k) dst[dn.off[1] + (long long)so.M3 * j + k] = src[so.off[1] + (long long)so.M3 * i + k];
    dst[dn.off[2] + j] = src[so.off[2] + i];
    for (int k = 0; k < 3; ++k) dst[dn.off[3] + 3LL * j + k] = src[so.off[3] + 3LL * i + k];
    for (int k = 0; k < 4; ++k) dst[dn.off[4] + 4LL * j + k] = src[so.off[4] + 4LL * i + k];
}
__device__ __forceinline__ void copy_segments(const ArenaMap& so, const ArenaMap& dn, int C, int i, int j,
                                              const float* __restrict__ src, float* __restrict__ dst) {
    for (int k = 0; k < C; ++k) dst[dn.off[5] + (long long)C * j + k] = src[so.off[5] + (long long)C * i + k];
}
__device__ __forceinline__ void zero_gaussian(const ArenaMap& dn, int C, int j, float* __restrict__ dst) {
    for (int k = 0; k < 3; ++k) dst[dn.off[0] + 3LL * j + k] = 0.0f;
    for (int k = 0; k < dn.M3; ++k) dst[dn.off[1] + (long long)dn.M3 * j + k] = 0.0f;
    dst[dn.off[2] + j] = 0.0f;
    for (int k = 0; k < 3; ++k) dst[dn.off[3] + 3LL * j + k] = 0.0f;
    for (int k = 0; k < 4; ++k) dst[dn.off[4] + 4LL * j + k] = 0.0f;
    for (int k = 0; k < C; ++k) dst[dn.off[5] + (long long)C * j + k] = 0.0f;
}

__global__ void __launch_bounds__(TR_THREADS) k_densify_apply(
    ArenaMap so, ArenaMap dn, int P, int C, DensifyK d, int base_clone, int base_child, int n_child, int n_split,
    const uint32_t* __restrict__ cat, const uint32_t* __restrict__ rank, const float* __restrict__ param,
    const float* __restrict__ act, const float* __restrict__ m1, const float* __restrict__ m2,
    const float* __restrict__ normals, float* __restrict__ np, float* __restrict__ nm1, float* __restrict__ nm2) {
    const int i = blockIdx.x * TR_THREADS + threadIdx.x;
    if (i >= P) return;
    const size_t P_ = (size_t)P;
    if (cat[i]) {  // kept original: parameters and moments move
        const int j = (int)rank[i] - 1;
        copy_gaussian(so, dn, i, j, param, np);
        copy_segments(so, dn, C, i, j, param, np);
        copy_gaussian(so, dn, i, j, m1, nm1);
        copy_segments(so, dn, C, i, j, m1, nm1);
        copy_gaussian(so, dn, i, j, m2, nm2);
        copy_segments(so, dn, C, i, j, m2, nm2);
    }
    if (cat[P_ + i]) {  // kept clone: parameters copied, fresh moments
        const int j = base_clone + (int)rank[P_ + i] - 1;
        copy_gaussian(so, dn, i, j, param, np);
        copy_segments(so, dn, C, i, j, param, np);
        zero_gaussian(dn, C, j, nm1);
        zero_gaussian(dn, C, j, nm2);
    }
    if (cat[2 * P_ + i]) {  // kept split children
        const int r = (int)rank[3 * P_ + i] - 1;  // rank among all split-selected (normals row)
        const float* s = act + so.aoff[1] + 3LL * i;
        const float* q = param + so.off[4] + 4LL * i;
        // build_rotation (utils/general_utils.py:86-107): separately rounded torch ops
        const float nrm = __fsqrt_rn(__fadd_rn(__fadd_rn(__fadd_rn(__fmul_rn(q[0], q[0]), __fmul_rn(q[1], q[1])),
                                                         __fmul_rn(q[2], q[2])), __fmul_rn(q[3], q[3])));
        const float w = __fdiv_rn(q[0], nrm), x = __fdiv_rn(q[1], nrm), y = __fdiv_rn(q[2], nrm),
                    z = __fdiv_rn(q[3], nrm);
        auto two = [](float v) { return __fmul_rn(2.0f, v); };
        const float R[9] = {
            __fsub_rn(1.0f, two(__fadd_rn(__fmul_rn(y, y), __fmul_rn(z, z)))),
            two(__fsub_rn(__fmul_rn(x, y), __fmul_rn(w, z))),
            two(__fadd_rn(__fmul_rn(x, z), __fmul_rn(w, y))),
            two(__fadd_rn(__fmul_rn(x, y), __fmul_rn(w, z))),
            __fsub_rn(1.0f, two(__fadd_rn(__fmul_rn(x, x), __fmul_rn(z, z)))),
            two(__fsub_rn(__fmul_rn(y, z), __fmul_rn(w, x))),
            two(__fsub_rn(__fmul_rn(x, z), __fmul_rn(w, y))),
            two(__fadd_rn(__fmul_rn(y, z), __fmul_rn(w, x))),
            __fsub_rn(1.0f, two(__fadd_rn(__fmul_rn(x, x), __fmul_rn(y, y)))),
        };
        for (int c = 0; c < d.split_n; ++c) {
            const int j = base_child + c * n_child + (int)rank[2 * P_ + i] - 1;
            const float* zr = normals + 3LL * ((long long)c * n_split + r);
            const float smp[3] = {__fmul_rn(zr[0], s[0]), __fmul_rn(zr[1], s[1]), __fmul_rn(zr[2], s[2])};
            copy_gaussian(so, dn, i, j, param, np);
            copy_segments(so, dn, C, i, j, param, np);
            for (int k = 0; k < 3; ++k) {  // bmm(R, samples) + xyz
                float acc = __fmul_rn(R[3 * k], smp[0]);
                acc = __fmaf_rn(R[3 * k + 1], smp[1], acc);
                acc = __fmaf_rn(R[3 * k + 2], smp[2], acc);
                np[dn.off[0] + 3LL * j + k] = __fadd_rn(acc, param[so.off[0] + 3LL * i + k]);
                np[dn.off[3] + 3LL * j + k] = logf(__fmul_rn(s[k], d.inv_split_div));
            }
            zero_gaussian(dn, C, j, nm1);
            zero_gaussian(dn, C, j, nm2);
        }
    }
}


// ---- PLY rows <-> arena ----------------------------------------------------------
// One thread per (Gaussian, float).  rows_to_arena walks the arena floats of a
// Gaussian (k) and gathers its row column; arena_to_rows walks the row columns (f)
// and gathers the arena float, so the side that streams the most (the row store)
// is the coalesced one.
struct PlyMap {
    int K;                          // arena floats per Gaussian
    int F;                          // row floats
    int col[GSR_PLY_MAX_COLS];      // arena float k -> row column (-1: none)
    int inv[GSR_PLY_MAX_COLS];      // row column f -> arena float (-1: none)
    signed char blk[GSR_PLY_MAX_COLS];  // arena float k -> block
    unsigned char sub[GSR_PLY_MAX_COLS];  // arena float k -> index inside the Gaussian's block row
    int width[GSR_ARENA_BLOCKS];
};

__global__ void __launch_bounds__(TR_THREADS) k_ply_rows_to_arena(ArenaMap am, PlyMap pm, int n, int dst,
                                                                  const float* __restrict__ rows,
                                                                  float* __restrict__ param) {
    const long long t = (long long)blockIdx.x * TR_THREADS + threadIdx.x;
    if (t >= (long long)n * pm.K) return;
    const int i = (int)(t / pm.K), k = (int)(t % pm.K);
    const int c = pm.col[k];
    const float v = c >= 0 ? rows[(long long)i * pm.F + c] : 0.0f;
    const int b = pm.blk[k];
    param[am.off[b] + (long long)(dst + i) * pm.width[b] + pm.sub[k]] = v;
}

__global__ void __launch_bounds__(TR_THREADS) k_arena_to_ply_rows(ArenaMap am, PlyMap pm, int P,
                                                                  const float* __restrict__ param,
                                                                  float* __restrict__ rows) {
    const long long t = (long long)blockIdx.x * TR_THREADS + threadIdx.x;
    if (t >= (long long)P * pm.F) return;
    const int i = (int)(t / pm.F), f = (int)(t % pm.F);
    const int k = pm.inv[f];
    float v = 0.0f;
    if (k >= 0) {
        const int b = pm.blk[k];
        v = param[am.off[b] + (long long)i * pm.width[b] + pm.sub[k]];
    }
    rows[t] = v;
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


GSR_API size_t gsr_densify_ws_bytes(int P) { return densify_ws_size(P > 0 ? (size_t)P : 1); }

namespace {
DensifyK densify_k(const gsr_densify_args* a) {
    DensifyK d{};
    d.mode = a->mode;
    d.split_n = a->split_n;
    d.max_grad = a->max_grad;
    d.min_opacity = a->min_opacity;
    d.clone_max_scale = a->clone_max_scale;
    d.prune_max_scale = a->prune_max_scale;
    d.max_screen_size = a->max_screen_size;
    d.inv_split_div = 1.0f / a->split_divisor;
    return d;
}
}  // namespace

GSR_API int gsr_densify_plan(int P, int M, int C, const float* param, const float* act, const float* grad_accum,
                             const float* denom, const uint8_t* mask, const gsr_densify_args* a, void* ws,
                             int* counts, void* stream) {
    (void)param;
    if (int rc = check_sizes(P, M, C)) return rc;
    if (!a || !counts) return set_error("[gsr] gsr_densify_plan: null args/counts");
    if (a->mode < GSR_DENSIFY_AND_PRUNE || a->mode > GSR_SPLIT_ONLY) return set_error("[gsr] densify: bad mode");
    if (a->split_n < 1 || a->split_n > 16 || !(a->split_divisor > 0.0f))
        return set_error("[gsr] densify: split_n must be 1..16 with a positive divisor");
    for (int k = 0; k < 4; ++k) counts[k] = 0;
    if (P == 0) return 0;
    if (!ws) return set_error("[gsr] gsr_densify_plan: null workspace");
    if (a->mode == GSR_PRUNE_MASK ? !mask : (!act || !grad_accum || !denom))
        return set_error("[gsr] gsr_densify_plan: null input");
    hipStream_t st = (hipStream_t)stream;
    const ArenaMap am = arena_map(P, M, C);
    const DensifyWs w = densify_ws(P, ws);
    k_densify_classify<<<(P + TR_THREADS - 1) / TR_THREADS, TR_THREADS, 0, st>>>(am, P, densify_k(a), act,
                                                                                grad_accum, denom, mask, w.cat);
    for (int k = 0; k < 4; ++k)
        launch_scan_inclusive_gather(w.cat + (size_t)k * P, nullptr, w.rank + (size_t)k * P, P, w.scan[k],
                                     /*ws_zeroed=*/false, st, nullptr);
    k_densify_totals<<<1, 64, 0, st>>>(w.rank, P, w.totals);
    uint32_t host[4] = {0, 0, 0, 0};
    hipError_t e = hipMemcpyAsync(host, w.totals, sizeof(host), hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    if (e != hipSuccess) return set_error(std::string("[gsr] densify plan: ") + hipGetErrorString(e));
    const long long np = (long long)host[0] + host[1] + (long long)a->split_n * host[2];
    if (np >= (1LL << 31)) return set_error("[gsr] densify: result too large");
    for (int k = 0; k < 4; ++k) counts[k] = (int)host[k];
    return 0;
}

GSR_API int gsr_densify_apply(int P, int M, int C, const float* param, const float* act, const float* exp_avg,
                              const float* exp_avg_sq, const gsr_densify_args* a, const void* ws, const int* counts,
                              const float* normals, float* new_param, float* new_exp_avg, float* new_exp_avg_sq,
                              void* stream) {
    if (int rc = check_sizes(P, M, C)) return rc;
    if (!a || !counts) return set_error("[gsr] gsr_densify_apply: null args/counts");
    const long long np = (long long)counts[0] + counts[1] + (long long)a->split_n * counts[2];
    if (int rc = check_sizes((int)np, M, C)) return rc;
    if (P == 0 || np == 0) return 0;
    if (!ws || !param || !act || !exp_avg || !exp_avg_sq || !new_param || !new_exp_avg || !new_exp_avg_sq)
        return set_error("[gsr] gsr_densify_apply: null buffer");
    if (counts[2] > 0 && !normals) return set_error("[gsr] gsr_densify_apply: split children need normals");
    hipStream_t st = (hipStream_t)stream;
    const ArenaMap so = arena_map(P, M, C), dn = arena_map((int)np, M, C);
    const DensifyWs w = densify_ws(P, const_cast<void*>(ws));
    k_densify_apply<<<(P + TR_THREADS - 1) / TR_THREADS, TR_THREADS, 0, st>>>(
        so, dn, P, C, densify_k(a), counts[0], counts[0] + counts[1], counts[2], counts[3], w.cat, w.rank, param, act,
        exp_avg, exp_avg_sq, normals, new_param, new_exp_avg, new_exp_avg_sq);
    return launched("densify_apply");
}


namespace {
int ply_map(int M, int C, int row_floats, const int* col, PlyMap& pm) {
    const int K = 3 + 3 * M + 1 + 3 + 4 + C;
    if (K > GSR_PLY_MAX_COLS || row_floats <= 0 || row_floats > GSR_PLY_MAX_COLS || !col)
        return set_error("[gsr] ply: too many columns or no column map");
    pm.K = K;
    pm.F = row_floats;
    const int widths[GSR_ARENA_BLOCKS] = {3, 3 * M, 1, 3, 4, C};
    for (int f = 0; f < GSR_PLY_MAX_COLS; ++f) pm.inv[f] = -1;
    int k = 0;
    for (int b = 0; b < GSR_ARENA_BLOCKS; ++b) {
        pm.width[b] = widths[b];
        for (int j = 0; j < widths[b]; ++j, ++k) {
            const int c = col[k];
            if (c >= row_floats) return set_error("[gsr] ply: column index out of range");
            pm.col[k] = c < 0 ? -1 : c;
            pm.blk[k] = (signed char)b;
            pm.sub[k] = (unsigned char)j;
            if (c >= 0) {
                if (pm.inv[c] >= 0) return set_error("[gsr] ply: a row column is mapped twice");
                pm.inv[c] = k;
            }
        }
    }
    return 0;
}
}  // namespace

GSR_API int gsr_ply_rows_to_arena(int n, int row_floats, const float* rows, const int* col, int P, int M, int C,
                                  int dst, float* param, void* stream) {
    if (int rc = check_sizes(P, M, C)) return rc;
    if (n < 0 || dst < 0 || (long long)dst + n > P) return set_error("[gsr] ply: rows do not fit the arena");
    if (n == 0) return 0;
    if (!rows || !param) return set_error("[gsr] ply: null buffer");
    PlyMap pm;
    if (int rc = ply_map(M, C, row_floats, col, pm)) return rc;
    const long long items = (long long)n * pm.K;
    k_ply_rows_to_arena<<<(unsigned)((items + TR_THREADS - 1) / TR_THREADS), TR_THREADS, 0, (hipStream_t)stream>>>(
        arena_map(P, M, C), pm, n, dst, rows, param);
    return launched("ply_rows_to_arena");
}

GSR_API int gsr_arena_to_ply_rows(int P, int M, int C, const float* param, int row_floats, const int* col,
                                  float* rows, void* stream) {
    if (int rc = check_sizes(P, M, C)) return rc;
    if (P == 0) return 0;
    if (!rows || !param) return set_error("[gsr] ply: null buffer");
    PlyMap pm;
    if (int rc = ply_map(M, C, row_floats, col, pm)) return rc;
    const long long items = (long long)P * pm.F;
    k_arena_to_ply_rows<<<(unsigned)((items + TR_THREADS - 1) / TR_THREADS), TR_THREADS, 0, (hipStream_t)stream>>>(
        arena_map(P, M, C), pm, P, param, rows);
    return launched("arena_to_ply_rows");
}

}  // extern "C"
