// render.hip -- per-tile front-to-back alpha compositing (forward) and its
// back-to-front replay (backward).  Reference: DGR/cuda_rasterizer/
// forward.cu:258-392 (renderCUDA) and backward.cu:414-639 (renderCUDA bwd).
//
// MI355X mapping: ONE wave64 per 16x16 tile, 4 pixels per lane (lane l owns
// column l&15 of rows (l>>4) + 4k, k = 0..3).  Per batch of 64 sorted
// instances each lane fetches one 64-B record with three 16-B loads; the blend
// loop then broadcasts record j to the wave with v_readlane (scalar operands,
// no LDS, no block barriers).  Early termination is a wave ballot.
//
// Backward: instead of the reference's 12 float atomics per (pixel, Gaussian)
// pair, each lane first sums its 4 pixels in registers, the wave reduces the 12
// gradient channels with a transposed butterfly (14 cross-lane moves for 12
// values), and 12 lanes store ONE 48-B record per (tile, Gaussian) instance at
// the instance's slot.  The per-Gaussian backward kernel sums a Gaussian's
// slots in fixed order: deterministic, atomic-free gradients.
#include "gsr_internal.h"

// Numerics.  The blend thresholds alpha >= 1/255 and T*(1-alpha) >= 1e-4
// (forward.cu:352-359) make n_contrib and every contribution knife-edge
// sensitive to exp(): the full-precision expf (ocml, ~1 ulp, like the
// reference's CUDA expf) keeps threshold flips against the oracle to ~0 on the
// parity scenes, where __expf (v_exp_f32 of x*log2e, several ulp at |x|~5)
// flipped about one pair per 10^7.  GSR_FAST_EXP selects the fast form.
// The forward blend keeps FMA contraction (errors ~2e-7); the backward replay
// runs with contraction off so its long recurrences (T /= 1-alpha, accum_rec)
// round like the reference's sequential code.
#ifdef GSR_FAST_EXP
#define GSR_EXP(x) __expf(x)
#else
#define GSR_EXP(x) expf(x)
#endif

namespace gsr {
namespace {

__device__ __forceinline__ float bcast(float v, int j) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), j));
}
__device__ __forceinline__ uint32_t bcast_u(uint32_t v, int j) {
    return (uint32_t)__builtin_amdgcn_readlane((int)v, j);
}

constexpr float ALPHA_MIN = 1.0f / 255.0f;  // forward.cu:352
constexpr float T_MIN = 0.0001f;            // forward.cu:355

__global__ void __launch_bounds__(64) k_render_fwd(int W, int H, int gx, const uint2* __restrict__ ranges,
                                                   const uint32_t* __restrict__ point_list,
                                                   const float4* __restrict__ rec, const float* __restrict__ bg,
                                                   float* __restrict__ out_color, float* __restrict__ out_depth,
                                                   float* __restrict__ out_alpha, float* __restrict__ out_segment,
                                                   uint32_t* __restrict__ n_contrib) {
    const int tile = blockIdx.x;
    const int lane = threadIdx.x;
    const int tx = tile % gx, ty = tile / gx;
    const int px = tx * BX + (lane & 15);
    const int py0 = ty * BY + (lane >> 4);
    const float pfx = (float)px;
    float pfy[4], T[4], C0[4], C1[4], C2[4], S0[4], S1[4], Dp[4], Wt[4];
    uint32_t last[4];
    bool done[4], inside[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int py = py0 + 4 * k;
        pfy[k] = (float)py;
        inside[k] = px < W && py < H;
        done[k] = !inside[k];
        T[k] = 1.0f;
        C0[k] = C1[k] = C2[k] = S0[k] = S1[k] = Dp[k] = Wt[k] = 0.f;
        last[k] = 0;
    }
    const uint2 range = ranges[tile];
    const int n = (int)(range.y - range.x);

    for (int base = 0; base < n; base += 64) {
        if (!__any(!(done[0] && done[1] && done[2] && done[3]))) break;
        const int cnt = min(64, n - base);
        float4 ra = make_float4(0.f, 0.f, 0.f, 0.f), rb = ra, rc = ra;
        if (lane < cnt) {
            const uint32_t g = point_list[range.x + base + lane];
            const float4* R = rec + (size_t)g * REC_F4;
            ra = R[0];
            rb = R[1];
            rc = R[2];
        }
        for (int j = 0; j < cnt; ++j) {
            const float gx_ = bcast(ra.x, j), gy_ = bcast(ra.y, j);
            const float ca = bcast(ra.z, j), cb = bcast(ra.w, j), cc = bcast(rb.x, j), op = bcast(rb.y, j);
            bool ok[4];
            float alpha[4];
            bool any_ok = false;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const float dx = gx_ - pfx, dy = gy_ - pfy[k];
                const float power = -0.5f * (ca * dx * dx + cc * dy * dy) - cb * dx * dy;
                alpha[k] = fminf(0.99f, op * GSR_EXP(power));
                bool o = !done[k] && power <= 0.0f && alpha[k] >= ALPHA_MIN;
                const float test_T = T[k] * (1.f - alpha[k]);
                const bool term = o && test_T < T_MIN;
                done[k] = done[k] || term;
                ok[k] = o && !term;
                any_ok = any_ok || ok[k];
            }
            if (!__any(any_ok)) continue;
            const float dep = bcast(rb.z, j), s0 = bcast(rb.w, j);
            const float cr = bcast(rc.x, j), cg = bcast(rc.y, j), cbl = bcast(rc.z, j), s1 = bcast(rc.w, j);
            const uint32_t contributor = (uint32_t)(base + j + 1);
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const float a = ok[k] ? alpha[k] : 0.f;
                const float aT = a * T[k];
                C0[k] += cr * a * T[k];
                C1[k] += cg * a * T[k];
                C2[k] += cbl * a * T[k];
                Wt[k] += aT;
                Dp[k] += dep * a * T[k];
                S0[k] += s0 * a * T[k];
                S1[k] += s1 * a * T[k];
                T[k] = ok[k] ? T[k] * (1.f - alpha[k]) : T[k];
                last[k] = ok[k] ? contributor : last[k];
            }
        }
    }
    const float bg0 = bg[0], bg1 = bg[1], bg2 = bg[2];
    const size_t HW = (size_t)H * W;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        n_contrib[(size_t)tile * TILE_PIX + k * 64 + lane] = last[k];
        if (!inside[k]) continue;
        const size_t pix = (size_t)(py0 + 4 * k) * W + px;
        out_color[pix] = C0[k] + T[k] * bg0;
        out_color[HW + pix] = C1[k] + T[k] * bg1;
        out_color[2 * HW + pix] = C2[k] + T[k] * bg2;
        out_alpha[pix] = Wt[k];
        out_depth[pix] = Dp[k];
        out_segment[pix] = S0[k];
        out_segment[HW + pix] = S1[k];
    }
}

// Transposed butterfly: v[12] per lane -> the wave-wide sum of channel vidx in
// every lane with (lane & 3) == 0 && valid.
__device__ __forceinline__ float wave_reduce12(float v[12], int lane, int& vidx, bool& valid) {
    const bool h32 = lane & 32, h16 = lane & 16, h8 = lane & 8, h4 = lane & 4;
#pragma unroll
    for (int i = 0; i < 6; ++i) {
        const float send = h32 ? v[i] : v[i + 6];
        const float keep = h32 ? v[i + 6] : v[i];
        v[i] = keep + __shfl_xor(send, 32, 64);
    }
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        const float send = h16 ? v[i] : v[i + 3];
        const float keep = h16 ? v[i + 3] : v[i];
        v[i] = keep + __shfl_xor(send, 16, 64);
    }
    v[3] = 0.f;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const float send = h8 ? v[i] : v[i + 2];
        const float keep = h8 ? v[i + 2] : v[i];
        v[i] = keep + __shfl_xor(send, 8, 64);
    }
    {
        const float send = h4 ? v[0] : v[1];
        const float keep = h4 ? v[1] : v[0];
        v[0] = keep + __shfl_xor(send, 4, 64);
    }
    float r = v[0];
    r += __shfl_xor(r, 2, 64);
    r += __shfl_xor(r, 1, 64);
    const int w = (h8 ? 2 : 0) + (h4 ? 1 : 0);
    vidx = (h32 ? 6 : 0) + (h16 ? 3 : 0) + w;
    valid = ((lane & 3) == 0) && w < 3;
    return r;
}

__global__ void __launch_bounds__(64) k_render_bwd(int W, int H, int gx, const uint2* __restrict__ ranges,
                                                   const uint32_t* __restrict__ point_list,
                                                   const uint32_t* __restrict__ slot_vals,
                                                   const float4* __restrict__ rec, const float* __restrict__ bg,
                                                   const float* __restrict__ alphas,
                                                   const uint32_t* __restrict__ n_contrib,
                                                   const float* __restrict__ dL_dpixels,
                                                   const float* __restrict__ dL_dsegs,
                                                   const float* __restrict__ dL_ddepths,
                                                   const float* __restrict__ dL_dalphas,
                                                   float* __restrict__ contrib) {
#pragma clang fp contract(off)
    const int tile = blockIdx.x;
    const int lane = threadIdx.x;
    const int tx = tile % gx, ty = tile / gx;
    const int px = tx * BX + (lane & 15);
    const int py0 = ty * BY + (lane >> 4);
    const float pfx = (float)px;
    const size_t HW = (size_t)H * W;
    const float bg0 = bg[0], bg1 = bg[1], bg2 = bg[2];

    float pfy[4], T[4], Tfin[4], dp0[4], dp1[4], dp2[4], ds0[4], ds1[4], dd[4], da[4], bgdot[4];
    float ar0[4], ar1[4], ar2[4], as0[4], as1[4], ad[4], aa[4], la[4], lc0[4], lc1[4], lc2[4], ls0[4], ls1[4],
        ld[4];
    uint32_t lastc[4];
    uint32_t maxlast = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int py = py0 + 4 * k;
        pfy[k] = (float)py;
        const bool inside = px < W && py < H;
        const size_t pix = (size_t)py * W + px;
        lastc[k] = inside ? n_contrib[(size_t)tile * TILE_PIX + k * 64 + lane] : 0u;
        Tfin[k] = inside ? 1.f - alphas[pix] : 0.f;
        T[k] = Tfin[k];
        dp0[k] = inside ? dL_dpixels[pix] : 0.f;
        dp1[k] = inside ? dL_dpixels[HW + pix] : 0.f;
        dp2[k] = inside ? dL_dpixels[2 * HW + pix] : 0.f;
        ds0[k] = inside ? dL_dsegs[pix] : 0.f;
        ds1[k] = inside ? dL_dsegs[HW + pix] : 0.f;
        dd[k] = inside ? dL_ddepths[pix] : 0.f;
        da[k] = inside ? dL_dalphas[pix] : 0.f;
        float bgd = 0.f;
        bgd += bg0 * dp0[k];
        bgd += bg1 * dp1[k];
        bgd += bg2 * dp2[k];
        bgdot[k] = bgd;
        ar0[k] = ar1[k] = ar2[k] = as0[k] = as1[k] = ad[k] = aa[k] = 0.f;
        la[k] = lc0[k] = lc1[k] = lc2[k] = ls0[k] = ls1[k] = ld[k] = 0.f;
        maxlast = max(maxlast, lastc[k]);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) maxlast = max(maxlast, (uint32_t)__shfl_xor((int)maxlast, o, 64));
    const bool use_bg = __any(bgdot[0] != 0.f || bgdot[1] != 0.f || bgdot[2] != 0.f || bgdot[3] != 0.f);

    const uint2 range = ranges[tile];
    const int n = (int)(range.y - range.x);
    const float ddelx_dx = 0.5f * W, ddely_dy = 0.5f * H;

    // Instances behind every pixel's last contributor carry no gradient.
    for (int p = (int)maxlast + lane; p < n; p += 64) {
        float4* dst = reinterpret_cast<float4*>(contrib + (size_t)slot_vals[range.x + p] * 12);
        const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
        dst[0] = z;
        dst[1] = z;
        dst[2] = z;
    }

    for (int top = (int)maxlast; top > 0; top -= 64) {
        const int cnt = min(64, top);
        float4 ra = make_float4(0.f, 0.f, 0.f, 0.f), rb = ra, rc = ra;
        uint32_t uslot = 0;
        if (lane < cnt) {
            const uint32_t kidx = range.x + (uint32_t)(top - 1 - lane);
            const uint32_t g = point_list[kidx];
            uslot = slot_vals[kidx];
            const float4* R = rec + (size_t)g * REC_F4;
            ra = R[0];
            rb = R[1];
            rc = R[2];
        }
        for (int j = 0; j < cnt; ++j) {
            const uint32_t p = (uint32_t)(top - 1 - j);
            const uint32_t u = bcast_u(uslot, j);
            float* dst = contrib + (size_t)u * 12;
            const float gx_ = bcast(ra.x, j), gy_ = bcast(ra.y, j);
            const float ca = bcast(ra.z, j), cb = bcast(ra.w, j), cc = bcast(rb.x, j), op = bcast(rb.y, j);
            bool ok[4];
            float G[4], alpha[4], dxs[4], dys[4];
            bool any_ok = false;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const float dx = gx_ - pfx, dy = gy_ - pfy[k];
                dxs[k] = dx;
                dys[k] = dy;
                const float power = -0.5f * (ca * dx * dx + cc * dy * dy) - cb * dx * dy;
                G[k] = GSR_EXP(power);
                alpha[k] = fminf(0.99f, op * G[k]);
                ok[k] = p < lastc[k] && power <= 0.0f && alpha[k] >= ALPHA_MIN;
                any_ok = any_ok || ok[k];
            }
            if (!__any(any_ok)) {
                if (lane < 12) dst[lane] = 0.f;
                continue;
            }
            const float dep = bcast(rb.z, j), s0 = bcast(rb.w, j);
            const float c0 = bcast(rc.x, j), c1 = bcast(rc.y, j), c2 = bcast(rc.z, j), s1 = bcast(rc.w, j);
            float acc[12];
#pragma unroll
            for (int i = 0; i < 12; ++i) acc[i] = 0.f;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const bool o = ok[k];
                const float a = alpha[k];
                const float one_m = 1.f - a;
                const float Tn = o ? T[k] / one_m : T[k];
                T[k] = Tn;
                const float dch = a * Tn;
                // colour
                const float nar0 = la[k] * lc0[k] + (1.f - la[k]) * ar0[k];
                const float nar1 = la[k] * lc1[k] + (1.f - la[k]) * ar1[k];
                const float nar2 = la[k] * lc2[k] + (1.f - la[k]) * ar2[k];
                float dopa = 0.f;
                dopa += (c0 - nar0) * dp0[k];
                dopa += (c1 - nar1) * dp1[k];
                dopa += (c2 - nar2) * dp2[k];
                // segment
                const float nas0 = la[k] * ls0[k] + (1.f - la[k]) * as0[k];
                const float nas1 = la[k] * ls1[k] + (1.f - la[k]) * as1[k];
                dopa += (s0 - nas0) * ds0[k];
                dopa += (s1 - nas1) * ds1[k];
                // depth
                const float nad = la[k] * ld[k] + (1.f - la[k]) * ad[k];
                dopa += (dep - nad) * dd[k];
                // alpha (weight sum)
                const float naa = la[k] + (1.f - la[k]) * aa[k];
                dopa += (1.f - naa) * da[k];
                dopa *= Tn;
                if (use_bg) dopa += (-Tfin[k] / one_m) * bgdot[k];
                const float dL_dG = op * dopa;
                const float gdx = G[k] * dxs[k], gdy = G[k] * dys[k];
                const float dG_ddelx = -gdx * ca - gdy * cb;
                const float dG_ddely = -gdy * cc - gdx * cb;
                if (o) {
                    acc[0] += dch * dp0[k];
                    acc[1] += dch * dp1[k];
                    acc[2] += dch * dp2[k];
                    acc[3] += dch * ds0[k];
                    acc[4] += dch * ds1[k];
                    acc[5] += dch * dd[k];
                    acc[6] += dL_dG * dG_ddelx * ddelx_dx;
                    acc[7] += dL_dG * dG_ddely * ddely_dy;
                    acc[8] += -0.5f * gdx * dxs[k] * dL_dG;
                    acc[9] += -0.5f * gdx * dys[k] * dL_dG;
                    acc[10] += -0.5f * gdy * dys[k] * dL_dG;
                    acc[11] += G[k] * dopa;
                    ar0[k] = nar0; ar1[k] = nar1; ar2[k] = nar2;
                    as0[k] = nas0; as1[k] = nas1;
                    ad[k] = nad;
                    aa[k] = naa;
                    lc0[k] = c0; lc1[k] = c1; lc2[k] = c2;
                    ls0[k] = s0; ls1[k] = s1;
                    ld[k] = dep;
                    la[k] = a;
                }
            }
            int vidx;
            bool valid;
            const float r = wave_reduce12(acc, lane, vidx, valid);
            if (valid) dst[vidx] = r;
        }
    }
}

}  // namespace

void launch_render_forward(int W, int H, int gx, int gy, const uint2* ranges, const uint32_t* point_list,
                           const float4* rec, const float* bg, float* out_color, float* out_depth, float* out_alpha,
                           float* out_segment, uint32_t* n_contrib, hipStream_t st) {
    const int T = gx * gy;
    if (T == 0) return;
    hipLaunchKernelGGL(k_render_fwd, dim3(T), dim3(64), 0, st, W, H, gx, ranges, point_list, rec, bg, out_color,
                       out_depth, out_alpha, out_segment, n_contrib);
}

void launch_render_backward(int W, int H, int gx, int gy, const uint2* ranges, const uint32_t* point_list,
                            const uint32_t* slot_vals, const float4* rec, const float* bg, const float* alpha,
                            const uint32_t* n_contrib, const float* dL_dcolor, const float* dL_dsegment,
                            const float* dL_ddepth, const float* dL_dalpha, float* contrib, hipStream_t st) {
    const int T = gx * gy;
    if (T == 0) return;
    hipLaunchKernelGGL(k_render_bwd, dim3(T), dim3(64), 0, st, W, H, gx, ranges, point_list, slot_vals, rec, bg,
                       alpha, n_contrib, dL_dcolor, dL_dsegment, dL_ddepth, dL_dalpha, contrib);
}

}  // namespace gsr
