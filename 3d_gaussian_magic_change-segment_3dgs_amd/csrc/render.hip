// render.hip -- per-tile front-to-back alpha compositing (forward) and its
// back-to-front replay (backward).  Reference: DGR/cuda_rasterizer/
// forward.cu:258-392 (renderCUDA) and backward.cu:414-639 (renderCUDA bwd).
//
// MI355X mapping: ONE wave64 per 16x16 tile, 4 pixels per lane.  Forward: lane l
// owns pixel (l&7, l>>3) of each 8x8 quadrant k of the tile (quadrant-gated);
// backward: lane l owns column l&15 of rows (l>>4) + 4k, k = 0..3 (16x4 strips, one
// dx per lane for the moment sums).  Per batch of 64 sorted instances each lane
// fetches one 64-B record with three 16-B loads (two-stage prefetch); the batch is
// parked in LDS and the blend loop reads record j with a wave-uniform broadcast
// ds_read (no v_readlane, no block barriers: one wave per block).  Early
// termination is tracked as per-quadrant live masks in SGPRs (ballots).
//
// Per pair, the four pixel "powers" are computed first and compared with the
// Gaussian's log-space opacity threshold ln(1/(255*o)) (minus a 1e-3 guard):
// when no pixel of the tile can reach alpha >= 1/255 the pair is skipped
// before any exp().  Pairs that pass are decided with the exact test of the
// reference (alpha >= 1/255 with the blend exp below), so the skip never changes a
// result.
//
// Backward: instead of the reference's 12 float atomics per (pixel, Gaussian)
// pair, each lane sums its 4 pixels in registers, the wave reduces the 12
// gradient channels with a transposed butterfly on v_permlane32_swap /
// v_permlane16_swap / DPP (34 VALU ops, no LDS round trips), and 12 lanes
// store ONE 48-B record per replayed (tile, Gaussian) instance at the
// instance's slot and set the slot's byte in a written-flag array.  Instances that no
// pixel replays (behind every last contributor, or out of reach) write nothing.
// The per-Gaussian backward kernel sums a Gaussian's written slots in slot
// order: deterministic, atomic-free gradients.  Record (q = G * dL_dalpha per pixel,
// d = (dx, dy) = mean2D - pixel):
//   [sum dch*dL_dcolor.rgb, sum dch*dL_dseg0/1, sum dch*dL_ddepth,
//    sum q, sum q dx, sum q dy, sum q dx^2, sum q dx dy, sum q dy^2]
// from which k_gaussian_backward forms dopacity = sum q and the reference's
// mean2D / conic gradients with the Gaussian's own conic and opacity.
#include "gsr_internal.h"

#include <type_traits>

// Numerics.  The blend thresholds alpha >= 1/255 and T*(1-alpha) >= 1e-4
// (forward.cu:352-359) make n_contrib and every contribution knife-edge
// sensitive to exp(), and the reference's backward recovers T from
// T_final = 1 - sum(alpha*T) (backward.cu:468), amplifying any last-ulp alpha
// difference by 1/T_final.  gsr therefore evaluates exp() with gsr_expf below:
// IEEE operations only (fma, add, mul, integer shift), so the CPU oracle computes the
// very same bits (oracle/gsr_oracle.cpp: gsr_expf).  Max error 0.88 ulp,
// correctly rounded on 99.53% of inputs (tests/test_oracle_golden.py pins it
// against double-precision exp; the reference's CUDA expf is specified at 2 ulp).
// GSR_FAST_EXP selects __expf (v_exp_f32, several ulp) for experiments.
// power, alpha, T and the weight sum run without FMA contraction (see the
// kernels); only non-amplified sums use explicit FMAs.
__device__ __forceinline__ float gsr_expf(float x) {
    // exp(clamp(x, -87, 88)).  k = round(x log2 e) via the 1.5*2^23 shifter (one FMA,
    // the integer lands in the low mantissa bits), Cody-Waite ln2 = hi + lo, degree-6
    // minimax polynomial on [-ln2/2, ln2/2] (1 + r + c2 r^2 + ... + c6 r^6, fp32
    // coefficients, Horner with FMAs), then times 2^k assembled from the shifter's
    // bits (k in [-126, 127], so the product is an exact scaling).  Outside the clamp
    // the value is meaningless for blending anyway: alpha < 1/255 below -87 and the
    // blend rejects power > 0.  Exhaustive check over every fp32 in [-87, 0]: max 0.88
    // ulp, correctly rounded on 99.53% (the degree-7 Taylor form it replaced: 0.94 ulp).
    const float xc = __builtin_amdgcn_fmed3f(x, -87.0f, 88.0f);
    const float kf = __builtin_fmaf(xc, 1.44269502f, 12582912.0f);
    const float k = kf - 12582912.0f;
    float r = __builtin_fmaf(-k, 0.693145751953125f, xc);
    r = __builtin_fmaf(-k, 1.42860677e-06f, r);
    float p = 0.001381461275741458f;
    p = __builtin_fmaf(p, r, 0.008368710055947304f);
    p = __builtin_fmaf(p, r, 0.04166838899254799f);
    p = __builtin_fmaf(p, r, 0.1666652113199234f);
    p = __builtin_fmaf(p, r, 0.4999999403953552f);
    p = __builtin_fmaf(p, r, 1.0f);
    p = __builtin_fmaf(p, r, 1.0f);
    const float scale = __uint_as_float((__float_as_uint(kf) << 23) + 0x3f800000u);
    return p * scale;
}
// gsr_expf without the clamp, for lanes whose argument is known to lie in [-87, 88]: the
// blend loops call it only under a lane mask of pixels with power >= the Gaussian's
// opacity floor (>= -5.6) and use the result only under that mask (other lanes get a
// meaningless, possibly non-finite value that every use masks out).  Same bits as
// gsr_expf on that range.
__device__ __forceinline__ float gsr_expf_nc(float x) {
    const float kf = __builtin_fmaf(x, 1.44269502f, 12582912.0f);
    const float k = kf - 12582912.0f;
    float r = __builtin_fmaf(-k, 0.693145751953125f, x);
    r = __builtin_fmaf(-k, 1.42860677e-06f, r);
    float p = 0.001381461275741458f;
    p = __builtin_fmaf(p, r, 0.008368710055947304f);
    p = __builtin_fmaf(p, r, 0.04166838899254799f);
    p = __builtin_fmaf(p, r, 0.1666652113199234f);
    p = __builtin_fmaf(p, r, 0.4999999403953552f);
    p = __builtin_fmaf(p, r, 1.0f);
    p = __builtin_fmaf(p, r, 1.0f);
    const float scale = __uint_as_float((__float_as_uint(kf) << 23) + 0x3f800000u);
    return p * scale;
}
#ifdef GSR_FAST_EXP
#define GSR_EXP(x) __expf(x)
#define GSR_EXP_NC(x) __expf(x)
#else
#define GSR_EXP(x) gsr_expf(x)
#define GSR_EXP_NC(x) gsr_expf_nc(x)
#endif

#ifdef GSR_STATS
// Instrumented build (tools/render_stats.py): wave-uniform loop counters, 16 per
// kernel (fwd at 0, bwd at 16): 0 visited, 1 near-skip, 2 prefiltered out, 3 full,
// 4 ok pixels, 5 batches, 6 zero-tail (bwd), 7 instances, 8 strips processed.
__device__ unsigned long long g_gsr_stats[32];
extern "C" __attribute__((visibility("default"))) int gsr_stats_read(unsigned long long* host, int reset) {
    if (hipMemcpyFromSymbol(host, HIP_SYMBOL(g_gsr_stats), sizeof(g_gsr_stats)) != hipSuccess) return -1;
    if (reset) {
        unsigned long long z[32] = {};
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_gsr_stats), z, sizeof(z)) != hipSuccess) return -1;
    }
    return 0;
}
#define STAT_DECL unsigned long long st_[16] = {};
#define STAT(i, v) (st_[i] += (v))
#define STAT_FLUSH(off)                                                          \
    if (threadIdx.x == 0)                                                        \
        for (int i_ = 0; i_ < 16; ++i_) atomicAdd(&g_gsr_stats[(off) + i_], st_[i_]);
#define POPC(a) __popcll(__ballot(a))
#else
#define STAT_DECL
#define STAT(i, v)
#define STAT_FLUSH(off)
#define POPC(a) 0
#endif

#ifdef GSR_WAVE_TRACE
// Timeline build (tools/wave_trace.py): per wave of the last launch of each render
// kernel, {start, end} of s_memrealtime (100 MHz, chip-wide), the tile, its list length
// and the last list position the wave visits, and the wave's HW_ID.
__device__ unsigned long long g_gsr_wtrace[2][32768][4];
extern "C" __attribute__((visibility("default"))) int gsr_wave_trace_read(unsigned long long* host) {
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_gsr_wtrace), sizeof(g_gsr_wtrace)) == hipSuccess ? 0 : -1;
}
#define WT_BEGIN const unsigned long long wt0_ = __builtin_amdgcn_s_memrealtime();
#define WT_END(kind, tile, n, depth)                                                                 \
    if (threadIdx.x == 0 && blockIdx.x < 32768) {                                                     \
        const unsigned long long wt1_ = __builtin_amdgcn_s_memrealtime();                             \
        unsigned long long* w_ = g_gsr_wtrace[kind][blockIdx.x];                                      \
        w_[0] = wt0_;                                                                                 \
        w_[1] = wt1_;                                                                                 \
        w_[2] = (unsigned long long)(tile) | ((unsigned long long)(unsigned)(n) << 32);               \
        w_[3] = (unsigned long long)((unsigned)(depth) & 0xffffffu) |                                 \
                ((unsigned long long)(__builtin_amdgcn_s_getreg((20) | (0 << 6) | (3 << 11)) & 15u) << 24) | \
                ((unsigned long long)__builtin_amdgcn_s_getreg((4) | (0 << 6) | (31 << 11)) << 32); \
    }
#else
#define WT_BEGIN
#define WT_END(kind, tile, n, depth)
#endif

namespace gsr {
namespace {

// Wave-wide "any": a ballot compared in SALU (HIP's __any materialises the
// predicate in a VGPR and compares it again on the VALU).
__device__ __forceinline__ bool wave_any(bool p) { return __builtin_amdgcn_ballot_w64(p) != 0; }

constexpr float ALPHA_MIN = 1.0f / 255.0f;  // forward.cu:352
constexpr float T_MIN = 0.0001f;            // forward.cu:355
constexpr float POWER_GUARD = 1e-3f;        // skip guard in ln-space (alpha factor e^-0.001)

// Lowest power at which o * exp(power) can still reach 1/255 (minus the guard).
__device__ __forceinline__ float power_floor(float opacity) {
#ifdef GSR_NO_SKIP
    return -INFINITY;
#endif
    return -__logf(255.0f * opacity) - POWER_GUARD;
}

// Batch fetch: lane l loads the 48 B of one instance's record.  Loads are issued
// unconditionally (callers clamp list positions into the tile's list, so g is always
// a valid id): with no branch around them the number of loads in flight is static
// and the waitcnt before the current batch's first use leaves the prefetched batch
// in flight (a predicated load makes the compiler fall back to vmcnt(0)).
struct Batch {
    float4 a, b, c;
};
__device__ __forceinline__ Batch fetch_batch(const float4* __restrict__ rec, uint32_t g) {
    const float4* R = rec + (size_t)g * REC_F4;
    return Batch{R[0], R[1], R[2]};
}

// Lane-parallel batch prefilter: can ANY pixel centre of the tile rectangle
// [x0,x1] x [y0,y1] reach power >= pm for the Gaussian (x, y, conic a, b, c)?
// power = -q/2 with q(u,v) = a u^2 + 2 b u v + c v^2 convex (a, c, det > 0), so the
// minimum of q over the rectangle is 0 when the centre lies inside, otherwise on
// one of the four edges, where it is a 1-D quadratic minimised in closed form.
// The test is conservative: the margin covers fp32 rounding of the terms, and a
// non-convex conic always passes.  Skipping a Gaussian here only avoids work that
// the exact per-pixel tests of the blend loop would have rejected.
__device__ __forceinline__ bool tile_hit(float x, float y, float a, float b, float c, float pm, float x0,
                                         float x1, float y0, float y1) {
    if (!(a > 0.f && c > 0.f && a * c > b * b)) return true;
    const float ul = x0 - x, uh = x1 - x, vl = y0 - y, vh = y1 - y;
    const float ra = __builtin_amdgcn_rcpf(a), rc = __builtin_amdgcn_rcpf(c);
    auto q = [&](float u, float v) { return (a * u + 2.f * b * v) * u + c * v * v; };
    const float v_l = fminf(fmaxf(-b * ul * rc, vl), vh), v_h = fminf(fmaxf(-b * uh * rc, vl), vh);
    const float u_l = fminf(fmaxf(-b * vl * ra, ul), uh), u_h = fminf(fmaxf(-b * vh * ra, ul), uh);
    float qmin = fminf(fminf(q(ul, v_l), q(uh, v_h)), fminf(q(u_l, vl), q(u_h, vh)));
    const bool inside = ul <= 0.f && uh >= 0.f && vl <= 0.f && vh >= 0.f;
    qmin = inside ? 0.f : qmin;
    const float U = fmaxf(-ul, uh), V = fmaxf(-vl, vh);
    const float margin = 1e-2f + 1e-5f * (a * U * U + 2.f * fabsf(b) * U * V + c * V * V);
    return qmin <= -2.f * pm + margin;
}

__global__ void __launch_bounds__(64) k_render_fwd(int W, int H, int gx, const uint32_t* __restrict__ order,
                                                   const uint2* __restrict__ ranges,
                                                   const uint32_t* __restrict__ point_list,
                                                   const float4* __restrict__ rec, const float* __restrict__ bg,
                                                   float* __restrict__ out_color, float* __restrict__ out_depth,
                                                   float* __restrict__ out_alpha, float* __restrict__ out_segment,
                                                   uint32_t* __restrict__ n_contrib) {
    // The backward recovers T from T_final = 1 - sum(alpha*T) (backward.cu:468) and
    // divides back through every contributor, which amplifies a last-bit difference
    // in the weight sum by 1/T_final.  power, alpha, T and the weight sum are therefore
    // rounded exactly as the reference writes them (no contraction); only the
    // colour/depth/segment sums, which nothing amplifies, use explicit FMAs.
#pragma clang fp contract(off)
    WT_BEGIN
    const int tile = (int)order[blockIdx.x];
    const int lane = threadIdx.x;
    const int tx = tile % gx, ty = tile / gx;
    // Lane l owns pixel (l & 7, l >> 3) of each 8x8 quadrant k of the tile (k & 1: right
    // half, k >> 1: bottom half).  Square quadrants are gated tighter than 16x4 strips:
    // 8.7% fewer (quadrant, Gaussian) blends at the metric scene (tools/render_stats.py).
    const int px0 = tx * BX + (lane & 7), py0 = ty * BY + (lane >> 3);
    const float pfx[2] = {(float)px0, (float)(px0 + 8)};
    const float pfy[2] = {(float)py0, (float)(py0 + 8)};
    // live[k]: lanes whose pixel of quadrant k is inside the image and not terminated,
    // kept as a wave mask in SGPRs (no per-pair VALU compare); T stays at its value at
    // termination, which is the T the output uses (forward.cu:355-357 breaks before T).
    float T[4], C0[4], C1[4], C2[4], S0[4], S1[4], Dp[4], Wt[4];
    uint32_t last[4];
    uint64_t live[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int px = px0 + 8 * (k & 1), py = py0 + 8 * (k >> 1);
        live[k] = __builtin_amdgcn_ballot_w64(px < W && py < H);
        T[k] = 1.0f;
        C0[k] = C1[k] = C2[k] = S0[k] = S1[k] = Dp[k] = Wt[k] = 0.f;
        last[k] = 0;
    }
    const uint2 range = ranges[tile];
    const int n = (int)(range.y - range.x);
    STAT_DECL
    STAT(7, n);
    const float x0 = (float)(tx * BX), y0 = (float)(ty * BY);
    const float x1 = (float)min(tx * BX + BX - 1, W - 1), y1 = (float)min(ty * BY + BY - 1, H - 1);

    // Two-stage software pipeline over batches of 64 instances: while batch b is
    // blended, the records of batch b+1 and the ids of batch b+2 are in flight
    // (the id -> record dependency would otherwise stall every batch start).
    // The batch's records are parked in LDS and read back with a wave-uniform address
    // (a broadcast ds_read): the blend loop then spends no VALU issue slots on
    // v_readlane broadcasts.  One wave per block, so the barriers are free.
    __shared__ float4 srec[64][4];
    const uint32_t* plist = point_list + range.x;
    const int nlast = max(n - 1, 0);  // list positions are clamped to the last one
    uint32_t g_next = n > 0 ? plist[min(lane, nlast)] : 0u;
    Batch cur;
    if (n > 0) cur = fetch_batch(rec, g_next);
    if (n > 0) g_next = plist[min(64 + lane, nlast)];
    for (int base = 0; base < n; base += 64) {
        if (!(live[0] | live[1] | live[2] | live[3])) break;
        const int cnt = min(64, n - base);
        STAT(5, 1);
        const Batch nxt = fetch_batch(rec, g_next);
        g_next = plist[min(base + 128 + lane, nlast)];
        const float4 ra = cur.a, rb = cur.b, rc = cur.c;
        cur = nxt;
        const float pmin = power_floor(rb.y);
        uint64_t todo = __ballot(lane < cnt && tile_hit(ra.x, ra.y, ra.z, ra.w, rb.x, pmin, x0, x1, y0, y1));
        STAT(2, cnt - __popcll(todo));
        __syncthreads();  // previous batch's reads are done
        srec[lane][0] = ra;                                      // x, y, conic a, b
        srec[lane][1] = make_float4(rb.x, pmin, rb.y, rb.w);     // conic c, power floor, opacity, seg0
        srec[lane][2] = rc;                                      // r, g, b, seg1
        srec[lane][3] = make_float4(rb.z, 0.f, 0.f, 0.f);        // depth
        __syncthreads();
        while (todo) {
            const int j = (int)__builtin_ctzll(todo);
            todo &= todo - 1;
            const float4 q0 = srec[j][0], q1 = srec[j][1];
            const float gx_ = q0.x, gy_ = q0.y, ca = q0.z, cb = q0.w, cc = q1.x, pm = q1.y;
            // power = -0.5 (a dx dx + c dy dy) - b dx dy, rounded as forward.cu:349 writes
            // it; the products are shared by the two quadrants of a column / row.
            const float dx0 = gx_ - pfx[0], dx1 = gx_ - pfx[1];
            const float dy0 = gy_ - pfy[0], dy1 = gy_ - pfy[1];
            const float ax[2] = {ca * dx0 * dx0, ca * dx1 * dx1}, bx[2] = {cb * dx0, cb * dx1};
            const float cy[2] = {cc * dy0 * dy0, cc * dy1 * dy1}, dyv[2] = {dy0, dy1};
            float power[4];
            uint64_t near[4];  // per quadrant: live lanes within reach
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                // -0.5 S is exact, so -(0.5 S) - B as one fma(-0.5, S, -B): the same bits
                power[k] = __builtin_fmaf(-0.5f, ax[k & 1] + cy[k >> 1], -(bx[k & 1] * dyv[k >> 1]));
                near[k] = __builtin_amdgcn_ballot_w64(power[k] >= pm) & live[k];
            }
            STAT(0, 1);
            if (!(near[0] | near[1] | near[2] | near[3])) {
                STAT(1, 1);
                continue;
            }
            STAT(3, 1);
            const float4 q2 = srec[j][2], q3 = srec[j][3];
            const float op = q1.z, dep = q3.x, s0 = q1.w;
            const float cr = q2.x, cg = q2.y, cbl = q2.z, s1 = q2.w;
            // in a VGPR once per pair: the per-quadrant v_cndmask below may read only one SGPR
            // (its lane mask), so a scalar contributor would be re-moved into a VGPR per quadrant
            uint32_t contributor = (uint32_t)(base + j + 1);
            asm volatile("" : "+v"(contributor));
            // Quadrant k is blended only if one of its pixels can pass; the exact
            // reference tests below decide per pixel.
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                if (!near[k]) continue;
                STAT(8, 1);
                // lanes of near[k] (live, power >= the opacity floor) are the only ones that
                // can pass; every result below is used only under that mask
                const float alpha = fminf(0.99f, op * GSR_EXP_NC(power[k]));
                const uint64_t m_o = near[k] & __builtin_amdgcn_ballot_w64(power[k] <= 0.0f) &
                                     __builtin_amdgcn_ballot_w64(alpha >= ALPHA_MIN);
                const float test_T = T[k] * (1.f - alpha);
                const uint64_t m_done = m_o & __builtin_amdgcn_ballot_w64(test_T < T_MIN);  // forward.cu:355-357
                live[k] &= ~m_done;
                const bool ok = __builtin_amdgcn_inverse_ballot_w64(m_o & ~m_done);
                STAT(4, POPC(ok));
                const float aT = (ok ? alpha : 0.f) * T[k];
                C0[k] = __builtin_fmaf(cr, aT, C0[k]);
                C1[k] = __builtin_fmaf(cg, aT, C1[k]);
                C2[k] = __builtin_fmaf(cbl, aT, C2[k]);
                Wt[k] += aT;  // weight += alpha * T (forward.cu:364), exact rounding
                Dp[k] = __builtin_fmaf(dep, aT, Dp[k]);
                S0[k] = __builtin_fmaf(s0, aT, S0[k]);
                S1[k] = __builtin_fmaf(s1, aT, S1[k]);
                T[k] = ok ? test_T : T[k];
                last[k] = ok ? contributor : last[k];
            }
        }
    }
    STAT_FLUSH(0)
    WT_END(0, tile, n, (int)__builtin_amdgcn_readfirstlane(max(max(last[0], last[1]), max(last[2], last[3]))))
    const float bg0 = bg[0], bg1 = bg[1], bg2 = bg[2];
    const size_t HW = (size_t)H * W;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        n_contrib[(size_t)tile * TILE_PIX + k * 64 + lane] = last[k];
        const int px = px0 + 8 * (k & 1), py = py0 + 8 * (k >> 1);
        if (!(px < W && py < H)) continue;
        const size_t pix = (size_t)py * W + px;
        out_color[pix] = C0[k] + T[k] * bg0;
        out_color[HW + pix] = C1[k] + T[k] * bg1;
        out_color[2 * HW + pix] = C2[k] + T[k] * bg2;
        out_alpha[pix] = Wt[k];
        out_depth[pix] = Dp[k];
        out_segment[pix] = S0[k];
        out_segment[HW + pix] = S1[k];
    }
}

template <int CTRL>
__device__ __forceinline__ float dpp(float v) {
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}

// Transposed butterfly over the wave: v[12] per lane -> lane l (with (l & 3) == 0
// and valid) holds the wave-wide sum of channel vidx.  xor-32 and xor-16 halves
// are exchanged by v_permlane32_swap / v_permlane16_swap (no selects: the swap
// itself routes each half), xor-8 by DPP row_ror:8, xor-4 by row_half_mirror
// (partner differs in bit 2), the last two steps by quad_perm DPP adds.
__device__ __forceinline__ float wave_reduce12(float v[12], int lane, int& vidx, bool& valid) {
    float s6[6];
#pragma unroll
    for (int i = 0; i < 6; ++i) {
        auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v[i]), __float_as_uint(v[i + 6]), false, false);
        s6[i] = __uint_as_float(r[0]) + __uint_as_float(r[1]);  // lanes <32: ch i, lanes >=32: ch i+6
    }
    float s3[4];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(s6[i]), __float_as_uint(s6[i + 3]), false, false);
        s3[i] = __uint_as_float(r[0]) + __uint_as_float(r[1]);  // row q holds ch 3q + i
    }
    s3[3] = 0.f;
    const bool h8 = lane & 8, h4 = lane & 4;
    float s2[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const float send = h8 ? s3[i] : s3[i + 2];
        const float keep = h8 ? s3[i + 2] : s3[i];
        s2[i] = keep + dpp<0x128>(send);  // row_ror:8 == xor 8 inside a row
    }
    const float send = h4 ? s2[0] : s2[1];
    const float keep = h4 ? s2[1] : s2[0];
    float r = keep + dpp<0x141>(send);  // row_half_mirror: partner differs in bit 2
    r += dpp<0x4E>(r);                  // quad_perm [2,3,0,1]
    r += dpp<0xB1>(r);                  // quad_perm [1,0,3,2]
    const int w = (h8 ? 2 : 0) + (h4 ? 1 : 0);
    vidx = 3 * (lane >> 4) + w;
    valid = ((lane & 3) == 0) && w < 3;
    return r;
}

// q = num / den as v_rcp_f32 plus one Newton correction of the quotient (4 VALU ops
// instead of the ~10 of div_scale/fmas/fixup; the corrected quotient is the correctly
// rounded one except in rare cases).  The replay divides T back through every contributor
// (backward.cu:574), so the quotient's rounding compounds along the pixel's list: with the
// bare num * rcp(den) (<= 1.5 ulp per step, GSR_FAST_DIV) one element of dscales / drot of
// C3 view 5 of 8 reached 1.2e-5 / 1.4e-5 of the tensor maximum (the reference's own
// fp32-order noise there: 9e-6); with the correction 4.1e-6 / 5.4e-6, the same as the IEEE
// quotient (GSR_IEEE_DIV, 50 us slower) (profiles/round3_div_study.txt).
__device__ __forceinline__ float fdiv(float num, float den) {
#if defined(GSR_IEEE_DIV)
    return num / den;
#elif defined(GSR_FAST_DIV)
    return num * __builtin_amdgcn_rcpf(den);
#else
    const float r = __builtin_amdgcn_rcpf(den);
    const float q = num * r;
    const float e = __builtin_fmaf(-q, den, num);
    return __builtin_fmaf(e, r, q);
#endif
}

__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(4))) k_render_bwd(int W, int H, int gx, const uint32_t* __restrict__ order,
                                                   const uint2* __restrict__ ranges,
                                                   const uint32_t* __restrict__ point_list,
                                                   const uint32_t* __restrict__ slot_vals,
                                                   const float4* __restrict__ rec, const float* __restrict__ bg,
                                                   const float* __restrict__ alphas,
                                                   const uint32_t* __restrict__ n_contrib,
                                                   const float* __restrict__ dL_dpixels,
                                                   const float* __restrict__ dL_dsegs,
                                                   const float* __restrict__ dL_ddepths,
                                                   const float* __restrict__ dL_dalphas,
                                                   float* __restrict__ contrib, uint8_t* __restrict__ written) {
#pragma clang fp contract(off)
    WT_BEGIN
    const int tile = (int)order[blockIdx.x];
    const int lane = threadIdx.x;
    const int tx = tile % gx, ty = tile / gx;
    const int px = tx * BX + (lane & 15);
    const int py0 = ty * BY + (lane >> 4);
    const float pfx = (float)px;
    const size_t HW = (size_t)H * W;
    const float bg0 = bg[0], bg1 = bg[1], bg2 = bg[2];

    // Per-pixel replay state.  The reference keeps seven per-channel accum_rec
    // registers (colour, segment, depth, alpha) plus last_alpha/last_colour and folds
    // them in at the NEXT contributor (backward.cu:567-606).  Here each pixel keeps
    // only their projection on its upstream gradient, Dk = sum_ch accum_rec[ch] *
    // dL_dch (alpha channel: colour 1), folded right after the contributor that owns
    // (a, c): Dk' = a * cdot + (1 - a) * Dk with cdot = sum_ch c[ch] * dL_dch, and the
    // reference's sum_ch (c[ch] - accum_rec[ch]) * dL_dch is cdot - Dk.  Equal in exact
    // arithmetic; the fp32 rounding differs from the per-channel form at the 1e-7
    // level (tests/test_gpu_parity.py tolerances), and 24 registers per lane are freed.
    float pfy[4], T[4], Tfin[4], dp0[4], dp1[4], dp2[4], ds0[4], ds1[4], dd[4], da[4], bgdot[4];
    float Dk[4];
    uint32_t lastc[4];
    uint32_t maxlast = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int py = py0 + 4 * k;
        pfy[k] = (float)py;
        const bool inside = px < W && py < H;
        const size_t pix = inside ? (size_t)py * W + px : 0;
        // n_contrib is in the forward's quadrant layout (entry 64 k' + 8 (row & 7) + (col & 7))
        const int r = (lane >> 4) + 4 * k, c = lane & 15;
        const int fidx = 64 * (2 * (r >> 3) + (c >> 3)) + 8 * (r & 7) + (c & 7);
        lastc[k] = inside ? n_contrib[(size_t)tile * TILE_PIX + fidx] : 0u;
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
        Dk[k] = 0.f;
        maxlast = max(maxlast, lastc[k]);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) maxlast = max(maxlast, (uint32_t)__shfl_xor((int)maxlast, o, 64));
    const bool use_bg = wave_any(bgdot[0] != 0.f || bgdot[1] != 0.f || bgdot[2] != 0.f || bgdot[3] != 0.f);

    const uint2 range = ranges[tile];
    const int n = (int)(range.y - range.x);
    const float x0 = (float)(tx * BX), y0 = (float)(ty * BY);
    const float x1 = (float)min(tx * BX + BX - 1, W - 1), y1 = (float)min(ty * BY + BY - 1, H - 1);

    STAT_DECL
    STAT(7, n);
    STAT(6, n > (int)maxlast ? n - (int)maxlast : 0);
    // Same two-stage batch pipeline and LDS record broadcast as the forward, walking
    // the list back to front: lane l of the batch with upper end `top` owns position top-1-l.
    __shared__ float4 srec[64][4];
    const int top0 = (int)__builtin_amdgcn_readfirstlane(maxlast);
    const uint32_t* plist = point_list + range.x;
    const uint32_t* slist = slot_vals + range.x;
    // list positions below 0 are clamped to 0 (unconditional loads, see fetch_batch)
    uint32_t g_next = 0u, u_next = 0u;
    Batch cur;
    if (top0 > 0) {
        g_next = plist[max(top0 - 1 - lane, 0)];
        u_next = slist[max(top0 - 1 - lane, 0)];
        cur = fetch_batch(rec, g_next);
    }
    uint32_t u_cur = u_next;
    if (top0 > 0) {
        g_next = plist[max(top0 - 65 - lane, 0)];
        u_next = slist[max(top0 - 65 - lane, 0)];
    }
    // The background term of dL_dalpha (backward.cu:597) is only live when bg . dL_dpix
    // is non-zero somewhere in the tile: the loop is specialised on it.
    auto replay = [&](auto use_bg_c) {
        constexpr bool UB = decltype(use_bg_c)::value;
        for (int top = top0; top > 0; top -= 64) {
            const int cnt = min(64, top);
            STAT(5, 1);
            const Batch nxt = fetch_batch(rec, g_next);
            const uint32_t u_nxt = u_next;
            g_next = plist[max(top - 129 - lane, 0)];
            u_next = slist[max(top - 129 - lane, 0)];
            const float4 ra = cur.a, rb = cur.b, rc = cur.c;
            const uint32_t uslot = u_cur;
            cur = nxt;
            u_cur = u_nxt;
            const float pmin = power_floor(rb.y);
            const bool hit = lane < cnt && tile_hit(ra.x, ra.y, ra.z, ra.w, rb.x, pmin, x0, x1, y0, y1);
            uint64_t todo = __ballot(hit);
            // Lanes replaying every position of this batch (p < n_contrib for all p < top) and
            // whether any lane starts replaying inside it: only then is p < n_contrib
            // tested per instance.
            uint64_t act_all[4];
            bool varying = false;
    #pragma unroll
            for (int k = 0; k < 4; ++k) {
                act_all[k] = __builtin_amdgcn_ballot_w64(lastc[k] >= (uint32_t)top);
                varying |= lastc[k] < (uint32_t)top && lastc[k] > (uint32_t)(top - cnt);
            }
            const bool vary = wave_any(varying);
            STAT(9, vary);
            STAT(2, cnt - __popcll(todo));
            __syncthreads();  // previous batch's reads are done
            srec[lane][0] = ra;                                                   // x, y, conic a, b
            srec[lane][1] = make_float4(rb.x, pmin, rb.y, rb.w);                  // conic c, power floor, opacity, seg0
            srec[lane][2] = rc;                                                   // r, g, b, seg1
            srec[lane][3] = make_float4(rb.z, __uint_as_float(uslot), 0.f, 0.f);  // depth, record slot
            __syncthreads();
            while (todo) {
                const int j = (int)__builtin_ctzll(todo);
                todo &= todo - 1;
                const uint32_t p = (uint32_t)(top - 1 - j);
                const float4 q0 = srec[j][0], q1 = srec[j][1];
                const float gx_ = q0.x, gy_ = q0.y, ca = q0.z, cb = q0.w, cc = q1.x, pm = q1.y;
                float power[4], dys[4];
                uint64_t act[4] = {act_all[0], act_all[1], act_all[2], act_all[3]};
                if (vary) {
    #pragma unroll
                    for (int k = 0; k < 4; ++k) act[k] = __builtin_amdgcn_ballot_w64(p < lastc[k]);
                }
                uint64_t near[4];  // per strip: lanes whose pixel replays p and is within reach
                const float dx = gx_ - pfx;
                const float adxdx = ca * dx * dx, bdx = cb * dx;
    #pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const float dy = gy_ - pfy[k];
                    dys[k] = dy;
                    power[k] = __builtin_fmaf(-0.5f, adxdx + cc * dy * dy, -(bdx * dy));  // == -0.5 S - B
                    near[k] = act[k] & __builtin_amdgcn_ballot_w64(power[k] >= pm);
                }
                STAT(0, 1);
                if (!(near[0] | near[1] | near[2] | near[3])) {
                    STAT(1, 1);
                    continue;
                }
                STAT(3, 1);
                                const float4 q2 = srec[j][2], q3 = srec[j][3];
                const float op = q1.z, dep = q3.x, s0 = q1.w;
                const float c0 = q2.x, c1 = q2.y, c2 = q2.z, s1 = q2.w;
                const uint32_t u = __float_as_uint(q3.y);
                float* dst = contrib + (size_t)u * 12;
                float acc[12];
    #pragma unroll
                for (int i = 0; i < 12; ++i) acc[i] = -0.0f;  // -0 + x == x: the first add folds away
                // Strip k (rows 4k..4k+3) is replayed only if one of its pixels can pass.
    #pragma unroll
                for (int k = 0; k < 4; ++k) {
                    if (!near[k]) continue;
                    STAT(8, 1);
                    // near[k]: lanes replaying p (p < n_contrib) within reach (power >= the
                    // opacity floor); G is used only under o, a subset of near[k]
                    const float G = GSR_EXP_NC(power[k]);
                    const float a = fminf(0.99f, op * G);
                    const bool o = __builtin_amdgcn_inverse_ballot_w64(
                        near[k] & __builtin_amdgcn_ballot_w64(power[k] <= 0.0f) &
                        __builtin_amdgcn_ballot_w64(a >= ALPHA_MIN));
                    STAT(4, POPC(o));
                    // a_m = alpha of a replayed pair, else 0: it masks dch and the Dk fold, and
                    // makes Tn == T exactly off o (T / 1), so T needs no select; off o, a itself
                    // may be anything (-inf * 0 would poison the quotient's correction step)
                    const float a_m = o ? a : 0.f;
                    const float one_m = 1.f - a_m;
                    const float Tn = fdiv(T[k], one_m);
                    const float dch_m = a_m * Tn;
                    float cdot = __builtin_fmaf(c0, dp0[k], da[k]);  // alpha channel (colour 1) first
                    cdot = __builtin_fmaf(c1, dp1[k], cdot);
                    cdot = __builtin_fmaf(c2, dp2[k], cdot);
                    cdot = __builtin_fmaf(s0, ds0[k], cdot);
                    cdot = __builtin_fmaf(s1, ds1[k], cdot);
                    cdot = __builtin_fmaf(dep, dd[k], cdot);
                    const float diff = cdot - Dk[k];
                    float dopa = diff * Tn;
                    if (UB) dopa += (-Tfin[k] * __builtin_amdgcn_rcpf(one_m)) * bgdot[k];

                    acc[0] = __builtin_fmaf(dch_m, dp0[k], acc[0]);
                    acc[1] = __builtin_fmaf(dch_m, dp1[k], acc[1]);
                    acc[2] = __builtin_fmaf(dch_m, dp2[k], acc[2]);
                    acc[3] = __builtin_fmaf(dch_m, ds0[k], acc[3]);
                    acc[4] = __builtin_fmaf(dch_m, ds1[k], acc[4]);
                    acc[5] = __builtin_fmaf(dch_m, dd[k], acc[5]);
                    // q = G * dL_dalpha: the opacity gradient term (backward.cu:636); the
                    // mean2D / conic terms (backward.cu:612-631) are op * q times a
                    // polynomial in (dx, dy) with per-Gaussian coefficients, so only the
                    // moments of q are summed here (see the record layout above).
                    const float qg = o ? G * dopa : 0.f;  // select after the product: G may be non-finite off o
                    const float qdy = qg * dys[k];
                    acc[6] += qg;
                    acc[8] += qdy;
                    acc[11] = __builtin_fmaf(qdy, dys[k], acc[11]);
                    // fold this contributor into the accumulators seen by the next one (front side)
                    // Dk' = a cdot + (1 - a) Dk, as Dk + a (cdot - Dk); unchanged when a_m = 0
                    Dk[k] = __builtin_fmaf(a_m, diff, Dk[k]);
                    T[k] = Tn;
                }
#ifdef GSR_MOMENT_MEAN
                acc[7] = dx * acc[6];   // sum q dx   (dx is shared by the lane's 4 pixels)
                acc[9] = dx * acc[7];   // sum q dx^2
                acc[10] = dx * acc[8];  // sum q dx dy
#else
                // The mean2D channels carry the conic-weighted sums per lane,
                // sum q (a dx + b dy) and sum q (b dx + c dy), as the reference's per-pixel
                // dG_ddelx / dG_ddely terms (backward.cu:612-621), instead of the moments
                // Qx, Qy combined after the reduction: for an elongated Gaussian a Qx and
                // b Qy nearly cancel, which amplified the moments' rounding ~100x there.
                {
                    const float qx = dx * acc[6];  // sum q dx (dx is shared by the lane's 4 pixels)
                    const float qy = acc[8];
                    acc[9] = dx * qx;              // sum q dx^2
                    acc[10] = dx * qy;             // sum q dx dy
                    acc[7] = __builtin_fmaf(ca, qx, cb * qy);
                    acc[8] = __builtin_fmaf(cc, qy, cb * qx);
                }
#endif
                int vidx;
                bool valid;
                const float r = wave_reduce12(acc, lane, vidx, valid);
                if (valid) dst[vidx] = r;
                // Byte u marks slot u as written: one plain store of one byte by the whole
                // wave (a uniform address; no atomic, no lane election).
                written[u] = 1;
            }
        }
    };
    if (use_bg)
        replay(std::true_type{});
    else
        replay(std::false_type{});
    STAT_FLUSH(16)
    WT_END(1, tile, n, top0)
}

}  // namespace

void launch_render_forward(int W, int H, int gx, int gy, const uint32_t* order, const uint2* ranges,
                           const uint32_t* point_list, const float4* rec, const float* bg, float* out_color,
                           float* out_depth, float* out_alpha, float* out_segment, uint32_t* n_contrib,
                           hipStream_t st) {
    const int T = gx * gy;
    if (T == 0) return;
    hipLaunchKernelGGL(k_render_fwd, dim3(T), dim3(64), 0, st, W, H, gx, order, ranges, point_list, rec, bg,
                       out_color, out_depth, out_alpha, out_segment, n_contrib);
}

void launch_render_backward(int W, int H, int gx, int gy, const uint32_t* order, const uint2* ranges,
                            const uint32_t* point_list, const uint32_t* slot_vals, const float4* rec,
                            const float* bg, const float* alpha, const uint32_t* n_contrib, const float* dL_dcolor,
                            const float* dL_dsegment, const float* dL_ddepth, const float* dL_dalpha, float* contrib,
                            uint8_t* written, hipStream_t st) {
    const int T = gx * gy;
    if (T == 0) return;
    hipLaunchKernelGGL(k_render_bwd, dim3(T), dim3(64), 0, st, W, H, gx, order, ranges, point_list, slot_vals, rec,
                       bg, alpha, n_contrib, dL_dcolor, dL_dsegment, dL_ddepth, dL_dalpha, contrib, written);
}

}  // namespace gsr
