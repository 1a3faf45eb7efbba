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
// d = (dx, dy) = mean2D - pixel, conic (a, b, c)), 12 floats:
//   [0..5]  sum dch*dL_dcolor.rgb, sum dch*dL_dseg0/1, sum dch*dL_ddepth
//   [6]     sum q
//   [7] [8] sum q (a dx + b dy), sum q (b dx + c dy)   (the reference's dG_ddelx / dG_ddely
//           weighting, backward.cu:612-621, formed per lane before the reduction)
//   [9..11] sum q dx^2, sum q dx dy, sum q dy^2
// from which k_gaussian_backward (preprocess.hip) forms dopacity = sum q and the reference's
// mean2D / conic gradients with the Gaussian's own conic and opacity.
#include "gsr_internal.h"

// Two translation units: this file's forward part (GSR_RENDER_PART 1) and render_bwd.hip,
// which includes it for the backward part (2), each built with its own machine-scheduler
// strategy (Makefile).  Diagnostic builds (GSR_WAVE_TRACE / GSR_STATS, whose trace buffers
// are per translation unit) compile both parts here (0).
#ifndef GSR_RENDER_PART
#if defined(GSR_WAVE_TRACE) || defined(GSR_STATS)
#define GSR_RENDER_PART 0
#else
#define GSR_RENDER_PART 1
#endif
#endif

#include <type_traits>

// Numerics.  The blend thresholds alpha >= 1/255 and T*(1-alpha) >= 1e-4
// (forward.cu:352-359) make n_contrib and every contribution knife-edge
// sensitive to exp(), and the reference's backward recovers T from
// T_final = 1 - sum(alpha*T) (backward.cu:468), amplifying any last-ulp alpha
// difference by 1/T_final.  gsr therefore evaluates exp() with gsr_expf below:
// IEEE operations only (fma, add, mul, integer shift), so the CPU oracle computes the
// very same bits (oracle/gsr_oracle.cpp: gsr_expf).  On the blend's range [-5.6, 0] (powers at
// or above the opacity floor, power_floor) max error 0.887 ulp, correctly rounded on 99.64% of
// inputs (exhaustive; tests/test_oracle_golden.py pins it against double-precision exp; the
// reference's CUDA expf is specified at 2 ulp).
// GSR_FAST_EXP selects __expf (v_exp_f32, several ulp) for experiments.
// power, alpha, T and the weight sum run without FMA contraction (see the
// kernels); only non-amplified sums use explicit FMAs.
// ln 2 rounded to fp32: the reduction x - k ln2 is one FMA.  Its error, |k| * 1.9e-9, is at most
// 1.5e-8 on the blend's range (|k| <= 8) and grows to 2.4e-7 (< 5 ulp) at -87 and 88, where only rejected
// pairs land (alpha < 1/255 with the power floor's 1e-3 margin).  The two-step Cody-Waite form it
// replaced (hi + lo, one more FMA per exp): max 0.874 ulp, correctly rounded 99.71% on [-5.6, 0].
constexpr float GSR_LN2 = 0.693147182464599609375f;
__device__ __forceinline__ float gsr_expf(float x) {
    // exp(clamp(x, -87, 88)).  k = round(x log2 e) via the 1.5*2^23 shifter (one FMA,
    // the integer lands in the low mantissa bits), r = x - k ln2 (one FMA), degree-6
    // minimax polynomial on [-ln2/2, ln2/2] (1 + r + c2 r^2 + ... + c6 r^6, fp32
    // coefficients, Horner with FMAs), then times 2^k assembled from the shifter's
    // bits (k in [-126, 127], so the product is an exact scaling).  Outside the clamp
    // the value is meaningless for blending anyway: alpha < 1/255 below -87 and the
    // blend rejects power > 0.
    const float xc = __builtin_amdgcn_fmed3f(x, -87.0f, 88.0f);
    const float kf = __builtin_fmaf(xc, 1.44269502f, 12582912.0f);
    const float k = kf - 12582912.0f;
    const float r = __builtin_fmaf(-k, GSR_LN2, xc);
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
// gsr_expf without the clamp, for lanes whose argument is known to lie in [-87, 0]: the
// blend loops call it only under a lane mask of pixels with power >= the Gaussian's
// opacity floor (>= -5.6) and use the result only under that mask (other lanes get a
// meaningless, possibly non-finite value that every use masks out).  Same bits as
// gsr_expf on [-125 ln2, 0]: there p * 2^k is a normal number, so scaling by 2^k is exact
// and equals adding k to p's exponent field -- one v_lshl_add_u32 instead of building 2^k
// and multiplying.
__device__ __forceinline__ float gsr_expf_nc(float x) {
    const float kf = __builtin_fmaf(x, 1.44269502f, 12582912.0f);
    const float k = kf - 12582912.0f;
    const float r = __builtin_fmaf(-k, GSR_LN2, x);
    float p = 0.001381461275741458f;
    p = __builtin_fmaf(p, r, 0.008368710055947304f);
    p = __builtin_fmaf(p, r, 0.04166838899254799f);
    p = __builtin_fmaf(p, r, 0.1666652113199234f);
    p = __builtin_fmaf(p, r, 0.4999999403953552f);
    p = __builtin_fmaf(p, r, 1.0f);
    p = __builtin_fmaf(p, r, 1.0f);
#ifdef GSR_EXP_MUL
    const float scale = __uint_as_float((__float_as_uint(kf) << 23) + 0x3f800000u);
    return p * scale;
#else
    // kf's low mantissa bits hold k (two's complement), so kf_bits << 23 == k << 23 (mod 2^32)
    return __uint_as_float((__float_as_uint(kf) << 23) + __float_as_uint(p));
#endif
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
// 4 ok pixels, 5 batches, 6 zero-tail (bwd), 7 instances, 8 strips processed, 13 instances
// fetched (their records read: the render kernels' per-instance HBM traffic).
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
    if ((threadIdx.x & 63) == 0)                                                 \
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
// kernel, {start, end} of s_memrealtime (100 MHz, chip-wide), the tile, its list length,
// the last list position the wave visits, XCC and HW_ID.  Entry = the wave's slot
// (forward: block; backward: 2 * block + wave).
__device__ unsigned long long g_gsr_wtrace[2][32768][4];
extern "C" __attribute__((visibility("default"))) int gsr_wave_trace_read(unsigned long long* host, int reset) {
    if (hipMemcpyFromSymbol(host, HIP_SYMBOL(g_gsr_wtrace), sizeof(g_gsr_wtrace)) != hipSuccess) return -1;
    if (reset) {
        void* d = nullptr;
        if (hipGetSymbolAddress(&d, HIP_SYMBOL(g_gsr_wtrace)) != hipSuccess) return -1;
        if (hipMemset(d, 0, sizeof(g_gsr_wtrace)) != hipSuccess) return -1;
    }
    return 0;
}
#define WT_BEGIN const unsigned long long wt0_ = __builtin_amdgcn_s_memrealtime();
#define WT_END(kind, slot, tile, n, depth, mode)                                                        \
    if ((threadIdx.x & 63) == 0 && (slot) < 32768) {                                                  \
        const unsigned long long wt1_ = __builtin_amdgcn_s_memrealtime();                             \
        unsigned long long* w_ = g_gsr_wtrace[kind][slot];                                            \
        w_[0] = wt0_;                                                                                 \
        w_[1] = wt1_;                                                                                 \
        w_[2] = (unsigned long long)(tile) | ((unsigned long long)(mode) << 24) |                    \
                ((unsigned long long)(unsigned)(n) << 32);                                            \
        w_[3] = (unsigned long long)((unsigned)(depth) & 0xffffffu) |                                 \
                ((unsigned long long)(__builtin_amdgcn_s_getreg((20) | (0 << 6) | (3 << 11)) & 15u) << 24) | \
                ((unsigned long long)__builtin_amdgcn_s_getreg((4) | (0 << 6) | (31 << 11)) << 32); \
    }
#else
#define WT_BEGIN
#define WT_END(kind, slot, tile, n, depth, mode)
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
// The backward's batch fetch also takes the Gaussian's tile rectangle and first record slot in its
// block (record part 3, in the 32-B sector of part 2) and its block's slot base bbase[g / SLOT_BLOCK]
// (gsr_internal.h): the instance's slot is then r.z + bb + (ty - y0) (x1 - x0) + (tx - x0) -- no
// per-instance slot array to read.  The parts are added when the batch is used, not here: an add
// at the fetch would wait for the prefetch loads.
struct BatchB {
    float4 a, b, c;
    uint3 r;
    uint32_t bb;
};
__device__ __forceinline__ BatchB fetch_batch_b(const float4* __restrict__ rec, const uint32_t* __restrict__ bbase,
                                                uint32_t g) {
    const float4* R = rec + (size_t)g * REC_F4;
    const uint4 r3 = *reinterpret_cast<const uint4*>(R + 3);
    return BatchB{R[0], R[1], R[2], make_uint3(r3.x, r3.y, r3.z), bbase[g / SLOT_BLOCK]};
}
__device__ __forceinline__ uint32_t batch_slot(const BatchB& b, int tx, int ty) {
    const uint32_t x0 = b.r.x & 0xFFFFu, y0 = b.r.x >> 16, x1 = b.r.y & 0xFFFFu;
    return b.r.z + b.bb + ((uint32_t)ty - y0) * (x1 - x0) + ((uint32_t)tx - x0);
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

// Forward of one tile (NQ = 4: all four 8x8 quadrants, one wave) or of half of it (NQ = 2:
// quadrants q0, q0 + 1, i.e. the top or the bottom 16x8 half).  The schedule gives the
// heaviest tiles (list length >= 2^(B-1) instances, B = the split bucket) two waves each:
// a wave's time grows with the list positions it visits, and at the metric scene the
// longest single-wave tiles ran 160-240 us of the 245-us launch, while the chip was less
// than half busy for the last 37% of it (tools/wave_trace.py, profiles/round3_wave_trace.txt).
// Every pixel is computed by the same code either way: results are bit-identical.
// File a rendered tile under its depth in the backward's queue (TileSched).  A split
// tile's halves finish independently: each adds (depth << 1) | 1 to the tile's word, so
// the second to finish (odd old value) reads the other half's depth from the value its
// own add returned -- one relaxed atomic, no fences (an acquire / release pair costs an
// L2 write-back + invalidate on this multi-XCD part: the split forward ran 50% slower
// with it).  Lane 0 only.
// Quarter tiles (4 parts): the word holds (max depth << 2) | parts done, updated by a
// compare-and-swap loop; the part that completes the count files the tile.
// List segments.  The backward replays a tile's list back to front, and its wave time grows with
// the positions it replays; with one wave per tile the deepest tiles, four or five to a SIMD from
// the start, set the kernel's end (profiles/round4_wave_trace.txt: per-SIMD work 1874..2407 list
// positions, the kernel ends with the most loaded SIMD).  So the forward, when its list walk
// reaches position ck (a multiple of 64, gsr_set_option "bwd_ckpt"), stores each pixel's
// transmittance Tc and its seven channel sums (colour, segment, depth, weight) there, and at its
// end turns them into the backward's replay state at ck (CKPT_FLOATS channels):
//   [0]    T(ck) as the backward's chain has it: T_final * Tc / T_end, where T_final = 1 - weight
//          sum is the reference's (backward.cu:468) and T_end the forward's last product -- the
//          back's divisions would have reached T_final / prod_{j >= ck} (1 - alpha_j) with the same
//          T_final rounding, which dominates for small T_final, and T_end / Tc is that product;
//   [1..7] the channel sums from ck on, / Tc: the normalised suffix sums of Dk (bwd_tile) for every
//          channel (the reference's accum_rec, backward.cu:567-606).  The colour, segment and depth
//          sums restart from 0 at ck, so these are accumulated directly (as differences of prefix
//          sums they lost eps * sum_final / Tc to cancellation, which the replay amplifies by
//          1 / (1 - alpha) per front contributor: one C3 dscales element went from 4e-6 to 1.2e-5
//          of its maximum); the weight sum from ck on is T(ck) - T_end (telescoping), since the
//          weight sum itself must not restart (T_final = 1 - weight sum);
//   [8]    T_end / Tc: the product of (1 - alpha) over the suffix, which scales the background term
// so Dk(ck) = sum_ch dL_ch [ch] + (bg . dL_dpix) [8].  A tile replayed deeper than ck + CK_MIN_BACK
// is filed as two independent queue entries: the back [ck, d) starts at the end of the list as
// before, the front [0, ck) from the checkpoint.  Every list position is replayed by exactly one
// of them (records and written flags unchanged).
constexpr uint32_t BQ_FRONT = 1u << 30, BQ_BACK = 2u << 30, BQ_TILE = BQ_FRONT - 1;
#ifndef GSR_CK_MIN_BACK
#define GSR_CK_MIN_BACK 64
#endif
constexpr uint32_t CK_MIN_BACK = GSR_CK_MIN_BACK;  // a back segment of at least one batch
#ifndef GSR_BWD_CKPT
#define GSR_BWD_CKPT 256
#endif
static int g_bwd_ckpt = GSR_BWD_CKPT;
#ifndef GSR_FWD_XCD_PAIRS
#define GSR_FWD_XCD_PAIRS 0
#endif
static int g_fwd_xcd_pairs = GSR_FWD_XCD_PAIRS;  // gsr_set_option("fwd_xcd_pairs", 0 / 1)
__device__ __forceinline__ void publish_depth(const TileSched& ts, int T, int tile, int parts, uint32_t d, int ck) {
    if (parts == 2) {
        const uint32_t old = atomicAdd(&ts.tdone[tile], (d << 1) | 1u);
        if (!(old & 1u)) return;  // first half: the second files the tile
        d = max(d, old >> 1);
    } else if (parts == 4) {
        uint32_t old = ts.tdone[tile], assumed;
        do {
            assumed = old;
            const uint32_t nv = (max(assumed >> 2, d) << 2) | ((assumed & 3u) + 1u);
            old = atomicCAS(&ts.tdone[tile], assumed, nv);
        } while (old != assumed);
        if ((old & 3u) != 3u) return;  // not the last quarter
        d = max(d, old >> 2);
    }
    if (d == 0) return;  // nothing for the backward to replay
    const size_t cap = bq_cap(T);
    if (ck > 0 && d >= (uint32_t)ck + CK_MIN_BACK) {
        // two list segments: the front [0, ck) from the forward's checkpoint, the back [ck, d)
        const uint32_t bf = depth_bucket((uint32_t)ck), bb = depth_bucket(d - (uint32_t)ck);
        ts.bq_list[(size_t)bf * cap + atomicAdd(&ts.bq_cnt[bf], 1u)] = (uint32_t)tile | BQ_FRONT;
        ts.bq_list[(size_t)bb * cap + atomicAdd(&ts.bq_cnt[bb], 1u)] = (uint32_t)tile | BQ_BACK;
        return;
    }
    const uint32_t b = depth_bucket(d);
    ts.bq_list[(size_t)b * cap + atomicAdd(&ts.bq_cnt[b], 1u)] = (uint32_t)tile;
}

template <int NQ>
__device__ __forceinline__ void fwd_tile(int W, int H, int gx, int ntiles, int tile, int q0, int wslot, const TileSched& ts,
                                         const uint2* __restrict__ ranges, const uint32_t* __restrict__ point_list,
                                         const float4* __restrict__ rec, const float* __restrict__ bg,
                                         float* __restrict__ out_color, float* __restrict__ out_depth,
                                         float* __restrict__ out_alpha, float* __restrict__ out_segment,
                                         uint32_t* __restrict__ n_contrib, float* __restrict__ ckpt, int ck,
                                         float4 (*srec)[4]) {
    // The backward recovers T from T_final = 1 - sum(alpha*T) (backward.cu:468) and
    // divides back through every contributor, which amplifies a last-bit difference
    // in the weight sum by 1/T_final.  power, alpha, T and the weight sum are therefore
    // rounded exactly as the reference writes them (no contraction); only the
    // colour/depth/segment sums, which nothing amplifies, use explicit FMAs.
#pragma clang fp contract(off)
    WT_BEGIN
    // quadrant rows / columns covered: 2 x 2 (whole tile), 1 x 2 (half), 1 x 1 (quarter)
    constexpr int NR = NQ == 4 ? 2 : 1, NC = NQ == 1 ? 1 : 2;
    const int lane = threadIdx.x & 63;
    const int tx = tile % gx, ty = tile / gx;
    const int r0 = q0 >> 1;                    // first quadrant row
    const int c0 = NQ == 1 ? (q0 & 1) : 0;     // first quadrant column
    // Lane l owns pixel (l & 7, l >> 3) of each 8x8 quadrant k of the tile (k & 1: right
    // half, k >> 1: bottom half).  Square quadrants are gated tighter than 16x4 strips:
    // 8.7% fewer (quadrant, Gaussian) blends at the metric scene (tools/render_stats.py).
    // Quadrant kk of this wave is k = q0 + kk: column c0 + kk % NC, row r0 + kk / NC.
    const int px0 = tx * BX + (lane & 7), py0 = ty * BY + (lane >> 3);
    float pfx[NC];
#pragma unroll
    for (int cc = 0; cc < NC; ++cc) pfx[cc] = (float)(px0 + 8 * (c0 + cc));
    float pfy[NR];
#pragma unroll
    for (int rr = 0; rr < NR; ++rr) pfy[rr] = (float)(py0 + 8 * (r0 + rr));
    // live[kk]: lanes whose pixel of quadrant kk is inside the image and not terminated,
    // kept as a wave mask in SGPRs (no per-pair VALU compare); T stays at its value at
    // termination, which is the T the output uses (forward.cu:355-357 breaks before T).
    float T[NQ], C0[NQ], C1[NQ], C2[NQ], S0[NQ], S1[NQ], Dp[NQ], Wt[NQ];
    uint32_t last[NQ];
    uint64_t live[NQ];
#pragma unroll
    for (int kk = 0; kk < NQ; ++kk) {
        const int k = q0 + kk;
        const int px = px0 + 8 * (k & 1), py = py0 + 8 * (k >> 1);
        live[kk] = __builtin_amdgcn_ballot_w64(px < W && py < H);
        T[kk] = 1.0f;
        C0[kk] = C1[kk] = C2[kk] = S0[kk] = S1[kk] = Dp[kk] = Wt[kk] = 0.f;
        last[kk] = 0;
    }
    const uint2 range = ranges[tile];
    const int n = (int)(range.y - range.x);
    STAT_DECL
    STAT(7, n);
    // prefilter rectangle: the pixels this wave owns
    const float x0 = (float)(tx * BX + 8 * c0), y0 = (float)(ty * BY + 8 * r0);
    const float x1 = (float)min(tx * BX + 8 * (c0 + NC) - 1, W - 1), y1 = (float)min(ty * BY + 8 * (r0 + NR) - 1, H - 1);

    // Two-stage software pipeline over batches of 64 instances: while batch b is
    // blended, the records of batch b+1 and the ids of batch b+2 are in flight
    // (the id -> record dependency would otherwise stall every batch start).
    // The batch's records are parked in LDS and read back with a wave-uniform address
    // (a broadcast ds_read): the blend loop then spends no VALU issue slots on
    // v_readlane broadcasts.  One wave per block, so the barriers are free.
    const uint32_t* plist = point_list + range.x;
    const int nlast = max(n - 1, 0);  // list positions are clamped to the last one
    uint32_t g_next = n > 0 ? plist[min(lane, nlast)] : 0u;
    Batch cur;
    if (n > 0) cur = fetch_batch(rec, g_next);
    if (n > 0) g_next = plist[min(64 + lane, nlast)];
    bool wrote_ck = false;
    for (int base = 0; base < n; base += 64) {
        uint64_t any_live = 0;
#pragma unroll
        for (int kk = 0; kk < NQ; ++kk) any_live |= live[kk];
        if (!any_live) break;
        if (ck > 0 && base == ck) {  // list-segment checkpoint (publish_depth)
            // T and the colour / segment / depth sums so far, which then restart from 0: at the end
            // they hold the sums from ck on (no cancellation, publish_depth) and the outputs are the
            // two parts added (the weight sum runs on: T_final = 1 - weight sum must stay the
            // reference's).  Wave-uniform base + 32-bit lane offsets (saddr stores: no per-lane
            // 64-bit addresses for the compiler to keep live across the loop).
            float* cp = ckpt + (size_t)__builtin_amdgcn_readfirstlane(tile) * CKPT_FLOATS;
#pragma unroll
            for (int kk = 0; kk < NQ; ++kk) {
                const uint32_t o = 64u * (uint32_t)(q0 + kk) + (uint32_t)lane;
                cp[o + 0 * TILE_PIX] = T[kk];
                cp[o + 1 * TILE_PIX] = C0[kk];
                cp[o + 2 * TILE_PIX] = C1[kk];
                cp[o + 3 * TILE_PIX] = C2[kk];
                cp[o + 4 * TILE_PIX] = S0[kk];
                cp[o + 5 * TILE_PIX] = S1[kk];
                cp[o + 6 * TILE_PIX] = Dp[kk];
                C0[kk] = C1[kk] = C2[kk] = S0[kk] = S1[kk] = Dp[kk] = 0.f;
            }
            wrote_ck = true;
        }
        const int cnt = min(64, n - base);
        STAT(5, 1);
        STAT(13, cnt);  // instances fetched (records read)
        const Batch nxt = fetch_batch(rec, g_next);
        g_next = plist[min(base + 128 + lane, nlast)];
        const float4 ra = cur.a, rb = cur.b, rc = cur.c;
        cur = nxt;
        const float pmin = power_floor(rb.y);
#ifndef GSR_NO_LIVE_RECT
        // prefilter against the quadrants that still have live pixels (deep tiles end with a
        // few live quadrants; their instances need not reach the others)
        float lx0 = x0, lx1 = x1, ly0 = y0, ly1 = y1;
        {
            uint64_t cl = 0, cr = 0, rt = 0, rbm = 0;
#pragma unroll
            for (int kk = 0; kk < NQ; ++kk) {
                if (kk & 1) cr |= live[kk]; else cl |= live[kk];
                if (kk >> 1) rbm |= live[kk]; else rt |= live[kk];
            }
            if (NC == 2 && !cl) lx0 = x0 + 8.f;
            if (NC == 2 && !cr) lx1 = fminf(x1, x0 + 7.f);
            if (NR == 2 && !rt) ly0 = y0 + 8.f;
            if (NR == 2 && !rbm) ly1 = fminf(y1, y0 + 7.f);
        }
        uint64_t todo = __ballot(lane < cnt && tile_hit(ra.x, ra.y, ra.z, ra.w, rb.x, pmin, lx0, lx1, ly0, ly1));
#else
        uint64_t todo = __ballot(lane < cnt && tile_hit(ra.x, ra.y, ra.z, ra.w, rb.x, pmin, x0, x1, y0, y1));
#endif
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
            const float4 q0v = srec[j][0], q1v = srec[j][1];
            const float gx_ = q0v.x, gy_ = q0v.y, ca = q0v.z, cb = q0v.w, cc = q1v.x, pm = q1v.y;
            // power = -0.5 (a dx dx + c dy dy) - b dx dy, rounded as forward.cu:349 writes
            // it; the products are shared by the quadrants of a column / row.
            float ax[NC], bx[NC];
#pragma unroll
            for (int cc = 0; cc < NC; ++cc) {
                const float dxc = gx_ - pfx[cc];
                ax[cc] = ca * dxc * dxc;
                bx[cc] = cb * dxc;
            }
            float cy[NR], dyv[NR];
#pragma unroll
            for (int rr = 0; rr < NR; ++rr) {
                const float dy = gy_ - pfy[rr];
                cy[rr] = cc * dy * dy;
                dyv[rr] = dy;
            }
            float power[NQ];
            uint64_t near[NQ];  // per quadrant: live lanes within reach
            uint64_t any_near = 0;
#pragma unroll
            for (int kk = 0; kk < NQ; ++kk) {
#ifdef GSR_DEAD_SKIP
                if (!live[kk]) {  // a finished quadrant: no power, no ballot
                    near[kk] = 0;
                    power[kk] = 0.f;
                    continue;
                }
#endif
                // -0.5 S is exact, so -(0.5 S) - B as one fma(-0.5, S, -B): the same bits
                power[kk] = __builtin_fmaf(-0.5f, ax[kk % NC] + cy[kk / NC], -(bx[kk % NC] * dyv[kk / NC]));
                near[kk] = __builtin_amdgcn_ballot_w64(power[kk] >= pm) & live[kk];
                any_near |= near[kk];
            }
            STAT(0, 1);
            if (!any_near) {
                STAT(1, 1);
                continue;
            }
            STAT(3, 1);
            const float4 q2v = srec[j][2], q3v = srec[j][3];
            const float op = q1v.z, dep = q3v.x, s0 = q1v.w;
            const float cr = q2v.x, cg = q2v.y, cbl = q2v.z, s1 = q2v.w;
            // in a VGPR once per pair: the per-quadrant v_cndmask below may read only one SGPR
            // (its lane mask), so a scalar contributor would be re-moved into a VGPR per quadrant
            uint32_t contributor = (uint32_t)(base + j + 1);
            asm volatile("" : "+v"(contributor));
            // Quadrant kk is blended only if one of its pixels can pass; the exact
            // reference tests below decide per pixel.
#pragma unroll
            for (int kk = 0; kk < NQ; ++kk) {
                if (!near[kk]) continue;
                STAT(8, 1);
                // lanes of near[kk] (live, power >= the opacity floor) are the only ones that
                // can pass; every result below is used only under that mask
                const float alpha = fminf(0.99f, op * GSR_EXP_NC(power[kk]));
                const uint64_t m_o = near[kk] & __builtin_amdgcn_ballot_w64(power[kk] <= 0.0f) &
                                     __builtin_amdgcn_ballot_w64(alpha >= ALPHA_MIN);
                const float test_T = T[kk] * (1.f - alpha);
                const uint64_t m_done = m_o & __builtin_amdgcn_ballot_w64(test_T < T_MIN);  // forward.cu:355-357
                live[kk] &= ~m_done;
                const bool ok = __builtin_amdgcn_inverse_ballot_w64(m_o & ~m_done);
                STAT(4, POPC(ok));
                STAT(10, POPC(ok) == 0);
                const float aT = (ok ? alpha : 0.f) * T[kk];
                C0[kk] = __builtin_fmaf(cr, aT, C0[kk]);
                C1[kk] = __builtin_fmaf(cg, aT, C1[kk]);
                C2[kk] = __builtin_fmaf(cbl, aT, C2[kk]);
                Wt[kk] += aT;  // weight += alpha * T (forward.cu:364), exact rounding
                Dp[kk] = __builtin_fmaf(dep, aT, Dp[kk]);
                S0[kk] = __builtin_fmaf(s0, aT, S0[kk]);
                S1[kk] = __builtin_fmaf(s1, aT, S1[kk]);
                T[kk] = ok ? test_T : T[kk];
                last[kk] = ok ? contributor : last[kk];
            }
        }
    }
    STAT_FLUSH(0)
    uint32_t deepest = 0;
#pragma unroll
    for (int kk = 0; kk < NQ; ++kk) deepest = max(deepest, last[kk]);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) deepest = max(deepest, (uint32_t)__shfl_xor((int)deepest, o, 64));
    if (lane == 0) publish_depth(ts, ntiles, tile, 4 / NQ, deepest, ck);
    if (wrote_ck) {  // the checkpoint becomes the backward's replay state at ck (publish_depth)
        float* cp = ckpt + (size_t)__builtin_amdgcn_readfirstlane(tile) * CKPT_FLOATS;
#pragma unroll
        for (int kk = 0; kk < NQ; ++kk) {
            const uint32_t o = 64u * (uint32_t)(q0 + kk) + (uint32_t)lane;
            const float Tc = cp[o];
            const float b0 = cp[o + 1 * TILE_PIX], b1 = cp[o + 2 * TILE_PIX], b2 = cp[o + 3 * TILE_PIX];
            const float b3 = cp[o + 4 * TILE_PIX], b4 = cp[o + 5 * TILE_PIX], b5 = cp[o + 6 * TILE_PIX];
            const float rT = 1.0f / Tc;  // T(ck) > 0: at least T_MIN * 0.01 on any pixel
            cp[o + 0 * TILE_PIX] = (1.0f - Wt[kk]) * (Tc / T[kk]);
            cp[o + 1 * TILE_PIX] = C0[kk] * rT;
            cp[o + 2 * TILE_PIX] = C1[kk] * rT;
            cp[o + 3 * TILE_PIX] = C2[kk] * rT;
            cp[o + 4 * TILE_PIX] = S0[kk] * rT;
            cp[o + 5 * TILE_PIX] = S1[kk] * rT;
            cp[o + 6 * TILE_PIX] = Dp[kk] * rT;
            cp[o + 7 * TILE_PIX] = (Tc - T[kk]) * rT;  // weights from ck on: T(ck) - T_end (telescoping)
            cp[o + 8 * TILE_PIX] = T[kk] * rT;
            C0[kk] = b0 + C0[kk];  // the outputs: the sums before ck plus those from ck on
            C1[kk] = b1 + C1[kk];
            C2[kk] = b2 + C2[kk];
            S0[kk] = b3 + S0[kk];
            S1[kk] = b4 + S1[kk];
            Dp[kk] = b5 + Dp[kk];
        }
    }
    WT_END(0, wslot, tile, n, deepest, NQ)
    const float bg0 = bg[0], bg1 = bg[1], bg2 = bg[2];
    const size_t HW = (size_t)H * W;
#pragma unroll
    for (int kk = 0; kk < NQ; ++kk) {
        const int k = q0 + kk;
        n_contrib[(size_t)tile * TILE_PIX + k * 64 + lane] = last[kk];
        const int px = px0 + 8 * (k & 1), py = py0 + 8 * (k >> 1);
        if (!(px < W && py < H)) continue;
        const size_t pix = (size_t)py * W + px;
        out_color[pix] = C0[kk] + T[kk] * bg0;
        out_color[HW + pix] = C1[kk] + T[kk] * bg1;
        out_color[2 * HW + pix] = C2[kk] + T[kk] * bg2;
        out_alpha[pix] = Wt[kk];
        out_depth[pix] = Dp[kk];
        out_segment[pix] = S0[kk];
        out_segment[HW + pix] = S1[kk];
    }
}

// Block b < 4 Qs: quadrant (b & 3) of the heaviest tile order[b >> 2] (the first Qs entries
// of the heavy-first schedule, sched[SCHED_FWD_QUARTER]); then, up to Hs (sched[SCHED_FWD_SPLIT],
// Hs >= Qs), half (b & 1) of the next heavy tiles; then one wave per remaining tile.  The grid is
// sized for the worst case; blocks past the work return at once.  Quarter waves (option
// split4_fwd_bucket, off by default) measured slower at every threshold (metric scene, render_fwd
// 0.206 ms without; n >= 2048: 0.222, >= 1024: 0.233, >= 512: 0.246, >= 256: 0.241): each quarter
// wave repeats the batch loads, the prefilter and the per-instance record reads and ballots for
// one 8x8 quadrant (profiles/round3_quarter_sweep.txt).
// Minimum waves per SIMD for the register allocator: with 4 the kernel still fits 96 VGPRs (5
// waves/SIMD) but is scheduled differently, and measured 1.4% faster than with 5 (render_fwd
// 193.6 / 193.8 vs 195.9 / 197.1 us, profiles/round4_bwd_segments.txt); 6-8 were slower in round 3.
#if GSR_RENDER_PART != 2
#ifndef GSR_FWD_WAVES
#define GSR_FWD_WAVES 4
#endif
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(GSR_FWD_WAVES))) k_render_fwd(int W, int H, int gx, int T, const uint32_t* __restrict__ order,
                                                   uint32_t* __restrict__ sched,
                                                   const uint2* __restrict__ ranges,
                                                   const uint32_t* __restrict__ point_list,
                                                   const float4* __restrict__ rec, const float* __restrict__ bg,
                                                   float* __restrict__ out_color, float* __restrict__ out_depth,
                                                   float* __restrict__ out_alpha, float* __restrict__ out_segment,
                                                   uint32_t* __restrict__ n_contrib, float* __restrict__ ckpt, int ck,
                                                   int xcd_pairs) {
    __shared__ float4 srec[64][4];
    const TileSched ts = tile_sched(sched - T, T);
    if (blockIdx.x == 0 && threadIdx.x == 0) sched[SCHED_CKPT] = (uint32_t)ck;  // for the backward
    const uint32_t Hs = min(sched[SCHED_FWD_SPLIT], (uint32_t)T);
    const uint32_t Qs = min(sched[SCHED_FWD_QUARTER], Hs);
    const uint32_t b = blockIdx.x;
    if (b < 4 * Qs) {
        fwd_tile<1>(W, H, gx, T, (int)order[b >> 2], (int)(b & 3), (int)b, ts, ranges, point_list, rec, bg,
                    out_color, out_depth, out_alpha, out_segment, n_contrib, ckpt, ck, srec);
    } else if (b < 4 * Qs + 2 * (Hs - Qs)) {
        const uint32_t h = b - 4 * Qs;
        uint32_t ti = h >> 1, half = h & 1;
        if (xcd_pairs) {
            // the two halves of a tile read the same records: give them blocks b and b + 8, which
            // the dispatcher sends to the same XCD (round robin over the 8), so the second half
            // finds the records in that XCD's L2.  Chunks of 16 blocks = 8 tiles; the last
            // M % 8 tiles keep the adjacent pairing.
            const uint32_t M = Hs - Qs, full = (M / 8) * 16;
            if (h < full) {
                ti = 8 * (h / 16) + (h & 7);
                half = (h >> 3) & 1;
            }
        }
        fwd_tile<2>(W, H, gx, T, (int)order[Qs + ti], 2 * (int)half, (int)b, ts, ranges, point_list, rec,
                    bg, out_color, out_depth, out_alpha, out_segment, n_contrib, ckpt, ck, srec);
    } else {
        const uint32_t i = b - 2 * Qs - Hs;  // = Hs + (b - 4 Qs - 2 (Hs - Qs))
        if (i >= (uint32_t)T) return;
        fwd_tile<4>(W, H, gx, T, (int)order[i], 0, (int)b, ts, ranges, point_list, rec, bg, out_color, out_depth,
                    out_alpha, out_segment, n_contrib, ckpt, ck, srec);
    }
}
#endif  // GSR_RENDER_PART != 2

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
#ifndef GSR_DIV_NO_ASM
    // the correction as a three-address v_fma_f32: as v_fmac (destination = q's register) the
    // replay's loop-carried T needed a v_mov per strip to get back into its own register
    float t;
    asm("v_fma_f32 %0, %1, %2, %3" : "=v"(t) : "v"(e), "v"(r), "v"(q));
    return t;
#else
    return __builtin_fmaf(e, r, q);
#endif
#endif
}

// LDS of one backward block (two waves): each wave parks its own copy of the batch
// records; split tiles also exchange their per-wave partial records and the batch count.
struct BwdShared {
    float4 srec[2][64][4];  // per wave: the batch's records
    float part[2][64][12];  // split tiles: per-wave partial record of each batch instance
    float4 stage[2][64][3]; // unsplit tiles: per-wave records of the batch, stored at the next batch
    uint64_t tmask[2];      // split tiles: instances each wave produced a partial for
    uint32_t top[2];        // split tiles: per-wave deepest contributor
};

// LDS write -> read by other lanes of the SAME wave: a wave's LDS instructions execute in
// order, so a compiler barrier plus the LDS counter wait is enough (no s_barrier: in the
// unsplit mode the block's other wave renders another tile, or has already ended).
__device__ __forceinline__ void wave_lds_sync() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

// Backward of one tile (NS = 4 strips of 16x4 pixels, one wave) or of half of it (NS = 2:
// strips s0, s0 + 1 = the top or the bottom 16x8 half, SPLIT: the block's two waves
// cooperate on one tile).  A split tile's two waves walk the same batches (the deeper of
// the halves' last contributors bounds both); per batch each wave reduces its partial
// record of an instance into LDS, and after a block barrier the block sums the two
// partials in a fixed order (wave 0 + wave 1: deterministic) and stores the record.
template <int NS, bool SPLIT>
__device__ __forceinline__ void bwd_tile(int W, int H, int gx, int tile, int s0, int wslot,
                                         const uint2* __restrict__ ranges,
                                         const uint32_t* __restrict__ point_list,
                                         const uint32_t* __restrict__ bbase,
                                         const float4* __restrict__ rec, const float* __restrict__ bg,
                                         const float* __restrict__ alphas,
                                         const uint32_t* __restrict__ n_contrib,
                                         const float* __restrict__ dL_dpixels,
                                         const float* __restrict__ dL_dsegs,
                                         const float* __restrict__ dL_ddepths,
                                         const float* __restrict__ dL_dalphas,
                                         float* __restrict__ contrib, uint8_t* __restrict__ written,
                                         float4 (*srec)[4], BwdShared* sh, float4 (*stage)[3] = nullptr,
                                         int seg_lo = 0, int seg_hi = 0x7fffffff,
                                         const float* __restrict__ ckpt = nullptr) {
#pragma clang fp contract(off)
    WT_BEGIN
    const int lane = threadIdx.x & 63, wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int tx = tile % gx, ty = tile / gx;
    const int px = tx * BX + (lane & 15);
    const int py0 = ty * BY + (lane >> 4) + 4 * s0;
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
    // The background term of dL_dalpha, -T_final / (1 - alpha) * (bg . dL_dpix) per
    // contributor (backward.cu:593-597), is the same recurrence's contribution of a virtual
    // last contributor with colour bg (and 0 in the segment / depth / alpha channels) and
    // alpha 1: Dk starts at bg . dL_dpix instead of 0, and (cdot - Dk) * T then carries
    // -(bg . dL_dpix) T_final / (1 - alpha) at every contributor.  No bg-specialised loop, no
    // T_final / bg . dL_dpix registers and no extra rcp per replayed pair.
    float pfy[NS], T[NS], dp0[NS], dp1[NS], dp2[NS], ds0[NS], ds1[NS], dd[NS], da[NS];
    float Dk[NS];
    uint32_t lastc[NS];
    uint32_t maxlast = 0;
#pragma unroll
    for (int k = 0; k < NS; ++k) {
        const int py = py0 + 4 * k;
        pfy[k] = (float)py;
        const bool inside = px < W && py < H;
        const size_t pix = inside ? (size_t)py * W + px : 0;
        // n_contrib is in the forward's quadrant layout (entry 64 k' + 8 (row & 7) + (col & 7))
        const int r = (lane >> 4) + 4 * (s0 + k), c = lane & 15;
        const int fidx = 64 * (2 * (r >> 3) + (c >> 3)) + 8 * (r & 7) + (c & 7);
        lastc[k] = inside ? n_contrib[(size_t)tile * TILE_PIX + fidx] : 0u;
        T[k] = inside ? 1.f - alphas[pix] : 0.f;  // T_final (backward.cu:468)
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
        Dk[k] = bgd;
        if (ckpt != nullptr && lastc[k] > (uint32_t)seg_hi) {
            // front segment (publish_depth): the replay state at seg_hi from the forward's checkpoint
            const float* q = ckpt + (size_t)tile * CKPT_FLOATS + fidx;
            float d = bgd * q[8 * TILE_PIX];
            d = __builtin_fmaf(dp0[k], q[1 * TILE_PIX], d);
            d = __builtin_fmaf(dp1[k], q[2 * TILE_PIX], d);
            d = __builtin_fmaf(dp2[k], q[3 * TILE_PIX], d);
            d = __builtin_fmaf(ds0[k], q[4 * TILE_PIX], d);
            d = __builtin_fmaf(ds1[k], q[5 * TILE_PIX], d);
            d = __builtin_fmaf(dd[k], q[6 * TILE_PIX], d);
            d = __builtin_fmaf(da[k], q[7 * TILE_PIX], d);
            Dk[k] = d;
            T[k] = q[0];
        }
        maxlast = max(maxlast, lastc[k]);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) maxlast = max(maxlast, (uint32_t)__shfl_xor((int)maxlast, o, 64));
    int top0 = min((int)__builtin_amdgcn_readfirstlane(maxlast), seg_hi);
    if constexpr (SPLIT) {  // both waves walk the same batches (their barriers pair up)
        if (lane == 0) sh->top[wid] = (uint32_t)top0;
        __syncthreads();
        top0 = (int)max(sh->top[0], sh->top[1]);
    }

    const uint2 range = ranges[tile];
    const int n = (int)(range.y - range.x);
    // prefilter rectangle: the pixels this wave owns
    const float x0 = (float)(tx * BX), y0 = (float)(ty * BY + 4 * s0);
    const float x1 = (float)min(tx * BX + BX - 1, W - 1), y1 = (float)min(ty * BY + 4 * (s0 + NS) - 1, H - 1);

    STAT_DECL
    STAT(7, n);
    STAT(6, n > top0 ? n - top0 : 0);
    // Same two-stage batch pipeline and LDS record broadcast as the forward, walking
    // the list back to front: lane l of the batch with upper end `top` owns position top-1-l.
    const uint32_t* plist = point_list + range.x;
    // list positions below 0 are clamped to 0 (unconditional loads, see fetch_batch)
    uint32_t g_next = 0u;
    BatchB cur;
    if (top0 > 0) {
        g_next = plist[max(top0 - 1 - lane, 0)];
        cur = fetch_batch_b(rec, bbase, g_next);
    }
    if (top0 > 0) g_next = plist[max(top0 - 65 - lane, 0)];
    // Unsplit tiles park a batch's records in LDS (stage[j] = record of batch instance j) and
    // store them at the start of the next batch, ahead of its prefetch loads.  gfx950 counts
    // vector loads and stores in one in-order vmcnt: with the records stored inside the batch,
    // taking over the prefetched batch at its end waited for every record store's
    // acknowledgement (an s_waitcnt vmcnt(0) per batch).
    uint64_t prev_touched = 0;
    uint32_t prev_uslot = 0;
    auto flush = [&]() {
        if constexpr (!SPLIT) {
            if ((prev_touched >> lane) & 1ull) {
                float4* d = reinterpret_cast<float4*>(contrib + (size_t)prev_uslot * CONTRIB_STRIDE);
                const float4 a = stage[lane][0], b = stage[lane][1], c = stage[lane][2];
                d[0] = a;
                d[1] = b;
                d[2] = c;
                // byte u marks slot u as written
                written[prev_uslot] = 1;
            }
        }
    };
    auto replay = [&]() {
        for (int top = top0; top > seg_lo; top -= 64) {
            const int cnt = min(64, top - seg_lo);
            STAT(5, 1);
            STAT(13, cnt);  // instances fetched (records read)
            flush();
            const BatchB nxt = fetch_batch_b(rec, bbase, g_next);
            g_next = plist[max(top - 129 - lane, 0)];
            const float4 ra = cur.a, rb = cur.b, rc = cur.c;
            const uint32_t uslot = batch_slot(cur, tx, ty);  // the instance's record slot
            cur = nxt;
            const float pmin = power_floor(rb.y);
            // Lanes replaying every position of this batch (p < n_contrib for all p < top) and
            // whether any lane starts replaying inside it: only then is p < n_contrib
            // tested per instance.  Strips with no pixel replaying any position of the batch
            // are idle: no powers for them, and the prefilter rectangle shrinks to the rows of
            // the active strips (deep tiles start with few pixels replaying).
            uint64_t act_all[NS];
            bool varying = false;
            uint32_t active = 0;  // bit k: strip k has a pixel replaying in this batch
#pragma unroll
            for (int k = 0; k < NS; ++k) {
                act_all[k] = __builtin_amdgcn_ballot_w64(lastc[k] >= (uint32_t)top);
                varying |= lastc[k] < (uint32_t)top && lastc[k] > (uint32_t)(top - cnt);
                if (__builtin_amdgcn_ballot_w64(lastc[k] > (uint32_t)(top - cnt))) active |= 1u << k;
            }
            const bool vary = wave_any(varying);
#ifndef GSR_NO_LIVE_RECT
            const int kmin = active ? __builtin_ctz(active) : 0, kmax = active ? 31 - __builtin_clz(active) : 0;
            const float ay0 = y0 + 4.f * kmin, ay1 = fminf(y1, y0 + 4.f * kmax + 3.f);
            const bool hit = lane < cnt && tile_hit(ra.x, ra.y, ra.z, ra.w, rb.x, pmin, x0, x1, ay0, ay1);
#else
            const bool hit = lane < cnt && tile_hit(ra.x, ra.y, ra.z, ra.w, rb.x, pmin, x0, x1, y0, y1);
#endif
            uint64_t todo = __ballot(hit);
            STAT(9, vary);
            STAT(2, cnt - __popcll(todo));
            wave_lds_sync();  // this wave's reads of the previous batch are issued before the writes
            srec[lane][0] = ra;                                                   // x, y, conic a, b
            srec[lane][1] = make_float4(rb.x, pmin, rb.y, rb.w);                  // conic c, power floor, opacity, seg0
            srec[lane][2] = rc;                                                   // r, g, b, seg1
            srec[lane][3] = make_float4(rb.z, __uint_as_float(uslot), 0.f, 0.f);  // depth, record slot
            wave_lds_sync();
            uint64_t touched = 0;  // instances with a (partial, SPLIT) record from this wave
            while (todo) {
                const int j = (int)__builtin_ctzll(todo);
                todo &= todo - 1;
                const uint32_t p = (uint32_t)(top - 1 - j);
                const float4 q0 = srec[j][0], q1 = srec[j][1];
                const float gx_ = q0.x, gy_ = q0.y, ca = q0.z, cb = q0.w, cc = q1.x, pm = q1.y;
                float power[NS], dys[NS];
                uint64_t act[NS];
#pragma unroll
                for (int k = 0; k < NS; ++k) act[k] = act_all[k];
                if (vary) {
#pragma unroll
                    for (int k = 0; k < NS; ++k) act[k] = __builtin_amdgcn_ballot_w64(p < lastc[k]);
                }
                uint64_t near[NS];  // per strip: lanes whose pixel replays p and is within reach
                uint64_t any_near = 0;
                const float dx = gx_ - pfx;
                const float adxdx = ca * dx * dx, bdx = cb * dx;
#pragma unroll
                for (int k = 0; k < NS; ++k) {
#ifdef GSR_DEAD_SKIP
                    if (!(active & (1u << k))) {  // idle strip in this batch
                        near[k] = 0;
                        power[k] = dys[k] = 0.f;
                        continue;
                    }
#endif
#ifdef GSR_PFY_RECOMPUTE
                    const float dy = gy_ - (pfy[0] + 4.f * k);  // the same exact pixel-centre float
#else
                    const float dy = gy_ - pfy[k];
#endif
                    dys[k] = dy;
                    power[k] = __builtin_fmaf(-0.5f, adxdx + cc * dy * dy, -(bdx * dy));  // == -0.5 S - B
                    near[k] = act[k] & __builtin_amdgcn_ballot_w64(power[k] >= pm);
                    any_near |= near[k];
                }
                STAT(0, 1);
                if (!any_near) {
                    STAT(1, 1);
                    continue;
                }
                STAT(3, 1);
                const float4 q2 = srec[j][2], q3 = srec[j][3];
                const float op = q1.z, dep = q3.x, s0v = q1.w;
#ifdef GSR_STATS
                unsigned long long okst_ = st_[12];
#endif
                const float c0 = q2.x, c1 = q2.y, c2 = q2.z, s1v = q2.w;
                float acc[12];
#pragma unroll
                for (int i = 0; i < 12; ++i) acc[i] = -0.0f;  // -0 + x == x: the first add folds away
                // Strip k (rows 4k..4k+3) is replayed only if one of its pixels can pass.
#pragma unroll
                for (int k = 0; k < NS; ++k) {
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
                    STAT(10, POPC(o) == 0);
                    STAT(12, POPC(o) > 0);
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
                    cdot = __builtin_fmaf(s0v, ds0[k], cdot);
                    cdot = __builtin_fmaf(s1v, ds1[k], cdot);
                    cdot = __builtin_fmaf(dep, dd[k], cdot);
                    const float diff = cdot - Dk[k];
                    float dopa = diff * Tn;

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
                // The mean2D channels carry the conic-weighted sums per lane,
                // sum q (a dx + b dy) and sum q (b dx + c dy), as the reference's per-pixel
                // dG_ddelx / dG_ddely terms (backward.cu:612-621), instead of the moments
                // Qx, Qy combined after the reduction: for an elongated Gaussian a Qx and
                // b Qy nearly cancel, which amplified the moments' rounding ~100x there.
                {
                    const float qx = dx * acc[6];  // sum q dx (dx is shared by the lane's pixels)
                    const float qy = acc[8];
                    acc[9] = dx * qx;              // sum q dx^2
                    acc[10] = dx * qy;             // sum q dx dy
                    acc[7] = __builtin_fmaf(ca, qx, cb * qy);
                    acc[8] = __builtin_fmaf(cc, qy, cb * qx);
                }
#ifdef GSR_STATS
                STAT(11, st_[12] == okst_);
#endif
                int vidx;
                bool valid;
                const float r = wave_reduce12(acc, lane, vidx, valid);
                if constexpr (SPLIT) {
                    if (valid) sh->part[wid][j][vidx] = r;
                } else {
                    if (valid) reinterpret_cast<float*>(stage[j])[vidx] = r;
                }
                touched |= 1ull << j;
            }
            if constexpr (!SPLIT) {
                prev_touched = touched;
                prev_uslot = uslot;
            }
            if constexpr (SPLIT) {
                if (lane == 0) sh->tmask[wid] = touched;
                __syncthreads();
                // 128 threads: instance j = t / 2, channels 6 (t & 1) .. + 5; partials summed
                // wave 0 + wave 1 (0 + x == x for a half that had none)
                const int t = threadIdx.x, jj = t >> 1, h = t & 1;
                const uint64_t m0 = sh->tmask[0], m1 = sh->tmask[1];
                if (((m0 | m1) >> jj) & 1ull) {
                    const bool w0 = (m0 >> jj) & 1ull, w1 = (m1 >> jj) & 1ull;
                    const uint32_t u = __float_as_uint(sh->srec[0][jj][3].y);
                    float v[6];
#pragma unroll
                    for (int c = 0; c < 6; ++c)
                        v[c] = (w0 ? sh->part[0][jj][6 * h + c] : 0.f) + (w1 ? sh->part[1][jj][6 * h + c] : 0.f);
                    float2* d = reinterpret_cast<float2*>(contrib + (size_t)u * CONTRIB_STRIDE + 6 * h);
                    d[0] = make_float2(v[0], v[1]);
                    d[1] = make_float2(v[2], v[3]);
                    d[2] = make_float2(v[4], v[5]);
                    if (h == 0) written[u] = 1;
                }
                __syncthreads();  // the partials are read before the next batch overwrites them
            }
        }
    };
    replay();
    flush();
    STAT_FLUSH(16)
    // mode: strips | 16 front segment | 32 back segment (from seg_lo = ck)
    WT_END(1, wslot, tile, n, top0, NS | (seg_hi < 0x7fffffff ? 16 : 0) | (seg_lo > 0 ? 32 : 0))
}

#if GSR_RENDER_PART != 1
// The backward walks the forward's depth queue deepest first (TileSched): global work
// index i -> bucket (a wave prefix over the 63 bucket counts, descending) -> tile.  Tiles
// at least split_depth deep come first, one per block (top / bottom half on wave 0 / 1);
// then two tiles per block, one per wave.  The grid is sized for no split (T / 2 ... T
// blocks); blocks or waves past the queue return.  A tile's wave time grows with its
// depth (the list positions it replays), so deepest-first is the longest-first order.
// Returns the queue entry (tile | segment kind, publish_depth), or BQ_NONE past the queue.
constexpr uint32_t BQ_NONE = ~0u;
__device__ __forceinline__ uint32_t queue_tile(const TileSched& ts, int T, uint32_t i, uint32_t pre, uint32_t cnt) {
    // pre / cnt: this lane's bucket (63 - lane) exclusive prefix and count (lane 63: bucket 0, empty)
    const uint64_t m = __builtin_amdgcn_ballot_w64(cnt > 0 && pre <= i);
    if (!m) return BQ_NONE;
    const int L = 63 - __builtin_clzll(m);  // the last non-empty bucket starting at or before i
    const uint32_t pL = __builtin_amdgcn_readlane(pre, L), cL = __builtin_amdgcn_readlane(cnt, L);
    if (i >= pL + cL) return BQ_NONE;
    return (uint32_t)__builtin_amdgcn_readfirstlane((int)ts.bq_list[(size_t)(63 - L) * bq_cap(T) + (i - pL)]);
}

__global__ void __launch_bounds__(128) __attribute__((amdgpu_waves_per_eu(4))) k_render_bwd(
    int W, int H, int gx, int T, int split_depth, uint32_t* __restrict__ sched,
    const uint2* __restrict__ ranges, const uint32_t* __restrict__ point_list, const uint32_t* __restrict__ bbase,
    const float4* __restrict__ rec, const float* __restrict__ bg, const float* __restrict__ alphas,
    const uint32_t* __restrict__ n_contrib, const float* __restrict__ dL_dpixels, const float* __restrict__ dL_dsegs,
    const float* __restrict__ dL_ddepths, const float* __restrict__ dL_dalphas, float* __restrict__ contrib,
    uint8_t* __restrict__ written) {
    __shared__ BwdShared sh;
    const int lane = threadIdx.x & 63, wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const TileSched ts = tile_sched(sched - T, T);
    // lane l: bucket 63 - l (deepest first); exclusive prefix over the lanes
    const uint32_t cnt = lane < 63 ? ts.bq_cnt[63 - lane] : 0u;
    uint32_t pre = cnt;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = (uint32_t)__shfl_up((int)pre, o, 64);
        if (lane >= o) pre += y;
    }
    pre -= cnt;
    // split tiles: buckets >= depth_bucket(split_depth), i.e. lanes <= 63 - that bucket
    const int sb = split_depth > 0 ? (int)depth_bucket((uint32_t)split_depth) : 64;
    const uint32_t Hs = sb < 64 ? (uint32_t)__builtin_amdgcn_readlane(pre + cnt, 63 - sb) : 0u;
    const uint32_t b = blockIdx.x;
    const bool split = b < Hs;  // block-uniform
    const uint32_t e = queue_tile(ts, T, split ? b : Hs + 2 * (b - Hs) + (uint32_t)wid, pre, cnt);
    if (e == BQ_NONE) return;  // past the queue (a split block's waves share the tile: both return or neither)
    // the forward runs without list segments for this kernel (launch_render_forward); a segment
    // entry would be replayed whole, i.e. its records written twice with the same values
    const int tile = (int)(e & BQ_TILE);
    if (split) {
        bwd_tile<2, true>(W, H, gx, tile, 2 * wid, (int)(2 * b + wid), ranges, point_list, bbase, rec, bg,
                          alphas, n_contrib, dL_dpixels, dL_dsegs, dL_ddepths, dL_dalphas, contrib, written,
                          sh.srec[wid], &sh);
    } else {
        bwd_tile<4, false>(W, H, gx, tile, 0, (int)(2 * b + wid), ranges, point_list, bbase, rec, bg, alphas,
                           n_contrib, dL_dpixels, dL_dsegs, dL_ddepths, dL_dalphas, contrib, written, sh.srec[wid],
                           nullptr, sh.stage[wid]);
    }
}

// No split (split_bwd_depth = 0): one wave per block and tile, deepest first.
// Waves per SIMD.  With one wave per tile, 5 (96 VGPRs, ~11 values spilled and reloaded once per
// batch) ran 2.8% faster than 4 (profiles/round4_bwd_waves.txt); with list segments, whose
// entries are shorter and twice as many, 4 waves (no spills) run 1.5% faster than 5
// (k_render_bwd1 350.3 / 349.9 vs 354.7 / 356.8 us, profiles/round4_bwd_segments.txt).
#ifndef GSR_BWD1_WAVES
#define GSR_BWD1_WAVES 4
#endif
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(GSR_BWD1_WAVES))) k_render_bwd1(
    int W, int H, int gx, int T, uint32_t* __restrict__ sched,
    const uint2* __restrict__ ranges, const uint32_t* __restrict__ point_list, const uint32_t* __restrict__ bbase,
    const float4* __restrict__ rec, const float* __restrict__ bg, const float* __restrict__ alphas,
    const uint32_t* __restrict__ n_contrib, const float* __restrict__ dL_dpixels, const float* __restrict__ dL_dsegs,
    const float* __restrict__ dL_ddepths, const float* __restrict__ dL_dalphas, float* __restrict__ contrib,
    uint8_t* __restrict__ written, const float* __restrict__ ckpt) {
    __shared__ float4 srec[64][4];
    __shared__ float4 stage[64][3];
    const int lane = threadIdx.x & 63;
    const TileSched ts = tile_sched(sched - T, T);
    const uint32_t cnt = lane < 63 ? ts.bq_cnt[63 - lane] : 0u;
    uint32_t pre = cnt;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = (uint32_t)__shfl_up((int)pre, o, 64);
        if (lane >= o) pre += y;
    }
    pre -= cnt;
    const uint32_t e = queue_tile(ts, T, blockIdx.x, pre, cnt);
    if (e == BQ_NONE) return;
    // a whole tile, or one of its list segments [0, ck) / [ck, depth) (publish_depth)
    const uint32_t kind = e & ~BQ_TILE;
    const int ck = (int)ts.sched[SCHED_CKPT];
    bwd_tile<4, false>(W, H, gx, (int)(e & BQ_TILE), 0, (int)blockIdx.x, ranges, point_list, bbase, rec,
                       bg, alphas, n_contrib, dL_dpixels, dL_dsegs, dL_ddepths, dL_dalphas, contrib, written, srec,
                       nullptr, stage, kind == BQ_BACK ? ck : 0, kind == BQ_FRONT ? ck : 0x7fffffff,
                       kind == BQ_FRONT ? ckpt : nullptr);
}

#endif  // GSR_RENDER_PART != 1
}  // namespace

#if GSR_RENDER_PART != 2
void set_bwd_ckpt(int pos) { g_bwd_ckpt = pos > 0 ? (pos + 63) / 64 * 64 : 0; }
void set_fwd_xcd_pairs(int on) { g_fwd_xcd_pairs = on ? 1 : 0; }
int bwd_ckpt() { return g_bwd_ckpt; }

void launch_render_forward(int W, int H, int gx, int gy, const uint32_t* order, uint32_t* sched,
                           const uint2* ranges, const uint32_t* point_list, const float4* rec, const float* bg,
                           float* out_color, float* out_depth, float* out_alpha, float* out_segment,
                           uint32_t* n_contrib, float* ckpt, hipStream_t st) {
    const int T = gx * gy;
    if (T == 0) return;
    // list segments only for the one-wave backward (k_render_bwd1)
    const int ck = split_bwd_depth() <= 0 ? g_bwd_ckpt : 0;
    // grid for the worst case of the schedule: 2T blocks with halves only, 4T with quarters
    hipLaunchKernelGGL(k_render_fwd, dim3((split4_fwd_bucket() > 0 ? 4 : 2) * T), dim3(64), 0, st, W, H, gx, T, order,
                       sched, ranges, point_list,
                       rec, bg, out_color, out_depth, out_alpha, out_segment, n_contrib, ckpt, ck, g_fwd_xcd_pairs);
}
#endif  // GSR_RENDER_PART != 2

#if GSR_RENDER_PART != 1
void launch_render_backward(int W, int H, int gx, int gy, const uint32_t* order, uint32_t* sched,
                            const uint2* ranges, const uint32_t* point_list, const uint32_t* bbase,
                            const float4* rec, const float* bg, const float* alpha, const uint32_t* n_contrib,
                            const float* dL_dcolor, const float* dL_dsegment, const float* dL_ddepth,
                            const float* dL_dalpha, float* contrib, uint8_t* written, const float* ckpt,
                            hipStream_t st) {
    const int T = gx * gy;
    if (T == 0) return;
    (void)order;  // the backward follows the forward's depth queue
    if (split_bwd_depth() <= 0) {
        // up to two queue entries per tile (list segments); blocks past the queue return at once
        hipLaunchKernelGGL(k_render_bwd1, dim3(2 * T), dim3(64), 0, st, W, H, gx, T, sched, ranges, point_list,
                           bbase, rec, bg, alpha, n_contrib, dL_dcolor, dL_dsegment, dL_ddepth, dL_dalpha,
                           contrib, written, ckpt);
        return;
    }
    hipLaunchKernelGGL(k_render_bwd, dim3(T), dim3(128), 0, st, W, H, gx, T, split_bwd_depth(), sched, ranges,
                       point_list,
                       bbase, rec, bg, alpha, n_contrib, dL_dcolor, dL_dsegment, dL_ddepth, dL_dalpha, contrib,
                       written);
}

#endif  // GSR_RENDER_PART != 1

}  // namespace gsr
