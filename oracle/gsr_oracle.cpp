// ============================================================================
// gsr_oracle.cpp -- CPU restatement of the reference differentiable Gaussian
// rasterizer (submodules_local/diff-gaussian-rasterization, "DGR/").
//
// TEST INFRASTRUCTURE ONLY.  This file is the parity oracle and the CPU
// baseline.  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
// leg may load it; the product path (libgsr.so) never links or calls it.
//
// Parity status: the reference CUDA path cannot be built here (no nvcc/CUB,
// un-vendored glm submodule: DGR/.gitmodules:1-3), and the reference ships no
// tests, fixtures or golden vectors for this path.  The
// restatement is pinned by (a) golden vectors generated from the reference's
// own importable Python (utils/sh_utils.py eval_sh, utils/graphics_utils.py
// camera matrices: tests/golden/make_golden.py), and (b) a float64 PyTorch
// autograd restatement of the same math (tests/test_oracle_autograd.py) that
// checks this file's hand-derived backward against true derivatives.
//
// Numerics follow the reference line by line:
//   * glm column-major mat3 (m[col][row]); (A*B)[c][r] = sum_k A[k][r]*B[c][k],
//     evaluated left to right (glm type_mat3x3.inl operator*).
//   * ndc2Pix in double (DGR/cuda_rasterizer/auxiliary.h:41-44).
//   * (int) truncation in getRect (auxiliary.h:46-56).
//   * tie order of the (tile|depth) radix sort = original emission order
//     (rasterizer_impl.cu:304-312, CUB SortPairs is stable).
//   * sequential per-pixel blending (forward.cu:314-377, backward.cu:508-638).
// Built with -ffp-contract=off: every a*b+c is two roundings, the same
// evaluation order the HIP preprocess uses (it also disables contraction), so
// integer outputs (radii, tiles, keys, point_list, ranges) compare bit-exact.
// ============================================================================
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <numeric>
#include <string>
#include <vector>
#ifdef _OPENMP
#include <omp.h>
#include <parallel/algorithm>
#endif

namespace {

constexpr int BX = 16, BY = 16;          // DGR/cuda_rasterizer/config.h:17-18
constexpr int NCH = 3, NCLS = 2;         // config.h:15-16

// auxiliary.h:21-39
const float SH_C0 = 0.28209479177387814f;
const float SH_C1 = 0.4886025119029199f;
const float SH_C2[] = {1.0925484305920792f, -1.0925484305920792f, 0.31539156525252005f,
                       -1.0925484305920792f, 0.5462742152960396f};
const float SH_C3[] = {-0.5900435899266435f, 2.890611442640554f, -0.4570457994644658f,
                       0.3731763325901154f, -0.4570457994644658f, 1.445305721320277f,
                       -0.5900435899266435f};

struct v3 { float x, y, z; };
static inline v3 operator+(v3 a, v3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
static inline v3 operator-(v3 a, v3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
static inline v3 operator*(float s, v3 a) { return {s * a.x, s * a.y, s * a.z}; }
static inline v3 operator*(v3 a, float s) { return {a.x * s, a.y * s, a.z * s}; }
static inline v3 operator/(v3 a, float s) { return {a.x / s, a.y / s, a.z / s}; }
static inline float dot(v3 a, v3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }

// ---------------------------------------------------------------------------------------------
// nvcc contraction model (VERDICT r5 "Next" #1).  DGR is built with nvcc's defaults
// (DGR/setup.py:17-34: --fmad=true, no fast-math), so the reference binary contracts a*b+c into
// FMAs, while this oracle (-ffp-contract=off) and gsr round twice.  With g_contract != 0 the
// oracle evaluates the sites that decide integer outputs the way LLVM's DAG combiner (NVVM's
// code generator) contracts them:
//   * fadd/fsub of a bare product and anything: the product is fused (fma(a, b, +-z));
//   * of two bare products: the LEFT one is fused, the right one rounded (equal use counts;
//     CT_RIGHT fuses the right one instead, to bracket the model);
//   * a sum chain p0 + p1 + p2 (+ c): fma(a2, b2, fma(a0, b0, p1)) (+ c) -- the running sum
//     is no longer a bare product, so each later product is fused into it.
// Bits: CT_PRE = projection (auxiliary.h:58-77 transformPoint4x3/4x4, in_frustum :139-164),
// ndc2Pix (:41-44, in double), computeCov3D (forward.cu:118-152), computeCov2D (:74-113), the
// determinant / eigenvalue / radius lines (:219-232); CT_BLEND = the blend's power and its
// colour / weight / depth / segment sums (forward.cu:346, 362-366; the backward's power,
// backward.cu:541, so the replay sees the forward's decisions).  Default 0 = gsr's evaluation.
// ptxas may fuse further pairs on its own; the model does not claim to be the binary, it
// measures how many integer outputs a last-bit change of this kind moves.
enum { CT_PRE = 1, CT_BLEND = 2, CT_RIGHT = 4 };
static int g_contract = 0;
static inline float pp_add(int c, float a, float b, float x, float y) {  // a*b + x*y
    if (!c) return a * b + x * y;
    return (c & CT_RIGHT) ? std::fma(x, y, a * b) : std::fma(a, b, x * y);
}
static inline float pp_sub(int c, float a, float b, float x, float y) {  // a*b - x*y
    if (!c) return a * b - x * y;
    return (c & CT_RIGHT) ? std::fma(-x, y, a * b) : std::fma(a, b, -(x * y));
}
static inline float dot3c(int c, float a0, float b0, float a1, float b1, float a2, float b2) {
    if (!c) return a0 * b0 + a1 * b1 + a2 * b2;
    return std::fma(a2, b2, pp_add(c, a0, b0, a1, b1));
}
static inline int ct_pre() { return (g_contract & CT_PRE) ? (g_contract | CT_PRE) : 0; }
static inline int ct_blend() { return (g_contract & CT_BLEND) ? (g_contract | CT_BLEND) : 0; }

// glm mat3: m[col][row]; mat3(a..i) fills columns.
struct m3 { float m[3][3]; };
static inline m3 mk(float a, float b, float c, float d, float e, float f, float g, float h, float i) {
    m3 r;
    r.m[0][0] = a; r.m[0][1] = b; r.m[0][2] = c;
    r.m[1][0] = d; r.m[1][1] = e; r.m[1][2] = f;
    r.m[2][0] = g; r.m[2][1] = h; r.m[2][2] = i;
    return r;
}
static inline m3 mul(const m3& A, const m3& B, int ct = 0) {
    m3 R;
    for (int c = 0; c < 3; ++c)
        for (int r = 0; r < 3; ++r)
            R.m[c][r] = dot3c(ct, A.m[0][r], B.m[c][0], A.m[1][r], B.m[c][1], A.m[2][r], B.m[c][2]);
    return R;
}
static inline m3 tr(const m3& A) {
    m3 R;
    for (int c = 0; c < 3; ++c)
        for (int r = 0; r < 3; ++r) R.m[c][r] = A.m[r][c];
    return R;
}
static inline m3 smul(float s, const m3& A) {
    m3 R;
    for (int c = 0; c < 3; ++c)
        for (int r = 0; r < 3; ++r) R.m[c][r] = s * A.m[c][r];
    return R;
}
static inline v3 col(const m3& A, int c) { return {A.m[c][0], A.m[c][1], A.m[c][2]}; }

// auxiliary.h:41-44 (double arithmetic, float result)
static inline float ndc2Pix(float v, int S, int ct = 0) {
    if (ct) return (float)(std::fma((double)v + 1.0, (double)S, -1.0) * 0.5);
    return (float)(((v + 1.0) * S - 1.0) * 0.5);
}

// auxiliary.h:46-56
static inline void getRect(float px, float py, int max_radius, int gx, int gy,
                           int& minx, int& miny, int& maxx, int& maxy) {
    minx = std::min(gx, std::max(0, (int)((px - (float)max_radius) / (float)BX)));
    miny = std::min(gy, std::max(0, (int)((py - (float)max_radius) / (float)BY)));
    maxx = std::min(gx, std::max(0, (int)((((px + (float)max_radius) + (float)BX) - 1.0f) / (float)BX)));
    maxy = std::min(gy, std::max(0, (int)((((py + (float)max_radius) + (float)BY) - 1.0f) / (float)BY)));
}

// auxiliary.h:58-77
static inline v3 xform4x3(v3 p, const float* m, int ct = 0) {
    return {dot3c(ct, m[0], p.x, m[4], p.y, m[8], p.z) + m[12],
            dot3c(ct, m[1], p.x, m[5], p.y, m[9], p.z) + m[13],
            dot3c(ct, m[2], p.x, m[6], p.y, m[10], p.z) + m[14]};
}
struct v4 { float x, y, z, w; };
static inline v4 xform4x4(v3 p, const float* m, int ct = 0) {
    return {dot3c(ct, m[0], p.x, m[4], p.y, m[8], p.z) + m[12],
            dot3c(ct, m[1], p.x, m[5], p.y, m[9], p.z) + m[13],
            dot3c(ct, m[2], p.x, m[6], p.y, m[10], p.z) + m[14],
            dot3c(ct, m[3], p.x, m[7], p.y, m[11], p.z) + m[15]};
}
// auxiliary.h:89-97
static inline v3 xformVecT(v3 p, const float* m) {
    return {m[0] * p.x + m[1] * p.y + m[2] * p.z,
            m[4] * p.x + m[5] * p.y + m[6] * p.z,
            m[8] * p.x + m[9] * p.y + m[10] * p.z};
}
// auxiliary.h:107-117
static inline v3 dnormvdv(v3 v, v3 dv) {
    float sum2 = v.x * v.x + v.y * v.y + v.z * v.z;
    float invsum32 = 1.0f / std::sqrt(sum2 * sum2 * sum2);
    v3 r;
    r.x = ((+sum2 - v.x * v.x) * dv.x - v.y * v.x * dv.y - v.z * v.x * dv.z) * invsum32;
    r.y = (-v.x * v.y * dv.x + (sum2 - v.y * v.y) * dv.y - v.z * v.y * dv.z) * invsum32;
    r.z = (-v.x * v.z * dv.x - v.y * v.z * dv.y + (sum2 - v.z * v.z) * dv.z) * invsum32;
    return r;
}

}  // namespace

extern "C" {

// Host-side copy of the raster settings (reference GaussianRasterizationSettings,
// DGR/diff_gaussian_rasterization/__init__.py:168-180).
struct OracleSettings {
    int P, D, M, W, H;
    float tanfovx, tanfovy, scale_modifier;
    int prefiltered;
    float view[16], proj[16], campos[3], bg[3];
};

struct OracleInputs {
    const float* means3D;        // [P,3]
    const float* shs;            // [P,M,3] or NULL
    const float* colors_precomp; // [P,3] or NULL
    const float* segments;       // [P,2] or NULL (treated as zeros)
    const float* opacities;      // [P]
    const float* scales;         // [P,3] or NULL
    const float* rotations;      // [P,4] or NULL
    const float* cov3D_precomp;  // [P,6] or NULL
};

}  // extern "C"

namespace {

// Geometry/Binning/Image state of the reference (rasterizer_impl.h:29-65).
struct State {
    OracleSettings s;
    int gx = 0, gy = 0;
    std::vector<float> depths, means2D, cov3D, conic_opacity, rgb;  // [P], [P,2], [P,6], [P,4], [P,3]
    std::vector<uint8_t> clamped;                                    // [P,3]
    std::vector<int> radii;
    std::vector<uint32_t> tiles_touched, point_offsets;
    int num_rendered = 0;
    std::vector<uint64_t> keys;       // sorted keys [I]
    std::vector<uint32_t> point_list; // sorted gaussian ids [I]
    std::vector<uint32_t> ranges;     // [T,2]
    std::vector<uint32_t> n_contrib;  // [H*W]
    // per pixel: FNV-1a hash of the blend's decision sequence (forward.cu:343-361) -- the list
    // positions that blend and the one that terminates; equal hashes = identical decisions
    std::vector<uint64_t> dhash;      // [H*W]
    std::vector<float> alpha;         // out_alpha copy [H*W]
    std::vector<float> segments;      // [P,2] (zeros if absent)
    std::vector<float> gabs;          // [P,12] sum of |per-pixel gradient terms| (after backward)
};

// forward.cu:20-71
static v3 colorFromSH(int idx, int deg, int max_coeffs, const float* means, v3 campos,
                      const float* shs, uint8_t* clamped) {
    v3 pos = {means[3 * idx], means[3 * idx + 1], means[3 * idx + 2]};
    v3 dir = pos - campos;
    dir = dir / std::sqrt(dot(dir, dir));
    const float* b = shs + (size_t)idx * max_coeffs * 3;
    auto sh = [&](int i) { return v3{b[3 * i], b[3 * i + 1], b[3 * i + 2]}; };
    v3 result = SH_C0 * sh(0);
    if (deg > 0) {
        float x = dir.x, y = dir.y, z = dir.z;
        result = result - SH_C1 * y * sh(1) + SH_C1 * z * sh(2) - SH_C1 * x * sh(3);
        if (deg > 1) {
            float xx = x * x, yy = y * y, zz = z * z;
            float xy = x * y, yz = y * z, xz = x * z;
            result = result + SH_C2[0] * xy * sh(4) + SH_C2[1] * yz * sh(5) +
                     SH_C2[2] * (2.0f * zz - xx - yy) * sh(6) + SH_C2[3] * xz * sh(7) +
                     SH_C2[4] * (xx - yy) * sh(8);
            if (deg > 2) {
                result = result + SH_C3[0] * y * (3.0f * xx - yy) * sh(9) +
                         SH_C3[1] * xy * z * sh(10) + SH_C3[2] * y * (4.0f * zz - xx - yy) * sh(11) +
                         SH_C3[3] * z * (2.0f * zz - 3.0f * xx - 3.0f * yy) * sh(12) +
                         SH_C3[4] * x * (4.0f * zz - xx - yy) * sh(13) +
                         SH_C3[5] * z * (xx - yy) * sh(14) + SH_C3[6] * x * (xx - 3.0f * yy) * sh(15);
            }
        }
    }
    result = result + v3{0.5f, 0.5f, 0.5f};
    clamped[3 * idx + 0] = result.x < 0;
    clamped[3 * idx + 1] = result.y < 0;
    clamped[3 * idx + 2] = result.z < 0;
    return {std::max(result.x, 0.0f), std::max(result.y, 0.0f), std::max(result.z, 0.0f)};
}

// forward.cu:74-113
static void cov2D(v3 mean, float fx, float fy, float tanx, float tany, const float* c3,
                  const float* view, float out[3], int ct = 0) {
    v3 t = xform4x3(mean, view, ct);
    const float limx = 1.3f * tanx, limy = 1.3f * tany;
    const float txtz = t.x / t.z, tytz = t.y / t.z;
    t.x = std::min(limx, std::max(-limx, txtz)) * t.z;
    t.y = std::min(limy, std::max(-limy, tytz)) * t.z;
    m3 J = mk(fx / t.z, 0.0f, -(fx * t.x) / (t.z * t.z), 0.0f, fy / t.z, -(fy * t.y) / (t.z * t.z), 0, 0, 0);
    m3 W = mk(view[0], view[4], view[8], view[1], view[5], view[9], view[2], view[6], view[10]);
    m3 T = mul(W, J, ct);
    m3 Vrk = mk(c3[0], c3[1], c3[2], c3[1], c3[3], c3[4], c3[2], c3[4], c3[5]);
    m3 cov = mul(mul(tr(T), tr(Vrk), ct), T, ct);
    cov.m[0][0] += 0.3f;
    cov.m[1][1] += 0.3f;
    out[0] = cov.m[0][0]; out[1] = cov.m[0][1]; out[2] = cov.m[1][1];
}

// forward.cu:118-152
static void cov3D(v3 scale, float mod, const float* rot, float* out, int ct = 0) {
    m3 S = mk(1, 0, 0, 0, 1, 0, 0, 0, 1);
    S.m[0][0] = mod * scale.x; S.m[1][1] = mod * scale.y; S.m[2][2] = mod * scale.z;
    float r = rot[0], x = rot[1], y = rot[2], z = rot[3];
    m3 R;
    if (!ct) {
        R = mk(1.f - 2.f * (y * y + z * z), 2.f * (x * y - r * z), 2.f * (x * z + r * y),
               2.f * (x * y + r * z), 1.f - 2.f * (x * x + z * z), 2.f * (y * z - r * x),
               2.f * (x * z - r * y), 2.f * (y * z + r * x), 1.f - 2.f * (x * x + y * y));
    } else {  // 1 - 2*s: fsub(1, fmul(2, s)) -> fma(-2, s, 1)
        auto one_m2 = [&](float a, float b) { return std::fma(-2.f, pp_add(ct, a, a, b, b), 1.f); };
        R = mk(one_m2(y, z), 2.f * pp_sub(ct, x, y, r, z), 2.f * pp_add(ct, x, z, r, y),
               2.f * pp_add(ct, x, y, r, z), one_m2(x, z), 2.f * pp_sub(ct, y, z, r, x),
               2.f * pp_sub(ct, x, z, r, y), 2.f * pp_add(ct, y, z, r, x), one_m2(x, y));
    }
    m3 M = mul(S, R, ct);
    m3 Sig = mul(tr(M), M, ct);
    out[0] = Sig.m[0][0]; out[1] = Sig.m[0][1]; out[2] = Sig.m[0][2];
    out[3] = Sig.m[1][1]; out[4] = Sig.m[1][2]; out[5] = Sig.m[2][2];
}

// rasterizer_impl.cu:35-50
static uint32_t getHigherMsb(uint32_t n) {
    uint32_t msb = sizeof(n) * 4, step = msb;
    while (step > 1) {
        step /= 2;
        if (n >> msb) msb += step; else msb -= step;
    }
    if (n >> msb) msb++;
    return msb;
}

static std::string g_err;

// exp() of the blend (forward.cu:351, backward.cu:547).  The reference calls CUDA's
// expf (2 ulp); gsr's kernels and this oracle share gsr_expf: IEEE operations only
// (fma, add, mul, integer shift), max 0.887 ulp on the blend's range [-5.6, 0], so both compute
// identical bits and the knife-edge blend decisions (alpha >= 1/255, T(1-alpha) >= 1e-4) agree
// exactly.
// g_exp_libm = 1 switches to the C library's expf (noise-floor studies).
static int g_exp_libm = 0;
static inline float gsr_expf(float x) {
    // exp(clamp(x, -87, 88)): k = round(x log2 e) by the 1.5*2^23 shifter, r = x - k ln2 with
    // ln 2 rounded to fp32 (one FMA; error |k| * 1.9e-9), degree-6 minimax polynomial (Horner,
    // FMA), times 2^k built from the shifter's low bits.  Must stay bit-identical to
    // render.hip: gsr_expf.
    const float xc = std::fmin(std::fmax(x, -87.0f), 88.0f);
    const float kf = std::fma(xc, 1.44269502f, 12582912.0f);
    const float k = kf - 12582912.0f;
    const float r = std::fma(-k, 0.693147182464599609375f, xc);
    float p = 0.001381461275741458f;  // degree-6 minimax (1 + r + c2 r^2 + ... + c6 r^6)
    p = std::fma(p, r, 0.008368710055947304f);
    p = std::fma(p, r, 0.04166838899254799f);
    p = std::fma(p, r, 0.1666652113199234f);
    p = std::fma(p, r, 0.4999999403953552f);
    p = std::fma(p, r, 1.0f);
    p = std::fma(p, r, 1.0f);
    uint32_t kb;
    std::memcpy(&kb, &kf, 4);
    const uint32_t sb = (kb << 23) + 0x3f800000u;  // 2^k, k in [-126, 127]
    float scale;
    std::memcpy(&scale, &sb, 4);
    return p * scale;
}
static inline float oracle_exp(float x) { return g_exp_libm ? std::exp(x) : gsr_expf(x); }
// forward.cu:346 / backward.cu:541: -0.5*(cx*dx*dx + cz*dy*dy) - cy*dx*dy; cb != 0: as nvcc
// contracts it (see the contraction model above)
static inline float blend_power(int cb, const float* co, float dx, float dy) {
    if (!cb) return -0.5f * (co[0] * dx * dx + co[2] * dy * dy) - co[1] * dx * dy;
    const float q = pp_add(cb, co[0] * dx, dx, co[2] * dy, dy);
    return (cb & CT_RIGHT) ? std::fma(-(co[1] * dx), dy, -0.5f * q) : std::fma(-0.5f, q, -((co[1] * dx) * dy));
}
// g_exp_jitter != 0: every blend exp (forward and backward alike) moves by -n .. +n ulp
// (n = g_exp_jitter_ulps, default 1), chosen by a hash of (seed, Gaussian, pixel) -- the
// reference algorithm run with another exp of n-ulp accuracy around gsr_expf (CUDA's expf is
// specified at 2 ulp), to measure each output element's own sensitivity to last-bit alpha
// differences (tests/test_gpu_exp_budget.py).
static uint32_t g_exp_jitter = 0;
static int g_exp_jitter_ulps = 1;
static inline float jitter_exp(float G, uint32_t g, uint32_t pix) {
    if (!g_exp_jitter || !(G > 0.f)) return G;
    uint64_t h = ((uint64_t)g_exp_jitter << 40) ^ ((uint64_t)g << 20) ^ (uint64_t)pix;
    h ^= h >> 33;
    h *= 0xff51afd7ed558ccdull;
    h ^= h >> 33;
    h *= 0xc4ceb9fe1a85ec53ull;
    h ^= h >> 33;
    // -n .. +n ulp
    int r = (int)(h % (uint64_t)(2 * g_exp_jitter_ulps + 1)) - g_exp_jitter_ulps;
    for (; r < 0; ++r) G = std::nextafter(G, 0.0f);
    for (; r > 0; --r) G = std::nextafter(G, 2.0f * G);
    return G;
}
// 1: emulate the reference's fp32 accumulation (one fixed order of its atomics)
static int g_acc32 = 0;

}  // namespace

extern "C" {

const char* oracle_last_error(void) { return g_err.c_str(); }

void oracle_set_acc32(int on) { g_acc32 = on; }
void oracle_set_exp_libm(int on) { g_exp_libm = on; }
void oracle_set_exp_jitter(unsigned seed) { g_exp_jitter = seed; }
void oracle_set_exp_jitter_ulps(int n) { g_exp_jitter_ulps = n < 1 ? 1 : n; }
void oracle_set_contract(int mode) { g_contract = mode; }
int oracle_get_contract(void) { return g_contract; }
float oracle_expf(float x) { return gsr_expf(x); }

int oracle_num_threads(void) {
#ifdef _OPENMP
    return omp_get_max_threads();
#else
    return 1;
#endif
}
void oracle_set_num_threads(int n) {
#ifdef _OPENMP
    if (n > 0) omp_set_num_threads(n);
#else
    (void)n;
#endif
}

// Reference: CudaRasterizer::Rasterizer::forward (rasterizer_impl.cu:198-344).
// Outputs are planar CHW like the reference (forward.cu:383-391).
void* oracle_forward(const OracleSettings* sp, const OracleInputs* in, float* out_color,
                     float* out_depth, float* out_alpha, float* out_segment, int* radii_out) {
    State* st = new State();
    st->s = *sp;
    const OracleSettings& s = st->s;
    const int P = s.P, W = s.W, H = s.H;
    const float focal_y = H / (2.0f * s.tanfovy);
    const float focal_x = W / (2.0f * s.tanfovx);
    st->gx = (W + BX - 1) / BX;
    st->gy = (H + BY - 1) / BY;
    const int gx = st->gx, gy = st->gy;
    st->depths.assign(P, 0.f);
    st->means2D.assign(2 * (size_t)P, 0.f);
    st->cov3D.assign(6 * (size_t)P, 0.f);
    st->conic_opacity.assign(4 * (size_t)P, 0.f);
    st->rgb.assign(3 * (size_t)P, 0.f);
    st->clamped.assign(3 * (size_t)P, 0);
    st->radii.assign(P, 0);
    st->tiles_touched.assign(P, 0);
    st->segments.assign(2 * (size_t)P, 0.f);
    if (in->segments) std::memcpy(st->segments.data(), in->segments, sizeof(float) * 2 * (size_t)P);
    const v3 campos = {s.campos[0], s.campos[1], s.campos[2]};

    // preprocessCUDA (forward.cu:154-256)
    const int ct = ct_pre();
#pragma omp parallel for schedule(static)
    for (int idx = 0; idx < P; ++idx) {
        v3 p_orig = {in->means3D[3 * idx], in->means3D[3 * idx + 1], in->means3D[3 * idx + 2]};
        // in_frustum (auxiliary.h:139-164)
        v3 p_view = xform4x3(p_orig, s.view, ct);
        if (p_view.z <= 0.2f) continue;  // prefiltered trap is a device abort; not modelled
        v4 p_hom = xform4x4(p_orig, s.proj, ct);
        float p_w = 1.0f / (p_hom.w + 0.0000001f);
        v3 p_proj = {p_hom.x * p_w, p_hom.y * p_w, p_hom.z * p_w};
        const float* c3;
        if (in->cov3D_precomp) {
            c3 = in->cov3D_precomp + 6 * (size_t)idx;
        } else {
            v3 sc = {in->scales[3 * idx], in->scales[3 * idx + 1], in->scales[3 * idx + 2]};
            cov3D(sc, s.scale_modifier, in->rotations + 4 * (size_t)idx, &st->cov3D[6 * (size_t)idx], ct);
            c3 = &st->cov3D[6 * (size_t)idx];
        }
        float cov[3];
        cov2D(p_orig, focal_x, focal_y, s.tanfovx, s.tanfovy, c3, s.view, cov, ct);
        float det = pp_sub(ct, cov[0], cov[2], cov[1], cov[1]);
        if (det == 0.0f) continue;
        float det_inv = 1.f / det;
        float conic[3] = {cov[2] * det_inv, -cov[1] * det_inv, cov[0] * det_inv};
        float mid = 0.5f * (cov[0] + cov[2]);
        const float disc = ct ? std::fma(mid, mid, -det) : mid * mid - det;
        float lambda1 = mid + std::sqrt(std::max(0.1f, disc));
        float lambda2 = mid - std::sqrt(std::max(0.1f, disc));
        float my_radius = std::ceil(3.f * std::sqrt(std::max(lambda1, lambda2)));
        float pix_x = ndc2Pix(p_proj.x, W, ct), pix_y = ndc2Pix(p_proj.y, H, ct);
        int minx, miny, maxx, maxy;
        getRect(pix_x, pix_y, (int)my_radius, gx, gy, minx, miny, maxx, maxy);
        if ((uint32_t)((maxx - minx) * (maxy - miny)) == 0) continue;
        if (in->colors_precomp == nullptr) {
            v3 c = colorFromSH(idx, s.D, s.M, in->means3D, campos, in->shs, st->clamped.data());
            st->rgb[3 * idx + 0] = c.x; st->rgb[3 * idx + 1] = c.y; st->rgb[3 * idx + 2] = c.z;
        }
        st->depths[idx] = p_view.z;
        st->radii[idx] = (int)my_radius;
        st->means2D[2 * idx] = pix_x; st->means2D[2 * idx + 1] = pix_y;
        st->conic_opacity[4 * idx + 0] = conic[0];
        st->conic_opacity[4 * idx + 1] = conic[1];
        st->conic_opacity[4 * idx + 2] = conic[2];
        st->conic_opacity[4 * idx + 3] = in->opacities[idx];
        st->tiles_touched[idx] = (uint32_t)((maxy - miny) * (maxx - minx));
    }
    // InclusiveSum (rasterizer_impl.cu:281)
    st->point_offsets.resize(P);
    uint64_t acc = 0;
    for (int i = 0; i < P; ++i) { acc += st->tiles_touched[i]; st->point_offsets[i] = (uint32_t)acc; }
    const int I = P ? (int)st->point_offsets[P - 1] : 0;
    st->num_rendered = I;

    // duplicateWithKeys (rasterizer_impl.cu:68-111), then the stable sort on
    // bits [0, 32+bit) (:304-312).  The composite (key, unsorted position) is
    // unique, so an unstable sort of it equals CUB's stable pair sort.
    std::vector<std::pair<uint64_t, uint32_t>> kv((size_t)I);
#pragma omp parallel for schedule(dynamic, 1024)
    for (int idx = 0; idx < P; ++idx) {
        if (st->radii[idx] <= 0) continue;
        uint32_t off = idx == 0 ? 0 : st->point_offsets[idx - 1];
        int minx, miny, maxx, maxy;
        getRect(st->means2D[2 * idx], st->means2D[2 * idx + 1], st->radii[idx], gx, gy, minx, miny, maxx, maxy);
        uint32_t dbits;
        std::memcpy(&dbits, &st->depths[idx], 4);
        for (int y = miny; y < maxy; ++y)
            for (int x = minx; x < maxx; ++x) {
                uint64_t key = (uint64_t)(uint32_t)(y * gx + x);
                key <<= 32;
                key |= dbits;
                kv[off] = {key, (uint32_t)off};
                off++;
            }
    }
    std::vector<uint32_t> unsorted_val((size_t)I);
    for (int idx = 0; idx < P; ++idx) {
        if (st->radii[idx] <= 0) continue;
        uint32_t off = idx == 0 ? 0 : st->point_offsets[idx - 1];
        for (uint32_t k = 0; k < st->tiles_touched[idx]; ++k) unsorted_val[off + k] = (uint32_t)idx;
    }
    const int bit = (int)getHigherMsb((uint32_t)(gx * gy));
    const uint64_t mask = (32 + bit) >= 64 ? ~0ull : ((1ull << (32 + bit)) - 1);
    for (auto& e : kv) e.first &= mask;
#ifdef _OPENMP
    __gnu_parallel::sort(kv.begin(), kv.end());
#else
    std::sort(kv.begin(), kv.end());
#endif
    st->keys.resize(I);
    st->point_list.resize(I);
    for (int k = 0; k < I; ++k) {
        st->keys[k] = kv[k].first;
        st->point_list[k] = unsorted_val[kv[k].second];
    }
    // identifyTileRanges (rasterizer_impl.cu:113-138, memset :314)
    const int T = gx * gy;
    st->ranges.assign(2 * (size_t)T, 0);
    for (int k = 0; k < I; ++k) {
        uint32_t cur = (uint32_t)(st->keys[k] >> 32);
        if (k == 0) st->ranges[2 * cur] = 0;
        else {
            uint32_t prev = (uint32_t)(st->keys[k - 1] >> 32);
            if (cur != prev) { st->ranges[2 * prev + 1] = k; st->ranges[2 * cur] = k; }
        }
        if (k == I - 1) st->ranges[2 * cur + 1] = I;
    }

    // renderCUDA forward (forward.cu:258-392)
    st->n_contrib.assign((size_t)W * H, 0);
    st->dhash.assign((size_t)W * H, 0);
    st->alpha.assign((size_t)W * H, 0.f);
    const float* feat = in->colors_precomp ? in->colors_precomp : st->rgb.data();
    const float* segs = st->segments.data();
    const int cb = ct_blend();
#pragma omp parallel for schedule(dynamic, 1)
    for (int t = 0; t < T; ++t) {
        const int tx = t % gx, ty = t / gx;
        const uint32_t r0 = st->ranges[2 * t], r1 = st->ranges[2 * t + 1];
        for (int ly = 0; ly < BY; ++ly)
            for (int lx = 0; lx < BX; ++lx) {
                const int px = tx * BX + lx, py = ty * BY + ly;
                if (px >= W || py >= H) continue;
                const uint32_t pix_id = (uint32_t)W * py + px;
                const float pfx = (float)px, pfy = (float)py;
                float Tr = 1.0f, C[NCH] = {0, 0, 0}, S[NCLS] = {0, 0}, weight = 0, D = 0;
                uint32_t contributor = 0, last_contributor = 0;
                uint64_t dh = 1469598103934665603ull;  // FNV-1a over the decisions
                auto mix = [&](uint32_t v) {
                    for (int b = 0; b < 4; ++b) dh = (dh ^ ((v >> (8 * b)) & 0xffu)) * 1099511628211ull;
                };
                for (uint32_t k = r0; k < r1; ++k) {
                    contributor++;
                    const uint32_t g = st->point_list[k];
                    const float* co = &st->conic_opacity[4 * (size_t)g];
                    const float dx = st->means2D[2 * g] - pfx, dy = st->means2D[2 * g + 1] - pfy;
                    const float power = blend_power(cb, co, dx, dy);
                    if (power > 0.0f) continue;
                    const float alpha = std::min(0.99f, co[3] * jitter_exp(oracle_exp(power), g, pix_id));
                    if (alpha < 1.0f / 255.0f) continue;
                    const float test_T = Tr * (1 - alpha);
                    if (test_T < 0.0001f) {  // done = true
                        mix(contributor | 0x80000000u);
                        break;
                    }
                    mix(contributor);
                    if (!cb) {
                        for (int ch = 0; ch < NCH; ++ch) C[ch] += feat[g * NCH + ch] * alpha * Tr;
                        weight += alpha * Tr;
                        D += st->depths[g] * alpha * Tr;
                        for (int c = 0; c < NCLS; ++c) S[c] += segs[g * NCLS + c] * alpha * Tr;
                    } else {  // forward.cu:362-366 under contraction: x += (f*alpha)*T -> fma
                        for (int ch = 0; ch < NCH; ++ch) C[ch] = std::fma(feat[g * NCH + ch] * alpha, Tr, C[ch]);
                        weight = std::fma(alpha, Tr, weight);
                        D = std::fma(st->depths[g] * alpha, Tr, D);
                        for (int c = 0; c < NCLS; ++c) S[c] = std::fma(segs[g * NCLS + c] * alpha, Tr, S[c]);
                    }
                    Tr = test_T;
                    last_contributor = contributor;
                }
                st->n_contrib[pix_id] = last_contributor;
                st->dhash[pix_id] = dh;
                for (int ch = 0; ch < NCH; ++ch) out_color[(size_t)ch * H * W + pix_id] = C[ch] + Tr * s.bg[ch];
                out_alpha[pix_id] = weight;
                st->alpha[pix_id] = weight;
                out_depth[pix_id] = D;
                for (int c = 0; c < NCLS; ++c) out_segment[(size_t)c * H * W + pix_id] = S[c];
            }
    }
    if (radii_out) std::memcpy(radii_out, st->radii.data(), sizeof(int) * (size_t)P);
    return st;
}

void oracle_free(void* h) { delete (State*)h; }

int oracle_num_rendered(void* h) { return ((State*)h)->num_rendered; }

// Replace the forward's weight sums (out_alpha, [H*W]) that the backward recovers T_final from
// (backward.cu:468): lets a study run one backward from another forward's T_final.
int oracle_set_weight_sums(void* h, const float* alpha) {
    State* st = (State*)h;
    if (!alpha) return 1;
    std::memcpy(st->alpha.data(), alpha, st->alpha.size() * sizeof(float));
    return 0;
}

// Copies one named intermediate into dst; returns element count (or -1).
long oracle_get(void* h, const char* name, void* dst) {
    State* st = (State*)h;
    auto cp = [&](const void* src, size_t bytes, long n) {
        if (dst && bytes) std::memcpy(dst, src, bytes);
        return n;
    };
    std::string n(name);
    if (n == "depths") return cp(st->depths.data(), st->depths.size() * 4, st->depths.size());
    if (n == "means2D") return cp(st->means2D.data(), st->means2D.size() * 4, st->means2D.size());
    if (n == "cov3D") return cp(st->cov3D.data(), st->cov3D.size() * 4, st->cov3D.size());
    if (n == "conic_opacity") return cp(st->conic_opacity.data(), st->conic_opacity.size() * 4, st->conic_opacity.size());
    if (n == "rgb") return cp(st->rgb.data(), st->rgb.size() * 4, st->rgb.size());
    if (n == "clamped") return cp(st->clamped.data(), st->clamped.size(), st->clamped.size());
    if (n == "tiles_touched") return cp(st->tiles_touched.data(), st->tiles_touched.size() * 4, st->tiles_touched.size());
    if (n == "point_offsets") return cp(st->point_offsets.data(), st->point_offsets.size() * 4, st->point_offsets.size());
    if (n == "keys") return cp(st->keys.data(), st->keys.size() * 8, st->keys.size());
    if (n == "point_list") return cp(st->point_list.data(), st->point_list.size() * 4, st->point_list.size());
    if (n == "ranges") return cp(st->ranges.data(), st->ranges.size() * 4, st->ranges.size());
    if (n == "n_contrib") return cp(st->n_contrib.data(), st->n_contrib.size() * 4, st->n_contrib.size());
    if (n == "dhash") return cp(st->dhash.data(), st->dhash.size() * 8, st->dhash.size());
    if (n == "gabs") return cp(st->gabs.data(), st->gabs.size() * 4, st->gabs.size());
    g_err = "unknown field " + n;
    return -1;
}

// Reference: CudaRasterizer::Rasterizer::backward (rasterizer_impl.cu:348-458).
// grads: dmeans2D[P,3] dcolors[P,3] dopacity[P] dmeans3D[P,3] dcov3D[P,6]
//        dsh[P,M,3] dscales[P,3] drot[P,4] dsegments[P,2]  (all zero-filled by caller)
// Per-pixel contributions are summed per (tile, gaussian) instance in pixel
// row-major order, then per gaussian in sorted-instance order, so the oracle is
// bitwise reproducible for any thread count (the reference's atomicAdd order
// is arbitrary: backward.cu:575-636).
int oracle_backward(void* h, const OracleInputs* in, const float* dL_dpix, const float* dL_dpix_seg,
                    const float* dL_dpix_depth, const float* dL_dalphas, float* dmeans2D,
                    float* dcolors, float* dopacity, float* dmeans3D, float* dcov3D, float* dsh,
                    float* dscales, float* drot, float* dsegments) {
    State* st = (State*)h;
    const OracleSettings& s = st->s;
    const int P = s.P, W = s.W, H = s.H, gx = st->gx, gy = st->gy, T = gx * gy;
    const int I = st->num_rendered;
    const float focal_y = H / (2.0f * s.tanfovy);
    const float focal_x = W / (2.0f * s.tanfovx);
    const float* colors = in->colors_precomp ? in->colors_precomp : st->rgb.data();
    const float* segs = st->segments.data();
    // fp64 accumulation: the reference sums with atomicAdd in arbitrary order, so
    // the exact sum of the fp32 per-pixel terms is the centre of its outputs.
    std::vector<double> contrib((size_t)I * 12, 0.0), cabs((size_t)I * 12, 0.0);
    const float ddelx_dx = 0.5 * W, ddely_dy = 0.5 * H;
    const int cb = ct_blend();

    // renderCUDA backward (backward.cu:414-639)
#pragma omp parallel for schedule(dynamic, 1)
    for (int t = 0; t < T; ++t) {
        const int tx = t % gx, ty = t / gx;
        const uint32_t r0 = st->ranges[2 * t], r1 = st->ranges[2 * t + 1];
        for (int ly = 0; ly < BY; ++ly)
            for (int lx = 0; lx < BX; ++lx) {
                const int px = tx * BX + lx, py = ty * BY + ly;
                if (px >= W || py >= H) continue;
                const uint32_t pix_id = (uint32_t)W * py + px;
                const float pfx = (float)px, pfy = (float)py;
                const float T_final = 1 - st->alpha[pix_id];
                float Tr = T_final;
                uint32_t contributor = r1 - r0;
                const uint32_t last_contributor = st->n_contrib[pix_id];
                float accum_rec[NCH] = {0, 0, 0}, dL_dpixel[NCH];
                float accum_seg[NCLS] = {0, 0}, dL_dseg[NCLS];
                float accum_depth = 0, accum_alpha = 0;
                for (int i = 0; i < NCH; ++i) dL_dpixel[i] = dL_dpix[(size_t)i * H * W + pix_id];
                const float dL_dd = dL_dpix_depth[pix_id];
                const float dL_da = dL_dalphas[pix_id];
                for (int i = 0; i < NCLS; ++i) dL_dseg[i] = dL_dpix_seg[(size_t)i * H * W + pix_id];
                float last_alpha = 0, last_color[NCH] = {0, 0, 0}, last_seg[NCLS] = {0, 0}, last_depth = 0;
                for (uint32_t kk = r1; kk > r0; --kk) {
                    const uint32_t k = kk - 1;
                    contributor--;
                    if (contributor >= last_contributor) continue;
                    const uint32_t g = st->point_list[k];
                    const float* co = &st->conic_opacity[4 * (size_t)g];
                    const float dx = st->means2D[2 * g] - pfx, dy = st->means2D[2 * g + 1] - pfy;
                    const float power = blend_power(cb, co, dx, dy);
                    if (power > 0.0f) continue;
                    const float G = jitter_exp(oracle_exp(power), g, pix_id);
                    const float alpha = std::min(0.99f, co[3] * G);
                    if (alpha < 1.0f / 255.0f) continue;
                    Tr = Tr / (1.f - alpha);
                    const float dchannel_dcolor = alpha * Tr;
                    double* cb = &contrib[(size_t)k * 12];
                    double* ab = &cabs[(size_t)k * 12];
                    auto ADD = [&](int i, float t) {
                        if (g_acc32) cb[i] = (double)((float)cb[i] + t);
                        else cb[i] += t;
                        ab[i] += std::fabs((double)t);
                    };
                    float dL_dopa = 0.0f;
                    for (int ch = 0; ch < NCH; ++ch) {
                        const float c = colors[g * NCH + ch];
                        accum_rec[ch] = last_alpha * last_color[ch] + (1.f - last_alpha) * accum_rec[ch];
                        last_color[ch] = c;
                        dL_dopa += (c - accum_rec[ch]) * dL_dpixel[ch];
                        ADD(0 + ch, dchannel_dcolor * dL_dpixel[ch]);
                    }
                    for (int ch = 0; ch < NCLS; ++ch) {
                        const float c_s = segs[g * NCLS + ch];
                        accum_seg[ch] = last_alpha * last_seg[ch] + (1.f - last_alpha) * accum_seg[ch];
                        last_seg[ch] = c_s;
                        dL_dopa += (c_s - accum_seg[ch]) * dL_dseg[ch];
                        ADD(3 + ch, dchannel_dcolor * dL_dseg[ch]);
                    }
                    const float c_d = st->depths[g];
                    accum_depth = last_alpha * last_depth + (1.f - last_alpha) * accum_depth;
                    last_depth = c_d;
                    dL_dopa += (c_d - accum_depth) * dL_dd;
                    ADD(5, dchannel_dcolor * dL_dd);
                    accum_alpha = last_alpha + (1.f - last_alpha) * accum_alpha;
                    dL_dopa += (1 - accum_alpha) * dL_da;
                    dL_dopa *= Tr;
                    last_alpha = alpha;
                    float bg_dot = 0;
                    for (int i = 0; i < NCH; ++i) bg_dot += s.bg[i] * dL_dpixel[i];
                    dL_dopa += (-T_final / (1.f - alpha)) * bg_dot;
                    const float dL_dG = co[3] * dL_dopa;
                    const float gdx = G * dx, gdy = G * dy;
                    const float dG_ddelx = -gdx * co[0] - gdy * co[1];
                    const float dG_ddely = -gdy * co[2] - gdx * co[1];
                    ADD(6, dL_dG * dG_ddelx * ddelx_dx);
                    ADD(7, dL_dG * dG_ddely * ddely_dy);
                    ADD(8, -0.5f * gdx * dx * dL_dG);
                    ADD(9, -0.5f * gdx * dy * dL_dG);
                    ADD(10, -0.5f * gdy * dy * dL_dG);
                    ADD(11, G * dL_dopa);
                }
            }
    }
    // Gather per-gaussian sums: [dcolor3 dseg2 ddepth dmean2D.xy dconic.xyw dopacity]
    std::vector<double> gsum_d((size_t)P * 12, 0.0);
    st->gabs.assign((size_t)P * 12, 0.f);
    for (int k = 0; k < I; ++k) {
        const uint32_t g = st->point_list[k];
        for (int j = 0; j < 12; ++j) {
            double& d = gsum_d[(size_t)g * 12 + j];
            d = g_acc32 ? (double)((float)d + (float)contrib[(size_t)k * 12 + j]) : d + contrib[(size_t)k * 12 + j];
            st->gabs[(size_t)g * 12 + j] += (float)cabs[(size_t)k * 12 + j];
        }
    }
    std::vector<float> gsum(gsum_d.begin(), gsum_d.end());
    std::vector<float> ddepth(P);
    for (int g = 0; g < P; ++g) {
        const float* q = &gsum[(size_t)g * 12];
        for (int ch = 0; ch < 3; ++ch) dcolors[3 * g + ch] = q[ch];
        for (int c = 0; c < 2; ++c) dsegments[2 * g + c] = q[3 + c];
        ddepth[g] = q[5];
        dmeans2D[3 * g + 0] = q[6];
        dmeans2D[3 * g + 1] = q[7];
        dmeans2D[3 * g + 2] = 0.f;
        dopacity[g] = q[11];
    }
    const int* radii = st->radii.data();
    const v3 campos = {s.campos[0], s.campos[1], s.campos[2]};

#pragma omp parallel for schedule(static)
    for (int idx = 0; idx < P; ++idx) {
        if (!(radii[idx] > 0)) continue;
        const float* q = &gsum[(size_t)idx * 12];
        // computeCov2DCUDA (backward.cu:141-274)
        const float* c3 = in->cov3D_precomp ? in->cov3D_precomp + 6 * (size_t)idx : &st->cov3D[6 * (size_t)idx];
        const v3 mean = {in->means3D[3 * idx], in->means3D[3 * idx + 1], in->means3D[3 * idx + 2]};
        const float dconic[3] = {q[8], q[9], q[10]};
        v3 t = xform4x3(mean, s.view);
        const float limx = 1.3f * s.tanfovx, limy = 1.3f * s.tanfovy;
        const float txtz = t.x / t.z, tytz = t.y / t.z;
        t.x = std::min(limx, std::max(-limx, txtz)) * t.z;
        t.y = std::min(limy, std::max(-limy, tytz)) * t.z;
        const float x_grad_mul = txtz < -limx || txtz > limx ? 0 : 1;
        const float y_grad_mul = tytz < -limy || tytz > limy ? 0 : 1;
        const float hx = focal_x, hy = focal_y;
        m3 J = mk(hx / t.z, 0.0f, -(hx * t.x) / (t.z * t.z), 0.0f, hy / t.z, -(hy * t.y) / (t.z * t.z), 0, 0, 0);
        m3 Wm = mk(s.view[0], s.view[4], s.view[8], s.view[1], s.view[5], s.view[9], s.view[2], s.view[6], s.view[10]);
        m3 Vrk = mk(c3[0], c3[1], c3[2], c3[1], c3[3], c3[4], c3[2], c3[4], c3[5]);
        m3 Tm = mul(Wm, J);
        m3 c2 = mul(mul(tr(Tm), tr(Vrk)), Tm);
        const float a = c2.m[0][0] += 0.3f;
        const float b = c2.m[0][1];
        const float c = c2.m[1][1] += 0.3f;
        const float denom = a * c - b * b;
        float dL_da = 0, dL_db = 0, dL_dc = 0;
        const float denom2inv = 1.0f / ((denom * denom) + 0.0000001f);
        float dcv[6] = {0, 0, 0, 0, 0, 0};
        const auto& Tt = Tm.m;
        if (denom2inv != 0) {
            dL_da = denom2inv * (-c * c * dconic[0] + 2 * b * c * dconic[1] + (denom - a * c) * dconic[2]);
            dL_dc = denom2inv * (-a * a * dconic[2] + 2 * a * b * dconic[1] + (denom - a * c) * dconic[0]);
            dL_db = denom2inv * 2 * (b * c * dconic[0] - (denom + 2 * b * b) * dconic[1] + a * b * dconic[2]);
            dcv[0] = (Tt[0][0] * Tt[0][0] * dL_da + Tt[0][0] * Tt[1][0] * dL_db + Tt[1][0] * Tt[1][0] * dL_dc);
            dcv[3] = (Tt[0][1] * Tt[0][1] * dL_da + Tt[0][1] * Tt[1][1] * dL_db + Tt[1][1] * Tt[1][1] * dL_dc);
            dcv[5] = (Tt[0][2] * Tt[0][2] * dL_da + Tt[0][2] * Tt[1][2] * dL_db + Tt[1][2] * Tt[1][2] * dL_dc);
            dcv[1] = 2 * Tt[0][0] * Tt[0][1] * dL_da + (Tt[0][0] * Tt[1][1] + Tt[0][1] * Tt[1][0]) * dL_db + 2 * Tt[1][0] * Tt[1][1] * dL_dc;
            dcv[2] = 2 * Tt[0][0] * Tt[0][2] * dL_da + (Tt[0][0] * Tt[1][2] + Tt[0][2] * Tt[1][0]) * dL_db + 2 * Tt[1][0] * Tt[1][2] * dL_dc;
            dcv[4] = 2 * Tt[0][2] * Tt[0][1] * dL_da + (Tt[0][1] * Tt[1][2] + Tt[0][2] * Tt[1][1]) * dL_db + 2 * Tt[1][1] * Tt[1][2] * dL_dc;
        }
        const auto& V = Vrk.m;
        const float dL_dT00 = 2 * (Tt[0][0] * V[0][0] + Tt[0][1] * V[0][1] + Tt[0][2] * V[0][2]) * dL_da +
                              (Tt[1][0] * V[0][0] + Tt[1][1] * V[0][1] + Tt[1][2] * V[0][2]) * dL_db;
        const float dL_dT01 = 2 * (Tt[0][0] * V[1][0] + Tt[0][1] * V[1][1] + Tt[0][2] * V[1][2]) * dL_da +
                              (Tt[1][0] * V[1][0] + Tt[1][1] * V[1][1] + Tt[1][2] * V[1][2]) * dL_db;
        const float dL_dT02 = 2 * (Tt[0][0] * V[2][0] + Tt[0][1] * V[2][1] + Tt[0][2] * V[2][2]) * dL_da +
                              (Tt[1][0] * V[2][0] + Tt[1][1] * V[2][1] + Tt[1][2] * V[2][2]) * dL_db;
        const float dL_dT10 = 2 * (Tt[1][0] * V[0][0] + Tt[1][1] * V[0][1] + Tt[1][2] * V[0][2]) * dL_dc +
                              (Tt[0][0] * V[0][0] + Tt[0][1] * V[0][1] + Tt[0][2] * V[0][2]) * dL_db;
        const float dL_dT11 = 2 * (Tt[1][0] * V[1][0] + Tt[1][1] * V[1][1] + Tt[1][2] * V[1][2]) * dL_dc +
                              (Tt[0][0] * V[1][0] + Tt[0][1] * V[1][1] + Tt[0][2] * V[1][2]) * dL_db;
        const float dL_dT12 = 2 * (Tt[1][0] * V[2][0] + Tt[1][1] * V[2][1] + Tt[1][2] * V[2][2]) * dL_dc +
                              (Tt[0][0] * V[2][0] + Tt[0][1] * V[2][1] + Tt[0][2] * V[2][2]) * dL_db;
        const auto& Wt = Wm.m;
        const float dL_dJ00 = Wt[0][0] * dL_dT00 + Wt[0][1] * dL_dT01 + Wt[0][2] * dL_dT02;
        const float dL_dJ02 = Wt[2][0] * dL_dT00 + Wt[2][1] * dL_dT01 + Wt[2][2] * dL_dT02;
        const float dL_dJ11 = Wt[1][0] * dL_dT10 + Wt[1][1] * dL_dT11 + Wt[1][2] * dL_dT12;
        const float dL_dJ12 = Wt[2][0] * dL_dT10 + Wt[2][1] * dL_dT11 + Wt[2][2] * dL_dT12;
        const float tz = 1.f / t.z, tz2 = tz * tz, tz3 = tz2 * tz;
        const float dL_dtx = x_grad_mul * -hx * tz2 * dL_dJ02;
        const float dL_dty = y_grad_mul * -hy * tz2 * dL_dJ12;
        const float dL_dtz = -hx * tz2 * dL_dJ00 - hy * tz2 * dL_dJ11 + (2 * hx * t.x) * tz3 * dL_dJ02 + (2 * hy * t.y) * tz3 * dL_dJ12;
        v3 dmean = xformVecT({dL_dtx, dL_dty, dL_dtz}, s.view);
        if (dcov3D) for (int i = 0; i < 6; ++i) dcov3D[6 * idx + i] = dcv[i];

        // preprocessCUDA backward (backward.cu:343-412)
        const float* proj = s.proj;
        const float* view = s.view;
        const v3 m = mean;
        v4 m_hom = xform4x4(m, proj);
        float m_w = 1.0f / (m_hom.w + 0.0000001f);
        const float d2x = q[6], d2y = q[7];
        float mul1 = (proj[0] * m.x + proj[4] * m.y + proj[8] * m.z + proj[12]) * m_w * m_w;
        float mul2 = (proj[1] * m.x + proj[5] * m.y + proj[9] * m.z + proj[13]) * m_w * m_w;
        v3 dm;
        dm.x = (proj[0] * m_w - proj[3] * mul1) * d2x + (proj[1] * m_w - proj[3] * mul2) * d2y;
        dm.y = (proj[4] * m_w - proj[7] * mul1) * d2x + (proj[5] * m_w - proj[7] * mul2) * d2y;
        dm.z = (proj[8] * m_w - proj[11] * mul1) * d2x + (proj[9] * m_w - proj[11] * mul2) * d2y;
        dmean = dmean + dm;
        float mul3 = view[2] * m.x + view[6] * m.y + view[10] * m.z + view[14];
        v3 dm2;
        dm2.x = (view[2] - view[3] * mul3) * ddepth[idx];
        dm2.y = (view[6] - view[7] * mul3) * ddepth[idx];
        dm2.z = (view[10] - view[11] * mul3) * ddepth[idx];
        dmean = dmean + dm2;

        if (in->shs) {
            // computeColorFromSH backward (backward.cu:20-139)
            const int deg = s.D, max_coeffs = s.M;
            v3 dir_orig = m - campos;
            v3 dir = dir_orig / std::sqrt(dot(dir_orig, dir_orig));
            const float* bsh = in->shs + (size_t)idx * max_coeffs * 3;
            auto sh = [&](int i) { return v3{bsh[3 * i], bsh[3 * i + 1], bsh[3 * i + 2]}; };
            v3 dL_dRGB = {q[0], q[1], q[2]};
            dL_dRGB.x *= st->clamped[3 * idx + 0] ? 0 : 1;
            dL_dRGB.y *= st->clamped[3 * idx + 1] ? 0 : 1;
            dL_dRGB.z *= st->clamped[3 * idx + 2] ? 0 : 1;
            v3 dRGBdx = {0, 0, 0}, dRGBdy = {0, 0, 0}, dRGBdz = {0, 0, 0};
            const float x = dir.x, y = dir.y, z = dir.z;
            float* o = dsh + (size_t)idx * max_coeffs * 3;
            auto put = [&](int i, v3 v) { o[3 * i] = v.x; o[3 * i + 1] = v.y; o[3 * i + 2] = v.z; };
            put(0, SH_C0 * dL_dRGB);
            if (deg > 0) {
                const float s1 = -SH_C1 * y, s2 = SH_C1 * z, s3 = -SH_C1 * x;
                put(1, s1 * dL_dRGB); put(2, s2 * dL_dRGB); put(3, s3 * dL_dRGB);
                dRGBdx = -SH_C1 * sh(3);
                dRGBdy = -SH_C1 * sh(1);
                dRGBdz = SH_C1 * sh(2);
                if (deg > 1) {
                    const float xx = x * x, yy = y * y, zz = z * z, xy = x * y, yz = y * z, xz = x * z;
                    put(4, (SH_C2[0] * xy) * dL_dRGB);
                    put(5, (SH_C2[1] * yz) * dL_dRGB);
                    put(6, (SH_C2[2] * (2.f * zz - xx - yy)) * dL_dRGB);
                    put(7, (SH_C2[3] * xz) * dL_dRGB);
                    put(8, (SH_C2[4] * (xx - yy)) * dL_dRGB);
                    dRGBdx = dRGBdx + (SH_C2[0] * y * sh(4) + SH_C2[2] * 2.f * -x * sh(6) + SH_C2[3] * z * sh(7) + SH_C2[4] * 2.f * x * sh(8));
                    dRGBdy = dRGBdy + (SH_C2[0] * x * sh(4) + SH_C2[1] * z * sh(5) + SH_C2[2] * 2.f * -y * sh(6) + SH_C2[4] * 2.f * -y * sh(8));
                    dRGBdz = dRGBdz + (SH_C2[1] * y * sh(5) + SH_C2[2] * 2.f * 2.f * z * sh(6) + SH_C2[3] * x * sh(7));
                    if (deg > 2) {
                        put(9, (SH_C3[0] * y * (3.f * xx - yy)) * dL_dRGB);
                        put(10, (SH_C3[1] * xy * z) * dL_dRGB);
                        put(11, (SH_C3[2] * y * (4.f * zz - xx - yy)) * dL_dRGB);
                        put(12, (SH_C3[3] * z * (2.f * zz - 3.f * xx - 3.f * yy)) * dL_dRGB);
                        put(13, (SH_C3[4] * x * (4.f * zz - xx - yy)) * dL_dRGB);
                        put(14, (SH_C3[5] * z * (xx - yy)) * dL_dRGB);
                        put(15, (SH_C3[6] * x * (xx - 3.f * yy)) * dL_dRGB);
                        dRGBdx = dRGBdx + (SH_C3[0] * sh(9) * 3.f * 2.f * xy + SH_C3[1] * sh(10) * yz +
                                           SH_C3[2] * sh(11) * -2.f * xy + SH_C3[3] * sh(12) * -3.f * 2.f * xz +
                                           SH_C3[4] * sh(13) * (-3.f * xx + 4.f * zz - yy) +
                                           SH_C3[5] * sh(14) * 2.f * xz + SH_C3[6] * sh(15) * 3.f * (xx - yy));
                        dRGBdy = dRGBdy + (SH_C3[0] * sh(9) * 3.f * (xx - yy) + SH_C3[1] * sh(10) * xz +
                                           SH_C3[2] * sh(11) * (-3.f * yy + 4.f * zz - xx) +
                                           SH_C3[3] * sh(12) * -3.f * 2.f * yz + SH_C3[4] * sh(13) * -2.f * xy +
                                           SH_C3[5] * sh(14) * -2.f * yz + SH_C3[6] * sh(15) * -3.f * 2.f * xy);
                        dRGBdz = dRGBdz + (SH_C3[1] * sh(10) * xy + SH_C3[2] * sh(11) * 4.f * 2.f * yz +
                                           SH_C3[3] * sh(12) * 3.f * (2.f * zz - xx - yy) +
                                           SH_C3[4] * sh(13) * 4.f * 2.f * xz + SH_C3[5] * sh(14) * (xx - yy));
                    }
                }
            }
            v3 dL_ddir = {dot(dRGBdx, dL_dRGB), dot(dRGBdy, dL_dRGB), dot(dRGBdz, dL_dRGB)};
            v3 dmsh = dnormvdv(dir_orig, dL_ddir);
            dmean = dmean + dmsh;
        }
        dmeans3D[3 * idx + 0] = dmean.x;
        dmeans3D[3 * idx + 1] = dmean.y;
        dmeans3D[3 * idx + 2] = dmean.z;

        if (in->scales) {
            // computeCov3D backward (backward.cu:276-341)
            const float* rot = in->rotations + 4 * (size_t)idx;
            const float r = rot[0], x = rot[1], y = rot[2], z = rot[3];
            m3 R = mk(1.f - 2.f * (y * y + z * z), 2.f * (x * y - r * z), 2.f * (x * z + r * y),
                      2.f * (x * y + r * z), 1.f - 2.f * (x * x + z * z), 2.f * (y * z - r * x),
                      2.f * (x * z - r * y), 2.f * (y * z + r * x), 1.f - 2.f * (x * x + y * y));
            m3 S = mk(1, 0, 0, 0, 1, 0, 0, 0, 1);
            v3 sc = {in->scales[3 * idx], in->scales[3 * idx + 1], in->scales[3 * idx + 2]};
            v3 sv = s.scale_modifier * sc;
            S.m[0][0] = sv.x; S.m[1][1] = sv.y; S.m[2][2] = sv.z;
            m3 M = mul(S, R);
            m3 dSig = mk(dcv[0], 0.5f * dcv[1], 0.5f * dcv[2], 0.5f * dcv[1], dcv[3], 0.5f * dcv[4],
                         0.5f * dcv[2], 0.5f * dcv[4], dcv[5]);
            m3 dM = mul(smul(2.0f, M), dSig);
            m3 Rt = tr(R);
            m3 dMt = tr(dM);
            dscales[3 * idx + 0] = dot(col(Rt, 0), col(dMt, 0));
            dscales[3 * idx + 1] = dot(col(Rt, 1), col(dMt, 1));
            dscales[3 * idx + 2] = dot(col(Rt, 2), col(dMt, 2));
            for (int rr = 0; rr < 3; ++rr) dMt.m[0][rr] *= sv.x;
            for (int rr = 0; rr < 3; ++rr) dMt.m[1][rr] *= sv.y;
            for (int rr = 0; rr < 3; ++rr) dMt.m[2][rr] *= sv.z;
            const auto& d = dMt.m;
            drot[4 * idx + 0] = 2 * z * (d[0][1] - d[1][0]) + 2 * y * (d[2][0] - d[0][2]) + 2 * x * (d[1][2] - d[2][1]);
            drot[4 * idx + 1] = 2 * y * (d[1][0] + d[0][1]) + 2 * z * (d[2][0] + d[0][2]) + 2 * r * (d[1][2] - d[2][1]) - 4 * x * (d[2][2] + d[1][1]);
            drot[4 * idx + 2] = 2 * x * (d[1][0] + d[0][1]) + 2 * r * (d[2][0] - d[0][2]) + 2 * z * (d[1][2] + d[2][1]) - 4 * y * (d[2][2] + d[0][0]);
            drot[4 * idx + 3] = 2 * r * (d[0][1] - d[1][0]) + 2 * x * (d[2][0] + d[0][2]) + 2 * y * (d[1][2] + d[2][1]) - 4 * z * (d[1][1] + d[0][0]);
        }
    }
    return 0;
}

// Reference markVisible (rasterizer_impl.cu:54-66,141-153 -> auxiliary.h:139-164).
void oracle_mark_visible(int P, const float* means3D, const float* view, uint8_t* present) {
    for (int i = 0; i < P; ++i) {
        v3 p = {means3D[3 * i], means3D[3 * i + 1], means3D[3 * i + 2]};
        present[i] = xform4x3(p, view).z > 0.2f;
    }
}

}  // extern "C"
