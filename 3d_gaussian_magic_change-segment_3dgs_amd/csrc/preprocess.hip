// preprocess.hip -- per-Gaussian kernels: forward preprocess (projection, EWA
// covariance, SH colour, tile rectangle), frustum visibility, and the fused
// per-Gaussian backward (instance-gradient gather + computeCov2DCUDA +
// preprocessCUDA backward of the reference).
//
// Reference: DGR/cuda_rasterizer/forward.cu:18-256, backward.cu:18-412,
// auxiliary.h:41-164, rasterizer_impl.cu:54-66.
//
// FP contraction is OFF in this file: every product/sum is rounded as written,
// in the reference's (glm's) evaluation order.  Division and sqrt are IEEE
// correctly rounded (hipcc default -fhip-fp32-correctly-rounded-divide-sqrt),
// ndc2Pix runs in double.  With the same choices in the CPU oracle, radii,
// tiles_touched, depth bits, rectangles and therefore every key, point_list and
// range are bit-identical to the oracle.
#pragma clang fp contract(off)

#include "gsr_internal.h"

// Two translation units: this file (GSR_PRE_PART 1) and gaussian_bwd.hip, which includes it
// for k_gaussian_backward alone (2), built with its own machine-scheduler strategy (Makefile).
#ifndef GSR_PRE_PART
#define GSR_PRE_PART 1
#endif

namespace gsr {
namespace {

// auxiliary.h:21-39
__constant__ float C_SH0 = 0.28209479177387814f;
__constant__ float C_SH1 = 0.4886025119029199f;
__constant__ float C_SH2[5] = {1.0925484305920792f, -1.0925484305920792f, 0.31539156525252005f,
                               -1.0925484305920792f, 0.5462742152960396f};
__constant__ float C_SH3[7] = {-0.5900435899266435f, 2.890611442640554f, -0.4570457994644658f,
                               0.3731763325901154f, -0.4570457994644658f, 1.445305721320277f,
                               -0.5900435899266435f};

struct f3 { float x, y, z; };
__device__ __forceinline__ f3 operator+(f3 a, f3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
__device__ __forceinline__ f3 operator-(f3 a, f3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
__device__ __forceinline__ f3 operator*(float s, f3 a) { return {s * a.x, s * a.y, s * a.z}; }
__device__ __forceinline__ f3 operator*(f3 a, float s) { return {a.x * s, a.y * s, a.z * s}; }
__device__ __forceinline__ f3 operator/(f3 a, float s) { return {a.x / s, a.y / s, a.z / s}; }
__device__ __forceinline__ float dot3(f3 a, f3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }

// Column-major 3x3 with glm semantics: m[col][row].
struct M3 { float m[3][3]; };
__device__ __forceinline__ M3 mat3(float a, float b, float c, float d, float e, float f, float g, float h,
                                   float i) {
    M3 r;
    r.m[0][0] = a; r.m[0][1] = b; r.m[0][2] = c;
    r.m[1][0] = d; r.m[1][1] = e; r.m[1][2] = f;
    r.m[2][0] = g; r.m[2][1] = h; r.m[2][2] = i;
    return r;
}
// glm operator*(mat3, mat3): R[c][r] = A[0][r]*B[c][0] + A[1][r]*B[c][1] + A[2][r]*B[c][2]
__device__ __forceinline__ M3 mmul(const M3& A, const M3& B) {
    M3 R;
#pragma unroll
    for (int c = 0; c < 3; ++c)
#pragma unroll
        for (int r = 0; r < 3; ++r)
            R.m[c][r] = A.m[0][r] * B.m[c][0] + A.m[1][r] * B.m[c][1] + A.m[2][r] * B.m[c][2];
    return R;
}
__device__ __forceinline__ M3 mtr(const M3& A) {
    M3 R;
#pragma unroll
    for (int c = 0; c < 3; ++c)
#pragma unroll
        for (int r = 0; r < 3; ++r) R.m[c][r] = A.m[r][c];
    return R;
}

__device__ __forceinline__ f3 xform4x3(f3 p, const float* m) {
    return {m[0] * p.x + m[4] * p.y + m[8] * p.z + m[12], m[1] * p.x + m[5] * p.y + m[9] * p.z + m[13],
            m[2] * p.x + m[6] * p.y + m[10] * p.z + m[14]};
}
__device__ __forceinline__ float4 xform4x4(f3 p, const float* m) {
    return {m[0] * p.x + m[4] * p.y + m[8] * p.z + m[12], m[1] * p.x + m[5] * p.y + m[9] * p.z + m[13],
            m[2] * p.x + m[6] * p.y + m[10] * p.z + m[14], m[3] * p.x + m[7] * p.y + m[11] * p.z + m[15]};
}
__device__ __forceinline__ f3 xformVecT(f3 p, const float* m) {
    return {m[0] * p.x + m[1] * p.y + m[2] * p.z, m[4] * p.x + m[5] * p.y + m[6] * p.z,
            m[8] * p.x + m[9] * p.y + m[10] * p.z};
}

// auxiliary.h:41-44
__device__ __forceinline__ float ndc2pix(float v, int S) { return (float)(((v + 1.0) * S - 1.0) * 0.5); }

// auxiliary.h:46-56
__device__ __forceinline__ void get_rect(float px, float py, int r, int gx, int gy, int& x0, int& y0, int& x1,
                                         int& y1) {
    x0 = min(gx, max(0, (int)((px - (float)r) / (float)BX)));
    y0 = min(gy, max(0, (int)((py - (float)r) / (float)BY)));
    x1 = min(gx, max(0, (int)((((px + (float)r) + (float)BX) - 1.0f) / (float)BX)));
    y1 = min(gy, max(0, (int)((((py + (float)r) + (float)BY) - 1.0f) / (float)BY)));
}

__device__ __forceinline__ f3 ld3(const float* p) { return {p[0], p[1], p[2]}; }

// forward.cu:118-152 (quaternion used as given: normalised upstream)
__device__ __forceinline__ void cov3d_from(f3 scale, float mod, float4 q, float c[6]) {
    M3 S = mat3(1, 0, 0, 0, 1, 0, 0, 0, 1);
    S.m[0][0] = mod * scale.x;
    S.m[1][1] = mod * scale.y;
    S.m[2][2] = mod * scale.z;
    const float r = q.x, x = q.y, y = q.z, z = q.w;
    M3 R = mat3(1.f - 2.f * (y * y + z * z), 2.f * (x * y - r * z), 2.f * (x * z + r * y),
                2.f * (x * y + r * z), 1.f - 2.f * (x * x + z * z), 2.f * (y * z - r * x),
                2.f * (x * z - r * y), 2.f * (y * z + r * x), 1.f - 2.f * (x * x + y * y));
    M3 Mm = mmul(S, R);
    M3 Sig = mmul(mtr(Mm), Mm);
    c[0] = Sig.m[0][0]; c[1] = Sig.m[0][1]; c[2] = Sig.m[0][2];
    c[3] = Sig.m[1][1]; c[4] = Sig.m[1][2]; c[5] = Sig.m[2][2];
}

// Clamped camera-space mean, J, W, T of forward.cu:80-99 / backward.cu:166-192.
struct EwaTerms { f3 t; float txtz, tytz, limx, limy; M3 W, T; };
__device__ __forceinline__ EwaTerms ewa_terms(f3 mean, float fx, float fy, float tanx, float tany,
                                              const float* view) {
    EwaTerms e;
    f3 t = xform4x3(mean, view);
    e.limx = 1.3f * tanx;
    e.limy = 1.3f * tany;
    e.txtz = t.x / t.z;
    e.tytz = t.y / t.z;
    t.x = fminf(e.limx, fmaxf(-e.limx, e.txtz)) * t.z;
    t.y = fminf(e.limy, fmaxf(-e.limy, e.tytz)) * t.z;
    e.t = t;
    M3 J = mat3(fx / t.z, 0.0f, -(fx * t.x) / (t.z * t.z), 0.0f, fy / t.z, -(fy * t.y) / (t.z * t.z), 0, 0, 0);
    e.W = mat3(view[0], view[4], view[8], view[1], view[5], view[9], view[2], view[6], view[10]);
    e.T = mmul(e.W, J);
    return e;
}

__device__ __forceinline__ M3 vrk_of(const float* c) {
    return mat3(c[0], c[1], c[2], c[1], c[3], c[4], c[2], c[4], c[5]);
}

// One Gaussian's SH row (M coefficients x 3 floats, the first ncoef used).  Rows of
// a multiple of 4 floats (M = 16 in training) are fetched with 16-B loads: at a
// 192-B stride between lanes every load instruction touches 64 cache lines, so 12
// float4 loads cost a quarter of the memory-pipeline work of 48 dword loads.
// Streaming hints: the forward's SH row loads and the backward's dsh row stores are
// non-temporal (read / written once per view).  Measured at 1M, SH3: preprocess 83 -> 62 us,
// per-Gaussian backward 152 -> 150 us.  The backward's own SH row loads stay ordinary:
// non-temporal there cost 150 -> 220 us (thread-own 192-B rows re-touch each line 12 times).
// GSR_NO_NT_SH restores ordinary accesses.
#ifndef GSR_NO_NT_SH
#define GSR_NT_SH_LOAD
#define GSR_NT_SH_STORE
#endif
typedef float sh_v4 __attribute__((ext_vector_type(4)));
// The SH-row staging below is per wave (each wave parks and reads back only its own LDS rows),
// so a wave-level LDS fence replaces the block barriers: a wave's LDS instructions execute in
// order, so waiting for its own outstanding LDS operations (and keeping the compiler from moving
// LDS accesses across the point) orders its writes before its reads and its reads before the next
// pass's writes.  Without block barriers the four waves of a block no longer wait for each other
// at every pass, so their loads overlap more.
__device__ __forceinline__ void wave_lds_fence() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }
// Inclusive scan over the wave with DPP (row_shr inside 16-lane rows, then row_bcast 15 / 31).
__device__ __forceinline__ uint32_t wave_scan_incl(uint32_t x) {
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xF, 0xF, true);  // row_shr:1
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xF, 0xF, true);  // row_shr:2
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xF, 0xF, true);  // row_shr:4
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xF, 0xF, true);  // row_shr:8
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xA, 0xF, false); // row_bcast:15
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xC, 0xF, false); // row_bcast:31
    return x;
}

#ifdef GSR_BLOCK_SYNC  // (A/B: the block barriers the fence replaced)
#define GSR_WAVE_SYNC() __syncthreads()
#else
#define GSR_WAVE_SYNC() wave_lds_fence()
#endif

__device__ __forceinline__ float4 sh_ld(const float4* p) {
#ifdef GSR_NT_SH_LOAD
    const sh_v4 r = __builtin_nontemporal_load(reinterpret_cast<const sh_v4*>(p));
    return make_float4(r.x, r.y, r.z, r.w);
#else
    return *p;
#endif
}
__device__ __forceinline__ void sh_st(float4* p, float4 v) {
#ifdef GSR_NT_SH_STORE
    const sh_v4 r = {v.x, v.y, v.z, v.w};
    __builtin_nontemporal_store(r, reinterpret_cast<sh_v4*>(p));
#else
    *p = v;
#endif
}

struct ShRow {
    float v[48];
    __device__ __forceinline__ void load(const float* p, int M, int ncoef) {
        const int nf = 3 * ncoef;
        if (((3 * M) & 3) == 0 && (reinterpret_cast<uintptr_t>(p) & 15) == 0) {
            const float4* q = reinterpret_cast<const float4*>(p);
#pragma unroll
            for (int i = 0; i < 12; ++i)
                if (4 * i < nf) {
                    const float4 t = q[i];
                    v[4 * i] = t.x; v[4 * i + 1] = t.y; v[4 * i + 2] = t.z; v[4 * i + 3] = t.w;
                }
        } else {
#pragma unroll
            for (int i = 0; i < 48; ++i)
                if (i < nf) v[i] = p[i];
        }
    }
    __device__ __forceinline__ f3 operator()(int i) const { return {v[3 * i], v[3 * i + 1], v[3 * i + 2]}; }
};

// forward.cu:20-71: RGB from SH (deg <= 3), +0.5, clamp >= 0, record clamping.
template <typename SF>
__device__ __forceinline__ f3 color_from_sh(int deg, f3 dir, const SF& S, uint8_t& clamp_bits) {
    f3 result = C_SH0 * S(0);
    if (deg > 0) {
        const float x = dir.x, y = dir.y, z = dir.z;
        result = result - C_SH1 * y * S(1) + C_SH1 * z * S(2) - C_SH1 * x * S(3);
        if (deg > 1) {
            const float xx = x * x, yy = y * y, zz = z * z;
            const float xy = x * y, yz = y * z, xz = x * z;
            result = result + C_SH2[0] * xy * S(4) + C_SH2[1] * yz * S(5) +
                     C_SH2[2] * (2.0f * zz - xx - yy) * S(6) + C_SH2[3] * xz * S(7) +
                     C_SH2[4] * (xx - yy) * S(8);
            if (deg > 2) {
                result = result + C_SH3[0] * y * (3.0f * xx - yy) * S(9) + C_SH3[1] * xy * z * S(10) +
                         C_SH3[2] * y * (4.0f * zz - xx - yy) * S(11) +
                         C_SH3[3] * z * (2.0f * zz - 3.0f * xx - 3.0f * yy) * S(12) +
                         C_SH3[4] * x * (4.0f * zz - xx - yy) * S(13) + C_SH3[5] * z * (xx - yy) * S(14) +
                         C_SH3[6] * x * (xx - 3.0f * yy) * S(15);
            }
        }
    }
    result = result + f3{0.5f, 0.5f, 0.5f};
    clamp_bits = (uint8_t)((result.x < 0 ? 1 : 0) | (result.y < 0 ? 2 : 0) | (result.z < 0 ? 4 : 0));
    return {fmaxf(result.x, 0.0f), fmaxf(result.y, 0.0f), fmaxf(result.z, 0.0f)};
}

// The direction Jacobian of the SH colour, d(rgb)/d(dir) as three f3 over the colour
// channels (dx, dy, dz: the dRGBdx / dRGBdy / dRGBdz of backward.cu:54-107), written in
// the reference's evaluation order.  The forward evaluates it while the SH row is at
// hand (LDS) and stores it (GeomLayout::shjac, wave-blocked SoA); the backward then needs
// no SH coefficients at all: dL/ddir = (dx . dRGB, dy . dRGB, dz . dRGB)
// (backward.cu:109-111) from 36 B per Gaussian instead of a 192-B SH row.  The same
// expressions under the same contraction setting: bit-identical to evaluating them in
// the backward, as the reference and the oracle do.
template <typename SF>
__device__ __forceinline__ void sh_dir_jacobian(int deg, f3 dir, const SF& S, f3& dx, f3& dy, f3& dz) {
    dx = {0, 0, 0};
    dy = {0, 0, 0};
    dz = {0, 0, 0};
    const float x = dir.x, y = dir.y, z = dir.z;
    if (deg > 0) {
        dx = -C_SH1 * S(3);
        dy = -C_SH1 * S(1);
        dz = C_SH1 * S(2);
        if (deg > 1) {
            const float xx = x * x, yy = y * y, zz = z * z, xy = x * y, yz = y * z, xz = x * z;
            dx = dx + (C_SH2[0] * y * S(4) + C_SH2[2] * 2.f * -x * S(6) + C_SH2[3] * z * S(7) +
                       C_SH2[4] * 2.f * x * S(8));
            dy = dy + (C_SH2[0] * x * S(4) + C_SH2[1] * z * S(5) + C_SH2[2] * 2.f * -y * S(6) +
                       C_SH2[4] * 2.f * -y * S(8));
            dz = dz + (C_SH2[1] * y * S(5) + C_SH2[2] * 2.f * 2.f * z * S(6) + C_SH2[3] * x * S(7));
            if (deg > 2) {
                dx = dx + (C_SH3[0] * S(9) * 3.f * 2.f * xy + C_SH3[1] * S(10) * yz +
                           C_SH3[2] * S(11) * -2.f * xy + C_SH3[3] * S(12) * -3.f * 2.f * xz +
                           C_SH3[4] * S(13) * (-3.f * xx + 4.f * zz - yy) + C_SH3[5] * S(14) * 2.f * xz +
                           C_SH3[6] * S(15) * 3.f * (xx - yy));
                dy = dy + (C_SH3[0] * S(9) * 3.f * (xx - yy) + C_SH3[1] * S(10) * xz +
                           C_SH3[2] * S(11) * (-3.f * yy + 4.f * zz - xx) + C_SH3[3] * S(12) * -3.f * 2.f * yz +
                           C_SH3[4] * S(13) * -2.f * xy + C_SH3[5] * S(14) * -2.f * yz +
                           C_SH3[6] * S(15) * -3.f * 2.f * xy);
                dz = dz + (C_SH3[1] * S(10) * xy + C_SH3[2] * S(11) * 4.f * 2.f * yz +
                           C_SH3[3] * S(12) * 3.f * (2.f * zz - xx - yy) + C_SH3[4] * S(13) * 4.f * 2.f * xz +
                           C_SH3[5] * S(14) * (xx - yy));
            }
        }
    }
}

// Jacobian storage: per 64 consecutive Gaussians a block of 9 rows x 64 floats (component
// k of Gaussian i at block(i) + 64 k + (i & 63)): every access is a coalesced 256-B row
// and the 9 addresses of a thread are one base plus immediate offsets.
__device__ __forceinline__ float* jac_row(float* J, int idx) { return J + (size_t)(idx & ~63) * 9 + (idx & 63); }
__device__ __forceinline__ const float* jac_row(const float* J, int idx) {
    return J + (size_t)(idx & ~63) * 9 + (idx & 63);
}

// SH basis values bas[i] = dRGB/dsh[i] (backward.cu:46-107); entries >= (deg+1)^2 are 0.
__device__ __forceinline__ void sh_basis(int deg, f3 dir, float bas[16]) {
#pragma unroll
    for (int i = 0; i < 16; ++i) bas[i] = 0.f;
    const float x = dir.x, y = dir.y, z = dir.z;
    bas[0] = C_SH0;
    if (deg > 0) {
        bas[1] = -C_SH1 * y; bas[2] = C_SH1 * z; bas[3] = -C_SH1 * x;
        if (deg > 1) {
            const float xx = x * x, yy = y * y, zz = z * z, xy = x * y, yz = y * z, xz = x * z;
            bas[4] = C_SH2[0] * xy;
            bas[5] = C_SH2[1] * yz;
            bas[6] = C_SH2[2] * (2.f * zz - xx - yy);
            bas[7] = C_SH2[3] * xz;
            bas[8] = C_SH2[4] * (xx - yy);
            if (deg > 2) {
                bas[9] = C_SH3[0] * y * (3.f * xx - yy);
                bas[10] = C_SH3[1] * xy * z;
                bas[11] = C_SH3[2] * y * (4.f * zz - xx - yy);
                bas[12] = C_SH3[3] * z * (2.f * zz - 3.f * xx - 3.f * yy);
                bas[13] = C_SH3[4] * x * (4.f * zz - xx - yy);
                bas[14] = C_SH3[5] * z * (xx - yy);
                bas[15] = C_SH3[6] * x * (xx - 3.f * yy);
            }
        }
    }
}

struct Cam {
    float view[16], proj[16];
    f3 campos;
};

// Camera matrices live in device memory (the reference passes CUDA tensors); they are
// read through the constant address space, i.e. as scalar (SMEM) loads into SGPRs: the
// compiler cannot prove on its own that no store of the kernel aliases them, and plain
// loads become per-lane vector loads issued late behind the kernel's other memory work.
// (The forward preprocess keeps plain loads: measured faster there, 0.0695 vs 0.0736 ms.)
__device__ __forceinline__ void load_cam(const gsr_settings& s, Cam& c) {
#pragma unroll
    for (int i = 0; i < 16; ++i) { c.view[i] = s.viewmatrix[i]; c.proj[i] = s.projmatrix[i]; }
    c.campos = ld3(s.campos);
}
typedef const __attribute__((address_space(4))) float* const_fp;
__device__ __forceinline__ void load_cam_smem(const gsr_settings& s, Cam& c) {
    const const_fp V = (const_fp)s.viewmatrix, Pm = (const_fp)s.projmatrix, C = (const_fp)s.campos;
#pragma unroll
    for (int i = 0; i < 16; ++i) { c.view[i] = V[i]; c.proj[i] = Pm[i]; }
    c.campos = {C[0], C[1], C[2]};
}

// ------------------------------------------------------------------ forward --
// preprocessCUDA (forward.cu:154-256).  One thread per Gaussian.
__global__ void __launch_bounds__(256) k_preprocess(gsr_settings s, gsr_inputs in, int gx, int gy,
                                                    float4* __restrict__ rec, int* __restrict__ radii,
                                                    uint32_t* __restrict__ tiles_touched,
                                                    uint32_t* __restrict__ depth_keys,
                                                    uint8_t* __restrict__ clamped, ushort4* __restrict__ rect,
                                                    uint32_t* __restrict__ rect32, float* __restrict__ shjac,
                                                    float2* __restrict__ og,
                                                    uint32_t* __restrict__ btot,
                                                    void* zero_a, size_t zero_a16, void* zero_b, size_t zero_b16) {
    const int idx = blockIdx.x * blockDim.x + threadIdx.x;
    // clear the depth sort's and the scan's look-back counters (saves two memset launches)
    zero16(zero_a, zero_a16, idx, (size_t)gridDim.x * blockDim.x);
    zero16(zero_b, zero_b16, idx, (size_t)gridDim.x * blockDim.x);
    // No early exits: the SH rows are staged through LDS by the whole block below, so
    // every thread reaches the barriers; `ok` carries the reference's culls.
    const bool live = idx < s.P;
    const int sidx = live ? idx : 0;
    Cam cam;
    load_cam(s, cam);

    // SH3 rows through LDS (below): the first half-run's loads are issued before the
    // projection math so their latency overlaps it.
    const bool sh_lds = in.colors_precomp == nullptr && s.M == 16 && (reinterpret_cast<uintptr_t>(in.shs) & 15) == 0;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int wbase = blockIdx.x * blockDim.x + wave * 64;
    float4 shv[6];
    if (sh_lds) {
        const float4* src = reinterpret_cast<const float4*>(in.shs + (size_t)wbase * 48);
#pragma unroll
        for (int r = 0; r < 6; ++r) {
            const int f = lane + 64 * r;
            const int row = f / 12;
            shv[r] = (wbase + row < s.P) ? sh_ld(src + f) : make_float4(0.f, 0.f, 0.f, 0.f);
        }
    }

    const f3 p_orig = ld3(in.means3D + 3 * (size_t)sidx);
    const float opacity = in.opacities[sidx];
    // in_frustum (auxiliary.h:139-164)
    const f3 p_view = xform4x3(p_orig, cam.view);
    bool ok = live && p_view.z > 0.2f;
    const float4 p_hom = xform4x4(p_orig, cam.proj);
    const float p_w = 1.0f / (p_hom.w + 0.0000001f);
    const f3 p_proj = {p_hom.x * p_w, p_hom.y * p_w, p_hom.z * p_w};

    float c3[6];
    if (in.cov3D_precomp) {
        const float* c = in.cov3D_precomp + 6 * (size_t)sidx;
#pragma unroll
        for (int i = 0; i < 6; ++i) c3[i] = c[i];
    } else {
        const float4 q = *reinterpret_cast<const float4*>(in.rotations + 4 * (size_t)sidx);
        cov3d_from(ld3(in.scales + 3 * (size_t)sidx), s.scale_modifier, q, c3);
    }
    const float focal_y = s.H / (2.0f * s.tanfovy);
    const float focal_x = s.W / (2.0f * s.tanfovx);
    const EwaTerms e = ewa_terms(p_orig, focal_x, focal_y, s.tanfovx, s.tanfovy, cam.view);
    const M3 cov = mmul(mmul(mtr(e.T), mtr(vrk_of(c3))), e.T);
    const float cx = cov.m[0][0] + 0.3f, cy = cov.m[0][1], cz = cov.m[1][1] + 0.3f;

    const float det = (cx * cz - cy * cy);
    ok = ok && det != 0.0f;
    const float det_inv = 1.f / det;
    const float conic_x = cz * det_inv, conic_y = -cy * det_inv, conic_z = cx * det_inv;
    const float mid = 0.5f * (cx + cz);
    const float lambda1 = mid + sqrtf(fmaxf(0.1f, mid * mid - det));
    const float lambda2 = mid - sqrtf(fmaxf(0.1f, mid * mid - det));
    const float my_radius = ceilf(3.f * sqrtf(fmaxf(lambda1, lambda2)));
    const float px = ndc2pix(p_proj.x, s.W), py = ndc2pix(p_proj.y, s.H);
    int x0 = 0, y0 = 0, x1 = 0, y1 = 0;
    if (ok) get_rect(px, py, (int)my_radius, gx, gy, x0, y0, x1, y1);
    const uint32_t ntiles = (uint32_t)((x1 - x0) * (y1 - y0));
    ok = ok && ntiles != 0;
    // Record slots in Gaussian-index order: the block's exclusive scan of the tile counts here,
    // the blocks' bases from their totals btot in the depth sort's histogram kernel (bbase, see
    // block_bases): Gaussian idx's first slot is og[idx].y + bbase[idx / 256].  Neighbouring
    // Gaussians then own neighbouring slot ranges, which the per-Gaussian backward reads.  The wave
    // scan (DPP) runs here, the block combine after the SH work (slot_scan_finish), behind a bare
    // s_barrier: __syncthreads' fence would also wait for the SH loads in flight.
    __shared__ uint32_t s_wtot[4];
    const uint32_t t_ok = ok ? ntiles : 0u;
    const uint32_t t_incl = wave_scan_incl(t_ok);
    if (lane == 63) s_wtot[wave] = t_incl;
    auto slot_scan_finish = [&]() {
        wave_lds_fence();
        __builtin_amdgcn_s_barrier();  // (without it: the same time, round5_h_index_order_slots.txt)
        wave_lds_fence();
        uint32_t pre = 0;
#pragma unroll
        for (int w = 0; w < 4; ++w) pre += w < wave ? s_wtot[w] : 0u;
        const uint32_t slot = pre + t_incl - t_ok;
        if (threadIdx.x == 0) btot[blockIdx.x] = s_wtot[0] + s_wtot[1] + s_wtot[2] + s_wtot[3];
        if (live) og[idx] = make_float2(opacity, __uint_as_float(slot));  // (opacity, in-block first slot)
        return slot;
    };

    f3 rgb = {0.f, 0.f, 0.f};
    uint8_t cbits = 0;
    // the SH direction Jacobian goes straight out (ok is final here): no live range
    // across the LDS passes.  Coalesced 256-B rows (jac_row).
    auto store_jac = [&](f3 jx, f3 jy, f3 jz) {
        float* J = jac_row(shjac, idx);
        J[0] = jx.x; J[64] = jx.y; J[128] = jx.z;
        J[192] = jy.x; J[256] = jy.y; J[320] = jy.z;
        J[384] = jz.x; J[448] = jz.y; J[512] = jz.z;
    };
    const bool want_jac = shjac && s.D > 0;
    if (in.colors_precomp == nullptr) {
        f3 dir = p_orig - cam.campos;
        dir = dir / sqrtf(dot3(dir, dir));
        if (sh_lds) {
            // SH3 rows (192 B) through LDS: the wave loads 32 rows at a time as
            // consecutive float4s (a thread loading its own row issues loads 192 B
            // apart: 0.056 ms of a 0.100 ms kernel at 1M), then the 32 owners evaluate
            // their colour from LDS.  Rows padded to 52 floats (2-way bank aliasing).
            __shared__ float shrow[4][32][52];
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int g0 = wbase + 32 * h;
                if (h == 1) {
                    const float4* src = reinterpret_cast<const float4*>(in.shs + (size_t)g0 * 48);
#pragma unroll
                    for (int r = 0; r < 6; ++r) {
                        const int f = lane + 64 * r;
                        shv[r] = (g0 + f / 12 < s.P) ? sh_ld(src + f) : make_float4(0.f, 0.f, 0.f, 0.f);
                    }
                }
#pragma unroll
                for (int r = 0; r < 6; ++r) {
                    const int f = lane + 64 * r;  // float4 index in the 32-row run
                    const int row = f / 12, col = f - 12 * (f / 12);
                    *reinterpret_cast<float4*>(&shrow[wave][row][4 * col]) = shv[r];
                }
                GSR_WAVE_SYNC();
                if ((lane >> 5) == h && ok) {
                    const float* S = shrow[wave][lane & 31];
                    auto Sf = [&](int i) { return f3{S[3 * i], S[3 * i + 1], S[3 * i + 2]}; };
                    rgb = color_from_sh(s.D, dir, Sf, cbits);
                    if (want_jac) {
                        f3 jx, jy, jz;
                        sh_dir_jacobian(s.D, dir, Sf, jx, jy, jz);
                        store_jac(jx, jy, jz);
                    }
                }
                GSR_WAVE_SYNC();
            }
        } else if (ok) {
            // per-coefficient loads: here they overlap the projection math better than a
            // row of float4 loads issued up front (measured: 0.091 vs 0.100 ms at 1M)
            const float* sh = in.shs + (size_t)idx * s.M * 3;
            auto Sf = [&](int i) { return ld3(sh + 3 * i); };
            rgb = color_from_sh(s.D, dir, Sf, cbits);
            if (want_jac) {
                f3 jx, jy, jz;
                sh_dir_jacobian(s.D, dir, Sf, jx, jy, jz);
                store_jac(jx, jy, jz);
            }
        }
    } else if (ok) {
        rgb = ld3(in.colors_precomp + 3 * (size_t)idx);
    }
    const uint32_t slot0 = slot_scan_finish();
    if (!ok) {  // culled (the reference's early returns): no tiles, sorted last
        if (live) {
            radii[idx] = 0;
            tiles_touched[idx] = 0;
            depth_keys[idx] = 0xFFFFFFFFu;  // culled Gaussians sort last; they emit no instances
            clamped[idx] = 0;
            if (rect32) rect32[idx] = 0u;   // empty rect: no tiles
        }
        return;
    }
    float s0 = 0.f, s1 = 0.f;
    if (in.segments) {
        const float2 sg = *reinterpret_cast<const float2*>(in.segments + 2 * (size_t)idx);
        s0 = sg.x;
        s1 = sg.y;
    }
    float4* R = rec + (size_t)idx * REC_F4;
    R[0] = make_float4(px, py, conic_x, conic_y);
    R[1] = make_float4(conic_z, opacity, p_view.z, s0);
    R[2] = make_float4(rgb.x, rgb.y, rgb.z, s1);
    // R[3]: the tile rectangle (x0 | y0 << 16, x1 | y1 << 16), from which the render backward forms
    // an instance's record slot goff + (y - y0) (x1 - x0) + (x - x0) (binning_rows.hip) -- so the
    // binning writes no per-instance slot array.  All 64 B are written: with 48 written, the
    // record's second 32-B sector was a partial write (read-modify-write in memory; rocprof, round
    // 5: C5 preprocess 540 -> 447 us, the metric scene 69.1 -> 68.1 us).
    R[3] = make_float4(__uint_as_float((uint32_t)x0 | ((uint32_t)y0 << 16)),
                       __uint_as_float((uint32_t)x1 | ((uint32_t)y1 << 16)), __uint_as_float(slot0), 0.f);
    radii[idx] = (int)my_radius;
    tiles_touched[idx] = ntiles;
    depth_keys[idx] = __float_as_uint(p_view.z);
    clamped[idx] = cbits;
    if (!rect32)  // the unpacked rect is read only when the packed one is unavailable
        rect[idx] = make_ushort4((unsigned short)x0, (unsigned short)y0, (unsigned short)x1, (unsigned short)y1);
    if (rect32) rect32[idx] = (uint32_t)x0 | ((uint32_t)y0 << 8) | ((uint32_t)x1 << 16) | ((uint32_t)y1 << 24);
}

// checkFrustum (rasterizer_impl.cu:54-66)
__global__ void k_mark_visible(int P, const float* __restrict__ means3D, const float* __restrict__ view,
                               uint8_t* __restrict__ present) {
    const int idx = blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= P) return;
    float v[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) v[i] = view[i];
    present[idx] = xform4x3(ld3(means3D + 3 * (size_t)idx), v).z > 0.2f ? 1 : 0;
}

// Gather-sum of the written instance records of one Gaussian's slot range [lo, hi)
// (a Gaussian's slots are contiguous), in slot order: deterministic.  The sum runs in
// fp64 (rounded once at the end): a Gaussian covering hundreds of tiles otherwise adds
// a sequential fp32 rounding error per tile, which the cov2D backward amplifies by
// 1/det(cov2D)^2 for elongated Gaussians (C5: dscales off by 1.3e-5 of the tensor max
// in fp32).  The kernel is HBM-bound; the fp64 adds cost no time.
__device__ __forceinline__ void sum_records(const float* __restrict__ contrib, const uint8_t* __restrict__ written,
                                            uint32_t lo, uint32_t hi, float q[12]) {
    double d[12];
#pragma unroll
    for (int j = 0; j < 12; ++j) d[j] = 0.0;
    // Written flags (one byte per slot, 0 or 1) are read 32 at a time and folded into a
    // 32-bit mask (slot base + i -> bit i); then the written records of those 32 slots, four
    // per round with their loads issued together.  A Gaussian covering many tiles thus costs
    // one flag round trip per 32 slots instead of one per 8 (the gather was 66 of the
    // kernel's 143 us, most of it in the long ranges' serial round trips).  The record loads
    // of a round's empty places are predicated off: clamped duplicates of the first record
    // cost 6 us of address processing (0.1276 -> 0.1215 ms).  Sums stay in slot order.
    auto fold8 = [](uint64_t f) {  // byte i of f (0 or 1) -> bit i
        return (uint32_t)(((f & 0x0101010101010101ull) * 0x0102040810204080ull) >> 56);
    };
    auto records = [&](uint32_t base, uint32_t bits) {
        while (bits) {
            uint32_t u[4];
            bool v[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                v[k] = bits != 0;
                u[k] = v[k] ? base + (uint32_t)__builtin_ctz(bits) : u[0];
                bits &= bits - 1;
            }
            float4 r[4][3];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const float4* src = reinterpret_cast<const float4*>(contrib + (size_t)u[k] * CONTRIB_STRIDE);
                if (k == 0 || v[k]) {
                    r[k][0] = src[0]; r[k][1] = src[1]; r[k][2] = src[2];
                } else {
                    r[k][0] = r[k][1] = r[k][2] = make_float4(0.f, 0.f, 0.f, 0.f);
                }
            }
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                if (!v[k]) continue;
                d[0] += r[k][0].x; d[1] += r[k][0].y; d[2] += r[k][0].z; d[3] += r[k][0].w;
                d[4] += r[k][1].x; d[5] += r[k][1].y; d[6] += r[k][1].z; d[7] += r[k][1].w;
                d[8] += r[k][2].x; d[9] += r[k][2].y; d[10] += r[k][2].z; d[11] += r[k][2].w;
            }
        }
    };
    // two 16-byte loads per 32 slots, from 16-slot granules (the flag array is 256-B aligned;
    // four 8-byte loads from the range's first word took 0.8 us longer)
    const uint4* w16 = reinterpret_cast<const uint4*>(written);
    const uint32_t glo = lo >> 4, ghi = (hi - 1) >> 4;
    for (uint32_t gi = glo; gi <= ghi; gi += 2) {
        const uint4 f0 = w16[gi], f1 = w16[min(gi + 1, ghi)];
        uint32_t bits = fold8((uint64_t)f0.x | ((uint64_t)f0.y << 32)) |
                        fold8((uint64_t)f0.z | ((uint64_t)f0.w << 32)) << 8 |
                        fold8((uint64_t)f1.x | ((uint64_t)f1.y << 32)) << 16 |
                        fold8((uint64_t)f1.z | ((uint64_t)f1.w << 32)) << 24;
        const uint32_t base = gi << 4;  // slot of bit 0; base <= hi - 1
        if (lo > base) bits &= ~0u << (lo - base);              // lo - base < 16
        if (hi - base < 32u) bits &= (1u << (hi - base)) - 1u;  // drops a clamped duplicate granule too
        records(base, bits);
    }
#pragma unroll
    for (int j = 0; j < 12; ++j) q[j] = (float)d[j];
}

// Wave-cooperative form of sum_records for slots in Gaussian-index order (gsr_internal.h
// SLOT_BLOCK): the 64 lanes' ranges [lo, lo + n) tile one contiguous slot range, so the wave reads
// its written flags as one run (lane l: granule l of 16 slots, 1024 slots per round), lists the
// written slots in LDS by a wave scan, loads their records with one lane per record, and every lane
// then sums its own from LDS -- in slot order, in fp64, as sum_records: the same bits.  Every lane
// of the wave must call it (n = 0 for a lane without records).  W: the wave's LDS.
struct GatherLds {
    uint32_t gran[64];    // per granule: (written slots of the round before it) << 16 | its 16-bit mask
    uint16_t list[1024];  // the round's written slots, as offsets from the round's first slot
    float4 recs[64][3];   // one batch of their records
};
__device__ __forceinline__ void wave_gather(const float* __restrict__ contrib, const uint8_t* __restrict__ written,
                                            uint32_t lo, uint32_t n, float q[12], GatherLds& W) {
    const int lane = threadIdx.x & 63;
    double d[12];
#pragma unroll
    for (int j = 0; j < 12; ++j) d[j] = 0.0;
    const uint32_t hi = lo + n;
    // the wave's range [L, H): the ranges of lanes with records are ordered and adjacent
    uint32_t L = n ? lo : 0xFFFFFFFFu, H = n ? hi : 0u;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        L = min(L, (uint32_t)__shfl_xor((int)L, o, 64));
        H = max(H, (uint32_t)__shfl_xor((int)H, o, 64));
    }
    L = __builtin_amdgcn_readfirstlane(L);
    H = __builtin_amdgcn_readfirstlane(H);
    const uint4* w16 = reinterpret_cast<const uint4*>(written);
    auto fold8 = [](uint64_t f) { return (uint32_t)(((f & 0x0101010101010101ull) * 0x0102040810204080ull) >> 56); };
    for (uint32_t base = L & ~15u; base < H; base += 1024) {  // wave-uniform (L = ~0 when no lane has records)
        const uint32_t s0 = base + 16u * (uint32_t)lane;
        uint32_t m = 0;
        if (s0 < H) {
            const uint4 f = w16[s0 >> 4];
            m = fold8((uint64_t)f.x | ((uint64_t)f.y << 32)) | fold8((uint64_t)f.z | ((uint64_t)f.w << 32)) << 8;
            if (L > s0) m &= 0xFFFFu << min(L - s0, 16u);
            if (H - s0 < 16u) m &= (1u << (H - s0)) - 1u;
        }
        const uint32_t c = (uint32_t)__popc(m);
        const uint32_t incl = wave_scan_incl(c), excl = incl - c;
        const uint32_t total = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
        W.gran[lane] = (excl << 16) | m;
        for (uint32_t mm = m, k = excl; mm; mm &= mm - 1, ++k)
            W.list[k] = (uint16_t)(16u * (uint32_t)lane + (uint32_t)__builtin_ctz(mm));
        wave_lds_fence();
        // this lane's list positions [a, b) in the round
        auto pos = [&](uint32_t sl) -> uint32_t {
            if (sl <= base) return 0u;
            const uint32_t off = sl - base;
            if (off >= 1024u) return total;
            const uint32_t g = W.gran[off >> 4];
            return (g >> 16) + (uint32_t)__popc((g & 0xFFFFu) & ((1u << (off & 15u)) - 1u));
        };
        const uint32_t a = n ? pos(lo) : 0u, b = n ? pos(hi) : 0u;
        for (uint32_t r0 = 0; r0 < total; r0 += 64) {  // wave-uniform
            if (r0 + (uint32_t)lane < total) {
                const float4* src = reinterpret_cast<const float4*>(
                    contrib + (size_t)(base + W.list[r0 + lane]) * CONTRIB_STRIDE);
                const float4 x0 = src[0], x1 = src[1], x2 = src[2];
                W.recs[lane][0] = x0;
                W.recs[lane][1] = x1;
                W.recs[lane][2] = x2;
            }
            wave_lds_fence();
            const uint32_t j0 = max(a, r0), j1 = min(b, r0 + 64u);
            for (uint32_t j = j0; j < j1; ++j) {
                const float4 x0 = W.recs[j - r0][0], x1 = W.recs[j - r0][1], x2 = W.recs[j - r0][2];
                d[0] += x0.x; d[1] += x0.y; d[2] += x0.z; d[3] += x0.w;
                d[4] += x1.x; d[5] += x1.y; d[6] += x1.z; d[7] += x1.w;
                d[8] += x2.x; d[9] += x2.y; d[10] += x2.z; d[11] += x2.w;
            }
            wave_lds_fence();  // the batch is read before the next one overwrites it
        }
    }
#pragma unroll
    for (int j = 0; j < 12; ++j) q[j] = (float)d[j];
}

#if GSR_PRE_PART == 2
// ----------------------------------------------------------------- backward --
// One thread per Gaussian.  Sums the per-(tile, Gaussian) gradient records that
// the render backward wrote at the Gaussian's instance slots (replacing the
// reference's 12 per-pixel atomicAdds, backward.cu:575-636), then runs
// computeCov2DCUDA (backward.cu:141-274) and preprocessCUDA backward
// (backward.cu:343-412) on the sums.  Record layout (12 floats, render.hip):
//   [dcolor.rgb, dseg0, dseg1, ddepth, Q, Qx, Qy, Qxx, Qxy, Qyy]
// with Q* the moments of q = G * dL_dalpha over the Gaussian's pixels.  Since
// dL_dG = opacity * dL_dalpha and conic/opacity are per-Gaussian constants
// (backward.cu:612-636):
//   dopacity  = Q
//   dmean2D.x = -o (a Qx + b Qy) W/2,   dmean2D.y = -o (c Qy + b Qx) H/2
//   dconic    = -o/2 (Qxx, Qxy, Qyy)    for conic (a, b, c), opacity o.
#ifdef GSR_GBWD_WAVES  // (A/B: a minimum waves-per-SIMD for the register allocator)
#define GSR_GBWD_ATTR __attribute__((amdgpu_waves_per_eu(GSR_GBWD_WAVES)))
#else
#define GSR_GBWD_ATTR
#endif
__global__ void __launch_bounds__(256) GSR_GBWD_ATTR k_gaussian_backward(gsr_settings s, gsr_inputs in,
                                                           const int* __restrict__ radii,
                                                           const uint32_t* __restrict__ tiles_touched,
                                                           const float2* __restrict__ og,
                                                           const uint32_t* __restrict__ bbase,
                                                           const uint8_t* __restrict__ clamped,
                                                           const float* __restrict__ contrib,
                                                           const uint8_t* __restrict__ written,
                                                           const float* __restrict__ shjac, gsr_grads g,
                                                           float* __restrict__ shx) {
    // shx != NULL (gsr_backward_deferred_sh): the SH exchange rows of this view -- the
    // clamped dRGB [P,3] and the camera centre -- instead of dsh (g.dsh is NULL then)
    const int idx = blockIdx.x * blockDim.x + threadIdx.x;
    const int M = s.M;
    const size_t i3 = 3 * (size_t)idx;
    const bool live = idx < s.P;
    // per-wave LDS: the record gather's, then the dsh staging's (each wave uses only its own part,
    // so the two phases may share it without a block barrier): 21.5 KB per block, which leaves the
    // kernel at its VGPR-bound occupancy
    union WaveLds {
        GatherLds g;
        float4 srow[16][13];
    };
    __shared__ WaveLds s_wave[4];
    // Every per-Gaussian input that does not depend on the record sums is loaded up front
    // (clamped index for the tail threads), so that their latencies overlap each other
    // and the record gather instead of forming a chain of round trips after it.
    const int ci = live ? idx : 0;
    const size_t c3i = 3 * (size_t)ci;
    Cam cam;
    load_cam_smem(s, cam);
    const int rad = radii[ci];
    const float2 og_i = og[ci];
    const uint32_t lo_slot = __float_as_uint(og_i.y) + bbase[ci / SLOT_BLOCK], n_slot = tiles_touched[ci];
    const float op = og_i.x;
    const f3 mean = ld3(in.means3D + c3i);
    float c3[6];
    float4 quat = make_float4(0.f, 0.f, 0.f, 0.f);
    f3 scale = {0.f, 0.f, 0.f};
    if (in.cov3D_precomp) {
#pragma unroll
        for (int i = 0; i < 6; ++i) c3[i] = in.cov3D_precomp[6 * (size_t)ci + i];
    } else {
        quat = *reinterpret_cast<const float4*>(in.rotations + 4 * (size_t)ci);
        scale = ld3(in.scales + c3i);
    }
    const uint8_t cbits = in.shs ? clamped[ci] : 0;
    f3 jx = {0, 0, 0}, jy = {0, 0, 0}, jz = {0, 0, 0};
    if (in.shs && s.D > 0) {
        const float* J = jac_row(shjac, ci);
        jx = {J[0], J[64], J[128]};
        jy = {J[192], J[256], J[320]};
        jz = {J[384], J[448], J[512]};
    }
    const bool vis = live && rad > 0;
    // dsh rows (48 floats = 192 B per Gaussian) are written through LDS so that the
    // stores are contiguous runs of the wave's 12 KB output block: a thread storing
    // its own row issues 16-B stores 192 B apart, which measured at 0.09 ms of the
    // kernel's 0.21 ms (the same bytes take ~0.03 ms as coalesced runs).
    const bool stage_dsh = g.dsh && in.shs && M == 16 && (reinterpret_cast<uintptr_t>(g.dsh) & 15) == 0;
    float bas[16];
    float dc[3] = {0.f, 0.f, 0.f};
#pragma unroll
    for (int i = 0; i < 16; ++i) bas[i] = 0.f;
    if (shx && idx == 0) {
        float* c = shx + sh_rows_campos(s.P);
        c[0] = cam.campos.x; c[1] = cam.campos.y; c[2] = cam.campos.z; c[3] = 0.f;
    }
    if (shx && live && !vis) { shx[i3] = 0.f; shx[i3 + 1] = 0.f; shx[i3 + 2] = 0.f; }
    if (live && !vis) {
        // invisible: every gradient is zero (rasterize_points.cu:166-177 zero-init)
        if (g.dmeans2D) { g.dmeans2D[i3] = 0.f; g.dmeans2D[i3 + 1] = 0.f; g.dmeans2D[i3 + 2] = 0.f; }
        if (g.dcolors) { g.dcolors[i3] = 0.f; g.dcolors[i3 + 1] = 0.f; g.dcolors[i3 + 2] = 0.f; }
        if (g.dopacity) g.dopacity[idx] = 0.f;
        if (g.dmeans3D) { g.dmeans3D[i3] = 0.f; g.dmeans3D[i3 + 1] = 0.f; g.dmeans3D[i3 + 2] = 0.f; }
        if (g.dcov3D) for (int i = 0; i < 6; ++i) g.dcov3D[6 * (size_t)idx + i] = 0.f;
        if (g.dsh && in.shs && !stage_dsh) for (int i = 0; i < 3 * M; ++i) g.dsh[(size_t)idx * 3 * M + i] = 0.f;
        if (g.dscales && in.scales) { g.dscales[i3] = 0.f; g.dscales[i3 + 1] = 0.f; g.dscales[i3 + 2] = 0.f; }
        if (g.drot && in.scales) for (int i = 0; i < 4; ++i) g.drot[4 * (size_t)idx + i] = 0.f;
        if (g.dsegments) { g.dsegments[2 * (size_t)idx] = 0.f; g.dsegments[2 * (size_t)idx + 1] = 0.f; }
    }
    // gather-sum of the written instance records of the Gaussian's slot range
    // [lo_slot, lo_slot + tiles_touched), in slot order (deterministic)
    float q[12];
#ifndef GSR_GATHER_PER_LANE
    {
        wave_gather(contrib, written, lo_slot, vis ? n_slot : 0u, q, s_wave[threadIdx.x >> 6].g);
    }
#else
    if (vis) sum_records(contrib, written, lo_slot, lo_slot + n_slot, q);
#endif
    if (vis) {
        // the conic weighting of the mean2D channels happened per lane in the render backward
        const float dm2x = -op * q[7] * (0.5f * s.W);  // q[7] = sum q (a dx + b dy)
        const float dm2y = -op * q[8] * (0.5f * s.H);  // q[8] = sum q (b dx + c dy)
        if (g.dmeans2D) { g.dmeans2D[i3] = dm2x; g.dmeans2D[i3 + 1] = dm2y; g.dmeans2D[i3 + 2] = 0.f; }
        if (g.dcolors) { g.dcolors[i3] = q[0]; g.dcolors[i3 + 1] = q[1]; g.dcolors[i3 + 2] = q[2]; }
        if (g.dopacity) g.dopacity[idx] = q[6];
        if (g.dsegments) { g.dsegments[2 * (size_t)idx] = q[3]; g.dsegments[2 * (size_t)idx + 1] = q[4]; }

        const float focal_y = s.H / (2.0f * s.tanfovy);
        const float focal_x = s.W / (2.0f * s.tanfovx);

        // ---- computeCov2DCUDA (backward.cu:155-273)
        if (!in.cov3D_precomp) cov3d_from(scale, s.scale_modifier, quat, c3);  // == the forward's geom.cov3D
        const float dcx = -0.5f * op * q[9], dcy = -0.5f * op * q[10], dcz = -0.5f * op * q[11];
        const EwaTerms e = ewa_terms(mean, focal_x, focal_y, s.tanfovx, s.tanfovy, cam.view);
        const float x_grad_mul = e.txtz < -e.limx || e.txtz > e.limx ? 0 : 1;
        const float y_grad_mul = e.tytz < -e.limy || e.tytz > e.limy ? 0 : 1;
        const M3 Vrk = vrk_of(c3);
        const M3& T = e.T;
        const M3 cov2D = mmul(mmul(mtr(T), mtr(Vrk)), T);
        const float a = cov2D.m[0][0] + 0.3f;
        const float b = cov2D.m[0][1];
        const float c = cov2D.m[1][1] + 0.3f;
        const float denom = a * c - b * b;
        float dL_da = 0, dL_db = 0, dL_dc = 0;
        const float denom2inv = 1.0f / ((denom * denom) + 0.0000001f);
        float dcv[6] = {0, 0, 0, 0, 0, 0};
        const auto& Tt = T.m;
        if (denom2inv != 0) {
            dL_da = denom2inv * (-c * c * dcx + 2 * b * c * dcy + (denom - a * c) * dcz);
            dL_dc = denom2inv * (-a * a * dcz + 2 * a * b * dcy + (denom - a * c) * dcx);
            dL_db = denom2inv * 2 * (b * c * dcx - (denom + 2 * b * b) * dcy + a * b * dcz);
            dcv[0] = (Tt[0][0] * Tt[0][0] * dL_da + Tt[0][0] * Tt[1][0] * dL_db + Tt[1][0] * Tt[1][0] * dL_dc);
            dcv[3] = (Tt[0][1] * Tt[0][1] * dL_da + Tt[0][1] * Tt[1][1] * dL_db + Tt[1][1] * Tt[1][1] * dL_dc);
            dcv[5] = (Tt[0][2] * Tt[0][2] * dL_da + Tt[0][2] * Tt[1][2] * dL_db + Tt[1][2] * Tt[1][2] * dL_dc);
            dcv[1] = 2 * Tt[0][0] * Tt[0][1] * dL_da + (Tt[0][0] * Tt[1][1] + Tt[0][1] * Tt[1][0]) * dL_db +
                     2 * Tt[1][0] * Tt[1][1] * dL_dc;
            dcv[2] = 2 * Tt[0][0] * Tt[0][2] * dL_da + (Tt[0][0] * Tt[1][2] + Tt[0][2] * Tt[1][0]) * dL_db +
                     2 * Tt[1][0] * Tt[1][2] * dL_dc;
            dcv[4] = 2 * Tt[0][2] * Tt[0][1] * dL_da + (Tt[0][1] * Tt[1][2] + Tt[0][2] * Tt[1][1]) * dL_db +
                     2 * Tt[1][1] * Tt[1][2] * dL_dc;
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
        const auto& Wt = e.W.m;
        const float dL_dJ00 = Wt[0][0] * dL_dT00 + Wt[0][1] * dL_dT01 + Wt[0][2] * dL_dT02;
        const float dL_dJ02 = Wt[2][0] * dL_dT00 + Wt[2][1] * dL_dT01 + Wt[2][2] * dL_dT02;
        const float dL_dJ11 = Wt[1][0] * dL_dT10 + Wt[1][1] * dL_dT11 + Wt[1][2] * dL_dT12;
        const float dL_dJ12 = Wt[2][0] * dL_dT10 + Wt[2][1] * dL_dT11 + Wt[2][2] * dL_dT12;
        const float hx = focal_x, hy = focal_y;
        const f3 t = e.t;
        const float tz = 1.f / t.z, tz2 = tz * tz, tz3 = tz2 * tz;
        const float dL_dtx = x_grad_mul * -hx * tz2 * dL_dJ02;
        const float dL_dty = y_grad_mul * -hy * tz2 * dL_dJ12;
        const float dL_dtz = -hx * tz2 * dL_dJ00 - hy * tz2 * dL_dJ11 + (2 * hx * t.x) * tz3 * dL_dJ02 +
                             (2 * hy * t.y) * tz3 * dL_dJ12;
        f3 dmean = xformVecT({dL_dtx, dL_dty, dL_dtz}, cam.view);
        if (g.dcov3D)
#pragma unroll
            for (int i = 0; i < 6; ++i) g.dcov3D[6 * (size_t)idx + i] = dcv[i];

        // ---- preprocessCUDA backward (backward.cu:372-411)
        const float* proj = cam.proj;
        const float* view = cam.view;
        const f3 m = mean;
        const float4 m_hom = xform4x4(m, proj);
        const float m_w = 1.0f / (m_hom.w + 0.0000001f);
        const float d2x = dm2x, d2y = dm2y;
        const float mul1 = (proj[0] * m.x + proj[4] * m.y + proj[8] * m.z + proj[12]) * m_w * m_w;
        const float mul2 = (proj[1] * m.x + proj[5] * m.y + proj[9] * m.z + proj[13]) * m_w * m_w;
        f3 dm;
        dm.x = (proj[0] * m_w - proj[3] * mul1) * d2x + (proj[1] * m_w - proj[3] * mul2) * d2y;
        dm.y = (proj[4] * m_w - proj[7] * mul1) * d2x + (proj[5] * m_w - proj[7] * mul2) * d2y;
        dm.z = (proj[8] * m_w - proj[11] * mul1) * d2x + (proj[9] * m_w - proj[11] * mul2) * d2y;
        dmean = dmean + dm;
        const float ddepth = q[5];
        const float mul3 = view[2] * m.x + view[6] * m.y + view[10] * m.z + view[14];
        f3 dm2;
        dm2.x = (view[2] - view[3] * mul3) * ddepth;
        dm2.y = (view[6] - view[7] * mul3) * ddepth;
        dm2.z = (view[10] - view[11] * mul3) * ddepth;
        dmean = dmean + dm2;

        if (in.shs) {
            // computeColorFromSH backward (backward.cu:20-139), from the direction Jacobian
            // the forward stored (sh_dir_jacobian): no SH coefficient is read here
            const int deg = s.D;
            const f3 dir_orig = m - cam.campos;
            const f3 dir = dir_orig / sqrtf(dot3(dir_orig, dir_orig));
            const uint8_t cb = cbits;
            f3 dRGB = {q[0], q[1], q[2]};
            dRGB.x *= (cb & 1) ? 0 : 1;
            dRGB.y *= (cb & 2) ? 0 : 1;
            dRGB.z *= (cb & 4) ? 0 : 1;
            const f3 dx = jx, dy = jy, dz = jz;
            // dL/dsh[i] = basis_i * dRGB (backward.cu:46-110); coefficients >= (D+1)^2 get 0
            sh_basis(deg, dir, bas);
            dc[0] = dRGB.x;
            dc[1] = dRGB.y;
            dc[2] = dRGB.z;
            if (shx) {  // the exchange row: the clamped colour gradient (k_gaussian_backward_mv's form)
                shx[i3] = (cb & 1) ? 0.f : q[0];
                shx[i3 + 1] = (cb & 2) ? 0.f : q[1];
                shx[i3 + 2] = (cb & 4) ? 0.f : q[2];
            }
            if (g.dsh && !stage_dsh) {
                float* o = g.dsh + (size_t)idx * M * 3;
                auto val = [&](int f) { return f < 48 ? bas[f / 3] * dc[f % 3] : 0.f; };
                if (((3 * M) & 3) == 0 && (reinterpret_cast<uintptr_t>(o) & 15) == 0 && M <= 16) {
                    float4* o4 = reinterpret_cast<float4*>(o);
#pragma unroll
                    for (int i = 0; i < 12; ++i)
                        if (4 * i < 3 * M)
                            o4[i] = make_float4(val(4 * i), val(4 * i + 1), val(4 * i + 2), val(4 * i + 3));
                } else {
                    for (int f = 0; f < 3 * M; ++f) o[f] = f < 48 ? bas[f / 3] * dc[f % 3] : 0.f;
                }
            }
            const f3 dL_ddir = {dot3(dx, dRGB), dot3(dy, dRGB), dot3(dz, dRGB)};
            // dnormvdv (auxiliary.h:107-117)
            const f3 v = dir_orig, dv = dL_ddir;
            const float sum2 = v.x * v.x + v.y * v.y + v.z * v.z;
            const float invsum32 = 1.0f / sqrtf(sum2 * sum2 * sum2);
            f3 dn;
            dn.x = ((+sum2 - v.x * v.x) * dv.x - v.y * v.x * dv.y - v.z * v.x * dv.z) * invsum32;
            dn.y = (-v.x * v.y * dv.x + (sum2 - v.y * v.y) * dv.y - v.z * v.y * dv.z) * invsum32;
            dn.z = (-v.x * v.z * dv.x - v.y * v.z * dv.y + (sum2 - v.z * v.z) * dv.z) * invsum32;
            dmean = dmean + dn;
        }
        if (g.dmeans3D) { g.dmeans3D[i3] = dmean.x; g.dmeans3D[i3 + 1] = dmean.y; g.dmeans3D[i3 + 2] = dmean.z; }

        if (in.scales) {
            // computeCov3D backward (backward.cu:276-341)
            const float r = quat.x, x = quat.y, y = quat.z, z = quat.w;
            const M3 R = mat3(1.f - 2.f * (y * y + z * z), 2.f * (x * y - r * z), 2.f * (x * z + r * y),
                              2.f * (x * y + r * z), 1.f - 2.f * (x * x + z * z), 2.f * (y * z - r * x),
                              2.f * (x * z - r * y), 2.f * (y * z + r * x), 1.f - 2.f * (x * x + y * y));
            M3 S = mat3(1, 0, 0, 0, 1, 0, 0, 0, 1);
            const f3 sv = s.scale_modifier * scale;
            S.m[0][0] = sv.x;
            S.m[1][1] = sv.y;
            S.m[2][2] = sv.z;
            const M3 Mm = mmul(S, R);
            const M3 dSig = mat3(dcv[0], 0.5f * dcv[1], 0.5f * dcv[2], 0.5f * dcv[1], dcv[3], 0.5f * dcv[4],
                                 0.5f * dcv[2], 0.5f * dcv[4], dcv[5]);
            M3 M2;
#pragma unroll
            for (int cc = 0; cc < 3; ++cc)
#pragma unroll
                for (int rr = 0; rr < 3; ++rr) M2.m[cc][rr] = 2.0f * Mm.m[cc][rr];
            const M3 dM = mmul(M2, dSig);
            const M3 Rt = mtr(R);
            M3 dMt = mtr(dM);
            if (g.dscales) {
                g.dscales[i3 + 0] = Rt.m[0][0] * dMt.m[0][0] + Rt.m[0][1] * dMt.m[0][1] + Rt.m[0][2] * dMt.m[0][2];
                g.dscales[i3 + 1] = Rt.m[1][0] * dMt.m[1][0] + Rt.m[1][1] * dMt.m[1][1] + Rt.m[1][2] * dMt.m[1][2];
                g.dscales[i3 + 2] = Rt.m[2][0] * dMt.m[2][0] + Rt.m[2][1] * dMt.m[2][1] + Rt.m[2][2] * dMt.m[2][2];
            }
#pragma unroll
            for (int rr = 0; rr < 3; ++rr) {
                dMt.m[0][rr] *= sv.x;
                dMt.m[1][rr] *= sv.y;
                dMt.m[2][rr] *= sv.z;
            }
            const auto& d = dMt.m;
            if (g.drot) {
                float* dr = g.drot + 4 * (size_t)idx;
                dr[0] = 2 * z * (d[0][1] - d[1][0]) + 2 * y * (d[2][0] - d[0][2]) + 2 * x * (d[1][2] - d[2][1]);
                dr[1] = 2 * y * (d[1][0] + d[0][1]) + 2 * z * (d[2][0] + d[0][2]) + 2 * r * (d[1][2] - d[2][1]) -
                        4 * x * (d[2][2] + d[1][1]);
                dr[2] = 2 * x * (d[1][0] + d[0][1]) + 2 * r * (d[2][0] - d[0][2]) + 2 * z * (d[1][2] + d[2][1]) -
                        4 * y * (d[2][2] + d[0][0]);
                dr[3] = 2 * r * (d[0][1] - d[1][0]) + 2 * x * (d[2][0] + d[0][2]) + 2 * y * (d[1][2] + d[2][1]) -
                        4 * z * (d[1][1] + d[0][0]);
            }
        }
    }  // vis
    if (stage_dsh) {
        // pass p: lanes 16p..16p+15 of each wave park their rows (padded to 52 floats:
        // conflict-free ds_write_b128), then the wave stores those 16 rows = 3 KB as
        // 192 consecutive float4s.
        const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
        const int wbase = blockIdx.x * blockDim.x + wave * 64;
        auto val = [&](int f) { return bas[f / 3] * dc[f % 3]; };
#pragma unroll
        for (int p = 0; p < 4; ++p) {
            if ((lane >> 4) == p) {
                float4* row = s_wave[wave].srow[lane & 15];
#pragma unroll
                for (int i = 0; i < 12; ++i)
                    row[i] = make_float4(val(4 * i), val(4 * i + 1), val(4 * i + 2), val(4 * i + 3));
            }
            GSR_WAVE_SYNC();
            const int g0 = wbase + 16 * p;
            float4* dst = reinterpret_cast<float4*>(g.dsh + (size_t)g0 * 48);
#pragma unroll
            for (int r = 0; r < 3; ++r) {
                const int f = lane + 64 * r;  // float4 index in the 16-row run
                const int row = f / 12, col = f - 12 * (f / 12);
                if (g0 + row < s.P) sh_st(dst + f, s_wave[wave].srow[row][col]);
            }
            GSR_WAVE_SYNC();
        }
    }
}


#endif  // GSR_PRE_PART == 2
#if GSR_PRE_PART == 1
// ------------------------------------------------------- multi-view backward --
// Parameter gradients of B views summed (gsr_backward_multiview).  Two kernels:
//  k_gaussian_backward_mv: per Gaussian, loops over the views: record gather,
//    computeCov2DCUDA + preprocessCUDA backward per view (the view's camera) including
//    the SH direction term from the direction Jacobian the view's forward stored (no SH
//    row is read), sums dmean / dcov3D / dopacity / dsegments / dcolors over the views,
//    writes each view's dmeans2D, derives dscales / drot ONCE from the summed dcov3D
//    (linear), and leaves each view's clamped dRGB row for the dsh kernel;
//  k_sh_dsh: per Gaussian, dsh = sum over the views of basis(dir) x dRGB from means3D
//    and the rows (the SH exchange's rebuild after an all-gather of the rows, or the
//    local batch), stored once through LDS as coalesced runs.
// The shared inputs are read and the parameter gradients written once per batch.
// (130 VGPRs, 3 waves/SIMD; a 4-wave hint fits 128 without spills but measured slower: 439 vs 423 us
// per 8-view batch; 5 waves spill, 643 us -- profiles/round5_p_mv_occupancy.txt)
__global__ void __launch_bounds__(256) k_gaussian_backward_mv(int P, int D, int M, float scale_modifier,
                                                              gsr_inputs in, MvArgs a, gsr_grads g,
                                                              float* __restrict__ shx) {
    const int idx = blockIdx.x * blockDim.x + threadIdx.x;
    const size_t chunk = sh_rows_floats(P);
    if (shx && idx < a.B) {  // each view's camera centre travels with its dRGB rows
        float* c = shx + (size_t)idx * chunk + sh_rows_campos(P);
        const float* cp = a.v[idx].campos;
        c[0] = cp[0]; c[1] = cp[1]; c[2] = cp[2]; c[3] = 0.f;
    }
    // no early exit: the per-view record gathers are wave operations (wave_gather)
    const bool live = idx < P;
    const int ci = live ? idx : 0;
    const size_t i3 = 3 * (size_t)idx, c3i = 3 * (size_t)ci;
    const f3 mean = ld3(in.means3D + c3i);
    float c3[6];
    float4 quat = make_float4(0.f, 0.f, 0.f, 0.f);
    f3 scale = {0.f, 0.f, 0.f};
    if (in.cov3D_precomp) {
#pragma unroll
        for (int i = 0; i < 6; ++i) c3[i] = in.cov3D_precomp[6 * (size_t)ci + i];
    } else {
        quat = *reinterpret_cast<const float4*>(in.rotations + 4 * (size_t)ci);
        scale = ld3(in.scales + c3i);
        cov3d_from(scale, scale_modifier, quat, c3);
    }
    __shared__ GatherLds s_gl[SLOT_BLOCK / 64];
    const M3 Vrk = vrk_of(c3);
    const auto& V = Vrk.m;
    f3 dmean_sum = {0.f, 0.f, 0.f}, dcol = {0.f, 0.f, 0.f};
    float dcv_sum[6] = {0, 0, 0, 0, 0, 0};
    float dop = 0.f, dseg0 = 0.f, dseg1 = 0.f;
    // the next view's per-Gaussian inputs are loaded while this view's records are gathered (one
    // round trip less in each view's chain of loads -> flags -> records)
    struct MvIn {
        int rad;
        uint32_t tt;
        float2 og;
        uint32_t cb;
    };
    auto load_in = [&](int v) {
        const MvView& w = a.v[v];
        return MvIn{w.radii[ci], w.tiles_touched[ci], w.og[ci], in.shs ? (uint32_t)w.clamped[ci] : 0u};
    };
    MvIn cur = load_in(0);
    for (int v = 0; v < a.B; ++v) {  // uniform: the view's fields are scalar loads
        const MvView& w = a.v[v];
        const MvIn nxt = v + 1 < a.B ? load_in(v + 1) : cur;
        float* drgb_v = shx && live ? shx + (size_t)v * chunk + i3 : nullptr;
        const bool vis_v = live && cur.rad > 0;
        float q[12];
        const float2 og_v = cur.og;
        const uint32_t cbits_v = cur.cb;
        const uint32_t tt_v = cur.tt;
        cur = nxt;
        wave_gather(w.contrib, w.written, __float_as_uint(og_v.y) + w.bbase[ci / SLOT_BLOCK], vis_v ? tt_v : 0u, q,
                    s_gl[threadIdx.x >> 6]);
        if (!vis_v) {
            if (live && w.dmeans2D) { w.dmeans2D[i3] = 0.f; w.dmeans2D[i3 + 1] = 0.f; w.dmeans2D[i3 + 2] = 0.f; }
            if (drgb_v) { drgb_v[0] = 0.f; drgb_v[1] = 0.f; drgb_v[2] = 0.f; }
            continue;
        }
        const float op = og_v.x;
        const float dm2x = -op * q[7] * (0.5f * w.W);  // q[7] = sum q (a dx + b dy)
        const float dm2y = -op * q[8] * (0.5f * w.H);  // q[8] = sum q (b dx + c dy)
        if (w.dmeans2D) { w.dmeans2D[i3] = dm2x; w.dmeans2D[i3 + 1] = dm2y; w.dmeans2D[i3 + 2] = 0.f; }
        dcol = dcol + f3{q[0], q[1], q[2]};
        dop += q[6];
        dseg0 += q[3];
        dseg1 += q[4];
        f3 dRGB = {0.f, 0.f, 0.f};  // the clamped colour gradient (backward.cu:72-74)
        if (in.shs) {
            const uint32_t cbits = cbits_v;
            dRGB = {(cbits & 1) ? 0.f : q[0], (cbits & 2) ? 0.f : q[1], (cbits & 4) ? 0.f : q[2]};
        }
        if (drgb_v) {
            drgb_v[0] = dRGB.x;
            drgb_v[1] = dRGB.y;
            drgb_v[2] = dRGB.z;
        }
        const float* view = w.view;
        const float* proj = w.proj;
        const float focal_y = w.H / (2.0f * w.tanfovy);
        const float focal_x = w.W / (2.0f * w.tanfovx);
        // ---- computeCov2DCUDA (backward.cu:155-273) for this view
        const float dcx = -0.5f * op * q[9], dcy = -0.5f * op * q[10], dcz = -0.5f * op * q[11];
        const EwaTerms e = ewa_terms(mean, focal_x, focal_y, w.tanfovx, w.tanfovy, view);
        const float x_grad_mul = e.txtz < -e.limx || e.txtz > e.limx ? 0 : 1;
        const float y_grad_mul = e.tytz < -e.limy || e.tytz > e.limy ? 0 : 1;
        const M3& T = e.T;
        const M3 cov2D = mmul(mmul(mtr(T), mtr(Vrk)), T);
        const float a_ = cov2D.m[0][0] + 0.3f;
        const float b_ = cov2D.m[0][1];
        const float c_ = cov2D.m[1][1] + 0.3f;
        const float denom = a_ * c_ - b_ * b_;
        float dL_da = 0, dL_db = 0, dL_dc = 0;
        const float denom2inv = 1.0f / ((denom * denom) + 0.0000001f);
        const auto& Tt = T.m;
        if (denom2inv != 0) {
            dL_da = denom2inv * (-c_ * c_ * dcx + 2 * b_ * c_ * dcy + (denom - a_ * c_) * dcz);
            dL_dc = denom2inv * (-a_ * a_ * dcz + 2 * a_ * b_ * dcy + (denom - a_ * c_) * dcx);
            dL_db = denom2inv * 2 * (b_ * c_ * dcx - (denom + 2 * b_ * b_) * dcy + a_ * b_ * dcz);
            dcv_sum[0] += (Tt[0][0] * Tt[0][0] * dL_da + Tt[0][0] * Tt[1][0] * dL_db + Tt[1][0] * Tt[1][0] * dL_dc);
            dcv_sum[3] += (Tt[0][1] * Tt[0][1] * dL_da + Tt[0][1] * Tt[1][1] * dL_db + Tt[1][1] * Tt[1][1] * dL_dc);
            dcv_sum[5] += (Tt[0][2] * Tt[0][2] * dL_da + Tt[0][2] * Tt[1][2] * dL_db + Tt[1][2] * Tt[1][2] * dL_dc);
            dcv_sum[1] += 2 * Tt[0][0] * Tt[0][1] * dL_da + (Tt[0][0] * Tt[1][1] + Tt[0][1] * Tt[1][0]) * dL_db +
                          2 * Tt[1][0] * Tt[1][1] * dL_dc;
            dcv_sum[2] += 2 * Tt[0][0] * Tt[0][2] * dL_da + (Tt[0][0] * Tt[1][2] + Tt[0][2] * Tt[1][0]) * dL_db +
                          2 * Tt[1][0] * Tt[1][2] * dL_dc;
            dcv_sum[4] += 2 * Tt[0][2] * Tt[0][1] * dL_da + (Tt[0][1] * Tt[1][2] + Tt[0][2] * Tt[1][1]) * dL_db +
                          2 * Tt[1][1] * Tt[1][2] * dL_dc;
        }
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
        const auto& Wt = e.W.m;
        const float dL_dJ00 = Wt[0][0] * dL_dT00 + Wt[0][1] * dL_dT01 + Wt[0][2] * dL_dT02;
        const float dL_dJ02 = Wt[2][0] * dL_dT00 + Wt[2][1] * dL_dT01 + Wt[2][2] * dL_dT02;
        const float dL_dJ11 = Wt[1][0] * dL_dT10 + Wt[1][1] * dL_dT11 + Wt[1][2] * dL_dT12;
        const float dL_dJ12 = Wt[2][0] * dL_dT10 + Wt[2][1] * dL_dT11 + Wt[2][2] * dL_dT12;
        const float hx = focal_x, hy = focal_y;
        const f3 t = e.t;
        const float tz = 1.f / t.z, tz2 = tz * tz, tz3 = tz2 * tz;
        const float dL_dtx = x_grad_mul * -hx * tz2 * dL_dJ02;
        const float dL_dty = y_grad_mul * -hy * tz2 * dL_dJ12;
        const float dL_dtz = -hx * tz2 * dL_dJ00 - hy * tz2 * dL_dJ11 + (2 * hx * t.x) * tz3 * dL_dJ02 +
                             (2 * hy * t.y) * tz3 * dL_dJ12;
        f3 dmean = xformVecT({dL_dtx, dL_dty, dL_dtz}, view);
        // ---- preprocessCUDA backward (backward.cu:372-403) for this view
        const f3 m = mean;
        const float4 m_hom = xform4x4(m, proj);
        const float m_w = 1.0f / (m_hom.w + 0.0000001f);
        const float mul1 = (proj[0] * m.x + proj[4] * m.y + proj[8] * m.z + proj[12]) * m_w * m_w;
        const float mul2 = (proj[1] * m.x + proj[5] * m.y + proj[9] * m.z + proj[13]) * m_w * m_w;
        f3 dm;
        dm.x = (proj[0] * m_w - proj[3] * mul1) * dm2x + (proj[1] * m_w - proj[3] * mul2) * dm2y;
        dm.y = (proj[4] * m_w - proj[7] * mul1) * dm2x + (proj[5] * m_w - proj[7] * mul2) * dm2y;
        dm.z = (proj[8] * m_w - proj[11] * mul1) * dm2x + (proj[9] * m_w - proj[11] * mul2) * dm2y;
        dmean = dmean + dm;
        const float ddepth = q[5];
        const float mul3 = view[2] * m.x + view[6] * m.y + view[10] * m.z + view[14];
        f3 dmz;
        dmz.x = (view[2] - view[3] * mul3) * ddepth;
        dmz.y = (view[6] - view[7] * mul3) * ddepth;
        dmz.z = (view[10] - view[11] * mul3) * ddepth;
        dmean = dmean + dmz;
        if (in.shs && D > 0) {
            // the SH direction term of this view (backward.cu:109-111 + dnormvdv), from the
            // Jacobian its forward stored: the same arithmetic as k_gaussian_backward
            const float* J = jac_row(w.shjac, idx);
            const f3 jx = {J[0], J[64], J[128]}, jy = {J[192], J[256], J[320]}, jz = {J[384], J[448], J[512]};
            const f3 cam = {w.campos[0], w.campos[1], w.campos[2]};
            const f3 v = m - cam;
            const f3 dv = {dot3(jx, dRGB), dot3(jy, dRGB), dot3(jz, dRGB)};
            const float sum2 = v.x * v.x + v.y * v.y + v.z * v.z;
            const float invsum32 = 1.0f / sqrtf(sum2 * sum2 * sum2);
            f3 dn;
            dn.x = ((+sum2 - v.x * v.x) * dv.x - v.y * v.x * dv.y - v.z * v.x * dv.z) * invsum32;
            dn.y = (-v.x * v.y * dv.x + (sum2 - v.y * v.y) * dv.y - v.z * v.y * dv.z) * invsum32;
            dn.z = (-v.x * v.z * dv.x - v.y * v.z * dv.y + (sum2 - v.z * v.z) * dv.z) * invsum32;
            dmean = dmean + dn;
        }
        dmean_sum = dmean_sum + dmean;
    }
    if (!live) return;
    if (g.dcolors) { g.dcolors[i3] = dcol.x; g.dcolors[i3 + 1] = dcol.y; g.dcolors[i3 + 2] = dcol.z; }
    if (g.dopacity) g.dopacity[idx] = dop;
    if (g.dsegments) { g.dsegments[2 * (size_t)idx] = dseg0; g.dsegments[2 * (size_t)idx + 1] = dseg1; }
    if (g.dcov3D)
#pragma unroll
        for (int i = 0; i < 6; ++i) g.dcov3D[6 * (size_t)idx + i] = dcv_sum[i];
    if (g.dmeans3D) {
        g.dmeans3D[i3] = dmean_sum.x;
        g.dmeans3D[i3 + 1] = dmean_sum.y;
        g.dmeans3D[i3 + 2] = dmean_sum.z;
    }
    if (in.scales) {
        // computeCov3D backward (backward.cu:276-341) of the summed dcov3D (linear in it)
        const float* dcv = dcv_sum;
        const float r = quat.x, x = quat.y, y = quat.z, z = quat.w;
        const M3 R = mat3(1.f - 2.f * (y * y + z * z), 2.f * (x * y - r * z), 2.f * (x * z + r * y),
                          2.f * (x * y + r * z), 1.f - 2.f * (x * x + z * z), 2.f * (y * z - r * x),
                          2.f * (x * z - r * y), 2.f * (y * z + r * x), 1.f - 2.f * (x * x + y * y));
        M3 S = mat3(1, 0, 0, 0, 1, 0, 0, 0, 1);
        const f3 sv = scale_modifier * scale;
        S.m[0][0] = sv.x;
        S.m[1][1] = sv.y;
        S.m[2][2] = sv.z;
        const M3 Mm = mmul(S, R);
        const M3 dSig = mat3(dcv[0], 0.5f * dcv[1], 0.5f * dcv[2], 0.5f * dcv[1], dcv[3], 0.5f * dcv[4],
                             0.5f * dcv[2], 0.5f * dcv[4], dcv[5]);
        M3 M2;
#pragma unroll
        for (int cc = 0; cc < 3; ++cc)
#pragma unroll
            for (int rr = 0; rr < 3; ++rr) M2.m[cc][rr] = 2.0f * Mm.m[cc][rr];
        const M3 dM = mmul(M2, dSig);
        const M3 Rt = mtr(R);
        M3 dMt = mtr(dM);
        if (g.dscales) {
            g.dscales[i3 + 0] = Rt.m[0][0] * dMt.m[0][0] + Rt.m[0][1] * dMt.m[0][1] + Rt.m[0][2] * dMt.m[0][2];
            g.dscales[i3 + 1] = Rt.m[1][0] * dMt.m[1][0] + Rt.m[1][1] * dMt.m[1][1] + Rt.m[1][2] * dMt.m[1][2];
            g.dscales[i3 + 2] = Rt.m[2][0] * dMt.m[2][0] + Rt.m[2][1] * dMt.m[2][1] + Rt.m[2][2] * dMt.m[2][2];
        }
#pragma unroll
        for (int rr = 0; rr < 3; ++rr) {
            dMt.m[0][rr] *= sv.x;
            dMt.m[1][rr] *= sv.y;
            dMt.m[2][rr] *= sv.z;
        }
        const auto& d = dMt.m;
        if (g.drot) {
            float* dr = g.drot + 4 * (size_t)idx;
            dr[0] = 2 * z * (d[0][1] - d[1][0]) + 2 * y * (d[2][0] - d[0][2]) + 2 * x * (d[1][2] - d[2][1]);
            dr[1] = 2 * y * (d[1][0] + d[0][1]) + 2 * z * (d[2][0] + d[0][2]) + 2 * r * (d[1][2] - d[2][1]) -
                    4 * x * (d[2][2] + d[1][1]);
            dr[2] = 2 * x * (d[1][0] + d[0][1]) + 2 * r * (d[2][0] - d[0][2]) + 2 * z * (d[1][2] + d[2][1]) -
                    4 * y * (d[2][2] + d[0][0]);
            dr[3] = 2 * r * (d[0][1] - d[1][0]) + 2 * x * (d[2][0] + d[0][2]) + 2 * y * (d[1][2] + d[2][1]) -
                    4 * z * (d[1][1] + d[0][0]);
        }
    }
}

// dsh of the multi-view backward / the SH exchange: dsh[i] = sum over the views of
// basis_v x dRGB_v (backward.cu:46-110, the views in order, so every rank of an exchange
// computes the same bits; one view: the same products k_gaussian_backward stores).
// STAGED: M == 16 with 16-B aligned rows, the wave's 64 output rows go through LDS
// (coalesced 12-KB runs); otherwise a thread writes its own row.
template <bool STAGED>
__global__ void __launch_bounds__(256) k_sh_dsh(int P, int D, int M, const float* __restrict__ means3D, int V,
                                                const float* __restrict__ shx, float* __restrict__ dsh) {
    const size_t chunk = sh_rows_floats(P);
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int wbase = blockIdx.x * blockDim.x + wave * 64;
    const int idx = wbase + lane;
    const bool live = idx < P;
    if (!STAGED && !live) return;
    float acc[48];
#pragma unroll
    for (int i = 0; i < 48; ++i) acc[i] = 0.f;
    const f3 mean = live ? ld3(means3D + 3 * (size_t)idx) : f3{0.f, 0.f, 0.f};
    for (int v = 0; v < V; ++v) {  // views in order: every rank of an exchange sums identically
        const float* r = shx + (size_t)v * chunk;
        const f3 dRGB = live ? ld3(r + 3 * (size_t)idx) : f3{0.f, 0.f, 0.f};
        if (dRGB.x == 0.f && dRGB.y == 0.f && dRGB.z == 0.f) continue;  // invisible in this view (or a zero gradient)
        const f3 dir_orig = mean - ld3(r + sh_rows_campos(P));
        const f3 dir = dir_orig / sqrtf(dot3(dir_orig, dir_orig));
        float bas[16];
        sh_basis(D, dir, bas);
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            acc[3 * i] += bas[i] * dRGB.x;
            acc[3 * i + 1] += bas[i] * dRGB.y;
            acc[3 * i + 2] += bas[i] * dRGB.z;
        }
    }
    if (STAGED) {
        // as k_gaussian_backward's dsh: per pass, 16 lanes park their rows (52-float pitch,
        // conflict-free ds_write_b128) and the wave stores those 16 rows = 3 KB as 192
        // consecutive float4s
        __shared__ float4 srow[4][16][13];
#pragma unroll
        for (int p = 0; p < 4; ++p) {
            if ((lane >> 4) == p) {
                float4* row = srow[wave][lane & 15];
#pragma unroll
                for (int i = 0; i < 12; ++i)
                    row[i] = make_float4(acc[4 * i], acc[4 * i + 1], acc[4 * i + 2], acc[4 * i + 3]);
            }
            GSR_WAVE_SYNC();
            const int g0 = wbase + 16 * p;
            float4* dst = reinterpret_cast<float4*>(dsh + (size_t)g0 * 48);
#pragma unroll
            for (int r = 0; r < 3; ++r) {
                const int f = lane + 64 * r;
                const int row = f / 12, col = f - 12 * (f / 12);
                if (g0 + row < P) sh_st(dst + f, srow[wave][row][col]);
            }
            GSR_WAVE_SYNC();
        }
    } else {
        float* o = dsh + (size_t)idx * M * 3;
        for (int f = 0; f < 3 * M; ++f) o[f] = f < 48 ? acc[f] : 0.f;
    }
}
#endif  // GSR_PRE_PART == 1
}  // namespace

#if GSR_PRE_PART == 1
void launch_preprocess(const gsr_settings& s, const gsr_inputs& in, int gx, int gy, float4* rec, int* radii,
                       uint32_t* tiles_touched, uint32_t* depth_keys, uint8_t* clamped, ushort4* rect,
                       uint32_t* rect32, float* shjac, float2* og, uint32_t* btot, void* zero_a,
                       size_t zero_a_bytes, void* zero_b, size_t zero_b_bytes, hipStream_t st) {
    if (s.P == 0) return;
    hipLaunchKernelGGL(k_preprocess, dim3(cdiv(s.P, SLOT_BLOCK)), dim3(SLOT_BLOCK), 0, st, s, in, gx, gy, rec, radii,
                       tiles_touched, depth_keys, clamped, rect, rect32, shjac, og, btot, zero_a,
                       cdiv(zero_a_bytes, 16), zero_b, cdiv(zero_b_bytes, 16));
}

void launch_mark_visible(int P, const float* means3D, const float* view, uint8_t* present, hipStream_t st) {
    if (P == 0) return;
    hipLaunchKernelGGL(k_mark_visible, dim3(cdiv(P, 256)), dim3(256), 0, st, P, means3D, view, present);
}

void launch_gaussian_backward_multiview(int P, int D, int M, float scale_modifier, const gsr_inputs& in,
                                        const MvArgs& a, const gsr_grads& g, float* shx, bool defer_sh,
                                        hipStream_t st) {
    if (P == 0) return;
    float* shx_used = (in.shs && (defer_sh || g.dsh)) ? shx : nullptr;
    hipLaunchKernelGGL(k_gaussian_backward_mv, dim3(cdiv(P, 256)), dim3(256),
                       0, st, P, D, M, scale_modifier, in, a, g, shx_used);
    if (!shx_used || defer_sh) return;
    launch_sh_backward(P, D, M, in.means3D, a.B, shx_used, g.dsh, st);
}

void launch_sh_backward(int P, int D, int M, const float* means3D, int V, const float* shx, float* dsh,
                        hipStream_t st) {
    if (P == 0 || V == 0 || !dsh) return;
    const bool staged = M == 16 && (reinterpret_cast<uintptr_t>(dsh) & 15) == 0;
    if (staged)
        hipLaunchKernelGGL(k_sh_dsh<true>, dim3(cdiv(P, 256)), dim3(256), 0, st, P, D, M, means3D, V, shx, dsh);
    else
        hipLaunchKernelGGL(k_sh_dsh<false>, dim3(cdiv(P, 256)), dim3(256), 0, st, P, D, M, means3D, V, shx, dsh);
}
#endif  // GSR_PRE_PART == 1

#if GSR_PRE_PART == 2
void launch_gaussian_backward(const gsr_settings& s, const gsr_inputs& in, const int* radii,
                              const uint32_t* tiles_touched, const float2* og, const uint32_t* bbase,
                              const uint8_t* clamped, const float* contrib, const uint8_t* written,
                              const float* shjac, const gsr_grads& g, float* shx, hipStream_t st) {
    if (s.P == 0) return;
    hipLaunchKernelGGL(k_gaussian_backward, dim3(cdiv(s.P, 256)), dim3(256), 0, st, s, in, radii, tiles_touched,
                       og, bbase, clamped, contrib, written, shjac, g, in.shs ? shx : nullptr);
}

#endif  // GSR_PRE_PART == 2

}  // namespace gsr
