// knn.hip -- distCUDA2 (submodules_local/simple-knn/simple_knn.cu:181-220): the mean
// squared distance of every point to its 3 nearest neighbours, used once to
// initialise the Gaussian scales (scene/gaussian_model.py:143).
//
// Same spatial ordering as the reference (origin-including bounds, 10-bit Morton
// codes, stable radix sort -- here the library's LDS radix sort), but the search
// is organised for CDNA:
//   * boxes are 256 consecutive sorted points, one workgroup (4 wave64) per box,
//     one thread per query point;
//   * a candidate box's points are staged once into LDS and read by every thread of
//     the workgroup that still needs that box (ds_read broadcast), instead of each
//     thread re-reading them from L2;
//   * the own box is scanned first (a tight 3rd-best bound), then groups of 64
//     boxes ("super boxes") outward in Morton order; a super box, and then each of
//     its boxes, is rejected for the whole workgroup when its AABB is farther from
//     the workgroup's AABB than the largest current 3rd best (exact: such a box
//     cannot hold a neighbour of any of its queries), and per thread by the
//     point-box distance, with a workgroup vote so the LDS stage is skipped when
//     no thread needs the box.  Work is ~linear in P instead of the reference's
//     every-point-tests-every-box scan.
// The result is the exact 3-NN mean like the reference's; squared distances are
// d.x*d.x + d.y*d.y + d.z*d.z in fp32.
#include <float.h>

#include <algorithm>

#include "gsr_internal.h"
#include "../../include/gsr_train.h"

namespace gsr {
namespace {

constexpr int KNN_BOX = 256;
constexpr int KNN_THREADS = 256;
constexpr int KNN_BOUND_BLOCKS = 256;
constexpr int KNN_SUPER = 64;  // boxes per super box (level-2 culling)

__device__ __forceinline__ uint32_t spread10(uint32_t x) {
    x = (x | (x << 16)) & 0x030000FFu;
    x = (x | (x << 8)) & 0x0300F00Fu;
    x = (x | (x << 4)) & 0x030C30C3u;
    x = (x | (x << 2)) & 0x09249249u;
    return x;
}

// Per-block min/max of the points (x, y, z), then one block folds them with the
// reference's {0,0,0} reduction init.
__global__ void __launch_bounds__(KNN_THREADS) k_knn_bounds(int P, const float* __restrict__ pts,
                                                            float* __restrict__ partial) {
    float mn[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, mx[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
    for (int i = blockIdx.x * KNN_THREADS + threadIdx.x; i < P; i += gridDim.x * KNN_THREADS) {
        for (int k = 0; k < 3; ++k) {
            const float v = pts[3LL * i + k];
            mn[k] = fminf(mn[k], v);
            mx[k] = fmaxf(mx[k], v);
        }
    }
    __shared__ float s[6][KNN_THREADS];
    for (int k = 0; k < 3; ++k) {
        s[k][threadIdx.x] = mn[k];
        s[3 + k][threadIdx.x] = mx[k];
    }
    __syncthreads();
    for (int off = KNN_THREADS / 2; off > 0; off >>= 1) {
        if ((int)threadIdx.x < off) {
            for (int k = 0; k < 3; ++k) {
                s[k][threadIdx.x] = fminf(s[k][threadIdx.x], s[k][threadIdx.x + off]);
                s[3 + k][threadIdx.x] = fmaxf(s[3 + k][threadIdx.x], s[3 + k][threadIdx.x + off]);
            }
        }
        __syncthreads();
    }
    if (threadIdx.x < 6) partial[blockIdx.x * 8 + threadIdx.x] = s[threadIdx.x][0];
}

__global__ void k_knn_morton(int P, int nparts, const float* __restrict__ pts, const float* __restrict__ partial,
                             uint32_t* __restrict__ codes) {
    float mn[3] = {0.0f, 0.0f, 0.0f}, mx[3] = {0.0f, 0.0f, 0.0f};  // cub Reduce init {0,0,0}
    for (int b = 0; b < nparts; ++b) {  // uniform: scalar loads
        for (int k = 0; k < 3; ++k) {
            mn[k] = fminf(mn[k], partial[b * 8 + k]);
            mx[k] = fmaxf(mx[k], partial[b * 8 + 3 + k]);
        }
    }
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= P) return;
    uint32_t c = 0;
    for (int k = 0; k < 3; ++k) {
        const float q = ((pts[3LL * i + k] - mn[k]) / (mx[k] - mn[k])) * 1023.0f;
        const uint32_t u = q > 0.0f ? (uint32_t)q : 0u;  // float -> uint32 as the reference converts
        c |= spread10(u) << k;
    }
    codes[i] = c;
}

__global__ void k_knn_gather(int P, const float* __restrict__ pts, const uint32_t* __restrict__ order,
                             float4* __restrict__ sp) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= P) return;
    const uint32_t j = order[i];
    sp[i] = make_float4(pts[3LL * j], pts[3LL * j + 1], pts[3LL * j + 2], 0.0f);
}

__global__ void __launch_bounds__(KNN_THREADS) k_knn_boxes(int P, const float4* __restrict__ sp,
                                                           float4* __restrict__ boxes) {
    const int i = blockIdx.x * KNN_BOX + threadIdx.x;
    float4 p = i < P ? sp[i] : sp[blockIdx.x * KNN_BOX];
    __shared__ float s[6][KNN_THREADS];
    s[0][threadIdx.x] = p.x; s[1][threadIdx.x] = p.y; s[2][threadIdx.x] = p.z;
    s[3][threadIdx.x] = p.x; s[4][threadIdx.x] = p.y; s[5][threadIdx.x] = p.z;
    __syncthreads();
    for (int off = KNN_THREADS / 2; off > 0; off >>= 1) {
        if ((int)threadIdx.x < off) {
            for (int k = 0; k < 3; ++k) {
                s[k][threadIdx.x] = fminf(s[k][threadIdx.x], s[k][threadIdx.x + off]);
                s[3 + k][threadIdx.x] = fmaxf(s[3 + k][threadIdx.x], s[3 + k][threadIdx.x + off]);
            }
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        boxes[2 * blockIdx.x] = make_float4(s[0][0], s[1][0], s[2][0], 0.0f);
        boxes[2 * blockIdx.x + 1] = make_float4(s[3][0], s[4][0], s[5][0], 0.0f);
    }
}

__device__ __forceinline__ float box_dist(float4 mn, float4 mx, float4 p) {
    float dx = 0.0f, dy = 0.0f, dz = 0.0f;
    if (p.x < mn.x || p.x > mx.x) dx = fminf(fabsf(p.x - mn.x), fabsf(p.x - mx.x));
    if (p.y < mn.y || p.y > mx.y) dy = fminf(fabsf(p.y - mn.y), fabsf(p.y - mx.y));
    if (p.z < mn.z || p.z > mx.z) dz = fminf(fabsf(p.z - mn.z), fabsf(p.z - mx.z));
    return dx * dx + dy * dy + dz * dz;
}

__device__ __forceinline__ void update3(float4 q, float4 p, float& b0, float& b1, float& b2) {
    const float dx = p.x - q.x, dy = p.y - q.y, dz = p.z - q.z;
    float d = dx * dx + dy * dy + dz * dz;
    // keep the 3 smallest (same insertion as the reference's updateKBest)
    if (b0 > d) { const float t = b0; b0 = d; d = t; }
    if (b1 > d) { const float t = b1; b1 = d; d = t; }
    if (b2 > d) b2 = d;
}

// Squared distance between two AABBs (0 if they overlap).
__device__ __forceinline__ float box_box_dist(float4 amn, float4 amx, float4 bmn, float4 bmx) {
    const float dx = fmaxf(0.0f, fmaxf(amn.x - bmx.x, bmn.x - amx.x));
    const float dy = fmaxf(0.0f, fmaxf(amn.y - bmx.y, bmn.y - amx.y));
    const float dz = fmaxf(0.0f, fmaxf(amn.z - bmx.z, bmn.z - amx.z));
    return dx * dx + dy * dy + dz * dz;
}

__device__ __forceinline__ float wave_max(float v) {
    for (int off = 32; off > 0; off >>= 1) v = fmaxf(v, __shfl_xor(v, off, 64));
    return v;
}

// AABBs of KNN_SUPER consecutive boxes (one thread per super box).
__global__ void k_knn_super(int nbox, const float4* __restrict__ boxes, float4* __restrict__ sup) {
    const int sidx = blockIdx.x * blockDim.x + threadIdx.x;
    const int lo = sidx * KNN_SUPER;
    if (lo >= nbox) return;
    float4 mn = boxes[2 * lo], mx = boxes[2 * lo + 1];
    for (int c = lo + 1; c < min(nbox, lo + KNN_SUPER); ++c) {
        const float4 a = boxes[2 * c], z = boxes[2 * c + 1];
        mn = make_float4(fminf(mn.x, a.x), fminf(mn.y, a.y), fminf(mn.z, a.z), 0.0f);
        mx = make_float4(fmaxf(mx.x, z.x), fmaxf(mx.y, z.y), fmaxf(mx.z, z.z), 0.0f);
    }
    sup[2 * sidx] = mn;
    sup[2 * sidx + 1] = mx;
}

__global__ void __launch_bounds__(KNN_THREADS) k_knn_query(int P, int nbox, const float4* __restrict__ sp,
                                                           const float4* __restrict__ boxes,
                                                           const float4* __restrict__ sup,
                                                           const uint32_t* __restrict__ order,
                                                           float* __restrict__ out) {
    __shared__ float4 cand[KNN_BOX];
    __shared__ float wmax[KNN_THREADS / 64];
    const int b = blockIdx.x;
    const int i = b * KNN_BOX + threadIdx.x;
    const bool valid = i < P;
    const float4 q = valid ? sp[i] : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    const float4 qmn = boxes[2 * b], qmx = boxes[2 * b + 1];
    float b0 = FLT_MAX, b1 = FLT_MAX, b2 = FLT_MAX;
    float wg_thr = FLT_MAX;  // max over the workgroup's 3rd-best distances (uniform)

    // Scan box c (uniform call): stage it in LDS if any thread may find a neighbour.
    auto visit = [&](int c) {
        const float4 mn = boxes[2 * c], mx = boxes[2 * c + 1];
        // uniform rejection: no point of this box is nearer to any of our queries
        // than that query's current 3rd best
        if (box_box_dist(qmn, qmx, mn, mx) > wg_thr) return;
        const bool need = valid && box_dist(mn, mx, q) <= b2;
        if (!__syncthreads_or(need)) return;
        const int base = c * KNN_BOX;
        const int n = min(KNN_BOX, P - base);
        if ((int)threadIdx.x < n) cand[threadIdx.x] = sp[base + threadIdx.x];
        __syncthreads();
        if (need) {
            const int self = i - base;  // the query point itself is skipped by index
            for (int j = 0; j < n; ++j)
                if (j != self) update3(q, cand[j], b0, b1, b2);
        }
        const float m = wave_max(valid ? b2 : 0.0f);
        if ((threadIdx.x & 63) == 0) wmax[threadIdx.x >> 6] = m;
        __syncthreads();
        wg_thr = fmaxf(fmaxf(wmax[0], wmax[1]), fmaxf(wmax[2], wmax[3]));
        __syncthreads();
    };

    visit(b);  // own box first: a tight bound for everything after
    // then super boxes outward in Morton order, each rejected as a whole when possible
    const int nsup = (nbox + KNN_SUPER - 1) / KNN_SUPER, sb = b / KNN_SUPER;
    const int tmax = 2 * max(sb, nsup - 1 - sb) + 1;
    for (int t = 0; t < tmax; ++t) {  // uniform over the workgroup
        const int S = (t & 1) ? sb + ((t + 1) >> 1) : sb - (t >> 1);
        if (S < 0 || S >= nsup) continue;
        if (box_box_dist(qmn, qmx, sup[2 * S], sup[2 * S + 1]) > wg_thr) continue;
        const int lo = S * KNN_SUPER, hi = min(nbox, lo + KNN_SUPER);
        for (int c = lo; c < hi; ++c)
            if (c != b) visit(c);
    }
    if (valid) out[order[i]] = (b0 + b1 + b2) / 3.0f;
}

struct KnnWs {
    float* partial;
    uint32_t *codes, *codes_tmp, *codes_sorted, *idx_tmp, *order;
    float4 *sp, *boxes, *sup;
    void* sort;
};
size_t knn_ws_size(size_t P, KnnWs* w, char* base) {
    size_t o = 0;
    auto take = [&](size_t bytes) { char* p = base ? base + o : nullptr; o += align_up(bytes); return p; };
    const size_t nbox = cdiv(P, KNN_BOX);
    char* partial = take(KNN_BOUND_BLOCKS * 8 * 4);
    char* codes = take(P * 4);
    char* codes_tmp = take(P * 4);
    char* codes_sorted = take(P * 4);
    char* idx_tmp = take(P * 4);
    char* order = take(P * 4);
    char* sp = take(P * 16);
    char* boxes = take(nbox * 32);
    char* sup = take(cdiv(nbox, KNN_SUPER) * 32);
    char* sort = take(sort_ws_bytes(P, 4));
    if (w) {
        w->partial = (float*)partial;
        w->codes = (uint32_t*)codes;
        w->codes_tmp = (uint32_t*)codes_tmp;
        w->codes_sorted = (uint32_t*)codes_sorted;
        w->idx_tmp = (uint32_t*)idx_tmp;
        w->order = (uint32_t*)order;
        w->sp = (float4*)sp;
        w->boxes = (float4*)boxes;
        w->sup = (float4*)sup;
        w->sort = sort;
    }
    return o;
}

}  // namespace
}  // namespace gsr

using namespace gsr;

extern "C" {

GSR_API size_t gsr_knn_ws_bytes(int P) { return knn_ws_size(P > 0 ? (size_t)P : 1, nullptr, nullptr); }

GSR_API int gsr_dist_knn3(int P, const float* points, float* mean_dists, void* ws, void* stream) {
    if (P < 0) return set_error("[gsr] gsr_dist_knn3: P < 0");
    if (P == 0) return 0;
    if (!points || !mean_dists || !ws) return set_error("[gsr] gsr_dist_knn3: null buffer");
    hipStream_t st = (hipStream_t)stream;
    KnnWs w;
    knn_ws_size((size_t)P, &w, static_cast<char*>(ws));
    const int nbox = (int)cdiv((size_t)P, KNN_BOX);
    const int parts = (int)std::min<size_t>(KNN_BOUND_BLOCKS, cdiv((size_t)P, KNN_THREADS));
    k_knn_bounds<<<parts, KNN_THREADS, 0, st>>>(P, points, w.partial);
    const unsigned g = (unsigned)cdiv((size_t)P, 256);
    k_knn_morton<<<g, 256, 0, st>>>(P, parts, points, w.partial, w.codes);
    launch_radix_sort(w.codes, nullptr, w.codes_tmp, w.idx_tmp, w.codes_sorted, w.order, (size_t)P, 30, w.sort,
                      /*ws_zeroed=*/false, st);
    k_knn_gather<<<g, 256, 0, st>>>(P, points, w.order, w.sp);
    k_knn_boxes<<<nbox, KNN_THREADS, 0, st>>>(P, w.sp, w.boxes);
    const int nsup = (int)cdiv((size_t)nbox, KNN_SUPER);
    k_knn_super<<<(unsigned)cdiv((size_t)nsup, 64), 64, 0, st>>>(nbox, w.boxes, w.sup);
    k_knn_query<<<nbox, KNN_THREADS, 0, st>>>(P, nbox, w.sp, w.boxes, w.sup, w.order, mean_dists);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return set_error(std::string("[gsr] dist_knn3: ") + hipGetErrorString(e));
    return 0;
}

}  // extern "C"
