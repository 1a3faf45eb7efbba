// knn_oracle.cpp -- CPU restatement of distCUDA2 (simple-knn), TEST INFRASTRUCTURE
// ONLY (tests/, bench.py's cpu_baseline); never linked into the product.
//
// Follows submodules_local/simple-knn/simple_knn.cu step by step:
//   bounds      cub Reduce with init {0,0,0} (:188-199): min/max include the origin
//   morton      10-bit quantisation per axis, bit-interleaved x|y<<1|z<<2 (:48-71)
//   sort        stable radix sort of (code, index) (:209-212) -> std::stable_sort
//   boxes       AABBs of 1024 consecutive sorted points (:80-116, BOX_SIZE :12)
//   query       3 best of the +-3 sorted neighbours give `reject`; then every box
//               whose point-box distance is <= reject and <= the running 3rd best
//               is scanned in box order (:142-178); result = mean of the 3 best
//               squared distances, written at the original index.
// The three smallest squared distances are those of the exact 3 nearest
// neighbours (the pruning only skips boxes that cannot hold one), which the tests
// also check against a brute-force search.  -ffp-contract=off: each squared
// distance is d.x*d.x + d.y*d.y + d.z*d.z with separate roundings.
#include <stdint.h>
#include <algorithm>
#include <cfloat>
#include <cmath>
#include <numeric>
#include <vector>

#ifdef _OPENMP
#include <omp.h>
#endif

namespace {
constexpr int BOX = 1024;

struct F3 { float x, y, z; };

uint32_t spread10(uint32_t x) {
    x = (x | (x << 16)) & 0x030000FF;
    x = (x | (x << 8)) & 0x0300F00F;
    x = (x | (x << 4)) & 0x030C30C3;
    x = (x | (x << 2)) & 0x09249249;
    return x;
}

uint32_t to_u32(float v) {  // the reference's implicit float -> uint32_t conversion (values are in [0, 1023])
    if (!(v > 0.0f)) return 0u;
    return (uint32_t)v;
}

float sq(F3 a, F3 b) {
    const float dx = b.x - a.x, dy = b.y - a.y, dz = b.z - a.z;
    return dx * dx + dy * dy + dz * dz;
}

void update3(F3 ref, F3 p, float* best) {
    float d = sq(ref, p);
    for (int j = 0; j < 3; ++j) {
        if (best[j] > d) {
            const float t = best[j];
            best[j] = d;
            d = t;
        }
    }
}

struct Box { F3 mn, mx; };

float box_dist(const Box& b, F3 p) {
    float dx = 0, dy = 0, dz = 0;
    if (p.x < b.mn.x || p.x > b.mx.x) dx = std::min(std::fabs(p.x - b.mn.x), std::fabs(p.x - b.mx.x));
    if (p.y < b.mn.y || p.y > b.mx.y) dy = std::min(std::fabs(p.y - b.mn.y), std::fabs(p.y - b.mx.y));
    if (p.z < b.mn.z || p.z > b.mx.z) dz = std::min(std::fabs(p.z - b.mn.z), std::fabs(p.z - b.mx.z));
    return dx * dx + dy * dy + dz * dz;
}
}  // namespace

extern "C" {

// points: [P,3] float32; out: [P] mean squared distance to the 3 nearest neighbours.
void oracle_dist_knn3(int P, const float* points, float* out) {
    if (P <= 0) return;
    const F3* pts = reinterpret_cast<const F3*>(points);
    F3 mn{0, 0, 0}, mx{0, 0, 0};
    for (int i = 0; i < P; ++i) {
        mn.x = std::min(mn.x, pts[i].x); mn.y = std::min(mn.y, pts[i].y); mn.z = std::min(mn.z, pts[i].z);
        mx.x = std::max(mx.x, pts[i].x); mx.y = std::max(mx.y, pts[i].y); mx.z = std::max(mx.z, pts[i].z);
    }
    std::vector<uint32_t> code(P);
    for (int i = 0; i < P; ++i) {
        const uint32_t x = spread10(to_u32(((pts[i].x - mn.x) / (mx.x - mn.x)) * 1023.0f));
        const uint32_t y = spread10(to_u32(((pts[i].y - mn.y) / (mx.y - mn.y)) * 1023.0f));
        const uint32_t z = spread10(to_u32(((pts[i].z - mn.z) / (mx.z - mn.z)) * 1023.0f));
        code[i] = x | (y << 1) | (z << 2);
    }
    std::vector<uint32_t> idx(P);
    std::iota(idx.begin(), idx.end(), 0u);
    std::stable_sort(idx.begin(), idx.end(), [&](uint32_t a, uint32_t b) { return code[a] < code[b]; });
    const int nb = (P + BOX - 1) / BOX;
    std::vector<Box> boxes(nb);
    for (int b = 0; b < nb; ++b) {
        Box bx{{FLT_MAX, FLT_MAX, FLT_MAX}, {-FLT_MAX, -FLT_MAX, -FLT_MAX}};
        for (int i = b * BOX; i < std::min(P, (b + 1) * BOX); ++i) {
            const F3 p = pts[idx[i]];
            bx.mn.x = std::min(bx.mn.x, p.x); bx.mn.y = std::min(bx.mn.y, p.y); bx.mn.z = std::min(bx.mn.z, p.z);
            bx.mx.x = std::max(bx.mx.x, p.x); bx.mx.y = std::max(bx.mx.y, p.y); bx.mx.z = std::max(bx.mx.z, p.z);
        }
        boxes[b] = bx;
    }
#pragma omp parallel for schedule(dynamic, 256)
    for (int s = 0; s < P; ++s) {
        const F3 p = pts[idx[s]];
        float best[3] = {FLT_MAX, FLT_MAX, FLT_MAX};
        for (int i = std::max(0, s - 3); i <= std::min(P - 1, s + 3); ++i)
            if (i != s) update3(p, pts[idx[i]], best);
        const float reject = best[2];
        best[0] = best[1] = best[2] = FLT_MAX;
        for (int b = 0; b < nb; ++b) {
            const float d = box_dist(boxes[b], p);
            if (d > reject || d > best[2]) continue;
            for (int i = b * BOX; i < std::min(P, (b + 1) * BOX); ++i)
                if (i != s) update3(p, pts[idx[i]], best);
        }
        out[idx[s]] = (best[0] + best[1] + best[2]) / 3.0f;
    }
}

}  // extern "C"
