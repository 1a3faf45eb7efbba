// api.hip -- the C ABI of include/gsr.h: buffer carving and stage orchestration.
// Reference orchestration: DGR/cuda_rasterizer/rasterizer_impl.cu:198-458 and
// the host bindings DGR/rasterize_points.cu:35-242.
#include <stdio.h>
#include <stdlib.h>

#include <chrono>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

#include "gsr_internal.h"

namespace {
thread_local std::string g_last_error;

// ---- live stage timing (gsr_timing_*): hipEvents on the caller's stream.
constexpr int NUM_STAGES = 9;
const char* const STAGE_NAMES[NUM_STAGES] = {"preprocess", "depth_sort", "scan",       "duplicate",   "tile_sort",
                                             "ranges",     "render_fwd", "render_bwd", "gaussian_bwd"};
struct Timer {
    std::mutex mu;
    unsigned mask = 0;  // bit i: time stage i
    struct Rec { int stage; hipEvent_t a, b; };
    std::vector<Rec> pending;
    std::vector<hipEvent_t> pool;
    hipEvent_t get() {
        if (!pool.empty()) {
            hipEvent_t e = pool.back();
            pool.pop_back();
            return e;
        }
        // no system-scope fence on record: a fenced event costs ~10 us of pipeline
        // drain between the kernels it separates
        hipEvent_t e = nullptr;
        if (hipEventCreateWithFlags(&e, hipEventDisableSystemFence) != hipSuccess) e = nullptr;
        return e;
    }
};
Timer& timer() {
    static Timer t;
    return t;
}
struct StageScope {
    int stage;
    hipStream_t st;
    hipEvent_t a = nullptr;
    StageScope(int s, hipStream_t stream) : stage(s), st(stream) {
        Timer& T = timer();
        std::lock_guard<std::mutex> lk(T.mu);
        if (!((T.mask >> stage) & 1u)) return;
        a = T.get();
        if (a && hipEventRecord(a, st) != hipSuccess) {
            T.pool.push_back(a);
            a = nullptr;
        }
    }
    ~StageScope() {
        if (!a) return;
        Timer& T = timer();
        std::lock_guard<std::mutex> lk(T.mu);
        hipEvent_t b = T.get();
        if (!b || hipEventRecord(b, st) != hipSuccess) {
            T.pool.push_back(a);
            if (b) T.pool.push_back(b);
            return;
        }
        T.pending.push_back({stage, a, b});
    }
};

int fail(const std::string& msg) {
    g_last_error = msg;
    return 1;
}

// gsr.h gsr_backward contract guard: the colour source of each geom buffer's last forward.  The
// forward stores the SH direction Jacobian in geom only when it evaluated SH itself, so a
// backward given shs for a buffer whose forward took colors_precomp fails here instead of
// reading that field uninitialised.  Host-side bookkeeping only (no device read, no sync);
// a buffer the table does not hold (another process's, or evicted) is not checked.
struct GeomSource {
    int P;
    bool sh;
};
std::mutex g_src_mu;
std::unordered_map<const void*, GeomSource> g_src;
void note_source(const void* geom, int P, bool sh) {
    std::lock_guard<std::mutex> lk(g_src_mu);
    if (g_src.size() >= 4096) g_src.clear();
    g_src[geom] = GeomSource{P, sh};
}
int check_source(const void* geom, int P, bool sh) {
    std::lock_guard<std::mutex> lk(g_src_mu);
    const auto it = g_src.find(geom);
    if (it == g_src.end() || it->second.P != P || !sh || it->second.sh) return 0;
    return fail("[gsr] backward: shs given, but the forward of this geom buffer took colors_precomp (pass the "
                "forward's colour source; include/gsr.h gsr_backward)");
}

// Launch errors are checked after every stage; in debug mode the stream is also
// synchronised so that asynchronous faults are attributed to their stage
// (reference CHECK_CUDA, auxiliary.h:166-173).
int check(const char* stage, hipStream_t st, bool debug) {
    hipError_t e = hipGetLastError();
    if (e == hipSuccess && debug) e = hipStreamSynchronize(st);
    if (e != hipSuccess) return fail(std::string("[gsr] ") + stage + ": " + hipGetErrorString(e));
    return 0;
}

#define GSR_STAGE(name)                              \
    do {                                             \
        if (int rc_ = check(name, st, dbg)) return rc_; \
    } while (0)

template <typename T>
T* at(char* base, size_t off) {
    return reinterpret_cast<T*>(base + off);
}

int validate(const gsr_settings* s, const gsr_inputs* in, bool forward) {
    if (!s || !in) return fail("[gsr] null settings/inputs");
    if (s->P < 0 || s->W <= 0 || s->H <= 0) return fail("[gsr] invalid problem size");
    if (s->P == 0) return 0;
    if (!in->means3D || (forward && !in->opacities)) return fail("[gsr] means3D and opacities are required");
    if ((in->shs == nullptr) == (in->colors_precomp == nullptr))
        return fail("[gsr] Please provide excatly one of either SHs or precomputed colors!");
    const bool have_sr = in->scales && in->rotations;
    if (have_sr == (in->cov3D_precomp != nullptr) || ((in->scales == nullptr) != (in->rotations == nullptr)))
        return fail("[gsr] Please provide exactly one of either scale/rotation pair or precomputed 3D covariance!");
    if (in->shs && (s->D < 0 || s->D > 3 || s->M < (s->D + 1) * (s->D + 1)))
        return fail("[gsr] SH degree must be 0..3 with shs.shape[1] >= (degree+1)^2");
    if (!s->bg || !s->viewmatrix || !s->projmatrix || !s->campos) return fail("[gsr] missing camera tensors");
    if (((uintptr_t)in->rotations & 15) || ((uintptr_t)in->segments & 7))
        return fail("[gsr] rotations must be 16-byte and segments 8-byte aligned");
    if ((size_t)((s->W + gsr::BX - 1) / gsr::BX) > 65535 || (size_t)((s->H + gsr::BY - 1) / gsr::BY) > 65535)
        return fail("[gsr] image too large");
    return 0;
}

}  // namespace

namespace {

// num_rendered hand-off.  The scan writes the total into a host-mapped pinned word
// (one per host thread: calls from one thread are sequential, and this call waits for
// the value before returning); the host polls it, which returns as soon as the scan's
// last tile is done instead of after a copy kernel and a stream synchronisation.  If
// the stream drains without the value appearing (or pinned memory is unavailable) the
// total is copied the ordinary way.
constexpr uint32_t TOTAL_PENDING = 0xFFFFFFFFu;
// The word has ONE writer per call: the depth sort's histogram kernel when it runs (tally of
// tiles_touched, geometry_impl sets t_tallied), otherwise the offsets scan / level-1 binning.
thread_local bool t_tallied = false;
constexpr int TALLY_MAX_P = 1 << 17;
struct HostSlot {
    uint32_t* host = nullptr;  // CPU view
    uint32_t* dev = nullptr;   // GPU view of the same pinned word
};
// One word per call in flight: slot 0 for the calls that wait before returning, slots
// 1..HOST_SLOTS-1 for gsr_forward_deferred calls (a ticket each until gsr_forward_wait).  The
// calls of one host thread select their slot through t_slot.
constexpr int HOST_SLOTS = 1 + GSR_MAX_DEFERRED;
thread_local int t_slot = 0;
struct HostSlots {
    uint32_t* host = nullptr;
    uint32_t* dev = nullptr;
    bool busy[HOST_SLOTS] = {};
};
HostSlots& host_slots() {
    thread_local HostSlots hs;
    thread_local bool tried = false;
    if (!tried) {
        tried = true;
        const char* env = getenv("GSR_HOST_TOTAL");
        if (env && env[0] == '0') return hs;
        void* p = nullptr;
        void* d = nullptr;
        if (hipHostMalloc(&p, 64 * HOST_SLOTS, hipHostMallocMapped | hipHostMallocCoherent) == hipSuccess) {
            if (hipHostGetDevicePointer(&d, p, 0) == hipSuccess) {
                hs.host = (uint32_t*)p;
                hs.dev = (uint32_t*)d;
            } else {
                (void)hipHostFree(p);
            }
        }
    }
    return hs;
}
HostSlot host_total_slot() {  // the current call's word (64 B apart: one cache line each)
    HostSlots& hs = host_slots();
    if (!hs.host) return HostSlot{};
    return HostSlot{hs.host + 16 * t_slot, hs.dev + 16 * t_slot};
}
int wait_total(uint32_t* hslot, hipStream_t st, const uint32_t* dev_last, uint32_t* total) {
    if (hslot) {
        // hipStreamQuery enqueues a marker behind the work in flight, whose system-scope
        // release runs between the forward render and the backward launched after this wait
        // (a 6.8 us idle gap per step when the stream was queried every 256 spins): the
        // stream is queried only once the word is 5 ms late, then every millisecond.
        using clk = std::chrono::steady_clock;
        const clk::time_point t0 = clk::now();
        long next_ms = 5;
        for (unsigned spin = 0;; ++spin) {
            const uint32_t v = __atomic_load_n(hslot, __ATOMIC_ACQUIRE);
            if (v != TOTAL_PENDING) {
                *total = v;
                return 0;
            }
            if ((spin & 255u) == 255u &&
                std::chrono::duration_cast<std::chrono::milliseconds>(clk::now() - t0).count() >= next_ms) {
                ++next_ms;
                const hipError_t q = hipStreamQuery(st);
                if (q == hipSuccess) {  // drained: read once more, then fall back
                    const uint32_t w = __atomic_load_n(hslot, __ATOMIC_ACQUIRE);
                    if (w != TOTAL_PENDING) {
                        *total = w;
                        return 0;
                    }
                    break;
                }
                if (q != hipErrorNotReady) return fail(std::string("[gsr] num_rendered: ") + hipGetErrorString(q));
            }
        }
    }
    hipError_t e = hipMemcpyAsync(total, dev_last, sizeof(uint32_t), hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    if (e != hipSuccess) return fail(std::string("[gsr] num_rendered copy: ") + hipGetErrorString(e));
    return 0;
}

}  // namespace

namespace gsr {
int set_error(const std::string& msg) { return fail(msg); }
}  // namespace gsr


namespace gsr {
namespace {
// HBM streaming-copy reference for the roofline (bench.py): each thread moves U float4s,
// all loads issued before the stores, non-temporal on both sides.
template <int U>
__global__ void __launch_bounds__(256) k_stream_copy(const float4* __restrict__ src, float4* __restrict__ dst,
                                                     size_t n) {
    const size_t base = ((size_t)blockIdx.x * 256 * U) + threadIdx.x;
    float4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const size_t i = base + (size_t)u * 256;
        if (i < n) {
            const float* s = (const float*)(src + i);
            v[u] = make_float4(__builtin_nontemporal_load(s), __builtin_nontemporal_load(s + 1),
                               __builtin_nontemporal_load(s + 2), __builtin_nontemporal_load(s + 3));
        }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const size_t i = base + (size_t)u * 256;
        if (i < n) {
            float* d = (float*)(dst + i);
            __builtin_nontemporal_store(v[u].x, d);
            __builtin_nontemporal_store(v[u].y, d + 1);
            __builtin_nontemporal_store(v[u].z, d + 2);
            __builtin_nontemporal_store(v[u].w, d + 3);
        }
    }
}
}  // namespace
}  // namespace gsr

extern "C" {

const char* gsr_last_error(void) { return g_last_error.c_str(); }

const char* gsr_version(void) { return "gsr 0.1 (gfx950)"; }

static bool g_speculate = getenv("GSR_SPECULATE") == nullptr || getenv("GSR_SPECULATE")[0] != '0';
static bool g_rows_binning = getenv("GSR_ROWS_BINNING") == nullptr || getenv("GSR_ROWS_BINNING")[0] != '0';
// the multi-view backward's second stream (backward_multiview_impl)
static bool g_mv_streams = getenv("GSR_MV_STREAMS") == nullptr || getenv("GSR_MV_STREAMS")[0] != '0';
int gsr_set_option(const char* name, long long value) {
    if (!name) return fail("[gsr] option name is NULL");
    if (std::string(name) == "speculate") {  // gsr_forward's speculative stage B (default on)
        g_speculate = value != 0;
        return 0;
    }
    if (std::string(name) == "mv_streams") {  // multi-view backward on two streams (default on)
        g_mv_streams = value != 0;
        return 0;
    }
    if (std::string(name) == "rows_binning") {  // binning_rows.hip for grids <= 255 x 255 tiles (default on)
        g_rows_binning = value != 0;
        return 0;
    }
    if (std::string(name) == "split_fwd_bucket") {  // render forward: tiles with n >= 2^(v-1) on two waves; 0 = off
        gsr::set_split_buckets((int)value, gsr::split_bwd_depth());
        return 0;
    }
    if (std::string(name) == "split4_fwd_bucket") {  // render forward: tiles with n >= 2^(v-1) on four waves; 0 = off
        gsr::set_split4_bucket((int)value);
        return 0;
    }
    if (std::string(name) == "fwd_xcd_pairs") {  // forward: a split tile's halves on one XCD (b, b + 8)
        gsr::set_fwd_xcd_pairs((int)value);
        return 0;
    }
    if (std::string(name) == "fwd_order_cap") {  // forward tile order: lengths >= v share one bucket; 0 = off
        gsr::set_fwd_order_cap((int)value);
        return 0;
    }
    if (std::string(name) == "split_bwd_depth") {  // render backward: tiles this deep on two waves; 0 = off
        gsr::set_split_buckets(gsr::split_fwd_bucket(), (int)value);
        return 0;
    }
    if (std::string(name) == "bwd_ckpt") {  // render backward list segments at this position (x64); 0 = off
        gsr::set_bwd_ckpt((int)value);
        return 0;
    }
    if (std::string(name) == "sort_grouped") {  // depth sort: grouped look-back passes (default on)
        gsr::set_sort_grouped(value != 0);
        return 0;
    }
    if (std::string(name) == "sort_lookback_max") {
        gsr::set_sort_lookback_max(value < 0 ? 0 : (size_t)value);
        return 0;
    }
    if (gsr::set_train_option(name, value) == 0) return 0;
    return fail(std::string("[gsr] unknown option ") + name);
}

size_t gsr_geom_bytes(int P) { return gsr::geom_layout(P > 0 ? (size_t)P : 0).bytes; }
size_t gsr_binning_bytes(int num_rendered) { return gsr::bin_layout(num_rendered > 0 ? (size_t)num_rendered : 0).bytes; }
int gsr_binning_capacity(size_t bytes) {
    // largest C with gsr_binning_bytes(C) <= bytes (gsr_binning_bytes is non-decreasing)
    if (bytes < gsr_binning_bytes(0)) return -1;
    int lo = 0, hi = 0x7FFFFFFF;
    while (lo < hi) {
        const int mid = lo + (hi - lo + 1) / 2;
        if (gsr_binning_bytes(mid) <= bytes) lo = mid; else hi = mid - 1;
    }
    return lo;
}
size_t gsr_img_bytes(int W, int H) { return gsr::img_layout(W, H).bytes; }
size_t gsr_backward_scratch_bytes(int num_rendered) {
    return gsr::scratch_bytes(num_rendered > 0 ? (size_t)num_rendered : 0);
}

namespace {
// Layout capacity (instances) of a binning buffer: settings.binning_capacity if the caller
// laid the buffer out for more instances than num_rendered (gsr.h), else num_rendered.
size_t bin_cap(const gsr_settings* s, size_t I) {
    return s->binning_capacity > 0 && (size_t)s->binning_capacity > I ? (size_t)s->binning_capacity : I;
}
int geometry_impl(const gsr_settings* s, const gsr_inputs* in, void* geom, int* radii, void* stream,
                  int* num_rendered, bool wait);
int render_impl(const gsr_settings* s, const gsr_inputs* in, void* geom, void* binning, void* img, size_t cap,
                size_t n_host, const uint32_t* n_dev, float* out_color, float* out_depth, float* out_alpha,
                float* out_segment, void* stream);
}  // namespace

int gsr_forward_geometry(const gsr_settings* s, const gsr_inputs* in, void* geom, int* radii, void* stream,
                         int* num_rendered) {
    return geometry_impl(s, in, geom, radii, stream, num_rendered, true);
}

namespace {
int geometry_impl(const gsr_settings* s, const gsr_inputs* in, void* geom, int* radii, void* stream,
                  int* num_rendered, bool wait) {
    using namespace gsr;
    g_last_error.clear();
    if (int rc = validate(s, in, true)) return rc;
    if (!num_rendered) return fail("[gsr] num_rendered is NULL");
    *num_rendered = 0;
    const int P = s->P;
    if (P == 0) return 0;
    if (!geom || !radii) return fail("[gsr] geom/radii buffers are NULL");
    note_source(geom, P, in->shs != nullptr);
    hipStream_t st = (hipStream_t)stream;
    const bool dbg = s->debug != 0;
    const ImgLayout IL = img_layout(s->W, s->H);
    const GeomLayout L = geom_layout(P);
    char* g = aligned_base(geom);
    const bool packed = rect_packable(IL.gx, IL.gy);
    const HostSlot hs = host_total_slot();  // NULL views if pinned host memory is unavailable
    uint32_t* hslot = hs.host;
    bool tallied = false;  // the depth sort's histogram kernel posts num_rendered
    t_tallied = false;
    if (hslot) __atomic_store_n(hslot, TOTAL_PENDING, __ATOMIC_RELAXED);
    {
        StageScope sc(GSR_STAGE_PREPROCESS, st);
        const bool lb = sort_uses_lookback(P) || sort_grouped_size(P);  // look-back counters to clear
        launch_preprocess(*s, *in, IL.gx, IL.gy, at<float4>(g, L.rec), radii, at<uint32_t>(g, L.tiles_touched),
                          at<uint32_t>(g, L.depth_keys), at<uint8_t>(g, L.clamped), at<ushort4>(g, L.rect),
                          packed ? at<uint32_t>(g, L.rect32) : nullptr, at<float>(g, L.shjac), at<float2>(g, L.og),
                          at<uint32_t>(g, L.btot), g + L.ws, lb ? sort_zero_bytes(P, depth_sort_passes()) : 0,
                          g + L.ws_scan, scan_ws_bytes(P), st);
    }
    GSR_STAGE("preprocess");
    {
        // Depth order: 32-bit keys -> 4 passes (even: sorted keys land back in depth_keys).
        StageScope sc(GSR_STAGE_DEPTH_SORT, st);
        // only the order (+ rects) is used; the histogram kernel also sums tiles_touched into the
        // host-mapped num_rendered word (the binning kernels store the same value later)
        // (small scenes only: there the host waits on the word; at 1M Gaussians the host is
        // ~200 us ahead of the GPU and the tally's extra loads and 64-bit atomic cost
        // k_radix_hist 2 us: 10.5 -> 12.6 us)
        const bool tally = P <= TALLY_MAX_P;
        const SortFinal nokeys{nullptr, nullptr, 0, true, tally ? at<uint32_t>(g, L.tiles_touched) : nullptr,
                               tally ? hs.dev : nullptr, &tallied, at<uint32_t>(g, L.btot),
                               at<uint32_t>(g, L.bbase), (uint32_t)cdiv((size_t)P, (size_t)SLOT_BLOCK)};
        launch_radix_sort(at<uint32_t>(g, L.depth_keys), nullptr, at<uint32_t>(g, L.dkeys_alt),
                          at<uint32_t>(g, L.order_alt), at<uint32_t>(g, L.depth_keys), at<uint32_t>(g, L.order), P,
                          32, g + L.ws, /*ws_zeroed=*/true, st, packed ? at<uint32_t>(g, L.rect32) : nullptr,
                          packed ? at<uint32_t>(g, L.rect32_alt) : nullptr,
                          packed ? at<uint32_t>(g, L.rect32_sorted) : nullptr, &nokeys,
                          /*skip_sentinel=*/true);  // culled Gaussians (key ~0u) emit nothing
    }
    t_tallied = tallied;
    GSR_STAGE("depth sort");
    // gsr_forward's speculative stage B with row binning computes the offsets and num_rendered
    // in its level-1 kernels (binning_rows.hip, fused mode): no scan here
    if (!wait && packed && g_rows_binning) return 0;
    {
        StageScope sc(GSR_STAGE_SCAN, st);
        if (packed)  // tile counts from the depth-ordered packed rects: no gather
            launch_scan_inclusive_gather(at<uint32_t>(g, L.rect32_sorted), nullptr, at<uint32_t>(g, L.offsets), P,
                                         g + L.ws_scan, /*ws_zeroed=*/true, st, tallied ? nullptr : hs.dev,
                                         /*rect_mode=*/true);
        else
            launch_scan_inclusive_gather(at<uint32_t>(g, L.tiles_touched), at<uint32_t>(g, L.order),
                                         at<uint32_t>(g, L.offsets), P, g + L.ws_scan, /*ws_zeroed=*/true, st,
                                         tallied ? nullptr : hs.dev);
    }
    GSR_STAGE("scan");
    if (!wait) return 0;  // gsr_forward's speculative stage B: waits after launching it
    uint32_t total = 0;
    if (int rc = wait_total(hslot, st, at<uint32_t>(g, L.offsets) + (P - 1), &total)) return rc;
    if (total > 0x7FFFFFFFu) return fail("[gsr] num_rendered overflows int32");
    *num_rendered = (int)total;
    return 0;
}
}  // namespace

int gsr_forward_render(const gsr_settings* s, const gsr_inputs* in, void* geom, void* binning, void* img,
                       int num_rendered, float* out_color, float* out_depth, float* out_alpha, float* out_segment,
                       void* stream) {
    g_last_error.clear();
    const size_t I = num_rendered > 0 ? (size_t)num_rendered : 0;
    if (int rc = validate(s, in, true)) return rc;
    return render_impl(s, in, geom, binning, img, bin_cap(s, I), I, nullptr, out_color, out_depth, out_alpha,
                       out_segment, stream);
}

namespace {
// Stage B.  cap: the binning buffer's layout capacity; n_host: instances to sort (grid
// sizes); n_dev: when non-NULL, the device word holding num_rendered (speculative stage
// B, launched before the host knows it: the kernels clamp to min(*n_dev, n_host) and
// never write a slot >= cap).
int render_impl(const gsr_settings* s, const gsr_inputs* in, void* geom, void* binning, void* img, size_t cap,
                size_t n_host, const uint32_t* n_dev, float* out_color, float* out_depth, float* out_alpha,
                float* out_segment, void* stream) {
    using namespace gsr;
    if (!img || !out_color || !out_depth || !out_alpha || !out_segment) return fail("[gsr] null output buffer");
    hipStream_t st = (hipStream_t)stream;
    const bool dbg = s->debug != 0;
    const int P = s->P;
    const size_t I = n_host;
    const ImgLayout IL = img_layout(s->W, s->H);
    const int T = IL.gx * IL.gy;
    char* im = aligned_base(img);
    uint2* ranges = at<uint2>(im, IL.ranges);
    if (I == 0 && hipMemsetAsync(ranges, 0, (size_t)T * sizeof(uint2), st) != hipSuccess)
        return fail("[gsr] memset ranges");  // otherwise k_duplicate clears them
    const GeomLayout GL = geom_layout(P > 0 ? P : 0);
    char* g = P > 0 ? aligned_base(geom) : nullptr;
    const BinLayout BL = bin_layout(cap);
    char* b = I > 0 ? aligned_base(binning) : nullptr;
    uint32_t* point_list = nullptr;
    uint32_t* order = at<uint32_t>(im, IL.order);
    const bool rows = I > 0 && g_rows_binning && rect_packable(IL.gx, IL.gy);
    if (I > 0) {
        if (!geom || !binning) return fail("[gsr] geom/binning buffers are NULL");
        if (rows) {
            // tile lists by row-then-tile expansion of the depth-ordered Gaussians
            // (binning_rows.hip): level 1 under the "duplicate" stage, level 2 under
            // "tile_sort", ranges + tile order under "ranges"
            const uint32_t* n_total = at<uint32_t>(g, GL.offsets) + (P - 1);
            auto rb = [&](int stage) {
                launch_rows_binning(P, IL.gx, IL.gy, at<uint32_t>(g, GL.order), at<uint32_t>(g, GL.offsets),
                                    at<uint32_t>(g, GL.rect32_sorted), g + GL.ws, b + BL.ws,
                                    at<uint32_t>(b, BL.tkeys), at<uint32_t>(b, BL.vals_alt),
                                    at<uint32_t>(b, BL.point_list), ranges, order, at<uint4>(b, BL.written),
                                    cdiv(cap, 16), cap, n_total, st, stage, /*fused=*/true,
                                    n_dev && !t_tallied ? host_total_slot().dev : nullptr);
            };
            {
                StageScope sc(GSR_STAGE_DUPLICATE, st);
                rb(0);
            }
            GSR_STAGE("rows");
            {
                StageScope sc(GSR_STAGE_TILE_SORT, st);
                rb(1);
            }
            GSR_STAGE("tiles");
            {
                StageScope sc(GSR_STAGE_RANGES, st);
                rb(2);
            }
            GSR_STAGE("tile ranges + order");
        } else {
            {
                StageScope sc(GSR_STAGE_DUPLICATE, st);
                launch_duplicate(P, at<uint32_t>(g, GL.order), at<uint32_t>(g, GL.offsets),
                                 at<uint32_t>(g, GL.tiles_touched), at<ushort4>(g, GL.rect),
                                 rect_packable(IL.gx, IL.gy) ? at<uint32_t>(g, GL.rect32_sorted) : nullptr, IL.gx,
                                 at<uint32_t>(b, BL.tkeys), at<uint32_t>(b, BL.slot_gid), ranges, T, (uint32_t)cap,
                                 st);
            }
            GSR_STAGE("duplicate");
            const int bits = (int)higher_msb((uint32_t)T);
            const int passes = (bits + RADIX_BITS - 1) / RADIX_BITS;
            // even pass count: sorted keys return to tkeys; odd: they land in tkeys_alt.
            uint32_t* kin = at<uint32_t>(b, BL.tkeys);
            uint32_t* kalt = at<uint32_t>(b, BL.tkeys_alt);
            uint32_t* kout = (passes % 2 == 0) ? kin : kalt;
            uint32_t* ktmp = (passes % 2 == 0) ? kalt : kin;
            {
                // key = tile, payload = (instance slot u, Gaussian id): the slot orders ties by
                // (depth, gaussian); the id travels along so point_list needs no gather.
                StageScope sc(GSR_STAGE_TILE_SORT, st);
                // the last pass also produces the tile ranges (identifyTileRanges,
                // rasterizer_impl.cu:113-138) and clears the backward's written-slot flags
                const SortFinal fin{ranges, at<uint4>(b, BL.written), cdiv(cap, 16)};
                launch_radix_sort(kin, nullptr, ktmp, at<uint32_t>(b, BL.vals_alt), kout,
                                  at<uint32_t>(b, BL.slot_vals), I, bits, b + BL.ws, /*ws_zeroed=*/false, st,
                                  at<uint32_t>(b, BL.slot_gid), at<uint32_t>(b, BL.gid_alt),
                                  at<uint32_t>(b, BL.point_list), &fin, /*skip_sentinel=*/false, n_dev);
            }
            GSR_STAGE("tile sort");
        }
        point_list = at<uint32_t>(b, BL.point_list);
    }
    if (!rows) {
        StageScope sc(GSR_STAGE_RANGES, st);
        launch_tile_order(ranges, T, order, st);
    }
    GSR_STAGE("tile order");
    {
        StageScope sc(GSR_STAGE_RENDER_FWD, st);
        launch_render_forward(s->W, s->H, IL.gx, IL.gy, order, order + T, ranges, point_list,
                              g ? at<float4>(g, GL.rec) : nullptr, s->bg, out_color, out_depth, out_alpha,
                              out_segment, at<uint32_t>(im, IL.n_contrib), at<float>(im, IL.ckpt), st);
    }
    GSR_STAGE("render");
    return 0;
}
}  // namespace

int gsr_forward_deferred(const gsr_settings* s, const gsr_inputs* in, void* geom, int* radii, void* binning,
                         size_t binning_bytes, void* img, float* out_color, float* out_depth, float* out_alpha,
                         float* out_segment, void* stream, int* ticket) {
    using namespace gsr;
    g_last_error.clear();
    if (!ticket) return fail("[gsr] forward_deferred: ticket is NULL");
    *ticket = -1;
    const size_t C = s && s->binning_capacity > 0 ? (size_t)s->binning_capacity : 0;
    if (!s || s->P <= 0 || C == 0 || !binning || gsr_binning_bytes((int)C) > binning_bytes)
        return fail("[gsr] forward_deferred: needs P > 0 and a binning buffer laid out for binning_capacity > 0");
    HostSlots& hs = host_slots();
    int k = 1;
    while (k < HOST_SLOTS && hs.busy[k]) ++k;
    if (k == HOST_SLOTS) return fail("[gsr] forward_deferred: too many calls in flight (gsr_forward_wait each)");
    t_slot = k;
    int nr = 0;
    int rc = geometry_impl(s, in, geom, radii, stream, &nr, false);
    if (rc == 0) {
        const GeomLayout L = geom_layout((size_t)s->P);
        const uint32_t* n_dev = at<uint32_t>(aligned_base(geom), L.offsets) + (s->P - 1);
        rc = render_impl(s, in, geom, binning, img, C, C, n_dev, out_color, out_depth, out_alpha, out_segment,
                         stream);
    }
    t_slot = 0;
    if (rc) {
        // kernels already queued may still store into slot k's word: let them finish before the
        // slot can be handed out again
        (void)hipStreamSynchronize((hipStream_t)stream);
        return rc;
    }
    hs.busy[k] = true;
    *ticket = k;
    return 0;
}

int gsr_forward_wait(int ticket, const gsr_settings* s, const void* geom, void* stream, int* num_rendered) {
    using namespace gsr;
    g_last_error.clear();
    if (ticket < 1 || ticket >= HOST_SLOTS) return fail("[gsr] forward_wait: not a pending ticket");
    HostSlots& hs = host_slots();
    if (!hs.busy[ticket]) return fail("[gsr] forward_wait: not a pending ticket");
    // a bad call keeps the ticket pending: its kernels may still store into the slot's word,
    // so the slot must not be handed to the next gsr_forward_deferred
    if (!s || !geom || !num_rendered || s->P <= 0) return fail("[gsr] forward_wait: null argument");
    const GeomLayout L = geom_layout((size_t)s->P);
    const uint32_t* n_dev = at<uint32_t>(aligned_base(const_cast<void*>(geom)), L.offsets) + (s->P - 1);
    uint32_t total = 0;
    const int rc = wait_total(hs.host ? hs.host + 16 * ticket : nullptr, (hipStream_t)stream, n_dev, &total);
    if (rc) (void)hipStreamSynchronize((hipStream_t)stream);  // nothing may store the word after release
    hs.busy[ticket] = false;
    if (rc) return rc;
    if (total > 0x7FFFFFFFu) return fail("[gsr] num_rendered overflows int32");
    *num_rendered = (int)total;
    return total > (uint32_t)s->binning_capacity ? GSR_NEED_BINNING : 0;
}

int gsr_forward(const gsr_settings* s, const gsr_inputs* in, void* geom, int* radii, void* binning,
                size_t binning_bytes, void* img, float* out_color, float* out_depth, float* out_alpha,
                float* out_segment, void* stream, int* num_rendered) {
    using namespace gsr;
    const size_t C = s && s->binning_capacity > 0 ? (size_t)s->binning_capacity : 0;
    if (g_speculate && C > 0 && s->P > 0 && binning && gsr_binning_bytes((int)C) <= binning_bytes) {
        // Speculative stage B: launched right behind stage A into the caller's buffer laid out
        // for C instances, the kernels reading num_rendered from device memory; the host waits
        // for num_rendered only afterwards, so no host round trip stalls the GPU.
        if (int rc = geometry_impl(s, in, geom, radii, stream, num_rendered, false)) {
            (void)hipStreamSynchronize((hipStream_t)stream);  // queued kernels may still store the slot word
            return rc;
        }
        const GeomLayout L = geom_layout((size_t)s->P);
        const uint32_t* n_dev = at<uint32_t>(aligned_base(geom), L.offsets) + (s->P - 1);
        if (int rc = render_impl(s, in, geom, binning, img, C, C, n_dev, out_color, out_depth, out_alpha,
                                 out_segment, stream)) {
            (void)hipStreamSynchronize((hipStream_t)stream);
            return rc;
        }
        uint32_t total = 0;
        if (int rc = wait_total(host_total_slot().host, (hipStream_t)stream, n_dev, &total)) return rc;
        if (total > 0x7FFFFFFFu) return fail("[gsr] num_rendered overflows int32");
        *num_rendered = (int)total;
        return total > C ? GSR_NEED_BINNING : 0;  // over capacity: stage B's results are void
    }
    if (int rc = gsr_forward_geometry(s, in, geom, radii, stream, num_rendered)) return rc;
    if (*num_rendered > 0 && (binning == nullptr || gsr_binning_bytes(*num_rendered) > binning_bytes))
        return GSR_NEED_BINNING;
    return gsr_forward_render(s, in, geom, binning, img, *num_rendered, out_color, out_depth, out_alpha,
                              out_segment, stream);
}

namespace {
int backward_impl(const gsr_settings* s, const gsr_inputs* in, const int* radii, void* geom, void* binning,
                  void* img, int num_rendered, const float* alpha, const float* dL_dcolor, const float* dL_dsegment,
                  const float* dL_ddepth, const float* dL_dalpha, void* scratch, const gsr_grads* grads,
                  float* sh_rows, void* stream);
}  // namespace

int gsr_backward(const gsr_settings* s, const gsr_inputs* in, const int* radii, void* geom, void* binning,
                 void* img, int num_rendered, const float* alpha, const float* dL_dcolor, const float* dL_dsegment,
                 const float* dL_ddepth, const float* dL_dalpha, void* scratch, const gsr_grads* grads,
                 void* stream) {
    return backward_impl(s, in, radii, geom, binning, img, num_rendered, alpha, dL_dcolor, dL_dsegment, dL_ddepth,
                         dL_dalpha, scratch, grads, nullptr, stream);
}

int gsr_backward_deferred_sh(const gsr_settings* s, const gsr_inputs* in, const int* radii, void* geom,
                             void* binning, void* img, int num_rendered, const float* alpha, const float* dL_dcolor,
                             const float* dL_dsegment, const float* dL_ddepth, const float* dL_dalpha,
                             void* scratch, const gsr_grads* grads, float* sh_rows, void* stream) {
    if (!sh_rows || !in || !in->shs) {
        g_last_error = "[gsr] deferred SH backward: sh_rows and shs are required";
        return 1;
    }
    return backward_impl(s, in, radii, geom, binning, img, num_rendered, alpha, dL_dcolor, dL_dsegment, dL_ddepth,
                         dL_dalpha, scratch, grads, sh_rows, stream);
}

namespace {
int backward_impl(const gsr_settings* s, const gsr_inputs* in, const int* radii, void* geom, void* binning,
                  void* img, int num_rendered, const float* alpha, const float* dL_dcolor, const float* dL_dsegment,
                  const float* dL_ddepth, const float* dL_dalpha, void* scratch, const gsr_grads* grads,
                  float* sh_rows, void* stream) {
    using namespace gsr;
    g_last_error.clear();
    if (int rc = validate(s, in, false)) return rc;
    if (!grads) return fail("[gsr] grads is NULL");
    const int P = s->P;
    if (P == 0) return 0;
    if (!geom || !img || !radii || !alpha || !dL_dcolor || !dL_dsegment || !dL_ddepth || !dL_dalpha)
        return fail("[gsr] null buffer");
    if (int rc = check_source(geom, P, in->shs != nullptr)) return rc;
    hipStream_t st = (hipStream_t)stream;
    const bool dbg = s->debug != 0;
    const size_t I = num_rendered > 0 ? (size_t)num_rendered : 0;
    const ImgLayout IL = img_layout(s->W, s->H);
    char* im = aligned_base(img);
    const GeomLayout GL = geom_layout(P);
    char* g = aligned_base(geom);
    float* contrib = nullptr;
    uint8_t* written = nullptr;
    if (I > 0) {
        if (!binning || !scratch) return fail("[gsr] binning/scratch buffer is NULL");
        const BinLayout BL = bin_layout(bin_cap(s, I));
        char* b = aligned_base(binning);
        contrib = reinterpret_cast<float*>(aligned_base(scratch));
        written = at<uint8_t>(b, BL.written);  // cleared by the forward's tile sort
        {
            StageScope sc(GSR_STAGE_RENDER_BWD, st);
            launch_render_backward(s->W, s->H, IL.gx, IL.gy, at<uint32_t>(im, IL.order),
                                   at<uint32_t>(im, IL.order) + IL.gx * IL.gy, at<uint2>(im, IL.ranges),
                                   at<uint32_t>(b, BL.point_list), at<uint32_t>(g, GL.bbase),
                                   at<float4>(g, GL.rec), s->bg, alpha, at<uint32_t>(im, IL.n_contrib), dL_dcolor,
                                   dL_dsegment, dL_ddepth, dL_dalpha, contrib, written, at<float>(im, IL.ckpt), st);
        }
        GSR_STAGE("render backward");
    }
    {
        StageScope sc(GSR_STAGE_GAUSSIAN_BWD, st);
        gsr_grads gr = *grads;
        if (sh_rows) gr.dsh = nullptr;  // deferred: the exchange writes dsh from the rows
        launch_gaussian_backward(*s, *in, radii, at<uint32_t>(g, GL.tiles_touched), at<float2>(g, GL.og),
                                 at<uint32_t>(g, GL.bbase),
                                 at<uint8_t>(g, GL.clamped), contrib, written,
                                 at<float>(g, GL.shjac), gr, sh_rows, st);
    }
    GSR_STAGE("gaussian backward");
    return 0;
}
}  // namespace

size_t gsr_multiview_scratch_bytes(int P, int B) {
    return gsr::align_up(gsr::sh_rows_floats(P > 0 ? P : 0) * (size_t)(B > 0 ? B : 0) * 4) + gsr::ALIGN;
}

size_t gsr_sh_rows_floats(int P) { return gsr::sh_rows_floats(P > 0 ? P : 0); }

namespace {
// The multi-view backward alternates its views' render backwards between the caller's stream
// and an auxiliary stream of libgsr's (one per device, created on first use), so that one
// view's render backward fills the tail of the previous one instead of the chip idling half
// empty behind the deepest tiles; the per-Gaussian pass waits for both.  The views write
// disjoint scratch, and the caller's stream waits for the auxiliary one before anything that
// follows, so the caller sees one stream's ordering.  gsr_set_option("mv_streams", 0) or a
// debug call (stage-by-stage synchronisation) keeps everything on the caller's stream.
struct AuxStream {
    hipStream_t st = nullptr;
};
hipStream_t aux_stream() {
    static std::mutex mu;
    static AuxStream aux[64];
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return nullptr;
    std::lock_guard<std::mutex> lk(mu);
    if (!aux[dev].st && hipStreamCreateWithFlags(&aux[dev].st, hipStreamNonBlocking) != hipSuccess) aux[dev].st = nullptr;
    return aux[dev].st;
}
// per thread and device: the fork and join events of one multi-view call (re-recorded by the
// next call of the same thread only after this call enqueued its waits)
struct ForkJoin {
    hipEvent_t fork = nullptr, join = nullptr;
};
bool fork_join(ForkJoin*& fj) {
    thread_local ForkJoin t[64];
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return false;
    fj = &t[dev];
    if (!fj->fork && hipEventCreateWithFlags(&fj->fork, hipEventDisableTiming) != hipSuccess) return false;
    if (!fj->join && hipEventCreateWithFlags(&fj->join, hipEventDisableTiming) != hipSuccess) return false;
    return true;
}

int backward_multiview_impl(int B, const gsr_view_state* views, const gsr_inputs* in, void* mv_scratch,
                            float* sh_rows, const gsr_grads* grads, void* stream) {
    using namespace gsr;
    g_last_error.clear();
    const bool defer = sh_rows != nullptr;
    if (defer && (!in || !in->shs)) return fail("[gsr] deferred SH backward: shs must be present");
    if (defer && (reinterpret_cast<uintptr_t>(sh_rows) & 15)) return fail("[gsr] deferred SH backward: sh_rows must be 16-B aligned");
    if (B < 1 || B > GSR_MAX_VIEWS) return fail("[gsr] multiview: B must be 1..16");
    if (!views || !in || !grads) return fail("[gsr] multiview: null argument");
    const gsr_settings* s0 = views[0].s;
    if (!s0) return fail("[gsr] multiview: view 0 has no settings");
    for (int v = 0; v < B; ++v) {
        const gsr_view_state& V = views[v];
        if (!V.s) return fail("[gsr] multiview: a view has no settings");
        if (int rc = validate(V.s, in, false)) return rc;
        if (V.s->P != s0->P || V.s->D != s0->D || V.s->M != s0->M || V.s->scale_modifier != s0->scale_modifier)
            return fail("[gsr] multiview: P, D, M and scale_modifier must be equal across views");
    }
    const int P = s0->P;
    if (P == 0) return 0;
    if (in->shs && !mv_scratch && !defer) return fail("[gsr] multiview: scratch is NULL");
    // Every view is validated before any work is queued: once odd views run on the auxiliary
    // stream, an early return would leave the caller's stream unordered after work that still
    // reads and writes the caller's buffers.
    for (int v = 0; v < B; ++v) {
        const gsr_view_state& V = views[v];
        if (!V.geom || !V.img || !V.radii || !V.alpha || !V.dL_dcolor || !V.dL_dsegment || !V.dL_ddepth ||
            !V.dL_dalpha)
            return fail("[gsr] multiview: null buffer");
        // each view's SH direction Jacobian comes from its forward (as in gsr_backward)
        if (int rc = check_source(V.geom, P, in->shs != nullptr)) return rc;
        if (V.num_rendered > 0 && (!V.binning || !V.scratch))
            return fail("[gsr] multiview: binning/scratch buffer is NULL");
    }
    hipStream_t st = (hipStream_t)stream;
    const bool dbg = s0->debug != 0;
    hipStream_t aux = (B > 1 && g_mv_streams && !dbg) ? aux_stream() : nullptr;
    ForkJoin* fj = nullptr;
    if (aux && (!fork_join(fj) || hipEventRecord(fj->fork, st) != hipSuccess ||
                hipStreamWaitEvent(aux, fj->fork, 0) != hipSuccess))
        aux = nullptr;
    bool aux_used = false;
    // a failure after the fork still joins: the caller's stream waits for the auxiliary work
    auto join = [&]() -> bool {
        return !aux || !aux_used ||
               (hipEventRecord(fj->join, aux) == hipSuccess && hipStreamWaitEvent(st, fj->join, 0) == hipSuccess);
    };
    MvArgs a{};
    a.B = B;
    for (int v = 0; v < B; ++v) {
        const gsr_view_state& V = views[v];
        const gsr_settings* s = V.s;
        const size_t I = V.num_rendered > 0 ? (size_t)V.num_rendered : 0;
        const ImgLayout IL = img_layout(s->W, s->H);
        char* im = aligned_base(V.img);
        const GeomLayout GL = geom_layout(P);
        char* g = aligned_base(V.geom);
        float* contrib = nullptr;
        uint8_t* written = nullptr;
        if (I > 0) {
            const BinLayout BL = bin_layout(bin_cap(V.s, I));
            char* b = aligned_base(V.binning);
            contrib = reinterpret_cast<float*>(aligned_base(V.scratch));
            written = at<uint8_t>(b, BL.written);
            const hipStream_t sv = (aux && (v & 1)) ? aux : st;  // odd views on the auxiliary stream
            aux_used |= sv == aux;
            {
                StageScope sc(GSR_STAGE_RENDER_BWD, sv);
                launch_render_backward(s->W, s->H, IL.gx, IL.gy, at<uint32_t>(im, IL.order),
                                       at<uint32_t>(im, IL.order) + IL.gx * IL.gy, at<uint2>(im, IL.ranges),
                                       at<uint32_t>(b, BL.point_list),
                                       at<uint32_t>(g, GL.bbase), at<float4>(g, GL.rec), s->bg, V.alpha,
                                       at<uint32_t>(im, IL.n_contrib), V.dL_dcolor, V.dL_dsegment, V.dL_ddepth,
                                       V.dL_dalpha, contrib, written, at<float>(im, IL.ckpt), sv);
            }
            if (int rc = check("render backward", sv, dbg)) {
                (void)join();
                return rc;
            }
        } else {
            // nothing rendered: every radius is 0 and the records are never read
            written = nullptr;
        }
        MvView& w = a.v[v];
        w.radii = V.radii;
        w.tiles_touched = at<uint32_t>(g, GL.tiles_touched);
        w.bbase = at<uint32_t>(g, GL.bbase);
        w.clamped = at<uint8_t>(g, GL.clamped);
        w.contrib = contrib;
        w.written = written;
        w.og = at<float2>(g, GL.og);
        w.shjac = at<float>(g, GL.shjac);
        w.view = s->viewmatrix;
        w.proj = s->projmatrix;
        w.campos = s->campos;
        w.dmeans2D = V.dmeans2D;
        w.W = s->W;
        w.H = s->H;
        w.tanfovx = s->tanfovx;
        w.tanfovy = s->tanfovy;
    }
    // join: the per-Gaussian pass (and the caller) after every view's render backward (nothing to
    // join when no view went to the auxiliary stream, e.g. the odd views rendered nothing)
    if (!join()) return fail("[gsr] multiview: stream join failed");
    {
        StageScope sc(GSR_STAGE_GAUSSIAN_BWD, st);
        float* shx = defer ? sh_rows : reinterpret_cast<float*>(in->shs ? aligned_base(mv_scratch) : nullptr);
        launch_gaussian_backward_multiview(P, s0->D, s0->M, s0->scale_modifier, *in, a, *grads, shx, defer, st);
    }
    GSR_STAGE("gaussian backward (multiview)");
    return 0;
}
}  // namespace

int gsr_backward_multiview(int B, const gsr_view_state* views, const gsr_inputs* in, void* mv_scratch,
                           const gsr_grads* grads, void* stream) {
    return backward_multiview_impl(B, views, in, mv_scratch, nullptr, grads, stream);
}

int gsr_backward_multiview_deferred_sh(int B, const gsr_view_state* views, const gsr_inputs* in, float* sh_rows,
                                       const gsr_grads* grads, void* stream) {
    if (!sh_rows) {
        g_last_error = "[gsr] deferred SH backward: sh_rows is NULL";
        return 1;
    }
    return backward_multiview_impl(B, views, in, nullptr, sh_rows, grads, stream);
}

int gsr_sh_backward(int V, int P, int D, int M, const float* shs, const float* means3D, const float* sh_rows,
                    float* dsh, float* dmeans3D, void* stream) {
    using namespace gsr;
    g_last_error.clear();
    if (V < 0 || P < 0 || D < 0 || D > 3 || M < 1 || M < (D + 1) * (D + 1))
        return fail("[gsr] sh backward: bad V / P / D / M");
    if (P == 0) return 0;
    if (!means3D || (V > 0 && !sh_rows)) return fail("[gsr] sh backward: null argument");
    if (V == 0) {
        if (dsh) (void)hipMemsetAsync(dsh, 0, (size_t)P * M * 3 * 4, (hipStream_t)stream);
        return 0;
    }
    (void)shs;
    (void)dmeans3D;  // the views' direction terms are in dmeans3D already (the multi-view backward)
    launch_sh_backward(P, D, M, means3D, V, sh_rows, dsh, (hipStream_t)stream);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail(std::string("[gsr] sh backward: ") + hipGetErrorString(e));
    return 0;
}

int gsr_num_stages(void) { return NUM_STAGES; }

const char* gsr_stage_name(int stage) { return (stage >= 0 && stage < NUM_STAGES) ? STAGE_NAMES[stage] : ""; }

void gsr_timing_enable(int stage_mask) {
    Timer& T = timer();
    std::lock_guard<std::mutex> lk(T.mu);
    T.mask = (unsigned)stage_mask;
}

int gsr_timing_collect(double* ms, long long* counts) {
    Timer& T = timer();
    std::lock_guard<std::mutex> lk(T.mu);
    for (auto& r : T.pending) {
        float t = 0.f;
        if (hipEventSynchronize(r.b) == hipSuccess && hipEventElapsedTime(&t, r.a, r.b) == hipSuccess) {
            if (ms) ms[r.stage] += t;
            if (counts) counts[r.stage] += 1;
        }
        T.pool.push_back(r.a);
        T.pool.push_back(r.b);
    }
    T.pending.clear();
    return NUM_STAGES;
}

long long gsr_debug_copy(const char* name, int P, int W, int H, int num_rendered, int binning_capacity,
                         void* geom, void* binning, void* img, void* dst, void* stream) {
    using namespace gsr;
    g_last_error.clear();
    if (!name) {
        fail("[gsr] debug_copy: null argument");
        return -1;
    }
    const std::string n(name);
    const size_t Pz = P > 0 ? (size_t)P : 0, I = num_rendered > 0 ? (size_t)num_rendered : 0;
    const GeomLayout GL = geom_layout(Pz);
    const BinLayout BL = bin_layout(binning_capacity > 0 && (size_t)binning_capacity > I ? (size_t)binning_capacity : I);
    const ImgLayout IL = img_layout(W, H);
    const size_t T = (size_t)IL.gx * IL.gy;
    const char* src = nullptr;
    size_t bytes = 0;
    auto G = [&](size_t off, size_t b) { bytes = b; if (geom) src = aligned_base(geom) + off; };
    auto B = [&](size_t off, size_t b) { bytes = b; if (binning) src = aligned_base(binning) + off; };
    auto M = [&](size_t off, size_t b) { bytes = b; if (img) src = aligned_base(img) + off; };
    if (n == "tiles_touched") G(GL.tiles_touched, Pz * 4);
    else if (n == "rec") G(GL.rec, Pz * 64);
    else if (n == "clamped") G(GL.clamped, Pz);
    else if (n == "order") G(GL.order, Pz * 4);
    else if (n == "goff") G(GL.og + 4, Pz * 4);  // the odd words of the (opacity, goff) pairs
    else if (n == "bbase") G(GL.bbase, cdiv(Pz, (size_t)SLOT_BLOCK) * 4);
    else if (n == "point_list") B(BL.point_list, I * 4);
    else if (n == "slot_vals") {
        // only the radix binning (grids beyond 255 x 255 tiles, or row binning switched off)
        // writes it; the row binning derives record slots from the record
        if (g_rows_binning && rect_packable(IL.gx, IL.gy)) {
            fail("[gsr] debug_copy: slot_vals is not materialised by the row binning");
            return -1;
        }
        B(BL.slot_vals, I * 4);
    }
    else if (n == "written") B(BL.written, I);  // the backward's written-record flags (1 byte per slot)
    else if (n == "ranges") M(IL.ranges, T * 8);
    else if (n == "n_contrib_tiles") M(IL.n_contrib, T * TILE_PIX * 4);
    else if (n == "tile_order") M(IL.order, tile_sched_words(T) * 4);  // heavy-first order + TileSched
    else {
        fail("[gsr] debug_copy: unknown field");
        return -1;
    }
    if (!dst) return (long long)bytes;  // size query: no device access
    if (bytes == 0 || !src) return 0;   // empty, or the buffer holding it was not passed
    if (n == "goff") {  // strided: 4 of every 8 bytes
        if (hipMemcpy2DAsync(dst, 4, src, 8, 4, Pz, hipMemcpyDeviceToDevice, (hipStream_t)stream) != hipSuccess)
            return -1;
        return (long long)bytes;
    }
    if (hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, (hipStream_t)stream) != hipSuccess) return -1;
    return (long long)bytes;
}

int gsr_mark_visible(int P, const float* means3D, const float* viewmatrix, const float* projmatrix,
                     uint8_t* present, void* stream) {
    (void)projmatrix;  // the reference computes p_proj but only tests view-space z (auxiliary.h:154)
    g_last_error.clear();
    if (P < 0) return fail("[gsr] invalid P");
    if (P == 0) return 0;
    if (!means3D || !viewmatrix || !present) return fail("[gsr] null buffer");
    hipStream_t st = (hipStream_t)stream;
    gsr::launch_mark_visible(P, means3D, viewmatrix, present, st);
    if (int rc = check("mark_visible", st, false)) return rc;
    return 0;
}


int gsr_stream_copy(const void* src, void* dst, size_t bytes, int per_thread, void* stream) {
    g_last_error.clear();
    if (!src || !dst || bytes % 16) return fail("[gsr] stream_copy: null buffer or size not a multiple of 16");
    const size_t n = bytes / 16;
    if (n == 0) return 0;
    hipStream_t st = (hipStream_t)stream;
    const auto* s4 = (const float4*)src;
    auto* d4 = (float4*)dst;
    switch (per_thread) {
        case 1: hipLaunchKernelGGL(gsr::k_stream_copy<1>, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, s4, d4, n); break;
        case 2: hipLaunchKernelGGL(gsr::k_stream_copy<2>, dim3((unsigned)((n + 511) / 512)), dim3(256), 0, st, s4, d4, n); break;
        case 4: hipLaunchKernelGGL(gsr::k_stream_copy<4>, dim3((unsigned)((n + 1023) / 1024)), dim3(256), 0, st, s4, d4, n); break;
        default: return fail("[gsr] stream_copy: per_thread must be 1, 2 or 4");
    }
    if (int rc = check("stream_copy", st, false)) return rc;
    return 0;
}

}  // extern "C"
