// gsr_internal.h -- shared layout + launch declarations of libgsr (not part of the ABI).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stddef.h>

#include <algorithm>
#include <string>

#include "../../include/gsr.h"

namespace gsr {

// Sets the thread-local gsr_last_error() message; returns 1 (api.hip).
int set_error(const std::string& msg);
// Training-kernel launch options (train.hip); -1 = unknown name.
int set_train_option(const std::string& name, long long value);

constexpr int BX = GSR_BLOCK_X, BY = GSR_BLOCK_Y;
constexpr int NCH = GSR_NUM_CHANNELS, NCLS = GSR_NUM_CLASS;
constexpr int TILE_PIX = BX * BY;  // 256 pixels per tile, 4 per lane of one wave64

// Per-Gaussian render record (64 B, one HBM sector pair, never crosses a 128 B line):
//   r0 = {x, y, conic.x, conic.y}   r1 = {conic.z, opacity, depth, seg0}
//   r2 = {r, g, b, seg1}            r3 = reserved (0)
constexpr int REC_F4 = 4;

// Radix sort / scan tiling (256-thread blocks = 4 wave64s, 16 items per thread).
constexpr int SORT_THREADS = 256, SORT_ITEMS = 16, SORT_TILE = SORT_THREADS * SORT_ITEMS;
// Look-back scan tiles of 8192 values, 16 waves x 8 per thread (r2, metric scene: the depth-
// order scan 9.7 -> 8.4 us and the tile sort's level-2 scan ~4 us faster than 4 waves x 16;
// tools/bench_stage_variants.sh with -DGSR_SCAN_THREADS / -DGSR_SCAN_ITEMS)
#ifndef GSR_SCAN_THREADS
#define GSR_SCAN_THREADS 1024
#endif
#ifndef GSR_SCAN_ITEMS
#define GSR_SCAN_ITEMS 8
#endif
constexpr int SCAN_THREADS = GSR_SCAN_THREADS, SCAN_ITEMS = GSR_SCAN_ITEMS, SCAN_TILE = SCAN_THREADS * SCAN_ITEMS;
constexpr int RADIX_BITS = 8, RADIX = 1 << RADIX_BITS;

constexpr size_t ALIGN = 256;
inline size_t align_up(size_t x) { return (x + ALIGN - 1) & ~(ALIGN - 1); }
__host__ __device__ inline size_t cdiv(size_t a, size_t b) { return (a + b - 1) / b; }

// Zero n4 16-B words with a grid-stride loop: lets a kernel that runs anyway clear
// the next stage's counters instead of a separate memset launch.
// Heavy-first tile schedule bucket: the bit length of a tile's instance count (0 = empty).
__device__ __forceinline__ uint32_t len_bucket(uint2 r) {
    const uint32_t len = r.y - r.x;
    return len ? 32 - __clz(len) : 0;
}
// Finer schedule bucket of the row-binning path: quarter octaves, 4 * bit length + the two bits
// below the leading one (0 = empty, up to 131).  Bit length B <-> fine buckets [4B, 4B + 3].
constexpr int FINE_BUCKETS = 132;
__host__ __device__ inline uint32_t len_fbucket_n(uint32_t len) {
    if (!len) return 0;
    uint32_t bl = 0;
    for (uint32_t v = len; v; v >>= 1) ++bl;
    const uint32_t sub = bl >= 3 ? (len >> (bl - 3)) & 3u : (len << (3 - bl)) & 3u;
    return 4 * bl + sub;
}
// fb_cap > 0: every tile at or above that fine bucket shares it (the forward's work follows the
// depth at which its pixels terminate, not the list length, once the list is long: such tiles are
// then issued in no particular order among themselves; gsr_set_option "fwd_order_cap")
__device__ __forceinline__ uint32_t len_fbucket(uint2 r, uint32_t fb_cap = 0) {
    const uint32_t len = r.y - r.x;
    if (!len) return 0;
    const uint32_t bl = 32 - __clz(len);
    const uint32_t sub = bl >= 3 ? (len >> (bl - 3)) & 3u : (len << (3 - bl)) & 3u;
    const uint32_t b = 4 * bl + sub;
    return fb_cap && b > fb_cap ? fb_cap : b;
}
// Bucket-count words of the row binning's tile order (k_tiles_scatter counts the non-empty fine
// buckets, k_tile_order_counted ranks the tiles): counts at [0, 132), positions at [256, 388).
constexpr int TILE_BUCKET_WORDS = 512, TILE_BUCKET_POS = 256;
__device__ __forceinline__ void zero16(void* p, size_t n4, size_t tid, size_t nthreads) {
    uint4* q = static_cast<uint4*>(p);
    for (size_t i = tid; i < n4; i += nthreads) q[i] = make_uint4(0u, 0u, 0u, 0u);
}

inline size_t sort_blocks(size_t n) { return n ? cdiv(n, SORT_TILE) : 0; }
constexpr int MAX_SORT_PASSES = 4;

// Workspaces of the single-pass (decoupled look-back) scan and radix sort: tile
// counters, pass histograms and per-tile status words, zeroed before each use.
struct ScanWs {
    void* base;
    size_t bytes;
    uint32_t* counter;
    uint64_t* status;
};
inline size_t scan_ws_bytes(size_t n) { return ALIGN + cdiv(n > 0 ? n : 1, SCAN_TILE) * 8; }
inline ScanWs scan_ws(size_t n, void* p) {
    char* c = static_cast<char*>(p);
    return {p, scan_ws_bytes(n), reinterpret_cast<uint32_t*>(c), reinterpret_cast<uint64_t*>(c + ALIGN)};
}
// Sort workspace header: words [0, passes) are the look-back tile counters, words
// [SPAN_WORD, SPAN_WORD + 2) the OR of the keys and of their complements (k_radix_hist);
// [TALLY_WORD, TALLY_WORD + 2) one 64-bit word: blocks done << 40 | tally sum (k_radix_hist).
constexpr int SPAN_WORD = 16, TALLY_WORD = 18;
struct SortWs {
    void* base;
    size_t header;      // bytes of counter + pass histograms
    uint32_t* counter;  // [passes] tile counters (look-back mode)
    uint32_t* hist;     // [passes][RADIX] global digit histograms (look-back mode)
    uint64_t* status;   // [passes][tiles][RADIX] look-back status words
    uint32_t* table;    // [RADIX][tiles] per-tile histograms (table mode; aliases status)
    void* scan;         // scan workspace of the table (table mode)
};
constexpr int MIN_SORT_ITEMS = 4;
inline size_t sort_tiles(size_t n, int items) { return n ? cdiv(n, (size_t)SORT_THREADS * items) : 0; }
size_t sort_grp_status_words(size_t nt);
inline size_t sort_ws_bytes(size_t n, int passes) {
    const size_t nt = sort_tiles(n, MIN_SORT_ITEMS);
    // look-back status words of either look-back mode (the grouped one adds a word row per group
    // of tiles; sort_lb_zero_bytes must never exceed this)
    const size_t lb = (size_t)passes * sort_grp_status_words(nt) * 8;
    const size_t tb = align_up(nt * RADIX * 4) + scan_ws_bytes(nt * RADIX);
    return ALIGN + align_up((size_t)MAX_SORT_PASSES * RADIX * 4) + (lb > tb ? lb : tb);
}
// Status words of one grouped look-back pass over nt tiles (binning.hip: per tile, then per
// group of tiles, RADIX words each).
// Bytes of the workspace a look-back sort of n keys in `passes` passes needs zeroed (either
// look-back mode: the grouped one's status words are the larger).
inline size_t sort_lb_zero_bytes(size_t n, int passes, int items) {
    return ALIGN + align_up((size_t)MAX_SORT_PASSES * RADIX * 4) +
           (size_t)passes * sort_grp_status_words(sort_tiles(n, items)) * 8;
}
inline SortWs sort_ws(size_t n, void* p) {
    char* c = static_cast<char*>(p);
    const size_t hdr = ALIGN + align_up((size_t)MAX_SORT_PASSES * RADIX * 4);
    const size_t nt = sort_tiles(n, MIN_SORT_ITEMS);
    return {p, hdr, reinterpret_cast<uint32_t*>(c), reinterpret_cast<uint32_t*>(c + ALIGN),
            reinterpret_cast<uint64_t*>(c + hdr), reinterpret_cast<uint32_t*>(c + hdr),
            c + hdr + align_up(nt * RADIX * 4)};
}

// binning_rows.hip workspace sizes (used by the layouts below)
size_t rows_bin_geom_ws_bytes(size_t P, int gy);
size_t rows_bin_ws_bytes(size_t cap);

// ---- geometry buffer (reference GeometryState, rasterizer_impl.cu:155-171) ----
struct GeomLayout {
    size_t rec, tiles_touched, depth_keys, clamped, rect, order, order_alt, dkeys_alt, offsets, ws,
        ws_scan, rect32, rect32_alt, rect32_sorted, shjac, og, btot, bbase, bytes;
};
// Record slots are numbered in Gaussian-index order, per block of SLOT_BLOCK Gaussians (the
// preprocess's blocks): Gaussian g's instance slots start at goff[g] + bbase[g / SLOT_BLOCK], where
// goff (the second word of GeomLayout::og[g]) is the exclusive scan of the tile counts inside g's
// block and bbase[b] the slots of the blocks before b (block_bases, binning.hip, from the blocks'
// totals btot).
constexpr int SLOT_BLOCK = 256;
inline GeomLayout geom_layout(size_t P) {
    GeomLayout L{};
    size_t o = 0;
    auto take = [&](size_t bytes) { size_t r = o; o = align_up(o + bytes); return r; };
    L.rec = take(P * 64);
    L.tiles_touched = take(P * 4);
    L.depth_keys = take(P * 4);
    L.clamped = take(P);
    L.rect = take(P * 8);
    L.order = take(P * 4);
    L.order_alt = take(P * 4);
    L.dkeys_alt = take(P * 4);
    L.offsets = take(P * 4);
    // depth sort; afterwards the row binning's level-1 table (binning_rows.hip)
    L.ws = take(std::max(sort_ws_bytes(P, MAX_SORT_PASSES), rows_bin_geom_ws_bytes(P, 255)));
    L.ws_scan = take(scan_ws_bytes(P));              // tiles_touched scan
    // tile rect packed as x0 | y0 << 8 | x1 << 16 | y1 << 24 (grids up to 255 x 255 tiles):
    // the depth sort carries it, so the scan and the duplicate read it in depth order
    // instead of gathering tiles_touched[g] / rect[g] at random
    L.rect32 = take(P * 4);
    L.rect32_alt = take(P * 4);
    L.rect32_sorted = take(P * 4);
    // d(rgb)/d(dir) of the SH colour, 9 x 64 floats per 64 Gaussians (preprocess writes
    // it, the backward reads it instead of the 192-B SH rows; preprocess.hip sh_dir_jacobian)
    L.shjac = take(cdiv(P, 64) * 64 * 9 * 4);
    // (opacity, in-block first record slot) of each Gaussian, for the per-Gaussian backward (which
    // recomputes the conic and so reads no 64-B record: the record's 32-B half cost a scattered
    // sector read); one 8-B stream instead of two 4-B ones
    L.og = take(P * 8);
    L.btot = take(cdiv(P, (size_t)SLOT_BLOCK) * 4);
    L.bbase = take(cdiv(P, (size_t)SLOT_BLOCK) * 4);
    L.bytes = o + ALIGN;
    return L;
}

// ---- binning buffer (reference BinningState, rasterizer_impl.cu:181-194) ----
struct BinLayout {
    size_t tkeys, tkeys_alt, vals_alt, slot_vals, slot_gid, gid_alt, point_list, written, ws, bytes;
};
inline BinLayout bin_layout(size_t I) {
    BinLayout L{};
    size_t o = 0;
    auto take = [&](size_t bytes) { size_t r = o; o = align_up(o + bytes); return r; };
    L.tkeys = take(I * 4);
    L.tkeys_alt = take(I * 4);
    L.vals_alt = take(I * 4);
    L.slot_vals = take(I * 4);
    L.slot_gid = take(I * 4);
    L.gid_alt = take(I * 4);
    L.point_list = take(I * 4);
    L.written = take(cdiv(I, 16) * 16);  // backward: 1 byte per instance slot (zeroed by the tile sort's last pass)
    L.ws = take(std::max(sort_ws_bytes(I, MAX_SORT_PASSES), rows_bin_ws_bytes(I)));  // tile sort or row binning
    L.bytes = o + ALIGN;
    return L;
}

// ---- backward scratch: per-instance gradient records ----
// Backward scratch: one 48-B gradient record per instance slot.  (64-B records, whole 32-B sectors
// per record, measured slower: the per-Gaussian gather touches more lines, round 5.)
constexpr int CONTRIB_STRIDE = 12;
inline size_t scratch_bytes(size_t I) { return align_up(I * CONTRIB_STRIDE * sizeof(float)) + ALIGN; }

// ---- image buffer (reference ImageState, rasterizer_impl.cu:173-179) ----
// After the T entries of the tile order (img buffer), the render schedule:
//   sched[SCHED_WORDS]  written by the tile-order kernels: [SCHED_FWD_SPLIT] = how many of
//                       the heaviest tiles the forward splits over two waves;
//   bq_cnt[BQ_BUCKETS], bq_list[BQ_BUCKETS][T]: the backward's queue -- the forward files
//                       every tile it rendered under its depth (deepest contributor, in
//                       steps of BQ_STEP list positions) and the backward walks the buckets
//                       deepest first;
//   tdone[T]:           split forward tiles: sum over finished halves of (depth << 1) | 1.
// bq_cnt and tdone are zeroed by the tile-order kernels.  A queue entry is a tile index with a
// list-segment kind in bits 30-31 (BQ_WHOLE / BQ_FRONT / BQ_BACK, render.hip): a tile replayed
// deeper than the forward's checkpoint position sched[SCHED_CKPT] is filed as two entries, so a
// bucket holds up to 2T entries.
constexpr int SCHED_FWD_SPLIT = 0, SCHED_FWD_QUARTER = 1, SCHED_CKPT = 2, SCHED_WORDS = 4;
constexpr int BQ_BUCKETS = 64, BQ_STEP = 16;
struct TileSched {
    uint32_t *sched, *bq_cnt, *tdone, *bq_list;
};
__host__ __device__ inline TileSched tile_sched(uint32_t* order, int T) {
    TileSched s;
    s.sched = order + T;
    s.bq_cnt = s.sched + SCHED_WORDS;
    s.tdone = s.bq_cnt + BQ_BUCKETS;
    s.bq_list = s.tdone + T;
    return s;
}
__host__ __device__ inline size_t bq_cap(size_t T) { return 2 * T; }  // entries per bucket
inline size_t tile_sched_words(size_t T) { return T + SCHED_WORDS + BQ_BUCKETS + T + BQ_BUCKETS * bq_cap(T); }
// depth (1-based deepest contributor) -> backward bucket; 0 = nothing to replay
__host__ __device__ inline uint32_t depth_bucket(uint32_t d) {
    const uint32_t b = (d + BQ_STEP - 1) / BQ_STEP;
    return b < (uint32_t)BQ_BUCKETS ? b : (uint32_t)BQ_BUCKETS - 1;
}
// Forward checkpoint of a tile (render.hip, list segments): 9 channels x 4 quadrants x 64 lanes
// floats -- the backward's replay state at the checkpoint position (render.hip publish_depth).
constexpr int CKPT_FLOATS = 9 * TILE_PIX;
struct ImgLayout {
    size_t ranges, n_contrib, order, ckpt, bytes;
    int gx, gy;
};
inline ImgLayout img_layout(int W, int H) {
    ImgLayout L{};
    L.gx = (W + BX - 1) / BX;
    L.gy = (H + BY - 1) / BY;
    size_t T = (size_t)L.gx * L.gy;
    size_t o = 0;
    auto take = [&](size_t bytes) { size_t r = o; o = align_up(o + bytes); return r; };
    L.ranges = take(T * 8);
    L.n_contrib = take(T * TILE_PIX * 4);  // tile-major: [tile][local pixel]
    L.order = take(tile_sched_words(T) * 4);  // heavy-first tile order + the render schedule (TileSched)
    L.ckpt = take(T * CKPT_FLOATS * 4);       // forward checkpoints for the backward's list segments
    L.bytes = o + ALIGN;
    return L;
}

inline char* aligned_base(void* p) {
    uintptr_t u = reinterpret_cast<uintptr_t>(p);
    return reinterpret_cast<char*>((u + ALIGN - 1) & ~(uintptr_t)(ALIGN - 1));
}

// ---- launchers (defined in the .hip files) ----
// preprocess.hip
void launch_preprocess(const gsr_settings& s, const gsr_inputs& in, int gx, int gy, float4* rec,
                       int* radii, uint32_t* tiles_touched, uint32_t* depth_keys, uint8_t* clamped,
                       ushort4* rect, uint32_t* rect32, float* shjac, float2* og, uint32_t* btot,
                       void* zero_a, size_t zero_a_bytes, void* zero_b, size_t zero_b_bytes, hipStream_t st);
// the packed rect (GeomLayout::rect32) fits grids of up to 255 x 255 tiles (4080 px)
inline bool rect_packable(int gx, int gy) { return gx <= 255 && gy <= 255; }
void launch_mark_visible(int P, const float* means3D, const float* view, uint8_t* present, hipStream_t st);
// Per-view inputs of the multi-view per-Gaussian backward (preprocess.hip).
struct MvView {
    const int* radii;
    const uint32_t* tiles_touched;
    const float2* og;     // the view's forward GeomLayout::og (opacity, in-block first slot)
    const uint32_t* bbase;
    const uint8_t* clamped;
    const float* contrib;
    const uint8_t* written;
    const float* shjac;  // the view's SH direction Jacobian (its forward's GeomLayout::shjac)
    const float* view;
    const float* proj;
    const float* campos;
    float* dmeans2D;
    int W, H;
    float tanfovx, tanfovy;
};
struct MvArgs {
    int B;
    MvView v[GSR_MAX_VIEWS];
};
// SH exchange rows of one view (gsr_sh_rows_floats): the view's clamped colour
// gradient dRGB [P,3], then its camera centre (4 floats) at a 64-float boundary.
__host__ __device__ inline size_t sh_rows_campos(int P) { return ((size_t)3 * P + 63) & ~(size_t)63; }
__host__ __device__ inline size_t sh_rows_floats(int P) { return sh_rows_campos(P) + 64; }
void launch_gaussian_backward_multiview(int P, int D, int M, float scale_modifier, const gsr_inputs& in,
                                        const MvArgs& a, const gsr_grads& g, float* shx, bool defer_sh,
                                        hipStream_t st);
// dsh [P,M,3] = sum over V views' rows of basis(dir) x dRGB (reads means3D and the rows only)
void launch_sh_backward(int P, int D, int M, const float* means3D, int V, const float* shx, float* dsh,
                        hipStream_t st);
void launch_gaussian_backward(const gsr_settings& s, const gsr_inputs& in, const int* radii,
                              const uint32_t* tiles_touched, const float2* og, const uint32_t* bbase,
                              const uint8_t* clamped, const float* contrib, const uint8_t* written,
                              const float* shjac, const gsr_grads& g, float* shx, hipStream_t st);
// binning.hip
// Optional last-pass outputs of a sort: ranges[key] = [first, last + 1) of each key's run in
// the sorted order (atomicMin/atomicMax per run and tile; empty keys keep {~0u, 0}, which
// k_tile_order turns into {0, 0}); the sorted keys themselves are then not written.  zero
// / zero16: a buffer of zero16 x 16 B cleared on the way.
struct SortFinal {
    uint2* ranges;
    uint4* zero;
    size_t zero16;
    bool no_keys;  // the sorted keys are not needed: the last pass writes none
    // optional: the histogram kernel (look-back / grouped modes) also sums tally[0, n) and its
    // last block stores the sum into tally_host (a host-mapped word): num_rendered from the
    // depth sort's first kernel, before any binning kernel has run
    // (set true when it does: the caller must then leave the word to it alone -- a later
    // store of the same call's value could land after the host has re-armed the word for
    // its next call)
    const uint32_t* tally = nullptr;
    uint32_t* tally_host = nullptr;
    bool* tally_used = nullptr;
    // optional: the record slots' block bases (SLOT_BLOCK): bb_base[b] = sum of bb_tot[0, b) for
    // b < bb_n, computed by the histogram kernel's block 0 (or a one-block kernel when the sort
    // runs without it)
    const uint32_t* bb_tot = nullptr;
    uint32_t* bb_base = nullptr;
    uint32_t bb_n = 0;
};
void launch_radix_sort(const uint32_t* keys_in, const uint32_t* vals_in /*NULL = identity*/, uint32_t* keys_tmp,
                       uint32_t* vals_tmp, uint32_t* keys_out, uint32_t* vals_out, size_t n, int key_bits,
                       void* ws, bool ws_zeroed, hipStream_t st, const uint32_t* vals2_in = nullptr,
                       uint32_t* vals2_tmp = nullptr, uint32_t* vals2_out = nullptr, const SortFinal* fin = nullptr,
                       bool skip_sentinel = false, const uint32_t* n_dev = nullptr);
// n_dev: optional device word; the sort then covers min(*n_dev, n) keys (n sizes the grids)
int depth_sort_passes();
int sort_lb_items();
bool sort_uses_lookback(size_t n);
void set_sort_lookback_max(size_t n);
void set_sort_grouped(bool on);  // grouped look-back passes for sorts of <= 1024 tiles (default on)
bool sort_grouped_size(size_t n);  // a key-only sort of n keys (e.g. the depth sort) takes the grouped passes
// bytes of the sort workspace a look-back / grouped sort of n keys needs zeroed (its tile size)
size_t sort_zero_bytes(size_t n, int passes);
// Both tile-order launchers also write order[T + SCHED_FWD_SPLIT]: the number of tiles in
// length buckets >= the forward's split bucket (set_split_buckets; 0 = no split), and zero
// the backward queue's counters (TileSched).  bwd_depth: the backward splits tiles whose
// deepest contributor is at least this deep (0 = no split; a render.hip launch argument).
void set_split_buckets(int fwd_bucket, int bwd_depth);  // negative: the built-in default
// forward quarter tiles: tiles with n >= 2^(B-1) get four waves (0 = off; negative: default)
void set_split4_bucket(int fwd_bucket);
// forward tile order: list lengths at or above this many instances share one schedule bucket (0 = off)
void set_fwd_order_cap(int instances);
// forward: the two halves of a split tile on blocks b and b + 8 (one XCD) instead of b and b + 1
void set_fwd_xcd_pairs(int on);
uint32_t fwd_order_fb_cap();
int split4_fwd_bucket();
int split_bwd_depth();
int split_fwd_bucket();
void launch_tile_order(uint2* ranges, int T, uint32_t* order, hipStream_t st);
// the same from bucket counts already taken (row binning): many blocks, no serial pass
void launch_tile_order_counted(const uint2* ranges, int T, uint32_t* bucket_words, uint32_t* order, hipStream_t st);
// value(j) = src[gather[j]] (gather != NULL), src[j], or, with rect_mode, the tile count
// (x1 - x0)(y1 - y0) of the packed rect src[j]
void launch_scan_inclusive_gather(const uint32_t* src, const uint32_t* gather_idx, uint32_t* out, size_t n,
                                  void* ws, bool ws_zeroed, hipStream_t st, uint32_t* host_total = nullptr,
                                  bool rect_mode = false);
// exclusive scan of n (or min(n, *n_dev)) values; W zeroed beforehand
void launch_scan_exclusive(const uint32_t* src, uint32_t* out, size_t n, const uint32_t* n_dev, const ScanWs& W,
                           hipStream_t st);
// binning_rows.hip: tile lists by row-then-tile expansion (grids up to 255 x 255 tiles).
// stage 0: level 1 (rows); 1: level 2 (point_list, written flags
// cleared); 2: ranges + heavy-first tile order.  geom_ws: rows_bin_geom_ws_bytes(P, gy)
// bytes (the depth sort's workspace, free by then); bin_ws: rows_bin_ws_bytes(cap).
// fused: level 1 also computes the depth-ordered instance offsets (written to offsets, as the
// depth-order scan writes them; num_rendered also to host_total when non-NULL), so the scan need
// not run first.
void launch_rows_binning(int P, int gx, int gy, const uint32_t* order, uint32_t* offsets, const uint32_t* rect,
                         void* geom_ws, void* bin_ws, uint32_t* e_gid, uint32_t* e_x,
                         uint32_t* point_list, uint2* ranges, uint32_t* tile_order,
                         uint4* written, size_t written16, size_t cap, const uint32_t* n_total, hipStream_t st,
                         int stage, bool fused, uint32_t* host_total);
void launch_duplicate(int P, const uint32_t* order, const uint32_t* offsets, const uint32_t* tiles_touched,
                      const ushort4* rect, const uint32_t* rect_sorted, int gx, uint32_t* tkeys,
                      uint32_t* slot_gid, uint2* ranges, int T, uint32_t cap, hipStream_t st);
// render.hip
// sched = order + T (TileSched).  Forward grid 2T single-wave blocks in the heavy-first
// order (split tiles first); backward grid T two-wave blocks over the forward's depth
// queue, deepest first (tiles at least split_bwd_depth() deep on both waves of a block).
void launch_render_forward(int W, int H, int gx, int gy, const uint32_t* order, uint32_t* sched,
                           const uint2* ranges, const uint32_t* point_list, const float4* rec, const float* bg,
                           float* out_color, float* out_depth, float* out_alpha, float* out_segment,
                           uint32_t* n_contrib, float* ckpt, hipStream_t st);
void launch_render_backward(int W, int H, int gx, int gy, const uint32_t* order, uint32_t* sched,
                            const uint2* ranges, const uint32_t* point_list, const uint32_t* bbase,
                            const float4* rec, const float* bg, const float* alpha, const uint32_t* n_contrib,
                            const float* dL_dcolor, const float* dL_dsegment, const float* dL_ddepth,
                            const float* dL_dalpha, float* contrib, uint8_t* written, const float* ckpt,
                            hipStream_t st);
// list-segment checkpoint position of the render forward (0 = off; gsr_set_option "bwd_ckpt")
void set_bwd_ckpt(int pos);
int bwd_ckpt();

uint32_t higher_msb(uint32_t n);

}  // namespace gsr
