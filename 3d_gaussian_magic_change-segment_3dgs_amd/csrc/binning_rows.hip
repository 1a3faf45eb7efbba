// binning_rows.hip -- per-tile instance lists by two stable expansions of the
// depth-ordered Gaussians, rows first, then tiles.  Replaces, for grids of up to
// 255 x 255 tiles (4080 x 4080 px), the reference's duplicateWithKeys +
// DeviceRadixSort::SortPairs + identifyTileRanges (DGR/cuda_rasterizer/
// rasterizer_impl.cu:68-138, :291-322); wider grids keep binning.hip's duplicate + radix
// sort.
//
// Input: the Gaussians in depth order r = 0..P-1 (binning.hip's depth sort): the id
// order[r], the packed tile rectangle rect[r] = x0 | y0 << 8 | x1 << 16 | y1 << 24 and
// the inclusive scan offsets[r] of the tile counts (the instance slots of r start at
// offsets[r - 1]).  Output: point_list (Gaussian ids grouped by tile, by depth inside a
// tile: the reference's sorted (tile << 32 | depth) order, bit for bit), ranges and the
// heavy-first tile order.  (An instance's record slot is not written here: the render backward
// forms it from the Gaussian's first slot and its rectangle, gsr_internal.h SLOT_BLOCK.)
//
//   level 1 (rows):  Gaussian r -> one entry per tile row y0..y1-1 of its rectangle,
//                    grouped by row, in depth order inside a row;
//   level 2 (tiles): row entry -> one instance per tile x0..x1-1 of its row, grouped by
//                    tile, in depth order inside a tile.
// Each level is a chunked stable counting sort (bucket = row, or tile column of the row):
//   count:   per chunk of RB_CH items, the bucket histogram (a difference array in LDS:
//            two atomics per item) -> table[bucket][chunk];
//   scan:    one exclusive scan of the bucket-major table (k_scan) gives every
//            (bucket, chunk) the position of its first item;
//   scatter: the chunk marks in LDS, per bucket, the RB_CH-bit set of its items that
//            cover the bucket; an item's rank in its bucket is the popcount of the set
//            bits below its own (stable and deterministic, no ordered atomics); the
//            chunk's output is assembled in LDS in bucket order and written as runs.
// Level-2 chunks never straddle rows (row y's entries form ceil(R_y / RB_CH) chunks), so
// a chunk's buckets are the gx columns of one row.  Bytes per instance: 4 written
// (point_list) plus ~12 written and read per row entry (~2.9 instances each at
// the metric scene), against ~52 for duplicate + two radix passes over (key, slot, id).
#include "gsr_internal.h"

#ifdef GSR_SORT_TRACE
// Timeline build (tools/sort_trace.py): per block of k_rows_scatter [0], k_tiles_count [1] and
// k_tiles_scatter [2]: s_memrealtime at entry, after the row map, at the end, chunks | XCC << 16.
__device__ unsigned long long g_gsr_btrace[3][4096][4];
extern "C" __attribute__((visibility("default"))) int gsr_bin_trace_read(unsigned long long* host, int reset) {
    if (hipMemcpyFromSymbol(host, HIP_SYMBOL(g_gsr_btrace), sizeof(g_gsr_btrace)) != hipSuccess) return -1;
    if (reset) {
        void* d = nullptr;
        if (hipGetSymbolAddress(&d, HIP_SYMBOL(g_gsr_btrace)) != hipSuccess) return -1;
        if (hipMemset(d, 0, sizeof(g_gsr_btrace)) != hipSuccess) return -1;
    }
    return 0;
}
#define BT_T(var) const unsigned long long var = __builtin_amdgcn_s_memrealtime();
#define BT_END(k, t0, t1, nch)                                                                          \
    if (threadIdx.x == 0 && blockIdx.x < 4096) {                                                       \
        unsigned long long* w_ = g_gsr_btrace[k][blockIdx.x];                                          \
        w_[0] = t0; w_[1] = t1; w_[2] = __builtin_amdgcn_s_memrealtime();                              \
        w_[3] = (unsigned long long)(nch) | ((unsigned long long)(__builtin_amdgcn_s_getreg((20) | (0 << 6) | (3 << 11)) & 15u) << 16); \
    }
#else
#define BT_T(var)
#define BT_END(k, t0, t1, nch)
#endif

namespace gsr {

namespace {

constexpr int RB_CH1 = 1024;          // level 1: depth-ordered Gaussians per chunk = threads per block
constexpr int RB_S1 = RB_CH1 / 32 + 1; // its LDS words per bucket row (bitmask words + pad)
constexpr int RB_STAGE1 = 4 * RB_CH1;  // its row entries assembled in LDS (more: direct writes)
#ifndef GSR_RB_CH
#define GSR_RB_CH 512
#endif
// Level-2 grid: 768 blocks = three 512-thread blocks per CU on 256 CUs (k_tiles_scatter's LDS
// allows three), one resident round grid-striding over the chunks (2048 blocks ran ~2.7 rounds
// of block start-up: tile sort 0.0688 -> 0.0653 ms at the metric scene)
#ifndef GSR_RB_GRID2
#define GSR_RB_GRID2 768
#endif
constexpr int RB_CH = GSR_RB_CH;      // level 2: row entries per chunk = threads per block
static_assert(RB_CH == 512 || RB_CH == 1024, "level-2 chunks: 16 or 32 bitmask words per bucket, at most 1024 threads");
constexpr int RB_W = RB_CH / 32;      // bitmask words per bucket
// LDS words per bucket row of bits / pre: one pad word so that the words of different
// buckets fall in different banks (with a stride of 16 words, lanes touching buckets 4
// apart hit one bank: 13M bank-conflict cycles per tile-scatter launch at the metric scene)
constexpr int RB_S = RB_W + 1;
constexpr int RB_STAGE = 4 * RB_CH;    // outputs a chunk assembles in LDS (more: direct writes)
constexpr int RB_MAXB = 256;          // buckets per chunk (<= 255 rows / columns)
constexpr int RB_GRID2 = GSR_RB_GRID2;  // blocks of the level-2 kernels (grid-stride over chunks)

// Inclusive scans of x over groups of W = 16, 32 or 64 consecutive lanes with DPP (row_shr
// inside a 16-lane row, then row_bcast15 / row_bcast31 across rows): no LDS round trip per step
// (the ds_bpermute shuffles they replace were the latency chain of every level-2 chunk).
template <int W>
__device__ __forceinline__ uint32_t scan_incl(uint32_t x) {
    // row_shr stays inside a 16-lane row, not inside a smaller group: W < 16 would add the previous
    // group's lanes (wrong ranks, so wrong point_list entries)
    static_assert(W == 16 || W == 32 || W == 64, "scan_incl: groups of 16, 32 or 64 lanes");
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xF, 0xF, true);  // row_shr:1
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xF, 0xF, true);  // row_shr:2
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xF, 0xF, true);  // row_shr:4
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xF, 0xF, true);  // row_shr:8
    if (W >= 32) x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xA, 0xF, false);  // row_bcast:15
    if (W >= 64) x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xC, 0xF, false);  // row_bcast:31
    return x;
}

// Exclusive scan of n <= 256 LDS values v[0..n) by wave 0 (4 values per lane): out[k] =
// sum of v[0..k); *tot = sum of all.  Every thread of the block must call it (barrier).
__device__ void lds_scan256(const uint32_t* v, int n, uint32_t* out, uint32_t* tot) {
    if (threadIdx.x < 64) {
        const int l = threadIdx.x;
        uint32_t a[4], s = 0;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int k = 4 * l + i;
            a[i] = k < n ? v[k] : 0u;
            s += a[i];
        }
        const uint32_t x = scan_incl<64>(s);
        uint32_t e = x - s;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int k = 4 * l + i;
            if (k < n) out[k] = e;
            e += a[i];
        }
        if (l == 63) *tot = x;
    }
    __syncthreads();
}

// bits[b * RB_S + w]: bit i of word w = item 32 w + i of the chunk covers bucket b.
// pre[b * RB_S + w] = items of bucket b in words < w; cnt[b] = items of bucket b.
// CH: items per chunk (= threads per block), CH / 32 bitmask words per bucket row of
// CH / 32 + 1 LDS words.  Every word is loaded before the first scan (one LDS latency).
template <int CH>
__device__ void bucket_prefix(const uint32_t* bits, int nb, uint32_t* pre, uint32_t* cnt) {
    constexpr int W = CH / 32, S = W + 1;
    constexpr int PER_WAVE = 64 / W, STEP = PER_WAVE * (CH / 64), ITER = (RB_MAXB + STEP - 1) / STEP;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int bl = PER_WAVE * wave + lane / W, w = lane % W;
    uint32_t c[ITER];
#pragma unroll
    for (int i = 0; i < ITER; ++i) {
        const int b = bl + i * STEP;
        c[i] = b < nb ? (uint32_t)__popc(bits[b * S + w]) : 0u;
    }
#pragma unroll
    for (int i = 0; i < ITER; ++i) {
        if (i * STEP >= nb) break;  // uniform
        const int b = bl + i * STEP;
        const uint32_t x = scan_incl<W>(c[i]);
        if (b < nb) {
            pre[b * S + w] = x - c[i];
            if (w == W - 1) cnt[b] = x;
        }
    }
    __syncthreads();
}

__device__ __forceinline__ void unpack_rect(uint32_t pr, int& x0, int& y0, int& x1, int& y1) {
    x0 = (int)(pr & 255u);
    y0 = (int)((pr >> 8) & 255u);
    x1 = (int)((pr >> 16) & 255u);
    y1 = (int)(pr >> 24);
}

// ---------------------------------------------------------------- level 1 --
// table1[y * nch1 + c] = Gaussians of chunk c (RB_CH1 depth-ordered Gaussians) covering row y.
// fused: table1[gy * nch1 + c] = the chunk's instances (sum of its Gaussians' tile counts), a row
// after the others, so that the one scan of table1 also yields every chunk's first instance
// slot (k_rows_scatter then computes the per-Gaussian offsets: no separate scan of the counts).
__global__ void __launch_bounds__(RB_CH1) k_rows_count(int P, int gy, int nch1, const uint32_t* __restrict__ rect,
                                                      uint32_t* __restrict__ table1, void* zero, size_t nzero16,
                                                      int fused) {
    __shared__ int d[RB_MAXB + 1];
    __shared__ uint32_t e[RB_MAXB + 1];
    __shared__ uint32_t tot, s_inst;
    for (int i = threadIdx.x; i <= gy; i += RB_CH1) d[i] = 0;
    if (threadIdx.x == 0) s_inst = 0;
    __syncthreads();
    const int r = blockIdx.x * RB_CH1 + threadIdx.x;
    uint32_t ntile = 0;
    if (r < P) {
        int x0, y0, x1, y1;
        unpack_rect(rect[r], x0, y0, x1, y1);
        if (x1 > x0 && y1 > y0) {
            atomicAdd(&d[y0], 1);
            atomicAdd(&d[y1], -1);
            ntile = (uint32_t)((x1 - x0) * (y1 - y0));
        }
    }
    if (fused) {
        const uint32_t ws = (uint32_t)__builtin_amdgcn_readlane((int)scan_incl<64>(ntile), 63);
        if ((threadIdx.x & 63) == 0 && ws) atomicAdd(&s_inst, ws);
    }
    __syncthreads();
    lds_scan256(reinterpret_cast<const uint32_t*>(d), gy + 1, e, &tot);  // e[y + 1] = rows' counts
    for (int y = threadIdx.x; y < gy; y += RB_CH1) table1[(size_t)y * nch1 + blockIdx.x] = e[y + 1];
    if (fused && threadIdx.x == 0) table1[(size_t)gy * nch1 + blockIdx.x] = s_inst;
    // the scan's status words, cleared after the rect load (one in-order vmcnt for loads and stores)
    zero16(zero, nzero16, (size_t)blockIdx.x * RB_CH1 + threadIdx.x, (size_t)gridDim.x * RB_CH1);
}

// Level-1 entries (E1, grouped by row): e_gid = Gaussian id, e_x = x0 | x1 << 8.
// Dynamic LDS: bits + pre, 2 x gy x RB_S1 words, sized by the grid rather than the 255
// bound (gy = 68 at 1080p: 18 KB; 67 KB at gy = 255, covered by the 4080-px-tall case of
// tests/test_gpu_parity.py::test_rows_binning_matches_radix_path).  Every global load is
// issued before the first barrier.
// fused (k_rows_count's extra table row): the Gaussians' instance offsets are computed here --
// the chunk's first slot from the scanned table plus an exclusive block scan of the tile counts
// -- and written to offsets (inclusive, as the scan of binning.hip writes them); the thread of
// Gaussian P - 1 also stores num_rendered into host-mapped memory when host_total is given.
// Otherwise the offsets are read (the depth-order scan ran).
__global__ void __launch_bounds__(RB_CH1) k_rows_scatter(int P, int gy, int nch1, const uint32_t* __restrict__ order,
                                                        uint32_t* __restrict__ offsets,
                                                        const uint32_t* __restrict__ rect,
                                                        const uint32_t* __restrict__ base1,
                                                        uint32_t* __restrict__ e_gid,
                                                        uint32_t* __restrict__ e_x, uint32_t cap, int fused,
                                                        uint32_t* host_total) {
    extern __shared__ uint32_t dyn[];
    uint32_t* bits = dyn;
    uint32_t* pre = dyn + gy * RB_S1;
    __shared__ uint32_t cnt[RB_MAXB], lst[RB_MAXB], gb[RB_MAXB];
    __shared__ uint32_t s_gid[RB_STAGE1], s_x[RB_STAGE1];
    __shared__ uint32_t tot;
    __shared__ uint32_t s_wsum[RB_CH1 / 64];
    BT_T(bt0)
    const int tid = threadIdx.x;
    const int r = blockIdx.x * RB_CH1 + tid;
    int x0 = 0, y0 = 0, x1 = 0, y1 = 0;
    uint32_t g = 0, off = 0, cbase = 0;
    if (r < P) {
        unpack_rect(rect[r], x0, y0, x1, y1);
        g = order[r];
        if (!fused) off = r == 0 ? 0u : offsets[r - 1];
    }
    if (fused) cbase = base1[(size_t)gy * nch1 + blockIdx.x] - base1[(size_t)gy * nch1];
    for (int i = tid; i < gy * RB_S1; i += RB_CH1) bits[i] = 0;
    for (int y = tid; y < gy; y += RB_CH1) gb[y] = base1[(size_t)y * nch1 + blockIdx.x];
    const uint32_t ntile = (x1 > x0 && y1 > y0) ? (uint32_t)((x1 - x0) * (y1 - y0)) : 0u;
    uint32_t incl = 0;
    if (fused) {
        incl = scan_incl<64>(ntile);
        if ((tid & 63) == 63) s_wsum[tid >> 6] = incl;
    }
    __syncthreads();
    if (fused) {
        uint32_t wpre = 0;
        for (int w = 0; w < (tid >> 6); ++w) wpre += s_wsum[w];
        off = cbase + wpre + incl - ntile;
        if (r < P) {
            offsets[r] = off + ntile;
            if (r == P - 1 && host_total)
                __hip_atomic_store(host_total, off + ntile, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
    const bool vis = x1 > x0 && y1 > y0;
    const uint32_t bit = 1u << (tid & 31), wd = (uint32_t)tid >> 5;
    if (vis)
        for (int y = y0; y < y1; ++y) atomicOr(&bits[y * RB_S1 + wd], bit);
    __syncthreads();
    bucket_prefix<RB_CH1>(bits, gy, pre, cnt);
    lds_scan256(cnt, gy, lst, &tot);
    const bool staged = tot <= (uint32_t)RB_STAGE1;  // uniform
    if (vis) {
        const uint32_t below = bit - 1u;
        for (int y = y0; y < y1; ++y) {
            const uint32_t rank = pre[y * RB_S1 + wd] + (uint32_t)__popc(bits[y * RB_S1 + wd] & below);
            const uint32_t xr = (uint32_t)x0 | ((uint32_t)x1 << 8) | ((uint32_t)y << 16);
            if (staged) {
                const uint32_t lp = lst[y] + rank;
                s_gid[lp] = g;
                s_x[lp] = xr;
            } else {
                const uint32_t gp = gb[y] + rank;
                if (gp < cap) {
                    e_gid[gp] = g;
                    e_x[gp] = xr & 0xFFFFu;
                }
            }
        }
    }
    if (!staged) return;
    __syncthreads();
    for (uint32_t i = tid; i < tot; i += RB_CH1) {
        const uint32_t xr = s_x[i], y = xr >> 16;
        const uint32_t gp = gb[y] + (i - lst[y]);
        if (gp < cap) {
            e_gid[gp] = s_gid[i];
            e_x[gp] = xr & 0xFFFFu;
        }
    }
    BT_END(0, bt0, bt0, 1)
}

// ---------------------------------------------------------------- level 2 --
// Row map of the level-2 chunks from the level-1 table: rs[y] = first entry of row y
// (rs[gy] = entries), nsub[y] = chunks of row y, c0[y] = first chunk of row y; returns the
// number of chunks.  Clamped to the entry capacity (a speculative stage B whose
// num_rendered exceeds the buffer writes nothing past it; its results are discarded).
struct RowMap {
    uint32_t rs[RB_MAXB + 1], nsub[RB_MAXB + 1], c0[RB_MAXB + 1], nch2;
};
__device__ void build_row_map(RowMap& m, int gy, int nch1, const uint32_t* table1, const uint32_t* base1,
                              uint32_t cap) {
    const int tid = threadIdx.x;
    for (int y = tid; y < gy; y += blockDim.x) m.rs[y] = min(base1[(size_t)y * nch1], cap);
    if (tid == 0) {
        const size_t last = (size_t)gy * nch1 - 1;
        m.rs[gy] = min(base1[last] + table1[last], cap);
    }
    __syncthreads();
    for (int y = tid; y < gy; y += blockDim.x) m.nsub[y] = (uint32_t)cdiv(m.rs[y + 1] - m.rs[y], RB_CH);
    __syncthreads();
    lds_scan256(m.nsub, gy, m.c0, &m.nch2);
    if (tid == 0) m.c0[gy] = m.nch2;
    __syncthreads();
}
// row of chunk c (< nch2, block-uniform): the last row y with c0[y] <= c = the number of rows
// y < gy with c0[y] <= c, minus one (c0 is non-decreasing, c0[0] = 0), counted by four
// ballots per wave over independent LDS reads (a binary search was 8 dependent LDS reads)
__device__ __forceinline__ int chunk_row(const RowMap& m, int gy, uint32_t c) {
    const int lane = threadIdx.x & 63;
    uint32_t v[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) v[i] = lane + 64 * i < gy ? m.c0[lane + 64 * i] : 0xFFFFFFFFu;
    int k = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) k += __popcll(__ballot(v[i] <= c));
    return k - 1;
}
__device__ __forceinline__ size_t tile_slot(const RowMap& m, int gx, int y, int x, uint32_t s) {
    return (size_t)gx * m.c0[y] + (size_t)x * m.nsub[y] + s;  // (row, column, sub-chunk) order
}

// table2[tile_slot(y, x, s)] = entries of sub-chunk s of row y covering column x.
// Also clears the tile ranges (rows without entries keep {0, 0}: rasterizer_impl.cu:316).
__global__ void __launch_bounds__(RB_CH) k_tiles_count(int gx, int gy, int nch1, const uint32_t* __restrict__ table1,
                                                       const uint32_t* __restrict__ base1,
                                                       const uint32_t* __restrict__ e_x, uint32_t* __restrict__ table2,
                                                       uint32_t* __restrict__ len2, uint32_t cap, void* zero,
                                                       size_t nzero16, uint2* __restrict__ ranges,
                                                       uint32_t* __restrict__ bucket_words) {
    __shared__ RowMap m;
    __shared__ int d[RB_MAXB + 1];
    __shared__ uint32_t e[RB_MAXB + 1];
    __shared__ uint32_t tot;
    BT_T(bt0)
    build_row_map(m, gy, nch1, table1, base1, cap);
    BT_T(bt1)
    if (blockIdx.x == 0 && threadIdx.x == 0) *len2 = (uint32_t)gx * m.nch2;
    uint32_t nch_ = 0;
    // chunk c -> row, sub-chunk and this thread's entry (the next chunk's entry is loaded while
    // the current one is counted, and waited for before the current chunk's stores: gfx950's
    // vmcnt is one in-order counter for loads and stores)
    struct Chunk {
        int y;
        uint32_t s, xr;
        bool valid;
    };
    auto fetch = [&](uint32_t c) {
        Chunk k;
        k.y = chunk_row(m, gy, c);
        k.s = c - m.c0[k.y];
        const uint32_t e0 = m.rs[k.y] + k.s * RB_CH, n = min((uint32_t)RB_CH, m.rs[k.y + 1] - e0);
        k.valid = threadIdx.x < n;
        k.xr = k.valid ? e_x[e0 + threadIdx.x] : 0u;
        return k;
    };
    uint32_t c = blockIdx.x;
    Chunk cur{};
    if (c < m.nch2) cur = fetch(c);
    while (c < m.nch2) {
        ++nch_;
        for (int i = threadIdx.x; i <= gx; i += RB_CH) d[i] = 0;
        __syncthreads();
        if (cur.valid) {
            atomicAdd(&d[cur.xr & 255u], 1);
            atomicAdd(&d[(cur.xr >> 8) & 255u], -1);
        }
        const uint32_t cn = c + gridDim.x;
        Chunk nxt{};
        if (cn < m.nch2) nxt = fetch(cn);
        __syncthreads();
        lds_scan256(reinterpret_cast<const uint32_t*>(d), gx + 1, e, &tot);  // e[x + 1] = column counts
        asm volatile("" ::"v"(nxt.xr));
        for (int x = threadIdx.x; x < gx; x += RB_CH) table2[tile_slot(m, gx, cur.y, x, cur.s)] = e[x + 1];
        // no barrier: d was last read before lds_scan256's barrier, e is rewritten after two more
        c = cn;
        cur = nxt;
    }
    // clears for the next kernels, issued after this kernel's loads (one in-order vmcnt: stores
    // ahead of the row map's loads would delay them)
    zero16(zero, nzero16, (size_t)blockIdx.x * RB_CH + threadIdx.x, (size_t)gridDim.x * RB_CH);  // scan-2 words
    for (int t = blockIdx.x * RB_CH + threadIdx.x; t < gx * gy; t += gridDim.x * RB_CH) ranges[t] = make_uint2(0u, 0u);
    // (strided: GSR_RB_CH may be below TILE_BUCKET_WORDS; a word left set would push
    // k_tile_order_counted's positions past the order array)
    if (blockIdx.x == 0)
        for (int t = threadIdx.x; t < TILE_BUCKET_WORDS; t += RB_CH) bucket_words[t] = 0u;
    BT_END(1, bt0, bt1, nch_)
    (void)nch_;
}

// point_list; the ranges of every non-empty row (from the chunk s = 0 of the
// row: the first entry of (y, x, 0) and of the next column, clamped to the capacity, empty
// tiles {0, 0}); also clears the backward's written-slot flags.  The next chunk's entries
// and bucket bases are loaded while the current one is ranked (software pipeline: a chunk
// otherwise waits on two dependent global round trips).  Dynamic LDS: bits + pre,
// 2 x gx x RB_S words.
__global__ void __launch_bounds__(RB_CH) k_tiles_scatter(int gx, int gy, int nch1, const uint32_t* __restrict__ table1,
                                                         const uint32_t* __restrict__ base1,
                                                         const uint32_t* __restrict__ base2,
                                                         const uint32_t* __restrict__ e_gid,
                                                         const uint32_t* __restrict__ e_x,
                                                         uint32_t* __restrict__ point_list, uint32_t cap,
                                                         const uint32_t* __restrict__ n_total,
                                                         uint2* __restrict__ ranges, uint4* zero, size_t nzero16,
                                                         uint32_t* __restrict__ bucket_words, uint32_t fb_cap) {
    extern __shared__ uint32_t dyn[];
    uint32_t* bits = dyn;
    uint32_t* pre = dyn + gx * RB_S;
    __shared__ RowMap m;
    __shared__ uint32_t cnt[RB_MAXB], lst[RB_MAXB], gb[RB_MAXB];
    __shared__ uint32_t s_gid[RB_STAGE], s_gp[RB_STAGE];
    __shared__ uint32_t tot;
    __shared__ uint32_t s_bc[FINE_BUCKETS];  // this row's tiles per fine schedule bucket (k_tile_order_counted)
    BT_T(bt0)
    const int tid = threadIdx.x;
    build_row_map(m, gy, nch1, table1, base1, cap);
    BT_T(bt1)
    uint32_t nch_ = 0;
    const uint32_t len2 = (uint32_t)gx * m.nch2, itot = min(*n_total, cap);
    const uint32_t bit = 1u << (tid & 31), wd = (uint32_t)tid >> 5, below = bit - 1u;
    // chunk c -> its row, sub-chunk, entries, this thread's entry and bucket base (prefetch)
    struct Chunk {
        int y;
        uint32_t s, e0, n, g, xr, gbv;
    };
    auto fetch = [&](uint32_t c) {
        Chunk k;
        k.y = chunk_row(m, gy, c);
        k.s = c - m.c0[k.y];
        k.e0 = m.rs[k.y] + k.s * RB_CH;
        k.n = min((uint32_t)RB_CH, m.rs[k.y + 1] - k.e0);
        k.g = k.xr = 0;
        if ((uint32_t)tid < k.n) {
            k.g = e_gid[k.e0 + tid];
            k.xr = e_x[k.e0 + tid];
        }
        k.gbv = tid < gx ? base2[tile_slot(m, gx, k.y, tid, k.s)] : 0u;
        return k;
    };
    uint32_t c = blockIdx.x;
    Chunk cur;
    if (c < m.nch2) cur = fetch(c);
    while (c < m.nch2) {
        const int y = cur.y;
        for (int i = tid; i < gx * RB_S; i += RB_CH) bits[i] = 0;
        if (tid < gx) gb[tid] = cur.gbv;
        if (tid < FINE_BUCKETS) s_bc[tid] = 0;
        __syncthreads();
        const bool live = (uint32_t)tid < cur.n;
        const int x0 = (int)(cur.xr & 255u), x1 = (int)((cur.xr >> 8) & 255u);
        if (live)
            for (int x = x0; x < x1; ++x) atomicOr(&bits[x * RB_S + wd], bit);
        if (cur.s == 0 && tid < gx) {  // this row's tile ranges
            const uint32_t a = min(gb[tid], cap);
            uint32_t b;
            if (tid + 1 < gx) {
                b = base2[tile_slot(m, gx, y, tid + 1, 0)];
            } else {
                const size_t nx = (size_t)gx * m.c0[y + 1];
                b = nx < len2 ? base2[nx] : itot;
            }
            b = min(b, cap);
            const uint2 rg = b > a ? make_uint2(a, b) : make_uint2(0u, 0u);
            ranges[(size_t)y * gx + tid] = rg;
            const uint32_t bk = len_fbucket(rg, fb_cap);
            if (bk) atomicAdd(&s_bc[bk], 1u);
        }
        const uint32_t cn = c + gridDim.x;
        Chunk nxt{};
        if (cn < m.nch2) nxt = fetch(cn);  // in flight while this chunk is ranked
        __syncthreads();
        if (cur.s == 0 && tid < FINE_BUCKETS && s_bc[tid]) atomicAdd(&bucket_words[tid], s_bc[tid]);
        bucket_prefix<RB_CH>(bits, gx, pre, cnt);
        lds_scan256(cnt, gx, lst, &tot);
        const bool staged = tot <= (uint32_t)RB_STAGE;  // uniform
        if (live)
            for (int x = x0; x < x1; ++x) {
                const uint32_t rank = pre[x * RB_S + wd] + (uint32_t)__popc(bits[x * RB_S + wd] & below);
                if (staged) {
                    const uint32_t lp = lst[x] + rank;
                    s_gid[lp] = cur.g;
                    s_gp[lp] = gb[x] + rank;
                } else {
                    const uint32_t gp = gb[x] + rank;
                    if (gp < cap) point_list[gp] = cur.g;
                }
            }
        // The next chunk's prefetched values are waited for here, before this chunk's output
        // stores: gfx950 counts loads and stores in one in-order vmcnt, so a first use after
        // a store loop of unknown length becomes vmcnt(0) -- a wait for every store's
        // acknowledgement once per chunk.
        asm volatile("" ::"v"(nxt.g), "v"(nxt.xr), "v"(nxt.gbv));
        if (staged) {
            __syncthreads();
            for (uint32_t i = tid; i < tot; i += RB_CH) {
                const uint32_t gp = s_gp[i];
                if (gp < cap) point_list[gp] = s_gid[i];
            }
        } else {
            __syncthreads();  // gb and bits are rewritten at the top of the next chunk
        }
        // (staged: bits and gb were last read before the barrier above; the staging arrays
        // are next written after three more barriers)
        c = cn;
        cur = nxt;
        ++nch_;
    }
    // the backward's written-slot flags, cleared after this kernel's loads (in-order vmcnt)
    for (size_t i = (size_t)blockIdx.x * RB_CH + tid; i < nzero16; i += (size_t)gridDim.x * RB_CH)
        zero[i] = make_uint4(0u, 0u, 0u, 0u);
    BT_END(2, bt0, bt1, nch_)
    (void)nch_;
}

}  // namespace

size_t rows_bin_geom_ws_bytes(size_t P, int gy) {
    const size_t n1 = (size_t)(gy + 1) * cdiv(P > 0 ? P : 1, RB_CH1);  // + the fused mode's instance row
    return 2 * align_up(n1 * 4) + scan_ws_bytes(n1);
}

size_t rows_bin_ws_bytes(size_t cap) {
    const size_t n2 = (size_t)RB_MAXB * (RB_MAXB + cdiv(cap > 0 ? cap : 1, RB_CH));
    return ALIGN + align_up(TILE_BUCKET_WORDS * 4) + 2 * align_up(n2 * 4) + scan_ws_bytes(n2);
}

void launch_rows_binning(int P, int gx, int gy, const uint32_t* order, uint32_t* offsets, const uint32_t* rect,
                         void* geom_ws, void* bin_ws, uint32_t* e_gid, uint32_t* e_x,
                         uint32_t* point_list, uint2* ranges, uint32_t* tile_order,
                         uint4* written, size_t written16, size_t cap, const uint32_t* n_total, hipStream_t st,
                         int stage, bool fused, uint32_t* host_total) {
    const int nch1 = (int)cdiv(P, RB_CH1);
    const size_t n1a = (size_t)(gy + 1) * nch1;              // table rows (+ the fused mode's instance row)
    const size_t n1 = (size_t)(gy + (fused ? 1 : 0)) * nch1;  // entries scanned
    char* gw = static_cast<char*>(geom_ws);
    uint32_t* table1 = reinterpret_cast<uint32_t*>(gw);
    uint32_t* base1 = reinterpret_cast<uint32_t*>(gw + align_up(n1a * 4));
    void* scan1 = gw + 2 * align_up(n1a * 4);
    const ScanWs S1 = scan_ws(n1, scan1);
    const size_t n2 = (size_t)gx * (gy + cdiv(cap, RB_CH));  // table-2 entries bound
    char* bw = static_cast<char*>(bin_ws);
    uint32_t* len2 = reinterpret_cast<uint32_t*>(bw);
    uint32_t* bucket_words = reinterpret_cast<uint32_t*>(bw + ALIGN);
    char* bw2 = bw + ALIGN + align_up(TILE_BUCKET_WORDS * 4);
    uint32_t* table2 = reinterpret_cast<uint32_t*>(bw2);
    uint32_t* base2 = reinterpret_cast<uint32_t*>(bw2 + align_up(n2 * 4));
    void* scan2 = bw2 + 2 * align_up(n2 * 4);
    const ScanWs S2 = scan_ws(n2, scan2);
    const uint32_t cap32 = (uint32_t)(cap < 0xFFFFFFFFull ? cap : 0xFFFFFFFFull);
    if (stage == 0) {  // level 1: rows
        hipLaunchKernelGGL(k_rows_count, dim3(nch1), dim3(RB_CH1), 0, st, P, gy, nch1, rect, table1, S1.base,
                           cdiv(S1.bytes, 16), (int)fused);
        launch_scan_exclusive(table1, base1, n1, nullptr, S1, st);
        hipLaunchKernelGGL(k_rows_scatter, dim3(nch1), dim3(RB_CH1), 2 * gy * RB_S1 * 4, st, P, gy, nch1, order,
                           offsets, rect, base1, e_gid, e_x, cap32, (int)fused, host_total);
    } else if (stage == 1) {  // level 2: tiles (+ ranges)
        const int grid2 = (int)std::min<size_t>(RB_GRID2, gy + cdiv(cap, RB_CH));
        hipLaunchKernelGGL(k_tiles_count, dim3(grid2), dim3(RB_CH), 0, st, gx, gy, nch1, table1, base1, e_x, table2,
                           len2, cap32, S2.base, cdiv(S2.bytes, 16), ranges, bucket_words);
        launch_scan_exclusive(table2, base2, n2, len2, S2, st);
        hipLaunchKernelGGL(k_tiles_scatter, dim3(grid2), dim3(RB_CH), 2 * gx * RB_S * 4, st, gx, gy, nch1, table1,
                           base1, base2, e_gid, e_x, point_list, cap32, n_total, ranges, written,
                           written16, bucket_words, fwd_order_fb_cap());
    } else {  // heavy-first tile order from the bucket counts (binning.hip)
        launch_tile_order_counted(ranges, gx * gy, bucket_words, tile_order, st);
    }
}

}  // namespace gsr
