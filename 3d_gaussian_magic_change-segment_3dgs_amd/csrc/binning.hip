// binning.hip -- prefix scan, stable LSD radix sort, key duplication and tile
// ranges.  Replaces the reference's CUB DeviceScan / DeviceRadixSort calls and
// the duplicateWithKeys / identifyTileRanges kernels
// (DGR/cuda_rasterizer/rasterizer_impl.cu:68-138, :281, :304-322).
//
// Ordering contract (bit-exact with the reference): the reference sorts
// (tile << 32 | depth_bits) with a stable sort whose input is emitted in
// Gaussian-index order, so inside a tile the order is (depth_bits, gaussian).
// gsr reaches the same total order in two cheaper steps:
//   1. stable sort of the P depth keys (value = gaussian id)  -> order[]
//   2. instances are emitted in that depth order, so the instance slot u is
//      increasing in (depth, gaussian); a stable sort of the I tile keys with
//      u as the value then yields (tile, depth, gaussian) -- the reference's
//      order -- after only ceil(log2(T)/8) passes over I instead of
//      ceil((32+log2 T)/8) passes over 64-bit keys.
#include "gsr_internal.h"

#ifdef GSR_SORT_TRACE
// Timeline build (tools/sort_trace.py): per tile of each look-back radix pass (slot = shift /
// 8), s_memrealtime (100 MHz) at entry, after the tile index, after the ranking barrier, after
// the look-back barrier and at the end, plus the XCC id.
__device__ unsigned long long g_gsr_strace[5][1024][6];  // [4]: k_radix_hist blocks
extern "C" __attribute__((visibility("default"))) int gsr_sort_trace_read(unsigned long long* host, int reset) {
    if (hipMemcpyFromSymbol(host, HIP_SYMBOL(g_gsr_strace), sizeof(g_gsr_strace)) != hipSuccess) return -1;
    if (reset) {
        void* d = nullptr;
        if (hipGetSymbolAddress(&d, HIP_SYMBOL(g_gsr_strace)) != hipSuccess) return -1;
        if (hipMemset(d, 0, sizeof(g_gsr_strace)) != hipSuccess) return -1;
    }
    return 0;
}
#define ST_T(var) const unsigned long long var = __builtin_amdgcn_s_memrealtime();
#else
#define ST_T(var)
#endif

namespace gsr {

namespace {

__device__ __forceinline__ uint64_t lanemask_lt() {
    const uint32_t lane = threadIdx.x & 63;
    return lane ? (~0ull >> (64 - lane)) : 0ull;
}

// ------------------------------------------------- decoupled look-back ----
// Single-pass prefix sums (scan, radix scatter) publish one 64-bit status word per
// (tile, lane of the sum): flag in the high half (1 = tile aggregate, 2 = inclusive
// prefix), value in the low half.  Tiles take their index from an atomic counter in
// launch order, so every tile a block waits on has already started: the spin always
// terminates.  Status words are zeroed (memset) before each launch.  A status word
// carries its own payload, so relaxed agent-scope atomics suffice: they are coherent
// across the XCDs' L2s (sc1) without the L2 write-back / invalidate that
// release / acquire ordering costs on MI355X.
constexpr uint64_t LB_AGG = 1ull << 32, LB_PRE = 2ull << 32;
__device__ __forceinline__ void lb_store(uint64_t* p, uint64_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t lb_load(uint64_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// Sum of the values of tiles 0..t-1 of one column (stride between tiles).
__device__ __forceinline__ uint32_t lb_lookback(uint64_t* col, size_t stride, int t) {
    uint32_t excl = 0;
    int i = t - 1;
    while (i >= 0) {
        const uint64_t w = lb_load(col + (size_t)i * stride);
        const uint32_t f = (uint32_t)(w >> 32);
        if (f == 0) {
            __builtin_amdgcn_s_sleep(1);
            continue;
        }
        excl += (uint32_t)w;
        if (f == 2) break;
        --i;
    }
    return excl;
}
// The same, reading N predecessors per dependent step (one thread per column; used by
// the radix scatter, where 256 digit columns walk back in parallel).  N = 1, 2, 4, 8, 16,
// 32 measured at the 1M-key depth sort: 87, 84, 83, 84, 87, 93 us -- the look-back loads,
// not the chain length, are what a wider window costs.
#ifndef GSR_LB_STEP
#define GSR_LB_STEP 8
#endif
template <int N>
__device__ __forceinline__ uint32_t lb_lookback_n(uint64_t* col, size_t stride, int t) {
    uint32_t excl = 0;
    int i = t - 1;
    while (true) {
        uint64_t w[N];
#pragma unroll
        for (int k = 0; k < N; ++k) {
            const int j = i - k;
            w[k] = j >= 0 ? lb_load(col + (size_t)j * stride) : LB_PRE;
        }
        int consumed = 0;
        bool done = false, stall = false;
#pragma unroll
        for (int k = 0; k < N; ++k) {
            if (done || stall) continue;
            const uint32_t f = (uint32_t)(w[k] >> 32);
            if (f == 0) {
                stall = true;
                continue;
            }
            excl += (uint32_t)w[k];
            ++consumed;
            done = f == 2;
        }
        if (done) return excl;
        i -= consumed;
        if (stall) __builtin_amdgcn_s_sleep(1);
    }
}
// The same, by a whole wave over a window of 64 predecessors per step: lane l inspects
// tile i - l; the window is summed up to the nearest inclusive prefix (tiles below 0
// count as an inclusive 0).  A window with an unpublished tile before that point is
// re-read.  O(t / 64) dependent loads instead of O(t) when many tiles start together.
__device__ __forceinline__ uint32_t lb_lookback_wave(uint64_t* col, int t) {
    const int lane = threadIdx.x & 63;
    uint32_t excl = 0;
    int i = t - 1;
    while (true) {
        const int j = i - lane;
        const uint64_t w = j >= 0 ? lb_load(col + j) : LB_PRE;
        const uint32_t f = (uint32_t)(w >> 32);
        const uint64_t inc = __ballot(f == 2u), unpub = __ballot(f == 0u);
        const int stop = inc ? (int)__builtin_ctzll(inc) : 63;
        const uint64_t need = stop == 63 ? ~0ull : ((2ull << stop) - 1ull);
        if (unpub & need) {
            __builtin_amdgcn_s_sleep(1);
            continue;
        }
        uint32_t v = lane <= stop ? (uint32_t)w : 0u;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) v += (uint32_t)__shfl_xor((int)v, o, 64);
        excl += v;
        if (inc) return excl;
        i -= 64;
    }
}
__device__ __forceinline__ int lb_tile_index(uint32_t* counter) {
    __shared__ int s_tile;
    if (threadIdx.x == 0) s_tile = (int)atomicAdd(counter, 1u);
    __syncthreads();
    return s_tile;
}

// Exclusive scan over a block of WAVES wave64s.  wsum: __shared__ uint32_t[WAVES].
template <int WAVES>
__device__ __forceinline__ uint32_t block_exclusive_scan_w(uint32_t v, uint32_t* wsum, uint32_t* total) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    uint32_t x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        uint32_t y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
    }
    if (lane == 63) wsum[wid] = x;
    __syncthreads();
    uint32_t pre = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < WAVES; ++w) {
        const uint32_t s = wsum[w];
        if (w < wid) pre += s;
        tot += s;
    }
    __syncthreads();
    *total = tot;
    return pre + x - v;
}

// ---------------------------------------------------------------- scan ----
// out[i] = sum_{j<=i (INCLUSIVE) / j<i} value(j), value(j) = gather ? src[gather[j]] : src[j], in one
// pass: each tile of SCAN_TILE values is staged through LDS (coalesced loads/stores),
// reduced, its prefix found by look-back, then scanned.
// n_dev (optional): a device word; the scan then covers min(n, *n_dev) values (n sizes the
// grid; tiles past the device count return at once -- no later tile depends on them).
template <bool INCLUSIVE>
__global__ void __launch_bounds__(SCAN_THREADS) k_scan(const uint32_t* __restrict__ src,
                                                       const uint32_t* __restrict__ gather, size_t n,
                                                       uint32_t* __restrict__ out, uint64_t* status,
                                                       uint32_t* counter, uint32_t* host_total, int rect_mode,
                                                       const uint32_t* n_dev) {
    __shared__ uint32_t tile[SCAN_TILE + SCAN_TILE / 32];
    __shared__ uint32_t wsum[SCAN_THREADS / 64];
    __shared__ uint32_t s_excl;
    if (n_dev) n = min(n, (size_t)*n_dev);
    const int t = lb_tile_index(counter);
    const size_t base = (size_t)t * SCAN_TILE;
    if (base >= n && t > 0) return;  // uniform: past the device count
    auto pad = [](int i) { return i + (i >> 5); };
    uint32_t v[SCAN_ITEMS], sum = 0;
    if (gather) {
        uint32_t gi[SCAN_ITEMS];
#pragma unroll
        for (int i = 0; i < SCAN_ITEMS; ++i) {
            const size_t idx = base + i * SCAN_THREADS + threadIdx.x;
            gi[i] = idx < n ? gather[idx] : 0u;
        }
#pragma unroll
        for (int i = 0; i < SCAN_ITEMS; ++i) {
            const size_t idx = base + i * SCAN_THREADS + threadIdx.x;
            v[i] = idx < n ? src[gi[i]] : 0u;
        }
    } else {
#pragma unroll
        for (int i = 0; i < SCAN_ITEMS; ++i) {
            const size_t idx = base + i * SCAN_THREADS + threadIdx.x;
            v[i] = idx < n ? src[idx] : 0u;
        }
        if (rect_mode)  // packed rect -> tile count (x1 - x0)(y1 - y0)
#pragma unroll
            for (int i = 0; i < SCAN_ITEMS; ++i)
                v[i] = (((v[i] >> 16) & 255u) - (v[i] & 255u)) * ((v[i] >> 24) - ((v[i] >> 8) & 255u));
    }
#pragma unroll
    for (int i = 0; i < SCAN_ITEMS; ++i) tile[pad(i * SCAN_THREADS + threadIdx.x)] = v[i];
    __syncthreads();
#pragma unroll
    for (int i = 0; i < SCAN_ITEMS; ++i) {
        v[i] = tile[pad(threadIdx.x * SCAN_ITEMS + i)];
        sum += v[i];
    }
    uint32_t total;
    uint32_t pre = block_exclusive_scan_w<SCAN_THREADS / 64>(sum, wsum, &total);
    if (threadIdx.x < 64) {  // wave 0: publish, look back over 64 tiles at a time, publish
        uint32_t excl = 0;
        if (t == 0) {
            if (threadIdx.x == 0) lb_store(status, LB_PRE | total);
        } else {
            if (threadIdx.x == 0) lb_store(status + t, LB_AGG | total);
            excl = lb_lookback_wave(status, t);
            if (threadIdx.x == 0) lb_store(status + t, LB_PRE | (excl + total));
        }
        if (threadIdx.x == 0) s_excl = excl;
    }
    __syncthreads();
    pre += s_excl;
#pragma unroll
    for (int i = 0; i < SCAN_ITEMS; ++i) {
        const uint32_t nx = pre + v[i];
        tile[pad(threadIdx.x * SCAN_ITEMS + i)] = INCLUSIVE ? nx : pre;
        pre = nx;
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < SCAN_ITEMS; ++i) {
        const int li = i * SCAN_THREADS + threadIdx.x;
        const size_t idx = base + li;
        if (idx < n) out[idx] = tile[pad(li)];
        // the grand total, straight into host-mapped memory (system-scope store): the
        // host polls it instead of waiting for a copy + stream synchronisation
        if (host_total && idx == n - 1)
            __hip_atomic_store(host_total, tile[pad(li)], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

// ---------------------------------------------------------- radix sort ----
// Digit histograms of every pass at once (one read of the keys): LDS counters per
// block, then one global atomic per (pass, digit, block).  hist[p * RADIX + d].
// Also which key bits vary over the keys that matter (all keys, or all but the 0xFFFFFFFF
// sentinel when skip_sentinel: culled Gaussians of the depth sort, whose position is
// irrelevant): span[0] = OR of the keys, span[1] = OR of their complements (zero-initialised
// words), so bit b varies iff it is set in span[0] & span[1].  A pass whose digit bits are all
// constant over the keys that matter is the identity on them and is skipped (identity_pass).
// The ORs are wave-reduced with DPP row rotations and four v_readlane (round 2 took min / max
// digit spans per pass with 48 dependent lane shuffles per wave: 6.8 us of LDS phase per block).
// Keys per thread of k_radix_hist: fewer, fuller blocks mean fewer global atomics at the
// end (one per nonzero (pass, digit) per block).
// 16 waves x 4 keys per thread per block (a 4-wave block with 16 keys per thread left
// under one wave per SIMD at 1M keys: latency-bound, 16 us; 2 or 8 keys measured no better
// there).  Larger sorts keep the grid near 366 blocks (8 keys per thread up to 4M keys, 16
// beyond): at 6M keys the 1465 blocks of 4096 keys issued ~1.5M global atomics (41 us).
constexpr int HIST_THREADS = 1024;
inline int hist_items(size_t n) { return n <= (2u << 20) ? 4 : n <= (4u << 20) ? 8 : 16; }
__device__ __forceinline__ uint32_t wave_or(uint32_t x) {
    x |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x121, 0xF, 0xF, false);  // row_ror:1
    x |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x122, 0xF, 0xF, false);  // row_ror:2
    x |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x124, 0xF, 0xF, false);  // row_ror:4
    x |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x128, 0xF, 0xF, false);  // row_ror:8
    return (uint32_t)__builtin_amdgcn_readlane((int)x, 0) | (uint32_t)__builtin_amdgcn_readlane((int)x, 16) |
           (uint32_t)__builtin_amdgcn_readlane((int)x, 32) | (uint32_t)__builtin_amdgcn_readlane((int)x, 48);
}
// A pass over digit bits [shift, shift + bits) is the identity on the keys that matter.
__device__ __forceinline__ bool identity_pass(const uint32_t* span, int shift, int bits) {
    return (((span[0] & span[1]) >> shift) & ((1u << bits) - 1u)) == 0u;
}
// Record-slot block bases (gsr_internal.h SLOT_BLOCK): bbase[b] = sum of btot[0, b), b < nb, in
// segments of BB_SEG totals, segment k by the histogram kernel's k-th extra block (the blocks run
// concurrently: one block doing every segment made the kernel ~9 us longer at C5).  Block k adds
// up the totals before its segment (all loads up front) and scans its own (BB_RUN consecutive
// totals per thread, the runs' sums scanned across the block).
constexpr int BB_RUN = 8, BB_SEG = BB_RUN * HIST_THREADS;
__device__ __forceinline__ uint32_t block_sum(uint32_t x, uint32_t* s_w) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) x += (uint32_t)__shfl_xor((int)x, o, 64);
    if ((threadIdx.x & 63) == 0) s_w[threadIdx.x >> 6] = x;
    __syncthreads();
    uint32_t t = 0;
#pragma unroll
    for (int w = 0; w < HIST_THREADS / 64; ++w) t += s_w[w];
    __syncthreads();
    return t;
}
__device__ void block_bases(const uint32_t* __restrict__ btot, uint32_t nb, uint32_t* __restrict__ bbase, uint32_t seg) {
    __shared__ uint32_t s_w[HIST_THREADS / 64];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const uint32_t r0 = seg * BB_SEG;
    // totals before the segment: up to 8 per thread per round, loaded together
    uint32_t pre_sum = 0;
    for (uint32_t c0 = 0; c0 < r0; c0 += BB_SEG) {
        uint32_t a[BB_RUN];
#pragma unroll
        for (int k = 0; k < BB_RUN; ++k) {
            const uint32_t i = c0 + (uint32_t)k * HIST_THREADS + threadIdx.x;
            a[k] = i < r0 ? btot[i] : 0u;
        }
#pragma unroll
        for (int k = 0; k < BB_RUN; ++k) pre_sum += a[k];
    }
    const uint32_t carry = r0 ? block_sum(pre_sum, s_w) : 0u;
    const uint32_t i0 = r0 + BB_RUN * threadIdx.x;
    uint32_t v[BB_RUN], s = 0;
#pragma unroll
    for (int k = 0; k < BB_RUN; ++k) {
        v[k] = i0 + k < nb ? btot[i0 + k] : 0u;
        s += v[k];
    }
    uint32_t x = s;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = (uint32_t)__shfl_up((int)x, o, 64);
        if (lane >= o) x += y;
    }
    if (lane == 63) s_w[wid] = x;
    __syncthreads();
    uint32_t pre = carry;
#pragma unroll
    for (int w = 0; w < HIST_THREADS / 64; ++w) pre += w < wid ? s_w[w] : 0u;
    pre += x - s;
#pragma unroll
    for (int k = 0; k < BB_RUN; ++k) {
        if (i0 + k < nb) bbase[i0 + k] = pre;
        pre += v[k];
    }
}
inline uint32_t block_base_segments(uint32_t nb) { return (nb + BB_SEG - 1) / BB_SEG; }
__global__ void __launch_bounds__(HIST_THREADS) k_block_bases(const uint32_t* __restrict__ btot, uint32_t nb,
                                                              uint32_t* __restrict__ bbase) {
    block_bases(btot, nb, bbase, blockIdx.x);
}

template <int HIST_ITEMS>
__global__ void __launch_bounds__(HIST_THREADS) k_radix_hist(const uint32_t* __restrict__ keys, size_t n,
                                                             int passes, int per_pass, int key_bits,
                                                             uint32_t* __restrict__ hist, uint32_t* span,
                                                             int skip_sentinel, const uint32_t* n_dev,
                                                             const uint32_t* __restrict__ tally,
                                                             unsigned long long* tally_word, uint32_t* tally_host,
                                                             const uint32_t* __restrict__ bb_tot, uint32_t bb_n,
                                                             uint32_t* __restrict__ bb_base) {
    // the record-slot block bases run on extra blocks past the histogram's (beside them: a
    // histogram block that also did them set the kernel's end, +3 us at the metric scene)
    const uint32_t nseg = bb_base ? (bb_n + BB_SEG - 1) / BB_SEG : 0u, hblocks = gridDim.x - nseg;
    if (blockIdx.x >= hblocks) {  // block-uniform
        block_bases(bb_tot, bb_n, bb_base, blockIdx.x - hblocks);
        return;
    }
    ST_T(st0)
    if (n_dev) n = min(n, (size_t)*n_dev);
    __shared__ uint32_t cnt[4][RADIX];
    __shared__ uint32_t s_span[3];
    if (threadIdx.x < RADIX)
#pragma unroll
        for (int p = 0; p < 4; ++p) cnt[p][threadIdx.x] = 0;
    if (threadIdx.x < 3) s_span[threadIdx.x] = 0;
    __syncthreads();
    uint32_t ork = 0, ornk = 0;
    // all loads issued before any use (a strided loop with one dependent load per
    // iteration is latency-bound)
    const size_t base = (size_t)blockIdx.x * HIST_THREADS * HIST_ITEMS + threadIdx.x;
    uint32_t kk[HIST_ITEMS], tsum = 0;
#pragma unroll
    for (int i = 0; i < HIST_ITEMS; ++i) {
        const size_t idx = base + (size_t)i * HIST_THREADS;
        kk[i] = idx < n ? keys[idx] : 0u;
    }
    if (tally) {
#pragma unroll
        for (int i = 0; i < HIST_ITEMS; ++i) {
            const size_t idx = base + (size_t)i * HIST_THREADS;
            tsum += idx < n ? tally[idx] : 0u;
        }
    }
#ifdef GSR_SORT_TRACE
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    ST_T(st1)
#endif
#pragma unroll
    for (int i = 0; i < HIST_ITEMS; ++i) {
        const size_t idx = base + (size_t)i * HIST_THREADS;
        const bool valid = idx < n;
        const uint32_t k = kk[i];
        const uint64_t vmask = __ballot(valid);
        const bool matters = valid && !(skip_sentinel && k == 0xFFFFFFFFu);
        if (matters) {
            ork |= k;
            ornk |= ~k;
        }
#pragma unroll
        for (int p = 0; p < 4; ++p) {
            if (p >= passes) break;
            const int shift = p * per_pass;
            const int bits = min(per_pass, key_bits - shift);
            const uint32_t d = (k >> shift) & ((1u << bits) - 1u);
            // wave-aggregated: a digit shared by the whole wave (the high digits of keys
            // with a narrow range) is one LDS atomic, not 64 serialised on one address
            const uint32_t d0 = __builtin_amdgcn_readfirstlane(d);
            if (__ballot(valid && d == d0) == vmask) {
                if ((threadIdx.x & 63) == 0 && vmask) atomicAdd(&cnt[p][d0], (uint32_t)__popcll(vmask));
            } else if (valid) {
                atomicAdd(&cnt[p][d], 1u);
            }
        }
    }
    ork = wave_or(ork);
    ornk = wave_or(ornk);
    if (tally) {
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) tsum += (uint32_t)__shfl_xor((int)tsum, o, 64);
    }
    if ((threadIdx.x & 63) == 0) {
        if (ork) atomicOr(&s_span[0], ork);
        if (ornk) atomicOr(&s_span[1], ornk);
        if (tsum) atomicAdd(&s_span[2], tsum);
    }
    __syncthreads();
    if (tally && threadIdx.x == 0) {
        // one 64-bit atomic carries both the sum and the count of blocks done, so the block
        // that completes the count holds the whole sum (no fences); sums < 2^40
        const unsigned long long mine = (1ull << 40) | s_span[2];
        const unsigned long long old =
            __hip_atomic_fetch_add(tally_word, mine, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if ((old >> 40) + 1 == hblocks)
            __hip_atomic_store(tally_host, (uint32_t)((old + mine) & ((1ull << 40) - 1)), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_SYSTEM);
    }
    ST_T(st2)
    if (threadIdx.x < RADIX)
        for (int p = 0; p < passes; ++p)
            if (cnt[p][threadIdx.x]) atomicAdd(&hist[p * RADIX + threadIdx.x], cnt[p][threadIdx.x]);
    if (threadIdx.x < 2 && s_span[threadIdx.x]) atomicOr(&span[threadIdx.x], s_span[threadIdx.x]);
#ifdef GSR_SORT_TRACE
    __syncthreads();
    if (threadIdx.x == 0 && blockIdx.x < 1024) {
        unsigned long long* w = g_gsr_strace[4][blockIdx.x];
        w[0] = st0; w[1] = st0; w[2] = st1; w[3] = st2; w[4] = __builtin_amdgcn_s_memrealtime();
        w[5] = __builtin_amdgcn_s_getreg((20) | (0 << 6) | (3 << 11)) & 15u;
    }
#endif
}

// Per-tile digit histogram -> hist[digit * ntiles + tile] (table-driven passes).  One
// LDS atomic per element: a ballot multisplit (one ballot per digit bit) made this
// kernel VALU-bound (tile sort 134 -> 120 us without it at the metric scene).
template <int ITEMS, int WAVES>
__global__ void __launch_bounds__(64 * WAVES) k_radix_upsweep(const uint32_t* __restrict__ keys, size_t n,
                                                              int shift, int bits, uint32_t* __restrict__ hist,
                                                              void* scan_ws, size_t scan_ws16, const uint32_t* n_dev) {
    if (n_dev) n = min(n, (size_t)*n_dev);
    constexpr int NT = 64 * WAVES;
    __shared__ uint32_t cnt[RADIX];
    zero16(scan_ws, scan_ws16, (size_t)blockIdx.x * NT + threadIdx.x, (size_t)gridDim.x * NT);
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const uint32_t ndig = 1u << bits, mask = ndig - 1u;
    for (int i = tid; i < RADIX; i += NT) cnt[i] = 0;
    __syncthreads();
    const size_t wbase = (size_t)blockIdx.x * (NT * ITEMS) + (size_t)wid * (64 * ITEMS);
    uint32_t key[ITEMS];
#pragma unroll
    for (int r = 0; r < ITEMS; ++r) {
        const size_t idx = wbase + (size_t)r * 64 + lane;
        key[r] = idx < n ? keys[idx] : 0u;
    }
#pragma unroll
    for (int r = 0; r < ITEMS; ++r) {
        const bool valid = wbase + (size_t)r * 64 + lane < n;
        const uint32_t digit = (key[r] >> shift) & mask;
        if (valid) atomicAdd(&cnt[digit], 1u);
    }
    __syncthreads();
    for (int d = tid; d < (int)ndig; d += NT) hist[(size_t)d * gridDim.x + blockIdx.x] = cnt[d];
}

// Stable scatter, staged through LDS, one launch per pass.  Wave w of the tile ranks the elements
// [1024 w, 1024 w + 1024) of the block's tile in 16 rounds of 64: a wave64
// multi-split by ballots gives each element its rank among equal digits of the
// round, and a per-wave digit counter in LDS (read by all lanes, then bumped by
// the digit's first lane -- ordered within the wave, no barrier) carries the
// rank across rounds.  One block scan then turns the 4 x 2^bits counters into
// block-local digit bases, a decoupled look-back over earlier tiles (per digit)
// gives the tile's global digit offsets, the tile is permuted into digit order in LDS, and
// written out with consecutive threads on consecutive positions of each digit's
// run (coalesced, unlike a direct per-element scatter).  Stable: element order
// inside a digit is (wave, round, lane) = input order.  vals_in == NULL means
// value = element index; vals2 is an optional second payload word.
// LB = true: the tile's global digit offsets come from a decoupled look-back over
// earlier tiles (one launch per pass; hist = the pass's global digit histogram).
// LB = false: they come from a scanned per-tile histogram table (hist[d * ntiles + t],
// k_radix_upsweep + k_scan<false>): more launches, but no look-back latency chain,
// which costs a cross-XCD round trip per hop on MI355X.
template <int ITEMS, int WAVES, bool LB>
__global__ void __launch_bounds__(64 * WAVES) k_radix_scatter(
    const uint32_t* __restrict__ keys_in, const uint32_t* __restrict__ vals_in, uint32_t* __restrict__ keys_out,
    uint32_t* __restrict__ vals_out, size_t n, int shift, int bits, const uint32_t* __restrict__ hist,
    uint64_t* status, uint32_t* counter, const uint32_t* __restrict__ vals2_in, uint32_t* __restrict__ vals2_out,
    SortFinal fin, const uint32_t* span, const uint32_t* n_dev) {
    constexpr int NT = 64 * WAVES, TILE = NT * ITEMS;
    ST_T(st0)
    if (n_dev) n = min(n, (size_t)*n_dev);
    for (size_t i = (size_t)blockIdx.x * NT + threadIdx.x; i < fin.zero16; i += (size_t)gridDim.x * NT)
        fin.zero[i] = make_uint4(0u, 0u, 0u, 0u);
    __shared__ uint32_t s_key[TILE], s_val[TILE], s_val2[TILE];
    __shared__ uint32_t wcnt[WAVES][RADIX];
    __shared__ uint32_t dbase[RADIX], gbase[RADIX];
    __shared__ uint32_t wsum[WAVES];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const uint32_t ndig = 1u << bits, mask = ndig - 1u;
    // span: the key bits that vary over the keys that matter (k_radix_hist)
    const bool ident = LB && span && identity_pass(span, shift, bits);
    const int t = LB ? lb_tile_index(counter) : (int)blockIdx.x;
    ST_T(st1)
    if (ident) {
        // Every key that matters has the same digit in this pass: a stable pass is the
        // identity on them, so the tile is copied through and the look-back chain is
        // skipped.  Uniform over the grid.
        for (size_t idx = (size_t)blockIdx.x * TILE + tid; idx < min(n, (size_t)(blockIdx.x + 1) * TILE);
             idx += NT) {
            const uint32_t k = keys_in[idx];
            if (keys_out) keys_out[idx] = k;
            vals_out[idx] = vals_in ? vals_in[idx] : (uint32_t)idx;
            if (vals2_out) vals2_out[idx] = vals2_in[idx];
            if (fin.ranges) {
                if (idx == 0 || keys_in[idx - 1] != k) atomicMin(&fin.ranges[k].x, (uint32_t)idx);
                if (idx == n - 1 || keys_in[idx + 1] != k) atomicMax(&fin.ranges[k].y, (uint32_t)(idx + 1));
            }
        }
#ifdef GSR_SORT_TRACE
        __syncthreads();
        if (threadIdx.x == 0 && t < 1024) {
            unsigned long long* w = g_gsr_strace[(shift >> 3) & 3][t];
            w[0] = st0; w[1] = st1; w[2] = 0; w[3] = 0; w[4] = __builtin_amdgcn_s_memrealtime();
            w[5] = __builtin_amdgcn_s_getreg((20) | (0 << 6) | (3 << 11)) & 15u;
        }
#endif
        return;
    }
#pragma unroll
    for (int i = 0; i < RADIX / 64; ++i) wcnt[wid][lane + 64 * i] = 0;
    const size_t bbase = (size_t)t * TILE;
    const size_t wbase = bbase + (size_t)wid * (64 * ITEMS);
    const uint64_t lt = lanemask_lt();
    uint32_t key[ITEMS], val[ITEMS], val2[ITEMS], rk[ITEMS];
#pragma unroll
    for (int r = 0; r < ITEMS; ++r) {
        const size_t idx = wbase + (size_t)r * 64 + lane;
        const bool valid = idx < n;
        key[r] = valid ? keys_in[idx] : 0u;
        val[r] = valid ? (vals_in ? vals_in[idx] : (uint32_t)idx) : 0u;
        val2[r] = (valid && vals2_in) ? vals2_in[idx] : 0u;
    }
#pragma unroll
    for (int r = 0; r < ITEMS; ++r) {
        const size_t idx = wbase + (size_t)r * 64 + lane;
        const bool valid = idx < n;
        const uint32_t digit = (key[r] >> shift) & mask;
        uint64_t peers = __ballot(valid);
        for (int b = 0; b < bits; ++b) {
            const bool set = (digit >> b) & 1u;
            const uint64_t m = __ballot(set);
            peers &= set ? m : ~m;
        }
        const uint32_t rank = __popcll(peers & lt);
        const uint32_t old = valid ? wcnt[wid][digit] : 0u;
        rk[r] = old + rank;
        if (valid && rank == 0) wcnt[wid][digit] = old + (uint32_t)__popcll(peers);
    }
    __syncthreads();
    ST_T(st2)
    // digit-major block offsets: dbase[d] = elements of digits < d; wave offsets inside d
    uint32_t tot = 0;
    if ((uint32_t)tid < ndig)
#pragma unroll
        for (int w = 0; w < WAVES; ++w) tot += wcnt[w][tid];
    uint32_t total;
    const uint32_t db = block_exclusive_scan_w<WAVES>(tot, wsum, &total);
    // global start of each digit (exclusive scan of the pass histogram)
    const uint32_t gstart =
        LB ? block_exclusive_scan_w<WAVES>((uint32_t)tid < ndig ? hist[tid] : 0u, wsum, &total) : 0u;
    if ((uint32_t)tid < ndig) {
        dbase[tid] = db;
        uint32_t o = db;
#pragma unroll
        for (int w = 0; w < WAVES; ++w) {
            const uint32_t cw = wcnt[w][tid];
            wcnt[w][tid] = o;
            o += cw;
        }
        if (LB) {
            // this tile's offset inside digit tid: decoupled look-back over earlier tiles
            uint64_t* col = status + tid;
            uint32_t excl = 0;
            if (t == 0) {
                lb_store(col, LB_PRE | tot);
            } else {
                lb_store(col + (size_t)t * RADIX, LB_AGG | tot);
                excl = lb_lookback_n<GSR_LB_STEP>(col, RADIX, t);
                lb_store(col + (size_t)t * RADIX, LB_PRE | (excl + tot));
            }
            gbase[tid] = gstart + excl;
        } else {
            gbase[tid] = hist[(size_t)tid * gridDim.x + t];
        }
    }
    __syncthreads();
    ST_T(st3)
#pragma unroll
    for (int r = 0; r < ITEMS; ++r) {
        const size_t idx = wbase + (size_t)r * 64 + lane;
        if (idx < n) {
            const uint32_t pos = wcnt[wid][(key[r] >> shift) & mask] + rk[r];
            s_key[pos] = key[r];
            s_val[pos] = val[r];
            s_val2[pos] = val2[r];
        }
    }
    __syncthreads();
    // 0 for a tile past n (speculative sorts size the grid by capacity, n by the device count)
    const int nvalid = bbase < n ? (int)min((size_t)TILE, n - bbase) : 0;
    for (int p = tid; p < nvalid; p += NT) {
        const uint32_t k = s_key[p];
        const uint32_t d = (k >> shift) & mask;
        const size_t g = (size_t)gbase[d] + (uint32_t)p - dbase[d];
        if (keys_out) keys_out[g] = k;
        vals_out[g] = s_val[p];
        if (vals2_out) vals2_out[g] = s_val2[p];
        if (fin.ranges) {
            // Last pass: the tile is in final order, so equal keys are adjacent here and a
            // key's run continues across tiles only at the tile's ends.
            if (p == 0 || s_key[p - 1] != k) atomicMin(&fin.ranges[k].x, (uint32_t)g);
            if (p == nvalid - 1 || s_key[p + 1] != k) atomicMax(&fin.ranges[k].y, (uint32_t)(g + 1));
        }
    }
#ifdef GSR_SORT_TRACE
    if (LB) {
        __syncthreads();
        if (threadIdx.x == 0 && t < 1024) {
            unsigned long long* w = g_gsr_strace[(shift >> 3) & 3][t];
            w[0] = st0; w[1] = st1; w[2] = st2; w[3] = st3; w[4] = __builtin_amdgcn_s_memrealtime();
            w[5] = __builtin_amdgcn_s_getreg((20) | (0 << 6) | (3 << 11)) & 15u;
        }
    }
#endif
}

// ------------------------------------------- grouped look-back passes ----
// The depth sort's passes for grids of at most GRP_MAX_TILES tiles (4M keys at 4096 keys per
// tile), measured per tile phase (tools/sort_trace.py, profiles/round3_sort_trace.txt): of a
// 17.8-us pass, 2.1 us went to the atomic that hands out tile indices, 6.8 us to the decoupled
// look-back (the inclusive prefix advanced 8 tiles per cross-XCD round trip: the last tiles
// finished their look-back 9 us after the first), and identity passes (a constant top byte)
// still cost a 7-us copy plus a launch gap.  Here:
//   * the tile index still comes from an atomic ticket in dispatch order (a tile waits only on
//     tiles that have started, whatever order the hardware dispatches workgroups in and however
//     many CUs a concurrent kernel -- RCCL's, in the data-parallel run -- holds), but the ticket's
//     round trip now overlaps the load of the pass plan instead of preceding the key loads;
//   * two-level look-back: a tile publishes its digit counts, sums those of the earlier tiles
//     of its group of 16 or 32 tiles (independent loads, no chain), and the group's last tile
//     publishes the group total; a tile adds the totals of the earlier groups.  About three
//     round trips instead of one per 8 tiles;
//   * the pass plan comes from the digit spans of every pass (k_radix_hist): passes that are
//     the identity on the keys that matter return at once, and the real passes ping-pong so
//     that the last real one writes the output arrays (buffers chosen on the device: no copy).
// Results are identical to the other modes (same stable order on the keys that matter).
// Group size: 16 tiles up to 256 tiles (the 1M-key depth sort), 32 up to GRP_MAX_TILES = 1024
// (C3's 3M-key depth sort 0.202 -> 0.161 ms).  Sorts of more than 1024 tiles of 4096 keys use
// tiles of 8192 keys (16 waves x 8), up to 8M keys; grouped passes over 1465 tiles of 4096 keys
// (C5, groups of 64) took 0.320 ms against 0.258 for the table passes.
constexpr int GRP_MIN = 16, GRP_MAX_TILES = 1024;
constexpr int GRP_BIG_ITEMS = 8;  // keys per thread of the 8192-key tiles
inline int grp_size(size_t nt) { return nt <= 256 ? 16 : 32; }
// Sum of the published values of words [lo, hi) of one digit column (stride RADIX between
// tiles / groups), LB_WIN loads in flight at a time.
template <int LB_WIN = 16>
__device__ __forceinline__ uint32_t lb_sum_window(uint64_t* col, int lo, int hi) {
    uint32_t acc = 0;
    for (int i = lo; i < hi;) {
        uint64_t w[LB_WIN];
#pragma unroll
        for (int k = 0; k < LB_WIN; ++k) w[k] = i + k < hi ? lb_load(col + (size_t)(i + k) * RADIX) : LB_AGG;
        bool stall = false;
        uint32_t part = 0;
#pragma unroll
        for (int k = 0; k < LB_WIN; ++k) {
            if (i + k >= hi) continue;
            stall |= (w[k] >> 32) == 0;
            part += (uint32_t)w[k];
        }
        if (stall) {
            __builtin_amdgcn_s_sleep(1);
            continue;
        }
        acc += part;
        i += LB_WIN;
    }
    return acc;
}
struct GrpBufs {
    const uint32_t* kin;
    const uint32_t* v2in;
    uint32_t *ktmp, *vtmp, *v2tmp;
    uint32_t *kout, *vout, *v2out;
};
template <int ITEMS, int WAVES>
__global__ void __launch_bounds__(64 * WAVES) k_radix_scatter_grp(GrpBufs B, size_t n, int pass, int passes,
                                                                  int per_pass, int key_bits,
                                                                  const uint32_t* __restrict__ hist,
                                                                  uint64_t* status, const uint32_t* span,
                                                                  int no_keys, uint32_t* counter, int grp) {
    constexpr int NT = 64 * WAVES, TILE = NT * ITEMS;
    ST_T(st0)
    __shared__ uint32_t s_key[TILE], s_val[TILE], s_val2[TILE];
    __shared__ uint32_t wcnt[WAVES][RADIX];
    __shared__ uint32_t dbase[RADIX], gbase[RADIX];
    __shared__ uint32_t wsum[WAVES];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    // the key bits that vary over the keys that matter (k_radix_hist), loaded while the tile
    // index is taken
    const uint32_t vary = span[0] & span[1];
    const int ntiles = (int)gridDim.x;
    const int t = lb_tile_index(counter);
    // the pass plan: real passes
    int nreal = 0, j = -1;
    for (int p = 0; p < passes; ++p) {
        const int sh = p * per_pass, nb = min(per_pass, key_bits - p * per_pass);
        const bool real = ((vary >> sh) & ((1u << nb) - 1u)) != 0u;
        if (real) {
            if (p == pass) j = nreal;
            ++nreal;
        }
    }
    if (nreal == 0 && pass == 0) {  // every pass is the identity: pass 0 runs (a stable copy)
        nreal = 1;
        j = 0;
    }
    ST_T(st1)
    if (j < 0) return;  // uniform: identity pass
    const bool to_out = ((nreal - 1 - j) & 1) == 0, from_out = j > 0 && ((nreal - j) & 1) == 0;
    const bool last = j == nreal - 1;
    // Keys: when the output key array is the input one (the depth sort, whose sorted keys are
    // not needed: no_keys), a pass must never write the array it or an earlier pass reads from
    // while other tiles may still be loading it, so the keys alternate tmp, in, tmp, ... from
    // pass 0 on; otherwise they follow the values (the last real pass writes the output).
    const bool kalias = B.kout == B.kin;
    const uint32_t* keys_in = j == 0 ? B.kin : (kalias ? ((j & 1) ? B.ktmp : B.kin) : (from_out ? B.kout : B.ktmp));
    uint32_t* keys_out = (last && no_keys) ? nullptr : (kalias ? ((j & 1) ? B.kout : B.ktmp) : (to_out ? B.kout : B.ktmp));
    const uint32_t* vals_in = j == 0 ? nullptr : (from_out ? B.vout : B.vtmp);
    const uint32_t* vals2_in = j == 0 ? B.v2in : (from_out ? B.v2out : B.v2tmp);
    uint32_t* vals_out = to_out ? B.vout : B.vtmp;
    uint32_t* vals2_out = B.v2in ? (to_out ? B.v2out : B.v2tmp) : nullptr;
    const int shift = pass * per_pass;
    const int bits = min(per_pass, key_bits - shift);
    const uint32_t ndig = 1u << bits, mask = ndig - 1u;
#pragma unroll
    for (int i = 0; i < RADIX / 64; ++i) wcnt[wid][lane + 64 * i] = 0;
    const size_t bbase = (size_t)t * TILE;
    const size_t wbase = bbase + (size_t)wid * (64 * ITEMS);
    const uint64_t lt = lanemask_lt();
    uint32_t key[ITEMS], val[ITEMS], val2[ITEMS], rk[ITEMS];
#pragma unroll
    for (int r = 0; r < ITEMS; ++r) {
        const size_t idx = wbase + (size_t)r * 64 + lane;
        const bool valid = idx < n;
        key[r] = valid ? keys_in[idx] : 0u;
        val[r] = valid ? (vals_in ? vals_in[idx] : (uint32_t)idx) : 0u;
        val2[r] = (valid && vals2_in) ? vals2_in[idx] : 0u;
    }
    // the pass's global digit counts (used after the ranking), issued after the keys: the
    // in-order load counter would otherwise make the ranking wait for this load as well
    const uint32_t hcount = (uint32_t)tid < ndig ? hist[pass * RADIX + tid] : 0u;
#pragma unroll
    for (int r = 0; r < ITEMS; ++r) {
        const size_t idx = wbase + (size_t)r * 64 + lane;
        const bool valid = idx < n;
        const uint32_t digit = (key[r] >> shift) & mask;
        uint64_t peers = __ballot(valid);
        for (int b = 0; b < bits; ++b) {
            const bool set = (digit >> b) & 1u;
            const uint64_t m = __ballot(set);
            peers &= set ? m : ~m;
        }
        const uint32_t rank = __popcll(peers & lt);
        const uint32_t old = valid ? wcnt[wid][digit] : 0u;
        rk[r] = old + rank;
        if (valid && rank == 0) wcnt[wid][digit] = old + (uint32_t)__popcll(peers);
    }
    __syncthreads();
    ST_T(st2)
    uint32_t tot = 0;
    if ((uint32_t)tid < ndig)
#pragma unroll
        for (int w = 0; w < WAVES; ++w) tot += wcnt[w][tid];
    if ((uint32_t)tid < ndig) {  // publish this tile's digit counts first: later tiles wait on them
        uint64_t* agg = status + (size_t)t * RADIX + tid;
        lb_store(agg, LB_AGG | tot);
    }
    uint32_t total;
    const uint32_t db = block_exclusive_scan_w<WAVES>(tot, wsum, &total);
    const uint32_t gstart = block_exclusive_scan_w<WAVES>(hcount, wsum, &total);
    if ((uint32_t)tid < ndig) {
        dbase[tid] = db;
        uint32_t o = db;
#pragma unroll
        for (int w = 0; w < WAVES; ++w) {
            const uint32_t cw = wcnt[w][tid];
            wcnt[w][tid] = o;
            o += cw;
        }
        const int g = t / grp, t0 = g * grp;
        uint64_t* const aggs = status + tid;                                  // [tile][RADIX]
        uint64_t* const grps = status + (size_t)ntiles * RADIX + tid;         // [group][RADIX]
        // earlier tiles of the group, then the totals of the earlier groups: windows of LB_WIN
        // independent loads, a window re-read until all of it is published
        // (8-deep windows with 8 keys per thread: the 16-deep ones pushed the kernel past 128 VGPRs)
        constexpr int WIN = ITEMS > 4 ? 8 : 16;
        const uint32_t in_grp = lb_sum_window<WIN>(aggs, t0, t);
        if (t == t0 + grp - 1 && t + 1 < ntiles)  // the group's total, for the later groups
            lb_store(grps + (size_t)g * RADIX, LB_AGG | (in_grp + tot));
        const uint32_t before = lb_sum_window<WIN>(grps, 0, g);
        gbase[tid] = gstart + before + in_grp;
    }
    __syncthreads();
    ST_T(st3)
#pragma unroll
    for (int r = 0; r < ITEMS; ++r) {
        const size_t idx = wbase + (size_t)r * 64 + lane;
        if (idx < n) {
            const uint32_t pos = wcnt[wid][(key[r] >> shift) & mask] + rk[r];
            s_key[pos] = key[r];
            s_val[pos] = val[r];
            s_val2[pos] = val2[r];
        }
    }
    __syncthreads();
    const int nvalid = bbase < n ? (int)min((size_t)TILE, n - bbase) : 0;
    for (int p = tid; p < nvalid; p += NT) {
        const uint32_t k = s_key[p];
        const uint32_t d = (k >> shift) & mask;
        const size_t g = (size_t)gbase[d] + (uint32_t)p - dbase[d];
        if (keys_out) keys_out[g] = k;
        vals_out[g] = s_val[p];
        if (vals2_out) vals2_out[g] = s_val2[p];
    }
#ifdef GSR_SORT_TRACE
    __syncthreads();
    if (threadIdx.x == 0 && t < 1024) {
        unsigned long long* w = g_gsr_strace[pass & 3][t];
        w[0] = st0; w[1] = st1; w[2] = st2; w[3] = st3; w[4] = __builtin_amdgcn_s_memrealtime();
        w[5] = __builtin_amdgcn_s_getreg((20) | (0 << 6) | (3 << 11)) & 15u;
    }
#endif
}

// ----------------------------------------------------------- duplicate ----
// One thread per depth-ordered Gaussian: emit its tiles (y outer, x inner, as
// rasterizer_impl.cu:98-108) into consecutive instance slots.  A block's 256
// consecutive depth-ordered Gaussians own one contiguous slot range; when it fits
// in LDS the keys are assembled there and written out with consecutive threads on
// consecutive slots (per-thread runs at scattered offsets would make every store
// instruction touch 64 partial lines).  Oversized ranges are written directly.
constexpr int DUP_CAP = 4096;
__global__ void __launch_bounds__(256) k_duplicate(int P, const uint32_t* __restrict__ order,
                                                   const uint32_t* __restrict__ offsets,
                                                   const uint32_t* __restrict__ tiles_touched,
                                                   const ushort4* __restrict__ rect,
                                                   const uint32_t* __restrict__ rect_sorted, int gx,
                                                   uint32_t* __restrict__ tkeys, uint32_t* __restrict__ slot_gid,
                                                   uint2* __restrict__ ranges, int T,
                                                   uint32_t cap) {
    __shared__ uint32_t s_key[DUP_CAP], s_gid[DUP_CAP];
    // ranges start at {~0u, 0} for the tile sort's atomicMin / atomicMax; empty tiles end
    // up {0, 0} (rasterizer_impl.cu:316 memset) in k_tile_order
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < T; i += gridDim.x * blockDim.x)
        ranges[i] = make_uint2(~0u, 0u);
    const int r0 = blockIdx.x * blockDim.x;
    const int r = r0 + threadIdx.x;
    const int rl = min(r0 + (int)blockDim.x, P) - 1;
    const uint32_t bbase = r0 == 0 ? 0u : offsets[r0 - 1];
    // cap: slots the binning buffer holds; a speculative launch (gsr_forward) may see more
    // instances than that, and then writes none past it (the host re-runs this stage)
    const uint32_t bend_full = offsets[rl];
    const bool staged = bend_full - bbase <= (uint32_t)DUP_CAP;
    const uint32_t bend = min(bend_full, max(cap, bbase));
    if (r < P) {
        const uint32_t g = order[r];
        // packed rect in depth order (coalesced) when available, else gathered by id
        ushort4 rc;
        uint32_t cnt;
        if (rect_sorted) {
            const uint32_t pr = rect_sorted[r];
            rc = make_ushort4(pr & 255u, (pr >> 8) & 255u, (pr >> 16) & 255u, pr >> 24);
            cnt = (uint32_t)(rc.z - rc.x) * (uint32_t)(rc.w - rc.y);
        } else {
            cnt = tiles_touched[g];
            rc = cnt ? rect[g] : make_ushort4(0, 0, 0, 0);
        }
        if (cnt != 0) {
            uint32_t off = r == 0 ? 0u : offsets[r - 1];
            if (staged) {
                uint32_t lo = off - bbase;
                for (int y = rc.y; y < rc.w; ++y)
                    for (int x = rc.x; x < rc.z; ++x, ++lo) {
                        s_key[lo] = (uint32_t)(y * gx + x);
                        s_gid[lo] = g;
                    }
            } else {
                for (int y = rc.y; y < rc.w; ++y)
                    for (int x = rc.x; x < rc.z; ++x, ++off) {
                        if (off >= cap) break;
                        tkeys[off] = (uint32_t)(y * gx + x);
                        slot_gid[off] = g;
                    }
            }
        }
    }
    if (!staged) return;  // uniform per block
    __syncthreads();
    const int n = (int)(bend - bbase);
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
        tkeys[bbase + i] = s_key[i];
        slot_gid[bbase + i] = s_gid[i];
    }
}

// Heavy-first tile schedule for the render kernels: tiles bucketed by the bit
// length of their instance count, longest bucket first.  The hardware dispatcher
// hands workgroups out in index order as slots free up, so issuing the heavy
// tiles first turns it into a longest-processing-time-first scheduler (the
// natural row-major order leaves the dense centre tiles for the end).  Order
// within a bucket is arbitrary: it changes timing only, never a result.

// Counters are private to each wave (LDS [wave][bucket]): a lane's atomic contends only
// with its own wave's lanes inside one instruction.  Shared counters serialised across
// the whole block when most tiles share a bucket (at the 6M-Gaussian config every tile
// length has the same bit length: 0.1 ms).
constexpr int ORDER_THREADS = 1024, ORDER_WAVES = ORDER_THREADS / 64;
// sched[SCHED_*] = tiles in length buckets >= the kernel's split bucket B (the heavy-first
// order lists buckets 32, 31, ..., so that is bucket B - 1's offset); B = 0: no split.
__device__ __forceinline__ void write_sched(uint32_t* sched, const uint32_t* boff, int split_fwd, int split4_fwd) {
    sched[SCHED_FWD_SPLIT] = split_fwd > 0 && split_fwd <= 33 ? boff[split_fwd - 1] : 0u;
    sched[SCHED_FWD_QUARTER] = split4_fwd > 0 && split4_fwd <= 33 ? boff[split4_fwd - 1] : 0u;
}
__global__ void __launch_bounds__(ORDER_THREADS) k_tile_order(uint2* __restrict__ ranges, int T,
                                                              uint32_t* __restrict__ order, int split_fwd,
                                                              int split4_fwd) {
    __shared__ uint32_t wcnt[ORDER_WAVES][33];
    const int tid = threadIdx.x, wave = tid >> 6;
    for (int i = tid; i < ORDER_WAVES * 33; i += ORDER_THREADS) (&wcnt[0][0])[i] = 0;
    {  // the forward's backward queue starts empty
        const TileSched ts = tile_sched(order, T);
        for (int i = tid; i < BQ_BUCKETS; i += ORDER_THREADS) ts.bq_cnt[i] = 0u;
        for (int i = tid; i < T; i += ORDER_THREADS) ts.tdone[i] = 0u;
    }
    __syncthreads();
#pragma unroll 4
    for (int t = tid; t < T; t += ORDER_THREADS) {
        uint2 r = ranges[t];
        if (r.x == ~0u) {  // no instance (the tile sort's atomicMin never touched it): {0, 0}
            r = make_uint2(0u, 0u);
            ranges[t] = r;
        }
        atomicAdd(&wcnt[wave][len_bucket(r)], 1u);
    }
    __syncthreads();
    __shared__ uint32_t btot[33], boff[33];
    if (tid < 33) {  // per bucket: wave bases inside the bucket, and its total
        uint32_t run = 0;
        for (int w = 0; w < ORDER_WAVES; ++w) {
            const uint32_t c = wcnt[w][tid];
            wcnt[w][tid] = run;
            run += c;
        }
        btot[tid] = run;
    }
    __syncthreads();
    if (tid < 64) {  // heavy buckets first: exclusive scan over buckets 32, 31, ..., 0
        const uint32_t v = tid < 33 ? btot[32 - tid] : 0u;
        uint32_t x = v;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = (uint32_t)__shfl_up((int)x, o, 64);
            if (tid >= o) x += y;
        }
        if (tid < 33) boff[32 - tid] = x - v;
    }
    __syncthreads();
    if (tid == 0) write_sched(order + T, boff, split_fwd, split4_fwd);
#pragma unroll 4
    for (int t = tid; t < T; t += ORDER_THREADS) {
        const uint32_t b = len_bucket(ranges[t]);
        order[boff[b] + atomicAdd(&wcnt[wave][b], 1u)] = (uint32_t)t;
    }
}

// The same schedule when the non-empty buckets were counted upstream (row binning:
// k_tiles_scatter adds each row's fine-bucket counts into bw[0, 132)): one thread per tile over
// many blocks instead of one block walking every tile twice (11-12 us at 8160 tiles,
// latency-bound on one CU).  Fine buckets (quarter octaves of the list length, len_fbucket):
// inside one octave the lengths differ up to 2x, and the dispatcher then hands out tiles of
// very different work in arbitrary order.  A wave's lanes that share a bucket are grouped by an
// 8-ballot match and take one global atomic position per group (bw[TILE_BUCKET_POS + b]).
// Empty tiles (bucket 0, including rows the binning never visited) go last, so their count is
// not needed.
__global__ void __launch_bounds__(256) k_tile_order_counted(const uint2* __restrict__ ranges, int T,
                                                            uint32_t* bw, uint32_t* __restrict__ order,
                                                            int split_fwd, int split4_fwd, uint32_t fb_cap) {
    __shared__ uint32_t boff[FINE_BUCKETS];
    const int tid = threadIdx.x;
    if (tid < 64) {  // heavy first: exclusive offsets over buckets 131, 130, ..., 1; then bucket 0
        // lane l: heavy-order positions 3l .. 3l + 2 = buckets 131 - 3l - i
        uint32_t v[3], s = 0;
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            const int b = FINE_BUCKETS - 1 - (3 * tid + i);
            v[i] = b >= 1 ? bw[b] : 0u;
            s += v[i];
        }
        uint32_t x = s;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = (uint32_t)__shfl_up((int)x, o, 64);
            if (tid >= o) x += y;
        }
        uint32_t e = x - s;
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            const int b = FINE_BUCKETS - 1 - (3 * tid + i);
            if (b >= 1) boff[b] = e;
            e += v[i];
        }
        if (tid == 63) boff[0] = x;  // every non-empty tile comes first
    }
    __syncthreads();
    // forward split: tiles with n >= 2^(B-1) = fine buckets >= 4B
    if (blockIdx.x == 0 && tid == 0) {
        order[T + SCHED_FWD_SPLIT] = split_fwd > 0 && 4 * split_fwd <= FINE_BUCKETS ? boff[4 * split_fwd - 1] : 0u;
        order[T + SCHED_FWD_QUARTER] =
            split4_fwd > 0 && 4 * split4_fwd <= FINE_BUCKETS ? boff[4 * split4_fwd - 1] : 0u;
    }
    {  // the forward's backward queue starts empty
        const TileSched ts = tile_sched(order, T);
        if (blockIdx.x == 0 && tid < BQ_BUCKETS) ts.bq_cnt[tid] = 0u;
        const int t0 = blockIdx.x * 256 + tid;
        if (t0 < T) ts.tdone[t0] = 0u;
    }
    const int t = blockIdx.x * 256 + tid;
    const bool valid = t < T;
    const uint32_t b = valid ? len_fbucket(ranges[t], fb_cap) : 0u;
    uint64_t peers = __ballot(valid);
#pragma unroll
    for (int k = 0; k < 8; ++k) {  // buckets 0..131
        const bool set = (b >> k) & 1u;
        const uint64_t m = __ballot(set);
        peers &= set ? m : ~m;
    }
    const uint64_t lt = lanemask_lt();
    uint32_t base = 0;
    if (valid && (peers & lt) == 0) base = atomicAdd(&bw[TILE_BUCKET_POS + b], (uint32_t)__popcll(peers));
    const int leader = valid ? (int)__builtin_ctzll(peers) : 0;
    base = (uint32_t)__shfl((int)base, leader, 64);
    if (valid) order[boff[b] + base + (uint32_t)__popcll(peers & lt)] = (uint32_t)t;
}

}  // namespace

// rasterizer_impl.cu:35-50
uint32_t higher_msb(uint32_t n) {
    uint32_t msb = sizeof(n) * 4, step = msb;
    while (step > 1) {
        step /= 2;
        if (n >> msb) msb += step; else msb -= step;
    }
    if (n >> msb) msb++;
    return msb;
}

void launch_scan_inclusive_gather(const uint32_t* src, const uint32_t* gather_idx, uint32_t* out, size_t n,
                                  void* ws, bool ws_zeroed, hipStream_t st, uint32_t* host_total, bool rect_mode) {
    if (n == 0) return;
    const ScanWs W = scan_ws(n, ws);
    if (!ws_zeroed) (void)hipMemsetAsync(W.base, 0, W.bytes, st);
    hipLaunchKernelGGL(k_scan<true>, dim3(cdiv(n, SCAN_TILE)), dim3(SCAN_THREADS), 0, st, src, gather_idx, n, out,
                       W.status, W.counter, host_total, (int)rect_mode, nullptr);
}

// Sorting modes (measured on MI355X): small sorts are launch-bound and use one
// look-back scatter launch per pass; large sorts are bandwidth-bound and use the
// table-driven passes, whose per-pass histogram + scan launches cost less than the
// look-back chain over thousands of tiles.
#ifndef GSR_SORT_LB_MAX
#define GSR_SORT_LB_MAX (4u << 20)
#endif
#ifndef GSR_LB_ITEMS
#define GSR_LB_ITEMS 4
#endif
#ifndef GSR_LB_WAVES
#define GSR_LB_WAVES 16
#endif
#ifndef GSR_TB_WAVES
#define GSR_TB_WAVES 16
#endif
#ifndef GSR_TB_ITEMS
#define GSR_TB_ITEMS 4
#endif

int depth_sort_passes() { return 4; }
int sort_lb_items() { return GSR_LB_ITEMS * GSR_LB_WAVES / 4; }  // in units of 256-element rows
static size_t g_sort_lb_max = GSR_SORT_LB_MAX;  // gsr_set_option("sort_lookback_max", n)
void set_sort_lookback_max(size_t n) { g_sort_lb_max = n; }
bool sort_uses_lookback(size_t n) { return n <= g_sort_lb_max; }
#ifndef GSR_SORT_GROUPED
#define GSR_SORT_GROUPED 1
#endif
static bool g_sort_grouped = GSR_SORT_GROUPED;  // gsr_set_option("sort_grouped", 0 / 1)
void set_sort_grouped(bool on) { g_sort_grouped = on; }
size_t sort_grp_status_words(size_t nt) { return (nt + cdiv(nt, GRP_MIN)) * RADIX; }
// grouped passes for sorts of up to GRP_MAX_TILES tiles (whatever sort_lookback_max, which at 0
// forces the histogram-table passes for every sort)
// keys per tile of the grouped passes (in 256-key units): 4096 keys, or 8192 beyond 1024 tiles
static int grp_items(size_t n) {
#ifdef GSR_GRP_BIG_ALWAYS  // experiment: 8192-key tiles for every grouped sort
    return GRP_BIG_ITEMS * GSR_LB_WAVES / 4;
#endif
    return sort_tiles(n, sort_lb_items()) <= (size_t)GRP_MAX_TILES ? sort_lb_items() : GRP_BIG_ITEMS * GSR_LB_WAVES / 4;
}
bool sort_grouped_size(size_t n) {
    return g_sort_grouped && g_sort_lb_max > 0 && sort_tiles(n, grp_items(n)) <= (size_t)GRP_MAX_TILES;
}
size_t sort_zero_bytes(size_t n, int passes) {
    // the grouped passes' tiles (8192 keys beyond 1024 tiles of 4096) or the classic look-back's
    return sort_lb_zero_bytes(n, passes, sort_grouped_size(n) ? grp_items(n) : sort_lb_items());
}

// A tile is 64 * WAVES * ITEMS elements; sort_tiles(n, WAVES * ITEMS / 4) counts them.
template <int ITEMS, int WAVES, bool LB>
static void launch_scatter(size_t n, const uint32_t* kin, const uint32_t* vin, uint32_t* kout, uint32_t* vout,
                           int shift, int bits, const uint32_t* hist, uint64_t* status, uint32_t* counter,
                           const uint32_t* v2in, uint32_t* v2out, SortFinal fin, const uint32_t* span,
                           const uint32_t* n_dev, hipStream_t st) {
    static_assert(WAVES * ITEMS % 4 == 0, "tile must be a multiple of 256 elements");
    hipLaunchKernelGGL((k_radix_scatter<ITEMS, WAVES, LB>), dim3(sort_tiles(n, WAVES * ITEMS / 4)),
                       dim3(64 * WAVES), 0, st, kin, vin, kout, vout, n, shift, bits, hist, status, counter, v2in,
                       v2out, fin, span, n_dev);
}

// Stable LSD sort of (keys, vals[, vals2]) on the low key_bits bits.  Ping-pongs
// between the _tmp and _out arrays; the result always lands in the _out arrays.
// keys_in / vals_in / vals2_in are not modified.
void launch_radix_sort(const uint32_t* keys_in, const uint32_t* vals_in, uint32_t* keys_tmp, uint32_t* vals_tmp,
                       uint32_t* keys_out, uint32_t* vals_out, size_t n, int key_bits, void* ws, bool ws_zeroed,
                       hipStream_t st, const uint32_t* vals2_in, uint32_t* vals2_tmp, uint32_t* vals2_out,
                       const SortFinal* final_out, bool skip_sentinel, const uint32_t* n_dev) {
    if (n == 0) return;
    if (key_bits < 1) key_bits = 1;
    const int passes = (key_bits + RADIX_BITS - 1) / RADIX_BITS;
    const int per_pass = (key_bits + passes - 1) / passes;  // balanced: 13 bits -> 7 + 6
    const SortWs W = sort_ws(n, ws);
    const bool lb = sort_uses_lookback(n);
    // (an output key array that is the input one is supported only when the sorted keys are not
    // wanted: k_radix_scatter_grp then alternates the keys between the input and tmp arrays)
    const bool grp = sort_grouped_size(n) && !n_dev && !vals_in &&
                     (!final_out || (!final_out->ranges && final_out->zero16 == 0)) &&
                     (keys_out != keys_in || (final_out && final_out->no_keys));
    const bool tally = (lb || grp) && final_out && final_out->tally && final_out->tally_host && !n_dev;
    if (final_out && final_out->tally_used) *final_out->tally_used = tally;
    const bool bb = final_out && final_out->bb_base && final_out->bb_n;  // record-slot block bases
    const bool bb_in_hist = bb && (lb || grp);
    if (lb || grp) {
        const size_t nt = sort_tiles(n, sort_lb_items());
        if (!ws_zeroed) (void)hipMemsetAsync(W.base, 0, sort_zero_bytes(n, passes), st);
        const int hi = hist_items(n);
        auto hist_kern = hi == 4 ? k_radix_hist<4> : hi == 8 ? k_radix_hist<8> : k_radix_hist<16>;
        const size_t hblocks = cdiv(n, (size_t)HIST_THREADS * hi) + (bb_in_hist ? block_base_segments(final_out->bb_n) : 0);
        hipLaunchKernelGGL(hist_kern, dim3((unsigned)hblocks), dim3(HIST_THREADS), 0, st, keys_in,
                           n, passes, per_pass, key_bits, W.hist, W.counter + SPAN_WORD, (int)skip_sentinel, n_dev,
                           tally ? final_out->tally : nullptr,
                           reinterpret_cast<unsigned long long*>(W.counter + TALLY_WORD),
                           final_out ? final_out->tally_host : nullptr, bb_in_hist ? final_out->bb_tot : nullptr,
                           bb_in_hist ? final_out->bb_n : 0u, bb_in_hist ? final_out->bb_base : nullptr);
    }
    if (bb && !bb_in_hist) {
        // no histogram kernel: the bases on their own
        hipLaunchKernelGGL(k_block_bases, dim3(block_base_segments(final_out->bb_n)), dim3(HIST_THREADS), 0, st,
                           final_out->bb_tot, final_out->bb_n, final_out->bb_base);
    }
    if (grp) {
        // grouped look-back passes with the pass plan on the device (k_radix_scatter_grp)
        const bool big = grp_items(n) != sort_lb_items();
        const size_t nt = sort_tiles(n, grp_items(n));
        const GrpBufs B{keys_in, vals2_in, keys_tmp, vals_tmp, vals2_tmp, keys_out, vals_out, vals2_out};
        const int no_keys = final_out && final_out->no_keys ? 1 : 0;
        for (int p = 0; p < passes; ++p) {
            auto kern = big ? k_radix_scatter_grp<GRP_BIG_ITEMS, GSR_LB_WAVES> : k_radix_scatter_grp<GSR_LB_ITEMS, GSR_LB_WAVES>;
            hipLaunchKernelGGL(kern, dim3((unsigned)nt), dim3(64 * GSR_LB_WAVES), 0, st, B, n, p, passes, per_pass,
                               key_bits, W.hist, W.status + (size_t)p * sort_grp_status_words(nt), W.counter + SPAN_WORD,
                               no_keys, W.counter + p, grp_size(nt));
        }
        return;
    }
    const uint32_t* kin = keys_in;
    const uint32_t* vin = vals_in;
    const uint32_t* v2in = vals2_in;
    for (int p = 0; p < passes; ++p) {
        const int shift = p * per_pass;
        const int bits = key_bits - shift < per_pass ? key_bits - shift : per_pass;
        // last pass writes the output pair; earlier passes alternate so that holds
        const bool to_out = ((passes - 1 - p) % 2) == 0;
        uint32_t* kout = to_out ? keys_out : keys_tmp;
        uint32_t* vout = to_out ? vals_out : vals_tmp;
        uint32_t* v2out = vals2_in ? (to_out ? vals2_out : vals2_tmp) : nullptr;
        const bool last = p == passes - 1;
        const SortFinal fin = (last && final_out) ? *final_out : SortFinal{nullptr, nullptr, 0, false};
        if (fin.ranges || fin.no_keys) kout = nullptr;  // the ranges replace the sorted keys
        if (lb) {
            const size_t nt = sort_tiles(n, sort_lb_items());
            launch_scatter<GSR_LB_ITEMS, GSR_LB_WAVES, true>(n, kin, vin, kout, vout, shift, bits,
                                                             W.hist + p * RADIX, W.status + (size_t)p * nt * RADIX,
                                                             W.counter + p, v2in, v2out, fin,
                                                             W.counter + SPAN_WORD, n_dev, st);
        } else {
            const size_t nt = sort_tiles(n, GSR_TB_ITEMS * GSR_TB_WAVES / 4);
            const size_t len = ((size_t)1 << bits) * nt;
            const ScanWs S = scan_ws(len, W.scan);
            hipLaunchKernelGGL((k_radix_upsweep<GSR_TB_ITEMS, GSR_TB_WAVES>), dim3(nt), dim3(64 * GSR_TB_WAVES), 0, st,
                               kin, n, shift,
                               bits, W.table, S.base, cdiv(S.bytes, 16), n_dev);
            hipLaunchKernelGGL(k_scan<false>, dim3(cdiv(len, SCAN_TILE)), dim3(SCAN_THREADS), 0, st, W.table,
                               nullptr, len, W.table, S.status, S.counter, nullptr, 0, nullptr);
            launch_scatter<GSR_TB_ITEMS, GSR_TB_WAVES, false>(n, kin, vin, kout, vout, shift, bits, W.table, nullptr,
                                                              nullptr, v2in, v2out, fin, nullptr, n_dev, st);
        }
        kin = kout;
        vin = vout;
        v2in = v2out;
    }
}

void launch_scan_exclusive(const uint32_t* src, uint32_t* out, size_t n, const uint32_t* n_dev, const ScanWs& W,
                           hipStream_t st) {
    if (n == 0) return;
    hipLaunchKernelGGL(k_scan<false>, dim3(cdiv(n, SCAN_TILE)), dim3(SCAN_THREADS), 0, st, src, nullptr, n, out,
                       W.status, W.counter, nullptr, 0, n_dev);
}

// Split buckets (gsr_set_option "split_fwd_bucket" / "split_bwd_depth"; a negative value
// restores the default): tiles whose list length has at least this bit length
// (n >= 2^(B-1)) get two waves.  Forward default B = 8 (n >= 128: at the metric scene every
// tile that goes deeper than a few dozen positions): a SIMD serves its waves oldest first and
// ends when its tiles' total work is done, so the ~5300 deep tiles dealt over 1024 SIMDs x 5
// wave slots left the most loaded SIMD 25% behind the median (profiles/round3_wave_trace_simd.txt);
// twice as many half-size units even that out: render_fwd 0.227 -> 0.204 ms
// (profiles/round3_split_sweep.txt: B = 7 0.203-0.205, 9 0.207-0.213, 1 0.206, 10-12 slower).
#ifndef GSR_SPLIT_FWD
#define GSR_SPLIT_FWD 8
#endif
#ifndef GSR_SPLIT_BWD_DEPTH
#define GSR_SPLIT_BWD_DEPTH 0
#endif
#ifndef GSR_SPLIT4_FWD
#define GSR_SPLIT4_FWD 0
#endif
static int g_split_fwd = GSR_SPLIT_FWD, g_split_bwd_depth = GSR_SPLIT_BWD_DEPTH, g_split4_fwd = GSR_SPLIT4_FWD;
void set_split4_bucket(int b) { g_split4_fwd = b >= 0 ? b : GSR_SPLIT4_FWD; }
int split4_fwd_bucket() { return g_split4_fwd; }
void set_split_buckets(int fwd_bucket, int bwd_depth) {
    g_split_fwd = fwd_bucket >= 0 ? fwd_bucket : GSR_SPLIT_FWD;
    g_split_bwd_depth = bwd_depth >= 0 ? bwd_depth : GSR_SPLIT_BWD_DEPTH;
}
int split_bwd_depth() { return g_split_bwd_depth; }
int split_fwd_bucket() { return g_split_fwd; }

#ifndef GSR_FWD_ORDER_CAP
#define GSR_FWD_ORDER_CAP 0
#endif
static uint32_t g_fwd_order_fb_cap = len_fbucket_n(GSR_FWD_ORDER_CAP);
void set_fwd_order_cap(int instances) { g_fwd_order_fb_cap = instances > 0 ? len_fbucket_n((uint32_t)instances) : 0u; }
uint32_t fwd_order_fb_cap() { return g_fwd_order_fb_cap; }

void launch_tile_order_counted(const uint2* ranges, int T, uint32_t* bucket_words, uint32_t* order,
                               hipStream_t st) {
    if (T == 0) return;
    hipLaunchKernelGGL(k_tile_order_counted, dim3((unsigned)cdiv((size_t)T, 256)), dim3(256), 0, st, ranges, T,
                       bucket_words, order, g_split_fwd, g_split4_fwd, g_fwd_order_fb_cap);
}

void launch_tile_order(uint2* ranges, int T, uint32_t* order, hipStream_t st) {
    if (T == 0) return;
    hipLaunchKernelGGL(k_tile_order, dim3(1), dim3(1024), 0, st, ranges, T, order, g_split_fwd, g_split4_fwd);
}

void launch_duplicate(int P, const uint32_t* order, const uint32_t* offsets, const uint32_t* tiles_touched,
                      const ushort4* rect, const uint32_t* rect_sorted, int gx, uint32_t* tkeys,
                      uint32_t* slot_gid, uint2* ranges, int T, uint32_t cap, hipStream_t st) {
    if (P == 0) return;
    hipLaunchKernelGGL(k_duplicate, dim3(cdiv(P, 256)), dim3(256), 0, st, P, order, offsets, tiles_touched, rect,
                       rect_sorted, gx, tkeys, slot_gid, ranges, T, cap);
}


}  // namespace gsr
