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

namespace gsr {

namespace {

__device__ __forceinline__ uint64_t lanemask_lt() {
    const uint32_t lane = threadIdx.x & 63;
    return lane ? (~0ull >> (64 - lane)) : 0ull;
}

// Exclusive scan of one value per thread over a 256-thread block.
// wsum: __shared__ uint32_t[4].  Returns the exclusive prefix; *total = block sum.
__device__ __forceinline__ uint32_t block_exclusive_scan(uint32_t v, uint32_t* wsum, uint32_t* total) {
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
    for (int w = 0; w < 4; ++w) {
        uint32_t s = wsum[w];
        if (w < wid) pre += s;
        tot += s;
    }
    __syncthreads();
    *total = tot;
    return pre + x - v;
}

// ---------------------------------------------------------------- scan ----
// value(i) = gather ? src[gather[i]] : src[i]
__global__ void __launch_bounds__(SCAN_THREADS) k_scan_reduce(const uint32_t* __restrict__ src,
                                                              const uint32_t* __restrict__ gather, size_t n,
                                                              uint32_t* __restrict__ parts) {
    __shared__ uint32_t wsum[4];
    const size_t base = (size_t)blockIdx.x * SCAN_TILE;
    uint32_t acc = 0;
#pragma unroll
    for (int i = 0; i < SCAN_ITEMS; ++i) {
        size_t idx = base + (size_t)i * SCAN_THREADS + threadIdx.x;
        if (idx < n) acc += gather ? src[gather[idx]] : src[idx];
    }
    uint32_t tot;
    block_exclusive_scan(acc, wsum, &tot);
    if (threadIdx.x == 0) parts[blockIdx.x] = tot;
}

// Single block: exclusive scan of parts[0..np) in place.
__global__ void __launch_bounds__(SCAN_THREADS) k_scan_parts(uint32_t* __restrict__ parts, size_t np) {
    __shared__ uint32_t wsum[4];
    uint32_t carry = 0;
    for (size_t base = 0; base < np; base += (size_t)SCAN_THREADS * SCAN_ITEMS) {
        uint32_t v[SCAN_ITEMS];
        uint32_t s = 0;
        const size_t mine = base + (size_t)threadIdx.x * SCAN_ITEMS;
#pragma unroll
        for (int i = 0; i < SCAN_ITEMS; ++i) {
            v[i] = (mine + i < np) ? parts[mine + i] : 0u;
            s += v[i];
        }
        uint32_t tot;
        uint32_t pre = block_exclusive_scan(s, wsum, &tot) + carry;
#pragma unroll
        for (int i = 0; i < SCAN_ITEMS; ++i) {
            if (mine + i < np) parts[mine + i] = pre;
            pre += v[i];
        }
        carry += tot;
    }
}

// out[i] = (inclusive ? sum_{j<=i} : sum_{j<i}) value(j); tile staged through LDS so
// both the loads and the stores are coalesced.
template <bool INCLUSIVE>
__global__ void __launch_bounds__(SCAN_THREADS) k_scan_down(const uint32_t* __restrict__ src,
                                                            const uint32_t* __restrict__ gather, size_t n,
                                                            const uint32_t* __restrict__ parts,
                                                            uint32_t* __restrict__ out) {
    __shared__ uint32_t tile[SCAN_TILE + SCAN_TILE / 32];
    __shared__ uint32_t wsum[4];
    const size_t base = (size_t)blockIdx.x * SCAN_TILE;
    auto pad = [](int i) { return i + (i >> 5); };
#pragma unroll
    for (int i = 0; i < SCAN_ITEMS; ++i) {
        int li = i * SCAN_THREADS + threadIdx.x;
        size_t idx = base + li;
        tile[pad(li)] = idx < n ? (gather ? src[gather[idx]] : src[idx]) : 0u;
    }
    __syncthreads();
    uint32_t v[SCAN_ITEMS], s = 0;
#pragma unroll
    for (int i = 0; i < SCAN_ITEMS; ++i) {
        v[i] = tile[pad(threadIdx.x * SCAN_ITEMS + i)];
        s += v[i];
    }
    uint32_t tot;
    uint32_t pre = block_exclusive_scan(s, wsum, &tot) + parts[blockIdx.x];
#pragma unroll
    for (int i = 0; i < SCAN_ITEMS; ++i) {
        uint32_t nx = pre + v[i];
        tile[pad(threadIdx.x * SCAN_ITEMS + i)] = INCLUSIVE ? nx : pre;
        pre = nx;
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < SCAN_ITEMS; ++i) {
        int li = i * SCAN_THREADS + threadIdx.x;
        size_t idx = base + li;
        if (idx < n) out[idx] = tile[pad(li)];
    }
}

// ---------------------------------------------------------- radix sort ----
// Per-block digit histogram -> hist[digit * nblocks + block].
__global__ void __launch_bounds__(SORT_THREADS) k_radix_upsweep(const uint32_t* __restrict__ keys, size_t n,
                                                                int shift, uint32_t mask,
                                                                uint32_t* __restrict__ hist) {
    __shared__ uint32_t cnt[RADIX];
    cnt[threadIdx.x] = 0;
    __syncthreads();
    const size_t base = (size_t)blockIdx.x * SORT_TILE;
#pragma unroll
    for (int i = 0; i < SORT_ITEMS; ++i) {
        size_t idx = base + (size_t)i * SORT_THREADS + threadIdx.x;
        if (idx < n) atomicAdd(&cnt[(keys[idx] >> shift) & mask], 1u);
    }
    __syncthreads();
    if (threadIdx.x <= mask) hist[(size_t)threadIdx.x * gridDim.x + blockIdx.x] = cnt[threadIdx.x];
}

// Stable scatter, staged through LDS.  Wave w of the block ranks the elements
// [1024 w, 1024 w + 1024) of the block's tile in 16 rounds of 64: a wave64
// multi-split by ballots gives each element its rank among equal digits of the
// round, and a per-wave digit counter in LDS (read by all lanes, then bumped by
// the digit's first lane -- ordered within the wave, no barrier) carries the
// rank across rounds.  One block scan then turns the 4 x 2^bits counters into
// block-local digit bases, the tile is permuted into digit order in LDS, and
// written out with consecutive threads on consecutive positions of each digit's
// run (coalesced, unlike a direct per-element scatter).  Stable: element order
// inside a digit is (wave, round, lane) = input order.  vals_in == NULL means
// value = element index; vals2 is an optional second payload word.
__global__ void __launch_bounds__(SORT_THREADS) k_radix_scatter(
    const uint32_t* __restrict__ keys_in, const uint32_t* __restrict__ vals_in, uint32_t* __restrict__ keys_out,
    uint32_t* __restrict__ vals_out, size_t n, int shift, int bits, const uint32_t* __restrict__ hist,
    const uint32_t* __restrict__ vals2_in, uint32_t* __restrict__ vals2_out) {
    __shared__ uint32_t s_key[SORT_TILE], s_val[SORT_TILE], s_val2[SORT_TILE];
    __shared__ uint32_t wcnt[4][RADIX];
    __shared__ uint32_t dbase[RADIX], gbase[RADIX];
    __shared__ uint32_t wsum[4];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const uint32_t ndig = 1u << bits, mask = ndig - 1u;
    const int nb = (int)gridDim.x;
#pragma unroll
    for (int i = 0; i < RADIX / 64; ++i) wcnt[wid][lane + 64 * i] = 0;
    if ((uint32_t)tid < ndig) gbase[tid] = hist[(size_t)tid * nb + blockIdx.x];
    const size_t bbase = (size_t)blockIdx.x * SORT_TILE;
    const size_t wbase = bbase + (size_t)wid * (SORT_TILE / 4);
    const uint64_t lt = lanemask_lt();
    uint32_t key[SORT_ITEMS], val[SORT_ITEMS], val2[SORT_ITEMS], rk[SORT_ITEMS];
#pragma unroll
    for (int r = 0; r < SORT_ITEMS; ++r) {
        const size_t idx = wbase + (size_t)r * 64 + lane;
        const bool valid = idx < n;
        key[r] = valid ? keys_in[idx] : 0u;
        val[r] = valid ? (vals_in ? vals_in[idx] : (uint32_t)idx) : 0u;
        val2[r] = (valid && vals2_in) ? vals2_in[idx] : 0u;
    }
#pragma unroll
    for (int r = 0; r < SORT_ITEMS; ++r) {
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
    // digit-major block offsets: dbase[d] = elements of digits < d; wave offsets inside d
    uint32_t c[4], tot = 0;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
        c[w] = (uint32_t)tid < ndig ? wcnt[w][tid] : 0u;
        tot += c[w];
    }
    uint32_t total;
    const uint32_t db = block_exclusive_scan(tot, wsum, &total);
    if ((uint32_t)tid < ndig) {
        dbase[tid] = db;
        uint32_t o = db;
#pragma unroll
        for (int w = 0; w < 4; ++w) {
            wcnt[w][tid] = o;
            o += c[w];
        }
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < SORT_ITEMS; ++r) {
        const size_t idx = wbase + (size_t)r * 64 + lane;
        if (idx < n) {
            const uint32_t pos = wcnt[wid][(key[r] >> shift) & mask] + rk[r];
            s_key[pos] = key[r];
            s_val[pos] = val[r];
            s_val2[pos] = val2[r];
        }
    }
    __syncthreads();
    const int nvalid = (int)min((size_t)SORT_TILE, n - bbase);
    for (int p = tid; p < nvalid; p += SORT_THREADS) {
        const uint32_t k = s_key[p];
        const uint32_t d = (k >> shift) & mask;
        const size_t g = (size_t)gbase[d] + (uint32_t)p - dbase[d];
        keys_out[g] = k;
        vals_out[g] = s_val[p];
        if (vals2_out) vals2_out[g] = s_val2[p];
    }
}

// ----------------------------------------------------------- duplicate ----
// One thread per depth-ordered Gaussian: emit its tiles (y outer, x inner, as
// rasterizer_impl.cu:98-108) into consecutive instance slots.
__global__ void __launch_bounds__(256) k_duplicate(int P, const uint32_t* __restrict__ order,
                                                   const uint32_t* __restrict__ offsets,
                                                   const uint32_t* __restrict__ tiles_touched,
                                                   const ushort4* __restrict__ rect, int gx,
                                                   uint32_t* __restrict__ tkeys, uint32_t* __restrict__ slot_gid,
                                                   uint32_t* __restrict__ goff) {
    const int r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= P) return;
    const uint32_t g = order[r];
    const uint32_t cnt = tiles_touched[g];
    if (cnt == 0) return;
    uint32_t off = r == 0 ? 0u : offsets[r - 1];
    goff[g] = off;
    const ushort4 rc = rect[g];
    for (int y = rc.y; y < rc.w; ++y)
        for (int x = rc.x; x < rc.z; ++x) {
            tkeys[off] = (uint32_t)(y * gx + x);
            slot_gid[off] = g;
            ++off;
        }
}

// Tile ranges [first, last+1) from the sorted tile keys (identifyTileRanges,
// rasterizer_impl.cu:113-138).
__global__ void __launch_bounds__(256) k_finalize(size_t I, const uint32_t* __restrict__ tkeys,
                                                  uint2* __restrict__ ranges) {
    const size_t k = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= I) return;
    const uint32_t t = tkeys[k];
    if (k == 0 || tkeys[k - 1] != t) ranges[t].x = (uint32_t)k;
    if (k == I - 1 || tkeys[k + 1] != t) ranges[t].y = (uint32_t)(k + 1);
}

// Heavy-first tile schedule for the render kernels: tiles bucketed by the bit
// length of their instance count, longest bucket first.  The hardware dispatcher
// hands workgroups out in index order as slots free up, so issuing the heavy
// tiles first turns it into a longest-processing-time-first scheduler (the
// natural row-major order leaves the dense centre tiles for the end).  Order
// within a bucket is arbitrary: it changes timing only, never a result.
__global__ void __launch_bounds__(1024) k_tile_order(const uint2* __restrict__ ranges, int T,
                                                     uint32_t* __restrict__ order) {
    __shared__ uint32_t hist[33], off[33];
    const int tid = threadIdx.x;
    if (tid < 33) hist[tid] = 0;
    __syncthreads();
    for (int t = tid; t < T; t += blockDim.x) {
        const uint2 r = ranges[t];
        const uint32_t len = r.y - r.x;
        atomicAdd(&hist[len ? 32 - __clz(len) : 0], 1u);
    }
    __syncthreads();
    if (tid == 0) {
        uint32_t run = 0;
        for (int b = 32; b >= 0; --b) {
            off[b] = run;
            run += hist[b];
        }
    }
    __syncthreads();
    for (int t = tid; t < T; t += blockDim.x) {
        const uint2 r = ranges[t];
        const uint32_t len = r.y - r.x;
        order[atomicAdd(&off[len ? 32 - __clz(len) : 0], 1u)] = (uint32_t)t;
    }
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

static void scan_exclusive_inplace(uint32_t* data, size_t n, uint32_t* parts, hipStream_t st) {
    const size_t nb = cdiv(n, SCAN_TILE);
    hipLaunchKernelGGL(k_scan_reduce, dim3(nb), dim3(SCAN_THREADS), 0, st, data, nullptr, n, parts);
    hipLaunchKernelGGL(k_scan_parts, dim3(1), dim3(SCAN_THREADS), 0, st, parts, nb);
    hipLaunchKernelGGL(k_scan_down<false>, dim3(nb), dim3(SCAN_THREADS), 0, st, data, nullptr, n, parts, data);
}

void launch_scan_inclusive_gather(const uint32_t* src, const uint32_t* gather_idx, uint32_t* out, size_t n,
                                  uint32_t* parts, hipStream_t st) {
    if (n == 0) return;
    const size_t nb = cdiv(n, SCAN_TILE);
    hipLaunchKernelGGL(k_scan_reduce, dim3(nb), dim3(SCAN_THREADS), 0, st, src, gather_idx, n, parts);
    hipLaunchKernelGGL(k_scan_parts, dim3(1), dim3(SCAN_THREADS), 0, st, parts, nb);
    hipLaunchKernelGGL(k_scan_down<true>, dim3(nb), dim3(SCAN_THREADS), 0, st, src, gather_idx, n, parts, out);
}

// Stable LSD sort of (keys, vals) on the low key_bits bits.  Ping-pongs between
// (keys_tmp, vals_tmp) and (keys_out, vals_out); the result always lands in
// (keys_out, vals_out).  keys_in/vals_in are not modified.
void launch_radix_sort(const uint32_t* keys_in, const uint32_t* vals_in, uint32_t* keys_tmp, uint32_t* vals_tmp,
                       uint32_t* keys_out, uint32_t* vals_out, size_t n, int key_bits, uint32_t* hist,
                       uint32_t* parts, hipStream_t st, const uint32_t* vals2_in, uint32_t* vals2_tmp,
                       uint32_t* vals2_out) {
    if (n == 0) return;
    if (key_bits < 1) key_bits = 1;
    const int passes = (key_bits + RADIX_BITS - 1) / RADIX_BITS;
    const int per_pass = (key_bits + passes - 1) / passes;  // balanced: 13 bits -> 7 + 6
    const size_t nb = sort_blocks(n);
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
        hipLaunchKernelGGL(k_radix_upsweep, dim3(nb), dim3(SORT_THREADS), 0, st, kin, n, shift,
                           (1u << bits) - 1u, hist);
        scan_exclusive_inplace(hist, ((size_t)1 << bits) * nb, parts, st);
        hipLaunchKernelGGL(k_radix_scatter, dim3(nb), dim3(SORT_THREADS), 0, st, kin, vin, kout, vout, n, shift,
                           bits, hist, v2in, v2out);
        kin = kout;
        vin = vout;
        v2in = v2out;
    }
}

void launch_tile_order(const uint2* ranges, int T, uint32_t* order, hipStream_t st) {
    if (T == 0) return;
    hipLaunchKernelGGL(k_tile_order, dim3(1), dim3(1024), 0, st, ranges, T, order);
}

void launch_duplicate(int P, const uint32_t* order, const uint32_t* offsets, const uint32_t* tiles_touched,
                      const ushort4* rect, int gx, uint32_t* tkeys, uint32_t* slot_gid, uint32_t* goff,
                      hipStream_t st) {
    if (P == 0) return;
    hipLaunchKernelGGL(k_duplicate, dim3(cdiv(P, 256)), dim3(256), 0, st, P, order, offsets, tiles_touched, rect,
                       gx, tkeys, slot_gid, goff);
}

void launch_finalize(size_t I, const uint32_t* tkeys, uint2* ranges, hipStream_t st) {
    if (I == 0) return;
    hipLaunchKernelGGL(k_finalize, dim3(cdiv(I, 256)), dim3(256), 0, st, I, tkeys, ranges);
}

}  // namespace gsr
