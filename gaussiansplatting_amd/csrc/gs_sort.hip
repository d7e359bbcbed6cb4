// gs_sort.hip — stable LSD radix sort of 32-bit keys (with a 32-bit payload) and a
// device-wide exclusive scan, both driven by a device-resident element count so the
// frame never has to read P back to the host.
//
// The (tile | depth) 64-bit key order of the reference (tiled_rasterizer.mm:27-102, a CPU
// 8x8-bit LSD sort over pair<u64,u32>) is produced in two stages:
//   1. the 31 significant depth-key bits are sorted once over the N Gaussians;
//   2. pairs are emitted in that depth order, and a stable LSD pass over only the
//      ceil(log2(T)) tile bits orders them by tile.
// Stability of both stages gives exactly the order (tile, depth key, Gaussian index).
//
// One pass = hist (per-block digit counts) -> digit_scan (per digit over blocks) -> scatter
// (wave-level multisplit ranking, stable). Blocks own contiguous slices; the slice size is
// derived on the device from the element count, so a fixed grid serves any P.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "gs_device.hpp"
#include "gs_internal.hpp"
#include "gs_emit.hpp"

namespace gs {

// Inter-workgroup words inside a launch (scan status words): global agent-scope accesses, which
// are coherent across the XCDs' L2s; each word is its own payload (flag bits + value).
typedef __attribute__((address_space(1))) uint32_t gu32;
typedef __attribute__((address_space(1))) unsigned long long gu64;

// Workgroup barrier for LDS hand-offs only: waits for this wave's LDS operations, not for its
// outstanding global stores (a __syncthreads() would also drain the status-word stores, a memory
// round trip, before the barrier). The scan kernels exchange nothing through global memory inside
// a workgroup.
__device__ __forceinline__ void lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// Exclusive scan of one value per digit over threads 0..255 (every thread of the block calls it;
// threads >= 256 contribute nothing and get garbage). ws: 4 LDS words.
__device__ __forceinline__ uint32_t scan256_excl(uint32_t v, uint32_t t, uint32_t* ws) {
    const uint32_t lane = t & 63u, w = t >> 6;
    uint32_t inc = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(inc, o, 64);
        if (lane >= (uint32_t)o) inc += y;
    }
    if (w < 4u && lane == 63u) ws[w] = inc;
    lds_barrier();
    uint32_t base = 0;
#pragma unroll
    for (uint32_t k = 0; k < 4u; k++) base += k < w ? ws[k] : 0u;
    lds_barrier();
    return base + inc - v;
}

__device__ __forceinline__ uint32_t ld_agent(const uint32_t* p) {
    return __hip_atomic_load((const gu32*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_agent(uint32_t* p, uint32_t v) {
    __hip_atomic_store((gu32*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned long long ld_agent64(const unsigned long long* p) {
    return __hip_atomic_load((const gu64*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_agent64(unsigned long long* p, unsigned long long v) {
    __hip_atomic_store((gu64*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

constexpr int kSortThreads = 256;
constexpr int kSortItems = 8;
constexpr uint32_t kSortTile = kSortThreads * kSortItems;  // 2048 elements per block step
constexpr int kSortWaves = kSortThreads / 64;

__device__ __forceinline__ uint32_t sort_count(const uint32_t* n_dev, uint32_t n_host) {
    return n_dev ? *n_dev : n_host;
}

// Slice of block b: [b*S, min((b+1)*S, n)), S = ceil(n / B) rounded up to kSortTile.
__device__ __forceinline__ void sort_slice(uint32_t n, uint32_t b, uint32_t nblocks,
                                           uint32_t& begin, uint32_t& end) {
    uint32_t per = (n + nblocks - 1u) / nblocks;
    per = (per + kSortTile - 1u) / kSortTile * kSortTile;
    const uint64_t b0 = (uint64_t)per * b;
    begin = b0 < n ? (uint32_t)b0 : n;
    const uint64_t e0 = b0 + per;
    end = e0 < n ? (uint32_t)e0 : n;
}

// (ranges_init: the tile ranges the following scatter builds by atomics start as (~0, 0))
// per-slice digit counts: 1024 threads per slice (the sort's at most 512 slices then fill the device)
constexpr uint32_t kRhThreads = 1024;
template <typename KI>
__global__ __launch_bounds__(kRhThreads) void radix_hist_kernel(
    const KI* __restrict__ keys, const uint32_t* n_dev, uint32_t n_host, uint32_t shift,
    uint32_t mask, uint32_t* __restrict__ hist /* [256][nblocks] */, uint2* __restrict__ ranges_init,
    uint32_t ranges_n) {
    constexpr uint32_t kRhWaves = kRhThreads / 64;
    __shared__ uint32_t h[kRhWaves][256];
    const uint32_t t = threadIdx.x, w = t >> 6;
    if (ranges_init)
        for (uint32_t d = blockIdx.x * kRhThreads + t; d < ranges_n; d += gridDim.x * kRhThreads)
            ranges_init[d] = make_uint2(0xffffffffu, 0u);
    for (uint32_t i = t; i < kRhWaves * 256; i += kRhThreads) (&h[0][0])[i] = 0u;
    __syncthreads();
    const uint32_t n = sort_count(n_dev, n_host);
    uint32_t begin, end;
    sort_slice(n, blockIdx.x, gridDim.x, begin, end);
    // 16 loads in flight per thread before they are counted
    constexpr uint32_t kH = 16;
    for (uint32_t i0 = begin; i0 < end; i0 += kH * kRhThreads) {
        uint32_t k[kH];
#pragma unroll
        for (uint32_t q = 0; q < kH; q++) {
            const uint32_t i = i0 + q * kRhThreads + t;
            k[q] = i < end ? (uint32_t)keys[i] : 0u;
        }
#pragma unroll
        for (uint32_t q = 0; q < kH; q++)
            if (i0 + q * kRhThreads + t < end) atomicAdd(&h[w][(k[q] >> shift) & mask], 1u);
    }
    __syncthreads();
    if (t < 256u) {
        uint32_t s = 0;
#pragma unroll
        for (uint32_t ww = 0; ww < kRhWaves; ww++) s += h[ww][t];
        hist[t * gridDim.x + blockIdx.x] = s;
    }
}

// One block per digit: exclusive scan of hist[d][0..B) in place; totals[d] = row sum.
__global__ __launch_bounds__(256) void radix_digit_scan_kernel(uint32_t* __restrict__ hist,
                                                                uint32_t nblocks,
                                                                uint32_t* __restrict__ totals) {
    __shared__ uint32_t part[256];
    const uint32_t d = blockIdx.x, t = threadIdx.x;
    uint32_t* row = hist + (size_t)d * nblocks;
    const uint32_t per = (nblocks + 255u) / 256u;
    const uint32_t b0 = t * per;
    uint32_t s = 0;
    for (uint32_t k = 0; k < per; k++)
        if (b0 + k < nblocks) s += row[b0 + k];
    part[t] = s;
    __syncthreads();
    // Hillis-Steele inclusive scan of the 256 partials
    for (uint32_t o = 1; o < 256; o <<= 1) {
        const uint32_t v = t >= o ? part[t - o] : 0u;
        __syncthreads();
        part[t] += v;
        __syncthreads();
    }
    uint32_t run = t ? part[t - 1] : 0u;
    for (uint32_t k = 0; k < per; k++)
        if (b0 + k < nblocks) {
            const uint32_t c = row[b0 + k];
            row[b0 + k] = run;
            run += c;
        }
    if (t == 255) totals[d] = part[255];
}

// Stable scatter. Element order inside a block step is (wave, item, lane), which is the
// memory order, so ranks computed by wave ballots + per-wave counters are stable. Each 2048-element
// step is first reordered by digit in LDS, then written out so that consecutive lanes store
// consecutive positions of a digit run (coalesced) instead of 64 scattered buckets per instruction.
// Keys are read as KI and written as KO (u16 between the tile passes when the tile id fits). With
// ranges_out (the last pass of the tile sort) no keys are written: the first and last element of
// each key's run inside a step take atomicMin / atomicMax of their positions into ranges_out[key],
// which the pass's histogram kernel set to (~0, 0); the output is sorted by key, so the extremes
// over all steps are the key's range (empty keys stay (~0, 0): chunk_base_kernel fills them in).
// pairs per thread and step of the scatter (config 5, 69M pairs: 4 -> 1.25 ms, 8 -> 1.12, 16 -> 1.04,
// 32 -> 1.12 for both passes, round 3)
constexpr int kRsItems = 16;
// scatter workgroup (a step is kRsThreads * kRsItems pairs; config 5 both passes: 256 -> 647 us,
// 512 -> 639, 1024 -> 811 per frame)
constexpr int kRsThreads = 512;
constexpr uint32_t kRsMaxBlocks = 512;
static_assert(kRsMaxBlocks <= kMaxSortBlocks, "histogram rows");
// The keys are staged in LDS at their input width (u16 between the tile passes) and no per-item
// digit / valid arrays are kept (recomputed from the key and the index): 38.9 -> 30.7 KB of LDS per
// 256 threads, 650 -> 645 us per config-5 frame. (More waves per SIMD instead of items per thread:
// 12 items at 5 waves 673 us, 8 items at 6 waves 735 us.)
template <typename KI, typename KO, int NT>
__global__ __launch_bounds__(NT) void radix_scatter_kernel(
    const KI* __restrict__ keys_in, const uint32_t* __restrict__ vals_in,
    const uint32_t* n_dev, uint32_t n_host, uint32_t shift, uint32_t nbits,
    const uint32_t* hist, const uint32_t* __restrict__ totals,
    KO* __restrict__ keys_out, uint32_t* __restrict__ vals_out,
    uint32_t* __restrict__ inverse_out, uint2* __restrict__ ranges_out, uint32_t* hist_clear) {
    using SK = KI;
    constexpr uint32_t NW = NT / 64, kRsTile = NT * kRsItems;
    static_assert(NT >= 256 && NT % 64 == 0, "threads 0..255 own the digits");
    __shared__ uint32_t s_off[256];               // running global start of each digit
    __shared__ uint32_t s_cnt[NW][256];           // per-wave counts -> per-wave local offsets
    __shared__ uint32_t s_loc[256];               // block-local start of each digit in the step
    __shared__ SK s_key[kRsTile];
    __shared__ uint32_t s_val[kRsTile];
    __shared__ uint32_t s_ws[4];
    const uint32_t t = threadIdx.x, w = t >> 6, lane = t & 63u;
    const bool dig = t < 256u;  // this thread owns digit t
    const uint32_t mask = (1u << nbits) - 1u;

    // digit bases: exclusive scan of totals
    if (dig) s_loc[t] = totals[t];
    __syncthreads();
    for (uint32_t o = 1; o < 256; o <<= 1) {
        const uint32_t v = (dig && t >= o) ? s_loc[t - o] : 0u;
        __syncthreads();
        if (dig) s_loc[t] += v;
        __syncthreads();
    }
    if (dig) s_off[t] = (t ? s_loc[t - 1] : 0u) + hist[t * gridDim.x + blockIdx.x];
    // (hist_clear: the last pass leaves the histogram zero for the next frame's emission, which
    // counts the first pass's digits into it; each block clears the column only it reads)
    if (dig && hist_clear) hist_clear[t * gridDim.x + blockIdx.x] = 0u;
    __syncthreads();

    const uint32_t n = sort_count(n_dev, n_host);
    uint32_t begin, end;
    sort_slice(n, blockIdx.x, gridDim.x, begin, end);
    const uint64_t lt = lanemask_lt();

    // (loading the next step while this one is ranked -- 167 VGPRs, 3 waves per SIMD -- made both
    // config-5 passes slower: 656 -> 716 us per frame, scripts/ab_cfg5.sh)
    for (uint32_t step = begin; step < end; step += kRsTile) {
        const uint32_t ibase = step + w * (kRsItems * 64u) + lane;
        uint32_t k[kRsItems], v[kRsItems], rk[kRsItems];
        auto okf = [&](int i) { return ibase + (uint32_t)i * 64u < end; };
        auto dgf = [&](int i) { return (k[i] >> shift) & mask; };
#pragma unroll
        for (int i = 0; i < kRsItems; i++) {
            const uint32_t idx = ibase + (uint32_t)i * 64u;
            const bool in = idx < end;
            k[i] = in ? (uint32_t)keys_in[idx] : 0u;
            v[i] = vals_in ? (in ? vals_in[idx] : 0u) : idx;
        }
#pragma unroll
        for (int j = 0; j < 4; j++) s_cnt[w][lane + 64u * j] = 0u;
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int i = 0; i < kRsItems; i++) {
            const bool oki = okf(i);
            const uint32_t d = dgf(i);
            uint64_t m = __ballot(oki);
            for (uint32_t bit = 0; bit < nbits; bit++) {
                const bool on = (d >> bit) & 1u;
                const uint64_t bb = __ballot(on);
                m &= on ? bb : ~bb;
            }
            const uint32_t below = (uint32_t)__popcll(m & lt);
            uint32_t c = 0;
            if (oki) c = s_cnt[w][d];
            __builtin_amdgcn_wave_barrier();
            rk[i] = c + below;
            const uint32_t leader = 63u - (uint32_t)__clzll(m);
            if (oki && lane == leader) s_cnt[w][d] = c + (uint32_t)__popcll(m);
            __builtin_amdgcn_wave_barrier();
        }
        __syncthreads();
        // per digit (thread t = digit): wave offsets within the digit, digit total of the step
        uint32_t tot = 0;
        if (dig) {
#pragma unroll
            for (uint32_t ww = 0; ww < NW; ww++) {
                const uint32_t c = s_cnt[ww][t];
                s_cnt[ww][t] = tot;
                tot += c;
            }
        }
        // block-local exclusive scan of the digit totals -> s_loc (wave shuffles: two barriers
        // instead of the sixteen of a Hillis-Steele scan in LDS; every thread takes the barriers)
        const uint32_t ex = scan256_excl(tot, t, s_ws);
        if (dig) s_loc[t] = ex;
        lds_barrier();
        // reorder the step by digit in LDS
#pragma unroll
        for (int i = 0; i < kRsItems; i++) {
            if (!okf(i)) continue;
            const uint32_t d = dgf(i);
            const uint32_t lp = s_loc[d] + s_cnt[w][d] + rk[i];
            s_key[lp] = (SK)k[i];
            s_val[lp] = v[i];
        }
        __syncthreads();
        const uint32_t cnt = min(kRsTile, end - step);
        for (uint32_t i = t; i < cnt; i += NT) {
            const uint32_t kk = s_key[i], vv = s_val[i];
            const uint32_t d = (kk >> shift) & mask;
            const uint32_t pos = s_off[d] + (i - s_loc[d]);
            if (keys_out) keys_out[pos] = (KO)kk;
            if (vals_out) vals_out[pos] = vv;
            if (inverse_out) inverse_out[vv] = pos;
            if (ranges_out) {  // (an equal key is always in the same digit run of the step)
                if (i == 0u || (uint32_t)s_key[i - 1u] != kk) atomicMin(&ranges_out[kk].x, pos);
                if (i + 1u == cnt || (uint32_t)s_key[i + 1u] != kk) atomicMax(&ranges_out[kk].y, pos + 1u);
            }
        }
        __syncthreads();
        if (dig) s_off[t] += tot;
        __syncthreads();
    }
}


// ---- one-pass stable counting sort of the pairs by tile key (T <= kTileSortMaxTiles) ----------
// The tile key has only ceil(log2 T) significant bits (13 at 1080p; read as u16), so instead of two
// LSD passes the pairs are counted once per (block, tile) and scattered once:
//   tile_hist      per-block tile counts -> hist[b][t] (block-major rows, coalesced);
//   tile_colscan   per tile, exclusive prefixes over blocks inside chunks of 16 blocks (in place)
//                  and the chunk totals csum[c][t];
//   tile_finish    per tile, exclusive prefixes over the chunks (in place) and the tile total;
//                  across the tiles (full fan-in) the ranges, the list-chunk bases and the
//                  forward's launch order (no separate ranges pass);
//   tile_scatter   each wave owns a contiguous quarter of its block's slice; per-wave tile counts
//                  (packed u16 pairs in LDS) give the wave prefixes, then rows are ranked with
//                  ballots. Order inside a tile = memory order = depth order: stable.
// Only the packed values are written; the sorted keys are implied by the ranges. Every loop over
// global memory issues 8 independent loads per lane before using them (1 block per CU here, so
// latency is hidden by batching, not by occupancy).
constexpr uint32_t kColChunk = 16;

// Blocks actually used for P pairs. The grid is sized from the host's bound on P (which may be
// the whole pair capacity); blocks past the count derived from the device-resident P exit at once,
// so the histogram and the column scans are sized by the real P.
__host__ __device__ inline uint32_t tile_blocks_for(uint64_t p) {
    uint64_t b = (p + 4 * kSortTile - 1) / (4 * kSortTile);
    if (b > kTileSortMaxBlocks) b = kTileSortMaxBlocks;
    if (b < 1) b = 1;
    return (uint32_t)b;
}

__global__ __launch_bounds__(kSortThreads) void tile_hist_kernel(const uint16_t* __restrict__ keys,
                                                                 const uint32_t* n_dev, uint32_t T,
                                                                 uint32_t* __restrict__ hist,
                                                                 uint32_t* __restrict__ zero_words,
                                                                 uint32_t nzero) {
    extern __shared__ uint32_t h_tile[];
    const uint32_t n = *n_dev, B = tile_blocks_for(n);
    const uint32_t t = threadIdx.x;
    // the tile-level scan's status words (tile_finish_kernel), zeroed here instead of by a memset
    for (uint32_t z = blockIdx.x * kSortThreads + t; z < nzero; z += gridDim.x * kSortThreads) zero_words[z] = 0u;
    for (uint32_t vb = blockIdx.x; vb < B; vb += gridDim.x) {  // grid <= kTileSortMaxBlocks
        for (uint32_t d = t; d < T; d += kSortThreads) h_tile[d] = 0u;
        __syncthreads();
        uint32_t begin, end;
        sort_slice(n, vb, B, begin, end);
        for (uint32_t r = begin; r < end; r += kSortTile) {
            uint32_t d[kSortItems];
#pragma unroll
            for (int k = 0; k < kSortItems; k++) {
                const uint32_t i = r + (uint32_t)k * kSortThreads + t;
                d[k] = i < end ? (uint32_t)keys[i] : 0xffffffffu;
            }
#pragma unroll
            for (int k = 0; k < kSortItems; k++)
                if (d[k] < T) atomicAdd(&h_tile[d[k]], 1u);
        }
        __syncthreads();
        uint32_t* row = hist + (size_t)vb * T;
        for (uint32_t d = t; d < T; d += kSortThreads) row[d] = h_tile[d];
        __syncthreads();
    }
}

__global__ __launch_bounds__(256) void tile_colscan_kernel(uint32_t* __restrict__ hist, uint32_t T,
                                                           const uint32_t* n_dev,
                                                           uint32_t* __restrict__ csum, uint32_t b_fixed) {
    const uint32_t d = blockIdx.x * 256u + threadIdx.x;
    const uint32_t B = b_fixed ? b_fixed : tile_blocks_for(*n_dev);
    if (d >= T) return;
    for (uint32_t c = blockIdx.y; c * kColChunk < B; c += gridDim.y) {
        const uint32_t b0 = c * kColChunk;
        const uint32_t bn = min(kColChunk, B - b0);
        uint32_t v[kColChunk];
#pragma unroll
        for (uint32_t k = 0; k < kColChunk; k++) v[k] = k < bn ? hist[(size_t)(b0 + k) * T + d] : 0u;
        uint32_t run = 0;
#pragma unroll
        for (uint32_t k = 0; k < kColChunk; k++) {
            if (k < bn) hist[(size_t)(b0 + k) * T + d] = run;
            run += v[k];
        }
        csum[(size_t)c * T + d] = run;
    }
}

__device__ __forceinline__ uint32_t half16(uint32_t word, uint32_t d) { return (word >> (16u * (d & 1u))) & 0xffffu; }

template <int W>
__global__ __launch_bounds__(64 * W) void tile_scatter_kernel(
    const uint16_t* __restrict__ keys, const uint32_t* __restrict__ vals, const uint32_t* n_dev,
    uint32_t T, uint32_t nbits, const uint32_t* __restrict__ hist, const uint32_t* __restrict__ csum,
    const uint2* __restrict__ ranges, uint32_t* __restrict__ vals_out) {
    constexpr uint32_t NT = 64u * W;
    constexpr int R = kSortItems;  // rows per batch
    extern __shared__ uint32_t sm_tile[];
    const uint32_t n = *n_dev, B = tile_blocks_for(n);
    const uint32_t Th = (T + 1u) >> 1;
    uint32_t* base = sm_tile;         // [T] global start of each tile's run for this block
    uint32_t* rel = sm_tile + T;      // [W][Th] packed u16 per-wave counters (see phase 2)
    const uint32_t t = threadIdx.x, w = t >> 6, lane = t & 63u;
    const uint64_t lt = lanemask_lt();
    uint32_t* wrel = rel + w * Th;
    // XCD-aware slice order: workgroups are dispatched round-robin over the 8 XCDs, so with a grid
    // of a multiple of 8 the workgroups of XCD x take the consecutive slices [x Q, (x + 1) Q). Each
    // tile's output segment is then written in 8 contiguous parts, each from one L2, which merges
    // the short per-slice runs into whole lines before they leave (the runs average ~2 pairs:
    // without this every store is a partial line).
    const bool xcdmap = (gridDim.x & 7u) == 0u;
    const uint32_t Q = (B + 7u) >> 3;
    for (uint32_t it = blockIdx.x; xcdmap ? (it >> 3) < Q : it < B; it += gridDim.x) {  // grid <= kTileSortMaxBlocks
        const uint32_t vb = xcdmap ? (it & 7u) * Q + (it >> 3) : it;
        if (vb >= B) continue;
        uint32_t begin, end;
        sort_slice(n, vb, B, begin, end);
        // base gathers in flight while the counters are cleared
        const uint32_t* hrow = hist + (size_t)vb * T;
        const uint32_t* crow = csum + (size_t)(vb / kColChunk) * T;
        for (uint32_t d0 = 0; d0 < T; d0 += R * NT) {
            uint32_t x[R];
#pragma unroll
            for (int k = 0; k < R; k++) {
                const uint32_t d = d0 + (uint32_t)k * NT + t;
                x[k] = d < T ? ranges[d].x + crow[d] + hrow[d] : 0u;
            }
            if (d0 == 0)
                for (uint32_t q = t; q < W * Th; q += NT) rel[q] = 0u;
#pragma unroll
            for (int k = 0; k < R; k++) {
                const uint32_t d = d0 + (uint32_t)k * NT + t;
                if (d < T) base[d] = x[k];
            }
        }
        // the slice in chunks of at most kTileSortMaxSlice pairs, so every packed u16 counter fits
        for (uint32_t cb = begin; cb < end; cb += (uint32_t)kTileSortMaxSlice) {
            const uint32_t ce = min(cb + (uint32_t)kTileSortMaxSlice, end);
            uint32_t per = (ce - cb + W - 1u) / W;
            per = (per + 63u) & ~63u;
            const uint32_t wb = min(cb + w * per, ce), we = min(wb + per, ce);
            __syncthreads();
            if (cb != begin) {  // re-arm the counters (a wave's count keeps the later waves' share)
                for (uint32_t q = t; q < W * Th; q += NT) rel[q] = 0u;
                __syncthreads();
            }
            // phase 1: per-wave tile counts of the chunk
            for (uint32_t r = wb; r < we; r += R * 64u) {
                uint32_t d[R];
#pragma unroll
                for (int k = 0; k < R; k++) {
                    const uint32_t i = r + (uint32_t)k * 64u + lane;
                    d[k] = i < we ? (uint32_t)keys[i] : 0xffffffffu;
                }
#pragma unroll
                for (int k = 0; k < R; k++)
                    if (d[k] < T) atomicAdd(&wrel[d[k] >> 1], 1u << (16u * (d[k] & 1u)));
            }
            __syncthreads();
            // phase 2 (both halves of a word by one thread): counts -> per-wave "remaining" counts
            // (this and later waves' pairs of the tile), and base advances to the end of the
            // chunk's run. Phase 3 places a pair at base - remaining + (rank in its row) and
            // counts its own wave's remaining down.
            for (uint32_t q = t; q < Th; q += NT) {
                uint32_t c[W];
#pragma unroll
                for (int ww = 0; ww < W; ww++) c[ww] = rel[ww * Th + q];
                uint32_t lo = 0, hi = 0;
#pragma unroll
                for (int ww = W - 1; ww >= 0; ww--) {
                    lo += c[ww] & 0xffffu;
                    hi += c[ww] >> 16;
                    rel[ww * Th + q] = lo | (hi << 16);
                }
                base[2u * q] += lo;
                if (2u * q + 1u < T) base[2u * q + 1u] += hi;
            }
            __syncthreads();
            // phase 3: rank rows in memory order, next batch's loads in flight. The match masks of
            // a batch are independent (interleaved by the compiler); the counter reads and
            // decrements go back to back (LDS operations of a wave complete in order, so row k+1
            // reads the count after row k's update).
            uint32_t nd[R], nv[R];
#pragma unroll
            for (int k = 0; k < R; k++) {
                const uint32_t i = wb + (uint32_t)k * 64u + lane;
                nd[k] = i < we ? (uint32_t)keys[i] : 0u;
                nv[k] = i < we ? vals[i] : 0u;
            }
            for (uint32_t r = wb; r < we; r += R * 64u) {
                uint32_t d[R], v[R];
#pragma unroll
                for (int k = 0; k < R; k++) {
                    d[k] = nd[k];
                    v[k] = nv[k];
                }
                const uint32_t rn = r + R * 64u;
                if (rn < we) {
#pragma unroll
                    for (int k = 0; k < R; k++) {
                        const uint32_t i = rn + (uint32_t)k * 64u + lane;
                        nd[k] = i < we ? (uint32_t)keys[i] : 0u;
                        nv[k] = i < we ? vals[i] : 0u;
                    }
                }
                uint64_t m[R];
#pragma unroll
                for (int k = 0; k < R; k++) m[k] = __ballot(r + (uint32_t)k * 64u + lane < we);
                for (uint32_t bit = 0; bit < nbits; bit++) {
#pragma unroll
                    for (int k = 0; k < R; k++) {
                        const bool on = (d[k] >> bit) & 1u;
                        const uint64_t bb = __ballot(on);
                        m[k] &= on ? bb : ~bb;
                    }
                }
                // Every lane issues the counter update (the group leader subtracts the group's size,
                // the others 0), so the batch's LDS operations go out back to back without exec-mask
                // branches; the leader's returned value (this wave's remaining count of the tile,
                // this row included) is then fetched by its group with ds_bpermute.
                uint32_t old[R], bs[R], pos[R];
#pragma unroll
                for (int k = 0; k < R; k++) {
                    const bool ok = r + (uint32_t)k * 64u + lane < we;
                    const uint32_t leader = 63u - (uint32_t)__clzll(m[k]);
                    const uint32_t dec = (ok && lane == leader) ? (uint32_t)__popcll(m[k]) << (16u * (d[k] & 1u)) : 0u;
                    old[k] = __hip_atomic_fetch_sub(&wrel[d[k] >> 1], dec, __ATOMIC_RELAXED,
                                                    __HIP_MEMORY_SCOPE_WORKGROUP);
                }
#pragma unroll
                for (int k = 0; k < R; k++) bs[k] = base[d[k]];
#pragma unroll
                for (int k = 0; k < R; k++) {
                    const uint32_t leader = 63u - (uint32_t)__clzll(m[k]);
                    const uint32_t lold = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(leader << 2), (int)old[k]);
                    pos[k] = bs[k] + (uint32_t)__popcll(m[k] & lt) - half16(lold, d[k]);
                }
#pragma unroll
                for (int k = 0; k < R; k++)
                    if (r + (uint32_t)k * 64u + lane < we) vals_out[pos[k]] = v[k];
            }
        }
        __syncthreads();
    }
}

// ---- the one-pass tile sort straight from the Gaussians (per-tile depth sort path) ----------
// The pairs are never written in Gaussian order: the histogram counts each slice's Gaussians' rects
// (tile_hist_rect_kernel) and the scatter walks their pairs (wave_walk_pairs, the emission's own
// walk), so the 6 B per pair of emitted keys and values are neither written nor read twice. Slice
// vb = the wave chunks (64 Gaussians) [vb C / B, (vb + 1) C / B).
//   kOwn = false: the slot offsets goff and P come from offsets_scan_kernel; B = tile_blocks_for(P)
//     as the colscan / finish kernels read it; block 0 of the histogram does the emission's frame
//     duties.
//   kOwn = true (the pair buffers hold the worst case, so no slot can overflow): no offset scan. The
//     scatter's walk numbers the slots inside each wave (a DPP scan of the counts); the histogram keeps
//     each chunk's and each slice's pair count (chunk_tot, slice_tot) and resets the frame's error
//     words (frame_reset, before tile_finish can set one); the scatter derives from the counts the
//     slice's first slot, each chunk's first slot and so goff and the raster records' slot field
//     (what offsets_scan_kernel wrote), and P, which its block 0 stores and publishes
//     (frame_publish). B = b_fixed, from N.
constexpr uint32_t kGidThreads = 1024;
constexpr uint32_t kGidWaves = kGidThreads / 64u;
__device__ __forceinline__ void gid_slice(uint32_t n, uint32_t vb, uint32_t B, uint32_t& c0, uint32_t& c1) {
    const uint64_t nch = (n + 63u) / 64u;
    c0 = (uint32_t)(nch * vb / B);
    c1 = (uint32_t)(nch * (vb + 1u) / B);
}

// The histogram without walking the pairs: a Gaussian's pairs are exactly the tiles of its rect
// (count = the rect's area), so a slice's per-tile counts are the 2-D prefix sums of a difference grid
// with +1 / -1 at the rect's four corners: 4 LDS atomics per Gaussian instead of one per pair, then
// one DPP scan per grid row and one per grid column (a wave each). (The pairs beyond the buffers'
// capacity never need cutting here: the forward grows the buffers to P before the tile sort.)
template <bool kOwn>
__global__ __launch_bounds__(kGidThreads) void tile_hist_rect_kernel(
    uint32_t n, const uint32_t* __restrict__ count, const uint2* __restrict__ rect, uint32_t tiles_x,
    const uint32_t* p_dev, uint64_t cap, uint32_t T, uint32_t* __restrict__ hist, uint32_t* __restrict__ zero_words,
    uint32_t nzero, uint32_t* __restrict__ overflow, uint32_t* __restrict__ host_mirror,
    uint32_t* __restrict__ hist_rezero, uint32_t b_fixed, uint32_t* __restrict__ slice_tot,
    uint32_t* __restrict__ chunk_tot) {
    extern __shared__ uint32_t D[];  // [(tiles_y + 1) (tiles_x + 1)] difference grid, then the slice total
    const uint32_t tiles_y = T / tiles_x, px = tiles_x + 1u, cells = (tiles_y + 1u) * px;
    const uint32_t P = kOwn ? 0u : *p_dev, B = kOwn ? b_fixed : tile_blocks_for(P);
    const uint32_t t = threadIdx.x, lane = t & 63u, w = t >> 6;
    // (the frame's error words are reset here, before tile_finish can set one; with kOwn P is only
    // known to the scatter, which publishes it)
    if (blockIdx.x == 0) {
        if (kOwn)
            frame_reset(t, kGidThreads, overflow, host_mirror, hist_rezero);
        else
            emit_frame_duties(t, kGidThreads, P, cap, overflow, host_mirror, hist_rezero);
    }
    for (uint32_t z = blockIdx.x * kGidThreads + t; z < nzero; z += gridDim.x * kGidThreads) zero_words[z] = 0u;
    for (uint32_t vb = blockIdx.x; vb < B; vb += gridDim.x) {
        for (uint32_t d = t; d <= cells; d += kGidThreads) D[d] = 0u;
        __syncthreads();
        uint32_t c0, c1;
        gid_slice(n, vb, B, c0, c1);
        // two chunks per step, each lane's count and rect loaded together (no dependent round trip)
        for (uint32_t c = c0 + w; c < c1; c += 2u * kGidWaves) {
            uint32_t cnt[2];
            uint2 r[2];
#pragma unroll
            for (uint32_t h = 0; h < 2u; h++) {
                const uint32_t i = (c + h * kGidWaves) * 64u + lane;
                const bool ok = c + h * kGidWaves < c1 && i < n;
                cnt[h] = ok ? count[i] : 0u;
                r[h] = ok ? rect[i] : make_uint2(0u, 0u);
            }
#pragma unroll
            for (uint32_t h = 0; h < 2u; h++) {
                const uint32_t ch = c + h * kGidWaves;
                if (kOwn && ch < c1) {
                    const uint32_t tot = (uint32_t)__builtin_amdgcn_readlane((int)wave_scan_dpp(cnt[h], 0u, DppAdd{}), 63);
                    if (lane == 0) {
                        chunk_tot[ch] = tot;
                        atomicAdd(&D[cells], tot);
                    }
                }
                if (cnt[h]) {
                    const uint32_t x0 = r[h].x & 0xffffu, y0 = r[h].x >> 16;
                    const uint32_t x1 = (r[h].y & 0xffffu) + 1u, y1 = (r[h].y >> 16) + 1u;  // (exclusive)
                    atomicAdd(&D[y0 * px + x0], 1u);
                    atomicAdd(&D[y0 * px + x1], 0xffffffffu);
                    atomicAdd(&D[y1 * px + x0], 0xffffffffu);
                    atomicAdd(&D[y1 * px + x1], 1u);
                }
            }
        }
        __syncthreads();
        for (uint32_t y = w; y < tiles_y; y += kGidWaves) {  // along x, one wave per row
            uint32_t carry = 0;
            for (uint32_t x0 = 0; x0 < tiles_x; x0 += 64u) {
                const uint32_t x = x0 + lane;
                const uint32_t v = x < tiles_x ? D[y * px + x] : 0u;
                const uint32_t inc = wave_scan_dpp(v, 0u, DppAdd{});
                if (x < tiles_x) D[y * px + x] = carry + inc;
                carry += (uint32_t)__builtin_amdgcn_readlane((int)inc, 63);
            }
        }
        __syncthreads();
        for (uint32_t x = w; x < tiles_x; x += kGidWaves) {  // along y, one wave per column
            uint32_t carry = 0;
            for (uint32_t y0 = 0; y0 < tiles_y; y0 += 64u) {
                const uint32_t y = y0 + lane;
                const uint32_t v = y < tiles_y ? D[y * px + x] : 0u;
                const uint32_t inc = wave_scan_dpp(v, 0u, DppAdd{});
                if (y < tiles_y) D[y * px + x] = carry + inc;
                carry += (uint32_t)__builtin_amdgcn_readlane((int)inc, 63);
            }
        }
        __syncthreads();
        uint32_t* row = hist + (size_t)vb * T;
        for (uint32_t y = w; y < tiles_y; y += kGidWaves)
            for (uint32_t x = lane; x < tiles_x; x += 64u) row[y * tiles_x + x] = D[y * px + x];
        if (kOwn && t == 0) slice_tot[vb] = D[cells];
        __syncthreads();
    }
}

template <bool kOwn>
__global__ __launch_bounds__(kGidThreads) void tile_scatter_gid_kernel(
    uint32_t n, const uint32_t* __restrict__ count, uint32_t* __restrict__ goff, const uint2* __restrict__ rect,
    uint32_t tiles_x, uint32_t* p_dev, uint64_t cap, uint32_t T, const uint32_t* __restrict__ hist,
    const uint32_t* __restrict__ csum, const uint2* __restrict__ ranges, uint32_t* __restrict__ vals_out,
    uint32_t b_fixed, const uint32_t* __restrict__ slice_tot, const uint32_t* __restrict__ chunk_tot,
    float4* __restrict__ rec, uint32_t* __restrict__ overflow,
    uint32_t* __restrict__ host_mirror, uint32_t* __restrict__ hist_rezero, uint32_t ncofs, uint32_t scap) {
    extern __shared__ uint32_t cur[];  // [T] next slot of each tile's run for this slice; [2] (P);
                                       // [16] wave sums; [ncofs] (kOwn) the slice's chunks' first
                                       // slots; [scap] staged values; [scap] u16 staged tiles
    uint32_t* const sb = cur + T;
    uint32_t* const wsum = cur + T + 2u;
    uint32_t* const cofs = cur + T + 2u + kGidWaves;
    uint32_t* const svals = cofs + ncofs;
    uint16_t* const stile = reinterpret_cast<uint16_t*>(svals + scap);
    const uint32_t t = threadIdx.x, lane = t & 63u, w = t >> 6;
    uint32_t P = 0, B = b_fixed;
    if (kOwn) {
        // every slice's pair count (<= 256 of them): this block's base is the sum of those before
        if (w == 0) {
            uint32_t all = 0;
            for (uint32_t s0 = 0; s0 < B; s0 += 64u) all += s0 + lane < B ? slice_tot[s0 + lane] : 0u;
            all = (uint32_t)__builtin_amdgcn_readlane((int)wave_scan_dpp(all, 0u, DppAdd{}), 63);
            if (lane == 0) sb[1] = all;
        }
        __syncthreads();
        P = sb[1];
        if (blockIdx.x == 0) {
            if (t == 0) *p_dev = P;
            frame_publish(t, P, cap, overflow, host_mirror);
        }
    } else {
        P = *p_dev;
        B = tile_blocks_for(P);
    }
    const uint32_t stop = kOwn ? 0xffffffffu : ((uint64_t)P < cap ? P : (uint32_t)cap);
    // XCD-aware slice order (as tile_scatter_kernel): XCD x takes the consecutive slices [x Q, x Q + Q)
    const bool xcdmap = (gridDim.x & 7u) == 0u;
    const uint32_t Q = (B + 7u) >> 3;
    for (uint32_t it = blockIdx.x; xcdmap ? (it >> 3) < Q : it < B; it += gridDim.x) {
        const uint32_t vb = xcdmap ? (it & 7u) * Q + (it >> 3) : it;
        if (vb >= B) continue;
        const uint32_t* hrow = hist + (size_t)vb * T;
        const uint32_t* crow = csum + (size_t)(vb / kColChunk) * T;
        const bool more = vb + 1u < B;
        const uint32_t* hnext = hist + (size_t)(more ? vb + 1u : vb) * T;
        const uint32_t* cnext = csum + (size_t)((more ? vb + 1u : vb) / kColChunk) * T;
        // Tile d's run for this slice is [G, Gn) of the sorted list (G from this slice's column
        // prefix, Gn from the next slice's, or the range end). Staged (the slice's pairs fit the LDS
        // stage): the pairs are placed tile by tile in LDS at local offsets (an exclusive scan of
        // the run lengths), then written out in that order, so the stores of a wave hit consecutive
        // addresses inside each run instead of one scattered 4-B store per pair.
        bool staged = false;
        uint32_t total = 0;
        {
            // wave w owns the tiles [w tw, w tw + tw), 64 consecutive tiles per round: coalesced loads
            // of the ranges and column prefixes, conflict-free LDS stores of the cursors (a thread owning
            // 8 consecutive tiles put every fourth lane on one bank)
            constexpr uint32_t kRounds = (kTileSortMaxTiles + kGidThreads - 1u) / kGidThreads;
            const uint32_t tw = (((T + kGidWaves - 1u) / kGidWaves) + 63u) & ~63u;
            uint32_t g[kRounds], run_in[kRounds], wtot = 0;
#pragma unroll
            for (uint32_t k = 0; k < kRounds; k++) {
                const uint32_t d = w * tw + k * 64u + lane;
                uint32_t len = 0;
                g[k] = 0u;
                if (k * 64u < tw && d < T) {
                    const uint2 rg = ranges[d];
                    g[k] = rg.x + crow[d] + hrow[d];
                    len = (more ? rg.x + cnext[d] + hnext[d] : rg.y) - g[k];
                }
                const uint32_t inc = k * 64u < tw ? wave_scan_dpp(len, 0u, DppAdd{}) : 0u;
                run_in[k] = wtot + inc - len;
                wtot += (uint32_t)__builtin_amdgcn_readlane((int)inc, 63);
            }
            if (lane == 0) wsum[w] = wtot;
            __syncthreads();
            uint32_t run = 0;
#pragma unroll
            for (uint32_t k = 0; k < kGidWaves; k++) {
                run += k < w ? wsum[k] : 0u;
                total += wsum[k];
            }
            staged = total <= scap;
#pragma unroll
            for (uint32_t k = 0; k < kRounds; k++) {
                const uint32_t d = w * tw + k * 64u + lane;
                if (k * 64u < tw && d < T) cur[d] = staged ? run + run_in[k] : g[k];
            }
        }
        uint32_t c0, c1;
        gid_slice(n, vb, B, c0, c1);
        if (kOwn && w == 0) {
            // the slice's first slot (the pair counts of the slices before it), then each chunk's
            // first slot: the exclusive scan of the chunks' pair counts (the histogram's) in order
            uint32_t run = 0;
            for (uint32_t s0 = 0; s0 < vb; s0 += 64u) run += s0 + lane < vb ? slice_tot[s0 + lane] : 0u;
            run = (uint32_t)__builtin_amdgcn_readlane((int)wave_scan_dpp(run, 0u, DppAdd{}), 63);
            for (uint32_t k0 = 0; k0 < c1 - c0; k0 += 64u) {
                const uint32_t x = k0 + lane < c1 - c0 ? chunk_tot[c0 + k0 + lane] : 0u;
                const uint32_t inc = wave_scan_dpp(x, 0u, DppAdd{});
                if (k0 + lane < c1 - c0) cofs[k0 + lane] = run + inc - x;
                run += (uint32_t)__builtin_amdgcn_readlane((int)inc, 63);
            }
        }
        __syncthreads();
        // each chunk's counts, rects (and goff) loaded one chunk ahead: the next chunk's loads are in
        // flight while this one is walked
        auto load_chunk = [&](uint32_t c, uint32_t& cg, uint2& r, uint32_t& go) {
            const uint32_t i = c * 64u + lane;
            const bool ok = c < c1 && i < n;
            cg = ok ? count[i] : 0u;
            r = ok ? rect[i] : make_uint2(0u, 0u);
            if (!kOwn) go = ok ? goff[i] : 0xffffffffu;  // past n: never a slot's Gaussian
        };
        uint32_t cgN = 0, goN = 0;
        uint2 rN = make_uint2(0u, 0u);
        load_chunk(c0 + w, cgN, rN, goN);
        for (uint32_t c = c0 + w; c < c1; c += kGidWaves) {
            auto place = [&](uint32_t, uint32_t tile, uint32_t v) {
                const uint32_t p = atomicAdd(&cur[tile], 1u);
                if (staged) {
                    svals[p] = v;
                    stile[p] = (uint16_t)tile;
                } else {
                    vals_out[p] = v;
                }
            };
            const uint32_t cg = cgN, go = goN;
            const uint2 r = rN;
            load_chunk(c + kGidWaves, cgN, rN, goN);
            if (kOwn) {
                const uint32_t inc = wave_scan_dpp(cg, 0u, DppAdd{});
                const uint32_t o = inc - cg;  // the slot offsets inside the wave
                // the backward's partial-sum slots in Gaussian order (offsets_scan_kernel's goff and
                // the raster record's quad 3)
                const uint32_t i = c * 64u + lane;
                const uint32_t g = cofs[c - c0] + o;
                if (i < n) {
                    goff[i] = g;
                    if (cg) reinterpret_cast<uint32_t*>(rec + (size_t)i * kRecQuads + 3)[0] = g;
                }
                wave_walk_pairs_rect(c * 64u, n, lane, cg, o, r, tiles_x, stop, place);
            } else {
                wave_walk_pairs_rect(c * 64u, n, lane, cg, go, r, tiles_x, stop, place);
            }
        }
        __syncthreads();
        if (staged) {
            // a staged entry k of tile d goes to Gn - (d's local end) + k: cur[d] is now the end
            for (uint32_t d = t; d < T; d += kGidThreads)
                cur[d] = (more ? ranges[d].x + cnext[d] + hnext[d] : ranges[d].y) - cur[d];
            __syncthreads();
            for (uint32_t k = t; k < total; k += kGidThreads) vals_out[cur[stile[k]] + k] = svals[k];
            __syncthreads();
        }
    }
}

// XCD-group launch slot (gs_internal.hpp) of the tile with rank `rank` in the runs-in-order ranking
// (run x's tiles at [q[x], q[x + 1]), longest first): rank r in run x -> slot 8 r + x while the run
// has slots (ceil((T - x) / 8) of them); the e-th surplus tile overall takes the e-th free slot (runs
// in order, slots ascending). A bijection onto [0, T): the surplus equals the free slots.
__device__ uint32_t xcd_slot(uint32_t rank, uint32_t run, const uint32_t* q, uint32_t T) {
    const uint32_t r = rank - q[run];
    const uint32_t cap = (T - run + kXcdGroups - 1u) / kXcdGroups;
    if (r < cap) return r * kXcdGroups + run;
    uint32_t e = r - cap;
    for (uint32_t x = 0; x < run; x++) {
        const uint32_t len = q[x + 1] - q[x], cx = (T - x + kXcdGroups - 1u) / kXcdGroups;
        e += len > cx ? len - cx : 0u;
    }
    for (uint32_t x = 0; x < kXcdGroups; x++) {
        const uint32_t len = q[x + 1] - q[x], cx = (T - x + kXcdGroups - 1u) / kXcdGroups;
        const uint32_t fr = cx > len ? cx - len : 0u;
        if (e < fr) return (len + e) * kXcdGroups + x;
        e -= fr;
    }
    return rank;  // not reached
}

// Per tile: exclusive prefixes of the chunk totals (in place) and the tile total; then, across the
// tiles, the ranges (exclusive scan of the totals), the list-chunk bases (scan of ceil(len / 64))
// and the blend launch order. One tile per thread, at most kFinBlocks blocks, all resident at once,
// two rounds of full fan-in over flagged 64-bit words (every block reads every block's words; no
// chain of inclusive prefixes): round 1 the blocks' two sums (-> ranges, chunk bases and the total
// work), round 2 the blocks' 256 launch-bucket counts. The launch order is bucketed by list length,
// longest first; in XCD-group order (gs_internal.hpp) a bucket is (work run x, 32 log-length levels),
// whose scan ranks every tile inside its run, and the rank gives the launch slot. The order inside a
// bucket is irrelevant to the results.
constexpr uint32_t kFinBlocks = (kTileSortMaxTiles + 255u) / 256u;
constexpr uint32_t kFinWords = 2u + 256u;  // per block: total, chunk total, 256 bucket counts
constexpr float kFwdLevels = 2.5f;  // log-length levels per doubling inside an XCD group (32 levels)
constexpr unsigned long long kFinFlag = 1ull << 63;
// bits of the frame's fan-in error word (GsFrameStats.scan_errors) set by a give-up spin
constexpr uint32_t kFanInErrFinish = 16u, kFanInErrReorder = 32u;

__global__ __launch_bounds__(256) void tile_finish_kernel(uint32_t* __restrict__ csum, uint32_t T,
                                                          const uint32_t* n_dev, unsigned long long* fin,
                                                          uint2* __restrict__ ranges, uint32_t* __restrict__ order,
                                                          uint32_t* __restrict__ chunk_base,
                                                          uint32_t* __restrict__ tile_cost,
                                                          unsigned long long* __restrict__ reorder_words,
                                                          uint32_t* __restrict__ err, uint32_t xcd,
                                                          uint32_t* __restrict__ xgroup, uint32_t b_fixed) {
    __shared__ uint32_t s_cnt[256];
    __shared__ uint64_t s_ws[2][4];
    __shared__ uint32_t s_bs[4];
    __shared__ uint64_t s_pre[3];
    __shared__ uint32_t s_q[kXcdGroups + 1];
    const uint32_t t = threadIdx.x, lane = t & 63u, wv = t >> 6, b = blockIdx.x;
    const uint32_t d = b * 256u + t;
    const uint32_t G = gridDim.x;
    s_cnt[t] = 0u;
    // this frame's forward work counters and the backward reorder's status words (tile_reorder_kernel)
    if (tile_cost && d < T) tile_cost[d] = 0u;
    if (reorder_words)
        for (uint32_t z = d; z < kFinBlocks * kFinWords; z += gridDim.x * 256u) reorder_words[z] = 0ull;
    // this tile's total over the chunks (exclusive chunk prefixes written back in place)
    uint32_t tot = 0;
    if (d < T) {
        const uint32_t C = ((b_fixed ? b_fixed : tile_blocks_for(*n_dev)) + kColChunk - 1) / kColChunk;
        for (uint32_t c0 = 0; c0 < C; c0 += 16u) {
            uint32_t x[16];
#pragma unroll
            for (uint32_t k = 0; k < 16u; k++) x[k] = c0 + k < C ? csum[(size_t)(c0 + k) * T + d] : 0u;
#pragma unroll
            for (uint32_t k = 0; k < 16u; k++) {
                if (c0 + k < C) csum[(size_t)(c0 + k) * T + d] = tot;
                tot += x[k];
            }
        }
    }
    const uint32_t nch = (tot + 63u) >> 6;
    // round 1: block-local exclusive scans of the totals and the chunk counts, then the sums of the
    // blocks before b (thread j reads block j's pair) and over all blocks
    uint64_t i0 = tot, i1 = nch;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint64_t y0 = __shfl_up(i0, o, 64), y1 = __shfl_up(i1, o, 64);
        if (lane >= (uint32_t)o) {
            i0 += y0;
            i1 += y1;
        }
    }
    if (lane == 63u) {
        s_ws[0][wv] = i0;
        s_ws[1][wv] = i1;
    }
    lds_barrier();
    uint64_t e0 = i0 - tot, e1 = i1 - nch, b0 = 0, b1 = 0;
#pragma unroll
    for (uint32_t k = 0; k < 4u; k++) {
        e0 += k < wv ? s_ws[0][k] : 0ull;
        e1 += k < wv ? s_ws[1][k] : 0ull;
        b0 += s_ws[0][k];
        b1 += s_ws[1][k];
    }
    unsigned long long* mine = fin + (size_t)b * kFinWords;
    if (t == 0) {
        st_agent64(mine, kFinFlag | b0);
        st_agent64(mine + 1, kFinFlag | b1);
    }
    uint64_t p0 = 0, p1 = 0, pall = 0;
    if (t < G) {
        unsigned long long v0 = ld_agent64(fin + (size_t)t * kFinWords);
        unsigned long long v1 = ld_agent64(fin + (size_t)t * kFinWords + 1u);
        uint32_t spins = 0;
        while (!(v0 & v1 & kFinFlag)) {  // every block is resident (at most kFinBlocks): it will publish
            if (++spins > (1u << 22)) {  // cannot happen (all blocks resident); reported, never a hang
                atomicOr(err, kFanInErrFinish);
                break;
            }
            __builtin_amdgcn_s_sleep(1);
            v0 = ld_agent64(fin + (size_t)t * kFinWords);
            v1 = ld_agent64(fin + (size_t)t * kFinWords + 1u);
        }
        pall = v0 & ~kFinFlag;
        p0 = t < b ? pall : 0ull;
        p1 = t < b ? v1 & ~kFinFlag : 0ull;
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {  // G <= kFinBlocks <= 64: all in wave 0
        p0 += __shfl_xor(p0, o, 64);
        p1 += __shfl_xor(p1, o, 64);
        pall += __shfl_xor(pall, o, 64);
    }
    if (t == 0) {
        s_pre[0] = p0;
        s_pre[1] = p1;
        s_pre[2] = pall;
    }
    lds_barrier();
    const uint32_t start = (uint32_t)(s_pre[0] + e0);
    // the launch bucket: longest first; in XCD groups, per run x of equal work (list length; a
    // per-tile constant added to the length measured within noise at 0, 16 and 64, round 3)
    uint32_t bucket, run = 0;
    if (xcd) {
        const uint64_t wtot = s_pre[2] > 0 ? s_pre[2] : 1u;
        const uint64_t wpre = start;
        const uint64_t xr = wpre * kXcdGroups / wtot;  // wpre < wtot unless every list is empty
        run = xr < kXcdGroups - 1u ? (uint32_t)xr : kXcdGroups - 1u;
        const uint32_t lv = min((uint32_t)(__log2f((float)tot + 1.0f) * kFwdLevels), 31u);
        bucket = run * 32u + (31u - lv);
    } else {
        bucket = 255u - min(tot >> 4, 255u);
    }
    const uint32_t lrank = d < T ? atomicAdd(&s_cnt[bucket], 1u) : 0u;
    lds_barrier();
    // round 2: the blocks' bucket counts
    st_agent64(mine + 2u + t, kFinFlag | s_cnt[t]);
    uint64_t gtot = 0, before = 0;  // bucket t: count over all blocks, over the blocks before b
    for (uint32_t j0 = 0; j0 < G; j0 += 16u) {
        unsigned long long v[16];
#pragma unroll
        for (uint32_t k = 0; k < 16u; k++)
            v[k] = j0 + k < G ? ld_agent64(fin + (size_t)(j0 + k) * kFinWords + 2u + t) : kFinFlag;
#pragma unroll
        for (uint32_t k = 0; k < 16u; k++) {
            uint32_t spins = 0;
            while (!(v[k] & kFinFlag)) {
                if (++spins > (1u << 22)) {
                    atomicOr(err, kFanInErrFinish);
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
                v[k] = ld_agent64(fin + (size_t)(j0 + k) * kFinWords + 2u + t);
            }
            const uint64_t c = v[k] & ~kFinFlag;
            gtot += c;
            before += j0 + k < b ? c : 0ull;
        }
    }
    // bucket bases: exclusive scan over the buckets of the global counts
    uint32_t gi = (uint32_t)gtot;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(gi, o, 64);
        if (lane >= (uint32_t)o) gi += y;
    }
    if (lane == 63u) s_bs[wv] = gi;
    lds_barrier();
    uint32_t bb = gi - (uint32_t)gtot;
#pragma unroll
    for (uint32_t k = 0; k < 4u; k++) bb += k < wv ? s_bs[k] : 0u;
    if ((t & 31u) == 0u) s_q[t >> 5] = bb;  // run x's first rank (bucket 32 x), XCD-group order
    if (t == 0) s_q[kXcdGroups] = T;
    s_cnt[t] = bb + (uint32_t)before;  // first launch-order slot of bucket t for this block
    lds_barrier();
    if (d < T) {
        ranges[d] = make_uint2(start, start + tot);
        chunk_base[d] = (uint32_t)(s_pre[1] + e1);
        const uint32_t slot = s_cnt[bucket] + lrank;
        const uint32_t ls = xcd ? xcd_slot(slot, run, s_q, T) : slot;
        if (order) order[ls] = d;
        if (xgroup) xgroup[d] = ls & (kXcdGroups - 1u);  // the XCD group the forward runs the tile in
    }
}

constexpr float kBwdLevels = 2.5f;  // log-work levels per doubling inside an XCD group (32 levels)
// The backward's launch order: tiles bucketed by the work the forward measured for them (blend
// steps summed over the tile's four waves, tile_cost) on a log scale, most work first. The
// backward's run time per tile follows that far better than the list length the forward's own
// order uses (the forward stops each band where its pixels saturate). One tile per thread, at most
// kFinBlocks resident blocks, full fan-in of the blocks' 256 bucket counts (as tile_finish_kernel).
__global__ __launch_bounds__(256) void tile_reorder_kernel(uint32_t T, const uint32_t* __restrict__ tile_cost,
                                                           unsigned long long* fin, uint32_t* __restrict__ order,
                                                           uint32_t* __restrict__ err, const uint32_t* __restrict__ xgroup) {
    __shared__ uint32_t s_cnt[256];
    __shared__ uint32_t s_w[4][256];
    __shared__ uint32_t s_bs[4];
    __shared__ uint32_t s_q[kXcdGroups + 1];
    const uint32_t t = threadIdx.x, lane = t & 63u, wv = t >> 6, b = blockIdx.x;
    const uint32_t d = b * 256u + t;
#pragma unroll
    for (int k = 0; k < 4; k++) s_w[k][t] = 0u;
    uint32_t bucket = 255u, run = 0;
    if (d < T && xgroup) {  // XCD groups of the forward, 32 levels (2.5 per doubling) inside each
        run = xgroup[d];
        const uint32_t lv = min((uint32_t)(__log2f((float)tile_cost[d] + 1.0f) * kBwdLevels), 31u);
        bucket = run * 32u + (31u - lv);
    } else if (d < T) {
        const float lc = __log2f((float)tile_cost[d] + 1.0f) * 16.0f;  // 16 buckets per doubling
        bucket = 255u - min((uint32_t)lc, 255u);
    }
    lds_barrier();
    // stable rank inside the bucket (tile order): peers by wave ballots over the bucket's bits, then
    // the waves' counts in wave order. A deterministic order keeps the backward's results
    // reproducible where the order decides how a tile is processed.
    uint64_t m = __ballot(d < T);
#pragma unroll
    for (int bit = 0; bit < 8; bit++) {
        const bool on = (bucket >> bit) & 1u;
        const uint64_t bb = __ballot(on);
        m &= on ? bb : ~bb;
    }
    const uint32_t below = (uint32_t)__popcll(m & (lane ? (~0ull >> (64u - lane)) : 0ull));
    if (d < T && lane == 63u - (uint32_t)__clzll(m)) s_w[wv][bucket] = (uint32_t)__popcll(m);
    lds_barrier();
    {
        uint32_t tot = 0;
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const uint32_t c = s_w[k][t];
            s_w[k][t] = tot;
            tot += c;
        }
        s_cnt[t] = tot;
    }
    lds_barrier();
    const uint32_t lrank = s_w[wv][bucket] + below;
    unsigned long long* mine = fin + (size_t)b * kFinWords;
    st_agent64(mine + 2u + t, kFinFlag | s_cnt[t]);
    const uint32_t G = gridDim.x;
    uint64_t gtot = 0, before = 0;
    for (uint32_t j0 = 0; j0 < G; j0 += 16u) {
        unsigned long long v[16];
#pragma unroll
        for (uint32_t k = 0; k < 16u; k++)
            v[k] = j0 + k < G ? ld_agent64(fin + (size_t)(j0 + k) * kFinWords + 2u + t) : kFinFlag;
#pragma unroll
        for (uint32_t k = 0; k < 16u; k++) {
            uint32_t spins = 0;
            while (!(v[k] & kFinFlag)) {  // every block is resident (at most kFinBlocks): it will publish
                if (++spins > (1u << 22)) {  // cannot happen (all blocks resident); reported, never a hang
                    atomicOr(err, kFanInErrReorder);
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
                v[k] = ld_agent64(fin + (size_t)(j0 + k) * kFinWords + 2u + t);
            }
            const uint64_t c = v[k] & ~kFinFlag;
            gtot += c;
            before += j0 + k < b ? c : 0ull;
        }
    }
    uint32_t gi = (uint32_t)gtot;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(gi, o, 64);
        if (lane >= (uint32_t)o) gi += y;
    }
    if (lane == 63u) s_bs[wv] = gi;
    lds_barrier();
    uint32_t bb = gi - (uint32_t)gtot;
#pragma unroll
    for (uint32_t k = 0; k < 4u; k++) bb += k < wv ? s_bs[k] : 0u;
    if ((t & 31u) == 0u) s_q[t >> 5] = bb;
    if (t == 0) s_q[kXcdGroups] = T;
    s_cnt[t] = bb + (uint32_t)before;
    lds_barrier();
    if (d < T) {
        const uint32_t slot = s_cnt[bucket] + lrank;
        order[xgroup ? xcd_slot(slot, run, s_q, T) : slot] = d;
    }
}

hipError_t tile_reorder(hipStream_t st, uint32_t T, const uint32_t* tile_cost, unsigned long long* words,
                        uint32_t* order, uint32_t* err, const uint32_t* xgroup) {
    if (T == 0 || T > kTileSortMaxTiles) return hipErrorInvalidValue;
    hipLaunchKernelGGL(tile_reorder_kernel, dim3((T + 255) / 256), dim3(256), 0, st, T, tile_cost, words, order, err,
                       xgroup);
    return hipGetLastError();
}

uint32_t tile_reorder_words() { return 2u * kFinBlocks * kFinWords; }

uint32_t tile_sort_blocks(uint64_t p_bound) { return tile_blocks_for(p_bound); }

static uint64_t tile_fin_offset(uint64_t B, uint32_t T) {  // u32 words; even (64-bit words follow)
    return ((uint64_t)T * (B + (B + kColChunk - 1) / kColChunk) + 1u) / 2u * 2u;
}

uint64_t tile_sort_scratch(uint64_t p_bound, uint32_t T) {
    // hist [B][T], chunk sums [C][T], then tile_finish_kernel's 64-bit words, then the slice totals of
    // tile_sort_gid's own-offsets mode
    return tile_fin_offset(tile_sort_blocks(p_bound), T) + 2ull * kFinBlocks * kFinWords + kTileSortMaxBlocks;
}

// the column scans and the tile-level scan (ranges, launch order) of the one-pass tile sort
static void tile_scan_launch(hipStream_t st, uint32_t T, uint32_t C, const uint32_t* p_dev, uint32_t* hist,
                             uint32_t* csum, unsigned long long* fin, uint2* ranges, uint32_t* order,
                             uint32_t* chunk_base, uint32_t* tile_cost, uint32_t* reorder_words, uint32_t* err,
                             bool xcd_groups, uint32_t* xgroup, uint32_t b_fixed = 0) {
    hipLaunchKernelGGL(tile_colscan_kernel, dim3((T + 255) / 256, std::min<uint32_t>(C, 16u)), dim3(256), 0, st, hist, T, p_dev,
                       csum, b_fixed);
    hipLaunchKernelGGL(tile_finish_kernel, dim3((T + 255) / 256), dim3(256), 0, st, csum, T, p_dev, fin, ranges,
                       order, chunk_base, tile_cost, reinterpret_cast<unsigned long long*>(reorder_words), err,
                       (uint32_t)(order != nullptr && xcd_groups), order != nullptr && xcd_groups ? xgroup : nullptr,
                       b_fixed);
}

uint32_t tile_sort_gid_blocks(uint32_t n) {
    // at least 4 chunks of 64 Gaussians per slice, at most one slice per CU
    const uint32_t nch = (n + 63u) / 64u;
    return std::max<uint32_t>(1u, std::min<uint32_t>(kTileSortMaxBlocks, (nch + 3u) / 4u));
}

hipError_t tile_sort_gid(hipStream_t st, uint32_t n, const uint32_t* count, uint32_t* goff, const uint2* rect,
                         uint32_t tiles_x, uint64_t cap, uint32_t* p_dev, uint64_t p_bound, uint32_t T,
                         uint32_t* scratch, uint32_t* vals_out, uint2* ranges, uint32_t* order, uint32_t* chunk_base,
                         uint32_t* tile_cost, uint32_t* reorder_words, uint32_t* err, bool xcd_groups,
                         uint32_t* xgroup, uint32_t* overflow, uint32_t* host_mirror, uint32_t* hist_rezero,
                         bool own_offsets, float4* rec, uint32_t* chunk_tot) {
    if (T == 0 || T > kTileSortMaxTiles || n == 0) return hipErrorInvalidValue;
    const uint32_t B = own_offsets ? tile_sort_gid_blocks(n) : tile_sort_blocks(p_bound);
    if (own_offsets && B > tile_sort_blocks(p_bound)) return hipErrorInvalidValue;  // scratch sized for p_bound
    const uint32_t C = (B + kColChunk - 1) / kColChunk;
    uint32_t* hist = scratch;
    uint32_t* csum = scratch + (size_t)T * B;
    const uint32_t grid = std::min<uint32_t>(B, kTileSortMaxBlocks);
    const uint32_t sgrid = (grid + 7u) & ~7u;
    // (the fan-in words and the slice totals sit where tile_sort_scratch(p_bound, T) puts them)
    const uint32_t Bs = tile_sort_blocks(p_bound);
    unsigned long long* fin = reinterpret_cast<unsigned long long*>(scratch + tile_fin_offset(Bs, T));
    uint32_t* slice_tot = scratch + tile_fin_offset(Bs, T) + 2ull * kFinBlocks * kFinWords;
    const uint32_t fin_words = 2u * kFinWords * ((T + 255u) / 256u);
    const uint32_t b_fixed = own_offsets ? B : 0u;
    const uint32_t nch = (n + 63u) / 64u;
    const uint32_t tiles_y = T / tiles_x;
    const size_t lds_rect = ((size_t)(tiles_y + 1u) * (tiles_x + 1u) + 1u) * sizeof(uint32_t);
    if (tiles_x * tiles_y != T || lds_rect > 160u * 1024u) return hipErrorInvalidValue;
    const uint32_t ncofs = own_offsets ? (nch + B - 1u) / B + 1u : 0u;
    const size_t lds_base = (T + 2u + kGidWaves + ncofs) * sizeof(uint32_t);
    if (lds_base > 160u * 1024u) return hipErrorInvalidValue;
    // the rest of the 160 KB stages up to scap pairs (6 B each) per slice
    const uint32_t scap = (uint32_t)((160u * 1024u - lds_base) / 6u) & ~1u;
    const size_t lds_scat = lds_base + (size_t)scap * 6u;
    if (own_offsets && !chunk_tot) return hipErrorInvalidValue;
    if (own_offsets)
        hipLaunchKernelGGL(tile_hist_rect_kernel<true>, dim3(grid), dim3(kGidThreads), lds_rect, st, n, count, rect,
                           tiles_x, p_dev, cap, T, hist, reinterpret_cast<uint32_t*>(fin), fin_words, overflow,
                           host_mirror, hist_rezero, b_fixed, slice_tot, chunk_tot);
    else
        hipLaunchKernelGGL(tile_hist_rect_kernel<false>, dim3(grid), dim3(kGidThreads), lds_rect, st, n, count, rect,
                           tiles_x, p_dev, cap, T, hist, reinterpret_cast<uint32_t*>(fin), fin_words, overflow,
                           host_mirror, hist_rezero, b_fixed, slice_tot, chunk_tot);
    tile_scan_launch(st, T, C, p_dev, hist, csum, fin, ranges, order, chunk_base, tile_cost, reorder_words, err,
                     xcd_groups, xgroup, b_fixed);
    if (own_offsets)
        hipLaunchKernelGGL(tile_scatter_gid_kernel<true>, dim3(sgrid), dim3(kGidThreads), lds_scat, st, n, count,
                           goff, rect, tiles_x, p_dev, cap, T, hist, csum, ranges, vals_out, b_fixed, slice_tot, chunk_tot, rec,
                           overflow, host_mirror, hist_rezero, ncofs, scap);
    else
        hipLaunchKernelGGL(tile_scatter_gid_kernel<false>, dim3(sgrid), dim3(kGidThreads), lds_scat, st, n, count,
                           goff, rect, tiles_x, p_dev, cap, T, hist, csum, ranges, vals_out, b_fixed, slice_tot, chunk_tot, rec,
                           overflow, host_mirror, hist_rezero, ncofs, scap);
    return hipGetLastError();
}

hipError_t tile_sort(hipStream_t st, const uint16_t* keys, const uint32_t* vals, const uint32_t* p_dev,
                     uint64_t p_bound, uint32_t T, uint32_t nbits, uint32_t* scratch,
                     uint32_t* vals_out, uint2* ranges, uint32_t* order, uint32_t* chunk_base,
                     uint32_t* tile_cost, uint32_t* reorder_words, uint32_t* err, bool xcd_groups,
                     uint32_t* xgroup) {
    if (T == 0 || T > kTileSortMaxTiles) return hipErrorInvalidValue;
    const uint32_t B = tile_sort_blocks(p_bound);
    const uint32_t C = (B + kColChunk - 1) / kColChunk;
    uint32_t* hist = scratch;
    uint32_t* csum = scratch + (size_t)T * B;
    const uint32_t grid = std::min<uint32_t>(B, kTileSortMaxBlocks);
    const uint32_t sgrid = (grid + 7u) & ~7u;  // the scatter's XCD-aware slice order wants a multiple of 8
    unsigned long long* fin = reinterpret_cast<unsigned long long*>(scratch + tile_fin_offset(B, T));
    const uint32_t fin_words = 2u * kFinWords * ((T + 255u) / 256u);
    hipLaunchKernelGGL(tile_hist_kernel, dim3(grid), dim3(kSortThreads), T * sizeof(uint32_t), st, keys,
                       p_dev, T, hist, reinterpret_cast<uint32_t*>(fin), fin_words);
    tile_scan_launch(st, T, C, p_dev, hist, csum, fin, ranges, order, chunk_base, tile_cost, reorder_words, err,
                     xcd_groups, xgroup);
    // 8 waves per block when their counters fit the 160 KB of LDS (T <= 8192), else 4
    const uint32_t lds8 = (T + 8u * ((T + 1u) >> 1)) * (uint32_t)sizeof(uint32_t);
    if (lds8 <= 160u * 1024u) {
        hipLaunchKernelGGL(tile_scatter_kernel<8>, dim3(sgrid), dim3(512), lds8, st, keys, vals, p_dev, T,
                           nbits, hist, csum, ranges, vals_out);
    } else {
        const uint32_t lds4 = (T + 4u * ((T + 1u) >> 1)) * (uint32_t)sizeof(uint32_t);
        hipLaunchKernelGGL(tile_scatter_kernel<4>, dim3(sgrid), dim3(256), lds4, st, keys, vals, p_dev, T,
                           nbits, hist, csum, ranges, vals_out);
    }
    return hipGetLastError();
}

// ---- device-wide exclusive scan of u32 (optionally gathered through a permutation) ------
constexpr int kScanThreads = 256;
constexpr int kScanItems = 8;
constexpr uint32_t kScanTile = kScanThreads * kScanItems;

__device__ __forceinline__ uint32_t scan_load(const uint32_t* __restrict__ in,
                                              const uint32_t* __restrict__ perm, uint32_t i) {
    return perm ? in[perm[i]] : in[i];
}

__global__ __launch_bounds__(kScanThreads) void scan_reduce_kernel(
    const uint32_t* __restrict__ in, const uint32_t* __restrict__ perm, uint32_t n,
    uint32_t* __restrict__ block_sums) {
    __shared__ uint32_t ws[kScanThreads / 64];
    const uint32_t base = blockIdx.x * kScanTile;
    uint32_t s = 0;
#pragma unroll
    for (int i = 0; i < kScanItems; i++) {
        const uint32_t idx = base + (uint32_t)i * kScanThreads + threadIdx.x;
        if (idx < n) s += scan_load(in, perm, idx);
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) s += __shfl_xor(s, o, 64);
    if ((threadIdx.x & 63u) == 0) ws[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) block_sums[blockIdx.x] = ws[0] + ws[1] + ws[2] + ws[3];
}

// Single block: exclusive scan of block sums; writes the grand total (u32, saturating flag).
__global__ __launch_bounds__(1024) void scan_block_sums_kernel(uint32_t* __restrict__ sums,
                                                                uint32_t nb,
                                                                uint32_t* __restrict__ total,
                                                                uint32_t* __restrict__ overflow) {
    __shared__ uint32_t part[1024];
    const uint32_t t = threadIdx.x;
    const uint32_t per = (nb + 1023u) / 1024u;
    const uint32_t b0 = t * per;
    uint64_t s = 0;
    for (uint32_t k = 0; k < per; k++)
        if (b0 + k < nb) s += sums[b0 + k];
    part[t] = (uint32_t)s;
    __syncthreads();
    for (uint32_t o = 1; o < 1024; o <<= 1) {
        const uint32_t v = t >= o ? part[t - o] : 0u;
        __syncthreads();
        part[t] += v;
        __syncthreads();
    }
    uint64_t run = t ? part[t - 1] : 0u;
    for (uint32_t k = 0; k < per; k++)
        if (b0 + k < nb) {
            const uint32_t c = sums[b0 + k];
            sums[b0 + k] = (uint32_t)run;
            run += c;
        }
    if (t == 1023) {
        *total = part[1023];
        if (overflow) *overflow = 0u;
    }
}

__global__ __launch_bounds__(kScanThreads) void scan_final_kernel(
    const uint32_t* __restrict__ in, const uint32_t* __restrict__ perm, uint32_t n,
    const uint32_t* __restrict__ block_offsets, uint32_t* __restrict__ out) {
    __shared__ uint32_t ws[kScanThreads / 64];
    // blocked arrangement: thread t owns items [t*8, t*8+8) of the tile
    const uint32_t base = blockIdx.x * kScanTile + threadIdx.x * kScanItems;
    uint32_t v[kScanItems];
    uint32_t s = 0;
#pragma unroll
    for (int i = 0; i < kScanItems; i++) {
        const uint32_t idx = base + (uint32_t)i;
        v[i] = idx < n ? scan_load(in, perm, idx) : 0u;
        s += v[i];
    }
    // wave inclusive scan of per-thread sums
    const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
    uint32_t inc = s;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(inc, o, 64);
        if (lane >= (uint32_t)o) inc += y;
    }
    if (lane == 63u) ws[w] = inc;
    __syncthreads();
    uint32_t wo = 0;
    for (uint32_t k = 0; k < w; k++) wo += ws[k];
    uint32_t run = block_offsets[blockIdx.x] + wo + inc - s;
#pragma unroll
    for (int i = 0; i < kScanItems; i++) {
        const uint32_t idx = base + (uint32_t)i;
        if (idx < n) out[idx] = run;
        run += v[i];
    }
}

// ---- single-sweep depth sort and emission-offset scan ----------------------------------------
// The depth sort over the N Gaussians as one scatter kernel per 8-bit digit, 4 passes (instead of hist +
// digit scan + scatter per digit): every digit's global histogram is built by project_kernel as it
// writes the keys (gs_raster.hip), and a scatter block learns its per-digit offset among the blocks
// before it by decoupled look-back — it takes a partition ticket, publishes its digit counts
// (flag "aggregate"), walks back over the predecessors' words until one carries an inclusive prefix,
// then publishes its own inclusive prefix. A status word holds its flag in the top two bits and the
// count in the low 30 (N < 2^30). The word is the payload (no separate flag), stored and polled
// with agent-scope atomics, which are coherent across the XCDs' L2s. A block only waits on blocks
// that took their tickets before it, and those are resident and publish their aggregate without
// waiting on anyone, so the walk always ends; the spin is still bounded (error word, no hang).
constexpr uint32_t kOsThreads = 1024;  // scatter block; threads 0..255 own one digit each
// Keys per thread and partition. A partition is one 1024-thread workgroup, and one fits a CU (its
// LDS and registers), so a pass over n keys runs ceil(parts / 256) rounds of partitions on the
// 256-CU device, and its time follows rounds x partition size. Above kOsSmallKeys the size is picked
// from 8, 10 and 12 keys per thread to minimise that product (config 5, 5.2M keys: 8 -> 635
// partitions in 3 rounds, 10 -> 508 in 2: depth sort 203 -> 172 us; 12: 180 us); below it every
// partition is resident at once and a pass costs one partition's latency, which shrinks with its
// size: 4 keys per thread (config 2, 100k keys: 55 -> 43 us; 5 keys 45, 3 keys 41 us). Host and
// device derive the choice from n alike.
constexpr uint32_t kOsItemsSmall = 4;
constexpr uint32_t kOsSmallKeys = 1u << 21;
constexpr uint32_t kOsRoundParts = 256;  // partitions resident at once (one per CU)
__host__ __device__ inline uint32_t os_items(uint32_t n) {
    if (n <= kOsSmallKeys) return kOsItemsSmall;
    uint32_t best = 8u, cost = 0xffffffffu;
    for (uint32_t it = 8u; it <= 12u; it += 2u) {
        const uint32_t parts = (n + kOsThreads * it - 1u) / (kOsThreads * it);
        const uint32_t c = (parts + kOsRoundParts - 1u) / kOsRoundParts * it;
        if (c < cost) {
            cost = c;
            best = it;
        }
    }
    return best;
}
constexpr uint32_t kOsWaves = kOsThreads / 64;
static_assert(kOsThreads >= 256 && kOsThreads <= 1024, "one thread per digit");
// offsets_scan_kernel: 512 threads of 8 or 12 consecutive ranks, held to 64 VGPRs so four blocks
// share a CU (1024 resident); the rank count per thread minimises rounds of resident partitions x
// partition size, as os_items does (config 5, 5.2M ranks: 8 -> 1270 partitions in 2 rounds, 12 ->
// 847 in one)
constexpr uint32_t kOffThreads = 512;
constexpr uint32_t kScanRoundParts = 1024;
__host__ __device__ inline uint32_t scan_items(uint32_t n) {
    uint32_t best = 8u, cost = 0xffffffffu;
    for (uint32_t it = 8u; it <= 12u; it += 4u) {
        const uint32_t parts = (n + kOffThreads * it - 1u) / (kOffThreads * it);
        const uint32_t c = (parts + kScanRoundParts - 1u) / kScanRoundParts * it;
        if (c < cost) {
            cost = c;
            best = it;
        }
    }
    return best;
}
constexpr uint32_t kOsFlagAgg = 1u << 30, kOsFlagPre = 2u << 30, kOsValMask = (1u << 30) - 1u;
constexpr uint32_t kOsSpinLimit = 1u << 22;
constexpr uint32_t kOsLook = 16;  // look-back window (predecessor words per round trip)

#ifdef GS_OS_TRACE  // diagnostics build only: per-block phase timestamps of the sweep kernels
__device__ unsigned long long g_os_trace[6][4096][4];
#define OS_TRACE(kern, part, phase) \
    do { if (threadIdx.x == 0 && (part) < 4096u) g_os_trace[kern][part][phase] = wall_clock64(); } while (0)
extern "C" __attribute__((visibility("default"))) int gs_debug_os_trace(void* host, size_t bytes) {
    return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_os_trace), bytes < sizeof(g_os_trace) ? bytes : sizeof(g_os_trace));
}
#else
#define OS_TRACE(kern, part, phase) do { } while (0)
#endif
__host__ __device__ inline uint32_t os_parts(uint32_t n) {
    const uint32_t tile = kOsThreads * os_items(n);
    return (n + tile - 1u) / tile;
}
// the most partitions any n <= n_cap takes (the scratch bound: the smallest partitions, 4 keys per
// thread up to kOsSmallKeys, then at least 8)
__host__ __device__ inline uint32_t os_parts_bound(uint32_t n_cap) {
    const uint32_t small = os_parts(n_cap < kOsSmallKeys ? n_cap : kOsSmallKeys);
    const uint32_t large = (n_cap + kOsThreads * 8u - 1u) / (kOsThreads * 8u);
    return small > large ? small : large;
}
__host__ __device__ inline uint32_t scan_parts(uint32_t n) {
    const uint32_t tile = kOffThreads * scan_items(n);
    return (n + tile - 1u) / tile;
}
// the most scan partitions any n <= n_cap takes (8 ranks per thread)
__host__ __device__ inline uint32_t scan_parts_bound(uint32_t n_cap) { return (n_cap + kOffThreads * 8u - 1u) / (kOffThreads * 8u); }
// digit p = bits [8p, 8p + nbits) of the key; the last digit has the remaining key bits
__host__ __device__ constexpr uint32_t os_digit_bits(uint32_t p) { return p + 1u < kOsPasses ? 8u : kDepthKeyBits - 8u * p; }
__host__ __device__ constexpr uint32_t os_digit_mask(uint32_t p) { return (1u << os_digit_bits(p)) - 1u; }

// scratch words: [0, 1024) digit histograms, [1024, 1040) tickets and error word (the head: zeroed by
// the emission kernel for the next frame), then the depth passes' status words [kOsPasses][parts][256]
// and the offset scan's 64-bit status words [scan parts] (zeroed by project_kernel)
constexpr uint32_t kOsHistWords = kOsPasses * 256u;
constexpr uint32_t kOsCtrWords = 16;
constexpr uint32_t kOsCtrCulled = 8;
constexpr uint32_t kOsHeadWords = kOsHistWords + kOsCtrWords;
__host__ __device__ inline uint64_t os_status_words(uint32_t n) { return (uint64_t)kOsPasses * os_parts(n) * 256u; }

static_assert(kOsHeadWords == kSweepHeadWords && kOsHistWords == kSweepHistWords &&
                  kOsCtrCulled == kSweepCtrCulled && kOsCtrWords - 1u == kSweepCtrError,
              "sweep head layout shared with gs_raster.hip");
uint32_t depth_sweep_zero_words(uint32_t n) {
    return (uint32_t)(os_status_words(n) + 2ull * scan_parts(n) + 4u);
}
uint32_t depth_sweep_error_word() { return kOsHistWords + kOsCtrWords - 1u; }

uint64_t depth_sweep_words(uint32_t n_cap) {
    return kOsHeadWords + (uint64_t)kOsPasses * os_parts_bound(n_cap) * 256u + 2ull * scan_parts_bound(n_cap) + 4u;
}

// Exclusive prefixes over partitions by full fan-in, for two scans over the same partitions: the
// block publishes its two totals as one flagged 64-bit word (bit 63 the flag, ta in bits 32..62,
// tb in 0..31: a partition's totals are below 2^31), then its threads read every earlier
// partition's word at once (spinning on words not yet published) and reduce. No chain of inclusive
// prefixes, so a block waits one round trip once its predecessors have published, however many
// there are. Sums below 2^32 (every count is at most 256 and n below 2^24). Every thread of the
// block calls it.
template <uint32_t NT>
__device__ void fanin_packed(unsigned long long* st, uint32_t part, uint32_t ta, uint32_t tb, uint32_t t,
                             uint32_t (*s_red)[NT / 64], uint32_t* err, uint32_t& ea, uint32_t& eb) {
    constexpr unsigned long long kFlag = 1ull << 63;
    if (t == 0) st_agent64(st + part, kFlag | (unsigned long long)ta << 32 | tb);
    uint32_t suma = 0, sumb = 0;
    for (uint32_t j = t; j < part; j += NT) {
        unsigned long long v = ld_agent64(st + j);
        uint32_t spins = 0;
        while (!(v & kFlag)) {  // not yet published (its block is resident: tickets)
            if (++spins > kOsSpinLimit) {
                atomicOr(err, 8u);
                break;
            }
            __builtin_amdgcn_s_sleep(1);
            v = ld_agent64(st + j);
        }
        suma += (uint32_t)(v >> 32) & 0x7fffffffu;
        sumb += (uint32_t)v;
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
        suma += __shfl_xor(suma, o, 64);
        sumb += __shfl_xor(sumb, o, 64);
    }
    if ((t & 63u) == 0u) {
        s_red[0][t >> 6] = suma;
        s_red[1][t >> 6] = sumb;
    }
    lds_barrier();
    ea = eb = 0;
#pragma unroll
    for (uint32_t k = 0; k < NT / 64; k++) {
        ea += s_red[0][k];
        eb += s_red[1][k];
    }
    lds_barrier();
}

// One stable digit pass (digit = bits [8 pass, 8 pass + nbits) of the key) over one partition of
// kOsTile keys; ranks inside the partition as radix_scatter_kernel (wave ballots in memory order),
// partition offsets per digit by look-back.
template <bool kFirst, uint32_t kOsItems>
__global__ __launch_bounds__(kOsThreads) void onesweep_kernel(
    const uint32_t* __restrict__ keys_in, const uint32_t* __restrict__ vals_in, uint32_t n,
    uint32_t pass, uint32_t* sweep, uint32_t* __restrict__ keys_out, uint32_t* __restrict__ vals_out,
    const uint32_t* __restrict__ count) {
    constexpr uint32_t kOsTile = kOsThreads * kOsItems;  // (the host launches os_items(n))
    __shared__ uint32_t s_ticket;
    __shared__ uint32_t s_ws[4];
    __shared__ uint32_t s_off[256];
    __shared__ uint32_t s_loc[256];
    __shared__ uint32_t s_cnt[kOsWaves][256];
    __shared__ uint32_t s_key[kOsTile];
    __shared__ uint32_t s_val[kOsTile];
    const uint32_t t = threadIdx.x, w = t >> 6, lane = t & 63u;
    const uint32_t shift = 8u * pass, nbits = os_digit_bits(pass);
    const uint32_t mask = os_digit_mask(pass);
    uint32_t* ctr = sweep + kOsHistWords;
    if (t == 0) s_ticket = __hip_atomic_fetch_add((gu32*)(ctr + pass), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    lds_barrier();
    const uint32_t part = s_ticket;
    OS_TRACE(1 + pass, part, 0);
    const uint32_t begin = part * kOsTile;
    const uint32_t end = min(begin + kOsTile, n);
    const uint64_t lt = lanemask_lt();

    uint32_t k[kOsItems], v[kOsItems], dg[kOsItems], rk[kOsItems];
    bool ok[kOsItems];
    // all loads of the partition in flight at once (clamped indices, no per-item branches)
#pragma unroll
    for (int i = 0; i < (int)kOsItems; i++) {
        const uint32_t idx = begin + w * (kOsItems * 64u) + (uint32_t)i * 64u + lane;
        ok[i] = idx < end;
        const uint32_t ci = ok[i] ? idx : end - 1u;
        k[i] = keys_in[ci];
        // pass 0 builds the payload: gid | (tile count - 1) << 24 (count in 1..256; the culled
        // ranks, count 0, are the last n - visible and never read it), so the offset scan needs no
        // gather of count[gid]
        v[i] = kFirst ? count[ci] : vals_in[ci];
    }
#pragma unroll
    for (int i = 0; i < (int)kOsItems; i++) {
        if (kFirst) {
            const uint32_t idx = begin + w * (kOsItems * 64u) + (uint32_t)i * 64u + lane;
            v[i] = idx | (v[i] ? (v[i] - 1u) << kDsortCountShift : 0u);
        }
        dg[i] = (k[i] >> shift) & mask;
    }
    // global digit starts: exclusive scan of this pass's histogram (loads above in flight)
    const uint32_t gbase = scan256_excl(t < 256u ? sweep[pass * 256u + t] : 0u, t, s_ws);
#pragma unroll
    for (int j = 0; j < 4; j++) s_cnt[w][lane + 64u * j] = 0u;
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int i = 0; i < (int)kOsItems; i++) {
        uint64_t m = __ballot(ok[i]);
        for (uint32_t bit = 0; bit < nbits; bit++) {
            const bool on = (dg[i] >> bit) & 1u;
            const uint64_t bb = __ballot(on);
            m &= on ? bb : ~bb;
        }
        const uint32_t below = (uint32_t)__popcll(m & lt);
        uint32_t c = 0;
        if (ok[i]) c = s_cnt[w][dg[i]];
        __builtin_amdgcn_wave_barrier();
        rk[i] = c + below;
        const uint32_t leader = 63u - (uint32_t)__clzll(m);
        if (ok[i] && lane == leader) s_cnt[w][dg[i]] = c + (uint32_t)__popcll(m);
        __builtin_amdgcn_wave_barrier();
    }
    lds_barrier();
    OS_TRACE(1 + pass, part, 1);
    uint32_t tot = 0;
    if (t < 256u) {
#pragma unroll
        for (int ww = 0; ww < (int)kOsWaves; ww++) {
            const uint32_t c = s_cnt[ww][t];
            s_cnt[ww][t] = tot;
            tot += c;
        }
        // publish this partition's digit count, look back for the counts of the partitions before it
        uint32_t* status = sweep + kOsHeadWords + (size_t)pass * os_parts(n) * 256u;
        uint32_t excl = 0;
        if (part == 0) {
            st_agent(status + t, kOsFlagPre | tot);
        } else {
            st_agent(status + (size_t)part * 256u + t, kOsFlagAgg | tot);
            // windowed walk: the next kOsLook predecessors' words in one round trip, summed from the
            // nearest back to the first inclusive prefix (below partition 0: a virtual zero prefix)
            int32_t j = (int32_t)part - 1;  // nearest predecessor not yet accounted for
            uint32_t spins = 0;
            for (;;) {
                uint32_t sv[kOsLook];
#pragma unroll
                for (int q = 0; q < (int)kOsLook; q++)
                    sv[q] = j - q >= 0 ? ld_agent(status + (size_t)(j - q) * 256u + t) : kOsFlagPre;
                bool done = false, stall = false;
                uint32_t acc = 0;
                int32_t used = 0;
#pragma unroll
                for (int q = 0; q < (int)kOsLook; q++) {
                    const bool live = !done && !stall;
                    const uint32_t f = sv[q] & (kOsFlagAgg | kOsFlagPre);
                    stall = stall || (live && !f);
                    if (live && f) {
                        acc += sv[q] & kOsValMask;
                        used = q + 1;
                        done = (f & kOsFlagPre) != 0u;
                    }
                }
                excl += acc;
                j -= used;
                if (done) break;
                if (stall) {
                    if (++spins > kOsSpinLimit) {  // cannot happen (see above); never hang the GPU
                        atomicOr(ctr + kOsCtrWords - 1u, 1u);
                        break;
                    }
                    __builtin_amdgcn_s_sleep(1);
                }
            }
            st_agent(status + (size_t)part * 256u + t, kOsFlagPre | (excl + tot));
        }
        s_off[t] = gbase + excl;
    }
    // block-local exclusive scan of the digit counts -> s_loc
    const uint32_t loc = scan256_excl(tot, t, s_ws);
    OS_TRACE(1 + pass, part, 2);
    if (t < 256u) s_loc[t] = loc;
    lds_barrier();
#pragma unroll
    for (int i = 0; i < (int)kOsItems; i++) {
        if (!ok[i]) continue;
        const uint32_t lp = s_loc[dg[i]] + s_cnt[w][dg[i]] + rk[i];
        s_key[lp] = k[i];
        s_val[lp] = v[i];
    }
    lds_barrier();
    const uint32_t cnt = end > begin ? end - begin : 0u;
    for (uint32_t i = t; i < cnt; i += kOsThreads) {
        const uint32_t kk = s_key[i], vv = s_val[i];
        const uint32_t d = (kk >> shift) & mask;
        const uint32_t pos = s_off[d] + (i - s_loc[d]);
        if (keys_out) keys_out[pos] = kk;
        vals_out[pos] = vv;
    }
    OS_TRACE(1 + pass, part, 3);
}

// Emission offsets in one pass: offset[i] = sum of count[dsorted[0..i)], P = the total, and the
// emission windows' owners (window_starts_kernel's job: rank i owns the windows whose first slot
// lies in [offset[i], min(offset[i] + count, cap))); with them goff, the same scan over the counts in
// Gaussian order. kDepth: the global depth order (dsorted given); otherwise the emission is in
// Gaussian order and only goff (and the records' slot field) is written. Partitions learn their
// prefixes by one full fan-in over packed 64-bit status words (fanin_packed). Held to 64 VGPRs (8
// waves per SIMD): at 113 (4 waves, 512 partitions resident of config 5's 1270) it took 78 us, the
// partitions starting over 69 us; now 42 us.
template <uint32_t kSI, bool kDepth>
__global__ __launch_bounds__(kOffThreads, 8) void offsets_scan_kernel(
    uint32_t n, const uint32_t* __restrict__ count, const uint32_t* __restrict__ dsorted,
    uint32_t* sweep, uint32_t* __restrict__ offset, uint32_t* __restrict__ p_dev,
    uint32_t* __restrict__ wstart, uint64_t cap, uint32_t* __restrict__ goff, float4* __restrict__ rec) {
    __shared__ uint32_t s_ticket;
    __shared__ uint32_t s_ws[2][kOffThreads / 64], s_red[2][kOffThreads / 64];
    __shared__ uint32_t s_excl[2];
    const uint32_t t = threadIdx.x, w = t >> 6, lane = t & 63u;
    uint32_t* ctr = sweep + kOsHistWords;
    if (t == 0) s_ticket = __hip_atomic_fetch_add((gu32*)(ctr + kOsPasses), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    lds_barrier();
    const uint32_t part = s_ticket;
    OS_TRACE(5, part, 0);
    constexpr uint32_t kScanPart = kOffThreads * kSI;
    const uint32_t base = part * kScanPart + t * kSI;  // blocked: thread t owns kSI consecutive ranks
    // c: the tile counts in depth order (from the sort payload: ranks below `visible` were emitted),
    // or, with no depth sort (per-tile depth sort after the tile sort, gs_segsort.hip: emission in
    // Gaussian order), the counts themselves; cg: the counts in Gaussian order. Read twice: for the
    // thread's sums here, and again (from L2) after the partition's prefix is known, so no array is
    // live across the fan-in and the kernel stays at 8 waves per SIMD. 16-B loads and stores, by the
    // threads with ranks below n, also past n (the four buffers have 16 words of padding; the ranks
    // past n are masked).
    const uint32_t visible = kDepth ? n - sweep[kOsHistWords + kOsCtrCulled] : n;
    const bool live = base < n;
    uint32_t c[kSI], cg[kSI];
    auto load = [&](uint32_t b0) {  // (b0 == base, or 0 for the threads past n: no branch around the loads)
#pragma unroll
        for (int q = 0; q < (int)kSI; q += 4) {
            const uint4 x = *reinterpret_cast<const uint4*>(count + b0 + q);
            cg[q] = x.x; cg[q + 1] = x.y; cg[q + 2] = x.z; cg[q + 3] = x.w;
            if (kDepth) {
                const uint4 a = *reinterpret_cast<const uint4*>(dsorted + b0 + q);
                c[q] = a.x; c[q + 1] = a.y; c[q + 2] = a.z; c[q + 3] = a.w;
            }
        }
#pragma unroll
        for (int i = 0; i < (int)kSI; i++) {
            const uint32_t idx = base + (uint32_t)i;
            cg[i] = idx < n ? cg[i] : 0u;  // (all ranks of a thread past n)
            c[i] = kDepth ? (idx < visible ? (c[i] >> kDsortCountShift) + 1u : 0u) : cg[i];
        }
    };
    load(live ? base : 0u);
    uint32_t s = 0, sg = 0;
#pragma unroll
    for (int i = 0; i < (int)kSI; i++) {
        s += c[i];
        sg += cg[i];
    }
    uint32_t inc = s, incg = sg;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(inc, o, 64), yg = __shfl_up(incg, o, 64);
        if (lane >= (uint32_t)o) {
            inc += y;
            incg += yg;
        }
    }
    if (lane == 63u) {
        s_ws[0][w] = inc;
        s_ws[1][w] = incg;
    }
    lds_barrier();
    uint32_t wo = 0, btot = 0, wog = 0, btotg = 0;  // (a partition's totals are below 2^32)
#pragma unroll
    for (uint32_t k = 0; k < kOffThreads / 64; k++) {
        wo += k < w ? s_ws[0][k] : 0u;
        btot += s_ws[0][k];
        wog += k < w ? s_ws[1][k] : 0u;
        btotg += s_ws[1][k];
    }
    unsigned long long* status = reinterpret_cast<unsigned long long*>(sweep + kOsHeadWords + os_status_words(n));
    {
        OS_TRACE(5, part, 1);
        uint32_t excl, exclg;
        fanin_packed<kOffThreads>(status, part, btot, btotg, t, s_red, ctr + kOsCtrWords - 1u, excl, exclg);
        OS_TRACE(5, part, 2);
        if (t == 0) {
            s_excl[0] = excl;
            s_excl[1] = exclg;
            if ((uint64_t)(part + 1u) * kScanPart >= n) *p_dev = excl + btot;  // the last partition
        }
    }
    lds_barrier();
    const uint32_t run0 = s_excl[0] + wo + (inc - s);  // this thread's first emission offset
    uint32_t run = run0, rung = s_excl[1] + wog + (incg - sg);
    uint32_t base2 = live ? base : 0u;
    asm volatile("" : "+v"(base2));  // opaque to the compiler: a real second read, not the first one's registers kept live
    load(base2);
#pragma unroll
    for (int i = 0; i < (int)kSI; i++) {  // c, cg -> their running prefixes
        const uint32_t nx = run + c[i];
        c[i] = run;
        run = nx;
        const uint32_t ng = rung + cg[i];
        cg[i] = rung;
        rung = ng;
    }
    // offset: the emission offsets (Gaussian-order emission reads goff instead). goff: the partial-sum
    // slots of the backward in Gaussian order, goff[gid] = the tile counts of the Gaussians before gid,
    // so each Gaussian's slots follow the previous Gaussian's and the chain kernel's reads of them are
    // contiguous.
    // (16-B stores, past n into the buffers' padding in the last partition)
#pragma unroll
    for (int q = 0; q < (int)kSI && live; q += 4) {
        if (kDepth) *reinterpret_cast<uint4*>(offset + base + q) = make_uint4(c[q], c[q + 1], c[q + 2], c[q + 3]);
        *reinterpret_cast<uint4*>(goff + base + q) = make_uint4(cg[q], cg[q + 1], cg[q + 2], cg[q + 3]);
    }
    // the emission windows whose first slot lies in this thread's slots [run0, run0 + s) below cap:
    // each one's owner is the last of the thread's ranks starting at or before that slot (a rank
    // with no slots starts where the next one does, so it is never the last); ~0.1 windows per
    // thread at config 5
    if (kDepth && run0 < cap) {
        const uint64_t end = (uint64_t)run0 + s < cap ? (uint64_t)run0 + s : cap;
        for (uint64_t wd = ((uint64_t)run0 + kEmitWin - 1) / kEmitWin; wd * kEmitWin < end; wd++) {
            const uint32_t x = (uint32_t)(wd * kEmitWin - run0);
            uint32_t k = 0;
#pragma unroll
            for (int i = 0; i < (int)kSI; i++) k += c[i] - run0 <= x ? 1u : 0u;
            wstart[wd] = base + k - 1u;
        }
    }
    // ... and (rec given: the per-tile order) into the raster record's quad 3 (.x), next to the splat data the backward gathers
    // anyway: its slot base then costs no gather of its own (a random 4-B read of goff per walked
    // list entry, ~240 MB of line fetches per frame at the bench workload)
    if (!kDepth && rec)
#pragma unroll
        for (int i = 0; i < (int)kSI; i++)
            if (base + (uint32_t)i < n && (i + 1 < (int)kSI ? cg[i + 1] != cg[i] : rung != cg[i]))
                reinterpret_cast<uint32_t*>(rec + (size_t)(base + (uint32_t)i) * kRecQuads + 3)[0] = cg[i];
    OS_TRACE(5, part, 3);
}

hipError_t depth_sort_onesweep(hipStream_t st, const uint32_t* dkey, const uint32_t* count, uint32_t n,
                               uint32_t* sweep, uint32_t* const kbuf[2], uint32_t* const vbuf[2],
                               uint32_t* dsorted) {
    if (n == 0) return hipSuccess;
    const uint32_t parts = os_parts(n);
    // (the digit histograms come from project_kernel; it also zeroed this frame's status words)
    const uint32_t* kin = dkey;
    const uint32_t* vin = nullptr;
    // ping-pong so that the next-to-last pass writes the buffer that is not `dsorted` (the caller
    // passes vbuf[1] as dsorted; the last pass must not scatter in place whatever the pass count)
    static_assert(kOsPasses >= 2, "ping-pong");
    const uint32_t flip = (dsorted == vbuf[0] ? 1u : 0u) ^ ((kOsPasses - 2u) & 1u);
    for (uint32_t p = 0; p < kOsPasses; p++) {
        const bool last = p + 1 == kOsPasses;
        const uint32_t o = (p & 1u) ^ flip;
        const uint32_t it = os_items(n);
        auto kern = it == 4u    ? (p == 0 ? onesweep_kernel<true, 4u> : onesweep_kernel<false, 4u>)
                    : it == 8u  ? (p == 0 ? onesweep_kernel<true, 8u> : onesweep_kernel<false, 8u>)
                    : it == 10u ? (p == 0 ? onesweep_kernel<true, 10u> : onesweep_kernel<false, 10u>)
                                : (p == 0 ? onesweep_kernel<true, 12u> : onesweep_kernel<false, 12u>);
        hipLaunchKernelGGL(kern, dim3(parts), dim3(kOsThreads), 0, st, kin, vin, n, p, sweep,
                           last ? nullptr : kbuf[o], last ? dsorted : vbuf[o], count);
        kin = kbuf[o];
        vin = vbuf[o];
    }
    return hipGetLastError();
}

hipError_t offsets_scan(hipStream_t st, uint32_t n, const uint32_t* count, const uint32_t* dsorted,
                        uint32_t* sweep, uint32_t* offset, uint32_t* p_dev, uint32_t* wstart, uint64_t cap,
                        uint32_t* goff, float4* rec) {
    if (n == 0) return hipMemsetAsync(p_dev, 0, sizeof(uint32_t), st);
    const uint32_t it = scan_items(n);
    auto kern = dsorted ? (it == 8u ? offsets_scan_kernel<8u, true> : offsets_scan_kernel<12u, true>)
                        : (it == 8u ? offsets_scan_kernel<8u, false> : offsets_scan_kernel<12u, false>);
    hipLaunchKernelGGL(kern, dim3(scan_parts(n)), dim3(kOffThreads), 0, st, n, count, dsorted, sweep, offset, p_dev,
                       wstart, cap, goff, rec);
    return hipGetLastError();
}

// ---- host launchers -----------------------------------------------------------------

uint32_t sort_blocks_for(uint64_t n_bound) {
    uint64_t b = (n_bound + kSortTile - 1) / kSortTile;
    if (b < 1) b = 1;
    // at most the scatter's resident workgroups (2 per CU at 128 VGPRs, 256 CUs): one round of long
    // slices instead of four rounds of 2048 (config 5, both passes: 607 -> 544 us)
    if (b > kRsMaxBlocks) b = kRsMaxBlocks;
    return (uint32_t)b;
}

template <typename KI, typename KO>
static void radix_pass_t(hipStream_t st, const RadixPass& p) {
    const uint32_t B = p.nblocks;
    const KI* kin = static_cast<const KI*>(p.keys_in);
    if (!p.hist_ready)
        hipLaunchKernelGGL(radix_hist_kernel<KI>, dim3(B), dim3(kRhThreads), 0, st, kin, p.n_dev, p.n_host,
                           p.shift, (1u << p.nbits) - 1u, p.hist, p.ranges_out, p.ranges_n);
    hipLaunchKernelGGL(radix_digit_scan_kernel, dim3(256), dim3(256), 0, st, p.hist, B, p.totals);
    hipLaunchKernelGGL((radix_scatter_kernel<KI, KO, kRsThreads>), dim3(B), dim3(kRsThreads), 0, st, kin,
                       p.vals_in, p.n_dev,
                       p.n_host, p.shift, p.nbits, p.hist, p.totals, static_cast<KO*>(p.keys_out), p.vals_out,
                       p.inverse_out, p.ranges_out, p.clear_hist ? p.hist : nullptr);
}

hipError_t radix_pass(hipStream_t st, const RadixPass& p) {
    if ((p.key_bytes_in != 2 && p.key_bytes_in != 4) || (p.key_bytes_out != 2 && p.key_bytes_out != 4))
        return hipErrorInvalidValue;
    if (p.key_bytes_in == 4)
        p.key_bytes_out == 4 ? radix_pass_t<uint32_t, uint32_t>(st, p) : radix_pass_t<uint32_t, uint16_t>(st, p);
    else
        p.key_bytes_out == 4 ? radix_pass_t<uint16_t, uint32_t>(st, p) : radix_pass_t<uint16_t, uint16_t>(st, p);
    return hipGetLastError();
}

uint32_t scan_blocks_for(uint32_t n) { return (n + kScanTile - 1) / kScanTile; }

hipError_t exclusive_scan(hipStream_t st, const uint32_t* in, const uint32_t* perm, uint32_t n,
                          uint32_t* out, uint32_t* block_sums, uint32_t* total,
                          uint32_t* overflow) {
    const uint32_t nb = scan_blocks_for(n);
    if (nb == 0) {
        return hipMemsetAsync(total, 0, sizeof(uint32_t), st);
    }
    hipLaunchKernelGGL(scan_reduce_kernel, dim3(nb), dim3(kScanThreads), 0, st, in, perm, n,
                       block_sums);
    hipLaunchKernelGGL(scan_block_sums_kernel, dim3(1), dim3(1024), 0, st, block_sums, nb, total,
                       overflow);
    hipLaunchKernelGGL(scan_final_kernel, dim3(nb), dim3(kScanThreads), 0, st, in, perm, n,
                       block_sums, out);
    return hipGetLastError();
}

}  // namespace gs
