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

#include "gs_device.hpp"
#include "gs_internal.hpp"

namespace gs {

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

__global__ __launch_bounds__(kSortThreads) void radix_hist_kernel(
    const uint32_t* __restrict__ keys, const uint32_t* n_dev, uint32_t n_host, uint32_t shift,
    uint32_t mask, uint32_t* __restrict__ hist /* [256][nblocks] */) {
    __shared__ uint32_t h[kSortWaves][256];
    const uint32_t t = threadIdx.x, w = t >> 6;
    for (uint32_t i = t; i < kSortWaves * 256; i += kSortThreads) (&h[0][0])[i] = 0u;
    __syncthreads();
    const uint32_t n = sort_count(n_dev, n_host);
    uint32_t begin, end;
    sort_slice(n, blockIdx.x, gridDim.x, begin, end);
    for (uint32_t i = begin + t; i < end; i += kSortThreads) {
        const uint32_t d = (keys[i] >> shift) & mask;
        atomicAdd(&h[w][d], 1u);
    }
    __syncthreads();
    const uint32_t s = h[0][t] + h[1][t] + h[2][t] + h[3][t];
    hist[t * gridDim.x + blockIdx.x] = s;
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
__global__ __launch_bounds__(kSortThreads) void radix_scatter_kernel(
    const uint32_t* __restrict__ keys_in, const uint32_t* __restrict__ vals_in,
    const uint32_t* n_dev, uint32_t n_host, uint32_t shift, uint32_t nbits,
    const uint32_t* __restrict__ hist, const uint32_t* __restrict__ totals,
    uint32_t* __restrict__ keys_out, uint32_t* __restrict__ vals_out,
    uint32_t* __restrict__ inverse_out) {
    __shared__ uint32_t s_off[256];               // running global start of each digit
    __shared__ uint32_t s_cnt[kSortWaves][256];   // per-wave counts -> per-wave local offsets
    __shared__ uint32_t s_loc[256];               // block-local start of each digit in the step
    __shared__ uint32_t s_key[kSortTile];
    __shared__ uint32_t s_val[kSortTile];
    const uint32_t t = threadIdx.x, w = t >> 6, lane = t & 63u;
    const uint32_t mask = (1u << nbits) - 1u;

    // digit bases: exclusive scan of totals
    s_loc[t] = totals[t];
    __syncthreads();
    for (uint32_t o = 1; o < 256; o <<= 1) {
        const uint32_t v = t >= o ? s_loc[t - o] : 0u;
        __syncthreads();
        s_loc[t] += v;
        __syncthreads();
    }
    const uint32_t base = t ? s_loc[t - 1] : 0u;
    s_off[t] = base + hist[t * gridDim.x + blockIdx.x];
    __syncthreads();

    const uint32_t n = sort_count(n_dev, n_host);
    uint32_t begin, end;
    sort_slice(n, blockIdx.x, gridDim.x, begin, end);
    const uint64_t lt = lanemask_lt();

    for (uint32_t step = begin; step < end; step += kSortTile) {
        uint32_t k[kSortItems], v[kSortItems], dg[kSortItems], rk[kSortItems];
        bool ok[kSortItems];
#pragma unroll
        for (int i = 0; i < kSortItems; i++) {
            const uint32_t idx = step + w * (kSortItems * 64u) + (uint32_t)i * 64u + lane;
            ok[i] = idx < end;
            k[i] = ok[i] ? keys_in[idx] : 0u;
            v[i] = vals_in ? (ok[i] ? vals_in[idx] : 0u) : idx;
            dg[i] = (k[i] >> shift) & mask;
        }
#pragma unroll
        for (int j = 0; j < 4; j++) s_cnt[w][lane + 64u * j] = 0u;
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int i = 0; i < kSortItems; i++) {
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
        __syncthreads();
        // per digit (thread t = digit): wave offsets within the digit, digit total of the step
        uint32_t tot = 0;
#pragma unroll
        for (int ww = 0; ww < kSortWaves; ww++) {
            const uint32_t c = s_cnt[ww][t];
            s_cnt[ww][t] = tot;
            tot += c;
        }
        // block-local exclusive scan of the digit totals -> s_loc
        s_loc[t] = tot;
        __syncthreads();
        for (uint32_t o = 1; o < 256; o <<= 1) {
            const uint32_t x = t >= o ? s_loc[t - o] : 0u;
            __syncthreads();
            s_loc[t] += x;
            __syncthreads();
        }
        const uint32_t loc_start = s_loc[t] - tot;
        __syncthreads();
        s_loc[t] = loc_start;
        __syncthreads();
        // reorder the step by digit in LDS
#pragma unroll
        for (int i = 0; i < kSortItems; i++) {
            if (!ok[i]) continue;
            const uint32_t lp = s_loc[dg[i]] + s_cnt[w][dg[i]] + rk[i];
            s_key[lp] = k[i];
            s_val[lp] = v[i];
        }
        __syncthreads();
        const uint32_t cnt = min(kSortTile, end - step);
        for (uint32_t i = t; i < cnt; i += kSortThreads) {
            const uint32_t kk = s_key[i], vv = s_val[i];
            const uint32_t d = (kk >> shift) & mask;
            const uint32_t pos = s_off[d] + (i - s_loc[d]);
            if (keys_out) keys_out[pos] = kk;
            if (vals_out) vals_out[pos] = vv;
            if (inverse_out) inverse_out[vv] = pos;
        }
        __syncthreads();
        s_off[t] += tot;
        __syncthreads();
    }
}


// ---- one-pass stable counting sort of the pairs by tile key (T <= kTileSortMaxTiles) ----------
// The tile key has only ceil(log2 T) significant bits (13 at 1080p), so instead of two 8-bit LSD
// passes the pairs are counted once per (block, tile) and scattered once:
//   tile_hist      per-block tile counts -> hist[b][t] (block-major rows, coalesced);
//   tile_colscan   per tile, exclusive prefixes over blocks inside chunks of 16 blocks (in place)
//                  and the chunk totals csum[c][t];
//   tile_totals    per tile, exclusive prefixes over the chunks (in place) and the tile total;
//   tile_starts    one workgroup: exclusive scan of the tile totals -> the tile ranges (no
//                  separate ranges pass);
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

__global__ __launch_bounds__(kSortThreads) void tile_hist_kernel(const uint32_t* __restrict__ keys,
                                                                 const uint32_t* n_dev, uint32_t T,
                                                                 uint32_t* __restrict__ hist) {
    extern __shared__ uint32_t h_tile[];
    const uint32_t n = *n_dev, B = tile_blocks_for(n);
    const uint32_t t = threadIdx.x;
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
                d[k] = i < end ? keys[i] : 0xffffffffu;
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
                                                           uint32_t* __restrict__ csum) {
    const uint32_t d = blockIdx.x * 256u + threadIdx.x;
    const uint32_t B = tile_blocks_for(*n_dev);
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

// per tile: exclusive prefixes of the chunk totals (in place) and the tile total -> ranges[d].y
__global__ __launch_bounds__(256) void tile_totals_kernel(uint32_t* __restrict__ csum, uint32_t T,
                                                          const uint32_t* n_dev,
                                                          uint2* __restrict__ ranges) {
    const uint32_t d = blockIdx.x * 256u + threadIdx.x;
    if (d >= T) return;
    const uint32_t C = (tile_blocks_for(*n_dev) + kColChunk - 1) / kColChunk;
    uint32_t run = 0;
    for (uint32_t c0 = 0; c0 < C; c0 += 16u) {
        uint32_t x[16];
#pragma unroll
        for (uint32_t k = 0; k < 16u; k++) x[k] = c0 + k < C ? csum[(size_t)(c0 + k) * T + d] : 0u;
#pragma unroll
        for (uint32_t k = 0; k < 16u; k++) {
            if (c0 + k < C) csum[(size_t)(c0 + k) * T + d] = run;
            run += x[k];
        }
    }
    ranges[d] = make_uint2(0u, run);
}

// one workgroup: exclusive scan of the tile totals -> ranges; with `order`, also the blend launch
// order (tile_order_kernel's bucketing, gs_raster.hip) from the totals already in registers
__global__ __launch_bounds__(1024) void tile_starts_kernel(uint32_t T, uint2* __restrict__ ranges,
                                                           uint32_t* __restrict__ order,
                                                           uint32_t* __restrict__ chunk_base) {
    __shared__ uint32_t wsum[16], wsum2[16];
    __shared__ uint32_t cnt[256];
    const uint32_t t = threadIdx.x, lane = t & 63u, w = t >> 6;
    constexpr uint32_t kPer = (kTileSortMaxTiles + 1023u) / 1024u;
    const uint32_t d0 = t * kPer;
    if (t < 256u) cnt[t] = 0u;
    uint32_t tot[kPer];
    uint32_t s = 0;
#pragma unroll
    for (uint32_t k = 0; k < kPer; k++) {
        tot[k] = d0 + k < T ? ranges[d0 + k].y : 0u;
        s += tot[k];
    }
    uint32_t s2 = 0;  // list chunks of 64 entries
#pragma unroll
    for (uint32_t k = 0; k < kPer; k++) s2 += (tot[k] + 63u) >> 6;
    uint32_t inc = s, inc2 = s2;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(inc, o, 64), y2 = __shfl_up(inc2, o, 64);
        if (lane >= (uint32_t)o) {
            inc += y;
            inc2 += y2;
        }
    }
    if (lane == 63u) {
        wsum[w] = inc;
        wsum2[w] = inc2;
    }
    __syncthreads();
    uint32_t start = inc - s, cstart = inc2 - s2;
    for (uint32_t k = 0; k < w; k++) {
        start += wsum[k];
        cstart += wsum2[k];
    }
#pragma unroll
    for (uint32_t k = 0; k < kPer; k++) {
        if (d0 + k < T) {
            ranges[d0 + k] = make_uint2(start, start + tot[k]);
            chunk_base[d0 + k] = cstart;
            if (order) atomicAdd(&cnt[255u - min(tot[k] >> 4, 255u)], 1u);
        }
        start += tot[k];
        cstart += (tot[k] + 63u) >> 6;
    }
    if (!order) return;
    __syncthreads();
    if (t < 64u) {  // exclusive scan of the 256 bucket counts by one wave
        uint32_t v[4], c = 0;
#pragma unroll
        for (int k = 0; k < 4; k++) {
            v[k] = cnt[4 * t + k];
            c += v[k];
        }
        uint32_t ci = c;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(ci, o, 64);
            if (t >= (uint32_t)o) ci += y;
        }
        uint32_t run = ci - c;
#pragma unroll
        for (int k = 0; k < 4; k++) {
            cnt[4 * t + k] = run;
            run += v[k];
        }
    }
    __syncthreads();
#pragma unroll
    for (uint32_t k = 0; k < kPer; k++)
        if (d0 + k < T) order[atomicAdd(&cnt[255u - min(tot[k] >> 4, 255u)], 1u)] = d0 + k;
}

__device__ __forceinline__ uint32_t half16(uint32_t word, uint32_t d) { return (word >> (16u * (d & 1u))) & 0xffffu; }

template <int W>
__global__ __launch_bounds__(64 * W) void tile_scatter_kernel(
    const uint32_t* __restrict__ keys, const uint32_t* __restrict__ vals, const uint32_t* n_dev,
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
    for (uint32_t it = blockIdx.x; it < B; it += gridDim.x) {  // grid <= kTileSortMaxBlocks
        // XCD-aware slice order: workgroups are dispatched round-robin over the 8 XCDs, so map
        // the workgroups of one XCD to consecutive slices. Each tile's output segment is then
        // written mostly from one L2, which merges the short per-slice runs into whole lines
        // before they leave (the runs average ~2 pairs: without this every store is a partial line).
        const uint32_t vb = (B == gridDim.x && (B & 7u) == 0u) ? (it & 7u) * (B >> 3) + (it >> 3) : it;
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
                    d[k] = i < we ? keys[i] : 0xffffffffu;
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
                nd[k] = i < we ? keys[i] : 0u;
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
                        nd[k] = i < we ? keys[i] : 0u;
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

uint32_t tile_sort_blocks(uint64_t p_bound) { return tile_blocks_for(p_bound); }

uint64_t tile_sort_scratch(uint64_t p_bound, uint32_t T) {
    const uint64_t B = tile_sort_blocks(p_bound);
    return (uint64_t)T * (B + (B + kColChunk - 1) / kColChunk);
}

hipError_t tile_sort(hipStream_t st, const uint32_t* keys, const uint32_t* vals, const uint32_t* p_dev,
                     uint64_t p_bound, uint32_t T, uint32_t nbits, uint32_t* scratch,
                     uint32_t* vals_out, uint2* ranges, uint32_t* order, uint32_t* chunk_base) {
    if (T == 0 || T > kTileSortMaxTiles) return hipErrorInvalidValue;
    const uint32_t B = tile_sort_blocks(p_bound);
    const uint32_t C = (B + kColChunk - 1) / kColChunk;
    uint32_t* hist = scratch;
    uint32_t* csum = scratch + (size_t)T * B;
    const uint32_t grid = std::min<uint32_t>(B, kTileSortMaxBlocks);
    hipLaunchKernelGGL(tile_hist_kernel, dim3(grid), dim3(kSortThreads), T * sizeof(uint32_t), st, keys,
                       p_dev, T, hist);
    hipLaunchKernelGGL(tile_colscan_kernel, dim3((T + 255) / 256, std::min<uint32_t>(C, 16u)), dim3(256), 0, st, hist, T, p_dev,
                       csum);
    hipLaunchKernelGGL(tile_totals_kernel, dim3((T + 255) / 256), dim3(256), 0, st, csum, T, p_dev, ranges);
    hipLaunchKernelGGL(tile_starts_kernel, dim3(1), dim3(1024), 0, st, T, ranges, order, chunk_base);
    // 8 waves per block when their counters fit the 160 KB of LDS (T <= 8192), else 4
    const uint32_t lds8 = (T + 8u * ((T + 1u) >> 1)) * (uint32_t)sizeof(uint32_t);
    if (lds8 <= 160u * 1024u) {
        hipLaunchKernelGGL(tile_scatter_kernel<8>, dim3(grid), dim3(512), lds8, st, keys, vals, p_dev, T,
                           nbits, hist, csum, ranges, vals_out);
    } else {
        const uint32_t lds4 = (T + 4u * ((T + 1u) >> 1)) * (uint32_t)sizeof(uint32_t);
        hipLaunchKernelGGL(tile_scatter_kernel<4>, dim3(grid), dim3(256), lds4, st, keys, vals, p_dev, T,
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

// ---- host launchers -----------------------------------------------------------------

uint32_t sort_blocks_for(uint64_t n_bound) {
    uint64_t b = (n_bound + kSortTile - 1) / kSortTile;
    if (b < 1) b = 1;
    if (b > kMaxSortBlocks) b = kMaxSortBlocks;
    return (uint32_t)b;
}

hipError_t radix_pass(hipStream_t st, const RadixPass& p) {
    const uint32_t B = p.nblocks;
    hipLaunchKernelGGL(radix_hist_kernel, dim3(B), dim3(kSortThreads), 0, st, p.keys_in, p.n_dev,
                       p.n_host, p.shift, (1u << p.nbits) - 1u, p.hist);
    hipLaunchKernelGGL(radix_digit_scan_kernel, dim3(256), dim3(256), 0, st, p.hist, B, p.totals);
    hipLaunchKernelGGL(radix_scatter_kernel, dim3(B), dim3(kSortThreads), 0, st, p.keys_in,
                       p.vals_in, p.n_dev, p.n_host, p.shift, p.nbits, p.hist, p.totals,
                       p.keys_out, p.vals_out, p.inverse_out);
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
