// gs_raster.hip — the tiled rasterizer's per-Gaussian and pair-emission kernels on gfx950.
//
//   project_kernel       one thread per Gaussian: projectGaussians (tiled_shaders.metal:102-304)
//                        + the generateTilePairs filter (:755-774); writes the 64-B raster
//                        record, tile rect, tile count and depth key, and the depth sort's digit
//                        histograms.
//   window_starts_kernel the emission windows' owners after a capacity growth (offsets_scan_kernel
//                        marks them itself otherwise).
//   emit_slots_kernel    generateTilePairs' emission (:784-793) in depth order, at offsets from a
//                        prefix scan (deterministic, no atomic counter), coalesced 2048-slot windows.
//   ranges_kernel,       tile ranges / list-chunk bases + launch order for the two-pass tile sort
//   chunk_base_kernel    (buildTileRanges, sort.metal:553-589; the one-pass sort derives them in
//                        tile_finish_kernel).
// The blend kernels are in gs_blend.hip, the per-Gaussian chain in gs_chain.hip.
//
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "gs_device.hpp"
#include "gs_internal.hpp"
#include "gs_emit.hpp"

namespace gs {

// ---------------------------------------------------------------------------------------
// With `hist` (the single-sweep depth sort, gs_sort.hip), the kernel also builds the four digit
// histograms of the depth keys it writes (per-block LDS histograms, one global atomic per non-empty
// bin and block — hence 1024-thread blocks) and counts the Gaussians it does not emit: the sort
// needs no histogram pass of its own. `hist` must be zero on entry (the emission kernel re-zeroes
// it for the next frame). `zero_words` are the frame's other scan words (tickets, status words).
__global__ __launch_bounds__(kProjectThreads) void project_kernel(
    const GsGaussian* __restrict__ g, uint32_t n, GsTiledUniforms u, float4* __restrict__ rec,
    uint32_t* __restrict__ count,
    uint32_t* __restrict__ dkey, uint2* __restrict__ rect, GsProjected* __restrict__ dbg,
    uint32_t* __restrict__ zero_words, uint32_t nzero, uint32_t* __restrict__ hist) {
    __shared__ uint32_t h_lds[kSweepHistWords + 1];  // digit histograms, then the culled count
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    // the frame's sort/scan words (zeroed here instead of by a separate memset launch)
    for (uint32_t z = i; z < nzero; z += gridDim.x * blockDim.x) zero_words[z] = 0u;
    if (hist) {  // (block-uniform)
        for (uint32_t z = threadIdx.x; z <= kSweepHistWords; z += blockDim.x) h_lds[z] = 0u;
        __syncthreads();
    }
    if (i < n) {
    const GaussianIn gin = load_gaussian(g, i);
    Projected p;
    project(gin, u, p);
    const uint32_t cnt = pair_count(p);
    if (hist) {
        const uint32_t k = cnt ? depth_key(p.depth) : 0xffffffffu;
#pragma unroll
        for (uint32_t d = 0; d < kSweepPasses; d++) atomicAdd(&h_lds[d * 256u + ((k >> (8u * d)) & sweep_digit_mask(d))], 1u);
        if (!cnt) atomicAdd(&h_lds[kSweepHistWords], 1u);
    }
    if (!dbg) {  // a debug re-projection (gs_debug_projected) leaves the frame's buffers alone
        count[i] = cnt;
        dkey[i] = cnt ? depth_key(p.depth) : 0xffffffffu;
    }
    // A Gaussian with no tile pairs is never gathered (every reader of the record and the rect looks
    // at its count first): neither is written for it. (Config 5: most of its projections.)
    if (!dbg && cnt) {
        float4* r = rec + (size_t)i * kRecQuads;
        r[0] = make_float4(p.sx, p.sy, p.c0, p.c1);
        r[1] = make_float4(p.c2, p.opacity, p.r, p.g);
        float ex, ey, kq;
        cull_extents(p.c0, p.c1, p.c2, p.opacity, ex, ey, kq);
        // w: |conic|_1 in the forward's evaluation order (tiled_shaders.metal:350-351)
        r[2] = make_float4(p.b, ex, ey, fabsf(p.c0) + fabsf(p.c1) + fabsf(p.c2));
        // quad 3: .x = goff, the backward's partial-sum slot base on the per-tile order (filled in by
        //         the tile scatter or the offset scan; the global order's backward reads goff itself),
        //         .y = culling-ellipse bound
        r[3] = make_float4(0.0f, kq, 0.0f, 0.0f);
        rect[i] = make_uint2((p.tminx & 0xffffu) | (p.tminy << 16), (p.tmaxx & 0xffffu) | (p.tmaxy << 16));
    }
    if (dbg) {
        GsProjected o;
        o.screen_pos[0] = p.sx; o.screen_pos[1] = p.sy;
        o.conic[0] = p.c0; o.conic[1] = p.c1; o.conic[2] = p.c2;
        o.depth = p.depth;
        o.opacity = p.opacity;
        o.color[0] = p.r; o.color[1] = p.g; o.color[2] = p.b;
        o.radius = p.radius;
        o.tile_min_x = p.tminx; o.tile_min_y = p.tminy;
        o.tile_max_x = p.tmaxx; o.tile_max_y = p.tmaxy;
        o._pad1 = 0.0f;
        o.view_pos_xy[0] = p.vx; o.view_pos_xy[1] = p.vy;
        o.cov2d[0] = p.ca; o.cov2d[1] = p.cb; o.cov2d[2] = p.cc;
        o._pad2 = 0.0f;
        dbg[i] = o;
    }
    }
    if (hist) {
        __syncthreads();
        for (uint32_t z = threadIdx.x; z < kSweepHistWords; z += blockDim.x)
            if (h_lds[z]) atomicAdd(&hist[z], h_lds[z]);
        if (threadIdx.x == 0 && h_lds[kSweepHistWords]) atomicAdd(&hist[kSweepHistWords + kSweepCtrCulled], h_lds[kSweepHistWords]);
    }
}

// ---------------------------------------------------------------------------------------
// Slot-parallel pair emission: a persistent grid walks the output in kEmitWin-slot windows. The
// depth rank owning each window's first slot comes from window_starts_kernel (one thread per rank
// marks the window starts inside its slot range, no search); the window's ranks and offsets are
// staged in LDS, and a max-scan over the ranks' first slots gives every slot its owner. Every store is
// coalesced, and the work per thread does not depend on a Gaussian's tile count.
__global__ __launch_bounds__(256) void window_starts_kernel(uint32_t n, const uint32_t* __restrict__ offset,
                                                            const uint32_t* __restrict__ p_dev, uint64_t cap,
                                                            uint32_t* __restrict__ wstart) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint64_t P = *p_dev;
    const uint64_t Pc = P < cap ? P : cap;
    const uint64_t o = offset[i];
    uint64_t e = i + 1u < n ? (uint64_t)offset[i + 1u] : P;
    e = e < Pc ? e : Pc;
    for (uint64_t w = (o + kEmitWin - 1) / kEmitWin; w * kEmitWin < e; w++) wstart[w] = i;
}

// Pair emission in Gaussian order (the per-tile depth sort path, gs_segsort.hip): the emission
// offsets are the slot offsets goff. One wave per 64 consecutive Gaussians: the wave's slots
// [goff[first], goff[last] + count[last]) are walked 64 at a time, one slot per lane (coalesced
// stores); a slot's Gaussian is the last of the 64 whose goff is at most the slot (a binary search
// over the lanes' goff by cross-lane reads; a culled Gaussian shares its successor's goff and never
// wins). No window owners and no rank staging: culled Gaussians anywhere in the order cost nothing.
__global__ __launch_bounds__(256) void emit_gid_kernel(
    uint32_t n, const uint32_t* __restrict__ count, const uint32_t* __restrict__ goff,
    const uint2* __restrict__ rect, const uint32_t* __restrict__ p_dev, uint32_t tiles_x,
    uint32_t* __restrict__ tile0, uint32_t* __restrict__ val0, uint64_t cap, uint32_t* __restrict__ overflow,
    uint32_t* __restrict__ host_mirror, uint32_t* __restrict__ hist_rezero, uint32_t key16) {
    const uint32_t t = threadIdx.x, lane = t & 63u;
    const uint32_t P = *p_dev;
    if (blockIdx.x == 0) emit_frame_duties(t, 256u, P, cap, overflow, host_mirror, hist_rezero);
    const uint32_t first = blockIdx.x * 256u + t - lane;  // the wave's first Gaussian
    if (first >= n) return;
    const uint32_t stop = (uint64_t)P < cap ? P : (uint32_t)cap;
    wave_walk_pairs(first, n, lane, count, goff, rect, tiles_x, stop, [&](uint32_t s, uint32_t tile, uint32_t v) {
        if (key16)
            reinterpret_cast<uint16_t*>(tile0)[s] = (uint16_t)tile;
        else
            tile0[s] = tile;
        val0[s] = v;
    });
}

__global__ __launch_bounds__(256) void emit_slots_kernel(
    uint32_t n, const uint32_t* __restrict__ dsorted, const uint2* __restrict__ rect,
    const uint32_t* __restrict__ offset, const uint32_t* __restrict__ wstart,
    const uint32_t* __restrict__ p_dev, uint32_t tiles_x,
    uint32_t* __restrict__ tile0, uint32_t* __restrict__ val0, uint32_t* __restrict__ goff,
    float4* __restrict__ rec, uint64_t cap, uint32_t* __restrict__ overflow,
    uint32_t* __restrict__ host_mirror, uint32_t* __restrict__ hist_rezero, uint32_t key16,
    uint32_t* __restrict__ lsd_hist, uint32_t lsd_blocks, uint32_t lsd_mask) {
    constexpr uint32_t kR = kEmitWin + 1;  // ranks staged per window
    __shared__ uint32_t s_off[kR];
    __shared__ uint32_t s_gid[kR];
    __shared__ uint32_t s_org[kR];    // first tile of the rect (ty0 * tiles_x + tx0)
    __shared__ uint32_t s_shape[kR];  // rect width (<= 256, 9 bits) | magic ceil(2^16 / width) << 9
    __shared__ uint32_t s_own[kEmitWin];
    __shared__ uint32_t s_wmax[4];
    __shared__ uint32_t s_hist[256];  // (lsd_hist) the window's first-pass digit counts
    const uint32_t t = threadIdx.x, lane = t & 63u, wv = t >> 6;
    const uint32_t P = *p_dev;
    const uint64_t Pc = P < cap ? P : cap;
    if (blockIdx.x == 0) emit_frame_duties(t, 256u, P, cap, overflow, host_mirror, hist_rezero);
    const uint32_t nwin = (uint32_t)((Pc + kEmitWin - 1) / kEmitWin);
    // lsd_hist: the LSD tile sort's first-pass histogram, hist[digit][sort block], counted here
    // instead of by a pass over the emitted keys. A sort block's slice is a multiple of 2048 slots
    // (gs_sort.hip sort_slice), so every window lies in one slice; a workgroup walks a contiguous run
    // of windows, so it adds its counts to the histogram once per slice it meets (one per window
    // across a strided walk: 8.6M global atomics at config 5, 178 -> 609 us).
    uint32_t lsd_per = 1, cur = 0xffffffffu;
    if (lsd_hist) {
        lsd_per = (P + lsd_blocks - 1u) / lsd_blocks;
        lsd_per = (lsd_per + 2047u) / 2048u * 2048u;
        lsd_per = lsd_per ? lsd_per : 2048u;
    }
    auto flush = [&]() {  // (after a barrier: the slice's counts are all in s_hist)
        const uint32_t c = s_hist[t];
        if (cur != 0xffffffffu && t <= lsd_mask && c) atomicAdd(&lsd_hist[t * lsd_blocks + cur], c);
        s_hist[t] = 0u;
    };
    const uint32_t per_blk = (nwin + gridDim.x - 1u) / gridDim.x;
    const uint32_t w0 = blockIdx.x * per_blk, w1 = min(nwin, w0 + per_blk);
    for (uint32_t wdw = w0; wdw < w1; wdw++) {
        const uint32_t s0 = wdw * kEmitWin;
        if (lsd_hist && s0 / lsd_per != cur) {  // (block-uniform)
            __syncthreads();
            flush();
            cur = s0 / lsd_per;
        }
        const uint32_t s1 = (uint32_t)min((uint64_t)s0 + kEmitWin, Pc);
        // ranks lo .. (start rank of the next window): every one but possibly the last owns a slot
        // here, so at most kEmitWin + 1 of them; the extra one (offset >= s1) is ignored
        const uint32_t lo = wstart[wdw];
        const uint32_t last = wdw + 1u < nwin ? wstart[wdw + 1u] : n - 1u;
        const uint32_t cnt = min(last - lo + 1u, kR);
        __syncthreads();
        for (uint32_t q = t; q < kEmitWin; q += 256u) s_own[q] = 0u;
        __syncthreads();
        // per rank: offset, Gaussian, rect origin and width (one gather per Gaussian, not per slot);
        // the rank's first slot in the window marks its ownership run
        for (uint32_t k = t; k < cnt; k += 256u) {
            const uint32_t o = offset[lo + k], gid = dsorted[lo + k] & kDsortGidMask;
            const uint2 r = rect[gid];
            const uint32_t x0 = r.x & 0xffffu, y0 = r.x >> 16, x1 = r.y & 0xffffu;
            const uint32_t rw = x1 - x0 + 1u;
            s_off[k] = o;
            s_gid[k] = gid;
            s_org[k] = y0 * tiles_x + x0;
            s_shape[k] = rw | (((65536u + rw - 1u) / rw) << 9);
            if (o < s1) s_own[o > s0 ? o - s0 : 0u] = k;
        }
        __syncthreads();
        // inclusive max-scan of the run heads: owner rank of every slot (thread t: slots kSpt t .. + kSpt - 1)
        constexpr uint32_t kSpt = kEmitWin / 256u;
        uint32_t v[kSpt], m = 0;
#pragma unroll
        for (uint32_t q = 0; q < kSpt; q++) {
            m = max(m, s_own[kSpt * t + q]);
            v[q] = m;
        }
        uint32_t inc = m;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(inc, o, 64);
            if (lane >= (uint32_t)o) inc = max(inc, y);
        }
        if (lane == 63u) s_wmax[wv] = inc;
        __syncthreads();
        uint32_t carry = __shfl_up(inc, 1, 64);
        carry = lane ? carry : 0u;
        for (uint32_t k = 0; k < wv; k++) carry = max(carry, s_wmax[k]);
#pragma unroll
        for (uint32_t q = 0; q < kSpt; q++) s_own[kSpt * t + q] = max(v[q], carry);
        __syncthreads();
        for (uint32_t s = s0 + t; s < s1; s += 256u) {
            const uint32_t k = s_own[s - s0];
            const uint32_t j = s - s_off[k];
            const uint32_t shape = s_shape[k];
            const uint32_t rw = shape & 0x1ffu;
            const uint32_t dy = (j * (shape >> 9)) >> 16;  // j / rw, exact for j < 256, rw <= 256
            const uint32_t gid = s_gid[k];
            const uint32_t tile = s_org[k] + dy * tiles_x + (j - dy * rw);  // row-major (:784-793)
            if (key16)
                reinterpret_cast<uint16_t*>(tile0)[s] = (uint16_t)tile;
            else
                tile0[s] = tile;
            val0[s] = (gid << kPairJBits) | j;
            if (lsd_hist) atomicAdd(&s_hist[tile & lsd_mask], 1u);
        }
    }
    if (lsd_hist && w0 < w1) {
        __syncthreads();
        flush();
    }
}

// ---------------------------------------------------------------------------------------
// ranges[t] = (start, end) over the sorted pairs; empty tiles get start = end = lower bound.
__global__ __launch_bounds__(256) void ranges_kernel(const uint32_t* __restrict__ s_tile,
                                                     const uint32_t* __restrict__ p_dev,
                                                     uint32_t num_tiles, uint2* __restrict__ ranges) {
    const uint32_t P = *p_dev;
    for (uint64_t s = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; s <= P;
         s += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t cur = s < P ? s_tile[s] : num_tiles;
        const int64_t prev = s > 0 ? (int64_t)s_tile[s - 1] : -1;
        if (s > 0 && (int64_t)cur == prev) continue;
        if (prev >= 0) ranges[prev].y = (uint32_t)s;
        const uint32_t hi = cur < num_tiles ? cur : num_tiles - 1u;
        for (int64_t t = prev + 1; t <= (int64_t)hi; t++) {
            ranges[t].x = (uint32_t)s;
            if ((uint32_t)t < cur) ranges[t].y = (uint32_t)s;
        }
    }
}

// The same ranges by binary search, as the reference's buildTileRanges (sort.metal:553-589: a
// lower-bound search per tile): one thread per tile searches the sorted keys for its first and
// its successor's first pair (two independent chains of ~log2 P dependent loads). At config 5
// (69M pairs) this reads ~2 x 26 lines per tile instead of streaming all 276 MB of keys.
__global__ __launch_bounds__(256) void ranges_search_kernel(const uint32_t* __restrict__ s_tile,
                                                            const uint32_t* __restrict__ p_dev,
                                                            uint32_t num_tiles, uint2* __restrict__ ranges) {
    const uint32_t d = blockIdx.x * blockDim.x + threadIdx.x;
    if (d >= num_tiles) return;
    const uint32_t P = *p_dev;
    uint32_t lo0 = 0, hi0 = P, lo1 = 0, hi1 = P;
    while (lo0 < hi0 || lo1 < hi1) {
        if (lo0 < hi0) {
            const uint32_t m = lo0 + ((hi0 - lo0) >> 1);
            if (s_tile[m] < d) lo0 = m + 1u; else hi0 = m;
        }
        if (lo1 < hi1) {
            const uint32_t m = lo1 + ((hi1 - lo1) >> 1);
            if (s_tile[m] <= d) lo1 = m + 1u; else hi1 = m;
        }
    }
    ranges[d] = make_uint2(lo0, lo1);
}

// ---------------------------------------------------------------------------------------
// chunk_base[t] = sum over t' < t of ceil(len(t') / 64): where tile t's band cull masks live
// (the one-pass tile sort computes this inside tile_finish_kernel).
// With `tile_cost`, it also zeroes this frame's forward work counters and the backward reorder's
// status words (what tile_finish_kernel does on the one-pass path). With `fill_empty` the ranges
// come from the LSD scatter's atomics, where an empty tile is (~0, 0): every range is rewritten as
// (start, start + len) from the scan of the lengths, which gives an empty tile the lower bound of
// its key as the binary search does.
__global__ __launch_bounds__(1024) void chunk_base_kernel(uint2* __restrict__ ranges, uint32_t T,
                                                          uint32_t* __restrict__ chunk_base,
                                                          uint32_t* __restrict__ tile_cost,
                                                          unsigned long long* __restrict__ reorder_words,
                                                          uint32_t nreorder, uint32_t fill_empty,
                                                          uint32_t* __restrict__ order) {
    // rounds of 8192 tiles, 8 consecutive tiles per thread: one load, one block scan and one store
    // per round (1080p: one round; the 1024-tile rounds with three barriers each took 17 us)
    constexpr uint32_t kPer = 8;
    __shared__ uint32_t wsum[16], wlen[16];
    __shared__ uint32_t carry, lcarry;
    __shared__ uint32_t cnt[256];
    const uint32_t t = threadIdx.x, lane = t & 63u, w = t >> 6;
    if (t == 0) carry = lcarry = 0u;
    if (t < 256u) cnt[t] = 0u;
    if (tile_cost) {
        for (uint32_t d = t; d < T; d += 1024u) tile_cost[d] = 0u;
        for (uint32_t z = t; z < nreorder; z += 1024u) reorder_words[z] = 0ull;
    }
    auto bucket = [](uint32_t len) { return 255u - min(len >> 4, 255u); };  // longest first
    for (uint32_t b0 = 0; b0 < T; b0 += 1024u * kPer) {
        __syncthreads();
        const uint32_t d0 = b0 + kPer * t;
        uint32_t len[kPer], sc = 0, sl = 0;
#pragma unroll
        for (uint32_t k = 0; k < kPer; k++) {
            const uint2 r = d0 + k < T ? ranges[d0 + k] : make_uint2(0u, 0u);
            len[k] = r.x == 0xffffffffu ? 0u : r.y - r.x;
            sc += (len[k] + 63u) >> 6;
            sl += len[k];
        }
        uint32_t inc = sc, linc = sl;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(inc, o, 64), yl = __shfl_up(linc, o, 64);
            if (lane >= (uint32_t)o) {
                inc += y;
                linc += yl;
            }
        }
        if (lane == 63u) {
            wsum[w] = inc;
            wlen[w] = linc;
        }
        __syncthreads();
        uint32_t ex = carry + inc - sc, lex = lcarry + linc - sl;
        for (uint32_t k = 0; k < w; k++) {
            ex += wsum[k];
            lex += wlen[k];
        }
#pragma unroll
        for (uint32_t k = 0; k < kPer; k++) {
            const uint32_t d = d0 + k;
            if (d < T) {
                chunk_base[d] = ex;
                if (fill_empty) ranges[d] = make_uint2(lex, lex + len[k]);
                if (order) atomicAdd(&cnt[bucket(len[k])], 1u);
            }
            ex += (len[k] + 63u) >> 6;
            lex += len[k];
        }
        __syncthreads();
        if (t == 1023u) {
            carry = ex;
            lcarry = lex;
        }
    }
    if (!order) return;
    // the blend launch order (until round 5 its own single-workgroup launch): longest first, bucket
    // starts by one wave's scan; each thread reads back only the ranges it wrote itself above
    __syncthreads();
    if (t < 64u) {
        uint32_t v[4], sv = 0;
#pragma unroll
        for (int k = 0; k < 4; k++) {
            v[k] = cnt[4 * t + k];
            sv += v[k];
        }
        uint32_t inc = sv;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(inc, o, 64);
            if (t >= (uint32_t)o) inc += y;
        }
        uint32_t run = inc - sv;
#pragma unroll
        for (int k = 0; k < 4; k++) {
            cnt[4 * t + k] = run;
            run += v[k];
        }
    }
    __syncthreads();
    for (uint32_t b0 = 0; b0 < T; b0 += 1024u * kPer) {
        const uint32_t d0 = b0 + kPer * t;
#pragma unroll
        for (uint32_t k = 0; k < kPer; k++)
            if (d0 + k < T) {
                const uint2 r = ranges[d0 + k];
                order[atomicAdd(&cnt[bucket(r.x == 0xffffffffu ? 0u : r.y - r.x)], 1u)] = d0 + k;
            }
    }
}

// ---------------------------------------------------------------------------------------
// The sorted tile keys are not materialised by the one-pass tile sort: a slot's tile is the
// range that contains it (binary search over the monotone range starts).
__global__ void debug_pairs_kernel(const uint2* __restrict__ ranges, uint32_t num_tiles,
                                   const uint32_t* __restrict__ s_val,
                                   const uint32_t* __restrict__ dkey,
                                   const uint32_t* __restrict__ p_dev, uint64_t cap,
                                   uint64_t* __restrict__ keys, uint32_t* __restrict__ values) {
    const uint64_t P = *p_dev;
    for (uint64_t s = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; s < P && s < cap;
         s += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t gi = s_val[s] >> kPairJBits;
        if (keys) {
            uint32_t lo = 0, hi = num_tiles;  // last tile with start <= s and a non-empty range
            while (hi - lo > 1u) {
                const uint32_t mid = (lo + hi) >> 1;
                if (ranges[mid].x <= s) lo = mid; else hi = mid;
            }
            while (lo + 1u < num_tiles && ranges[lo].y <= s) lo++;
            keys[s] = ((uint64_t)lo << 32) | dkey[gi];
        }
        if (values) values[s] = gi;
    }
}

__global__ void debug_ranges_kernel(const uint2* __restrict__ r, uint32_t num_tiles,
                                    GsTileRange* __restrict__ out) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= num_tiles) return;
    out[t].start = r[t].x;
    out[t].count = r[t].y - r[t].x;
}

// ---- launchers --------------------------------------------------------------------------
static inline uint32_t div_up(uint64_t a, uint32_t b) { return (uint32_t)((a + b - 1) / b); }

hipError_t launch_project(hipStream_t st, const GsGaussian* g, uint32_t n,
                          const GsTiledUniforms& u, const GaussianBuffers& gb,
                          GsProjected* debug_out, uint32_t* zero_words, uint32_t nzero,
                          uint32_t* hist) {
    if (n == 0) return nzero ? hipMemsetAsync(zero_words, 0, nzero * sizeof(uint32_t), st) : hipSuccess;
    hipLaunchKernelGGL(project_kernel, dim3(div_up(n, kProjectThreads)), dim3(kProjectThreads), 0, st, g,
                       n, u, gb.rec, gb.count, gb.dkey, gb.rect, debug_out, zero_words, nzero, hist);
    return hipGetLastError();
}

hipError_t launch_emit(hipStream_t st, uint32_t n, const GaussianBuffers& gb,
                       const uint32_t* dsorted, const PairBuffers& pb, uint32_t tiles_x,
                       const uint32_t* p_dev, uint64_t p_bound, uint32_t* overflow,
                       bool wstart_ready, uint32_t* host_mirror, uint32_t* hist_rezero, bool key16,
                       uint32_t* lsd_hist, uint32_t lsd_blocks, uint32_t lsd_mask) {
    if (n == 0) return hipSuccess;
    if (!dsorted) {  // Gaussian order (per-tile depth sort): one wave per 64 Gaussians
        hipLaunchKernelGGL(emit_gid_kernel, dim3(div_up(n, 256)), dim3(256), 0, st, n, gb.count, gb.goff, gb.rect,
                           p_dev, tiles_x, pb.tile0, pb.val0, pb.cap, overflow, host_mirror, hist_rezero,
                           (uint32_t)key16);
        return hipGetLastError();
    }
    // A persistent grid of exactly the resident workgroups: each walks every grid-th window, so no
    // partial last round of workgroups runs its windows alone (4096 workgroups against the 1792 a
    // 256-CU device holds at 7 per CU left 0.29 of a round to the tail)
    static uint32_t resident = 0;
    if (!resident) {
        int per_cu = 0, dev = 0, cus = 0;
        if (hipGetDevice(&dev) == hipSuccess &&
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess &&
            hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, emit_slots_kernel, 256, 0) == hipSuccess &&
            per_cu > 0 && cus > 0)
            resident = (uint32_t)(per_cu * cus);
        else
            resident = 4096u;
    }
    uint32_t blocks = div_up(std::min<uint64_t>(p_bound, pb.cap), kEmitWin);
    blocks = blocks < 1u ? 1u : (blocks > resident ? resident : blocks);
    if (!wstart_ready)  // (offsets_scan marks the windows' owners itself)
        hipLaunchKernelGGL(window_starts_kernel, dim3(div_up(n, 256)), dim3(256), 0, st, n, gb.offset, p_dev,
                           pb.cap, pb.wstart);
    hipLaunchKernelGGL(emit_slots_kernel, dim3(blocks), dim3(256), 0, st, n, dsorted, gb.rect, gb.offset,
                       pb.wstart, p_dev, tiles_x, pb.tile0, pb.val0, gb.goff, gb.rec, pb.cap, overflow,
                       host_mirror, hist_rezero, (uint32_t)key16, lsd_hist, lsd_blocks, lsd_mask);
    return hipGetLastError();
}

hipError_t launch_ranges(hipStream_t st, const uint32_t* s_tile, const uint32_t* p_dev,
                         uint64_t p_bound, uint32_t num_tiles, uint2* ranges) {
    // a streaming pass over the keys while they are few, a binary search per tile beyond
    if (p_bound > 64ull * num_tiles) {
        hipLaunchKernelGGL(ranges_search_kernel, dim3(div_up(num_tiles, 256)), dim3(256), 0, st, s_tile, p_dev,
                           num_tiles, ranges);
        return hipGetLastError();
    }
    uint32_t blocks = div_up(p_bound + 1, 256);
    if (blocks > 4096) blocks = 4096;
    hipLaunchKernelGGL(ranges_kernel, dim3(blocks), dim3(256), 0, st, s_tile, p_dev, num_tiles,
                       ranges);
    return hipGetLastError();
}

hipError_t launch_chunk_base(hipStream_t st, uint2* ranges, uint32_t num_tiles,
                             uint32_t* chunk_base, uint32_t* tile_cost, unsigned long long* reorder_words,
                             uint32_t nreorder, bool fill_empty, uint32_t* order) {
    if (num_tiles == 0) return hipSuccess;
    hipLaunchKernelGGL(chunk_base_kernel, dim3(1), dim3(1024), 0, st, ranges, num_tiles, chunk_base, tile_cost,
                       reorder_words, nreorder, (uint32_t)fill_empty, order);
    return hipGetLastError();
}

hipError_t launch_debug_pairs(hipStream_t st, const PairBuffers& pb, const GaussianBuffers& gb,
                              const uint2* ranges, uint32_t num_tiles, const uint32_t* p_dev,
                              uint64_t cap, uint64_t* keys, uint32_t* values) {
    hipLaunchKernelGGL(debug_pairs_kernel, dim3(1024), dim3(256), 0, st, ranges, num_tiles, pb.s_val,
                       gb.dkey, p_dev, cap, keys, values);
    return hipGetLastError();
}

hipError_t launch_debug_ranges(hipStream_t st, const uint2* ranges, uint32_t num_tiles,
                               GsTileRange* out) {
    if (num_tiles == 0) return hipSuccess;
    hipLaunchKernelGGL(debug_ranges_kernel, dim3(div_up(num_tiles, 256)), dim3(256), 0, st,
                       ranges, num_tiles, out);
    return hipGetLastError();
}

}  // namespace gs
