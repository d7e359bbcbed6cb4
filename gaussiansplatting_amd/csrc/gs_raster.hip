// gs_raster.hip — the tiled rasterizer's per-Gaussian and per-tile kernels on gfx950.
//
//   project_kernel    one thread per Gaussian: projectGaussians (tiled_shaders.metal:102-304)
//                     + the generateTilePairs filter (:755-774); writes the 36-B raster record
//                     (3 coalesced SoA streams), tile rect, tile count and depth key.
//   emit_kernel       one thread per depth-ranked Gaussian: writes its tile keys row-major
//                     (:784-793) into slots given by a prefix scan (deterministic, no atomics).
//   ranges_kernel     tile ranges by boundary detection over the sorted tile keys
//                     (replaces buildTileRanges' binary search, sort.metal:553-589).
//   forward_kernel    one 16x16 tile per 256-thread workgroup: the splat list is staged
//                     through LDS in 256-entry chunks and blended front to back in IEEE half
//                     (tiledForward, tiled_shaders.metal:307-385). It also records the float
//                     transmittance the backward would recompute (:430-460) so the backward
//                     needs one list traversal instead of two.
//   backward_kernel   one tile per wave, 4 pixels per lane, reverse traversal; the 9 linear
//                     per-(pixel, Gaussian) partials are summed per lane and reduced across the
//                     wave, then stored once per (tile, Gaussian) slot — no float atomics.
//   (the per-Gaussian chain that consumes the partials lives in gs_chain.hip)
//
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "gs_device.hpp"
#include "gs_internal.hpp"

namespace gs {

// ---------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void project_kernel(
    const GsGaussian* __restrict__ g, uint32_t n, GsTiledUniforms u, float4* __restrict__ rec,
    uint32_t* __restrict__ count,
    uint32_t* __restrict__ dkey, uint2* __restrict__ rect, GsProjected* __restrict__ dbg) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const GaussianIn gin = load_gaussian(g, i);
    Projected p;
    project(gin, u, p);
    const uint32_t cnt = pair_count(p);
    if (!dbg) {  // a debug re-projection (gs_debug_projected) leaves the frame's buffers alone
        float4* r = rec + (size_t)i * kRecQuads;
        r[0] = make_float4(p.sx, p.sy, p.c0, p.c1);
        r[1] = make_float4(p.c2, p.opacity, p.r, p.g);
        float ex, ey, kq;
        cull_extents(p.c0, p.c1, p.c2, p.opacity, ex, ey, kq);
        // w: |conic|_1 in the forward's evaluation order (tiled_shaders.metal:350-351)
        r[2] = make_float4(p.b, ex, ey, fabsf(p.c0) + fabsf(p.c1) + fabsf(p.c2));
        // quad 3: .x = first emission slot (filled in by emit), .y = culling-ellipse bound
        r[3] = make_float4(0.0f, kq, 0.0f, 0.0f);
        count[i] = cnt;
        dkey[i] = cnt ? depth_key(p.depth) : 0xffffffffu;
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

// ---------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void emit_kernel(
    uint32_t n, const uint32_t* __restrict__ dsorted, const uint32_t* __restrict__ count,
    const uint2* __restrict__ rect, const uint32_t* __restrict__ offset, uint32_t tiles_x,
    uint32_t* __restrict__ tile0, uint32_t* __restrict__ val0, uint32_t* __restrict__ goff,
    float4* __restrict__ rec,
    uint64_t cap, uint32_t* __restrict__ overflow) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t gid = dsorted[i];
    const uint32_t c = count[gid];
    if (c == 0) return;
    const uint64_t o = offset[i];
    if (o + c > cap) {
        atomicOr(overflow, 1u);
        return;
    }
    goff[gid] = (uint32_t)o;
    reinterpret_cast<uint32_t*>(rec + (size_t)gid * kRecQuads + 3)[0] = (uint32_t)o;
    const uint2 r = rect[gid];
    const uint32_t x0 = r.x & 0xffffu, y0 = r.x >> 16, x1 = r.y & 0xffffu, y1 = r.y >> 16;
    uint32_t k = (uint32_t)o, j = 0;
    const uint32_t packed = gid << kPairJBits;
    for (uint32_t ty = y0; ty <= y1; ty++)
        for (uint32_t tx = x0; tx <= x1; tx++) {
            tile0[k] = ty * tiles_x + tx;
            val0[k] = packed | j;
            k++;
            j++;
        }
}

// ---------------------------------------------------------------------------------------
// Slot-parallel pair emission: a persistent grid walks the output in 2048-slot windows. For a
// window the owning depth ranks are found by binary search over the emission offsets (they are
// monotone; the non-emitting Gaussians all sort to the end, so every rank inside a window owns
// at least one slot), staged in LDS, and each thread resolves its slots with an LDS binary search.
// Every store is coalesced, and the work per thread no longer depends on a Gaussian's tile count.
constexpr uint32_t kEmitWin = 2048;

__device__ __forceinline__ uint32_t upper_bound_u32(const uint32_t* __restrict__ a, uint32_t n, uint32_t v) {
    uint32_t lo = 0, hi = n;
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (a[mid] <= v) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

__global__ __launch_bounds__(256) void emit_slots_kernel(
    uint32_t n, const uint32_t* __restrict__ dsorted, const uint2* __restrict__ rect,
    const uint32_t* __restrict__ offset, const uint32_t* __restrict__ p_dev, uint32_t tiles_x,
    uint32_t* __restrict__ tile0, uint32_t* __restrict__ val0, uint32_t* __restrict__ goff,
    float4* __restrict__ rec, uint64_t cap, uint32_t* __restrict__ overflow) {
    __shared__ uint32_t s_off[kEmitWin + 1];
    __shared__ uint32_t s_gid[kEmitWin];
    __shared__ uint32_t s_lo, s_cnt;
    const uint32_t t = threadIdx.x;
    const uint32_t P = *p_dev;
    const uint64_t Pc = P < cap ? P : cap;
    if (blockIdx.x == 0 && t == 0 && (uint64_t)P > cap) atomicOr(overflow, 1u);
    const uint32_t nwin = (uint32_t)((Pc + kEmitWin - 1) / kEmitWin);
    for (uint32_t wdw = blockIdx.x; wdw < nwin; wdw += gridDim.x) {
        const uint32_t s0 = wdw * kEmitWin;
        const uint32_t s1 = (uint32_t)min((uint64_t)s0 + kEmitWin, Pc);
        __syncthreads();
        if (t == 0) {
            const uint32_t lo = upper_bound_u32(offset, n, s0) - 1u;
            const uint32_t hi = upper_bound_u32(offset, n, s1 - 1u) - 1u;
            s_lo = lo;
            s_cnt = hi - lo + 1u;
        }
        __syncthreads();
        const uint32_t lo = s_lo, cnt = s_cnt;  // cnt <= kEmitWin (each rank owns >= 1 slot)
        for (uint32_t k = t; k < cnt; k += 256u) {
            s_off[k] = offset[lo + k];
            s_gid[k] = dsorted[lo + k];
        }
        __syncthreads();
        for (uint32_t s = s0 + t; s < s1; s += 256u) {
            const uint32_t k = upper_bound_u32(s_off, cnt, s) - 1u;
            const uint32_t gid = s_gid[k];
            const uint32_t j = s - s_off[k];
            const uint2 r = rect[gid];
            const uint32_t x0 = r.x & 0xffffu, y0 = r.x >> 16, x1 = r.y & 0xffffu;
            const uint32_t rw = x1 - x0 + 1u;
            const uint32_t ty = y0 + j / rw, tx = x0 + j % rw;  // row-major (:784-793)
            tile0[s] = ty * tiles_x + tx;
            val0[s] = (gid << kPairJBits) | j;
            if (j == 0u) {
                goff[gid] = s;
                reinterpret_cast<uint32_t*>(rec + (size_t)gid * kRecQuads + 3)[0] = s;
            }
        }
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

// ---------------------------------------------------------------------------------------
// Launch order of the blend kernels: tiles bucketed by list length, longest first, so the long
// tiles start in the first wave of workgroups and the tail of the launch is made of short ones
// (longest-processing-time-first). The order inside a bucket is irrelevant to the results.
__global__ __launch_bounds__(1024) void tile_order_kernel(const uint2* __restrict__ ranges,
                                                          uint32_t num_tiles,
                                                          uint32_t* __restrict__ order) {
    __shared__ uint32_t cnt[256];
    const uint32_t t = threadIdx.x;
    if (t < 256) cnt[t] = 0u;
    __syncthreads();
    for (uint32_t i = t; i < num_tiles; i += 1024u) {
        const uint2 r = ranges[i];
        atomicAdd(&cnt[255u - min((r.y - r.x) >> 4, 255u)], 1u);
    }
    __syncthreads();
    if (t < 64) {  // exclusive scan of the 256 bucket counts by one wave
        uint32_t v[4], s = 0;
#pragma unroll
        for (int k = 0; k < 4; k++) {
            v[k] = cnt[4 * t + k];
            s += v[k];
        }
        uint32_t inc = s;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(inc, o, 64);
            if (t >= (uint32_t)o) inc += y;
        }
        uint32_t run = inc - s;
#pragma unroll
        for (int k = 0; k < 4; k++) {
            cnt[4 * t + k] = run;
            run += v[k];
        }
    }
    __syncthreads();
    for (uint32_t i = t; i < num_tiles; i += 1024u) {
        const uint2 r = ranges[i];
        order[atomicAdd(&cnt[255u - min((r.y - r.x) >> 4, 255u)], 1u)] = i;
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
                          GsProjected* debug_out) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(project_kernel, dim3(div_up(n, 256)), dim3(256), 0, st, g, n, u, gb.rec,
                       gb.count, gb.dkey, gb.rect, debug_out);
    return hipGetLastError();
}

hipError_t launch_emit(hipStream_t st, uint32_t n, const GaussianBuffers& gb,
                       const uint32_t* dsorted, const PairBuffers& pb, uint32_t tiles_x,
                       const uint32_t* p_dev, uint64_t p_bound, uint32_t* overflow) {
    if (n == 0) return hipSuccess;
#if GS_EMIT_SLOTS
    uint32_t blocks = div_up(std::min<uint64_t>(p_bound, pb.cap), kEmitWin);
    blocks = blocks < 1u ? 1u : (blocks > 4096u ? 4096u : blocks);
    hipLaunchKernelGGL(emit_slots_kernel, dim3(blocks), dim3(256), 0, st, n, dsorted, gb.rect, gb.offset,
                       p_dev, tiles_x, pb.tile0, pb.val0, gb.goff, gb.rec, pb.cap, overflow);
#else
    (void)p_dev;
    (void)p_bound;
    hipLaunchKernelGGL(emit_kernel, dim3(div_up(n, 256)), dim3(256), 0, st, n, dsorted, gb.count,
                       gb.rect, gb.offset, tiles_x, pb.tile0, pb.val0, gb.goff, gb.rec, pb.cap, overflow);
#endif
    return hipGetLastError();
}

hipError_t launch_ranges(hipStream_t st, const uint32_t* s_tile, const uint32_t* p_dev,
                         uint64_t p_bound, uint32_t num_tiles, uint2* ranges) {
    uint32_t blocks = div_up(p_bound + 1, 256);
    if (blocks > 4096) blocks = 4096;
    hipLaunchKernelGGL(ranges_kernel, dim3(blocks), dim3(256), 0, st, s_tile, p_dev, num_tiles,
                       ranges);
    return hipGetLastError();
}

hipError_t launch_tile_order(hipStream_t st, const uint2* ranges, uint32_t num_tiles,
                             uint32_t* order) {
    if (num_tiles == 0) return hipSuccess;
    hipLaunchKernelGGL(tile_order_kernel, dim3(1), dim3(1024), 0, st, ranges, num_tiles, order);
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
