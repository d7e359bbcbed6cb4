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

#include "gs_device.hpp"
#include "gs_internal.hpp"

namespace gs {

// ---------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void project_kernel(
    const GsGaussian* __restrict__ g, uint32_t n, GsTiledUniforms u, float4* __restrict__ rec_a,
    float4* __restrict__ rec_b, float* __restrict__ rec_c, uint32_t* __restrict__ count,
    uint32_t* __restrict__ dkey, uint2* __restrict__ rect, GsProjected* __restrict__ dbg) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const GaussianIn gin = load_gaussian(g, i);
    Projected p;
    project(gin, u, p);
    const uint32_t cnt = pair_count(p);
    rec_a[i] = make_float4(p.sx, p.sy, p.c0, p.c1);
    rec_b[i] = make_float4(p.c2, p.opacity, p.r, p.g);
    rec_c[i] = p.b;
    count[i] = cnt;
    dkey[i] = cnt ? depth_key(p.depth) : 0xffffffffu;
    rect[i] = make_uint2((p.tminx & 0xffffu) | (p.tminy << 16), (p.tmaxx & 0xffffu) | (p.tmaxy << 16));
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
    uint32_t* __restrict__ tile0, uint32_t* __restrict__ gid0, uint64_t cap,
    uint32_t* __restrict__ overflow) {
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
    const uint2 r = rect[gid];
    const uint32_t x0 = r.x & 0xffffu, y0 = r.x >> 16, x1 = r.y & 0xffffu, y1 = r.y >> 16;
    uint32_t k = (uint32_t)o;
    for (uint32_t ty = y0; ty <= y1; ty++)
        for (uint32_t tx = x0; tx <= x1; tx++) {
            tile0[k] = ty * tiles_x + tx;
            gid0[k] = gid;
            k++;
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

__device__ __forceinline__ uint32_t quantize_unorm8(float c) {
    return (uint32_t)rintf(fminf(fmaxf(c, 0.0f), 1.0f) * 255.0f);
}

// ---------------------------------------------------------------------------------------
constexpr int kFwdThreads = 256;

__global__ __launch_bounds__(kFwdThreads) void forward_kernel(
    uint32_t w, uint32_t h, uint32_t tiles_x, const float4* __restrict__ rec_a,
    const float4* __restrict__ rec_b, const float* __restrict__ rec_c,
    const uint32_t* __restrict__ s_gid, const uint2* __restrict__ ranges,
    const uint32_t* __restrict__ p_dev, uint32_t* __restrict__ last_idx,
    float* __restrict__ t_final, uint32_t* __restrict__ rgba8, float* __restrict__ rgb) {
    __shared__ float4 la[kFwdThreads];
    __shared__ float4 lb[kFwdThreads];
    __shared__ float lc[kFwdThreads];

    const uint32_t tile = blockIdx.x;
    const uint32_t tx = tile % tiles_x, ty = tile / tiles_x;
    const uint32_t x = tx * kTile + (threadIdx.x & 15u);
    const uint32_t y = ty * kTile + (threadIdx.x >> 4);
    const bool inside = x < w && y < h;
    const uint32_t pix = y * w + x;
    if (*p_dev == 0u) {  // tiled_rasterizer.mm:463-467: return before rendering
        if (inside) last_idx[pix] = 0xffffffffu;
        return;
    }
    const uint2 range = ranges[tile];
    const float px = (float)x + 0.5f, py = (float)y + 0.5f;

    const _Float16 hEps = (_Float16)0.0001f;
    const _Float16 hAlphaMax = (_Float16)0.99f;
    const _Float16 hAlphaMin = (_Float16)(1.0f / 255.0f);
    const _Float16 hPowMin = (_Float16)(-4.5f);
    const _Float16 hZero = (_Float16)0.0f;
    const _Float16 hOne = (_Float16)1.0f;

    _Float16 cr = hZero, cg = hZero, cb = hZero, T = hOne;
    float Tf = 1.0f, Tsnap = 1.0f;
    bool fdone = false;
    uint32_t last = 0xffffffffu;
    bool done = !inside;

    for (uint32_t base = range.x; base < range.y; base += kFwdThreads) {
        if (__syncthreads_count(!done) == 0) break;
        const uint32_t idx = base + threadIdx.x;
        if (idx < range.y) {
            const uint32_t gidx = s_gid[idx];
            la[threadIdx.x] = rec_a[gidx];
            lb[threadIdx.x] = rec_b[gidx];
            lc[threadIdx.x] = rec_c[gidx];
        }
        __syncthreads();
        const uint32_t cnt = min((uint32_t)kFwdThreads, range.y - base);
        if (!done) {
            for (uint32_t j = 0; j < cnt; j++) {
                const float4 A = la[j];
                const float4 B = lb[j];
                const float dx = px - A.x, dy = py - A.y;
                const float pw = -0.5f * (A.z * dx * dx + 2.0f * A.w * dx * dy + B.x * dy * dy);
                // float transmittance of the backward's T_final loop (tiled_shaders.metal:430-460)
                if (!fdone && !(pw > 0.0f || pw < -4.5f)) {
                    const float Gf = gs_expf(pw);
                    const float af = fminf(B.y * Gf, 0.99f);
                    if (!(af < 1.0f / 255.0f)) {
                        const float tt = Tf * (1.0f - af);
                        if (tt < 0.0001f) fdone = true;
                        else Tf = tt;
                    }
                }
                // half-precision blend (tiled_shaders.metal:350-373)
                const float cmag = fabsf(A.z) + fabsf(A.w) + fabsf(B.x);
                if (cmag < 0.0001f) continue;
                const _Float16 power = (_Float16)pw;
                if (power > hZero || power < hPowMin) continue;
                const _Float16 G = (_Float16)gs_expf((float)power);
                _Float16 alpha = (_Float16)B.y * G;
                alpha = alpha < hAlphaMax ? alpha : hAlphaMax;
                if (alpha < hAlphaMin) continue;
                cr = cr + ((_Float16)B.z * alpha) * T;
                cg = cg + ((_Float16)B.w * alpha) * T;
                cb = cb + ((_Float16)lc[j] * alpha) * T;
                T = T * (hOne - alpha);
                last = base + j;
                Tsnap = Tf;
                if (!(T > hEps)) {
                    done = true;
                    break;
                }
            }
        }
        __syncthreads();
    }
    if (!inside) return;
    cr = cr + hOne * T;
    cg = cg + hOne * T;
    cb = cb + hOne * T;
    last_idx[pix] = last;
    t_final[pix] = Tsnap;
    const float fr = (float)cr, fg = (float)cg, fb = (float)cb;
    rgba8[pix] = quantize_unorm8(fr) | (quantize_unorm8(fg) << 8) | (quantize_unorm8(fb) << 16) |
                 (255u << 24);
    if (rgb) {
        rgb[3 * pix + 0] = fr;
        rgb[3 * pix + 1] = fg;
        rgb[3 * pix + 2] = fb;
    }
}

// ---------------------------------------------------------------------------------------
constexpr int kBwdPix = 4;  // pixels per lane; one wave covers the 16x16 tile

__global__ __launch_bounds__(64) void backward_kernel(
    uint32_t w, uint32_t h, uint32_t tiles_x, const float4* __restrict__ rec_a,
    const float4* __restrict__ rec_b, const float* __restrict__ rec_c,
    const uint32_t* __restrict__ s_gid, const uint32_t* __restrict__ s_slot,
    const uint2* __restrict__ ranges, const uint32_t* __restrict__ last_idx,
    const float* __restrict__ t_final, const uint32_t* __restrict__ rendered,
    const uint32_t* __restrict__ gt, float* __restrict__ partial) {
    __shared__ float4 la[64];
    __shared__ float4 lb[64];
    __shared__ float lc[64];
    __shared__ uint32_t lslot[64];
    __shared__ float lpart[64][9];

    const uint32_t tile = blockIdx.x;
    const uint32_t lane = threadIdx.x;
    const uint32_t tx = tile % tiles_x, ty = tile / tiles_x;
    const uint2 range = ranges[tile];

    float pxv[kBwdPix], pyv[kBwdPix], T[kBwdPix], acc[kBwdPix][3], dl[kBwdPix][3];
    uint32_t last[kBwdPix];
    bool act[kBwdPix];
    uint32_t my_end = 0;
#pragma unroll
    for (int k = 0; k < kBwdPix; k++) {
        const uint32_t x = tx * kTile + (lane & 15u);
        const uint32_t y = ty * kTile + (lane >> 4) + 4u * (uint32_t)k;
        pxv[k] = (float)x + 0.5f;
        pyv[k] = (float)y + 0.5f;
        act[k] = false;
        last[k] = 0;
        T[k] = 1.0f;
        acc[k][0] = acc[k][1] = acc[k][2] = 1.0f;
        dl[k][0] = dl[k][1] = dl[k][2] = 0.0f;
        if (x < w && y < h) {
            const uint32_t pix = y * w + x;
            const uint32_t li = last_idx[pix];
            if (li != 0xffffffffu) {
                act[k] = true;
                last[k] = li;
                T[k] = t_final[pix];
                const uint32_t rr = rendered[pix], gg = gt[pix];
#pragma unroll
                for (int c = 0; c < 3; c++) {
                    const float r = (float)((rr >> (8 * c)) & 0xffu) / 255.0f;
                    const float t = (float)((gg >> (8 * c)) & 0xffu) / 255.0f;
                    const float d = r - t;
                    dl[k][c] = (d > 0.0f ? 1.0f : (d < 0.0f ? -1.0f : 0.0f)) / 3.0f;
                }
                my_end = max(my_end, li + 1u);
            }
        }
    }
    uint32_t end_max = wave_max_u32(my_end);
    if (end_max < range.x) end_max = range.x;

    // slots of this tile that no pixel reaches: zero partials
    for (uint32_t s = end_max + lane; s < range.y; s += 64u) {
        float* dst = partial + (size_t)s_slot[s] * 9u;
#pragma unroll
        for (int q = 0; q < 9; q++) dst[q] = 0.0f;
    }

    for (uint32_t hi = end_max; hi > range.x;) {
        const uint32_t lo = hi - range.x > 64u ? hi - 64u : range.x;
        const uint32_t cnt = hi - lo;
        if (lane < cnt) {
            const uint32_t s = lo + lane;
            const uint32_t gidx = s_gid[s];
            la[lane] = rec_a[gidx];
            lb[lane] = rec_b[gidx];
            lc[lane] = rec_c[gidx];
            lslot[lane] = s_slot[s];
        }
        __syncthreads();
        for (int j = (int)cnt - 1; j >= 0; j--) {
            const uint32_t s = lo + (uint32_t)j;
            const float4 A = la[j];
            const float4 B = lb[j];
            const float col[3] = {B.z, B.w, lc[j]};
            float p9[9];
#pragma unroll
            for (int q = 0; q < 9; q++) p9[q] = 0.0f;
            bool any = false;
#pragma unroll
            for (int k = 0; k < kBwdPix; k++) {
                if (!act[k] || s > last[k]) continue;
                const float dx = pxv[k] - A.x, dy = pyv[k] - A.y;
                const float power = -0.5f * (A.z * dx * dx + 2.0f * A.w * dx * dy + B.x * dy * dy);
                if (power > 0.0f || power < -4.5f) continue;
                const float G = gs_expf(power);
                const float alpha = fminf(B.y * G, 0.99f);
                if (alpha < 1.0f / 255.0f) continue;
                T[k] = T[k] / fmaxf(1.0f - alpha, 0.0001f);
                const float weight = alpha * T[k];
                float dd = dl[k][0] * (col[0] - acc[k][0]);
                dd = dd + dl[k][1] * (col[1] - acc[k][1]);
                dd = dd + dl[k][2] * (col[2] - acc[k][2]);
                const float dL_dAlpha = T[k] * dd;
#pragma unroll
                for (int c = 0; c < 3; c++) acc[k][c] = alpha * col[c] + (1.0f - alpha) * acc[k][c];
                const float wg = dL_dAlpha * G;
                p9[0] += dl[k][0] * weight;
                p9[1] += dl[k][1] * weight;
                p9[2] += dl[k][2] * weight;
                p9[3] += wg;
                p9[4] += wg * dx;
                p9[5] += wg * dy;
                p9[6] += wg * dx * dx;
                p9[7] += wg * dx * dy;
                p9[8] += wg * dy * dy;
                any = true;
            }
            if (__ballot(any)) {
#pragma unroll
                for (int q = 0; q < 9; q++) p9[q] = wave_sum(p9[q]);
            }
            if (lane == 0) {
#pragma unroll
                for (int q = 0; q < 9; q++) lpart[j][q] = p9[q];
            }
        }
        __syncthreads();
        if (lane < cnt) {
            float* dst = partial + (size_t)lslot[lane] * 9u;
#pragma unroll
            for (int q = 0; q < 9; q++) dst[q] = lpart[lane][q];
        }
        __syncthreads();
        hi = lo;
    }
}

// ---------------------------------------------------------------------------------------
__global__ void debug_pairs_kernel(const uint32_t* __restrict__ s_tile,
                                   const uint32_t* __restrict__ s_gid,
                                   const uint32_t* __restrict__ dkey,
                                   const uint32_t* __restrict__ p_dev, uint64_t cap,
                                   uint64_t* __restrict__ keys, uint32_t* __restrict__ values) {
    const uint64_t P = *p_dev;
    for (uint64_t s = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; s < P && s < cap;
         s += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t gi = s_gid[s];
        if (keys) keys[s] = ((uint64_t)s_tile[s] << 32) | dkey[gi];
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
    hipLaunchKernelGGL(project_kernel, dim3(div_up(n, 256)), dim3(256), 0, st, g, n, u, gb.rec_a,
                       gb.rec_b, gb.rec_c, gb.count, gb.dkey, gb.rect, debug_out);
    return hipGetLastError();
}

hipError_t launch_emit(hipStream_t st, uint32_t n, const GaussianBuffers& gb,
                       const uint32_t* dsorted, const PairBuffers& pb, uint32_t tiles_x,
                       uint32_t* overflow) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(emit_kernel, dim3(div_up(n, 256)), dim3(256), 0, st, n, dsorted, gb.count,
                       gb.rect, gb.offset, tiles_x, pb.tile0, pb.gid0, pb.cap, overflow);
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

hipError_t launch_forward(hipStream_t st, const LaunchGeom& geo, const GsTiledUniforms& u,
                          const GaussianBuffers& gb, const PairBuffers& pb, const uint2* ranges,
                          const uint32_t* p_dev, const PixelBuffers& px, uint32_t* rgba8,
                          float* rgb) {
    (void)u;
    hipLaunchKernelGGL(forward_kernel, dim3(geo.num_tiles), dim3(kFwdThreads), 0, st, geo.w,
                       geo.h, geo.tiles_x, gb.rec_a, gb.rec_b, gb.rec_c, pb.s_gid, ranges, p_dev,
                       px.last_idx, px.t_final, rgba8, rgb);
    return hipGetLastError();
}

hipError_t launch_backward(hipStream_t st, const LaunchGeom& geo, const GsTiledUniforms& u,
                           const GaussianBuffers& gb, const PairBuffers& pb,
                           const uint2* ranges, const PixelBuffers& px, const uint32_t* rendered,
                           const uint32_t* gt) {
    (void)u;
    hipLaunchKernelGGL(backward_kernel, dim3(geo.num_tiles), dim3(64), 0, st, geo.w, geo.h,
                       geo.tiles_x, gb.rec_a, gb.rec_b, gb.rec_c, pb.s_gid, pb.s_slot, ranges,
                       px.last_idx, px.t_final, rendered, gt, pb.partial);
    return hipGetLastError();
}

hipError_t launch_debug_pairs(hipStream_t st, const PairBuffers& pb, const GaussianBuffers& gb,
                              const uint32_t* p_dev, uint64_t cap, uint64_t* keys,
                              uint32_t* values) {
    hipLaunchKernelGGL(debug_pairs_kernel, dim3(1024), dim3(256), 0, st, pb.s_tile, pb.s_gid,
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
