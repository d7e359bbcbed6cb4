// gs_emit.hpp — device helpers shared by the pair emission (gs_raster.hip) and the one-pass tile sort's
// Gaussian-order kernels (gs_sort.hip): the walk over a wave's pairs in Gaussian order and the
// once-per-frame duties of whichever kernel emits the frame's pairs.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "gs_device.hpp"
#include "gs_internal.hpp"

namespace gs {

// Once per frame, in two parts that may run in different kernels (block 0, all its threads):
// frame_reset, before anything of the frame can raise an error bit: report the sweep's scan error
// word to the host and re-zero the sweep head for the next frame's project_kernel; zero the frame's
// fan-in error word; a new partial-slot frame tag. frame_publish, once P is
// known: the overflow flag, and P + flag into mapped host memory. emit_frame_duties does both.
__device__ __forceinline__ void frame_reset(uint32_t t, uint32_t nthreads, uint32_t* __restrict__ overflow,
                                            uint32_t* __restrict__ host_mirror, uint32_t* __restrict__ hist_rezero) {
    if (hist_rezero) {
        if (t == 0 && host_mirror)
            __hip_atomic_store(host_mirror + 2, hist_rezero[kSweepHistWords + kSweepCtrError], __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_SYSTEM);
        __syncthreads();
        for (uint32_t z = t; z < kSweepHeadWords; z += nthreads) hist_rezero[z] = 0u;
    }
    if (t == 0) {
        overflow[kScalarFanInError - 1u] = 0u;  // the frame's fan-in error word (overflow = scalars + 1)
        // a new frame tag for the partial-sum slots; 0 is skipped on wrap (slots are zeroed at
        // allocation, so tag 0 must never be current)
        const uint32_t ntag = overflow[kScalarFrameTag - 1u] + 1u;
        overflow[kScalarFrameTag - 1u] = ntag ? ntag : 1u;
    }
}

__device__ __forceinline__ void frame_publish(uint32_t t, uint32_t P, uint64_t cap, uint32_t* __restrict__ overflow,
                                              uint32_t* __restrict__ host_mirror) {
    if (t == 0) {
        // the frame's overflow flag (no memset launch) and P + flag into host memory for the host's
        // next-frame decisions (no copy launch; the host reads them only after a sync, or stale)
        const uint32_t of = (uint64_t)P > cap ? 1u : 0u;
        *overflow = of;
        if (host_mirror) {
            __hip_atomic_store(host_mirror, P, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            __hip_atomic_store(host_mirror + 1, of, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
}

__device__ __forceinline__ void emit_frame_duties(uint32_t t, uint32_t nthreads, uint32_t P, uint64_t cap,
                                                  uint32_t* __restrict__ overflow, uint32_t* __restrict__ host_mirror,
                                                  uint32_t* __restrict__ hist_rezero) {
    frame_reset(t, nthreads, overflow, host_mirror, hist_rezero);
    frame_publish(t, P, cap, overflow, host_mirror);
}

// The pairs of the 64 Gaussians [first, first + 64) in Gaussian order (one wave; lane l holds Gaussian
// first + l with its tile count c and slot offset o, non-decreasing over the lanes, any base): their
// slots [o of lane 0, max(o + c)) are walked 64 at a time, one slot per lane; a slot's Gaussian is the
// last of the 64 whose o is at most the slot (a binary search over the lanes' o by cross-lane reads;
// a culled Gaussian shares its successor's o and never wins). f(slot, tile, value) for every slot
// below `stop`; value = gid << kPairJBits | j, j the slot's index inside the Gaussian's rect, whose
// tiles run row-major (tiled_rasterizer.mm:784-793). Wave-uniform control flow: every lane must call.
// (_rect: with the lane's rect already loaded, e.g. prefetched; only read where c > 0)
template <class F>
__device__ __forceinline__ void wave_walk_pairs_rect(uint32_t first, uint32_t n, uint32_t lane, uint32_t c, uint32_t o,
                                                     uint2 r, uint32_t tiles_x, uint32_t stop, F&& f) {
    const uint32_t i = first + lane;
    uint32_t org = 0, shape = 1u | (65536u << 9);
    if (c) {
        const uint32_t x0 = r.x & 0xffffu, y0 = r.x >> 16, x1 = r.y & 0xffffu;
        const uint32_t rw = x1 - x0 + 1u;
        org = y0 * tiles_x + x0;
        shape = rw | (((65536u + rw - 1u) / rw) << 9);  // width | magic ceil(2^16 / width)
    }
    const uint32_t begin = (uint32_t)__builtin_amdgcn_readfirstlane((int)o);
    const uint32_t end = wave_max_dpp(i < n ? o + c : 0u);
    const uint32_t last = end < stop ? end : stop;
    for (uint32_t s0 = begin; s0 < last; s0 += 64u) {
        const uint32_t s = s0 + lane;
        // largest lane L with o[L] <= s (o is non-decreasing over the lanes)
        uint32_t L = 0;
#pragma unroll
        for (uint32_t step = 32u; step >= 1u; step >>= 1) {
            const uint32_t ol = (uint32_t)__builtin_amdgcn_ds_bpermute((int)((L + step) << 2), (int)o);
            if (ol <= s) L += step;
        }
        const uint32_t oL = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(L << 2), (int)o);
        const uint32_t sh = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(L << 2), (int)shape);
        const uint32_t og = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(L << 2), (int)org);
        if (s < last) {
            const uint32_t j = s - oL;
            const uint32_t rw = sh & 0x1ffu;
            const uint32_t dy = (j * (sh >> 9)) >> 16;  // j / rw, exact for j < 256, rw <= 256
            f(s, og + dy * tiles_x + (j - dy * rw), ((first + L) << kPairJBits) | j);
        }
    }
}

template <class F>
__device__ __forceinline__ void wave_walk_pairs_at(uint32_t first, uint32_t n, uint32_t lane, uint32_t c, uint32_t o,
                                                   const uint2* __restrict__ rect, uint32_t tiles_x, uint32_t stop,
                                                   F&& f) {
    const uint32_t i = first + lane;
    wave_walk_pairs_rect(first, n, lane, c, o, c ? rect[i] : make_uint2(0u, 0u), tiles_x, stop, f);
}

// ... at the Gaussian-order slot offsets goff (past n: never a slot's Gaussian)
template <class F>
__device__ __forceinline__ void wave_walk_pairs(uint32_t first, uint32_t n, uint32_t lane,
                                                const uint32_t* __restrict__ count, const uint32_t* __restrict__ goff,
                                                const uint2* __restrict__ rect, uint32_t tiles_x, uint32_t stop, F&& f) {
    const uint32_t i = first + lane;
    const uint32_t c = i < n ? count[i] : 0u;
    const uint32_t o = i < n ? goff[i] : 0xffffffffu;
    wave_walk_pairs_at(first, n, lane, c, o, rect, tiles_x, stop, f);
}

}  // namespace gs
