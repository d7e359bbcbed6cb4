// gs_segsort.hip — per-tile depth sort of the tile lists (the one-pass path's replacement for the
// global depth sort of the N Gaussians).
//
// The reference orders the (tile, Gaussian) pairs by the 64-bit key (tile << 32 | depthKey) and,
// among equal keys, by its sort's input order (tiled_rasterizer.mm:27-102, 498-512); the values
// compared in parity are ordered (tile, depthKey, Gaussian index). Here the pairs are emitted in
// Gaussian order (at the Gaussian-order slot offsets goff), the stable one-pass counting sort by tile
// (gs_sort.hip) leaves every tile's list in Gaussian order, and this kernel sorts each list by the
// depth key of its Gaussian, stably: the result is (tile, depthKey, gid), bit-exact with the global
// depth sort it replaces (4 look-back passes over the N keys, 77 us at the bench workload).
//
// One 256-thread workgroup per tile, in the blend's launch order (longest lists first). A tile's
// keys differ only below the highest bit where its smallest and largest key differ, so LSD passes
// of 8-bit digits run over those bits only (3-4 passes for a scene's depth range). A pass ranks the
// keys held in registers with wave ballots (stable: memory order, as the other scatters) and
// per-wave digit counters in LDS.
//   n <= kSegCap (2048): the whole list lives in registers, each pass scatters into LDS;
//   n >  kSegCap       : chunks of kSegCap, a digit histogram sweep then a rank-and-scatter sweep
//                        per pass, ping-ponging through the pair buffers the tile sort has finished
//                        with (L2-resident), the last pass copied back into the list.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "gs_device.hpp"
#include "gs_internal.hpp"

namespace gs {

constexpr uint32_t kSegThreads = 256;
constexpr uint32_t kSegWaves = kSegThreads / 64;
constexpr uint32_t kSegItems = 8;                        // rows of 64 per wave
constexpr uint32_t kSegCap = kSegThreads * kSegItems;   // 2048 pairs per register-resident chunk

__device__ __forceinline__ void seg_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// exclusive scan of one value per thread over the 256 threads; ws: 4 LDS words
__device__ __forceinline__ uint32_t seg_scan256(uint32_t v, uint32_t t, uint32_t* ws) {
    const uint32_t lane = t & 63u, w = t >> 6;
    uint32_t inc = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(inc, o, 64);
        if (lane >= (uint32_t)o) inc += y;
    }
    if (lane == 63u) ws[w] = inc;
    seg_barrier();
    uint32_t base = 0;
#pragma unroll
    for (uint32_t k = 0; k < kSegWaves; k++) base += k < w ? ws[k] : 0u;
    seg_barrier();
    return base + inc - v;
}

struct SegShared {
    uint32_t key[kSegCap];
    uint32_t val[kSegCap];
    uint32_t cnt[kSegWaves][256];  // per-wave digit counters, then their exclusive prefixes
    uint32_t loc[256];             // digit start inside the chunk (register path) / the tile (chunked path)
    uint32_t run[256];             // chunked path: the digit's pairs in earlier chunks
    uint32_t ws[kSegWaves];
    uint32_t red[2][kSegWaves];
};

// Ranks the wave's R rows (row i = elements [64 (w R + i), +64) of the chunk) by digit, in memory
// order: rk[i] = this element's position among the wave's earlier elements of its digit. Updates
// S.cnt[w][digit] to the wave's per-digit counts. R is wave-uniform.
__device__ __forceinline__ void seg_rank(SegShared& S, uint32_t w, uint32_t lane, uint32_t R, const bool (&ok)[kSegItems],
                                         const uint32_t (&dg)[kSegItems], uint32_t nb, uint32_t (&rk)[kSegItems]) {
    const uint64_t lt = lanemask_lt();
#pragma unroll
    for (uint32_t i = 0; i < kSegItems; i++) {
        if (i >= R) break;
        uint64_t m = __ballot(ok[i]);
        for (uint32_t bit = 0; bit < nb; bit++) {
            const bool on = (dg[i] >> bit) & 1u;
            const uint64_t bb = __ballot(on);
            m &= on ? bb : ~bb;
        }
        const uint32_t below = (uint32_t)__popcll(m & lt);
        uint32_t c = 0;
        if (ok[i]) c = S.cnt[w][dg[i]];
        __builtin_amdgcn_wave_barrier();
        rk[i] = c + below;
        const uint32_t leader = 63u - (uint32_t)__clzll(m);
        if (ok[i] && lane == leader) S.cnt[w][dg[i]] = c + (uint32_t)__popcll(m);
        __builtin_amdgcn_wave_barrier();
    }
}

// After seg_rank by every wave: S.cnt[w][d] <- the count of digit d in the waves before w; returns
// thread t's digit total over the waves (t = digit).
__device__ __forceinline__ uint32_t seg_wave_prefix(SegShared& S, uint32_t t) {
    uint32_t tot = 0;
#pragma unroll
    for (uint32_t ww = 0; ww < kSegWaves; ww++) {
        const uint32_t c = S.cnt[ww][t];
        S.cnt[ww][t] = tot;
        tot += c;
    }
    return tot;
}

__global__ __launch_bounds__(kSegThreads) void tile_depth_sort_kernel(
    const uint2* __restrict__ ranges, const uint32_t* __restrict__ order, uint32_t T,
    const uint32_t* __restrict__ dkey, uint32_t* __restrict__ s_val, uint32_t* __restrict__ ka,
    uint32_t* __restrict__ va, uint32_t* __restrict__ kb, uint32_t* __restrict__ vb) {
    __shared__ SegShared S;
    const uint32_t t = threadIdx.x, w = t >> 6, lane = t & 63u;
    const uint32_t tile = order ? order[blockIdx.x] : blockIdx.x;
    if (tile >= T) return;
    const uint2 r = ranges[tile];
    const uint32_t n = r.y - r.x;
    if (n <= 1u) return;
    const uint32_t nchunks = (n + kSegCap - 1u) / kSegCap;
    uint32_t* const list = s_val + r.x;

    // the chunk's rows: wave w owns rows [w R, w R + R) of the chunk (memory order = wave order)
    auto chunk_rows = [&](uint32_t c) {
        const uint32_t cn = min(kSegCap, n - c * kSegCap);
        const uint32_t nrows = (cn + 63u) >> 6;
        return (nrows + kSegWaves - 1u) / kSegWaves;
    };
    uint32_t k[kSegItems], v[kSegItems], dg[kSegItems], rk[kSegItems];
    bool ok[kSegItems];
    // src 0: the list itself, keys gathered from the Gaussians' depth keys; 1: (ka, va); 2: (kb, vb)
    auto load_chunk = [&](uint32_t c, uint32_t R, uint32_t src) {
        const uint32_t c0 = c * kSegCap;
#pragma unroll
        for (uint32_t i = 0; i < kSegItems; i++) {
            const uint32_t e = c0 + (w * R + i) * 64u + lane;
            ok[i] = i < R && e < n;
            const uint32_t ee = ok[i] ? e : 0u;
            v[i] = src == 0u ? list[ee] : (src == 1u ? va[r.x + ee] : vb[r.x + ee]);
            if (src == 1u) k[i] = ka[r.x + ee];
            if (src == 2u) k[i] = kb[r.x + ee];
        }
        if (src == 0u) {
#pragma unroll
            for (uint32_t i = 0; i < kSegItems; i++) k[i] = dkey[v[i] >> kPairJBits];
        }
    };

    // the bits the tile's keys differ in: [0, hb)
    uint32_t kmin = 0xffffffffu, kmax = 0u;
    for (uint32_t c = 0; c < nchunks; c++) {
        const uint32_t R = chunk_rows(c);
        load_chunk(c, R, 0u);
#pragma unroll
        for (uint32_t i = 0; i < kSegItems; i++)
            if (ok[i]) {
                kmin = min(kmin, k[i]);
                kmax = max(kmax, k[i]);
            }
    }
    kmin = wave_min_u32(kmin);
    kmax = wave_max_u32(kmax);
    if (lane == 0) {
        S.red[0][w] = kmin;
        S.red[1][w] = kmax;
    }
    seg_barrier();
#pragma unroll
    for (uint32_t q = 0; q < kSegWaves; q++) {
        kmin = min(kmin, S.red[0][q]);
        kmax = max(kmax, S.red[1][q]);
    }
    const uint32_t hb = (kmin ^ kmax) ? 32u - (uint32_t)__clz(kmin ^ kmax) : 0u;
    if (hb == 0u) return;  // one key: the list is already in Gaussian order
    const uint32_t npass = (hb + 7u) >> 3;

    if (nchunks == 1u) {
        // ---- register-resident list, LDS scatter per pass (chunk 0 is still loaded) ----
        const uint32_t R = chunk_rows(0);
        for (uint32_t p = 0; p < npass; p++) {
            const uint32_t shift = 8u * p, nb = min(8u, hb - shift);
#pragma unroll
            for (uint32_t q = 0; q < kSegWaves; q++) S.cnt[q][t] = 0u;
            seg_barrier();
#pragma unroll
            for (uint32_t i = 0; i < kSegItems; i++) dg[i] = (k[i] >> shift) & ((1u << nb) - 1u);
            seg_rank(S, w, lane, R, ok, dg, nb, rk);
            seg_barrier();
            const uint32_t tot = seg_wave_prefix(S, t);
            S.loc[t] = seg_scan256(tot, t, S.ws);
            seg_barrier();
#pragma unroll
            for (uint32_t i = 0; i < kSegItems; i++)
                if (ok[i]) {
                    const uint32_t pos = S.loc[dg[i]] + S.cnt[w][dg[i]] + rk[i];
                    S.key[pos] = k[i];
                    S.val[pos] = v[i];
                }
            seg_barrier();
#pragma unroll
            for (uint32_t i = 0; i < kSegItems; i++)
                if (ok[i]) {
                    const uint32_t e = (w * R + i) * 64u + lane;
                    k[i] = S.key[e];
                    v[i] = S.val[e];
                }
            seg_barrier();
        }
#pragma unroll
        for (uint32_t i = 0; i < kSegItems; i++)
            if (ok[i]) list[(w * R + i) * 64u + lane] = v[i];
        return;
    }

    // ---- chunked: per pass a histogram sweep, then rank + scatter chunk by chunk ----
    uint32_t src = 0u;
    for (uint32_t p = 0; p < npass; p++) {
        const uint32_t shift = 8u * p, nb = min(8u, hb - shift);
        const uint32_t dst = p & 1u ? 2u : 1u;
        uint32_t* const kd = (dst == 1u ? ka : kb) + r.x;
        uint32_t* const vd = (dst == 1u ? va : vb) + r.x;
        // digit histogram of the whole list (S.cnt[w] as per-wave histograms)
#pragma unroll
        for (uint32_t q = 0; q < kSegWaves; q++) S.cnt[q][t] = 0u;
        S.run[t] = 0u;
        seg_barrier();
        for (uint32_t c = 0; c < nchunks; c++) {
            load_chunk(c, chunk_rows(c), src);
#pragma unroll
            for (uint32_t i = 0; i < kSegItems; i++)
                if (ok[i]) atomicAdd(&S.cnt[w][(k[i] >> shift) & ((1u << nb) - 1u)], 1u);
        }
        seg_barrier();
        uint32_t tot = 0;
#pragma unroll
        for (uint32_t q = 0; q < kSegWaves; q++) tot += S.cnt[q][t];
        S.loc[t] = seg_scan256(tot, t, S.ws);  // digit starts over the whole list
        for (uint32_t c = 0; c < nchunks; c++) {
            const uint32_t R = chunk_rows(c);
            load_chunk(c, R, src);
#pragma unroll
            for (uint32_t q = 0; q < kSegWaves; q++) S.cnt[q][t] = 0u;
            seg_barrier();
#pragma unroll
            for (uint32_t i = 0; i < kSegItems; i++) dg[i] = (k[i] >> shift) & ((1u << nb) - 1u);
            seg_rank(S, w, lane, R, ok, dg, nb, rk);
            seg_barrier();
            const uint32_t ctot = seg_wave_prefix(S, t);
            seg_barrier();
#pragma unroll
            for (uint32_t i = 0; i < kSegItems; i++)
                if (ok[i]) {
                    const uint32_t pos = S.loc[dg[i]] + S.run[dg[i]] + S.cnt[w][dg[i]] + rk[i];
                    kd[pos] = k[i];
                    vd[pos] = v[i];
                }
            seg_barrier();
            S.run[t] += ctot;  // (thread t owns digit t)
        }
        // this pass's stores are read back by other waves of the workgroup in the next pass
        __syncthreads();
        src = dst;
    }
    // the sorted values back into the list
    const uint32_t* const vs = (src == 1u ? va : vb) + r.x;
    for (uint32_t e = t; e < n; e += kSegThreads) list[e] = vs[e];
}

hipError_t launch_tile_depth_sort(hipStream_t st, const uint2* ranges, const uint32_t* order, uint32_t T,
                                  const uint32_t* dkey, uint32_t* s_val, uint32_t* ka, uint32_t* va, uint32_t* kb,
                                  uint32_t* vb) {
    if (T == 0) return hipSuccess;
    hipLaunchKernelGGL(tile_depth_sort_kernel, dim3(T), dim3(kSegThreads), 0, st, ranges, order, T, dkey, s_val, ka,
                       va, kb, vb);
    return hipGetLastError();
}

}  // namespace gs
