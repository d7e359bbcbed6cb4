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
// A tile's keys differ only below the highest bit where its smallest and largest key differ, so
// LSD passes of 8-bit digits run over those bits only (3-4 passes for a scene's depth range: 25 bits
// on every tile of the bench frame). A pass ranks the keys held in registers with wave ballots (stable:
// memory order, as the other scatters) and digit counters in LDS, then scatters into LDS.
//   n <= kWaveCap (1024: every list of the bench frame, whose longest is 846): ONE wave per tile,
//        up to 16 rows of 64 in registers, no workgroup barrier at all (tile_depth_sort_wave_kernel;
//        four independent waves per workgroup, the tiles in the blend's launch order). The
//        workgroup-per-tile form of the same passes took 82 us at the bench workload: each of its
//        ~24 barriers per tile waited on the one wave that held most rows;
//   n >  kWaveCap: the wave appends the tile to a list that tile_depth_sort_kernel (256 threads per
//        tile, launched next) works through: n <= kSegCap (2048) in registers with an LDS scatter;
//        above, chunks of kSegCap, a digit histogram sweep then a rank-and-scatter sweep per pass,
//        ping-ponging through the pair buffers the tile sort has finished with (L2-resident), the last
//        pass copied back into the list.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "gs_device.hpp"
#include "gs_internal.hpp"

#include <algorithm>

namespace gs {

#ifndef GS_SEG_THREADS
#define GS_SEG_THREADS 256
#endif
#ifndef GS_SEG_ITEMS
#define GS_SEG_ITEMS 8
#endif
constexpr uint32_t kSegThreads = GS_SEG_THREADS;
constexpr uint32_t kSegWaves = kSegThreads / 64;
constexpr uint32_t kSegItems = GS_SEG_ITEMS;             // rows of 64 per wave
constexpr uint32_t kSegCap = kSegThreads * kSegItems;   // 2048 pairs per register-resident chunk

__device__ __forceinline__ void seg_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// exclusive scan of one value per thread over the block (digit t for t < 256, 0 above); ws: a word per wave
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

__device__ void tile_depth_sort_block(SegShared& S, uint32_t tile, const uint2* __restrict__ ranges,
                                      const uint32_t* __restrict__ dkey, uint32_t* __restrict__ s_val,
                                      uint32_t* __restrict__ ka, uint32_t* __restrict__ va, uint32_t* __restrict__ kb,
                                      uint32_t* __restrict__ vb) {
    const uint32_t t = threadIdx.x, w = t >> 6, lane = t & 63u;
    const uint2 r = ranges[tile];
    const uint32_t n = r.y - r.x;
    if (n <= 1u) return;
    const uint32_t nchunks = (n + kSegCap - 1u) / kSegCap;
#ifdef GS_SEG_SKIP_CHUNKED  // diagnostics only (wrong results): the register path's cost alone
    if (nchunks > 1u) return;
#endif
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
            if (t < 256u)
#pragma unroll
                for (uint32_t q = 0; q < kSegWaves; q++) S.cnt[q][t] = 0u;
            seg_barrier();
#pragma unroll
            for (uint32_t i = 0; i < kSegItems; i++) dg[i] = (k[i] >> shift) & ((1u << nb) - 1u);
            seg_rank(S, w, lane, R, ok, dg, nb, rk);
            seg_barrier();
            const uint32_t tot = t < 256u ? seg_wave_prefix(S, t) : 0u;
            const uint32_t loc = seg_scan256(tot, t, S.ws);
            if (t < 256u) S.loc[t] = loc;
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
        if (t < 256u) {
#pragma unroll
            for (uint32_t q = 0; q < kSegWaves; q++) S.cnt[q][t] = 0u;
            S.run[t] = 0u;
        }
        seg_barrier();
        for (uint32_t c = 0; c < nchunks; c++) {
            load_chunk(c, chunk_rows(c), src);
#pragma unroll
            for (uint32_t i = 0; i < kSegItems; i++)
                if (ok[i]) atomicAdd(&S.cnt[w][(k[i] >> shift) & ((1u << nb) - 1u)], 1u);
        }
        seg_barrier();
        uint32_t tot = 0;
        if (t < 256u)
#pragma unroll
            for (uint32_t q = 0; q < kSegWaves; q++) tot += S.cnt[q][t];
        const uint32_t loc = seg_scan256(tot, t, S.ws);  // digit starts over the whole list
        if (t < 256u) S.loc[t] = loc;
        for (uint32_t c = 0; c < nchunks; c++) {
            const uint32_t R = chunk_rows(c);
            load_chunk(c, R, src);
            if (t < 256u)
#pragma unroll
                for (uint32_t q = 0; q < kSegWaves; q++) S.cnt[q][t] = 0u;
            seg_barrier();
#pragma unroll
            for (uint32_t i = 0; i < kSegItems; i++) dg[i] = (k[i] >> shift) & ((1u << nb) - 1u);
            seg_rank(S, w, lane, R, ok, dg, nb, rk);
            seg_barrier();
            const uint32_t ctot = t < 256u ? seg_wave_prefix(S, t) : 0u;
            seg_barrier();
#pragma unroll
            for (uint32_t i = 0; i < kSegItems; i++)
                if (ok[i]) {
                    const uint32_t pos = S.loc[dg[i]] + S.run[dg[i]] + S.cnt[w][dg[i]] + rk[i];
                    kd[pos] = k[i];
                    vd[pos] = v[i];
                }
            seg_barrier();
            if (t < 256u) S.run[t] += ctot;  // (thread t owns digit t)
        }
        // this pass's stores are read back by other waves of the workgroup in the next pass
        __syncthreads();
        src = dst;
    }
    // the sorted values back into the list
    const uint32_t* const vs = (src == 1u ? va : vb) + r.x;
    for (uint32_t e = t; e < n; e += kSegThreads) list[e] = vs[e];
}

// the lists one wave could not take (n > kWaveCap), one workgroup each, grid-stride over the list
__global__ __launch_bounds__(kSegThreads) void tile_depth_sort_kernel(
    const uint2* __restrict__ ranges, const uint32_t* __restrict__ big_list, const uint32_t* __restrict__ big_count,
    const uint32_t* __restrict__ dkey, uint32_t* __restrict__ s_val, uint32_t* __restrict__ ka,
    uint32_t* __restrict__ va, uint32_t* __restrict__ kb, uint32_t* __restrict__ vb) {
    __shared__ SegShared S;
    const uint32_t nbig = *big_count;
    for (uint32_t b = blockIdx.x; b < nbig; b += gridDim.x) {
        tile_depth_sort_block(S, big_list[b], ranges, dkey, s_val, ka, va, kb, vb);
        __syncthreads();  // S is reused by the next list
    }
}

// ---- one wave per tile ----------------------------------------------------------------------
// Between passes a list entry travels as one word: its key bits not yet sorted on, above its index in
// the list (10 bits): 4 B of LDS per entry instead of key + value, so twice the waves fit a CU. After
// the last pass the sorted indices pick the list's values (staged once in the same LDS words).
// Lists whose keys differ in more than 30 bits do not fit the word (22 key bits after the first
// pass) and go to the workgroup kernel with the long lists.
constexpr uint32_t kWaveRows = 16;
constexpr uint32_t kWaveCap = 64u * kWaveRows;  // 1024
constexpr uint32_t kWaveIdxBits = 10;
constexpr uint32_t kWaveWaves = 4;              // independent waves per workgroup
struct WaveShared {
    uint32_t word[kWaveCap];
    uint32_t cnt[256];
};

__global__ __launch_bounds__(64 * kWaveWaves) void tile_depth_sort_wave_kernel(
    const uint2* __restrict__ ranges, const uint32_t* __restrict__ order, uint32_t T,
    const uint32_t* __restrict__ dkey, const uint2* __restrict__ kv, uint32_t* __restrict__ s_val,
    uint32_t* __restrict__ big_list, uint32_t* __restrict__ big_count) {
    __shared__ WaveShared SW[kWaveWaves];
    const uint32_t w = threadIdx.x >> 6, lane = threadIdx.x & 63u;
    const uint32_t pos = blockIdx.x * kWaveWaves + w;
    if (pos >= T) return;
    const uint32_t tile = __builtin_amdgcn_readfirstlane(order ? order[pos] : pos);
    const uint2 r = ranges[tile];
    const uint32_t n = __builtin_amdgcn_readfirstlane(r.y - r.x);
    uint32_t* const list = s_val + r.x;
    // with kv the list exists only as the tile sort's (value, key) pairs: every entry must be written
    // here, whatever happens to the list below
    const bool from_kv = kv != nullptr;
    const uint2* const kvl = kv + r.x;
    if (n == 0u) return;
    if (n == 1u || n > kWaveCap) {
        if (from_kv)
            for (uint32_t e = lane; e < n; e += 64u) list[e] = kvl[e].x;
        if (n > kWaveCap && lane == 0) big_list[atomicAdd(big_count, 1u)] = tile;
        return;
    }
    WaveShared& L = SW[w];
    const uint32_t R = (n + 63u) >> 6;  // rows, wave-uniform
    // q: the entry's key (first pass), then (unsorted key bits << kWaveIdxBits) | list index
    uint32_t q[kWaveRows], rk[kWaveRows];
    if (from_kv) {  // the keys came with the pairs (one-pass tile sort): coalesced, no gather
#pragma unroll
        for (uint32_t i = 0; i < kWaveRows; i++) {
            const uint32_t e = i * 64u + lane;
            q[i] = (i < R && e < n) ? kvl[e].y : kvl[0].y;
        }
    } else {
#pragma unroll
        for (uint32_t i = 0; i < kWaveRows; i++) {
            const uint32_t e = i * 64u + lane;
            q[i] = (i < R && e < n) ? list[e] : list[0];
        }
#pragma unroll
        for (uint32_t i = 0; i < kWaveRows; i++) q[i] = i < R ? dkey[q[i] >> kPairJBits] : 0u;
    }
    uint32_t kmin = 0xffffffffu, kmax = 0u;
#pragma unroll
    for (uint32_t i = 0; i < kWaveRows; i++) {
        if (i < R && i * 64u + lane < n) {
            kmin = min(kmin, q[i]);
            kmax = max(kmax, q[i]);
        }
    }
    // (wave-uniform values in scalar registers: the pass and bit loops below are then scalar loops,
    // and the row loops unroll with fixed registers)
    kmin = (uint32_t)__builtin_amdgcn_readfirstlane((int)wave_min_u32(kmin));
    kmax = (uint32_t)__builtin_amdgcn_readfirstlane((int)wave_max_u32(kmax));
    // sorted on key - kmin (same order): its bits [0, hb) are all that vary (25-26 bits for depths
    // spanning a factor of 100)
    const uint32_t hb = kmax != kmin ? 32u - (uint32_t)__clz(kmax - kmin) : 0u;
    if (hb == 0u || hb > 32u - kWaveIdxBits + 8u) {
        // one key: the list is already in order; or the key bits left after the first pass do not
        // fit a word: the workgroup kernel sorts the list in place
        if (from_kv)
            for (uint32_t e = lane; e < n; e += 64u) list[e] = kvl[e].x;
        if (hb != 0u && lane == 0) big_list[atomicAdd(big_count, 1u)] = tile;
        return;
    }
#pragma unroll
    for (uint32_t i = 0; i < kWaveRows; i++) q[i] -= kmin;
    const uint64_t lt = lanemask_lt();
    // passes of 8-bit digits over [0, hb) (the bits of key - kmin above hb are zero: a short last
    // digit costs nothing extra, and fixed-width digits keep the loops free of bit-count branches)
    for (uint32_t shift = 0; shift < hb; shift += 8u) {
        // the digit: the key's low byte on the first pass, then the word's lowest unsorted key bits
        const uint32_t dsh = shift == 0u ? 0u : kWaveIdxBits;
#pragma unroll
        for (uint32_t c = 0; c < 4u; c++) L.cnt[4u * lane + c] = 0u;
        __builtin_amdgcn_wave_barrier();
        // rank the rows in memory order, four at a time: ballot match over the 8 digit bits; the
        // group leader adds the group's size to its digit's counter with a returning LDS atomic (the
        // rows' atomics go out back to back, applied in order), and its group reads the old count
        // from the leader's lane
#pragma unroll
        for (uint32_t i0 = 0; i0 < kWaveRows; i0 += 4u) {
            if (i0 < R) {
                uint64_t m[4];
                uint32_t old[4], ldr[4];
#pragma unroll
                for (uint32_t k = 0; k < 4u; k++) {
                    const uint32_t i = i0 + k;
                    const bool ok = i < R && i * 64u + lane < n;
                    const uint32_t d = (q[i] >> dsh) & 0xffu;
                    uint64_t mm = __ballot(ok);
#pragma unroll
                    for (uint32_t bit = 0; bit < 8u; bit++) {
                        const bool on = (d >> bit) & 1u;
                        const uint64_t bb = __ballot(on);
                        mm &= on ? bb : ~bb;
                    }
                    m[k] = mm;
                    ldr[k] = 63u - (uint32_t)__clzll(mm);
                    const uint32_t add = (ok && lane == ldr[k]) ? (uint32_t)__popcll(mm) : 0u;
                    old[k] = __hip_atomic_fetch_add(&L.cnt[d], add, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                }
#pragma unroll
                for (uint32_t k = 0; k < 4u; k++) {
                    const uint32_t lold = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(ldr[k] << 2), (int)old[k]);
                    rk[i0 + k] = lold + (uint32_t)__popcll(m[k] & lt);
                }
            }
        }
        __builtin_amdgcn_wave_barrier();
        // digit starts: exclusive scan of the 256 counts, four per lane
        uint32_t c4[4], s4 = 0;
#pragma unroll
        for (uint32_t c = 0; c < 4u; c++) {
            c4[c] = L.cnt[4u * lane + c];
            s4 += c4[c];
        }
        uint32_t inc = s4;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(inc, o, 64);
            if (lane >= (uint32_t)o) inc += y;
        }
        uint32_t run = inc - s4;
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (uint32_t c = 0; c < 4u; c++) {
            L.cnt[4u * lane + c] = run;
            run += c4[c];
        }
        __builtin_amdgcn_wave_barrier();
        // scatter the words with this digit's bits dropped (the list index kept below them)
#pragma unroll
        for (uint32_t i = 0; i < kWaveRows; i++) {
            if (i < R) {
                const uint32_t e = i * 64u + lane;
                if (e < n) {
                    const uint32_t p = L.cnt[(q[i] >> dsh) & 0xffu] + rk[i];
                    const uint32_t idx = shift == 0u ? e : (q[i] & ((1u << kWaveIdxBits) - 1u));
                    const uint32_t rest = shift == 0u ? q[i] >> 8 : q[i] >> (kWaveIdxBits + 8u);
                    L.word[p] = (rest << kWaveIdxBits) | idx;
                }
            }
        }
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (uint32_t i = 0; i < kWaveRows; i++) {
            if (i < R) {
                const uint32_t e = i * 64u + lane;
                if (e < n) q[i] = L.word[e];
            }
        }
        __builtin_amdgcn_wave_barrier();
    }
    // the values in sorted order: stage the list's values by index, pick them by the sorted indices
    uint32_t v[kWaveRows];
#pragma unroll
    for (uint32_t i = 0; i < kWaveRows; i++) {
        const uint32_t e = i * 64u + lane;
        v[i] = (i < R && e < n) ? (from_kv ? kvl[e].x : list[e]) : 0u;
    }
#pragma unroll
    for (uint32_t i = 0; i < kWaveRows; i++) {
        const uint32_t e = i * 64u + lane;
        if (i < R && e < n) L.word[e] = v[i];
    }
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (uint32_t i = 0; i < kWaveRows; i++) {
        const uint32_t e = i * 64u + lane;
        if (i < R && e < n) v[i] = L.word[q[i] & ((1u << kWaveIdxBits) - 1u)];
    }
#pragma unroll
    for (uint32_t i = 0; i < kWaveRows; i++) {
        const uint32_t e = i * 64u + lane;
        if (i < R && e < n) list[e] = v[i];
    }
}

hipError_t launch_tile_depth_sort(hipStream_t st, const uint2* ranges, const uint32_t* order, uint32_t T,
                                  const uint32_t* dkey, const uint2* kv, uint32_t* s_val, uint32_t* ka,
                                  uint32_t* va, uint32_t* kb, uint32_t* vb, uint32_t* big_list, uint32_t* big_count) {
    if (T == 0) return hipSuccess;
    hipLaunchKernelGGL(tile_depth_sort_wave_kernel, dim3((T + kWaveWaves - 1) / kWaveWaves), dim3(64 * kWaveWaves), 0,
                       st, ranges, order, T, dkey, kv, s_val, big_list, big_count);
    // the long lists: a workgroup each (the count is on the device; surplus blocks exit at once)
    hipLaunchKernelGGL(tile_depth_sort_kernel, dim3(std::min<uint32_t>(T, 1024u)), dim3(kSegThreads), 0, st, ranges,
                       big_list, big_count, dkey, s_val, ka, va, kb, vb);
    return hipGetLastError();
}

}  // namespace gs
