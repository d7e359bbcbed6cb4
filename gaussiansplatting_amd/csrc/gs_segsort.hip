// gs_segsort.hip — per-tile depth sort of the tile lists the forward does not sort itself (the
// per-tile order's replacement for the global depth sort of the N Gaussians).
//
// The reference orders the (tile, Gaussian) pairs by the 64-bit key (tile << 32 | depthKey) and,
// among equal keys, by its sort's input order (tiled_rasterizer.mm:27-102, 498-512); the values
// compared in parity are ordered (tile, depthKey, Gaussian index). Here the one-pass counting sort by
// tile (gs_sort.hip) builds every tile's list straight from the Gaussians, in any order inside it
// (tile_hist_rect_kernel + tile_scatter_gid_kernel; on the LSD tile path the lists come in Gaussian
// order from emit_gid_kernel), and every list is sorted by (depth key, Gaussian index): bit-exact with
// the global depth sort it replaces (4 look-back passes over the N keys, 77 us at the bench
// workload), whatever order the list arrived in.
//   n <= kFwdSortMax (1024: every list of the bench frame, whose longest is 861): the forward
//        workgroup sorts its own list in LDS before blending it (fwd_sort_list, gs_blend.hip);
//   longer lists: tile_long_sort_kernel below, one launch before the forward, a 256-thread workgroup
//        per list: a bucket pass over a 64-bit (key, Gaussian, j) word and a rank by counting inside
//        the bucket for up to kBlkCap (4096) entries; longer lists are first cut by an MSD bucket split
//        into segments of at most ~kMsdSeg entries that the bucket sort finishes one after another; a
//        segment of nearly equal depths takes LSD passes of 8-bit digits over the Gaussian index's
//        varying bits, then the key's (n <= kSegCap (2048) in registers with an LDS scatter; above,
//        chunks of kSegCap, a digit histogram sweep then a rank-and-scatter sweep per pass,
//        ping-ponging through the pair buffers the tile sort has finished with, L2-resident, the last
//        pass copied back into the list).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "gs_device.hpp"
#include "gs_internal.hpp"

#include <algorithm>

namespace gs {

constexpr uint32_t kSegThreads = 256;
constexpr uint32_t kSegWaves = kSegThreads / 64;
constexpr uint32_t kSegItems = 8;                        // rows of 64 per wave
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
    uint32_t red[4][kSegWaves];
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

// A list of n entries at pair position `base`, read from `in` (base-relative) and written sorted to
// `out` (may be `in`); the ping-pong scratch is used at the same positions.
__device__ void seg_lsd_block(SegShared& S, uint32_t base, uint32_t n, const uint32_t* in, uint32_t* out,
                              const uint32_t* __restrict__ dkey, uint32_t* __restrict__ ka, uint32_t* __restrict__ va,
                              uint32_t* __restrict__ kb, uint32_t* __restrict__ vb) {
    const uint32_t t = threadIdx.x, w = t >> 6, lane = t & 63u;
    const uint2 r = make_uint2(base, base + n);
    if (n <= 1u) {
        if (n == 1u && t == 0 && out != in) out[0] = in[0];
        return;
    }
    const uint32_t nchunks = (n + kSegCap - 1u) / kSegCap;
    const uint32_t* const list = in;

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

    // the bits the tile's keys differ in, [0, hb), and its Gaussian indices, [0, gb)
    uint32_t kmin = 0xffffffffu, kmax = 0u, gmin = 0xffffffffu, gmax = 0u;
    for (uint32_t c = 0; c < nchunks; c++) {
        const uint32_t R = chunk_rows(c);
        load_chunk(c, R, 0u);
#pragma unroll
        for (uint32_t i = 0; i < kSegItems; i++)
            if (ok[i]) {
                kmin = min(kmin, k[i]);
                kmax = max(kmax, k[i]);
                gmin = min(gmin, v[i] >> kPairJBits);
                gmax = max(gmax, v[i] >> kPairJBits);
            }
    }
    kmin = wave_min_u32(kmin);
    kmax = wave_max_u32(kmax);
    gmin = wave_min_u32(gmin);
    gmax = wave_max_u32(gmax);
    if (lane == 0) {
        S.red[0][w] = kmin;
        S.red[1][w] = kmax;
        S.red[2][w] = gmin;
        S.red[3][w] = gmax;
    }
    seg_barrier();
#pragma unroll
    for (uint32_t q = 0; q < kSegWaves; q++) {
        kmin = min(kmin, S.red[0][q]);
        kmax = max(kmax, S.red[1][q]);
        gmin = min(gmin, S.red[2][q]);
        gmax = max(gmax, S.red[3][q]);
    }
    const uint32_t hb = (kmin ^ kmax) ? 32u - (uint32_t)__clz(kmin ^ kmax) : 0u;
    const uint32_t gb = (gmin ^ gmax) ? 32u - (uint32_t)__clz(gmin ^ gmax) : 0u;
    // LSD on (key, Gaussian): the Gaussian's bytes first, then the key's, so the result does not
    // depend on the order the list arrived in (bits above hb / gb are equal on the whole list)
    const uint32_t gpass = (gb + 7u) >> 3;
    const uint32_t npass = gpass + ((hb + 7u) >> 3);
    auto digit = [&](uint32_t kk, uint32_t vv, uint32_t p) -> uint32_t {
        return p < gpass ? ((vv >> kPairJBits) >> (8u * p)) & 0xffu : (kk >> (8u * (p - gpass))) & 0xffu;
    };
    if (npass == 0u) {  // one key and one Gaussian: already in order
        if (out != in)
            for (uint32_t e = t; e < n; e += kSegThreads) out[e] = in[e];
        return;
    }

    if (nchunks == 1u) {
        // ---- register-resident list, LDS scatter per pass (chunk 0 is still loaded) ----
        const uint32_t R = chunk_rows(0);
        for (uint32_t p = 0; p < npass; p++) {
            if (t < 256u)
#pragma unroll
                for (uint32_t q = 0; q < kSegWaves; q++) S.cnt[q][t] = 0u;
            seg_barrier();
#pragma unroll
            for (uint32_t i = 0; i < kSegItems; i++) dg[i] = digit(k[i], v[i], p);
            seg_rank(S, w, lane, R, ok, dg, 8u, rk);
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
        seg_barrier();  // (out may be in: every wave has loaded its rows)
#pragma unroll
        for (uint32_t i = 0; i < kSegItems; i++)
            if (ok[i]) out[(w * R + i) * 64u + lane] = v[i];
        return;
    }

    // ---- chunked: per pass a histogram sweep, then rank + scatter chunk by chunk ----
    uint32_t src = 0u;
    for (uint32_t p = 0; p < npass; p++) {
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
                if (ok[i]) atomicAdd(&S.cnt[w][digit(k[i], v[i], p)], 1u);
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
            for (uint32_t i = 0; i < kSegItems; i++) dg[i] = digit(k[i], v[i], p);
            seg_rank(S, w, lane, R, ok, dg, 8u, rk);
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
    // the sorted values into the output
    const uint32_t* const vs = (src == 1u ? va : vb) + r.x;
    for (uint32_t e = t; e < n; e += kSegThreads) out[e] = vs[e];
}

// ---- the bucket sort of a list of up to kBlkCap entries, one workgroup ------------------------
// The list arrives in any order (the any-order tile scatter places a slice's pairs with LDS
// atomics), so the sort does not rely on it. An entry's word K = (key - kmin, gid - gmin, j) packed
// in 64 bits, j the pair's tile index inside its Gaussian's rect (the value is gid << 8 | j): K
// compares as (depth key, Gaussian) and decodes back to the value, so no value is gathered. One
// bucket pass on the top kBlkBucketBits significant bits of K (histogram with LDS atomics, a scan, a
// scatter with returning LDS atomics: the order inside a bucket is arbitrary), then each bucket slot
// counts the words of its bucket below its own: its place in the list. 16 entries per thread, 4096
// buckets; false (list untouched) when the largest bucket exceeds kBucketMax (nearly equal depths:
// the LSD passes take the list).
constexpr uint32_t kBlkRows = 16;
constexpr uint32_t kBlkCap = kSegThreads * kBlkRows;  // 4096
constexpr uint32_t kBlkBuckets = 4096;
constexpr uint32_t kBlkBucketBits = 12;
constexpr uint32_t kBlkPerThread = kBlkBuckets / kSegThreads;
constexpr uint32_t kBucketMax = 64;
// MSD split of a list above kBlkCap (tile_long_sort_kernel): the top kLongBuckets significant bits
// of K cut the list into buckets; bucket b goes to segment floor(start_b / kMsdSeg), so a segment
// holds at most kMsdSeg + (its last bucket) entries and is finished by the bucket sort whenever
// that is at most kBlkCap.
constexpr uint32_t kMsdSeg = 3072;
// Bucket b's counter lives at bk(b) = b + b / 16: the scans give each thread 16 consecutive buckets,
// and without the pad word the 16-word stride put every other lane of a wave on the same LDS bank
// (SQ_LDS_BANK_CONFLICT above the kernels' own LDS issue cycles, profiles/r04_sq_counters.txt).
__device__ __forceinline__ uint32_t bk(uint32_t b) { return b + (b >> 4); }
static_assert(kBlkBuckets / kSegThreads == 16, "bk(): 16 buckets per thread");
struct BucketShared {
    uint64_t word[kBlkCap];
    uint32_t cur[kBlkBuckets + kBlkBuckets / 16];
    uint32_t red[5][kSegWaves];
};
static_assert(kBlkBuckets % kSegThreads == 0, "buckets per thread");

__device__ bool tile_depth_sort_bucket_block(BucketShared& S, uint32_t n, const uint32_t* list, uint32_t* out,
                                             const uint32_t* __restrict__ dkey) {
    const uint32_t t = threadIdx.x, w = t >> 6, lane = t & 63u;
    const uint32_t R = (n + kSegThreads - 1u) / kSegThreads;  // rows of kSegThreads, uniform
    uint32_t v[kBlkRows], q[kBlkRows];
#pragma unroll
    for (uint32_t i = 0; i < kBlkRows; i++) {
        const uint32_t e = i * kSegThreads + t;
        v[i] = (i < R && e < n) ? list[e] : 0u;
    }
#pragma unroll
    for (uint32_t i = 0; i < kBlkRows; i++) q[i] = (i < R && i * kSegThreads + t < n) ? dkey[v[i] >> kPairJBits] : 0u;
    uint32_t kmin = 0xffffffffu, kmax = 0u, gl = 0xffffffffu, gh = 0u;
#pragma unroll
    for (uint32_t i = 0; i < kBlkRows; i++)
        if (i < R && i * kSegThreads + t < n) {
            kmin = min(kmin, q[i]);
            kmax = max(kmax, q[i]);
            gl = min(gl, v[i] >> kPairJBits);
            gh = max(gh, v[i] >> kPairJBits);
        }
    kmin = wave_min_dpp(kmin);
    kmax = wave_max_dpp(kmax);
    gl = wave_min_dpp(gl);
    gh = wave_max_dpp(gh);
    if (lane == 0) {
        S.red[0][w] = kmin;
        S.red[1][w] = kmax;
        S.red[2][w] = gl;
        S.red[3][w] = gh;
    }
#pragma unroll
    for (uint32_t c = 0; c < kBlkPerThread; c++) S.cur[bk(kBlkPerThread * t + c)] = 0u;
    seg_barrier();
#pragma unroll
    for (uint32_t k = 0; k < kSegWaves; k++) {
        kmin = min(kmin, S.red[0][k]);
        kmax = max(kmax, S.red[1][k]);
        gl = min(gl, S.red[2][k]);
        gh = max(gh, S.red[3][k]);
    }
    const uint32_t gmin = gl;
    const uint32_t hb = kmax != kmin ? 32u - (uint32_t)__clz(kmax - kmin) : 0u;
    const uint32_t gb = gh != gl ? 32u - (uint32_t)__clz(gh - gl) : 0u;
    const uint32_t sig = hb + gb;
    const uint32_t dsh = kPairJBits + (sig > kBlkBucketBits ? sig - kBlkBucketBits : 0u);
    const uint32_t gsh = gb + kPairJBits;
    const uint32_t vmask = (uint32_t)((1ull << gsh) - 1ull);
    uint64_t K[kBlkRows];
#pragma unroll
    for (uint32_t i = 0; i < kBlkRows; i++)
        K[i] = ((uint64_t)(q[i] - kmin) << gsh) | (uint64_t)(v[i] - (gmin << kPairJBits));
#pragma unroll
    for (uint32_t i = 0; i < kBlkRows; i++)
        if (i < R && i * kSegThreads + t < n) atomicAdd(&S.cur[bk((uint32_t)(K[i] >> dsh) & (kBlkBuckets - 1u))], 1u);
    seg_barrier();
    uint32_t cb[kBlkPerThread], sb = 0, mbl = 0;
#pragma unroll
    for (uint32_t c = 0; c < kBlkPerThread; c++) {
        cb[c] = S.cur[bk(kBlkPerThread * t + c)];
        sb += cb[c];
        mbl = max(mbl, cb[c]);
    }
    const uint32_t inc = wave_scan_dpp(sb, 0u, DppAdd{});
    mbl = wave_max_dpp(mbl);
    if (lane == 63u) S.red[4][w] = inc;
    if (lane == 0) S.red[0][w] = mbl;
    seg_barrier();
    uint32_t mb = 0, run = inc - sb;
#pragma unroll
    for (uint32_t k = 0; k < kSegWaves; k++) {
        mb = max(mb, S.red[0][k]);
        run += k < w ? S.red[4][k] : 0u;
    }
    if (mb > kBucketMax) return false;  // (uniform; the list is untouched)
#pragma unroll
    for (uint32_t c = 0; c < kBlkPerThread; c++) {
        S.cur[bk(kBlkPerThread * t + c)] = run;
        run += cb[c];
    }
    seg_barrier();
#pragma unroll
    for (uint32_t i = 0; i < kBlkRows; i++)
        if (i < R && i * kSegThreads + t < n) {
            const uint32_t p = atomicAdd(&S.cur[bk((uint32_t)(K[i] >> dsh) & (kBlkBuckets - 1u))], 1u);
            S.word[p] = K[i];
        }
    seg_barrier();
    uint64_t kp[kBlkRows];
    uint32_t bs[kBlkRows], bn[kBlkRows], below[kBlkRows];
#pragma unroll
    for (uint32_t i = 0; i < kBlkRows; i++) {
        const uint32_t p = i * kSegThreads + t;
        kp[i] = (i < R && p < n) ? S.word[p] : ~0ull;
        const uint32_t d = (uint32_t)(kp[i] >> dsh) & (kBlkBuckets - 1u);
        const uint32_t b0 = (i < R && d) ? S.cur[bk(d - 1u)] : 0u, b1 = i < R ? S.cur[bk(d)] : 0u;
        bs[i] = b0;
        bn[i] = b1 - b0;
        below[i] = 0u;
    }
    for (uint32_t j = 0; j < mb; j++) {
        uint64_t x[kBlkRows];
#pragma unroll
        for (uint32_t i = 0; i < kBlkRows; i++)
            if (i < R) x[i] = S.word[min(bs[i] + j, kBlkCap - 1u)];
#pragma unroll
        for (uint32_t i = 0; i < kBlkRows; i++)
            if (i < R) below[i] += (j < bn[i] && x[i] < kp[i]) ? 1u : 0u;
    }
#pragma unroll
    for (uint32_t i = 0; i < kBlkRows; i++) {
        const uint32_t p = i * kSegThreads + t;
        if (i < R && p < n) out[bs[i] + below[i]] = ((uint32_t)kp[i] & vmask) + (gmin << kPairJBits);
    }
    return true;
}

// ---- the lists longer than the forward sorts itself -----------------------------------------
// One launch, no job list: workgroup b takes the tiles b, b + grid, ... whose lists exceed skip_max
// entries. Up to kBlkCap: the bucket sort in place (the LSD passes for nearly equal depths). Longer:
// the workgroup cuts the list by an MSD bucket split (the K range, a histogram of K's top
// kLongBuckets significant bits, the buckets' starts, the values scattered into `scratch` at their
// buckets' slots) into segments of at most kMsdSeg + (the last bucket) entries, ordered among
// themselves, and sorts them one after the other from the scratch into the list. (Round 4 sorted
// lists of up to 1024 entries one wave per tile in a kernel of their own and handed the rest to a
// workgroup kernel through a job list; the forward now sorts the short ones, round 5.)
constexpr uint32_t kLongBuckets = 1024;
constexpr uint32_t kLongSegs = 1024;  // segments of one list (n <= ~3.1M); above: the LSD passes whole
struct LongSplitShared {
    uint32_t cur[kLongBuckets + kLongBuckets / 4];  // bucket b at b + b / 4 (4 per thread)
    uint32_t seg[2 * kLongSegs];
    uint32_t red[5][kSegWaves];
};
__device__ __forceinline__ uint32_t lb(uint32_t b) { return b + (b >> 2); }
static_assert(kLongBuckets == 4u * kSegThreads, "4 buckets per thread");

__global__ __launch_bounds__(kSegThreads) void tile_long_sort_kernel(
    const uint2* __restrict__ ranges, uint32_t T, uint32_t skip_max, const uint32_t* __restrict__ dkey,
    uint32_t* __restrict__ s_val, uint32_t* __restrict__ scratch, uint32_t* __restrict__ ka,
    uint32_t* __restrict__ va, uint32_t* __restrict__ kb, uint32_t* __restrict__ vb) {
    __shared__ union {
        SegShared s;
        BucketShared b;
        LongSplitShared m;
    } U;
    __shared__ uint32_t seg_bcast[2];
    __shared__ uint64_t s_long[2];
    const uint32_t t = threadIdx.x, w = t >> 6, lane = t & 63u;
    // the workgroup's tiles (blockIdx.x + k * gridDim.x) are screened 64 at a time by wave 0, one
    // range load per lane, so a frame with few or no long lists costs one load round trip per
    // workgroup instead of one per tile; the long ones are then sorted one after the other
    for (uint32_t k0 = 0; blockIdx.x + k0 * gridDim.x < T; k0 += 64u) {
        if (w == 0) {
            const uint32_t tl = blockIdx.x + (k0 + lane) * gridDim.x;
            bool need = false;
            if (tl < T) {
                const uint2 rr = ranges[tl];
                need = rr.y - rr.x > skip_max && rr.y - rr.x >= 2u;
            }
            const uint64_t m = __ballot(need);
            if (lane == 0) s_long[(k0 >> 6) & 1u] = m;  // (double-buffered: one barrier per screen)
        }
        __syncthreads();
        for (uint64_t todo = s_long[(k0 >> 6) & 1u]; todo; todo &= todo - 1ull) {
            const uint32_t tile = blockIdx.x + (k0 + (uint32_t)__builtin_ctzll(todo)) * gridDim.x;
            const uint2 r = ranges[tile];
            const uint32_t n = r.y - r.x;
            uint32_t* const list = s_val + r.x;
            if (n <= kBlkCap) {
                const bool done = tile_depth_sort_bucket_block(U.b, n, list, list, dkey);
                __syncthreads();
                if (!done) {
                    seg_lsd_block(U.s, r.x, n, list, list, dkey, ka, va, kb, vb);
                    __syncthreads();
                }
                continue;
            }
            const uint32_t nseg = (n - 1u) / kMsdSeg + 1u;
            if (nseg > kLongSegs) {
                seg_lsd_block(U.s, r.x, n, list, list, dkey, ka, va, kb, vb);
                __syncthreads();
                continue;
            }
            constexpr uint32_t kU = 4;  // rows of 256 in flight per step
            uint32_t kmin = 0xffffffffu, kmax = 0u, gl = 0xffffffffu, gh = 0u;
            for (uint32_t e0 = 0; e0 < n; e0 += kSegThreads * kU) {
                uint32_t v[kU], q[kU];
    #pragma unroll
                for (uint32_t u = 0; u < kU; u++) {
                    const uint32_t e = e0 + u * kSegThreads + t;
                    v[u] = e < n ? list[e] : 0u;
                }
    #pragma unroll
                for (uint32_t u = 0; u < kU; u++) q[u] = e0 + u * kSegThreads + t < n ? dkey[v[u] >> kPairJBits] : 0u;
    #pragma unroll
                for (uint32_t u = 0; u < kU; u++)
                    if (e0 + u * kSegThreads + t < n) {
                        kmin = min(kmin, q[u]);
                        kmax = max(kmax, q[u]);
                        gl = min(gl, v[u] >> kPairJBits);
                        gh = max(gh, v[u] >> kPairJBits);
                    }
            }
            kmin = wave_min_dpp(kmin);
            kmax = wave_max_dpp(kmax);
            gl = wave_min_dpp(gl);
            gh = wave_max_dpp(gh);
            if (lane == 0) {
                U.m.red[0][w] = kmin;
                U.m.red[1][w] = kmax;
                U.m.red[2][w] = gl;
                U.m.red[3][w] = gh;
            }
    #pragma unroll
            for (uint32_t c = 0; c < 4; c++) U.m.cur[lb(4u * t + c)] = 0u;
            for (uint32_t k = t; k < nseg; k += kSegThreads) {
                U.m.seg[2u * k] = 0xffffffffu;
                U.m.seg[2u * k + 1u] = 0u;
            }
            __syncthreads();
    #pragma unroll
            for (uint32_t k = 0; k < kSegWaves; k++) {
                kmin = min(kmin, U.m.red[0][k]);
                kmax = max(kmax, U.m.red[1][k]);
                gl = min(gl, U.m.red[2][k]);
                gh = max(gh, U.m.red[3][k]);
            }
            const uint32_t gmin = gl;
            const uint32_t hb = kmax != kmin ? 32u - (uint32_t)__clz(kmax - kmin) : 0u;
            const uint32_t gb = gh != gl ? 32u - (uint32_t)__clz(gh - gl) : 0u;
            const uint32_t sig = hb + gb;
            constexpr uint32_t kLongBits = 10;
            static_assert((1u << kLongBits) == kLongBuckets, "bucket bits");
            const uint32_t dsh = kPairJBits + (sig > kLongBits ? sig - kLongBits : 0u);
            const uint32_t gsh = gb + kPairJBits;
            auto bucket = [&](uint32_t v, uint32_t q) {
                const uint64_t K = ((uint64_t)(q - kmin) << gsh) | (uint64_t)(v - (gmin << kPairJBits));
                return (uint32_t)(K >> dsh) & (kLongBuckets - 1u);
            };
            for (uint32_t e0 = 0; e0 < n; e0 += kSegThreads * kU) {
                uint32_t v[kU], q[kU];
    #pragma unroll
                for (uint32_t u = 0; u < kU; u++) {
                    const uint32_t e = e0 + u * kSegThreads + t;
                    v[u] = e < n ? list[e] : 0u;
                }
    #pragma unroll
                for (uint32_t u = 0; u < kU; u++) q[u] = e0 + u * kSegThreads + t < n ? dkey[v[u] >> kPairJBits] : 0u;
    #pragma unroll
                for (uint32_t u = 0; u < kU; u++)
                    if (e0 + u * kSegThreads + t < n) atomicAdd(&U.m.cur[lb(bucket(v[u], q[u]))], 1u);
            }
            __syncthreads();
            uint32_t cb[4], sb = 0;
    #pragma unroll
            for (uint32_t c = 0; c < 4; c++) {
                cb[c] = U.m.cur[lb(4u * t + c)];
                sb += cb[c];
            }
            const uint32_t inc = wave_scan_dpp(sb, 0u, DppAdd{});
            if (lane == 63u) U.m.red[4][w] = inc;
            __syncthreads();
            uint32_t run = inc - sb;
    #pragma unroll
            for (uint32_t k = 0; k < kSegWaves; k++) run += k < w ? U.m.red[4][k] : 0u;
    #pragma unroll
            for (uint32_t c = 0; c < 4; c++) {
                U.m.cur[lb(4u * t + c)] = run;
                if (cb[c]) {
                    const uint32_t k = run / kMsdSeg;
                    atomicMin(&U.m.seg[2u * k], run);
                    atomicMax(&U.m.seg[2u * k + 1u], run + cb[c]);
                }
                run += cb[c];
            }
            __syncthreads();
            for (uint32_t e0 = 0; e0 < n; e0 += kSegThreads * kU) {
                uint32_t v[kU], q[kU];
    #pragma unroll
                for (uint32_t u = 0; u < kU; u++) {
                    const uint32_t e = e0 + u * kSegThreads + t;
                    v[u] = e < n ? list[e] : 0u;
                }
    #pragma unroll
                for (uint32_t u = 0; u < kU; u++) q[u] = e0 + u * kSegThreads + t < n ? dkey[v[u] >> kPairJBits] : 0u;
    #pragma unroll
                for (uint32_t u = 0; u < kU; u++)
                    if (e0 + u * kSegThreads + t < n)
                        scratch[r.x + atomicAdd(&U.m.cur[lb(bucket(v[u], q[u]))], 1u)] = v[u];
            }
            // the scatter's stores are read back by other waves of the workgroup; the segments' bounds
            // leave LDS (for registers: segment k in thread k % 256) before it becomes the sorts' space
            __syncthreads();
            constexpr uint32_t kSegPerThread = kLongSegs / kSegThreads;
            uint32_t slo[kSegPerThread], shi[kSegPerThread];
    #pragma unroll
            for (uint32_t j = 0; j < kSegPerThread; j++) {
                const uint32_t k = j * kSegThreads + t;
                slo[j] = k < nseg ? U.m.seg[2u * k] : 0u;
                shi[j] = k < nseg ? U.m.seg[2u * k + 1u] : 0u;
            }
            __syncthreads();
            for (uint32_t k = 0; k < nseg; k++) {
                if (t == k % kSegThreads) {
                    const uint32_t j = k / kSegThreads;
                    uint32_t lo = slo[0], hi = shi[0];
    #pragma unroll
                    for (uint32_t jj = 1; jj < kSegPerThread; jj++)
                        if (jj == j) {
                            lo = slo[jj];
                            hi = shi[jj];
                        }
                    seg_bcast[0] = lo;
                    seg_bcast[1] = hi;
                }
                __syncthreads();
                const uint32_t lo = seg_bcast[0], hi = seg_bcast[1];
                __syncthreads();
                if (hi <= lo) continue;  // (uniform: an empty segment)
                const uint32_t m = hi - lo;
                const uint32_t* in = scratch + r.x + lo;
                uint32_t* out = list + lo;
                const bool done = m <= kBlkCap && tile_depth_sort_bucket_block(U.b, m, in, out, dkey);
                __syncthreads();
                if (!done) {
                    seg_lsd_block(U.s, r.x + lo, m, in, out, dkey, ka, va, kb, vb);
                    __syncthreads();
                }
            }
            __syncthreads();
        }
    }
}

hipError_t launch_tile_depth_sort(hipStream_t st, const uint2* ranges, uint32_t T, const uint32_t* dkey,
                                  uint32_t* s_val, uint32_t* ka, uint32_t* va, uint32_t* kb, uint32_t* vb,
                                  uint32_t* scratch) {
    if (T == 0) return hipSuccess;
    hipLaunchKernelGGL(tile_long_sort_kernel, dim3(std::min<uint32_t>(T, 1024u)), dim3(kSegThreads), 0, st, ranges,
                       T, kFwdSortMax, dkey, s_val, scratch, ka, va, kb, vb);
    return hipGetLastError();
}

}  // namespace gs
