// gs_blend.hip — per-tile front-to-back blend (forward) and its reverse pass (backward).
//
//   forward_quad_kernel  tiledForward (tiled_shaders.metal:307-385). One 16x16 tile per 256-thread
//                        workgroup, four independent waves, one 8x8 pixel band each, every band wave
//                        split into four 16-lane groups (one 4x4 quadrant each). On the per-tile depth
//                        order the workgroup first sorts its tile's list in LDS (fwd_sort_list). A wave
//                        gathers its tile's list 64 records per step (prefetched one step ahead, entries
//                        two), culls them against its band's quadrants (box + ellipse test; the band's
//                        ballot is handed to the backward), lists each quadrant's survivors and blends
//                        them one splat pair per group and step, in IEEE half exactly as the reference.
//                        It also tracks the float transmittance the reference backward recomputes before
//                        its reverse loop (:430-460) on the hardware exp, recomputing exactly the rare
//                        pixels whose break decision falls inside the track's error bound, and stores it
//                        per pixel, so the backward makes one traversal instead of two.
//   backward_kernel      tiledBackward (:388-738). One wave per tile, 4 pixels per lane (one in each
//                        8x8 band). Per splat: the forward's band ballots, per-pixel contribution, the 9
//                        linear partials summed over the lane's pixels, then a pair of splats' 18 sums
//                        across the wave (permlane32/16 swaps, select + row_ror, 3 DPP steps) and one
//                        store per pair, with the frame tag of each reached slot. No float atomics;
//                        deterministic.
//
// Without a launch order, tiles are mapped to workgroups XCD-aware: blocks b and b+8 share an XCD
// under round-robin dispatch, so each XCD gets a contiguous run of tiles (L2 reuse).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "gs_device.hpp"
#include "gs_internal.hpp"

namespace gs {

__device__ __forceinline__ uint32_t quantize_unorm8(float c) {
    return (uint32_t)rintf(fminf(fmaxf(c, 0.0f), 1.0f) * 255.0f);
}

// does the splat's culling box reach the pixel-centre rectangle [x0, x1] x [y0, y1]?
__device__ __forceinline__ bool box_hits(float sx, float sy, float ex, float ey, float x0, float x1,
                                         float y0, float y1) {
    return !(sx + ex < x0 || sx - ex > x1 || sy + ey < y0 || sy - ey > y1);
}

#ifdef GS_BLEND_TRACE  // diagnostics build only: per-workgroup start/end timestamps and CU id
__device__ unsigned long long g_blend_trace[2][16384][2];
__device__ unsigned int g_blend_hw[2][16384];
extern "C" __attribute__((visibility("default"))) int gs_debug_blend_trace(void* host, void* hw, size_t n) {
    hipError_t e = hipMemcpyFromSymbol(host, HIP_SYMBOL(g_blend_trace), n < sizeof(g_blend_trace) ? n : sizeof(g_blend_trace));
    if (e != hipSuccess) return (int)e;
    return (int)hipMemcpyFromSymbol(hw, HIP_SYMBOL(g_blend_hw), sizeof(g_blend_hw));
}
#define BLEND_TRACE(k, phase) \
    do { if (threadIdx.x == 0 && blockIdx.x < 16384u) { g_blend_trace[k][blockIdx.x][phase] = wall_clock64(); \
         if (phase == 0) g_blend_hw[k][blockIdx.x] = __smid(); } } while (0)
#else
#define BLEND_TRACE(k, phase) do { } while (0)
#endif

#ifdef GS_BLEND_STATS  // diagnostics build only: work counters of the blend kernels
__device__ unsigned long long g_blend_stats[32];
extern "C" __attribute__((visibility("default"))) int gs_debug_blend_stats(void* host, int reset) {
    hipError_t e = hipMemcpyFromSymbol(host, HIP_SYMBOL(g_blend_stats), sizeof(g_blend_stats));
    if (e == hipSuccess && reset) {
        unsigned long long z[32] = {};
        e = hipMemcpyToSymbol(HIP_SYMBOL(g_blend_stats), z, sizeof(z));
    }
    return (int)e;
}
#define BSTAT(i, v) (st_[i] += (unsigned long long)(v))
#define BSTAT_DECL unsigned long long st_[16] = {};
#define BSTAT_FLUSH(base) do { if ((threadIdx.x & 63u) == 0) for (int q_ = 0; q_ < 16; q_++) \
        if (st_[q_]) atomicAdd(&g_blend_stats[(base) + q_], st_[q_]); } while (0)
#else
#define BSTAT(i, v) do { } while (0)
#define BSTAT_DECL
#define BSTAT_FLUSH(base) do { } while (0)
#endif

// ---------------------------------------------------------------------------------------
constexpr int kFwdThreads = 256;  // four independent waves per 16x16 tile, one pixel band each
constexpr uint32_t kFwdStep = 2;  // splats per group and blend step
constexpr uint32_t kBandW = 8;  // band kBandW x kBandH = 64 pixels
constexpr uint32_t kBandH = 64u / kBandW;

__device__ __forceinline__ uint32_t pack_h2(_Float16 lo, _Float16 hi) {
    return (uint32_t)__builtin_bit_cast(uint16_t, lo) | ((uint32_t)__builtin_bit_cast(uint16_t, hi) << 16);
}

__device__ __forceinline__ float readlane_f(float v, uint32_t l) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}

// Relative bound on |T_hw / T_pinned - 1| for the float T_final track after n splats (T >= ~1e-4):
// per splat the weights differ by <= kExpRelErr (measured exhaustively on the device over every
// float power in [-4.5, 0], gs_debug_float_exp_check), which (1 - alpha) amplifies by
// alpha / (1 - alpha) <= 21.5 * -ln(1 - alpha) for alpha <= 0.99, summed to <= 21.5 * ln(1e4) = 198
// while T stays above the threshold; each splat taken adds <= 2.4e-7 of rounding between the two
// tracks.
constexpr float kExpRelErr = 4.0e-7f;
__device__ __forceinline__ float tfinal_track_bound(uint32_t n) {
    return (kExpRelErr + 1.2e-7f) * 198.0f + 2.5e-7f * (float)n + 2.0e-5f;
}

// The exact float T_final of one pixel (tiled_shaders.metal:430-460, the pinned exp, every decision
// in float as the reference): the wave walks the pixel's list [range.x, last] 64 entries at a time,
// each lane evaluating one entry's alpha, then multiplies the contributing factors in list order.
// Used only for the rare pixels whose hardware-exp track came within its error bound of the
// T < 1e-4 break.
__device__ float tfinal_exact(float px, float py, uint32_t first, uint32_t last, const float4* __restrict__ rec,
                              const uint32_t* list, uint32_t list_off, uint32_t lane) {
    float T = 1.0f;
    for (uint32_t b0 = first; b0 <= last; b0 += 64u) {
        const uint32_t idx = b0 + lane;
        float a = 0.0f;
        bool contrib = false;
        if (idx <= last) {
            const float4* r = rec + (size_t)(list[idx - list_off] >> kPairJBits) * kRecQuads;
            const float4 qa = r[0], qb = r[1];
            const float dx = px - qa.x, dy = py - qa.y;
            const float pw = -0.5f * ((qa.z * dx * dx + (2.0f * qa.w) * dx * dy) + qb.x * dy * dy);
            if (!(pw > 0.0f || pw < -4.5f)) {
                a = __builtin_amdgcn_fmed3f(qb.y * gs_expf_core(pw), -1.0f, 0.99f);
                contrib = !(a < 1.0f / 255.0f);
            }
        }
        uint64_t cm = __builtin_amdgcn_ballot_w64(contrib);
        while (cm) {
            const uint32_t j = (uint32_t)__builtin_ctzll(cm);
            cm &= cm - 1ull;
            const float test = T * (1.0f - readlane_f(a, j));
            if (test < 0.0001f) return T;
            T = test;
        }
    }
    return T;
}

// In-forward depth order of the tile's list (sort_dkey != null: the per-tile depth order, lists of
// 2..kFwdSortCap entries; longer ones were sorted by gs_segsort.hip's kernels before the forward):
// the workgroup's four waves sort the list (the 64-bit word K = (depth key - min, Gaussian - min, j),
// which compares as (depth key, Gaussian) and decodes back to the value; one bucket pass on K's top
// kFwdSortBits significant bits, each slot ranked by counting the smaller words of its bucket), keep
// the sorted values in LDS for the blend and store them to s_val for the backward. (Round 4 sorted
// every list in a wave kernel of its own: its per-tile load -> gather -> store chain cost 42 us at
// the bench frame; the forward's own list loads now come from LDS.)
constexpr uint32_t kFwdSortCap = 1024;
constexpr uint32_t kFwdSortBits = 10;
constexpr uint32_t kFwdSortBuckets = 1u << kFwdSortBits;
constexpr uint32_t kFwdSortRows = kFwdSortCap / kFwdThreads;  // 4 entries per thread
__device__ __forceinline__ uint32_t fsb(uint32_t b) { return b + (b >> 2); }  // 4 buckets per thread: padded
struct FwdSortShared {
    uint64_t word[kFwdSortCap];
    uint32_t cur[kFwdSortBuckets + kFwdSortBuckets / 4];
    uint32_t red[5][kFwdThreads / 64];
};

// Sorts list[0, n) (2 <= n <= kFwdSortCap) into sv (LDS) and list (global). Whole workgroup.
__device__ void fwd_sort_list(FwdSortShared& S, uint32_t* sv, uint32_t* list, uint32_t n,
                              const uint32_t* __restrict__ dkey, uint32_t t) {
    const uint32_t w = t >> 6, lane = t & 63u;
    uint32_t v[kFwdSortRows], q[kFwdSortRows];
#pragma unroll
    for (uint32_t i = 0; i < kFwdSortRows; i++) {
        const uint32_t e = i * kFwdThreads + t;
        v[i] = e < n ? list[e] : 0u;
    }
#pragma unroll
    for (uint32_t i = 0; i < kFwdSortRows; i++) q[i] = i * kFwdThreads + t < n ? dkey[v[i] >> kPairJBits] : 0u;
    uint32_t kmin = 0xffffffffu, kmax = 0u, gl = 0xffffffffu, gh = 0u;
#pragma unroll
    for (uint32_t i = 0; i < kFwdSortRows; i++)
        if (i * kFwdThreads + t < n) {
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
    for (uint32_t c = 0; c < 4; c++) S.cur[fsb(4u * t + c)] = 0u;
    __syncthreads();
#pragma unroll
    for (uint32_t k = 0; k < kFwdThreads / 64; k++) {
        kmin = min(kmin, S.red[0][k]);
        kmax = max(kmax, S.red[1][k]);
        gl = min(gl, S.red[2][k]);
        gh = max(gh, S.red[3][k]);
    }
    const uint32_t gmin = gl;
    const uint32_t hb = kmax != kmin ? 32u - (uint32_t)__clz(kmax - kmin) : 0u;
    const uint32_t gb = gh != gl ? 32u - (uint32_t)__clz(gh - gl) : 0u;
    const uint32_t sig = hb + gb;
    const uint32_t dsh = kPairJBits + (sig > kFwdSortBits ? sig - kFwdSortBits : 0u);
    const uint32_t gsh = gb + kPairJBits;
    const uint32_t vmask = (uint32_t)((1ull << gsh) - 1ull);
    uint64_t K[kFwdSortRows];
#pragma unroll
    for (uint32_t i = 0; i < kFwdSortRows; i++) {
        K[i] = ((uint64_t)(q[i] - kmin) << gsh) | (uint64_t)(v[i] - (gmin << kPairJBits));
        if (i * kFwdThreads + t < n) atomicAdd(&S.cur[fsb((uint32_t)(K[i] >> dsh) & (kFwdSortBuckets - 1u))], 1u);
    }
    __syncthreads();
    uint32_t cb[4], sb = 0, mbl = 0;
#pragma unroll
    for (uint32_t c = 0; c < 4; c++) {
        cb[c] = S.cur[fsb(4u * t + c)];
        sb += cb[c];
        mbl = max(mbl, cb[c]);
    }
    const uint32_t inc = wave_scan_dpp(sb, 0u, DppAdd{});
    mbl = wave_max_dpp(mbl);
    if (lane == 63u) S.red[4][w] = inc;
    if (lane == 0) S.red[0][w] = mbl;
    __syncthreads();
    uint32_t mb = 0, run = inc - sb;
#pragma unroll
    for (uint32_t k = 0; k < kFwdThreads / 64; k++) {
        mb = max(mb, S.red[0][k]);
        run += k < w ? S.red[4][k] : 0u;
    }
#pragma unroll
    for (uint32_t c = 0; c < 4; c++) {
        S.cur[fsb(4u * t + c)] = run;
        run += cb[c];
    }
    __syncthreads();
#pragma unroll
    for (uint32_t i = 0; i < kFwdSortRows; i++)
        if (i * kFwdThreads + t < n) {
            const uint32_t p = atomicAdd(&S.cur[fsb((uint32_t)(K[i] >> dsh) & (kFwdSortBuckets - 1u))], 1u);
            S.word[p] = K[i];
        }
    __syncthreads();
    // slot p of bucket d = [end of d - 1, end of d): its place is the bucket's start + the number of
    // the bucket's smaller words (any bucket size: a tile of nearly equal depths only loops longer)
    uint64_t kp[kFwdSortRows];
    uint32_t bs[kFwdSortRows], bn[kFwdSortRows], below[kFwdSortRows];
#pragma unroll
    for (uint32_t i = 0; i < kFwdSortRows; i++) {
        const uint32_t p = i * kFwdThreads + t;
        kp[i] = p < n ? S.word[p] : ~0ull;
        const uint32_t d = (uint32_t)(kp[i] >> dsh) & (kFwdSortBuckets - 1u);
        const uint32_t b0 = d ? S.cur[fsb(d - 1u)] : 0u, b1 = S.cur[fsb(d)];
        bs[i] = b0;
        bn[i] = b1 - b0;
        below[i] = 0u;
    }
    for (uint32_t j = 0; j < mb; j++) {
        uint64_t x[kFwdSortRows];
#pragma unroll
        for (uint32_t i = 0; i < kFwdSortRows; i++) x[i] = S.word[min(bs[i] + j, kFwdSortCap - 1u)];
#pragma unroll
        for (uint32_t i = 0; i < kFwdSortRows; i++) below[i] += (j < bn[i] && x[i] < kp[i]) ? 1u : 0u;
    }
#pragma unroll
    for (uint32_t i = 0; i < kFwdSortRows; i++)
        if (i * kFwdThreads + t < n) {
            const uint32_t val = ((uint32_t)kp[i] & vmask) + (gmin << kPairJBits);
            sv[bs[i] + below[i]] = val;
            list[bs[i] + below[i]] = val;  // for the backward (and the debug getters)
        }
    __syncthreads();  // sv complete; the word / bucket space becomes the waves' blend lists
}

// ---------------------------------------------------------------------------------------
// Quadrant-group forward (round 5: 0.353 -> 0.333 ms at the bench frame against the band-list forward
// of rounds 1-4, which walked one compacted list per 8x8 band). The band's 64 lanes are four 16-lane groups,
// each owning a 4x4 quadrant of the 8x8 band; every group walks its own compacted list of the
// chunk's splats that reach its quadrant, so a splat that covers one quadrant of the band costs one
// group's lanes instead of the whole wave's (an 8x8 band's lanes are 48 % in range on the bench
// frame, a 4x4 quadrant's 70 %; scripts/lane_util.py: 21 % fewer pair steps, measured 2.256M ->
// 1.787M). The chunk's records sit in LDS at their chunk position (two 16-B words each), the
// groups' lists hold positions; a step of the wave is one splat pair of each group's list (groups
// with fewer entries run no-op pads), per splat in plain (unpacked) float: the pair's records come
// from two LDS addresses, and packing their fields for v_pk_* would cost moves for nothing
// (v_pk_*_f32 issues at half rate). Per pixel the splats arrive in list order.
struct FwdRec {
    float4 a;  // sx, sy, c0, 2 c1
    uint4 b;   // c2, op (float bits), half(r) | half(g) << 16, half(b) | half(op or 0) << 16
};
constexpr uint32_t kQuadPad = 64;  // the record no pixel reaches (pads a group's odd / short list)

// The four 4x4 quadrants of the band rectangle (x0, y0) + [0, 7]^2 that the culling ellipse
// {q(p - s) <= kq} may reach, as a 4-bit mask (done after the band's box test passed). q uses the
// lower-bound form A' = (1-e) c0 - e|c1|, B' = c1, C' = (1-e) c2 - e|c1|, which is <= the
// float-evaluated q for every offset (|2 c1 dx dy| <= |c1| (dx^2 + dy^2)). If s lies outside a
// quadrant's pixel-centre rectangle, the minimum of the convex q over it lies on an edge facing s:
// along such an edge q is a 1-D quadratic, minimised at a clamped stationary point. Evaluated in fp32
// (fp64 VALU issues at half rate): its rounding is bounded by a few ulps of M(d) = c0 dx^2 + c2 dy^2
// + |c1| (dx^2 + dy^2), and with e = 1e-3 the lower-bound form lies e M(d) below the exact q, which
// covers the blend's own float rounding and this evaluation's (relative 3e-7 of M at the edge
// minimiser, at most the conic's condition number -- <= ~400 past the det / (A C) >= 1e-2 guard, the
// 20:1 aspect clamp's range -- times M at any pixel of the rectangle). Degenerate or near-singular
// forms are never culled. The form's constants are shared by the four quadrants.
__device__ __forceinline__ uint32_t ellipse_quads_hits_f32(float sx, float sy, float c0, float c1, float c2,
                                                           float kq, float ex, float ey, float x0, float y0) {
    const float e = 1e-3f;
    const float ac1 = fabsf(c1);
    const float A = (1.0f - e) * c0 - e * ac1, C = (1.0f - e) * c2 - e * ac1;
    const float B = c1;
    const bool degenerate = !(A > 0.0f) || !(C > 0.0f) || !(A * C - B * B > 1e-2f * A * C);
    const float K = kq * (1.0f + 1e-5f) + 1e-6f;
    const float rC = __builtin_amdgcn_rcpf(C), rA = __builtin_amdgcn_rcpf(A);
    uint32_t m = 0;
#pragma unroll
    for (uint32_t q = 0; q < 4; q++) {
        const float qx0 = x0 + (float)((q & 1u) * 4u), qy0 = y0 + (float)((q >> 1) * 4u);
        const float qx1 = qx0 + 3.0f, qy1 = qy0 + 3.0f;
        if (!box_hits(sx, sy, ex, ey, qx0, qx1, qy0, qy1)) continue;
        const bool outx0 = sx < qx0, outx1 = sx > qx1, outy0 = sy < qy0, outy1 = sy > qy1;
        bool hit = degenerate || !(outx0 || outx1 || outy0 || outy1);
        if (!hit) {
            float best = 3.0e38f;
            if (outx0 || outx1) {
                const float dx = (outx0 ? qx0 : qx1) - sx;
                float dy = -B * dx * rC;
                dy = __builtin_amdgcn_fmed3f(dy, qy0 - sy, qy1 - sy);
                best = fminf(best, A * dx * dx + 2.0f * B * dx * dy + C * dy * dy);
            }
            if (outy0 || outy1) {
                const float dy = (outy0 ? qy0 : qy1) - sy;
                float dx = -B * dy * rA;
                dx = __builtin_amdgcn_fmed3f(dx, qx0 - sx, qx1 - sx);
                best = fminf(best, A * dx * dx + 2.0f * B * dx * dy + C * dy * dy);
            }
            hit = best <= K;
        }
        m |= hit ? 1u << q : 0u;
    }
    return m;
}

// waves per SIMD the register budget is cut for (unbounded: 70 VGPRs, 7 waves, 0.340 ms against 0.333
// with 2 spilled VGPRs at 8)
constexpr int kFwdQuadWaves = 8;
__global__ __launch_bounds__(kFwdThreads, kFwdQuadWaves) void forward_quad_kernel(
    uint32_t w, uint32_t h, uint32_t tiles_x, uint32_t num_tiles, const uint32_t* __restrict__ order,
    const float4* __restrict__ rec, uint32_t* __restrict__ s_val,
    const uint2* __restrict__ ranges,
    const uint32_t* __restrict__ p_dev, uint32_t* __restrict__ last_idx,
    float* __restrict__ t_final, uint32_t* __restrict__ rgba8, float* __restrict__ rgb,
    const uint32_t* __restrict__ chunk_base, uint64_t* __restrict__ band_mask,
    uint32_t* __restrict__ tile_cost, const uint32_t* __restrict__ sort_dkey, uint32_t* __restrict__ walk) {
    struct QuadLists {
        FwdRec recs[kFwdThreads / 64][65];
        uint32_t qlist[kFwdThreads / 64][4][66];
    };
    __shared__ union {
        QuadLists q;
        FwdSortShared srt;
    } U;
    __shared__ uint32_t sv[kFwdSortCap];

    BLEND_TRACE(0, 0);
    const uint32_t tile = order ? order[blockIdx.x] : xcd_tile(blockIdx.x, num_tiles);
    const uint32_t tx = tile % tiles_x, ty = tile / tiles_x;
    const uint32_t t = threadIdx.x, wv = t >> 6, lane = t & 63u;
    constexpr uint32_t kBandsX = kTile / kBandW;
    const uint32_t bxo = (wv % kBandsX) * kBandW, byo = (wv / kBandsX) * kBandH;
    // lane -> pixel: group g = lane / 16 owns quadrant (g & 1, g >> 1) of the band
    const uint32_t grp = lane >> 4, gp = lane & 15u;
    const uint32_t qxo = (grp & 1u) * 4u, qyo = (grp >> 1) * 4u;
    const uint32_t x = tx * kTile + bxo + qxo + (gp & 3u);
    const uint32_t y = ty * kTile + byo + qyo + (gp >> 2);
    const bool inside = x < w && y < h;
    const uint32_t pix = y * w + x;
    if (*p_dev == 0u) {  // tiled_rasterizer.mm:463-467: return before rendering
        if (inside) last_idx[pix] = 0xffffffffu;
        return;
    }
    const uint2 range = ranges[tile];
    const uint32_t nlist = range.y - range.x;
    const bool own = sort_dkey != nullptr && nlist >= 2u && nlist <= kFwdSortCap;
    if (own) fwd_sort_list(U.srt, sv, s_val + range.x, nlist, sort_dkey, t);
    const uint32_t* const lsrc = own ? sv : s_val;
    const uint32_t loff = own ? range.x : 0u;
    uint64_t* bmask_out = band_mask + (size_t)chunk_base[tile] * 4u + wv;
    const float px = (float)x + 0.5f, py = (float)y + 0.5f;
    const float bx0 = (float)(tx * kTile + bxo) + 0.5f, bx1 = bx0 + (float)(kBandW - 1);
    const float by0 = (float)(ty * kTile + byo) + 0.5f, by1 = by0 + (float)(kBandH - 1);
    const uint64_t lt = lanemask_lt();
    FwdRec* R = U.q.recs[wv];
    uint32_t (*QL)[66] = U.q.qlist[wv];
    if (lane == 0) {  // the pad record: no pixel reaches it (power -inf), alpha 0 everywhere
        R[kQuadPad].a = make_float4(3.0e38f, 0.0f, 1.0f, 0.0f);
        R[kQuadPad].b = make_uint4(0u, 0u, 0u, 0u);
    }

    const _Float16 hEps = (_Float16)0.0001f;
    const _Float16 hAlphaMax = (_Float16)0.99f;
    const _Float16 hAlphaMin = (_Float16)(1.0f / 255.0f);
    const _Float16 hPowMin = (_Float16)(-4.5f);
    const _Float16 hZero = (_Float16)0.0f;
    const _Float16 hOne = (_Float16)1.0f;

    gs_h2 crg = (gs_h2)hZero;
    _Float16 cb = hZero, T = inside ? hOne : hZero;
    float Tf = 1.0f, Tsnap = 1.0f;
    uint32_t last = 0xffffffffu;
    bool tflag = false;

    float4 ra, rb, rc;
    float rk = 0.0f;
    auto fetch = [&](uint32_t idx, uint32_t v) {
        if (idx < range.y) {
            const float4* r = rec + (size_t)(v >> kPairJBits) * kRecQuads;
            ra = r[0];
            rb = r[1];
            rc = r[2];
            rk = r[3].y;
        }
    };
    auto entry = [&](uint32_t idx) { return idx < range.y ? lsrc[idx - loff] : 0u; };
    fetch(range.x + lane, entry(range.x + lane));
    uint32_t vnext = entry(range.x + 64u + lane);
    uint32_t work = 0, walked = 0;
    BSTAT_DECL
    BSTAT(0, 1);
    for (uint32_t base = range.x; base < range.y; base += 64u) {
        if (!__builtin_amdgcn_ballot_w64(T > hEps)) break;
        walked = min(base + 64u, range.y) - range.x;
        // cull this step's 64 records against the band's four quadrants; the band's mask for the
        // backward is their union
        uint32_t qm = 0;
        if (base + lane < range.y && box_hits(ra.x, ra.y, rc.y, rc.z, bx0, bx1, by0, by1))
            qm = ellipse_quads_hits_f32(ra.x, ra.y, ra.z, ra.w, rb.x, rk, rc.y, rc.z, bx0, by0);
        const uint64_t m = __ballot(qm != 0u);
        if (lane == 0) bmask_out[(size_t)((base - range.x) >> 6) * 4u] = m;  // for the backward
        if (qm) {
            FwdRec e;
            e.a = make_float4(ra.x, ra.y, ra.z, 2.0f * ra.w);  // the form's 2 cy, exact
            e.b = make_uint4(__float_as_uint(rb.x), __float_as_uint(rb.y),
                             pack_h2((_Float16)rb.z, (_Float16)rb.w),
                             pack_h2((_Float16)rc.x, rc.w < 0.0001f ? hZero : (_Float16)rb.y));
            R[lane] = e;  // (as two 16-B arrays, conflict-free stores: forward 0.3302 -> 0.3327 ms, not kept)
        }
        uint32_t nq[4];
#pragma unroll
        for (uint32_t q = 0; q < 4; q++) {
            const uint64_t mq = __builtin_amdgcn_ballot_w64((qm >> q) & 1u);
            nq[q] = (uint32_t)__popcll(mq);
            if ((qm >> q) & 1u) QL[q][__popcll(mq & lt)] = lane;
        }
        const uint32_t nsel = (uint32_t)__popcll(m);
        work += nsel;
        BSTAT(1, min(64u, range.y - base));
        BSTAT(2, nsel);
        BSTAT(6, 1);
        const uint32_t nmax = max(max(nq[0], nq[1]), max(nq[2], nq[3]));
        const uint32_t nown = grp == 0 ? nq[0] : (grp == 1 ? nq[1] : (grp == 2 ? nq[2] : nq[3]));
        const float tb = tfinal_track_bound(work);
        const float tlo = 0.0001f * (1.0f - tb), thi = 0.0001f * (1.0f + tb);
        fetch(base + 64u + lane, vnext);  // prefetch the next step while this one is blended
        vnext = entry(base + 128u + lane);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        const uint32_t* myq = QL[grp];
        // (reading the next pair's list positions one step ahead costs 5 spilled VGPRs at 8 waves per
        // SIMD: forward 0.333 -> 0.353 ms; 0.344 ms unbounded at 7 waves)
        for (uint32_t i = 0; i < nmax; i += kFwdStep) {
            const uint2 jj = *reinterpret_cast<const uint2*>(&myq[i]);
            const uint32_t jv[2] = {i < nown ? jj.x : kQuadPad, i + 1u < nown ? jj.y : kQuadPad};
            const FwdRec E[2] = {R[jv[0]], R[jv[1]]};
            float pw[2];
            _Float16 power[2];
            bool fin[2], hin[2];
            uint64_t range_mask = 0;
#pragma unroll
            for (int e = 0; e < 2; e++) {
                const float dx = px - E[e].a.x, dy = py - E[e].a.y;
                // -0.5 * (cx dx^2 + 2 cy dx dy + cz dy^2), left to right (:354-356)
                pw[e] = -0.5f * ((E[e].a.z * dx * dx + E[e].a.w * dx * dy) + __uint_as_float(E[e].b.x) * dy * dy);
                fin[e] = !(pw[e] > 0.0f || pw[e] < -4.5f);
                power[e] = (_Float16)pw[e];
                hin[e] = !(power[e] > hZero || power[e] < hPowMin);
                range_mask |= (__builtin_amdgcn_ballot_w64(!(pw[e] > 0.0f)) & __builtin_amdgcn_ballot_w64(!(pw[e] < -4.5f))) |
                              (__builtin_amdgcn_ballot_w64(!(power[e] > hZero)) &
                               __builtin_amdgcn_ballot_w64(!(power[e] < hPowMin)));
            }
            BSTAT(3, 1);
            if (!(__builtin_amdgcn_ballot_w64(T > hEps) & range_mask)) continue;
            BSTAT(4, 1);
#pragma unroll
            for (int e = 0; e < 2; e++) {
                const _Float16 G = (_Float16)__builtin_amdgcn_exp2f((float)power[e] * 1.44269504f);
                const float Gf = __builtin_amdgcn_exp2f(pw[e] * 1.44269504f);
                const float op = __uint_as_float(E[e].b.y);
                const bool alive = T > hEps;
                const bool live = alive && Tf > 0.0f && fin[e];
                float opg = op * Gf;
                if (live && fabsf(opg - 1.0f / 255.0f) <= 2e-6f * (1.0f / 255.0f)) opg = op * gs_expf_core(pw[e]);
                const float af = __builtin_amdgcn_fmed3f(opg, -1.0f, 0.99f);
                const bool okf = live && !(af < 1.0f / 255.0f);
                const float tt = Tf * (1.0f - af);
                const bool brk = okf && tt < thi;
                tflag = tflag || (brk && !(tt < tlo));
                Tf = okf ? (brk ? -Tf : tt) : Tf;
                const uint32_t bov = E[e].b.w;
                const _Float16 oph = __builtin_bit_cast(_Float16, (uint16_t)(bov >> 16));
                _Float16 alpha = oph * G;
                alpha = alpha < hAlphaMax ? alpha : hAlphaMax;
                const bool okh = alive && hin[e] && !(alpha < hAlphaMin);
                alpha = okh ? alpha : hZero;
                BSTAT(5, __popcll(__builtin_amdgcn_ballot_w64(okh)));
                const gs_h2 col_rg = __builtin_bit_cast(gs_h2, E[e].b.z);
                const _Float16 col_b = __builtin_bit_cast(_Float16, (uint16_t)(bov & 0xffffu));
                crg = crg + (col_rg * alpha) * T;
                cb = cb + (col_b * alpha) * T;
                T = T * (hOne - alpha);
                last = okh ? base + jv[e] : last;
                Tsnap = okh ? fabsf(Tf) : Tsnap;
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
    uint64_t fl = __builtin_amdgcn_ballot_w64(tflag && last != 0xffffffffu);
    while (fl) {
        const uint32_t f = (uint32_t)__builtin_ctzll(fl);
        fl &= fl - 1ull;
        const float Tx = tfinal_exact(readlane_f(px, f), readlane_f(py, f), range.x,
                                      (uint32_t)__builtin_amdgcn_readlane((int)last, f), rec, lsrc, loff, lane);
        if (lane == f) Tsnap = Tx;
    }
    BLEND_TRACE(0, 1);
    BSTAT_FLUSH(0);
    if (tile_cost && lane == 0 && work) atomicAdd(&tile_cost[tile], work);
    if (lane == 0) walk[tile * 4u + wv] = walked;
    if (!inside) return;
    const gs_h2 bgT = (gs_h2)(hOne * T);
    crg = crg + bgT;
    cb = cb + hOne * T;
    last_idx[pix] = last;
    t_final[pix] = Tsnap;
    const float fr = (float)crg.x, fg = (float)crg.y, fb = (float)cb;
    rgba8[pix] = quantize_unorm8(fr) | (quantize_unorm8(fg) << 8) | (quantize_unorm8(fb) << 16) |
                 (255u << 24);
    if (rgb) {
        rgb[3 * pix + 0] = fr;
        rgb[3 * pix + 1] = fg;
        rgb[3 * pix + 2] = fb;
    }
}

// ---------------------------------------------------------------------------------------
// Cross-lane reduction of the per-lane partial sums of a splat pair: 18 values v[j], j = 9e + q
// (splat e of the pair, partial q). Each stage halves the lanes a value is spread over while
// packing different values into different lane groups, so no lane ever adds a value it does not
// keep:
//   stage A  v_permlane32_swap: 9 registers, lanes 0-31 / 32-63 hold different values
//   stage B  v_permlane16_swap: 5 registers, the four 16-lane rows hold different values
//   stage C  select + DPP row_ror:8: 3 registers, the two 8-lane halves of a row hold different values
//   stage D  3 DPP steps (row_half_mirror, quad_perm) sum each 8-lane group
// Value j ends in register c = j / 8 of the 8-lane group g = bitrev3(j % 8) (all 8 lanes of the
// group hold it). 46 VALU per pair instead of 57 for the plain two-swap + four-DPP-step tree, and
// the 18 sums leave in one store instruction. The summation tree is fixed: deterministic.
template <int CTRL>
__device__ __forceinline__ float dpp_row_add(float v) {
    return v + __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xf, 0xf, true));
}

__device__ __forceinline__ float swap32_add(float a, float b) {
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(a), __float_as_uint(b), false, false);
    return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

__device__ __forceinline__ float swap16_add(float a, float b) {
    const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(a), __float_as_uint(b), false, false);
    return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

// stage C on a register pair: lanes 0-7 of each row keep a (+ the partner's a), lanes 8-15 keep b
__device__ __forceinline__ float swap8_add(float a, float b, bool lower) {
    const float send = lower ? b : a, keep = lower ? a : b;
    return keep + __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(send), 0x128, 0xf, 0xf, true));
}

__device__ __forceinline__ void reduce_pair(const float (&P)[2][9], float (&z)[3], bool lower) {
    float u[9];
#pragma unroll
    for (int a = 0; a < 9; a++) {
        const int j0 = 2 * a, j1 = 2 * a + 1;
        u[a] = swap32_add(P[j0 / 9][j0 % 9], P[j1 / 9][j1 % 9]);
    }
    float w[5];
#pragma unroll
    for (int b = 0; b < 4; b++) w[b] = swap16_add(u[2 * b], u[2 * b + 1]);
    w[4] = swap16_add(u[8], 0.0f);
    z[0] = swap8_add(w[0], w[1], lower);
    z[1] = swap8_add(w[2], w[3], lower);
    z[2] = swap8_add(w[4], 0.0f, lower);
#pragma unroll
    for (int c = 0; c < 3; c++) z[c] = dpp_row_add<0x141>(z[c]);  // row_half_mirror
#pragma unroll
    for (int c = 0; c < 3; c++) z[c] = dpp_row_add<0x4e>(z[c]);   // quad_perm [2,3,0,1]
#pragma unroll
    for (int c = 0; c < 3; c++) z[c] = dpp_row_add<0xb1>(z[c]);   // quad_perm [1,0,3,2]
}

constexpr int kBwdBands = 4;  // the 16x16 tile as four 64-pixel bands (the forward waves' bands)
__host__ __device__ constexpr uint32_t kBwdBandX0(uint32_t k) { return (k % (kTile / kBandW)) * kBandW; }
__host__ __device__ constexpr uint32_t kBwdBandY0(uint32_t k) { return (k / (kTile / kBandW)) * kBandH; }
constexpr int kBwdSlots = 64 + 2;
constexpr uint32_t kNoSlot = 0xffffffffu;

// Per-wave compacted splat list (reverse list order), structure-of-arrays for float2 pair loads.
struct alignas(8) BwdList {
    float sx[kBwdSlots], sy[kBwdSlots], c0[kBwdSlots], c1[kBwdSlots], c2[kBwdSlots], op[kBwdSlots];
    float cr[kBwdSlots], cg[kBwdSlots], cb[kBwdSlots];
    uint32_t slot[kBwdSlots];  // partial-sum slot (kNoSlot for the pad entry)
    uint32_t sidx[kBwdSlots];  // sorted-list index
    uint32_t mask[kBwdSlots];  // the bands that the splat reaches
};
static_assert(kBwdSlots % 2 == 0, "pair loads: every array 8-byte aligned");

// entry pair (i, i + 1), i even, of one of the list's arrays as one 8-byte LDS load: indexing an
// 8-byte-aligned view makes every field of the pair a ds_read_b64 off one address register
// (byte offsets up to 64 KB), instead of ds_read2_b32 pairs whose 1-KB offset reach needs a fresh
// base register per few fields
template <typename V, typename A>
__device__ __forceinline__ V pair_at(const A& arr, uint32_t i) {
    return reinterpret_cast<const V*>(arr)[i >> 1];
}

// List split (gs_set_backward_split): a job is a whole tile, or one part of a split tile's list --
// the chunks [cmid, nchunk) (back part, processed first by the reverse pass) or [0, cmid) (front
// quarter). The back-part wave stores its per-pixel state (T and the accumulated-colour sum A of
// the four bands) in kSplitStateWords 64-bit words, each carrying the frame tag in its high half
// (relaxed agent-scope atomics: the tag travels with the value, no fences), and the front-quarter
// wave, launched later, spins until every word it reads carries the current tag, then clears them
// (tag 0 is never a frame tag): a second backward of the same forward -- same tag -- eager or
// replayed from a HIP graph, waits for its own back part instead of reading this one's words, and
// no host-side state is involved. (Round 5 left the words and had the host clear them before a
// second backward of one forward, which a captured graph could not see. A device-side sequence
// number advanced by the launch's last split job instead cost the backward 0.39 -> 0.96 ms: every
// job's agent-scope load and atomic on the one word went to the memory side.) Launch positions: [0, S)
// back parts of the first S tiles of the order, [S, T) the remaining tiles whole, [T8, T8 + S)
// the front quarters (T8 = T rounded up to a multiple of 8). (A band split -- two waves per heavy tile, two 8x8 bands each, the second
// wave's sums in a second slot array -- duplicated the list walk and the pair reductions and was
// measured slower: 0.4575 -> 0.473 ms, chain +17 us.) Dispatch is in launch order within each XCD and back parts never wait, so every
// wait ends (bounded anyway: a give-up sets kFanInErrSplit in the frame's error word). Each list
// entry is still processed by exactly one wave with the same per-pixel operations in the same
// order, so the gradients are bit-identical to the unsplit pass; the jobs are shorter,
// which balances the kernel's tail (about two tiles per wave slot otherwise).
constexpr uint32_t kFanInErrSplit = 64u;
// the front part's share of a split list's chunks, in sixteenths (backward_kernel's measurements)
constexpr uint32_t kBwdFront16ths = 4;
__device__ __forceinline__ unsigned long long ld_agent_u64(const unsigned long long* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_agent_u64(unsigned long long* p, unsigned long long v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// One wave per tile (launch position blockIdx.x), one pixel of each of the four bands per lane.
// (Two waves per tile, two bands each with their own partial slots, measured slower: 0.489 ->
// 0.590 ms backward and 0.097 -> 0.146 ms chain, at 7 instead of 5 waves per SIMD.)
// (__launch_bounds__(64, 5) squeezes it into 96 VGPRs with spills: 0.482 -> 0.516 ms before the
// frame tags, 0.4575 -> 0.4598 ms after; (64, 6): 80 VGPRs + 36 spilled, 0.390 -> 0.401 ms, round 5)
constexpr int kBwdMinWaves = 4;
__global__ __launch_bounds__(64, kBwdMinWaves) void backward_kernel(
    uint32_t w, uint32_t h, uint32_t tiles_x, uint32_t num_tiles, const uint32_t* __restrict__ order,
    const float4* __restrict__ rec, const uint32_t* __restrict__ s_val, const uint32_t* __restrict__ goff,
    const uint2* __restrict__ ranges, const uint32_t* __restrict__ last_idx, const float* __restrict__ t_final,
    const uint32_t* __restrict__ rendered, const uint32_t* __restrict__ gt, float* __restrict__ partial,
    const uint32_t* __restrict__ chunk_base, const uint64_t* __restrict__ band_mask,
    const uint32_t* __restrict__ frame_tag, uint32_t nsplit,
    unsigned long long* __restrict__ split_state, uint32_t* __restrict__ split_err,
    reach_t* __restrict__ reached, uint32_t* __restrict__ walk) {
    __shared__ BwdList L;
    BLEND_TRACE(1, 0);
    const uint32_t tl = blockIdx.x;
    // launch position -> (position in the order, part: 0 whole tile, 1 back part, 2 front quarter):
    // [0, S) the back parts of the first S tiles of the order, [S, T) the other tiles whole,
    // [T8, T8 + S) the front quarters last, when their back parts have long finished (front quarters right after
    // the back parts waited on back parts that had just started: backward 0.396 -> 0.48-0.50 ms with
    // S = 2048 or 4096). nsplit > 0 only with an order (the host checks).
    // The front quarters start at T rounded up to a multiple of 8 (blocks [T, T8) are empty), so a
    // front quarter's launch position is congruent to its back part's modulo 8: both run on the XCD
    // of the tile's group (blocks b and b + 8 share an XCD) at every image size.
    const uint32_t t8 = (num_tiles + 7u) & ~7u;
    if (tl >= num_tiles && tl < t8) return;
    const uint32_t part = tl < nsplit ? 1u : (tl < num_tiles ? 0u : 2u);
    const uint32_t pos = tl < num_tiles ? tl : tl - t8;
    // wave-uniform: the tile's range, chunk base and band masks come in through scalar loads
    const uint32_t tile = __builtin_amdgcn_readfirstlane(order ? order[pos] : xcd_tile(pos, num_tiles));
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t tx = tile % tiles_x, ty = tile / tiles_x;
    const uint2 range = ranges[tile];
    constexpr int NB = kBwdBands;

    // The accumulated colour behind the splat (accum_rec, tiled_shaders.metal:470, 514) only enters
    // the gradients through dL/dalpha = T sum_c dl_c (c_c - accum_c): one float per pixel,
    // A = sum_c dl_c accum_c, recurred as A' = alpha D + (1 - alpha) A with D = sum_c dl_c c_c.
    // Three fewer recurrences per evaluation (6 VALU) and 8 fewer VGPRs per lane (94: five waves per
    // SIMD instead of four): backward 0.436 -> 0.399 ms. Its float drift stays within the gradient
    // bar (the conditioning class covers the dot product's cancellation; tests/_helpers.py).
    float T[NB], As[NB], dl[NB][3], pxk[NB], pyk[NB];
    uint32_t last[NB];
    uint32_t my_end = 0;
    // the four bands' pixel loads go out together (one round trip; pixels outside the image
    // read pixel 0 and are ignored)
    uint32_t li_[NB], rr_[NB], gg_[NB];
    float tf_[NB];
    bool in_[NB];
#pragma unroll
    for (int b = 0; b < NB; b++) {
        const uint32_t x = tx * kTile + kBwdBandX0((uint32_t)b) + lane % kBandW;
        const uint32_t y = ty * kTile + kBwdBandY0((uint32_t)b) + lane / kBandW;
        pxk[b] = (float)x + 0.5f;  // pixel centre (tiled_shaders.metal:328)
        pyk[b] = (float)y + 0.5f;
        in_[b] = x < w && y < h;
        const uint32_t pix = in_[b] ? y * w + x : 0u;
        li_[b] = last_idx[pix];
        tf_[b] = t_final[pix];
        rr_[b] = rendered[pix];
        gg_[b] = gt[pix];
    }
#pragma unroll
    for (int b = 0; b < NB; b++) {
        const bool act = in_[b] && li_[b] != 0xffffffffu;
        T[b] = act ? tf_[b] : 1.0f;
#pragma unroll
        for (int c = 0; c < 3; c++) {
            const float r = (float)((rr_[b] >> (8 * c)) & 0xffu) / 255.0f;
            const float t = (float)((gg_[b] >> (8 * c)) & 0xffu) / 255.0f;
            const float d = r - t;
            dl[b][c] = act ? (d > 0.0f ? 1.0f : (d < 0.0f ? -1.0f : 0.0f)) / 3.0f : 0.0f;
        }
        As[b] = (dl[b][0] + dl[b][1]) + dl[b][2];  // the background: accum = 1 in every channel
        if (act) my_end = max(my_end, li_[b] + 1u);
        // inactive (no pixel or no contribution): last = 0, an exclusive bound no list index
        // s >= range.x >= 0 is below; active: one past the pixel's last contributing entry
        last[b] = act ? li_[b] + 1u : 0u;
    }
    uint32_t end_max = __builtin_amdgcn_readfirstlane(wave_max_u32(my_end));
    if (end_max < range.x) end_max = range.x;
    if (part != 2u && lane == 0u) walk[4u * num_tiles + tile] = end_max - range.x;  // (work counter)
    // per band: one past the last list entry any of its 64 pixels still uses; splats beyond it
    // cannot touch the band (its pixels' reverse loops start below)
    uint32_t band_end[NB];
#pragma unroll
    for (int b = 0; b < NB; b++) band_end[b] = __builtin_amdgcn_readfirstlane(wave_max_u32(last[b]));

    BSTAT_DECL
    BSTAT(0, 1);
    BSTAT(3, range.y - end_max);
    // Slots this tile does not reach (beyond every pixel's last contributor, or culled from every
    // band) are not written: they keep an older frame tag, which the chain reads as zero.
    const uint32_t tag = *frame_tag;

    // this lane's share of a pair's 18 reduced sums: value j = 9e + q of register c = lane % 8
    // (< 3) in group g = lane / 8, j = 8c + bitrev3(g) (reduce_pair); the lanes of j = 18, 19 (pad
    // values) store the frame tag of slot 0, 1 (word 9)
    const bool lower = (lane & 15u) < 8u;
    const uint32_t rc_ = lane & 7u, rg_ = lane >> 3;
    const uint32_t rj = 8u * rc_ + (((rg_ & 1u) << 2) | (rg_ & 2u) | (rg_ >> 2));
    const bool rvalid = rc_ < 3u && rj < 20u;
    const bool rtag = rj >= 18u;
    const bool re = rtag ? rj == 19u : rj >= 9u;
    const uint32_t rq = rtag ? 9u : (re ? rj - 9u : rj);
    // this lane's store address is base + slot * stride: its tag word, or its float of the slot's run
    float* const rbase = partial + rq;  // (the tag lanes: word 9)
    constexpr uint32_t rstride = kSlotWords;

    const uint64_t gt_mask = lane == 63u ? 0ull : (~0ull << (lane + 1u));
    // The list is walked in the forward's 64-entry chunks (from the range start), last first, so
    // each chunk's band cull masks are the forward waves' ballots for the same records: no culling
    // math here. A band's mask is only read below its band_end, which its forward wave reached.
    const uint64_t* bm_tile = band_mask + (size_t)chunk_base[tile] * 4u;
    // Records of chunk c are prefetched one chunk ahead, its list entries (s_val) two chunks ahead,
    // so the record gathers never wait for the entry load that forms their address.
    float4 ra, rb, rc;
    uint32_t rgoff = 0, rpj = 0, rgid = 0;
    uint64_t rm[NB];
    auto entry = [&](uint32_t c) {
        const uint32_t lo_ = range.x + 64u * c;
        return lane < min(lo_ + 64u, end_max) - lo_ ? s_val[lo_ + lane] : 0u;
    };
    auto fetch = [&](uint32_t c, uint32_t v) {  // records of chunk c
        const uint32_t lo_ = range.x + 64u * c;
        if (lane < min(lo_ + 64u, end_max) - lo_) {
            const float4* r = rec + (size_t)(v >> kPairJBits) * kRecQuads;
            ra = r[0];
            rb = r[1];
            rc = r[2];
            // goff[gid]: on the global order read from goff (the offset scan's 4-B copies into 64-B record
            // lines cost more than this gather: config 5 offset scan 150 -> 81 us), on the per-tile
            // order the copy the tile scatter put into the record's quad 3 (no extra gather: bench
            // backward 623 vs 812 MB per launch)
            rgoff = goff ? goff[v >> kPairJBits] : __float_as_uint(r[3].x);
            rpj = v & kPairJMask;
            rgid = v >> kPairJBits;
        }
        const uint64_t* bm = bm_tile + (size_t)c * 4u;
#pragma unroll
        for (int b = 0; b < NB; b++) rm[b] = bm[b];
    };
    const uint32_t nchunk = end_max > range.x ? ((end_max - range.x - 1u) >> 6) + 1u : 0u;
    // this job's chunks [clo, chi): both parts of a split tile derive cmid from the same data
    // the front quarter of the chunks (the front entries cost more each: every pixel still
    // reaches them); measured on the bench frame: front 1/4 0.436 ms, 1/8 0.442, 3/8 0.450, 1/2 0.451,
    // 5/8 0.453, unsplit 0.452 (round 2); with the XCD-group order (round 3): 4/16 0.395, 3/16 0.415,
    // 5/16 0.406, 2/16 0.424, 6/16 0.416
    const uint32_t cmid = (nchunk * kBwdFront16ths) >> 4;
    const uint32_t clo = part == 1u ? cmid : 0u;
    uint32_t chi = part == 2u ? cmid : nchunk;
    unsigned long long* hand = split_state + (size_t)pos * kSplitStateWords;
    if (part == 2u) {  // the front quarter continues from the back part's per-pixel state
        unsigned long long v[2 * NB];
        uint32_t spins = 0;
        bool gave_up = false;
        for (;;) {
#pragma unroll
            for (int q = 0; q < 2 * NB; q++) v[q] = ld_agent_u64(hand + q * 64u + lane);
            bool ok = true;
#pragma unroll
            for (int q = 0; q < 2 * NB; q++) ok &= (uint32_t)(v[q] >> 32) == tag;
            if (__builtin_amdgcn_ballot_w64(!ok) == 0ull) break;
            if (++spins > (1u << 22)) {  // cannot happen (the back part never waits); reported, never a hang
                if (lane == 0) atomicOr(split_err, kFanInErrSplit);
                gave_up = true;
                break;
            }
            __builtin_amdgcn_s_sleep(2);
        }
        if (gave_up) {
            // process the whole list from the initial per-pixel state instead: the back part's
            // entries get the same values it writes (same operations, same order), so the result
            // stays exact; its words are left alone (they are its, not this pass's, to clear)
            chi = nchunk;
        } else {
#pragma unroll
            for (int b = 0; b < NB; b++) {
                T[b] = __uint_as_float((uint32_t)v[2 * b]);
                As[b] = __uint_as_float((uint32_t)v[2 * b + 1]);
            }
            // consumed: clear them, so the next backward of this forward waits for its own back part
#pragma unroll
            for (int q = 0; q < 2 * NB; q++) st_agent_u64(hand + q * 64u + lane, 0ull);
        }
    }
    uint32_t vnext = 0;
    if (chi > clo) fetch(chi - 1u, entry(chi - 1u));
    if (chi > clo + 1u) vnext = entry(chi - 2u);
    for (uint32_t c = chi; c-- > clo;) {
        const uint32_t lo = range.x + 64u * c;
        const uint32_t hi = min(lo + 64u, end_max);
        const uint32_t cnt = hi - lo;
        (void)cnt;
        const uint32_t rslot = rgoff + rpj;
        // the owning lane's band mask from the forward's ballots; culled splats get zero partials
        uint32_t bmask = 0;
#pragma unroll
        for (int b = 0; b < NB; b++)
            if (lo + lane < band_end[b] && ((rm[b] >> lane) & 1ull)) bmask |= 1u << b;
        const uint64_t sel = __ballot(bmask != 0);
        // compact the selected splats, highest list index first
        const uint32_t nsel = (uint32_t)__popcll(sel);
        BSTAT(1, cnt);
        BSTAT(2, nsel);
        BSTAT(10, 1);
        BSTAT(8, (nsel + 1u) / 2u);
        if (bmask) {
            const uint32_t o = (uint32_t)__popcll(sel & gt_mask);
            L.sx[o] = ra.x;
            L.sy[o] = ra.y;
            L.c0[o] = ra.z;
            L.c1[o] = 2.0f * ra.w;  // the form's 2 cy, exact (power-of-two scaling)
            L.c2[o] = rb.x;
            L.op[o] = rb.y;
            L.cr[o] = rb.z;
            L.cg[o] = rb.w;
            L.cb[o] = rc.x;
            L.slot[o] = rslot;
            L.sidx[o] = lo + lane;
            L.mask[o] = bmask;
            reached[rgid] = (reach_t)tag;  // the chain reads this Gaussian's slots
        }
        if ((nsel & 1u) && lane == 0) {  // pad to a pair with an entry that reaches no band
            L.sx[nsel] = 0.0f;
            L.sy[nsel] = 0.0f;
            L.c0[nsel] = 0.0f;
            L.c1[nsel] = 0.0f;
            L.c2[nsel] = 0.0f;
            L.op[nsel] = 0.0f;
            L.cr[nsel] = 0.0f;
            L.cg[nsel] = 0.0f;
            L.cb[nsel] = 0.0f;
            L.slot[nsel] = kNoSlot;
            L.sidx[nsel] = 0u;
            L.mask[nsel] = 0u;
        }
        if (c > clo) {  // prefetch the next (lower) chunk while this one is processed
            fetch(c - 1u, vnext);
            if (c > clo + 1u) vnext = entry(c - 2u);
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        // the entries' band masks in a register (lane o: entry o): the per-splat band branches read
        // them with v_readlane, no LDS round trip in front of every splat
        const uint32_t maskv = L.mask[lane];
        // a pair's fields (two entries per float2 load). Loading the next pair's during this one's
        // evaluation was measured slower (+22 VGPRs: 4 instead of 5 waves per SIMD, 0.486 -> 0.496 ms)
        struct PairFields {
            gs_f2 sx, sy, c0, c1, c2, op, cr, cg, cb;
            uint2 sidx;
        };
        auto load_pair = [&](uint32_t i, PairFields& F) {
            F.sx = pair_at<gs_f2>(L.sx, i);
            F.sy = pair_at<gs_f2>(L.sy, i);
            F.c0 = pair_at<gs_f2>(L.c0, i);
            F.c1 = pair_at<gs_f2>(L.c1, i);
            F.c2 = pair_at<gs_f2>(L.c2, i);
            F.op = pair_at<gs_f2>(L.op, i);
            F.cr = pair_at<gs_f2>(L.cr, i);
            F.cg = pair_at<gs_f2>(L.cg, i);
            F.cb = pair_at<gs_f2>(L.cb, i);
            F.sidx = pair_at<uint2>(L.sidx, i);
        };
        PairFields F;
        for (uint32_t i = 0; i < nsel; i += 2) {
            const uint32_t mk2[2] = {(uint32_t)__builtin_amdgcn_readlane((int)maskv, i),
                                     (uint32_t)__builtin_amdgcn_readlane((int)maskv, i + 1u)};
            load_pair(i, F);
            const gs_f2 sx2 = F.sx, sy2 = F.sy, c02 = F.c0, c12 = F.c1, c22 = F.c2, op2 = F.op;
            const gs_f2 cr2 = F.cr, cg2 = F.cg, cb2 = F.cb;
            const uint2 sidx2 = F.sidx;
            // the two splats one after the other (list order); their 9 sums stay per lane
            float P[2][9];
#ifdef GS_BLEND_STATS
            bool anyp = false;
#endif
#pragma unroll
            for (int e = 0; e < 2; e++) {
#pragma unroll
                for (int q = 0; q < 9; q++) P[e][q] = -0.0f;  // -0 + x == x: the first add folds away
                // the list entries are wave-uniform: band tests become scalar branches
                const uint32_t mk = mk2[e];
                if (!mk) continue;
                const float sx = e ? sx2.y : sx2.x, sy = e ? sy2.y : sy2.x;
                const float c0 = e ? c02.y : c02.x, c1 = e ? c12.y : c12.x, c2 = e ? c22.y : c22.x;
                const float op = e ? op2.y : op2.x;
                const float col[3] = {e ? cr2.y : cr2.x, e ? cg2.y : cg2.x, e ? cb2.y : cb2.x};
                const uint32_t sidx = e ? sidx2.y : sidx2.x;
#pragma unroll
                for (int k = 0; k < NB; k++) {
                    if (!((mk >> k) & 1u)) continue;
                    BSTAT(4, 1);
                    const float dx = pxk[k] - sx;
                    const float dy = pyk[k] - sy;
                    // power = -0.5 q; the scaling by -0.5 is exact, so the range tests run on q
                    // (power > 0 <=> q < 0, power < -4.5 <=> q > 9) and the exponent folds the
                    // -0.5 into its constant (rounding commutes with power-of-two scaling)
                    const float qf = c0 * dx * dx + c1 * dx * dy + c2 * dy * dy;
                    const bool inr = sidx < last[k] && !(qf < 0.0f || qf > 9.0f);
                    // wave-uniform skip; below it the pixel's update is branch-free, so the 9 sums
                    // need no per-path copies. (Ballots of the compares themselves: the lane mask
                    // stays in SGPRs, no bool round trip through a VGPR.)
                    if (!(__builtin_amdgcn_ballot_w64(sidx < last[k]) & __builtin_amdgcn_ballot_w64(!(qf < 0.0f)) &
                          __builtin_amdgcn_ballot_w64(!(qf > 9.0f))))
                        continue;
                    BSTAT(5, 1);
                    BSTAT(6, __popcll(__builtin_amdgcn_ballot_w64(inr)));
#ifdef GS_BLEND_STATS
                    anyp = true;
#endif
                    // G feeds gradient values, and one decision: alpha < 1/255. The hardware
                    // exp2 (v_exp_f32) is within 3.3e-7 of the pinned exp over this range
                    // (gs_debug_float_exp_check); only where op * G lies within 2e-6 (relative) of
                    // the threshold can the test differ, and there the pinned exp decides.
                    float G = __builtin_amdgcn_exp2f(qf * -0.72134752f);  // (-0.5 qf) * log2(e)
                    float opg = op * G;
                    if (inr && fabsf(opg - 1.0f / 255.0f) <= 2e-6f * (1.0f / 255.0f)) {
                        G = gs_expf_core(-0.5f * qf);
                        opg = op * G;
                    }
                    const float alpha = __builtin_amdgcn_fmed3f(opg, -1.0f, 0.99f);  // min(opg, 0.99), opg >= 0
                    const bool cb = inr && !(alpha < 1.0f / 255.0f);
                    BSTAT(7, __popcll(__builtin_amdgcn_ballot_w64(cb)));
                    // a non-contributing pixel gets alpha 0: T, acc and weight then keep their values
                    // exactly (rcp(1) = 1, fma(0, d, a) = a, 0 * T = 0) without selects
                    const float ac = cb ? alpha : 0.0f;
                    const float oma = 1.0f - ac;
                    // T feeds gradient values only (no decision): v_rcp instead of IEEE division
                    // (the reference's max(1 - alpha, 1e-4) never binds: alpha <= 0.99)
                    const float Tn = T[k] * __builtin_amdgcn_rcpf(oma);
                    T[k] = Tn;
                    // Gradient terms only (no decision depends on them): fused multiply-adds are
                    // fine here; the reference's own float atomics reassociate these sums anyway.
                    float Dc = dl[k][0] * col[0];
                    Dc = __builtin_fmaf(dl[k][1], col[1], Dc);
                    Dc = __builtin_fmaf(dl[k][2], col[2], Dc);
                    const float dd = Dc - As[k];
                    As[k] = __builtin_fmaf(ac, Dc, oma * As[k]);
                    const float weight = ac * Tn;
                    const float wg = cb ? (Tn * dd) * G : 0.0f;  // dL/dalpha * G
                    const float wdx = wg * dx, wdy = wg * dy;
                    P[e][0] = __builtin_fmaf(dl[k][0], weight, P[e][0]);
                    P[e][1] = __builtin_fmaf(dl[k][1], weight, P[e][1]);
                    P[e][2] = __builtin_fmaf(dl[k][2], weight, P[e][2]);
                    P[e][3] += wg;
                    P[e][4] += wdx;
                    P[e][5] += wdy;
                    P[e][6] = __builtin_fmaf(wdx, dx, P[e][6]);
                    P[e][7] = __builtin_fmaf(wdx, dy, P[e][7]);
                    P[e][8] = __builtin_fmaf(wdy, dy, P[e][8]);
                }
            }
#ifdef GS_BLEND_STATS
            if (!anyp) BSTAT(9, 1);
#endif
            float z[3];
            reduce_pair(P, z, lower);
            // one store instruction for the pair's 18 sums (two runs of 9 contiguous floats) and the
            // two slots' frame tags
            const uint2 slot = pair_at<uint2>(L.slot, i);
            const uint32_t sl = re ? slot.y : slot.x;
            const float val = rtag ? __uint_as_float(tag) : (rc_ == 0u ? z[0] : (rc_ == 1u ? z[1] : z[2]));
            float* dst = rbase + (size_t)sl * rstride;
            if (rvalid && sl != kNoSlot) *dst = val;
        }
        // every lane has consumed the list before the next chunk overwrites it
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
    if (part == 1u) {  // hand the per-pixel state to the front quarter (tag in every word)
        const unsigned long long tg = (unsigned long long)tag << 32;
#pragma unroll
        for (int b = 0; b < NB; b++) {
            st_agent_u64(hand + (2 * b) * 64u + lane, tg | __float_as_uint(T[b]));
            st_agent_u64(hand + (2 * b + 1) * 64u + lane, tg | __float_as_uint(As[b]));
        }
    }
    BSTAT_FLUSH(16);
    BLEND_TRACE(1, 1);
}

// ---- launchers --------------------------------------------------------------------------
// Exhaustive check behind the forward's hardware half exp: for every half power h in [-4.5, 0] (all
// the forward's weight inputs that reach a pixel), does the hardware path the forward uses,
// half(v_exp_f32(float(h) * log2 e)), round to the same half as half(gs_expf_core(float(h)))?
// out[0] = mismatches, out[1] = largest float ulp distance between the two exps.
__global__ __launch_bounds__(256) void half_exp_check_kernel(uint32_t* __restrict__ out) {
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    const _Float16 hv = __builtin_bit_cast(_Float16, (uint16_t)i);
    if (!(hv <= (_Float16)0.0f && hv >= (_Float16)-4.5f)) return;
    const float pf = (float)hv;
    const float hw = __builtin_amdgcn_exp2f(pf * 1.44269504f);
    const float pin = gs_expf_core(pf);
    const int32_t d = (int32_t)__float_as_uint(hw) - (int32_t)__float_as_uint(pin);
    atomicMax(&out[1], (uint32_t)(d < 0 ? -d : d));
    if (__builtin_bit_cast(uint16_t, (_Float16)hw) != __builtin_bit_cast(uint16_t, (_Float16)pin))
        atomicAdd(&out[0], 1u);
}

// Exhaustive check behind kExpRelErr: over every float power x in [-4.5, 0] (all the T_final
// track's and the backward's weight inputs that reach a pixel), the largest relative difference
// between the hardware path v_exp_f32(x * log2 e) and the pinned exp gs_expf_core(x), as float bits
// (non-negative floats order as unsigned integers). Grid-stride over the 0x80000000..0xc0900000
// bit patterns (-0 .. -4.5; +0 gives 1 on both paths).
__global__ __launch_bounds__(256) void float_exp_check_kernel(uint32_t* __restrict__ out) {
    constexpr uint32_t lo = 0x80000000u, hi = 0xc0900000u;
    float worst = 0.0f;
    for (uint32_t b = lo + blockIdx.x * 256u + threadIdx.x; b <= hi && b >= lo; b += gridDim.x * 256u) {
        const float x = __uint_as_float(b);
        const float hw = __builtin_amdgcn_exp2f(x * 1.44269504f);
        const float pin = gs_expf_core(x);
        worst = fmaxf(worst, fabsf(hw - pin) / pin);
    }
    const uint32_t wmax = wave_max_u32(__float_as_uint(worst));
    if ((threadIdx.x & 63u) == 0u) atomicMax(out, wmax);
}

hipError_t launch_float_exp_check(hipStream_t st, uint32_t* d_out) {
    hipError_t e = hipMemsetAsync(d_out, 0, sizeof(uint32_t), st);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(float_exp_check_kernel, dim3(16384), dim3(256), 0, st, d_out);
    return hipGetLastError();
}

hipError_t launch_half_exp_check(hipStream_t st, uint32_t* d_out) {
    hipError_t e = hipMemsetAsync(d_out, 0, 2 * sizeof(uint32_t), st);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(half_exp_check_kernel, dim3(65536 / 256), dim3(256), 0, st, d_out);
    return hipGetLastError();
}

hipError_t launch_forward(hipStream_t st, const LaunchGeom& geo, const GsTiledUniforms& u,
                          const GaussianBuffers& gb, const PairBuffers& pb, const uint2* ranges,
                          const uint32_t* p_dev, const PixelBuffers& px, uint32_t* rgba8,
                          float* rgb) {
    (void)u;
    hipLaunchKernelGGL(forward_quad_kernel, dim3(geo.num_tiles), dim3(kFwdThreads), 0, st, geo.w,
                       geo.h, geo.tiles_x, geo.num_tiles, geo.tile_order, gb.rec, pb.s_val,
                       ranges, p_dev, px.last_idx, px.t_final, rgba8, rgb, geo.chunk_base, geo.band_mask,
                       geo.tile_cost, geo.fwd_sort_dkey, geo.walk);
    return hipGetLastError();
}

hipError_t launch_backward(hipStream_t st, const LaunchGeom& geo, const GsTiledUniforms& u,
                           const GaussianBuffers& gb, const PairBuffers& pb,
                           const uint2* ranges, const PixelBuffers& px, const uint32_t* rendered,
                           const uint32_t* gt) {
    (void)u;
    const uint32_t* order = geo.bwd_order ? geo.bwd_order : geo.tile_order;
    const uint32_t nsplit = (order && geo.split_state) ? std::min(geo.split_tiles, geo.num_tiles) : 0u;
    // front quarters at [T8, T8 + S), T8 = T rounded up to a multiple of 8 (backward_kernel)
    const uint32_t grid = nsplit ? ((geo.num_tiles + 7u) & ~7u) + nsplit : geo.num_tiles;
    hipLaunchKernelGGL(backward_kernel, dim3(grid), dim3(64), 0, st, geo.w, geo.h, geo.tiles_x,
                       geo.num_tiles, order, gb.rec, pb.s_val, geo.goff_direct ? gb.goff : nullptr,
                       ranges, px.last_idx, px.t_final, rendered, gt, pb.partial, geo.chunk_base, geo.band_mask,
                       geo.frame_tag, nsplit, geo.split_state, geo.split_err, gb.reached,
                       geo.walk);
    return hipGetLastError();
}

}  // namespace gs
