// gs_chain.hip — per-Gaussian gradient chain of tiledBackward (tiled_shaders.metal:517-736).
//
// Everything after dL/dconic, dL/dscreen, dL/dcolour and dL/dopacity is linear with
// per-Gaussian coefficients, so the backward blend only reduces 9 partial sums per
// (tile, Gaussian) slot and this kernel applies the chain once per Gaussian:
//   S0..2 = sum dL/dpixel_c * alpha * T          (colour)
//   S3    = sum w,  w = dL/dalpha * G             (raw opacity: * sig (1 - sig))
//   S4,S5 = sum w dx, sum w dy                    (screen position: * sig * conic)
//   S6..8 = sum w dx^2, w dx dy, w dy^2           (conic: * -sig/2, -sig, -sig/2)
// One thread per Gaussian sums its current-frame slots (frame tag, gs_internal.hpp
// kScalarFrameTag) in slot order (deterministic, no atomics). (Summing the Gaussians with more than
// 24 slots by a whole wave each, against the per-thread loop's imbalance, was measured slower:
// config 5 chain 0.74 -> 1.52 ms.) The sums and the chain are evaluated in fp64: the
// conic -> cov2D -> Sigma -> (scale, quaternion) chain cancels heavily for near-degenerate
// covariances, and fp64 costs nothing at N threads.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "gs_adam.hpp"
#include "gs_device.hpp"
#include "gs_internal.hpp"

namespace gs {

// Gradient rows (include/gs_rasterizer.h GS_GRAD_ROW_FLOATS, 56 B per Gaussian; what the RCCL
// reduction moves): [0..2] position [3] opacity [4..6] log-scale [7..10] rotation [11] sh0 [12] sh4
// [13] sh8. A row starts 8-B aligned (56 i), so it is written as seven 8-B stores; the per-view
// viewspace gradient (not reduced, density statistics only) as one 8-B store into its own rows.
__device__ __forceinline__ void store_rows(float* __restrict__ rows, float* __restrict__ vs, uint32_t i,
                                           const float* out) {
    float2* dst = reinterpret_cast<float2*>(rows + (size_t)i * kGradRowFloats);
    dst[0] = make_float2(out[0], out[1]);
    dst[1] = make_float2(out[2], out[3]);
    dst[2] = make_float2(out[4], out[5]);
    dst[3] = make_float2(out[6], out[8]);
    dst[4] = make_float2(out[9], out[10]);
    dst[5] = make_float2(out[11], out[12]);
    dst[6] = make_float2(out[16], out[20]);
    if (vs) reinterpret_cast<float2*>(vs)[i] = make_float2(out[24], out[25]);
}

// The chain from the nine summed partials to the 16 gradient fields (tiled_shaders.metal:503-696),
// in fp64; out[] keeps zeros when every sum is zero.
__device__ __forceinline__ void chain_apply(const GaussianIn& gin, const GsTiledUniforms& u, const double (&S)[9],
                                            float (&out)[28]) {
    bool nz = false;
#pragma unroll
    for (int q = 0; q < 9; q++) nz |= S[q] != 0.0;
    if (nz) {
        Projected p;
        project(gin, u, p);  // bit-identical to the forward's projection
        const double sig = p.opacity;
        const double SH = (double)kShC0;
        // colour (tiled_shaders.metal:503-507, 699-704)
        out[12] = (p.r <= 0.01f || p.r >= 0.99f) ? 0.0f : (float)(S[0] * SH);
        out[16] = (p.g <= 0.01f || p.g >= 0.99f) ? 0.0f : (float)(S[1] * SH);
        out[20] = (p.b <= 0.01f || p.b >= 0.99f) ? 0.0f : (float)(S[2] * SH);
        // raw opacity (:517-519)
        out[3] = (float)(S[3] * (sig * (1.0 - sig)));
        // screen position (:528-536)
        const double c0 = p.c0, c1 = p.c1, c2 = p.c2;
        const double dSx = sig * (c0 * S[4] + c1 * S[5]);
        const double dSy = sig * (c2 * S[5] + c1 * S[4]);
        out[24] = (float)dSx;
        out[25] = (float)dSy;
        // view -> world position with unclamped tx/tz and no cov-through-mean term (:540-565)
        const double fx = u.focal[0], fy = u.focal[1];
        const double z = p.depth;
        const double txtz = (double)p.vx / z, tytz = (double)p.vy / z;
        const double dV[3] = {dSx * fx / z, dSy * fy / z, -dSx * fx * txtz / z - dSy * fy * tytz / z};
        Mat3d W;
#pragma unroll
        for (int a = 0; a < 3; a++)
#pragma unroll
            for (int b = 0; b < 3; b++) W.c[a][b] = u.view[a * 4 + b];
#pragma unroll
        for (int a = 0; a < 3; a++) out[a] = (float)(W.c[a][0] * dV[0] + W.c[a][1] * dV[1] + W.c[a][2] * dV[2]);
        // conic -> cov2D, off-diagonal doubled as in the reference (:570-596)
        const double dCo0 = -0.5 * sig * S[6];
        const double dCo1 = -sig * S[7];
        const double dCo2 = -0.5 * sig * S[8];
        const double ca = p.ca, cb = p.cb, cc = p.cc;
        const double den = ca * cc - cb * cb;
        const double d2i = 1.0 / (den * den + 1e-7);
        const double dCx = d2i * (-cc * cc * dCo0 + 2.0 * cb * cc * dCo1 + (den - ca * cc) * dCo2);
        const double dCz = d2i * (-ca * ca * dCo2 + 2.0 * ca * cb * dCo1 + (den - ca * cc) * dCo0);
        const double dCy = d2i * 2.0 * (cb * cc * dCo0 - (den + 2.0 * cb * cb) * dCo1 + ca * cb * dCo2);
        // cov2D -> Sigma3D = T^T dC T, T = J W (:602-631)
        Mat3d J = {};
        J.c[0][0] = fx / z;
        J.c[2][0] = -fx * txtz / z;
        J.c[1][1] = fy / z;
        J.c[2][1] = -fy * tytz / z;
        const Mat3d Tm = mul(J, W);
        Mat3d D = {};
        D.c[0][0] = dCx; D.c[0][1] = dCy;
        D.c[1][0] = dCy; D.c[1][1] = dCz;
        Mat3d dC3 = mul(mul(transpose(Tm), D), Tm);
        // T^T D T is symmetric; the two triangles round differently in the products above, and
        // for an isotropic Gaussian at identity rotation (every COLMAP-initialised one) the
        // quaternion gradient is exactly their difference: the reference's float terms are
        // exactly 0 there, so take one symmetric value instead of leaving 1e-16-relative residue
#pragma unroll
        for (int a = 0; a < 3; a++)
#pragma unroll
            for (int b = a + 1; b < 3; b++) {
                const double t = 0.5 * (dC3.c[a][b] + dC3.c[b][a]);
                dC3.c[a][b] = t;
                dC3.c[b][a] = t;
            }
        // Sigma3D -> log-scale and the raw (un-normalised) quaternion, no 20:1 clamp (:635-696)
        const double s0 = gs_expf(clampf(gin.sx, -kMaxLogScale, kMaxLogScale));
        const double s1 = gs_expf(clampf(gin.sy, -kMaxLogScale, kMaxLogScale));
        const double s2 = gs_expf(clampf(gin.sz, -kMaxLogScale, kMaxLogScale));
        const double qr = gin.qw, qx = gin.qx, qy = gin.qy, qz = gin.qz;
        Mat3d R;
        R.c[0][0] = 1.0 - 2.0 * (qy * qy + qz * qz);
        R.c[0][1] = 2.0 * (qx * qy + qr * qz);
        R.c[0][2] = 2.0 * (qx * qz - qr * qy);
        R.c[1][0] = 2.0 * (qx * qy - qr * qz);
        R.c[1][1] = 1.0 - 2.0 * (qx * qx + qz * qz);
        R.c[1][2] = 2.0 * (qy * qz + qr * qx);
        R.c[2][0] = 2.0 * (qx * qz + qr * qy);
        R.c[2][1] = 2.0 * (qy * qz - qr * qx);
        R.c[2][2] = 1.0 - 2.0 * (qx * qx + qy * qy);
        const double sc[3] = {s0, s1, s2};
        Mat3d M;
#pragma unroll
        for (int a = 0; a < 3; a++)
#pragma unroll
            for (int b = 0; b < 3; b++) M.c[a][b] = R.c[a][b] * sc[a];
        Mat3d dC3x2;
#pragma unroll
        for (int a = 0; a < 3; a++)
#pragma unroll
            for (int b = 0; b < 3; b++) dC3x2.c[a][b] = 2.0 * dC3.c[a][b];
        const Mat3d dM = mul(dC3x2, M);
        const Mat3d RtdM = mul(transpose(R), dM);
        out[4] = (float)(RtdM.c[0][0] * s0);
        out[5] = (float)(RtdM.c[1][1] * s1);
        out[6] = (float)(RtdM.c[2][2] * s2);
        Mat3d dR;
#pragma unroll
        for (int a = 0; a < 3; a++)
#pragma unroll
            for (int b = 0; b < 3; b++) dR.c[a][b] = dM.c[a][b] * sc[a];
        const Mat3d m = transpose(dR);
        out[8] = (float)(2.0 * (qz * (m.c[0][1] - m.c[1][0]) + qy * (m.c[2][0] - m.c[0][2]) +
                                qx * (m.c[1][2] - m.c[2][1])));
        out[9] = (float)(2.0 * (qy * (m.c[1][0] + m.c[0][1]) + qz * (m.c[2][0] + m.c[0][2]) +
                                qr * (m.c[1][2] - m.c[2][1]) - 2.0 * qx * (m.c[2][2] + m.c[1][1])));
        out[10] = (float)(2.0 * (qx * (m.c[1][0] + m.c[0][1]) + qr * (m.c[2][0] - m.c[0][2]) +
                                 qz * (m.c[1][2] + m.c[2][1]) - 2.0 * qy * (m.c[2][2] + m.c[0][0])));
        out[11] = (float)(2.0 * (qr * (m.c[0][1] - m.c[1][0]) + qx * (m.c[2][0] + m.c[0][2]) +
                                 qy * (m.c[1][2] + m.c[2][1]) - 2.0 * qz * (m.c[1][1] + m.c[0][0])));
    }
}

__device__ __forceinline__ void chain_store(uint32_t i, const float (&out)[28], GsGradients* __restrict__ grad,
                                            float* __restrict__ rows, float* __restrict__ vs) {
    if (rows) {
        store_rows(rows, vs, i, out);
        return;
    }
    float4* dst = reinterpret_cast<float4*>(grad + i);
#pragma unroll
    for (int q = 0; q < 7; q++) dst[q] = make_float4(out[4 * q], out[4 * q + 1], out[4 * q + 2], out[4 * q + 3]);
}

// The sums of Gaussian i's current-frame slots (slots the backward did not reach this frame carry
// an older tag and count as zero) and its chain, in fp64, into out[] (zeros where every sum is zero).
// Blocks of kB slots: the whole tagged 40-B slots are loaded at once and a stale slot's sums dropped
// after the load, one round trip per block. (Reading the tags first and then only the current slots'
// sums -- round 5's compacting chain, where most slots were stale -- was slower on config 5's reached
// Gaussians, whose slots are mostly current: 279 against 260 us per frame.)
__device__ __forceinline__ void chain_gaussian(const GsGaussian* gsrc, uint32_t i, const GsTiledUniforms& u,
                                               const uint32_t* __restrict__ count, const uint32_t* __restrict__ goff,
                                               const float* __restrict__ partial, const float* __restrict__ zero9,
                                               uint32_t tag, float (&out)[28]) {
    // the Gaussian record's loads go out with the partial sums' (independent latencies)
    const GaussianIn gin = load_gaussian(gsrc, i);
    const uint32_t c = count[i];
    const uint32_t o = goff[i];
    double S[9];
#pragma unroll
    for (int q = 0; q < 9; q++) S[q] = 0.0;
    constexpr uint32_t kB = 4;  // (tagged slots, bench chain: 3 / 4 / 6 / 8 slots 102.5 / 97.3 / 99.7 / 103.7 us)
    for (uint32_t e = o; e < o + c; e += kB) {
        float2 v[5 * kB];
#pragma unroll
        for (uint32_t k = 0; k < kB; k++) {
            const float2* src = reinterpret_cast<const float2*>(partial + (size_t)min(e + k, o + c - 1u) * kSlotWords);
#pragma unroll
            for (int q = 0; q < 5; q++) v[5 * k + q] = src[q];
        }
#pragma unroll
        for (uint32_t k = 0; k < kB; k++) {
            const bool cur = e + k < o + c && __float_as_uint(v[5 * k + 4].y) == tag;
#pragma unroll
            for (int q = 0; q < 9; q++) {
                const float x = (q & 1) ? v[5 * k + q / 2].y : v[5 * k + q / 2].x;
                S[q] += cur ? (double)x : 0.0;
            }
        }
    }
    chain_apply(gin, u, S, out);
}

// What happens to one Gaussian's gradient: stored (as a 56-B row + viewspace, or a GaussianGradients
// record), or, with kStep (gs_backward_step), fed to the density statistics and to Adam on the
// Gaussian itself (gs_adam.hpp: the same arithmetic as gs_density_accumulate_rows +
// gs_adam_step_rows, so the same bits), skipping the 64-B row write and read-back, the separate
// kernels' Gaussian re-read and two launches. Each Gaussian is read and updated by the one thread
// that owns it, after its chain has read it; in this mode the Gaussians are read through step.g
// (written by Adam), never through the restrict-qualified `g` of the kernels, which is then unused.
template <bool kStep>
__device__ __forceinline__ void chain_finish(uint32_t i, const float (&o)[28], GsGradients* __restrict__ grad,
                                             float* __restrict__ rows, float* __restrict__ vs, const ChainStep& step) {
    if constexpr (kStep) {
        if (step.accum) density_accumulate_one(step.accum, step.dcount, step.pos_accum, i, o[0], o[1], o[2], o[24], o[25]);
        adam_update(step.g, i, o, step.m, step.v, step.P);
    } else {
        chain_store(i, o, grad, rows, vs);
    }
}

// The plain chain (scenes where most Gaussians are reached, e.g. the bench frame): one thread per
// Gaussian; an unreached one (its list entries never selected: only stale slots) gets a zero
// gradient without reading its slots' tags or its record.
template <bool kStep>
__global__ __launch_bounds__(256) void chain_kernel(
    const GsGaussian* __restrict__ g, uint32_t n, GsTiledUniforms u,
    const uint32_t* __restrict__ count, const uint32_t* __restrict__ goff,
    const float* __restrict__ partial, const float* __restrict__ zero9,
    GsGradients* __restrict__ grad, float* __restrict__ rows, float* __restrict__ vs, uint32_t first, uint32_t end,
    const uint32_t* __restrict__ frame_tag, const reach_t* __restrict__ reached, ChainStep step) {
    const uint32_t i = first + blockIdx.x * 256u + threadIdx.x;
    if (i >= end || i >= n) return;
    const uint32_t tag = *frame_tag;
    float out[28];
#pragma unroll
    for (int q = 0; q < 28; q++) out[q] = 0.0f;
    if (count[i] != 0u && reached[i] == (reach_t)tag)
        chain_gaussian(kStep ? step.g : g, i, u, count, goff, partial, zero9, tag, out);
    chain_finish<kStep>(i, out, grad, rows, vs, step);
}

// The compacting path (scenes where most Gaussians are not reached, e.g. config 5: 160k of 5.2M
// reached, their 3.8M of the 69M slots), in two launches (round 6) over disjoint sets:
//   chain_screen_kernel  one thread per Gaussian. The "still" ones -- unreached (zero gradient) and,
//                        with kStep, with zero moments and zero cold lanes, for which Adam reduces
//                        exactly to the clamps and the renormalisation (adam_update_still); without
//                        kStep every unreached one, its zero gradient stored -- are finished here, a
//                        streaming pass at low register pressure (with kStep every Gaussian's record
//                        is loaded with its flags: one round trip). The others are listed per
//                        workgroup (ballot order) in `list` [block * 256 + k], their number in
//                        `lcount` [block].
//   chain_list_kernel    one thread per listed Gaussian (a workgroup takes kListBlocks screen blocks'
//                        lists): sums, chain, and the store or the density statistics + Adam. All
//                        listed Gaussians are in flight at once, one per thread, so their slot
//                        gathers' round trips overlap across the grid.
// Round 5 did both in one 512-thread kernel that compacted the reached ones of each workgroup into
// its first threads: a workgroup's ~15 reached Gaussians (3 %) kept it resident through one nearly
// empty wave's slot gathers and fp64 chain, and the fused tail moved its 1.0 GB at 1.76 TB/s (0.57 ms
// per config-5 frame); a first round-6 version compacted 8192 Gaussians per workgroup but still ran
// each thread's 1-3 chains one after another at 2 waves per SIMD (0.41 ms).
// is Gaussian i finished by the screen pass? (kStep: `cold` = the optimizer's cold word or flag)
// (The live unreached Gaussians are stepped by the list pass: doing their Adam -- moments to decay --
// in the screen pass instead raised its registers to ~120 and measured screen 133 -> 239 us, list
// 197 -> 154 us per config-5 frame; listing them apart for a third kernel, Adam alone, measured list
// 153 + decay 58 us against list 195 us: no gain.)
template <bool kStep>
__device__ __forceinline__ bool chain_still(bool heavy, bool cold, const ChainStep& step, uint32_t i) {
    if constexpr (kStep) return !heavy && !cold && step.P.live && step.P.live[i] == 0u;
    return !heavy;
}

template <bool kStep>
__device__ __forceinline__ bool step_cold(const ChainStep& step) {
    if constexpr (kStep) return step.P.cold != 0u || (step.P.cold_word && *step.P.cold_word != 0u);
    return false;
}

template <bool kStep>
__global__ __launch_bounds__(256) void chain_screen_kernel(
    uint32_t n, const uint32_t* __restrict__ count, GsGradients* __restrict__ grad, float* __restrict__ rows,
    float* __restrict__ vs, uint32_t first, uint32_t end, const uint32_t* __restrict__ frame_tag,
    const reach_t* __restrict__ reached, ChainStep step, uint32_t* __restrict__ list, uint32_t* __restrict__ lcount) {
    __shared__ uint32_t s_w[4];
    const uint32_t t = threadIdx.x, w = t >> 6, lane = t & 63u;
    const uint32_t i = first + blockIdx.x * 256u + t;
    const bool valid = i < end && i < n;
    float4 g0[7];
    if constexpr (kStep) {  // (the record's loads go out with the flags': screen 133 -> 125 us at config 5)
        const float4* gp = reinterpret_cast<const float4*>(step.g + (valid ? i : first));
#pragma unroll
        for (int q = 0; q < 7; q++) g0[q] = gp[q];
    }
    const bool heavy = valid && count[i] != 0u && reached[i] == (reach_t)*frame_tag;
    const bool still = valid && chain_still<kStep>(heavy, step_cold<kStep>(step), step, i);
    const bool listed = valid && !still;
    const uint64_t m = __ballot(listed);
    if (lane == 0) s_w[w] = (uint32_t)__popcll(m);
    __syncthreads();
    const uint32_t c0 = s_w[0], c1 = s_w[1], c2 = s_w[2];
    if (listed) {
        const uint32_t off = (w > 0 ? c0 : 0u) + (w > 1 ? c1 : 0u) + (w > 2 ? c2 : 0u);
        list[blockIdx.x * 256u + off + (uint32_t)__popcll(m & lanemask_lt())] = i;
    }
    if (t == 0) lcount[blockIdx.x] = c0 + c1 + c2 + s_w[3];
    if (!still) return;
    if constexpr (kStep) {
        // (a zero gradient adds nothing to the density statistics: its magnitude is 0)
        adam_still_from(reinterpret_cast<float4*>(step.g + i), g0);
    } else {
        float zero[28];
#pragma unroll
        for (int q = 0; q < 28; q++) zero[q] = 0.0f;
        chain_store(i, zero, grad, rows, vs);
    }
}

constexpr uint32_t kListBlocksMax = 16;  // screen blocks (of 256 Gaussians) per list workgroup, at most
constexpr uint32_t kListThreads = 128;

template <bool kStep>
// (at 3 waves per SIMD: 168 VGPRs and a 16-B spill; unbounded, 211 VGPRs and 2 waves, the config-5
// list pass took 217 instead of 191 us)
__global__ __launch_bounds__(kListThreads, 3) void chain_list_kernel(
    const GsGaussian* __restrict__ g, GsTiledUniforms u, const uint32_t* __restrict__ count,
    const uint32_t* __restrict__ goff, const float* __restrict__ partial, const float* __restrict__ zero9,
    GsGradients* __restrict__ grad, float* __restrict__ rows, float* __restrict__ vs, uint32_t nblocks,
    uint32_t lblocks, const uint32_t* __restrict__ frame_tag, const reach_t* __restrict__ reached, ChainStep step,
    const uint32_t* __restrict__ list, const uint32_t* __restrict__ lcount) {
    __shared__ uint32_t s_pre[kListBlocksMax + 1];
    const uint32_t t = threadIdx.x;
    const uint32_t b0 = blockIdx.x * lblocks;
    if (t == 0) {
        uint32_t run = 0;
        for (uint32_t k = 0; k < kListBlocksMax; k++) {
            s_pre[k] = run;
            run += k < lblocks && b0 + k < nblocks ? lcount[b0 + k] : 0u;
        }
        s_pre[kListBlocksMax] = run;
    }
    __syncthreads();
    const uint32_t total = s_pre[kListBlocksMax];
    const uint32_t tag = *frame_tag;
    for (uint32_t k = t; k < total; k += kListThreads) {
        uint32_t c = 0;
#pragma unroll
        for (uint32_t q = 1; q < kListBlocksMax; q++) c += k >= s_pre[q] ? 1u : 0u;
        const uint32_t i = list[(b0 + c) * 256u + (k - s_pre[c])];
        float out[28];
#pragma unroll
        for (int q = 0; q < 28; q++) out[q] = 0.0f;
        if (count[i] != 0u && reached[i] == (reach_t)tag)  // (else: kStep, unreached, moments to decay)
            chain_gaussian(kStep ? step.g : g, i, u, count, goff, partial, zero9, tag, out);
        chain_finish<kStep>(i, out, grad, rows, vs, step);
    }
}

__global__ __launch_bounds__(256) void unpack_kernel(const float* __restrict__ rows, const float* __restrict__ vs,
                                                     uint32_t n, GsGradients* __restrict__ grad) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float2* src = reinterpret_cast<const float2*>(rows + (size_t)i * kGradRowFloats);
    const float2 a = src[0], b = src[1], c = src[2], d = src[3], e = src[4], f = src[5], g = src[6];
    const float2 v = vs ? reinterpret_cast<const float2*>(vs)[i] : make_float2(0.0f, 0.0f);
    float4* dst = reinterpret_cast<float4*>(grad + i);
    dst[0] = make_float4(a.x, a.y, b.x, b.y);     // position, opacity
    dst[1] = make_float4(c.x, c.y, d.x, 0.0f);    // log-scale, pad
    dst[2] = make_float4(d.y, e.x, e.y, f.x);     // rotation
    dst[3] = make_float4(f.y, 0.0f, 0.0f, 0.0f);  // sh0..3
    dst[4] = make_float4(g.x, 0.0f, 0.0f, 0.0f);  // sh4..7
    dst[5] = make_float4(g.y, 0.0f, 0.0f, 0.0f);  // sh8..11
    dst[6] = make_float4(v.x, v.y, 0.0f, 0.0f);   // viewspace, pad
}

static inline uint32_t blocks_of(uint64_t n) { return (uint32_t)((n + 255) / 256); }

hipError_t launch_chain(hipStream_t st, const GsGaussian* g, uint32_t n,
                        const GsTiledUniforms& u, const GaussianBuffers& gb,
                        const PairBuffers& pb, GsGradients* grad, float* rows, float* vs, uint32_t first,
                        uint32_t count, const uint32_t* frame_tag, bool compact, const ChainStep* step,
                        bool list_dense) {
    if (count == 0) return hipSuccess;
    const ChainStep cs = step ? *step : ChainStep{};
    if (!compact) {
        auto go = [&](auto kernel) {
            hipLaunchKernelGGL(kernel, dim3((count + 255u) / 256u), dim3(256), 0, st, g, n, u, gb.count, gb.goff,
                               pb.partial, pb.ptag_zero, grad, rows, vs, first, first + count, frame_tag, gb.reached, cs);
        };
        step ? go(chain_kernel<true>) : go(chain_kernel<false>);
        return hipGetLastError();
    }
    // (the two launches touch disjoint Gaussians: the still ones in the first, the listed ones in the second)
    const uint32_t nb = (count + 255u) / 256u;
    // screen blocks per list workgroup: about one listed Gaussian per thread where few are listed (deep
    // scenes: config 5 lists ~4 % of its Gaussians), fewer blocks where many are
    const uint32_t lblocks = list_dense ? 2u : kListBlocksMax;
    auto go = [&](auto screen, auto lst) {
        hipLaunchKernelGGL(screen, dim3(nb), dim3(256), 0, st, n, gb.count, grad, rows, vs, first, first + count, frame_tag,
                           gb.reached, cs, gb.chain_list, gb.chain_lcount);
        hipLaunchKernelGGL(lst, dim3((nb + lblocks - 1u) / lblocks), dim3(kListThreads), 0, st, g, u, gb.count,
                           gb.goff, pb.partial, pb.ptag_zero, grad, rows, vs, nb, lblocks, frame_tag, gb.reached, cs,
                           gb.chain_list, gb.chain_lcount);
    };
    if (step)
        go(chain_screen_kernel<true>, chain_list_kernel<true>);
    else
        go(chain_screen_kernel<false>, chain_list_kernel<false>);
    return hipGetLastError();
}

hipError_t launch_unpack(hipStream_t st, const float* rows, const float* vs, uint32_t n, GsGradients* grad) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(unpack_kernel, dim3(blocks_of(n)), dim3(256), 0, st, rows, vs, n, grad);
    return hipGetLastError();
}

}  // namespace gs
