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

// kCompact (scenes where most Gaussians are not reached, e.g. config 5's 5.2M, of which a minority
// is, spread over nearly every wave): every thread whose Gaussian the backward never reached writes
// its zero gradient at once, the reached ones are compacted in LDS (ballot order: deterministic)
// and summed and chained by the first threads, so the fp64 path runs in as few waves as there are
// reached Gaussians (config 5 chain 0.46 -> 0.35 ms); where at least half of a workgroup's Gaussians
// are reached each thread keeps its own. The workgroup barrier costs ~6 us where nearly everything
// is reached (the bench frame), so the host takes the plain kernel there (launch_chain).
//
// kStep (gs_backward_step): instead of storing the gradient, the thread feeds it to the density
// statistics and to Adam on its own Gaussian (gs_adam.hpp: the same arithmetic as
// gs_density_accumulate_rows + gs_adam_step_rows, so the same bits), skipping the 64-B row write and
// read-back, the separate kernels' Gaussian re-read and two launches. Each Gaussian is read and
// updated by the one thread that owns it (compacted or not), after its chain has read it; in this
// mode the Gaussians are read through step.g (written by Adam), never through the restrict-qualified
// `g`, which is then unused.
template <bool kCompact, bool kStep>
__global__ __launch_bounds__(kCompact ? 512 : 256) void chain_kernel(
    const GsGaussian* __restrict__ g, uint32_t n, GsTiledUniforms u,
    const uint32_t* __restrict__ count, const uint32_t* __restrict__ goff,
    const float* __restrict__ partial, const float* __restrict__ zero9,
    GsGradients* __restrict__ grad, float* __restrict__ rows, float* __restrict__ vs, uint32_t first, uint32_t end,
    const uint32_t* __restrict__ frame_tag, const reach_t* __restrict__ reached, ChainStep step) {
    auto finish = [&](uint32_t gi, const float(&o)[28]) {
        if constexpr (kStep) {
            if (step.accum) density_accumulate_one(step.accum, step.dcount, step.pos_accum, gi, o[0], o[1], o[2], o[24], o[25]);
            adam_update(step.g, gi, o, step.m, step.v, step.P);
        } else {
            chain_store(gi, o, grad, rows, vs);
        }
    };
    constexpr uint32_t NT = kCompact ? 512u : 256u;
    __shared__ uint32_t s_list[kCompact ? NT : 1u];
    __shared__ uint32_t s_wave[NT / 64u];
    const uint32_t t = threadIdx.x;
    const uint32_t mine = first + blockIdx.x * NT + t;
    const bool valid = mine < end && mine < n;
    const uint32_t tag = *frame_tag;
    // a Gaussian whose list entries the backward never selected has only stale slots: zero gradient
    // without reading its slots' tags or its record (most of config 5's 69M slots)
    const bool heavy = valid && count[mine] != 0u && reached[mine] == (reach_t)tag;
    uint32_t i = mine;
    if (kCompact) {
        const uint32_t lane = t & 63u, wv = t >> 6;
        if (valid && !heavy) {
            float zero[28];
#pragma unroll
            for (int q = 0; q < 28; q++) zero[q] = 0.0f;
            finish(mine, zero);
        }
        const uint64_t m = __ballot(heavy);
        if (lane == 0) s_wave[wv] = (uint32_t)__popcll(m);
        __syncthreads();
        uint32_t base = 0, nheavy = 0;
#pragma unroll
        for (uint32_t k = 0; k < NT / 64u; k++) {
            base += k < wv ? s_wave[k] : 0u;
            nheavy += s_wave[k];
        }
        if (heavy) s_list[base + (uint32_t)__popcll(m & lanemask_lt())] = mine;
        __syncthreads();
        const bool compact = 2u * nheavy < NT;
        if (compact ? t >= nheavy : !heavy) return;
        i = compact ? s_list[t] : mine;
    } else if (!valid) {
        return;
    }
    float out[28];
#pragma unroll
    for (int q = 0; q < 28; q++) out[q] = 0.0f;
    const uint32_t c = count[i];
    if (kCompact || heavy) {
        // the Gaussian record's loads go out with the partial sums' (independent latencies)
        const GaussianIn gin = load_gaussian(kStep ? step.g : g, i);
        const uint32_t o = goff[i];
        double S[9];
#pragma unroll
        for (int q = 0; q < 9; q++) S[q] = 0.0;
        // Slots the backward did not reach this frame carry an older tag and count as zero. Blocks
        // of kB slots. Where most of a Gaussian's slots are current (the plain kernel's scenes) the
        // whole tagged 40-B slots are loaded at once and a stale slot's sums dropped after the load:
        // one round trip per block. Where most are stale (the compacting kernel's deep scenes) the
        // tags are read first and only current slots' sums are loaded, a stale slot or one past the
        // Gaussian's last reading a cached block of zeros instead (no branch around the loads).
        constexpr uint32_t kB = 4;  // (tagged slots, bench chain: 3 / 4 / 6 / 8 slots 102.5 / 97.3 / 99.7 / 103.7 us)
        if constexpr (!kCompact) {
            for (uint32_t e = o; e < o + c; e += kB) {
                float2 v[5 * kB];
#pragma unroll
                for (uint32_t k = 0; k < kB; k++) {
                    const float2* src =
                        reinterpret_cast<const float2*>(partial + (size_t)min(e + k, o + c - 1u) * kSlotWords);
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
        } else {
            for (uint32_t e = o; e < o + c; e += kB) {
                uint32_t tg[kB];
#pragma unroll
                for (uint32_t k = 0; k < kB; k++)
                    tg[k] = e + k >= o + c ? 0u : __float_as_uint(partial[(size_t)(e + k) * kSlotWords + 9u]);
                float v[9 * kB];
#pragma unroll
                for (uint32_t k = 0; k < kB; k++) {
                    const float* src =
                        (e + k < o + c && tg[k] == tag) ? partial + (size_t)(e + k) * kSlotWords : zero9;
#pragma unroll
                    for (int q = 0; q < 9; q++) v[9 * k + q] = src[q];
                }
#pragma unroll
                for (uint32_t k = 0; k < kB; k++)
#pragma unroll
                    for (int q = 0; q < 9; q++) S[q] += (double)v[9 * k + q];
            }
        }
        chain_apply(gin, u, S, out);
    }
    finish(i, out);
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
                        uint32_t count, const uint32_t* frame_tag, bool compact, const ChainStep* step) {
    if (count == 0) return hipSuccess;
    const ChainStep cs = step ? *step : ChainStep{};
    auto go = [&](auto kernel, uint32_t nt) {
        hipLaunchKernelGGL(kernel, dim3((count + nt - 1u) / nt), dim3(nt), 0, st, g, n, u, gb.count, gb.goff,
                           pb.partial, pb.ptag_zero, grad, rows, vs, first, first + count, frame_tag,
                           gb.reached, cs);
    };
    if (step)
        compact ? go(chain_kernel<true, true>, 512u) : go(chain_kernel<false, true>, 256u);
    else
        compact ? go(chain_kernel<true, false>, 512u) : go(chain_kernel<false, false>, 256u);
    return hipGetLastError();
}

hipError_t launch_unpack(hipStream_t st, const float* rows, const float* vs, uint32_t n, GsGradients* grad) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(unpack_kernel, dim3(blocks_of(n)), dim3(256), 0, st, rows, vs, n, grad);
    return hipGetLastError();
}

}  // namespace gs
