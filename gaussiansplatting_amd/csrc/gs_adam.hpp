// gs_adam.hpp — the per-Gaussian Adam update (adamStep, shaders.metal:536-713) and the density
// statistics update (accumulateGradients, density_control.mm:121-185) as device functions, shared
// by their own kernels (gs_optim.hip, gs_density.hip) and by the chain kernel's fused training-step
// mode (gs_chain.hip, gs_backward_step): the same arithmetic in the same order, so either path gives
// the same bits.
//
// Evaluation order follows the MSL text operation by operation (no FMA contraction: the files that
// include this are built with -ffp-contract=off).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/gs_rasterizer.h"

namespace gs {

struct AdamParams {
    float lr[5];       // position, log-scale, rotation, raw opacity, sh
    float beta1, beta2, eps, clip;
    float bc1, bc2;    // 1 - beta^t, computed on the host
    uint32_t cold;     // 1: the cold moment lanes may be non-zero (always, for gradient records)
    const uint32_t* cold_word;  // nullable: the optimizer's device word -- non-zero once a records step or
                                // a written state may have made a cold lane non-zero (gs_adam.flag)
    uint8_t* live;     // nullable: per Gaussian, 0 = its moment records are all zero (not loaded)
};

// Moment records in HBM: [i][6] float4 = 24 lanes, lanes 0-2 position, 3 opacity, 4-6 log-scale, 7
// pad, 8-11 rotation, then the 12 SH coefficients with the three DC ones (sh 0, 4, 8: the only SH
// fields the rasterizer's gradients have, tiled_shaders.metal:699-704) in lanes 12-14 and the nine
// others in lanes 15-23 ("cold"). While no gradient has ever had a non-zero cold field their moments
// stay exactly zero (m = b1 * 0 + (1 - b1) * 0) and their step exactly 0, so the rows / fused
// updates read and write quads 0-3 only (64 of 96 B per moment record); gs_adam_read_state /
// write_state convert to and from the reference's order (sh 0..11 in lanes 12-23).
__host__ __device__ constexpr int mom_sh_lane(int k) {
    return k == 0 ? 12 : k == 4 ? 13 : k == 8 ? 14 : k < 4 ? 14 + k : k < 8 ? 13 + k : 12 + k;
}

__device__ __forceinline__ float clampc(float x, float lo, float hi) { return fminf(fmaxf(x, lo), hi); }

// One Adam moment update + the bias-corrected step of one scalar parameter component
// (shaders.metal:595-611 for each component): returns lr * m_hat / (sqrt(v_hat) + eps).
__device__ __forceinline__ float adam_delta(float grad, float& m, float& v, float lr, const AdamParams& P) {
    const float gc = clampc(grad, -P.clip, P.clip);
    m = P.beta1 * m + (1.0f - P.beta1) * gc;
    v = P.beta2 * v + (1.0f - P.beta2) * gc * gc;
    const float m_hat = m / P.bc1;
    const float v_hat = v / P.bc2;
    return lr * m_hat / (sqrtf(v_hat) + P.eps);
}

// Adam on Gaussian i in place from its gradient d[] in the GaussianGradients float layout
// (pos 0-2, opacity 3, scale 4-6, rot 8-11, sh 12-23; the viewspace floats 24-27 are not read).
// Moment records as above (mom_sh_lane); quads 4-5 are read and written only when P.cold or the
// optimizer's device word says a cold lane may be non-zero (read on the device, so a replayed HIP
// graph sees a records step that came after its capture).
__device__ __forceinline__ void adam_update(GsGaussian* __restrict__ gs, uint32_t i, const float (&d)[28],
                                            float4* __restrict__ mom_m, float4* __restrict__ mom_v,
                                            const AdamParams& P) {
    float4* gp = reinterpret_cast<float4*>(gs + i);
    float g[28];
    float4 g0[7];  // as loaded: a quad whose update left every bit as it was is not stored
#pragma unroll
    for (int q = 0; q < 7; q++) {
        const float4 a = gp[q];
        g0[q] = a;
        g[4 * q] = a.x; g[4 * q + 1] = a.y; g[4 * q + 2] = a.z; g[4 * q + 3] = a.w;
    }
    // GsGaussian floats: pos 0-2, scale 4-6, rot 8-11, opacity 12, sh 13-24
    // skip invalid gradients and corrupted Gaussians (:566-576)
    if (__builtin_isnan(d[0]) || __builtin_isnan(d[3]) || __builtin_isnan(d[12]) ||
        __builtin_isinf(d[0]) || __builtin_isinf(d[3]))
        return;
    if (__builtin_isnan(g[0]) || __builtin_isinf(g[0]) || fabsf(g[0]) > 1e6f) return;

    float4* mp = mom_m + (size_t)i * 6u;
    float4* vp = mom_v + (size_t)i * 6u;
    const bool cold = P.cold != 0u || (P.cold_word && *P.cold_word != 0u);
    // a Gaussian whose moments were never non-zero (P.live: no gradient has reached it since the
    // state was zeroed) reads none of its 128-192 B of moments
    const bool live = !P.live || P.live[i] != 0u;
    float m[24], v[24];
    float4 m0[6], v0[6];
#pragma unroll
    for (int q = 0; q < 6; q++) {
        const float4 z = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
        const bool ld = live && (q < 4 || cold);
        const float4 a = ld ? mp[q] : z, b = ld ? vp[q] : z;
        m0[q] = a;
        v0[q] = b;
        m[4 * q] = a.x; m[4 * q + 1] = a.y; m[4 * q + 2] = a.z; m[4 * q + 3] = a.w;
        v[4 * q] = b.x; v[4 * q + 1] = b.y; v[4 * q + 2] = b.z; v[4 * q + 3] = b.w;
    }

    // position with the update-magnitude limit and the sanity check (:585-627)
    {
        float up[3];
#pragma unroll
        for (int k = 0; k < 3; k++) up[k] = adam_delta(d[k], m[k], v[k], P.lr[0], P);
        const float mag = sqrtf(up[0] * up[0] + up[1] * up[1] + up[2] * up[2]);
        if (mag > 0.1f) {
            const float s = 0.1f / mag;
#pragma unroll
            for (int k = 0; k < 3; k++) up[k] = up[k] * s;
        }
        float np[3];
#pragma unroll
        for (int k = 0; k < 3; k++) np[k] = g[k] - up[k];
        if (!__builtin_isnan(np[0]) && !__builtin_isnan(np[1]) && !__builtin_isnan(np[2]) &&
            fabsf(np[0]) < 1e6f && fabsf(np[1]) < 1e6f && fabsf(np[2]) < 1e6f) {
#pragma unroll
            for (int k = 0; k < 3; k++) g[k] = np[k];
        }
    }
    // log-scale, clamped to +-MAX_SCALE_TRAIN = 4 (:632-656)
#pragma unroll
    for (int k = 0; k < 3; k++) {
        const float ns = g[4 + k] - adam_delta(d[4 + k], m[4 + k], v[4 + k], P.lr[1], P);
        g[4 + k] = clampc(ns, -4.0f, 4.0f);
    }
    // rotation, renormalised (:659-673)
    {
        float nr[4];
#pragma unroll
        for (int k = 0; k < 4; k++) nr[k] = g[8 + k] - adam_delta(d[8 + k], m[8 + k], v[8 + k], P.lr[2], P);
        const float len = sqrtf(nr[0] * nr[0] + nr[1] * nr[1] + nr[2] * nr[2] + nr[3] * nr[3]);
        if (len > 0.001f) {
#pragma unroll
            for (int k = 0; k < 4; k++) g[8 + k] = nr[k] / len;
        } else {
            g[8] = 1.0f; g[9] = 0.0f; g[10] = 0.0f; g[11] = 0.0f;
        }
    }
    // raw opacity, clamped to +-8 (:676-690)
    g[12] = clampc(g[12] - adam_delta(d[3], m[3], v[3], P.lr[3], P), -8.0f, 8.0f);
    // SH, clamped to +-2 (:693-712)
#pragma unroll
    for (int k = 0; k < 12; k++) {
        const int l = mom_sh_lane(k);
        const float nsh = g[13 + k] - adam_delta(d[12 + k], m[l], v[l], P.lr[4], P);
        g[13 + k] = clampc(nsh, -2.0f, 2.0f);
    }
    // Only the quads whose bits changed are stored: a Gaussian no view reaches keeps zero moments
    // and, but for its clamps and the quaternion renormalisation, its parameters (config 5: most of
    // the 5.2M), so most of its 96 B of parameter and 128 B of moment writes are the same bits.
    auto same = [](float4 a, float4 b) {
        return ((__float_as_uint(a.x) ^ __float_as_uint(b.x)) | (__float_as_uint(a.y) ^ __float_as_uint(b.y)) |
                (__float_as_uint(a.z) ^ __float_as_uint(b.z)) | (__float_as_uint(a.w) ^ __float_as_uint(b.w))) == 0u;
    };
#pragma unroll
    for (int q = 0; q < 7; q++) {
        const float4 nq = make_float4(g[4 * q], g[4 * q + 1], g[4 * q + 2], g[4 * q + 3]);
        if (!same(nq, g0[q])) gp[q] = nq;
    }
    bool wrote = false;
#pragma unroll
    for (int q = 0; q < 6; q++) {
        if (q >= 4 && !cold) continue;
        const float4 nm = make_float4(m[4 * q], m[4 * q + 1], m[4 * q + 2], m[4 * q + 3]);
        const float4 nv = make_float4(v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3]);
        if (!same(nm, m0[q])) { mp[q] = nm; wrote = true; }
        if (!same(nv, v0[q])) { vp[q] = nv; wrote = true; }
    }
    if (wrote && !live) P.live[i] = 1u;  // (its zero records just changed)
}

// adam_update with an all-zero gradient on a Gaussian whose moment records are all zero (live flag
// 0) and whose cold lanes are zero: every adam_delta is exactly +0 (m = v = +0, m_hat = v_hat = +0,
// lr * 0 / (sqrt(0) + eps) = +0) and no moment changes, so what remains is x - 0 = x for every
// parameter followed by the same clamps, the same position check and the same quaternion
// renormalisation, bit for bit; only the quads whose bits changed are stored, as there.
// (g0: the Gaussian's seven 16-B quads as loaded from gp, for callers that issue the loads early)
__device__ __forceinline__ void adam_still_from(float4* __restrict__ gp, const float4 (&g0)[7]) {
    float g[28];
#pragma unroll
    for (int q = 0; q < 7; q++) {
        g[4 * q] = g0[q].x; g[4 * q + 1] = g0[q].y; g[4 * q + 2] = g0[q].z; g[4 * q + 3] = g0[q].w;
    }
    if (__builtin_isnan(g[0]) || __builtin_isinf(g[0]) || fabsf(g[0]) > 1e6f) return;
    // (position: the update is 0, so the new position is the old one and the check changes nothing)
#pragma unroll
    for (int k = 0; k < 3; k++) g[4 + k] = clampc(g[4 + k], -4.0f, 4.0f);
    {
        const float len = sqrtf(g[8] * g[8] + g[9] * g[9] + g[10] * g[10] + g[11] * g[11]);
        if (len > 0.001f) {
            const float nr[4] = {g[8], g[9], g[10], g[11]};
#pragma unroll
            for (int k = 0; k < 4; k++) g[8 + k] = nr[k] / len;
        } else {
            g[8] = 1.0f; g[9] = 0.0f; g[10] = 0.0f; g[11] = 0.0f;
        }
    }
    g[12] = clampc(g[12], -8.0f, 8.0f);
#pragma unroll
    for (int k = 0; k < 12; k++) g[13 + k] = clampc(g[13 + k], -2.0f, 2.0f);
#pragma unroll
    for (int q = 0; q < 7; q++) {
        const float4 nq = make_float4(g[4 * q], g[4 * q + 1], g[4 * q + 2], g[4 * q + 3]);
        if (((__float_as_uint(nq.x) ^ __float_as_uint(g0[q].x)) | (__float_as_uint(nq.y) ^ __float_as_uint(g0[q].y)) |
             (__float_as_uint(nq.z) ^ __float_as_uint(g0[q].z)) | (__float_as_uint(nq.w) ^ __float_as_uint(g0[q].w))) != 0u)
            gp[q] = nq;
    }
}

__device__ __forceinline__ void adam_update_still(GsGaussian* __restrict__ gs, uint32_t i) {
    float4* gp = reinterpret_cast<float4*>(gs + i);
    float4 g0[7];
#pragma unroll
    for (int q = 0; q < 7; q++) g0[q] = gp[q];
    adam_still_from(gp, g0);
}

// accumulateGradients for Gaussian i (density_control.mm:121-185): the viewspace gradient's
// magnitude (capped at 1) and the position gradient, where the magnitude is finite and positive.
__device__ __forceinline__ void density_accumulate_one(float* __restrict__ accum, uint32_t* __restrict__ count,
                                                       float* __restrict__ pos_accum, uint32_t i, float px,
                                                       float py, float pz, float vx, float vy) {
    float gm = sqrtf(vx * vx + vy * vy);
    gm = (1.0f < gm) ? 1.0f : gm;  // std::min(gradMag, 1.0f)
    if (!__builtin_isnan(gm) && !__builtin_isinf(gm) && gm > 0.0f) {
        accum[i] += gm;
        count[i] += 1u;
        pos_accum[3 * i + 0] += px;
        pos_accum[3 * i + 1] += py;
        pos_accum[3 * i + 2] += pz;
    }
}

}  // namespace gs
