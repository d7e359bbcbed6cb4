// gs_optim.hip — the training step's optimizer on gfx950.
//
//   adam_kernel            adamStep (shaders.metal:536-713): one thread per Gaussian, in place.
//                          Pure streaming: 112 B Gaussian + 112 B gradient + 2 x 96 B moments in,
//                          112 B + 2 x 96 B out per Gaussian — HBM-bound, all loads/stores 16 B.
//   adam_follow_kernel     moments follow a density apply (survivor -> its new slot, new
//                          Gaussians zero); one thread per input Gaussian.
//   opacity_reset_kernel   mtl_engine.mm:1173-1186.
//
// Evaluation order follows the MSL text operation by operation (no FMA contraction in this file).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "gs_adam.hpp"
#include "gs_device.hpp"
#include "gs_internal.hpp"

namespace gs {

// kRows: the gradient comes from a 56-B gradient row (gs_rasterizer.h GS_GRAD_ROW_FLOATS; row k
// belongs to Gaussian first + k) with the other GaussianGradients fields zero -- the same update,
// bit for bit, for half the gradient bytes (config 5: the 112-B records are never written).
template <bool kRows>
__global__ __launch_bounds__(256) void adam_kernel(GsGaussian* __restrict__ gs,
                                                   const GsGradients* __restrict__ grads,
                                                   const float* __restrict__ rows, uint32_t first, uint32_t end,
                                                   float4* __restrict__ mom_m, float4* __restrict__ mom_v,
                                                   AdamParams P) {
    const uint32_t i = first + blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= end) return;
    float d[28];
    if (kRows) {
        const float2* r = reinterpret_cast<const float2*>(rows + (size_t)(i - first) * kGradRowFloats);
        float rv[14];
#pragma unroll
        for (int q = 0; q < 7; q++) {
            const float2 a = r[q];
            rv[2 * q] = a.x;
            rv[2 * q + 1] = a.y;
        }
#pragma unroll
        for (int q = 0; q < 28; q++) d[q] = 0.0f;
#pragma unroll
        for (int q = 0; q < 7; q++) d[q] = rv[q];  // position, opacity, log-scale
#pragma unroll
        for (int q = 0; q < 4; q++) d[8 + q] = rv[7 + q];  // rotation
        d[12] = rv[11];
        d[16] = rv[12];
        d[20] = rv[13];
    } else {
        const float4* dp = reinterpret_cast<const float4*>(grads + i);
#pragma unroll
        for (int q = 0; q < 7; q++) {
            const float4 b = dp[q];
            d[4 * q] = b.x; d[4 * q + 1] = b.y; d[4 * q + 2] = b.z; d[4 * q + 3] = b.w;
        }
    }
    adam_update(gs, i, d, mom_m, mom_v, P);
}

// marker: 0 keep, 1 prune, 2 clone (original + copy), 3 split (two children); offset = first
// output slot (gs_density.hip). The moments move with the survivors; new Gaussians start at 0.
__global__ __launch_bounds__(256) void adam_follow_kernel(const uint32_t* __restrict__ marker,
                                                          const uint32_t* __restrict__ offset, uint32_t n,
                                                          const float4* __restrict__ m_in,
                                                          const float4* __restrict__ v_in,
                                                          float4* __restrict__ m_out, float4* __restrict__ v_out,
                                                          uint8_t* __restrict__ live_out) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t mk = marker[i];
    if (mk == 1u) return;
    const uint32_t o = offset[i];
    const float4 z = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    uint32_t nz = 0;
#pragma unroll
    for (int q = 0; q < 6; q++) {
        const bool keep = mk == 0u || mk == 2u;
        const float4 a = keep ? m_in[(size_t)i * 6u + q] : z, b = keep ? v_in[(size_t)i * 6u + q] : z;
        nz |= __float_as_uint(a.x) | __float_as_uint(a.y) | __float_as_uint(a.z) | __float_as_uint(a.w) |
              __float_as_uint(b.x) | __float_as_uint(b.y) | __float_as_uint(b.z) | __float_as_uint(b.w);
        m_out[(size_t)o * 6u + q] = a;
        v_out[(size_t)o * 6u + q] = b;
        if (mk >= 2u) {
            m_out[(size_t)(o + 1) * 6u + q] = z;
            v_out[(size_t)(o + 1) * 6u + q] = z;
        }
    }
    live_out[o] = nz ? 1u : 0u;
    if (mk >= 2u) live_out[o + 1] = 0u;
}

// zero the given lanes of the moment records [start, end): mask bit b clears float b (0..23); with
// every lane cleared the records are all zero again (live flag 0)
__global__ __launch_bounds__(256) void adam_zero_kernel(float* __restrict__ m, float* __restrict__ v,
                                                        uint32_t start, uint32_t end, uint32_t mask,
                                                        uint8_t* __restrict__ live) {
    const uint32_t i = start + blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= end) return;
    if (live && mask == 0xffffffu) live[i] = 0u;
#pragma unroll
    for (int b = 0; b < 24; b++)
        if ((mask >> b) & 1u) {
            m[(size_t)i * 24u + b] = 0.0f;
            v[(size_t)i * 24u + b] = 0.0f;
        }
}

__global__ __launch_bounds__(256) void opacity_reset_kernel(GsGaussian* __restrict__ g, uint32_t n,
                                                            float max_raw) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    if (g[i].opacity > max_raw) g[i].opacity = max_raw;
}

static inline uint32_t blocks_of(uint64_t n) { return (uint32_t)((n + 255) / 256); }

AdamParams make_adam_params(const float lrs[5], float beta1, float beta2, float eps, float clip, float bc1,
                            float bc2) {
    AdamParams P;
    for (int k = 0; k < 5; k++) P.lr[k] = lrs[k];
    P.beta1 = beta1;
    P.beta2 = beta2;
    P.eps = eps;
    P.clip = clip;
    P.bc1 = bc1;
    P.bc2 = bc2;
    P.cold = 1u;
    P.cold_word = nullptr;
    P.live = nullptr;
    return P;
}

// The moment records between the reference's lane order (sh 0..11 in lanes 12-23: gs_adam_read_state
// / write_state) and the HBM order (mom_sh_lane). to_hbm: also flags a non-zero cold lane in *cold
// (the rows / fused updates then keep processing quads 4-5).
__global__ __launch_bounds__(256) void adam_layout_kernel(const float* __restrict__ in_m, const float* __restrict__ in_v,
                                                          float* __restrict__ out_m, float* __restrict__ out_v,
                                                          uint32_t n, uint32_t to_hbm, uint32_t* __restrict__ cold,
                                                          uint8_t* __restrict__ live) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    bool nz = false, any = false;
#pragma unroll
    for (int l = 0; l < 24; l++) {
        int src = l, dst = l;
        if (l >= 12) {
            if (to_hbm) dst = mom_sh_lane(l - 12);
            else src = mom_sh_lane(l - 12);
        }
        const float a = in_m[(size_t)i * 24u + src], b = in_v[(size_t)i * 24u + src];
        out_m[(size_t)i * 24u + dst] = a;
        out_v[(size_t)i * 24u + dst] = b;
        if (to_hbm && dst >= 15) nz |= (__float_as_uint(a) | __float_as_uint(b)) != 0u;
        any |= (__float_as_uint(a) | __float_as_uint(b)) != 0u;
    }
    if (nz) atomicOr(cold, 1u);
    if (to_hbm && live) live[i] = any ? 1u : 0u;
}

hipError_t launch_adam(hipStream_t st, GsGaussian* g, const GsGradients* grad, const float* rows,
                       uint32_t first, uint32_t count, float4* m, float4* v, const float lrs[5], float beta1,
                       float beta2, float eps, float clip, float bc1, float bc2, const uint32_t* cold_word,
                       uint8_t* live) {
    if (count == 0) return hipSuccess;
    AdamParams P = make_adam_params(lrs, beta1, beta2, eps, clip, bc1, bc2);
    P.live = live;
    P.cold = rows ? 0u : 1u;  // the records' cold SH fields may be anything
    P.cold_word = cold_word;
    if (rows)
        hipLaunchKernelGGL(adam_kernel<true>, dim3(blocks_of(count)), dim3(256), 0, st, g, grad, rows, first,
                           first + count, m, v, P);
    else
        hipLaunchKernelGGL(adam_kernel<false>, dim3(blocks_of(count)), dim3(256), 0, st, g, grad, rows, first,
                           first + count, m, v, P);
    return hipGetLastError();
}

hipError_t launch_adam_follow(hipStream_t st, const uint32_t* marker, const uint32_t* offset,
                              uint32_t n, const float4* m_in, const float4* v_in, float4* m_out,
                              float4* v_out, uint8_t* live_out) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(adam_follow_kernel, dim3(blocks_of(n)), dim3(256), 0, st, marker, offset, n,
                       m_in, v_in, m_out, v_out, live_out);
    return hipGetLastError();
}

hipError_t launch_adam_zero(hipStream_t st, float* m, float* v, uint32_t start, uint32_t end,
                            uint32_t mask, uint8_t* live) {
    if (end <= start) return hipSuccess;
    hipLaunchKernelGGL(adam_zero_kernel, dim3(blocks_of(end - start)), dim3(256), 0, st, m, v,
                       start, end, mask, live);
    return hipGetLastError();
}

hipError_t launch_adam_layout(hipStream_t st, const float* in_m, const float* in_v, float* out_m, float* out_v,
                              uint32_t n, bool to_hbm, uint32_t* cold, uint8_t* live) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(adam_layout_kernel, dim3(blocks_of(n)), dim3(256), 0, st, in_m, in_v, out_m, out_v, n,
                       to_hbm ? 1u : 0u, cold, live);
    return hipGetLastError();
}

hipError_t launch_opacity_reset(hipStream_t st, GsGaussian* g, uint32_t n, float max_raw) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(opacity_reset_kernel, dim3(blocks_of(n)), dim3(256), 0, st, g, n, max_raw);
    return hipGetLastError();
}

}  // namespace gs
