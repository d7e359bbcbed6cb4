// gs_density.hip — DensityController hooks on the GPU (density_control.mm).
//
//   density_accumulate_kernel   accumulateGradients (:121-185), one thread per Gaussian.
//   density_mark_kernel         apply's first pass (:258-348): prune / clone / split markers,
//                               per-block counts folded into 3 global counters.
//   density_cap_kernel          the MAX_GAUSSIANS reduction (:360-382) — clones first, then
//                               splits, in index order — driven by exclusive scans of flags.
//   density_emit_kernel         apply's second pass (:393-483) into a compacted buffer; split
//                               offsets use a counter-based RNG keyed by (seed, index).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "gs_adam.hpp"
#include "gs_device.hpp"
#include "gs_internal.hpp"

namespace gs {

constexpr float kDcGradThreshold = 0.0002f;  // density_control.mm:21
constexpr float kDcOpacityPrune = 0.005f;    // :24
constexpr float kDcMaxScaleLog = 4.0f;       // :33
constexpr float kDcLogSplit = -0.47000363f;  // logf(1.0f / 1.6f), :425-426

__global__ __launch_bounds__(256) void density_accumulate_kernel(
    const GsGradients* __restrict__ grad, uint32_t n, float* __restrict__ accum,
    uint32_t* __restrict__ count, float* __restrict__ pos_accum) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float4* gp = reinterpret_cast<const float4*>(grad + i);
    const float4 g0 = gp[0];  // position xyz, opacity
    const float4 g6 = gp[6];  // viewspace xy @96
    density_accumulate_one(accum, count, pos_accum, i, g0.x, g0.y, g0.z, g6.x, g6.y);
}

// the same accumulation from gradient rows (position = row[0..2]) and the per-view viewspace rows
__global__ __launch_bounds__(256) void density_accumulate_rows_kernel(
    const float* __restrict__ rows, const float2* __restrict__ vs, uint32_t n, float* __restrict__ accum,
    uint32_t* __restrict__ count, float* __restrict__ pos_accum) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float2* r = reinterpret_cast<const float2*>(rows + (size_t)i * kGradRowFloats);
    const float2 p01 = r[0], p2o = r[1];
    const float2 v = vs[i];
    density_accumulate_one(accum, count, pos_accum, i, p01.x, p01.y, p2o.x, v.x, v.y);
}

__device__ __forceinline__ float dc_max_scale(const GaussianIn& g) {
    return fmaxf(fmaxf(gs_expf(clampf(g.sx, -kDcMaxScaleLog, kDcMaxScaleLog)),
                       gs_expf(clampf(g.sy, -kDcMaxScaleLog, kDcMaxScaleLog))),
                 gs_expf(clampf(g.sz, -kDcMaxScaleLog, kDcMaxScaleLog)));
}

struct DensityParams {
    uint32_t can_densify;
    uint32_t screen_prune;
    float split_thr;
    float prune_thr;
    float focal;
    float image_width;
    float avg_depth;
};

__global__ __launch_bounds__(256) void density_mark_kernel(
    const GsGaussian* __restrict__ g, uint32_t n, const float* __restrict__ accum,
    const uint32_t* __restrict__ count, DensityParams prm, uint32_t* __restrict__ marker,
    uint32_t* __restrict__ counters /* [pruned, cloned, split] */) {
    __shared__ uint32_t sc[3];
    if (threadIdx.x < 3) sc[threadIdx.x] = 0u;
    __syncthreads();
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) {
        const GaussianIn gin = load_gaussian(g, i);
        const float opacity = 1.0f / (1.0f + gs_expf(-gin.op));
        const float avg = count[i] > 0u ? accum[i] / (float)count[i] : 0.0f;
        const float ms = dc_max_scale(gin);
        bool prune = opacity < kDcOpacityPrune;
        if (prm.screen_prune) {
            if (ms > prm.prune_thr) prune = true;
            const float safe_depth = fmaxf(prm.avg_depth, 0.1f);
            const float sr = prm.focal * ms * 3.0f / safe_depth;
            const float frac = sr / prm.image_width;
            if (frac * prm.image_width > 40.0f) prune = true;
        }
        uint32_t m = 0u;
        if (prune) m = 1u;
        else if (prm.can_densify && avg > kDcGradThreshold) m = ms > prm.split_thr ? 3u : 2u;
        marker[i] = m;
        if (m) atomicAdd(&sc[m - 1u], 1u);
    }
    __syncthreads();
    if (threadIdx.x < 3 && sc[threadIdx.x]) atomicAdd(&counters[threadIdx.x], sc[threadIdx.x]);
}

// flag[i] = (marker[i] == want)
__global__ __launch_bounds__(256) void density_flag_kernel(const uint32_t* __restrict__ marker,
                                                           uint32_t n, uint32_t want,
                                                           uint32_t* __restrict__ flag) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) flag[i] = marker[i] == want ? 1u : 0u;
}

// demote the first `excess` markers equal to `want` (by index) to keep (0)
__global__ __launch_bounds__(256) void density_demote_kernel(uint32_t* __restrict__ marker,
                                                             uint32_t n, uint32_t want,
                                                             const uint32_t* __restrict__ rank,
                                                             uint64_t excess) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n && marker[i] == want && rank[i] < excess) marker[i] = 0u;
}

// out slots per Gaussian: keep 1, prune 0, clone 2, split 2
__global__ __launch_bounds__(256) void density_slots_kernel(const uint32_t* __restrict__ marker,
                                                            uint32_t n, uint32_t* __restrict__ slots) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) {
        const uint32_t m = marker[i];
        slots[i] = m == 1u ? 0u : (m == 0u ? 1u : 2u);
    }
}

__device__ __forceinline__ float density_uniform(uint64_t seed, uint64_t index, uint32_t comp) {
    uint64_t z = seed + (index * 3u + comp + 1u) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z = z ^ (z >> 31);
    const float uu = (float)(z >> 40) * 5.9604644775390625e-08f;
    return (uu - 0.5f) * 2.0f;
}

__global__ __launch_bounds__(256) void density_emit_kernel(const GsGaussian* __restrict__ in,
                                                           uint32_t n,
                                                           const uint32_t* __restrict__ marker,
                                                           const uint32_t* __restrict__ offset,
                                                           uint64_t seed,
                                                           GsGaussian* __restrict__ out) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t m = marker[i];
    if (m == 1u) return;
    const GsGaussian g = in[i];
    const uint32_t o = offset[i];
    if (m == 0u) {
        out[o] = g;
        return;
    }
    if (m == 2u) {
        out[o] = g;
        out[o + 1] = g;
        return;
    }
    float sc[3];
#pragma unroll
    for (int k = 0; k < 3; k++) sc[k] = gs_expf(clampf(g.scale[k], -kDcMaxScaleLog, kDcMaxScaleLog));
    float rx = density_uniform(seed, i, 0);
    float ry = density_uniform(seed, i, 1);
    float rz = density_uniform(seed, i, 2);
    const float rn = sqrtf(rx * rx + ry * ry + rz * rz);
    if (rn > 0.001f) {
        rx /= rn; ry /= rn; rz /= rn;
    }
    const float off[3] = {rx * sc[0], ry * sc[1], rz * sc[2]};
    const Mat3 R = quat_to_mat(g.rotation[0], g.rotation[1], g.rotation[2], g.rotation[3]);
    float ro[3];
#pragma unroll
    for (int r = 0; r < 3; r++) {
        float s = R.c[0][r] * off[0];
        s = s + R.c[1][r] * off[1];
        s = s + R.c[2][r] * off[2];
        ro[r] = s;
    }
    GsGaussian c1 = g, c2 = g;
#pragma unroll
    for (int k = 0; k < 3; k++) {
        c1.position[k] = g.position[k] + ro[k];
        c2.position[k] = g.position[k] - ro[k];
        c1.scale[k] = g.scale[k] + kDcLogSplit;
        c2.scale[k] = c1.scale[k];
    }
    out[o] = c1;
    out[o + 1] = c2;
}

// ---- launchers ------------------------------------------------------------------------
static inline uint32_t blocks_for(uint64_t n) { return (uint32_t)((n + 255) / 256); }

hipError_t launch_density_accumulate(hipStream_t st, const GsGradients* grad, uint32_t n,
                                     float* accum, uint32_t* count, float* pos_accum) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(density_accumulate_kernel, dim3(blocks_for(n)), dim3(256), 0, st, grad, n,
                       accum, count, pos_accum);
    return hipGetLastError();
}

hipError_t launch_density_accumulate_rows(hipStream_t st, const float* rows, const float* vs, uint32_t n,
                                          float* accum, uint32_t* count, float* pos_accum) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(density_accumulate_rows_kernel, dim3((n + 255u) / 256u), dim3(256), 0, st, rows,
                       reinterpret_cast<const float2*>(vs), n, accum, count, pos_accum);
    return hipGetLastError();
}

hipError_t launch_density_mark(hipStream_t st, const GsGaussian* g, uint32_t n,
                               const float* accum, const uint32_t* count, uint32_t can_densify,
                               uint32_t screen_prune, float split_thr, float prune_thr,
                               float focal, float image_width, float avg_depth, uint32_t* marker,
                               uint32_t* counters) {
    if (n == 0) return hipSuccess;
    DensityParams prm{can_densify, screen_prune, split_thr, prune_thr, focal, image_width, avg_depth};
    hipLaunchKernelGGL(density_mark_kernel, dim3(blocks_for(n)), dim3(256), 0, st, g, n, accum,
                       count, prm, marker, counters);
    return hipGetLastError();
}

hipError_t launch_density_demote(hipStream_t st, uint32_t* marker, uint32_t n, uint32_t want,
                                 uint64_t excess, uint32_t* flag, uint32_t* rank,
                                 uint32_t* block_sums, uint32_t* total) {
    if (n == 0 || excess == 0) return hipSuccess;
    hipLaunchKernelGGL(density_flag_kernel, dim3(blocks_for(n)), dim3(256), 0, st, marker, n, want,
                       flag);
    hipError_t e = exclusive_scan(st, flag, nullptr, n, rank, block_sums, total, nullptr);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(density_demote_kernel, dim3(blocks_for(n)), dim3(256), 0, st, marker, n,
                       want, rank, excess);
    return hipGetLastError();
}

hipError_t launch_density_slots(hipStream_t st, const uint32_t* marker, uint32_t n,
                                uint32_t* slots) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(density_slots_kernel, dim3(blocks_for(n)), dim3(256), 0, st, marker, n,
                       slots);
    return hipGetLastError();
}

hipError_t launch_density_emit(hipStream_t st, const GsGaussian* in, uint32_t n,
                               const uint32_t* marker, const uint32_t* offset, uint64_t seed,
                               GsGaussian* out) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(density_emit_kernel, dim3(blocks_for(n)), dim3(256), 0, st, in, n, marker,
                       offset, seed, out);
    return hipGetLastError();
}

}  // namespace gs
