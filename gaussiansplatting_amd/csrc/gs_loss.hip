// gs_loss.hip — the training loss of MTLEngine::computeLoss (mtl_engine.mm:769-853) on gfx950
// (SURVEY.md §8f row 3): per-pixel L1 (shaders.metal:320-339), D-SSIM over an 11x11 Gaussian
// window (:361-482), the (1 - lambda) L1 + lambda D-SSIM combination (:485-510) and the mean.
//
//   loss_kernel     one 16x16 pixel tile per 256-thread workgroup. The tile's grey values
//                   (r+g+b)/3 of both images plus a 5-pixel clamped halo are staged in LDS once
//                   (26x26 x 2 floats); every pixel then runs the reference's two window passes
//                   in the reference's order (dy outer, dx inner), so the maps are bit-identical
//                   to the CPU restatement. The tile's combined losses are summed in fp64 with a
//                   fixed tree (deterministic; the reference uses float atomics).
//   loss_final      one workgroup: the per-tile fp64 partial sums in tile order -> the mean.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "gs_device.hpp"
#include "gs_internal.hpp"

namespace gs {

constexpr int kLossR = 5;                  // SSIM_WINDOW_RADIUS
constexpr int kLossW = kTile + 2 * kLossR;  // staged tile width (26)

__device__ __forceinline__ float unorm8(uint32_t v, int c) { return (float)((v >> (8 * c)) & 0xffu) / 255.0f; }

__device__ __forceinline__ double wave_sum_f64(double v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

__global__ __launch_bounds__(256) void loss_kernel(const uint32_t* __restrict__ rendered,
                                                   const uint32_t* __restrict__ gt, uint32_t w,
                                                   uint32_t h, float lambda,
                                                   float* __restrict__ maps, double* __restrict__ partial) {
    __shared__ float sw[11 * 11];  // window weights, dy-major
    __shared__ float sx[kLossW][kLossW];
    __shared__ float sy[kLossW][kLossW];
    __shared__ double sred[4];
    const uint32_t tiles_x = (w + kTile - 1) / kTile;
    const uint32_t tx = blockIdx.x % tiles_x, ty = blockIdx.x / tiles_x;
    const uint32_t t = threadIdx.x;
    const int x0 = (int)(tx * kTile) - kLossR, y0 = (int)(ty * kTile) - kLossR;
    if (t < 121u) {  // w = exp(-dist_sq / two_sigma_sq), sigma = 1.5 (:393-395, 410-411), pinned exp
        const int dx = (int)(t % 11u) - kLossR, dy = (int)(t / 11u) - kLossR;
        const float dist_sq = (float)(dx * dx + dy * dy);
        sw[t] = gs_expf(-dist_sq / (2.0f * 1.5f * 1.5f));
    }
    // stage grey values with the reference's clamp-to-edge addressing (:404-406)
    for (uint32_t k = t; k < (uint32_t)(kLossW * kLossW); k += 256u) {
        const int ly = (int)k / kLossW, lx = (int)k % kLossW;
        int px = x0 + lx, py = y0 + ly;
        px = px < 0 ? 0 : (px > (int)w - 1 ? (int)w - 1 : px);
        py = py < 0 ? 0 : (py > (int)h - 1 ? (int)h - 1 : py);
        const uint32_t r = rendered[(size_t)py * w + px], g = gt[(size_t)py * w + px];
        sx[ly][lx] = (unorm8(r, 0) + unorm8(r, 1) + unorm8(r, 2)) / 3.0f;
        sy[ly][lx] = (unorm8(g, 0) + unorm8(g, 1) + unorm8(g, 2)) / 3.0f;
    }
    __syncthreads();
    const uint32_t lx = t & 15u, ly = t >> 4;
    const uint32_t x = tx * kTile + lx, y = ty * kTile + ly;
    double contrib = 0.0;
    if (x < w && y < h) {
        const size_t pix = (size_t)y * w + x;
        // L1 (:332-334)
        const uint32_t r = rendered[pix], g = gt[pix];
        const float l1 = (fabsf(unorm8(r, 0) - unorm8(g, 0)) + fabsf(unorm8(r, 1) - unorm8(g, 1)) +
                          fabsf(unorm8(r, 2) - unorm8(g, 2))) / 3.0f;
        // SSIM, first pass: weighted means (:398-428)
        float mu_x = 0.0f, mu_y = 0.0f, wsum = 0.0f;
        for (int dy = 0; dy < 11; dy++)
#pragma unroll
            for (int dx = 0; dx < 11; dx++) {
                const float wt = sw[dy * 11 + dx];
                wsum += wt;
                mu_x += wt * sx[ly + dy][lx + dx];
                mu_y += wt * sy[ly + dy][lx + dx];
            }
        mu_x /= wsum;
        mu_y /= wsum;
        // second pass: variances and covariance (:431-468)
        float vx = 0.0f, vy = 0.0f, cxy = 0.0f;
        wsum = 0.0f;
        for (int dy = 0; dy < 11; dy++)
#pragma unroll
            for (int dx = 0; dx < 11; dx++) {
                const float wt = sw[dy * 11 + dx];
                wsum += wt;
                const float a = sx[ly + dy][lx + dx] - mu_x;
                const float b = sy[ly + dy][lx + dx] - mu_y;
                vx += wt * a * a;
                vy += wt * b * b;
                cxy += wt * a * b;
            }
        vx /= wsum;
        vy /= wsum;
        cxy /= wsum;
        const float C1 = 0.01f * 0.01f, C2 = 0.03f * 0.03f;  // :356-358
        const float num = (2.0f * mu_x * mu_y + C1) * (2.0f * cxy + C2);
        const float den = (mu_x * mu_x + mu_y * mu_y + C1) * (vx + vy + C2);
        const float ssim = num / den;
        const float dssim = fminf(fmaxf((1.0f - ssim) / 2.0f, 0.0f), 1.0f);
        const float comb = (1.0f - lambda) * l1 + lambda * dssim;  // :508
        if (maps) {
            const size_t np = (size_t)w * h;
            maps[pix] = l1;
            maps[np + pix] = dssim;
            maps[2 * np + pix] = comb;
        }
        contrib = (double)comb;
    }
    contrib = wave_sum_f64(contrib);
    if ((t & 63u) == 0u) sred[t >> 6] = contrib;
    __syncthreads();
    if (t == 0) partial[blockIdx.x] = (sred[0] + sred[1]) + (sred[2] + sred[3]);
}

__global__ __launch_bounds__(1024) void loss_final_kernel(const double* __restrict__ partial,
                                                          uint32_t nblocks, uint64_t npix,
                                                          float* __restrict__ loss) {
    __shared__ double s[16];
    const uint32_t t = threadIdx.x;
    double acc = 0.0;
    for (uint32_t b = t; b < nblocks; b += 1024u) acc += partial[b];
    acc = wave_sum_f64(acc);
    if ((t & 63u) == 0u) s[t >> 6] = acc;
    __syncthreads();
    if (t == 0) {
        double tot = 0.0;
        for (int k = 0; k < 16; k++) tot += s[k];
        *loss = (float)(tot / (double)npix);
    }
}

uint32_t loss_blocks(uint32_t w, uint32_t h) { return ((w + kTile - 1) / kTile) * ((h + kTile - 1) / kTile); }

hipError_t launch_loss(hipStream_t st, const uint32_t* rendered, const uint32_t* gt, uint32_t w,
                       uint32_t h, float lambda, float* maps, double* partial, float* loss) {
    const uint32_t nb = loss_blocks(w, h);
    if (nb == 0) return hipSuccess;
    hipLaunchKernelGGL(loss_kernel, dim3(nb), dim3(256), 0, st, rendered, gt, w, h, lambda, maps,
                       partial);
    hipLaunchKernelGGL(loss_final_kernel, dim3(1), dim3(1024), 0, st, partial, nb,
                       (uint64_t)w * h, loss);
    return hipGetLastError();
}

}  // namespace gs
