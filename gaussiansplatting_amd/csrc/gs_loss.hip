// gs_loss.hip — the training loss of MTLEngine::computeLoss (mtl_engine.mm:769-853) on gfx950
// (SURVEY.md §8f row 3): per-pixel L1 (shaders.metal:320-339), D-SSIM over an 11x11 Gaussian
// window (:361-482), the (1 - lambda) L1 + lambda D-SSIM combination (:485-510) and the mean.
//
//   loss_kernel     one 16x16 pixel tile per one-wave workgroup, four pixels per lane. The tile's
//                   grey values (r+g+b)/3 of both images plus a 5-pixel clamped halo are staged in
//                   LDS once (26x26 x 2 floats); every pixel then runs the reference's two window
//                   passes in the reference's order (dy outer, dx inner), so the maps are
//                   bit-identical to the CPU restatement. The tile's combined losses are summed in
//                   fp64 with a fixed tree (deterministic; the reference uses float atomics).
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

// One wave per 16x16 tile, four vertically adjacent pixels per lane (lane l: column l % 16, rows
// 4 (l / 16) .. + 3). Staged row r (0..13 of the lane's window rows) is read once per (r, dx) and
// feeds all four pixels, pixel p with the weight of dy = r - p -- zero where r - p lies outside
// [0, 10], which adds an exact +0 (every term is finite) -- so each pixel still sums its taps
// dy-major, dx-minor: the reference's order, bit-identical maps. The four weights of a (r, dx) sit
// in one 16-B LDS word (one broadcast read). wsum is the same 121-term sum for every pixel, formed
// once. Row stride 28 floats: the lane halves (rows 4 apart, 112 dwords = 16 banks) read disjoint
// banks. (Round 4: one pixel per thread, 3 LDS reads per tap, 155 us at 1080p.)
constexpr uint32_t kLossPx = 4;                     // pixels per lane
constexpr uint32_t kLossStride = 28;
constexpr uint32_t kLossRows = kLossPx + 2 * kLossR;  // staged rows one lane reads (14)
// (Rows 0-2 and 11-13 only for the pixels whose window holds them -- 27 % fewer taps -- compiled to
// 203 VGPRs, 2 waves per SIMD, whatever the row loop's shape: not kept.)

// One staged row of the two window passes for the lane's pixels P0..P1 (the pixels whose window
// holds the row); the row's weights for the four pixels come from one 16-B LDS word per dx.
template <int P0, int P1>
__device__ __forceinline__ void loss_means_row(const float* rx, const float* ry, const float4* wrow,
                                               float (&mx)[kLossPx], float (&my)[kLossPx]) {
#pragma unroll
    for (int dx = 0; dx < 11; dx++) {
        const float a = rx[dx], b = ry[dx];
        const float4 w4 = wrow[dx];
        const float wv[kLossPx] = {w4.x, w4.y, w4.z, w4.w};
#pragma unroll
        for (int p = P0; p <= P1; p++) {
            mx[p] += wv[p] * a;
            my[p] += wv[p] * b;
        }
    }
}
template <int P0, int P1>
__device__ __forceinline__ void loss_moments_row(const float* rx, const float* ry, const float4* wrow,
                                                 const float (&mx)[kLossPx], const float (&my)[kLossPx],
                                                 float (&vx)[kLossPx], float (&vy)[kLossPx], float (&cxy)[kLossPx]) {
#pragma unroll
    for (int dx = 0; dx < 11; dx++) {
        const float sa = rx[dx], sb = ry[dx];
        const float4 w4 = wrow[dx];
        const float wv[kLossPx] = {w4.x, w4.y, w4.z, w4.w};
#pragma unroll
        for (int p = P0; p <= P1; p++) {
            const float a = sa - mx[p];
            const float b = sb - my[p];
            vx[p] += wv[p] * a * a;
            vy[p] += wv[p] * b * b;
            cxy[p] += wv[p] * a * b;
        }
    }
}

__global__ __launch_bounds__(64) void loss_kernel(const uint32_t* __restrict__ rendered,
                                                  const uint32_t* __restrict__ gt, uint32_t w,
                                                  uint32_t h, float lambda,
                                                  float* __restrict__ maps, double* __restrict__ partial) {
    __shared__ float sx[kLossW][kLossStride];
    __shared__ float sy[kLossW][kLossStride];
    __shared__ float4 swt[kLossRows][11];  // (r, dx) -> the weights of dy = r - p, p = 0..3
    const uint32_t tiles_x = (w + kTile - 1) / kTile;
    const uint32_t tx = blockIdx.x % tiles_x, ty = blockIdx.x / tiles_x;
    const uint32_t t = threadIdx.x;
    const int x0 = (int)(tx * kTile) - kLossR, y0 = (int)(ty * kTile) - kLossR;
    // w = exp(-dist_sq / two_sigma_sq), sigma = 1.5 (:393-395, 410-411), pinned exp
    for (uint32_t k = t; k < kLossRows * 11u; k += 64u) {
        const int r = (int)(k / 11u), dx = (int)(k % 11u) - kLossR;
        float wv[kLossPx];
#pragma unroll
        for (int p = 0; p < (int)kLossPx; p++) {
            const int dy = r - p - kLossR;
            const float dist_sq = (float)(dx * dx + dy * dy);
            wv[p] = (r - p >= 0 && r - p <= 10) ? gs_expf(-dist_sq / (2.0f * 1.5f * 1.5f)) : 0.0f;
        }
        swt[k / 11u][k % 11u] = make_float4(wv[0], wv[1], wv[2], wv[3]);
    }
    // stage grey values with the reference's clamp-to-edge addressing (:404-406)
    for (uint32_t k = t; k < (uint32_t)(kLossW * kLossW); k += 64u) {
        const int ly = (int)k / kLossW, lx = (int)k % kLossW;
        int px = x0 + lx, py = y0 + ly;
        px = px < 0 ? 0 : (px > (int)w - 1 ? (int)w - 1 : px);
        py = py < 0 ? 0 : (py > (int)h - 1 ? (int)h - 1 : py);
        const uint32_t r = rendered[(size_t)py * w + px], g = gt[(size_t)py * w + px];
        sx[ly][lx] = (unorm8(r, 0) + unorm8(r, 1) + unorm8(r, 2)) / 3.0f;
        sy[ly][lx] = (unorm8(g, 0) + unorm8(g, 1) + unorm8(g, 2)) / 3.0f;
    }
    __syncthreads();
    float wsum = 0.0f;  // (:398-428's running sum of the weights, identical for every pixel)
#pragma unroll 1
    for (int dy = 0; dy < 11; dy++)
#pragma unroll
        for (int dx = 0; dx < 11; dx++) wsum += swt[dy][dx].x;
    const uint32_t lx = t & 15u, ly0 = (t >> 4) * kLossPx;
    // SSIM, first pass: weighted means (:398-428)
    float mu_x[kLossPx], mu_y[kLossPx];
#pragma unroll
    for (uint32_t p = 0; p < kLossPx; p++) mu_x[p] = mu_y[p] = 0.0f;
#pragma unroll 1
    for (uint32_t r = 0; r < kLossRows; r++) loss_means_row<0, 3>(&sx[ly0 + r][lx], &sy[ly0 + r][lx], swt[r], mu_x, mu_y);
#pragma unroll
    for (uint32_t p = 0; p < kLossPx; p++) {
        mu_x[p] /= wsum;
        mu_y[p] /= wsum;
    }
    // second pass: variances and covariance (:431-468)
    float vx[kLossPx], vy[kLossPx], cxy[kLossPx];
#pragma unroll
    for (uint32_t p = 0; p < kLossPx; p++) vx[p] = vy[p] = cxy[p] = 0.0f;
#pragma unroll 1
    for (uint32_t r = 0; r < kLossRows; r++)
        loss_moments_row<0, 3>(&sx[ly0 + r][lx], &sy[ly0 + r][lx], swt[r], mu_x, mu_y, vx, vy, cxy);
    double contrib = 0.0;
#pragma unroll
    for (uint32_t p = 0; p < kLossPx; p++) {
        const uint32_t x = tx * kTile + lx, y = ty * kTile + ly0 + p;
        if (x >= w || y >= h) continue;
        const size_t pix = (size_t)y * w + x;
        // L1 (:332-334)
        const uint32_t r = rendered[pix], g = gt[pix];
        const float l1 = (fabsf(unorm8(r, 0) - unorm8(g, 0)) + fabsf(unorm8(r, 1) - unorm8(g, 1)) +
                          fabsf(unorm8(r, 2) - unorm8(g, 2))) / 3.0f;
        const float C1 = 0.01f * 0.01f, C2 = 0.03f * 0.03f;  // :356-358
        const float vxp = vx[p] / wsum, vyp = vy[p] / wsum, cxyp = cxy[p] / wsum;
        const float num = (2.0f * mu_x[p] * mu_y[p] + C1) * (2.0f * cxyp + C2);
        const float den = (mu_x[p] * mu_x[p] + mu_y[p] * mu_y[p] + C1) * (vxp + vyp + C2);
        const float ssim = num / den;
        const float dssim = fminf(fmaxf((1.0f - ssim) / 2.0f, 0.0f), 1.0f);
        const float comb = (1.0f - lambda) * l1 + lambda * dssim;  // :508
        if (maps) {
            const size_t np = (size_t)w * h;
            maps[pix] = l1;
            maps[np + pix] = dssim;
            maps[2 * np + pix] = comb;
        }
        contrib += (double)comb;
    }
    contrib = wave_sum_f64(contrib);
    if (t == 0) partial[blockIdx.x] = contrib;
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
    hipLaunchKernelGGL(loss_kernel, dim3(nb), dim3(64), 0, st, rendered, gt, w, h, lambda, maps,
                       partial);
    hipLaunchKernelGGL(loss_final_kernel, dim3(1), dim3(1024), 0, st, partial, nb,
                       (uint64_t)w * h, loss);
    return hipGetLastError();
}

}  // namespace gs
