// gs_tiled_rasterizer.hpp — C++ host mirror of the reference's operator classes over the C-ABI.
//
//   gsplat::TiledRasterizer    <- GuassianSplatting/tiled_rasterizer.hpp:56-124
//   gsplat::DensityController  <- GuassianSplatting/density_control.hpp:22-48
//
// Same method names and argument meaning, with MTL objects replaced by device pointers and a
// hipStream_t (the reference's MTL::CommandQueue). Error behaviour follows the reference: a
// failure is printed to stderr and the call returns (here: false) instead of throwing
// (tiled_rasterizer.mm:187-198, 457-460).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdio>

#include "gs_rasterizer.h"

namespace gsplat {

inline bool gs_ok(int rc, const char* where) {
    if (rc == GS_OK) return true;
    std::fprintf(stderr, "%s failed (%d): %s\n", where, rc, gs_last_error());
    return false;
}

class TiledRasterizer {
public:
    // TiledRasterizer(MTL::Device*, MTL::Library*, uint32_t maxGaussians)
    TiledRasterizer(int device, uint32_t maxGaussians, uint32_t maxWidth = 0, uint32_t maxHeight = 0) {
        gs_ok(gs_create(device, maxGaussians, maxWidth, maxHeight, &h_), "TiledRasterizer");
    }
    ~TiledRasterizer() { gs_destroy(h_); }
    TiledRasterizer(const TiledRasterizer&) = delete;
    TiledRasterizer& operator=(const TiledRasterizer&) = delete;

    bool valid() const { return h_ != nullptr; }
    bool reservePairs(uint64_t maxPairs) { return gs_ok(gs_reserve_pairs(h_, maxPairs), "reservePairs"); }

    // forward(queue, gaussianBuffer, gaussianCount, uniforms, outputTexture)
    bool forward(hipStream_t queue, const GsGaussian* gaussianBuffer, size_t gaussianCount,
                 const GsTiledUniforms& uniforms, uint32_t* outputTexture, uint32_t width,
                 uint32_t height, float* outputRgb = nullptr) {
        return gs_ok(gs_forward(h_, queue, gaussianBuffer, gaussianCount, &uniforms, width, height,
                                outputTexture, outputRgb),
                     "TiledRasterizer::forward");
    }

    // backward(queue, gaussianBuffer, gradientBuffer, gaussianCount, uniforms, rendered, gt)
    bool backward(hipStream_t queue, const GsGaussian* gaussianBuffer, GsGradients* gradientBuffer,
                  size_t gaussianCount, const GsTiledUniforms& uniforms,
                  const uint32_t* renderedTexture, const uint32_t* groundTruthTexture) {
        return gs_ok(gs_backward(h_, queue, gaussianBuffer, gradientBuffer, gaussianCount,
                                 &uniforms, renderedTexture, groundTruthTexture),
                     "TiledRasterizer::backward");
    }

    // backward in two parts (gs_backward_blend + gs_backward_chain over a range of Gaussians),
    // for callers that overlap the chain with a collective
    bool backwardBlend(hipStream_t queue, const GsGaussian* gaussianBuffer, size_t gaussianCount,
                       const GsTiledUniforms& uniforms, const uint32_t* renderedTexture,
                       const uint32_t* groundTruthTexture) {
        return gs_ok(gs_backward_blend(h_, queue, gaussianBuffer, gaussianCount, &uniforms,
                                       renderedTexture, groundTruthTexture),
                     "TiledRasterizer::backwardBlend");
    }
    bool backwardChain(hipStream_t queue, const GsGaussian* gaussianBuffer, GsGradients* gradientBuffer,
                       float* packed16, size_t gaussianCount, const GsTiledUniforms& uniforms,
                       size_t first, size_t count) {
        return gs_ok(gs_backward_chain(h_, queue, gaussianBuffer, gradientBuffer, packed16,
                                       gaussianCount, &uniforms, first, count),
                     "TiledRasterizer::backwardChain");
    }

    bool frameStats(GsFrameStats* out) { return gs_ok(gs_frame_stats(h_, out), "frameStats"); }
    gs_handle* handle() const { return h_; }

private:
    gs_handle* h_ = nullptr;
};

class DensityController {
public:
    // DensityController(MTL::Device*, MTL::Library*)
    explicit DensityController(int device, uint32_t maxGaussians = 0) {
        gs_ok(gs_density_create(device, maxGaussians, &d_), "DensityController");
    }
    ~DensityController() { gs_density_destroy(d_); }
    DensityController(const DensityController&) = delete;
    DensityController& operator=(const DensityController&) = delete;

    // static void setSceneExtent(float) — per controller here (the reference uses a file static)
    void setSceneExtent(float extent) { gs_density_set_scene_extent(d_, extent); }
    void setMaxGaussians(uint64_t maxGaussians) { gs_density_set_max_gaussians(d_, maxGaussians); }

    bool accumulateGradients(hipStream_t queue, const GsGradients* gradients, size_t gaussianCount) {
        return gs_ok(gs_density_accumulate(d_, queue, gradients, gaussianCount),
                     "DensityController::accumulateGradients");
    }
    bool resetAccumulator(size_t gaussianCount, hipStream_t queue = nullptr) {
        return gs_ok(gs_density_reset(d_, queue, gaussianCount), "resetAccumulator");
    }

    // apply(queue, gaussianBuffer&, ..., gaussianCount&, iteration, ...): like the reference it
    // replaces the caller's buffer; the old one is released with gs_free when `ownsBuffer`.
    GsDensityStats apply(hipStream_t queue, GsGaussian*& gaussianBuffer, size_t& gaussianCount,
                         size_t iteration, float focalLength = 500.0f, float imageWidth = 800.0f,
                         float avgDepth = 5.0f, uint64_t seed = 0, bool ownsBuffer = true) {
        GsDensityStats stats = {0, 0, 0, 0};
        GsGaussian* out = nullptr;
        size_t n = 0;
        if (!gs_ok(gs_density_apply(d_, queue, gaussianBuffer, gaussianCount, &out, &n, iteration,
                                    focalLength, imageWidth, avgDepth, seed, &stats),
                   "DensityController::apply"))
            return stats;
        if (ownsBuffer) gs_free(gaussianBuffer);
        gaussianBuffer = out;
        gaussianCount = n;
        return stats;
    }

    gs_density* handle() const { return d_; }

private:
    gs_density* d_ = nullptr;
};

// AdamOptimizer(MTL::Device*, MTL::Library*, size_t numGaussians) <- optimizer.hpp:22-95
class AdamOptimizer {
public:
    explicit AdamOptimizer(int device, uint32_t numGaussians = 0) {
        gs_ok(gs_adam_create(device, numGaussians, &a_), "AdamOptimizer");
    }
    ~AdamOptimizer() { gs_adam_destroy(a_); }
    AdamOptimizer(const AdamOptimizer&) = delete;
    AdamOptimizer& operator=(const AdamOptimizer&) = delete;

    // step(queue, gaussians, gradients, lr_position, lr_scale, lr_rotation, lr_opacity, lr_sh)
    bool step(hipStream_t queue, GsGaussian* gaussians, const GsGradients* gradients, size_t numGaussians,
              float lr_position = 0.00016f, float lr_scale = 0.005f, float lr_rotation = 0.001f,
              float lr_opacity = 0.05f, float lr_sh = 0.0025f) {
        const float lrs[5] = {lr_position, lr_scale, lr_rotation, lr_opacity, lr_sh};
        return gs_ok(gs_adam_step(a_, queue, gaussians, gradients, numGaussians, lrs), "AdamOptimizer::step");
    }
    bool reset(hipStream_t queue = nullptr) { return gs_ok(gs_adam_reset(a_, queue), "AdamOptimizer::reset"); }
    bool resizeIfNeeded(size_t n, hipStream_t queue = nullptr) {
        return gs_ok(gs_adam_resize(a_, queue, n), "AdamOptimizer::resizeIfNeeded");
    }
    bool resetStateForNewGaussians(size_t startIdx, size_t n, hipStream_t queue = nullptr) {
        return gs_ok(gs_adam_reset_new(a_, queue, startIdx, n), "AdamOptimizer::resetStateForNewGaussians");
    }
    bool resetOpacityMomentum(size_t n, hipStream_t queue = nullptr) {
        return gs_ok(gs_adam_reset_opacity_momentum(a_, queue, n), "AdamOptimizer::resetOpacityMomentum");
    }
    bool resetScaleMomentum(size_t n, hipStream_t queue = nullptr) {
        return gs_ok(gs_adam_reset_scale_momentum(a_, queue, n), "AdamOptimizer::resetScaleMomentum");
    }
    // moments follow a DensityController::apply (survivors keep theirs, new Gaussians start at 0)
    bool followDensity(const DensityController& dc, size_t nIn, size_t nOut, hipStream_t queue = nullptr) {
        return gs_ok(gs_adam_follow_density(a_, queue, dc.handle(), nIn, nOut), "AdamOptimizer::followDensity");
    }
    uint32_t getTimestep() const {
        uint32_t t = 0;
        gs_adam_timestep(a_, &t);
        return t;
    }

private:
    gs_adam* a_ = nullptr;
};

// MTLEngine::computeLoss (mtl_engine.mm:769-853): L1 + lambda D-SSIM, mean over the image
class Loss {
public:
    explicit Loss(int device) { gs_ok(gs_loss_create(device, &l_), "Loss"); }
    ~Loss() { gs_loss_destroy(l_); }
    Loss(const Loss&) = delete;
    Loss& operator=(const Loss&) = delete;
    // d_loss: one float on the device; d_maps (nullable): [3][h][w] L1, D-SSIM, combined
    bool compute(hipStream_t queue, const uint32_t* rendered, const uint32_t* gt, uint32_t w, uint32_t h,
                 float lambdaDssim, float* d_loss, float* d_maps = nullptr) {
        return gs_ok(gs_loss_compute(l_, queue, rendered, gt, w, h, lambdaDssim, d_loss, d_maps),
                     "Loss::compute");
    }

private:
    gs_loss* l_ = nullptr;
};

// the training loop's opacity reset (mtl_engine.mm:1173-1186)
inline bool resetOpacity(hipStream_t queue, GsGaussian* gaussians, size_t n, float maxRaw = -4.6f) {
    return gs_ok(gs_opacity_reset(queue, gaussians, n, maxRaw), "resetOpacity");
}

}  // namespace gsplat
