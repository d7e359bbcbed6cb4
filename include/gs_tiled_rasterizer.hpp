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

private:
    gs_density* d_ = nullptr;
};

}  // namespace gsplat
