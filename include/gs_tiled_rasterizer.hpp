// gs_tiled_rasterizer.hpp — C++ host mirror of the reference's operator classes over the C-ABI.
//
//   gsplat::TiledRasterizer    <- GuassianSplatting/tiled_rasterizer.hpp:56-124
//   gsplat::DensityController  <- GuassianSplatting/density_control.hpp:20-62
//   gsplat::AdamOptimizer      <- GuassianSplatting/optimizer.hpp:23-95
//
// Same method names, argument lists and meaning, with the Metal objects replaced: an
// MTL::CommandQueue is a hipStream_t, an MTL::Buffer of records a device pointer of the same
// record type, an RGBA8Unorm MTL::Texture a gsplat::Texture (device image + its size, which an
// MTL::Texture carries). With those substitutions the reference's own call sites compile unchanged
// (tests/cpp/refcall_shape.cpp keeps mtl_engine.mm's argument lists and is compiled by
// tests/test_capi.py). Error behaviour follows the reference: a failure is printed to stderr and
// the call returns (here: false / zero statistics) instead of throwing (tiled_rasterizer.mm:187-198,
// 457-460).
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

// An RGBA8Unorm render target or image (the reference's MTL::Texture, mtl_engine.mm:722): device
// memory [height][width], each texel packed R | G << 8 | B << 16 | A << 24.
struct Texture {
    uint32_t* data = nullptr;
    uint32_t width = 0, height = 0;
};

// simd_float3 (16 B) of the reference's position buffer (mtl_engine.mm:285-290)
struct alignas(16) Float3 {
    float x, y, z, _pad;
};
static_assert(sizeof(Float3) == 16, "simd_float3 is 16 B");

// DensityStats (density_control.hpp:13-17)
struct DensityStats {
    uint32_t numPruned = 0;
    uint32_t numCloned = 0;
    uint32_t numSplit = 0;
};

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
    bool setTileSortPath(int mode) { return gs_ok(gs_set_tile_sort_path(h_, mode), "setTileSortPath"); }
    bool setBackwardSplit(int tiles) { return gs_ok(gs_set_backward_split(h_, tiles), "setBackwardSplit"); }
    bool setChainCompact(int mode) { return gs_ok(gs_set_chain_compact(h_, mode), "setChainCompact"); }

    // forward(queue, gaussianBuffer, gaussianCount, uniforms, outputTexture) (tiled_rasterizer.hpp:63-67)
    bool forward(hipStream_t queue, const GsGaussian* gaussianBuffer, size_t gaussianCount,
                 const GsTiledUniforms& uniforms, Texture* outputTexture, float* outputRgb = nullptr) {
        if (!outputTexture) return gs_ok(GS_E_INVALID, "TiledRasterizer::forward (null texture)");
        return forward(queue, gaussianBuffer, gaussianCount, uniforms, outputTexture->data,
                       outputTexture->width, outputTexture->height, outputRgb);
    }
    // the same with the render target as a raw device image of the given size
    bool forward(hipStream_t queue, const GsGaussian* gaussianBuffer, size_t gaussianCount,
                 const GsTiledUniforms& uniforms, uint32_t* outputTexture, uint32_t width,
                 uint32_t height, float* outputRgb = nullptr) {
        return gs_ok(gs_forward(h_, queue, gaussianBuffer, gaussianCount, &uniforms, width, height,
                                outputTexture, outputRgb),
                     "TiledRasterizer::forward");
    }

    // backward(queue, gaussianBuffer, gradientBuffer, gaussianCount, uniforms, rendered,
    //          groundTruth) (tiled_rasterizer.hpp:69-75)
    bool backward(hipStream_t queue, const GsGaussian* gaussianBuffer, GsGradients* gradientBuffer,
                  size_t gaussianCount, const GsTiledUniforms& uniforms, const Texture* renderedTexture,
                  const Texture* groundTruthTexture) {
        if (!renderedTexture || !groundTruthTexture)
            return gs_ok(GS_E_INVALID, "TiledRasterizer::backward (null texture)");
        return backward(queue, gaussianBuffer, gradientBuffer, gaussianCount, uniforms,
                        renderedTexture->data, groundTruthTexture->data);
    }
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
    // gradientBuffer, or gradient rows (GS_GRAD_ROW_FLOATS per Gaussian) + per-view viewspace rows
    bool backwardChain(hipStream_t queue, const GsGaussian* gaussianBuffer, GsGradients* gradientBuffer,
                       float* rows14, float* viewspace2, size_t gaussianCount, const GsTiledUniforms& uniforms,
                       size_t first, size_t count) {
        return gs_ok(gs_backward_chain(h_, queue, gaussianBuffer, gradientBuffer, rows14, viewspace2,
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
    // DensityController(MTL::Device*, MTL::Library*) (density_control.hpp:22). `capacity` only
    // pre-sizes the accumulators (they grow with the largest count seen); `maxGaussians` is the
    // population cap of apply, the reference's MAX_GAUSSIANS (1.5M, density_control.mm:27,
    // 360-382): 0 = unlimited.
    explicit DensityController(int device, uint32_t capacity = 0, uint64_t maxGaussians = 0) {
        gs_ok(gs_density_create(device, capacity, &d_), "DensityController");
        if (d_ && maxGaussians) gs_density_set_max_gaussians(d_, maxGaussians);
    }
    ~DensityController() { gs_density_destroy(d_); }
    DensityController(const DensityController&) = delete;
    DensityController& operator=(const DensityController&) = delete;

    // static void setSceneExtent(float) (density_control.hpp:48): process-wide like the reference's
    // file static (density_control.mm:41, 79-84); every controller applies with the current value
    static void setSceneExtent(float extent) {
        sceneExtentRef() = extent;
        sceneExtentSetRef() = true;
    }
    static float sceneExtent() { return sceneExtentRef(); }
    void setMaxGaussians(uint64_t maxGaussians) { gs_density_set_max_gaussians(d_, maxGaussians); }

    // accumulateGradients(queue, gradients, gaussianCount) (density_control.hpp:40-42)
    bool accumulateGradients(hipStream_t queue, const GsGradients* gradients, size_t gaussianCount) {
        return gs_ok(gs_density_accumulate(d_, queue, gradients, gaussianCount),
                     "DensityController::accumulateGradients");
    }
    // resetAccumulator(gaussianCount) (density_control.hpp:45)
    bool resetAccumulator(size_t gaussianCount, hipStream_t queue = nullptr) {
        return gs_ok(gs_density_reset(d_, queue, gaussianCount), "resetAccumulator");
    }

    // apply with the reference's argument list (density_control.hpp:26-37; the call at
    // mtl_engine.mm:1142-1149 compiles unchanged). Like the reference it replaces the caller's
    // Gaussian buffer (the old one is released with gs_free, the new one is library memory; release
    // it with gs_free) and position buffer (hipFree / hipMalloc) and rewrites the count.
    // gradThreshold, minOpacity and maxScale are accepted and ignored exactly as the reference
    // ignores them (it uses its file constants: density_control.mm:246-247, 289, 313); gradientAccum
    // is unused there too. The split offsets are keyed by the iteration (seed), so replicas on
    // several GPUs densify identically.
    DensityStats apply(hipStream_t queue, GsGaussian*& gaussianBuffer, Float3*& positionBuffer,
                       void* gradientAccum, size_t& gaussianCount, size_t iteration,
                       float gradThreshold = 0.0002f, float minOpacity = 0.005f, float maxScale = 0.5f,
                       float focalLength = 500.0f, float imageWidth = 800.0f, float avgDepth = 5.0f) {
        (void)gradientAccum;
        (void)gradThreshold;
        (void)minOpacity;
        (void)maxScale;
        const GsDensityStats s = apply(queue, gaussianBuffer, gaussianCount, iteration, focalLength,
                                       imageWidth, avgDepth, /*seed*/ iteration, /*ownsBuffer*/ true);
        DensityStats out;
        out.numPruned = s.num_pruned;
        out.numCloned = s.num_cloned;
        out.numSplit = s.num_split;
        // the position buffer follows the new Gaussians (density_control.mm:471-489)
        Float3* pos = nullptr;
        if (hipMalloc(reinterpret_cast<void**>(&pos), (gaussianCount ? gaussianCount : 1) * sizeof(Float3)) != hipSuccess) {
            gs_ok(GS_E_NOMEM, "DensityController::apply (position buffer)");
            return out;
        }
        if (gaussianCount &&
            hipMemcpy2DAsync(pos, sizeof(Float3), gaussianBuffer, sizeof(GsGaussian), sizeof(Float3),
                             gaussianCount, hipMemcpyDeviceToDevice, queue) != hipSuccess)
            gs_ok(GS_E_HIP, "DensityController::apply (position copy)");
        if (positionBuffer) (void)hipFree(positionBuffer);
        positionBuffer = pos;
        return out;
    }

    // apply(queue, gaussianBuffer&, gaussianCount&, iteration, ...) without the position buffer:
    // replaces the caller's buffer; the old one is released with gs_free when `ownsBuffer`.
    GsDensityStats apply(hipStream_t queue, GsGaussian*& gaussianBuffer, size_t& gaussianCount,
                         size_t iteration, float focalLength = 500.0f, float imageWidth = 800.0f,
                         float avgDepth = 5.0f, uint64_t seed = 0, bool ownsBuffer = true) {
        GsDensityStats stats = {0, 0, 0, 0};
        GsGaussian* out = nullptr;
        size_t n = 0;
        // the process-wide extent (the reference's static) overrides the handle's only once it has
        // been set; an extent set through the C-ABI on handle() is kept otherwise
        if (sceneExtentSetRef()) gs_density_set_scene_extent(d_, sceneExtentRef());
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
    static float& sceneExtentRef() {
        static float extent = 1.0f;  // density_control.mm:41
        return extent;
    }
    static bool& sceneExtentSetRef() {
        static bool set = false;
        return set;
    }
    gs_density* d_ = nullptr;
};

// AdamOptimizer(MTL::Device*, MTL::Library*, size_t numGaussians) <- optimizer.hpp:23-95. The
// optimizer tracks the Gaussian count like the reference (constructor, resizeIfNeeded); the
// count-free methods act on it. (The reference dispatches its step over the buffer capacity,
// optimizer.mm:288; here every step covers exactly the current count.)
class AdamOptimizer {
public:
    explicit AdamOptimizer(int device, size_t numGaussians = 0) : n_(numGaussians) {
        gs_ok(gs_adam_create(device, (uint32_t)numGaussians, &a_), "AdamOptimizer");
    }
    ~AdamOptimizer() { gs_adam_destroy(a_); }
    AdamOptimizer(const AdamOptimizer&) = delete;
    AdamOptimizer& operator=(const AdamOptimizer&) = delete;

    // step(queue, gaussians, gradients, lr_position, lr_scale, lr_rotation, lr_opacity, lr_sh)
    // (optimizer.hpp:29-41; the call at mtl_engine.mm:1001-1006)
    bool step(hipStream_t queue, GsGaussian* gaussians, const GsGradients* gradients,
              float lr_position = 0.00016f, float lr_scale = 0.005f, float lr_rotation = 0.001f,
              float lr_opacity = 0.05f, float lr_sh = 0.0025f) {
        return step(queue, gaussians, gradients, n_, lr_position, lr_scale, lr_rotation, lr_opacity, lr_sh);
    }
    // the same over an explicit count
    bool step(hipStream_t queue, GsGaussian* gaussians, const GsGradients* gradients, size_t numGaussians,
              float lr_position = 0.00016f, float lr_scale = 0.005f, float lr_rotation = 0.001f,
              float lr_opacity = 0.05f, float lr_sh = 0.0025f) {
        const float lrs[5] = {lr_position, lr_scale, lr_rotation, lr_opacity, lr_sh};
        return gs_ok(gs_adam_step(a_, queue, gaussians, gradients, numGaussians, lrs), "AdamOptimizer::step");
    }
    bool reset(hipStream_t queue = nullptr) { return gs_ok(gs_adam_reset(a_, queue), "AdamOptimizer::reset"); }
    // resizeIfNeeded(newNumGaussians) (optimizer.hpp:46): grow keeping the state; the count follows
    bool resizeIfNeeded(size_t n, hipStream_t queue = nullptr) {
        n_ = n;
        return gs_ok(gs_adam_resize(a_, queue, n), "AdamOptimizer::resizeIfNeeded");
    }
    // resetStateForNewGaussians(startIdx) (optimizer.hpp:55): zero the moments of [startIdx, count)
    bool resetStateForNewGaussians(size_t startIdx) { return resetStateForNewGaussians(startIdx, n_); }
    bool resetStateForNewGaussians(size_t startIdx, size_t n, hipStream_t queue = nullptr) {
        return gs_ok(gs_adam_reset_new(a_, queue, startIdx, n), "AdamOptimizer::resetStateForNewGaussians");
    }
    // resetOpacityMomentum() / resetScaleMomentum() (optimizer.hpp:49-52)
    bool resetOpacityMomentum() { return resetOpacityMomentum(n_); }
    bool resetOpacityMomentum(size_t n, hipStream_t queue = nullptr) {
        return gs_ok(gs_adam_reset_opacity_momentum(a_, queue, n), "AdamOptimizer::resetOpacityMomentum");
    }
    bool resetScaleMomentum() { return resetScaleMomentum(n_); }
    bool resetScaleMomentum(size_t n, hipStream_t queue = nullptr) {
        return gs_ok(gs_adam_reset_scale_momentum(a_, queue, n), "AdamOptimizer::resetScaleMomentum");
    }
    // moments follow a DensityController::apply (survivors keep theirs, new Gaussians start at 0)
    bool followDensity(const DensityController& dc, size_t nIn, size_t nOut, hipStream_t queue = nullptr) {
        n_ = nOut;
        return gs_ok(gs_adam_follow_density(a_, queue, dc.handle(), nIn, nOut), "AdamOptimizer::followDensity");
    }
    uint32_t getTimestep() const {
        uint32_t t = 0;
        gs_adam_timestep(a_, &t);
        return t;
    }
    size_t count() const { return n_; }

private:
    gs_adam* a_ = nullptr;
    size_t n_ = 0;
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
