// refcall_shape.cpp — compile-only check that the reference's own call sites of the hot path's
// operator classes compile against include/gs_tiled_rasterizer.hpp once the Metal types are
// substituted: MTL::CommandQueue* -> hipStream_t, MTL::Buffer* of records ->
// a device pointer of the record type, MTL::Texture* -> gsplat::Texture*. Every call keeps the
// argument list of the reference line it cites. Nothing here runs (tests/test_capi.py compiles it
// with hipcc -fsyntax-only).
#include "gs_tiled_rasterizer.hpp"

namespace {

// MTLEngine's members used by trainStep / train (mtl_engine.hpp:80-140), substituted
struct EngineShape {
    hipStream_t commandQueue = nullptr;
    GsGaussian* gaussianBuffer = nullptr;
    gsplat::Float3* positionBuffer = nullptr;
    GsGradients* gaussianGradients = nullptr;
    gsplat::Texture* renderTarget = nullptr;
    size_t gaussianCount = 0;
    size_t totalIterations = 0;
    float sceneExtent = 1.0f;
    gsplat::TiledRasterizer* tiledRasterizer = nullptr;
    gsplat::DensityController* densityController = nullptr;
    gsplat::AdamOptimizer* optimizer = nullptr;

    float trainStep(gsplat::Texture* groundTruth, const GsTiledUniforms& uniforms, float lr_position,
                    float lr_scale, float lr_rotation, float lr_opacity, float lr_sh) {
        // mtl_engine.mm:973
        tiledRasterizer->forward(commandQueue, gaussianBuffer, gaussianCount, uniforms, renderTarget);
        // mtl_engine.mm:994-995
        tiledRasterizer->backward(commandQueue, gaussianBuffer, gaussianGradients, gaussianCount,
                                  uniforms, renderTarget, groundTruth);
        // mtl_engine.mm:998
        densityController->accumulateGradients(commandQueue, gaussianGradients, gaussianCount);
        // mtl_engine.mm:1001-1006
        optimizer->step(commandQueue, gaussianBuffer, gaussianGradients,
                        lr_position,
                        lr_scale,
                        lr_rotation,
                        lr_opacity,
                        lr_sh);
        return 0.0f;
    }

    void densify(float focalLength, float imageWidth, float avgDepth) {
        size_t oldCount = gaussianCount;
        // mtl_engine.mm:1142-1149
        densityController->apply(commandQueue, gaussianBuffer, positionBuffer,
                                 nullptr, gaussianCount, totalIterations,
                                 0.0002f,
                                 0.005f,  // min_opacity: official uses 0.005
                                 0.1f * sceneExtent,
                                 focalLength,
                                 imageWidth,
                                 avgDepth);
        // mtl_engine.mm:1159-1166
        if (optimizer) {
            optimizer->resizeIfNeeded(gaussianCount);
            if (gaussianCount > oldCount) {
                optimizer->resetStateForNewGaussians(oldCount);
            }
        }
    }

    void opacityReset() {
        // mtl_engine.mm:1188-1191
        optimizer->resetOpacityMomentum();
        optimizer->resetScaleMomentum();
        densityController->resetAccumulator(gaussianCount);
    }
};

}  // namespace

// MTLEngine::init (mtl_engine.mm:314-327) and one training iteration's sequence
void refcall_shape(float sceneExtent, GsTiledUniforms uniforms, gsplat::Texture* gt) {
    gsplat::DensityController::setSceneExtent(sceneExtent);  // mtl_engine.mm:314, a static call
    gsplat::DensityStats s{};                                // density_control.hpp:13-17
    (void)(s.numPruned + s.numCloned + s.numSplit);
    EngineShape e;
    e.trainStep(gt, uniforms, 0.00016f, 0.005f, 0.001f, 0.025f, 0.0025f);
    e.densify(1920.0f, 1920.0f, 2.0f * sceneExtent);
    e.opacityReset();
}
