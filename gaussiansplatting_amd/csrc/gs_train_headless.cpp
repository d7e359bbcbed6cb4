// gs_train_headless.cpp — headless C++ caller of the hot path, replaying the per-view sequence
// of MTLEngine::trainStep / train (mtl_engine.mm:856-1192): forward -> loss (L1 + 0.2 D-SSIM) ->
// backward -> density accumulate -> Adam; then, with the reference's conditions, densification
// when DENSIFY_FROM_ITER (500) < iteration < DENSIFY_UNTIL_ITER (15000) and iteration % D == 0
// (apply + moments follow, :1108-1167), and the opacity reset when iteration % R == 0 and
// 0 < iteration < 15000 (raw opacity clamp, opacity and scale momentum resets, accumulator reset,
// :1173-1192). The iteration counter starts at --start-iter (the reference counts from 0; a test
// starts past 500 to reach densification in a few steps). No window, no loaders: the seeded
// synthetic scene of SURVEY.md §8d stands in for COLMAP + images. `--train 0` times the rasterizer
// alone. After a densification the Adam moments follow the Gaussians (survivors keep theirs, new
// ones start at zero: the official 3DGS behaviour); `--ref-moments 1` keeps the reference's own
// behaviour instead: the state is resized and only the tail past the old count is zeroed, the
// survivors' moments staying where they were (mtl_engine.mm:1159-1166).
//
//   gs_train_headless [--n N] [--width W] [--height H] [--seed S] [--steps K] [--warmup W]
//                     [--train 0|1] [--densify-every D] [--opacity-reset-every R] [--start-iter I]
//                     [--ref-moments 0|1]
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../../include/gs_tiled_rasterizer.hpp"

static uint64_t splitmix(uint64_t seed, uint64_t k) {
    uint64_t z = seed + (k + 1) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

static double u01(uint64_t seed, uint64_t k) { return (double)(splitmix(seed, k) >> 40) * 0x1p-24; }

int main(int argc, char** argv) {
    uint32_t n = 1000000, w = 1920, h = 1080, steps = 20, warmup = 3;
    uint32_t train = 1, densify_every = 0, opacity_reset_every = 0, ref_moments = 0;
    uint64_t seed = 3, start_iter = 0;
    const uint64_t kDensifyFrom = 500, kDensifyUntil = 15000;  // mtl_engine.mm:1054-1055
    for (int i = 1; i + 1 < argc; i += 2) {
        if (!strcmp(argv[i], "--n")) n = (uint32_t)atol(argv[i + 1]);
        else if (!strcmp(argv[i], "--width")) w = (uint32_t)atol(argv[i + 1]);
        else if (!strcmp(argv[i], "--height")) h = (uint32_t)atol(argv[i + 1]);
        else if (!strcmp(argv[i], "--seed")) seed = (uint64_t)atoll(argv[i + 1]);
        else if (!strcmp(argv[i], "--steps")) steps = (uint32_t)atol(argv[i + 1]);
        else if (!strcmp(argv[i], "--warmup")) warmup = (uint32_t)atol(argv[i + 1]);
        else if (!strcmp(argv[i], "--train")) train = (uint32_t)atol(argv[i + 1]);
        else if (!strcmp(argv[i], "--densify-every")) densify_every = (uint32_t)atol(argv[i + 1]);
        else if (!strcmp(argv[i], "--opacity-reset-every")) opacity_reset_every = (uint32_t)atol(argv[i + 1]);
        else if (!strcmp(argv[i], "--start-iter")) start_iter = (uint64_t)atoll(argv[i + 1]);
        else if (!strcmp(argv[i], "--ref-moments")) ref_moments = (uint32_t)atol(argv[i + 1]);
    }
    const double kShC0 = 0.28209479177387814, kPi = 3.14159265358979323846;
    std::vector<GsGaussian> g(n);
    const double f = w, cx = w / 2.0, cy = h / 2.0;
    for (uint32_t i = 0; i < n; i++) {
        double u[13];
        for (int k = 0; k < 13; k++) u[k] = u01(seed, 13ull * i + k);
        GsGaussian& q = g[i];
        std::memset(&q, 0, sizeof(q));
        const double z = 2.0 + 8.0 * u[0];
        q.position[0] = (float)((u[1] * w - cx) * z / f);
        q.position[1] = (float)((u[2] * h - cy) * z / f);
        q.position[2] = (float)z;
        for (int k = 0; k < 3; k++) q.scale[k] = (float)std::log(0.5 * std::pow(10.0, u[3 + k]) * z / f);
        const double a = std::sqrt(1.0 - u[6]), b = std::sqrt(u[6]);
        q.rotation[0] = (float)(a * std::sin(2 * kPi * u[7]));
        q.rotation[1] = (float)(a * std::cos(2 * kPi * u[7]));
        q.rotation[2] = (float)(b * std::sin(2 * kPi * u[8]));
        q.rotation[3] = (float)(b * std::cos(2 * kPi * u[8]));
        const double p = 0.05 + 0.9 * u[9];
        q.opacity = (float)std::log(p / (1.0 - p));
        for (int k = 0; k < 3; k++) q.sh[4 * k] = (float)((u[10 + k] - 0.5) / kShC0);
    }
    std::vector<uint32_t> gt((size_t)w * h);
    for (size_t i = 0; i < gt.size(); i++) {
        uint32_t px = 255u << 24;
        for (int c = 0; c < 3; c++) px |= (uint32_t)(splitmix(seed + 1000, 3 * i + c) >> 56) << (8 * c);
        gt[i] = px;
    }
    GsTiledUniforms u;
    std::memset(&u, 0, sizeof(u));
    for (int k = 0; k < 4; k++) u.view[5 * k] = 1.0f;
    u.proj[0] = 2.0f * (float)f / (float)w;
    u.proj[5] = 2.0f * (float)f / (float)h;
    u.proj[8] = 2.0f * (float)cx / (float)w - 1.0f;
    u.proj[9] = 2.0f * (float)cy / (float)h - 1.0f;
    u.proj[10] = 1000.0f / (1000.0f - 0.1f);
    u.proj[11] = 1.0f;
    u.proj[14] = -(1000.0f * 0.1f) / (1000.0f - 0.1f);
    std::memcpy(u.view_proj, u.proj, sizeof(u.proj));  // identity view
    u.screen_size[0] = (float)w;
    u.screen_size[1] = (float)h;
    u.focal[0] = u.focal[1] = (float)f;

    // gradients sized for growth: densification can at most double the population per apply
    const size_t cap = (size_t)n * 4;
    GsGaussian* dg = nullptr;
    GsGradients* dgrad = nullptr;
    uint32_t *drgba = nullptr, *dgt = nullptr;
    float* dloss = nullptr;
    if (hipMalloc(&dg, sizeof(GsGaussian) * n) != hipSuccess ||
        hipMalloc(&dgrad, sizeof(GsGradients) * cap) != hipSuccess ||
        hipMalloc(&drgba, sizeof(uint32_t) * w * h) != hipSuccess ||
        hipMalloc(&dgt, sizeof(uint32_t) * w * h) != hipSuccess ||
        hipMalloc(&dloss, sizeof(float)) != hipSuccess) {
        std::fprintf(stderr, "allocation failed\n");
        return 1;
    }
    hipMemcpy(dg, g.data(), sizeof(GsGaussian) * n, hipMemcpyHostToDevice);
    hipMemcpy(dgt, gt.data(), sizeof(uint32_t) * w * h, hipMemcpyHostToDevice);
    hipStream_t st;
    hipStreamCreate(&st);

    gsplat::TiledRasterizer rast(0, (uint32_t)cap, w, h);
    // the population cap of densification is the buffers' capacity (the reference's MAX_GAUSSIANS
    // plays that role: density_control.mm:27, 360-382)
    gsplat::DensityController dens(0, (uint32_t)cap, cap);
    gsplat::AdamOptimizer adam(0, cap);
    gsplat::Loss loss(0);
    if (!rast.valid()) return 1;
    gsplat::DensityController::setSceneExtent(1.1f * 0.25f * 3.5f);  // the 8-camera rig's spread
    dens.resetAccumulator(n, st);
    const uint32_t tiles = ((w + 15) / 16) * ((h + 15) / 16);
    rast.reservePairs((uint64_t)n * (tiles < 256 ? tiles : 256));
    size_t count = n;
    bool lib_owned = false;  // after the first apply the buffer belongs to the library (gs_free)
    uint64_t iter = start_iter;
    uint64_t applies = 0, pruned = 0, cloned = 0, split = 0, resets = 0;
    auto step = [&]() {
        ++iter;
        bool ok = rast.forward(st, dg, count, u, drgba, w, h);
        if (ok && train) ok = loss.compute(st, drgba, dgt, w, h, 0.2f, dloss);
        ok = ok && rast.backward(st, dg, dgrad, count, u, drgba, dgt) &&
             dens.accumulateGradients(st, dgrad, count);
        if (ok && train) ok = adam.step(st, dg, dgrad, count);
        // shouldDensify (mtl_engine.mm:1112-1114)
        const bool densify = densify_every && iter > kDensifyFrom && iter < kDensifyUntil && iter % densify_every == 0;
        if (ok && train && densify) {
            const size_t n_in = count;
            GsGaussian* before = dg;
            const GsDensityStats s = dens.apply(st, dg, count, iter, (float)f, (float)w, 6.0f, iter, /*ownsBuffer*/ false);
            if (dg != before) {
                if (lib_owned) gs_free(before); else hipFree(before);
                lib_owned = true;
            }
            if (count > cap) return false;
            applies++;
            pruned += s.num_pruned;
            cloned += s.num_cloned;
            split += s.num_split;
            if (ref_moments) {  // mtl_engine.mm:1159-1166: resize, zero only the new tail
                ok = adam.resizeIfNeeded(count, st) &&
                     (count <= n_in || adam.resetStateForNewGaussians(n_in, count, st));
            } else {
                ok = adam.followDensity(dens, n_in, count, st);
            }
            ok = ok && dens.resetAccumulator(count, st);
        }
        // opacity reset (mtl_engine.mm:1173-1192): after densification, with both momentum resets
        // and the accumulator reset
        if (ok && train && opacity_reset_every && iter % opacity_reset_every == 0 && iter > 0 && iter < kDensifyUntil) {
            resets++;
            ok = gsplat::resetOpacity(st, dg, count) && adam.resetOpacityMomentum(count, st) &&
                 adam.resetScaleMomentum(count, st) && dens.resetAccumulator(count, st);
        }
        return ok;
    };
    for (uint32_t i = 0; i < warmup; i++)
        if (!step()) return 1;
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipStreamSynchronize(st);
    hipEventRecord(e0, st);
    for (uint32_t i = 0; i < steps; i++)
        if (!step()) return 1;
    hipEventRecord(e1, st);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    GsFrameStats fs;
    rast.frameStats(&fs);
    float hloss = 0.0f;
    hipMemcpy(&hloss, dloss, sizeof(float), hipMemcpyDeviceToHost);
    const double per = ms / steps;
    std::printf("{\"n\": %zu, \"n_initial\": %u, \"width\": %u, \"height\": %u, \"pairs\": %llu, \"train\": %u, "
                "\"loss\": %.6f, \"ms_per_step\": %.4f, \"gaussians_x_views_per_s\": %.4e, \"last_iter\": %llu, "
                "\"applies\": %llu, \"pruned\": %llu, \"cloned\": %llu, \"split\": %llu, \"opacity_resets\": %llu, "
                "\"moments\": \"%s\"}\n",
                count, n, w, h, (unsigned long long)fs.num_pairs, train, hloss, per, count / (per * 1e-3),
                (unsigned long long)iter, (unsigned long long)applies, (unsigned long long)pruned,
                (unsigned long long)cloned, (unsigned long long)split, (unsigned long long)resets,
                ref_moments ? "reference" : "follow");
    if (lib_owned) gs_free(dg); else hipFree(dg);
    dg = nullptr;
    hipFree(dgrad); hipFree(drgba); hipFree(dgt); hipFree(dloss);
    hipStreamDestroy(st);
    return 0;
}
