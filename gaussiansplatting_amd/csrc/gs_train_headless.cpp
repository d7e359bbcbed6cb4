// gs_train_headless.cpp — headless C++ caller of the hot path, replaying the reference's main()
// sequence (main.mm:392-413): scene -> train (mtl_engine.mm:1047-1221, per view MTLEngine::trainStep
// :856-1025: forward -> loss (L1 + 0.2 D-SSIM) -> backward -> density accumulate -> Adam; then, with
// the reference's conditions, densification when DENSIFY_FROM_ITER (500) < iteration <
// DENSIFY_UNTIL_ITER (15000) and iteration % D == 0 (apply + moments follow, :1108-1167), and the
// opacity reset when iteration % R == 0 and 0 < iteration < 15000 (raw opacity clamp, opacity and
// scale momentum resets, accumulator reset, :1173-1192)) -> exportTrainingViews (:1224-1306, one
// PPM per training image) -> PLYExporter::exportPLY.
//
// Scene: `--colmap DIR` loads a COLMAP binary model (gs_colmap_load), initialises the Gaussians
// from its sparse points (gaussiansFromColmap, main.mm:59-187) and trains over its images in file
// order, one view per iteration (mtl_engine.mm:1085-1093), each rendered at its camera's size with
// the view uniforms of mtl_engine.mm:866-924; the ground truth of image i is `--gt-dir`'s PPM named
// after the image (its extension replaced by .ppm), else the seeded RGBA8 of SURVEY.md §8d (stream
// seed + 1000 + i; images are out of scope). Without --colmap the seeded synthetic scene of
// SURVEY.md §8d, one view at --width x --height, stands in for COLMAP + images. The iteration
// counter starts at --start-iter (the reference counts from 0; a test starts past 500 to reach
// densification in a few steps). `--train 0` times the rasterizer alone. After a densification the
// Adam moments follow the Gaussians (survivors keep theirs, new ones start at zero: the official
// 3DGS behaviour); `--ref-moments 1` keeps the reference's own behaviour instead: the state is
// resized and only the tail past the old count is zeroed (mtl_engine.mm:1159-1166).
//
//   gs_train_headless [--n N] [--width W] [--height H] [--seed S] [--steps K] [--warmup W]
//                     [--train 0|1] [--densify-every D] [--opacity-reset-every R] [--start-iter I]
//                     [--ref-moments 0|1] [--colmap DIR] [--gt-dir DIR]
//                     [--export-views DIR] [--ply OUT.ply] [--dump-gaussians OUT.bin]
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <string>
#include <vector>

#include "../../include/gs_tiled_rasterizer.hpp"

static uint64_t splitmix(uint64_t seed, uint64_t k) {
    uint64_t z = seed + (k + 1) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

static double u01(uint64_t seed, uint64_t k) { return (double)(splitmix(seed, k) >> 40) * 0x1p-24; }

static bool fail_msg(const char* what) {
    std::fprintf(stderr, "%s: %s\n", what, gs_last_error());
    return false;
}

// One training view: its uniforms, render size, ground truth (device) and the apply's camera terms.
struct View {
    GsTiledUniforms u;
    uint32_t w, h, image_id;
    float focal;
    uint32_t* dgt;
};

static void synthetic_gt(std::vector<uint32_t>& gt, uint64_t seed, uint32_t view, uint32_t w, uint32_t h) {
    gt.assign((size_t)w * h, 0u);
    for (size_t i = 0; i < gt.size(); i++) {  // scene.synthetic_ground_truth
        uint32_t px = 255u << 24;
        for (int c = 0; c < 3; c++) px |= (uint32_t)(splitmix(seed + 1000 + view, 3 * i + c) >> 56) << (8 * c);
        gt[i] = px;
    }
}

int main(int argc, char** argv) {
    uint32_t n = 1000000, w = 1920, h = 1080, steps = 20, warmup = 3;
    uint32_t train = 1, densify_every = 0, opacity_reset_every = 0, ref_moments = 0;
    uint64_t seed = 3, start_iter = 0;
    std::string colmap_dir, gt_dir, export_dir, ply_out, dump_out;
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
        else if (!strcmp(argv[i], "--colmap")) colmap_dir = argv[i + 1];
        else if (!strcmp(argv[i], "--gt-dir")) gt_dir = argv[i + 1];
        else if (!strcmp(argv[i], "--export-views")) export_dir = argv[i + 1];
        else if (!strcmp(argv[i], "--ply")) ply_out = argv[i + 1];
        else if (!strcmp(argv[i], "--dump-gaussians")) dump_out = argv[i + 1];
        else {
            std::fprintf(stderr, "unknown option %s\n", argv[i]);
            return 2;
        }
    }
    const double kShC0 = 0.28209479177387814, kPi = 3.14159265358979323846;
    std::vector<GsGaussian> g;
    std::vector<View> views;
    std::vector<std::vector<uint32_t>> gts;
    float extent = 1.1f * 0.25f * 3.5f;  // the synthetic 8-camera rig's spread
    if (!colmap_dir.empty()) {
        gs_colmap* cm = nullptr;
        if (gs_colmap_load(colmap_dir.c_str(), &cm) != GS_OK) return fail_msg("gs_colmap_load"), 1;
        uint32_t ncam = 0, nimg = 0;
        uint64_t npts = 0, ng = 0;
        gs_colmap_counts(cm, &ncam, &nimg, &npts);
        if (nimg == 0) return std::fprintf(stderr, "COLMAP model without images\n"), 1;
        if (gs_colmap_scene_extent(cm, &extent) != GS_OK) return fail_msg("gs_colmap_scene_extent"), 1;
        if (gs_gaussians_from_colmap(cm, extent, nullptr, 0, &ng) != GS_OK) return fail_msg("gs_gaussians_from_colmap"), 1;
        g.resize(ng);
        if (gs_gaussians_from_colmap(cm, extent, g.data(), ng, &ng) != GS_OK) return fail_msg("gs_gaussians_from_colmap"), 1;
        n = (uint32_t)ng;
        w = h = 0;
        for (uint32_t i = 0; i < nimg; i++) {
            GsColmapImage img;
            GsColmapCamera cam;
            if (gs_colmap_image(cm, i, &img) != GS_OK || gs_colmap_camera_by_id(cm, img.camera_id, &cam) != GS_OK)
                return fail_msg("COLMAP image / camera"), 1;
            View v{};
            v.w = cam.width;
            v.h = cam.height;
            v.image_id = img.id;
            v.focal = cam.fx;  // mtl_engine.mm:1118-1121 (images at the camera's size: scale 1)
            if (gs_colmap_uniforms(&cam, &img, v.w, v.h, &v.u) != GS_OK) return fail_msg("gs_colmap_uniforms"), 1;
            std::vector<uint32_t> gt;
            if (!gt_dir.empty()) {
                std::string name = img.name;
                const size_t dot = name.rfind('.');
                if (dot != std::string::npos) name = name.substr(0, dot);
                const std::string path = gt_dir + "/" + name + ".ppm";
                uint32_t pw = 0, ph = 0;
                gt.resize((size_t)v.w * v.h);
                if (gs_ppm_load(path.c_str(), gt.data(), gt.size(), &pw, &ph) != GS_OK) return fail_msg("gs_ppm_load"), 1;
                if (pw != v.w || ph != v.h) return std::fprintf(stderr, "%s: size differs from its camera\n", path.c_str()), 1;
            } else {
                synthetic_gt(gt, seed, i, v.w, v.h);
            }
            w = std::max(w, v.w);
            h = std::max(h, v.h);
            views.push_back(v);
            gts.push_back(std::move(gt));
        }
        gs_colmap_free(cm);
    } else {
        g.resize(n);
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
        View v{};
        std::memset(&v.u, 0, sizeof(v.u));
        for (int k = 0; k < 4; k++) v.u.view[5 * k] = 1.0f;
        v.u.proj[0] = 2.0f * (float)f / (float)w;
        v.u.proj[5] = 2.0f * (float)f / (float)h;
        v.u.proj[8] = 2.0f * (float)cx / (float)w - 1.0f;
        v.u.proj[9] = 2.0f * (float)cy / (float)h - 1.0f;
        v.u.proj[10] = 1000.0f / (1000.0f - 0.1f);
        v.u.proj[11] = 1.0f;
        v.u.proj[14] = -(1000.0f * 0.1f) / (1000.0f - 0.1f);
        std::memcpy(v.u.view_proj, v.u.proj, sizeof(v.u.proj));  // identity view
        v.u.screen_size[0] = (float)w;
        v.u.screen_size[1] = (float)h;
        v.u.focal[0] = v.u.focal[1] = (float)f;
        v.w = w;
        v.h = h;
        v.image_id = 0;
        v.focal = (float)f;
        std::vector<uint32_t> gt;
        synthetic_gt(gt, seed, 0, w, h);
        views.push_back(v);
        gts.push_back(std::move(gt));
    }

    // gradients sized for growth: densification can at most double the population per apply
    const size_t cap = std::max<size_t>((size_t)n * 4, 1024);
    GsGaussian* dg = nullptr;
    GsGradients* dgrad = nullptr;
    uint32_t* drgba = nullptr;
    float* dloss = nullptr;
    if (hipMalloc(&dg, sizeof(GsGaussian) * std::max<uint32_t>(n, 1)) != hipSuccess ||
        hipMalloc(&dgrad, sizeof(GsGradients) * cap) != hipSuccess ||
        hipMalloc(&drgba, sizeof(uint32_t) * w * h) != hipSuccess ||
        hipMalloc(&dloss, sizeof(float)) != hipSuccess) {
        std::fprintf(stderr, "allocation failed\n");
        return 1;
    }
    for (size_t i = 0; i < views.size(); i++) {
        if (hipMalloc(&views[i].dgt, sizeof(uint32_t) * gts[i].size()) != hipSuccess) {
            std::fprintf(stderr, "allocation failed\n");
            return 1;
        }
        hipMemcpy(views[i].dgt, gts[i].data(), sizeof(uint32_t) * gts[i].size(), hipMemcpyHostToDevice);
    }
    if (n) hipMemcpy(dg, g.data(), sizeof(GsGaussian) * n, hipMemcpyHostToDevice);
    hipMemset(dloss, 0, sizeof(float));
    hipStream_t st;
    hipStreamCreate(&st);

    gsplat::TiledRasterizer rast(0, (uint32_t)cap, w, h);
    // the population cap of densification is the buffers' capacity (the reference's MAX_GAUSSIANS
    // plays that role: density_control.mm:27, 360-382)
    gsplat::DensityController dens(0, (uint32_t)cap, cap);
    gsplat::AdamOptimizer adam(0, cap);
    gsplat::Loss loss(0);
    if (!rast.valid()) return 1;
    gsplat::DensityController::setSceneExtent(extent);
    dens.resetAccumulator(n, st);
    const uint32_t tiles = ((w + 15) / 16) * ((h + 15) / 16);
    rast.reservePairs((uint64_t)std::max<uint32_t>(n, 1) * (tiles < 256 ? tiles : 256));
    size_t count = n;
    bool lib_owned = false;  // after the first apply the buffer belongs to the library (gs_free)
    uint64_t iter = start_iter;
    uint64_t applies = 0, pruned = 0, cloned = 0, split = 0, resets = 0;
    const float avg_depth = colmap_dir.empty() ? 6.0f : 2.0f * extent;  // mtl_engine.mm:1127
    auto step = [&]() {
        // the images in order, one per iteration (mtl_engine.mm:1085-1093)
        const View& v = views[(size_t)((iter - start_iter) % views.size())];
        ++iter;
        bool ok = rast.forward(st, dg, count, v.u, drgba, v.w, v.h);
        if (ok && train) ok = loss.compute(st, drgba, v.dgt, v.w, v.h, 0.2f, dloss);
        ok = ok && rast.backward(st, dg, dgrad, count, v.u, drgba, v.dgt) &&
             dens.accumulateGradients(st, dgrad, count);
        if (ok && train) ok = adam.step(st, dg, dgrad, count);
        // shouldDensify (mtl_engine.mm:1112-1114)
        const bool densify = densify_every && iter > kDensifyFrom && iter < kDensifyUntil && iter % densify_every == 0;
        if (ok && train && densify) {
            const size_t n_in = count;
            GsGaussian* before = dg;
            const GsDensityStats s = dens.apply(st, dg, count, iter, v.focal, (float)v.w, avg_depth, iter,
                                                /*ownsBuffer*/ false);
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
    GsFrameStats fs{};
    if (steps + warmup) rast.frameStats(&fs);
    float hloss = 0.0f;
    hipMemcpy(&hloss, dloss, sizeof(float), hipMemcpyDeviceToHost);
    const double per = steps ? ms / steps : 0.0;
    // exportTrainingViews (mtl_engine.mm:1224-1306): every training image rendered at its camera's
    // size, saved as image_%04u_render.ppm (the COLMAP image id)
    uint64_t exported = 0;
    if (!export_dir.empty()) {
        std::vector<uint32_t> host((size_t)w * h);
        for (const View& v : views) {
            if (!rast.forward(st, dg, count, v.u, drgba, v.w, v.h)) return 1;
            hipStreamSynchronize(st);
            hipMemcpy(host.data(), drgba, sizeof(uint32_t) * v.w * v.h, hipMemcpyDeviceToHost);
            char name[64];
            std::snprintf(name, sizeof(name), "image_%04u_render.ppm", v.image_id);
            const std::string path = export_dir + "/" + name;
            if (gs_ppm_save(path.c_str(), host.data(), v.w, v.h) != GS_OK) return fail_msg("gs_ppm_save"), 1;
            exported++;
        }
    }
    std::vector<GsGaussian> final_g;
    if (!ply_out.empty() || !dump_out.empty()) {
        hipStreamSynchronize(st);
        final_g.resize(count);
        if (count) hipMemcpy(final_g.data(), dg, sizeof(GsGaussian) * count, hipMemcpyDeviceToHost);
    }
    uint64_t ply_written = 0;
    if (!ply_out.empty() && gs_ply_save(ply_out.c_str(), final_g.data(), count, &ply_written) != GS_OK)
        return fail_msg("gs_ply_save"), 1;
    if (!dump_out.empty()) {  // the raw 112-B records (tests compare renders against them)
        FILE* fp = std::fopen(dump_out.c_str(), "wb");
        if (!fp || std::fwrite(final_g.data(), sizeof(GsGaussian), count, fp) != count) {
            std::fprintf(stderr, "failed to write %s\n", dump_out.c_str());
            if (fp) std::fclose(fp);
            return 1;
        }
        std::fclose(fp);
    }
    std::printf("{\"n\": %zu, \"n_initial\": %u, \"width\": %u, \"height\": %u, \"views\": %zu, \"pairs\": %llu, "
                "\"train\": %u, \"loss\": %.6f, \"ms_per_step\": %.4f, \"gaussians_x_views_per_s\": %.4e, "
                "\"last_iter\": %llu, \"applies\": %llu, \"pruned\": %llu, \"cloned\": %llu, \"split\": %llu, "
                "\"opacity_resets\": %llu, \"moments\": \"%s\", \"scene\": \"%s\", \"extent\": %.6f, "
                "\"exported_views\": %llu, \"ply_written\": %llu}\n",
                count, n, views[0].w, views[0].h, views.size(), (unsigned long long)fs.num_pairs, train, hloss, per,
                per > 0 ? count / (per * 1e-3) : 0.0, (unsigned long long)iter, (unsigned long long)applies,
                (unsigned long long)pruned, (unsigned long long)cloned, (unsigned long long)split,
                (unsigned long long)resets, ref_moments ? "reference" : "follow", colmap_dir.empty() ? "synthetic" : "colmap",
                extent, (unsigned long long)exported, (unsigned long long)ply_written);
    if (lib_owned) gs_free(dg); else hipFree(dg);
    dg = nullptr;
    for (View& v : views) hipFree(v.dgt);
    hipFree(dgrad); hipFree(drgba); hipFree(dloss);
    hipStreamDestroy(st);
    return 0;
}
