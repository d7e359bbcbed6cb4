// san_main.cpp — host-only driver for the AddressSanitizer + UndefinedBehaviorSanitizer build
// (`make sanitize` -> build/san/gs_san; tests/test_sanitize.py). It runs the code that parses
// untrusted files — the COLMAP binary model and 3DGS PLY readers of gs_io.cpp (the reference's
// colmap_loader.cpp:26-189 and ply_loader.cpp:61-290) — and the CPU oracle (oracle/gs_oracle.c)
// under the sanitizers:
//
//   gs_san colmap DIR          status of gs_colmap_load (+ counts, extent, initial Gaussians)
//   gs_san ply FILE            status of gs_ply_load (+ count)
//   gs_san ppm FILE            status of gs_ppm_load (+ size)
//   gs_san oracle N W H SEED   one oracle forward + backward on a seeded synthetic scene
//
// Prints one line "status=<code> ..." per command; the exit code is 0 unless the driver itself
// failed (a sanitizer report exits with the sanitizer's own code).
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "gs_rasterizer.h"
#include "gs_oracle.h"

namespace {

int run_colmap(const char* dir) {
    gs_colmap* c = nullptr;
    const int rc = gs_colmap_load(dir, &c);
    if (rc != GS_OK) {
        std::printf("status=%d error=%s\n", rc, gs_last_error());
        return 0;
    }
    uint32_t nc = 0, ni = 0;
    uint64_t np = 0;
    gs_colmap_counts(c, &nc, &ni, &np);
    float extent = 0.0f;
    gs_colmap_scene_extent(c, &extent);
    uint64_t n = 0;
    gs_gaussians_from_colmap(c, extent, nullptr, 0, &n);
    std::vector<GsGaussian> g(n > 0 ? n : 1);
    const int rg = gs_gaussians_from_colmap(c, extent, g.data(), n, &n);
    GsTiledUniforms u;
    int ru = GS_OK;
    if (ni > 0) {
        GsColmapImage img;
        GsColmapCamera cam;
        gs_colmap_image(c, 0, &img);
        if (gs_colmap_camera_by_id(c, img.camera_id, &cam) == GS_OK) ru = gs_colmap_uniforms(&cam, &img, 320, 240, &u);
    }
    gs_colmap_free(c);
    std::printf("status=0 cameras=%u images=%u points=%llu gaussians_rc=%d uniforms_rc=%d\n", nc, ni,
                (unsigned long long)np, rg, ru);
    return 0;
}

int run_ply(const char* path) {
    uint64_t n = 0;
    int rc = gs_ply_load(path, nullptr, 0, &n);
    if (rc != GS_OK) {
        std::printf("status=%d error=%s\n", rc, gs_last_error());
        return 0;
    }
    std::vector<GsGaussian> g(n > 0 ? n : 1);
    rc = gs_ply_load(path, g.data(), n, &n);
    std::printf("status=%d count=%llu\n", rc, (unsigned long long)n);
    return 0;
}

int run_ppm(const char* path) {
    uint32_t w = 0, h = 0;
    int rc = gs_ppm_load(path, nullptr, 0, &w, &h);
    if (rc != GS_OK) {
        std::printf("status=%d error=%s\n", rc, gs_last_error());
        return 0;
    }
    std::vector<uint32_t> img((size_t)w * h);
    rc = gs_ppm_load(path, img.data(), img.size(), &w, &h);
    std::printf("status=%d size=%ux%u\n", rc, w, h);
    return 0;
}

uint64_t splitmix(uint64_t seed, uint64_t k) {
    uint64_t z = seed + (k + 1) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

double u01(uint64_t seed, uint64_t k) { return (double)(splitmix(seed, k) >> 40) * 0x1p-24; }

// SURVEY.md §8d's seeded scene (gaussiansplatting_amd/scene.py synthetic_gaussians)
int run_oracle(uint32_t n, uint32_t w, uint32_t h, uint64_t seed) {
    const double kShC0 = 0.28209479177387814, kPi = 3.14159265358979323846;
    std::vector<GsGaussian> g(n > 0 ? n : 1);
    const double f = w, cx = w / 2.0, cy = h / 2.0;
    for (uint32_t i = 0; i < n; i++) {
        double u[13];
        for (int k = 0; k < 13; k++) u[k] = u01(seed, 13ull * i + (uint64_t)k);
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
    GsTiledUniforms un;
    std::memset(&un, 0, sizeof(un));
    for (int k = 0; k < 4; k++) un.view[5 * k] = 1.0f;
    un.proj[0] = 2.0f * (float)f / (float)w;
    un.proj[5] = 2.0f * (float)f / (float)h;
    un.proj[8] = 2.0f * (float)cx / (float)w - 1.0f;
    un.proj[9] = 2.0f * (float)cy / (float)h - 1.0f;
    un.proj[10] = 1000.0f / (1000.0f - 0.1f);
    un.proj[11] = 1.0f;
    un.proj[14] = -(1000.0f * 0.1f) / (1000.0f - 0.1f);
    std::memcpy(un.view_proj, un.proj, sizeof(un.proj));
    un.screen_size[0] = (float)w;
    un.screen_size[1] = (float)h;
    un.focal[0] = un.focal[1] = (float)f;
    const uint32_t tx = (w + 15) / 16, ty = (h + 15) / 16;
    const uint64_t cap = (uint64_t)(n > 0 ? n : 1) * (tx * ty < 256 ? tx * ty : 256);
    std::vector<GsProjected> proj(n > 0 ? n : 1);
    std::vector<uint64_t> keys(cap);
    std::vector<uint32_t> vals(cap), last((size_t)w * h), rgba((size_t)w * h), gt((size_t)w * h);
    std::vector<GsTileRange> ranges((size_t)tx * ty);
    std::vector<float> rgb((size_t)w * h * 3);
    const uint64_t P = gso_forward(g.data(), n, &un, w, h, cap, proj.data(), keys.data(), vals.data(),
                                   ranges.data(), last.data(), rgba.data(), rgb.data(), 2);
    for (size_t i = 0; i < gt.size(); i++) gt[i] = (uint32_t)(splitmix(seed + 1000, i) >> 32) | 0xff000000u;
    un.num_tiles_x = tx;
    un.num_tiles_y = ty;
    un.num_gaussians = n;
    std::vector<double> grad((size_t)(n > 0 ? n : 1) * 28), ab(grad.size()), nz(grad.size());
    gso_backward(g.data(), proj.data(), n, vals.data(), ranges.data(), &un, w, h, last.data(), rgba.data(),
                 gt.data(), grad.data(), ab.data(), nz.data(), 2);
    double s = 0.0;
    for (double v : grad) s += std::fabs(v);
    std::printf("status=0 pairs=%llu grad_abs_sum=%.6e\n", (unsigned long long)P, s);
    return 0;
}

}  // namespace

int main(int argc, char** argv) {
    if (argc >= 3 && !std::strcmp(argv[1], "colmap")) return run_colmap(argv[2]);
    if (argc >= 3 && !std::strcmp(argv[1], "ply")) return run_ply(argv[2]);
    if (argc >= 3 && !std::strcmp(argv[1], "ppm")) return run_ppm(argv[2]);
    if (argc >= 6 && !std::strcmp(argv[1], "oracle"))
        return run_oracle((uint32_t)std::atol(argv[2]), (uint32_t)std::atol(argv[3]), (uint32_t)std::atol(argv[4]),
                          (uint64_t)std::atoll(argv[5]));
    std::fprintf(stderr, "usage: gs_san colmap DIR | ply FILE | oracle N W H SEED\n");
    return 2;
}
