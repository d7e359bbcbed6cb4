// gs_capi.cpp — the extern "C" boundary (include/gs_rasterizer.h) over the HIP kernels.
//
// Host orchestration of one frame (replaces TiledRasterizer::forward/backward,
// tiled_rasterizer.mm:275-722). Everything is stream-ordered on the caller's stream; the only
// host syncs are (a) one 4-byte readback of P while the pair capacity is below the worst case
// (see gs_reserve_pairs) and (b) gs_frame_stats / debug getters / density apply.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstddef>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/gs_rasterizer.h"
#include "gs_internal.hpp"

namespace gs {
hipError_t launch_adam(hipStream_t st, GsGaussian* g, const GsGradients* grad, const float* rows,
                       uint32_t first, uint32_t count, float4* m, float4* v, const float lrs[5], float beta1,
                       float beta2, float eps, float clip, float bc1, float bc2, const uint32_t* cold_word,
                       uint8_t* live);
hipError_t launch_adam_layout(hipStream_t st, const float* in_m, const float* in_v, float* out_m, float* out_v,
                              uint32_t n, bool to_hbm, uint32_t* cold, uint8_t* live);
hipError_t launch_adam_follow(hipStream_t st, const uint32_t* marker, const uint32_t* offset,
                              uint32_t n, const float4* m_in, const float4* v_in, float4* m_out,
                              float4* v_out, uint8_t* live_out);
hipError_t launch_adam_zero(hipStream_t st, float* m, float* v, uint32_t start, uint32_t end,
                            uint32_t mask, uint8_t* live);
hipError_t launch_opacity_reset(hipStream_t st, GsGaussian* g, uint32_t n, float max_raw);
uint32_t loss_blocks(uint32_t w, uint32_t h);
hipError_t launch_loss(hipStream_t st, const uint32_t* rendered, const uint32_t* gt, uint32_t w,
                       uint32_t h, float lambda, float* maps, double* partial, float* loss);
hipError_t launch_density_accumulate(hipStream_t st, const GsGradients* grad, uint32_t n,
                                     float* accum, uint32_t* count, float* pos_accum);
hipError_t launch_density_accumulate_rows(hipStream_t st, const float* rows, const float* vs, uint32_t n,
                                          float* accum, uint32_t* count, float* pos_accum);
hipError_t launch_density_mark(hipStream_t st, const GsGaussian* g, uint32_t n,
                               const float* accum, const uint32_t* count, uint32_t can_densify,
                               uint32_t screen_prune, float split_thr, float prune_thr,
                               float focal, float image_width, float avg_depth, uint32_t* marker,
                               uint32_t* counters);
hipError_t launch_density_demote(hipStream_t st, uint32_t* marker, uint32_t n, uint32_t want,
                                 uint64_t excess, uint32_t* flag, uint32_t* rank,
                                 uint32_t* block_sums, uint32_t* total);
hipError_t launch_density_slots(hipStream_t st, const uint32_t* marker, uint32_t n,
                                uint32_t* slots);
hipError_t launch_density_emit(hipStream_t st, const GsGaussian* in, uint32_t n,
                               const uint32_t* marker, const uint32_t* offset, uint64_t seed,
                               GsGaussian* out);
}  // namespace gs

using namespace gs;

// Layout contract: the reference's record layouts.
static_assert(sizeof(GsGaussian) == 112, "Gaussian is 112 B (ply_loader.hpp:14-20)");
static_assert(offsetof(GsGaussian, scale) == 16 && offsetof(GsGaussian, rotation) == 32 &&
                  offsetof(GsGaussian, opacity) == 48 && offsetof(GsGaussian, sh) == 52,
              "Gaussian offsets (tiled_shaders.metal:11-22)");
static_assert(sizeof(GsProjected) == 88, "ProjectedGaussian is 88 B (tiled_rasterizer.mm:121)");
static_assert(offsetof(GsProjected, conic) == 8 && offsetof(GsProjected, depth) == 20 &&
                  offsetof(GsProjected, opacity) == 24 && offsetof(GsProjected, color) == 28 &&
                  offsetof(GsProjected, radius) == 40 && offsetof(GsProjected, tile_min_x) == 44 &&
                  offsetof(GsProjected, tile_min_y) == 48 && offsetof(GsProjected, tile_max_x) == 52 &&
                  offsetof(GsProjected, tile_max_y) == 56 && offsetof(GsProjected, view_pos_xy) == 64 &&
                  offsetof(GsProjected, cov2d) == 72,
              "ProjectedGaussian offsets (tiled_rasterizer.mm:122-133)");
static_assert(sizeof(GsTiledUniforms) == 240, "TiledUniforms is 240 B");
static_assert(offsetof(GsTiledUniforms, proj) == 64 && offsetof(GsTiledUniforms, view_proj) == 128 &&
                  offsetof(GsTiledUniforms, screen_size) == 192 && offsetof(GsTiledUniforms, focal) == 200 &&
                  offsetof(GsTiledUniforms, camera_pos) == 208 && offsetof(GsTiledUniforms, num_tiles_x) == 224 &&
                  offsetof(GsTiledUniforms, num_gaussians) == 232,
              "TiledUniforms offsets (tiled_rasterizer.hpp:42-53)");
static_assert(sizeof(GsGradients) == 112, "GaussianGradients is 112 B (gradients.hpp:11-31)");
static_assert(offsetof(GsGradients, opacity) == 12 && offsetof(GsGradients, scale) == 16 &&
                  offsetof(GsGradients, rotation) == 32 && offsetof(GsGradients, sh) == 48 &&
                  offsetof(GsGradients, viewspace) == 96,
              "GaussianGradients offsets (tiled_shaders.metal:65-80)");
static_assert(sizeof(GsTileRange) == 8, "TileRange is 8 B");

namespace {

thread_local std::string g_last_error;

int fail(int code, const std::string& msg) {
    g_last_error = msg;
    return code;
}

}  // namespace

namespace gs {
int io_fail(int code, const std::string& msg) { return fail(code, msg); }
}  // namespace gs

namespace {

#define GS_HIP(call)                                                                       \
    do {                                                                                   \
        hipError_t e_ = (call);                                                            \
        if (e_ != hipSuccess)                                                              \
            return fail(GS_E_HIP, std::string(#call " failed: ") + hipGetErrorString(e_)); \
    } while (0)

template <typename T>
hipError_t dalloc(T** p, uint64_t count) {
    *p = nullptr;
    if (count == 0) count = 1;
    return hipMalloc(reinterpret_cast<void**>(p), count * sizeof(T));
}

template <typename T>
void dfree(T*& p) {
    if (p) (void)hipFree(p);
    p = nullptr;
}


uint32_t tile_bits(uint32_t num_tiles) {
    uint32_t b = 1;
    while ((1ull << b) < num_tiles) b++;
    return b;
}

}  // namespace

struct gs_handle {
    int device = 0;
    GaussianBuffers gb;
    PairBuffers pb;
    PixelBuffers px;
    uint2* ranges = nullptr;
    uint32_t* tile_order = nullptr;
    uint32_t* xgroup = nullptr;  // per tile: XCD group of the forward launch slot
    uint32_t* chunk_base = nullptr;  // per tile: first index of its 64-entry list chunks
    uint32_t* tile_cost = nullptr;   // per tile: the forward's blend work
    uint32_t* bwd_order = nullptr;   // per tile: the backward's launch order
    uint32_t* reorder_words = nullptr;  // tile_reorder's status words (zeroed by the tile sort)
    uint32_t* walk = nullptr;        // [5 T] the blends' walked list entries (LaunchGeom::walk)
    bool bwd_order_ready = false;    // bwd_order holds this frame's order
    uint64_t* band_mask = nullptr;   // [chunk][4] forward cull ballots for the backward
    uint64_t band_mask_cap = 0;      // chunks
    uint32_t ranges_cap = 0;
    uint32_t* hist = nullptr;    // [256][kMaxSortBlocks]
    uint32_t* totals = nullptr;  // [256]
    uint32_t* thist = nullptr;   // one-pass tile sort scratch: hist [B][T] + chunk bases [C][T]
    uint64_t thist_cap = 0;
    uint32_t* scalars = nullptr; // [0] P, [1] overflow, [2] scratch total, [4] fan-in error word
    uint32_t* pinned = nullptr;  // host-pinned readback of scalars
    uint32_t* pinned_dev = nullptr;  // its device-side address (the emission kernel writes P there)
    hipStream_t last_stream = nullptr;
    // state carried from forward to backward (tiled_rasterizer.mm:675-722)
    bool have_forward = false;
    bool have_partials = false;  // a backward blend ran after the last forward
    bool sweep_dirty = false;    // the sweep head may be non-zero (see gs_forward)
    const GsGaussian* last_g = nullptr;
    uint32_t last_n = 0;
    GsTiledUniforms last_u{};
    LaunchGeom geo;
    uint32_t depth_passes = 0, tile_passes = 0, tile_path = 0;
    int tile_sort_path = 0;  // gs_set_tile_sort_path
    int backward_split = -1; // gs_set_backward_split (< 0 automatic: every tile)
    int chain_compact = -1;  // gs_set_chain_compact (< 0 automatic: deep lists, see chain_impl)
    int depth_sort = 0;      // gs_set_depth_sort (0 automatic, 1 global, 2 per tile)
    unsigned long long* split_state = nullptr;  // [split tile][kSplitStateWords] backward list-split handover
    uint32_t split_cap = 0;  // tiles split_state holds (allocated by the first backward)
    uint32_t last_overflowed = 0;
    // optional per-stage HIP-event timing (gs_set_stage_timing / gs_stage_times)
    bool timing = false;
    struct Mark {
        int stage;
        hipEvent_t ev;
    };
    std::vector<Mark> marks;
    std::vector<hipEvent_t> event_pool;
};

namespace {
enum {
    kStageProject = 0,
    kStageDepthSort,
    kStageScan,
    kStageEmit,
    kStageTileSort,
    kStageRanges,
    kStageForwardBlend,
    kStageBackwardBlend,
    kStageChain,
    kNumStages
};

// Records an event on `st` that opens `stage` (-1 closes the previous stage).
void tmark(gs_handle* h, hipStream_t st, int stage) {
    if (!h->timing) return;
    hipEvent_t ev;
    if (!h->event_pool.empty()) {
        ev = h->event_pool.back();
        h->event_pool.pop_back();
    } else if (hipEventCreate(&ev) != hipSuccess) {
        return;
    }
    if (hipEventRecord(ev, st) != hipSuccess) {
        h->event_pool.push_back(ev);
        return;
    }
    h->marks.push_back({stage, ev});
}
}  // namespace

struct gs_density {
    int device = 0;
    float scene_extent = 1.0f;  // density_control.mm:41
    float* accum = nullptr;
    uint32_t* count = nullptr;
    float* pos_accum = nullptr;
    uint32_t* marker = nullptr;
    uint32_t* flag = nullptr;
    uint32_t* rank = nullptr;
    uint32_t* slots = nullptr;
    uint32_t* offset = nullptr;
    uint32_t* block_sums = nullptr;
    uint32_t* scalars = nullptr;  // [0..2] counters, [3] total
    uint32_t* pinned = nullptr;
    size_t cap = 0;
    uint64_t max_gaussians = 0;  // 0 = unlimited (the reference caps at 1.5M, :27)
    // the last apply's (marker, offset) describe n_in -> n_out; 0 = identity (no apply ran)
    uint64_t last_in = 0, last_out = 0;
    bool last_mapped = false;
};

struct gs_loss {
    int device = 0;
    double* partial = nullptr;  // per-tile fp64 partial sums
    uint32_t cap = 0;
};

struct gs_adam {
    int device = 0;
    float4* m = nullptr;  // [cap][6] first moments
    float4* v = nullptr;  // [cap][6] second moments
    size_t cap = 0;
    uint32_t t = 0;
    float beta1 = 0.9f, beta2 = 0.999f, eps = 1e-8f, clip = 0.5f;  // optimizer.mm:274-276, shaders.metal:582
    // device word: some cold moment lane (gs_adam.hpp: the SH coefficients without rasterizer
    // gradients) may be non-zero -- set by a records step or a written state with one, cleared by a
    // reset, read by the update kernels themselves (never baked into a captured launch)
    uint32_t* flag = nullptr;
    uint8_t* live = nullptr;   // [cap] 0: the Gaussian's moment records are all zero (gs_adam.hpp)
};

namespace {

void free_gaussian_buffers(GaussianBuffers& b) {
    dfree(b.rec); dfree(b.count); dfree(b.dkey); dfree(b.rect);
    dfree(b.dsort_k[0]); dfree(b.dsort_k[1]); dfree(b.dsort_v[0]); dfree(b.dsort_v[1]);
    dfree(b.offset); dfree(b.goff); dfree(b.scan_sums); dfree(b.sweep); dfree(b.reached);
    dfree(b.chain_list); dfree(b.chain_lcount);
    b.cap = 0;
}

void free_pair_buffers(PairBuffers& b) {
    dfree(b.tile0); dfree(b.val0); dfree(b.tile1); dfree(b.val1);
    dfree(b.s_tile); dfree(b.s_val); dfree(b.partial); dfree(b.ptag_zero); dfree(b.wstart);
    b.cap = 0;
}

int ensure_gaussians(gs_handle* h, size_t n) {
    if (h->gb.cap >= n && h->gb.cap > 0) return GS_OK;
    GS_HIP(hipDeviceSynchronize());
    free_gaussian_buffers(h->gb);
    size_t cap = std::max<size_t>(n, 1024);
    GaussianBuffers& b = h->gb;
    GS_HIP(dalloc(&b.rec, cap * kRecQuads));
    // (count, the sorted payload, offset and goff padded by 16 words: offsets_scan_kernel's last
    // thread with ranks below n loads and stores 8 or 12 words from its first rank, 16-B vectors)
    const size_t cap16 = (cap + 15) / 16 * 16 + 16;
    GS_HIP(dalloc(&b.count, cap16)); GS_HIP(dalloc(&b.dkey, cap)); GS_HIP(dalloc(&b.rect, cap));
    GS_HIP(dalloc(&b.dsort_k[0], cap)); GS_HIP(dalloc(&b.dsort_k[1], cap));
    GS_HIP(dalloc(&b.dsort_v[0], cap16)); GS_HIP(dalloc(&b.dsort_v[1], cap16));
    GS_HIP(dalloc(&b.offset, cap16)); GS_HIP(dalloc(&b.goff, cap16));
    GS_HIP(dalloc(&b.scan_sums, scan_blocks_for((uint32_t)cap) + 1));
    GS_HIP(dalloc(&b.sweep, depth_sweep_words((uint32_t)cap)));
    GS_HIP(hipMemset(b.sweep, 0, depth_sweep_words((uint32_t)cap) * sizeof(uint32_t)));
    GS_HIP(dalloc(&b.reached, cap));
    GS_HIP(hipMemset(b.reached, 0, cap * sizeof(reach_t)));
    GS_HIP(dalloc(&b.chain_list, (cap + 255) / 256 * 256));
    GS_HIP(dalloc(&b.chain_lcount, (cap + 255) / 256));
    b.cap = cap;
    return GS_OK;
}

int ensure_pairs(gs_handle* h, uint64_t need) {
    if (h->pb.cap >= need && h->pb.cap > 0) return GS_OK;
    if (need > 0xffffffffull) return fail(GS_E_CAPACITY, "pair capacity above 2^32 requested");
    GS_HIP(hipDeviceSynchronize());
    uint64_t cap = std::max<uint64_t>(need, h->pb.cap + h->pb.cap / 2);
    cap = std::max<uint64_t>(cap, 1 << 16);
    cap = std::min<uint64_t>(cap, 0xffffffffull);
    free_pair_buffers(h->pb);
    PairBuffers& b = h->pb;
    hipError_t e = hipSuccess;
    if ((e = dalloc(&b.tile0, cap)) != hipSuccess || (e = dalloc(&b.val0, cap)) != hipSuccess ||
        (e = dalloc(&b.tile1, cap)) != hipSuccess || (e = dalloc(&b.val1, cap)) != hipSuccess ||
        (e = dalloc(&b.s_tile, cap)) != hipSuccess || (e = dalloc(&b.s_val, cap)) != hipSuccess ||
        (e = dalloc(&b.partial, cap * kSlotWords)) != hipSuccess ||
        (e = dalloc(&b.ptag_zero, 16)) != hipSuccess ||
        (e = dalloc(&b.wstart, cap / kEmitWin + 2)) != hipSuccess) {
        free_pair_buffers(h->pb);
        return fail(GS_E_NOMEM, std::string("pair buffer allocation failed: ") + hipGetErrorString(e));
    }
    // frame tags start at 1: a zeroed slot never belongs to the current frame
    GS_HIP(hipMemset(b.partial, 0, cap * kSlotWords * sizeof(float)));
    GS_HIP(hipMemset(b.ptag_zero, 0, 16 * sizeof(float)));
    b.cap = cap;
    return GS_OK;
}

int ensure_pixels(gs_handle* h, uint64_t npix, uint32_t ntiles) {
    if (h->px.cap < npix || h->px.cap == 0) {
        GS_HIP(hipDeviceSynchronize());
        dfree(h->px.last_idx); dfree(h->px.t_final);
        GS_HIP(dalloc(&h->px.last_idx, npix));
        GS_HIP(dalloc(&h->px.t_final, npix));
        h->px.cap = npix;
    }
    if (h->ranges_cap < ntiles || h->ranges == nullptr) {
        GS_HIP(hipDeviceSynchronize());
        dfree(h->ranges);
        dfree(h->tile_order);
        dfree(h->xgroup);
        dfree(h->chunk_base);
        dfree(h->tile_cost);
        dfree(h->bwd_order);
        dfree(h->reorder_words);
        dfree(h->walk);
        dfree(h->split_state);
        GS_HIP(dalloc(&h->ranges, ntiles));
        GS_HIP(dalloc(&h->tile_order, ntiles));
        GS_HIP(dalloc(&h->xgroup, ntiles));
        GS_HIP(dalloc(&h->chunk_base, ntiles));
        GS_HIP(dalloc(&h->tile_cost, ntiles));
        GS_HIP(dalloc(&h->bwd_order, ntiles));
        GS_HIP(dalloc(&h->reorder_words, tile_reorder_words()));
        GS_HIP(dalloc(&h->walk, 5ull * ntiles));
        GS_HIP(hipMemset(h->walk, 0, 5ull * ntiles * sizeof(uint32_t)));
        h->split_cap = 0;  // (the list split's state is allocated by the first backward: ensure_split_state)
        h->ranges_cap = ntiles;
    }
    return GS_OK;
}

// The list split's hand-over words, 4 KB per tile, for every tile of the grid (ensure_pixels'
// per-tile capacity), zeroed (the words carry the frame tag in their high half; tag 0 is never
// current). Allocated by the first backward, so a handle that only renders never holds them (33 MB
// at 1080p, 133 MB at 4K), and never inside a stream capture: a graph that captures a backward needs
// an eager backward on the handle first (every caller here warms up eagerly).
int ensure_split_state(gs_handle* h, hipStream_t st, uint32_t tiles) {
    if (tiles <= h->split_cap && h->split_state) return GS_OK;
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    GS_HIP(hipStreamIsCapturing(st, &cs));
    if (cs != hipStreamCaptureStatusNone)
        return fail(GS_E_STATE, "gs_backward: the list split's state is allocated by the first backward, which "
                                "cannot be inside a stream capture (run one backward eagerly first)");
    const uint32_t cap = std::max(tiles, h->ranges_cap);
    GS_HIP(hipStreamSynchronize(st));
    dfree(h->split_state);
    h->split_cap = 0;
    GS_HIP(dalloc(&h->split_state, (uint64_t)cap * kSplitStateWords));
    GS_HIP(hipMemset(h->split_state, 0, (uint64_t)cap * kSplitStateWords * sizeof(unsigned long long)));
    h->split_cap = cap;
    return GS_OK;
}

}  // namespace

extern "C" {

const char* gs_last_error(void) { return g_last_error.c_str(); }
int gs_abi_version(void) { return GS_ABI_VERSION; }

int gs_create(int device, uint32_t max_gaussians, uint32_t max_w, uint32_t max_h,
              gs_handle** out) {
    if (!out) return fail(GS_E_INVALID, "gs_create: out is null");
    *out = nullptr;
    int ndev = 0;
    GS_HIP(hipGetDeviceCount(&ndev));
    if (device < 0 || device >= ndev) return fail(GS_E_INVALID, "gs_create: bad device index");
    GS_HIP(hipSetDevice(device));
    gs_handle* h = new (std::nothrow) gs_handle();
    if (!h) return fail(GS_E_NOMEM, "gs_create: host allocation failed");
    h->device = device;
    int rc = GS_OK;
    do {
        if (hipMalloc(reinterpret_cast<void**>(&h->hist), sizeof(uint32_t) * 256 * kMaxSortBlocks) != hipSuccess ||
            hipMalloc(reinterpret_cast<void**>(&h->totals), sizeof(uint32_t) * 256) != hipSuccess ||
            hipMalloc(reinterpret_cast<void**>(&h->scalars), sizeof(uint32_t) * 16) != hipSuccess ||
            hipHostMalloc(reinterpret_cast<void**>(&h->pinned), sizeof(uint32_t) * 16, hipHostMallocMapped) != hipSuccess ||
            hipHostGetDevicePointer(reinterpret_cast<void**>(&h->pinned_dev), h->pinned, 0) != hipSuccess) {
            rc = fail(GS_E_NOMEM, "gs_create: scratch allocation failed");
            break;
        }
        std::memset(h->pinned, 0, sizeof(uint32_t) * 16);
        // (the LSD tile sort's histogram is zero between frames: the depth-order emission counts the
        // first pass's digits into it, the last pass's scatter clears it)
        if (hipMemset(h->scalars, 0, sizeof(uint32_t) * 16) != hipSuccess ||
            hipMemset(h->hist, 0, sizeof(uint32_t) * 256 * kMaxSortBlocks) != hipSuccess) {
            rc = fail(GS_E_HIP, "gs_create: memset failed");
            break;
        }
        if (max_gaussians && (rc = ensure_gaussians(h, max_gaussians)) != GS_OK) break;
        if (max_gaussians && (rc = ensure_pairs(h, (uint64_t)max_gaussians * 8)) != GS_OK) break;
        if (max_w && max_h) {
            const uint32_t nt = ((max_w + 15) / 16) * ((max_h + 15) / 16);
            if ((rc = ensure_pixels(h, (uint64_t)max_w * max_h, nt)) != GS_OK) break;
        }
    } while (0);
    if (rc != GS_OK) {
        gs_destroy(h);
        return rc;
    }
    *out = h;
    return GS_OK;
}

int gs_destroy(gs_handle* h) {
    if (!h) return GS_OK;
    (void)hipSetDevice(h->device);
    (void)hipDeviceSynchronize();
    free_gaussian_buffers(h->gb);
    free_pair_buffers(h->pb);
    dfree(h->px.last_idx); dfree(h->px.t_final);
    dfree(h->ranges); dfree(h->tile_order); dfree(h->xgroup); dfree(h->chunk_base); dfree(h->tile_cost); dfree(h->bwd_order); dfree(h->reorder_words); dfree(h->walk); dfree(h->split_state); dfree(h->band_mask); dfree(h->hist); dfree(h->totals); dfree(h->thist); dfree(h->scalars);
    if (h->pinned) (void)hipHostFree(h->pinned);
    for (auto& m : h->marks) (void)hipEventDestroy(m.ev);
    for (auto& e : h->event_pool) (void)hipEventDestroy(e);
    delete h;
    return GS_OK;
}

int gs_set_tile_sort_path(gs_handle* h, int mode) {
    if (!h) return fail(GS_E_INVALID, "gs_set_tile_sort_path: null handle");
    if (mode < 0 || mode > 2) return fail(GS_E_INVALID, "gs_set_tile_sort_path: mode must be 0, 1 or 2");
    h->tile_sort_path = mode;
    return GS_OK;
}

int gs_set_depth_sort(gs_handle* h, int mode) {
    if (!h) return fail(GS_E_INVALID, "gs_set_depth_sort: null handle");
    if (mode < 0 || mode > 2) return fail(GS_E_INVALID, "gs_set_depth_sort: mode must be 0, 1 or 2");
    h->depth_sort = mode;
    return GS_OK;
}

int gs_set_chain_compact(gs_handle* h, int mode) {
    if (!h) return fail(GS_E_INVALID, "gs_set_chain_compact: null handle");
    h->chain_compact = mode;
    return GS_OK;
}

int gs_set_backward_split(gs_handle* h, int tiles) {
    if (!h) return fail(GS_E_INVALID, "gs_set_backward_split: null handle");
    h->backward_split = tiles;
    return GS_OK;
}

int gs_reserve_pairs(gs_handle* h, uint64_t max_pairs) {
    if (!h) return fail(GS_E_INVALID, "gs_reserve_pairs: null handle");
    GS_HIP(hipSetDevice(h->device));
    return ensure_pairs(h, max_pairs);
}

int gs_forward(gs_handle* h, void* stream, const GsGaussian* d_g, size_t n,
               const GsTiledUniforms* uniforms, uint32_t w, uint32_t hgt,
               uint32_t* d_rgba8_out, float* d_rgb_f32_out) {
    if (!h || !uniforms || !d_rgba8_out) return fail(GS_E_INVALID, "gs_forward: null argument");
    if (n > 0 && !d_g) return fail(GS_E_INVALID, "gs_forward: null Gaussians");
    if (w == 0 || hgt == 0 || w > 65535u * 16u || hgt > 65535u * 16u)
        return fail(GS_E_INVALID, "gs_forward: bad image size");
    if (n > (1u << 24)) return fail(GS_E_INVALID, "gs_forward: more than 16M Gaussians per call");
    if ((uint32_t)uniforms->screen_size[0] != w || (uint32_t)uniforms->screen_size[1] != hgt)
        return fail(GS_E_INVALID, "gs_forward: uniforms.screen_size must equal (w, h)");
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    GS_HIP(hipSetDevice(h->device));
    h->have_forward = false;
    h->have_partials = false;

    LaunchGeom geo;
    geo.w = w;
    geo.h = hgt;
    geo.tiles_x = (w + GS_TILE_SIZE - 1) / GS_TILE_SIZE;
    geo.tiles_y = (hgt + GS_TILE_SIZE - 1) / GS_TILE_SIZE;
    geo.num_tiles = geo.tiles_x * geo.tiles_y;
    GsTiledUniforms u = *uniforms;  // tiled_rasterizer.mm:308-312
    u.num_tiles_x = geo.tiles_x;
    u.num_tiles_y = geo.tiles_y;
    u.num_gaussians = (uint32_t)n;
    const uint32_t nn = (uint32_t)n;

    int rc;
    if ((rc = ensure_gaussians(h, n)) != GS_OK) return rc;
    if ((rc = ensure_pixels(h, (uint64_t)w * hgt, geo.num_tiles)) != GS_OK) return rc;
    if (h->pb.cap == 0 && (rc = ensure_pairs(h, std::max<uint64_t>(8ull * n, 1 << 16))) != GS_OK)
        return rc;

    uint32_t* P_dev = h->scalars + 0;
    uint32_t* overflow = h->scalars + 1;
    GaussianBuffers& gb = h->gb;

    // Depth order: the global sort of the N depth keys before emission (pairs emitted in depth
    // order), or the per-tile order: with the one-pass tile sort the tile lists are built straight
    // from the Gaussians (no pairs emitted; on the LSD path pairs emitted in Gaussian order), then
    // every list sorted by (depth, Gaussian) on its own (gs_segsort.hip). The tile-sort path is
    // chosen from the previous frame's P, as below; both orders are exact.
    const uint32_t prev_p = h->pinned[0];
    const bool one_pass_wanted = h->tile_sort_path == 1 ||
                                 (h->tile_sort_path == 0 && prev_p <= kTileSortOnePassMaxPairs);
    const bool one_pass = geo.num_tiles <= kTileSortMaxTiles && one_pass_wanted;
    // auto: the per-tile sort's cost follows P (and long lists), the global sort's N, so the per-tile
    // sort only while the previous frame had at most kSegPairsPerGaussian pairs per Gaussian (bench
    // frame 4.7: 1.03-1.05 vs 1.11 ms; config 2's large splats 75: 0.59 vs 0.51 ms)
    const bool seg_sort = h->depth_sort == 2 ||
                          (h->depth_sort == 0 && one_pass && (uint64_t)prev_p <= kSegPairsPerGaussian * (uint64_t)nn);

    // 1. project + per-Gaussian tile count and depth key
    tmark(h, st, kStageProject);
    // The sweep head (digit histograms, tickets) must be zero here: the kernel with the frame duties
    // (emission, or the per-tile order's histogram) re-zeroes it every frame; a frame that stopped
    // between projection and that kernel leaves it dirty
    if (h->sweep_dirty) GS_HIP(hipMemsetAsync(gb.sweep, 0, kSweepHeadWords * sizeof(uint32_t), st));
    h->sweep_dirty = nn > 0;
    // (the depth sort's digit histograms only when the global sort runs)
    GS_HIP(launch_project(st, d_g, nn, u, gb, nullptr, gb.sweep + kSweepHeadWords,
                          nn ? depth_sweep_zero_words(nn) : 0u, nn && !seg_sort ? gb.sweep : nullptr));

    // 2. depth sort of the Gaussians (31 significant key bits, 4 stable passes)
    uint32_t* dsorted = seg_sort ? nullptr : gb.dsort_v[1];
    h->depth_passes = 0;
    if (nn > 0 && !seg_sort) {
        tmark(h, st, kStageDepthSort);
        GS_HIP(depth_sort_onesweep(st, gb.dkey, gb.count, nn, gb.sweep, gb.dsort_k, gb.dsort_v, dsorted));
        h->depth_passes = kOsPasses;
    }
    // 3. emission offsets (+ P and the emission windows' owners) in one look-back scan
    // (the per-tile sort's walks number the slots themselves when no slot can overflow: the pair
    // buffers hold the worst case N min(256, T); its scatter then writes goff, the records' slot
    // field and P, and no offset scan runs)
    const uint64_t worst = (uint64_t)nn * std::min<uint32_t>(256u, geo.num_tiles);
    const bool own_offsets = seg_sort && one_pass && nn > 0 &&
                             h->pb.cap >= worst && tile_sort_gid_blocks(nn) <= tile_sort_blocks(std::max<uint64_t>(worst, 1));
    // (stage marks only around stages that launch something: an empty stage would time the event
    // records themselves)
    if (!own_offsets) tmark(h, st, kStageScan);
    if (!own_offsets)
        GS_HIP(offsets_scan(st, nn, gb.count, dsorted, gb.sweep, gb.offset, P_dev, h->pb.wstart, h->pb.cap, gb.goff,
                            dsorted ? nullptr : gb.rec));  // (the global order's backward reads goff)
    bool wstart_ready = true;

    // 4. capacity: sync-free when the reserve covers the worst case
    const uint64_t bound = (uint64_t)nn * std::min<uint32_t>(256u, geo.num_tiles);
    uint64_t p_bound = std::min<uint64_t>(bound, h->pb.cap);
    h->last_overflowed = 0;
    if (h->pb.cap < bound) {
        GS_HIP(hipMemcpyAsync(h->pinned, P_dev, sizeof(uint32_t), hipMemcpyDeviceToHost, st));
        GS_HIP(hipStreamSynchronize(st));
        const uint64_t P = h->pinned[0];
        if (P > h->pb.cap) {
            h->last_overflowed = 1;
            if ((rc = ensure_pairs(h, P)) != GS_OK) return rc;
            wstart_ready = false;  // the window owners were marked in (and clamped to) the old buffers
        }
        p_bound = P;
    }
    PairBuffers& pb = h->pb;
    {  // band cull masks: at most P/64 + T chunks
        const uint64_t need = h->pb.cap / 64 + geo.num_tiles + 1;
        if (need > h->band_mask_cap) {
            GS_HIP(hipStreamSynchronize(st));
            dfree(h->band_mask);
            h->band_mask_cap = 0;
            GS_HIP(dalloc(&h->band_mask, need * 4));
            h->band_mask_cap = need;
        }
    }

    // 5. emit (tile key, Gaussian) pairs (in depth order, or in Gaussian order for the per-tile order
    // on the LSD path); tile ids of at most 16 bits as u16 (both tile sorts read them so: the
    // one-pass sort's T <= kTileSortMaxTiles always fits)
    const uint32_t tb = tile_bits(geo.num_tiles);
    const bool key16 = tb <= 16u;
    // (the per-tile depth sort's one-pass tile sort walks the Gaussians itself: no pairs emitted)
    const bool fused = one_pass && seg_sort && nn > 0;
    // The LSD tile sort (below): its passes, blocks and first digit width; the depth-order emission
    // counts the first pass's digits per sort block itself (no histogram pass over the emitted keys)
    // when that pass is not also the last (the last pass's histogram kernel initialises the ranges)
    const uint32_t lsd_passes = (tb + 7) / 8;
    const uint32_t lsd_B = sort_blocks_for(std::max<uint64_t>(p_bound, 1));
    const uint32_t lsd_nbits0 = (tb + lsd_passes - 1) / lsd_passes;
    const bool lsd_hist1 = !one_pass && !fused && dsorted != nullptr && lsd_passes >= 2;
    if (!fused) tmark(h, st, kStageEmit);
    if (!fused)
        GS_HIP(launch_emit(st, nn, gb, dsorted, pb, geo.tiles_x, P_dev, p_bound, overflow, wstart_ready,
                           h->pinned_dev, gb.sweep, key16, lsd_hist1 ? h->hist : nullptr, lsd_B,
                           (1u << lsd_nbits0) - 1u));
    h->sweep_dirty = false;

    // 6. stable sort of the (tile, gid<<8|j) pairs by tile, 7. tile ranges
    tmark(h, st, kStageTileSort);
    // Path choice (both give identical results): the one-pass counting sort wins while a
    // (slice, tile) run is short enough that its scattered stores cost less than a second pass;
    // above ~16M pairs the two coalesced 8-bit passes are faster (config 5: 69M pairs). The host
    // does not know this frame's P without a sync, so the previous frame's count (read back
    // asynchronously at the end of every forward) decides; a stale value only picks the other path.
    if (one_pass) {
        // one counting pass over the ceil(log2 T) tile bits; the ranges fall out of its scan
        const uint64_t pb1 = std::max<uint64_t>(p_bound, 1);
        const uint64_t need = tile_sort_scratch(pb1, geo.num_tiles);
        if (need > h->thist_cap) {
            GS_HIP(hipStreamSynchronize(st));
            dfree(h->thist);
            h->thist_cap = 0;
            GS_HIP(dalloc(&h->thist, need));
            h->thist_cap = need;
        }
        static_assert(kTileSortMaxTiles <= 65536u, "one-pass tile sort reads u16 keys");
        if (fused)
            GS_HIP(tile_sort_gid(st, nn, gb.count, gb.goff, gb.rect, geo.tiles_x, pb.cap, P_dev, pb1, geo.num_tiles,
                                 h->thist, pb.s_val, h->ranges, h->tile_order, h->chunk_base, h->tile_cost,
                                 h->reorder_words, h->scalars + kScalarFanInError, true, h->xgroup, overflow,
                                 h->pinned_dev, gb.sweep, own_offsets,
                                 gb.rec, gb.offset /* (the depth-order offsets: unused on this path) */));
        else
            GS_HIP(tile_sort(st, reinterpret_cast<const uint16_t*>(pb.tile0), pb.val0, P_dev, pb1, geo.num_tiles, tb, h->thist, pb.s_val,
                             h->ranges, h->tile_order, h->chunk_base, h->tile_cost, h->reorder_words,
                             h->scalars + kScalarFanInError, true, h->xgroup));
        geo.xgroup = h->xgroup;
        geo.tile_cost = h->tile_cost;
        h->tile_passes = 1;
        h->tile_path = 1;  // (its ranges come out of the sort: no separate ranges stage)
    } else {
        const uint32_t tpasses = lsd_passes;
        const uint32_t B = lsd_B;
        // tile ids of at most 16 bits travel between the passes as u16, and the last pass writes no
        // keys: it builds the ranges itself (atomics at the key runs' ends; chunk_base fills the
        // empty tiles) -- config 5 moves 552 MB less
        const bool narrow = key16;
        const uint32_t* kin = pb.tile0;
        const uint32_t* vin = pb.val0;
        uint32_t* kbuf[2] = {pb.tile1, pb.tile0};
        uint32_t* vbuf[2] = {pb.val1, pb.val0};
        uint32_t shift = 0;
        for (uint32_t p = 0; p < tpasses; p++) {
            RadixPass rp;
            rp.keys_in = kin;
            rp.key_bytes_in = narrow ? 2u : 4u;
            rp.key_bytes_out = narrow ? 2u : 4u;
            rp.vals_in = vin;
            rp.n_dev = P_dev;
            rp.shift = shift;
            // the tile bits spread evenly over the passes (13 -> 7 + 6, not 8 + 5): fewer digits per
            // pass make the scatter's per-(block step, digit) runs longer (more whole-line stores)
            rp.nbits = (tb - shift + (tpasses - p) - 1) / (tpasses - p);
            shift += rp.nbits;
            rp.nblocks = B;
            rp.hist = h->hist;
            rp.hist_ready = p == 0 && lsd_hist1;  // (counted by the emission)
            rp.clear_hist = p + 1 == tpasses;     // (zero again for the next frame's emission)
            rp.totals = h->totals;
            if (p + 1 == tpasses) {
                rp.keys_out = narrow ? nullptr : pb.s_tile;
                rp.vals_out = pb.s_val;
                if (narrow) {
                    rp.ranges_out = h->ranges;
                    rp.ranges_n = geo.num_tiles;
                }
            } else {
                rp.keys_out = kbuf[p & 1u];
                rp.vals_out = vbuf[p & 1u];
            }
            GS_HIP(radix_pass(st, rp));
            kin = kbuf[p & 1u];
            vin = vbuf[p & 1u];
        }
        h->tile_passes = tpasses;
        h->tile_path = 2;
        tmark(h, st, kStageRanges);
        if (!narrow) GS_HIP(launch_ranges(st, pb.s_tile, P_dev, p_bound, geo.num_tiles, h->ranges));
        // the forward's work counters (the backward's launch order, tile_reorder) work on this path too
        const bool reorder = geo.num_tiles <= kTileSortMaxTiles;
        GS_HIP(launch_chunk_base(st, h->ranges, geo.num_tiles, h->chunk_base, reorder ? h->tile_cost : nullptr,
                                 reorder ? reinterpret_cast<unsigned long long*>(h->reorder_words) : nullptr,
                                 reorder ? tile_reorder_words() / 2u : 0u, narrow,
                                 h->tile_order));  // (+ the blend launch order)
        if (reorder) geo.tile_cost = h->tile_cost;
    }
    geo.tile_order = h->tile_order;
    // 7b. the per-tile depth sort: every list, in whatever order the tile sort left it, to (depth,
    // Gaussian) order: lists of up to kFwdSortMax entries by the forward itself, longer ones before it
    // (their segments ping-pong through the emission / LSD buffers, which the tile sort has finished with)
    if (seg_sort && nn > 0) {
        tmark(h, st, kStageDepthSort);
        GS_HIP(launch_tile_depth_sort(st, h->ranges, geo.num_tiles, gb.dkey, pb.s_val, pb.tile1, pb.val1, pb.tile0,
                                      pb.val0, pb.s_tile));
        geo.fwd_sort_dkey = gb.dkey;
    }
    geo.goff_direct = !seg_sort;  // (the records carry the slot base only on the per-tile order)
    geo.chunk_base = h->chunk_base;
    geo.band_mask = h->band_mask;
    geo.frame_tag = h->scalars + kScalarFrameTag;
    geo.walk = h->walk;

    // 8. blend
    tmark(h, st, kStageForwardBlend);
    GS_HIP(launch_forward(st, geo, u, gb, pb, h->ranges, P_dev, h->px, d_rgba8_out, d_rgb_f32_out));
    tmark(h, st, -1);

    // (P and the overflow flag reach h->pinned from the emission kernel; with no Gaussians there is
    // no emission and P = 0)
    if (nn == 0) {
        GS_HIP(hipMemsetAsync(overflow, 0, kScalarFanInError * sizeof(uint32_t), st));  // [1, 4]
        GS_HIP(hipMemcpyAsync(h->pinned, h->scalars, 2 * sizeof(uint32_t), hipMemcpyDeviceToHost, st));
    }
    h->last_stream = st;
    h->have_forward = true;
    h->last_g = d_g;
    h->last_n = nn;
    h->last_u = u;
    h->geo = geo;
    h->bwd_order_ready = false;
    return GS_OK;
}

// Checks shared by the backward entry points; fills the backward's uniforms.
static int backward_check(gs_handle* h, const char* who, const GsGaussian* d_g, size_t n,
                          const GsTiledUniforms* uniforms, GsTiledUniforms& u) {
    if (!h || !uniforms) return fail(GS_E_INVALID, std::string(who) + ": null argument");
    if (!h->have_forward) return fail(GS_E_STATE, std::string(who) + ": no preceding gs_forward");
    if ((uint32_t)n != h->last_n || d_g != h->last_g)
        return fail(GS_E_STATE, std::string(who) + ": Gaussians differ from the preceding gs_forward");
    u = *uniforms;  // tiled_rasterizer.mm:690-694
    u.num_tiles_x = h->geo.tiles_x;
    u.num_tiles_y = h->geo.tiles_y;
    u.num_gaussians = (uint32_t)n;
    if (std::memcmp(u.view, h->last_u.view, sizeof(u.view)) != 0 ||
        std::memcmp(u.focal, h->last_u.focal, sizeof(u.focal)) != 0)
        return fail(GS_E_STATE, std::string(who) + ": uniforms differ from the preceding gs_forward");
    return GS_OK;
}

static int blend_impl(gs_handle* h, hipStream_t st, const GsTiledUniforms& u,
                      const uint32_t* d_rendered_rgba8, const uint32_t* d_gt_rgba8) {
    if (!d_rendered_rgba8 || !d_gt_rgba8) return fail(GS_E_INVALID, "gs_backward: null image");
    GS_HIP(hipSetDevice(h->device));
    tmark(h, st, kStageBackwardBlend);
    LaunchGeom geo = h->geo;
    if (geo.tile_cost && h->last_n) {  // the backward's launch order from the forward's measured work
        if (!h->bwd_order_ready) GS_HIP(tile_reorder(st, geo.num_tiles, geo.tile_cost,
                                                     reinterpret_cast<unsigned long long*>(h->reorder_words),
                                                     h->bwd_order, h->scalars + kScalarFanInError, geo.xgroup));
        h->bwd_order_ready = true;
        geo.bwd_order = h->bwd_order;
    }
    // the list split needs an order (heaviest first: the forward's measured work, else list length)
    if (geo.bwd_order || geo.tile_order) {
        geo.split_tiles = h->backward_split < 0 ? geo.num_tiles
                                                : std::min<uint32_t>((uint32_t)h->backward_split, geo.num_tiles);
        if (geo.split_tiles) {
            int rc = ensure_split_state(h, st, geo.split_tiles);
            if (rc != GS_OK) return rc;
            geo.split_state = h->split_state;
            geo.split_err = h->scalars + kScalarFanInError;
        }
    }
    GS_HIP(launch_backward(st, geo, u, h->gb, h->pb, h->ranges, h->px, d_rendered_rgba8, d_gt_rgba8));
    h->have_partials = true;
    h->last_stream = st;
    return GS_OK;
}

static int chain_impl(gs_handle* h, hipStream_t st, const GsGaussian* d_g, GsGradients* d_grad,
                      float* d_rows, float* d_vs, const GsTiledUniforms& u, uint32_t first, uint32_t count,
                      const ChainStep* step = nullptr) {
    GS_HIP(hipSetDevice(h->device));
    tmark(h, st, kStageChain);
    // The compacting chain pays off where most Gaussians are not reached: deep lists, whose pixels
    // saturate long before their ends (config 5: P = 13 N). The latest P the host has seen (mirrored
    // by the emission kernel; no sync) decides; both kernels give bit-identical gradients.
    const bool deep = (uint64_t)h->pinned[0] > kChainCompactPairsPerGaussian * (uint64_t)h->last_n;
    const bool compact = h->chain_compact < 0 ? deep : h->chain_compact > 0;
    GS_HIP(launch_chain(st, d_g, h->last_n, u, h->gb, h->pb, d_grad, d_rows, d_vs, first, count,
                        h->scalars + kScalarFrameTag, compact, step, !deep));
    tmark(h, st, -1);
    h->last_stream = st;
    return GS_OK;
}

static int backward_impl(gs_handle* h, void* stream, const GsGaussian* d_g, GsGradients* d_grad,
                         float* d_rows, float* d_vs, size_t n, const GsTiledUniforms* uniforms,
                         const uint32_t* d_rendered_rgba8, const uint32_t* d_gt_rgba8) {
    GsTiledUniforms u;
    int rc;
    if ((rc = backward_check(h, "gs_backward", d_g, n, uniforms, u)) != GS_OK) return rc;
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    if ((rc = blend_impl(h, st, u, d_rendered_rgba8, d_gt_rgba8)) != GS_OK) return rc;
    return chain_impl(h, st, d_g, d_grad, d_rows, d_vs, u, 0u, (uint32_t)n);
}

int gs_backward(gs_handle* h, void* stream, const GsGaussian* d_g, GsGradients* d_grad,
                size_t n, const GsTiledUniforms* uniforms, const uint32_t* d_rendered_rgba8,
                const uint32_t* d_gt_rgba8) {
    if (!d_grad) return fail(GS_E_INVALID, "gs_backward: null argument");
    return backward_impl(h, stream, d_g, d_grad, nullptr, nullptr, n, uniforms, d_rendered_rgba8,
                         d_gt_rgba8);
}

int gs_backward_packed(gs_handle* h, void* stream, const GsGaussian* d_g, float* d_rows14,
                       float* d_viewspace2, size_t n, const GsTiledUniforms* uniforms,
                       const uint32_t* d_rendered_rgba8, const uint32_t* d_gt_rgba8) {
    if (!d_rows14) return fail(GS_E_INVALID, "gs_backward_packed: null argument");
    return backward_impl(h, stream, d_g, nullptr, d_rows14, d_viewspace2, n, uniforms, d_rendered_rgba8,
                         d_gt_rgba8);
}

int gs_backward_blend(gs_handle* h, void* stream, const GsGaussian* d_g, size_t n,
                      const GsTiledUniforms* uniforms, const uint32_t* d_rendered_rgba8,
                      const uint32_t* d_gt_rgba8) {
    GsTiledUniforms u;
    int rc;
    if ((rc = backward_check(h, "gs_backward_blend", d_g, n, uniforms, u)) != GS_OK) return rc;
    return blend_impl(h, reinterpret_cast<hipStream_t>(stream), u, d_rendered_rgba8, d_gt_rgba8);
}

int gs_backward_chain(gs_handle* h, void* stream, const GsGaussian* d_g, GsGradients* d_grad,
                      float* d_rows14, float* d_viewspace2, size_t n, const GsTiledUniforms* uniforms,
                      size_t first, size_t count) {
    GsTiledUniforms u;
    int rc;
    if ((rc = backward_check(h, "gs_backward_chain", d_g, n, uniforms, u)) != GS_OK) return rc;
    if (!h->have_partials) return fail(GS_E_STATE, "gs_backward_chain: no preceding gs_backward_blend");
    if ((d_grad == nullptr) == (d_rows14 == nullptr))
        return fail(GS_E_INVALID, "gs_backward_chain: exactly one of d_grad, d_rows14");
    if (d_grad && d_viewspace2)
        return fail(GS_E_INVALID, "gs_backward_chain: d_viewspace2 goes with d_rows14 (records hold their own)");
    if (first > n || count > n - first) return fail(GS_E_INVALID, "gs_backward_chain: range outside [0, n)");
    return chain_impl(h, reinterpret_cast<hipStream_t>(stream), d_g, d_grad, d_rows14, d_viewspace2, u,
                      (uint32_t)first, (uint32_t)count);
}

static int density_ensure(gs_density* d, size_t n);
int adam_grow(gs_adam* a, hipStream_t st, size_t n);

int gs_backward_step(gs_handle* h, void* stream, GsGaussian* d_g, size_t n, const GsTiledUniforms* uniforms,
                     const uint32_t* d_rendered_rgba8, const uint32_t* d_gt_rgba8, gs_density* d, gs_adam* a,
                     const float lrs[5]) {
    if (!a || !lrs) return fail(GS_E_INVALID, "gs_backward_step: null argument");
    GsTiledUniforms u;
    int rc;
    if ((rc = backward_check(h, "gs_backward_step", d_g, n, uniforms, u)) != GS_OK) return rc;
    if (n > (1u << 30)) return fail(GS_E_INVALID, "gs_backward_step: count too large");
    if (a->device != h->device || (d && d->device != h->device))
        return fail(GS_E_INVALID, "gs_backward_step: optimizer / density state on another device");
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    GS_HIP(hipSetDevice(h->device));
    // the state the unfused sequence would grow (gs_density_accumulate_rows, gs_adam_step_rows)
    if (d && (rc = density_ensure(d, n)) != GS_OK) return rc;
    if ((rc = adam_grow(a, st, n)) != GS_OK) return rc;
    if ((rc = blend_impl(h, st, u, d_rendered_rgba8, d_gt_rgba8)) != GS_OK) return rc;
    a->t++;  // optimizer.mm:250
    const float p1 = (float)std::pow((double)a->beta1, (double)a->t);
    const float p2 = (float)std::pow((double)a->beta2, (double)a->t);
    ChainStep cs;
    cs.g = d_g;
    if (d) {
        cs.accum = d->accum;
        cs.dcount = d->count;
        cs.pos_accum = d->pos_accum;
    }
    cs.m = a->m;
    cs.v = a->v;
    cs.P = make_adam_params(lrs, a->beta1, a->beta2, a->eps, a->clip, 1.0f - p1, 1.0f - p2);
    cs.P.cold = 0u;
    cs.P.cold_word = a->flag;
    cs.P.live = a->live;
    rc = chain_impl(h, st, d_g, nullptr, nullptr, nullptr, u, 0u, (uint32_t)n, &cs);
    if (rc != GS_OK) a->t--;  // nothing was stepped
    return rc;
}

int gs_unpack_gradients(void* stream, const float* d_rows14, const float* d_viewspace2, GsGradients* d_grad,
                        size_t n) {
    if (n && (!d_rows14 || !d_grad)) return fail(GS_E_INVALID, "gs_unpack_gradients: null argument");
    GS_HIP(launch_unpack(reinterpret_cast<hipStream_t>(stream), d_rows14, d_viewspace2, (uint32_t)n, d_grad));
    return GS_OK;
}

int gs_set_stage_timing(gs_handle* h, int enable) {
    if (!h) return fail(GS_E_INVALID, "gs_set_stage_timing: null handle");
    h->timing = enable != 0;
    return GS_OK;
}

int gs_stage_times(gs_handle* h, double* ms_out, uint32_t* calls_out, int max_stages) {
    if (!h || !ms_out) return fail(GS_E_INVALID, "gs_stage_times: null argument");
    GS_HIP(hipSetDevice(h->device));
    for (auto& e : h->marks) GS_HIP(hipEventSynchronize(e.ev));
    double acc[kNumStages] = {0};
    uint32_t calls[kNumStages] = {0};
    for (size_t k = 0; k + 1 < h->marks.size(); k++) {
        const int s = h->marks[k].stage;
        if (s < 0) continue;
        float ms = 0.0f;
        GS_HIP(hipEventElapsedTime(&ms, h->marks[k].ev, h->marks[k + 1].ev));
        acc[s] += ms;
        calls[s]++;
    }
    for (int s = 0; s < max_stages && s < kNumStages; s++) {
        ms_out[s] = acc[s];
        if (calls_out) calls_out[s] = calls[s];
    }
    for (auto& e : h->marks) h->event_pool.push_back(e.ev);
    h->marks.clear();
    return kNumStages;
}

int gs_frame_stats(gs_handle* h, GsFrameStats* out) {
    if (!h || !out) return fail(GS_E_INVALID, "gs_frame_stats: null argument");
    GS_HIP(hipSetDevice(h->device));
    GS_HIP(hipStreamSynchronize(h->last_stream));
    std::memset(out, 0, sizeof(*out));
    if (h->have_forward) {
        uint32_t s[kScalarFrameTag + 1];
        GS_HIP(hipMemcpy(s, h->scalars, sizeof(s), hipMemcpyDeviceToHost));
        out->num_pairs = s[0];
        out->overflowed = h->last_overflowed | s[1];
        out->scan_errors = s[kScalarFanInError];  // the tile sort's and the backward order's fan-ins
        uint32_t vis = 0;
        // visible = Gaussians with a non-zero tile count; reached = those whose list entries the last
        // backward selected (their reached tag is the frame tag's low byte) and their slots
        if (h->last_n) {
            std::vector<uint32_t> cnt(h->last_n);
            std::vector<reach_t> rch(h->have_partials ? h->last_n : 0);
            GS_HIP(hipMemcpy(cnt.data(), h->gb.count, sizeof(uint32_t) * h->last_n, hipMemcpyDeviceToHost));
            if (h->have_partials)
                GS_HIP(hipMemcpy(rch.data(), h->gb.reached, sizeof(reach_t) * h->last_n, hipMemcpyDeviceToHost));
            const reach_t tag = (reach_t)s[kScalarFrameTag];
            for (uint32_t i = 0; i < h->last_n; i++) {
                vis += cnt[i] != 0;
                if (h->have_partials && cnt[i] && rch[i] == tag) {
                    out->reached_gaussians++;
                    out->reached_slots += cnt[i];
                }
            }
        }
        out->num_visible = vis;
        // the blends' walked list entries (when the frame rendered: P > 0)
        const uint32_t T = h->geo.num_tiles;
        if (s[0] && T) {
            std::vector<uint32_t> wk(5ull * T);
            GS_HIP(hipMemcpy(wk.data(), h->walk, wk.size() * sizeof(uint32_t), hipMemcpyDeviceToHost));
            for (uint32_t t = 0; t < T; t++) {
                out->fwd_walked_entries += std::max(std::max(wk[4 * t], wk[4 * t + 1]), std::max(wk[4 * t + 2], wk[4 * t + 3]));
                if (h->have_partials) out->bwd_walked_entries += wk[4ull * T + t];
            }
        }
        if (h->last_n) out->scan_errors |= h->pinned[2];  // the sweep's, mirrored by the emission kernel
        out->num_tiles = h->geo.num_tiles;
        out->width = h->geo.w;
        out->height = h->geo.h;
    }
    out->pair_capacity = h->pb.cap;
    out->sort_passes_depth = h->depth_passes;
    out->sort_passes_tile = h->tile_passes;
    out->tile_sort_path = h->tile_path;
    return GS_OK;
}

int gs_debug_num_pairs(gs_handle* h, uint64_t* out) {
    if (!h || !out) return fail(GS_E_INVALID, "gs_debug_num_pairs: null argument");
    if (!h->have_forward) return fail(GS_E_STATE, "gs_debug_num_pairs: no forward");
    GS_HIP(hipSetDevice(h->device));
    GS_HIP(hipStreamSynchronize(h->last_stream));
    uint32_t p = 0;
    GS_HIP(hipMemcpy(&p, h->scalars, sizeof(p), hipMemcpyDeviceToHost));
    *out = p;
    return GS_OK;
}

int gs_debug_sorted_pairs(gs_handle* h, void* stream, uint64_t* d_keys, uint32_t* d_values,
                          uint64_t cap) {
    if (!h) return fail(GS_E_INVALID, "gs_debug_sorted_pairs: null handle");
    if (!h->have_forward) return fail(GS_E_STATE, "gs_debug_sorted_pairs: no forward");
    GS_HIP(hipSetDevice(h->device));
    GS_HIP(launch_debug_pairs(reinterpret_cast<hipStream_t>(stream), h->pb, h->gb, h->ranges,
                              h->geo.num_tiles, h->scalars, cap,
                              d_keys, d_values));
    return GS_OK;
}

int gs_debug_tile_ranges(gs_handle* h, void* stream, GsTileRange* d_ranges, uint32_t cap) {
    if (!h || !d_ranges) return fail(GS_E_INVALID, "gs_debug_tile_ranges: null argument");
    if (!h->have_forward) return fail(GS_E_STATE, "gs_debug_tile_ranges: no forward");
    if (cap < h->geo.num_tiles) return fail(GS_E_INVALID, "gs_debug_tile_ranges: cap too small");
    GS_HIP(hipSetDevice(h->device));
    GS_HIP(launch_debug_ranges(reinterpret_cast<hipStream_t>(stream), h->ranges, h->geo.num_tiles,
                               d_ranges));
    return GS_OK;
}

int gs_debug_last_idx(gs_handle* h, void* stream, uint32_t* d_last_idx, uint64_t cap) {
    if (!h || !d_last_idx) return fail(GS_E_INVALID, "gs_debug_last_idx: null argument");
    if (!h->have_forward) return fail(GS_E_STATE, "gs_debug_last_idx: no forward");
    const uint64_t npix = (uint64_t)h->geo.w * h->geo.h;
    if (cap < npix) return fail(GS_E_INVALID, "gs_debug_last_idx: cap too small");
    GS_HIP(hipSetDevice(h->device));
    GS_HIP(hipMemcpyAsync(d_last_idx, h->px.last_idx, npix * sizeof(uint32_t),
                          hipMemcpyDeviceToDevice, reinterpret_cast<hipStream_t>(stream)));
    return GS_OK;
}

int gs_debug_projected(gs_handle* h, void* stream, GsProjected* d_proj, size_t cap) {
    if (!h || !d_proj) return fail(GS_E_INVALID, "gs_debug_projected: null argument");
    if (!h->have_forward) return fail(GS_E_STATE, "gs_debug_projected: no forward");
    if (cap < h->last_n) return fail(GS_E_INVALID, "gs_debug_projected: cap too small");
    GS_HIP(hipSetDevice(h->device));
    // projection is a pure function of (Gaussians, uniforms): re-run it with a debug sink
    GS_HIP(launch_project(reinterpret_cast<hipStream_t>(stream), h->last_g, h->last_n, h->last_u,
                          h->gb, d_proj));
    return GS_OK;
}

int gs_debug_half_exp_check(int device, uint32_t* mismatches, uint32_t* max_ulps) {
    if (!mismatches || !max_ulps) return fail(GS_E_INVALID, "gs_debug_half_exp_check: null argument");
    int ndev = 0;
    GS_HIP(hipGetDeviceCount(&ndev));
    if (device < 0 || device >= ndev) return fail(GS_E_INVALID, "gs_debug_half_exp_check: bad device index");
    GS_HIP(hipSetDevice(device));
    uint32_t* d = nullptr;
    GS_HIP(hipMalloc(&d, 2 * sizeof(uint32_t)));
    uint32_t out[2] = {0, 0};
    hipError_t e = launch_half_exp_check(nullptr, d);
    if (e == hipSuccess) e = hipMemcpy(out, d, sizeof(out), hipMemcpyDeviceToHost);
    (void)hipFree(d);
    if (e != hipSuccess) return fail(GS_E_HIP, std::string("gs_debug_half_exp_check: ") + hipGetErrorString(e));
    *mismatches = out[0];
    *max_ulps = out[1];
    return GS_OK;
}

int gs_debug_float_exp_check(int device, float* max_rel) {
    if (!max_rel) return fail(GS_E_INVALID, "gs_debug_float_exp_check: null argument");
    int ndev = 0;
    GS_HIP(hipGetDeviceCount(&ndev));
    if (device < 0 || device >= ndev) return fail(GS_E_INVALID, "gs_debug_float_exp_check: bad device index");
    GS_HIP(hipSetDevice(device));
    uint32_t* d = nullptr;
    GS_HIP(hipMalloc(&d, sizeof(uint32_t)));
    uint32_t out = 0;
    hipError_t e = launch_float_exp_check(nullptr, d);
    if (e == hipSuccess) e = hipMemcpy(&out, d, sizeof(out), hipMemcpyDeviceToHost);
    (void)hipFree(d);
    if (e != hipSuccess) return fail(GS_E_HIP, std::string("gs_debug_float_exp_check: ") + hipGetErrorString(e));
    std::memcpy(max_rel, &out, sizeof(float));
    return GS_OK;
}

// ---- density control -------------------------------------------------------------------

static int density_ensure(gs_density* d, size_t n) {
    if (d->cap >= n && d->cap > 0) return GS_OK;
    GS_HIP(hipDeviceSynchronize());
    size_t cap = std::max<size_t>(n, 1024);
    float* na = nullptr; uint32_t* nc = nullptr; float* np = nullptr;
    GS_HIP(dalloc(&na, cap)); GS_HIP(dalloc(&nc, cap)); GS_HIP(dalloc(&np, cap * 3));
    GS_HIP(hipMemset(na, 0, cap * sizeof(float)));
    GS_HIP(hipMemset(nc, 0, cap * sizeof(uint32_t)));
    GS_HIP(hipMemset(np, 0, cap * 3 * sizeof(float)));
    if (d->cap) {  // keep accumulated statistics across growth
        GS_HIP(hipMemcpy(na, d->accum, d->cap * sizeof(float), hipMemcpyDeviceToDevice));
        GS_HIP(hipMemcpy(nc, d->count, d->cap * sizeof(uint32_t), hipMemcpyDeviceToDevice));
        GS_HIP(hipMemcpy(np, d->pos_accum, d->cap * 3 * sizeof(float), hipMemcpyDeviceToDevice));
    }
    // the last apply's marker / offset survive growth (gs_adam_follow_density reads them after
    // the apply's own accumulator reset has grown the buffers to the new count)
    uint32_t* nm = nullptr; uint32_t* no = nullptr;
    GS_HIP(dalloc(&nm, cap)); GS_HIP(dalloc(&no, cap));
    if (d->cap) {
        GS_HIP(hipMemcpy(nm, d->marker, d->cap * sizeof(uint32_t), hipMemcpyDeviceToDevice));
        GS_HIP(hipMemcpy(no, d->offset, d->cap * sizeof(uint32_t), hipMemcpyDeviceToDevice));
    }
    dfree(d->accum); dfree(d->count); dfree(d->pos_accum);
    dfree(d->marker); dfree(d->flag); dfree(d->rank); dfree(d->slots); dfree(d->offset);
    dfree(d->block_sums);
    d->accum = na; d->count = nc; d->pos_accum = np;
    d->marker = nm; d->offset = no;
    GS_HIP(dalloc(&d->flag, cap)); GS_HIP(dalloc(&d->rank, cap));
    GS_HIP(dalloc(&d->slots, cap));
    GS_HIP(dalloc(&d->block_sums, scan_blocks_for((uint32_t)cap) + 1));
    d->cap = cap;
    return GS_OK;
}

int gs_density_create(int device, uint32_t max_gaussians, gs_density** out) {
    if (!out) return fail(GS_E_INVALID, "gs_density_create: out is null");
    *out = nullptr;
    int ndev = 0;
    GS_HIP(hipGetDeviceCount(&ndev));
    if (device < 0 || device >= ndev) return fail(GS_E_INVALID, "gs_density_create: bad device");
    GS_HIP(hipSetDevice(device));
    gs_density* d = new (std::nothrow) gs_density();
    if (!d) return fail(GS_E_NOMEM, "gs_density_create: host allocation failed");
    d->device = device;
    int rc = GS_OK;
    if (hipMalloc(reinterpret_cast<void**>(&d->scalars), 16 * sizeof(uint32_t)) != hipSuccess ||
        hipHostMalloc(reinterpret_cast<void**>(&d->pinned), 16 * sizeof(uint32_t), 0) != hipSuccess)
        rc = fail(GS_E_NOMEM, "gs_density_create: scratch allocation failed");
    if (rc == GS_OK) rc = density_ensure(d, std::max<uint32_t>(max_gaussians, 1));
    if (rc != GS_OK) {
        gs_density_destroy(d);
        return rc;
    }
    *out = d;
    return GS_OK;
}

int gs_density_destroy(gs_density* d) {
    if (!d) return GS_OK;
    (void)hipSetDevice(d->device);
    (void)hipDeviceSynchronize();
    dfree(d->accum); dfree(d->count); dfree(d->pos_accum);
    dfree(d->marker); dfree(d->flag); dfree(d->rank); dfree(d->slots); dfree(d->offset);
    dfree(d->block_sums); dfree(d->scalars);
    if (d->pinned) (void)hipHostFree(d->pinned);
    delete d;
    return GS_OK;
}

int gs_density_set_max_gaussians(gs_density* d, uint64_t max_gaussians) {
    if (!d) return fail(GS_E_INVALID, "gs_density_set_max_gaussians: null handle");
    d->max_gaussians = max_gaussians;
    return GS_OK;
}

int gs_density_set_scene_extent(gs_density* d, float extent) {
    if (!d) return fail(GS_E_INVALID, "gs_density_set_scene_extent: null handle");
    d->scene_extent = extent;
    return GS_OK;
}

int gs_density_reset(gs_density* d, void* stream, size_t n) {
    if (!d) return fail(GS_E_INVALID, "gs_density_reset: null handle");
    GS_HIP(hipSetDevice(d->device));
    int rc = density_ensure(d, n);
    if (rc != GS_OK) return rc;
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    if (n) {
        GS_HIP(hipMemsetAsync(d->accum, 0, n * sizeof(float), st));
        GS_HIP(hipMemsetAsync(d->count, 0, n * sizeof(uint32_t), st));
        GS_HIP(hipMemsetAsync(d->pos_accum, 0, n * 3 * sizeof(float), st));
    }
    return GS_OK;
}

int gs_density_accumulate(gs_density* d, void* stream, const GsGradients* d_grad, size_t n) {
    if (!d || (n && !d_grad)) return fail(GS_E_INVALID, "gs_density_accumulate: null argument");
    GS_HIP(hipSetDevice(d->device));
    int rc = density_ensure(d, n);
    if (rc != GS_OK) return rc;
    GS_HIP(launch_density_accumulate(reinterpret_cast<hipStream_t>(stream), d_grad, (uint32_t)n,
                                     d->accum, d->count, d->pos_accum));
    return GS_OK;
}

int gs_density_accumulate_rows(gs_density* d, void* stream, const float* d_rows14, const float* d_viewspace2,
                               size_t n) {
    if (!d || (n && (!d_rows14 || !d_viewspace2)))
        return fail(GS_E_INVALID, "gs_density_accumulate_rows: null argument");
    GS_HIP(hipSetDevice(d->device));
    int rc = density_ensure(d, n);
    if (rc != GS_OK) return rc;
    GS_HIP(launch_density_accumulate_rows(reinterpret_cast<hipStream_t>(stream), d_rows14, d_viewspace2,
                                          (uint32_t)n, d->accum, d->count, d->pos_accum));
    return GS_OK;
}

int gs_density_accumulate_rows_range(gs_density* d, void* stream, const float* d_rows14,
                                     const float* d_viewspace2, size_t first, size_t count) {
    if (!d || (count && (!d_rows14 || !d_viewspace2)))
        return fail(GS_E_INVALID, "gs_density_accumulate_rows_range: null argument");
    if (first > (1u << 30) || count > (1u << 30) - first)
        return fail(GS_E_INVALID, "gs_density_accumulate_rows_range: range too large");
    GS_HIP(hipSetDevice(d->device));
    int rc = density_ensure(d, first + count);
    if (rc != GS_OK) return rc;
    // the rows kernel indexes rows, viewspace and accumulators alike: offset all of them to `first`
    GS_HIP(launch_density_accumulate_rows(reinterpret_cast<hipStream_t>(stream), d_rows14 + first * GS_GRAD_ROW_FLOATS,
                                          d_viewspace2 + first * 2, (uint32_t)count, d->accum + first,
                                          d->count + first, d->pos_accum + first * 3));
    return GS_OK;
}

int gs_density_read(gs_density* d, void* stream, float* d_accum, uint32_t* d_count,
                    float* d_pos_accum, size_t n) {
    if (!d) return fail(GS_E_INVALID, "gs_density_read: null handle");
    if (n > d->cap) return fail(GS_E_INVALID, "gs_density_read: n above capacity");
    GS_HIP(hipSetDevice(d->device));
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    if (n && d_accum)
        GS_HIP(hipMemcpyAsync(d_accum, d->accum, n * sizeof(float), hipMemcpyDeviceToDevice, st));
    if (n && d_count)
        GS_HIP(hipMemcpyAsync(d_count, d->count, n * sizeof(uint32_t), hipMemcpyDeviceToDevice, st));
    if (n && d_pos_accum)
        GS_HIP(hipMemcpyAsync(d_pos_accum, d->pos_accum, n * 3 * sizeof(float),
                              hipMemcpyDeviceToDevice, st));
    return GS_OK;
}

int gs_density_write(gs_density* d, void* stream, const float* d_accum, const uint32_t* d_count,
                     const float* d_pos_accum, size_t n) {
    if (!d) return fail(GS_E_INVALID, "gs_density_write: null handle");
    if (n > d->cap) return fail(GS_E_INVALID, "gs_density_write: n above capacity");
    GS_HIP(hipSetDevice(d->device));
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    if (n && d_accum)
        GS_HIP(hipMemcpyAsync(d->accum, d_accum, n * sizeof(float), hipMemcpyDeviceToDevice, st));
    if (n && d_count)
        GS_HIP(hipMemcpyAsync(d->count, d_count, n * sizeof(uint32_t), hipMemcpyDeviceToDevice, st));
    if (n && d_pos_accum)
        GS_HIP(hipMemcpyAsync(d->pos_accum, d_pos_accum, n * 3 * sizeof(float),
                              hipMemcpyDeviceToDevice, st));
    return GS_OK;
}

int gs_density_apply(gs_density* d, void* stream, const GsGaussian* d_in, size_t n_in,
                     GsGaussian** d_out, size_t* n_out, uint64_t iteration, float focal,
                     float image_width, float avg_depth, uint64_t seed, GsDensityStats* stats) {
    if (!d || !d_out || !n_out || (n_in && !d_in))
        return fail(GS_E_INVALID, "gs_density_apply: null argument");
    if (n_in > (1u << 30)) return fail(GS_E_INVALID, "gs_density_apply: count too large");
    GS_HIP(hipSetDevice(d->device));
    int rc = density_ensure(d, n_in);
    if (rc != GS_OK) return rc;
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    const uint32_t n = (uint32_t)n_in;
    GsDensityStats s = {0, 0, 0, 0};
    *d_out = nullptr;
    *n_out = 0;
    d->last_mapped = false;
    d->last_in = n;
    d->last_out = n;
    if (iteration >= 15000u) {  // density_control.mm:216-220: stop, reset, no change
        GsGaussian* o = nullptr;
        GS_HIP(dalloc(&o, n));
        if (n) GS_HIP(hipMemcpyAsync(o, d_in, n * sizeof(GsGaussian), hipMemcpyDeviceToDevice, st));
        if ((rc = gs_density_reset(d, stream, n)) != GS_OK) return rc;
        GS_HIP(hipStreamSynchronize(st));
        *d_out = o;
        *n_out = n;
        if (stats) *stats = s;
        return GS_OK;
    }
    const uint32_t can_densify = iteration > 500u ? 1u : 0u;
    const uint32_t screen_prune = iteration > 3000u ? 1u : 0u;
    GS_HIP(hipMemsetAsync(d->scalars, 0, 4 * sizeof(uint32_t), st));
    GS_HIP(launch_density_mark(st, d_in, n, d->accum, d->count, can_densify, screen_prune,
                               0.01f * d->scene_extent /* PERCENT_DENSE, density_control.mm:26 */,
                               0.1f * d->scene_extent /* :247 */, focal, image_width,
                               avg_depth, d->marker, d->scalars));
    GS_HIP(hipMemcpyAsync(d->pinned, d->scalars, 3 * sizeof(uint32_t), hipMemcpyDeviceToHost, st));
    GS_HIP(hipStreamSynchronize(st));
    s.num_pruned = d->pinned[0];
    s.num_cloned = d->pinned[1];
    s.num_split = d->pinned[2];
    uint64_t new_count = (uint64_t)n - s.num_pruned + s.num_cloned + s.num_split;
    if (d->max_gaussians && new_count > d->max_gaussians) {  // density_control.mm:360-382
        uint64_t excess = new_count - d->max_gaussians;
        const uint64_t dc = std::min<uint64_t>(excess, s.num_cloned);
        GS_HIP(launch_density_demote(st, d->marker, n, 2u, dc, d->flag, d->rank, d->block_sums,
                                     d->scalars + 4));
        s.num_cloned -= (uint32_t)dc;
        excess -= dc;
        const uint64_t ds = std::min<uint64_t>(excess, s.num_split);
        GS_HIP(launch_density_demote(st, d->marker, n, 3u, ds, d->flag, d->rank, d->block_sums,
                                     d->scalars + 4));
        s.num_split -= (uint32_t)ds;
        new_count = (uint64_t)n - s.num_pruned + s.num_cloned + s.num_split;
    }
    GS_HIP(launch_density_slots(st, d->marker, n, d->slots));
    if (n) GS_HIP(exclusive_scan(st, d->slots, nullptr, n, d->offset, d->block_sums, d->scalars + 4, nullptr));
    GsGaussian* o = nullptr;
    GS_HIP(dalloc(&o, new_count));
    GS_HIP(launch_density_emit(st, d_in, n, d->marker, d->offset, seed, o));
    GS_HIP(hipStreamSynchronize(st));
    // density_control.mm:493 reset accumulators for the next interval
    if ((rc = gs_density_reset(d, stream, new_count)) != GS_OK) {
        (void)hipFree(o);
        return rc;
    }
    GS_HIP(hipStreamSynchronize(st));
    *d_out = o;
    *n_out = (size_t)new_count;
    d->last_mapped = true;
    d->last_out = new_count;
    if (stats) *stats = s;
    return GS_OK;
}

// ---- Adam optimizer ------------------------------------------------------------------------
namespace {
int adam_grow(gs_adam* a, hipStream_t st, size_t n) {
    if (n <= a->cap) return GS_OK;
    const size_t cap = std::max<size_t>(n, a->cap + a->cap / 2);
    float4 *m = nullptr, *v = nullptr;
    uint8_t* live = nullptr;
    GS_HIP(dalloc(&m, cap * 6));
    GS_HIP(dalloc(&v, cap * 6));
    GS_HIP(dalloc(&live, cap));
    GS_HIP(hipMemsetAsync(m, 0, cap * 6 * sizeof(float4), st));
    GS_HIP(hipMemsetAsync(v, 0, cap * 6 * sizeof(float4), st));
    GS_HIP(hipMemsetAsync(live, 0, cap, st));
    if (a->cap) {  // keep the contents (optimizer.mm:101-112)
        GS_HIP(hipMemcpyAsync(m, a->m, a->cap * 6 * sizeof(float4), hipMemcpyDeviceToDevice, st));
        GS_HIP(hipMemcpyAsync(v, a->v, a->cap * 6 * sizeof(float4), hipMemcpyDeviceToDevice, st));
        GS_HIP(hipMemcpyAsync(live, a->live, a->cap, hipMemcpyDeviceToDevice, st));
    }
    GS_HIP(hipStreamSynchronize(st));
    dfree(a->m);
    dfree(a->v);
    dfree(a->live);
    a->m = m;
    a->v = v;
    a->live = live;
    a->cap = cap;
    return GS_OK;
}

// moment-record lanes: 0-2 position, 3 opacity, 4-6 log-scale, 7 pad, 8-11 rotation, 12-23 sh
constexpr uint32_t kMomAll = 0xffffffu, kMomOpacity = 1u << 3, kMomScale = 0x70u;
}  // namespace

int gs_adam_create(int device, uint32_t max_gaussians, gs_adam** out) {
    if (!out) return fail(GS_E_INVALID, "gs_adam_create: out is null");
    *out = nullptr;
    int ndev = 0;
    GS_HIP(hipGetDeviceCount(&ndev));
    if (device < 0 || device >= ndev) return fail(GS_E_INVALID, "gs_adam_create: bad device index");
    GS_HIP(hipSetDevice(device));
    gs_adam* a = new (std::nothrow) gs_adam();
    if (!a) return fail(GS_E_NOMEM, "gs_adam_create: host allocation failed");
    a->device = device;
    int rc = GS_OK;
    if (dalloc(&a->flag, 1) != hipSuccess || hipMemset(a->flag, 0, sizeof(uint32_t)) != hipSuccess)
        rc = fail(GS_E_NOMEM, "gs_adam_create: flag allocation failed");
    if (rc == GS_OK) rc = adam_grow(a, nullptr, std::max<size_t>(max_gaussians, 1));
    if (rc != GS_OK) {
        gs_adam_destroy(a);
        return rc;
    }
    *out = a;
    return GS_OK;
}

int gs_adam_destroy(gs_adam* a) {
    if (!a) return GS_OK;
    (void)hipSetDevice(a->device);
    (void)hipDeviceSynchronize();
    dfree(a->m);
    dfree(a->v);
    dfree(a->flag);
    dfree(a->live);
    delete a;
    return GS_OK;
}

int gs_adam_reset(gs_adam* a, void* stream) {
    if (!a) return fail(GS_E_INVALID, "gs_adam_reset: null handle");
    GS_HIP(hipSetDevice(a->device));
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    a->t = 0;
    GS_HIP(hipMemsetAsync(a->flag, 0, sizeof(uint32_t), st));
    GS_HIP(hipMemsetAsync(a->live, 0, a->cap, st));
    GS_HIP(hipMemsetAsync(a->m, 0, a->cap * 6 * sizeof(float4), st));
    GS_HIP(hipMemsetAsync(a->v, 0, a->cap * 6 * sizeof(float4), st));
    return GS_OK;
}

int gs_adam_step(gs_adam* a, void* stream, GsGaussian* d_g, const GsGradients* d_grad, size_t n,
                 const float lrs[5]) {
    if (!a || !lrs || (n && (!d_g || !d_grad))) return fail(GS_E_INVALID, "gs_adam_step: null argument");
    if (n > (1u << 30)) return fail(GS_E_INVALID, "gs_adam_step: count too large");
    GS_HIP(hipSetDevice(a->device));
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    int rc = adam_grow(a, st, n);
    if (rc != GS_OK) return rc;
    a->t++;  // optimizer.mm:250
    // bias corrections 1 - beta^t (shaders.metal:579-580), pow correctly rounded on the host
    const float p1 = (float)std::pow((double)a->beta1, (double)a->t);
    const float p2 = (float)std::pow((double)a->beta2, (double)a->t);
    GS_HIP(launch_adam(st, d_g, d_grad, nullptr, 0u, (uint32_t)n, a->m, a->v, lrs, a->beta1, a->beta2, a->eps,
                       a->clip, 1.0f - p1, 1.0f - p2, nullptr, a->live));
    if (n) GS_HIP(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(a->flag), 1, 1, st));  // (the records' cold SH fields are not inspected)
    return GS_OK;
}

static int adam_rows_impl(gs_adam* a, void* stream, GsGaussian* d_g, const float* d_rows14, size_t first,
                          size_t count, const float lrs[5], const char* who) {
    if (!a || !lrs || (count && (!d_g || !d_rows14))) return fail(GS_E_INVALID, std::string(who) + ": null argument");
    if (first > (1u << 30) || count > (1u << 30) - first) return fail(GS_E_INVALID, std::string(who) + ": range too large");
    if (a->t == 0) return fail(GS_E_STATE, std::string(who) + ": no gs_adam_begin_step before the first range");
    GS_HIP(hipSetDevice(a->device));
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    int rc = adam_grow(a, st, first + count);
    if (rc != GS_OK) return rc;
    const float p1 = (float)std::pow((double)a->beta1, (double)a->t);
    const float p2 = (float)std::pow((double)a->beta2, (double)a->t);
    GS_HIP(launch_adam(st, d_g, nullptr, d_rows14, (uint32_t)first, (uint32_t)count, a->m, a->v, lrs, a->beta1,
                       a->beta2, a->eps, a->clip, 1.0f - p1, 1.0f - p2, a->flag, a->live));
    return GS_OK;
}

int gs_adam_step_rows(gs_adam* a, void* stream, GsGaussian* d_g, const float* d_rows14, size_t first,
                      size_t count, const float lrs[5]) {
    if (!a) return fail(GS_E_INVALID, "gs_adam_step_rows: null argument");
    a->t++;  // optimizer.mm:250
    int rc = adam_rows_impl(a, stream, d_g, d_rows14, first, count, lrs, "gs_adam_step_rows");
    if (rc != GS_OK) a->t--;  // nothing was stepped
    return rc;
}

int gs_adam_begin_step(gs_adam* a) {
    if (!a) return fail(GS_E_INVALID, "gs_adam_begin_step: null handle");
    a->t++;  // optimizer.mm:250, once per optimizer step whatever the number of ranges
    return GS_OK;
}

int gs_adam_step_rows_range(gs_adam* a, void* stream, GsGaussian* d_g, const float* d_rows14, size_t first,
                            size_t count, const float lrs[5]) {
    return adam_rows_impl(a, stream, d_g, d_rows14, first, count, lrs, "gs_adam_step_rows_range");
}

int gs_adam_timestep(gs_adam* a, uint32_t* t_out) {
    if (!a || !t_out) return fail(GS_E_INVALID, "gs_adam_timestep: null argument");
    *t_out = a->t;
    return GS_OK;
}

int gs_adam_resize(gs_adam* a, void* stream, size_t n) {
    if (!a) return fail(GS_E_INVALID, "gs_adam_resize: null handle");
    GS_HIP(hipSetDevice(a->device));
    return adam_grow(a, reinterpret_cast<hipStream_t>(stream), n);
}

int gs_adam_reset_new(gs_adam* a, void* stream, size_t start, size_t n) {
    if (!a) return fail(GS_E_INVALID, "gs_adam_reset_new: null handle");
    GS_HIP(hipSetDevice(a->device));
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    int rc = adam_grow(a, st, n);
    if (rc != GS_OK) return rc;
    GS_HIP(launch_adam_zero(st, reinterpret_cast<float*>(a->m), reinterpret_cast<float*>(a->v),
                            (uint32_t)std::min(start, n), (uint32_t)n, kMomAll, a->live));
    return GS_OK;
}

int gs_adam_reset_opacity_momentum(gs_adam* a, void* stream, size_t n) {
    if (!a) return fail(GS_E_INVALID, "gs_adam_reset_opacity_momentum: null handle");
    GS_HIP(hipSetDevice(a->device));
    GS_HIP(launch_adam_zero(reinterpret_cast<hipStream_t>(stream), reinterpret_cast<float*>(a->m),
                            reinterpret_cast<float*>(a->v), 0u, (uint32_t)std::min(n, a->cap), kMomOpacity,
                            a->live));
    return GS_OK;
}

int gs_adam_reset_scale_momentum(gs_adam* a, void* stream, size_t n) {
    if (!a) return fail(GS_E_INVALID, "gs_adam_reset_scale_momentum: null handle");
    GS_HIP(hipSetDevice(a->device));
    GS_HIP(launch_adam_zero(reinterpret_cast<hipStream_t>(stream), reinterpret_cast<float*>(a->m),
                            reinterpret_cast<float*>(a->v), 0u, (uint32_t)std::min(n, a->cap), kMomScale,
                            a->live));
    return GS_OK;
}

int gs_adam_follow_density(gs_adam* a, void* stream, const gs_density* d, size_t n_in, size_t n_out) {
    if (!a || !d) return fail(GS_E_INVALID, "gs_adam_follow_density: null argument");
    if (d->last_in != n_in || d->last_out != n_out || n_in > d->cap)
        return fail(GS_E_STATE, "gs_adam_follow_density: counts do not match the last gs_density_apply");
    GS_HIP(hipSetDevice(a->device));
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    int rc = adam_grow(a, st, n_in);
    if (rc != GS_OK) return rc;
    if (!d->last_mapped) return GS_OK;  // the apply changed nothing
    const size_t cap = std::max<size_t>(std::max<size_t>(n_out, a->cap), 1);
    float4 *m = nullptr, *v = nullptr;
    uint8_t* live = nullptr;
    GS_HIP(dalloc(&m, cap * 6));
    GS_HIP(dalloc(&v, cap * 6));
    GS_HIP(dalloc(&live, cap));
    GS_HIP(hipMemsetAsync(m, 0, cap * 6 * sizeof(float4), st));
    GS_HIP(hipMemsetAsync(v, 0, cap * 6 * sizeof(float4), st));
    GS_HIP(hipMemsetAsync(live, 0, cap, st));
    GS_HIP(launch_adam_follow(st, d->marker, d->offset, (uint32_t)n_in, a->m, a->v, m, v, live));
    GS_HIP(hipStreamSynchronize(st));
    dfree(a->m);
    dfree(a->v);
    dfree(a->live);
    a->m = m;
    a->v = v;
    a->live = live;
    a->cap = cap;
    return GS_OK;
}

int gs_adam_read_state(gs_adam* a, void* stream, float* d_m, float* d_v, size_t n) {
    if (!a || (n && (!d_m || !d_v))) return fail(GS_E_INVALID, "gs_adam_read_state: null argument");
    if (n > a->cap) return fail(GS_E_INVALID, "gs_adam_read_state: n exceeds the state size");
    GS_HIP(hipSetDevice(a->device));
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    GS_HIP(launch_adam_layout(st, reinterpret_cast<const float*>(a->m), reinterpret_cast<const float*>(a->v), d_m,
                              d_v, (uint32_t)n, false, nullptr, nullptr));
    return GS_OK;
}

int gs_adam_write_state(gs_adam* a, void* stream, const float* d_m, const float* d_v, size_t n) {
    if (!a || (n && (!d_m || !d_v))) return fail(GS_E_INVALID, "gs_adam_write_state: null argument");
    GS_HIP(hipSetDevice(a->device));
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    int rc = adam_grow(a, st, n);
    if (rc != GS_OK) return rc;
    // (a non-zero cold lane in the written state sets the device word; nothing is read back, so the
    // call stays stream-ordered and capturable)
    if (n)
        GS_HIP(launch_adam_layout(st, d_m, d_v, reinterpret_cast<float*>(a->m), reinterpret_cast<float*>(a->v),
                                  (uint32_t)n, true, a->flag, a->live));
    return GS_OK;
}

int gs_opacity_reset(void* stream, GsGaussian* d_g, size_t n, float max_raw) {
    if (n && !d_g) return fail(GS_E_INVALID, "gs_opacity_reset: null Gaussians");
    GS_HIP(launch_opacity_reset(reinterpret_cast<hipStream_t>(stream), d_g, (uint32_t)n, max_raw));
    return GS_OK;
}

// ---- training loss ---------------------------------------------------------------------------
int gs_loss_create(int device, gs_loss** out) {
    if (!out) return fail(GS_E_INVALID, "gs_loss_create: out is null");
    *out = nullptr;
    int ndev = 0;
    GS_HIP(hipGetDeviceCount(&ndev));
    if (device < 0 || device >= ndev) return fail(GS_E_INVALID, "gs_loss_create: bad device index");
    gs_loss* l = new (std::nothrow) gs_loss();
    if (!l) return fail(GS_E_NOMEM, "gs_loss_create: host allocation failed");
    l->device = device;
    *out = l;
    return GS_OK;
}

int gs_loss_destroy(gs_loss* l) {
    if (!l) return GS_OK;
    (void)hipSetDevice(l->device);
    (void)hipDeviceSynchronize();
    dfree(l->partial);
    delete l;
    return GS_OK;
}

int gs_loss_compute(gs_loss* l, void* stream, const uint32_t* d_rendered, const uint32_t* d_gt,
                    uint32_t w, uint32_t h, float lambda_dssim, float* d_loss, float* d_maps) {
    if (!l || !d_rendered || !d_gt || !d_loss) return fail(GS_E_INVALID, "gs_loss_compute: null argument");
    if (w == 0 || h == 0 || w > 65535u * 16u || h > 65535u * 16u)
        return fail(GS_E_INVALID, "gs_loss_compute: bad image size");
    GS_HIP(hipSetDevice(l->device));
    const uint32_t nb = loss_blocks(w, h);
    if (nb > l->cap) {
        GS_HIP(hipDeviceSynchronize());
        dfree(l->partial);
        l->cap = 0;
        GS_HIP(dalloc(&l->partial, nb));
        l->cap = nb;
    }
    GS_HIP(launch_loss(reinterpret_cast<hipStream_t>(stream), d_rendered, d_gt, w, h, lambda_dssim, d_maps,
                       l->partial, d_loss));
    return GS_OK;
}

int gs_free(void* d_ptr) {
    if (d_ptr) GS_HIP(hipFree(d_ptr));
    return GS_OK;
}

}  // extern "C"
