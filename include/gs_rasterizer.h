/*
 * gs_rasterizer.h — C-ABI of the MI355X-native tiled 3D Gaussian Splatting rasterizer.
 *
 * This is the drop-in boundary for the reference's hot path
 *   TiledRasterizer::{forward,backward}     (GuassianSplatting/tiled_rasterizer.hpp:56-124)
 *   DensityController::{accumulateGradients,apply,resetAccumulator,setSceneExtent}
 *                                            (GuassianSplatting/density_control.hpp:22-48)
 * All record types below are byte-for-byte the reference layouts (static_asserted in
 * gaussiansplatting_amd/csrc/gs_capi.cpp and, compiled with gcc, in tests/test_capi.py).
 *
 * Conventions
 *   - every entry point returns int status: GS_OK (0) or a negative GS_E* code;
 *     gs_last_error() returns a thread-local message for the last failure.
 *     No C++ exception crosses this boundary.
 *   - every pointer named d_* is device (HBM) memory on the handle's device.
 *   - `stream` is a hipStream_t passed as void* (NULL = the null stream). All compute
 *     calls are stream-asynchronous; only the calls documented "synchronous" block.
 *   - one handle = one device + one stream at a time; handles are not thread-safe.
 *   - gs_backward must follow gs_forward on the same handle with the same Gaussians,
 *     count and uniforms (the reference has the same contract: tiled_rasterizer.mm:675-722
 *     reuses the forward's projected/sorted/tileRange/lastIdx state).
 */
#ifndef GS_RASTERIZER_H
#define GS_RASTERIZER_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GS_ABI_VERSION 5

/* status codes */
#define GS_OK 0
#define GS_E_INVALID (-1)   /* bad argument (null pointer, size out of range, ...) */
#define GS_E_HIP (-2)       /* a HIP runtime call failed */
#define GS_E_NOMEM (-3)     /* device allocation failed */
#define GS_E_STATE (-4)     /* call order violated (backward without forward, ...) */
#define GS_E_CAPACITY (-5)  /* a capacity limit could not be satisfied */

#define GS_TILE_SIZE 16u
#define GS_MAX_TILES_PER_GAUSSIAN 256u /* tiled_shaders.metal:743 */

/* ---- records (reference layouts) -------------------------------------------------- */

/* Gaussian: 112 B AoS.  ply_loader.hpp:14-20 / tiled_shaders.metal:11-22 */
typedef struct GsGaussian {
    float position[3]; /* @0  */
    float _pad0;       /* @12 */
    float scale[3];    /* @16 LOG scale */
    float _pad1;       /* @28 */
    float rotation[4]; /* @32 (w,x,y,z) stored as .x=w .y=x .z=y .w=z */
    float opacity;     /* @48 raw, pre-sigmoid */
    float sh[12];      /* @52 channel-major R0..3 G0..3 B0..3; DC = sh[0], sh[4], sh[8] */
    float _pad2[3];    /* @100 */
} GsGaussian;

/* ProjectedGaussian: 88 B.  tiled_rasterizer.hpp:24-39 / tiled_shaders.metal:27-42 */
typedef struct GsProjected {
    float screen_pos[2]; /* @0  */
    float conic[3];      /* @8  */
    float depth;         /* @20 */
    float opacity;       /* @24 sigmoid(clamp(raw, +-8)) */
    float color[3];      /* @28 */
    float radius;        /* @40 */
    uint32_t tile_min_x; /* @44 */
    uint32_t tile_min_y; /* @48 */
    uint32_t tile_max_x; /* @52 */
    uint32_t tile_max_y; /* @56 */
    float _pad1;         /* @60 */
    float view_pos_xy[2];/* @64 */
    float cov2d[3];      /* @72 (a, b, c) after the +0.3 low-pass */
    float _pad2;         /* @84 */
} GsProjected;

/* TiledUniforms: 240 B, column-major float4x4s.  tiled_rasterizer.hpp:42-53 /
 * tiled_shaders.metal:51-62; filled by the caller (mtl_engine.mm:912-924). */
typedef struct GsTiledUniforms {
    float view[16];       /* @0   world->view, column-major (view[4*c + r]) */
    float proj[16];       /* @64  */
    float view_proj[16];  /* @128 proj * view */
    float screen_size[2]; /* @192 */
    float focal[2];       /* @200 fx, fy */
    float camera_pos[3];  /* @208 (16-B slot) */
    float _pad_cam;       /* @220 */
    uint32_t num_tiles_x; /* @224 overwritten by the rasterizer (tiled_rasterizer.mm:309) */
    uint32_t num_tiles_y; /* @228 overwritten */
    uint32_t num_gaussians;/* @232 overwritten */
    uint32_t _pad2;       /* @236 */
} GsTiledUniforms;

/* GaussianGradients: 112 B.  gradients.hpp:11-31 / tiled_shaders.metal:65-80.
 * Only 16 of the 28 floats are ever non-zero (sh[0], sh[4], sh[8] of the SH block). */
typedef struct GsGradients {
    float position[3];   /* @0  */
    float opacity;       /* @12 d/d(raw opacity) */
    float scale[3];      /* @16 d/d(log scale) */
    float _pad1;         /* @28 */
    float rotation[4];   /* @32 d/d(w,x,y,z) of the raw (un-normalised) quaternion */
    float sh[12];        /* @48 */
    float viewspace[2];  /* @96 dL/dScreenPos (x, y) */
    float _pad2[2];      /* @104 */
} GsGradients;

/* TileRange: 8 B.  tiled_shaders.metal:45-48 / tiled_rasterizer.hpp:16-19 */
typedef struct GsTileRange {
    uint32_t start;
    uint32_t count;
} GsTileRange;

/* DensityStats.  density_control.hpp:12-16 */
typedef struct GsDensityStats {
    uint32_t num_pruned;
    uint32_t num_cloned;
    uint32_t num_split;
    uint32_t _pad;
} GsDensityStats;

/* Per-frame statistics of the last gs_forward/gs_backward (host readback; synchronous). */
typedef struct GsFrameStats {
    uint64_t num_pairs;      /* P: emitted (tile, Gaussian) pairs */
    uint64_t pair_capacity;  /* current P capacity */
    uint32_t num_visible;    /* Gaussians that emitted >= 1 pair */
    uint32_t num_tiles;
    uint32_t width, height;
    uint32_t sort_passes_depth, sort_passes_tile;
    uint32_t overflowed;     /* 1 if P exceeded capacity (the frame was re-run after growth) */
    uint32_t scan_errors;    /* 0; non-zero if a cross-workgroup scan gave up waiting (never expected) */
    uint32_t tile_sort_path; /* the tile sort the frame took: 1 one-pass counting sort, 2 8-bit LSD */
    uint32_t _pad;
    /* Work the blends did (the roofline's walked bytes): the list entries whose records
     * the forward read (per tile, the farthest of its four band waves: every band stops once its
     * pixels are saturated) and the backward read (per tile, up to its last contributing entry);
     * the Gaussians whose entries the last backward selected, and their partial-sum slots. */
    uint64_t fwd_walked_entries;
    uint64_t bwd_walked_entries;
    uint64_t reached_gaussians;
    uint64_t reached_slots;
} GsFrameStats;

typedef struct gs_handle gs_handle;
typedef struct gs_density gs_density;

/* ---- lifetime --------------------------------------------------------------------- */

const char* gs_last_error(void);
int gs_abi_version(void);

/* Replaces TiledRasterizer(MTL::Device*, MTL::Library*, uint32_t maxGaussians)
 * (tiled_rasterizer.hpp:59).  max_w/max_h pre-size the per-pixel scratch (0 = lazily). */
int gs_create(int device, uint32_t max_gaussians, uint32_t max_w, uint32_t max_h,
              gs_handle** out);
/* Replaces ~TiledRasterizer (tiled_rasterizer.mm:160-177). */
int gs_destroy(gs_handle* h);

/* Reserve room for `max_pairs` (tile, Gaussian) pairs.  While the capacity is below
 * n*min(256, tiles) the forward reads P back once per frame (one 4-byte D2H sync) to
 * grow; at or above it the whole frame is sync-free.  Replaces ensurePairsCapacity
 * (tiled_rasterizer.mm:242-272) without its 100M / 50M clamps. */
int gs_reserve_pairs(gs_handle* h, uint64_t max_pairs);

/* Tile-sort path of the following frames: 0 = automatic (the one-pass counting sort while the
 * previous frame's P <= 16M and tiles <= 12288, else two 8-bit LSD passes), 1 = the one-pass sort
 * whenever tiles <= 12288, 2 = always LSD.  Both paths give identical results (tests pin each at
 * config 5's ~69M pairs); gs_frame_stats reports the one taken (tile_sort_path).  No reference counterpart: the
 * reference sorts 64-bit keys on the CPU (tiled_rasterizer.mm:27-102, 498-505). */
int gs_set_tile_sort_path(gs_handle* h, int mode);

/* Depth ordering of the following frames' tile lists: 0 = automatic (the per-tile sort when the
 * one-pass tile sort is taken and the previous frame had at most 16 pairs per Gaussian, else the
 * global sort), 1 = a global depth sort of the N Gaussians before the pairs are emitted in depth
 * order, 2 = the tile lists built straight from the Gaussians (in any order inside a list), then every
 * list sorted by (depth key, Gaussian index) on its own.  Both
 * give the reference's (tile, depth, Gaussian) order exactly (tests pin each); gs_frame_stats reports
 * the global passes taken (sort_passes_depth, 0 with the per-tile sort).  No reference counterpart:
 * the reference sorts 64-bit (tile | depth) keys on the CPU (tiled_rasterizer.mm:27-102). */
int gs_set_depth_sort(gs_handle* h, int mode);

/* Backward list split of the following frames: the first `tiles` tiles of the backward's launch order
 * (the forward's measured work, heaviest first inside each XCD group; every tile by default) each run
 * as two backward waves over two parts of their list -- the back three quarters first
 * (the reverse pass starts there), then the front quarter, which continues from the back part's
 * per-pixel transmittance and accumulated colour (handed over through memory).  Every (tile, Gaussian) entry
 * is still processed once, by one wave, with the same per-pixel float operations in the same order:
 * the gradients are bit-identical to the unsplit backward (tested).  Shorter jobs balance the
 * kernel's tail.  tiles < 0: automatic (every tile), 0: off.  No reference counterpart (the
 * reference's backward is one thread per pixel, tiled_shaders.metal:388-738). */
int gs_set_backward_split(gs_handle* h, int tiles);

/* Gradient chain kernel of the following backwards: < 0 automatic (the compacting kernel when the
 * latest frame had more than 8 pairs per Gaussian -- deep lists, where most Gaussians reach no
 * pixel), 0 = the plain per-Gaussian kernel, 1 = the compacting kernel.  Bit-identical gradients
 * (tested); a performance choice only. */
int gs_set_chain_compact(gs_handle* h, int mode);

/* ---- hot path --------------------------------------------------------------------- */

/* Replaces TiledRasterizer::forward (tiled_rasterizer.hpp:63-67, .mm:275-672):
 * project -> per-tile keys -> (tile|depth) radix sort -> tile ranges -> front-to-back blend.
 * d_rgba8_out: w*h packed RGBA8 (R in the low byte), the RGBA8Unorm render target.
 * d_rgb_f32_out (nullable): w*h*3 floats, the blended colour before 8-bit quantisation.
 * When P == 0 the reference returns before rendering (tiled_rasterizer.mm:463-467):
 * the output buffers are then left untouched. */
int gs_forward(gs_handle* h, void* stream, const GsGaussian* d_gaussians, size_t n,
               const GsTiledUniforms* uniforms, uint32_t w, uint32_t hgt,
               uint32_t* d_rgba8_out, float* d_rgb_f32_out);

/* Replaces TiledRasterizer::backward (tiled_rasterizer.hpp:69-75, .mm:675-722).
 * Writes every record of d_grad[0..n) (the reference memsets then accumulates).
 * d_rendered_rgba8 must be the forward's RGBA8 output; d_gt_rgba8 the ground truth. */
int gs_backward(gs_handle* h, void* stream, const GsGaussian* d_gaussians,
                GsGradients* d_grad, size_t n, const GsTiledUniforms* uniforms,
                const uint32_t* d_rendered_rgba8, const uint32_t* d_gt_rgba8);

/* Gradient rows: the 14 live fields of a summed gradient, 14 floats (56 B) per Gaussian,
 *   [0..2] position [3] opacity [4..6] log-scale [7..10] rotation (w,x,y,z)
 *   [11] sh[0] [12] sh[4] [13] sh[8]
 * -- the buffer the multi-GPU path reduces over the ranks (56 B instead of 112 B per Gaussian).
 * The screen-space gradient (GaussianGradients.viewspace) is not part of a row: it only feeds the
 * density statistics, which are non-linear per view and accumulated per view before any reduce
 * (SURVEY.md section 8e), so it goes to a separate per-rank buffer of 2 floats per Gaussian.
 * gs_backward_packed = gs_backward with the gradients written as rows (+ viewspace rows when
 * d_viewspace2 is non-null); the fields are bit-identical to gs_backward's. */
#define GS_GRAD_ROW_FLOATS 14
int gs_backward_packed(gs_handle* h, void* stream, const GsGaussian* d_gaussians,
                       float* d_rows14, float* d_viewspace2, size_t n, const GsTiledUniforms* uniforms,
                       const uint32_t* d_rendered_rgba8, const uint32_t* d_gt_rgba8);
/* gs_backward in two parts, for callers that overlap the per-Gaussian chain with other work
 * (the multi-GPU path reduces the first chunks of gradient rows while later chunks are
 * still being computed):
 *   gs_backward_blend  the per-tile blend backward (tiled_shaders.metal:388-738 up to the
 *                      per-pixel partial sums); same preconditions as gs_backward;
 *   gs_backward_chain  the per-Gaussian chain for Gaussians [first, first + count) into either
 *                      d_grad (GaussianGradients records) or d_rows14 (+ d_viewspace2, nullable),
 *                      all indexed by Gaussian; exactly one of d_grad, d_rows14 is non-null. Any
 *                      number of calls, any ranges, after one gs_backward_blend.
 * gs_backward == gs_backward_blend + gs_backward_chain(0, n) (bit-identical results). */
int gs_backward_blend(gs_handle* h, void* stream, const GsGaussian* d_gaussians, size_t n,
                      const GsTiledUniforms* uniforms, const uint32_t* d_rendered_rgba8,
                      const uint32_t* d_gt_rgba8);
int gs_backward_chain(gs_handle* h, void* stream, const GsGaussian* d_gaussians,
                      GsGradients* d_grad, float* d_rows14, float* d_viewspace2, size_t n,
                      const GsTiledUniforms* uniforms, size_t first, size_t count);
/* Rows (n x 14 floats) + viewspace (n x 2 floats; NULL = zero) -> GaussianGradients records (all 28
 * floats written). */
int gs_unpack_gradients(void* stream, const float* d_rows14, const float* d_viewspace2,
                        GsGradients* d_grad, size_t n);

/* Per-stage HIP-event timing. When enabled, forward/backward record events between stages on
 * the caller's stream; gs_stage_times (synchronous) returns the summed milliseconds and call
 * counts per stage since the last read and returns the number of stages (9):
 *   0 project  1 depth sort  2 offset scan  3 pair emission  4 tile sort  5 tile ranges
 *   6 forward blend  7 backward blend  8 per-Gaussian chain */
int gs_set_stage_timing(gs_handle* h, int enable);
int gs_stage_times(gs_handle* h, double* ms_out, uint32_t* calls_out, int max_stages);

/* Synchronous: waits for the handle's last stream work. */
int gs_frame_stats(gs_handle* h, GsFrameStats* out);

/* ---- debug getters (parity tests; stream-ordered copies into caller device memory) - */

/* num_pairs: synchronous readback of P. */
int gs_debug_num_pairs(gs_handle* h, uint64_t* out);
/* Sorted 64-bit keys ((tile << 32) | sortable depth bits) and values (Gaussian index),
 * exactly the reference's sorted pair arrays (tiled_rasterizer.mm:506-512). cap = entries. */
int gs_debug_sorted_pairs(gs_handle* h, void* stream, uint64_t* d_keys, uint32_t* d_values,
                          uint64_t cap);
int gs_debug_tile_ranges(gs_handle* h, void* stream, GsTileRange* d_ranges, uint32_t cap);
int gs_debug_last_idx(gs_handle* h, void* stream, uint32_t* d_last_idx, uint64_t cap);
int gs_debug_projected(gs_handle* h, void* stream, GsProjected* d_proj, size_t cap);
/* Synchronous exhaustive check of the forward's half weight on `device`: over every half power in
 * [-4.5, 0], how many hardware-exp halves differ from the pinned exp's (must be 0; the forward
 * relies on it) and the largest float ulp distance between the two exps. */
int gs_debug_half_exp_check(int device, uint32_t* mismatches, uint32_t* max_ulps);
/* Synchronous exhaustive check of the float weight's hardware exp on `device`: over every float
 * power in [-4.5, 0], the largest relative difference between v_exp_f32(x log2 e) and the pinned
 * exp. The forward's T_final track and its break window rely on it staying below 4e-7. */
int gs_debug_float_exp_check(int device, float* max_rel);
/* Synchronous measured HBM copy bandwidth on `device` (SURVEY.md §8d asks for one next to the 8 TB/s
 * spec): a 16-B-per-lane streaming read + write kernel over two `bytes`-sized buffers (well past the
 * 256 MiB Infinity Cache), plain and non-temporal, 1/2/4/8 workgroups per CU, `reps` launches each;
 * *gbs_out = the best (read + write bytes / s, in GB/s); variants_out (nullable) gets up to
 * max_variants of the individual rates (plain 1/2/4/8, then non-temporal 1/2/4/8). Measurement only:
 * no reference counterpart. */
int gs_debug_copy_bandwidth(int device, uint64_t bytes, int reps, double* gbs_out, double* variants_out,
                            int max_variants);

/* ---- density control hooks ---------------------------------------------------------- */

/* Replaces DensityController(MTL::Device*, MTL::Library*) (density_control.hpp:22) with the
 * 1.5M cap lifted: `max_gaussians` only pre-sizes the accumulators, which grow to the largest
 * count seen; the population cap is gs_density_set_max_gaussians. */
int gs_density_create(int device, uint32_t max_gaussians, gs_density** out);
int gs_density_destroy(gs_density* d);
/* The reference caps the population at MAX_GAUSSIANS = 1.5M (density_control.mm:27, 360-382);
 * here the cap is a setting: 0 (default) = unlimited, otherwise clones then splits are
 * dropped in index order exactly as the reference does. */
int gs_density_set_max_gaussians(gs_density* d, uint64_t max_gaussians);
/* Replaces DensityController::setSceneExtent (density_control.mm:79-84). */
int gs_density_set_scene_extent(gs_density* d, float extent);
/* Replaces DensityController::resetAccumulator (density_control.mm:113-118). */
int gs_density_reset(gs_density* d, void* stream, size_t n);
/* Replaces DensityController::accumulateGradients (density_control.mm:121-185). */
int gs_density_accumulate(gs_density* d, void* stream, const GsGradients* d_grad, size_t n);
/* gs_density_accumulate from gradient rows (the position gradient, rows [0..2]) and the per-view
 * viewspace rows of gs_backward_packed: the same accumulators, bit-identical, without the
 * GaussianGradients records. */
int gs_density_accumulate_rows(gs_density* d, void* stream, const float* d_rows14,
                               const float* d_viewspace2, size_t n);
/* gs_density_accumulate_rows over the Gaussians [first, first + count) only (rows and viewspace
 * point at row 0): a data-parallel caller accumulates each chunk of its own view's rows between the
 * chunk's chain and its all-reduce, so the statistics see this rank's position gradient, not the
 * sum over ranks. */
int gs_density_accumulate_rows_range(gs_density* d, void* stream, const float* d_rows14,
                                     const float* d_viewspace2, size_t first, size_t count);
/* Read back the accumulators (parity tests): accum[n] f32, count[n] u32, pos_accum[n*3] f32. */
int gs_density_read(gs_density* d, void* stream, float* d_accum, uint32_t* d_count,
                    float* d_pos_accum, size_t n);
/* Overwrite the accumulators (same layouts; null pointers leave a field alone). With views
 * sharded over ranks, each rank accumulates its own views; before gs_density_apply the ranks
 * all-reduce (sum) what gs_density_read returns and write it back, so every replica densifies
 * identically. No reference counterpart (the reference is one device). */
int gs_density_write(gs_density* d, void* stream, const float* d_accum, const uint32_t* d_count,
                     const float* d_pos_accum, size_t n);

/* Replaces DensityController::apply (density_control.mm:188-501), on the GPU.
 * Decides prune / clone / split per Gaussian and compacts into a NEW buffer that the library
 * allocates (the reference also allocates a new buffer and frees the caller's,
 * density_control.mm:385-490); *d_out receives it, *n_out its count; free it with gs_free.
 * The caller keeps ownership of d_in.  The split offsets use a counter-based RNG keyed by
 * (seed, gaussian index) instead of rand() (density_control.mm:440-442).  Synchronous. */
int gs_density_apply(gs_density* d, void* stream, const GsGaussian* d_in, size_t n_in,
                     GsGaussian** d_out, size_t* n_out, uint64_t iteration, float focal,
                     float image_width, float avg_depth, uint64_t seed,
                     GsDensityStats* stats);

/* ---- Adam optimizer and opacity reset ---------------------------
 * Replaces AdamOptimizer (optimizer.hpp:22-95; kernel adamStep, shaders.metal:536-713) and the
 * training loop's opacity reset (mtl_engine.mm:1173-1192). The moments live in the handle as one
 * 96-B record per Gaussian for m and for v: (pos xyz, opacity) (log-scale xyz, 0) (rotation)
 * (sh 0..11). beta1 = 0.9, beta2 = 0.999, epsilon = 1e-8, gradient clip 0.5 (optimizer.mm:274-278,
 * shaders.metal:582). The bias corrections 1 - beta^t are computed on the host with a correctly
 * rounded pow (the reference's in-kernel Metal pow is implementation-defined). */
typedef struct gs_adam gs_adam;

/* AdamOptimizer(device, library, numGaussians) (optimizer.mm:11-40): zeroed state, t = 0. */
int gs_adam_create(int device, uint32_t max_gaussians, gs_adam** out);
int gs_adam_destroy(gs_adam* a);
/* AdamOptimizer::reset (optimizer.mm:80-92): t = 0, all moments zero. */
int gs_adam_reset(gs_adam* a, void* stream);
/* AdamOptimizer::step (optimizer.mm:241-296): t += 1, then one update of every Gaussian in place.
 * lrs = {position, log-scale, rotation, raw opacity, sh} (optimizer.hpp:29-41). */
int gs_adam_step(gs_adam* a, void* stream, GsGaussian* d_g, const GsGradients* d_grad, size_t n,
                 const float lrs[5]);
/* gs_adam_step from gradient rows (GS_GRAD_ROW_FLOATS per Gaussian, the other GaussianGradients
 * fields zero: bit-identical to gs_adam_step on the unpacked records) for the Gaussians
 * [first, first + count): row k holds the gradient of Gaussian first + k; d_g and the moments are
 * indexed by Gaussian. t += 1 per call. A data-parallel caller that reduce-scatters the rows calls it
 * on its own shard and all-gathers the updated Gaussians. */
int gs_adam_step_rows(gs_adam* a, void* stream, GsGaussian* d_g, const float* d_rows14, size_t first,
                      size_t count, const float lrs[5]);
/* The same update split over several ranges of one optimizer step (e.g. chunks pipelined behind
 * their all-reduce): gs_adam_begin_step advances t once (optimizer.mm:250), then every
 * gs_adam_step_rows_range call updates its [first, first + count) at that t without advancing it.
 * GS_E_STATE before the first begin. */
int gs_adam_begin_step(gs_adam* a);
int gs_adam_step_rows_range(gs_adam* a, void* stream, GsGaussian* d_g, const float* d_rows14, size_t first,
                            size_t count, const float lrs[5]);
int gs_adam_timestep(gs_adam* a, uint32_t* t_out);
/* AdamOptimizer::resizeIfNeeded (optimizer.mm:95-135): grow to n keeping contents, new space 0. */
int gs_adam_resize(gs_adam* a, void* stream, size_t n);
/* resetStateForNewGaussians(startIdx) (optimizer.mm:150-185): zero the moments of [start, n). */
int gs_adam_reset_new(gs_adam* a, void* stream, size_t start, size_t n);
/* resetOpacityMomentum / resetScaleMomentum (optimizer.mm:137-147), over the first n records. */
int gs_adam_reset_opacity_momentum(gs_adam* a, void* stream, size_t n);
int gs_adam_reset_scale_momentum(gs_adam* a, void* stream, size_t n);
/* After gs_density_apply on (n_in -> n_out) Gaussians: make the moments follow the Gaussians.
 * Survivors keep their moments, clones' copies and split children start at zero (the official
 * 3DGS densification). The reference instead leaves the state un-permuted and only zeroes the
 * tail (mtl_engine.mm:1159-1166); that behaviour is gs_adam_resize + gs_adam_reset_new. */
int gs_adam_follow_density(gs_adam* a, void* stream, const gs_density* d, size_t n_in,
                           size_t n_out);
/* Copy the moments out (parity tests): d_m, d_v: n * 24 floats each. */
int gs_adam_read_state(gs_adam* a, void* stream, float* d_m, float* d_v, size_t n);
/* Overwrite the moments of [0, n) (same layout; the state grows to n if needed). A data-parallel
 * caller whose ranks each step their own shard (gs_adam_step_rows) all-gathers the moments through
 * read/write before gs_adam_follow_density, which needs every Gaussian's. */
int gs_adam_write_state(gs_adam* a, void* stream, const float* d_m, const float* d_v, size_t n);
/* Opacity reset (mtl_engine.mm:1173-1186): raw opacity = min(raw opacity, max_raw) for [0, n);
 * the reference uses max_raw = -4.6 (sigmoid^-1(0.01), :1056). */
int gs_opacity_reset(void* stream, GsGaussian* d_g, size_t n, float max_raw);

/* One training step's backward, fused through the optimizer (mtl_engine.mm:1085-1120's
 * tiledBackward -> accumulateGradients -> adamStep for one view): the blend backward, then per
 * Gaussian the chain, the density statistics (d: nullable, skipped when NULL) and Adam (t += 1) on
 * the Gaussian in place, in one kernel. Bit-identical to gs_backward_packed + gs_density_accumulate_rows
 * + gs_adam_step_rows(0, n) on the same inputs, without the gradient rows in HBM. Same preconditions
 * as gs_backward (the preceding gs_forward on these Gaussians); d_g is updated in place. */
int gs_backward_step(gs_handle* h, void* stream, GsGaussian* d_gaussians, size_t n,
                     const GsTiledUniforms* uniforms, const uint32_t* d_rendered_rgba8,
                     const uint32_t* d_gt_rgba8, gs_density* d, gs_adam* a, const float lrs[5]);

/* ---- training loss ---------------------------------------------
 * Replaces MTLEngine::computeLoss (mtl_engine.mm:769-853) with its kernels computeL1Loss,
 * computeSSIM, computeCombinedLoss and reduceLoss (shaders.metal:320-510): per pixel
 * L1 = mean |rendered - gt| over RGB, D-SSIM = clamp((1 - SSIM) / 2, 0, 1) of the grey images over
 * an 11x11 Gaussian window (sigma 1.5, clamp-to-edge), combined = (1 - lambda) L1 + lambda D-SSIM;
 * *d_loss = mean of the combined map (deterministic fp64 sum; the reference sums with float
 * atomics). Images are RGBA8 [h][w] as everywhere in this ABI. d_maps (nullable) receives three
 * [h][w] float maps: L1, D-SSIM, combined. Stream-ordered; the reference's default lambda is 0.2. */
typedef struct gs_loss gs_loss;
int gs_loss_create(int device, gs_loss** out);
int gs_loss_destroy(gs_loss* l);
int gs_loss_compute(gs_loss* l, void* stream, const uint32_t* d_rendered_rgba8,
                    const uint32_t* d_gt_rgba8, uint32_t w, uint32_t h, float lambda_dssim,
                    float* d_loss, float* d_maps);

/* ---- scene formats and initialisation, host-side ----------------
 * COLMAP binary model (colmap_loader.cpp:26-197), scene extent (:232-264), the initial Gaussians
 * from the sparse points (main.mm:59-187), TiledUniforms from a COLMAP camera + image
 * (mtl_engine.mm:637-682, 866-924), 3DGS PLY read / write (ply_loader.cpp:61-290,
 * ply_exporter.hpp:18-163) and the PPM dump of a render (mtl_engine.mm:19-63).
 * All buffers here are HOST memory. */
typedef struct GsColmapCamera {
    uint32_t id, width, height;
    int32_t model;        /* COLMAP model id; 0, 2, 3: f cx cy ...; else fx fy cx cy ... */
    float fx, fy, cx, cy;
} GsColmapCamera;

typedef struct GsColmapImage {
    uint32_t id;
    uint32_t camera_id;
    float rotation[4];    /* (w, x, y, z), world-to-camera */
    float translation[3];
    float _pad;
    char name[256];       /* NUL-terminated, truncated if longer */
} GsColmapImage;

typedef struct GsColmapPoint {
    float position[3];
    float color[3];       /* rgb8 / 255 */
    float error;
} GsColmapPoint;

typedef struct gs_colmap gs_colmap;

/* loadColmap(dir): dir/cameras.bin, dir/images.bin, dir/points3D.bin. */
int gs_colmap_load(const char* dir, gs_colmap** out);
int gs_colmap_free(gs_colmap* c);
int gs_colmap_counts(const gs_colmap* c, uint32_t* n_cameras, uint32_t* n_images, uint64_t* n_points);
/* cameras in ascending id order (the reference's std::map); images in file order */
int gs_colmap_camera(const gs_colmap* c, uint32_t index, GsColmapCamera* out);
int gs_colmap_camera_by_id(const gs_colmap* c, uint32_t id, GsColmapCamera* out);
int gs_colmap_image(const gs_colmap* c, uint32_t index, GsColmapImage* out);
int gs_colmap_points(const gs_colmap* c, GsColmapPoint* out, uint64_t cap);
/* getCameraWorldPosition (colmap_loader.cpp:200-229) */
int gs_colmap_camera_position(const GsColmapImage* img, float out_xyz[3]);
/* computeSceneExtent (colmap_loader.cpp:232-264): 1.1 x max camera distance from the centroid */
int gs_colmap_scene_extent(const gs_colmap* c, float* out);
/* gaussiansFromColmap (main.mm:59-187): one Gaussian per sparse point; out == NULL: count only */
int gs_gaussians_from_colmap(const gs_colmap* c, float scene_extent, GsGaussian* out, uint64_t cap,
                             uint64_t* n_out);
/* TiledUniforms of image `img` rendered at (width, height) (mtl_engine.mm:866-924): the COLMAP
 * intrinsics scaled to the render size, near 0.1, far 1000. */
int gs_colmap_uniforms(const GsColmapCamera* cam, const GsColmapImage* img, uint32_t width,
                       uint32_t height, GsTiledUniforms* out);
/* load_ply: out == NULL returns the count in *n_out only; invalid positions are skipped, linear
 * scales are detected and converted, log-scales clamped to +-8, quaternions normalised. */
int gs_ply_load(const char* path, GsGaussian* out, uint64_t cap, uint64_t* n_out);
/* PLYExporter::exportPLY: binary little-endian, invalid positions skipped; *n_written (nullable). */
int gs_ply_save(const char* path, const GsGaussian* g, uint64_t n, uint64_t* n_written);
/* saveTextureToPPM: P6, RGB of an RGBA8 [h][w] host image. */
int gs_ppm_save(const char* path, const uint32_t* rgba8, uint32_t w, uint32_t h);
/* A P6 PPM (maxval 255, what gs_ppm_save writes) into an RGBA8 [h][w] host image, alpha 255: the
 * headless caller's ground truth (the reference decodes images with stb_image, image_loader.mm:13-41).
 * rgba8 == NULL: the size only. GS_E_INVALID if w * h > cap_pixels or the file is malformed. */
int gs_ppm_load(const char* path, uint32_t* rgba8, uint64_t cap_pixels, uint32_t* w_out, uint32_t* h_out);

/* Frees memory returned by the library (gs_density_apply). */
int gs_free(void* d_ptr);

#ifdef __cplusplus
}
#endif

#endif /* GS_RASTERIZER_H */
