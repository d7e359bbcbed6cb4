/*
 * gs_oracle.h — TEST INFRASTRUCTURE ONLY (parity checker and CPU baseline).
 *
 * A CPU restatement, in plain C11, of the reference's Metal hot path
 * (ctaylo41/GaussianSplatting @ /root/reference/GuassianSplatting). Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it. The product
 * (gaussiansplatting_amd) never links or calls it.
 *
 * PARITY UNPINNED: the reference is Objective-C++/MSL on Apple Metal; it cannot be built
 * or run in this image (no Metal compiler or runtime, no <simd/simd.h>, no GCD) and it
 * ships no tests, golden vectors or recorded outputs. This restatement
 * follows the MSL text line by line with an explicit IEEE evaluation order (no FMA
 * contraction, left-to-right sums, Metal column-major matrix semantics, the shared
 * deterministic exp below); "reference semantics" is defined as this restatement.
 * It is cross-checked by an independent pure-Python restatement for small cases
 * (tests/test_oracle_kat.py) and by the reference's own runtime self-checks turned
 * into assertions (struct offsets, tile-range coverage == P, sorted keys monotone).
 */
#ifndef GS_ORACLE_H
#define GS_ORACLE_H

#include <stdint.h>
#include <stddef.h>
#include "../include/gs_rasterizer.h"

#ifdef __cplusplus
extern "C" {
#endif

/* deterministic exp (Cody-Waite + degree-6 polynomial, explicit fmaf) */
float gso_expf(float x);
/* IEEE binary16 round-to-nearest-even of a float, returned as float */
float gso_half(float x);
uint16_t gso_half_bits(float x);

/* tiled_shaders.metal:102-304 projectGaussians. u->num_tiles_x/_y/num_gaussians must be set. */
void gso_project(const GsGaussian* g, uint32_t n, const GsTiledUniforms* u, GsProjected* out,
                 int threads);

/* tiled_shaders.metal:745-794 generateTilePairs, emitting in Gaussian-index order (the reference
 * reserves slots with a global atomic, so its emission order is nondeterministic).
 * Returns the counter value (may exceed max_pairs); pairs of a Gaussian whose slot range
 * overflows are dropped whole (:780). */
uint64_t gso_generate_pairs(const GsProjected* p, uint32_t n, uint32_t num_tiles_x,
                            uint64_t max_pairs, uint64_t* keys, uint32_t* values);

/* tiled_rasterizer.mm:27-102 parallelRadixSort: stable LSD, 8 passes x 8 bits over the full
 * 64-bit key, per-thread histograms over `threads` contiguous chunks. (The reference uses an
 * unstable std::sort below 1000 pairs; this restatement is stable at every size.) */
void gso_sort_pairs(uint64_t* keys, uint32_t* values, uint64_t n, int threads);

/* sort.metal:553-589 buildTileRanges: lower-bound binary search + linear count per tile. */
void gso_build_tile_ranges(const uint64_t* keys, uint64_t n_pairs, uint32_t num_tiles,
                           GsTileRange* ranges, int threads);

/* tiled_shaders.metal:307-385 tiledForward (half accumulation, white background).
 * rgba8: packed R | G<<8 | B<<16 | 255<<24 (RGBA8Unorm write of float4(color, 1)). */
void gso_forward_blend(const GsProjected* p, uint32_t n, const uint32_t* sorted_values,
                       const GsTileRange* ranges, const GsTiledUniforms* u, uint32_t w,
                       uint32_t h, uint32_t* last_idx, uint32_t* rgba8, float* rgb_f32,
                       int threads);

/* tiled_shaders.metal:388-738 tiledBackward. Accumulates the 16 live gradient fields in double
 * (grad_out: n*28 doubles laid out like GsGradients), and the sum of |term| per field
 * (abs_out, same layout, nullable) that the parity tolerance is scaled by, and the sum of
 * |float term - fp64 term| (noise_out, nullable): the reference's own rounding noise. */
void gso_backward(const GsGaussian* g, const GsProjected* p, uint32_t n,
                  const uint32_t* sorted_values, const GsTileRange* ranges,
                  const GsTiledUniforms* u, uint32_t w, uint32_t h, const uint32_t* last_idx,
                  const uint32_t* rendered_rgba8, const uint32_t* gt_rgba8, double* grad_out,
                  double* abs_out, double* noise_out, int threads);

/* gso_backward's float sums plus their fp64 shadow (each term recomputed in double): where a
 * float intermediate of the reference overflows, the float sum is NaN and the shadow is finite. */
void gso_backward_shadow(const GsGaussian* g, const GsProjected* p, uint32_t n,
                         const uint32_t* sorted_values, const GsTileRange* ranges,
                         const GsTiledUniforms* u, uint32_t w, uint32_t h, const uint32_t* last_idx,
                         const uint32_t* rendered_rgba8, const uint32_t* gt_rgba8, double* grad_out,
                         double* shadow_out, int threads);

/* One pass producing all five: float sums, |term| sums, rounding noise, the fp64 shadow and the
 * first-order conditioning bound of the per-pixel float steps (sum |term| * r, see gs_oracle.c
 * COND_EXP_REL); abs_out, noise_out, shadow_out, cond_out nullable. */
void gso_backward_full(const GsGaussian* g, const GsProjected* p, uint32_t n,
                       const uint32_t* sorted_values, const GsTileRange* ranges,
                       const GsTiledUniforms* u, uint32_t w, uint32_t h, const uint32_t* last_idx,
                       const uint32_t* rendered_rgba8, const uint32_t* gt_rgba8, double* grad_out,
                       double* abs_out, double* noise_out, double* shadow_out, double* cond_out,
                       int threads);

/* Whole TiledRasterizer::forward (tiled_rasterizer.mm:275-672) + backward (:675-722).
 * Returns P (clamped to max_pairs). keys/values need max_pairs entries. When P == 0 the
 * reference returns before rendering: rgba8/rgb_f32 are left untouched and last_idx is all
 * 0xFFFFFFFF, ranges all zero (tiled_rasterizer.mm:316-317, 463-467). */
uint64_t gso_forward(const GsGaussian* g, uint32_t n, const GsTiledUniforms* u_in, uint32_t w,
                     uint32_t h, uint64_t max_pairs, GsProjected* proj, uint64_t* keys,
                     uint32_t* values, GsTileRange* ranges, uint32_t* last_idx, uint32_t* rgba8,
                     float* rgb_f32, int threads);

/* density_control.mm:121-185 accumulateGradients. */
void gso_density_accumulate(const GsGradients* grads, uint32_t n, float* accum, uint32_t* count,
                            float* pos_accum);

/* density_control.mm:188-501 apply, with the split offsets drawn from gso_density_uniform
 * (counter-based, keyed by seed and Gaussian index) instead of rand(). Returns the new count;
 * out needs room for 2*n records; markers (n u32, nullable) receives 0 keep/1 prune/2 clone/3 split. */
uint64_t gso_density_apply(const GsGaussian* in, uint32_t n, const float* accum,
                           const uint32_t* count, uint64_t iteration, float scene_extent,
                           float focal, float image_width, float avg_depth, uint64_t seed,
                           uint64_t max_gaussians, GsGaussian* out, uint32_t* markers,
                           GsDensityStats* stats);
/* uniform in [-1, 1) for (seed, index, component) */
float gso_density_uniform(uint64_t seed, uint64_t index, uint32_t component);

/* adamStep (shaders.metal:536-713) over the reference's own state layout (optimizer.mm:46-73):
 * m_pos/v_pos [3n], m_scale/v_scale [3n], m_rot/v_rot [4n], m_op/v_op [n], m_sh/v_sh [12n].
 * bc1 = 1 - beta1^t, bc2 = 1 - beta2^t (pinned: correctly rounded pow, then a float subtraction). */
void gso_adam_step(GsGaussian* g, const GsGradients* grad, uint32_t n, float* m_pos, float* m_scale,
                   float* m_rot, float* m_op, float* m_sh, float* v_pos, float* v_scale, float* v_rot,
                   float* v_op, float* v_sh, const float lrs[5], float beta1, float beta2, float eps,
                   float bc1, float bc2);
/* mtl_engine.mm:1173-1186 */
void gso_opacity_reset(GsGaussian* g, uint32_t n, float max_raw);

/* computeL1Loss / computeSSIM / computeCombinedLoss (shaders.metal:320-510) on RGBA8 images;
 * maps = [3][h][w] (L1, D-SSIM, combined); returns the mean of the combined map (fp64 sum). */
double gso_loss(const uint32_t* rendered, const uint32_t* gt, uint32_t w, uint32_t h, float lambda,
                float* maps, int threads);

#ifdef __cplusplus
}
#endif

#endif
