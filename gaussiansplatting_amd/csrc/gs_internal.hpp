// gs_internal.hpp — host-side internals shared by the kernel launchers and the C-ABI.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/gs_rasterizer.h"
#include "gs_adam.hpp"

namespace gs {

constexpr uint32_t kMaxSortBlocks = 2048;
// handle scalars (gs_capi.cpp): [0] P, [1] overflow flag, [2] scratch total, [4] the frame's fan-in
// error word (tile_finish / tile_reorder give-ups; zeroed with the overflow flag by pair emission)
constexpr uint32_t kScalarFanInError = 4;
// scalars[5]: the frame tag, incremented by the emission kernel once per forward (device-side, so a
// replayed HIP graph gets a new tag every frame). Every partial-sum slot the backward reaches
// gets the tag of its frame (PairBuffers::ptag); the chain reads the tags of a Gaussian's slots
// and only the partial sums of current ones, so slots no pixel reaches are never written (the tags
// are zeroed at allocation, and frame tags start at 1).
constexpr uint32_t kScalarFrameTag = 5;

// The backward's per-Gaussian reached tags: one byte (the frame tag's low byte). The tag is only a
// filter in front of the slots' own 32-bit tags, so a match left from 256 frames earlier costs the
// chain a read of stale slots and nothing else. (1 MB instead of 4 MB at 1M Gaussians; the
// backward's 1.9M scattered stores still write back a 32-B sector each, 55 MB per bench launch
// with bytes as with words (PMC, round 5). Without the filter the chain reads every slot of every
// emitted Gaussian: bench chain +27 us, config 5 +0.8 ms.)
using reach_t = uint8_t;

struct RadixPass {
    const void* keys_in = nullptr;      // key_bytes_in per key (u32 or u16)
    uint32_t key_bytes_in = 4, key_bytes_out = 4;
    const uint32_t* vals_in = nullptr;  // nullptr: value = element index
    const uint32_t* n_dev = nullptr;    // nullptr: use n_host
    uint32_t n_host = 0;
    uint32_t shift = 0;
    uint32_t nbits = 8;
    uint32_t nblocks = 1;
    uint32_t* hist = nullptr;    // [256][nblocks]
    bool hist_ready = false;     // hist already holds this pass's counts (the emission counted them)
    bool clear_hist = false;     // the scatter zeroes hist once it has read it
    uint32_t* totals = nullptr;  // [256]
    void* keys_out = nullptr;          // nullable; key_bytes_out per key
    uint32_t* vals_out = nullptr;
    uint32_t* inverse_out = nullptr;   // inverse_out[value] = pos
    uint2* ranges_out = nullptr;       // nullable: per key [first, last + 1) of the output (radix_scatter_kernel)
    uint32_t ranges_n = 0;             // keys < ranges_n
};

uint32_t sort_blocks_for(uint64_t n_bound);
hipError_t radix_pass(hipStream_t st, const RadixPass& p);
uint32_t scan_blocks_for(uint32_t n);
// one-pass tile sort (gs_sort.hip); scratch = tile_sort_scratch(p_bound, T) u32
constexpr uint32_t kTileSortMaxTiles = 12288;  // LDS: 12 B per tile
constexpr uint32_t kTileSortMaxBlocks = 256;  // one slice per CU (128 / 512 slices: 104 / 94 us vs 88)
constexpr uint64_t kTileSortMaxSlice = 63488;  // scatter chunk (31 x 2048): packed u16 counters fit
constexpr uint32_t kTileSortOnePassMaxPairs = 16u << 20;  // above: two-pass LSD (see gs_capi.cpp)
constexpr uint64_t kChainCompactPairsPerGaussian = 8;  // chain_impl: compacting chain above this P / N
uint32_t tile_sort_blocks(uint64_t p_bound);
uint64_t tile_sort_scratch(uint64_t p_bound, uint32_t T);
hipError_t tile_sort(hipStream_t st, const uint16_t* keys, const uint32_t* vals, const uint32_t* p_dev,
                     uint64_t p_bound, uint32_t T, uint32_t nbits, uint32_t* scratch,
                     uint32_t* vals_out, uint2* ranges, uint32_t* order /* nullable */,
                     uint32_t* chunk_base, uint32_t* tile_cost /* nullable: zeroed */,
                     uint32_t* reorder_words /* nullable: zeroed, tile_reorder_words() u32 */,
                     uint32_t* err /* the frame's fan-in error word */, bool xcd_groups,
                     uint32_t* xgroup /* nullable: per tile, the XCD group of its forward launch slot */);
// the same sort with no emitted pairs (per-tile depth sort path): the histogram and the scatter walk
// the Gaussians' rects in Gaussian order, the lists come out in any order inside a tile; the kernel
// that knows P does the emission's frame duties
constexpr uint64_t kSegPairsPerGaussian = 16;  // gs_set_depth_sort auto: per-tile sort up to this P / N
uint32_t tile_sort_gid_blocks(uint32_t n);  // slices of the own-offsets mode
hipError_t tile_sort_gid(hipStream_t st, uint32_t n, const uint32_t* count, uint32_t* goff, const uint2* rect,
                         uint32_t tiles_x, uint64_t cap, uint32_t* p_dev, uint64_t p_bound, uint32_t T,
                         uint32_t* scratch, uint32_t* vals_out, uint2* ranges, uint32_t* order, uint32_t* chunk_base,
                         uint32_t* tile_cost, uint32_t* reorder_words, uint32_t* err, bool xcd_groups,
                         uint32_t* xgroup, uint32_t* overflow, uint32_t* host_mirror, uint32_t* hist_rezero,
                         bool own_offsets /* no offsets_scan before: goff, the records' slot field and P from the
                                             scatter; only with the pair buffers at the worst case */,
                         float4* rec, uint32_t* chunk_tot /* own offsets: ceil(n / 64) words of scratch */);
// XCD-group launch order of the blend (tile_finish_kernel): the tiles are cut into kXcdGroups
// contiguous row-major runs of equal work (list length), and run x's tiles,
// longest first, take the launch slots 8k + x (blocks b and b + 8 share an XCD, so a run's tiles, and
// the splats they share, are read through one XCD's L2). A run with more tiles than its slots puts
// its last (lightest) tiles into the free slots of the runs with fewer.
constexpr uint32_t kXcdGroups = 8;
// the backward's launch order from the forward's measured per-tile work (gs_sort.hip)
uint32_t tile_reorder_words();
hipError_t tile_reorder(hipStream_t st, uint32_t T, const uint32_t* tile_cost, unsigned long long* words,
                        uint32_t* order, uint32_t* err, const uint32_t* xgroup /* nullable */);
hipError_t exclusive_scan(hipStream_t st, const uint32_t* in, const uint32_t* perm, uint32_t n,
                          uint32_t* out, uint32_t* block_sums, uint32_t* total,
                          uint32_t* overflow);
// Single-sweep depth sort (one look-back scatter per 8-bit digit; histograms from project_kernel) and the
// one-pass emission-offset scan that also marks the emission windows' owners (gs_sort.hip).
constexpr uint32_t kDepthKeyBits = 31;  // bit 31 of every emitted depth key is set
constexpr uint32_t kOsPasses = (kDepthKeyBits + 7) / 8;
// sweep scratch head: [0, kSweepHistWords) the digit histograms (built by project_kernel, zeroed by
// the emission kernel for the next frame), then 16 counter words (tickets, culled count, error)
constexpr uint32_t kSweepPasses = kOsPasses;
constexpr uint32_t kSweepHistWords = kSweepPasses * 256u;
constexpr uint32_t kSweepCtrCulled = 8;
constexpr uint32_t kSweepCtrError = 15;
constexpr uint32_t kSweepHeadWords = kSweepHistWords + 16u;
__host__ __device__ constexpr uint32_t sweep_digit_mask(uint32_t p) {
    return (1u << (p + 1u < kSweepPasses ? 8u : kDepthKeyBits - 8u * p)) - 1u;
}
uint64_t depth_sweep_words(uint32_t n_cap);
// leading words of the sweep scratch that must be zero before depth_sort_onesweep (the caller
// zeroes them: project_kernel does, in the forward)
uint32_t depth_sweep_zero_words(uint32_t n);  // words after the head that project_kernel zeroes
uint32_t depth_sweep_error_word();  // index of the sweep's error word (GsFrameStats.scan_errors)
// dsorted[r] = gid | (count - 1) << kDsortCountShift (gid < 2^24; consumers mask with kDsortGidMask)
constexpr uint32_t kDsortCountShift = 24;
constexpr uint32_t kDsortGidMask = (1u << kDsortCountShift) - 1u;
hipError_t depth_sort_onesweep(hipStream_t st, const uint32_t* dkey, const uint32_t* count, uint32_t n,
                               uint32_t* sweep, uint32_t* const kbuf[2], uint32_t* const vbuf[2],
                               uint32_t* dsorted);
// also the backward's partial-sum slots in Gaussian order: goff[gid] (and into the records' quad 3 when
// `rec` is given: the per-tile order's identity path; the global order's backward reads goff itself)
hipError_t offsets_scan(hipStream_t st, uint32_t n, const uint32_t* count, const uint32_t* dsorted,
                        uint32_t* sweep, uint32_t* offset, uint32_t* p_dev, uint32_t* wstart, uint64_t cap,
                        uint32_t* goff, float4* rec);

// Per-Gaussian raster record, 64 B = one aligned half cache line, so a blend kernel's gather of
// a splat touches one line (written by project; the last quad by pair emission):
//   rec[4i+0] = (screen x, screen y, conic.x, conic.y)
//   rec[4i+1] = (conic.z, opacity, r, g)
//   rec[4i+2] = (b, cull half-extent x, cull half-extent y, |conic|_1)
//   rec[4i+3] = (per-tile order only: the partial-sum slot base goff[i] as bits, copied by the tile
//                scatter or the offset scan -- the global order's backward reads goff[gid] instead;
//                culling-ellipse bound kq, 0, 0)
constexpr uint32_t kRecQuads = 4;

struct GaussianBuffers {
    float4* rec = nullptr;
    uint32_t* count = nullptr;  // tiles emitted (0 = not emitted)
    uint32_t* dkey = nullptr;   // sortable depth key; 0xFFFFFFFF when not emitted
    uint2* rect = nullptr;      // (min_x | min_y << 16, max_x | max_y << 16) tile rect
    uint32_t* dsort_k[2] = {nullptr, nullptr};
    uint32_t* dsort_v[2] = {nullptr, nullptr};
    uint32_t* offset = nullptr;  // first emission slot, by depth rank
    uint32_t* goff = nullptr;    // first partial-sum slot, by Gaussian index: the exclusive scan of
                                 // the tile counts in Gaussian order (offsets_scan_kernel, which
                                 // on the per-tile order mirrors it into the raster record's quad 3 .x)
    uint32_t* scan_sums = nullptr;
    uint32_t* sweep = nullptr;   // depth_sweep_words(cap): single-sweep sort / scan scratch
    reach_t* reached = nullptr;  // per Gaussian: the frame tag's low byte when the backward selected one
                                 // of its list entries (any band of any tile); the chain skips the
                                 // others (all their slots are stale). Zeroed at allocation.
    uint32_t* chain_list = nullptr;    // compacting chain: per 256-Gaussian block the listed Gaussians
    uint32_t* chain_lcount = nullptr;  // ... and their number (gs_chain.hip chain_screen_kernel)
    size_t cap = 0;
};

// A pair's value is packed as (gid << 8) | j: the Gaussian index (< 2^24) and the pair's index j
// (< 256) inside the Gaussian's row-major tile rect. Its emission slot is goff[gid] + j, where the
// backward stores the pair's 9 partial sums; the chain then reads each Gaussian's slots contiguously.
constexpr uint32_t kPairJBits = 8;
constexpr uint32_t kPairJMask = (1u << kPairJBits) - 1u;

// A partial-sum slot: the 9 sums and the slot's frame tag as a 10th word. The backward writes a
// reached slot as one 40-B run (two 32-B sectors at any slot index) instead of 36 B of sums plus a
// 4-B tag in its own array, whose scattered stores each wrote back a sector of their own (56 MB per
// bench launch for 7.6 MB of tags, PMC, round 5); the chain reads the tag with the sums.
constexpr uint32_t kSlotWords = 10u;

struct PairBuffers {
    uint32_t* tile0 = nullptr;  // emission order tile key (sort ping-pong A)
    uint32_t* val0 = nullptr;   // emission order packed value
    uint32_t* tile1 = nullptr;  // sort ping-pong B
    uint32_t* val1 = nullptr;
    uint32_t* s_tile = nullptr;  // sorted tile key
    uint32_t* s_val = nullptr;   // sorted packed value (gid = s_val >> 8: the reference's values)
    float* partial = nullptr;    // [slot][kSlotWords] backward partial sums per (tile, Gaussian) and
                                 // the frame tag (kScalarFrameTag) of the frame that wrote them
    float* ptag_zero = nullptr;  // 16 zero floats: what the chain reads for a stale slot
    uint32_t* wstart = nullptr;  // [cap / kEmitWin + 2] depth rank owning each emission window's first slot
    uint64_t cap = 0;
};

struct PixelBuffers {
    uint32_t* last_idx = nullptr;
    float* t_final = nullptr;
    uint64_t cap = 0;
};

struct LaunchGeom {
    uint32_t w = 0, h = 0, tiles_x = 0, tiles_y = 0, num_tiles = 0;
    const uint32_t* tile_order = nullptr;  // blend launch order (heaviest tiles first), or null
    const uint32_t* bwd_order = nullptr;   // backward launch order (by the forward's measured work), or null
    uint32_t* tile_cost = nullptr;         // per tile: blend steps of the forward (written by it)
    const uint32_t* xgroup = nullptr;      // per tile: XCD group of the forward's launch slot, or null
    // Band cull masks handed from the forward to the backward: for list chunk c (64 entries from
    // the tile's range start) of tile t, band_mask[(chunk_base[t] + c) * 4 + band] is the forward
    // wave's culling ballot for its 8x8 band (the backward's per-band test is the same test).
    const uint32_t* chunk_base = nullptr;  // exclusive scan over tiles of ceil(len / 64)
    uint64_t* band_mask = nullptr;
    const uint32_t* frame_tag = nullptr;   // the frame's partial-slot tag (scalars[kScalarFrameTag])
    // per-tile depth order sorted by the forward itself: the depth keys, or null (the lists arrive
    // sorted). Lists above kFwdSortMax entries are sorted before the forward.
    const uint32_t* fwd_sort_dkey = nullptr;
    bool goff_direct = false;  // the backward reads goff[gid] (global order: no slot-base copy in the records)
    // backward list split (gs_blend.hip): the first split_tiles tiles of the backward's order run as
    // a back-part and a front-quarter wave, the per-pixel state handed over in split_state
    // (kSplitStateWords u64 per split tile) and flagged with the frame tag (cleared by the consumer)
    uint32_t split_tiles = 0;
    unsigned long long* split_state = nullptr;
    uint32_t* split_err = nullptr;          // the frame's fan-in error word (a give-up spin sets a bit)
    // work counters (GsFrameStats walked entries): [tile * 4 + band] the list entries the forward's band
    // wave read, [4 T + tile] those the backward read (plain stores: a repeated pass writes the same)
    uint32_t* walk = nullptr;
};
constexpr uint32_t kSplitStateWords = 8u * 64u;  // 4 bands x (T, accumulated-colour sum) per lane

// kernel launchers (gs_raster.hip)
hipError_t launch_project(hipStream_t st, const GsGaussian* g, uint32_t n,
                          const GsTiledUniforms& u, const GaussianBuffers& gb,
                          GsProjected* debug_out, uint32_t* zero_words = nullptr, uint32_t nzero = 0,
                          uint32_t* hist = nullptr);
constexpr uint32_t kProjectThreads = 1024;  // project_kernel block (few blocks: few histogram atomics)
// emission window (slots) of emit_slots_kernel, a multiple of 256 (config 5: 2048 -> 229, 1024 -> 209,
// 512 -> 239 us per frame, scripts/ab_cfg5.sh)
constexpr uint32_t kEmitWin = 1024;
static_assert(kEmitWin % 256u == 0u && kEmitWin >= 256u, "emit_slots_kernel: slots per thread");
hipError_t launch_emit(hipStream_t st, uint32_t n, const GaussianBuffers& gb,
                       const uint32_t* dsorted, const PairBuffers& pb, uint32_t tiles_x,
                       const uint32_t* p_dev, uint64_t p_bound, uint32_t* overflow,
                       bool wstart_ready, uint32_t* host_mirror, uint32_t* hist_rezero, bool key16,
                       uint32_t* lsd_hist = nullptr, uint32_t lsd_blocks = 0, uint32_t lsd_mask = 0);
hipError_t launch_chunk_base(hipStream_t st, uint2* ranges, uint32_t num_tiles,
                             uint32_t* chunk_base, uint32_t* tile_cost = nullptr,
                             unsigned long long* reorder_words = nullptr, uint32_t nreorder = 0,
                             bool fill_empty = false, uint32_t* order = nullptr);  // order: + tile_order's job
hipError_t launch_ranges(hipStream_t st, const uint32_t* s_tile, const uint32_t* p_dev,
                         uint64_t p_bound, uint32_t num_tiles, uint2* ranges);
hipError_t launch_forward(hipStream_t st, const LaunchGeom& geo, const GsTiledUniforms& u,
                          const GaussianBuffers& gb, const PairBuffers& pb, const uint2* ranges,
                          const uint32_t* p_dev, const PixelBuffers& px, uint32_t* rgba8,
                          float* rgb);
hipError_t launch_backward(hipStream_t st, const LaunchGeom& geo, const GsTiledUniforms& u,
                           const GaussianBuffers& gb, const PairBuffers& pb,
                           const uint2* ranges, const PixelBuffers& px, const uint32_t* rendered,
                           const uint32_t* gt);
// gs_backward_step: the chain kernel hands each Gaussian's gradient straight to the density
// statistics (nullable accum) and to Adam on the Gaussian itself, instead of writing gradient rows
struct ChainStep {
    GsGaussian* g = nullptr;  // the Gaussians the chain reads (updated in place by Adam)
    float* accum = nullptr;
    uint32_t* dcount = nullptr;
    float* pos_accum = nullptr;
    float4* m = nullptr;
    float4* v = nullptr;
    AdamParams P = {};
};
AdamParams make_adam_params(const float lrs[5], float beta1, float beta2, float eps, float clip, float bc1,
                            float bc2);
hipError_t launch_chain(hipStream_t st, const GsGaussian* g, uint32_t n,
                        const GsTiledUniforms& u, const GaussianBuffers& gb,
                        const PairBuffers& pb, GsGradients* grad, float* rows, float* viewspace,
                        uint32_t first, uint32_t count, const uint32_t* frame_tag, bool compact,
                        const ChainStep* step = nullptr, bool list_dense = false);
// per-tile depth sort of the tile lists longer than the forward sorts itself (gs_segsort.hip): each
// such list, in any order, -> (depth, gid) order, in place in s_val; lists above 4096 entries are
// first cut by an MSD bucket split into `scratch` (pair capacity). (ka, va), (kb, vb): pair-capacity
// ping-pong of the LSD passes (segments above 4096 entries, or of nearly equal depths).
constexpr uint32_t kFwdSortMax = 1024;  // lists the forward sorts itself (gs_blend.hip kFwdSortCap)
hipError_t launch_tile_depth_sort(hipStream_t st, const uint2* ranges, uint32_t T, const uint32_t* dkey,
                                  uint32_t* s_val, uint32_t* ka, uint32_t* va, uint32_t* kb, uint32_t* vb,
                                  uint32_t* scratch);
hipError_t launch_half_exp_check(hipStream_t st, uint32_t* d_out);
hipError_t launch_float_exp_check(hipStream_t st, uint32_t* d_out);
hipError_t launch_unpack(hipStream_t st, const float* rows, const float* viewspace, uint32_t n,
                         GsGradients* grad);
constexpr uint32_t kGradRowFloats = GS_GRAD_ROW_FLOATS;  // gradient rows (gs_rasterizer.h)
hipError_t launch_debug_pairs(hipStream_t st, const PairBuffers& pb, const GaussianBuffers& gb,
                              const uint2* ranges, uint32_t num_tiles, const uint32_t* p_dev,
                              uint64_t cap, uint64_t* keys, uint32_t* values);
hipError_t launch_debug_ranges(hipStream_t st, const uint2* ranges, uint32_t num_tiles,
                               GsTileRange* out);

}  // namespace gs
