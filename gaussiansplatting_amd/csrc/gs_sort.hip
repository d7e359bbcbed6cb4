// gs_sort.hip — stable LSD radix sort of 32-bit keys (with a 32-bit payload) and a
// device-wide exclusive scan, both driven by a device-resident element count so the
// frame never has to read P back to the host.
//
// The (tile | depth) 64-bit key order of the reference (tiled_rasterizer.mm:27-102, a CPU
// 8x8-bit LSD sort over pair<u64,u32>) is produced in two stages:
//   1. the 31 significant depth-key bits are sorted once over the N Gaussians;
//   2. pairs are emitted in that depth order, and a stable LSD pass over only the
//      ceil(log2(T)) tile bits orders them by tile.
// Stability of both stages gives exactly the order (tile, depth key, Gaussian index).
//
// One pass = hist (per-block digit counts) -> digit_scan (per digit over blocks) -> scatter
// (wave-level multisplit ranking, stable). Blocks own contiguous slices; the slice size is
// derived on the device from the element count, so a fixed grid serves any P.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "gs_device.hpp"
#include "gs_internal.hpp"

namespace gs {

constexpr int kSortThreads = 256;
constexpr int kSortItems = 8;
constexpr uint32_t kSortTile = kSortThreads * kSortItems;  // 2048 elements per block step
constexpr int kSortWaves = kSortThreads / 64;

__device__ __forceinline__ uint32_t sort_count(const uint32_t* n_dev, uint32_t n_host) {
    return n_dev ? *n_dev : n_host;
}

// Slice of block b: [b*S, min((b+1)*S, n)), S = ceil(n / B) rounded up to kSortTile.
__device__ __forceinline__ void sort_slice(uint32_t n, uint32_t b, uint32_t nblocks,
                                           uint32_t& begin, uint32_t& end) {
    uint32_t per = (n + nblocks - 1u) / nblocks;
    per = (per + kSortTile - 1u) / kSortTile * kSortTile;
    const uint64_t b0 = (uint64_t)per * b;
    begin = b0 < n ? (uint32_t)b0 : n;
    const uint64_t e0 = b0 + per;
    end = e0 < n ? (uint32_t)e0 : n;
}

__global__ __launch_bounds__(kSortThreads) void radix_hist_kernel(
    const uint32_t* __restrict__ keys, const uint32_t* n_dev, uint32_t n_host, uint32_t shift,
    uint32_t mask, uint32_t* __restrict__ hist /* [256][nblocks] */) {
    __shared__ uint32_t h[kSortWaves][256];
    const uint32_t t = threadIdx.x, w = t >> 6;
    for (uint32_t i = t; i < kSortWaves * 256; i += kSortThreads) (&h[0][0])[i] = 0u;
    __syncthreads();
    const uint32_t n = sort_count(n_dev, n_host);
    uint32_t begin, end;
    sort_slice(n, blockIdx.x, gridDim.x, begin, end);
    for (uint32_t i = begin + t; i < end; i += kSortThreads) {
        const uint32_t d = (keys[i] >> shift) & mask;
        atomicAdd(&h[w][d], 1u);
    }
    __syncthreads();
    const uint32_t s = h[0][t] + h[1][t] + h[2][t] + h[3][t];
    hist[t * gridDim.x + blockIdx.x] = s;
}

// One block per digit: exclusive scan of hist[d][0..B) in place; totals[d] = row sum.
__global__ __launch_bounds__(256) void radix_digit_scan_kernel(uint32_t* __restrict__ hist,
                                                                uint32_t nblocks,
                                                                uint32_t* __restrict__ totals) {
    __shared__ uint32_t part[256];
    const uint32_t d = blockIdx.x, t = threadIdx.x;
    uint32_t* row = hist + (size_t)d * nblocks;
    const uint32_t per = (nblocks + 255u) / 256u;
    const uint32_t b0 = t * per;
    uint32_t s = 0;
    for (uint32_t k = 0; k < per; k++)
        if (b0 + k < nblocks) s += row[b0 + k];
    part[t] = s;
    __syncthreads();
    // Hillis-Steele inclusive scan of the 256 partials
    for (uint32_t o = 1; o < 256; o <<= 1) {
        const uint32_t v = t >= o ? part[t - o] : 0u;
        __syncthreads();
        part[t] += v;
        __syncthreads();
    }
    uint32_t run = t ? part[t - 1] : 0u;
    for (uint32_t k = 0; k < per; k++)
        if (b0 + k < nblocks) {
            const uint32_t c = row[b0 + k];
            row[b0 + k] = run;
            run += c;
        }
    if (t == 255) totals[d] = part[255];
}

// Stable scatter. Element order inside a block step is (wave, item, lane), which is the
// memory order, so ranks computed by wave ballots + per-wave counters are stable. Each 2048-element
// step is first reordered by digit in LDS, then written out so that consecutive lanes store
// consecutive positions of a digit run (coalesced) instead of 64 scattered buckets per instruction.
__global__ __launch_bounds__(kSortThreads) void radix_scatter_kernel(
    const uint32_t* __restrict__ keys_in, const uint32_t* __restrict__ vals_in,
    const uint32_t* n_dev, uint32_t n_host, uint32_t shift, uint32_t nbits,
    const uint32_t* __restrict__ hist, const uint32_t* __restrict__ totals,
    uint32_t* __restrict__ keys_out, uint32_t* __restrict__ vals_out,
    uint32_t* __restrict__ inverse_out) {
    __shared__ uint32_t s_off[256];               // running global start of each digit
    __shared__ uint32_t s_cnt[kSortWaves][256];   // per-wave counts -> per-wave local offsets
    __shared__ uint32_t s_loc[256];               // block-local start of each digit in the step
    __shared__ uint32_t s_key[kSortTile];
    __shared__ uint32_t s_val[kSortTile];
    const uint32_t t = threadIdx.x, w = t >> 6, lane = t & 63u;
    const uint32_t mask = (1u << nbits) - 1u;

    // digit bases: exclusive scan of totals
    s_loc[t] = totals[t];
    __syncthreads();
    for (uint32_t o = 1; o < 256; o <<= 1) {
        const uint32_t v = t >= o ? s_loc[t - o] : 0u;
        __syncthreads();
        s_loc[t] += v;
        __syncthreads();
    }
    const uint32_t base = t ? s_loc[t - 1] : 0u;
    s_off[t] = base + hist[t * gridDim.x + blockIdx.x];
    __syncthreads();

    const uint32_t n = sort_count(n_dev, n_host);
    uint32_t begin, end;
    sort_slice(n, blockIdx.x, gridDim.x, begin, end);
    const uint64_t lt = lanemask_lt();

    for (uint32_t step = begin; step < end; step += kSortTile) {
        uint32_t k[kSortItems], v[kSortItems], dg[kSortItems], rk[kSortItems];
        bool ok[kSortItems];
#pragma unroll
        for (int i = 0; i < kSortItems; i++) {
            const uint32_t idx = step + w * (kSortItems * 64u) + (uint32_t)i * 64u + lane;
            ok[i] = idx < end;
            k[i] = ok[i] ? keys_in[idx] : 0u;
            v[i] = vals_in ? (ok[i] ? vals_in[idx] : 0u) : idx;
            dg[i] = (k[i] >> shift) & mask;
        }
#pragma unroll
        for (int j = 0; j < 4; j++) s_cnt[w][lane + 64u * j] = 0u;
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int i = 0; i < kSortItems; i++) {
            uint64_t m = __ballot(ok[i]);
            for (uint32_t bit = 0; bit < nbits; bit++) {
                const bool on = (dg[i] >> bit) & 1u;
                const uint64_t bb = __ballot(on);
                m &= on ? bb : ~bb;
            }
            const uint32_t below = (uint32_t)__popcll(m & lt);
            uint32_t c = 0;
            if (ok[i]) c = s_cnt[w][dg[i]];
            __builtin_amdgcn_wave_barrier();
            rk[i] = c + below;
            const uint32_t leader = 63u - (uint32_t)__clzll(m);
            if (ok[i] && lane == leader) s_cnt[w][dg[i]] = c + (uint32_t)__popcll(m);
            __builtin_amdgcn_wave_barrier();
        }
        __syncthreads();
        // per digit (thread t = digit): wave offsets within the digit, digit total of the step
        uint32_t tot = 0;
#pragma unroll
        for (int ww = 0; ww < kSortWaves; ww++) {
            const uint32_t c = s_cnt[ww][t];
            s_cnt[ww][t] = tot;
            tot += c;
        }
        // block-local exclusive scan of the digit totals -> s_loc
        s_loc[t] = tot;
        __syncthreads();
        for (uint32_t o = 1; o < 256; o <<= 1) {
            const uint32_t x = t >= o ? s_loc[t - o] : 0u;
            __syncthreads();
            s_loc[t] += x;
            __syncthreads();
        }
        const uint32_t loc_start = s_loc[t] - tot;
        __syncthreads();
        s_loc[t] = loc_start;
        __syncthreads();
        // reorder the step by digit in LDS
#pragma unroll
        for (int i = 0; i < kSortItems; i++) {
            if (!ok[i]) continue;
            const uint32_t lp = s_loc[dg[i]] + s_cnt[w][dg[i]] + rk[i];
            s_key[lp] = k[i];
            s_val[lp] = v[i];
        }
        __syncthreads();
        const uint32_t cnt = min(kSortTile, end - step);
        for (uint32_t i = t; i < cnt; i += kSortThreads) {
            const uint32_t kk = s_key[i], vv = s_val[i];
            const uint32_t d = (kk >> shift) & mask;
            const uint32_t pos = s_off[d] + (i - s_loc[d]);
            if (keys_out) keys_out[pos] = kk;
            if (vals_out) vals_out[pos] = vv;
            if (inverse_out) inverse_out[vv] = pos;
        }
        __syncthreads();
        s_off[t] += tot;
        __syncthreads();
    }
}


// ---- device-wide exclusive scan of u32 (optionally gathered through a permutation) ------
constexpr int kScanThreads = 256;
constexpr int kScanItems = 8;
constexpr uint32_t kScanTile = kScanThreads * kScanItems;

__device__ __forceinline__ uint32_t scan_load(const uint32_t* __restrict__ in,
                                              const uint32_t* __restrict__ perm, uint32_t i) {
    return perm ? in[perm[i]] : in[i];
}

__global__ __launch_bounds__(kScanThreads) void scan_reduce_kernel(
    const uint32_t* __restrict__ in, const uint32_t* __restrict__ perm, uint32_t n,
    uint32_t* __restrict__ block_sums) {
    __shared__ uint32_t ws[kScanThreads / 64];
    const uint32_t base = blockIdx.x * kScanTile;
    uint32_t s = 0;
#pragma unroll
    for (int i = 0; i < kScanItems; i++) {
        const uint32_t idx = base + (uint32_t)i * kScanThreads + threadIdx.x;
        if (idx < n) s += scan_load(in, perm, idx);
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) s += __shfl_xor(s, o, 64);
    if ((threadIdx.x & 63u) == 0) ws[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) block_sums[blockIdx.x] = ws[0] + ws[1] + ws[2] + ws[3];
}

// Single block: exclusive scan of block sums; writes the grand total (u32, saturating flag).
__global__ __launch_bounds__(1024) void scan_block_sums_kernel(uint32_t* __restrict__ sums,
                                                                uint32_t nb,
                                                                uint32_t* __restrict__ total,
                                                                uint32_t* __restrict__ overflow) {
    __shared__ uint32_t part[1024];
    const uint32_t t = threadIdx.x;
    const uint32_t per = (nb + 1023u) / 1024u;
    const uint32_t b0 = t * per;
    uint64_t s = 0;
    for (uint32_t k = 0; k < per; k++)
        if (b0 + k < nb) s += sums[b0 + k];
    part[t] = (uint32_t)s;
    __syncthreads();
    for (uint32_t o = 1; o < 1024; o <<= 1) {
        const uint32_t v = t >= o ? part[t - o] : 0u;
        __syncthreads();
        part[t] += v;
        __syncthreads();
    }
    uint64_t run = t ? part[t - 1] : 0u;
    for (uint32_t k = 0; k < per; k++)
        if (b0 + k < nb) {
            const uint32_t c = sums[b0 + k];
            sums[b0 + k] = (uint32_t)run;
            run += c;
        }
    if (t == 1023) {
        *total = part[1023];
        if (overflow) *overflow = 0u;
    }
}

__global__ __launch_bounds__(kScanThreads) void scan_final_kernel(
    const uint32_t* __restrict__ in, const uint32_t* __restrict__ perm, uint32_t n,
    const uint32_t* __restrict__ block_offsets, uint32_t* __restrict__ out) {
    __shared__ uint32_t ws[kScanThreads / 64];
    // blocked arrangement: thread t owns items [t*8, t*8+8) of the tile
    const uint32_t base = blockIdx.x * kScanTile + threadIdx.x * kScanItems;
    uint32_t v[kScanItems];
    uint32_t s = 0;
#pragma unroll
    for (int i = 0; i < kScanItems; i++) {
        const uint32_t idx = base + (uint32_t)i;
        v[i] = idx < n ? scan_load(in, perm, idx) : 0u;
        s += v[i];
    }
    // wave inclusive scan of per-thread sums
    const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
    uint32_t inc = s;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(inc, o, 64);
        if (lane >= (uint32_t)o) inc += y;
    }
    if (lane == 63u) ws[w] = inc;
    __syncthreads();
    uint32_t wo = 0;
    for (uint32_t k = 0; k < w; k++) wo += ws[k];
    uint32_t run = block_offsets[blockIdx.x] + wo + inc - s;
#pragma unroll
    for (int i = 0; i < kScanItems; i++) {
        const uint32_t idx = base + (uint32_t)i;
        if (idx < n) out[idx] = run;
        run += v[i];
    }
}

// ---- host launchers -----------------------------------------------------------------

uint32_t sort_blocks_for(uint64_t n_bound) {
    uint64_t b = (n_bound + kSortTile - 1) / kSortTile;
    if (b < 1) b = 1;
    if (b > kMaxSortBlocks) b = kMaxSortBlocks;
    return (uint32_t)b;
}

hipError_t radix_pass(hipStream_t st, const RadixPass& p) {
    const uint32_t B = p.nblocks;
    hipLaunchKernelGGL(radix_hist_kernel, dim3(B), dim3(kSortThreads), 0, st, p.keys_in, p.n_dev,
                       p.n_host, p.shift, (1u << p.nbits) - 1u, p.hist);
    hipLaunchKernelGGL(radix_digit_scan_kernel, dim3(256), dim3(256), 0, st, p.hist, B, p.totals);
    hipLaunchKernelGGL(radix_scatter_kernel, dim3(B), dim3(kSortThreads), 0, st, p.keys_in,
                       p.vals_in, p.n_dev, p.n_host, p.shift, p.nbits, p.hist, p.totals,
                       p.keys_out, p.vals_out, p.inverse_out);
    return hipGetLastError();
}

uint32_t scan_blocks_for(uint32_t n) { return (n + kScanTile - 1) / kScanTile; }

hipError_t exclusive_scan(hipStream_t st, const uint32_t* in, const uint32_t* perm, uint32_t n,
                          uint32_t* out, uint32_t* block_sums, uint32_t* total,
                          uint32_t* overflow) {
    const uint32_t nb = scan_blocks_for(n);
    if (nb == 0) {
        return hipMemsetAsync(total, 0, sizeof(uint32_t), st);
    }
    hipLaunchKernelGGL(scan_reduce_kernel, dim3(nb), dim3(kScanThreads), 0, st, in, perm, n,
                       block_sums);
    hipLaunchKernelGGL(scan_block_sums_kernel, dim3(1), dim3(1024), 0, st, block_sums, nb, total,
                       overflow);
    hipLaunchKernelGGL(scan_final_kernel, dim3(nb), dim3(kScanThreads), 0, st, in, perm, n,
                       block_sums, out);
    return hipGetLastError();
}

}  // namespace gs
