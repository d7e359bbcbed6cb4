// gs_membw.hip — the measured HBM copy roofline the bench reports next to the 8 TB/s spec
// ("also report a measured device-copy bandwidth").
//
// A streaming read + write of 16 B per lane: every thread copies kUnroll float4s per grid-stride
// round, all loads issued before the stores, so each wave keeps kUnroll x 1 KiB of reads in flight.
// The buffers are sized well past the 256 MiB Infinity Cache (MI355X_MICROARCH.md "Infinity Cache"),
// so every byte comes from and goes to HBM. Variants: plain loads/stores, or non-temporal ones (the
// stream is touched once); grid sizes of 1-8 workgroups per CU. gs_debug_copy_bandwidth reports the
// best (the guide measures 6.29 TB/s for a float4 copy; round 5 reported a torch copy_ at 4.8-5.0).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "../../include/gs_rasterizer.h"

namespace gs {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));  // (the non-temporal builtins take native vectors)

template <int kUnroll, bool kNt>
__global__ __launch_bounds__(256) void copy_stream_kernel(const u32x4* __restrict__ src, u32x4* __restrict__ dst,
                                                          uint64_t n16) {
    const uint64_t stride = (uint64_t)gridDim.x * 256u;
    uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x;
    for (; i + (kUnroll - 1) * stride < n16; i += kUnroll * stride) {
        u32x4 v[kUnroll];
#pragma unroll
        for (int k = 0; k < kUnroll; k++)
            v[k] = kNt ? __builtin_nontemporal_load(src + i + k * stride) : src[i + k * stride];
#pragma unroll
        for (int k = 0; k < kUnroll; k++) {
            if (kNt)
                __builtin_nontemporal_store(v[k], dst + i + k * stride);
            else
                dst[i + k * stride] = v[k];
        }
    }
    for (; i < n16; i += stride) dst[i] = src[i];
}

}  // namespace gs

using namespace gs;

extern "C" int gs_debug_copy_bandwidth(int device, uint64_t bytes, int reps, double* gbs_out, double* variants_out,
                                       int max_variants) {
    if (!gbs_out || reps <= 0 || bytes < (1u << 20)) return GS_E_INVALID;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev) return GS_E_INVALID;
    if (hipSetDevice(device) != hipSuccess) return GS_E_HIP;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) != hipSuccess) return GS_E_HIP;
    const uint64_t n16 = bytes / 16u;
    u32x4 *a = nullptr, *b = nullptr;
    if (hipMalloc(&a, n16 * 16u) != hipSuccess) return GS_E_NOMEM;
    if (hipMalloc(&b, n16 * 16u) != hipSuccess) {
        (void)hipFree(a);
        return GS_E_NOMEM;
    }
    hipEvent_t e0 = nullptr, e1 = nullptr;
    int rc = GS_OK;
    double best = 0.0;
    int nv = 0;
    if (hipMemset(a, 1, n16 * 16u) != hipSuccess || hipEventCreate(&e0) != hipSuccess ||
        hipEventCreate(&e1) != hipSuccess)
        rc = GS_E_HIP;
    const uint32_t cus = (uint32_t)std::max(prop.multiProcessorCount, 1);
    for (int nt = 0; nt < 2 && rc == GS_OK; nt++) {
        for (uint32_t per_cu : {1u, 2u, 4u, 8u}) {
            const uint32_t grid = cus * per_cu;
            auto launch = [&]() {
                if (nt)
                    hipLaunchKernelGGL((copy_stream_kernel<4, true>), dim3(grid), dim3(256), 0, nullptr, a, b, n16);
                else
                    hipLaunchKernelGGL((copy_stream_kernel<4, false>), dim3(grid), dim3(256), 0, nullptr, a, b, n16);
            };
            launch();  // warm
            (void)hipEventRecord(e0, nullptr);
            for (int r = 0; r < reps; r++) launch();
            (void)hipEventRecord(e1, nullptr);
            float ms = 0.0f;
            if (hipGetLastError() != hipSuccess || hipEventSynchronize(e1) != hipSuccess ||
                hipEventElapsedTime(&ms, e0, e1) != hipSuccess || ms <= 0.0f) {
                rc = GS_E_HIP;
                break;
            }
            const double gbs = 2.0 * (double)(n16 * 16u) * reps / (ms * 1e-3) / 1e9;  // read + write
            if (variants_out && nv < max_variants) variants_out[nv] = gbs;
            nv++;
            best = std::max(best, gbs);
        }
    }
    if (e0) (void)hipEventDestroy(e0);
    if (e1) (void)hipEventDestroy(e1);
    (void)hipFree(a);
    (void)hipFree(b);
    if (rc == GS_OK) *gbs_out = best;
    return rc;
}
