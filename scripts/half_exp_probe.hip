// half_exp_probe.hip — exhaustive check, over every half power the forward blend can see
// (all 16-bit halves in [-4.5, 0]), of the hardware exp2 path the forward uses for the half weight
// (v_exp_f32(float(h) * log2 e)) against the pinned gs_expf_core(float(h)): the largest ulp
// distance, and for each tie window W the number of half-rounding mismatches the window misses.
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -std=c++17 -o scripts/half_exp_probe scripts/half_exp_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>

#include "../gaussiansplatting_amd/csrc/gs_device.hpp"

constexpr int kMaxW = 17;

__global__ void probe(unsigned int* maxd, unsigned int* mism, unsigned int* missed) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= 65536u) return;
    const _Float16 h = __builtin_bit_cast(_Float16, (uint16_t)i);
    if (!(h <= (_Float16)0.0f && h >= (_Float16)-4.5f)) return;
    const float pf = (float)h;
    const float hw = __builtin_amdgcn_exp2f(pf * 1.44269504f);
    const float pin = gs::gs_expf_core(pf);
    const int32_t d = (int32_t)__float_as_uint(hw) - (int32_t)__float_as_uint(pin);
    atomicMax(maxd, (uint32_t)(d < 0 ? -d : d));
    if (__builtin_bit_cast(uint16_t, (_Float16)hw) != __builtin_bit_cast(uint16_t, (_Float16)pin)) {
        atomicAdd(mism, 1u);
        const uint32_t low = __float_as_uint(hw) & 0x1fffu;
        for (int w = 0; w < kMaxW; w++)
            if (!(low - (0x1000u - (uint32_t)w) <= 2u * (uint32_t)w)) atomicAdd(&missed[w], 1u);
    }
}

int main() {
    unsigned int* d;
    hipMalloc(&d, (2 + kMaxW) * sizeof(unsigned int));
    hipMemset(d, 0, (2 + kMaxW) * sizeof(unsigned int));
    hipLaunchKernelGGL(probe, dim3(256), dim3(256), 0, 0, d, d + 1, d + 2);
    unsigned int h[2 + kMaxW];
    hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    printf("max ulp distance hw vs pinned: %u; half-rounding mismatches: %u\n", h[0], h[1]);
    for (int w = 0; w < kMaxW; w++) printf("window %2d: %u mismatches outside the window\n", w, h[2 + w]);
    return 0;
}
