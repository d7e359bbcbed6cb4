// exp_probe.hip — exhaustive check of the gfx950 v_exp_f32 (2^t) against the correctly rounded
// float of 2^t (fp64 exp2 rounded to f32), over every float t in [-24, 24].
// Decides whether exp(x) := RN_f32(2^RN_f32(x * log2(e))) can be evaluated with one v_exp_f32.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdint>
#include <cstring>

__global__ void probe(uint32_t lo_bits, uint32_t count, int negative, unsigned long long* mism,
                      uint32_t* samples) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < count; i += stride) {
        uint32_t bits = lo_bits + (uint32_t)i;
        if (negative) bits |= 0x80000000u;
        const float t = __uint_as_float(bits);
        const float hw = __builtin_amdgcn_exp2f(t);
        const float ref = (float)exp2((double)t);
        if (__float_as_uint(hw) != __float_as_uint(ref)) {
            const unsigned long long k = atomicAdd(mism, 1ull);
            if (k < 16) samples[k] = bits;
        }
    }
}

int main() {
    unsigned long long* d_m;
    uint32_t* d_s;
    hipMalloc(&d_m, sizeof(unsigned long long));
    hipMalloc(&d_s, 16 * sizeof(uint32_t));
    // magnitudes from 2^-30 up to 24.0
    const uint32_t lo = 0x30800000u;  // 2^-30
    const uint32_t hi = 0x41c00000u;  // 24.0
    for (int neg = 0; neg < 2; neg++) {
        hipMemset(d_m, 0, sizeof(unsigned long long));
        hipLaunchKernelGGL(probe, dim3(8192), dim3(256), 0, 0, lo, hi - lo + 1, neg, d_m, d_s);
        unsigned long long m = 0;
        uint32_t s[16];
        hipMemcpy(&m, d_m, sizeof(m), hipMemcpyDeviceToHost);
        hipMemcpy(s, d_s, sizeof(s), hipMemcpyDeviceToHost);
        printf("%s: %u inputs, %llu mismatches\n", neg ? "negative" : "positive", hi - lo + 1, m);
        for (int k = 0; k < (m < 16 ? (int)m : 16); k++) {
            float t;
            std::memcpy(&t, &s[k], 4);
            printf("  t=%a (%.9g)\n", t, t);
        }
    }
    return 0;
}
