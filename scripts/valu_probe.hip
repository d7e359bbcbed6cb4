// VALU issue-cost probe on gfx950: independent FMA chains, scalar f32 vs packed f32 vs packed f16.
// Prints ns per wave-instruction per SIMD for each flavour (1024 SIMDs, 8 waves each).
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f2 __attribute__((ext_vector_type(2)));
typedef _Float16 h2 __attribute__((ext_vector_type(2)));
constexpr int kIters = 4096, kAcc = 8;

__global__ __launch_bounds__(64) void k_fma(float* out, float b, float c) {
    float a[kAcc];
    for (int i = 0; i < kAcc; i++) a[i] = threadIdx.x + i;
    for (int it = 0; it < kIters; it++)
#pragma unroll
        for (int i = 0; i < kAcc; i++) a[i] = __builtin_fmaf(a[i], b, c);
    float s = 0; for (int i = 0; i < kAcc; i++) s += a[i];
    out[blockIdx.x * 64 + threadIdx.x] = s;
}
__global__ __launch_bounds__(64) void k_mul(float* out, float b, float c) {
    float a[kAcc];
    for (int i = 0; i < kAcc; i++) a[i] = threadIdx.x + i;
    for (int it = 0; it < kIters; it++)
#pragma unroll
        for (int i = 0; i < kAcc; i++) a[i] = a[i] * b;
    float s = 0; for (int i = 0; i < kAcc; i++) s += a[i];
    out[blockIdx.x * 64 + threadIdx.x] = s + c;
}
__global__ __launch_bounds__(64) void k_pkfma(float* out, float b, float c) {
    f2 a[kAcc];
    for (int i = 0; i < kAcc; i++) { a[i].x = threadIdx.x + i; a[i].y = i; }
    const f2 bb = (f2)(b), cc = (f2)(c);
    for (int it = 0; it < kIters; it++)
#pragma unroll
        for (int i = 0; i < kAcc; i++) a[i] = __builtin_elementwise_fma(a[i], bb, cc);
    float s = 0; for (int i = 0; i < kAcc; i++) s += a[i].x + a[i].y;
    out[blockIdx.x * 64 + threadIdx.x] = s;
}
__global__ __launch_bounds__(64) void k_pkmul(float* out, float b, float c) {
    f2 a[kAcc];
    for (int i = 0; i < kAcc; i++) { a[i].x = threadIdx.x + i; a[i].y = i; }
    f2 bb; bb.x = b; bb.y = c;
    for (int it = 0; it < kIters; it++)
#pragma unroll
        for (int i = 0; i < kAcc; i++) a[i] = a[i] * bb;
    float s = 0; for (int i = 0; i < kAcc; i++) s += a[i].x + a[i].y;
    out[blockIdx.x * 64 + threadIdx.x] = s;
}
__global__ __launch_bounds__(64) void k_pkh(float* out, float b, float c) {
    h2 a[kAcc];
    for (int i = 0; i < kAcc; i++) { a[i].x = (_Float16)(threadIdx.x + i); a[i].y = (_Float16)i; }
    const h2 bb = (h2)((_Float16)b), cc = (h2)((_Float16)c);
    for (int it = 0; it < kIters; it++)
#pragma unroll
        for (int i = 0; i < kAcc; i++) a[i] = a[i] * bb + cc;
    float s = 0; for (int i = 0; i < kAcc; i++) s += (float)a[i].x + (float)a[i].y;
    out[blockIdx.x * 64 + threadIdx.x] = s;
}

__global__ __launch_bounds__(64) void k_exp(float* out, float b, float c) {
    float a[kAcc];
    for (int i = 0; i < kAcc; i++) a[i] = (threadIdx.x + i) * 1e-3f;
    for (int it = 0; it < kIters; it++)
#pragma unroll
        for (int i = 0; i < kAcc; i++) a[i] = __builtin_amdgcn_exp2f(a[i]);
    float s = 0; for (int i = 0; i < kAcc; i++) s += a[i];
    out[blockIdx.x * 64 + threadIdx.x] = s + b + c;
}
__global__ __launch_bounds__(64) void k_rcp(float* out, float b, float c) {
    float a[kAcc];
    for (int i = 0; i < kAcc; i++) a[i] = 1.0f + (threadIdx.x + i) * 1e-3f;
    for (int it = 0; it < kIters; it++)
#pragma unroll
        for (int i = 0; i < kAcc; i++) a[i] = __builtin_amdgcn_rcpf(a[i]);
    float s = 0; for (int i = 0; i < kAcc; i++) s += a[i];
    out[blockIdx.x * 64 + threadIdx.x] = s + b + c;
}
// half the instructions are v_exp_f32, half v_fma_f32 (independent)
__global__ __launch_bounds__(64) void k_mix(float* out, float b, float c) {
    float a[kAcc], e[kAcc];
    for (int i = 0; i < kAcc; i++) { a[i] = threadIdx.x + i; e[i] = (threadIdx.x + i) * 1e-3f; }
    for (int it = 0; it < kIters; it++)
#pragma unroll
        for (int i = 0; i < kAcc; i++) { a[i] = __builtin_fmaf(a[i], b, c); e[i] = __builtin_amdgcn_exp2f(e[i]); }
    float s = 0; for (int i = 0; i < kAcc; i++) s += a[i] + e[i];
    out[blockIdx.x * 64 + threadIdx.x] = s;
}
template <typename K>
static void run(const char* name, K kern, float* d, int blocks, double instr_per_wave_iter) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(64), 0, 0, d, 0.999f, 0.001f);
    hipEventRecord(e0);
    for (int r = 0; r < 5; r++) hipLaunchKernelGGL(kern, dim3(blocks), dim3(64), 0, 0, d, 0.999f, 0.001f);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    const double waves = 5.0 * blocks;
    const double instr = waves * kIters * instr_per_wave_iter;
    printf("%-8s %8.3f ms  %.3f ns per wave-instr per SIMD (1024 SIMDs)\n", name, ms,
           ms * 1e6 * 1024 / instr);
}

int main() {
    float* d; hipMalloc(&d, sizeof(float) * 64 * 8192 * 4);
    for (int wps : {1, 2, 4, 8}) {
        const int blocks = 1024 * wps;
        printf("waves per SIMD = %d\n", wps);
        run("fma", k_fma, d, blocks, kAcc);
        run("mul", k_mul, d, blocks, kAcc);
        run("pk_fma", k_pkfma, d, blocks, kAcc);
        run("pk_mul", k_pkmul, d, blocks, kAcc);
        run("pk_f16", k_pkh, d, blocks, 2 * kAcc);
        run("exp", k_exp, d, blocks, kAcc);
        run("rcp", k_rcp, d, blocks, kAcc);
        run("mix", k_mix, d, blocks, 2 * kAcc);
    }
    return 0;
}
