// gs_device.hpp — device-side math shared by the MI355X kernels.
//
// Numerical contract: the whole library is compiled with -ffp-contract=off,
// division and sqrt are IEEE correctly rounded (hipcc default), exp is gs_expf below, and
// every expression keeps the evaluation order of the reference MSL
// (GuassianSplatting/tiled_shaders.metal). That makes tile rects, depth keys and the
// per-pixel half-precision blend bit-reproducible against the CPU oracle.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/gs_rasterizer.h"

namespace gs {

constexpr float kShC0 = 0.28209479177387814f;   // tiled_shaders.metal:83
constexpr uint32_t kTile = 16u;                 // :84
constexpr float kMaxRadius = 512.0f;            // :85
constexpr float kMaxLogScale = 5.0f;            // :87
constexpr float kMinOpacity = 0.005f;           // :742
constexpr uint32_t kMaxTilesPerGaussian = 256u; // :743

// Deterministic exp: Cody-Waite reduction + degree-6 polynomial with explicit fmaf.
// Domain used by the hot path |x| <= 8; valid for x in [-87, 88].
// gs_expf_core: the same computation without the range guards, for callers that have already
// bounded x (the blend kernels call it only after the power test, x in [-4.5, 0]).
__device__ __forceinline__ float gs_expf_core(float x) {
    float k = rintf(x * 1.44269502f);
    float r = fmaf(k, -0.693145751953125f, x);
    r = fmaf(k, -1.42860677e-06f, r);
    float p = 1.98756915e-4f;
    p = fmaf(p, r, 1.39819995e-3f);
    p = fmaf(p, r, 8.33345191e-3f);
    p = fmaf(p, r, 4.16657959e-2f);
    p = fmaf(p, r, 1.66666655e-1f);
    p = fmaf(p, r, 5.00000012e-1f);
    float r2 = r * r;
    float y = fmaf(p, r2, r) + 1.0f;
    // v_ldexp_f32: the scaling by 2^k (exact, rounded once like gs_expf's multiply), one instruction
    return __builtin_amdgcn_ldexpf(y, (int)k);
}

typedef float gs_f2 __attribute__((ext_vector_type(2)));
typedef _Float16 gs_h2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ float gs_expf(float x) {
    if (x != x) return x;
    if (x > 88.0f) return __builtin_inff();
    if (x < -87.0f) return 0.0f;
    float k = rintf(x * 1.44269502f);
    float r = fmaf(k, -0.693145751953125f, x);
    r = fmaf(k, -1.42860677e-06f, r);
    float p = 1.98756915e-4f;
    p = fmaf(p, r, 1.39819995e-3f);
    p = fmaf(p, r, 8.33345191e-3f);
    p = fmaf(p, r, 4.16657959e-2f);
    p = fmaf(p, r, 1.66666655e-1f);
    p = fmaf(p, r, 5.00000012e-1f);
    float r2 = r * r;
    float y = fmaf(p, r2, r) + 1.0f;
    int ki = (int)k;
    return y * __uint_as_float((uint32_t)(ki + 127) << 23);
}

__device__ __forceinline__ float clampf(float x, float lo, float hi) {
    return fminf(fmaxf(x, lo), hi);
}

// Metal float3x3: c[col][row]; product (A*B)[j][i] = sum_k A[k][i]*B[j][k] in k order.
struct Mat3 {
    float c[3][3];
};

__device__ __forceinline__ Mat3 mul(const Mat3& A, const Mat3& B) {
    Mat3 C;
#pragma unroll
    for (int j = 0; j < 3; j++)
#pragma unroll
        for (int i = 0; i < 3; i++) {
            float s = A.c[0][i] * B.c[j][0];
            s = s + A.c[1][i] * B.c[j][1];
            s = s + A.c[2][i] * B.c[j][2];
            C.c[j][i] = s;
        }
    return C;
}

__device__ __forceinline__ Mat3 transpose(const Mat3& A) {
    Mat3 T;
#pragma unroll
    for (int c = 0; c < 3; c++)
#pragma unroll
        for (int r = 0; r < 3; r++) T.c[c][r] = A.c[r][c];
    return T;
}

// fp64 3x3 for the per-Gaussian gradient chain (same column-major semantics).
struct Mat3d {
    double c[3][3];
};

__device__ __forceinline__ Mat3d mul(const Mat3d& A, const Mat3d& B) {
    Mat3d C;
#pragma unroll
    for (int j = 0; j < 3; j++)
#pragma unroll
        for (int i = 0; i < 3; i++)
            C.c[j][i] = A.c[0][i] * B.c[j][0] + A.c[1][i] * B.c[j][1] + A.c[2][i] * B.c[j][2];
    return C;
}

__device__ __forceinline__ Mat3d transpose(const Mat3d& A) {
    Mat3d T;
#pragma unroll
    for (int c = 0; c < 3; c++)
#pragma unroll
        for (int r = 0; r < 3; r++) T.c[c][r] = A.c[r][c];
    return T;
}

// quatToMat (tiled_shaders.metal:91-99); q = (w, x, y, z).
__device__ __forceinline__ Mat3 quat_to_mat(float w, float x, float y, float z) {
    Mat3 R;
    R.c[0][0] = 1.0f - 2.0f * (y * y + z * z);
    R.c[0][1] = 2.0f * (x * y + w * z);
    R.c[0][2] = 2.0f * (x * z - w * y);
    R.c[1][0] = 2.0f * (x * y - w * z);
    R.c[1][1] = 1.0f - 2.0f * (x * x + z * z);
    R.c[1][2] = 2.0f * (y * z + w * x);
    R.c[2][0] = 2.0f * (x * z + w * y);
    R.c[2][1] = 2.0f * (y * z - w * x);
    R.c[2][2] = 1.0f - 2.0f * (x * x + y * y);
    return R;
}

__device__ __forceinline__ Mat3 view_rot(const GsTiledUniforms& u) {
    Mat3 W;
#pragma unroll
    for (int c = 0; c < 3; c++)
#pragma unroll
        for (int r = 0; r < 3; r++) W.c[c][r] = u.view[c * 4 + r];
    return W;
}

// float4x4 * float4 row r (column-major), summed over columns in order.
__device__ __forceinline__ float mat4_row(const float* M, int r, float x, float y, float z) {
    float s = M[0 * 4 + r] * x;
    s = s + M[1 * 4 + r] * y;
    s = s + M[2 * 4 + r] * z;
    s = s + M[3 * 4 + r] * 1.0f;
    return s;
}

// Load the 56 bytes of a 112-B Gaussian record the hot path consumes, as 16-B vector loads.
struct GaussianIn {
    float px, py, pz;
    float sx, sy, sz;
    float qw, qx, qy, qz;
    float op;
    float sh0, sh4, sh8;
};

__device__ __forceinline__ GaussianIn load_gaussian(const GsGaussian* __restrict__ g, uint32_t i) {
    const float4* p = reinterpret_cast<const float4*>(g + i);  // 112 B = 7 x 16 B
    float4 a = p[0];  // pos, pad
    float4 b = p[1];  // scale, pad
    float4 c = p[2];  // rotation
    float4 d = p[3];  // opacity @48, sh0 @52, sh1, sh2
    float4 e = p[4];  // sh3 @64, sh4 @68, sh5, sh6
    float4 f = p[5];  // sh7 @80, sh8 @84, sh9, sh10
    GaussianIn o;
    o.px = a.x; o.py = a.y; o.pz = a.z;
    o.sx = b.x; o.sy = b.y; o.sz = b.z;
    o.qw = c.x; o.qx = c.y; o.qy = c.z; o.qz = c.w;
    o.op = d.x; o.sh0 = d.y; o.sh4 = e.y; o.sh8 = f.y;
    return o;
}

// Full projected record (the GsProjected fields) of one Gaussian —
// projectGaussians (tiled_shaders.metal:102-304) with its early-exit partial fills.
struct Projected {
    float sx, sy;          // screen_pos
    float c0, c1, c2;      // conic
    float depth;
    float opacity;
    float r, g, b;         // color
    float radius;
    uint32_t tminx, tminy, tmaxx, tmaxy;
    float vx, vy;          // view_pos_xy
    float ca, cb, cc;      // cov2d
};

__device__ __forceinline__ void project(const GaussianIn& gin, const GsTiledUniforms& u,
                                        Projected& p) {
    p.sx = p.sy = 0.0f;
    p.c0 = p.c1 = p.c2 = 0.0f;
    p.depth = 0.0f;
    p.opacity = 0.0f;
    p.r = p.g = p.b = 0.0f;
    p.radius = 0.0f;
    p.tminx = 0xffffffffu; p.tmaxx = 0u;
    p.tminy = 0xffffffffu; p.tmaxy = 0u;
    p.vx = p.vy = 0.0f;
    p.ca = p.cb = p.cc = 0.0f;

    if (__builtin_isnan(gin.px) || __builtin_isnan(gin.py) || __builtin_isnan(gin.pz) ||
        __builtin_isnan(gin.sx) || __builtin_isnan(gin.sy) || __builtin_isnan(gin.sz) ||
        fabsf(gin.px) > 1e6f || fabsf(gin.py) > 1e6f || fabsf(gin.pz) > 1e6f)
        return;

    const float vwx = mat4_row(u.view, 0, gin.px, gin.py, gin.pz);
    const float vwy = mat4_row(u.view, 1, gin.px, gin.py, gin.pz);
    const float vwz = mat4_row(u.view, 2, gin.px, gin.py, gin.pz);
    const float clx = mat4_row(u.view_proj, 0, gin.px, gin.py, gin.pz);
    const float cly = mat4_row(u.view_proj, 1, gin.px, gin.py, gin.pz);
    const float clw = mat4_row(u.view_proj, 3, gin.px, gin.py, gin.pz);
    if (clw <= 0.1f || vwz <= 0.1f) return;

    const float ndcx = clx / clw, ndcy = cly / clw;
    if (fabsf(ndcx) > 1.2f || fabsf(ndcy) > 1.2f) return;

    p.sx = (ndcx * 0.5f + 0.5f) * u.screen_size[0];
    p.sy = (ndcy * 0.5f + 0.5f) * u.screen_size[1];
    p.depth = vwz;
    p.vx = vwx;
    p.vy = vwy;

    float s0 = gs_expf(clampf(gin.sx, -kMaxLogScale, kMaxLogScale));
    float s1 = gs_expf(clampf(gin.sy, -kMaxLogScale, kMaxLogScale));
    float s2 = gs_expf(clampf(gin.sz, -kMaxLogScale, kMaxLogScale));
    const float smax = fmaxf(fmaxf(s0, s1), s2);
    const float smin = fminf(fminf(s0, s1), s2);
    if (smax > 20.0f * smin) {
        const float target = 20.0f * smin;
        const float f = target / smax;
        s0 = s0 * f; s1 = s1 * f; s2 = s2 * f;
    }

    float qd = gin.qw * gin.qw;
    qd = qd + gin.qx * gin.qx;
    qd = qd + gin.qy * gin.qy;
    qd = qd + gin.qz * gin.qz;
    const float ql = sqrtf(qd);
    float qw = 1.0f, qx = 0.0f, qy = 0.0f, qz = 0.0f;
    if (ql > 0.001f) {
        qw = gin.qw / ql; qx = gin.qx / ql; qy = gin.qy / ql; qz = gin.qz / ql;
    }

    const Mat3 R = quat_to_mat(qw, qx, qy, qz);
    Mat3 S = {};
    S.c[0][0] = s0; S.c[1][1] = s1; S.c[2][2] = s2;
    const Mat3 M = mul(R, S);
    const Mat3 Sigma = mul(M, transpose(M));

    const float z = vwz;
    const float fx = u.focal[0], fy = u.focal[1];
    const float limx = 1.3f * fx / z;
    const float limy = 1.3f * fy / z;
    const float txtz = clampf(vwx / z, -limx, limx);
    const float tytz = clampf(vwy / z, -limy, limy);
    Mat3 J = {};
    J.c[0][0] = fx / z;
    J.c[2][0] = -fx * txtz / z;
    J.c[1][1] = fy / z;
    J.c[2][1] = -fy * tytz / z;
    const Mat3 T = mul(J, view_rot(u));
    const Mat3 cov = mul(mul(T, Sigma), transpose(T));

    float a = cov.c[0][0];
    const float b = cov.c[1][0];
    float c = cov.c[1][1];
    a += 0.3f;
    c += 0.3f;
    p.ca = a; p.cb = b; p.cc = c;

    const float det = a * c - b * b;
    if (det < 0.0001f) return;
    const float inv_det = 1.0f / det;
    p.c0 = c * inv_det;
    p.c1 = -b * inv_det;
    p.c2 = a * inv_det;
    const float mid = 0.5f * (a + c);
    const float disc = mid * mid - det;
    const float l1 = mid + sqrtf(fmaxf(0.1f, disc));
    const float rr = 3.0f * sqrtf(l1);
    p.radius = fminf(ceilf(rr), kMaxRadius);
    if (p.radius <= 0.0f) return;

    const float rad = p.radius;
    int minx = (int)(p.sx - rad); minx = minx < 0 ? 0 : minx;
    int miny = (int)(p.sy - rad); miny = miny < 0 ? 0 : miny;
    int maxx = (int)(p.sx + rad);
    int maxy = (int)(p.sy + rad);
    const int swm1 = (int)u.screen_size[0] - 1, shm1 = (int)u.screen_size[1] - 1;
    maxx = maxx > swm1 ? swm1 : maxx;
    maxy = maxy > shm1 ? shm1 : maxy;
    if (minx > maxx || miny > maxy) {
        p.radius = 0.0f;
        return;
    }
    p.tminx = (uint32_t)minx / kTile;
    p.tminy = (uint32_t)miny / kTile;
    const uint32_t tmx = (uint32_t)maxx / kTile, tmy = (uint32_t)maxy / kTile;
    p.tmaxx = tmx < u.num_tiles_x - 1u ? tmx : u.num_tiles_x - 1u;
    p.tmaxy = tmy < u.num_tiles_y - 1u ? tmy : u.num_tiles_y - 1u;
    if ((p.tmaxx - p.tminx + 1u) * (p.tmaxy - p.tminy + 1u) > 256u) {
        p.radius = 0.0f;
        return;
    }
    const float rop = clampf(gin.op, -8.0f, 8.0f);
    p.opacity = 1.0f / (1.0f + gs_expf(-rop));
    p.r = clampf(kShC0 * gin.sh0 + 0.5f, 0.0f, 1.0f);
    p.g = clampf(kShC0 * gin.sh4 + 0.5f, 0.0f, 1.0f);
    p.b = clampf(kShC0 * gin.sh8 + 0.5f, 0.0f, 1.0f);
}

// generateTilePairs filter (tiled_shaders.metal:755-770): number of tiles to emit, or 0.
__device__ __forceinline__ uint32_t pair_count(const Projected& p) {
    if (p.radius <= 0.0f) return 0u;
    if (p.tminx > p.tmaxx || p.tminy > p.tmaxy) return 0u;
    if (p.opacity < kMinOpacity) return 0u;
    if (p.tminx > 10000u || p.tmaxx > 10000u || p.tminy > 10000u || p.tmaxy > 10000u) return 0u;
    const uint32_t cnt = (p.tmaxx - p.tminx + 1u) * (p.tmaxy - p.tminy + 1u);
    return cnt > kMaxTilesPerGaussian ? 0u : cnt;
}

// Conservative half-extents (pixels) of the region where a splat can contribute. A pixel must
// pass the power test (power >= -4.5 in float, or in half: q = -2 power <= 9.0039) AND the alpha
// test (opacity * G >= 1/255, i.e. q <= 2 ln(255 opacity) in float; the half path's roundings of
// opacity, power, G and the product loosen that by < 8.4e-3 in q), so the bound uses
// K = min(9.01, 2 ln(255 opacity) + 0.02). The float evaluation of q can lose a few ulp of
// |c0 dx^2| + |2 c1 dx dy| + |c2 dy^2| to cancellation, so the ellipse is that of the perturbed
// conic ((1-e) c0, (1+e)|c1|, (1-e) c2), e = 1e-5 — a superset of every pixel the exact kernels
// can accept. A near-singular conic gets infinite extents (never culled); a splat too faint to
// ever pass the alpha test gets -inf (always culled). Used only to skip work, never to decide.
__device__ __forceinline__ void cull_extents(float c0, float c1, float c2, float opacity, float& ex,
                                             float& ey, float& kq) {
    const double e = 1e-5;
    // float log is ample: its error (~1e-7) is far inside the 0.02 margin
    const double Kop = (double)(2.0f * __logf(255.0f * opacity)) + 0.02;
    if (!(Kop > 0.0)) {
        ex = ey = -__builtin_inff();
        kq = -1.0f;
        return;
    }
    const double K = Kop < 9.01 ? Kop : 9.01;
    kq = (float)(K * (1.0 + 1e-6));
    const double A = (1.0 - e) * (double)c0, C = (1.0 - e) * (double)c2;
    const double B = (1.0 + e) * fabs((double)c1);
    const double D = A * C - B * B;
    if (!(D > 1e-30 * A * C) || !(A > 0.0) || !(C > 0.0)) {
        ex = ey = __builtin_inff();
        return;
    }
    ex = (float)(sqrt(K * C / D) * (1.0 + 1e-6) + 1e-3);
    ey = (float)(sqrt(K * A / D) * (1.0 + 1e-6) + 1e-3);
}

// Sortable depth key (tiled_shaders.metal:773-774).
__device__ __forceinline__ uint32_t depth_key(float depth) {
    uint32_t k = __float_as_uint(depth);
    return (k & 0x80000000u) ? ~k : (k | 0x80000000u);
}

// Wave-64 helpers ---------------------------------------------------------------------
__device__ __forceinline__ uint64_t lanemask_lt() {
    const uint32_t lane = __lane_id();
    return lane == 0 ? 0ull : (~0ull >> (64u - lane));
}

__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
        const uint32_t w = __shfl_xor(v, o, 64);
        v = w > v ? w : v;
    }
    return v;
}

// Workgroup b -> tile with the tiles cut into 8 contiguous runs, run x on XCD x (workgroups are
// dispatched round-robin over the 8 XCDs: b and b + 8 share one), so neighbouring tiles -- which share
// most of their splats -- are read through one L2.
__device__ __forceinline__ uint32_t xcd_tile(uint32_t b, uint32_t n) {
    const uint32_t xcd = b & 7u, idx = b >> 3, q = n >> 3, r = n & 7u;
    return (xcd < r ? xcd * (q + 1u) : r * (q + 1u) + (xcd - r) * q) + idx;
}

// Inclusive wave scan with DPP moves (VALU latency, no LDS crossbar round trips): Hillis-Steele
// inside each row of 16 lanes (row_shr 1, 2, 4, 8), then row_bcast:15 into rows 1 and 3 and
// row_bcast:31 into rows 2 and 3. A lane whose DPP source is outside its row (or whose row is masked
// off) takes `id`, the operator's identity.
template <class Op>
__device__ __forceinline__ uint32_t wave_scan_dpp(uint32_t v, uint32_t id, Op op) {
    v = op(v, (uint32_t)__builtin_amdgcn_update_dpp((int)id, (int)v, 0x111, 0xf, 0xf, false));
    v = op(v, (uint32_t)__builtin_amdgcn_update_dpp((int)id, (int)v, 0x112, 0xf, 0xf, false));
    v = op(v, (uint32_t)__builtin_amdgcn_update_dpp((int)id, (int)v, 0x114, 0xf, 0xf, false));
    v = op(v, (uint32_t)__builtin_amdgcn_update_dpp((int)id, (int)v, 0x118, 0xf, 0xf, false));
    v = op(v, (uint32_t)__builtin_amdgcn_update_dpp((int)id, (int)v, 0x142, 0xa, 0xf, false));
    v = op(v, (uint32_t)__builtin_amdgcn_update_dpp((int)id, (int)v, 0x143, 0xc, 0xf, false));
    return v;
}
struct DppAdd {
    __device__ uint32_t operator()(uint32_t a, uint32_t b) const { return a + b; }
};
struct DppMin {
    __device__ uint32_t operator()(uint32_t a, uint32_t b) const { return a < b ? a : b; }
};
struct DppMax {
    __device__ uint32_t operator()(uint32_t a, uint32_t b) const { return a > b ? a : b; }
};
// wave-wide min / max, as a scalar (lane 63 of the inclusive scan)
__device__ __forceinline__ uint32_t wave_min_dpp(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_readlane((int)wave_scan_dpp(v, 0xffffffffu, DppMin{}), 63);
}
__device__ __forceinline__ uint32_t wave_max_dpp(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_readlane((int)wave_scan_dpp(v, 0u, DppMax{}), 63);
}

__device__ __forceinline__ uint32_t wave_min_u32(uint32_t v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
        const uint32_t w = __shfl_xor(v, o, 64);
        v = w < v ? w : v;
    }
    return v;
}

}  // namespace gs
