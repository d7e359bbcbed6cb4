/*
 * gs_oracle.c — TEST INFRASTRUCTURE ONLY (parity checker and CPU baseline).
 *
 * CPU restatement of the reference hot path; see gs_oracle.h for the scope and the
 * "parity unpinned" statement. Each function cites the reference file:line it restates.
 * Build: oracle/Makefile (gcc -O3 -ffp-contract=off -fopenmp). No FMA contraction is
 * allowed anywhere in this file: every float expression is evaluated in the order written.
 */
#include "gs_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define REF_SH_C0 0.28209479177387814f /* tiled_shaders.metal:83 */
#define REF_TILE 16u                   /* :84 */
#define REF_MAX_RADIUS 512.0f          /* :85 */
#define REF_MAX_SCALE 5.0f             /* :87 */
#define REF_MIN_OPACITY 0.005f         /* :742 */
#define REF_MAX_TILES 256u             /* :743 */

/* ----------------------------------------------------------------------------------
 * Deterministic exp. Metal's exp() under MTL_FAST_MATH is implementation-defined, so the
 * reference semantics pin exp to this routine (the product kernels use the same algorithm).
 * Domain used by the hot path: |x| <= 8. Valid for x in [-87, 88].
 * ---------------------------------------------------------------------------------- */
float gso_expf(float x) {
    if (x != x) return x;
    if (x > 88.0f) return INFINITY;
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
    union { uint32_t u; float f; } s;
    s.u = (uint32_t)(ki + 127) << 23;
    return y * s.f;
}

/* IEEE binary16, round to nearest even (handles subnormals, overflow to inf, NaN). */
uint16_t gso_half_bits(float f) {
    union { float f; uint32_t u; } v = {f};
    uint32_t x = v.u;
    uint32_t sign = (x >> 16) & 0x8000u;
    uint32_t ax = x & 0x7fffffffu;
    if (ax >= 0x7f800000u) return (uint16_t)(sign | (ax > 0x7f800000u ? 0x7e00u : 0x7c00u));
    if (ax >= 0x477ff000u) return (uint16_t)(sign | 0x7c00u); /* >= 65520 rounds to inf */
    if (ax < 0x38800000u) {                                   /* below 2^-14: subnormal */
        if (ax < 0x33000000u) return (uint16_t)sign;           /* < 2^-25: rounds to 0 */
        uint32_t e = ax >> 23;
        uint32_t m = (ax & 0x7fffffu) | 0x800000u;
        uint32_t shift = 126u - e; /* value = m * 2^(e-150); half subnormal q = value / 2^-24 */
        uint32_t q = m >> shift;
        uint32_t rem = m & ((1u << shift) - 1u);
        uint32_t half = 1u << (shift - 1u);
        if (rem > half || (rem == half && (q & 1u))) q++;
        return (uint16_t)(sign | q);
    }
    uint32_t e = (ax >> 23) - 112u;
    uint32_t m = ax & 0x7fffffu;
    uint32_t q = (e << 10) | (m >> 13);
    uint32_t rem = m & 0x1fffu;
    if (rem > 0x1000u || (rem == 0x1000u && (q & 1u))) q++;
    return (uint16_t)(sign | q);
}

static float half_bits_to_float(uint16_t h) {
    uint32_t sign = (uint32_t)(h & 0x8000u) << 16;
    uint32_t e = (h >> 10) & 0x1fu;
    uint32_t m = h & 0x3ffu;
    union { uint32_t u; float f; } v;
    if (e == 0) {
        float f = (float)m * 5.9604644775390625e-08f; /* 2^-24, exact */
        return sign ? -f : f;
    }
    if (e == 31) v.u = sign | 0x7f800000u | (m << 13);
    else v.u = sign | ((e + 112u) << 23) | (m << 13);
    return v.f;
}

float gso_half(float x) { return half_bits_to_float(gso_half_bits(x)); }

/* Half arithmetic: the float result of two binary16 operands rounded once to binary16 is the
 * correctly rounded binary16 result (24 >= 2*11 + 2), so these are IEEE half operations. */
static inline float hmul(float a, float b) { return gso_half(a * b); }
static inline float hadd(float a, float b) { return gso_half(a + b); }
static inline float hsub(float a, float b) { return gso_half(a - b); }

/* ---------------------------------------------------------------------------------- */
/* Metal float3x3 semantics: m[c][r] is column c, row r; (A*B)[j][i] = sum_k A[k][i]*B[j][k]. */
typedef struct { float m[3][3]; } mat3;

static mat3 mat3_mul(const mat3* A, const mat3* B) {
    mat3 C;
    for (int j = 0; j < 3; j++)
        for (int i = 0; i < 3; i++) {
            float s = A->m[0][i] * B->m[j][0];
            s = s + A->m[1][i] * B->m[j][1];
            s = s + A->m[2][i] * B->m[j][2];
            C.m[j][i] = s;
        }
    return C;
}

static mat3 mat3_transpose(const mat3* A) {
    mat3 T;
    for (int c = 0; c < 3; c++)
        for (int r = 0; r < 3; r++) T.m[c][r] = A->m[r][c];
    return T;
}

static mat3 mat3_scale(const mat3* A, float s) {
    mat3 B;
    for (int c = 0; c < 3; c++)
        for (int r = 0; r < 3; r++) B.m[c][r] = s * A->m[c][r];
    return B;
}

/* tiled_shaders.metal:91-99 quatToMat: q.x=w, q.y=x, q.z=y, q.w=z; columns listed. */
static mat3 quat_to_mat(const float q[4]) {
    float w = q[0], x = q[1], y = q[2], z = q[3];
    mat3 R;
    R.m[0][0] = 1.0f - 2.0f * (y * y + z * z);
    R.m[0][1] = 2.0f * (x * y + w * z);
    R.m[0][2] = 2.0f * (x * z - w * y);
    R.m[1][0] = 2.0f * (x * y - w * z);
    R.m[1][1] = 1.0f - 2.0f * (x * x + z * z);
    R.m[1][2] = 2.0f * (y * z + w * x);
    R.m[2][0] = 2.0f * (x * z + w * y);
    R.m[2][1] = 2.0f * (y * z - w * x);
    R.m[2][2] = 1.0f - 2.0f * (x * x + y * y);
    return R;
}

/* float4x4 (column-major, m[4c+r]) * float4: sum over columns in order. */
static void mat4_mul_vec(const float* M, const float v[4], float out[4]) {
    for (int r = 0; r < 4; r++) {
        float s = M[0 * 4 + r] * v[0];
        s = s + M[1 * 4 + r] * v[1];
        s = s + M[2 * 4 + r] * v[2];
        s = s + M[3 * 4 + r] * v[3];
        out[r] = s;
    }
}

static inline float clampf(float x, float lo, float hi) { return fminf(fmaxf(x, lo), hi); }

/* tiled_shaders.metal:102-304 */
static void project_one(const GsGaussian* gp, const GsTiledUniforms* u, GsProjected* out) {
    GsGaussian g = *gp;
    GsProjected proj;
    memset(&proj, 0, sizeof(proj));
    proj.radius = 0.0f;
    proj.tile_min_x = 0xffffffffu;
    proj.tile_max_x = 0u;
    proj.tile_min_y = 0xffffffffu;
    proj.tile_max_y = 0u;

    /* :120-125 */
    if (isnan(g.position[0]) || isnan(g.position[1]) || isnan(g.position[2]) ||
        isnan(g.scale[0]) || isnan(g.scale[1]) || isnan(g.scale[2]) ||
        fabsf(g.position[0]) > 1e6f || fabsf(g.position[1]) > 1e6f ||
        fabsf(g.position[2]) > 1e6f) {
        *out = proj;
        return;
    }
    /* :128-138 */
    float world[4] = {g.position[0], g.position[1], g.position[2], 1.0f};
    float view[4], clip[4];
    mat4_mul_vec(u->view, world, view);
    mat4_mul_vec(u->view_proj, world, clip);
    if (clip[3] <= 0.1f || view[2] <= 0.1f) {
        *out = proj;
        return;
    }
    /* :141-147 */
    float ndc[3] = {clip[0] / clip[3], clip[1] / clip[3], clip[2] / clip[3]};
    if (fabsf(ndc[0]) > 1.2f || fabsf(ndc[1]) > 1.2f) {
        *out = proj;
        return;
    }
    /* :150-157 */
    proj.screen_pos[0] = (ndc[0] * 0.5f + 0.5f) * u->screen_size[0];
    proj.screen_pos[1] = (ndc[1] * 0.5f + 0.5f) * u->screen_size[1];
    proj.depth = view[2];
    proj.view_pos_xy[0] = view[0];
    proj.view_pos_xy[1] = view[1];
    /* :160-170 */
    float scale[3];
    for (int k = 0; k < 3; k++) scale[k] = gso_expf(clampf(g.scale[k], -REF_MAX_SCALE, REF_MAX_SCALE));
    float max_s = fmaxf(fmaxf(scale[0], scale[1]), scale[2]);
    float min_s = fminf(fminf(scale[0], scale[1]), scale[2]);
    if (max_s > 20.0f * min_s) {
        float target = 20.0f * min_s;
        float f = target / max_s;
        for (int k = 0; k < 3; k++) scale[k] = scale[k] * f;
    }
    /* :173-175 length(q) = sqrt(dot(q, q)) summed x, y, z, w (= w, x, y, z of the quaternion) */
    float q[4] = {g.rotation[0], g.rotation[1], g.rotation[2], g.rotation[3]};
    float qdot = q[0] * q[0];
    qdot = qdot + q[1] * q[1];
    qdot = qdot + q[2] * q[2];
    qdot = qdot + q[3] * q[3];
    float qlen = sqrtf(qdot);
    if (qlen > 0.001f) {
        for (int k = 0; k < 4; k++) q[k] = q[k] / qlen;
    } else {
        q[0] = 1.0f; q[1] = 0.0f; q[2] = 0.0f; q[3] = 0.0f;
    }
    /* :180-190 */
    mat3 R = quat_to_mat(q);
    mat3 S;
    memset(&S, 0, sizeof(S));
    S.m[0][0] = scale[0]; S.m[1][1] = scale[1]; S.m[2][2] = scale[2];
    mat3 M = mat3_mul(&R, &S);
    mat3 Mt = mat3_transpose(&M);
    mat3 Sigma = mat3_mul(&M, &Mt);
    /* :193-215 */
    float z_cam = view[2];
    float fx = u->focal[0], fy = u->focal[1];
    float limx = 1.3f * fx / z_cam;
    float limy = 1.3f * fy / z_cam;
    float txtz = clampf(view[0] / z_cam, -limx, limx);
    float tytz = clampf(view[1] / z_cam, -limy, limy);
    float J00 = fx / z_cam;
    float J02 = -fx * txtz / z_cam;
    float J11 = fy / z_cam;
    float J12 = -fy * tytz / z_cam;
    mat3 J;
    memset(&J, 0, sizeof(J));
    J.m[0][0] = J00; J.m[1][1] = J11; J.m[2][0] = J02; J.m[2][1] = J12;
    /* :218-225 */
    mat3 W;
    for (int c = 0; c < 3; c++)
        for (int r = 0; r < 3; r++) W.m[c][r] = u->view[c * 4 + r];
    mat3 T = mat3_mul(&J, &W);
    mat3 Tt = mat3_transpose(&T);
    mat3 TS = mat3_mul(&T, &Sigma);
    mat3 cov = mat3_mul(&TS, &Tt);
    /* :228-237 */
    float a = cov.m[0][0];
    float b = cov.m[1][0];
    float c = cov.m[1][1];
    a += 0.3f;
    c += 0.3f;
    proj.cov2d[0] = a; proj.cov2d[1] = b; proj.cov2d[2] = c;
    /* :240-244 */
    float det = a * c - b * b;
    if (det < 0.0001f) {
        *out = proj;
        return;
    }
    /* :247-255 */
    float inv_det = 1.0f / det;
    proj.conic[0] = c * inv_det;
    proj.conic[1] = -b * inv_det;
    proj.conic[2] = a * inv_det;
    float mid = 0.5f * (a + c);
    float disc = mid * mid - det;
    float l1 = mid + sqrtf(fmaxf(0.1f, disc));
    float raw_radius = 3.0f * sqrtf(l1);
    proj.radius = fminf(ceilf(raw_radius), REF_MAX_RADIUS);
    /* :258-261 */
    if (proj.radius <= 0.0f) {
        *out = proj;
        return;
    }
    /* :264-275 int() conversion truncates toward zero */
    float r = proj.radius;
    int min_x = (int)(proj.screen_pos[0] - r); if (min_x < 0) min_x = 0;
    int min_y = (int)(proj.screen_pos[1] - r); if (min_y < 0) min_y = 0;
    int max_x = (int)(proj.screen_pos[0] + r);
    int max_y = (int)(proj.screen_pos[1] + r);
    int sw = (int)u->screen_size[0] - 1, sh = (int)u->screen_size[1] - 1;
    if (max_x > sw) max_x = sw;
    if (max_y > sh) max_y = sh;
    if (min_x > max_x || min_y > max_y) {
        proj.radius = 0.0f;
        *out = proj;
        return;
    }
    /* :278-290 */
    proj.tile_min_x = (uint32_t)min_x / REF_TILE;
    proj.tile_min_y = (uint32_t)min_y / REF_TILE;
    uint32_t tmx = (uint32_t)max_x / REF_TILE, tmy = (uint32_t)max_y / REF_TILE;
    proj.tile_max_x = tmx < u->num_tiles_x - 1u ? tmx : u->num_tiles_x - 1u;
    proj.tile_max_y = tmy < u->num_tiles_y - 1u ? tmy : u->num_tiles_y - 1u;
    uint32_t tiles_x = proj.tile_max_x - proj.tile_min_x + 1u;
    uint32_t tiles_y = proj.tile_max_y - proj.tile_min_y + 1u;
    if (tiles_x * tiles_y > 256u) {
        proj.radius = 0.0f;
        *out = proj;
        return;
    }
    /* :293-301 */
    float raw_op = clampf(g.opacity, -8.0f, 8.0f);
    proj.opacity = 1.0f / (1.0f + gso_expf(-raw_op));
    proj.color[0] = clampf(REF_SH_C0 * g.sh[0] + 0.5f, 0.0f, 1.0f);
    proj.color[1] = clampf(REF_SH_C0 * g.sh[4] + 0.5f, 0.0f, 1.0f);
    proj.color[2] = clampf(REF_SH_C0 * g.sh[8] + 0.5f, 0.0f, 1.0f);
    *out = proj;
}

void gso_project(const GsGaussian* g, uint32_t n, const GsTiledUniforms* u, GsProjected* out,
                 int threads) {
    (void)threads;
#pragma omp parallel for schedule(static) num_threads(threads > 0 ? threads : 1)
    for (int64_t i = 0; i < (int64_t)n; i++) project_one(&g[i], u, &out[i]);
}

/* tiled_shaders.metal:745-794 */
static int pair_count_of(const GsProjected* p, uint32_t* tile_count, uint32_t* depth_key) {
    if (p->radius <= 0.0f) return 0;
    if (p->tile_min_x > p->tile_max_x || p->tile_min_y > p->tile_max_y) return 0;
    if (p->opacity < REF_MIN_OPACITY) return 0;
    if (p->tile_min_x > 10000u || p->tile_max_x > 10000u || p->tile_min_y > 10000u ||
        p->tile_max_y > 10000u)
        return 0;
    uint32_t tx = p->tile_max_x - p->tile_min_x + 1u;
    uint32_t ty = p->tile_max_y - p->tile_min_y + 1u;
    uint32_t cnt = tx * ty;
    if (cnt > REF_MAX_TILES) return 0;
    union { float f; uint32_t u; } d = {p->depth};
    uint32_t k = d.u;
    k = (k & 0x80000000u) ? ~k : (k | 0x80000000u);
    *tile_count = cnt;
    *depth_key = k;
    return 1;
}

uint64_t gso_generate_pairs(const GsProjected* p, uint32_t n, uint32_t num_tiles_x,
                            uint64_t max_pairs, uint64_t* keys, uint32_t* values) {
    uint64_t counter = 0;
    for (uint32_t gid = 0; gid < n; gid++) {
        uint32_t cnt, dk;
        if (!pair_count_of(&p[gid], &cnt, &dk)) continue;
        uint64_t pos = counter;
        counter += cnt;
        if (pos + cnt > max_pairs) continue; /* :780 whole Gaussian dropped */
        uint64_t idx = 0;
        for (uint32_t ty = p[gid].tile_min_y; ty <= p[gid].tile_max_y; ty++)
            for (uint32_t tx = p[gid].tile_min_x; tx <= p[gid].tile_max_x; tx++) {
                uint32_t tile = ty * num_tiles_x + tx;
                keys[pos + idx] = ((uint64_t)tile << 32) | (uint64_t)dk;
                values[pos + idx] = gid;
                idx++;
            }
    }
    return counter;
}

/* tiled_rasterizer.mm:27-102 */
void gso_sort_pairs(uint64_t* keys, uint32_t* values, uint64_t n, int threads) {
    if (n < 2) return;
    int nt = threads > 0 ? threads : 1;
    uint64_t* tk = (uint64_t*)malloc(n * sizeof(uint64_t));
    uint32_t* tv = (uint32_t*)malloc(n * sizeof(uint32_t));
    uint32_t(*hist)[256] = (uint32_t(*)[256])calloc((size_t)nt, sizeof(uint32_t[256]));
    uint64_t* sk = keys; uint32_t* sv = values;
    uint64_t* dk = tk;   uint32_t* dv = tv;
    uint64_t chunk = (n + (uint64_t)nt - 1) / (uint64_t)nt;
    for (int pass = 0; pass < 8; pass++) {
        int shift = pass * 8;
#pragma omp parallel for schedule(static, 1) num_threads(nt)
        for (int t = 0; t < nt; t++) {
            memset(hist[t], 0, sizeof(hist[t]));
            uint64_t s = (uint64_t)t * chunk, e = s + chunk < n ? s + chunk : n;
            for (uint64_t i = s; i < e; i++) hist[t][(sk[i] >> shift) & 0xffu]++;
        }
        uint32_t sum = 0;
        for (int d = 0; d < 256; d++)
            for (int t = 0; t < nt; t++) {
                uint32_t c = hist[t][d];
                hist[t][d] = sum;
                sum += c;
            }
#pragma omp parallel for schedule(static, 1) num_threads(nt)
        for (int t = 0; t < nt; t++) {
            uint64_t s = (uint64_t)t * chunk, e = s + chunk < n ? s + chunk : n;
            for (uint64_t i = s; i < e; i++) {
                uint32_t d = (uint32_t)((sk[i] >> shift) & 0xffu);
                uint32_t o = hist[t][d]++;
                dk[o] = sk[i];
                dv[o] = sv[i];
            }
        }
        uint64_t* x = sk; sk = dk; dk = x;
        uint32_t* y = sv; sv = dv; dv = y;
    }
    /* 8 passes: the data is back in the caller's arrays */
    free(tk); free(tv); free(hist);
}

/* sort.metal:553-589 */
void gso_build_tile_ranges(const uint64_t* keys, uint64_t n_pairs, uint32_t num_tiles,
                           GsTileRange* ranges, int threads) {
    (void)threads;
#pragma omp parallel for schedule(static) num_threads(threads > 0 ? threads : 1)
    for (int64_t id = 0; id < (int64_t)num_tiles; id++) {
        uint32_t target = (uint32_t)id;
        uint64_t lo = 0, hi = n_pairs;
        while (lo < hi) {
            uint64_t mid = (lo + hi) / 2;
            if ((uint32_t)(keys[mid] >> 32) < target) lo = mid + 1; else hi = mid;
        }
        uint64_t cnt = 0;
        for (uint64_t i = lo; i < n_pairs; i++) {
            if ((uint32_t)(keys[i] >> 32) != target) break;
            cnt++;
        }
        ranges[id].start = (uint32_t)lo;
        ranges[id].count = (uint32_t)cnt;
    }
}

static inline uint32_t quantize_unorm8(float c) {
    float x = fminf(fmaxf(c, 0.0f), 1.0f) * 255.0f;
    return (uint32_t)rintf(x);
}

/* tiled_shaders.metal:307-385 */
void gso_forward_blend(const GsProjected* p, uint32_t n, const uint32_t* sorted_values,
                       const GsTileRange* ranges, const GsTiledUniforms* u, uint32_t w,
                       uint32_t h, uint32_t* last_idx, uint32_t* rgba8, float* rgb_f32,
                       int threads) {
    const float H_T_EPS = gso_half(0.0001f);
    const float H_ALPHA_MAX = gso_half(0.99f);
    const float H_ALPHA_MIN = gso_half(1.0f / 255.0f);
    const float H_POW_MIN = gso_half(-4.5f);
    uint32_t sw = (uint32_t)u->screen_size[0], shh = (uint32_t)u->screen_size[1];
#pragma omp parallel for schedule(dynamic, 4) num_threads(threads > 0 ? threads : 1)
    for (int64_t yy = 0; yy < (int64_t)h; yy++) {
        for (uint32_t x = 0; x < w; x++) {
            uint32_t y = (uint32_t)yy;
            if (x >= sw || y >= shh) continue;
            uint32_t tile = (y / REF_TILE) * u->num_tiles_x + (x / REF_TILE);
            GsTileRange range = ranges[tile];
            float col[3] = {0.0f, 0.0f, 0.0f};
            float T = 1.0f;
            float px = (float)x + 0.5f, py = (float)y + 0.5f;
            uint32_t last = 0;
            int has = 0;
            for (uint32_t i = 0; i < range.count && T > H_T_EPS; i++) {
                uint32_t sidx = range.start + i;
                uint32_t gidx = sorted_values[sidx];
                if (gidx >= n) continue;
                const GsProjected* pg = &p[gidx];
                if (pg->radius <= 0.0f) continue;
                float dx = px - pg->screen_pos[0];
                float dy = py - pg->screen_pos[1];
                float cmag = fabsf(pg->conic[0]) + fabsf(pg->conic[1]) + fabsf(pg->conic[2]);
                if (cmag < 0.0001f) continue;
                float pw = -0.5f * (pg->conic[0] * dx * dx + 2.0f * pg->conic[1] * dx * dy +
                                    pg->conic[2] * dy * dy);
                float power = gso_half(pw);
                if (power > 0.0f || power < H_POW_MIN) continue;
                float G = gso_half(gso_expf(power));
                float alpha = fminf(hmul(gso_half(pg->opacity), G), H_ALPHA_MAX);
                if (alpha < H_ALPHA_MIN) continue;
                for (int k = 0; k < 3; k++)
                    col[k] = hadd(col[k], hmul(hmul(gso_half(pg->color[k]), alpha), T));
                T = hmul(T, hsub(1.0f, alpha));
                last = sidx;
                has = 1;
            }
            for (int k = 0; k < 3; k++) col[k] = hadd(col[k], hmul(1.0f, T));
            uint32_t pix = y * sw + x;
            last_idx[pix] = has ? last : 0xffffffffu;
            if (rgba8)
                rgba8[pix] = quantize_unorm8(col[0]) | (quantize_unorm8(col[1]) << 8) |
                             (quantize_unorm8(col[2]) << 16) | (255u << 24);
            if (rgb_f32) {
                rgb_f32[3 * pix + 0] = col[0];
                rgb_f32[3 * pix + 1] = col[1];
                rgb_f32[3 * pix + 2] = col[2];
            }
        }
    }
}

/* field offsets (in floats) of GsGradients */
enum { GF_PX = 0, GF_PY = 1, GF_PZ = 2, GF_OP = 3, GF_SX = 4, GF_SY = 5, GF_SZ = 6,
       GF_QW = 8, GF_QX = 9, GF_QY = 10, GF_QZ = 11, GF_SH0 = 12, GF_SH4 = 16, GF_SH8 = 20,
       GF_VX = 24, GF_VY = 25, GF_NFLOATS = 28 };

static inline float signf_metal(float x) { return x > 0.0f ? 1.0f : (x < 0.0f ? -1.0f : 0.0f); }

/* fp64 shadow of the per-contribution computation (tiled_shaders.metal:427-696) with the float
 * path's decisions: exact exp, and T_final, the reverse T recurrence, accum_rec and dL/dalpha
 * carried in fp64 alongside their float versions. |float term - double term| summed per field
 * estimates the reference's own rounding noise, which the gradient tolerance must admit: T drifts
 * over a long list, dL/dalpha = T dot(dL/dpixel, colour - accum) cancels when accum ~ colour, and
 * the chain (conic -> cov2D -> Sigma -> scale / quaternion) cancels for near-degenerate
 * covariances. */
typedef struct { double m[3][3]; } mat3d;

static mat3d mat3d_mul(const mat3d* A, const mat3d* B) {
    mat3d C;
    for (int j = 0; j < 3; j++)
        for (int i = 0; i < 3; i++)
            C.m[j][i] = A->m[0][i] * B->m[j][0] + A->m[1][i] * B->m[j][1] + A->m[2][i] * B->m[j][2];
    return C;
}

static mat3d mat3d_transpose(const mat3d* A) {
    mat3d T;
    for (int c = 0; c < 3; c++)
        for (int r = 0; r < 3; r++) T.m[c][r] = A->m[r][c];
    return T;
}

static void chain_terms_double(const GsProjected* pg, const GsGaussian* go, const GsTiledUniforms* u,
                               const float dLp[3], double weight, double dL_dAlpha, double G, float dx,
                               float dy, double out[16]) {
    const double SH = (double)REF_SH_C0;
    for (int k = 0; k < 3; k++) {
        double v = (double)dLp[k] * (double)weight * SH;
        if (pg->color[k] <= 0.01f || pg->color[k] >= 0.99f) v = 0.0;
        out[k] = v;
    }
    const double sig = pg->opacity, Gd = G, dxd = dx, dyd = dy, dA = dL_dAlpha;
    out[3] = dA * (sig * (1.0 - sig) * Gd);
    const double dLdG = dA * sig;
    const double c0 = pg->conic[0], c1 = pg->conic[1], c2 = pg->conic[2];
    const double dSx = dLdG * (Gd * dxd * c0 + Gd * dyd * c1);
    const double dSy = dLdG * (Gd * dyd * c2 + Gd * dxd * c1);
    const double z = pg->depth, fx = u->focal[0], fy = u->focal[1];
    const double tx = pg->view_pos_xy[0] / z, ty = pg->view_pos_xy[1] / z;
    const double dV[3] = {dSx * fx / z, dSy * fy / z, -dSx * fx * tx / z - dSy * fy * ty / z};
    mat3d W;
    for (int c = 0; c < 3; c++)
        for (int r = 0; r < 3; r++) W.m[c][r] = u->view[c * 4 + r];
    for (int i = 0; i < 3; i++) out[4 + i] = W.m[i][0] * dV[0] + W.m[i][1] * dV[1] + W.m[i][2] * dV[2];
    out[7] = dSx;
    out[8] = dSy;
    const double dCo0 = -0.5 * dLdG * Gd * dxd * dxd;
    const double dCo1 = -0.5 * dLdG * Gd * 2.0 * dxd * dyd;
    const double dCo2 = -0.5 * dLdG * Gd * dyd * dyd;
    const double ca = pg->cov2d[0], cb = pg->cov2d[1], cc = pg->cov2d[2];
    const double den = ca * cc - cb * cb;
    const double d2i = 1.0 / (den * den + 1e-7);
    const double dCx = d2i * (-cc * cc * dCo0 + 2.0 * cb * cc * dCo1 + (den - ca * cc) * dCo2);
    const double dCz = d2i * (-ca * ca * dCo2 + 2.0 * ca * cb * dCo1 + (den - ca * cc) * dCo0);
    const double dCy = d2i * 2.0 * (cb * cc * dCo0 - (den + 2.0 * cb * cb) * dCo1 + ca * cb * dCo2);
    mat3d J;
    memset(&J, 0, sizeof(J));
    J.m[0][0] = fx / z; J.m[1][1] = fy / z; J.m[2][0] = -fx * tx / z; J.m[2][1] = -fy * ty / z;
    mat3d Tm = mat3d_mul(&J, &W);
    mat3d D;
    memset(&D, 0, sizeof(D));
    D.m[0][0] = dCx; D.m[0][1] = dCy; D.m[1][0] = dCy; D.m[1][1] = dCz;
    mat3d TmT = mat3d_transpose(&Tm);
    mat3d tmp = mat3d_mul(&TmT, &D);
    mat3d dC3 = mat3d_mul(&tmp, &Tm);
    double sc[3];
    for (int k = 0; k < 3; k++) sc[k] = gso_expf(clampf(go->scale[k], -REF_MAX_SCALE, REF_MAX_SCALE));
    const double qr = go->rotation[0], qx = go->rotation[1], qy = go->rotation[2], qz = go->rotation[3];
    mat3d R;
    R.m[0][0] = 1.0 - 2.0 * (qy * qy + qz * qz); R.m[0][1] = 2.0 * (qx * qy + qr * qz); R.m[0][2] = 2.0 * (qx * qz - qr * qy);
    R.m[1][0] = 2.0 * (qx * qy - qr * qz); R.m[1][1] = 1.0 - 2.0 * (qx * qx + qz * qz); R.m[1][2] = 2.0 * (qy * qz + qr * qx);
    R.m[2][0] = 2.0 * (qx * qz + qr * qy); R.m[2][1] = 2.0 * (qy * qz - qr * qx); R.m[2][2] = 1.0 - 2.0 * (qx * qx + qy * qy);
    mat3d M;
    for (int c = 0; c < 3; c++)
        for (int r = 0; r < 3; r++) M.m[c][r] = R.m[c][r] * sc[c];
    mat3d dC3x2;
    for (int c = 0; c < 3; c++)
        for (int r = 0; r < 3; r++) dC3x2.m[c][r] = 2.0 * dC3.m[c][r];
    mat3d dM = mat3d_mul(&dC3x2, &M);
    mat3d Rt = mat3d_transpose(&R);
    mat3d RtdM = mat3d_mul(&Rt, &dM);
    out[9] = RtdM.m[0][0] * sc[0];
    out[10] = RtdM.m[1][1] * sc[1];
    out[11] = RtdM.m[2][2] * sc[2];
    mat3d dR;
    for (int c = 0; c < 3; c++)
        for (int r = 0; r < 3; r++) dR.m[c][r] = dM.m[c][r] * sc[c];
    mat3d m = mat3d_transpose(&dR);
    out[12] = 2.0 * (qz * (m.m[0][1] - m.m[1][0]) + qy * (m.m[2][0] - m.m[0][2]) + qx * (m.m[1][2] - m.m[2][1]));
    out[13] = 2.0 * (qy * (m.m[1][0] + m.m[0][1]) + qz * (m.m[2][0] + m.m[0][2]) +
                     qr * (m.m[1][2] - m.m[2][1]) - 2.0 * qx * (m.m[2][2] + m.m[1][1]));
    out[14] = 2.0 * (qx * (m.m[1][0] + m.m[0][1]) + qr * (m.m[2][0] - m.m[0][2]) +
                     qz * (m.m[1][2] + m.m[2][1]) - 2.0 * qy * (m.m[2][2] + m.m[0][0]));
    out[15] = 2.0 * (qr * (m.m[0][1] - m.m[1][0]) + qx * (m.m[2][0] + m.m[0][2]) +
                     qy * (m.m[1][2] + m.m[2][1]) - 2.0 * qz * (m.m[1][1] + m.m[0][0]));
}

/* First-order rounding bound of the per-pixel float steps (condacc): a float evaluation of the
 * same expressions in another order, with an exp within COND_EXP_REL of the pinned one (the
 * hardware exp: <= 4e-7, gs_debug_float_exp_check; Metal's fast-math exp is unspecified), differs
 * from the reference's per-pixel term by at most |term| * r, where r adds up
 *   - the exp error of the term's own G and of every alpha the pixel's T went through: T is a
 *     product / quotient of (1 - alpha) factors and d(1 - alpha) / (1 - alpha) = -alpha / (1 - alpha)
 *     d(alpha), so T's relative error is <= COND_EXP_REL * sum alpha / (1 - alpha) (forward track
 *     and reverse recurrence), plus one rounding per step;
 *   - for the terms through dL/dalpha = T dot(dL/dpixel, colour - accum): the dot product's
 *     condition number (sum |dl| (|c| + |accum|) / |dot|), with accum's own error bounded by its
 *     contracting recurrence (accum' = a c + (1 - a) accum: each step's error is damped by 1 - a).
 * It is what "defined to float precision" means for these terms; the tests hold a GPU entry that
 * misses the plain bar to it. */
#define COND_EXP_REL 4.0e-7
#define COND_U 5.9604644775390625e-08 /* 2^-24 */

/* tiled_shaders.metal:388-738, one pixel; adds every term into acc (and |term| into abs). */
static void backward_pixel(const GsGaussian* g, const GsProjected* p, uint32_t n,
                           const uint32_t* sorted_values, const GsTileRange* ranges,
                           const GsTiledUniforms* u, uint32_t x, uint32_t y,
                           const uint32_t* last_idx, const uint32_t* rendered,
                           const uint32_t* gt, double* acc, double* absacc, double* noiseacc,
                           double* shadowacc, double* condacc) {
    uint32_t sw = (uint32_t)u->screen_size[0];
    uint32_t pix = y * sw + x;
    uint32_t last = last_idx[pix];
    if (last == 0xffffffffu) return;
    uint32_t tile = (y / REF_TILE) * u->num_tiles_x + (x / REF_TILE);
    GsTileRange range = ranges[tile];
    float px = (float)x + 0.5f, py = (float)y + 0.5f;
    /* :418-423 RGBA8Unorm reads: channel / 255 */
    float dLp[3];
    for (int k = 0; k < 3; k++) {
        float r = (float)((rendered[pix] >> (8 * k)) & 0xffu) / 255.0f;
        float t = (float)((gt[pix] >> (8 * k)) & 0xffu) / 255.0f;
        dLp[k] = signf_metal(r - t) / 3.0f;
    }
    /* :427-460 */
    uint32_t end = last + 1u < range.start + range.count ? last + 1u : range.start + range.count;
    float T_final = 1.0f;
    double Td_final = 1.0;  /* fp64 shadow (noise estimate only) */
    double cA = 0.0, cN = 0.0;  /* conditioning: sum alpha / (1 - alpha), steps (condacc) */
    for (uint32_t s = range.start; s < end; s++) {
        uint32_t gi = sorted_values[s];
        if (gi >= n) continue;
        const GsProjected* pg = &p[gi];
        if (pg->radius <= 0.0f) continue;
        float dx = px - pg->screen_pos[0], dy = py - pg->screen_pos[1];
        float power = -0.5f * (pg->conic[0] * dx * dx + 2.0f * pg->conic[1] * dx * dy +
                               pg->conic[2] * dy * dy);
        if (power > 0.0f || power < -4.5f) continue;
        float G = gso_expf(power);
        float alpha = fminf(pg->opacity * G, 0.99f);
        if (alpha < 1.0f / 255.0f) continue;
        float test_T = T_final * (1.0f - alpha);
        if (test_T < 0.0001f) break;
        T_final = test_T;
        if (noiseacc || shadowacc) Td_final *= 1.0 - fmin((double)pg->opacity * exp((double)power), 0.99);
        cA += (double)alpha / (1.0 - (double)alpha);
        cN += 1.0;
    }
    /* :464-737 */
    float T = T_final;
    float accum[3] = {1.0f, 1.0f, 1.0f};
    double Td = Td_final, accd[3] = {1.0, 1.0, 1.0};
    double cS = 0.0;  /* accum's error amplification: S' = 1 + (1 - alpha) S */
    float fx = u->focal[0], fy = u->focal[1];
    mat3 viewRot;
    for (int c = 0; c < 3; c++)
        for (int r = 0; r < 3; r++) viewRot.m[c][r] = u->view[c * 4 + r];
    for (int64_t s = (int64_t)end - 1; s >= (int64_t)range.start; s--) {
        uint32_t gi = sorted_values[s];
        if (gi >= n) continue;
        const GsProjected* pg = &p[gi];
        if (pg->radius <= 0.0f) continue;
        float dx = px - pg->screen_pos[0], dy = py - pg->screen_pos[1];
        float power = -0.5f * (pg->conic[0] * dx * dx + 2.0f * pg->conic[1] * dx * dy +
                               pg->conic[2] * dy * dy);
        if (power > 0.0f || power < -4.5f) continue;
        float G = gso_expf(power);
        float alpha = fminf(pg->opacity * G, 0.99f);
        if (alpha < 1.0f / 255.0f) continue;
        T = T / fmaxf(1.0f - alpha, 0.0001f);
        float weight = alpha * T;
        float dLc[3] = {dLp[0] * weight, dLp[1] * weight, dLp[2] * weight};
        for (int k = 0; k < 3; k++)
            if (pg->color[k] <= 0.01f || pg->color[k] >= 0.99f) dLc[k] = 0.0f;
        float dd = dLp[0] * (pg->color[0] - accum[0]);
        dd = dd + dLp[1] * (pg->color[1] - accum[1]);
        dd = dd + dLp[2] * (pg->color[2] - accum[2]);
        float dL_dAlpha = T * dd;
        double r_col = 0.0, r_alpha = 0.0;  /* relative conditioning bounds (condacc) */
        if (condacc) {
            cA += (double)alpha / (1.0 - (double)alpha);
            cN += 1.0;
            r_col = COND_EXP_REL * (1.0 + cA) + COND_U * (3.0 + cN);
            double amax = 0.0, num = 0.0;
            for (int k = 0; k < 3; k++) {
                const double dlk = fabs((double)dLp[k]);
                amax = fmax(amax, fmax(fabs((double)accum[k]), fabs((double)pg->color[k])));
                num += dlk * (fabs((double)pg->color[k]) + fabs((double)accum[k])) * 3.0 * COND_U;
            }
            num += (2.0 * COND_U + COND_EXP_REL) * cS * amax * (fabs((double)dLp[0]) + fabs((double)dLp[1]) + fabs((double)dLp[2]));
            r_alpha = r_col + (dd != 0.0f ? num / fabs((double)dd) : 1.0);
            cS = 1.0 + (1.0 - (double)alpha) * cS;
        }
        for (int k = 0; k < 3; k++) accum[k] = alpha * pg->color[k] + (1.0f - alpha) * accum[k];
        float sig = pg->opacity;
        float dAlpha_dRawOp = sig * (1.0f - sig) * G;
        float dL_dRawOp = dL_dAlpha * dAlpha_dRawOp;
        float dL_dG = dL_dAlpha * sig;
        float gdx = G * dx, gdy = G * dy;
        float dG_ddelx = -gdx * pg->conic[0] - gdy * pg->conic[1];
        float dG_ddely = -gdy * pg->conic[2] - gdx * pg->conic[1];
        float dSx = dL_dG * -dG_ddelx;
        float dSy = dL_dG * -dG_ddely;
        float z = pg->depth;
        float txtz = pg->view_pos_xy[0] / z;
        float tytz = pg->view_pos_xy[1] / z;
        float dV[3];
        dV[0] = dSx * fx / z;
        dV[1] = dSy * fy / z;
        dV[2] = -dSx * fx * txtz / z - dSy * fy * tytz / z;
        /* transpose(viewRot) * dV */
        mat3 vrT = mat3_transpose(&viewRot);
        float dW[3];
        for (int i = 0; i < 3; i++) {
            float sacc = vrT.m[0][i] * dV[0];
            sacc = sacc + vrT.m[1][i] * dV[1];
            sacc = sacc + vrT.m[2][i] * dV[2];
            dW[i] = sacc;
        }
        float dCo[3];
        dCo[0] = -0.5f * dL_dG * G * dx * dx;
        dCo[1] = -0.5f * dL_dG * G * 2.0f * dx * dy;
        dCo[2] = -0.5f * dL_dG * G * dy * dy;
        float ca = pg->cov2d[0], cb = pg->cov2d[1], cc = pg->cov2d[2];
        float denom = ca * cc - cb * cb;
        float denom2inv = 1.0f / ((denom * denom) + 0.0000001f);
        float dCv[3];
        dCv[0] = denom2inv * (-cc * cc * dCo[0] + 2.0f * cb * cc * dCo[1] + (denom - ca * cc) * dCo[2]);
        dCv[2] = denom2inv * (-ca * ca * dCo[2] + 2.0f * ca * cb * dCo[1] + (denom - ca * cc) * dCo[0]);
        dCv[1] = denom2inv * 2.0f * (cb * cc * dCo[0] - (denom + 2.0f * cb * cb) * dCo[1] + ca * cb * dCo[2]);
        float tx = pg->view_pos_xy[0] / z, ty = pg->view_pos_xy[1] / z;
        float J00 = fx / z, J02 = -fx * tx / z, J11 = fy / z, J12 = -fy * ty / z;
        mat3 J;
        memset(&J, 0, sizeof(J));
        J.m[0][0] = J00; J.m[1][1] = J11; J.m[2][0] = J02; J.m[2][1] = J12;
        mat3 Tm = mat3_mul(&J, &viewRot);
        mat3 dC2;
        memset(&dC2, 0, sizeof(dC2));
        dC2.m[0][0] = dCv[0]; dC2.m[0][1] = dCv[1];
        dC2.m[1][0] = dCv[1]; dC2.m[1][1] = dCv[2];
        mat3 TmT = mat3_transpose(&Tm);
        mat3 tmp = mat3_mul(&TmT, &dC2);
        mat3 dC3 = mat3_mul(&tmp, &Tm);
        const GsGaussian* go = &g[gi];
        float sc[3];
        for (int k = 0; k < 3; k++) sc[k] = gso_expf(clampf(go->scale[k], -REF_MAX_SCALE, REF_MAX_SCALE));
        float qr = go->rotation[0], qx = go->rotation[1], qy = go->rotation[2], qz = go->rotation[3];
        mat3 R = quat_to_mat(go->rotation);
        mat3 S;
        memset(&S, 0, sizeof(S));
        S.m[0][0] = sc[0]; S.m[1][1] = sc[1]; S.m[2][2] = sc[2];
        mat3 M = mat3_mul(&R, &S);
        mat3 dC3x2 = mat3_scale(&dC3, 2.0f);
        mat3 dM = mat3_mul(&dC3x2, &M);
        mat3 Rt = mat3_transpose(&R);
        mat3 RtdM = mat3_mul(&Rt, &dM);
        float dLS[3] = {RtdM.m[0][0] * sc[0], RtdM.m[1][1] * sc[1], RtdM.m[2][2] * sc[2]};
        mat3 dR;
        for (int c = 0; c < 3; c++)
            for (int r = 0; r < 3; r++) dR.m[c][r] = dM.m[c][r] * sc[c];
        mat3 m = mat3_transpose(&dR);
        float dq[4];
        dq[0] = 2.0f * (qz * (m.m[0][1] - m.m[1][0]) + qy * (m.m[2][0] - m.m[0][2]) +
                        qx * (m.m[1][2] - m.m[2][1]));
        dq[1] = 2.0f * (qy * (m.m[1][0] + m.m[0][1]) + qz * (m.m[2][0] + m.m[0][2]) +
                        qr * (m.m[1][2] - m.m[2][1]) - 2.0f * qx * (m.m[2][2] + m.m[1][1]));
        dq[2] = 2.0f * (qx * (m.m[1][0] + m.m[0][1]) + qr * (m.m[2][0] - m.m[0][2]) +
                        qz * (m.m[1][2] + m.m[2][1]) - 2.0f * qy * (m.m[2][2] + m.m[0][0]));
        dq[3] = 2.0f * (qr * (m.m[0][1] - m.m[1][0]) + qx * (m.m[2][0] + m.m[0][2]) +
                        qy * (m.m[1][2] + m.m[2][1]) - 2.0f * qz * (m.m[1][1] + m.m[0][0]));
        /* :699-736 the 16 atomics */
        float terms[16] = {dLc[0] * REF_SH_C0, dLc[1] * REF_SH_C0, dLc[2] * REF_SH_C0,
                           dL_dRawOp, dW[0], dW[1], dW[2], dSx, dSy,
                           dLS[0], dLS[1], dLS[2], dq[0], dq[1], dq[2], dq[3]};
        static const int field[16] = {GF_SH0, GF_SH4, GF_SH8, GF_OP, GF_PX, GF_PY, GF_PZ,
                                      GF_VX, GF_VY, GF_SX, GF_SY, GF_SZ, GF_QW, GF_QX, GF_QY,
                                      GF_QZ};
        double* a = acc + (size_t)gi * GF_NFLOATS;
        double* ab = absacc ? absacc + (size_t)gi * GF_NFLOATS : NULL;
        double* nz = noiseacc ? noiseacc + (size_t)gi * GF_NFLOATS : NULL;
        double* sh = shadowacc ? shadowacc + (size_t)gi * GF_NFLOATS : NULL;
        double* cd = condacc ? condacc + (size_t)gi * GF_NFLOATS : NULL;
        double dterms[16];
        if (nz || sh) {
            const double Gd = exp((double)power);
            const double ad = fmin((double)pg->opacity * Gd, 0.99);
            Td = Td / fmax(1.0 - ad, 0.0001);
            double ddd = 0.0;
            for (int k = 0; k < 3; k++) ddd += (double)dLp[k] * ((double)pg->color[k] - accd[k]);
            for (int k = 0; k < 3; k++) accd[k] = ad * (double)pg->color[k] + (1.0 - ad) * accd[k];
            chain_terms_double(pg, go, u, dLp, ad * Td, Td * ddd, Gd, dx, dy, dterms);
        }
        for (int k = 0; k < 16; k++) {
            a[field[k]] += (double)terms[k];
            if (ab) ab[field[k]] += fabs((double)terms[k]);
            if (nz) nz[field[k]] += fabs((double)terms[k] - dterms[k]);
            if (sh) sh[field[k]] += dterms[k];
            if (cd) cd[field[k]] += fabs((double)terms[k]) * (k < 3 ? r_col : r_alpha);
        }
    }
}

/* Sums per Gaussian field over all pixels: out[0] the float terms (the reference's values),
 * out[1] |float term|, out[2] |float term - fp64 term|, out[3] the fp64 shadow terms (finite where
 * a float intermediate of the reference overflows). NULL outputs are skipped (out[0] required). */
static void backward_impl(const GsGaussian* g, const GsProjected* p, uint32_t n,
                          const uint32_t* sorted_values, const GsTileRange* ranges,
                          const GsTiledUniforms* u, uint32_t w, uint32_t h, const uint32_t* last_idx,
                          const uint32_t* rendered_rgba8, const uint32_t* gt_rgba8, double* out[5],
                          int threads) {
    int nt = threads > 0 ? threads : 1;
    size_t per = (size_t)n * GF_NFLOATS;
    for (int k = 0; k < 5; k++)
        if (out[k]) memset(out[k], 0, per * sizeof(double));
    uint32_t sw = (uint32_t)u->screen_size[0], shh = (uint32_t)u->screen_size[1];
    uint32_t rows = h < shh ? h : shh, cols = w < sw ? w : sw;
    if (nt == 1) {
        for (uint32_t y = 0; y < rows; y++)
            for (uint32_t x = 0; x < cols; x++)
                backward_pixel(g, p, n, sorted_values, ranges, u, x, y, last_idx,
                               rendered_rgba8, gt_rgba8, out[0], out[1], out[2], out[3], out[4]);
        return;
    }
    /* per-thread double accumulators over static row blocks, summed in thread order */
    double* tacc[5];
    for (int k = 0; k < 5; k++)
        tacc[k] = out[k] ? (double*)calloc((size_t)nt * per, sizeof(double)) : NULL;
#pragma omp parallel for schedule(static, 1) num_threads(nt)
    for (int t = 0; t < nt; t++) {
        uint32_t y0 = (uint32_t)(((uint64_t)rows * (uint64_t)t) / (uint64_t)nt);
        uint32_t y1 = (uint32_t)(((uint64_t)rows * (uint64_t)(t + 1)) / (uint64_t)nt);
        double* mine[5];
        for (int k = 0; k < 5; k++) mine[k] = tacc[k] ? tacc[k] + (size_t)t * per : NULL;
        for (uint32_t y = y0; y < y1; y++)
            for (uint32_t x = 0; x < cols; x++)
                backward_pixel(g, p, n, sorted_values, ranges, u, x, y, last_idx,
                               rendered_rgba8, gt_rgba8, mine[0], mine[1], mine[2], mine[3], mine[4]);
    }
    for (int k = 0; k < 5; k++) {
        if (!out[k]) continue;
        const double* ta = tacc[k];
        double* o = out[k];
#pragma omp parallel for schedule(static) num_threads(nt)
        for (int64_t i = 0; i < (int64_t)per; i++) {
            double s = 0.0;
            for (int t = 0; t < nt; t++) s += ta[(size_t)t * per + (size_t)i];
            o[i] = s;
        }
        free(tacc[k]);
    }
}

void gso_backward(const GsGaussian* g, const GsProjected* p, uint32_t n,
                  const uint32_t* sorted_values, const GsTileRange* ranges,
                  const GsTiledUniforms* u, uint32_t w, uint32_t h, const uint32_t* last_idx,
                  const uint32_t* rendered_rgba8, const uint32_t* gt_rgba8, double* grad_out,
                  double* abs_out, double* noise_out, int threads) {
    double* out[5] = {grad_out, abs_out, noise_out, NULL, NULL};
    backward_impl(g, p, n, sorted_values, ranges, u, w, h, last_idx, rendered_rgba8, gt_rgba8, out,
                  threads);
}

/* The fp64 shadow of gso_backward: each per-pixel term recomputed in double from the same float
 * inputs (G, T, accum in fp64), summed. Where a float intermediate of the reference overflows
 * (huge splats: inf - inf in the dSigma chain) the float sum is NaN and this one is finite. */
void gso_backward_shadow(const GsGaussian* g, const GsProjected* p, uint32_t n,
                         const uint32_t* sorted_values, const GsTileRange* ranges,
                         const GsTiledUniforms* u, uint32_t w, uint32_t h, const uint32_t* last_idx,
                         const uint32_t* rendered_rgba8, const uint32_t* gt_rgba8, double* grad_out,
                         double* shadow_out, int threads) {
    double* out[5] = {grad_out, NULL, NULL, shadow_out, NULL};
    backward_impl(g, p, n, sorted_values, ranges, u, w, h, last_idx, rendered_rgba8, gt_rgba8, out,
                  threads);
}

/* All sums of one pass: the float terms, |float term|, the rounding noise, the fp64 shadow and the
 * conditioning bound (NULL outputs skipped; grad_out required). */
void gso_backward_full(const GsGaussian* g, const GsProjected* p, uint32_t n,
                       const uint32_t* sorted_values, const GsTileRange* ranges,
                       const GsTiledUniforms* u, uint32_t w, uint32_t h, const uint32_t* last_idx,
                       const uint32_t* rendered_rgba8, const uint32_t* gt_rgba8, double* grad_out,
                       double* abs_out, double* noise_out, double* shadow_out, double* cond_out,
                       int threads) {
    double* out[5] = {grad_out, abs_out, noise_out, shadow_out, cond_out};
    backward_impl(g, p, n, sorted_values, ranges, u, w, h, last_idx, rendered_rgba8, gt_rgba8, out,
                  threads);
}

/* tiled_rasterizer.mm:275-672 */
uint64_t gso_forward(const GsGaussian* g, uint32_t n, const GsTiledUniforms* u_in, uint32_t w,
                     uint32_t h, uint64_t max_pairs, GsProjected* proj, uint64_t* keys,
                     uint32_t* values, GsTileRange* ranges, uint32_t* last_idx, uint32_t* rgba8,
                     float* rgb_f32, int threads) {
    GsTiledUniforms u = *u_in;
    u.num_tiles_x = (w + REF_TILE - 1u) / REF_TILE;
    u.num_tiles_y = (h + REF_TILE - 1u) / REF_TILE;
    u.num_gaussians = n;
    uint32_t num_tiles = u.num_tiles_x * u.num_tiles_y;
    memset(last_idx, 0xff, (size_t)w * h * sizeof(uint32_t));
    gso_project(g, n, &u, proj, threads);
    uint64_t total = gso_generate_pairs(proj, n, u.num_tiles_x, max_pairs, keys, values);
    if (total > max_pairs) total = max_pairs;
    if (total == 0) {
        memset(ranges, 0, (size_t)num_tiles * sizeof(GsTileRange));
        return 0;
    }
    gso_sort_pairs(keys, values, total, threads);
    gso_build_tile_ranges(keys, total, num_tiles, ranges, threads);
    gso_forward_blend(proj, n, values, ranges, &u, w, h, last_idx, rgba8, rgb_f32, threads);
    return total;
}

/* density_control.mm:121-185 */
void gso_density_accumulate(const GsGradients* grads, uint32_t n, float* accum, uint32_t* count,
                            float* pos_accum) {
    for (uint32_t i = 0; i < n; i++) {
        float gm = sqrtf(grads[i].viewspace[0] * grads[i].viewspace[0] +
                         grads[i].viewspace[1] * grads[i].viewspace[1]);
        gm = (1.0f < gm) ? 1.0f : gm; /* std::min(gradMag, 1.0f): NaN stays NaN */
        if (!isnan(gm) && !isinf(gm) && gm > 0.0f) {
            accum[i] += gm;
            count[i]++;
            pos_accum[3 * i + 0] += grads[i].position[0];
            pos_accum[3 * i + 1] += grads[i].position[1];
            pos_accum[3 * i + 2] += grads[i].position[2];
        }
    }
}

/* counter-based replacement for rand() in density_control.mm:440-442 */
float gso_density_uniform(uint64_t seed, uint64_t index, uint32_t component) {
    uint64_t z = seed + (index * 3u + component + 1u) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z = z ^ (z >> 31);
    float uu = (float)(z >> 40) * 5.9604644775390625e-08f; /* [0, 1) */
    return (uu - 0.5f) * 2.0f;
}

#define DC_GRAD_THRESHOLD 0.0002f /* density_control.mm:21 */
#define DC_OPACITY_PRUNE 0.005f   /* :24 */
#define DC_PERCENT_DENSE 0.01f    /* :26 */
#define DC_FROM 500u              /* :29 */
#define DC_UNTIL 15000u           /* :31 */
#define DC_MAX_SCALE_LOG 4.0f     /* :33 */
#define DC_RESET_INTERVAL 3000u   /* :35 */
/* logf(1.0f / 1.6f) (density_control.mm:425-426), pinned as a constant */
#define DC_LOG_SPLIT (-0.47000363f)

static float dc_max_scale(const GsGaussian* g) {
    return fmaxf(fmaxf(gso_expf(clampf(g->scale[0], -DC_MAX_SCALE_LOG, DC_MAX_SCALE_LOG)),
                       gso_expf(clampf(g->scale[1], -DC_MAX_SCALE_LOG, DC_MAX_SCALE_LOG))),
                 gso_expf(clampf(g->scale[2], -DC_MAX_SCALE_LOG, DC_MAX_SCALE_LOG)));
}

/* density_control.mm:188-501 */
uint64_t gso_density_apply(const GsGaussian* in, uint32_t n, const float* accum,
                           const uint32_t* count, uint64_t iteration, float scene_extent,
                           float focal, float image_width, float avg_depth, uint64_t seed,
                           uint64_t max_gaussians, GsGaussian* out, uint32_t* markers_out,
                           GsDensityStats* stats) {
    GsDensityStats st = {0, 0, 0, 0};
    if (iteration >= DC_UNTIL) {
        memcpy(out, in, (size_t)n * sizeof(GsGaussian));
        if (stats) *stats = st;
        if (markers_out) memset(markers_out, 0, (size_t)n * sizeof(uint32_t));
        return n;
    }
    int can_densify = iteration > DC_FROM && iteration < DC_UNTIL;
    int screen_prune = iteration > DC_RESET_INTERVAL;
    float split_thr = DC_PERCENT_DENSE * scene_extent;
    float prune_thr = 0.1f * scene_extent;
    uint32_t* mk = (uint32_t*)malloc((size_t)(n ? n : 1) * sizeof(uint32_t));
    for (uint32_t i = 0; i < n; i++) {
        const GsGaussian* g = &in[i];
        float opacity = 1.0f / (1.0f + gso_expf(-g->opacity));
        float avg_grad = count[i] > 0 ? accum[i] / (float)count[i] : 0.0f;
        float max_s = dc_max_scale(g);
        int prune = opacity < DC_OPACITY_PRUNE;
        if (screen_prune) {
            if (max_s > prune_thr) prune = 1;
            /* computeApproxScreenRadius (density_control.mm:56-76) */
            float safe_depth = fmaxf(avg_depth, 0.1f);
            float screen_r = focal * max_s * 3.0f / safe_depth;
            float frac = screen_r / image_width;
            if (frac * image_width > 40.0f) prune = 1;
        }
        if (prune) { mk[i] = 1; st.num_pruned++; }
        else if (can_densify && avg_grad > DC_GRAD_THRESHOLD) {
            if (max_s > split_thr) { mk[i] = 3; st.num_split++; }
            else { mk[i] = 2; st.num_cloned++; }
        } else mk[i] = 0;
    }
    uint64_t new_count = (uint64_t)n - st.num_pruned + st.num_cloned + st.num_split;
    if (max_gaussians > 0 && new_count > max_gaussians) { /* :360-382 */
        uint64_t excess = new_count - max_gaussians;
        for (uint32_t i = 0; i < n && excess > 0; i++)
            if (mk[i] == 2) { mk[i] = 0; st.num_cloned--; excess--; }
        for (uint32_t i = 0; i < n && excess > 0; i++)
            if (mk[i] == 3) { mk[i] = 0; st.num_split--; excess--; }
    }
    uint64_t w = 0;
    for (uint32_t i = 0; i < n; i++) {
        const GsGaussian* g = &in[i];
        uint32_t m = mk[i];
        if (m == 1) continue;
        if (m == 0) { out[w++] = *g; continue; }
        if (m == 2) { out[w++] = *g; out[w++] = *g; continue; }
        float sc[3];
        for (int k = 0; k < 3; k++) sc[k] = gso_expf(clampf(g->scale[k], -DC_MAX_SCALE_LOG, DC_MAX_SCALE_LOG));
        float rx = gso_density_uniform(seed, i, 0);
        float ry = gso_density_uniform(seed, i, 1);
        float rz = gso_density_uniform(seed, i, 2);
        float rn = sqrtf(rx * rx + ry * ry + rz * rz);
        if (rn > 0.001f) { rx /= rn; ry /= rn; rz /= rn; }
        float off[3] = {rx * sc[0], ry * sc[1], rz * sc[2]};
        mat3 R = quat_to_mat(g->rotation);
        float ro[3];
        for (int r = 0; r < 3; r++) { /* simd_mul(R, v) = sum_k column_k * v_k */
            float s = R.m[0][r] * off[0];
            s = s + R.m[1][r] * off[1];
            s = s + R.m[2][r] * off[2];
            ro[r] = s;
        }
        GsGaussian c1 = *g, c2 = *g;
        for (int k = 0; k < 3; k++) {
            c1.position[k] = g->position[k] + ro[k];
            c2.position[k] = g->position[k] - ro[k];
            c1.scale[k] = g->scale[k] + DC_LOG_SPLIT;
            c2.scale[k] = c1.scale[k];
        }
        out[w++] = c1;
        out[w++] = c2;
    }
    if (markers_out) memcpy(markers_out, mk, (size_t)n * sizeof(uint32_t));
    free(mk);
    if (stats) *stats = st;
    return w;
}

/* ----------------------------------------------------------------------------------
 * Adam (shaders.metal:536-713). Metal float3/float4 arithmetic is per component; length() is
 * sqrt of the dot product accumulated x, y, z(, w) in order; clamp(x, a, b) = fmin(fmax(x, a), b).
 * ---------------------------------------------------------------------------------- */
static float ref_clamp(float x, float a, float b) { return fminf(fmaxf(x, a), b); }

void gso_adam_step(GsGaussian* gs, const GsGradients* grads, uint32_t n, float* m_pos, float* m_scale,
                   float* m_rot, float* m_op, float* m_sh, float* v_pos, float* v_scale, float* v_rot,
                   float* v_op, float* v_sh, const float lrs[5], float beta1, float beta2, float eps,
                   float bc1, float bc2) {
    const float clip = 0.5f; /* :582 */
    for (uint32_t tid = 0; tid < n; tid++) {
        const GsGradients* g = &grads[tid];
        GsGaussian* G = &gs[tid];
        /* :566-576 */
        if (isnan(g->position[0]) || isnan(g->opacity) || isnan(g->sh[0]) || isinf(g->position[0]) ||
            isinf(g->opacity))
            continue;
        if (isnan(G->position[0]) || isinf(G->position[0]) || fabsf(G->position[0]) > 1e6f) continue;
        { /* position :585-627 */
            float grad[3], m[3], v[3], upd[3];
            for (int k = 0; k < 3; k++) {
                grad[k] = ref_clamp(g->position[k], -clip, clip);
                m[k] = beta1 * m_pos[tid * 3 + k] + (1.0f - beta1) * grad[k];
                v[k] = beta2 * v_pos[tid * 3 + k] + (1.0f - beta2) * grad[k] * grad[k];
                m_pos[tid * 3 + k] = m[k];
                v_pos[tid * 3 + k] = v[k];
            }
            for (int k = 0; k < 3; k++) {
                const float m_hat = m[k] / bc1, v_hat = v[k] / bc2;
                upd[k] = lrs[0] * m_hat / (sqrtf(v_hat) + eps);
            }
            const float mag = sqrtf(upd[0] * upd[0] + upd[1] * upd[1] + upd[2] * upd[2]);
            if (mag > 0.1f)
                for (int k = 0; k < 3; k++) upd[k] = upd[k] * (0.1f / mag);
            float np[3];
            for (int k = 0; k < 3; k++) np[k] = G->position[k] - upd[k];
            if (!isnan(np[0]) && !isnan(np[1]) && !isnan(np[2]) && fabsf(np[0]) < 1e6f &&
                fabsf(np[1]) < 1e6f && fabsf(np[2]) < 1e6f)
                for (int k = 0; k < 3; k++) G->position[k] = np[k];
        }
        for (int k = 0; k < 3; k++) { /* log-scale :632-656, MAX_SCALE_TRAIN = 4 (:55) */
            const float grad = ref_clamp(g->scale[k], -clip, clip);
            const float m = beta1 * m_scale[tid * 3 + k] + (1.0f - beta1) * grad;
            const float v = beta2 * v_scale[tid * 3 + k] + (1.0f - beta2) * grad * grad;
            m_scale[tid * 3 + k] = m;
            v_scale[tid * 3 + k] = v;
            const float m_hat = m / bc1, v_hat = v / bc2;
            const float ns = G->scale[k] - lrs[1] * m_hat / (sqrtf(v_hat) + eps);
            G->scale[k] = ref_clamp(ns, -4.0f, 4.0f);
        }
        { /* rotation :659-673 */
            float nr[4];
            for (int k = 0; k < 4; k++) {
                const float grad = ref_clamp(g->rotation[k], -clip, clip);
                const float m = beta1 * m_rot[tid * 4 + k] + (1.0f - beta1) * grad;
                const float v = beta2 * v_rot[tid * 4 + k] + (1.0f - beta2) * grad * grad;
                m_rot[tid * 4 + k] = m;
                v_rot[tid * 4 + k] = v;
                const float m_hat = m / bc1, v_hat = v / bc2;
                nr[k] = G->rotation[k] - lrs[2] * m_hat / (sqrtf(v_hat) + eps);
            }
            const float len = sqrtf(nr[0] * nr[0] + nr[1] * nr[1] + nr[2] * nr[2] + nr[3] * nr[3]);
            if (len > 0.001f) {
                for (int k = 0; k < 4; k++) G->rotation[k] = nr[k] / len;
            } else {
                G->rotation[0] = 1.0f;
                G->rotation[1] = G->rotation[2] = G->rotation[3] = 0.0f;
            }
        }
        { /* raw opacity :676-690 */
            const float grad = ref_clamp(g->opacity, -clip, clip);
            const float m = beta1 * m_op[tid] + (1.0f - beta1) * grad;
            const float v = beta2 * v_op[tid] + (1.0f - beta2) * grad * grad;
            m_op[tid] = m;
            v_op[tid] = v;
            const float m_hat = m / bc1, v_hat = v / bc2;
            G->opacity = ref_clamp(G->opacity - lrs[3] * m_hat / (sqrtf(v_hat) + eps), -8.0f, 8.0f);
        }
        for (int i = 0; i < 12; i++) { /* sh :693-712 */
            const float grad = ref_clamp(g->sh[i], -clip, clip);
            const uint32_t idx = tid * 12 + (uint32_t)i;
            const float m = beta1 * m_sh[idx] + (1.0f - beta1) * grad;
            const float v = beta2 * v_sh[idx] + (1.0f - beta2) * grad * grad;
            m_sh[idx] = m;
            v_sh[idx] = v;
            const float m_hat = m / bc1, v_hat = v / bc2;
            const float nsh = G->sh[i] - lrs[4] * m_hat / (sqrtf(v_hat) + eps);
            G->sh[i] = ref_clamp(nsh, -2.0f, 2.0f);
        }
    }
}

void gso_opacity_reset(GsGaussian* g, uint32_t n, float max_raw) {
    for (uint32_t i = 0; i < n; i++)
        if (g[i].opacity > max_raw) g[i].opacity = max_raw; /* mtl_engine.mm:1182-1184 */
}

/* ----------------------------------------------------------------------------------
 * Loss (shaders.metal:320-510). Texture reads of RGBA8Unorm give c / 255.0f.
 * ---------------------------------------------------------------------------------- */
static float ref_unorm(uint32_t v, int c) { return (float)((v >> (8 * c)) & 0xffu) / 255.0f; }

static float ref_grey(uint32_t v) { return (ref_unorm(v, 0) + ref_unorm(v, 1) + ref_unorm(v, 2)) / 3.0f; }

double gso_loss(const uint32_t* rendered, const uint32_t* gt, uint32_t w, uint32_t h, float lambda,
                float* maps, int threads) {
    const float sigma = 1.5f;
    const float two_sigma_sq = 2.0f * sigma * sigma; /* :393-395 */
    const float C1 = 0.01f * 0.01f, C2 = 0.03f * 0.03f;
    const size_t np = (size_t)w * h;
    double total = 0.0;
#ifdef _OPENMP
#pragma omp parallel for schedule(static) num_threads(threads > 0 ? threads : 1) reduction(+ : total)
#endif
    for (long long yy = 0; yy < (long long)h; yy++) {
        const uint32_t y = (uint32_t)yy;
        for (uint32_t x = 0; x < w; x++) {
            const size_t pix = (size_t)y * w + x;
            /* computeL1Loss :332-334 */
            const uint32_t r = rendered[pix], g = gt[pix];
            const float l1 = (fabsf(ref_unorm(r, 0) - ref_unorm(g, 0)) + fabsf(ref_unorm(r, 1) - ref_unorm(g, 1)) +
                              fabsf(ref_unorm(r, 2) - ref_unorm(g, 2))) / 3.0f;
            /* computeSSIM :398-482 */
            float mu_x = 0.0f, mu_y = 0.0f, weight_sum = 0.0f;
            for (int dy = -5; dy <= 5; dy++)
                for (int dx = -5; dx <= 5; dx++) {
                    int px = (int)x + dx, py = (int)y + dy;
                    px = px < 0 ? 0 : (px > (int)w - 1 ? (int)w - 1 : px);
                    py = py < 0 ? 0 : (py > (int)h - 1 ? (int)h - 1 : py);
                    const float dist_sq = (float)(dx * dx + dy * dy);
                    const float wt = gso_expf(-dist_sq / two_sigma_sq);
                    weight_sum += wt;
                    mu_x += wt * ref_grey(rendered[(size_t)py * w + px]);
                    mu_y += wt * ref_grey(gt[(size_t)py * w + px]);
                }
            mu_x /= weight_sum;
            mu_y /= weight_sum;
            float sx2 = 0.0f, sy2 = 0.0f, sxy = 0.0f;
            weight_sum = 0.0f;
            for (int dy = -5; dy <= 5; dy++)
                for (int dx = -5; dx <= 5; dx++) {
                    int px = (int)x + dx, py = (int)y + dy;
                    px = px < 0 ? 0 : (px > (int)w - 1 ? (int)w - 1 : px);
                    py = py < 0 ? 0 : (py > (int)h - 1 ? (int)h - 1 : py);
                    const float dist_sq = (float)(dx * dx + dy * dy);
                    const float wt = gso_expf(-dist_sq / two_sigma_sq);
                    weight_sum += wt;
                    const float dxv = ref_grey(rendered[(size_t)py * w + px]) - mu_x;
                    const float dyv = ref_grey(gt[(size_t)py * w + px]) - mu_y;
                    sx2 += wt * dxv * dxv;
                    sy2 += wt * dyv * dyv;
                    sxy += wt * dxv * dyv;
                }
            sx2 /= weight_sum;
            sy2 /= weight_sum;
            sxy /= weight_sum;
            const float num = (2.0f * mu_x * mu_y + C1) * (2.0f * sxy + C2);
            const float den = (mu_x * mu_x + mu_y * mu_y + C1) * (sx2 + sy2 + C2);
            const float ssim = num / den;
            const float dssim = fminf(fmaxf((1.0f - ssim) / 2.0f, 0.0f), 1.0f);
            const float comb = (1.0f - lambda) * l1 + lambda * dssim; /* :508 */
            if (maps) {
                maps[pix] = l1;
                maps[np + pix] = dssim;
                maps[2 * np + pix] = comb;
            }
            total += (double)comb;
        }
    }
    return np ? total / (double)np : 0.0;
}
