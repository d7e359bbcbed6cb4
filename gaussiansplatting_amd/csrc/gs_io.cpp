// gs_io.cpp — host-side scene formats and initialisation for the hot path's callers
// (SURVEY.md §8f row 4): COLMAP binary model, scene extent, initial Gaussians from the sparse
// points, TiledUniforms of a COLMAP view, 3DGS PLY read/write, PPM dump. Plain C++17 on the host
// (the reference's versions are host C++ too); float arithmetic follows the reference's
// expression order, with no FMA contraction (built -ffp-contract=off).
#include <algorithm>
#include <cctype>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <map>
#include <memory>
#include <new>
#include <sstream>
#include <string>
#include <vector>

#include "../../include/gs_rasterizer.h"

namespace gs {
int io_fail(int code, const std::string& msg);  // gs_capi.cpp (thread-local last error)
}

using gs::io_fail;

struct gs_colmap {
    std::map<uint32_t, GsColmapCamera> cameras;  // the reference keeps a std::map by id
    std::vector<GsColmapImage> images;
    std::vector<GsColmapPoint> points;
};

namespace {

// getParamCount (colmap_loader.cpp:14-23)
int param_count(int model) {
    switch (model) {
        case 0: return 3;
        case 1: return 4;
        case 2: return 4;
        case 3: return 5;
        case 4: return 8;
        default: return 4;
    }
}

template <typename T>
bool rd(std::ifstream& f, T& v) {
    return static_cast<bool>(f.read(reinterpret_cast<char*>(&v), sizeof(T)));
}

// Bytes left between the read position and the end of the file. COLMAP and PLY files are
// untrusted input: every element count read from them is checked against this before it sizes an
// allocation or a loop, so a lying header fails as "truncated" instead of allocating 2^60 rows.
uint64_t bytes_left(std::ifstream& f) {
    const std::streampos here = f.tellg();
    if (here < 0) return 0;
    f.seekg(0, std::ios::end);
    const std::streampos end = f.tellg();
    f.seekg(here);
    return end > here ? (uint64_t)(end - here) : 0;
}

// a * b without wrap-around; false when the product exceeds 2^64 - 1
bool mul_ok(uint64_t a, uint64_t b, uint64_t& out) {
    if (a != 0 && b > UINT64_MAX / a) return false;
    out = a * b;
    return true;
}

// `count` records of at least `min_record` bytes each fit in what is left of the file
bool count_fits(std::ifstream& f, uint64_t count, uint64_t min_record) {
    uint64_t need = 0;
    return mul_ok(count, min_record, need) && need <= bytes_left(f);
}

// skip `n` records of `size` bytes, refusing to seek past the end of the file
bool skip_records(std::ifstream& f, uint64_t n, uint64_t size) {
    uint64_t skip = 0;
    if (!mul_ok(n, size, skip) || skip > bytes_left(f)) return false;
    f.seekg((std::streamoff)skip, std::ios::cur);
    return static_cast<bool>(f);
}

// smallest on-disk record of each COLMAP binary file (colmap_loader.cpp:26-182)
constexpr uint64_t kMinCameraBytes = 4 + 4 + 8 + 8 + 3 * 8;         // id, model, w, h, >= 3 params
constexpr uint64_t kMinImageBytes = 4 + 4 * 8 + 3 * 8 + 4 + 1 + 8;  // id, q, t, camera, "\0", n2d
constexpr uint64_t kMinPointBytes = 8 + 3 * 8 + 3 + 8 + 8;          // id, xyz, rgb, error, track

int load_cameras(const std::string& path, gs_colmap& c) {  // colmap_loader.cpp:26-80
    std::ifstream f(path, std::ios::binary);
    if (!f.is_open()) return io_fail(GS_E_INVALID, "failed to open " + path);
    uint64_t num = 0;
    if (!rd(f, num)) return io_fail(GS_E_INVALID, "truncated " + path);
    if (!count_fits(f, num, kMinCameraBytes))
        return io_fail(GS_E_INVALID, "truncated " + path + ": camera count exceeds the file");
    for (uint64_t i = 0; i < num; i++) {
        uint32_t id = 0;
        int32_t model = 0;
        uint64_t w = 0, h = 0;
        if (!rd(f, id) || !rd(f, model) || !rd(f, w) || !rd(f, h)) return io_fail(GS_E_INVALID, "truncated " + path);
        std::vector<double> p((size_t)param_count(model));
        if (!f.read(reinterpret_cast<char*>(p.data()), (std::streamsize)(sizeof(double) * p.size())))
            return io_fail(GS_E_INVALID, "truncated " + path);
        GsColmapCamera cam{};
        cam.id = id;
        cam.width = (uint32_t)w;
        cam.height = (uint32_t)h;
        cam.model = model;
        if (model == 0 || model == 2 || model == 3) {
            cam.fx = cam.fy = (float)p[0];
            cam.cx = (float)p[1];
            cam.cy = (float)p[2];
        } else {
            cam.fx = (float)p[0];
            cam.fy = (float)p[1];
            cam.cx = (float)p[2];
            cam.cy = (float)p[3];
        }
        c.cameras[id] = cam;
    }
    return GS_OK;
}

int load_images(const std::string& path, gs_colmap& c) {  // colmap_loader.cpp:83-140
    std::ifstream f(path, std::ios::binary);
    if (!f.is_open()) return io_fail(GS_E_INVALID, "failed to open " + path);
    uint64_t num = 0;
    if (!rd(f, num)) return io_fail(GS_E_INVALID, "truncated " + path);
    if (!count_fits(f, num, kMinImageBytes))
        return io_fail(GS_E_INVALID, "truncated " + path + ": image count exceeds the file");
    for (uint64_t i = 0; i < num; i++) {
        uint32_t id = 0, cam = 0;
        double q[4], t[3];
        if (!rd(f, id)) return io_fail(GS_E_INVALID, "truncated " + path);
        for (double& v : q)
            if (!rd(f, v)) return io_fail(GS_E_INVALID, "truncated " + path);
        for (double& v : t)
            if (!rd(f, v)) return io_fail(GS_E_INVALID, "truncated " + path);
        if (!rd(f, cam)) return io_fail(GS_E_INVALID, "truncated " + path);
        std::string name;
        char ch = 0;
        while (f.read(&ch, 1) && ch != '\0') name += ch;
        if (!f) return io_fail(GS_E_INVALID, "truncated " + path + ": unterminated image name");
        uint64_t n2d = 0;
        if (!rd(f, n2d)) return io_fail(GS_E_INVALID, "truncated " + path);
        if (!skip_records(f, n2d, 24))  // x, y (f64) + point3D id (i64) per 2D point
            return io_fail(GS_E_INVALID, "truncated " + path + ": 2D point count exceeds the file");
        GsColmapImage im{};
        im.id = id;
        im.camera_id = cam;
        for (int k = 0; k < 4; k++) im.rotation[k] = (float)q[k];
        for (int k = 0; k < 3; k++) im.translation[k] = (float)t[k];
        std::strncpy(im.name, name.c_str(), sizeof(im.name) - 1);
        c.images.push_back(im);
    }
    return GS_OK;
}

int load_points(const std::string& path, gs_colmap& c) {  // colmap_loader.cpp:143-182
    std::ifstream f(path, std::ios::binary);
    if (!f.is_open()) return io_fail(GS_E_INVALID, "failed to open " + path);
    uint64_t num = 0;
    if (!rd(f, num)) return io_fail(GS_E_INVALID, "truncated " + path);
    if (!count_fits(f, num, kMinPointBytes))
        return io_fail(GS_E_INVALID, "truncated " + path + ": point count exceeds the file");
    c.points.reserve((size_t)num);
    for (uint64_t i = 0; i < num; i++) {
        uint64_t pid = 0, track = 0;
        double x, y, z, err;
        uint8_t r, g, b;
        if (!rd(f, pid) || !rd(f, x) || !rd(f, y) || !rd(f, z) || !rd(f, r) || !rd(f, g) || !rd(f, b) ||
            !rd(f, err) || !rd(f, track))
            return io_fail(GS_E_INVALID, "truncated " + path);
        if (!skip_records(f, track, 8))  // (image id, point2D index) per track element
            return io_fail(GS_E_INVALID, "truncated " + path + ": track length exceeds the file");
        GsColmapPoint p{};
        p.position[0] = (float)x;
        p.position[1] = (float)y;
        p.position[2] = (float)z;
        p.color[0] = r / 255.0f;
        p.color[1] = g / 255.0f;
        p.color[2] = b / 255.0f;
        p.error = (float)err;
        c.points.push_back(p);
    }
    return GS_OK;
}

void camera_position(const GsColmapImage& img, float out[3]) {  // colmap_loader.cpp:200-229
    const float qw = img.rotation[0], qx = img.rotation[1], qy = img.rotation[2], qz = img.rotation[3];
    const float r00 = 1 - 2 * (qy * qy + qz * qz);
    const float r01 = 2 * (qx * qy - qz * qw);
    const float r02 = 2 * (qx * qz + qy * qw);
    const float r10 = 2 * (qx * qy + qz * qw);
    const float r11 = 1 - 2 * (qx * qx + qz * qz);
    const float r12 = 2 * (qy * qz - qx * qw);
    const float r20 = 2 * (qx * qz - qy * qw);
    const float r21 = 2 * (qy * qz + qx * qw);
    const float r22 = 1 - 2 * (qx * qx + qy * qy);
    const float tx = img.translation[0], ty = img.translation[1], tz = img.translation[2];
    out[0] = -(r00 * tx + r10 * ty + r20 * tz);
    out[1] = -(r01 * tx + r11 * ty + r21 * tz);
    out[2] = -(r02 * tx + r12 * ty + r22 * tz);
}

// computeMeanNearestNeighborDistance(points, i, 3) (main.mm:18-57): the 3 smallest distances to
// the other points, summed in the order the reference pops its max-heap (largest first).
float mean_nn3(const std::vector<GsColmapPoint>& pts, size_t idx) {
    float best[3];
    int cnt = 0;
    const float* p = pts[idx].position;
    for (size_t i = 0; i < pts.size(); i++) {
        if (i == idx) continue;
        const float dx = pts[i].position[0] - p[0];
        const float dy = pts[i].position[1] - p[1];
        const float dz = pts[i].position[2] - p[2];
        const float d = std::sqrt(dx * dx + dy * dy + dz * dz);
        if (cnt < 3) {
            best[cnt++] = d;
            std::sort(best, best + cnt);
        } else if (d < best[2]) {
            best[2] = d;
            std::sort(best, best + 3);
        }
    }
    float sum = 0.0f;
    for (int k = cnt - 1; k >= 0; k--) sum += best[k];
    return cnt > 0 ? sum / (float)cnt : 0.1f;
}

void matmul_colmajor(const float* a, const float* b, float* out) {  // (A*B), summed in k order
    for (int j = 0; j < 4; j++)
        for (int i = 0; i < 4; i++) {
            float s = 0.0f;
            for (int k = 0; k < 4; k++) s = s + a[k * 4 + i] * b[j * 4 + k];
            out[j * 4 + i] = s;
        }
}

// ---- PLY ---------------------------------------------------------------------------------
struct PlyProp {
    std::string name;
    int size = 4;
    char kind = 'f';  // 'f' float, 'd' double, 'i' signed int, 'u' unsigned int
};

bool ply_type(const std::string& t, PlyProp& p) {
    if (t == "char" || t == "int8") { p.size = 1; p.kind = 'i'; }
    else if (t == "uchar" || t == "uint8") { p.size = 1; p.kind = 'u'; }
    else if (t == "short" || t == "int16") { p.size = 2; p.kind = 'i'; }
    else if (t == "ushort" || t == "uint16") { p.size = 2; p.kind = 'u'; }
    else if (t == "int" || t == "int32") { p.size = 4; p.kind = 'i'; }
    else if (t == "uint" || t == "uint32") { p.size = 4; p.kind = 'u'; }
    else if (t == "float" || t == "float32") { p.size = 4; p.kind = 'f'; }
    else if (t == "double" || t == "float64") { p.size = 8; p.kind = 'd'; }
    else return false;
    return true;
}

double ply_value(const unsigned char* b, const PlyProp& p) {
    switch (p.kind) {
        case 'f': { float v; std::memcpy(&v, b, 4); return v; }
        case 'd': { double v; std::memcpy(&v, b, 8); return v; }
        case 'i':
            if (p.size == 1) { int8_t v; std::memcpy(&v, b, 1); return v; }
            if (p.size == 2) { int16_t v; std::memcpy(&v, b, 2); return v; }
            { int32_t v; std::memcpy(&v, b, 4); return v; }
        default:
            if (p.size == 1) return b[0];
            if (p.size == 2) { uint16_t v; std::memcpy(&v, b, 2); return v; }
            { uint32_t v; std::memcpy(&v, b, 4); return v; }
    }
}

struct PlyElement {
    std::string name;
    uint64_t count = 0;
    std::vector<PlyProp> props;
    bool has_list = false;
};

int ply_read_vertices(const char* path, std::vector<PlyProp>& props, std::vector<float>& data,
                      uint64_t& count) {
    std::ifstream f(path, std::ios::binary);
    if (!f.is_open()) return io_fail(GS_E_INVALID, std::string("failed to open ") + path);
    std::string line;
    if (!std::getline(f, line) || line.rfind("ply", 0) != 0) return io_fail(GS_E_INVALID, "not a PLY file");
    bool binary = false, ascii = false;
    std::vector<PlyElement> els;
    while (std::getline(f, line)) {
        if (!line.empty() && line.back() == '\r') line.pop_back();
        std::istringstream ss(line);
        std::string tok;
        ss >> tok;
        if (tok == "format") {
            std::string fmt;
            ss >> fmt;
            binary = fmt == "binary_little_endian";
            ascii = fmt == "ascii";
        } else if (tok == "element") {
            PlyElement e;
            ss >> e.name >> e.count;
            els.push_back(e);
        } else if (tok == "property") {
            if (els.empty()) return io_fail(GS_E_INVALID, "PLY property before element");
            std::string t, name;
            ss >> t;
            if (t == "list") {
                els.back().has_list = true;
                continue;
            }
            ss >> name;
            PlyProp p;
            p.name = name;
            if (!ply_type(t, p)) return io_fail(GS_E_INVALID, "unsupported PLY property type " + t);
            els.back().props.push_back(p);
        } else if (tok == "end_header") {
            break;
        }
    }
    if (!binary && !ascii) return io_fail(GS_E_INVALID, "PLY: only binary_little_endian and ascii are supported");
    for (const PlyElement& e : els) {
        if (e.name == "vertex") {
            if (e.has_list) return io_fail(GS_E_INVALID, "PLY: list property in vertex element");
            props = e.props;
            count = e.count;
            const size_t np = props.size();
            size_t stride = 0;
            for (const PlyProp& p : props) stride += (size_t)p.size;
            // the header's count must fit the data that follows it: a binary row is `stride` bytes,
            // an ASCII value at least one character (a digit; the separators between values
            // count too, but the last value of the file need not be followed by one)
            if (!count_fits(f, count, binary ? (uint64_t)stride : (uint64_t)np))
                return io_fail(GS_E_INVALID, "truncated PLY: vertex count exceeds the file");
            uint64_t cells = 0;
            if (!mul_ok(count, (uint64_t)np, cells) || cells > (uint64_t)SIZE_MAX / sizeof(float))
                return io_fail(GS_E_INVALID, "PLY: vertex count too large");
            data.resize((size_t)cells);
            if (binary) {
                std::vector<unsigned char> row(stride);
                for (uint64_t i = 0; i < count; i++) {
                    if (!f.read(reinterpret_cast<char*>(row.data()), (std::streamsize)stride))
                        return io_fail(GS_E_INVALID, "truncated PLY vertex data");
                    size_t o = 0;
                    for (size_t k = 0; k < np; k++) {
                        data[(size_t)i * np + k] = (float)ply_value(row.data() + o, props[k]);
                        o += (size_t)props[k].size;
                    }
                }
            } else {
                for (uint64_t i = 0; i < count; i++)
                    for (size_t k = 0; k < np; k++) {
                        double v;
                        if (!(f >> v)) return io_fail(GS_E_INVALID, "truncated PLY vertex data");
                        data[(size_t)i * np + k] = (float)v;
                    }
            }
            return GS_OK;
        }
        // an element before the vertices: skip its data (fixed-size rows only)
        if (e.has_list) return io_fail(GS_E_INVALID, "PLY: list element before the vertices");
        if (binary) {
            size_t stride = 0;
            for (const PlyProp& p : e.props) stride += (size_t)p.size;
            if (!skip_records(f, e.count, stride))
                return io_fail(GS_E_INVALID, "truncated PLY: element '" + e.name + "' exceeds the file");
        } else {
            for (uint64_t i = 0; i < e.count; i++)
                if (!std::getline(f, line))
                    return io_fail(GS_E_INVALID, "truncated PLY: element '" + e.name + "' exceeds the file");
        }
    }
    return io_fail(GS_E_INVALID, "PLY has no vertex element");
}

// detectLinearScales (ply_loader.cpp:18-56)
bool detect_linear_scales(const std::vector<float>& s, uint64_t count) {
    if (count == 0) return false;
    int pos = 0, neg = 0;
    float mx = -3.402823466e38f, mn = 3.402823466e38f;
    const uint64_t sample = std::min<uint64_t>(count, 1000);
    for (uint64_t i = 0; i < sample; i++)
        for (int j = 0; j < 3; j++) {
            const float v = s[(size_t)i * 3 + j];
            if (v > 0) pos++;
            if (v < 0) neg++;
            mx = std::max(mx, v);
            mn = std::min(mn, v);
        }
    (void)pos;
    if (neg > 0) return false;
    if (mx <= 1.0f && mn > 0.0f) return true;
    return false;
}

// No C++ exception crosses the C-ABI (include/gs_rasterizer.h): a host allocation failure or a
// library error inside an entry point becomes a status code.
template <typename F>
int guarded(const char* who, F&& body) {
    try {
        return body();
    } catch (const std::bad_alloc&) {
        return io_fail(GS_E_NOMEM, std::string(who) + ": host allocation failed");
    } catch (const std::exception& e) {
        return io_fail(GS_E_INVALID, std::string(who) + ": " + e.what());
    } catch (...) {
        return io_fail(GS_E_INVALID, std::string(who) + ": unknown error");
    }
}

}  // namespace

extern "C" {

int gs_colmap_load(const char* dir, gs_colmap** out) {
    return guarded("gs_colmap_load", [&]() -> int {
    if (!dir || !out) return io_fail(GS_E_INVALID, "gs_colmap_load: null argument");
    *out = nullptr;
    std::unique_ptr<gs_colmap> c(new gs_colmap());
    const std::string d(dir);
    int rc;
    if ((rc = load_cameras(d + "/cameras.bin", *c)) != GS_OK || (rc = load_images(d + "/images.bin", *c)) != GS_OK ||
        (rc = load_points(d + "/points3D.bin", *c)) != GS_OK)
        return rc;
    *out = c.release();
    return GS_OK;
    });
}

int gs_colmap_free(gs_colmap* c) {
    delete c;
    return GS_OK;
}

int gs_colmap_counts(const gs_colmap* c, uint32_t* nc, uint32_t* ni, uint64_t* np) {
    if (!c) return io_fail(GS_E_INVALID, "gs_colmap_counts: null handle");
    if (nc) *nc = (uint32_t)c->cameras.size();
    if (ni) *ni = (uint32_t)c->images.size();
    if (np) *np = (uint64_t)c->points.size();
    return GS_OK;
}

int gs_colmap_camera(const gs_colmap* c, uint32_t index, GsColmapCamera* out) {
    if (!c || !out) return io_fail(GS_E_INVALID, "gs_colmap_camera: null argument");
    if (index >= c->cameras.size()) return io_fail(GS_E_INVALID, "gs_colmap_camera: index out of range");
    auto it = c->cameras.begin();
    std::advance(it, index);
    *out = it->second;
    return GS_OK;
}

int gs_colmap_camera_by_id(const gs_colmap* c, uint32_t id, GsColmapCamera* out) {
    if (!c || !out) return io_fail(GS_E_INVALID, "gs_colmap_camera_by_id: null argument");
    auto it = c->cameras.find(id);
    if (it == c->cameras.end()) return io_fail(GS_E_INVALID, "gs_colmap_camera_by_id: no such camera");
    *out = it->second;
    return GS_OK;
}

int gs_colmap_image(const gs_colmap* c, uint32_t index, GsColmapImage* out) {
    if (!c || !out) return io_fail(GS_E_INVALID, "gs_colmap_image: null argument");
    if (index >= c->images.size()) return io_fail(GS_E_INVALID, "gs_colmap_image: index out of range");
    *out = c->images[index];
    return GS_OK;
}

int gs_colmap_points(const gs_colmap* c, GsColmapPoint* out, uint64_t cap) {
    if (!c || (!out && cap)) return io_fail(GS_E_INVALID, "gs_colmap_points: null argument");
    if (cap < c->points.size()) return io_fail(GS_E_INVALID, "gs_colmap_points: cap too small");
    if (!c->points.empty()) std::memcpy(out, c->points.data(), c->points.size() * sizeof(GsColmapPoint));
    return GS_OK;
}

int gs_colmap_camera_position(const GsColmapImage* img, float out_xyz[3]) {
    if (!img || !out_xyz) return io_fail(GS_E_INVALID, "gs_colmap_camera_position: null argument");
    camera_position(*img, out_xyz);
    return GS_OK;
}

int gs_colmap_scene_extent(const gs_colmap* c, float* out) {  // colmap_loader.cpp:232-264
    return guarded("gs_colmap_scene_extent", [&]() -> int {
    if (!c || !out) return io_fail(GS_E_INVALID, "gs_colmap_scene_extent: null argument");
    std::vector<float> pos(c->images.size() * 3);
    for (size_t i = 0; i < c->images.size(); i++) camera_position(c->images[i], &pos[i * 3]);
    float cen[3] = {0.0f, 0.0f, 0.0f};
    for (size_t i = 0; i < c->images.size(); i++)
        for (int k = 0; k < 3; k++) cen[k] += pos[i * 3 + k];
    for (int k = 0; k < 3; k++) cen[k] /= (float)c->images.size();
    float maxd = 0.0f;
    for (size_t i = 0; i < c->images.size(); i++) {
        const float dx = pos[i * 3] - cen[0], dy = pos[i * 3 + 1] - cen[1], dz = pos[i * 3 + 2] - cen[2];
        maxd = std::max(maxd, std::sqrt(dx * dx + dy * dy + dz * dz));
    }
    *out = maxd * 1.1f;
    return GS_OK;
    });
}

int gs_gaussians_from_colmap(const gs_colmap* c, float scene_extent, GsGaussian* out, uint64_t cap,
                             uint64_t* n_out) {
    return guarded("gs_gaussians_from_colmap", [&]() -> int {
    if (!c || !n_out) return io_fail(GS_E_INVALID, "gs_gaussians_from_colmap: null argument");
    const size_t n = c->points.size();
    *n_out = n;
    if (!out) return GS_OK;
    if (cap < n) return io_fail(GS_E_INVALID, "gs_gaussians_from_colmap: cap too small");
    const float kShC0 = 0.28209479177387814f;
    std::vector<float> scales(n);
    if (n > 10000) {  // main.mm:90-111: median over a strided sample
        const size_t sample = std::min<size_t>(1000, n);
        const size_t step = n / sample;
        std::vector<size_t> idx;
        for (size_t i = 0; i < n; i += step) idx.push_back(i);
        std::vector<float> ss(idx.size());
        for (long long k = 0; k < (long long)idx.size(); k++) ss[(size_t)k] = mean_nn3(c->points, idx[(size_t)k]);
        std::sort(ss.begin(), ss.end());
        const float med = ss[ss.size() / 2];
        std::fill(scales.begin(), scales.end(), med);
    } else {
        for (long long i = 0; i < (long long)n; i++) scales[(size_t)i] = mean_nn3(c->points, (size_t)i);
    }
    for (size_t i = 0; i < n; i++) {  // main.mm:124-166
        const GsColmapPoint& pt = c->points[i];
        GsGaussian g;
        std::memset(&g, 0, sizeof(g));
        for (int k = 0; k < 3; k++) g.position[k] = pt.position[k];
        const float mn = 0.0001f * scene_extent, mx = 0.1f * scene_extent;
        const float s = std::clamp(scales[i], mn, mx);
        const float ls = std::log(s);
        for (int k = 0; k < 3; k++) g.scale[k] = ls;
        g.rotation[0] = 1.0f;
        g.opacity = 0.0f;
        g.sh[0] = (pt.color[0] - 0.5f) / kShC0;
        g.sh[4] = (pt.color[1] - 0.5f) / kShC0;
        g.sh[8] = (pt.color[2] - 0.5f) / kShC0;
        out[i] = g;
    }
    return GS_OK;
    });
}

int gs_colmap_uniforms(const GsColmapCamera* cam, const GsColmapImage* img, uint32_t width,
                       uint32_t height, GsTiledUniforms* out) {
    if (!cam || !img || !out) return io_fail(GS_E_INVALID, "gs_colmap_uniforms: null argument");
    if (!width || !height || !cam->width || !cam->height) return io_fail(GS_E_INVALID, "gs_colmap_uniforms: zero size");
    // intrinsics scaled to the render size (mtl_engine.mm:873-881)
    const float sx = (float)width / (float)cam->width, sy = (float)height / (float)cam->height;
    const float fx = cam->fx * sx, fy = cam->fy * sy, cx = cam->cx * sx, cy = cam->cy * sy;
    // viewMatrixFromColmap (:637-659), [col][row]
    const float w = img->rotation[0], x = img->rotation[1], y = img->rotation[2], z = img->rotation[3];
    float view[16] = {0};
    view[0] = 1 - 2 * (y * y + z * z); view[1] = 2 * (x * y + w * z); view[2] = 2 * (x * z - w * y);
    view[4] = 2 * (x * y - w * z); view[5] = 1 - 2 * (x * x + z * z); view[6] = 2 * (y * z + w * x);
    view[8] = 2 * (x * z + w * y); view[9] = 2 * (y * z - w * x); view[10] = 1 - 2 * (x * x + y * y);
    view[12] = img->translation[0]; view[13] = img->translation[1]; view[14] = img->translation[2];
    view[15] = 1.0f;
    // projectionFromColmap (:662-682), near 0.1, far 1000 (:913)
    const float fw = (float)width, fh = (float)height, nz = 0.1f, fz = 1000.0f;
    float proj[16] = {0};
    proj[0] = 2.0f * fx / fw;
    proj[5] = 2.0f * fy / fh;
    proj[8] = 2.0f * cx / fw - 1.0f;
    proj[9] = 2.0f * cy / fh - 1.0f;
    proj[10] = fz / (fz - nz);
    proj[11] = 1.0f;
    proj[14] = -(fz * nz) / (fz - nz);
    std::memset(out, 0, sizeof(*out));
    std::memcpy(out->view, view, sizeof(view));
    std::memcpy(out->proj, proj, sizeof(proj));
    matmul_colmajor(proj, view, out->view_proj);
    out->screen_size[0] = fw;
    out->screen_size[1] = fh;
    out->focal[0] = fx;
    out->focal[1] = fy;
    // cameraPos = -(R^T t) (:918-922)
    for (int i = 0; i < 3; i++)
        out->camera_pos[i] = -(view[i * 4 + 0] * img->translation[0] + view[i * 4 + 1] * img->translation[1] +
                               view[i * 4 + 2] * img->translation[2]);
    out->num_tiles_x = (width + GS_TILE_SIZE - 1) / GS_TILE_SIZE;
    out->num_tiles_y = (height + GS_TILE_SIZE - 1) / GS_TILE_SIZE;
    return GS_OK;
}

int gs_ply_load(const char* path, GsGaussian* out, uint64_t cap, uint64_t* n_out) {
    return guarded("gs_ply_load", [&]() -> int {
    if (!path || !n_out) return io_fail(GS_E_INVALID, "gs_ply_load: null argument");
    std::vector<PlyProp> props;
    std::vector<float> data;
    uint64_t count = 0;
    int rc = ply_read_vertices(path, props, data, count);
    if (rc != GS_OK) return rc;
    auto col = [&](const char* name) -> int {
        for (size_t k = 0; k < props.size(); k++)
            if (props[k].name == name) return (int)k;
        return -1;
    };
    const char* req[] = {"x", "y", "z", "scale_0", "scale_1", "scale_2", "rot_0", "rot_1", "rot_2", "rot_3",
                         "opacity", "f_dc_0", "f_dc_1", "f_dc_2"};
    int ci[14];
    for (int k = 0; k < 14; k++)
        if ((ci[k] = col(req[k])) < 0) return io_fail(GS_E_INVALID, std::string("PLY lacks property ") + req[k]);
    int rest[9];
    bool has_rest = true;
    for (int k = 0; k < 9; k++) {
        const std::string nm = "f_rest_" + std::to_string(k);
        if ((rest[k] = col(nm.c_str())) < 0) has_rest = false;
    }
    const size_t np = props.size();
    auto at = [&](uint64_t i, int k) { return data[(size_t)i * np + (size_t)k]; };
    std::vector<float> sc((size_t)count * 3);
    for (uint64_t i = 0; i < count; i++)
        for (int j = 0; j < 3; j++) sc[(size_t)i * 3 + j] = at(i, ci[3 + j]);
    const bool linear = detect_linear_scales(sc, count);
    uint64_t n = 0;
    for (uint64_t i = 0; i < count; i++) {  // ply_loader.cpp:173-250
        const float px = at(i, ci[0]), py = at(i, ci[1]), pz = at(i, ci[2]);
        if (std::isnan(px) || std::isnan(py) || std::isnan(pz) || std::isinf(px) || std::isinf(py) ||
            std::isinf(pz) || std::fabs(px) > 1e6f || std::fabs(py) > 1e6f || std::fabs(pz) > 1e6f)
            continue;
        if (out) {
            if (n >= cap) return io_fail(GS_E_INVALID, "gs_ply_load: cap too small");
            GsGaussian g;
            std::memset(&g, 0, sizeof(g));
            g.position[0] = px;
            g.position[1] = py;
            g.position[2] = pz;
            for (int j = 0; j < 3; j++) {
                float s = sc[(size_t)i * 3 + j];
                if (linear) s = std::log(std::max(s, 1e-8f));
                g.scale[j] = std::clamp(s, -8.0f, 8.0f);
            }
            float qw = at(i, ci[6]), qx = at(i, ci[7]), qy = at(i, ci[8]), qz = at(i, ci[9]);
            const float ql = std::sqrt(qw * qw + qx * qx + qy * qy + qz * qz);
            if (ql > 0.0001f) {
                qw /= ql; qx /= ql; qy /= ql; qz /= ql;
            } else {
                qw = 1.0f; qx = 0.0f; qy = 0.0f; qz = 0.0f;
            }
            g.rotation[0] = qw; g.rotation[1] = qx; g.rotation[2] = qy; g.rotation[3] = qz;
            g.opacity = at(i, ci[10]);
            g.sh[0] = at(i, ci[11]);
            g.sh[4] = at(i, ci[12]);
            g.sh[8] = at(i, ci[13]);
            if (has_rest) {  // interleaved by coefficient: (R, G, B) of coef 1, 2, 3
                const int map[9] = {1, 5, 9, 2, 6, 10, 3, 7, 11};
                for (int k = 0; k < 9; k++) g.sh[map[k]] = at(i, rest[k]);
            }
            out[n] = g;
        }
        n++;
    }
    *n_out = n;
    return GS_OK;
    });
}

int gs_ply_save(const char* path, const GsGaussian* gs, uint64_t n, uint64_t* n_written) {
    return guarded("gs_ply_save", [&]() -> int {
    if (!path || (n && !gs)) return io_fail(GS_E_INVALID, "gs_ply_save: null argument");
    std::ofstream f(path, std::ios::binary);
    if (!f.is_open()) return io_fail(GS_E_INVALID, std::string("failed to open ") + path + " for writing");
    auto valid = [](const GsGaussian& g) {
        return !std::isnan(g.position[0]) && !std::isinf(g.position[0]) && std::fabs(g.position[0]) < 1e6f;
    };
    uint64_t nv = 0;
    for (uint64_t i = 0; i < n; i++) nv += valid(gs[i]) ? 1 : 0;
    // header exactly as PLYExporter::exportPLY (ply_exporter.hpp:37-75)
    f << "ply\n" << "format binary_little_endian 1.0\n" << "element vertex " << nv << "\n";
    for (const char* p : {"x", "y", "z", "nx", "ny", "nz", "f_dc_0", "f_dc_1", "f_dc_2"}) f << "property float " << p << "\n";
    for (int i = 0; i < 9; i++) f << "property float f_rest_" << i << "\n";
    for (const char* p : {"opacity", "scale_0", "scale_1", "scale_2", "rot_0", "rot_1", "rot_2", "rot_3"})
        f << "property float " << p << "\n";
    f << "end_header\n";
    for (uint64_t i = 0; i < n; i++) {
        const GsGaussian& g = gs[i];
        if (!valid(g)) continue;
        const float row[26] = {g.position[0], g.position[1], g.position[2], 0.0f, 0.0f, 0.0f,
                               g.sh[0], g.sh[4], g.sh[8],
                               g.sh[1], g.sh[5], g.sh[9], g.sh[2], g.sh[6], g.sh[10], g.sh[3], g.sh[7], g.sh[11],
                               g.opacity, g.scale[0], g.scale[1], g.scale[2],
                               g.rotation[0], g.rotation[1], g.rotation[2], g.rotation[3]};
        f.write(reinterpret_cast<const char*>(row), sizeof(row));
    }
    if (!f) return io_fail(GS_E_INVALID, std::string("write failed: ") + path);
    if (n_written) *n_written = nv;
    return GS_OK;
    });
}

int gs_ppm_save(const char* path, const uint32_t* rgba8, uint32_t w, uint32_t h) {
    return guarded("gs_ppm_save", [&]() -> int {
    if (!path || (!rgba8 && w && h)) return io_fail(GS_E_INVALID, "gs_ppm_save: null argument");
    std::ofstream f(path, std::ios::binary);
    if (!f.is_open()) return io_fail(GS_E_INVALID, std::string("failed to open ") + path + " for writing");
    f << "P6\n" << w << " " << h << "\n255\n";
    std::vector<unsigned char> row((size_t)w * 3);
    for (uint32_t y = 0; y < h; y++) {
        for (uint32_t x = 0; x < w; x++) {
            const uint32_t v = rgba8[(size_t)y * w + x];
            row[(size_t)x * 3 + 0] = (unsigned char)(v & 0xffu);
            row[(size_t)x * 3 + 1] = (unsigned char)((v >> 8) & 0xffu);
            row[(size_t)x * 3 + 2] = (unsigned char)((v >> 16) & 0xffu);
        }
        f.write(reinterpret_cast<const char*>(row.data()), (std::streamsize)row.size());
    }
    if (!f) return io_fail(GS_E_INVALID, std::string("write failed: ") + path);
    return GS_OK;
    });
}

// The reference reads its ground-truth images through stb_image (image_loader.mm:13-41, out of scope);
// a P6 PPM (what gs_ppm_save writes) is the headless caller's stand-in for one.
int gs_ppm_load(const char* path, uint32_t* rgba8, uint64_t cap_pixels, uint32_t* w_out, uint32_t* h_out) {
    return guarded("gs_ppm_load", [&]() -> int {
    if (!path || !w_out || !h_out) return io_fail(GS_E_INVALID, "gs_ppm_load: null argument");
    std::ifstream f(path, std::ios::binary);
    if (!f.is_open()) return io_fail(GS_E_INVALID, std::string("failed to open ") + path);
    // header: magic, width, height, maxval, separated by whitespace and '#' comments
    auto token = [&](std::string& t) -> bool {
        t.clear();
        int c;
        while ((c = f.get()) != EOF) {
            if (c == '#') {
                while ((c = f.get()) != EOF && c != '\n') {}
                continue;
            }
            if (!std::isspace(c)) break;
        }
        if (c == EOF) return false;
        t.push_back((char)c);
        while ((c = f.peek()) != EOF && !std::isspace(c) && c != '#') {
            t.push_back((char)f.get());
            if (t.size() > 16) return false;
        }
        return true;
    };
    std::string magic, sw, sh, smax;
    if (!token(magic) || magic != "P6") return io_fail(GS_E_INVALID, std::string("not a binary PPM (P6): ") + path);
    if (!token(sw) || !token(sh) || !token(smax)) return io_fail(GS_E_INVALID, std::string("truncated PPM header: ") + path);
    auto parse = [](const std::string& t, uint64_t lim, uint64_t& v) {
        if (t.empty() || t.size() > 9) return false;
        v = 0;
        for (char ch : t) {
            if (ch < '0' || ch > '9') return false;
            v = v * 10 + (uint64_t)(ch - '0');
        }
        return v >= 1 && v <= lim;
    };
    uint64_t w = 0, h = 0, mx = 0;
    if (!parse(sw, 1u << 16, w) || !parse(sh, 1u << 16, h) || !parse(smax, 65535, mx))
        return io_fail(GS_E_INVALID, std::string("bad PPM header: ") + path);
    if (mx != 255) return io_fail(GS_E_INVALID, std::string("PPM maxval must be 255: ") + path);
    if (f.get() == EOF) return io_fail(GS_E_INVALID, std::string("truncated PPM: ") + path);  // one whitespace
    *w_out = (uint32_t)w;
    *h_out = (uint32_t)h;
    if (!rgba8) return GS_OK;
    if (w * h > cap_pixels) return io_fail(GS_E_INVALID, "gs_ppm_load: image larger than the output");
    std::vector<unsigned char> row((size_t)w * 3);
    for (uint64_t y = 0; y < h; y++) {
        if (!f.read(reinterpret_cast<char*>(row.data()), (std::streamsize)row.size()))
            return io_fail(GS_E_INVALID, std::string("truncated PPM pixel data: ") + path);
        for (uint64_t x = 0; x < w; x++)
            rgba8[y * w + x] = (uint32_t)row[3 * x] | ((uint32_t)row[3 * x + 1] << 8) |
                               ((uint32_t)row[3 * x + 2] << 16) | (255u << 24);
    }
    return GS_OK;
    });
}

}  // extern "C"
