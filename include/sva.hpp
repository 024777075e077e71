// sva.hpp -- C++ host mirror of the reference's interface for the stereo hot
// path, layered on the C-ABI in sva.h.  Header-only; no OpenCV, no torch.
//
// It keeps the reference's names, argument meaning and error behaviour so a
// call site in CameraStereoVision.cpp reads the same:
//   Camera               include/Camera.h:6-21, src/Camera.cpp:6-34
//   pairType             include/functions.h:8-19
//   getCameraPairs       src/functions.cpp:148-213 (incl. the :205 quirk, opt-out)
//   getGroups            src/functions.cpp:107-116
//   bresenham            src/functions.cpp:253-321
//   getAbsDiff           src/functions.cpp:215-218 (on raw 8-bit views)
//   computeDisparity     NEW: replaces the inline hot loop
//                        src/CameraStereoVision.cpp:44-95 with one GPU call
//   disparityToDepth     src/CameraStereoVision.cpp:47,98-100
//   getIdealRef / saveImage / loadImage / calculateAverageError
//                        src/functions.cpp:323-354 (OpenCV-YAML matrix files),
//   refError             src/CameraStereoVision.cpp:107-110,118-119
// Host-side helpers (Camera math, bresenham, pair tables) run on the CPU as in
// the reference -- they are per-call scalars, not the hot path.  Everything
// per-pixel runs on the GPU through sva.h.  Errors are reported as
// sva::Error exceptions on the C++ side (the reference throws cv::Exception on
// bad input); nothing throws across the C-ABI itself.
#pragma once

#include <algorithm>
#include <array>
#include <filesystem>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <sstream>
#include <stdexcept>
#include <string>
#include <vector>

#include "sva.h"

namespace sva {

struct Point2i {
    int x = 0, y = 0;
    Point2i() = default;
    Point2i(int x_, int y_) : x(x_), y(y_) {}
    Point2i operator+(const Point2i& o) const { return {x + o.x, y + o.y}; }
    Point2i operator-(const Point2i& o) const { return {x - o.x, y - o.y}; }
    bool operator==(const Point2i& o) const { return x == o.x && y == o.y; }
};

struct Point3d {
    double x = 0, y = 0, z = 0;
    Point3d() = default;
    Point3d(double x_, double y_, double z_) : x(x_), y(y_), z(z_) {}
    Point3d operator+(const Point3d& o) const { return {x + o.x, y + o.y, z + o.z}; }
    Point3d operator-(const Point3d& o) const { return {x - o.x, y - o.y, z - o.z}; }
    Point3d operator*(double s) const { return {x * s, y * s, z * s}; }
    Point3d operator/(double s) const { return {x / s, y / s, z / s}; }
};

inline double norm(const Point3d& p) { return std::sqrt(p.x * p.x + p.y * p.y + p.z * p.z); }
inline double norm(const Point2i& p) {
    return std::sqrt((double)p.x * p.x + (double)p.y * p.y);
}

struct Error : std::runtime_error {
    int status;
    Error(int s, const std::string& m) : std::runtime_error(m), status(s) {}
};

// class Camera -- include/Camera.h:6-21 (public fields, same constructor).
class Camera {
public:
    Camera(double focal_length, Point3d position, double pixel_size_)
        : pos3D(position), f(focal_length), pixel_size(pixel_size_) {}

    Point3d pos3D;
    double f;
    double pixel_size;

    // Camera::project (src/Camera.cpp:15-21): truncation toward zero.
    Point2i project(Point3d P) const {
        double mult = f / (P.z - pos3D.z) / pixel_size;
        return {int((P.x - pos3D.x) * mult), int((P.y - pos3D.y) * mult)};
    }
    // Camera::inv_project (src/Camera.cpp:25-33).
    Point3d inv_project(Point2i px) const {
        Point3d v{px.x * pixel_size, px.y * pixel_size, f};
        return v / norm(v);
    }
    sva_camera abi() const {
        sva_camera c;
        c.f = f;
        c.pos[0] = pos3D.x;
        c.pos[1] = pos3D.y;
        c.pos[2] = pos3D.z;
        c.pixel_size = pixel_size;
        return c;
    }
};

// include/functions.h:8-19
enum pairType {
    ORTHOGONAL,
    DIAGONAL,
    TO_CENTER,
    LINE_HORIZONTAL,
    LINE_VERTICAL,
    CROSS,
    JUMP_CROSS,
    TO_CENTER_SMALL,
    MID_LEFT,
    MID_TOP
};

// getCameraPairs(cameras, pairType) -- src/functions.cpp:148-197.
inline std::vector<std::array<int, 2>> getCameraPairs(const std::vector<Camera>& cameras,
                                                      const pairType pair) {
    std::vector<std::array<int, 2>> pairs;
    const int n = (int)cameras.size();
    switch (pair) {
        case TO_CENTER:
            for (int i = 0; i < n; i++)
                if (i != 12) pairs.push_back({12, i});
            break;
        case TO_CENTER_SMALL:
            for (int o : {6, 7, 8, 11, 13, 16, 17, 18}) pairs.push_back({12, o});
            break;
        case MID_LEFT: pairs.push_back({12, 11}); break;
        case MID_TOP: pairs.push_back({12, 7}); break;
        case LINE_HORIZONTAL:
            for (int i = 10; i < 15; i++)
                if (i != 12) pairs.push_back({12, i});
            break;
        case LINE_VERTICAL:
            for (int i = 2; i < 25; i += 5)
                if (i != 12) pairs.push_back({12, i});
            break;
        case CROSS:
            for (int o : {11, 13, 7, 17}) pairs.push_back({12, o});
            break;
        case JUMP_CROSS:
            for (int o : {10, 14, 2, 24}) pairs.push_back({12, o});
            break;
        default: break;  // ORTHOGONAL, DIAGONAL: empty in the reference too
    }
    return pairs;
}

// getCameraPairs(cameras, CROSS, cameraNum) -- src/functions.cpp:199-213.
// reference_quirks = true reproduces the reference exactly: the second entry
// is {cameraNum, +5} (the literal camera 5, :205) and the upward neighbour is
// only added for cameraNum - 5 > 0 (:202).  false gives the evident intent.
inline std::vector<std::array<int, 2>> getCameraPairs(const std::vector<Camera>& cameras,
                                                      const pairType pair, int cameraNum,
                                                      bool reference_quirks = true) {
    (void)cameras;
    std::vector<std::array<int, 2>> pairs;
    if (pair != CROSS) return pairs;
    if (reference_quirks ? (cameraNum - 5 > 0) : (cameraNum - 5 >= 0))
        pairs.push_back({cameraNum, cameraNum - 5});
    if (cameraNum + 5 < 25) pairs.push_back({cameraNum, reference_quirks ? 5 : cameraNum + 5});
    if (cameraNum % 5 > 0) pairs.push_back({cameraNum, cameraNum - 1});
    if (cameraNum % 5 < 4) pairs.push_back({cameraNum, cameraNum + 1});
    return pairs;
}

// getGroups -- src/functions.cpp:107-116 ("CHESS": CROSS groups of 0,2,..,24).
inline std::vector<std::vector<std::array<int, 2>>> getGroups(std::vector<Camera>& cameras,
                                                              const std::string& groupType,
                                                              bool reference_quirks = true) {
    std::vector<std::vector<std::array<int, 2>>> groups;
    if (groupType == "CHESS")
        for (int i = 0; i < 25; i += 2)
            groups.push_back(getCameraPairs(cameras, CROSS, i, reference_quirks));
    return groups;
}

// bresenham(point2, point1) -- src/functions.cpp:253-321 (first parameter is
// the caller's pixel1).  Emits from the lower x (|dy| < |dx|) or lower y.
inline std::vector<Point2i> bresenham(Point2i point2, Point2i point1) {
    std::vector<Point2i> pts;
    auto low = [&](int x0, int y0, int x1, int y1) {
        int dx = x1 - x0, dy = y1 - y0, yi = 1;
        if (dy < 0) { yi = -1; dy = -dy; }
        int D = 2 * dy - dx, y = y0;
        for (int x = x0; x <= x1; x++) {
            pts.push_back({x, y});
            if (D > 0) { y += yi; D -= 2 * dx; }
            D += 2 * dy;
        }
    };
    auto high = [&](int x0, int y0, int x1, int y1) {
        int dx = x1 - x0, dy = y1 - y0, xi = 1;
        if (dx < 0) { xi = -1; dx = -dx; }
        int D = 2 * dx - dy, x = x0;
        for (int y = y0; y <= y1; y++) {
            pts.push_back({x, y});
            if (D > 0) { x += xi; D -= 2 * dy; }
            D += 2 * dx;
        }
    };
    if (std::abs(point2.y - point1.y) < std::abs(point2.x - point1.x)) {
        if (point1.x > point2.x) low(point2.x, point2.y, point1.x, point1.y);
        else low(point1.x, point1.y, point2.x, point2.y);
    } else {
        if (point1.y > point2.y) high(point2.x, point2.y, point1.x, point1.y);
        else high(point1.x, point1.y, point2.x, point2.y);
    }
    return pts;
}

// Non-owning 8-bit image view (the part of cv::Mat the path uses).
struct ImageView {
    const uint8_t* data = nullptr;
    int width = 0, height = 0;
    size_t pitch = 0;  // bytes per row
    ImageView() = default;
    ImageView(const uint8_t* d, int w, int h, size_t p = 0)
        : data(d), width(w), height(h), pitch(p ? p : (size_t)w) {}
    ImageView roi(int x, int y, int w, int h) const {
        if (x < 0 || y < 0 || x + w > width || y + h > height)
            throw Error(SVA_ERR_INVALID_ARG, "roi outside image");  // cv::Mat throws here too
        return ImageView(data + (size_t)y * pitch + x, w, h, pitch);
    }
};

// getAbsDiff -- src/functions.cpp:215-218: sum |m1 - m2| as double.
// Compatibility helper for call sites outside the hot path (e.g. one-off
// checks); computeDisparity never calls it -- its SADs run on the GPU.
inline double getAbsDiff(const ImageView& m1, const ImageView& m2) {
    if (m1.width != m2.width || m1.height != m2.height)
        throw Error(SVA_ERR_INVALID_ARG, "getAbsDiff: size mismatch");
    int64_t s = 0;
    for (int v = 0; v < m1.height; v++)
        for (int u = 0; u < m1.width; u++) {
            int d = (int)m1.data[v * m1.pitch + u] - (int)m2.data[v * m2.pitch + u];
            s += d < 0 ? -d : d;
        }
    return (double)s;
}

// RAII owner of one sva context (one device, one stream).
class Engine {
public:
    explicit Engine(int device = 0) {
        int s = sva_create(device, &ctx_);
        if (s != SVA_OK) throw Error(s, std::string("sva_create: ") + sva_status_string(s));
    }
    ~Engine() {
        if (ctx_) sva_destroy(ctx_);
    }
    Engine(const Engine&) = delete;
    Engine& operator=(const Engine&) = delete;
    void* handle() const { return ctx_; }
    void check(int s) const {
        if (s != SVA_OK) throw Error(s, sva_last_error(ctx_));
    }
    // SVA_PATH_KERNEL_AUTO (default) or _COST_VOLUME, the same route (sva.h)
    void setPathKernel(int kernel) { check(sva_set_path_kernel(ctx_, kernel)); }

private:
    void* ctx_ = nullptr;
};

// Result of computeDisparity: the reference's CV_8UC1 map (values wrap mod
// 256, CameraStereoVision.cpp:89), the unwrapped map and a validity mask
// (the reference leaves skipped pixels uninitialised, :46).
struct DisparityMaps {
    int width = 0, height = 0;
    std::vector<uint8_t> disp_u8;
    std::vector<uint16_t> disp_u16;
    std::vector<uint8_t> valid;
};

// Replaces CameraStereoVision.cpp:44-95 (pairs loop incl. last-pair-wins).
// mask may be empty (width 0): every pixel selected.
inline DisparityMaps computeDisparity(Engine& eng, const std::vector<ImageView>& images,
                                      const std::vector<Camera>& cameras,
                                      const std::vector<std::array<int, 2>>& pairs,
                                      const ImageView& mask, int kernelSize,
                                      double t_near = 0.5, double t_far = 1.0) {
    if (pairs.empty()) throw Error(SVA_ERR_INVALID_ARG, "no camera pairs");
    const ImageView& first = images.at(pairs[0][0]);
    DisparityMaps out;
    out.width = first.width;
    out.height = first.height;
    const size_t n = (size_t)first.width * first.height;
    out.disp_u8.assign(n, 0);
    out.disp_u16.assign(n, 0);
    out.valid.assign(n, 0);
    std::vector<uint8_t> mask_dense;
    const uint8_t* mptr = nullptr;
    if (mask.data && mask.width) {
        if (mask.width != first.width || mask.height != first.height)
            throw Error(SVA_ERR_INVALID_ARG, "mask size mismatch");
        mask_dense.resize(n);
        for (int y = 0; y < mask.height; y++)
            for (int x = 0; x < mask.width; x++)
                mask_dense[(size_t)y * mask.width + x] = mask.data[(size_t)y * mask.pitch + x];
        mptr = mask_dense.data();
    }
    for (const auto& pr : pairs) {
        const ImageView& a = images.at(pr[0]);
        const ImageView& b = images.at(pr[1]);
        if (a.width != b.width || a.height != b.height || a.pitch != b.pitch)
            throw Error(SVA_ERR_INVALID_ARG, "pair images differ in size");
        const sva_camera ca = cameras.at(pr[0]).abi(), cb = cameras.at(pr[1]).abi();
        eng.check(sva_disparity_ref(eng.handle(), a.data, b.data, a.width, a.height, a.pitch, mptr,
                                    &ca, &cb, kernelSize, t_near, t_far, out.disp_u8.data(),
                                    out.disp_u16.data(), out.valid.data()));
    }
    return out;
}

// Mode S matcher on one rectified pair (north_star SGM).
inline std::vector<uint16_t> computeDisparitySGM(Engine& eng, const ImageView& left,
                                                 const ImageView& right,
                                                 const sva_sgm_params& p,
                                                 std::vector<float>* subpix = nullptr) {
    if (left.width != right.width || left.height != right.height || left.pitch != right.pitch)
        throw Error(SVA_ERR_INVALID_ARG, "pair images differ in size");
    std::vector<uint16_t> disp((size_t)left.width * left.height);
    float* sp = nullptr;
    if (subpix && p.subpixel) {
        subpix->resize(disp.size());
        sp = subpix->data();
    }
    eng.check(sva_disparity_sgm(eng.handle(), left.data, right.data, left.width, left.height,
                                left.pitch, &p, disp.data(), sp));
    return disp;
}

// CameraStereoVision.cpp:47,98-100 on the GPU (per-pixel f64; reference:
// multiply(disparity, pixelSize, .., CV_64F) then camDistance * f /
// pixSizeDisp, 0 where the divisor is 0).
inline std::vector<double> disparityToDepth(Engine& eng, const std::vector<uint8_t>& disparity,
                                            const Camera& c0, const Camera& c1) {
    const double camDistance = norm(c0.pos3D - c1.pos3D);
    std::vector<double> depth(disparity.size());
    eng.check(sva_disparity_to_depth(eng.handle(), disparity.data(), (int)disparity.size(),
                                     camDistance, c0.f, c0.pixel_size, depth.data()));
    return depth;
}

// ---- camera-array pairs ----------

// Match step of the pair (ref, other) on a planar array with grid pitch
// `pitch` (0.05 m in the reference, CameraStereoVision.cpp:34-39).  Camera
// `other` sits at grid offset g = round((other.pos3D - ref.pos3D) / pitch);
// Camera::project (Camera.cpp:15-21) maps a scene point at pixel q of `ref` to
// q - g * delta in `other`, so the step is -g reduced by the gcd of its
// components.  k = |major component of g|: the disparity along the major axis
// is k * delta and the baseline that converts it to depth is k * pitch.
struct PairStep {
    int dir = 0, dir_y = 0, k = 0;
    double baseline = 0.0;
};

inline PairStep pairStep(const Camera& ref, const Camera& other, double pitch = 0.05) {
    const int gx = (int)std::lround((other.pos3D.x - ref.pos3D.x) / pitch);
    const int gy = (int)std::lround((other.pos3D.y - ref.pos3D.y) / pitch);
    if (gx == 0 && gy == 0) throw Error(SVA_ERR_INVALID_ARG, "pairStep: cameras coincide");
    int a = std::abs(gx), b = std::abs(gy);
    while (b) { const int r = a % b; a = b; b = r; }
    PairStep s;
    s.dir = -gx / a;
    s.dir_y = -gy / a;
    s.k = std::max(std::abs(gx), std::abs(gy));
    s.baseline = s.k * pitch;
    return s;
}

// Mode S on an array pair: base parameters with the pair's step applied.
inline std::vector<uint16_t> computeDisparityPair(Engine& eng, const ImageView& ref,
                                                  const ImageView& other, const PairStep& step,
                                                  sva_sgm_params p) {
    p.dir = step.dir;
    p.dir_y = step.dir_y;
    return computeDisparitySGM(eng, ref, other, p);
}

// Median depth over the maps of one reference camera, f64,
// 0 where no map is valid.  maps[i] is W*H u16, baselines[i] its major-axis
// baseline (PairStep::baseline).
inline std::vector<double> fuseDepth(Engine& eng, const std::vector<std::vector<uint16_t>>& maps,
                                     int W, int H, const std::vector<double>& baselines, double f,
                                     double pixel_size, uint16_t invalid = 0xFFFF,
                                     std::vector<uint8_t>* n_valid = nullptr) {
    const size_t np = (size_t)W * H;
    if (maps.empty() || maps.size() != baselines.size())
        throw Error(SVA_ERR_INVALID_ARG, "fuseDepth: need one baseline per map");
    std::vector<uint16_t> packed(np * maps.size());
    for (size_t i = 0; i < maps.size(); i++) {
        if (maps[i].size() != np) throw Error(SVA_ERR_INVALID_ARG, "fuseDepth: map size");
        std::copy(maps[i].begin(), maps[i].end(), packed.begin() + i * np);
    }
    std::vector<double> depth(np);
    uint8_t* nv = nullptr;
    if (n_valid) {
        n_valid->resize(np);
        nv = n_valid->data();
    }
    eng.check(sva_fuse_depth(eng.handle(), packed.data(), (int)maps.size(), W, H,
                             baselines.data(), f, pixel_size, invalid, depth.data(), nv));
    return depth;
}

// ---- multi-GPU engine (sva.h "multi-GPU engine") ----------

// RAII owner of an sva_multi engine: pairs shard over `devices` (pair j ->
// devices[j mod n]) and over each device's streams; maps are gathered to
// devices[0] by RCCL (default) or peer copies (SVA_MULTI_GATHER_PEER).
class MultiEngine {
public:
    explicit MultiEngine(const std::vector<int>& devices, int streamsPerDevice = 2,
                         int flags = SVA_MULTI_GATHER_RCCL) {
        int s = sva_multi_create(devices.data(), (int)devices.size(), streamsPerDevice, flags, &m_);
        if (s != SVA_OK) throw Error(s, std::string("sva_multi_create: ") + sva_status_string(s));
    }
    ~MultiEngine() {
        if (m_) sva_multi_destroy(m_);
    }
    MultiEngine(const MultiEngine&) = delete;
    MultiEngine& operator=(const MultiEngine&) = delete;
    void* handle() const { return m_; }
    void check(int s) const {
        if (s != SVA_OK) throw Error(s, sva_multi_last_error(m_));
    }
    void synchronize() { check(sva_multi_synchronize(m_)); }

private:
    void* m_ = nullptr;
};

// One camera-array frame over a MultiEngine: replaces the pair loop of
// CameraStereoVision.cpp:55 for Mode S.  Every pair (getCameraPairs,
// functions.cpp:148-213) is matched along its own grid step (pairStep) with
// base parameters p; the maps of each reference camera are fused into one
// median depth map, in the order reference cameras first
// appear in `pairs`.  All images share width, height and pitch; f and
// pixel_size are the first reference camera's.  maps (nullable) receives
// every pair's u16 map in `pairs` order.
inline std::vector<std::vector<double>> computeArrayDepth(
    MultiEngine& m, const std::vector<ImageView>& images, const std::vector<Camera>& cameras,
    const std::vector<std::array<int, 2>>& pairs, const sva_sgm_params& p, double pitch = 0.05,
    std::vector<std::vector<uint16_t>>* maps = nullptr) {
    if (pairs.empty()) throw Error(SVA_ERR_INVALID_ARG, "computeArrayDepth: no camera pairs");
    const ImageView& first = images.at(pairs[0][0]);
    const int W = first.width, H = first.height;
    for (const auto& im : images)
        if (im.width != W || im.height != H || im.pitch != first.pitch)
            throw Error(SVA_ERR_INVALID_ARG, "computeArrayDepth: images differ in size");
    // group the pairs by reference camera (stable: first appearance order)
    std::vector<int> refs;
    for (const auto& pr : pairs)
        if (std::find(refs.begin(), refs.end(), pr[0]) == refs.end()) refs.push_back(pr[0]);
    std::vector<sva_array_pair> ap;
    std::vector<int32_t> group_start;
    std::vector<size_t> order;   // ap index -> index in pairs
    for (int r : refs) {
        group_start.push_back((int32_t)ap.size());
        for (size_t j = 0; j < pairs.size(); j++) {
            if (pairs[j][0] != r) continue;
            const PairStep st = pairStep(cameras.at(pairs[j][0]), cameras.at(pairs[j][1]), pitch);
            sva_array_pair a;
            a.ref = pairs[j][0];
            a.other = pairs[j][1];
            a.params = p;
            a.params.dir = st.dir;
            a.params.dir_y = st.dir_y;
            a.baseline = st.baseline;
            ap.push_back(a);
            order.push_back(j);
        }
    }
    group_start.push_back((int32_t)ap.size());
    std::vector<const uint8_t*> ptrs;
    for (const auto& im : images) ptrs.push_back(im.data);
    const size_t np = (size_t)W * H;
    const int ng = (int)refs.size();
    std::vector<double> depth(np * ng);
    std::vector<uint16_t> all(maps ? np * ap.size() : 0);
    const Camera& c0 = cameras.at(refs[0]);
    m.check(sva_array_depth(m.handle(), ptrs.data(), (int)ptrs.size(), W, H, first.pitch, ap.data(),
                            (int)ap.size(), group_start.data(), ng, c0.f, c0.pixel_size,
                            depth.data(), nullptr, maps ? all.data() : nullptr));
    if (maps) {
        maps->assign(pairs.size(), {});
        for (size_t i = 0; i < ap.size(); i++)
            (*maps)[order[i]].assign(all.begin() + i * np, all.begin() + (i + 1) * np);
    }
    std::vector<std::vector<double>> out(ng);
    for (int g = 0; g < ng; g++) out[g].assign(depth.begin() + g * np, depth.begin() + (g + 1) * np);
    return out;
}

// ---- refinement and 3-D output ----
// The reference's names and argument meaning; cv::Mat becomes ImageView (u8)
// or a dense W*H std::vector<double>.  Pixels a routine does not write keep
// the values of `init` (zeros when omitted) -- the reference leaves them
// uninitialised.

static_assert(sizeof(Point3d) == 3 * sizeof(double), "Point3d must be three packed doubles");

// shiftPerspectiveWithDisparity -- functions.cpp:55-77.
inline std::vector<uint8_t> shiftPerspectiveWithDisparity(Engine& eng, const Camera& inputCam,
                                                          const Camera& outputCam,
                                                          const ImageView& disparity,
                                                          const ImageView& image,
                                                          std::vector<uint8_t> init = {}) {
    if (disparity.width != image.width || disparity.height != image.height ||
        disparity.pitch != image.pitch)
        throw Error(SVA_ERR_INVALID_ARG, "shiftPerspectiveWithDisparity: plane mismatch");
    init.resize((size_t)image.height * image.pitch, 0);
    const sva_camera a = inputCam.abi(), b = outputCam.abi();
    eng.check(sva_shift_perspective(eng.handle(), &a, &b, disparity.data, image.data, image.width,
                                    image.height, image.pitch, init.data()));
    return init;
}

// improveWithDisparity -- functions.cpp:11-52.  `mask` replaces
// getFaceMask(centerImage) (:13; empty view = every pixel).  strict (default,
// as the reference): a masked pixel whose window leaves the image throws
// sva::Error, the analogue of the reference's cv::Exception on that ROI.
inline std::vector<uint8_t> improveWithDisparity(Engine& eng, const ImageView& disparity,
                                                 const ImageView& centerImage,
                                                 const std::vector<ImageView>& images,
                                                 const std::vector<std::array<Camera, 2>>& cameras,
                                                 int windowSize,
                                                 const ImageView& mask = ImageView(),
                                                 bool strict = true,
                                                 std::vector<uint8_t> init = {}) {
    const size_t pitch = centerImage.pitch;
    auto same = [&](const ImageView& v) {
        return v.width == centerImage.width && v.height == centerImage.height && v.pitch == pitch;
    };
    if (!same(disparity) || (mask.data && !same(mask)) || images.size() != cameras.size())
        throw Error(SVA_ERR_INVALID_ARG, "improveWithDisparity: plane or pair mismatch");
    std::vector<const uint8_t*> ptrs;
    std::vector<sva_camera> cams;
    for (size_t i = 0; i < images.size(); i++) {
        if (!same(images[i])) throw Error(SVA_ERR_INVALID_ARG, "improveWithDisparity: image size");
        ptrs.push_back(images[i].data);
        cams.push_back(cameras[i][0].abi());
        cams.push_back(cameras[i][1].abi());
    }
    init.resize((size_t)centerImage.height * pitch, 0);
    eng.check(sva_improve_with_disparity(eng.handle(), disparity.data, centerImage.data,
                                         ptrs.data(), cams.data(), (int)images.size(),
                                         centerImage.width, centerImage.height, pitch, mask.data,
                                         windowSize, strict ? 1 : 0, init.data()));
    return init;
}

// shiftPerspective2 -- functions.cpp:79-103 (depth map W*H f64).
inline std::vector<double> shiftPerspective2(Engine& eng, const Camera& inputCam,
                                             const Camera& outputCam,
                                             const std::vector<double>& depthMap, int W, int H,
                                             std::vector<double> init = {}) {
    if (depthMap.size() != (size_t)W * H) throw Error(SVA_ERR_INVALID_ARG, "depth map size");
    init.resize(depthMap.size(), 0.0);
    const sva_camera a = inputCam.abi(), b = outputCam.abi();
    eng.check(sva_shift_perspective2(eng.handle(), &a, &b, depthMap.data(), W, H, init.data()));
    return init;
}

// Points3DToDepthMap -- functions.cpp:118-132.
inline std::vector<double> Points3DToDepthMap(Engine& eng, const std::vector<Point3d>& points,
                                              const Camera& camera, int W, int H,
                                              std::vector<double> init = {}) {
    init.resize((size_t)W * H, 0.0);
    const sva_camera c = camera.abi();
    eng.check(sva_points_to_depth(eng.handle(), reinterpret_cast<const double*>(points.data()),
                                  (int64_t)points.size(), &c, W, H, init.data()));
    return init;
}

// DepthMapToPoints3D -- functions.cpp:134-146 (column-major order, depth > 0.1).
inline std::vector<Point3d> DepthMapToPoints3D(Engine& eng, const std::vector<double>& depthMap,
                                               const Camera& camera, int W, int H) {
    if (depthMap.size() != (size_t)W * H) throw Error(SVA_ERR_INVALID_ARG, "depth map size");
    std::vector<Point3d> pts((size_t)W * H);
    int64_t n = 0;
    const sva_camera c = camera.abi();
    eng.check(sva_depth_to_points(eng.handle(), depthMap.data(), W, H, &c,
                                  reinterpret_cast<double*>(pts.data()), &n));
    pts.resize((size_t)n);
    return pts;
}

// ---- ingestion ---------------------------------------

// getImagesPathsFromFolder -- functions.cpp:240-250, sorted by file name (the
// reference's directory_iterator order is unspecified).
inline std::vector<std::string> getImagesPathsFromFolder(const std::string& folderPath) {
    std::vector<std::string> filePaths;
    for (auto& p : std::filesystem::directory_iterator(folderPath))
        if (p.is_regular_file()) filePaths.push_back(p.path().u8string());
    std::sort(filePaths.begin(), filePaths.end());
    return filePaths;
}

// resize(img, img, Size(), 0.5, 0.5) -- CameraStereoVision.cpp:18 (INTER_LINEAR
// at exactly 2x = OpenCV's area path), on the GPU.  Returns a dense image of
// *outW x *outH.
inline std::vector<uint8_t> resizeHalf(Engine& eng, const ImageView& img, int* outW, int* outH) {
    int dw = 0, dh = 0;
    eng.check(sva_resize_half_size(img.width, img.height, &dw, &dh));
    std::vector<uint8_t> out((size_t)dw * dh);
    eng.check(sva_resize_half(eng.handle(), img.data, img.width, img.height, img.pitch,
                              out.data(), (size_t)(dw > 0 ? dw : 1)));
    if (outW) *outW = dw;
    if (outH) *outH = dh;
    return out;
}

// ---- evaluation ---------------------------------------

// A matrix of an OpenCV FileStorage "!!opencv-matrix" node: rows x cols x
// channels values of element code dt ('u' 'c' 'w' 's' 'i' 'f' 'd'), held as
// doubles (exact for every one of those types).
struct YamlMatrix {
    int rows = 0, cols = 0, channels = 1;
    char dt = 'd';
    std::vector<double> data;   // row-major, channels interleaved
};

namespace detail {
inline double yaml_number(const std::string& t) {
    if (t == ".Inf" || t == ".inf" || t == "+.Inf") return HUGE_VAL;
    if (t == "-.Inf" || t == "-.inf") return -HUGE_VAL;
    if (t == ".Nan" || t == ".nan" || t == ".NaN") return std::nan("");
    size_t used = 0;
    const double v = std::stod(t, &used);
    if (used != t.size()) throw Error(SVA_ERR_INVALID_ARG, "yaml: bad number '" + t + "'");
    return v;
}
inline std::string yaml_field(const std::string& body, const std::string& name) {
    std::istringstream in(body);
    std::string line;
    while (std::getline(in, line)) {
        const size_t a = line.find_first_not_of(" \t");
        if (a == std::string::npos || a == 0) continue;   // nested fields are indented
        if (line.compare(a, name.size() + 1, name + ":") == 0) {
            std::string v = line.substr(a + name.size() + 1);
            v.erase(0, v.find_first_not_of(" \t\""));
            v.erase(v.find_last_not_of(" \t\"\r") + 1);
            return v;
        }
    }
    throw Error(SVA_ERR_INVALID_ARG, "yaml: missing field " + name);
}
}  // namespace detail

// FileStorage(path, READ)[key] >> Mat for an "!!opencv-matrix" node.
inline YamlMatrix readYamlMatrix(const std::string& path, const std::string& key) {
    std::ifstream f(path);
    if (!f) throw Error(SVA_ERR_INVALID_ARG, "cannot open " + path);
    std::stringstream ss;
    ss << f.rdbuf();
    const std::string text = ss.str();
    const std::string head = key + ":";
    size_t pos = 0, start = std::string::npos;
    while ((pos = text.find(head, pos)) != std::string::npos) {
        const bool bol = pos == 0 || text[pos - 1] == '\n';
        const size_t eol = text.find('\n', pos);
        const std::string rest = text.substr(pos + head.size(), eol - pos - head.size());
        if (bol && rest.find("!!opencv-matrix") != std::string::npos) {
            start = eol;
            break;
        }
        pos += head.size();
    }
    if (start == std::string::npos) throw Error(SVA_ERR_INVALID_ARG, "yaml: no matrix " + key);
    // the node ends at the next unindented line
    size_t end = start;
    while (end < text.size()) {
        const size_t nl = text.find('\n', end + 1);
        const size_t ls = end + 1;
        if (ls < text.size() && text[ls] != ' ' && text[ls] != '\t' && text[ls] != '\n') break;
        if (nl == std::string::npos) { end = text.size(); break; }
        end = nl;
    }
    const std::string body = text.substr(start, end - start);
    YamlMatrix m;
    m.rows = std::stoi(detail::yaml_field(body, "rows"));
    m.cols = std::stoi(detail::yaml_field(body, "cols"));
    const std::string dt = detail::yaml_field(body, "dt");
    if (dt.empty() || std::string("ucwsifd").find(dt.back()) == std::string::npos)
        throw Error(SVA_ERR_INVALID_ARG, "yaml: unsupported dt " + dt);
    m.dt = dt.back();
    m.channels = dt.size() > 1 ? std::stoi(dt.substr(0, dt.size() - 1)) : 1;
    const size_t lb = body.find('['), rb = body.find(']', lb);
    if (lb == std::string::npos || rb == std::string::npos)
        throw Error(SVA_ERR_INVALID_ARG, "yaml: missing data");
    std::string tok;
    for (size_t i = lb + 1; i <= rb; i++) {
        const char ch = body[i];
        if (ch == ',' || ch == ']' || ch == ' ' || ch == '\n' || ch == '\t' || ch == '\r') {
            if (!tok.empty()) m.data.push_back(detail::yaml_number(tok));
            tok.clear();
        } else {
            tok += ch;
        }
    }
    if (m.data.size() != (size_t)m.rows * m.cols * m.channels)
        throw Error(SVA_ERR_INVALID_ARG, "yaml: data size does not match rows x cols");
    return m;
}

// FileStorage(path, WRITE) << key << Mat (a new file holding one node).
inline void writeYamlMatrix(const std::string& path, const std::string& key, const YamlMatrix& m) {
    if (m.data.size() != (size_t)m.rows * m.cols * m.channels)
        throw Error(SVA_ERR_INVALID_ARG, "yaml: data size does not match rows x cols");
    std::ofstream f(path);
    if (!f) throw Error(SVA_ERR_INVALID_ARG, "cannot write " + path);
    f << "%YAML:1.0\n---\n" << key << ": !!opencv-matrix\n   rows: " << m.rows
      << "\n   cols: " << m.cols << "\n   dt: ";
    if (m.channels > 1) f << m.channels;
    f << m.dt << "\n   data: [ ";
    const bool fl = m.dt == 'f' || m.dt == 'd';
    char buf[64];
    for (size_t i = 0; i < m.data.size(); i++) {
        const double v = m.data[i];
        if (fl && std::isnan(v)) std::snprintf(buf, sizeof buf, ".Nan");
        else if (fl && std::isinf(v)) std::snprintf(buf, sizeof buf, v > 0 ? ".Inf" : "-.Inf");
        else if (fl) std::snprintf(buf, sizeof buf, m.dt == 'f' ? "%.9g" : "%.17g", v);
        else std::snprintf(buf, sizeof buf, "%lld", (long long)v);
        f << buf << (i + 1 < m.data.size() ? ((i + 1) % 8 ? ", " : ",\n       ") : "");
    }
    f << " ]\n";
}

// getIdealRef -- functions.cpp:323-329 ("idealRef.yml", key "R").
inline YamlMatrix getIdealRef(const std::string& path = "idealRef.yml") {
    return readYamlMatrix(path, "R");
}
// saveImage / loadImage -- functions.cpp:331-346 (key "image").
inline void saveImage(const std::string& filename, const YamlMatrix& image) {
    writeYamlMatrix(filename, "image", image);
}
inline YamlMatrix loadImage(const std::string& filename) { return readYamlMatrix(filename, "image"); }

// resize(src, dst, Size(dw, dh)) INTER_LINEAR on a dense f64 matrix, on the GPU.
inline std::vector<double> resizeLinear(Engine& eng, const std::vector<double>& src, int sw, int sh,
                                        int dw, int dh) {
    if (src.size() != (size_t)sw * sh) throw Error(SVA_ERR_INVALID_ARG, "resize: size mismatch");
    std::vector<double> out((size_t)dw * dh);
    eng.check(sva_resize_linear_f64(eng.handle(), src.data(), sw, sh, out.data(), dw, dh));
    return out;
}

// CameraStereoVision.cpp:107-110,118-119: resize(depth, depth2, ref.size());
// error = (depth2 - ref) * scale -- on the GPU, returned at ref's size.
inline std::vector<double> refError(Engine& eng, const std::vector<double>& depth, int w, int h,
                                    const YamlMatrix& ref, double scale = 50.0) {
    if (depth.size() != (size_t)w * h || ref.channels != 1 ||
        ref.data.size() != (size_t)ref.rows * ref.cols)
        throw Error(SVA_ERR_INVALID_ARG, "refError: size mismatch");
    std::vector<double> err(ref.data.size());
    eng.check(sva_ref_error(eng.handle(), depth.data(), w, h, ref.data.data(), ref.cols, ref.rows,
                            scale, err.data()));
    return err;
}

// calculateAverageError -- functions.cpp:348-354: cv::mean(image, mask)[0] on
// the GPU.  mask (W*H, nullable = all) replaces dlib's getFaceMask.
inline double calculateAverageError(Engine& eng, const std::vector<double>& image, int w, int h,
                                    const std::vector<uint8_t>* mask = nullptr) {
    if (image.size() != (size_t)w * h || (mask && mask->size() != image.size()))
        throw Error(SVA_ERR_INVALID_ARG, "calculateAverageError: size mismatch");
    double mean = 0;
    eng.check(sva_masked_mean(eng.handle(), image.data(), mask ? mask->data() : nullptr, w, h,
                              &mean));
    return mean;
}

}  // namespace sva
