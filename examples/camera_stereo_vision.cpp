// camera_stereo_vision.cpp -- the reference's main() (src/CameraStereoVision.cpp)
// re-expressed on the MI355X engine through include/sva.hpp, as a drop-in
// demonstration: same 5x5 rig (:24-39), same pair tables (:42), the hot loop
// (:44-95) as one computeDisparity call, depth (:98-100), plus the north_star
// Mode S matcher, the TO_CENTER_SMALL array fusion and the refinement stage.
//
// No OpenCV here: images are synthetic (one texture seen by every camera
// through a fronto-parallel plane at depth Z, so the true disparity is known)
// and nothing is shown on screen.  Build:
//   g++ -std=c++17 -O2 -I include examples/camera_stereo_vision.cpp
//       -L stereovisionarray_amd -lsva -Wl,-rpath,$PWD/stereovisionarray_amd
// Run: ./camera_stereo_vision [width height]   (default 640 480)
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>

#include "sva.hpp"

using namespace sva;

int main(int argc, char** argv) {
    const int W = argc > 2 ? std::atoi(argv[1]) : 640, H = argc > 2 ? std::atoi(argv[2]) : 480;
    // Camera parameters (CameraStereoVision.cpp:24-39)
    const double f = 0.05, sensor_size = 0.036, pixelSize = sensor_size / W;
    std::vector<Camera> cameras;
    for (int y = 0; y < 5; y++)
        for (int x = 0; x < 5; x++)
            cameras.emplace_back(f, Point3d{-0.1 + x * 0.05, -0.1 + y * 0.05, -0.75}, pixelSize);

    // Synthetic scene: a textured plane at depth Z in front of the rig.  A
    // scene point seen at pixel q of camera 12 appears shifted by
    // -(grid offset) * d0 pixels in a neighbour, d0 = pitch * f / (Z * ps).
    // Z inside the reference's ray interval t in [0.5, 1] (:61-64), so Mode R
    // can find it; Mode S gets the smallest built D above d0.
    const int d0 = (int)std::lround(0.05 * f / (0.7 * pixelSize));
    const double Z = 0.05 * f / (d0 * pixelSize);   // the plane depth d0 encodes
    std::mt19937 rng(1234);
    const int M = 4 * d0 + 8;                       // texture margin
    std::vector<uint8_t> tex((size_t)(W + 2 * M) * (H + 2 * M));
    for (auto& t : tex) t = (uint8_t)(rng() & 255);
    std::vector<std::vector<uint8_t>> imgs(25, std::vector<uint8_t>((size_t)W * H));
    for (int c = 0; c < 25; c++) {
        const int gx = c % 5 - 2, gy = c / 5 - 2;
        for (int y = 0; y < H; y++)
            for (int x = 0; x < W; x++)
                imgs[c][(size_t)y * W + x] = tex[(size_t)(y + M + gy * d0) * (W + 2 * M) + x + M + gx * d0];
    }
    std::vector<ImageView> images;
    for (auto& im : imgs) images.emplace_back(im.data(), W, H);

    Engine engine(0);
    auto ms = [](auto t0) {
        return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    };

    // The reference's path (Mode R): pairs MID_LEFT, kernelSize 20, mask = all
    auto pairs = getCameraPairs(cameras, MID_LEFT);
    auto t0 = std::chrono::steady_clock::now();
    DisparityMaps dm = computeDisparity(engine, images, cameras, pairs, ImageView(), 20);
    const double t_ref = ms(t0);
    auto depth = disparityToDepth(engine, dm.disp_u8, cameras[pairs[0][0]], cameras[pairs[0][1]]);
    long nvalid = 0, nexact = 0;
    for (size_t i = 0; i < dm.valid.size(); i++)
        if (dm.valid[i]) {
            nvalid++;
            nexact += dm.disp_u16[i] == d0;
        }
    std::printf("Mode R (reference path, pair 12->11, k=20): %dx%d in %.2f ms, %ld px matched, "
                "%.1f %% at the true disparity %d\n",
                W, H, t_ref, nvalid, 100.0 * nexact / (nvalid ? nvalid : 1), d0);
    const size_t pc = (size_t)(H / 2) * W + W / 2;
    std::printf("  depth at the centre: %.4f m (plane at %.4f m from the rig)\n", depth[pc], Z);

    // north_star Mode S on the same pair (12 -> 11: match at x + d)
    sva_sgm_params p;
    sva_sgm_params_default(&p);
    p.D = d0 < 64 ? 64 : d0 < 128 ? 128 : d0 < 192 ? 192 : 256;
    p.dir = +1;
    t0 = std::chrono::steady_clock::now();
    auto ds = computeDisparitySGM(engine, images[12], images[11], p);
    const double t_sgm = ms(t0);
    long sexact = 0, sn = 0;
    for (int y = 8; y < H - 8; y++)
        for (int x = 8; x < W - 8 - d0; x++, sn++) sexact += ds[(size_t)y * W + x] == d0;
    std::printf("Mode S (census/SGM, D=%d): %.2f ms incl. host copies, %.1f %% of the interior "
                "at %d\n", p.D, t_sgm, 100.0 * sexact / sn, d0);

    // TO_CENTER_SMALL: 8 pairs on their own baseline steps, median-fused depth
    auto around = getCameraPairs(cameras, TO_CENTER_SMALL);
    std::vector<std::vector<uint16_t>> maps;
    std::vector<double> baselines;
    t0 = std::chrono::steady_clock::now();
    for (auto& pr : around) {
        PairStep st = pairStep(cameras[pr[0]], cameras[pr[1]]);
        maps.push_back(computeDisparityPair(engine, images[pr[0]], images[pr[1]], st, p));
        baselines.push_back(st.baseline);
    }
    std::vector<uint8_t> nv;
    auto fused = fuseDepth(engine, maps, W, H, baselines, f, pixelSize, 0xFFFF, &nv);
    std::printf("TO_CENTER_SMALL: 8 pairs + fusion in %.2f ms; fused depth at the centre %.4f m "
                "from %d maps\n", ms(t0), fused[pc], nv[pc]);

    // Refinement (functions.cpp:11-52) of the Mode R map with the CROSS pairs
    std::vector<std::array<Camera, 2>> camPairs;
    std::vector<ImageView> pairImages;
    for (auto& pr : getCameraPairs(cameras, CROSS)) {
        camPairs.push_back({cameras[pr[0]], cameras[pr[1]]});
        pairImages.push_back(images[pr[1]]);
    }
    std::vector<uint8_t> faceMask((size_t)W * H, 0);
    for (int y = H / 4; y < 3 * H / 4; y++)
        for (int x = W / 4; x < 3 * W / 4; x++) faceMask[(size_t)y * W + x] = 1;
    t0 = std::chrono::steady_clock::now();
    auto refined = improveWithDisparity(engine, ImageView(dm.disp_u8.data(), W, H), images[12],
                                        pairImages, camPairs, 21, ImageView(faceMask.data(), W, H));
    std::printf("improveWithDisparity (4 CROSS pairs, 20x20): %.2f ms; centre %d -> %d\n", ms(t0),
                dm.disp_u8[pc], refined[pc]);
    const bool ok = nvalid > 0 && 100.0 * nexact / nvalid > 50.0 && 100.0 * sexact / sn > 50.0 &&
                    std::fabs(fused[pc] - Z) < 0.05 * Z;
    std::printf("%s\n", ok ? "OK" : "UNEXPECTED RESULT");
    return ok ? 0 : 1;
}
