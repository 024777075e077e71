// C++ host-mirror tests (include/sva.hpp).  Built by tests/test_host_cpp.py.
//   ./test_host cpu   -- CPU-only checks (pair tables, bresenham, camera)
//   ./test_host gpu   -- computeDisparity / computeDisparitySGM through the C-ABI
#include <cstdio>
#include <cstring>
#include <fstream>
#include <random>

#include "sva.hpp"

static int failures = 0;
#define CHECK(c)                                                        \
    do {                                                                \
        if (!(c)) {                                                     \
            std::printf("FAIL %s:%d  %s\n", __FILE__, __LINE__, #c);    \
            failures++;                                                 \
        }                                                               \
    } while (0)

using namespace sva;

static std::vector<Camera> rig(int W) {
    // CameraStereoVision.cpp:24-39
    std::vector<Camera> cams;
    const double ps = 0.036 / W;
    for (int y = 0; y < 5; y++)
        for (int x = 0; x < 5; x++) cams.emplace_back(0.05, Point3d{-0.1 + x * 0.05, -0.1 + y * 0.05, -0.75}, ps);
    return cams;
}

static void yaml_tests() {
    // getIdealRef / saveImage / loadImage (functions.cpp:323-346): OpenCV's own text
    const std::string dir = std::filesystem::temp_directory_path().string();
    const std::string p = dir + "/sva_test_idealRef.yml";
    {
        std::ofstream f(p);
        f << "%YAML:1.0\n---\nR: !!opencv-matrix\n   rows: 2\n   cols: 3\n   dt: d\n"
             "   data: [ 1., 2.5000000000000000e+00, -3.2500000000000000e+00, .Inf,\n"
             "       -.Inf, .Nan ]\nimage: !!opencv-matrix\n   rows: 1\n   cols: 2\n"
             "   dt: \"3u\"\n   data: [ 1, 2, 3, 4, 5, 255 ]\n";
    }
    YamlMatrix R = getIdealRef(p);
    CHECK(R.rows == 2 && R.cols == 3 && R.dt == 'd' && R.data.size() == 6);
    CHECK(R.data[0] == 1.0 && R.data[1] == 2.5 && R.data[2] == -3.25);
    CHECK(std::isinf(R.data[3]) && R.data[3] > 0 && std::isinf(R.data[4]) && R.data[4] < 0);
    CHECK(std::isnan(R.data[5]));
    YamlMatrix im = loadImage(p);
    CHECK(im.rows == 1 && im.cols == 2 && im.channels == 3 && im.dt == 'u');
    CHECK(im.data.back() == 255.0);
    bool threw = false;
    try { readYamlMatrix(p, "missing"); } catch (const Error&) { threw = true; }
    CHECK(threw);
    // round trip through saveImage
    YamlMatrix m;
    m.rows = 3; m.cols = 4; m.dt = 'd';
    std::mt19937 rng(3);
    std::normal_distribution<double> nd;
    for (int i = 0; i < 12; i++) m.data.push_back(nd(rng));
    m.data[5] = HUGE_VAL;
    const std::string q = dir + "/sva_test_image.yml";
    saveImage(q, m);
    YamlMatrix back = loadImage(q);
    CHECK(back.rows == 3 && back.cols == 4 && back.dt == 'd' && back.data == m.data);
    std::remove(p.c_str());
    std::remove(q.c_str());
}

static void cpu_tests() {
    yaml_tests();
    auto cams = rig(640);
    // getCameraPairs (functions.cpp:148-197)
    CHECK(getCameraPairs(cams, MID_LEFT) == (std::vector<std::array<int, 2>>{{12, 11}}));
    CHECK(getCameraPairs(cams, TO_CENTER).size() == 24);
    CHECK(getCameraPairs(cams, TO_CENTER_SMALL).size() == 8);
    CHECK(getCameraPairs(cams, LINE_VERTICAL) ==
          (std::vector<std::array<int, 2>>{{12, 2}, {12, 7}, {12, 17}, {12, 22}}));
    CHECK(getCameraPairs(cams, JUMP_CROSS)[3] == (std::array<int, 2>{12, 24}));
    CHECK(getCameraPairs(cams, ORTHOGONAL).empty());
    // CROSS with cameraNum (functions.cpp:199-213) keeps the reference quirks
    auto q = getCameraPairs(cams, CROSS, 12);
    CHECK(q == (std::vector<std::array<int, 2>>{{12, 7}, {12, 5}, {12, 11}, {12, 13}}));
    auto fixed = getCameraPairs(cams, CROSS, 12, false);
    CHECK(fixed == (std::vector<std::array<int, 2>>{{12, 7}, {12, 17}, {12, 11}, {12, 13}}));
    CHECK(getCameraPairs(cams, CROSS, 5).size() == 2);   // 5-5 > 0 false, 5%5 == 0
    auto groups = getGroups(cams, "CHESS");
    CHECK(groups.size() == 13);
    CHECK(getGroups(cams, "OTHER").empty());
    // bresenham hand traces (same as tests/test_oracle_kat.py)
    auto b = bresenham({5, 5}, {4, 9});
    std::vector<Point2i> e{{5, 5}, {5, 6}, {5, 7}, {4, 8}, {4, 9}};
    CHECK(b == e);
    auto b2 = bresenham({3, 1}, {0, 0});
    std::vector<Point2i> e2{{0, 0}, {1, 0}, {2, 1}, {3, 1}};
    CHECK(b2 == e2);
    // Camera::project truncates toward zero
    Camera c(0.05, {0, 0, -0.75}, 0.036 / 640);
    Point2i p = c.project({0.01, -0.02, 0.25});
    CHECK(p.x == 8 && p.y == -17);
    Camera u(12.0, {0, 0, 0}, 1.0);
    Point3d v = u.inv_project({3, 4});
    CHECK(v.x == 3.0 / 13 && v.y == 4.0 / 13 && v.z == 12.0 / 13);
    // getAbsDiff on views
    uint8_t a[4] = {0, 255, 10, 20}, bb[4] = {255, 0, 20, 10};
    CHECK(getAbsDiff(ImageView(a, 2, 2), ImageView(bb, 2, 2)) == 530.0);
    bool threw = false;
    try { ImageView(a, 2, 2).roi(1, 1, 2, 2); } catch (const Error&) { threw = true; }
    CHECK(threw);
    // array pair steps on the reference rig (camera 12 at grid (2,2))
    auto rc = rig(640);
    PairStep s11 = pairStep(rc[12], rc[11]);   // left neighbour: match at x + d (12 -> 11)
    CHECK(s11.dir == 1 && s11.dir_y == 0 && s11.k == 1 && std::fabs(s11.baseline - 0.05) < 1e-12);
    PairStep s18 = pairStep(rc[12], rc[18]);   // (+1,+1) neighbour
    CHECK(s18.dir == -1 && s18.dir_y == -1 && s18.k == 1);
    PairStep s7 = pairStep(rc[12], rc[7]);     // above
    CHECK(s7.dir == 0 && s7.dir_y == 1 && s7.k == 1);
    PairStep s3 = pairStep(rc[12], rc[3]);     // grid offset (1,-2)
    CHECK(s3.dir == -1 && s3.dir_y == 2 && s3.k == 2 && std::fabs(s3.baseline - 0.1) < 1e-12);
    // getImagesPathsFromFolder: sorted listing of regular files
    auto dir = std::filesystem::temp_directory_path() / "sva_host_test_listing";
    std::filesystem::remove_all(dir);
    std::filesystem::create_directories(dir / "sub");
    for (const char* n : {"b.png", "a.png", "10.png"}) std::ofstream(dir / n) << "x";
    auto files = getImagesPathsFromFolder(dir.string());
    CHECK(files.size() == 3 && files[0] == (dir / "10.png").string() &&
          files[2] == (dir / "b.png").string());
    std::filesystem::remove_all(dir);
    PairStep s14 = pairStep(rc[12], rc[14]);   // (2,0): reduced to a unit step
    CHECK(s14.dir == -1 && s14.dir_y == 0 && s14.k == 2);
}

static void gpu_tests() {
    const int W = 192, H = 144;
    auto cams = rig(W);
    std::mt19937 rng(5);
    std::vector<std::vector<uint8_t>> imgs(25, std::vector<uint8_t>(W * H));
    for (auto& im : imgs)
        for (auto& px : im) px = (uint8_t)(rng() & 255);
    std::vector<ImageView> views;
    for (auto& im : imgs) views.emplace_back(im.data(), W, H);
    Engine eng(0);
    auto pairs = getCameraPairs(cams, CROSS);
    DisparityMaps m = computeDisparity(eng, views, cams, pairs, ImageView(), 8);
    // each pair individually through the C-ABI, last pair wins (:55)
    std::vector<uint8_t> d8(W * H, 0), val(W * H, 0);
    std::vector<uint16_t> d16(W * H, 0);
    for (auto& pr : pairs) {
        sva_camera a = cams[pr[0]].abi(), b = cams[pr[1]].abi();
        eng.check(sva_disparity_ref(eng.handle(), imgs[pr[0]].data(), imgs[pr[1]].data(), W, H, W,
                                    nullptr, &a, &b, 8, 0.5, 1.0, d8.data(), d16.data(), val.data()));
    }
    CHECK(m.disp_u8 == d8 && m.disp_u16 == d16 && m.valid == val);
    int nvalid = 0;
    for (auto v : m.valid) nvalid += v;
    CHECK(nvalid > W * H / 4);
    auto depth = disparityToDepth(eng, m.disp_u8, cams[12], cams[11]);
    CHECK(depth.size() == m.disp_u8.size());
    // Mode S through the C++ layer
    sva_sgm_params p;
    sva_sgm_params_default(&p);
    p.D = 64;
    p.subpixel = 1;
    std::vector<float> sub;
    auto ds = computeDisparitySGM(eng, views[12], views[13], p, &sub);
    CHECK(ds.size() == (size_t)W * H && sub.size() == ds.size());
    // AUTO and COST_VOLUME are one route; the census-fused kernel is gone (ABI v4)
    std::vector<float> sub_f;
    eng.setPathKernel(SVA_PATH_KERNEL_COST_VOLUME);
    auto df = computeDisparitySGM(eng, views[12], views[13], p, &sub_f);
    eng.setPathKernel(SVA_PATH_KERNEL_AUTO);
    CHECK(df == ds && sub_f == sub);
    bool threw = false;
    try {
        eng.setPathKernel(SVA_PATH_KERNEL_FUSED);
    } catch (const Error& e) {
        threw = e.status == SVA_ERR_UNSUPPORTED;
    }
    CHECK(threw);
    // any D <= 256: D = 50 runs padded to 64
    p.D = 50;
    auto d50 = computeDisparitySGM(eng, views[12], views[13], p);
    CHECK(d50.size() == ds.size());
    for (uint16_t v : d50) CHECK(v < 50);
    threw = false;
    try {
        p.D = 257;
        computeDisparitySGM(eng, views[12], views[13], p);
    } catch (const Error& e) {
        threw = e.status == SVA_ERR_UNSUPPORTED;
    }
    CHECK(threw);
    // array pair + fusion through the C++ layer: a constant vertical shift d0
    const int d0 = 9;
    std::vector<uint8_t> below(W * H);
    for (int y = 0; y < H; y++)
        for (int x = 0; x < W; x++) below[y * W + x] = imgs[12][std::min(H - 1, y + d0) * W + x];
    sva_sgm_params q;
    sva_sgm_params_default(&q);
    q.D = 64;
    PairStep st = pairStep(cams[12], cams[17]);   // camera 17 is one grid row below 12
    CHECK(st.dir == 0 && st.dir_y == -1);
    auto dv = computeDisparityPair(eng, views[12], ImageView(below.data(), W, H), st, q);
    int exact = 0, inner = 0;
    for (int y = d0 + 20; y < H - 20; y++)
        for (int x = 8; x < W - 8; x++) {
            inner++;
            exact += dv[y * W + x] == d0;
        }
    CHECK(exact == inner);
    std::vector<uint8_t> nv;
    auto z = fuseDepth(eng, {dv, dv}, W, H, {st.baseline, st.baseline}, cams[12].f,
                       cams[12].pixel_size, 0xFFFF, &nv);
    const int pc = (H / 2) * W + W / 2;
    CHECK(nv[pc] == 2 && z[pc] == (st.baseline * cams[12].f) / ((double)d0 * cams[12].pixel_size));

    // multi-GPU engine (here one device, two streams): the TO_CENTER_SMALL
    // frame equals per-pair matching on one context + fuseDepth
    {
        MultiEngine me({0}, 2);
        auto cpairs = getCameraPairs(cams, TO_CENTER_SMALL);
        std::vector<std::vector<uint16_t>> mm;
        auto fused = computeArrayDepth(me, views, cams, cpairs, q, 0.05, &mm);
        CHECK(fused.size() == 1 && mm.size() == cpairs.size());
        std::vector<std::vector<uint16_t>> single;
        std::vector<double> bl;
        bool same = true;
        for (size_t i = 0; i < cpairs.size(); i++) {
            PairStep s = pairStep(cams[cpairs[i][0]], cams[cpairs[i][1]]);
            single.push_back(computeDisparityPair(eng, views[cpairs[i][0]], views[cpairs[i][1]], s, q));
            bl.push_back(s.baseline);
            same = same && single.back() == mm[i];
        }
        CHECK(same);
        CHECK(fuseDepth(eng, single, W, H, bl, cams[12].f, cams[12].pixel_size) == fused[0]);
    }

    // refinement: img(x) = centre(x - dd - 2) => refined disparity dd + 2 (functions.cpp:11-52)
    const int dd = 6;
    std::vector<uint8_t> other(W * H, 0), dispc(W * H, dd), fmask(W * H, 0);
    for (int y = 0; y < H; y++)
        for (int x = dd + 2; x < W; x++) other[y * W + x] = imgs[12][y * W + x - dd - 2];
    for (int y = 40; y < 100; y++)
        for (int x = 60; x < 130; x++) fmask[y * W + x] = 1;
    Camera ca(0.05, Point3d{0.05, 0, -0.75}, 1e-4), cb(0.05, Point3d{0, 0, -0.75}, 1e-4);
    auto refined = improveWithDisparity(eng, ImageView(dispc.data(), W, H), views[12],
                                        {ImageView(other.data(), W, H)}, {{ca, cb}}, 21,
                                        ImageView(fmask.data(), W, H));
    bool allok = true;
    for (int y = 40; y < 100; y++)
        for (int x = 60; x < 130; x++) allok = allok && refined[y * W + x] == dd + 2;
    CHECK(allok && refined[0] == 0);
    bool threw2 = false;   // full mask: border windows leave the image -> throws like the ROI
    try {
        improveWithDisparity(eng, ImageView(dispc.data(), W, H), views[12],
                             {ImageView(other.data(), W, H)}, {{ca, cb}}, 21);
    } catch (const Error& e) {
        threw2 = e.status == SVA_ERR_INVALID_ARG;
    }
    CHECK(threw2);
    // depth -> points -> depth at constant depth 1 on the reference camera
    std::vector<double> dm((size_t)W * H, 1.0);
    auto pts = DepthMapToPoints3D(eng, dm, cams[12], W, H);
    CHECK(pts.size() == (size_t)W * H);
    auto back = Points3DToDepthMap(eng, pts, cams[12], W, H);
    CHECK(back[(size_t)(H / 2) * W + W / 2] == 1.0);   // the centre ray is the optical axis
    auto sh = shiftPerspective2(eng, cams[12], cams[11], dm, W, H);
    CHECK(sh.size() == dm.size());
    auto shifted = shiftPerspectiveWithDisparity(eng, cams[12], cams[11], ImageView(dispc.data(), W, H),
                                                 views[13]);
    CHECK(shifted[(size_t)10 * W + 10] == imgs[13][(size_t)10 * W + 10 + dd]);
    // ingestion resize (CameraStereoVision.cpp:18)
    int hw = 0, hh = 0;
    auto half = resizeHalf(eng, views[0], &hw, &hh);
    CHECK(hw == W / 2 && hh == H / 2 && half.size() == (size_t)hw * hh);
    const int s4 = imgs[0][0] + imgs[0][1] + imgs[0][W] + imgs[0][W + 1];
    CHECK(half[0] == (uint8_t)((s4 + 2) >> 2));

    // evaluation (CameraStereoVision.cpp:107-110; functions.cpp:348-354)
    const std::vector<double> row = {0.0, 10.0};
    CHECK(resizeLinear(eng, row, 2, 1, 4, 1) == (std::vector<double>{0.0, 2.5, 7.5, 10.0}));
    YamlMatrix ref;
    ref.rows = 1; ref.cols = 4; ref.dt = 'd';
    ref.data = {0.0, 2.0, 7.0, 10.0};
    CHECK(refError(eng, row, 2, 1, ref) == (std::vector<double>{0.0, 25.0, 25.0, 0.0}));
    const std::vector<double> img = {1.0, 2.0, 3.0, 4.0};
    const std::vector<uint8_t> msk = {1, 0, 1, 0};
    CHECK(calculateAverageError(eng, img, 2, 2, &msk) == 2.0);
    CHECK(calculateAverageError(eng, img, 2, 2) == 2.5);
}

int main(int argc, char** argv) {
    const bool gpu = argc > 1 && std::strcmp(argv[1], "gpu") == 0;
    if (gpu) gpu_tests();
    else cpu_tests();
    std::printf("%s: %d failure(s)\n", gpu ? "gpu" : "cpu", failures);
    return failures ? 1 : 0;
}
