#!/usr/bin/env python3
"""SURVEY.md §8f rows 1-4 throughput on the GPU vs the CPU oracle (1 thread),
at 1920x1080 with inputs resident in HBM (device entry points) and hipEvent
kernel times; one JSON line per routine:
  improveWithDisparity (4 CROSS pairs of camera 12, 20x20 windows, a centred
  face-sized mask, and without a mask), shiftPerspective2,
  DepthMapToPoints3D, Points3DToDepthMap, the ingestion resize, and the
  evaluation error map / masked mean."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def main():
    import torch
    import stereovisionarray_amd as sva
    from stereovisionarray_amd import synth
    import pyoracle

    W, H, reps = 1920, 1080, 10
    ctx = sva.Context(0)
    s = torch.cuda.Stream()
    torch.cuda.set_stream(s)
    ctx.set_stream(s.cuda_stream)
    dev = torch.device("cuda", 0)
    cams = synth.reference_array(0.036 / W)
    cam = [sva.Camera.make(*c) for c in cams]
    ocam = [pyoracle.OCamera.make(*c) for c in cams]

    def timed(fn, names):
        fn()
        torch.cuda.synchronize()
        ctx.set_timing(True)
        ctx.reset_timing()
        t0 = time.perf_counter()
        for _ in range(reps):
            fn()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / reps
        ctx.set_timing(False)
        ks = {}
        for n in names:
            ms, k = ctx.kernel_time(n)
            if k:
                ks[n] = round(ms / k, 4)
        return dt, ks

    # improveWithDisparity: 4 CROSS pairs, window 21 (20x20), face-sized mask
    center = synth.texture(H, W, 12)
    others = [synth.texture(H, W, 40 + i) for i in range(4)]
    pairs = [(cam[12], cam[b]) for b in (7, 17, 11, 13)]
    opairs = [(ocam[12], ocam[b]) for b in (7, 17, 11, 13)]
    rng = np.random.default_rng(0)
    disp = rng.integers(100, 160, size=(H, W)).astype(np.uint8)
    mask = np.zeros((H, W), np.uint8)
    mask[240:840, 660:1260] = 1                     # 600 x 600 face region
    d_disp, d_center, d_mask = (torch.from_numpy(a).to(dev) for a in (disp, center, mask))
    d_others = [torch.from_numpy(a).to(dev) for a in others]
    out = torch.zeros((H, W), dtype=torch.uint8, device=dev)
    dt, ks = timed(lambda: ctx.improve_with_disparity_d(
        d_disp.data_ptr(), d_center.data_ptr(), [o.data_ptr() for o in d_others], pairs, W, H, W,
        d_mask.data_ptr(), 21, False, out.data_ptr()), ["shift_perspective", "refine"])
    npx = int(mask.sum()) * len(pairs)
    sad_ops = npx * 11 * 400
    t0 = time.perf_counter()
    crow = slice(240, 264)        # CPU sample: 24 mask rows
    m2 = np.zeros_like(mask); m2[crow, 660:1260] = 1
    pyoracle.improve_with_disparity(disp, center, others, opairs, window=21, mask=m2)
    cdt = time.perf_counter() - t0
    cpx = int(m2.sum()) * len(pairs)
    print(json.dumps({"routine": "improveWithDisparity", "size": f"{W}x{H}", "pairs": 4,
                      "masked_px": int(mask.sum()), "gpu_ms": round(dt * 1e3, 3),
                      "kernels_ms": ks, "gpu_Mpx_pair_per_s": round(npx / dt / 1e6, 1),
                      "gpu_Gabsdiff_per_s": round(sad_ops / dt / 1e9, 1),
                      "cpu_Mpx_pair_per_s_1thread": round(cpx / cdt / 1e6, 4),
                      "cpu_sample": f"24 mask rows x 600 px x 4 pairs, {cdt:.2f} s",
                      "speedup": round((npx / dt) / (cpx / cdt), 1)}), flush=True)

    # the same without a mask: every pixel whose windows fit (the rest are skipped)
    dt, ks = timed(lambda: ctx.improve_with_disparity_d(
        d_disp.data_ptr(), d_center.data_ptr(), [o.data_ptr() for o in d_others], pairs, W, H, W,
        None, 21, False, out.data_ptr()), ["shift_perspective", "refine"])
    print(json.dumps({"routine": "improveWithDisparity_nomask", "size": f"{W}x{H}", "pairs": 4,
                      "gpu_ms": round(dt * 1e3, 3), "kernels_ms": ks,
                      "gpu_Mpx_pair_per_s": round(W * H * 4 / dt / 1e6, 1)}), flush=True)

    # shiftPerspective2 / Points3DToDepthMap / DepthMapToPoints3D
    depth = rng.uniform(0.3, 3.0, size=(H, W))
    d_depth = torch.from_numpy(depth).to(dev)
    d_out = torch.zeros((H, W), dtype=torch.float64, device=dev)
    c12, c11 = cam[12], cam[11]
    from stereovisionarray_amd import lib as L, _ptr
    import ctypes as ct

    def shift2():
        ctx._chk(L.sva_shift_perspective2_d(ctx.h, ct.byref(c12), ct.byref(c11),
                                            _ptr(d_depth.data_ptr()), W, H,
                                            _ptr(d_out.data_ptr())))
    dt, ks = timed(shift2, ["shift_perspective2"])
    t0 = time.perf_counter()
    pyoracle.shift_perspective2(ocam[12], ocam[11], depth)
    cdt = time.perf_counter() - t0
    print(json.dumps({"routine": "shiftPerspective2", "size": f"{W}x{H}",
                      "gpu_ms": round(dt * 1e3, 3), "kernels_ms": ks,
                      "cpu_ms_1thread": round(cdt * 1e3, 1),
                      "speedup": round(cdt / dt, 1)}), flush=True)

    pts = torch.zeros((W * H, 3), dtype=torch.float64, device=dev)
    n = [0]

    def d2p():
        n[0] = ctx.depth_to_points_d(d_depth.data_ptr(), W, H, c12, pts.data_ptr())
    dt, ks = timed(d2p, ["depth_to_points"])
    t0 = time.perf_counter()
    opts = pyoracle.depth_to_points(depth, ocam[12])
    cdt = time.perf_counter() - t0
    print(json.dumps({"routine": "DepthMapToPoints3D", "size": f"{W}x{H}", "points": n[0],
                      "gpu_ms": round(dt * 1e3, 3), "kernels_ms": ks,
                      "cpu_ms_1thread": round(cdt * 1e3, 1),
                      "speedup": round(cdt / dt, 1)}), flush=True)

    d_pts = torch.from_numpy(opts).to(dev)

    def p2d():
        ctx._chk(L.sva_points_to_depth_d(ctx.h, _ptr(d_pts.data_ptr()), opts.shape[0],
                                         ct.byref(c12), W, H, _ptr(d_out.data_ptr())))
    dt, ks = timed(p2d, ["points_to_depth"])
    t0 = time.perf_counter()
    pyoracle.points_to_depth(opts, ocam[12], W, H)
    cdt = time.perf_counter() - t0
    print(json.dumps({"routine": "Points3DToDepthMap", "size": f"{W}x{H}",
                      "points": int(opts.shape[0]), "gpu_ms": round(dt * 1e3, 3),
                      "kernels_ms": ks, "cpu_ms_1thread": round(cdt * 1e3, 1),
                      "speedup": round(cdt / dt, 1)}), flush=True)

    # ingestion: resize(img, img, Size(), 0.5, 0.5) of a 1080p u8 frame
    img = synth.texture(H, W, 9)
    d_img = torch.from_numpy(img).to(dev)
    hw, hh = sva.resize_half_size(W, H)
    d_half = torch.zeros((hh, hw), dtype=torch.uint8, device=dev)
    dt, ks = timed(lambda: ctx.resize_half_d(d_img.data_ptr(), W, H, W, d_half.data_ptr(), hw),
                   ["resize_half"])
    t0 = time.perf_counter()
    pyoracle.resize_half(img)
    cdt = time.perf_counter() - t0
    print(json.dumps({"routine": "resizeHalf", "size": f"{W}x{H}", "gpu_ms": round(dt * 1e3, 3),
                      "kernels_ms": ks, "cpu_ms_1thread": round(cdt * 1e3, 1),
                      "speedup": round(cdt / dt, 1)}), flush=True)

    # evaluation: error map of a 960x540 depth against a 1080p reference, and
    # the masked mean of that error (CameraStereoVision.cpp:107-110)
    dep = rng.uniform(0.3, 2.0, size=(hh, hw))
    refm = rng.uniform(0.3, 2.0, size=(H, W))
    d_dep, d_ref = torch.from_numpy(dep).to(dev), torch.from_numpy(refm).to(dev)
    d_err = torch.zeros((H, W), dtype=torch.float64, device=dev)
    dt, ks = timed(lambda: ctx.ref_error_d(d_dep.data_ptr(), hw, hh, d_ref.data_ptr(), W, H, 50.0,
                                           d_err.data_ptr()), ["resize_linear"])
    t0 = time.perf_counter()
    err = pyoracle.ref_error(dep, refm, 50.0)
    cdt = time.perf_counter() - t0
    print(json.dumps({"routine": "refError", "size": f"{hw}x{hh}->{W}x{H}",
                      "gpu_ms": round(dt * 1e3, 3), "kernels_ms": ks,
                      "cpu_ms_1thread": round(cdt * 1e3, 1), "speedup": round(cdt / dt, 1)}),
          flush=True)
    d_mask = torch.from_numpy(mask).to(dev)
    dt, ks = timed(lambda: ctx.masked_mean_d(d_err.data_ptr(), d_mask.data_ptr(), W, H),
                   ["masked_mean"])
    t0 = time.perf_counter()
    pyoracle.masked_mean(err, mask)
    cdt = time.perf_counter() - t0
    print(json.dumps({"routine": "calculateAverageError", "size": f"{W}x{H}",
                      "gpu_ms_incl_sync": round(dt * 1e3, 3), "kernels_ms": ks,
                      "cpu_ms_1thread": round(cdt * 1e3, 1), "speedup": round(cdt / dt, 1)}),
          flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
