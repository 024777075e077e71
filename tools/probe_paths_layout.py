#!/usr/bin/env python3
"""Path-kernel lane layouts, in-process A/B: the 16-lane
layout (SVA_PATH_KERNEL_COST_VOLUME) against one line per wave
(SVA_PATH_KERNEL_WIDE), alternating launch by launch on the same buffers, per
frame size: the whole frame (hipEvent around sva_disparity_sgm_d, sub-pixel
on) and the sgm_paths launch alone (its dispatch timer).  Maps are checked
equal between the layouts.

  python tools/probe_paths_layout.py [--iters 40] [--sizes 640x480x64,1920x1080x128]
"""
import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

SIZES = "640x480x64,640x480x128,640x480x256,960x540x64,960x540x128,1280x720x64,1280x720x128," \
        "1600x900x64,1920x1080x64,1920x1080x128"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=40)
    ap.add_argument("--sizes", default=SIZES)
    ap.add_argument("--dmin", type=int, default=0)
    a = ap.parse_args()
    import torch
    import stereovisionarray_amd as sva
    from stereovisionarray_amd import synth

    dev = torch.device("cuda", 0)
    s = torch.cuda.Stream(dev)
    torch.cuda.set_stream(s)
    ctx = sva.Context(0)
    ctx.set_stream(s.cuda_stream)
    kinds = {"16lane": sva.SVA_PATH_KERNEL_COST_VOLUME, "wide": sva.SVA_PATH_KERNEL_WIDE}
    for spec in a.sizes.split(","):
        W, H, D = (int(v) for v in spec.split("x"))
        L, R, _ = synth.stereo_pair(H, W, D, a.dmin, -1, seed=1)
        dL, dR = torch.from_numpy(L).to(dev), torch.from_numpy(R).to(dev)
        p = sva.default_params(D=D, dmin=a.dmin, subpixel=1)
        disp = {k: torch.zeros((H, W), dtype=torch.int16, device=dev) for k in kinds}
        sub = {k: torch.zeros((H, W), dtype=torch.float32, device=dev) for k in kinds}
        frame = {k: [] for k in kinds}
        paths = {k: [] for k in kinds}
        for it in range(a.iters + 3):
            for k, kind in kinds.items():
                ctx.set_path_kernel(kind)
                ctx.set_timing(sva.SVA_TIMING_PATHS if hasattr(sva, "SVA_TIMING_PATHS") else 2)
                ctx.reset_timing()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(s)
                ctx.disparity_sgm_d(dL.data_ptr(), dR.data_ptr(), W, H, W, p, disp[k].data_ptr(),
                                    sub[k].data_ptr())
                e1.record(s)
                e1.synchronize()
                ms, n = ctx.kernel_time("sgm_paths")
                ctx.set_timing(0)
                if it >= 3:
                    frame[k].append(e0.elapsed_time(e1))
                    paths[k].append(ms / max(n, 1))
        same = torch.equal(disp["16lane"], disp["wide"]) and torch.equal(sub["16lane"], sub["wide"])
        out = {"W": W, "H": H, "D": D, "maps_equal": bool(same)}
        for k in kinds:
            out[f"frame_{k}_ms"] = round(statistics.median(frame[k]), 4)
            out[f"paths_{k}_ms"] = round(statistics.median(paths[k]), 4)
        print(json.dumps(out), flush=True)
        assert same, "layouts disagree"
    ctx.set_path_kernel(sva.SVA_PATH_KERNEL_AUTO)
    ctx.close()


if __name__ == "__main__":
    main()
