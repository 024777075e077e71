#!/usr/bin/env python3
"""Does a frame's kernels run faster when consecutive frames use different
workspaces?  tools/ab_paths.py (two contexts alternating) measures sgm_paths
~2.5 % below bench.py (one context), same build, same frame.  Here, on one
stream: N frames on one context, then N frames alternating over two contexts,
then N frames on the first again; per-kernel hipEvent averages (SVA_TIMING_AGG,
as bench.py) and wall time per frame.

    python tools/probe_pingpong.py [--W 1920 --H 1080 --D 128] [--frames 60] [--rounds 3]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--W", type=int, default=1920)
    ap.add_argument("--H", type=int, default=1080)
    ap.add_argument("--D", type=int, default=128)
    ap.add_argument("--frames", type=int, default=60)
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    import torch
    import stereovisionarray_amd as sva
    from stereovisionarray_amd import synth
    W, H, D = a.W, a.H, a.D
    dev = torch.device("cuda", 0)
    s = torch.cuda.Stream(dev)
    torch.cuda.set_stream(s)
    L, R, _ = synth.stereo_pair(H, W, D, 0, -1, seed=1)
    dL, dR = torch.from_numpy(L).to(dev), torch.from_numpy(R).to(dev)
    p = sva.default_params(D=D, subpixel=1)
    disp = torch.zeros((H, W), dtype=torch.int16, device=dev)
    sub = torch.zeros((H, W), dtype=torch.float32, device=dev)
    ctxs = []
    for _ in range(3):
        c = sva.Context(0)
        c.set_stream(s.cuda_stream)
        c.reserve(W, H, D)
        ctxs.append(c)

    def run(order):
        for c in ctxs:
            c.set_timing(3)
            c.reset_timing()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for f in range(a.frames):
            c = ctxs[order[f % len(order)]]
            c.disparity_sgm_d(dL.data_ptr(), dR.data_ptr(), W, H, W, p, disp.data_ptr(), sub.data_ptr())
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t0) / a.frames * 1e3
        out = {}
        for k in ("sgm_paths", "wta_hv"):
            tot, n = 0.0, 0
            for c in ctxs:
                ms, cnt = c.kernel_time(k)
                tot += ms
                n += cnt
            out[k] = round(tot / n, 4)
        for c in ctxs:
            c.set_timing(0)
        return round(wall, 4), out

    for c in ctxs:     # warm-up
        for _ in range(10):
            c.disparity_sgm_d(dL.data_ptr(), dR.data_ptr(), W, H, W, p, disp.data_ptr(), sub.data_ptr())
    torch.cuda.synchronize()
    for r in range(a.rounds):
        for name, order in (("one_ctx_A", [0]), ("two_ctx_AB", [0, 1]), ("one_ctx_B", [1]),
                            ("three_ctx_ABC", [0, 1, 2])):
            wall, k = run(order)
            print(json.dumps({"round": r, "mode": name, "ms_per_frame": wall, "kernels_ms": k}),
                  flush=True)
    for c in ctxs:
        c.close()


if __name__ == "__main__":
    main()
