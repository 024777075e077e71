"""Launch-gap probe for the 1080p D=128 pipeline.

Per-frame wall time of back-to-back frames on one stream:
  plain      -- sva_disparity_sgm_d per frame, kernel timing off
  timed      -- the same with the hipEvent kernel timer on every launch
  timed_paths-- only the path kernel timed, by its own dispatch (bench.py)
  graph1     -- one frame captured into a hipGraph, replayed per frame
  graph10    -- ten frames captured into one hipGraph
Prints one JSON line.  Run on the GPU box: python tools/graph_probe.py
"""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import stereovisionarray_amd as sva  # noqa: E402
from stereovisionarray_amd import synth  # noqa: E402

W, H, D = 1920, 1080, 128
N = 60


def main():
    dev = torch.device("cuda", 0)
    ctx = sva.Context(0)
    s = torch.cuda.Stream(dev)
    torch.cuda.set_stream(s)
    ctx.set_stream(s.cuda_stream)
    ctx.reserve(W, H, D)
    L, R, _ = synth.stereo_pair(H, W, D, 0, -1, seed=1)
    Lt, Rt = torch.from_numpy(L).to(dev), torch.from_numpy(R).to(dev)
    disp = torch.zeros((H, W), dtype=torch.int16, device=dev)
    sub = torch.zeros((H, W), dtype=torch.float32, device=dev)
    p = sva.default_params(D=D, dmin=0, dir=-1, subpixel=1)

    def frame():
        ctx.disparity_sgm_d(Lt.data_ptr(), Rt.data_ptr(), W, H, W, p, disp.data_ptr(),
                            sub.data_ptr())

    def clock(fn, n):
        best = 1e9
        for _ in range(3):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(n):
                fn()
            torch.cuda.synchronize()
            best = min(best, (time.perf_counter() - t0) / n * 1e3)
        return best

    for _ in range(5):
        frame()
    ref = disp.clone()
    out = {"plain": clock(frame, N)}
    ctx.set_timing(True)
    out["timed"] = clock(frame, N)
    ctx.set_timing(sva.SVA_TIMING_PATHS)
    ctx.reset_timing()
    out["timed_paths"] = clock(frame, N)
    ms, n = ctx.kernel_time("sgm_paths")
    out["sgm_paths_event_ms"] = ms / max(n, 1)
    ctx.set_timing(False)

    g1 = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g1, stream=s):
        frame()
    out["graph1"] = clock(g1.replay, N)
    g10 = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g10, stream=s):
        for _ in range(10):
            frame()
    out["graph10"] = clock(g10.replay, N // 10) / 10
    torch.cuda.synchronize()
    out["graph_result_ok"] = bool(torch.equal(disp, ref))
    out["unit"] = "ms/frame (best of 3 rounds)"
    print(json.dumps({k: (round(v, 4) if isinstance(v, float) else v) for k, v in out.items()}),
          flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
