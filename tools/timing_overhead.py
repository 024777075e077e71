#!/usr/bin/env python3
"""Stream-time cost of the bench's live kernel timing: ms per 1080p D=128
frame for back-to-back frames with timing off (0), the roofline kernel's
dispatch events only (2), both aggregation kernels' dispatch events (3, what
bench.py's timed region uses) and every kernel event-timed (1).  Modes
alternate round by round on one context."""
import json
import statistics
import sys
import time
import os

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    import stereovisionarray_amd as sva
    from stereovisionarray_amd import synth
    frames, rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 20, 8
    W, H, D = (int(v) for v in sys.argv[2:5]) if len(sys.argv) > 4 else (1920, 1080, 128)
    dev = torch.device("cuda", 0)
    L, R, _ = synth.stereo_pair(H, W, D, 0, -1, seed=1)
    dL, dR = torch.from_numpy(L).to(dev), torch.from_numpy(R).to(dev)
    s = torch.cuda.Stream(dev)
    ctx = sva.Context(0)
    ctx.set_stream(s.cuda_stream)
    ctx.reserve(W, H, D)
    disp = torch.zeros((H, W), dtype=torch.int16, device=dev)
    sub = torch.zeros((H, W), dtype=torch.float32, device=dev)
    p = sva.default_params(D=D, subpixel=1)

    def run(mode):
        ctx.set_timing(mode)
        ctx.reset_timing()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(frames):
            ctx.disparity_sgm_d(dL.data_ptr(), dR.data_ptr(), W, H, W, p, disp.data_ptr(),
                                sub.data_ptr())
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / frames * 1e3
        ctx.set_timing(0)
        return dt

    modes = (0, 2, 3, 1)
    for m in modes:
        run(m)
    res = {m: [] for m in modes}
    for _ in range(rounds):
        for m in modes:
            res[m].append(run(m))
    # one isolated frame (host sync before and after), as tools/ab_paths.py times them
    iso = []
    for _ in range(rounds):
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        ctx.disparity_sgm_d(dL.data_ptr(), dR.data_ptr(), W, H, W, p, disp.data_ptr(), sub.data_ptr())
        e1.record(s)
        e1.synchronize()
        iso.append(e0.elapsed_time(e1))
    print(json.dumps({"W": W, "H": H, "D": D, "frames_per_run": frames, "rounds": rounds,
                      "isolated_frame_ms_median": round(statistics.median(iso), 4),
                      "ms_per_frame_median": {f"timing_{m}": round(statistics.median(v), 4)
                                              for m, v in res.items()},
                      "ms_per_frame_min": {f"timing_{m}": round(min(v), 4) for m, v in res.items()}}))


if __name__ == "__main__":
    main()
