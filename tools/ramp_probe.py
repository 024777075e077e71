#!/usr/bin/env python3
"""Per-frame times of back-to-back 1080p D=128 frames right after set-up, to
see where the start-up ramp of bench.py's first frames comes from (DESIGN.md
§6).  Run 1 starts right after ctx.reserve(); run 2 after an idle sleep.  A
ramp in run 1 only points at first touches of fresh memory; a ramp in both
at clocks / power state.

usage: ramp_probe.py [frames] [idle_s]
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    import stereovisionarray_amd as sva
    from stereovisionarray_amd import synth
    frames = int(sys.argv[1]) if len(sys.argv) > 1 else 80
    idle = float(sys.argv[2]) if len(sys.argv) > 2 else 3.0
    W, H, D = 1920, 1080, 128
    dev = torch.device("cuda", 0)
    L, R, _ = synth.stereo_pair(H, W, D, 0, -1, seed=1)
    dL, dR = torch.from_numpy(L).to(dev), torch.from_numpy(R).to(dev)
    s = torch.cuda.Stream(dev)
    torch.cuda.set_stream(s)
    ctx = sva.Context(0)
    ctx.set_stream(s.cuda_stream)
    t0 = time.perf_counter()
    ctx.reserve(W, H, D)
    torch.cuda.synchronize()
    reserve_ms = (time.perf_counter() - t0) * 1e3
    disp = torch.zeros((H, W), dtype=torch.int16, device=dev)
    sub = torch.zeros((H, W), dtype=torch.float32, device=dev)
    p = sva.default_params(D=D, subpixel=1)

    def run():
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(frames + 1)]
        torch.cuda.synchronize()
        ev[0].record(s)
        for f in range(frames):
            ctx.disparity_sgm_d(dL.data_ptr(), dR.data_ptr(), W, H, W, p, disp.data_ptr(),
                                sub.data_ptr())
            ev[f + 1].record(s)
        torch.cuda.synchronize()
        return [round(ev[f].elapsed_time(ev[f + 1]), 4) for f in range(frames)]

    first = run()
    time.sleep(idle)
    second = run()
    out = {"reserve_ms": round(reserve_ms, 2), "idle_s": idle,
           "run1_ms": first, "run2_ms": second}
    for k in ("run1_ms", "run2_ms"):
        v = out[k]
        out[k.replace("_ms", "_summary")] = {
            "first5": round(sum(v[:5]) / 5, 4), "5to25": round(sum(v[5:25]) / 20, 4),
            "last20": round(sum(v[-20:]) / 20, 4)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
