#!/usr/bin/env python3
"""Is the 4.3 vs 4.9 ms spread of sgm_paths at 4K D=256 a memory-side clock
state?  Runs back-to-back 4K D=256 frames for a while in one process (one
context, fixed buffers) and, beside them, samples `rocm-smi --showclocks`
(read-only) every ~0.5 s; prints sgm_paths hipEvent averages per batch of
frames next to the clock readings taken during that batch.

    python tools/probe_4k_clocks.py [--seconds 20]
"""
import argparse
import json
import os
import re
import subprocess
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def smi_clocks():
    try:
        r = subprocess.run(["rocm-smi", "--showclocks", "--json"], capture_output=True, text=True,
                           timeout=10)
        d = json.loads(r.stdout)
        card = next(iter(d.values()))
        return {k: v for k, v in card.items() if "clk" in k.lower()}
    except Exception as e:                                   # report, do not fail
        return {"error": str(e)[:80]}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=20.0)
    ap.add_argument("--batch", type=int, default=20)
    a = ap.parse_args()
    import torch
    import stereovisionarray_amd as sva
    from stereovisionarray_amd import synth
    W, H, D = 3840, 2160, 256
    dev = torch.device("cuda", 0)
    s = torch.cuda.Stream(dev)
    torch.cuda.set_stream(s)
    L, R, _ = synth.stereo_pair(H, W, D, 0, -1, seed=1)
    dL, dR = torch.from_numpy(L).to(dev), torch.from_numpy(R).to(dev)
    p = sva.default_params(D=D, subpixel=1)
    disp = torch.zeros((H, W), dtype=torch.int16, device=dev)
    sub = torch.zeros((H, W), dtype=torch.float32, device=dev)
    ctx = sva.Context(0)
    ctx.set_stream(s.cuda_stream)
    ctx.reserve(W, H, D)
    samples, stop = [], [False]

    def sampler():
        while not stop[0]:
            samples.append((time.time(), smi_clocks()))
            time.sleep(0.5)

    th = threading.Thread(target=sampler, daemon=True)
    th.start()
    t_end = time.time() + a.seconds
    while time.time() < t_end:
        t0 = time.time()
        ctx.set_timing(sva.SVA_TIMING_AGG)
        ctx.reset_timing()
        for _ in range(a.batch):
            ctx.disparity_sgm_d(dL.data_ptr(), dR.data_ptr(), W, H, W, p, disp.data_ptr(),
                                sub.data_ptr())
        torch.cuda.synchronize()
        t1 = time.time()
        ms, n = ctx.kernel_time("sgm_paths")
        ctx.set_timing(0)
        during = [c for (t, c) in samples if t0 <= t <= t1]
        print(json.dumps({"t": round(t0 - (t_end - a.seconds), 2), "sgm_paths_ms": round(ms / n, 4),
                          "clocks": during[-1] if during else None}), flush=True)
    stop[0] = True
    th.join(timeout=5)
    ctx.close()


if __name__ == "__main__":
    main()
