#!/usr/bin/env python3
"""Mode R (the reference's own Bresenham + 2k x 2k SAD path) throughput on the
GPU vs the CPU restatement on this host.

Unit: candidate evaluations per second ("Mdisp/s" in the reference's sense:
one disparity hypothesis = one 2k x 2k SAD), reference rig (5x5 grid, pair
12 -> 11, k = 20, t in [0.5, 1]), synthetic texture shifted by the rig's own
disparity so the minimum is real.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="640x480,1920x1080")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--cpu-rows", type=int, default=24, help="rows of the CPU sample")
    ap.add_argument("--pairs", default="12-11", help="reference-rig pairs, e.g. 12-11,12-7,12-6")
    ap.add_argument("--k", type=int, default=20, help="kernelSize (2k x 2k windows)")
    a = ap.parse_args()
    import torch
    import stereovisionarray_amd as sva
    from stereovisionarray_amd import synth
    import pyoracle

    ctx = sva.Context(0)
    s = torch.cuda.Stream()
    torch.cuda.set_stream(s)
    ctx.set_stream(s.cuda_stream)
    out = []
    import hashlib
    for spec, pair in [(s_, p_) for s_ in a.sizes.split(",") for p_ in a.pairs.split(",")]:
        W, H = map(int, spec.split("x"))
        i_ref, i_oth = map(int, pair.split("-"))
        k = a.k
        grid = synth.reference_array(0.036 / W)
        cr, co = sva.Camera.make(*grid[i_ref]), sva.Camera.make(*grid[i_oth])
        ocr, oco = pyoracle.OCamera.make(*grid[i_ref]), pyoracle.OCamera.make(*grid[i_oth])
        ref = synth.texture(H, W, 5)
        shift = int(round(0.05 * 0.05 / 1.0 / (0.036 / W) * 1.5))  # ~ mid-range disparity
        oth = np.roll(ref, shift, axis=1)
        # candidate count (oracle geometry on a sample of rows, exact count on GPU side below)
        d_ref = torch.from_numpy(ref).cuda()
        d_oth = torch.from_numpy(oth).cuda()
        d8 = torch.zeros((H, W), dtype=torch.uint8, device="cuda")
        d16 = torch.zeros((H, W), dtype=torch.int16, device="cuda")
        val = torch.zeros((H, W), dtype=torch.uint8, device="cuda")
        ends = torch.zeros((H, W, 4), dtype=torch.int32, device="cuda")
        ok = torch.zeros((H, W), dtype=torch.uint8, device="cuda")
        ctx.ref_endpoints_d(W, H, cr, co, k, 0.5, 1.0, ends.data_ptr(), ok.data_ptr())
        torch.cuda.synchronize()
        e = ends.cpu().numpy().astype(np.int64)
        okn = ok.cpu().numpy().astype(bool)
        n_cand = (np.maximum(np.abs(e[..., 0] - e[..., 2]), np.abs(e[..., 1] - e[..., 3])) + 1)[okn].sum()
        ctx.disparity_ref_d(d_ref.data_ptr(), d_oth.data_ptr(), W, H, W, None, cr, co, k, 0.5, 1.0,
                            d8.data_ptr(), d16.data_ptr(), val.data_ptr())
        torch.cuda.synchronize()
        ctx.set_timing(True)
        ctx.reset_timing()
        t0 = time.perf_counter()
        for _ in range(a.reps):
            ctx.disparity_ref_d(d_ref.data_ptr(), d_oth.data_ptr(), W, H, W, None, cr, co, k, 0.5,
                                1.0, d8.data_ptr(), d16.data_ptr(), val.data_ptr())
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / a.reps
        ctx.set_timing(False)
        ms_match, n = ctx.kernel_time("ref_match")
        gpu_rate = n_cand / dt / 1e6
        # CPU sample: a band of rows through the oracle, single thread
        y0 = H // 2
        band = slice(y0 - a.cpu_rows // 2 - k, y0 + a.cpu_rows // 2 + k)
        mask = np.zeros((H, W), np.uint8)
        mask[y0 - a.cpu_rows // 2: y0 + a.cpu_rows // 2, :] = 1
        t0 = time.perf_counter()
        _, _, _, ncpu = pyoracle.ref_pair(ref, oth, ocr, oco, k=k, mask=mask)
        cdt = time.perf_counter() - t0
        cpu_rate = ncpu / cdt / 1e6
        del band
        digest = hashlib.sha1(d16.cpu().numpy().tobytes() + val.cpu().numpy().tobytes()).hexdigest()[:16]
        out.append({"size": f"{W}x{H}", "pair": pair, "k": k,
                    "out_sha1": digest, "candidates": int(n_cand), "gpu_ms": round(dt * 1e3, 3),
                    "ref_match_ms": round(ms_match / max(n, 1), 3),
                    "gpu_Mcand_per_s": round(gpu_rate, 1),
                    "cpu_Mcand_per_s_1thread": round(cpu_rate, 3),
                    "cpu_sample": f"{a.cpu_rows} rows, {ncpu} candidates, {cdt:.2f} s",
                    "speedup": round(gpu_rate / cpu_rate, 1)})
        print(json.dumps(out[-1]), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
