#!/usr/bin/env python3
"""PCIe-inclusive rate of the host-buffer boundary (sva_disparity_sgm with
host images in and host maps out, synchronous), next to the device-resident
rate of the same frame.  1080p D=128; the sub-pixel map doubles the bytes
coming back, so both are shown."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import torch
    import stereovisionarray_amd as sva
    from stereovisionarray_amd import synth
    W, H, D, n = 1920, 1080, 128, 20
    L, R, _ = synth.stereo_pair(H, W, D, 0, -1, seed=1)
    ctx = sva.Context(0)
    out = {}
    for sub in (0, 1):
        p = sva.default_params(D=D, subpixel=sub)
        ctx.disparity_sgm(L, R, p)
        t0 = time.perf_counter()
        for _ in range(n):
            ctx.disparity_sgm(L, R, p)
        dt = (time.perf_counter() - t0) / n
        out[f"host_buffers_subpixel{sub}"] = {"ms_per_frame": round(dt * 1e3, 3),
                                              "Mdisp_per_s": round(W * H * D / dt / 1e6, 1)}
    dev = torch.device("cuda", 0)
    s = torch.cuda.Stream()
    torch.cuda.set_stream(s)
    ctx.set_stream(s.cuda_stream)
    dL, dR = torch.from_numpy(L).to(dev), torch.from_numpy(R).to(dev)
    disp = torch.zeros((H, W), dtype=torch.int16, device=dev)
    p = sva.default_params(D=D, subpixel=0)
    ctx.disparity_sgm_d(dL.data_ptr(), dR.data_ptr(), W, H, W, p, disp.data_ptr())
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        ctx.disparity_sgm_d(dL.data_ptr(), dR.data_ptr(), W, H, W, p, disp.data_ptr())
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / n
    out["device_buffers_subpixel0"] = {"ms_per_frame": round(dt * 1e3, 3),
                                       "Mdisp_per_s": round(W * H * D / dt / 1e6, 1)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
