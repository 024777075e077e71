#!/usr/bin/env python3
"""Progress of the 8 path directions inside one sgm_paths launch (experiment
build with -DSVA_PATHS_TRACE, ablibs/libsva_trace.so): every wave stamps
s_memrealtime (100 MHz) each 96 steps.  Prints, per direction group and
checkpoint, the spread of the waves' stamps (us after the first stamp), to see
whether the three downward directions read a cost row close enough in time
for the Infinity Cache to serve the re-reads."""
import ctypes as ct
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("SVA_LIB_PATH", os.path.join(ROOT, "ablibs", "libsva_trace.so"))
import stereovisionarray_amd as sva  # noqa: E402
from stereovisionarray_amd import synth  # noqa: E402

W, H, D = 1920, 1080, 128
SLOTS = 32
# code = 10 + 3*(rx+1) + (ry+1)
NAMES = {10 + 3 * (rx + 1) + (ry + 1): n for (rx, ry), n in {
    (1, 0): "h_lr", (-1, 0): "h_rl", (0, 1): "down", (0, -1): "up", (1, 1): "down_right",
    (-1, -1): "up_left", (-1, 1): "down_left", (1, -1): "up_right"}.items()}


def main():
    dev = torch.device("cuda", 0)
    ctx = sva.Context(0)
    s = torch.cuda.Stream(dev)
    torch.cuda.set_stream(s)
    ctx.set_stream(s.cuda_stream)
    L, R, _ = synth.stereo_pair(H, W, D, 0, -1, seed=1)
    Lt, Rt = torch.from_numpy(L).to(dev), torch.from_numpy(R).to(dev)
    disp = torch.zeros((H, W), dtype=torch.int16, device=dev)
    p = sva.default_params(D=D)
    for _ in range(4):
        ctx.disparity_sgm_d(Lt.data_ptr(), Rt.data_ptr(), W, H, W, p, disp.data_ptr())
    torch.cuda.synchronize()
    lib = sva.lib
    nw = (2 * ((H + 15) // 16) + 6 * ((W + 15) // 16)) * 4
    host = np.zeros(nw * SLOTS, np.uint64)
    assert lib.sva_debug_paths_trace_copy(ct.c_void_p(host.ctypes.data),
                                          ct.c_size_t(host.nbytes)) == 0
    tr = host.reshape(nw, SLOTS)
    stamps = tr[:, 1:].astype(np.int64)
    t0 = stamps[stamps > 0].min()
    out = {}
    for g, name in NAMES.items():
        rows = tr[:, 0] == g
        rows &= stamps[:, 0] > 0
        st = stamps[rows]
        res = []
        for k in range(0, SLOTS - 1):
            col = st[:, k]
            col = col[col > 0]
            if len(col) == 0:
                break
            us = (col - t0) / 100.0
            res.append([k * 96, round(float(np.percentile(us, 5)), 1),
                        round(float(np.median(us)), 1), round(float(np.percentile(us, 95)), 1),
                        int(len(col))])
        out[name] = res
    print(json.dumps({"unit": "us after the first stamp: [step, p5, median, p95, waves]",
                      "groups": out}))
    ctx.close()


if __name__ == "__main__":
    main()
