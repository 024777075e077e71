"""Census + cost per 2-D array pair: the census-word
route (census x2 -> hamming_cost2) against the matrix-core census_cost2
kernel, on one stream, 1080p, with the bytes compared.

  python tools/probe_cost2.py [--D 128] [--reps 20]
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import stereovisionarray_amd as sva  # noqa: E402
from stereovisionarray_amd import synth  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--D", type=int, default=128)
    ap.add_argument("--W", type=int, default=1920)
    ap.add_argument("--H", type=int, default=1080)
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    W, H, D = a.W, a.H, a.D
    dev = torch.device("cuda", 0)
    s = torch.cuda.Stream(dev)
    torch.cuda.set_stream(s)
    ctx = sva.Context(0)
    ctx.set_stream(s.cuda_stream)
    out = {"W": W, "H": H, "D": D, "unit": "ms per pair (hipEvent, median of reps)", "steps": {}}
    for sx, sy in [(0, -1), (-1, -1), (1, -1), (2, -1), (3, -1), (-1, 0)]:
        L, R, _ = synth.stereo_pair2(H, W, D, 0, sx, sy, seed=3)
        dL, dR = torch.from_numpy(L).to(dev), torch.from_numpy(R).to(dev)
        p = sva.default_params(D=D, dir=sx, dir_y=sy)
        cl = torch.zeros((H, W), dtype=torch.int64, device=dev)
        cr = torch.zeros((H, W), dtype=torch.int64, device=dev)
        C1 = torch.zeros((H, W, D), dtype=torch.uint8, device=dev)
        C2 = torch.ones((H, W, D), dtype=torch.uint8, device=dev)

        def old():
            ctx.census_d(dL.data_ptr(), W, H, W, cl.data_ptr())
            ctx.census_d(dR.data_ptr(), W, H, W, cr.data_ptr())
            ctx.cost_d(cl.data_ptr(), cr.data_ptr(), W, H, p, C1.data_ptr())

        def new():
            ctx.census_cost_d(dL.data_ptr(), dR.data_ptr(), W, H, W, p, C2.data_ptr())

        def time(f):
            ts = []
            for _ in range(a.reps):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(s)
                f()
                e1.record(s)
                e1.synchronize()
                ts.append(e0.elapsed_time(e1))
            return float(np.median(ts))

        for f in (old, new, old, new):
            f()
        torch.cuda.synchronize()
        res = {"census_words_route": round(time(old), 4), "census_cost_kernel": round(time(new), 4),
               "equal": bool(torch.equal(C1, C2))}
        res["old_again"] = round(time(old), 4)
        res["new_again"] = round(time(new), 4)
        out["steps"][f"{sx},{sy}"] = res
        print(json.dumps({f"{sx},{sy}": res}), flush=True)
    print(json.dumps(out))
    ctx.close()


if __name__ == "__main__":
    main()
