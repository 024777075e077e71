#!/usr/bin/env python3
"""Frame-level stream overlap experiment: consecutive 1080p D=128 frames on
1, 2 or 3 contexts (each its own HIP stream and workspaces), round-robin, so
frame i+1's census/cost/paths can fill frame i's sgm_paths tail (where only
the long horizontal lines still run).  Prints ms per frame for each setting,
interleaved over several rounds."""
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import stereovisionarray_amd as sva
    from stereovisionarray_amd import synth
    W, H, D = 1920, 1080, 128
    frames = int(os.environ.get("FRAMES", "40"))
    dev = torch.device("cuda", 0)
    L, R, _ = synth.stereo_pair(H, W, D, 0, -1, seed=1)
    dL, dR = torch.from_numpy(L).to(dev), torch.from_numpy(R).to(dev)
    p = sva.default_params(D=D, subpixel=1)
    ctxs, streams, outs = [], [], []
    for i in range(3):
        s = torch.cuda.Stream(dev)
        c = sva.Context(0)
        c.set_stream(s.cuda_stream)
        c.reserve(W, H, D)
        ctxs.append(c)
        streams.append(s)
        outs.append((torch.zeros((H, W), dtype=torch.int16, device=dev),
                     torch.zeros((H, W), dtype=torch.float32, device=dev)))

    def run(n):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for f in range(frames):
            k = f % n
            ctxs[k].disparity_sgm_d(dL.data_ptr(), dR.data_ptr(), W, H, W, p,
                                    outs[k][0].data_ptr(), outs[k][1].data_ptr())
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / frames * 1e3

    res = {1: [], 2: [], 3: []}
    for n in (1, 2, 3):
        run(n)
    for _ in range(5):
        for n in (1, 2, 3):
            res[n].append(run(n))
    print(json.dumps({f"contexts_{n}": round(statistics.median(v), 4) for n, v in res.items()}))
    ref = outs[0][0].cpu()
    for k in (1, 2):
        assert torch.equal(outs[k][0].cpu(), ref)


if __name__ == "__main__":
    main()
