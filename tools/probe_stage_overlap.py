#!/usr/bin/env python3
"""Upper bound of overlapping two consecutive stages of one frame: each pair
of stages run one after the other on one stream, and the same two launches
started together on two streams with no dependency between them (their
inputs are a previous frame's buffers, so the second stage computes from
stale but valid data).  The concurrent time is what a producer/consumer
fusion of the two stages could reach at best.

  python tools/probe_stage_overlap.py [--W 1920 --H 1080 --D 128 --reps 30]
"""
import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--W", type=int, default=1920)
    ap.add_argument("--H", type=int, default=1080)
    ap.add_argument("--D", type=int, default=128)
    ap.add_argument("--reps", type=int, default=30)
    a = ap.parse_args()
    import torch
    import stereovisionarray_amd as sva
    from stereovisionarray_amd import synth

    W, H, D = a.W, a.H, a.D
    dev = torch.device("cuda", 0)
    sA, sB = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    cA, cB = sva.Context(0), sva.Context(0)
    cA.set_stream(sA.cuda_stream)
    cB.set_stream(sB.cuda_stream)
    L, R, _ = synth.stereo_pair(H, W, D, 0, -1, seed=1)
    dL, dR = torch.from_numpy(L).to(dev), torch.from_numpy(R).to(dev)
    p = sva.default_params(D=D, subpixel=1)
    lay = sva.tile_layout(W, H, D)
    mk = lambda n: torch.zeros(n, dtype=torch.uint8, device=dev)  # noqa: E731
    C0, C1 = mk(lay.cost_bytes), mk(lay.cost_bytes)
    DG0, DG1 = mk(lay.diag_bytes), mk(lay.diag_bytes)
    HK0, HK1 = mk(lay.hckpt_bytes), mk(lay.hckpt_bytes)
    VK0, VK1 = mk(lay.vckpt_bytes), mk(lay.vckpt_bytes)
    disp = torch.zeros((H, W), dtype=torch.int16, device=dev)
    sub = torch.zeros((H, W), dtype=torch.float32, device=dev)

    def cc(ctx, C):
        ctx.census_cost_d(dL.data_ptr(), dR.data_ptr(), W, H, W, p, C.data_ptr())

    def tile(ctx, C, DG, HK, VK):
        ctx.paths_tile_d(C.data_ptr(), C.numel(), W, H, p, DG.data_ptr(), DG.numel(),
                         HK.data_ptr(), HK.numel(), VK.data_ptr(), VK.numel())

    def wta(ctx, C, DG, HK, VK):
        ctx.wta_hv_d(C.data_ptr(), C.numel(), DG.data_ptr(), DG.numel(), HK.data_ptr(), HK.numel(),
                     VK.data_ptr(), VK.numel(), W, H, p, disp.data_ptr(), sub.data_ptr())

    for C in (C0, C1):
        cc(cA, C)
    for args in ((C0, DG0, HK0, VK0), (C1, DG1, HK1, VK1)):
        tile(cA, *args)
    torch.cuda.synchronize()

    def timed(fn):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record(sA)
        sB.wait_event(e0)
        fn()
        eb = torch.cuda.Event()
        eb.record(sB)
        sA.wait_event(eb)
        e1.record(sA)
        e1.synchronize()
        return e0.elapsed_time(e1)

    cases = {
        "census_cost": lambda: cc(cA, C1),
        "paths_tile": lambda: tile(cA, C0, DG0, HK0, VK0),
        "wta_hv": lambda: wta(cA, C0, DG0, HK0, VK0),
        "seq census_cost+paths_tile": lambda: (cc(cA, C1), tile(cA, C0, DG0, HK0, VK0)),
        "par census_cost|paths_tile": lambda: (cc(cB, C1), tile(cA, C0, DG0, HK0, VK0)),
        "seq paths_tile+wta_hv": lambda: (tile(cA, C1, DG1, HK1, VK1), wta(cA, C0, DG0, HK0, VK0)),
        "par paths_tile|wta_hv": lambda: (tile(cB, C1, DG1, HK1, VK1), wta(cA, C0, DG0, HK0, VK0)),
        "seq frame stages": lambda: (cc(cA, C0), tile(cA, C0, DG0, HK0, VK0),
                                     wta(cA, C0, DG0, HK0, VK0)),
    }
    res = {k: [] for k in cases}
    for _ in range(3):
        for f in cases.values():
            timed(f)
    for _ in range(a.reps):
        for k, f in cases.items():
            res[k].append(timed(f))
    out = {"W": W, "H": H, "D": D, "unit": "ms, median of reps (hipEvent, both streams joined)"}
    out.update({k: round(statistics.median(v), 4) for k, v in res.items()})
    print(json.dumps(out), flush=True)
    cA.close()
    cB.close()


if __name__ == "__main__":
    main()
