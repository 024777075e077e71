#!/usr/bin/env python3
"""Why does sgm_paths at 4K D=256 run 4.3 ms in one process and 4.9 ms in
another on the same box, with the same bytes and clock?
Probe: time the path kernel (sva_paths_tile_d, SVA_TIMING_PATHS) with the
cost volume, the four diagonal volumes and the checkpoint planes placed by
the caller inside one big allocation, at chosen offsets from one another,
and the frame route on freshly created contexts with and without other
allocations made first.

    python tools/probe_4k_placement.py [--W 3840 --H 2160 --D 256] [--iters 8]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--W", type=int, default=3840)
    ap.add_argument("--H", type=int, default=2160)
    ap.add_argument("--D", type=int, default=256)
    ap.add_argument("--iters", type=int, default=8)
    ap.add_argument("--skews", default="0,256,4096,65536,1048576,2097152,2359296,33554432")
    ap.add_argument("--part", default="stage,frame")
    a = ap.parse_args()
    import torch
    import stereovisionarray_amd as sva
    from stereovisionarray_amd import synth
    W, H, D = a.W, a.H, a.D
    dev = torch.device("cuda", 0)
    s = torch.cuda.Stream(dev)
    torch.cuda.set_stream(s)
    L, R, _ = synth.stereo_pair(H, W, D, 0, -1, seed=1)
    dL, dR = torch.from_numpy(L).to(dev), torch.from_numpy(R).to(dev)
    p = sva.default_params(D=D, subpixel=1)

    def timed(ctx, fn, n):
        fn()
        torch.cuda.synchronize()
        ctx.set_timing(sva.SVA_TIMING_AGG)
        ctx.reset_timing()
        for _ in range(n):
            fn()
        torch.cuda.synchronize()
        out = {k: ctx.kernel_time(k) for k in ("sgm_paths", "wta_hv")}
        ctx.set_timing(0)
        return {k: round(ms / c, 4) for k, (ms, c) in out.items() if c}

    if "stage" in a.part:
        lay = sva.tile_layout(W, H, D)
        ctx = sva.Context(0)
        ctx.set_stream(s.cuda_stream)
        C = torch.zeros(lay.cost_bytes, dtype=torch.uint8, device=dev)
        if D >= 128:
            ctx.census_cost_d(dL.data_ptr(), dR.data_ptr(), W, H, W, p, C.data_ptr())
        torch.cuda.synchronize()
        big = lay.diag_bytes + lay.hckpt_bytes + lay.vckpt_bytes + (64 << 20)
        arena = torch.empty(big, dtype=torch.uint8, device=dev)
        base = arena.data_ptr()
        for skew in [int(v) for v in a.skews.split(",")]:
            diag = base + skew
            hck = diag + lay.diag_bytes
            vck = hck + lay.hckpt_bytes
            if vck + lay.vckpt_bytes > base + big:
                continue
            fn = lambda: ctx.paths_tile_d(C.data_ptr(), C.numel(), W, H, p, diag, lay.diag_bytes,
                                          hck, lay.hckpt_bytes, vck, lay.vckpt_bytes)
            t = timed(ctx, fn, a.iters)
            print(json.dumps({"part": "stage", "skew": skew, "C_mod_2M": C.data_ptr() % (2 << 20),
                              "diag_minus_C_mod_32M": (diag - C.data_ptr()) % (32 << 20),
                              "ms": t}), flush=True)
        del arena, C
        ctx.close()
        torch.cuda.synchronize()
        torch.cuda.empty_cache()

    if "sep" in a.part:
        # cost volume and diagonal volumes in separate allocations, with a
        # ballast allocation before them and between them
        lay = sva.tile_layout(W, H, D)
        for pre_gb, mid_gb in ((0, 0), (3, 0), (0, 3), (1, 0), (2, 0), (0, 1), (5, 0), (16, 0),
                               (0, 0)):
            pre = torch.empty(pre_gb << 30, dtype=torch.uint8, device=dev) if pre_gb else None
            ctx = sva.Context(0)
            ctx.set_stream(s.cuda_stream)
            C = torch.zeros(lay.cost_bytes, dtype=torch.uint8, device=dev)
            ctx.census_cost_d(dL.data_ptr(), dR.data_ptr(), W, H, W, p, C.data_ptr())
            mid = torch.empty(mid_gb << 30, dtype=torch.uint8, device=dev) if mid_gb else None
            dg = torch.empty(lay.diag_bytes, dtype=torch.uint8, device=dev)
            hk = torch.empty(lay.hckpt_bytes, dtype=torch.uint8, device=dev)
            vk = torch.empty(lay.vckpt_bytes, dtype=torch.uint8, device=dev)
            fn = lambda: ctx.paths_tile_d(C.data_ptr(), C.numel(), W, H, p, dg.data_ptr(),
                                          lay.diag_bytes, hk.data_ptr(), lay.hckpt_bytes,
                                          vk.data_ptr(), lay.vckpt_bytes)
            t = timed(ctx, fn, a.iters)
            G = 1 << 30
            print(json.dumps({"part": "sep", "pre_gb": pre_gb, "mid_gb": mid_gb,
                              "C_GB": round(C.data_ptr() / G, 3), "diag_GB": round(dg.data_ptr() / G, 3),
                              "C_mod_1G_MB": (C.data_ptr() % G) >> 20,
                              "diag_mod_1G_MB": (dg.data_ptr() % G) >> 20,
                              "ms": t}), flush=True)
            ctx.close()
            del pre, mid, C, dg, hk, vk
            torch.cuda.synchronize()
            torch.cuda.empty_cache()

    if "alloc" in a.part:
        # the same buffers from hipExtMallocWithFlags, default vs physically
        # contiguous, allocated and freed several times
        import ctypes as ct
        hip = None
        for name in ("libamdhip64.so", "libamdhip64.so.6", "libamdhip64.so.7"):
            try:
                hip = ct.CDLL(name)
                break
            except OSError:
                continue
        hip.hipExtMallocWithFlags.argtypes = [ct.POINTER(ct.c_void_p), ct.c_size_t, ct.c_uint]
        hip.hipFree.argtypes = [ct.c_void_p]
        lay = sva.tile_layout(W, H, D)
        ctx = sva.Context(0)
        ctx.set_stream(s.cuda_stream)
        for flags, label in ((0, "default"), (4, "contiguous")) * 3:
            ptrs = []
            ok = True
            for nbytes in (lay.cost_bytes, lay.diag_bytes, lay.hckpt_bytes, lay.vckpt_bytes):
                pp = ct.c_void_p()
                st = hip.hipExtMallocWithFlags(ct.byref(pp), nbytes, flags)
                if st != 0:
                    ok = False
                    print(json.dumps({"part": "alloc", "mode": label, "error": st}), flush=True)
                    break
                ptrs.append(pp.value)
            if ok:
                Cp, dg, hk, vk = ptrs
                ctx.census_cost_d(dL.data_ptr(), dR.data_ptr(), W, H, W, p, Cp)
                fn = lambda: ctx.paths_tile_d(Cp, lay.cost_bytes, W, H, p, dg, lay.diag_bytes, hk,
                                              lay.hckpt_bytes, vk, lay.vckpt_bytes)
                t = timed(ctx, fn, a.iters)
                print(json.dumps({"part": "alloc", "mode": label, "ms": t}), flush=True)
            torch.cuda.synchronize()
            for pp in ptrs:
                hip.hipFree(pp)
        ctx.close()

    if "frame" in a.part:
        disp = torch.zeros((H, W), dtype=torch.int16, device=dev)
        sub = torch.zeros((H, W), dtype=torch.float32, device=dev)
        for trial, ballast_gb in (("plain", 0), ("ballast_16GB_first", 16), ("plain_again", 0),
                                  ("ballast_3GB_first", 3)):
            ballast = torch.empty(ballast_gb << 30, dtype=torch.uint8, device=dev) if ballast_gb else None
            ctx = sva.Context(0)
            ctx.set_stream(s.cuda_stream)
            ctx.reserve(W, H, D)
            fn = lambda: ctx.disparity_sgm_d(dL.data_ptr(), dR.data_ptr(), W, H, W, p,
                                             disp.data_ptr(), sub.data_ptr())
            t = timed(ctx, fn, a.iters)
            print(json.dumps({"part": "frame", "trial": trial, "ms": t}), flush=True)
            ctx.close()
            del ballast
            torch.cuda.synchronize()
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
