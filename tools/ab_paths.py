#!/usr/bin/env python3
"""In-process A/B of kernel builds (list a build twice to see the noise
floor: positions in the alternation differ by up to +-2 %): load several libsva variants
(ctypes handles side by side), run sva_paths_d on the SAME device C / L
buffers, alternating variants launch by launch, and report the median
hipEvent time per variant (run-level effects -- memory placement, clocks --
hit every variant alike).

usage: ab_paths.py lib1.so lib2.so ... [--W 1920 --H 1080 --D 128 --iters 30]
"""
import argparse
import ctypes as ct
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="+")
    ap.add_argument("--W", type=int, default=1920)
    ap.add_argument("--H", type=int, default=1080)
    ap.add_argument("--D", type=int, default=128)
    ap.add_argument("--iters", type=int, default=30)
    ap.add_argument("--dir", type=int, default=-1)
    ap.add_argument("--dir-y", type=int, default=0,
                    help="2-D array step (census_cost / cost / sgm entries: census_cost2 for "
                         "supported steps)")
    ap.add_argument("--sub", action="store_true", help="wta_hv / sgm entries: also write the f32 sub-pixel map")
    ap.add_argument("--dmin", type=int, default=0)
    ap.add_argument("--kernels", action="store_true",
                    help="also report each variant's per-kernel hipEvent averages (timing mode 1 "
                         "on every handle; the event packets slow every variant alike)")
    ap.add_argument("--entry", default="paths",
                    choices=["paths", "sgm", "cost", "census", "census_cost", "tile", "wta_hv"])
    a = ap.parse_args()
    import numpy as np
    import torch
    import stereovisionarray_amd as sva   # preloads torch's HIP runtime
    from stereovisionarray_amd import synth

    W, H, D = a.W, a.H, a.D
    dev = torch.device("cuda", 0)
    s = torch.cuda.Stream()
    torch.cuda.set_stream(s)
    L, R, _ = synth.stereo_pair(H, W, D, 0, -1, seed=1)
    dL, dR = torch.from_numpy(L).to(dev), torch.from_numpy(R).to(dev)
    disp = torch.zeros((H, W), dtype=torch.int16, device=dev)
    subm = torch.zeros((H, W), dtype=torch.float32, device=dev)
    C = torch.zeros((H, W, D), dtype=torch.uint8, device=dev)
    L8 = torch.zeros((8, H, W, D), dtype=torch.uint8, device=dev)
    # the tile stages' planes (ABI v5: sized buffers); native widths only
    native = D in (64, 128, 192, 256)
    if a.entry in ("tile", "wta_hv") and not native:
        raise SystemExit(f"--entry {a.entry} needs D in 64/128/192/256")
    lay = sva.tile_layout(W, H, D) if native else None
    HCK = torch.zeros(lay.hckpt_bytes, dtype=torch.uint8, device=dev) if native else None
    # vertical checkpoints at the largest layout any variant reports: 6 planes
    # (§4.11 builds that recompute diagonals carry their row checkpoints here)
    VCK = torch.zeros(lay.vckpt_bytes // (6 - lay.diag_volumes) * 6, dtype=torch.uint8,
                      device=dev) if native else None
    vp = ct.c_void_p

    def tile_call(lib, h):
        return lib.sva_paths_tile_d(h, vp(C.data_ptr()), ct.c_size_t(C.numel()), W, H,
                                    ct.byref(p), vp(L8.data_ptr()), ct.c_size_t(L8.numel()),
                                    vp(HCK.data_ptr()), ct.c_size_t(HCK.numel()),
                                    vp(VCK.data_ptr()), ct.c_size_t(VCK.numel()))

    def wta_hv_call(lib, h):
        return lib.sva_wta_hv_d(h, vp(C.data_ptr()), ct.c_size_t(C.numel()), vp(L8.data_ptr()),
                                ct.c_size_t(L8.numel()), vp(HCK.data_ptr()),
                                ct.c_size_t(HCK.numel()), vp(VCK.data_ptr()),
                                ct.c_size_t(VCK.numel()), W, H, ct.byref(p),
                                vp(disp.data_ptr()), vp(subm.data_ptr()) if a.sub else None)
    p = sva.default_params(D=D, dmin=a.dmin, dir=a.dir, dir_y=a.dir_y, subpixel=1 if a.sub else 0)
    handles = []
    for path in a.libs:
        lib = ct.CDLL(os.path.abspath(path))
        h = ct.c_void_p()
        assert lib.sva_create(0, ct.byref(h)) == 0
        assert lib.sva_set_stream(h, ct.c_void_p(s.cuda_stream)) == 0
        lib.sva_kernel_time.argtypes = [ct.c_void_p, ct.c_char_p, ct.POINTER(ct.c_double),
                                        ct.POINTER(ct.c_int64)]
        handles.append((os.path.basename(path), lib, h))
    # a real cost volume: run the full pipeline once with the first library
    name0, lib0, h0 = handles[0]
    assert lib0.sva_disparity_sgm_d(h0, ct.c_void_p(dL.data_ptr()), ct.c_void_p(dR.data_ptr()), W,
                                    H, ct.c_size_t(W), ct.byref(p), ct.c_void_p(disp.data_ptr()),
                                    None) == 0
    C_src = C
    # build C with the cost stage of lib0 (census via stage calls)
    cl = torch.zeros((H, W), dtype=torch.int64, device=dev)
    cr = torch.zeros((H, W), dtype=torch.int64, device=dev)
    lib0.sva_census_d(h0, ct.c_void_p(dL.data_ptr()), W, H, ct.c_size_t(W), ct.c_void_p(cl.data_ptr()))
    lib0.sva_census_d(h0, ct.c_void_p(dR.data_ptr()), W, H, ct.c_size_t(W), ct.c_void_p(cr.data_ptr()))
    lib0.sva_cost_d(h0, ct.c_void_p(cl.data_ptr()), ct.c_void_p(cr.data_ptr()), W, H, ct.byref(p),
                    ct.c_void_p(C_src.data_ptr()))
    torch.cuda.synchronize()
    C_ref = C_src.clone()          # census -> cost bytes, checked against every census_cost variant
    # tile-stage volumes and checkpoints for the wta_hv entry (first library)
    if native and a.entry in ("tile", "wta_hv"):
        assert tile_call(lib0, h0) == 0
    torch.cuda.synchronize()
    times = {n: [] for n, _, _ in handles}
    ref = None
    for it in range(a.iters + 2):
        if a.kernels and it == 2:            # kernel timing over the measured iterations only
            for n, lib, h in handles:
                lib.sva_set_timing(h, 1)
                lib.sva_reset_timing(h)
        for n, lib, h in handles:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            if a.entry == "paths":
                st = lib.sva_paths_d(h, ct.c_void_p(C.data_ptr()), W, H, ct.byref(p),
                                     ct.c_void_p(L8.data_ptr()))
            elif a.entry == "tile":
                st = tile_call(lib, h)
            elif a.entry == "wta_hv":
                st = wta_hv_call(lib, h)
            elif a.entry == "census":
                st = lib.sva_census_d(h, ct.c_void_p(dL.data_ptr()), W, H, ct.c_size_t(W),
                                      ct.c_void_p(cl.data_ptr()))
            elif a.entry == "census_cost":
                st = lib.sva_census_cost_d(h, ct.c_void_p(dL.data_ptr()), ct.c_void_p(dR.data_ptr()),
                                           W, H, ct.c_size_t(W), ct.byref(p),
                                           ct.c_void_p(C.data_ptr()))
            elif a.entry == "cost":
                st = lib.sva_cost_d(h, ct.c_void_p(cl.data_ptr()), ct.c_void_p(cr.data_ptr()), W, H,
                                    ct.byref(p), ct.c_void_p(C.data_ptr()))
            else:
                st = lib.sva_disparity_sgm_d(h, ct.c_void_p(dL.data_ptr()), ct.c_void_p(dR.data_ptr()),
                                             W, H, ct.c_size_t(W), ct.byref(p),
                                             ct.c_void_p(disp.data_ptr()),
                                             ct.c_void_p(subm.data_ptr()) if a.sub else None)
            e1.record(s)
            assert st == 0, (n, st)
            e1.synchronize()
            if a.entry == "census_cost" and it == 0 and not os.environ.get("AB_NOCHECK"):
                assert torch.equal(C, C_ref), f"{n}: census_cost differs from census -> cost"
            if it >= 2:
                times[n].append(e0.elapsed_time(e1))
        if a.entry == "cost" and it == 0:
            outs = []
            for n, lib, h in handles:
                lib.sva_cost_d(h, ct.c_void_p(cl.data_ptr()), ct.c_void_p(cr.data_ptr()), W, H,
                               ct.byref(p), ct.c_void_p(C.data_ptr()))
                torch.cuda.synchronize()
                outs.append(torch.sum(C.view(torch.int64)).item())
            assert len(set(outs)) == 1, outs
        if a.entry in ("tile", "wta_hv") and it == 0:
            outs = []
            for n, lib, h in handles:
                if a.entry == "tile":
                    tile_call(lib, h)
                else:
                    wta_hv_call(lib, h)
                torch.cuda.synchronize()
                t = L8[:lay.diag_volumes] if a.entry == "tile" else disp
                outs.append(torch.sum(t.view(torch.int64) if t.dtype == torch.uint8 else
                                      t.to(torch.int64)).item())
                if a.entry == "tile":
                    outs[-1] = (outs[-1], torch.sum(HCK.view(torch.int64)).item(),
                                torch.sum(VCK.view(torch.int64)).item())
                if a.entry == "wta_hv" and a.sub:      # sub-pixel maps bit-identical
                    outs[-1] = (outs[-1], torch.sum(subm.view(torch.int32).to(torch.int64)).item())
            if not os.environ.get("AB_NOCHECK"):     # ablation builds compute other values
                assert len(set(outs)) == 1, outs
        if a.entry == "sgm" and it == 0:
            # every variant must produce the same disparities (and sub-pixel map)
            outs = []
            for n, lib, h in handles:
                lib.sva_disparity_sgm_d(h, ct.c_void_p(dL.data_ptr()), ct.c_void_p(dR.data_ptr()),
                                        W, H, ct.c_size_t(W), ct.byref(p),
                                        ct.c_void_p(disp.data_ptr()),
                                        ct.c_void_p(subm.data_ptr()) if a.sub else None)
                torch.cuda.synchronize()
                outs.append((disp.cpu().numpy().tobytes(),
                             subm.cpu().numpy().tobytes() if a.sub else b""))
            if not os.environ.get("AB_NOCHECK"):     # ablation builds compute other values
                assert all(o == outs[0] for o in outs), "variants disagree on the disparity map"
        if a.entry == "paths" and it == 0:
            # every variant must produce the same volumes
            outs = []
            for n, lib, h in handles:
                lib.sva_paths_d(h, ct.c_void_p(C.data_ptr()), W, H, ct.byref(p),
                                ct.c_void_p(L8.data_ptr()))
                torch.cuda.synchronize()
                outs.append(torch.sum(L8.view(torch.int64)).item())
            assert len(set(outs)) == 1, outs
    res = {n: {"median_ms": round(statistics.median(v), 4), "min_ms": round(min(v), 4)}
           for n, v in times.items()}
    if a.kernels:
        for n, lib, h in handles:
            ks = {}
            for k in ("cost", "census", "sgm_paths", "wta_hv"):
                tot, cnt = ct.c_double(0), ct.c_int64(0)
                lib.sva_kernel_time(h, k.encode(), ct.byref(tot), ct.byref(cnt))
                if cnt.value:
                    ks[k] = round(tot.value / cnt.value, 4)
            res[n]["kernels_ms"] = ks
    print(json.dumps({"W": W, "H": H, "D": D, "entry": a.entry, "iters": a.iters,
                      "variants": res}), flush=True)
    for n, lib, h in handles:
        lib.sva_destroy(h)


if __name__ == "__main__":
    main()
