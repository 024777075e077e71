#!/usr/bin/env python3
"""In-process A/B of Mode R (sva_disparity_ref_d) builds: several libsva
variants loaded side by side time the same reference-rig pair on the same
device buffers, alternating launch by launch; the u8/u16 maps and valid
masks must be byte-identical across variants.  Reports the median and min
per variant and, with --kernels, the ref_match kernel's hipEvent average.

usage: ab_refpath.py lib1.so lib2.so ... [--W 1920 --H 1080 --pair 12-11 --k 20 --iters 20]
"""
import argparse
import ctypes as ct
import json
import os
import statistics
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="+")
    ap.add_argument("--W", type=int, default=1920)
    ap.add_argument("--H", type=int, default=1080)
    ap.add_argument("--pair", default="12-11")
    ap.add_argument("--k", type=int, default=20)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--kernels", action="store_true")
    a = ap.parse_args()
    import torch
    import stereovisionarray_amd as sva   # preloads torch's HIP runtime
    from stereovisionarray_amd import synth
    W, H, k = a.W, a.H, a.k
    i_ref, i_oth = map(int, a.pair.split("-"))
    grid = synth.reference_array(0.036 / W)
    cr, co = sva.Camera.make(*grid[i_ref]), sva.Camera.make(*grid[i_oth])
    ref = synth.texture(H, W, 5)
    oth = np.roll(ref, int(round(0.05 * 0.05 / 0.75 / (0.036 / W))), axis=1)
    dev = torch.device("cuda", 0)
    s = torch.cuda.Stream()
    torch.cuda.set_stream(s)
    d_ref, d_oth = torch.from_numpy(ref).to(dev), torch.from_numpy(oth).to(dev)
    d8 = torch.zeros((H, W), dtype=torch.uint8, device=dev)
    d16 = torch.zeros((H, W), dtype=torch.int16, device=dev)
    val = torch.zeros((H, W), dtype=torch.uint8, device=dev)
    handles = []
    for path in a.libs:
        lib = ct.CDLL(os.path.abspath(path))
        h = ct.c_void_p()
        assert lib.sva_create(0, ct.byref(h)) == 0
        assert lib.sva_set_stream(h, ct.c_void_p(s.cuda_stream)) == 0
        lib.sva_disparity_ref_d.argtypes = [
            ct.c_void_p, ct.c_void_p, ct.c_void_p, ct.c_int, ct.c_int, ct.c_size_t, ct.c_void_p,
            ct.POINTER(sva.Camera), ct.POINTER(sva.Camera), ct.c_int, ct.c_double, ct.c_double,
            ct.c_void_p, ct.c_void_p, ct.c_void_p]
        lib.sva_kernel_time.argtypes = [ct.c_void_p, ct.c_char_p, ct.POINTER(ct.c_double),
                                        ct.POINTER(ct.c_int64)]
        handles.append((os.path.basename(path), lib, h))

    def run(lib, h):
        return lib.sva_disparity_ref_d(h, d_ref.data_ptr(), d_oth.data_ptr(), W, H, W, None,
                                       ct.byref(cr), ct.byref(co), k, 0.5, 1.0, d8.data_ptr(),
                                       d16.data_ptr(), val.data_ptr())

    outs = []
    for n, lib, h in handles:
        d8.zero_(), d16.zero_(), val.zero_()
        assert run(lib, h) == 0, n
        torch.cuda.synchronize()
        outs.append((d8.cpu().numpy().tobytes(), d16.cpu().numpy().tobytes(),
                     val.cpu().numpy().tobytes()))
    assert all(o == outs[0] for o in outs), "variants disagree on the Mode R maps"
    times = {n: [] for n, _, _ in handles}
    for it in range(a.iters + 2):
        if a.kernels and it == 2:
            for n, lib, h in handles:
                lib.sva_set_timing(h, 1)
                lib.sva_reset_timing(h)
        for n, lib, h in handles:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            assert run(lib, h) == 0
            e1.record(s)
            e1.synchronize()
            if it >= 2:
                times[n].append(e0.elapsed_time(e1))
    res = {n: {"median_ms": round(statistics.median(v), 4), "min_ms": round(min(v), 4)}
           for n, v in times.items()}
    if a.kernels:
        for n, lib, h in handles:
            tot, cnt = ct.c_double(0), ct.c_int64(0)
            lib.sva_kernel_time(h, b"ref_match", ct.byref(tot), ct.byref(cnt))
            if cnt.value:
                res[n]["ref_match_ms"] = round(tot.value / cnt.value, 4)
    print(json.dumps({"W": W, "H": H, "pair": a.pair, "k": k, "iters": a.iters,
                      "variants": res}), flush=True)
    for n, lib, h in handles:
        lib.sva_destroy(h)


if __name__ == "__main__":
    main()
