#!/usr/bin/env python3
"""Generate the frozen regression fixtures in tests/golden/ from the CPU oracle.

STATUS: these are NOT reference-generated golden vectors.  The reference
(Nahuel-M/StereoVisionArray) ships no tests or fixtures, and its hot-path
sources need OpenCV, which this image lacks, so it cannot be run here
("parity unpinned").  The oracle they come from is pinned by
the hand-derived KATs in tests/test_oracle_kat.py.  The fixtures freeze the
oracle's outputs on small seeded inputs so that any later change to the
oracle or to the kernels is caught (tests/test_golden.py checks both).

Inputs are regenerated from seeds (synth.texture, MT19937), so each fixture
only stores the expected outputs (uint arrays, np.savez_compressed, no
pickles).  Run:  python tests/golden/make_golden.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

CASES = {
    # Mode S: (W, H, D, dmin, dir/sx, sy, seed)
    "modes_96x64_d64": dict(W=96, H=64, D=64, dmin=0, sx=-1, sy=0, seed=101),
    "modes_80x72_d128_dmin5": dict(W=80, H=72, D=128, dmin=5, sx=1, sy=0, seed=102),
    "modes_64x90_d64_step_2_1": dict(W=64, H=90, D=64, dmin=0, sx=-2, sy=1, seed=103),
    # Mode R: reference rig pair (ref, other), k
    "moder_128x96_12_11_k8": dict(W=128, H=96, ref=12, other=11, k=8, seed=104),
    "moder_128x96_12_17_k6": dict(W=128, H=96, ref=12, other=17, k=6, seed=105),
}


def inputs(name, c):
    from stereovisionarray_amd import synth
    if name.startswith("modes"):
        L, R, _ = synth.stereo_pair2(c["H"], c["W"], c["D"], c["dmin"], c["sx"], c["sy"],
                                     seed=c["seed"]) if c["sy"] or abs(c["sx"]) != 1 else \
            synth.stereo_pair(c["H"], c["W"], c["D"], c["dmin"], c["sx"], seed=c["seed"])
        return L, R
    ref = synth.texture(c["H"], c["W"], c["seed"])
    oth = np.roll(ref, 7, axis=1)
    return ref, oth


def expected(name, c):
    import pyoracle
    from stereovisionarray_amd import synth
    a, b = inputs(name, c)
    if name.startswith("modes"):
        d, s = pyoracle.sgm2(a, b, c["D"], c["dmin"], c["sx"], c["sy"], subpixel=True)
        return {"disp": d, "subpix_bits": s.view(np.uint32)}
    cams = synth.reference_array(0.036 / c["W"])
    d8, d16, v, _ = pyoracle.ref_pair(a, b, pyoracle.OCamera.make(*cams[c["ref"]]),
                                      pyoracle.OCamera.make(*cams[c["other"]]), k=c["k"])
    return {"disp_u8": d8, "disp_u16": d16, "valid": v}


def main():
    for name, c in CASES.items():
        out = expected(name, c)
        np.savez_compressed(os.path.join(HERE, name + ".npz"), **out)
        print(name, {k: v.shape for k, v in out.items()})


if __name__ == "__main__":
    main()
