#!/usr/bin/env python3
"""Headline benchmark: Mode S (Census -> Hamming -> 8-path SGM -> WTA) in
Mdisparities/s (W*H*D per second) at 1920x1080, D=128 (BASELINE.json config 2).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N \
        --master-addr 127.0.0.1 --master-port P bench.py --gpus N --steps K --warmup W

A step = one full disparity computation of one synthetic 1080p pair per rank
(inputs already resident in HBM), followed for N > 1 by the path's one
exchange: an RCCL gather of the u16 disparity maps to rank 0 over xGMI.
Pairs are independent units (weak scaling: every rank matches its own pair).
Rank 0 prints one JSON line (the driver's contract), including the live
hipEvent roofline of the dominant kernel and the CPU baseline (the oracle,
single thread, the same 1080p D=128 frame) timed on this host.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0          # MI355X HBM3E peak (MI355X_MICROARCH.md)
AGG_BYTES_PER_DISP = 10.0      # 8 u8 C reads + 1 u16 S write

WORKLOADS = {
    "1080p_d128": dict(W=1920, H=1080, D=128),   # BASELINE configs[1]
    "4k_d256": dict(W=3840, H=2160, D=256),      # BASELINE configs[2]
    "1080p_d192": dict(W=1920, H=1080, D=192),   # BASELINE configs[4] per-pair shape
    "vga_d64": dict(W=640, H=480, D=64),         # BASELINE configs[0] shape
    "1080p_d64": dict(W=1920, H=1080, D=64),     # path-kernel selection sweep
    "1080p_d256": dict(W=1920, H=1080, D=256),   # path-kernel selection sweep
    "1080half_d128": dict(W=1920, H=540, D=128), # experiment: C fits the Infinity Cache
    # BASELINE configs[3] as SURVEY.md §8d spells it: getCameraPairs(TO_CENTER_SMALL)
    # = 12 <-> {6,7,8,11,13,16,17,18} (functions.cpp:156-165), one pair per GPU at
    # N=8, gather + median fusion around camera 12
    "center8": dict(W=1920, H=1080, D=128, rig="center8"),
    # BASELINE configs[3] wording: an 8-camera array (2x4 grid), all 28 pairwise
    # baselines, fused per reference camera
    "grid8_all": dict(W=1920, H=1080, D=128, rig="grid8_all"),
    # the reference's own frame size class: its renders are resized by 0.5
    # before matching (CameraStereoVision.cpp:17-18), and SURVEY §6 measures
    # D = 45-49 at 640 px; center8 at 960x540 D=64
    "center8_half_d64": dict(W=960, H=540, D=64, rig="center8"),
    # BASELINE configs[4]: 256 synthetic 1080p pairs (seeds 0-255), D=192,
    # sharded over the ranks (32 per GPU at N=8): fixed total, strong scaling
    "batch256_d192": dict(W=1920, H=1080, D=192, total_pairs=256),
}

ARRAY_PITCH = 0.05             # m between grid neighbours (CameraStereoVision.cpp:34-39)
ARRAY_F = 0.05                 # m
ARRAY_PS = 0.036 / 1920        # m / pixel


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=None,
                    help="timed steps (default 100; 20 for the 256-pair batch workload)")
    ap.add_argument("--warmup", type=int, default=None,
                    help="untimed steps before them (default 50; 5 for the batch workload). "
                         "The first ~20 frames after start-up run 3-4 %% slow (clocks, first "
                         "touches): with 5 warmups a 20-step run measured 0.935 ms per 1080p "
                         "frame, with 50 warmups 0.897 and 200 steps 0.892 "
                         "(profiles/r03_v8/bench_warmup_probe.log.txt)")
    ap.add_argument("--workload", default="1080p_d128", choices=sorted(WORKLOADS))
    ap.add_argument("--pairs-per-rank", type=int, default=1)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--pmc", default="live", choices=["live", "committed"],
                    help="roofline.traffic source: 'live' runs two rocprofv3 PMC passes "
                         "(FETCH_SIZE, WRITE_SIZE) of this workload as child processes on "
                         "rank 0 at N=1 and falls back to the committed profiles/pmc_*.json "
                         "if they fail; 'committed' reads the committed file only")
    ap.add_argument("--cpu-threads", type=int, default=1)
    ap.add_argument("--mode-r-only", action="store_true",
                    help="run only three GPU Mode R frames (pair 12->11, k=20, at --mode-r-size) "
                         "and exit: the child of the Mode R VALU counter pass")
    ap.add_argument("--mode-r-size", default="1920x1080",
                    help="WxH of the --mode-r-only frames: the parent passes the size of the "
                         "frame it timed (mode_r_child_args), so the counters and the kernel "
                         "time describe the same launch")
    ap.add_argument("--streams", type=int, default=0,
                    help="pairs of a step go round-robin to this many contexts, each with its "
                         "own HIP stream and workspaces, so pairs overlap (0 = auto: 2 when a "
                         "rank has several pairs per step and D != 192, else 1)")
    ap.add_argument("--batch", action="store_true",
                    help="a rank's pairs of a step go through sva_disparity_sgm_batch_d on one "
                         "context: one sgm_paths and one wta_hv launch per 8 frames "
                         "(DESIGN.md §4.10) instead of one launch each on --streams contexts")
    ap.add_argument("--no-overlap", action="store_true",
                    help="gather each step's maps synchronously on the compute stream")
    ap.add_argument("--rehearse-overlap", action="store_true",
                    help="N=1 only: run the overlapped-gather stream logic with a device copy "
                         "standing in for the RCCL gather (RCCL refuses 2 ranks on 1 GPU)")
    ap.add_argument("--rehearse-rccl", action="store_true",
                    help="N=1 only: a 1-rank RCCL process group runs the real overlapped "
                         "gather_maps on the comm stream (the N>1 code path on one GPU)")
    ap.add_argument("--placement-trials", type=int, default=0,
                    help="stage-buffer sets sva_reserve's placement check times (0: the "
                         "library default, which checks only frames with >= 4 GiB of stage "
                         "buffers; 1: no check)")
    ap.add_argument("--engine", default="auto", choices=["auto", "multi"],
                    help="auto: --gpus N > 1 without torch.distributed.run drives the N devices "
                         "from this one process through the C-ABI engine (sva_multi_create + "
                         "sva_batch_sgm_d, RCCL ncclCommInitAll gather); multi: that engine at "
                         "any N, N = 1 included")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="nccl = RCCL over xGMI (real runs); gloo = rehearsal with ranks "
                         "sharing one GPU, maps gathered through host memory")
    a = ap.parse_args()
    batch = "total_pairs" in WORKLOADS[a.workload]
    if a.steps is None:
        a.steps = 20 if batch else 100
    if a.warmup is None:
        a.warmup = 5 if batch else 50
    return a


def host_cpu():
    """CPU model and the thread budget this job may use."""
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    nproc = os.cpu_count() or 1
    budget = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or min(nproc, 16)
    return model, nproc, budget


def cpu_baseline(W, H, D, threads):
    """Oracle ('port') timing on this host: the same frame the GPU computes."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle  # CPU baseline leg only
    from stereovisionarray_amd import synth
    L, R, _ = synth.stereo_pair(H, W, D, 0, -1, seed=1)
    t0 = time.perf_counter()
    pyoracle.sgm(L, R, D, 0, -1, 10, 120, subpixel=True, threads=threads)
    dt = time.perf_counter() - t0
    model, nproc, _ = host_cpu()
    return {
        "value": round(W * H * D / dt / 1e6, 3),
        "unit": "Mdisp/s",
        "cores": threads,
        "kind": "port",
        "sample": f"oracle/sgm_oracle.c svo_sgm, one full {W}x{H} D={D} frame "
                  f"(census+cost+8 paths+WTA+subpixel), {threads} thread(s), {dt:.2f} s; "
                  f"host {model}, nproc {nproc}",
    }


def mode_r_beside(ctx, W, H, rows=24, k=20, reps=10):
    """The reference's own path (Mode R: Bresenham candidates + 2k x 2k SAD,
    CameraStereoVision.cpp:44-95), GPU vs its CPU restatement on this host,
    in candidate SADs per second.  Reference rig pair 12 -> 11, k = 20; the
    CPU leg runs a bounded sample of `rows` image rows (1 thread)."""
    import torch
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle  # CPU baseline leg only
    import stereovisionarray_amd as sva
    from stereovisionarray_amd import synth
    cams = synth.reference_array(0.036 / W)
    cr, co = sva.Camera.make(*cams[12]), sva.Camera.make(*cams[11])
    ref = synth.texture(H, W, 5)
    oth = np.roll(ref, int(round(0.05 * 0.05 / 0.75 / (0.036 / W))), axis=1)
    dev = torch.device("cuda", torch.cuda.current_device())
    d_ref, d_oth = torch.from_numpy(ref).to(dev), torch.from_numpy(oth).to(dev)
    d8 = torch.zeros((H, W), dtype=torch.uint8, device=dev)
    ends = torch.zeros((H, W, 4), dtype=torch.int32, device=dev)
    ok = torch.zeros((H, W), dtype=torch.uint8, device=dev)
    ctx.ref_endpoints_d(W, H, cr, co, k, 0.5, 1.0, ends.data_ptr(), ok.data_ptr())
    torch.cuda.synchronize()
    e = ends.cpu().numpy().astype(np.int64)
    okn = ok.cpu().numpy().astype(bool)
    n_cand = int((np.maximum(np.abs(e[..., 0] - e[..., 2]), np.abs(e[..., 1] - e[..., 3])) + 1)[okn].sum())
    run = lambda: ctx.disparity_ref_d(d_ref.data_ptr(), d_oth.data_ptr(), W, H, W, None, cr, co, k,
                                      0.5, 1.0, d8.data_ptr())
    for _ in range(3):          # warm-up (3 timed reps used to sit in the clock ramp)
        run()
    torch.cuda.synchronize()
    ctx.set_timing(1)
    ctx.reset_timing()
    t0 = time.perf_counter()
    for _ in range(reps):
        run()
    torch.cuda.synchronize()
    gdt = (time.perf_counter() - t0) / reps
    km, kn = ctx.kernel_time("ref_match")
    ctx.set_timing(0)
    mask = np.zeros((H, W), np.uint8)
    mask[H // 2 - rows // 2: H // 2 + rows // 2, :] = 1
    t0 = time.perf_counter()
    _, _, _, ncpu = pyoracle.ref_pair(ref, oth, pyoracle.OCamera.make(*cams[12]),
                                      pyoracle.OCamera.make(*cams[11]), k=k, mask=mask)
    cdt = time.perf_counter() - t0
    g, c = n_cand / gdt / 1e6, ncpu / cdt / 1e6
    sample = (f"oracle/refpath_oracle.c svo_ref_pair, {W}x{H} pair 12->11 k={k}: a bounded "
              f"sample of {rows} of the frame's {H} rows (the middle band, masked), "
              f"{ncpu} candidates, {cdt:.2f} s; the rate is per candidate SAD, so it does "
              "not depend on how many rows the sample holds")
    # pixel-SADs the plane kernel evaluates per candidate
    # the reference uses (sampled tiles, tools/mode_r_planes.py)
    try:
        sys.path.insert(0, os.path.join(ROOT, "tools"))
        import mode_r_planes
        red = mode_r_planes.pair_ratio(W, H, k, 12, 11, mode_r_planes.sample_tiles(W, H, k),
                                       ends=e, ok=okn)     # the GPU's own endpoints
    except Exception as e:                      # a report, never the bench's failure
        red = {"error": str(e)[:120]}
    return {"unit": "Mcandidate-SADs/s", "gpu": round(g, 1), "gpu_ms_per_frame": round(gdt * 1e3, 3),
            "sad_planes_per_candidate": red,
            "W": W, "H": H,
            "ref_match_kernel_ms": round(km / kn, 4) if kn else None,
            "cpu": round(c, 3), "cores": 1, "kind": "port", "sample": sample,
            "cpu_baseline": {"value": round(c, 3), "unit": "Mcandidate-SADs/s", "cores": 1,
                             "kind": "port", "sample": sample},
            "gpu_over_cpu": round(g / c, 1)}


def mode_r_child_args(W, H):
    """Arguments of the Mode R PMC child: the frame size mode_r_beside timed."""
    return ["--mode-r-only", "--mode-r-size", f"{int(W)}x{int(H)}"]


def parse_size(s):
    W, H = (int(v) for v in s.lower().split("x"))
    if W <= 0 or H <= 0:
        raise ValueError(f"bad frame size {s!r}")
    return W, H


def mode_r_only(size="1920x1080"):
    """Three GPU Mode R frames of mode_r_beside's workload (the PMC child).
    Writes the frame size it ran to $SVA_MODE_R_STAMP, so that the parent can
    refuse counters taken on a different frame."""
    import torch
    import stereovisionarray_amd as sva
    from stereovisionarray_amd import synth
    W, H = parse_size(size)
    k = 20
    cams = synth.reference_array(0.036 / W)
    cr, co = sva.Camera.make(*cams[12]), sva.Camera.make(*cams[11])
    ref = synth.texture(H, W, 5)
    oth = np.roll(ref, int(round(0.05 * 0.05 / 0.75 / (0.036 / W))), axis=1)
    dev = torch.device("cuda", 0)
    d_ref, d_oth = torch.from_numpy(ref).to(dev), torch.from_numpy(oth).to(dev)
    d8 = torch.zeros((H, W), dtype=torch.uint8, device=dev)
    ctx = sva.Context(0)
    for _ in range(3):
        ctx.disparity_ref_d(d_ref.data_ptr(), d_oth.data_ptr(), W, H, W, None, cr, co, k, 0.5, 1.0,
                            d8.data_ptr())
    torch.cuda.synchronize()
    ctx.close()
    stamp = os.environ.get("SVA_MODE_R_STAMP")
    if stamp:
        with open(stamp, "w") as f:
            json.dump({"W": W, "H": H, "k": k}, f)


def valu_roofline(kernel, c, t_ms, label):
    """VALU issue roofline of one kernel from one SQ counter pass (counters
    averaged per launch, `c`) and its hipEvent time `t_ms`:

      frac          = SQ_INSTS_VALU / (t x VALU_PEAK_PER_S), the chip's SIMD-32
                      issue rate at the 2.4 GHz peak clock (VERDICT r05 weak #2:
                      rounds 3-5 charged 4 cycles per wave64 instruction, which is
                      one wave's own issue interval, and so doubled every VALU
                      fraction);
      frac_of_mix_peak  against the rate tools/microbench_valu.hip measures for
                      this kernel's own static instruction mix at 8 waves/SIMD
                      (VALU_MIX_PEAK_PER_S), where one is measured;
      frac_at_clock = 2 x SQ_INSTS_VALU / (1,024 x GRBM_GUI_ACTIVE / 8): issue
                      slots used out of those the kernel's own active cycles
                      offered (clock-independent; the counter is summed over the
                      8 XCDs, MI355X_MICROARCH.md "DVFS give-back");
    plus the shares of SQ_WAVE_CYCLES that waves spent issuing VALU
    (SQ_ACTIVE_INST_VALU) and waiting (SQ_WAIT_INST_ANY: for an instruction's
    operands, SQ_WAIT_ANY: for anything)."""
    insts = c.get("SQ_INSTS_VALU")
    if not insts or not t_ms:
        raise RuntimeError(f"no {kernel} VALU counters or time")
    ach = insts / (t_ms * 1e-3)
    out = {"bound": "valu", "unit": "wave-instructions/s", "kernel": label,
           "sq_insts_valu": int(insts), "kernel_ms": round(t_ms, 4),
           "achieved_per_s": round(ach, 1), "peak_per_s": round(VALU_PEAK_PER_S, 1),
           "frac": round(ach / VALU_PEAK_PER_S, 4),
           "peak_source": VALU_PEAK_SOURCE}
    mix = VALU_MIX_PEAK_PER_S.get(kernel)
    if mix:
        out["mix_peak_per_s"] = mix
        out["frac_of_mix_peak"] = round(ach / mix, 4)
        out["mix_source"] = VALU_MIX_SOURCE
    g = c.get("GRBM_GUI_ACTIVE")
    dur = c.get("_dur_ns")
    if g:
        out["grbm_gui_active"] = int(g)
        out["frac_at_clock"] = round(VALU_ISSUE_CYCLES * insts / (SIMDS * g / XCDS), 4)
        if dur:
            out["clock_ghz"] = round(g / XCDS / dur, 3)
            out["pmc_kernel_ms"] = round(dur * 1e-6, 4)
    wc = c.get("SQ_WAVE_CYCLES")
    if wc:
        for key, name in (("SQ_ACTIVE_INST_VALU", "active_valu_share"),
                          ("SQ_WAIT_INST_ANY", "wait_inst_any_share"),
                          ("SQ_WAIT_ANY", "wait_any_share")):
            if key in c:
                out[name] = round(c[key] / wc, 4)
        out["sq"] = {k: int(v) for k, v in c.items() if k.startswith("SQ_")}
    return out


def mode_r_roofline(mr):
    """Mode R is VALU/latency-bound, so its roofline is the
    VALU issue rate (valu_roofline), the instructions from one live rocprofv3
    SQ pass over mode_r_only(), the kernel time from the hipEvent-timed
    ref_match launches of mode_r_beside.  The child runs mr's own frame size
    and stamps it; a mismatch is refused, so the fraction never divides one
    frame's instructions by another's time."""
    import tempfile
    outdir = tempfile.mkdtemp(prefix="sva_pmc_r_", dir="/tmp")
    stamp = os.path.join(outdir, "mode_r_stamp.json")
    res = _pmc_pass(SQ_VALU_COUNTERS, [], outdir,
                    child=mode_r_child_args(mr["W"], mr["H"]), env={"SVA_MODE_R_STAMP": stamp})
    with open(stamp) as f:
        ran = json.load(f)
    if (ran["W"], ran["H"]) != (mr["W"], mr["H"]):
        raise RuntimeError(f"Mode R PMC child ran {ran['W']}x{ran['H']}, timed {mr['W']}x{mr['H']}")
    c = res.get("ref_match", {})
    t_ms = mr.get("ref_match_kernel_ms")
    if not c.get("SQ_INSTS_VALU") or not t_ms:
        raise RuntimeError("no ref_plane3_kernel counters")
    out = valu_roofline("ref_match", c, t_ms, "ref_plane3_kernel<20>")
    out["frame"] = f"{mr['W']}x{mr['H']}"
    out["model"] = ("SQ_INSTS_VALU / (ref_match time x 1,024 SIMDs x 2.4 GHz / 2 cycles per "
                    "wave64 VALU instruction)")
    return out


def placement_report(ctxs):
    """sva_reserve's placement check (include/sva.h): per context, the path
    kernel's time on the stage-buffer set it kept and on the slowest set it
    timed; None when no context ran the check (stage buffers below 4 GiB)."""
    import stereovisionarray_amd as sva
    rows = []
    for c in ctxs:
        kept = c.get_debug(sva.SVA_DEBUG_PLACEMENT_NS)
        if kept > 0:
            rows.append({"kept_ms": round(kept * 1e-6, 4),
                         "worst_ms": round(c.get_debug(sva.SVA_DEBUG_PLACEMENT_WORST_NS) * 1e-6, 4)})
    if not rows:
        return None
    return {"contexts": rows,
            "note": "sgm_paths on each trial allocation of the cost / path / checkpoint buffers at "
                    "sva_reserve, best of 3 launches; the fastest set is kept (DESIGN.md §6.0000)"}


def steady_state_beside(step, ctxs, frames=300):
    """ms per frame of the same step on the same context once the GPU has been
    busy for a while (after the timed region and the CPU baseline): the
    driver's 5 / 20 run starts from idle and sits inside the clock ramp
    (DESIGN.md §6.00).  Context only, never `value`."""
    import torch
    for _ in range(200):
        step(False)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(frames):
        step(False)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / frames * 1e3
    return {"ms_per_frame": round(ms, 4), "frames": frames,
            "note": "200 + 300 more steps on the same context after the timed region; not the "
                    "headline value"}


def frame_overlap_beside(W, H, D, frames=40, rounds=2):
    """ms per frame for consecutive frames issued round-robin on 1 or 2
    contexts (each its own stream and workspaces).  The frame's kernels are
    HBM-bound, so a second stream gains only the launch gaps and the
    horizontal-line tail of the path kernel."""
    import torch
    import stereovisionarray_amd as sva
    from stereovisionarray_amd import synth
    dev = torch.device("cuda", torch.cuda.current_device())
    L, R, _ = synth.stereo_pair(H, W, D, 0, -1, seed=1)
    dL, dR = torch.from_numpy(L).to(dev), torch.from_numpy(R).to(dev)
    p = sva.default_params(D=D, subpixel=1)
    ctxs, streams, outs = [], [], []
    for _ in range(2):
        s = torch.cuda.Stream(dev)
        c = sva.Context(torch.cuda.current_device())
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
            i = f % n
            ctxs[i].disparity_sgm_d(dL.data_ptr(), dR.data_ptr(), W, H, W, p,
                                    outs[i][0].data_ptr(), outs[i][1].data_ptr())
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / frames * 1e3

    run(2)
    best = {}
    for _ in range(rounds):
        for n in (1, 2):
            t = run(n)
            best[n] = min(best.get(n, t), t)
    for c in ctxs:
        c.close()
    res = {f"{n}_streams": round(best[n], 4) for n in (1, 2)}
    res["unit"] = "ms/frame"
    res["note"] = (f"{frames} consecutive {W}x{H} D={D} frames round-robin on 1 or 2 contexts "
                   "(own stream + workspaces), best of 2 rounds; not the headline value")
    return res


def load_traffic(workload, kernel="sgm_paths"):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 PMC pass
    (profiles/pmc_<workload>.json, written by tools/pmc_traffic.py), or None."""
    p = os.path.join(ROOT, "profiles", f"pmc_{workload}.json")
    if not os.path.exists(p):
        return None
    try:
        with open(p) as f:
            d = json.load(f)
        return d.get("kernels", {}).get(kernel, {}).get("hbm_bytes_per_launch")
    except Exception:
        return None


def committed_traffic(workload):
    """{kernel: {"hbm_bytes_per_launch": ...}} from the committed PMC pass, or None."""
    p = os.path.join(ROOT, "profiles", f"pmc_{workload}.json")
    try:
        with open(p) as f:
            return json.load(f).get("kernels")
    except Exception:
        return None


# rocprofv3 kernel names -> bench timer names (the PMC pass reports per kernel)
PMC_KERNELS = {"sgm_paths_kernel": "sgm_paths", "wta_hv_kernel": "wta_hv",
               "census_cost_mma_kernel": "cost", "ref_plane3_kernel": "ref_match"}
MI355X_ENGINE_GHZ = 2.4   # peak engine clock (MI355X_MICROARCH.md)
SIMDS = 1024              # 256 CUs x 4 SIMDs
XCDS = 8                  # GRBM_GUI_ACTIVE is summed over the 8 XCDs
# MI355X_MICROARCH.md "Wave scheduling" (:53-54): each CU has 4 SIMD-32 units
# and a wave64 VALU instruction issues over 2 cycles; the 4 cycles of its
# 'vector-instruction ISSUE cost' row are what ONE wave alone sustains.
VALU_ISSUE_CYCLES = 2.0
VALU_PEAK_PER_S = SIMDS * MI355X_ENGINE_GHZ * 1e9 / VALU_ISSUE_CYCLES     # 1.2288e12
VALU_PEAK_SOURCE = ("1,024 SIMD-32 units x 2.4 GHz / 2 cycles per wave64 VALU instruction "
                    "(MI355X_MICROARCH.md Wave scheduling)")
# The same ceiling measured for each kernel's own instruction mix:
# tools/microbench_valu.hip kinds 18 / 19 (the static VALU mix of
# wta_hv_kernel<8,3,false> and of ref_plane3_kernel<20>'s per-plane body,
# tools/isa_mix.py), best of 1/2/4/8 waves per SIMD, chip-wide wave-instructions
# per second from the kernel's hipEvent time (profiles/r06_v1/microbench_valu.txt).
# Measured: 64-bit-encoded VALU (VOP3 / VOP3P / DPP: v_perm, v_add3, v_pk_*,
# v_sad_u8, DPP min/add) issue at about half the SIMD-32 rate on gfx950
# (0.47 of 1.229e12 at 8 waves/SIMD), 32-bit VOP2 at 0.84 (v_add_u32), and
# these kernels are ~90 % the former.  sgm_paths runs the same recurrence
# step as wta_hv, so it is graded on the wta_hv mix.
VALU_MIX_PEAK_PER_S = {"wta_hv": 5.931e11, "sgm_paths": 5.931e11, "ref_match": 6.348e11}
VALU_MIX_SOURCE = "tools/microbench_valu.hip mix kinds, profiles/r06_v1/microbench_valu.txt"
SQ_VALU_COUNTERS = ("SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_WAVE_CYCLES "
                    "SQ_BUSY_CYCLES GRBM_GUI_ACTIVE")
EA_COUNTERS = "TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum GRBM_GUI_ACTIVE"


def _pmc_pass(counter, args, outdir, child=None, env=None):
    """One rocprofv3 PMC pass (one counter group, kernel trace only) over a short
    run of this bench as a CHILD process; returns {timer name: mean counter per
    launch} (several counters: {timer name: {counter: mean}})."""
    import csv
    import shutil
    import subprocess
    prof = shutil.which("rocprofv3") or "/opt/rocm/bin/rocprofv3"
    counters = counter.split()
    d = os.path.join(outdir, counters[0].lower())
    child = child if child is not None else ["--steps", "3", "--warmup", "1", "--no-cpu-baseline",
                                             "--pmc", "committed", "--streams", "1"] + args
    cmd = ["timeout", "-s", "KILL", "150", prof, "--pmc"] + counters + ["--kernel-trace",
           "-d", d, "-o", "run", "--output-format", "csv", "--",
           sys.executable, os.path.abspath(__file__)] + child
    env = dict(os.environ, TMPDIR="/tmp", SVA_BENCH_PMC_CHILD="1", **(env or {}))
    r = subprocess.run(cmd, cwd="/tmp", env=env, capture_output=True, text=True, timeout=170)
    if r.returncode != 0:
        raise RuntimeError(f"rocprofv3 --pmc {counter} exited {r.returncode}: {r.stderr[-300:]}")
    path = os.path.join(d, "run_counter_collection.csv")
    agg, durs = {}, {}
    for row in csv.DictReader(open(path)):
        name = row["Kernel_Name"]
        for key, short in PMC_KERNELS.items():
            if key + "<" in name or key + "(" in name:
                agg.setdefault((short, row["Counter_Name"]), []).append(float(row["Counter_Value"]))
                try:
                    durs.setdefault(short, {})[row["Dispatch_Id"]] = \
                        float(row["End_Timestamp"]) - float(row["Start_Timestamp"])
                except (KeyError, ValueError):
                    pass
                break
    if len(counters) == 1:
        return {k: sum(v) / len(v) for (k, _), v in agg.items()}
    out = {}
    for (k, c), v in agg.items():
        out.setdefault(k, {})[c] = sum(v) / len(v)
    for k, dd in durs.items():      # kernel duration under this pass, ns
        if k in out and dd:
            out[k]["_dur_ns"] = sum(dd.values()) / len(dd)
    return out


def live_traffic(a):
    """HBM bytes per launch for every pipeline kernel from two live rocprofv3 PMC
    passes, corrected as MI355X_MICROARCH.md's HBM section prescribes: separate
    FETCH_SIZE and WRITE_SIZE runs (kB units), FETCH_SIZE doubled on gfx950 (it
    tallies 128-B streaming reads at 64 B), WRITE_SIZE exact for 16-B stores."""
    import tempfile
    outdir = tempfile.mkdtemp(prefix="sva_pmc_", dir="/tmp")
    args = ["--workload", a.workload, "--pairs-per-rank", str(a.pairs_per_rank)]
    if getattr(a, "batch", False):
        args.append("--batch")     # per-launch bytes of the batched launches the line grades
    fetch = _pmc_pass("FETCH_SIZE", args, outdir)
    write = _pmc_pass("WRITE_SIZE", args, outdir)
    out = {}
    for k in sorted(set(fetch) | set(write)):
        rd, wr = fetch.get(k, 0.0) * 1024 * 2.0, write.get(k, 0.0) * 1024
        out[k] = {"hbm_read_bytes": int(rd), "hbm_write_bytes": int(wr),
                  "hbm_bytes_per_launch": int(rd + wr)}
    return out


def engine_counters(a):
    """Two more live PMC passes over this workload (N = 1, rank 0): the SQ
    VALU set for every pipeline kernel, and the L2's memory-side requests with
    the engine clock for the dominant kernel (tells a
    slower box's clock from its memory)."""
    import tempfile
    outdir = tempfile.mkdtemp(prefix="sva_pmc_e_", dir="/tmp")
    args = ["--workload", a.workload, "--pairs-per-rank", str(a.pairs_per_rank)]
    return _pmc_pass(SQ_VALU_COUNTERS, args, outdir), _pmc_pass(EA_COUNTERS, args, outdir)


def ea_figures(c, t_ms):
    """roofline.engine: clock and TCC EA request bytes of one kernel.  Reads:
    RDREQ x 128 B (gfx950 tallies a 128-B streaming read as one 64-B request
    in FETCH_SIZE = RDREQ x 64 B, MI355X_MICROARCH.md HBM); writes:
    WRREQ_64B x 64 B + (WRREQ - WRREQ_64B) x 32 B."""
    rd, wr, w64 = (c.get(k) for k in ("TCC_EA0_RDREQ_sum", "TCC_EA0_WRREQ_sum",
                                       "TCC_EA0_WRREQ_64B_sum"))
    out = {"source": "live rocprofv3 --pmc " + EA_COUNTERS}
    g, dur = c.get("GRBM_GUI_ACTIVE"), c.get("_dur_ns")
    if g and dur:
        out["clock_ghz"] = round(g / XCDS / dur, 3)
        out["pmc_kernel_ms"] = round(dur * 1e-6, 4)
        out["grbm_gui_active"] = int(g)
    if rd is not None:
        out["ea_rdreq"] = int(rd)
        out["ea_read_bytes"] = int(rd * 128)
    if wr is not None and w64 is not None:
        out["ea_wrreq"] = int(wr)
        out["ea_wrreq_64b"] = int(w64)
        out["ea_write_bytes"] = int(w64 * 64 + (wr - w64) * 32)
    if "ea_read_bytes" in out and "ea_write_bytes" in out and t_ms:
        tot = out["ea_read_bytes"] + out["ea_write_bytes"]
        out["ea_bytes"] = tot
        out["ea_gbs_at_event_time"] = round(tot / (t_ms * 1e-3) / 1e9, 1)
    return out


def attach_engine(a, out, kernels, world):
    """valu_roofline per pipeline kernel and roofline.engine (clock + EA bytes)
    from engine_counters(), on rank 0 at N = 1 with --pmc live only."""
    under_prof = any(k.startswith("ROCPROF") for k in os.environ) or \
        os.environ.get("SVA_BENCH_PMC_CHILD")
    if a.pmc != "live" or world != 1 or under_prof or getattr(a, "batch", False):
        return
    try:
        sq, ea = engine_counters(a)
    except Exception as e:                           # keep the bench line; say why
        out["valu_roofline"] = {"error": str(e)[:200]}
        return
    labels = {"sgm_paths": "sgm_paths_kernel", "wta_hv": "wta_hv_kernel",
              "cost": "census_cost_mma_kernel"}
    vr = {}
    for k, label in labels.items():
        if k in sq and k in kernels:
            try:
                vr[k] = valu_roofline(k, sq[k], kernels[k]["avg_ms"], label)
            except RuntimeError:
                pass
    out["valu_roofline"] = vr
    rf = out.get("roofline")
    if rf and rf.get("kernel") in ea:
        rf["engine"] = ea_figures(ea[rf["kernel"]], rf.get("kernel_avg_ms"))
    ag = out.get("aggregation_roofline")
    if ag:
        ag["engine"] = {k: ea_figures(ea[k], kernels.get(k, {}).get("avg_ms"))
                        for k in AGG_KERNELS if k in ea}


def attach_traffic(a, out, world):
    """roofline.traffic: live PMC passes on rank 0 at N=1 (a.pmc == 'live', not
    when this process is itself a PMC child or already under a profiler), else
    the committed profiles/pmc_<workload>.json figure."""
    rf = out.get("roofline")
    if not rf:
        return
    under_prof = any(k.startswith("ROCPROF") for k in os.environ) or \
        os.environ.get("SVA_BENCH_PMC_CHILD")
    if a.pmc == "live" and world == 1 and not under_prof:
        try:
            t0 = time.time()
            kern = live_traffic(a)
            rf["traffic"] = kern.get(rf["kernel"], {}).get("hbm_bytes_per_launch")
            rf["traffic_source"] = ("live: rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of this "
                                    "workload (3 steps each, FETCH_SIZE x2 gfx950 correction), "
                                    f"{time.time() - t0:.1f} s")
            rf["traffic_per_kernel"] = kern
            if rf["traffic"]:
                rf["traffic_over_alg"] = round(rf["traffic"] / rf["alg_bytes_per_launch"], 3)
            ag = out.get("aggregation_roofline")
            if ag and all(k in kern for k in AGG_KERNELS):
                ag["traffic"] = sum(kern[k]["hbm_bytes_per_launch"] for k in AGG_KERNELS)
                ag["traffic_over_alg"] = round(ag["traffic"] / ag["alg_bytes_per_launch"], 3)
                ag["traffic_source"] = "live (the roofline's PMC passes)"
            return
        except Exception as e:                       # keep the bench line; say why
            rf["traffic_source"] = f"committed (live PMC pass failed: {str(e)[:200]})"
            return
    rf["traffic_source"] = f"committed profiles/pmc_{a.workload}.json"


def timed(a, step, world, dev, ctx):
    """W untimed steps, then exactly K steps between barrier + synchronize,
    max over ranks.  ctx: one context or a list (kernel timing on all)."""
    ctxs = ctx if isinstance(ctx, list) else [ctx]
    import torch
    import torch.distributed as dist
    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    for c in ctxs:
        # only the two aggregation kernels are event-timed in the timed region
        # (their own dispatch events): a timed launch costs a few us of stream
        # time, every kernel timed cost ~2.5 %
        c.set_timing(3)          # SVA_TIMING_AGG: sgm_paths + wta_hv
        c.reset_timing()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    for c in ctxs:
        c.set_timing(False)
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64,
                         device=dev if a.dist_backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    return elapsed


def breakdown(a, step, world, ctx, timed_kernels):
    """Per-kernel averages of every pipeline kernel from a short pass after the
    timed region (all launches event-timed); sgm_paths and wta_hv keep their
    timed-region figures, which the rooflines use."""
    import torch
    import torch.distributed as dist
    ctxs = ctx if isinstance(ctx, list) else [ctx]
    for c in ctxs:
        c.set_timing(1)          # SVA_TIMING_ALL
        c.reset_timing()
    for _ in range(min(a.steps, 5)):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    kernels = kernel_table(ctxs)
    for c in ctxs:
        c.set_timing(0)
    for k in AGG_KERNELS:
        if k in timed_kernels:
            kernels[k] = timed_kernels[k]
    return kernels


def exchange_report(a, step, world, rank, dev, ctxs, last, n_units, ms_per_step, recompute):
    """The path's one exchange, checked and timed once after the timed region
    (N > 1, or the 1-rank RCCL rehearsal):
      * the last step's maps are gathered again with a per-unit checksum that
        each owner computed before sending (dist.gather_maps_checked), and
        rank 0 checks every received map against it;
      * rank 0 recomputes one unit owned by another rank (unit 1, or unit 0
        at N = 1) from its seed and compares the bytes with the gathered map;
      * the gather alone is timed, and the steps are re-timed without it: the
        difference is the gather time the overlap does not hide.
    Returns the report on rank 0 (None elsewhere)."""
    import torch
    import torch.distributed as dist
    from stereovisionarray_amd import dist as sdist
    gloo = a.dist_backend == "gloo" and world > 1
    torch.cuda.synchronize()
    src = last.cpu() if gloo else last
    maps, ok = sdist.gather_maps_checked(src, n_units, dst=0)
    remote = None
    if rank == 0:
        u = 1 if n_units > 1 else 0
        mine = recompute(u)
        torch.cuda.synchronize()
        remote = {"unit": u, "owner_rank": u % world,
                  "equal": bool(torch.equal(mine.cpu(), maps[u].cpu()))}

    def max_over_ranks(x):
        if world == 1:
            return x
        t = torch.tensor([x], dtype=torch.float64, device="cpu" if gloo else dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    n = min(a.steps, 10)
    torch.cuda.synchronize()
    dist.barrier()
    t0 = time.perf_counter()
    for _ in range(n):
        sdist.gather_maps(src, n_units, dst=0)
    torch.cuda.synchronize()
    gather_ms = max_over_ranks((time.perf_counter() - t0) / n * 1e3)
    compute_ms = timed(a, lambda: step(False), world, dev, ctxs) / a.steps * 1e3
    if rank != 0:
        return None
    return {"backend": "gloo" if gloo else "rccl", "world": dist.get_world_size(),
            "rccl_world": None if gloo else dist.get_world_size(),
            "units_checked": n_units, "checksums_ok": ok, "remote_unit_recomputed": remote,
            "ok": bool(ok and remote["equal"]),
            "gather_ms": round(gather_ms, 4),
            "compute_only_ms_per_step": round(compute_ms, 4),
            "exposed_gather_ms_per_step": round(ms_per_step - compute_ms, 4),
            "map_bytes_per_unit": int(last[0].numel() * last.element_size())}


def kernel_table(ctx, names=("census", "cost", "sgm_paths", "wta_hv", "fuse_depth")):
    """Average hipEvent duration per kernel, pooled over one or several contexts
    (with --streams > 1 the launches overlap, so durations include contention)."""
    ctxs = ctx if isinstance(ctx, list) else [ctx]
    kernels = {}
    for name in names:
        ms = n = 0
        for c in ctxs:
            m1, n1 = c.kernel_time(name)
            ms, n = ms + m1, n + n1
        if n:
            kernels[name] = {"avg_ms": ms / n, "launches": n}
    return kernels


# Algorithmic bytes per launch of the path-aggregation kernel:
# SURVEY.md §8(d)'s aggregation model, 10 B/disp (8 u8 C reads + one u16 S
# write), whatever the kernel spills.
def roofline_of(kernels, W, H, D, workload, overlapped=False, frames_per_launch=1):
    name = "sgm_paths"
    agg = kernels.get(name)
    if not agg:
        return None
    model = "SURVEY §8d aggregation: 10 B/disp"
    alg_bytes = AGG_BYTES_PER_DISP * W * H * D * frames_per_launch
    achieved = alg_bytes / (agg["avg_ms"] * 1e-3) / 1e9
    out = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
           "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
           # the committed PMC file holds single-frame launches: a batched launch
           # (frames_per_launch > 1) gets its traffic from the live passes only
           "traffic": load_traffic(workload, name) if frames_per_launch == 1 else None,
           "kernel": name, "kernel_avg_ms": round(agg["avg_ms"], 4),
           "alg_bytes_per_launch": alg_bytes, "model": model}
    if overlapped:
        # pairs overlap on several streams: a launch's event span includes the
        # other stream's kernels, so this fraction is not the single-stream one
        out["overlapped"] = True
    if frames_per_launch != 1:
        out["frames_per_launch"] = frames_per_launch
    return out


# The aggregation as the tile pipeline splits it: sgm_paths
# runs all 8 recurrences and wta_hv re-runs the 4 horizontal / vertical ones
# per tile, sums S and picks d*.  Graded together over SURVEY.md §8(d)'s
# aggregation (10 B/disp) + WTA (2 B/disp + 2 B/px) bytes, from both kernels'
# timed-region hipEvent averages, so moving work between the two kernels
# cannot move the grade.
AGG_KERNELS = ("sgm_paths", "wta_hv")
# sva_disparity_sgm_batch_d (sva_tuning.h): calls are split into chunks of at
# most 8 frames, each aggregated in sub-batches of 4 frames per launch
BATCH_MAX_PAIRS = 8
BATCH_SUB_FRAMES = 4


def batch_groups(n, groups):
    """[j0, j1) of each of `groups` contiguous batch calls over n pairs."""
    g = max(1, min(groups, n))
    return [(n * i // g, n * (i + 1) // g) for i in range(g)] + [(n, n)] * (groups - g)


def batch_frames_per_launch(n, groups=1):
    """Mean frames per aggregation launch of `groups` batch calls over n pairs."""
    launches = frames = 0
    for j0, j1 in batch_groups(n, groups):
        m = j1 - j0
        for c0 in range(0, m, BATCH_MAX_PAIRS):
            cm = min(BATCH_MAX_PAIRS, m - c0)
            launches += -(-cm // BATCH_SUB_FRAMES)
            frames += cm
    return frames / launches if launches else 1


def aggregation_roofline_of(kernels, W, H, D, traffic_per_kernel=None, overlapped=False,
                            frames_per_launch=1):
    if not all(k in kernels for k in AGG_KERNELS):
        return None
    ms = sum(kernels[k]["avg_ms"] for k in AGG_KERNELS)
    alg = ((AGG_BYTES_PER_DISP + 2.0) * W * H * D + 2.0 * W * H) * frames_per_launch
    ach = alg / (ms * 1e-3) / 1e9
    out = {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
           "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": None,
           "kernels": list(AGG_KERNELS),
           "kernels_avg_ms": {k: round(kernels[k]["avg_ms"], 4) for k in AGG_KERNELS},
           "sum_ms": round(ms, 4), "alg_bytes_per_launch": alg,
           "model": "SURVEY §8d aggregation 10 B/disp + WTA 2 B/disp + 2 B/px, "
                    "sgm_paths + wta_hv timed-region averages"}
    if traffic_per_kernel and all(k in traffic_per_kernel for k in AGG_KERNELS) \
            and frames_per_launch == 1:      # committed bytes are single-frame launches
        out["traffic"] = sum(traffic_per_kernel[k]["hbm_bytes_per_launch"] for k in AGG_KERNELS)
        out["traffic_over_alg"] = round(out["traffic"] / alg, 3)
    if overlapped:
        out["overlapped"] = True
    if frames_per_launch != 1:
        out["frames_per_launch"] = frames_per_launch
    return out


def frame_roofline(W, H, D, ms_per_frame):
    """The whole frame against SURVEY §8d's per-stage algorithmic bytes:
    census 18 B/px, cost 16 B/px + 1 B/disp, aggregation 10 B/disp, WTA
    2 B/disp + 2 B/px, over the measured time per frame (all kernels and the
    launch gaps between them)."""
    alg = 13.0 * W * H * D + 36.0 * W * H
    ach = alg / (ms_per_frame * 1e-3) / 1e9
    return {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(ach / HBM_PEAK_GBS, 4), "alg_bytes_per_frame": alg,
            "ms_per_frame": round(ms_per_frame, 4),
            "model": "SURVEY §8d census+cost+aggregation+WTA: 13 B/disp + 36 B/px"}


def rig_of(name):
    """(grid positions, pairs, label).  Positions are in grid units relative to
    the first pair's reference camera, which therefore sees the texture
    unwarped (used by the sanity check)."""
    from stereovisionarray_amd import synth
    if name == "center8":
        g = [(i % 5 - 2, i // 5 - 2) for i in range(25)]      # 5x5, camera 12 at (0,0)
        return g, [(12, j) for j in (6, 7, 8, 11, 13, 16, 17, 18)], \
            "getCameraPairs(TO_CENTER_SMALL): 12 <-> {6,7,8,11,13,16,17,18}"
    g = synth.array_grid(2, 4)
    return g, synth.array_pairs(len(g)), "2x4 grid, all 28 pairwise baselines"


def run_array(a, wl, world, rank, local, dev):
    """BASELINE configs[3]: camera-array pairs at 1080p D=128.  Pair u
    (grouped by reference camera) is matched by rank u mod N along its own
    baseline step; the u16 maps are gathered to rank 0
    (RCCL), which fuses, per reference camera, the median depth over that
    camera's pairs.  Total work is fixed (strong scaling)."""
    import torch
    import torch.distributed as dist
    import stereovisionarray_amd as sva
    from stereovisionarray_amd import dist as sdist
    from stereovisionarray_amd import synth

    W, H, D = wl["W"], wl["H"], wl["D"]
    grid, pairs, rig_label = rig_of(wl["rig"])
    n_units = len(pairs)
    kmax = max(synth.pair_step(grid[i], grid[j])[2] for i, j in pairs)
    dmax = min((D - 1) // kmax, 100)
    delta = synth.array_delta(H, W, dmax)
    used = sorted({c for p in pairs for c in p})
    views_np = dict(zip(used, synth.array_views(H, W, [grid[c] for c in used], delta, seed=7)))

    ctx = sva.Context(local)
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    ctx.set_stream(stream.cuda_stream)
    ctx.reserve(W, H, D)
    mine = sdist.shard(n_units, rank, world)
    need = sorted({c for u in mine for c in pairs[u]})
    views = {c: torch.from_numpy(views_np[c]).to(dev) for c in need}
    jobs = []
    for u in mine:
        i, j = pairs[u]
        sx, sy, _ = synth.pair_step(grid[i], grid[j])
        jobs.append((views[i], views[j], sva.default_params(D=D, dmin=0, dir=sx, dir_y=sy)))
    disp = torch.zeros((len(mine), H, W), dtype=torch.int16, device=dev)
    # fusion groups on rank 0: reference camera i owns pairs [off, off + n)
    groups, off = [], 0
    for i in dict.fromkeys(p[0] for p in pairs):     # pairs are grouped by reference
        n = sum(1 for p in pairs if p[0] == i)
        bases = [synth.pair_step(grid[i], grid[j])[2] * ARRAY_PITCH
                 for (_, j) in pairs[off:off + n]]
        groups.append((i, off, n, bases))
        off += n
    depth = torch.zeros((len(groups), H, W), dtype=torch.float64, device=dev)
    nvalid = torch.zeros((len(groups), H, W), dtype=torch.uint8, device=dev)
    maps = {"all": None}
    # pairs alternate over n_streams contexts (own stream and workspaces) so
    # consecutive pairs overlap; gather and fusion wait for all of them.
    # Three streams (profiles/r03_v8/streams_arrays.log.txt, one box): center8
    # 311.2-315.0K (2) -> 319.7-321.0K (3) -> 309.3K (4) Mdisp/s; grid8_all
    # 316.2-316.9K (2) -> 316.4-318.1K (3) -> 305.2-308.1K (4).
    n_streams = a.streams if a.streams > 0 else (min(3, len(jobs)) if len(jobs) > 1 else 1)
    if a.batch and a.streams <= 0:
        n_streams = 1                    # the batch runs on one context (--streams S: S batches)
    ctxs, cstreams = [ctx], [stream]
    for _ in range(1, n_streams):
        s_ = torch.cuda.Stream(dev)
        c_ = sva.Context(local)
        c_.set_stream(s_.cuda_stream)
        c_.reserve(W, H, D)
        ctxs.append(c_)
        cstreams.append(s_)

    # compute-only steps (exchange_report) fuse a stand-in buffer of the full size
    # multi: the exchange runs (N > 1, or a 1-rank RCCL group with --rehearse-rccl)
    multi = world > 1 or a.rehearse_rccl
    stand_in = torch.zeros((n_units, H, W), dtype=torch.int16, device=dev) \
        if multi and rank == 0 else None
    # N > 1 over RCCL: step i computes into map buffer i % 2 while the gather
    # of step i - 1 and rank 0's fusion of it run on a comm stream (fused by a
    # context bound to that stream), as in main()
    overlap = multi and a.dist_backend == "nccl" and not a.no_overlap
    disps = [disp] + ([torch.zeros_like(disp)] if overlap else [])
    comm = torch.cuda.Stream(dev) if overlap else None
    fctx = None
    if overlap and rank == 0:
        fctx = sva.Context(local)
        fctx.set_stream(comm.cuda_stream)
    pending = [None] * len(disps)        # buffer -> event after its gather (+ fusion)
    it = [0]

    def fuse(c, allm):
        for g, (i, o, n, bases) in enumerate(groups):
            c.fuse_depth_d(allm[o].data_ptr(), n, W, H, bases, ARRAY_F, ARRAY_PS, 0xFFFF,
                           depth[g].data_ptr(), nvalid[g].data_ptr())
        maps["all"] = allm

    def step(exchange=True):
        b = it[0] % len(disps)
        it[0] += 1
        dsp = disps[b]
        if pending[b] is not None:       # this buffer's previous gather has read it
            stream.wait_event(pending[b])
            pending[b] = None
        if len(ctxs) > 1:                # the previous step's fusion has read disp
            go = torch.cuda.Event()
            go.record(stream)
            for s_ in cstreams[1:]:
                s_.wait_event(go)
        if a.batch:
            # --streams S: the pairs in S contiguous groups, one batch call per context
            for c_, (j0, j1) in zip(ctxs, batch_groups(len(jobs), len(ctxs))):
                if j1 > j0:
                    c_.disparity_sgm_batch_d([(L.data_ptr(), R.data_ptr(), p) for (L, R, p) in
                                              jobs[j0:j1]], W, H, W, dsp[j0].data_ptr())
        else:
            for jb, (L, R, p) in enumerate(jobs):
                ctxs[jb % len(ctxs)].disparity_sgm_d(L.data_ptr(), R.data_ptr(), W, H, W, p,
                                                     dsp[jb].data_ptr())
        for s_ in cstreams[1:]:
            done_ = torch.cuda.Event()
            done_.record(s_)
            stream.wait_event(done_)
        if multi and exchange and overlap:
            ev = torch.cuda.Event()
            ev.record(stream)
            with torch.cuda.stream(comm):
                comm.wait_event(ev)
                dsp.record_stream(comm)
                allm = sdist.gather_maps(dsp, n_units, dst=0)
                if rank == 0:
                    fuse(fctx, allm)
                e2 = torch.cuda.Event()
                e2.record(comm)
                pending[b] = e2
            return
        if multi and not exchange:
            allm = stand_in
        elif multi:
            if a.dist_backend == "nccl":
                allm = sdist.gather_maps(dsp, n_units, dst=0)
            else:
                allm = sdist.gather_maps(dsp.cpu(), n_units, dst=0)
                allm = allm.to(dev) if allm is not None else None
        else:
            allm = dsp
        if rank == 0:
            fuse(ctx, allm)

    elapsed = timed(a, step, world, dev, ctxs)
    kernels = breakdown(a, step, world, ctxs, kernel_table(ctxs))
    value = n_units * W * H * D * a.steps / elapsed / 1e6
    # committed PMC bytes per pair: the 1080p D=128 frame's for the 1080p rigs
    traffic_wl = "1080p_d128" if (W, H, D) == (1920, 1080, 128) else a.workload
    fpl = batch_frames_per_launch(len(jobs), len(ctxs)) if a.batch else 1
    exchange = None
    if multi:
        def recompute(u):
            i, j = pairs[u]
            sx, sy, _ = synth.pair_step(grid[i], grid[j])
            Ld = torch.from_numpy(views_np[i]).to(dev)
            Rd = torch.from_numpy(views_np[j]).to(dev)
            m = torch.zeros((H, W), dtype=torch.int16, device=dev)
            ctx.disparity_sgm_d(Ld.data_ptr(), Rd.data_ptr(), W, H, W,
                                sva.default_params(D=D, dmin=0, dir=sx, dir_y=sy), m.data_ptr())
            return m
        exchange = exchange_report(a, step, world, rank, dev, ctxs, disps[(it[0] - 1) % len(disps)],
                                   n_units, elapsed / a.steps * 1e3, recompute)
        step()                           # the compute-only steps fused the stand-in
        torch.cuda.synchronize()
    out = None
    if rank == 0:
        # sanity: camera 0 sees the texture unwarped, so its fused depth must be
        # the stripe-plane depth pitch*f/(delta*ps) away from stripe edges
        z0 = depth[0].cpu().numpy()
        truth = ARRAY_PITCH * ARRAY_F / (delta * ARRAY_PS)
        edge = np.zeros(W, bool)
        cuts = np.flatnonzero(np.diff(delta[0]) != 0)
        for c in cuts:
            edge[max(0, c - 48): c + 48] = True
        inner = np.zeros((H, W), bool)
        inner[D:H - D, D:W - D] = True
        inner &= ~edge[None, :]
        exact = float(np.mean(np.abs(z0[inner] - truth[inner]) <= 1e-9 * truth[inner]))
        out = {
            "metric": f"Mdisparities/sec (W·H·D/s), camera array ({rig_label}), "
                      f"{W}x{H} D={D}, gather + fuse",
            "value": round(value, 1),
            "unit": "Mdisp/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(elapsed / a.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "u16",
            "data": "synthetic array views of one MT19937 texture warped by 12 "
                    f"stripe planes (per-grid-unit disparity 4..{dmax} px)",
            "config": {"workload": f"{a.workload}: {rig_label}, {n_units} pairs {W}x{H} D={D} "
                                   "Mode S along each pair's baseline step, RCCL gather, "
                                   "per-camera median fusion on rank 0",
                       "W": W, "H": H, "D": D, "P1": 10, "P2": 120, "pairs": n_units,
                       "parallelism": f"pairs sharded over {world} rank(s), gather to rank 0"
                                      + (" overlapped with the next step" if overlap else ""),
                       "streams_per_rank": len(ctxs), "batched": bool(a.batch)},
            "kernels_ms": {k: round(v["avg_ms"], 4) for k, v in kernels.items()},
            "fused_maps_per_s": round(len(groups) * a.steps / elapsed, 2),
            "ref_interior_depth_exact_frac": round(exact, 4),
            "roofline": roofline_of(kernels, W, H, D, traffic_wl, overlapped=len(ctxs) > 1,
                                    frames_per_launch=fpl),
            "aggregation_roofline": aggregation_roofline_of(kernels, W, H, D,
                                                            committed_traffic(traffic_wl),
                                                            overlapped=len(ctxs) > 1,
                                                            frames_per_launch=fpl),
            "cpu_baseline": None,
        }
        if exchange is not None:
            out["exchange"] = exchange
        if world == 1 and not a.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(W, H, D, a.cpu_threads)
        print(json.dumps(out), flush=True)
    for c in ctxs + ([fctx] if fctx is not None else []):
        c.close()
    if multi:
        dist.destroy_process_group()
    if exchange is not None and not exchange["ok"]:
        raise SystemExit("multi-rank exchange check failed: " + json.dumps(exchange))


def launch_mode(a, env):
    """How this process runs the N GPUs of a step:
      'torchrun' -- started by torch.distributed.run (WORLD_SIZE set): one rank
                    per GPU, torch.distributed (RCCL) gather;
      'engine'   -- --gpus N > 1 without WORLD_SIZE, or --engine multi: this
                    process drives devices 0..N-1 through the C-ABI engine
                    (sva_multi_*), the route a C++ host takes;
      'single'   -- one process, one GPU."""
    world = int(env.get("WORLD_SIZE", "1"))
    if "WORLD_SIZE" in env and world > 1:
        if world != a.gpus:
            raise SystemExit(f"--gpus {a.gpus} but WORLD_SIZE={world}")
        if a.engine == "multi":
            raise SystemExit("--engine multi is one process for all GPUs; do not start it "
                             "under torch.distributed.run")
        return "torchrun"
    if a.engine == "multi" or a.gpus > 1:
        if a.rehearse_rccl or a.rehearse_overlap or a.dist_backend != "nccl":
            raise SystemExit("--rehearse-* / --dist-backend apply to the torchrun route only")
        return "engine"
    return "single"


def run_engine(a, wl):
    """--gpus N from ONE process through the C-ABI multi-GPU engine: pair u
    lives on device u mod N (sva_multi_plan), each device runs its pairs on its
    own contexts/streams, and sva_batch_sgm_d gathers the u16 disparity maps
    (and f32 sub-pixel maps) to device 0 with RCCL grouped send/recv on a
    single-process communicator (ncclCommInitAll).  Array workloads then fuse
    per reference camera on device 0.  Checked once after the timed region:
    every gathered map vs a single-context recompute on device 0, and the
    steps re-timed without the gather (each device's pairs through its own
    engine contexts) for the exposed gather time."""
    import torch
    import stereovisionarray_amd as sva
    from stereovisionarray_amd import synth

    N = a.gpus
    ndev = torch.cuda.device_count()
    if N > ndev:
        raise SystemExit(f"--gpus {N}: only {ndev} HIP device(s) visible")
    W, H, D = wl["W"], wl["H"], wl["D"]
    devs = [torch.device("cuda", d) for d in range(N)]
    torch.cuda.set_device(0)
    groups = []
    if "rig" in wl:
        grid, pairs, rig_label = rig_of(wl["rig"])
        kmax = max(synth.pair_step(grid[i], grid[j])[2] for i, j in pairs)
        dmax = min((D - 1) // kmax, 100)
        delta = synth.array_delta(H, W, dmax)
        used = sorted({c for q in pairs for c in q})
        views_np = dict(zip(used, synth.array_views(H, W, [grid[c] for c in used], delta, seed=7)))
        units = []
        for i, j in pairs:
            sx, sy, _ = synth.pair_step(grid[i], grid[j])
            units.append((views_np[i], views_np[j],
                          sva.default_params(D=D, dmin=0, dir=sx, dir_y=sy)))
        off = 0
        for i in dict.fromkeys(q[0] for q in pairs):
            n = sum(1 for q in pairs if q[0] == i)
            bases = [synth.pair_step(grid[i], grid[j])[2] * ARRAY_PITCH
                     for (_, j) in pairs[off:off + n]]
            groups.append((off, n, bases))
            off += n
        subpixel = 0
    else:
        total = wl.get("total_pairs", N * a.pairs_per_rank)
        seed0 = 0 if "total_pairs" in wl else 1
        units = []
        for u in range(total):
            L, R, _ = synth.stereo_pair(H, W, D, 0, -1, seed=seed0 + u)
            units.append((L, R, sva.default_params(D=D, dmin=0, dir=-1, subpixel=1)))
        subpixel = 1
    n_units = len(units)
    per_dev = -(-n_units // N)
    S = a.streams if a.streams > 0 else (1 if per_dev == 1 else 2)
    m = sva.Multi(list(range(N)), streams=S, flags=sva.SVA_MULTI_GATHER_RCCL)
    ctxs = [m.context(d, s) for d in range(N) for s in range(S)]
    for c in ctxs:
        c.reserve(W, H, D)
    dl, dr = [], []
    for u, (L, R, _) in enumerate(units):
        dl.append(torch.from_numpy(L).to(devs[u % N]))
        dr.append(torch.from_numpy(R).to(devs[u % N]))
    jobs = [(dl[u].data_ptr(), dr[u].data_ptr(), units[u][2]) for u in range(n_units)]
    maps = torch.zeros((n_units, H, W), dtype=torch.int16, device=devs[0])
    sub = torch.zeros((n_units, H, W), dtype=torch.float32, device=devs[0]) if subpixel else None
    depth = torch.zeros((max(len(groups), 1), H, W), dtype=torch.float64, device=devs[0])
    nvalid = torch.zeros((max(len(groups), 1), H, W), dtype=torch.uint8, device=devs[0])
    fctx = m.context(0, 0)                 # device 0, stream 0: where the gathered maps land

    def step():
        m.batch_sgm_d(jobs, W, H, W, maps.data_ptr(), sub.data_ptr() if sub is not None else None)
        for g, (o, n, bases) in enumerate(groups):
            fctx.fuse_depth_d(maps[o].data_ptr(), n, W, H, bases, ARRAY_F, ARRAY_PS, 0xFFFF,
                              depth[g].data_ptr(), nvalid[g].data_ptr())

    # compute-only re-timing: every pair on its engine context, no gather
    local = [torch.zeros((H, W), dtype=torch.int16, device=devs[u % N]) for u in range(n_units)]
    plan_ctx = [m.context(u % N, (u // N) % S) for u in range(n_units)]

    lmaps = torch.zeros_like(maps) if groups else None

    def step_local():
        # the same work as step() without the gather: array workloads fuse a
        # stand-in of the gathered maps, so the difference is the gather alone
        for u in range(n_units):
            plan_ctx[u].disparity_sgm_d(dl[u].data_ptr(), dr[u].data_ptr(), W, H, W,
                                        units[u][2], local[u].data_ptr())
        for g, (o, n, bases) in enumerate(groups):
            fctx.fuse_depth_d(lmaps[o].data_ptr(), n, W, H, bases, ARRAY_F, ARRAY_PS, 0xFFFF,
                              depth[g].data_ptr(), nvalid[g].data_ptr())

    def run(fn, k, timing):
        for c in ctxs:
            c.set_timing(timing)
            c.reset_timing()
        m.synchronize()
        t0 = time.perf_counter()
        for _ in range(k):
            fn()
        m.synchronize()
        return time.perf_counter() - t0

    run(step, a.warmup, 0)
    elapsed = run(step, a.steps, 3)                     # SVA_TIMING_AGG in the timed region
    timed_k = kernel_table(ctxs)
    run(step, min(a.steps, 5), 1)                       # every kernel, after the timed region
    kernels = kernel_table(ctxs)
    for k in AGG_KERNELS:
        if k in timed_k:
            kernels[k] = timed_k[k]
    for c in ctxs:
        c.set_timing(0)
    compute_ms = run(step_local, max(1, min(a.steps, 10)), 0) / max(1, min(a.steps, 10)) * 1e3
    # every gathered map vs a single-context recompute on device 0
    check = sva.Context(0)
    cs = torch.cuda.Stream(devs[0])
    check.set_stream(cs.cuda_stream)
    mism = []
    got = maps.cpu()
    checked = min(n_units, max(32, N))      # bounded: 32 units, every owner device
    for u in range(checked):
        L, R, p = units[u]
        ref = torch.zeros((H, W), dtype=torch.int16, device=devs[0])
        Ld, Rd = torch.from_numpy(L).to(devs[0]), torch.from_numpy(R).to(devs[0])
        torch.cuda.synchronize(devs[0])
        check.disparity_sgm_d(Ld.data_ptr(), Rd.data_ptr(), W, H, W, p, ref.data_ptr())
        check.synchronize()
        if not torch.equal(ref.cpu(), got[u]):
            mism.append(u)
    check.close()
    ms_per_step = elapsed / a.steps * 1e3
    value = n_units * W * H * D * a.steps / elapsed / 1e6
    model, nproc, _ = host_cpu()
    exchange = {"backend": "rccl", "route": "C-ABI engine: sva_multi_create + sva_batch_sgm_d, "
                "single-process communicator (ncclCommInitAll), grouped ncclSend/ncclRecv to "
                "device 0", "rccl_ranks": N, "devices": N, "streams_per_device": S,
                "units_checked": checked, "units_equal_single_context": checked - len(mism),
                "remote_unit_recomputed": {"unit": 1 % n_units, "owner_device": (1 % n_units) % N,
                                           "equal": (1 % n_units) not in mism},
                "ok": not mism,
                "compute_only_ms_per_step": round(compute_ms, 4),
                "exposed_gather_ms_per_step": round(ms_per_step - compute_ms, 4),
                "map_bytes_per_unit": W * H * 2 + (W * H * 4 if subpixel else 0)}
    if "rig" in wl:
        metric = (f"Mdisparities/sec (W·H·D/s), camera array ({rig_label}), {W}x{H} D={D}, "
                  "gather + fuse")
        work = (f"{a.workload}: {rig_label}, {n_units} pairs {W}x{H} D={D} Mode S along each "
                "pair's baseline step, gather + per-camera median fusion on device 0")
    else:
        metric = ("Mdisparities/sec (W·H·D/s) at 1080p D=128" if a.workload == "1080p_d128"
                  else f"Mdisparities/sec (W·H·D/s) {a.workload}")
        work = (f"{W}x{H} D={D} Mode S SGM (census 9x7, Hamming, 8 paths, WTA+subpixel), "
                f"{n_units} pair(s) per step")
    out = {
        "metric": metric,
        "value": round(value, 1),
        "unit": "Mdisp/s",
        "n_gpus": N,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": round(ms_per_step, 4),
        "higher_is_better": True,
        "scaling": "strong" if ("total_pairs" in wl or "rig" in wl) else "weak",
        "vs_baseline": None,
        "dtype": "u16",
        "data": "synthetic (MT19937 u8 texture" + (", array views)" if "rig" in wl else
                                                    ", 16-stripe piecewise-constant disparity)"),
        "config": {"workload": work, "W": W, "H": H, "D": D, "P1": 10, "P2": 120,
                   "pairs": n_units,
                   "parallelism": f"pairs sharded over {N} device(s) of one process "
                                  "(sva_multi engine), RCCL gather to device 0",
                   "streams_per_rank": S},
        "kernels_ms": {k: round(v["avg_ms"], 4) for k, v in kernels.items()},
        "roofline": roofline_of(kernels, W, H, D, "1080p_d128" if "rig" in wl else a.workload,
                                overlapped=S > 1),
        "aggregation_roofline": aggregation_roofline_of(
            kernels, W, H, D, committed_traffic("1080p_d128" if "rig" in wl else a.workload),
            overlapped=S > 1),
        "cpu_baseline": None,
        "exchange": exchange,
        "host": f"{model}, nproc {nproc}",
    }
    if N == 1 and S == 1 and "rig" not in wl:
        out["frame_roofline"] = frame_roofline(W, H, D, ms_per_step / n_units)
    if N == 1 and not a.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(W, H, D, a.cpu_threads)
    if out["roofline"]:
        out["roofline"]["traffic_source"] = (f"committed profiles/pmc_{a.workload}.json "
                                             "(live PMC passes run on the single-GPU route)")
    print(json.dumps(out), flush=True)
    for c in ctxs:
        c.close()
    m.close()
    if mism:
        raise SystemExit(f"engine gather check failed for units {mism[:8]}")


def main():
    a = parse()
    mode = launch_mode(a, os.environ)
    import torch
    import torch.distributed as dist
    import stereovisionarray_amd as sva
    from stereovisionarray_amd import dist as sdist
    from stereovisionarray_amd import synth

    if not torch.cuda.is_available():
        raise SystemExit("bench.py needs a HIP device (no CPU fallback)")
    if a.mode_r_only:
        return mode_r_only(a.mode_r_size)
    if mode == "engine":
        return run_engine(a, WORKLOADS[a.workload])
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if not torch.cuda.is_available():
        raise SystemExit("bench.py needs a HIP device (no CPU fallback)")
    ndev = torch.cuda.device_count()
    local = local % ndev if a.dist_backend == "gloo" else local
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    rccl1 = world == 1 and a.rehearse_rccl
    if rccl1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29561")
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if a.dist_backend == "nccl":
            dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
        else:
            dist.init_process_group("gloo", rank=rank, world_size=world)

    wl = WORKLOADS[a.workload]
    W, H, D = wl["W"], wl["H"], wl["D"]
    if "rig" in wl:
        return run_array(a, wl, world, rank, local, dev)
    P = a.pairs_per_rank
    if "total_pairs" in wl:
        if world > 1 and wl["total_pairs"] % world:
            raise SystemExit("total_pairs must divide evenly over the ranks")
        P = wl["total_pairs"] // world
    params = sva.default_params(D=D, dmin=0, dir=-1, subpixel=1)
    # Pairs overlap on 2 streams by default.  Round 2 kept D=192 on one stream
    # (1080p x 256 pairs: 1 stream 251.5K, 2 streams 244.1K Mdisp/s,
    # profiles/r02_v9/streams_ab.txt); with the tile pipeline
    # two streams win there too: 304.9-307.7K -> 317.9K Mdisp/s
    # (profiles/r03_v8/streams_batch256.log.txt).
    n_streams = a.streams if a.streams > 0 else (1 if P == 1 else 2)
    if a.batch and a.streams <= 0:
        n_streams = 1                    # the batch runs on one context (--streams S: S batches)
    ctx = sva.Context(local)
    stream = torch.cuda.Stream(dev)     # non-default stream shared by kernels, copies, RCCL
    torch.cuda.set_stream(stream)
    ctx.set_stream(stream.cuda_stream)
    ctx.set_debug(sva.SVA_DEBUG_PLACEMENT_TRIALS, a.placement_trials)
    ctx.reserve(W, H, D)
    # --streams S: pair j of a step runs on context j % S (own stream and
    # workspaces); the step's maps are complete once `stream` has waited on all
    ctxs, cstreams = [ctx], [stream]
    for _ in range(1, n_streams):
        s_ = torch.cuda.Stream(dev)
        c_ = sva.Context(local)
        c_.set_stream(s_.cuda_stream)
        c_.set_debug(sva.SVA_DEBUG_PLACEMENT_TRIALS, a.placement_trials)
        c_.reserve(W, H, D)
        ctxs.append(c_)
        cstreams.append(s_)

    n_units = world * P   # unit u = pair u, owned by rank u mod world (sdist.shard)
    seed0 = 0 if "total_pairs" in wl else 1   # config 5 seeds 0-255
    lefts, rights = [], []
    for u in sdist.shard(n_units, rank, world):
        L, R, _ = synth.stereo_pair(H, W, D, 0, -1, seed=seed0 + u)
        lefts.append(torch.from_numpy(L).to(dev))
        rights.append(torch.from_numpy(R).to(dev))
    batch_jobs = [(lefts[j].data_ptr(), rights[j].data_ptr(), params) for j in range(P)]
    # Two map buffers: step i computes into buffer i%2 on the compute stream
    # while the gather of step i-1 (buffer (i-1)%2) runs on a comm stream.
    overlap = (world > 1 and a.dist_backend == "nccl" and not a.no_overlap) or \
        (world == 1 and (a.rehearse_overlap or rccl1))
    nbuf = 2 if overlap else 1
    disps = [torch.zeros((P, H, W), dtype=torch.int16, device=dev) for _ in range(nbuf)]
    sub = torch.zeros((P, H, W), dtype=torch.float32, device=dev)
    comm = torch.cuda.Stream(dev) if nbuf == 2 else None
    gathered = [None] * nbuf            # buffer -> event recorded after its gather
    it = [0]
    rehearsal = [torch.zeros((P, H, W), dtype=torch.int16, device=dev)] if world == 1 else None

    def gather(disp):
        if world > 1:
            sdist.gather_maps(disp, n_units, dst=0)
        elif rccl1:                      # real RCCL gather in a 1-rank group
            rehearsal[0].copy_(sdist.gather_maps(disp, n_units, dst=0))
        else:                            # --rehearse-overlap stand-in for the RCCL gather
            rehearsal[0].copy_(disp)

    def step(exchange=True):
        b = it[0] % nbuf
        it[0] += 1
        disp = disps[b]
        if gathered[b] is not None:      # the previous gather of this buffer is done
            stream.wait_event(gathered[b])
            gathered[b] = None
        if len(ctxs) > 1:                # other streams start after this buffer is free
            go = torch.cuda.Event()
            go.record(stream)
            for s_ in cstreams[1:]:
                s_.wait_event(go)
        if a.batch:
            for c_, (j0, j1) in zip(ctxs, batch_groups(P, len(ctxs))):
                if j1 > j0:
                    c_.disparity_sgm_batch_d(batch_jobs[j0:j1], W, H, W, disp[j0].data_ptr(),
                                             sub[j0].data_ptr())
        else:
            for j in range(P):
                ctxs[j % len(ctxs)].disparity_sgm_d(lefts[j].data_ptr(), rights[j].data_ptr(), W,
                                                    H, W, params, disp[j].data_ptr(),
                                                    sub[j].data_ptr())
        for s_ in cstreams[1:]:
            done_ = torch.cuda.Event()
            done_.record(s_)
            stream.wait_event(done_)
        if exchange and (world > 1 or comm is not None):   # the path's one exchange (RCCL)
            if a.dist_backend == "gloo" and world > 1:
                sdist.gather_maps(disp.cpu(), n_units, dst=0)
            elif comm is None:
                gather(disp)
            else:
                done = torch.cuda.Event()
                done.record(stream)
                with torch.cuda.stream(comm):
                    comm.wait_event(done)
                    disp.record_stream(comm)
                    gather(disp)
                    ev = torch.cuda.Event()
                    ev.record(comm)
                    gathered[b] = ev

    elapsed = timed(a, step, world, dev, ctxs)
    kernels = breakdown(a, step, world, ctxs, kernel_table(ctxs))
    # sanity: the result is a real disparity map (exact on the stripe interiors)
    d0 = disps[0][0].cpu().numpy().view(np.uint16)
    if rehearsal is not None and comm is not None:
        last = disps[(it[0] - 1) % nbuf]
        assert torch.equal(rehearsal[0], last), "overlapped gather copied the wrong buffer"
    assert d0.max() < D, "disparity out of range"
    exchange = None
    if world > 1 or rccl1:
        def recompute(u):
            L, R, _ = synth.stereo_pair(H, W, D, 0, -1, seed=seed0 + u)
            Ld, Rd = torch.from_numpy(L).to(dev), torch.from_numpy(R).to(dev)
            m = torch.zeros((H, W), dtype=torch.int16, device=dev)
            ctx.disparity_sgm_d(Ld.data_ptr(), Rd.data_ptr(), W, H, W, params, m.data_ptr())
            return m
        exchange = exchange_report(a, step, world, rank, dev, ctxs, disps[(it[0] - 1) % nbuf],
                                   n_units, elapsed / a.steps * 1e3, recompute)

    units = world * P * a.steps
    disparities = units * W * H * D
    value = disparities / elapsed / 1e6
    ms_per_step = elapsed / a.steps * 1e3
    fpl = batch_frames_per_launch(P, len(ctxs)) if a.batch else 1
    roofline = roofline_of(kernels, W, H, D, a.workload, overlapped=len(ctxs) > 1,
                           frames_per_launch=fpl)
    out = {
        "metric": "Mdisparities/sec (W·H·D/s) at 1080p D=128" if a.workload == "1080p_d128"
                  else f"Mdisparities/sec (W·H·D/s) {a.workload}",
        "value": round(value, 1),
        "unit": "Mdisp/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": round(ms_per_step, 4),
        "higher_is_better": True,
        "scaling": "strong" if "total_pairs" in wl else "weak",
        "vs_baseline": None,
        "dtype": "u16",
        "data": "synthetic (MT19937 u8 texture, 16-stripe piecewise-constant disparity)",
        "config": {"workload": f"{W}x{H} D={D} Mode S SGM (census 9x7, Hamming, 8 paths, "
                               f"WTA+subpixel), {P} pair(s)/rank",
                   "W": W, "H": H, "D": D, "P1": 10, "P2": 120,
                   "parallelism": f"pairs sharded over {world} rank(s), RCCL gather to rank 0"
                                  + (" overlapped with the next step" if nbuf == 2 else ""),
                   "streams_per_rank": len(ctxs), "batched": bool(a.batch)},
        "kernels_ms": {k: round(v["avg_ms"], 4) for k, v in kernels.items()},
        "roofline": roofline,
        "aggregation_roofline": aggregation_roofline_of(kernels, W, H, D, committed_traffic(a.workload),
                                                        overlapped=len(ctxs) > 1,
                                                        frames_per_launch=fpl),
        "cpu_baseline": None,
    }
    if len(ctxs) == 1:
        out["frame_roofline"] = frame_roofline(W, H, D, ms_per_step / P)
    pl = placement_report(ctxs)
    if pl:
        out["placement"] = pl
    if exchange is not None:
        out["exchange"] = exchange
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(W, H, D, a.cpu_threads)
        _, _, budget = host_cpu()
        if budget > 1:   # the oracle at all (allowed) cores as well
            out["cpu_baseline_all_cores"] = cpu_baseline(W, H, D, budget)
        # the reference's own CPU path (Mode R) timed beside its GPU port
        out["mode_r"] = mode_r_beside(ctx, W, H)
        under_prof = any(k.startswith("ROCPROF") for k in os.environ) or \
            os.environ.get("SVA_BENCH_PMC_CHILD")
        if a.pmc == "live" and not under_prof:
            try:
                out["mode_r"]["roofline"] = mode_r_roofline(out["mode_r"])
            except Exception as e:                  # keep the bench line; say why
                out["mode_r"]["roofline"] = {"error": str(e)[:200]}
        if a.workload == "1080p_d128":
            out["frame_overlap"] = frame_overlap_beside(W, H, D)
            out["steady_state"] = steady_state_beside(step, ctxs)
    if rank == 0:
        attach_traffic(a, out, world)
        attach_engine(a, out, kernels, world)
        print(json.dumps(out), flush=True)
    for c in ctxs:
        c.close()
    if world > 1 or rccl1:
        dist.destroy_process_group()
    if exchange is not None and not exchange["ok"]:
        raise SystemExit("multi-rank exchange check failed: " + json.dumps(exchange))


if __name__ == "__main__":
    main()
