"""bench.py host logic that needs no GPU: where roofline.traffic comes from.

The live source runs rocprofv3 PMC passes as child processes; it must not run
at N > 1, inside a PMC child, or under a profiler, and a failed pass must
leave the committed figure with the reason in traffic_source.
"""
import argparse
import importlib.util
import os

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def bench():
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def line(bench):
    kernels = {"sgm_paths": {"avg_ms": 0.62}}
    return {"roofline": bench.roofline_of(kernels, 1920, 1080, 128, "1080p_d128")}


def args(pmc):
    return argparse.Namespace(pmc=pmc, workload="1080p_d128", path_kernel="auto",
                              pairs_per_rank=1)


def test_committed_source(bench):
    out = line(bench)
    bench.attach_traffic(args("committed"), out, 1)
    assert out["roofline"]["traffic_source"].startswith("committed")
    assert out["roofline"]["traffic"] == bench.load_traffic("1080p_d128", "sgm_paths")


def test_live_skipped_at_n_gt_1_and_under_profiler(bench, monkeypatch):
    called = []
    monkeypatch.setattr(bench, "live_traffic", lambda a: called.append(1) or {})
    out = line(bench)
    bench.attach_traffic(args("live"), out, 2)
    monkeypatch.setenv("ROCPROF_KERNEL_TRACE", "1")
    bench.attach_traffic(args("live"), out, 1)
    monkeypatch.delenv("ROCPROF_KERNEL_TRACE")
    monkeypatch.setenv("SVA_BENCH_PMC_CHILD", "1")
    bench.attach_traffic(args("live"), out, 1)
    assert not called
    assert out["roofline"]["traffic_source"].startswith("committed")


def test_live_failure_falls_back(bench, monkeypatch):
    def boom(a):
        raise RuntimeError("rocprofv3 --pmc FETCH_SIZE exited 137")
    monkeypatch.delenv("SVA_BENCH_PMC_CHILD", raising=False)
    for k in [k for k in os.environ if k.startswith("ROCPROF")]:
        monkeypatch.delenv(k)
    monkeypatch.setattr(bench, "live_traffic", boom)
    out = line(bench)
    bench.attach_traffic(args("live"), out, 1)
    rf = out["roofline"]
    assert "live PMC pass failed" in rf["traffic_source"] and "137" in rf["traffic_source"]
    assert rf["traffic"] == bench.load_traffic("1080p_d128", "sgm_paths")


def test_live_success_uses_kernel_bytes(bench, monkeypatch):
    monkeypatch.delenv("SVA_BENCH_PMC_CHILD", raising=False)
    for k in [k for k in os.environ if k.startswith("ROCPROF")]:
        monkeypatch.delenv(k)
    kern = {"sgm_paths": {"hbm_read_bytes": 2, "hbm_write_bytes": 1, "hbm_bytes_per_launch": 3}}
    monkeypatch.setattr(bench, "live_traffic", lambda a: kern)
    out = line(bench)
    bench.attach_traffic(args("live"), out, 1)
    rf = out["roofline"]
    assert rf["traffic"] == 3 and rf["traffic_source"].startswith("live")
    assert rf["traffic_per_kernel"] == kern


def test_aggregation_roofline(bench, monkeypatch):
    """sgm_paths + wta_hv graded together over SURVEY §8d's
    aggregation (10 B/disp) + WTA (2 B/disp + 2 B/px) bytes; live PMC bytes
    of both kernels fill its traffic."""
    W, H, D = 1920, 1080, 128
    kernels = {"sgm_paths": {"avg_ms": 0.5}, "wta_hv": {"avg_ms": 0.25}}
    ag = bench.aggregation_roofline_of(kernels, W, H, D)
    alg = 12.0 * W * H * D + 2.0 * W * H
    assert ag["alg_bytes_per_launch"] == alg and ag["sum_ms"] == 0.75
    assert abs(ag["achieved"] - alg / 0.75e-3 / 1e9) < 0.1
    assert abs(ag["frac"] - ag["achieved"] / 8000.0) < 1e-4
    assert bench.aggregation_roofline_of({"sgm_paths": {"avg_ms": 0.5}}, W, H, D) is None
    monkeypatch.delenv("SVA_BENCH_PMC_CHILD", raising=False)
    for k in [k for k in os.environ if k.startswith("ROCPROF")]:
        monkeypatch.delenv(k)
    kern = {"sgm_paths": {"hbm_bytes_per_launch": 3}, "wta_hv": {"hbm_bytes_per_launch": 4}}
    monkeypatch.setattr(bench, "live_traffic", lambda a: kern)
    out = line(bench)
    out["aggregation_roofline"] = ag
    bench.attach_traffic(args("live"), out, 1)
    assert out["aggregation_roofline"]["traffic"] == 7


def fake_mode_r_pass(seen, ran=None):
    """A stand-in PMC pass that records the child's arguments and stamps the
    frame size the child would have run (or `ran`)."""
    import json

    def fake(counter, args, outdir, child=None, env=None):
        seen["counter"], seen["child"] = counter, child
        i = child.index("--mode-r-size")
        W, H = (int(v) for v in (ran or child[i + 1]).split("x"))
        with open(env["SVA_MODE_R_STAMP"], "w") as f:
            json.dump({"W": W, "H": H, "k": 20}, f)
        return {"ref_match": {"SQ_INSTS_VALU": 300e6, "GRBM_GUI_ACTIVE": 2.0e6}}
    return fake


def test_mode_r_valu_roofline(bench, monkeypatch):
    """the VALU peak is the SIMD-32 issue rate,
    one wave64 instruction per 2 cycles per SIMD (MI355X_MICROARCH.md :53-54):
    SQ_INSTS_VALU / (kernel time x 1,024 x 2.4 GHz / 2) -- not the 4 cycles
    one wave alone sustains, which rounds 3-5 used."""
    seen = {}
    monkeypatch.setattr(bench, "_pmc_pass", fake_mode_r_pass(seen))
    rf = bench.mode_r_roofline({"ref_match_kernel_ms": 0.8, "W": 1920, "H": 1080})
    assert seen["counter"] == bench.SQ_VALU_COUNTERS
    assert "SQ_WAIT_INST_ANY" in seen["counter"] and "SQ_ACTIVE_INST_VALU" in seen["counter"]
    assert seen["child"] == ["--mode-r-only", "--mode-r-size", "1920x1080"]
    assert bench.VALU_ISSUE_CYCLES == 2.0 and abs(bench.VALU_PEAK_PER_S - 1.2288e12) < 1e3
    assert abs(rf["frac"] - 300e6 * 2 / (1024 * 2.4e9 * 0.8e-3)) < 1e-4
    assert rf["bound"] == "valu" and rf["sq_insts_valu"] == 300000000
    assert rf["frame"] == "1920x1080"
    with pytest.raises(RuntimeError):
        bench.mode_r_roofline({"ref_match_kernel_ms": None, "W": 1920, "H": 1080})


def test_mode_r_child_runs_the_timed_frame(bench, monkeypatch):
    """the PMC child gets the timed frame's W and H (the
    4K line once divided 1080p instruction counts by the 4K kernel time), and
    a child that ran another size is refused."""
    seen = {}
    monkeypatch.setattr(bench, "_pmc_pass", fake_mode_r_pass(seen))
    rf = bench.mode_r_roofline({"ref_match_kernel_ms": 4.7, "W": 3840, "H": 2160})
    assert seen["child"] == ["--mode-r-only", "--mode-r-size", "3840x2160"]
    assert rf["frame"] == "3840x2160"
    monkeypatch.setattr(bench, "_pmc_pass", fake_mode_r_pass(seen, ran="1920x1080"))
    with pytest.raises(RuntimeError, match="ran 1920x1080, timed 3840x2160"):
        bench.mode_r_roofline({"ref_match_kernel_ms": 4.7, "W": 3840, "H": 2160})
    assert bench.parse_size("3840x2160") == (3840, 2160)
    with pytest.raises(ValueError):
        bench.parse_size("0x10")


def test_batched_launch_gets_no_single_frame_traffic(bench):
    """a batched launch covers frames_per_launch frames, so the
    committed single-frame PMC bytes must not be set against its algorithmic
    bytes (that once reported traffic below the algorithmic minimum)."""
    k = {"sgm_paths": {"avg_ms": 4.0}, "wta_hv": {"avg_ms": 2.0}}
    rf = bench.roofline_of(k, 1920, 1080, 128, "1080p_d128", frames_per_launch=8)
    assert rf["traffic"] is None and rf["frames_per_launch"] == 8
    assert rf["alg_bytes_per_launch"] == 10.0 * 1920 * 1080 * 128 * 8
    committed = {"sgm_paths": {"hbm_bytes_per_launch": 3}, "wta_hv": {"hbm_bytes_per_launch": 4}}
    ag = bench.aggregation_roofline_of(k, 1920, 1080, 128, committed, frames_per_launch=8)
    assert ag["traffic"] is None
    ag1 = bench.aggregation_roofline_of(k, 1920, 1080, 128, committed)
    assert ag1["traffic"] == 7


def mode_args(**kw):
    d = dict(gpus=1, engine="auto", rehearse_rccl=False, rehearse_overlap=False,
             dist_backend="nccl")
    d.update(kw)
    return argparse.Namespace(**d)


def test_launch_mode(bench):
    """VERDICT r02 "next" #2: --gpus N > 1 without torch.distributed.run runs
    the single-process C-ABI engine; torchrun keeps its route."""
    assert bench.launch_mode(mode_args(), {}) == "single"
    assert bench.launch_mode(mode_args(gpus=2), {}) == "engine"
    assert bench.launch_mode(mode_args(gpus=8), {"WORLD_SIZE": "1"}) == "engine"
    assert bench.launch_mode(mode_args(engine="multi"), {}) == "engine"
    assert bench.launch_mode(mode_args(gpus=4), {"WORLD_SIZE": "4"}) == "torchrun"
    with pytest.raises(SystemExit):
        bench.launch_mode(mode_args(gpus=2), {"WORLD_SIZE": "4"})
    with pytest.raises(SystemExit):
        bench.launch_mode(mode_args(gpus=2, engine="multi"), {"WORLD_SIZE": "2"})
    with pytest.raises(SystemExit):
        bench.launch_mode(mode_args(gpus=2, dist_backend="gloo"), {})


def test_gpus_2_without_world_size_gets_past_argument_handling():
    """`python bench.py --gpus 2` with no WORLD_SIZE no longer demands
    torch.distributed.run: here (no HIP device) it stops at the device check,
    after argument handling and route selection."""
    import subprocess
    import sys
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["HIP_VISIBLE_DEVICES"] = ""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2",
                        "--steps", "1", "--warmup", "0"], capture_output=True, text=True,
                       env=env, timeout=300)
    assert r.returncode != 0
    assert "torch.distributed.run" not in r.stderr
    assert "needs a HIP device" in r.stderr or "HIP device(s) visible" in r.stderr


def test_batch_groups_and_frames_per_launch(bench):
    """--batch --streams S: S contiguous batch calls; the roofline's frames per
    aggregation launch follow sva_disparity_sgm_batch_d's chunks of 8 and
    sub-batches of 4 (sva_tuning.h kBatchMaxPairs, kBatchSubFrames)."""
    assert bench.batch_groups(8, 1) == [(0, 8)]
    assert bench.batch_groups(8, 3) == [(0, 2), (2, 5), (5, 8)]
    assert bench.batch_groups(2, 3) == [(0, 1), (1, 2), (2, 2)]
    cover = [j for j0, j1 in bench.batch_groups(11, 4) for j in range(j0, j1)]
    assert cover == list(range(11))
    assert bench.batch_frames_per_launch(8) == 4.0           # 8 -> 4 + 4
    assert bench.batch_frames_per_launch(256) == 4.0
    assert bench.batch_frames_per_launch(11) == 11 / 3       # 8 -> 4 + 4, 3
    assert bench.batch_frames_per_launch(8, 3) == 8 / 3      # 2, 3, 3 frames: one launch each


def test_valu_roofline_shares_and_clock(bench):
    """valu_roofline: issue fraction at the peak clock, at the kernel's own
    active cycles (GRBM_GUI_ACTIVE summed over 8 XCDs), and the SQ_WAVE_CYCLES
    shares spent issuing VALU and waiting."""
    c = {"SQ_INSTS_VALU": 120e6, "SQ_ACTIVE_INST_VALU": 120e6, "SQ_WAIT_INST_ANY": 90e6,
         "SQ_WAIT_ANY": 150e6, "SQ_WAVE_CYCLES": 600e6, "GRBM_GUI_ACTIVE": 8 * 500e3,
         "_dur_ns": 250e3}
    rf = bench.valu_roofline("wta_hv", c, 0.25, "wta_hv_kernel")
    assert abs(rf["frac"] - 120e6 / (0.25e-3 * 1.2288e12)) < 1e-4
    assert abs(rf["frac_at_clock"] - 2 * 120e6 / (1024 * 500e3)) < 1e-4
    assert rf["clock_ghz"] == 2.0
    assert rf["active_valu_share"] == 0.2 and rf["wait_inst_any_share"] == 0.15
    assert rf["wait_any_share"] == 0.25
    with pytest.raises(RuntimeError):
        bench.valu_roofline("wta_hv", {}, 0.25, "wta_hv_kernel")


def test_ea_figures(bench):
    """roofline.engine: engine clock from GRBM_GUI_ACTIVE
    over the pass's kernel duration, EA read bytes at 128 B per request
    (gfx950), write bytes from the 64-B and 32-B request counts."""
    c = {"TCC_EA0_RDREQ_sum": 1e6, "TCC_EA0_WRREQ_sum": 3e6, "TCC_EA0_WRREQ_64B_sum": 2e6,
         "GRBM_GUI_ACTIVE": 8 * 2.1e6, "_dur_ns": 1e6}
    e = bench.ea_figures(c, 1.0)
    assert e["clock_ghz"] == 2.1
    assert e["ea_read_bytes"] == 128e6 and e["ea_write_bytes"] == 2e6 * 64 + 1e6 * 32
    assert e["ea_bytes"] == e["ea_read_bytes"] + e["ea_write_bytes"]
    assert e["ea_gbs_at_event_time"] == round(e["ea_bytes"] / 1e-3 / 1e9, 1)


def test_engine_counters_skipped_off_the_live_route(bench, monkeypatch):
    called = []
    monkeypatch.setattr(bench, "engine_counters", lambda a: called.append(1) or ({}, {}))
    out = line(bench)
    a = args("committed")
    bench.attach_engine(a, out, {}, 1)
    bench.attach_engine(args("live"), out, {}, 2)
    assert not called and "valu_roofline" not in out


def test_placement_report(bench):
    """The bench line's `placement` field: the kept and slowest trial times of
    sva_reserve's placement check, per context; absent when no context ran it."""
    import stereovisionarray_amd as sva

    class FakeCtx:
        def __init__(self, kept, worst):
            self.v = {sva.SVA_DEBUG_PLACEMENT_NS: kept, sva.SVA_DEBUG_PLACEMENT_WORST_NS: worst}

        def get_debug(self, key):
            return self.v[key]

    assert bench.placement_report([FakeCtx(0, 0)]) is None
    r = bench.placement_report([FakeCtx(4_193_100, 4_838_900), FakeCtx(0, 0)])
    assert r["contexts"] == [{"kept_ms": 4.1931, "worst_ms": 4.8389}]
    assert "fastest set is kept" in r["note"]
