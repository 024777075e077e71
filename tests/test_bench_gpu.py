"""bench.py's N>1 exchange on one GPU: a 1-rank RCCL process group runs the
real overlapped gather (sdist.gather_maps on the comm stream, two map buffers)
and bench.py asserts that the last gathered buffer is the last computed one.
Also checks the driver's JSON contract fields on that line.
"""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_rehearse_rccl_gather():
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT="29573")
    r = subprocess.run([sys.executable, "bench.py", "--steps", "4", "--warmup", "2",
                        "--no-cpu-baseline", "--rehearse-rccl"],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    d = json.loads(lines[0])
    for key in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
                "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config",
                "roofline", "cpu_baseline"):
        assert key in d, key
    assert d["n_gpus"] == 1 and d["steps"] == 4 and d["value"] > 0
    assert "overlapped" in d["config"]["parallelism"]
    rf = d["roofline"]
    assert rf["bound"] == "hbm" and rf["unit"] == "GB/s" and 0 < rf["frac"] < 1
    assert abs(rf["frac"] - rf["achieved"] / rf["peak"]) < 1e-3
    assert rf["traffic"] is None or rf["traffic"] > 0
    fr = d["frame_roofline"]
    assert 0 < fr["frac"] < rf["frac"] and abs(fr["ms_per_frame"] - d["ms_per_step"]) < 1e-3
    # the exchange check (owner checksums, a recomputed unit, timing)
    ex = d["exchange"]
    assert ex["backend"] == "rccl" and ex["rccl_world"] == 1 and ex["ok"]
    assert ex["checksums_ok"] and ex["remote_unit_recomputed"]["equal"]
    assert ex["gather_ms"] > 0 and ex["map_bytes_per_unit"] == 1920 * 1080 * 2


def test_bench_array_rehearse_rccl():
    """The camera-array workload's overlapped gather + fusion on the comm
    stream, through a 1-rank RCCL group (bench.py run_array)."""
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT="29575")
    r = subprocess.run([sys.executable, "bench.py", "--workload", "center8", "--steps", "2",
                        "--warmup", "1", "--no-cpu-baseline", "--rehearse-rccl"],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    d = json.loads(lines[0])
    assert "overlapped" in d["config"]["parallelism"] and d["config"]["pairs"] == 8
    assert d["exchange"]["ok"] and d["exchange"]["units_checked"] == 8
    # the fused reference depth is the synthetic plane depth on the interior
    assert d["ref_interior_depth_exact_frac"] > 0.98
