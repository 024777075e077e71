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
