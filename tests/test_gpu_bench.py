"""The bench line the driver parses (README "bench.py contract"): one JSON line on stdout with
the metric of BASELINE.json, whole-job throughput, the roofline object of the dominant kernel
and the whole-step object.  A short run (3 timed outer iterations, no CPU baseline, no side
measurements) on the GPU."""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

pytestmark = pytest.mark.gpu


def test_bench_json_line():
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    out = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--steps", "3", "--warmup", "1",
                          "--no-cpu-baseline", "--no-gn", "--no-stencil"], cwd=REPO, env=env,
                         capture_output=True, text=True, timeout=180)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout[-2000:]
    d = json.loads(lines[0])
    base = json.load(open(os.path.join(REPO, "BASELINE.json")))
    assert base["metric"].startswith(d["metric"])   # the iters/s half of the metric (EPE needs Middlebury)
    for key in ("value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
                "vs_baseline", "dtype", "data", "config"):
        assert key in d, key
    assert d["unit"] == "iters/s" and d["n_gpus"] == 1 and d["steps"] == 3 and d["warmup"] == 1
    assert d["higher_is_better"] is True and d["dtype"] == "f64" and d["vs_baseline"] is None
    assert d["config"]["grid"] == [640, 480, 32] and "workload" in d["config"]
    assert d["value"] > 0 and abs(d["value"] * d["ms_per_step"] / 1e3 - 1.0) < 0.01
    assert 150 <= d["cg_iters_per_step"] <= 210   # scipy-rule CG steps per outer iteration at the bench grid
    r = d["roofline"]
    assert r["bound"] == "hbm" and r["unit"] == "GB/s" and r["peak"] == 8000.0 and r["kernel"] == "prox"
    assert abs(r["frac"] - r["achieved"] / r["peak"]) < 1e-3
    assert r["alg_bytes_per_launch"] == 64 * 640 * 480 * 32   # SURVEY §8(d) bytes per voxel x voxels
    st = r["step"]
    assert st["alg_bytes_per_voxel"] == sum(st["items"].values()) == 188
    assert "cpu_baseline" not in d or d["cpu_baseline"] is None
