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


def test_bench_two_ranks_batch_mode_one_gpu(tmp_path):
    """bench.py --gpus 2 as the driver launches it (torch.distributed.run, one process per rank,
    the file rendezvous), both ranks on this one GPU (FOTO_BENCH_DEVICES=0,0): the default batch
    mode -- one 640x480x32 solve per rank, value = both solves' outer iterations per second on the
    slowest rank's clock, "scaling": "weak".  (The time-sharded side run needs two GPUs for RCCL:
    --no-strong here; its call sequences are checked by tests/test_gpu_rccl_mock.py.)"""
    # (the two ranks started here the way torch.distributed.run starts them -- children of one
    # process, RANK / WORLD_SIZE / LOCAL_RANK / MASTER_PORT set -- without its torch import)
    procs = []
    for g in range(2):
        env = dict(os.environ, FOTO_BENCH_DEVICES="0,0", WORLD_SIZE="2", RANK=str(g), LOCAL_RANK=str(g),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT="29617")
        cmd = [sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--steps", "3", "--warmup", "1",
               "--no-cpu-baseline", "--no-gn", "--no-stencil", "--no-strong"]
        procs.append(subprocess.Popen(cmd, cwd=REPO, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                                      text=True))
    outs = [p.communicate(timeout=240) for p in procs]
    for p, (o, e) in zip(procs, outs):
        assert p.returncode == 0, e[-3000:]
    lines = [ln for o, _ in outs for ln in o.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, [o[-1000:] for o, _ in outs]   # rank 0 only
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["scaling"] == "weak" and d["steps"] == 3
    assert "data-parallel x2" in d["config"]["parallelism"]
    # two problems advanced in the timed region: value = 2 K / elapsed
    assert abs(d["value"] * d["ms_per_step"] / 1e3 - 2.0) < 0.02
    assert 150 <= d["cg_iters_per_step"] <= 210
    assert "strong" not in d


def test_bench_strong_side_run_failure_is_reported(tmp_path):
    """The batch mode's time-sharded side run runs in a child process per rank: here, with both
    ranks on one GPU, RCCL refuses the communicator (one device for two ranks), and the children
    fail -- the headline line must still come out of rank 0 with the failure reported in
    "strong", and both ranks must exit 0 (a crash or hang inside RCCL on the driver's 8-GPU node
    cannot cost the data-parallel measurement)."""
    procs = []
    for g in range(2):
        env = dict(os.environ, FOTO_BENCH_DEVICES="0,0", WORLD_SIZE="2", RANK=str(g), LOCAL_RANK=str(g),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT="29619", FOTO_BENCH_STRONG_TIMEOUT="90")
        cmd = [sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--steps", "3", "--warmup", "1",
               "--no-cpu-baseline", "--no-gn", "--no-stencil"]
        procs.append(subprocess.Popen(cmd, cwd=REPO, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                                      text=True))
    outs = [p.communicate(timeout=300) for p in procs]
    for p, (o, e) in zip(procs, outs):
        assert p.returncode == 0, e[-3000:]
    lines = [ln for o, _ in outs for ln in o.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, [o[-1000:] for o, _ in outs]
    d = json.loads(lines[0])
    print("strong:", d.get("strong"))
    assert d["scaling"] == "weak" and d["n_gpus"] == 2
    assert "strong" in d and ("error" in d["strong"] or "value" in d["strong"])
