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
sys.path.insert(0, REPO)
import bench  # noqa: E402  (the model table the line carries)

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


def _ranks(n, port, extra_env=None, args=()):
    """bench.py --gpus n as the driver launches it (torch.distributed.run: one process per rank,
    RANK / WORLD_SIZE / LOCAL_RANK / MASTER_PORT set, children of one process) without its torch
    import, every rank on this one GPU (FOTO_BENCH_DEVICES=0) and the time-sharded runs over the
    in-process RCCL transport (FOTO_BENCH_MOCK_RCCL=1: rank 0's child runs the n ranks as threads
    over libfoto_mockrccl.so -- real RCCL refuses two ranks on one device).  Returns rank 0's line."""
    procs = []
    for g in range(n):
        env = dict(os.environ, FOTO_BENCH_DEVICES="0", FOTO_BENCH_MOCK_RCCL="1", WORLD_SIZE=str(n), RANK=str(g),
                   LOCAL_RANK=str(g), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                   FOTO_BENCH_SHARD_TIMEOUT="150", **(extra_env or {}))
        cmd = [sys.executable, os.path.join(REPO, "bench.py"), "--gpus", str(n), "--steps", "3", "--warmup", "1",
               "--no-cpu-baseline", "--no-gn", "--no-stencil", *args]
        procs.append(subprocess.Popen(cmd, cwd=REPO, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                                      text=True))
    outs = [p.communicate(timeout=280) for p in procs]
    for p, (o, e) in zip(procs, outs):
        assert p.returncode == 0, e[-3000:]
    lines = [ln for o, _ in outs for ln in o.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, [o[-1000:] for o, _ in outs]   # rank 0 only
    d = json.loads(lines[0])
    print({k: d.get(k) for k in ("value", "ms_per_step", "rccl_ranks", "error")},
          {k: (d[k] or {}).get("value") if isinstance(d.get(k), dict) else None for k in ("batch", "c4")})
    return d


def _check_strong(d, n):
    assert d["n_gpus"] == n and d["scaling"] == "strong" and d["steps"] == 3
    assert d["rccl_ranks"] == n   # ncclCommCount of every rank's communicator
    assert "time-slab x%d" % n in d["config"]["parallelism"]
    assert d["value"] > 0 and abs(d["value"] * d["ms_per_step"] / 1e3 - 1.0) < 0.01
    assert 150 <= d["cg_iters_per_step"] <= 210
    sh = d["sharded"]
    assert sum(sh["planes_per_rank"]) == 32 and sh["rccl_ranks_per_rank"] == [n] * n
    st = d["roofline"]["step"]
    assert st["items"]["a2a_staging"] == round(32 * (n - 1) / n, 4)
    assert st["alg_bytes_per_rank"] == st["alg_bytes_per_voxel"] * st["voxels_per_rank"]
    assert d["roofline"]["kernel"] == "prox" and d["roofline"]["frac"] > 0
    assert sh["model_it_s"] == bench.MODEL_IT_S[(640, 480, 32)].get(n)
    b = d["batch"]   # the data-parallel number: a labelled side object, never the headline
    assert b["scaling"] == "weak" and b["n_gpus"] == n and abs(b["value"] * b["ms_per_step"] / 1e3 - n) < 0.02 * n


def test_bench_n2_line_time_sharded_headline():
    """N = 2: value = the one 640x480x32 solve time-sharded over the two ranks (RCCL branches),
    "scaling": "strong", rccl_ranks 2; config 4 (1024x1024x64) sharded the same way in "c4";
    the independent-solve throughput only in "batch"."""
    d = _ranks(2, 29617, args=("--c4-steps", "1", "--c4-warmup", "1"))
    _check_strong(d, 2)
    c4 = d["c4"]
    assert c4["value"] > 0 and c4["grid"] == [1024, 1024, 64] and c4["rccl_ranks"] == 2, c4
    assert c4["planes_per_rank"] == [32, 32]


def test_bench_n8_line_time_sharded_headline():
    """N = 8 (the driver's scaling node): four planes per rank, rccl_ranks 8."""
    d = _ranks(8, 29618, args=("--no-c4",))
    _check_strong(d, 8)
    assert d["sharded"]["planes_per_rank"] == [4] * 8
    assert d["c4"] is None


def test_bench_n4_line_with_c4():
    """N = 4, as the driver's scaling run launches it: eight planes per rank on the metric grid,
    and config 4 sharded over the same four ranks (16 planes each) in "c4"."""
    d = _ranks(4, 29620, args=("--c4-steps", "1", "--c4-warmup", "1"))
    _check_strong(d, 4)
    assert d["sharded"]["planes_per_rank"] == [8] * 4
    c4 = d["c4"]
    assert c4["value"] > 0 and c4["rccl_ranks"] == 4 and c4["planes_per_rank"] == [16] * 4, c4


def test_bench_rccl_failure_gives_null_value():
    """An RCCL failure (the mock refuses the communicator, as real RCCL refuses two ranks on one
    GPU): the headline value is null with the error in the line -- the batch number, which
    needs no collective, is still measured but stays in "batch" -- and every rank exits 0."""
    d = _ranks(2, 29619, extra_env={"FOTO_MOCK_FAIL_INIT": "1"}, args=("--no-c4",))
    assert d["value"] is None and d["ms_per_step"] is None and d["rccl_ranks"] is None
    assert "ncclCommInitRank" in d["error"] or "refused" in d["error"], d["error"]
    assert d["scaling"] == "strong" and d["batch"]["value"] > 0
