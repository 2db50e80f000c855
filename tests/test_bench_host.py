"""bench.py's multi-GPU host logic on the CPU (no GPU here): the file rendezvous's gather and
abort, the thread rendezvous of the mock-RCCL path, the per-rank step model of the time-sharded
solve, and the failure path of the N-GPU line -- with no device every rank's sharded child fails,
and rank 0 must still print the line with value null and the reason, never another number."""
import importlib.util
import json
import os
import subprocess
import sys
import threading

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def bench():
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(REPO, "bench.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def test_sharded_step_model(bench):
    m1 = bench.sharded_step_model((640, 480, 32), 1, 32)
    assert m1["items"]["a2a_staging"] == 0 and m1["alg_bytes_per_voxel"] == 188
    assert m1["xgmi_bytes_per_rank"] == 0
    m8 = bench.sharded_step_model((640, 480, 32), 8, 4)
    assert m8["voxels_per_rank"] == 4 * 640 * 480
    assert m8["alg_bytes_per_voxel"] == pytest.approx(188 + 28)
    assert m8["xgmi_bytes_per_rank"] == pytest.approx(14 * 4 * 640 * 480)


def test_thread_sync_gather_and_max(bench):
    W = 4
    ts = bench.ThreadSync(W)
    out = [None] * W

    def run(g):
        v = ts.view(g)
        v.barrier()
        out[g] = (v.gather({"r": g}), v.max(float(g) * 1.5))

    th = [threading.Thread(target=run, args=(g,)) for g in range(W)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=30)
    for g in range(W):
        assert out[g][0] == [{"r": k} for k in range(W)] and out[g][1] == 4.5


def test_file_rendezvous_gather_and_abort(bench, tmp_path):
    W = 3
    rs = [bench.FileRendezvous(g, W, timeout=20, dir=str(tmp_path / "rdv")) for g in range(W)]
    res = [None] * W
    th = [threading.Thread(target=lambda g=g: res.__setitem__(g, rs[g].gather(g * 10 or None))) for g in range(W)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=30)
    assert res == [[None, 10, 20]] * W
    rs[1].abort("boom")
    with pytest.raises(RuntimeError, match="rank 1: boom"):
        rs[0].barrier()


def test_n2_line_without_a_device_reports_null_value(tmp_path):
    """Two ranks launched the way torch.distributed.run launches them, on a host with no GPU: both
    sharded children fail (rank 0's before the RCCL id exists, rank 1's on the abort it leaves),
    and rank 0's line carries value null, the strong-scaling fields and both ranks' errors."""
    procs = []
    for g in range(2):
        env = dict(os.environ, WORLD_SIZE="2", RANK=str(g), LOCAL_RANK=str(g), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT="29741", FOTO_BENCH_SHARD_TIMEOUT="90", TMPDIR=str(tmp_path))
        cmd = [sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "1",
               "--no-batch", "--no-c4"]
        procs.append(subprocess.Popen(cmd, cwd=REPO, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                                      text=True))
    outs = [p.communicate(timeout=180) for p in procs]
    for p, (o, e) in zip(procs, outs):
        assert p.returncode == 0, e[-2000:]
    lines = [ln for o, _ in outs for ln in o.splitlines() if ln.startswith("{")]
    assert len(lines) == 1
    d = json.loads(lines[0])
    print(d["error"])
    assert d["value"] is None and d["scaling"] == "strong" and d["n_gpus"] == 2 and d["rccl_ranks"] is None
    assert "rank 0" in d["error"] and "rank 1" in d["error"], d["error"]
    assert d["batch"] is None and d["c4"] is None


def test_visible_device(bench, monkeypatch):
    for k in ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        monkeypatch.delenv(k, raising=False)
    assert bench.visible_device(5) == 5                  # every GPU visible: LOCAL_RANK
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "5")       # one GPU per process
    assert bench.visible_device(5) == 0
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "0,1,2,3,4,5,6,7")
    assert bench.visible_device(5) == 5
