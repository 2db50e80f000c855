"""The batch pipeline run.py, the drop-in for run.sh:1-167.

CPU: bash $RANDOM restatement vs bash itself (tests/golden/bin.npz), `prepare` on a tiny
synthetic dataset against the bin/ tools it composes, the run loop's outputs, skip
markers, restart and GPU sharding with the solver stubbed out.  GPU: real GN + FOTO solves
through libfoto.so on two small sequences, compared against main.py run directly.
"""
import json
import os

import numpy as np
import pytest
from PIL import Image

import run as pipeline
import utils
from _common import open_gray
from create_lum_dataset import lum_image
from normalize_image import normalize_pair


def test_bash_random_matches_bash(gold):
    d = gold("bin.npz")
    assert pipeline.bash_random(12345, len(d["bash_random_12345"])) == list(d["bash_random_12345"])


def _pattern(w, h, shift, seed):
    yy, xx = np.mgrid[0:h, 0:w].astype(float)
    rng = np.random.default_rng(seed)
    f = 0.5 + 0.3 * np.sin((xx - shift) / 4.0 + rng.uniform(0, 3)) * np.cos(yy / 5.0) + 0.05 * rng.random((h, w))
    return np.uint8(255 * np.clip(f, 0, 1))


def _make_data(root, seqs=("Army", "Grove", "Urban"), w=96, h=80):
    base = root / "data" / "middlebury-1" / "eval-data-gray"
    for i, s in enumerate(seqs):
        (base / s).mkdir(parents=True)
        Image.fromarray(_pattern(w, h, 0, i), "L").save(base / s / "frame10.png")
        Image.fromarray(_pattern(w, h, 1.5, i), "L").save(base / s / "frame11.png")
    (base / "README").write_text("not a sequence")      # skipped like `[ -d "$dir" ]`
    return base


def _args(root, *extra):
    return pipeline.parse_args([*extra, f"--data={root / 'data'}", f"--results={root / 'results'}"])


def test_prepare(tmp_path):
    base = _make_data(tmp_path)
    orig = {s: [np.asarray(Image.open(base / s / f"frame1{k}.png")) for k in (0, 1)] for s in ("Army", "Grove", "Urban")}
    pipeline.main(["prepare", f"--data={tmp_path / 'data'}"])
    lum = tmp_path / "data" / "middlebury-1-lum" / "eval-data-gray"
    seeds = pipeline.bash_random(12345, 3)
    for s, sd in zip(("Army", "Grove", "Urban"), seeds):
        # resized (50 %), then normalised in place
        r = [np.asarray(Image.fromarray(orig[s][k]).resize((48, 40), Image.LANCZOS)) for k in (0, 1)]
        n1, n2 = normalize_pair(r[0].ravel() / 255, r[1].ravel() / 255)
        got = [open_gray(str(base / s / f"frame1{k}.png"))[0] for k in (0, 1)]
        assert np.array_equal(np.uint8(255 * got[0]), np.uint8(255 * np.clip(n1, 0, 1)))
        assert np.array_equal(np.uint8(255 * got[1]), np.uint8(255 * np.clip(n2, 0, 1)))
        # lum: frame10 copied, frame11 lit with the s-th $RANDOM seed, both normalised
        l1 = r[0].ravel() / 255
        l2 = np.uint8(255 * np.clip(lum_image(r[1].ravel() / 255, 48, 40, sd), 0, 1)).ravel() / 255
        m1, m2 = normalize_pair(l1, l2)
        g = [open_gray(str(lum / s / f"frame1{k}.png"))[0] for k in (0, 1)]
        assert np.array_equal(np.uint8(255 * g[0]), np.uint8(255 * np.clip(m1, 0, 1)))
        assert np.array_equal(np.uint8(255 * g[1]), np.uint8(255 * np.clip(m2, 0, 1)))


def _stub_solver(monkeypatch, calls):
    """main.py stand-in: records argv, writes the files main.py would."""
    def fake(argv, log_path, writer=None):
        calls.append(argv)
        kv = dict(a[2:].split("=", 1) for a in argv if a.startswith("--") and "=" in a)
        f, w, h = open_gray(argv[0])
        u, v = np.full(w * h, 0.5), np.full(w * h, -0.25)
        utils.saveFlo(w, h, u, v, kv["out"])
        with open(kv["save-benchmark"], "w") as fh:
            fh.write("IE: 1.5\ntime: 0.1s")
        for k in ("save-reconstruction", "save-lum"):
            Image.fromarray(np.zeros((h, w), np.uint8), "L").save(kv[k])
        open(log_path, "w").close()
        return u, v, np.zeros(w * h)
    monkeypatch.setattr(pipeline, "run_main", fake)


def test_color_from_arrays_matches_flo_round_trip(tmp_path):
    """The background writer colours (u, v) directly; the PNG is byte-identical to colouring
    the saved .flo (run.sh:104 reads the .flo)."""
    rng = np.random.default_rng(3)
    w, h = 37, 23
    u, v = rng.normal(0, 2.5, w * h), rng.normal(0, 1.5, w * h)
    utils.saveFlo(w, h, u, v, str(tmp_path / "a.flo"))
    pipeline.color_flow(str(tmp_path / "a.flo"), str(tmp_path / "a.png"))
    pipeline.color_flow_arrays(u, v, w, h, str(tmp_path / "b.png"))
    assert np.array_equal(np.asarray(Image.open(tmp_path / "a.png")), np.asarray(Image.open(tmp_path / "b.png")))


def test_writer_markers_after_files_and_errors(tmp_path):
    import threading
    import time
    w = pipeline.Writer(threads=4)
    seen, lock = [], threading.Lock()

    def slow(i):
        time.sleep(0.01 * (i % 3))
        with lock:
            seen.append(i)
    for g in range(5):
        futs = [w.submit(slow, 10 * g + i) for i in range(4)]
        w.when_all(futs, lambda g=g: seen.append(("marker", g)))
    w.drain()
    time.sleep(0.05)   # callbacks run in the worker that finished last
    for g in range(5):
        k = seen.index(("marker", g))
        assert all(seen.index(10 * g + i) < k for i in range(4))

    def boom():
        raise OSError("disk full")
    f = w.submit(boom)
    w.when_all([f], lambda: seen.append("never"))
    with pytest.raises(OSError):
        w.close()
    assert "never" not in seen


def test_run_loop_markers_and_restart(tmp_path, monkeypatch):
    _make_data(tmp_path)
    pipeline.main(["prepare", f"--data={tmp_path / 'data'}"])
    calls = []
    _stub_solver(monkeypatch, calls)
    common = [f"--data={tmp_path / 'data'}", f"--results={tmp_path / 'results'}"]
    assert pipeline.main(["run", *common]) == 0
    assert len(calls) == 2 * 2 * 3                   # 2 datasets x 3 sequences x {GN, FOTO}
    gn = [c for c in calls if "--algo=GN" in c]
    foto = [c for c in calls if "--algo=foto" in c]
    assert all(set(pipeline.GN_ARGS) <= set(c) for c in gn) and len(gn) == 6
    assert all(set(pipeline.FOTO_ARGS) <= set(c) for c in foto) and len(foto) == 6
    for ds in ("middlebury-1", "middlebury-1-lum"):
        for s in ("Army", "Grove", "Urban"):
            out = tmp_path / "results" / ds / s
            for name in ("diff.png", ".out.gn.sucess", ".out.foto.sucess", "gn.png", "foto.png", "gn.flo", "foto.benchmark.txt"):
                assert (out / name).is_file(), (ds, s, name)
            f0, w, h = open_gray(str(tmp_path / "data" / ds / "eval-data-gray" / s / "frame10.png"))
            f1, w, h = open_gray(str(tmp_path / "data" / ds / "eval-data-gray" / s / "frame11.png"))
            import data_diff
            d = np.asarray(Image.open(out / "diff.png"))
            assert np.array_equal(d, np.uint8(255 * np.clip(data_diff.frame_diff(f0, f1), 0, 1)).reshape(h, w))
    rows = json.load(open(tmp_path / "results" / "summary.json"))
    assert len(rows) == 12 and all(r["IE"] == 1.5 for r in rows)
    # markers present: nothing re-solved (run.sh:98, 109)
    calls.clear()
    (tmp_path / "results" / "middlebury-1" / "Grove" / ".out.foto.sucess").unlink()
    pipeline.main(["run", *common])
    assert len(calls) == 1 and "--algo=foto" in calls[0] and "Grove" in calls[0][0]
    # restart wipes results (run.sh:76-79)
    calls.clear()
    pipeline.main(["restart", *common])
    assert len(calls) == 12


def test_sharding_covers_every_sequence_once(tmp_path, monkeypatch):
    _make_data(tmp_path, seqs=tuple(f"S{i}" for i in range(7)), w=40, h=32)
    calls = []
    _stub_solver(monkeypatch, calls)
    args = _args(tmp_path, "run")
    for world in (1, 2, 3, 8):
        seen = []
        for rank in range(world):
            mine = pipeline.shard(pipeline.jobs(args), rank, world)
            seen += [(d.name, s) for d, s in mine]
            assert len(mine) in (len(pipeline.jobs(args)) // world, -(-len(pipeline.jobs(args)) // world))
        assert sorted(seen) == sorted((d.name, s) for d, s in pipeline.jobs(args))
    # torch.distributed.run-style launch: each rank solves only its shard
    for rank in range(2):
        monkeypatch.setenv("WORLD_SIZE", "2")
        monkeypatch.setenv("RANK", str(rank))
        monkeypatch.setenv("LOCAL_RANK", str(rank))
        pipeline.main(["run", f"--data={tmp_path / 'data'}", f"--results={tmp_path / 'results'}"])
    assert len(calls) == 7 * 2                         # middlebury-1 only (no lum data), GN + FOTO
    assert len({c[0] for c in calls}) == 7
    devs = {c[0].split(os.sep)[-2]: [a for a in c if a.startswith("--device=")][0] for c in calls}
    assert devs["S0"] == "--device=0" and devs["S1"] == "--device=1"


def test_extra_dataset_with_ground_truth(tmp_path, monkeypatch):
    frames = tmp_path / "m2" / "other-data-gray"
    gtdir = tmp_path / "m2" / "other-gt-flow"
    for s in ("Dimetrodon", "Venus"):
        (frames / s).mkdir(parents=True)
        Image.fromarray(_pattern(40, 32, 0, 3), "L").save(frames / s / "frame10.png")
        Image.fromarray(_pattern(40, 32, 1, 3), "L").save(frames / s / "frame11.png")
    (gtdir / "Venus").mkdir(parents=True)
    utils.saveFlo(40, 32, np.ones(40 * 32), np.zeros(40 * 32), str(gtdir / "Venus" / "flow10.flo"))
    calls = []
    _stub_solver(monkeypatch, calls)
    pipeline.main(["run", f"--data={tmp_path / 'nodata'}", f"--results={tmp_path / 'results'}",
                   f"--dataset=middlebury-2={frames}:{gtdir}"])
    gt = {c[0].split(os.sep)[-2]: any(a.startswith("--ground-truth=") for a in c) for c in calls}
    assert gt == {"Dimetrodon": False, "Venus": True}


@pytest.mark.gpu
def test_pipeline_gpu_end_to_end(tmp_path):
    """Real solves (run.sh's GN and FOTO parameters) on two 48x40 sequences; the pipeline's
    flows equal main.py's run directly on the same frames, markers make a re-run a no-op."""
    import main as cli
    _make_data(tmp_path, seqs=("Army", "Grove"))
    common = [f"--data={tmp_path / 'data'}", f"--results={tmp_path / 'results'}"]
    pipeline.main(["prepare", common[0]])
    assert pipeline.main(["run", *common]) == 0
    rows = json.load(open(tmp_path / "results" / "summary.json"))
    assert len(rows) == 8 and all(np.isfinite(r["IE"]) for r in rows)
    seq = tmp_path / "data" / "middlebury-1-lum" / "eval-data-gray" / "Grove"
    for algo, args in pipeline.ALGOS:
        direct = tmp_path / f"direct_{algo}.flo"
        cli.main([str(seq / "frame10.png"), str(seq / "frame11.png"), f"--out={direct}", *args])
        a = utils.openFlo(str(direct))
        b = utils.openFlo(str(tmp_path / "results" / "middlebury-1-lum" / "Grove" / f"{algo}.flo"))
        assert a[:2] == b[:2] and np.array_equal(a[2], b[2]) and np.array_equal(a[3], b[3])
    before = os.path.getmtime(tmp_path / "results" / "middlebury-1" / "Army" / "foto.flo")
    pipeline.main(["run", *common])
    assert os.path.getmtime(tmp_path / "results" / "middlebury-1" / "Army" / "foto.flo") == before


@pytest.mark.gpu
def test_pipeline_gpu_vs_reference_cli(gold, tmp_path):
    """The pipeline's per-sequence run against the reference itself: tests/golden/cli.npz
    holds the reference main.py's results on a 36x28 PNG pair (make_golden.py, GN with
    run.sh's alpha / lambda, FOTO with Nt = 4, 8 outer iterations).  The same PNG bytes as a
    one-sequence dataset through run.py (FOTO parameters forwarded after `--`) give the same
    .flo to 1e-5 px and the same IE."""
    d = gold("cli.npz")
    frames = tmp_path / "frames"
    (frames / "Pair").mkdir(parents=True)
    d["png0"].tofile(frames / "Pair" / "frame10.png")
    d["png1"].tofile(frames / "Pair" / "frame11.png")
    assert pipeline.main(["run", f"--data={tmp_path / 'nodata'}", f"--results={tmp_path / 'results'}",
                          f"--dataset=ref={frames}", "--", "--Nt=4", "--max-it=8"]) == 0
    for algo, key in (("gn", "GN"), ("foto", "foto")):
        w, h, uu, vv = utils.openFlo(str(tmp_path / "results" / "ref" / "Pair" / f"{algo}.flo"))
        assert (w, h) == (36, 28)
        ref = np.frombuffer(d[f"{key}_flo"].tobytes()[12:], dtype=np.float32)
        np.testing.assert_allclose(np.stack([uu, vv], 1).ravel(), ref, rtol=0, atol=1e-5)
    rows = {r["algo"]: r for r in json.load(open(tmp_path / "results" / "summary.json")) if r["sequence"] == "Pair"}
    for algo, key in (("gn", "GN"), ("foto", "foto")):
        assert abs(float(rows[algo]["IE"]) - float(d[f"{key}_ie"])) < 1e-4


def test_worker_argv_round_trip(tmp_path):
    """`--gpus N` re-invokes run.py per GPU; the children must see the parent's options."""
    a = pipeline.parse_args(["run", "--gpus=4", f"--data={tmp_path}/d", "--results=r",
                                            "--dataset=m2=/x/frames:/x/gt", "--", "--cg-mode=2"])
    b = pipeline.parse_args(["run", "--gpus=4", "--worker-rank=3", *pipeline.forward_args(a)])
    assert (b.data, b.results, b.dataset, b.extra, b.worker_rank) == (a.data, a.results, a.dataset, ["--cg-mode=2"], 3)


def test_worker_device_map(tmp_path, monkeypatch):
    """--devices / FOTO_RUN_DEVICES put worker i on device LIST[i mod len] (several workers can
    share a GPU); without them worker i gets device i.  The parent only starts the children
    (HIP_VISIBLE_DEVICES per child) and never touches a device."""
    started = []

    class FakePopen:
        def __init__(self, cmd, env=None, **kw):
            started.append((cmd, env["HIP_VISIBLE_DEVICES"]))

        def wait(self):
            return 0

    monkeypatch.setattr(pipeline.subprocess, "Popen", FakePopen)
    monkeypatch.setattr(pipeline, "summarize", lambda args: [])
    monkeypatch.delenv("FOTO_RUN_DEVICES", raising=False)
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    common = [f"--data={tmp_path / 'd'}", f"--results={tmp_path / 'r'}"]
    assert pipeline.main(["run", "--gpus=3", *common]) == 0
    assert [d for _, d in started] == ["0", "1", "2"]
    assert [c[c.index("run") + 2] for c, _ in started] == ["--worker-rank=0", "--worker-rank=1", "--worker-rank=2"]
    started.clear()
    assert pipeline.main(["run", "--gpus=4", "--devices=0,0,1", *common]) == 0
    assert [d for _, d in started] == ["0", "0", "1", "0"]
    started.clear()
    started.clear()
    assert pipeline.main(["run", "--gpus=2", "--per-gpu=2", *common]) == 0   # 4 workers, 2 per GPU
    assert [d for _, d in started] == ["0", "1", "0", "1"]
    assert all("--gpus=4" in c for c, _ in started)
    started.clear()
    monkeypatch.setenv("FOTO_RUN_DEVICES", "5,5")
    assert pipeline.main(["run", "--gpus=2", *common]) == 0
    assert [d for _, d in started] == ["5", "5"]
    monkeypatch.setenv("FOTO_RUN_DEVICES", "a,b")
    with pytest.raises(SystemExit):
        pipeline.main(["run", "--gpus=2", *common])
