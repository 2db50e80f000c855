"""Two outer iterations in flight (foto_bb.cpp, c->pipe: single shard, fused prox + RHS, Gauss
CG -- the default path).  The host enqueues iteration i + 1 before it waits for iteration i's
crit (reference loop: benamou_brenier.py:204-258), so:

  * the stop rules (benamou_brenier.py:253-258) may end the run at i with i + 1 already on the
    stream: the rollback must leave phi, mu (and the F a later iterate() call starts from)
    exactly as a one-in-flight run leaves them;
  * a failed Gauss solve (K beyond the table; forced here with FOTO_GQ_KLIM) is redone with the
    s-step CG after the iteration behind it -- whose prox the done-flag chain skipped -- is
    dropped, and the loop enqueues that iteration again.

The kernels are the same in both loops, so the comparisons with FOTO_PIPE=0 are bit for bit."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

foto = pytest.importorskip("foto")
from foto.bb import BBSolver  # noqa: E402


def _run(d, monkeypatch, env, calls, **kw):
    for k in ("FOTO_PIPE", "FOTO_GQ_KLIM", "FOTO_CG_DEFER", "FOTO_HOST_CRIT", "FOTO_PHASE_EV"):
        monkeypatch.delenv(k, raising=False)
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    Nt, Ny, Nx = (int(v) for v in d["shape"])
    r, tol, eps, max_it = d["params"]
    with BBSolver(d["rho0"], d["rhoT"], Nt, Nx, Ny, r=r, reg_epsilon=eps, **kw) as s:
        for n, t, rules in calls:
            s.iterate(n, tol if t is None else t, rules)
        out = dict(crit=np.array(s.crit), its=np.array(s.cg_its), flow=s.flow(), phi=s.phi(), state=s.state(),
                   stats=s.stats())
    return out


def _same(a, b):
    assert np.array_equal(a["crit"], b["crit"])
    assert np.array_equal(a["its"], b["its"])
    for x, y in zip(a["flow"], b["flow"]):
        assert np.array_equal(x, y)
    assert np.array_equal(a["phi"], b["phi"])
    for x, y in zip(a["state"], b["state"]):
        assert np.array_equal(x, y)


def test_pipe_stop_rules_match_one_in_flight(gold, monkeypatch):
    """C1 golden run (46 outer iterations, the stop rule ends it): the pipelined loop drops the
    47th iteration it had enqueued; crit, CG counts, phi, mu, q and the flow equal the
    one-in-flight loop's, and the run meets the reference golden."""
    d = gold("bb_c1.npz")
    max_it = int(d["params"][3])
    a = _run(d, monkeypatch, {}, [(max_it, None, True)])
    b = _run(d, monkeypatch, {"FOTO_PIPE": "0"}, [(max_it, None, True)])
    _same(a, b)
    assert len(a["crit"]) == len(d["crit"])
    np.testing.assert_allclose(a["crit"], d["crit"], rtol=1e-5, atol=0)


def test_pipe_rollback_then_continue(gold, monkeypatch):
    """Stop early (a loose tolerance ends the run after a few iterations), then iterate again
    without the stop rules: the second call starts from the rolled-back state (F recomputed from
    q of the kept iteration) and reproduces the one-in-flight loop bit for bit."""
    d = gold("bb_c1.npz")
    calls = [(40, 0.5, True), (4, 0.0, False), (3, 0.0, True), (5, 0.0, False)]
    a = _run(d, monkeypatch, {}, calls)
    b = _run(d, monkeypatch, {"FOTO_PIPE": "0"}, calls)
    _same(a, b)
    assert len(a["crit"]) >= 9


@pytest.mark.parametrize("klim", ["1", "200"])
def test_pipe_gauss_redo(gold, monkeypatch, klim):
    """FOTO_GQ_KLIM makes every solve (1) or the solves with more than 200 CG iterations (C1:
    197-202, a mix) report status 2: each is redone with the s-step CG after the iteration
    behind it is dropped.  The run matches the one-in-flight loop under the same knob bit for
    bit and meets the reference golden (the s-step CG's bars)."""
    d = gold("bb_c1.npz")
    max_it = int(d["params"][3])
    a = _run(d, monkeypatch, {"FOTO_GQ_KLIM": klim}, [(max_it, None, True)])
    b = _run(d, monkeypatch, {"FOTO_GQ_KLIM": klim, "FOTO_PIPE": "0"}, [(max_it, None, True)])
    _same(a, b)
    n = len(a["crit"])
    assert n == len(d["crit"])
    redo = a["stats"]["cg_redo"]
    if klim == "1":
        assert redo == n
    else:
        assert 0 < redo < n
    assert np.max(np.abs(a["its"] - d["cg_its"])) <= 1
    np.testing.assert_allclose(a["crit"], d["crit"], rtol=1e-5, atol=0)


def test_pipe_exact_iteration_count(gold, monkeypatch):
    """Without the stop rules the loop enqueues exactly max_it iterations (never one beyond),
    and chunked calls equal one call."""
    d = gold("bb_tex.npz")
    a = _run(d, monkeypatch, {}, [(7, 0.0, False)])
    b = _run(d, monkeypatch, {}, [(3, 0.0, False), (1, 0.0, False), (3, 0.0, False)])
    c = _run(d, monkeypatch, {"FOTO_PIPE": "0"}, [(7, 0.0, False)])
    _same(a, b)
    _same(a, c)
    assert len(a["crit"]) == 7 and a["stats"]["outer_iters"] == 7


@pytest.mark.parametrize("klim", ["1", "200", None])
@pytest.mark.parametrize("vr", [2, 3])
def test_sharded_gauss_deferred(gold, monkeypatch, vr, klim):
    """Sharded Gauss CG enqueued whole (x^, all-to-all back, inverse DCTs and the prox guarded by
    each shard's done flag) and checked at the crit sync; a failed solve (FOTO_GQ_KLIM) is redone
    there with the s-step CG from b^ by every shard.  Bit-identical to the sharded solve waited
    for on the host (FOTO_CG_DEFER=0), which redoes the same solves before the inverse."""
    d = gold("bb_c1.npz")
    max_it = int(d["params"][3])
    env = {} if klim is None else {"FOTO_GQ_KLIM": klim}
    a = _run(d, monkeypatch, env, [(max_it, None, True)], virtual_ranks=vr)
    b = _run(d, monkeypatch, {**env, "FOTO_CG_DEFER": "0"}, [(max_it, None, True)], virtual_ranks=vr)
    monkeypatch.delenv("FOTO_CG_DEFER", raising=False)
    _same(a, b)
    n = len(a["crit"])
    assert n == len(d["crit"])
    assert a["stats"]["cg_redo"] == b["stats"]["cg_redo"]
    if klim == "1":
        assert a["stats"]["cg_redo"] == n
    assert np.max(np.abs(a["its"] - d["cg_its"])) <= 1
    np.testing.assert_allclose(a["crit"], d["crit"], rtol=1e-5, atol=0)


@pytest.mark.parametrize("klim", [None, "200"])
def test_host_readback_stores(gold, monkeypatch, klim):
    """The crit pair and the Gauss solve's header reach the host as stores of the kernels
    themselves into pinned, coherent slots (no copy launch); FOTO_HOST_CRIT=0 copies them on the
    stream instead.  Same run either way, including the redone solves (KLIM 200)."""
    d = gold("bb_c1.npz")
    max_it = int(d["params"][3])
    env = {} if klim is None else {"FOTO_GQ_KLIM": klim}
    a = _run(d, monkeypatch, env, [(max_it, None, True)])
    b = _run(d, monkeypatch, {**env, "FOTO_HOST_CRIT": "0"}, [(max_it, None, True)])
    _same(a, b)
    assert a["stats"]["cg_redo"] == b["stats"]["cg_redo"]
    np.testing.assert_allclose(a["crit"], d["crit"], rtol=1e-5, atol=0)


@pytest.mark.parametrize("klim", [None, "200"])
def test_phase_events_only_with_timing(gold, monkeypatch, klim):
    """The RHS / CG / prox phase events are recorded only with kernel timing on (or
    FOTO_PHASE_EV=1); the crit sync then uses a timing-free event.  Same run either way,
    including the redone solves (KLIM 200); the phase times are 0 without the events."""
    d = gold("bb_c1.npz")
    max_it = int(d["params"][3])
    env = {} if klim is None else {"FOTO_GQ_KLIM": klim}
    a = _run(d, monkeypatch, env, [(max_it, None, True)])
    c = _run(d, monkeypatch, {**env, "FOTO_PHASE_EV": "1"}, [(max_it, None, True)])
    _same(a, c)
    assert a["stats"]["cg_redo"] == c["stats"]["cg_redo"]
    assert c["stats"]["ms_cg"] > 0 and a["stats"]["ms_cg"] == 0
    np.testing.assert_allclose(a["crit"], d["crit"], rtol=1e-5, atol=0)


def test_callback_sees_its_own_iteration(gold, monkeypatch):
    """The iteration callback runs while iteration i + 1 is already on the stream.  In the
    pipelined loop phi(), state() and flow() called from it return iteration i's results (the
    record of the iteration in flight keeps them): each equals the final state of a run of
    i + 1 iterations.  The one-in-flight loop (FOTO_PIPE=0) refuses them there."""
    d = gold("bb_tex.npz")
    Nt, Ny, Nx = (int(v) for v in d["shape"])
    r, _, eps, _ = d["params"]
    for k in ("FOTO_PIPE", "FOTO_GQ_KLIM"):
        monkeypatch.delenv(k, raising=False)
    seen = {}
    with BBSolver(d["rho0"], d["rhoT"], Nt, Nx, Ny, r=r, reg_epsilon=eps) as s:
        def cb(i, crit, its, info):
            seen[i] = (s.phi(), s.state(), s.flow())
        s.iterate(5, 0.0, False, callback=cb)
    assert sorted(seen) == list(range(5))
    for n in (2, 4, 5):
        with BBSolver(d["rho0"], d["rhoT"], Nt, Nx, Ny, r=r, reg_epsilon=eps) as s:
            s.iterate(n, 0.0, False)
            ref = (s.phi(), s.state(), s.flow())
        phi, (mu, q), fl = seen[n - 1]
        assert np.array_equal(phi, ref[0])
        assert np.array_equal(mu, ref[1][0]) and np.array_equal(q, ref[1][1])
        for x, y in zip(fl, ref[2]):
            assert np.array_equal(x, y)
    monkeypatch.setenv("FOTO_PIPE", "0")
    errs = []
    with BBSolver(d["rho0"], d["rhoT"], Nt, Nx, Ny, r=r, reg_epsilon=eps) as s:
        def cb0(i, crit, its, info):
            try:
                s.phi()
            except foto.FotoError as e:
                errs.append(i)
        s.iterate(3, 0.0, False, callback=cb0)
        s.phi()   # after the call: fine
    assert errs == [0, 1]   # (the last callback runs with nothing in flight)
