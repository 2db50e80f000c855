"""The communication model beside the compute-only proxy curves (tools/proxy_scaling.py,
DESIGN.md section 5): a model, not a measurement, so its arithmetic is pinned here on the CPU --
the pipeline formula, the phi halo inside or beside the backward all-to-all, and the w_t plane
hidden behind the measured prox time when the overlap is on (foto_bb.cpp wt_overlap)."""
import importlib.util
import os

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture()
def model(monkeypatch):
    for k in ("FOTO_A2A_PARTS", "FOTO_A2A_HALO", "FOTO_WT_OVERLAP"):
        monkeypatch.delenv(k, raising=False)
    spec = importlib.util.spec_from_file_location("proxy_scaling", os.path.join(HERE, "..", "tools", "proxy_scaling.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def test_pipeline_formula(model):
    # one part: the transfer follows the compute, all of it exposed
    assert model.pipe_us(100.0, 40.0, 1) == pytest.approx(40.0)
    # transfer shorter than compute, many parts: only the last part's transfer stays exposed
    assert model.pipe_us(100.0, 40.0, 4) == pytest.approx(40.0 / 4)
    # transfer longer than compute: at least its excess over the compute stays exposed
    for p in (1, 2, 4, 8):
        assert model.pipe_us(100.0, 130.0, p) >= 30.0 - 1e-9


def test_one_rank_has_no_communication(model):
    model.NX, model.NY, model.NT = 640, 480, 32
    assert model.comm_model_us(1, 0.1) == (0.0, {})


def test_wt_plane_hidden_behind_the_prox(model, monkeypatch):
    model.NX, model.NY, model.NT = 1024, 1024, 64
    plane_us = model.NX * model.NY * 8 / (model.LINK_GBS * 1e3)
    _, slow = model.comm_model_us(8, 0.2, prox_ms=0.0)
    _, fast = model.comm_model_us(8, 0.2, prox_ms=1.0)
    assert slow["halo_wt"] == pytest.approx(plane_us + model.LAT_US)
    assert fast["halo_wt"] == 0.0
    monkeypatch.setenv("FOTO_WT_OVERLAP", "0")
    _, off = model.comm_model_us(8, 0.2, prox_ms=1.0)
    assert off["halo_wt"] == pytest.approx(plane_us + model.LAT_US)
    # slabs of fewer than three planes keep w_t after the prox (wt_overlap's rule)
    monkeypatch.delenv("FOTO_WT_OVERLAP")
    model.NT = 16
    _, thin = model.comm_model_us(8, 0.2, prox_ms=1.0)
    assert thin["halo_wt"] == pytest.approx(plane_us + model.LAT_US)


def test_phi_halo_inside_or_beside_the_backward_alltoall(model, monkeypatch):
    model.NX, model.NY, model.NT = 1024, 1024, 64   # planes of 2^20 voxels: halo inside by default
    _, inside = model.comm_model_us(8, 0.2, prox_ms=1.0)
    assert inside["halo_phi"] == 0.0
    monkeypatch.setenv("FOTO_A2A_HALO", "0")
    _, beside = model.comm_model_us(8, 0.2, prox_ms=1.0)
    assert beside["halo_phi"] > 0.0
    assert beside["alltoall_inv"] <= inside["alltoall_inv"]   # two planes fewer on the wire
