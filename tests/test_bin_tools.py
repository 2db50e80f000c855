"""Dataset-prep tools and the flow colour coding (row 4).

normalize_image.py / data_diff.py / create_lum_dataset.py are checked pixel-exact against
the outputs of the reference's own bin/ scripts (bin/normalize_image.py,
bin/data_diff.py, bin/create_lum_dataset.py) run on the same 48x40 PNG pair, recorded in
tests/golden/bin.npz by tests/golden/make_golden.py (gen_bin).  color_flow replaces a
prebuilt binary that is never run here: parity unpinned, checked on the published
algorithm's defining properties only.
"""
import os
import subprocess
import sys

import numpy as np
import pytest
from PIL import Image

from conftest import PKG

BIN = os.path.join(PKG, "bin")
sys.path.insert(0, BIN)
import color_flow  # noqa: E402
import create_lum_dataset  # noqa: E402
import data_diff  # noqa: E402
import normalize_image  # noqa: E402


def _u8(f, h, w):
    return np.uint8(255 * np.clip(f, 0, 1)).reshape(h, w)


def test_functions_match_reference_outputs(gold):
    d = gold("bin.npz")
    h, w = d["f1"].shape
    f1, f2 = d["f1"].ravel() / 255, d["f2"].ravel() / 255
    n1, n2 = normalize_image.normalize_pair(f1, f2)
    assert np.array_equal(_u8(n1, h, w), d["norm1"]) and np.array_equal(_u8(n2, h, w), d["norm2"])
    assert np.array_equal(_u8(data_diff.frame_diff(f1, f2), h, w), d["diff"])
    for sd in d["lum_seeds"]:
        assert np.array_equal(_u8(create_lum_dataset.lum_image(f2, w, h, int(sd)), h, w), d[f"lum_{sd}"])


def test_lum_does_not_modify_input(gold):
    d = gold("bin.npz")
    h, w = d["f2"].shape
    f = d["f2"].ravel() / 255
    keep = f.copy()
    create_lum_dataset.lum_image(f, w, h, 3)
    assert np.array_equal(f, keep)


def test_clis_match_reference_outputs(gold, tmp_path):
    """The scripts as run.sh calls them (run.sh:35-41, 95), PNG in, PNG out."""
    d = gold("bin.npz")
    p1, p2 = tmp_path / "frame10.png", tmp_path / "frame11.png"
    Image.fromarray(d["f1"], "L").save(p1)
    Image.fromarray(d["f2"], "L").save(p2)

    def run(script, *args):
        subprocess.run([sys.executable, os.path.join(BIN, script), *map(str, args)], check=True, cwd=tmp_path)

    def load(name):
        return np.asarray(Image.open(tmp_path / name).convert("L"))

    run("normalize_image.py", p1, p2, "n1.png", "n2.png")
    assert np.array_equal(load("n1.png"), d["norm1"]) and np.array_equal(load("n2.png"), d["norm2"])
    run("data_diff.py", p1, p2, "diff.png")
    assert np.array_equal(load("diff.png"), d["diff"])
    sd = int(d["lum_seeds"][0])
    run("create_lum_dataset.py", p2, "lum.png", sd)
    assert np.array_equal(load("lum.png"), d[f"lum_{sd}"])


def test_colorwheel_and_flow_coding():
    cw = color_flow.colorwheel()
    assert cw.shape == (55, 3)
    assert tuple(cw[0]) == (255, 0, 0)        # red
    assert tuple(cw[15]) == (255, 255, 0)     # RY -> yellow
    assert tuple(cw[21]) == (0, 255, 0)       # YG -> green
    assert tuple(cw[25]) == (0, 255, 255)     # GC -> cyan
    assert tuple(cw[36]) == (0, 0, 255)       # CB -> blue
    assert tuple(cw[49]) == (255, 0, 255)     # BM -> magenta
    w, h = 5, 3
    u = np.zeros(w * h); v = np.zeros(w * h)
    u[1] = 2.0                                 # the largest flow -> saturated
    u[2] = np.nan                              # unknown -> black
    v[3] = 2e9                                 # unknown -> black
    u[4] = -1.0                                # half magnitude
    img = color_flow.flow_to_color(u, v, w, h)
    assert img.shape == (h, w, 3) and img.dtype == np.uint8
    assert tuple(img[0, 0]) == (255, 255, 255)           # zero flow is white
    assert tuple(img[0, 2]) == (0, 0, 0) and tuple(img[0, 3]) == (0, 0, 0)
    # +x flow: a = atan2(-0.0, -1)/pi = -1 -> fk = 0 -> red, fully saturated (Middlebury: right = red)
    assert tuple(img[0, 1]) == (255, 0, 0)
    # -x flow at half radius: a = 0 -> fk = 27, halfway to white
    assert img[0, 4].min() >= 127
    # maxmotion smaller than the flow darkens out-of-range pixels (x 0.75)
    dark = color_flow.flow_to_color(u, v, w, h, maxmotion=1.0)
    assert tuple(dark[0, 1]) == (191, 0, 0)


def test_color_flow_cli(tmp_path):
    import utils
    w, h = 8, 6
    yy, xx = np.mgrid[0:h, 0:w]
    u, v = (xx - 3.5).ravel().astype(float), (yy - 2.5).ravel().astype(float)
    path = tmp_path / "f.flo"
    utils.saveFlo(w, h, u, v, str(path))
    subprocess.run([sys.executable, os.path.join(BIN, "color_flow.py"), str(path), str(tmp_path / "f.png")], check=True)
    img = np.asarray(Image.open(tmp_path / "f.png"))
    assert img.shape == (h, w, 3)
    assert np.array_equal(img, color_flow.flow_to_color(u, v, w, h))
