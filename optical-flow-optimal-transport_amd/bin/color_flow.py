"""Replacement for the reference's prebuilt bin/color_flow (run.sh:104): Middlebury flow
colour coding of a .flo file to a PNG.  The reference ships it only as a binary (it is
never run here), so this restates the published Middlebury flow-code algorithm
(colorcode.cpp / color_flow.cpp, Baker et al.): a 55-entry colour wheel (RY 15, YG 6,
GC 4, CB 11, BM 13, MR 6), hue from atan2(-v, -u), saturation from |flow| / maxrad
(maxrad = the largest known flow magnitude, or the optional maxmotion argument),
out-of-range flow darkened by 0.75, unknown flow (|u| or |v| > 1e9, NaN) black; float32
arithmetic as the C++.  Parity unpinned: no output of the binary is available.

usage: color_flow.py in.flo out.png [maxmotion]"""
import argparse
import os
import sys

import numpy as np
from PIL import Image

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

UNKNOWN_FLOW_THRESH = 1e9


def colorwheel():
    RY, YG, GC, CB, BM, MR = 15, 6, 4, 11, 13, 6
    cols = []
    cols += [(255, 255 * i // RY, 0) for i in range(RY)]
    cols += [(255 - 255 * i // YG, 255, 0) for i in range(YG)]
    cols += [(0, 255, 255 * i // GC) for i in range(GC)]
    cols += [(0, 255 - 255 * i // CB, 255) for i in range(CB)]
    cols += [(255 * i // BM, 0, 255) for i in range(BM)]
    cols += [(255, 0, 255 - 255 * i // MR) for i in range(MR)]
    return np.array(cols, dtype=np.float32)


def flow_to_color(u, v, w, h, maxmotion=0.0):
    """(h, w, 3) uint8 RGB image of the flow (u, v) (flattened row-major, length w*h)."""
    u = np.asarray(u, dtype=np.float32).reshape(h, w)
    v = np.asarray(v, dtype=np.float32).reshape(h, w)
    unknown = (np.abs(u) > UNKNOWN_FLOW_THRESH) | (np.abs(v) > UNKNOWN_FLOW_THRESH) | np.isnan(u) | np.isnan(v)
    rad = np.sqrt(u * u + v * v)
    maxrad = float(np.max(rad[~unknown])) if np.any(~unknown) else -1.0
    if maxmotion > 0:
        maxrad = maxmotion
    if maxrad <= 0:
        maxrad = 1.0
    fx = np.where(unknown, 0, u) / np.float32(maxrad)
    fy = np.where(unknown, 0, v) / np.float32(maxrad)
    cw = colorwheel()
    ncols = cw.shape[0]
    r = np.sqrt(fx * fx + fy * fy)
    a = np.arctan2(-fy, -fx) / np.float32(np.pi)
    fk = (a + np.float32(1.0)) / np.float32(2.0) * np.float32(ncols - 1)
    k0 = fk.astype(np.int32)
    k1 = (k0 + 1) % ncols
    f = fk - k0.astype(np.float32)
    img = np.zeros((h, w, 3), dtype=np.uint8)
    for b in range(3):
        col0 = cw[k0, b] / np.float32(255.0)
        col1 = cw[k1, b] / np.float32(255.0)
        col = (np.float32(1) - f) * col0 + f * col1
        col = np.where(r <= 1, np.float32(1) - r * (np.float32(1) - col), col * np.float32(0.75))
        img[..., b] = np.where(unknown, 0, (np.float32(255.0) * col).astype(np.int32)).astype(np.uint8)
    return img


def main(argv=None):
    ap = argparse.ArgumentParser(description="Middlebury flow colour coding")
    ap.add_argument("flo")
    ap.add_argument("png")
    ap.add_argument("maxmotion", nargs="?", type=float, default=0.0)
    a = ap.parse_args(argv)
    import utils
    w, h, u, v = utils.openFlo(a.flo)
    Image.fromarray(flow_to_color(u, v, w, h, a.maxmotion), "RGB").save(a.png)


if __name__ == "__main__":
    main()
