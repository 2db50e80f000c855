"""Drop-in for the reference's bin/data_diff.py (bin/data_diff.py:24-35): the frame
difference f2 - f1 rescaled to [0, 1], written as an 8-bit PNG."""
import argparse

import numpy as np

from _common import open_gray, save_gray


def frame_diff(f1, f2):
    diff = f2 - f1
    diff = diff - np.min(diff)
    return diff / np.max(diff)


def main(argv=None):
    ap = argparse.ArgumentParser(description="sample argument parser")
    ap.add_argument("f0", help="first frame")
    ap.add_argument("f1", help="second frame")
    ap.add_argument("out", help="output")
    a = ap.parse_args(argv)
    f1, w, h = open_gray(a.f0)
    f2, w, h = open_gray(a.f1)
    save_gray(frame_diff(f1, f2), w, h, a.out)


if __name__ == "__main__":
    main()
