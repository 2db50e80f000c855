"""Drop-in for the reference's bin/normalize_image.py (bin/normalize_image.py:17-30):
mass-normalise a frame pair (each divided by its sum, then both by the larger maximum)
and write them back as 8-bit PNGs.  Identical arithmetic (numpy), identical output."""
import argparse

import numpy as np

from _common import open_gray, save_gray


def normalize_pair(f1, f2):
    f1 = f1 / np.sum(f1)
    f2 = f2 / np.sum(f2)
    scale = max(np.max(f1), np.max(f2))
    return f1 / scale, f2 / scale


def main(argv=None):
    ap = argparse.ArgumentParser(description="sample argument parser")
    ap.add_argument("f1", help="frame 1")
    ap.add_argument("f2", help="frame 1")
    ap.add_argument("out1", help="output 1")
    ap.add_argument("out2", help="output 2")
    a = ap.parse_args(argv)
    f1, w, h = open_gray(a.f1)
    f2, w, h = open_gray(a.f2)
    f1, f2 = normalize_pair(f1, f2)
    save_gray(f1, w, h, a.out1)
    save_gray(f2, w, h, a.out2)


if __name__ == "__main__":
    main()
