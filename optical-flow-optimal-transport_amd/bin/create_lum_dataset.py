"""Drop-in for the reference's bin/create_lum_dataset.py (bin/create_lum_dataset.py:8-57):
add two random rectangles and two random discs of illumination (+-0.25) to a frame.

Same `random` calls in the same order (randint / uniform, seeded with `random.seed(seed)`),
so the same shapes; the per-pixel loops of the reference are slice / mask additions here,
each pixel receiving the same additions in the same order -- identical output."""
import argparse
import random

import numpy as np

from _common import open_gray, save_gray


def add_rectangle(f, w, h, L_x, L_y, r_x, r_y, v):
    g = f.reshape(h, w)
    g[int(r_y - L_y / 2):int(r_y + L_y / 2), int(r_x - L_x / 2):int(r_x + L_x / 2)] += v
    return f


def add_circle(f, w, h, R, c_x, c_y, v):
    jj, ii = np.mgrid[0:h, 0:w]
    mask = ((ii - c_x) ** 2 + (jj - c_y) ** 2 < R ** 2).ravel()
    f[mask] += v
    return f


def add_random_rectangle(f, w, h):
    L_x = random.randint(10, w - 1)
    L_y = random.randint(10, h - 1)
    r_x = random.randint(int(L_x / 2), int(w - L_x / 2))
    r_y = random.randint(int(L_y / 2), int(h - L_y / 2))
    v = random.uniform(-0.25, 0.25)
    return add_rectangle(f, w, h, L_x, L_y, r_x, r_y, v)


def add_random_circle(f, w, h):
    R = random.randint(10, min(w, h)) / 2
    c_x = random.randint(int(R), int(w - R))
    c_y = random.randint(int(R), int(h - R))
    v = random.uniform(-0.25, 0.25)
    return add_circle(f, w, h, R, c_x, c_y, v)


def lum_image(f, w, h, seed):
    random.seed(seed)
    f = np.array(f, dtype=np.float64)
    f = add_random_rectangle(f, w, h)
    f = add_random_rectangle(f, w, h)
    f = add_random_circle(f, w, h)
    f = add_random_circle(f, w, h)
    return f


def main(argv=None):
    ap = argparse.ArgumentParser(description="sample argument parser")
    ap.add_argument("f", help="frame")
    ap.add_argument("out", help="output")
    ap.add_argument("seed", type=int, help="random seed")
    a = ap.parse_args(argv)
    f, w, h = open_gray(a.f)
    save_gray(lum_image(f, w, h, a.seed), w, h, a.out)


if __name__ == "__main__":
    main()
