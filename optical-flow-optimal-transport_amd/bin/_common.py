"""Shared helpers of the dataset-prep tools (host code; PIL + numpy)."""
import os
import sys

import numpy as np
from PIL import Image

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def open_gray(path):
    """utils.openGrayscaleImage (utils.py:25-42): flattened grayscale in [0, 1], w, h."""
    f = np.asarray(Image.open(path).convert("L"))
    return f.flatten() / 255, f.shape[1], f.shape[0]


def save_gray(f, w, h, path):
    """np.uint8(255 * clip(f, 0, 1)) as an 8-bit grayscale PNG (the scripts' writer)."""
    Image.fromarray(np.uint8(255 * np.clip(f, 0, 1).reshape([h, w])), "L").save(path)
