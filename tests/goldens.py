"""Golden-vector access for the tests (data written by tools/make_goldens.py)."""
import json
import lzma
import os

import numpy as np

G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
with open(os.path.join(G, "goldens.json")) as _f:
    GOLD = json.load(_f)
SEED = GOLD["seed"]


def _un(b, dtype):
    return np.frombuffer(lzma.decompress(b.tobytes()), dtype)


def hits(name):
    d = np.load(os.path.join(G, f"hits_{name}.npz"), allow_pickle=False)
    H, W = (int(x) for x in d["shape"])
    return _un(d["face"], np.uint32).reshape(H, W), _un(d["tbits"], np.uint32).view(np.float32).reshape(H, W)


def render(name):
    d = np.load(os.path.join(G, f"render_{name}.npz"), allow_pickle=False)
    H, W = (int(x) for x in d["shape"])
    return (_un(d["rgb"], np.float32).reshape(H, W, 3), _un(d["fb"], np.uint32).reshape(H, W),
            _un(d["casts"], np.uint32).reshape(H, W))
