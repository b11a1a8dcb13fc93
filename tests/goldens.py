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


def frame_digest(a):
    """Digest of a whole frame's array: sha256 of its little-endian bytes, first 16 hex digits
    (tests/golden/fullframe.json, tools/make_fullframe_goldens.py)."""
    import hashlib
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()[:16]


def row_crcs(frames):
    """One CRC-32 per image row over that row's fb, ray_casts, face, t and RGB words, as one hex
    string (8 digits per row, row 0 first): localises a whole-frame digest mismatch."""
    import zlib
    H = frames["fb"].shape[0]
    keys = ("fb", "casts", "face", "t", "rgb")
    out = []
    for y in range(H):
        c = 0
        for k in keys:
            c = zlib.crc32(np.ascontiguousarray(frames[k][y]).tobytes(), c)
        out.append(f"{c:08x}")
    return "".join(out)


def fullframe():
    with open(os.path.join(G, "fullframe.json")) as f:
        return json.load(f)


def render(name):
    d = np.load(os.path.join(G, f"render_{name}.npz"), allow_pickle=False)
    H, W = (int(x) for x in d["shape"])
    return (_un(d["rgb"], np.float32).reshape(H, W, 3), _un(d["fb"], np.uint32).reshape(H, W),
            _un(d["casts"], np.uint32).reshape(H, W))
