"""Scene assets for the benchmark configs.

Dragon.obj is absent from the reference (``.MISSING_LARGE_BLOBS:1``); the benchmark uses the
survey's 139,128-triangle surrogate, stored losslessly in ``tests/golden/dragon_surrogate.npz``
(encoder: ``tools/encode_surrogate.py``). ``dragon_obj_path()`` regenerates the byte-identical
OBJ text (sha256-checked) so the product loader parses exactly what the reference parsed.
A real Dragon.obj can be dropped in with ``ATRAY_DRAGON_OBJ=/path/Dragon.obj``.
"""
from __future__ import annotations

import hashlib
import lzma
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SURROGATE_NPZ = os.path.join(ROOT, "tests", "golden", "dragon_surrogate.npz")
ASSET_DIR = os.path.join(ROOT, "tests", "golden", "assets")
CACHE_DIR = os.path.join(ROOT, "build", "assets")

# app.cpp:73 and the survey's probe framings
CENTERS = {
    "Cube": (-0.256, 0.22, -3.56),
    "Monkey": (-0.12, 0.89, -2.23),
    "Deer": (0.0, 1.0, -6.0),
    "Dragon": (0.0, -15.0, -38.0),
}


def _fmt6(mu: np.ndarray, negz: np.ndarray) -> list:
    """Fixed-point micro-units -> '%.6f' text, keeping '-0.000000' where the source had it."""
    out = []
    for m, z in zip(mu.tolist(), negz.tolist()):
        s = "-" if (m < 0 or z) else ""
        a = abs(m)
        out.append(f"{s}{a // 1000000}.{a % 1000000:06d}")
    return out


def pack(a: np.ndarray) -> np.ndarray:
    return np.frombuffer(lzma.compress(np.ascontiguousarray(a).tobytes(), preset=9), np.uint8)


def _unpack(b: np.ndarray, dtype, shape) -> np.ndarray:
    return np.frombuffer(lzma.decompress(b.tobytes()), dtype).reshape(shape)


def predict_normals_mu(vid: np.ndarray, U: np.ndarray) -> np.ndarray:
    """Flat face normals normalize(cross(b-a, c-a)) in float64 from the printed vertices, in
    micro-units; the fixture stores only the (small) residual to the surrogate's vn lines."""
    t = vid.reshape(-1, 3)
    P = U.astype(np.float64) / 1e6
    a, b, c = P[t[:, 0]], P[t[:, 1]], P[t[:, 2]]
    e1, e2 = b - a, c - a
    n = np.stack([e1[:, 1] * e2[:, 2] - e1[:, 2] * e2[:, 1],
                  e1[:, 2] * e2[:, 0] - e1[:, 0] * e2[:, 2],
                  e1[:, 0] * e2[:, 1] - e1[:, 1] * e2[:, 0]], 1)
    n = n / np.sqrt((n * n).sum(1, keepdims=True))
    return np.rint(n * 1e6).astype(np.int64)


def decode_surrogate_npz(path: str = SURROGATE_NPZ) -> bytes:
    d = np.load(path, allow_pickle=False)
    nu, nf = (int(x) for x in d["shape"])
    vid = np.cumsum(_unpack(d["vid"], np.int32, (3 * nf,)).astype(np.int64)).astype(np.int32)
    U = _unpack(d["U"], np.int32, (nu, 3))
    Uz = _unpack(d["Uz"], np.bool_, (nu, 3))
    N = (predict_normals_mu(vid, U) + _unpack(d["R"], np.int32, (nf, 3))).astype(np.int64)
    Nz = _unpack(d["Nz"], np.bool_, (nf, 3))
    vtxt = ["v " + " ".join(_fmt6(U[i], Uz[i])) for i in range(len(U))]
    parts = []
    for i in range(nf):
        nl = "vn " + " ".join(_fmt6(N[i], Nz[i]))
        parts.append(vtxt[vid[3 * i]]); parts.append(vtxt[vid[3 * i + 1]]); parts.append(vtxt[vid[3 * i + 2]])
        parts.append(nl); parts.append(nl); parts.append(nl)
    for i in range(nf):
        a = 3 * i + 1
        parts.append(f"f {a}//{a} {a+1}//{a+1} {a+2}//{a+2}")
    data = ("\n".join(parts) + "\n").encode()
    want = bytes(d["sha256"].tolist())
    if hashlib.sha256(data).digest() != want:
        raise RuntimeError("surrogate decode mismatch")
    return data


def dragon_obj_path() -> str:
    """Path of Dragon.obj for the benchmark: $ATRAY_DRAGON_OBJ, else the decoded surrogate."""
    env = os.environ.get("ATRAY_DRAGON_OBJ")
    if env:
        return env
    out = os.path.join(CACHE_DIR, "DragonSurrogate.obj")
    if not os.path.exists(out):
        os.makedirs(CACHE_DIR, exist_ok=True)
        tmp = out + f".tmp{os.getpid()}"
        with open(tmp, "wb") as f:
            f.write(decode_surrogate_npz())
        os.replace(tmp, out)
    return out


def asset_path(name: str) -> str:
    """Reference assets (Cube/Monkey/Deer/Simple) copied as fixtures into tests/golden/assets."""
    if name == "Dragon":
        return dragon_obj_path()
    return os.path.join(ASSET_DIR, f"{name}.obj")
