"""Input files of the benchmark configs.

The reference's shipped resources (resources/*.obj, *.grid, *.octree) are kept
gzip-compressed under <repo>/data/ and unpacked on first use into
<repo>/data/_unpacked/ (git-ignored). Nothing here reads /root/reference.
"""
from __future__ import annotations

import gzip
import os
import shutil

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
DATA = os.path.join(REPO, "data")
UNPACKED = os.path.join(DATA, "_unpacked")

FILES = ("cube.obj", "stanford-bunny.obj", "spot.obj", "example_grid.grid", "sdf_5.octree",
         "sdf_6.octree")


def path(name: str) -> str:
    """Absolute path of an unpacked input file (e.g. 'stanford-bunny.obj')."""
    out = os.path.join(UNPACKED, name)
    if os.path.exists(out):
        return out
    src = os.path.join(DATA, name + ".gz")
    if not os.path.exists(src):
        raise FileNotFoundError(f"no data file {name} (looked for {src})")
    os.makedirs(UNPACKED, exist_ok=True)
    tmp = out + f".tmp{os.getpid()}"
    with gzip.open(src, "rb") as fi, open(tmp, "wb") as fo:
        shutil.copyfileobj(fi, fo)
    os.replace(tmp, out)
    return out
