"""Generate the small golden frame fixtures in tests/golden/frames.npz.

The frames are rendered by the ORACLE (oracle/cpuref.cpp), whose output for the
reference's default camera reproduces the golden frame hashes that the survey
obtained from the reference's own unmodified translation units (SURVEY.md 8(c);
checked by tests/test_oracle.py). Inputs: the reference's shipped resources
(data/*.gz). Run from the repo root:  python tests/golden/make_golden.py
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle"),
                os.path.join(ROOT, "triangles-sdf-cpu-raytracing_amd")]

import cpuref  # noqa: E402
import scenes as S  # noqa: E402

CASES = [
    # (input, W, H, mode, camera position)
    ("cube.obj", 128, 128, "primary", (0.0, 0.0, 2.5)),
    ("cube.obj", 128, 128, "default", (1.2, 0.8, 2.0)),
    ("stanford-bunny.obj", 192, 108, "primary", (0.0, 0.0, 2.5)),
    ("stanford-bunny.obj", 192, 108, "default", (0.0, 0.0, 2.5)),
    ("stanford-bunny.obj", 192, 108, "color_plane", (1.5, 0.5, 2.0)),
    ("spot.obj", 160, 120, "default", (0.0, 0.5, 2.5)),
    ("example_grid.grid", 192, 108, "primary", (0.0, 0.0, 2.5)),
    ("example_grid.grid", 192, 108, "default", (0.9, 0.5, 2.3)),
    ("sdf_5.octree", 160, 120, "default", (0.0, 0.0, 2.5)),
    ("sdf_6.octree", 192, 108, "primary", (0.0, 0.0, 2.5)),
    ("sdf_6.octree", 192, 108, "default", (-1.1, 0.5, 2.2)),
]


def key(c):
    name, W, H, mode, pos = c
    return f"{name}|{W}x{H}|{mode}|{pos[0]:g},{pos[1]:g},{pos[2]:g}"


def main():
    arrays, index = {}, []
    for i, c in enumerate(CASES):
        name, W, H, mode, pos = c
        col, t = S.ref_frame(name, W, H, mode, pos)
        arrays[f"c{i}"] = col
        arrays[f"t{i}"] = t
        index.append({"case": key(c), "color": f"c{i}", "t": f"t{i}",
                      "fnv1a64": cpuref.fnv1a64_words(col), "coverage": int(np.isfinite(t).sum())})
    np.savez_compressed(os.path.join(HERE, "frames.npz"), **arrays)
    with open(os.path.join(HERE, "frames.json"), "w") as f:
        json.dump(index, f, indent=1)
    print(f"wrote {len(CASES)} frames")


if __name__ == "__main__":
    main()
