"""The C++ surface (include/rtamd.hpp) a reference user switches to.

CPU: the C header compiles as C11 and C++, the C++ wrapper compiles, and the
headless driver (apps/rt_render.cpp, written against rtamd.hpp only) is built.
GPU: the driver's frames reproduce SURVEY.md 8(c)'s golden hashes, i.e. the
reference's own render of the same scene through Renderer::draw.
"""
import json
import os
import subprocess

import pytest

import scenes as S
from conftest import ROOT
from rtamd import data

INCLUDE = os.path.join(ROOT, "include")
CLI = os.path.join(ROOT, "triangles-sdf-cpu-raytracing_amd", "lib", "rt_render")


def _compile(tmp_path, src, compiler, flags):
    f = tmp_path / src[0]
    f.write_text(src[1])
    r = subprocess.run([compiler, *flags, "-I", INCLUDE, "-fsyntax-only", str(f)],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr


def test_c_header_is_plain_c(tmp_path):
    _compile(tmp_path, ("a.c", '#include "rtamd.h"\nint main(void){return rt_abi_version();}\n'),
             "gcc", ["-std=c11", "-Wall", "-Wextra", "-Werror", "-pedantic"])


def test_cpp_wrapper_compiles(tmp_path):
    src = ('#include "rtamd.hpp"\n'
           "int main(){ rtamd::Renderer r; rtamd::FrameBuffer fb; fb.resize(4,4);\n"
           "  rtamd::SDFGrid g; (void)r; (void)g; return 0; }\n")
    _compile(tmp_path, ("a.cpp", src), "g++", ["-std=c++17", "-Wall", "-Wextra", "-Werror"])


def test_cli_built_and_fails_loudly_without_device(rt):
    assert os.path.exists(CLI), "rt_render not built (make in the package dir)"
    r = subprocess.run([CLI, "/nonexistent/model.obj"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 1 and "cannot open" in r.stderr
    if rt.device_count() == 0:
        r = subprocess.run([CLI, data.path("cube.obj"), "--size", "8", "8"], capture_output=True,
                           text=True, timeout=120)
        assert r.returncode == 1 and "rtamd:" in r.stderr


GOLDEN_CASES = [
    ("cube.obj", 256, 256, "primary"),
    ("cube.obj", 256, 256, "default"),
    ("stanford-bunny.obj", 1920, 1080, "default"),
    ("example_grid.grid", 1920, 1080, "primary"),
    ("sdf_6.octree", 3840, 2160, "default"),
]


@pytest.mark.gpu
@pytest.mark.parametrize("name,W,H,mode", GOLDEN_CASES)
def test_cli_reproduces_golden_hash(gpu, name, W, H, mode):
    args = [CLI, data.path(name), "--size", str(W), str(H), "--frames", "2"]
    if mode == "primary":
        args += ["--mode", "normal", "--plane", "0"]
    r = subprocess.run(args, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    out = json.loads(r.stdout)
    assert out["hash"] == S.GOLDEN[(name, W, H, mode)]
    key = (name, W, H, mode)
    if key in S.COVERAGE:
        assert out["covered"] == S.COVERAGE[key]


def test_cli_save_obj_matches_reference_writer(rt, ref, tmp_path):
    """rtamd::SaveMeshToObj through the C++ wrapper: the loaded, scaled mesh
    written byte for byte as cmesh4::SaveMeshToObj would (mesh.cpp:14-63).
    The file is written before the scene upload, so this runs without a GPU."""
    out = tmp_path / "cube_out.obj"
    subprocess.run([CLI, data.path("cube.obj"), "--size", "8", "8", "--save-obj", str(out)],
                   capture_output=True, text=True, timeout=120)
    v, i = ref.load_obj(data.path("cube.obj"))
    assert out.read_bytes() == ref.save_obj_text(v, i)


@pytest.mark.gpu
@pytest.mark.parametrize("name,W,H,mode", [GOLDEN_CASES[2], GOLDEN_CASES[4]])
@pytest.mark.parametrize("devices", ["0,0", "0"])
def test_cli_multi_device_reproduces_golden_hash(gpu, name, W, H, mode, devices):
    """The C++ Renderer over several devices of one process (Renderer::devices
    -> rt_multi_*, `rt_render --devices`): the same golden frames. On the
    one-GPU box "0,0" is two slots gathered by peer copies, "0" one slot
    gathered by RCCL."""
    args = [CLI, data.path(name), "--size", str(W), str(H), "--frames", "2", "--devices", devices]
    r = subprocess.run(args, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    # (RCCL prints its version banner to stdout when the communicator is made)
    out = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert out["devices"] == len(devices.split(","))
    assert out["hash"] == S.GOLDEN[(name, W, H, mode)]
