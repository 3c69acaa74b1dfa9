"""bench.py --gpus N without a launcher: spawn_ranks starts one rank process
per GPU with the torch.distributed.run environment, relays rank 0's JSON line
and exits with the worst rank's code; it never reports a line for a GPU count
it could not run (CPU: the rank command is a stand-in script)."""
import io
import json
import os
import sys
import textwrap

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402

RANK_SCRIPT = textwrap.dedent("""
    import json, os, sys, time
    r, n = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    mode = sys.argv[1]
    if mode == "fail" and r == 1:
        sys.exit(3)
    if mode == "hang" and r == 1:
        time.sleep(600)
    if mode == "hang" and r == 0:
        sys.exit(4)
    if r == 0:
        print("banner text")
        print(json.dumps({"rank": r, "world": n, "local": os.environ["LOCAL_RANK"],
                          "addr": os.environ["MASTER_ADDR"], "port": os.environ["MASTER_PORT"]}))
""")


def _run(tmp_path, mode, n=3, ndev=4, grace=60.0):
    script = tmp_path / "rank.py"
    script.write_text(RANK_SCRIPT)
    out = io.StringIO()
    rc = bench.spawn_ranks(n, out, grace_s=grace, cmd=[sys.executable, str(script), mode], ndev=ndev)
    return rc, out.getvalue()


def test_spawn_relays_rank0_line(tmp_path):
    rc, out = _run(tmp_path, "ok")
    assert rc == 0
    d = json.loads(out.strip())
    assert d["rank"] == 0 and d["world"] == 3 and d["local"] == "0" and d["addr"] == "127.0.0.1"


def test_spawn_failing_rank_reports_nothing(tmp_path):
    rc, out = _run(tmp_path, "fail")
    assert rc == 3 and out == ""


def test_spawn_kills_ranks_left_waiting(tmp_path):
    rc, out = _run(tmp_path, "hang", n=2, grace=1.0)
    assert rc == 9 and out == ""  # rank 0 exited 4, rank 1 killed (SIGKILL -> -9)


@pytest.mark.parametrize("ndev", [0, 2])
def test_spawn_refuses_too_few_gpus(tmp_path, ndev, monkeypatch):
    monkeypatch.delenv("RTAMD_DIST_BACKEND", raising=False)
    rc, out = _run(tmp_path, "ok", n=3, ndev=ndev)
    assert rc == 2 and out == ""


def test_gloo_ranks_may_share_gpus(tmp_path, monkeypatch):
    monkeypatch.setenv("RTAMD_DIST_BACKEND", "gloo")
    rc, out = _run(tmp_path, "ok", n=2, ndev=1)
    assert rc == 0 and json.loads(out)["world"] == 2
