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


PARENT_SCRIPT = textwrap.dedent("""
    import io, sys
    sys.path.insert(0, sys.argv[1])
    import bench
    sys.exit(bench.spawn_ranks(2, io.StringIO(), cmd=[sys.executable, sys.argv[2]], ndev=2))
""")

SLEEP_RANK = textwrap.dedent("""
    import os, sys, time
    d = os.path.dirname(os.path.abspath(__file__))
    with open(os.path.join(d, f"pid_{os.environ['RANK']}"), "w") as f:
        f.write(str(os.getpid()))
    time.sleep(600)
""")


def _alive(pid):
    try:
        os.kill(pid, 0)
    except ProcessLookupError:
        return False
    try:  # a zombie (exited, not yet reaped) counts as gone
        with open(f"/proc/{pid}/stat") as f:
            return f.read().split(")")[-1].split()[0] != "Z"
    except OSError:
        return False


@pytest.mark.parametrize("sig", ["SIGTERM", "SIGINT"])
def test_spawn_parent_signal_kills_every_rank(tmp_path, sig, monkeypatch):
    """The ranks run in sessions of their own, so a timeout's signal to the
    parent's process group never reaches them: the parent itself must kill
    every rank still running when it is told to stop."""
    import signal
    import subprocess
    import time
    monkeypatch.delenv("RTAMD_DIST_BACKEND", raising=False)
    (tmp_path / "parent.py").write_text(PARENT_SCRIPT)
    (tmp_path / "rank.py").write_text(SLEEP_RANK)
    p = subprocess.Popen([sys.executable, str(tmp_path / "parent.py"), ROOT, str(tmp_path / "rank.py")])
    try:
        t0 = time.monotonic()
        while not all((tmp_path / f"pid_{r}").exists() for r in range(2)):
            assert time.monotonic() - t0 < 120 and p.poll() is None, "ranks did not start"
            time.sleep(0.1)
        pids = [int((tmp_path / f"pid_{r}").read_text()) for r in range(2)]
        assert all(_alive(q) for q in pids)
        p.send_signal(getattr(signal, sig))
        assert p.wait(timeout=60) != 0
        t0 = time.monotonic()
        while any(_alive(q) for q in pids) and time.monotonic() - t0 < 20:
            time.sleep(0.1)
        assert not any(_alive(q) for q in pids), "a rank outlived its parent"
    finally:
        if p.poll() is None:
            p.kill()
