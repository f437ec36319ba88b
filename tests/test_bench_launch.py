"""bench.py's launch contract without a GPU: ``--gpus N`` alone starts N ranks itself
(spawn_ranks: fresh processes with torch.distributed.run's environment; the parent
never touches the GPU), a launcher's WORLD_SIZE must equal --gpus, and the ranks it
starts can form a process group (gloo, 2 ranks on CPU) -- DESIGN.md section 7."""

import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def test_launch_mode():
    assert bench.launch_mode(1, {}) == "single"
    assert bench.launch_mode(8, {}) == "spawn"
    assert bench.launch_mode(2, {"WORLD_SIZE": "2"}) == "rank"
    assert bench.launch_mode(1, {"WORLD_SIZE": "1", "LOCAL_RANK": "0"}) == "rank"
    with pytest.raises(SystemExit, match="WORLD_SIZE=2 but --gpus 1"):
        bench.launch_mode(1, {"WORLD_SIZE": "2"})
    with pytest.raises(SystemExit, match="WORLD_SIZE=4 but --gpus 8"):
        bench.launch_mode(8, {"WORLD_SIZE": "4"})
    with pytest.raises(SystemExit):
        bench.launch_mode(0, {})


def test_mismatched_world_size_exits_nonzero():
    env = dict(os.environ, WORLD_SIZE="3", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"],
                       env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode != 0
    assert "WORLD_SIZE=3 but --gpus 2" in r.stderr


_RANK_PROG = r"""
import os, sys, torch, torch.distributed as dist
dist.init_process_group("gloo")
r, n = dist.get_rank(), dist.get_world_size()
assert r == int(os.environ["RANK"]) == int(os.environ["LOCAL_RANK"])
assert os.environ["MASTER_ADDR"] == "127.0.0.1"
t = torch.tensor([float(r + 1)])
dist.all_reduce(t)
with open(os.path.join(sys.argv[1], f"rank{r}"), "w") as f:
    f.write(f"{n} {t.item()}")
dist.destroy_process_group()
sys.exit(int(os.environ.get("FAIL_RANK", "-1")) == r and 3 or 0)
"""


def test_spawn_ranks_forms_a_process_group(tmp_path):
    prog = [sys.executable, "-c", _RANK_PROG, str(tmp_path)]
    assert bench.spawn_ranks(2, [], program=prog) == 0
    for r in range(2):
        assert (tmp_path / f"rank{r}").read_text() == "2 3.0"


def test_spawn_ranks_reports_a_failed_rank(tmp_path):
    prog = [sys.executable, "-c", _RANK_PROG, str(tmp_path)]
    env = dict(os.environ, FAIL_RANK="1")
    assert bench.spawn_ranks(2, [], env=env, program=prog) == 3


_PARENT_PROG = r"""
import sys
sys.path.insert(0, sys.argv[1])
import bench
child = [sys.executable, "-c",
         "import os, sys, time; open(os.path.join(sys.argv[1], 'pid' + os.environ['RANK']), 'w')"
         ".write(str(os.getpid())); time.sleep(600)", sys.argv[2]]
sys.exit(bench.spawn_ranks(2, [], program=child))
"""


def test_spawn_ranks_terminated_parent_stops_its_ranks(tmp_path):
    """A SIGTERM to the spawning parent (a driver timeout) ends its ranks too: none
    keeps holding a GPU or waits in a collective after the parent is gone."""
    import signal
    import time
    parent = subprocess.Popen([sys.executable, "-c", _PARENT_PROG, ROOT, str(tmp_path)])
    pids = []
    deadline = time.time() + 120
    while time.time() < deadline and len(pids) < 2:
        pids = [int(p.read_text()) for p in tmp_path.glob("pid*") if p.read_text()]
        time.sleep(0.1)
    assert len(pids) == 2
    parent.send_signal(signal.SIGTERM)
    assert parent.wait(timeout=60) == 128 + signal.SIGTERM
    for pid in pids:
        for _ in range(100):
            try:
                os.kill(pid, 0)
            except ProcessLookupError:
                break
            time.sleep(0.1)
        else:
            raise AssertionError(f"rank {pid} outlived its parent")
