"""bench.py's own rank launcher (gsr_tools/launch.py; VERDICT r4 Next #1): `python3 bench.py
--gpus N` without torch.distributed.run starts its N ranks itself.  These tests run the
launcher over gloo ranks on the CPU: every rank sees the torch.distributed.run environment
(env:// rendezvous on 127.0.0.1), only rank 0's stdout reaches the parent's stdout, and a
failing rank fails the job (the survivors, stuck in a collective, are terminated)."""
import json
import os
import subprocess
import sys
import textwrap

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "3d_gaussian_magic_change-segment_3dgs_amd")

CHILD = textwrap.dedent("""
    import json, os, sys, time
    import torch, torch.distributed as dist
    sys.path.insert(0, os.environ["PKG"])
    from gsr_tools.launch import dist_timeout
    dist.init_process_group("gloo", timeout=dist_timeout())
    r, w = dist.get_rank(), dist.get_world_size()
    if os.environ.get("SLEEP_RANK") == str(r):
        time.sleep(600)                     # never joins the collective below

    assert os.environ["LOCAL_RANK"] == str(r) and os.environ["MASTER_ADDR"] == "127.0.0.1"
    fail = os.environ.get("FAIL_RANK")
    if fail is not None and int(fail) == r:
        sys.exit(3)
    t = torch.tensor([float(r + 1)])
    dist.all_reduce(t)
    print(f"rank {r} says hello")          # only rank 0's stdout may reach the parent's
    if r == 0:
        print(json.dumps({"world": w, "sum": t.item(), "launcher": os.environ.get("GSR_LAUNCHER")}))
    dist.barrier()
    dist.destroy_process_group()
    if os.environ.get("LINGER_RANK") == str(r):
        time.sleep(600)                     # finishes its work, then never exits
""")

PARENT = textwrap.dedent("""
    import os, sys
    sys.path.insert(0, {pkg!r})
    from gsr_tools import launch
    assert launch.needs_launch(int(sys.argv[1]))
    sys.exit(launch.spawn_ranks(int(sys.argv[1]), [sys.executable, sys.argv[2]], grace_s=3.0,
                                straggler_s=float(os.environ.get("STRAGGLER_S", "60")),
                                env=dict(os.environ, GSR_LAUNCHER="test")))
""")


def _run(tmp_path, world, extra_env=None):
    child = tmp_path / "child.py"
    child.write_text(CHILD)
    parent = tmp_path / "parent.py"
    parent.write_text(PARENT.format(pkg=PKG))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["PKG"] = PKG
    env.update(extra_env or {})
    return subprocess.run([sys.executable, str(parent), str(world), str(child)], env=env, capture_output=True,
                          text=True, timeout=180)


@pytest.mark.parametrize("world", [2, 3])
def test_spawn_ranks_relays_rank0_stdout(tmp_path, world):
    p = _run(tmp_path, world)
    assert p.returncode == 0, p.stderr
    # (gloo announces its connections on stdout; bench.py points fd 1 at stderr for that reason)
    lines = [x for x in p.stdout.strip().splitlines() if not x.startswith("[Gloo]")]
    assert lines[0] == "rank 0 says hello" and len(lines) == 2, p.stdout
    line = json.loads(lines[1])
    assert line == {"world": world, "sum": world * (world + 1) / 2, "launcher": "test"}
    for r in range(1, world):
        assert f"rank {r} says hello" in p.stderr


def test_spawn_ranks_propagates_failure(tmp_path):
    p = _run(tmp_path, 2, {"FAIL_RANK": "1"})
    assert p.returncode == 3, (p.returncode, p.stderr[-2000:])
    assert "rank 1 exited with status 3" in p.stderr


def test_rank_stuck_in_collective_fails_fast(tmp_path):
    """VERDICT r5 Next #7: one rank sleeps instead of joining a collective.  The others' gloo
    all_reduce times out after GSR_DIST_TIMEOUT_S (bench.py passes the same dist_timeout() to
    init_process_group), they exit non-zero, and the launcher terminates the sleeper after its
    grace period: the job ends non-zero within the timeout, not at the driver's limit."""
    import time
    t0 = time.monotonic()
    p = _run(tmp_path, 2, {"SLEEP_RANK": "1", "GSR_DIST_TIMEOUT_S": "5"})
    took = time.monotonic() - t0
    assert p.returncode != 0, p.stderr[-2000:]
    assert "terminating rank 1" in p.stderr
    assert took < 60, took


def test_rank_outliving_the_job_is_terminated(tmp_path):
    """A rank that keeps running long after another exited 0 (straggler grace) is terminated
    and the job exits with launch.STRAGGLER_STATUS."""
    sys.path.insert(0, PKG)
    from gsr_tools import launch
    p = _run(tmp_path, 2, {"LINGER_RANK": "1", "STRAGGLER_S": "3"})
    assert p.returncode == launch.STRAGGLER_STATUS, (p.returncode, p.stderr[-2000:])
    assert "still running" in p.stderr and "terminating rank 1" in p.stderr


def test_needs_launch():
    sys.path.insert(0, PKG)
    from gsr_tools import launch
    assert launch.needs_launch(2, {}) and not launch.needs_launch(1, {})
    assert not launch.needs_launch(8, {"WORLD_SIZE": "8"})
    env = launch.rank_env({"RANK": "5", "X": "1"}, 1, 4, 1234)
    assert env["RANK"] == "1" and env["WORLD_SIZE"] == "4" and env["MASTER_PORT"] == "1234" and env["X"] == "1"


def test_bench_launches_its_own_ranks():
    """bench.py's `--gpus N` path goes through the launcher before anything touches the GPU
    (the exit that demanded torch.distributed.run is gone)."""
    src = open(os.path.join(ROOT, "bench.py")).read()
    assert "must be launched with torch.distributed.run" not in src
    i_launch = src.index("launch.spawn_ranks(")
    assert i_launch < src.index("torch.cuda.set_device(")
