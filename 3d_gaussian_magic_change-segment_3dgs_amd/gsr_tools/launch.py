"""One process per GPU without an external launcher (bench.py --gpus N, N > 1).

The driver runs `python3 bench.py --gpus N ...` as a plain command.  When no
torch.distributed.run environment is present (WORLD_SIZE unset), the parent starts
the N rank processes itself -- each rank is the same script with RANK, LOCAL_RANK,
WORLD_SIZE, LOCAL_WORLD_SIZE, MASTER_ADDR=127.0.0.1 and MASTER_PORT set, exactly the
environment torch.distributed.run gives its workers -- waits for them and forwards
rank 0's stdout (the one JSON line) as its own.  Other ranks' stdout goes to stderr.

The parent never touches the GPU (no HIP call, no torch.cuda query that initialises
the runtime): it only spawns, waits and relays.  The ranks are child processes, not an
exec of the parent.  If one rank exits non-zero the others are given a grace period
(they are usually blocked in a collective with the dead rank) and then terminated by
their exact PIDs; the parent exits with the first failing rank's status.  A rank that
outlives a rank that finished normally by more than the straggler grace period (stuck in a
collective the finished rank never joins) is terminated too, and the job exits 124: a hang
ends the job instead of running into the driver's time limit.  Collectives themselves time
out after dist_timeout() seconds (bench.py passes it to init_process_group).
"""
import datetime
import os
import signal
import socket
import subprocess
import sys
import threading
import time

RANK_ENV = ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT",
            "GROUP_RANK", "ROLE_RANK", "ROLE_WORLD_SIZE")


STRAGGLER_STATUS = 124


def dist_timeout(env=None):
    """The process group's timeout (rendezvous and every collective): GSR_DIST_TIMEOUT_S,
    default 300 s -- long enough for a fresh box's first import of torch on every rank, short
    against the driver's limit."""
    env = os.environ if env is None else env
    return datetime.timedelta(seconds=float(env.get("GSR_DIST_TIMEOUT_S", "300")))


def free_port(host="127.0.0.1"):
    """A TCP port that is free on `host` right now (the rendezvous store binds it)."""
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind((host, 0))
        return s.getsockname()[1]


def rank_env(base, rank, world, port, addr="127.0.0.1"):
    """The environment of rank `rank` of a one-node job of `world` ranks (the variables
    torch.distributed.run sets for its workers; env:// rendezvous reads them)."""
    env = {k: v for k, v in base.items() if k not in RANK_ENV}
    env.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world), LOCAL_WORLD_SIZE=str(world),
               GROUP_RANK="0", ROLE_RANK=str(rank), ROLE_WORLD_SIZE=str(world),
               MASTER_ADDR=addr, MASTER_PORT=str(port))
    return env


def _pump(src, dst):
    """Copy a child's stdout to one of our file descriptors, line by line."""
    for line in iter(src.readline, b""):
        os.write(dst, line)
    src.close()


def spawn_ranks(world, argv, grace_s=30.0, poll_s=0.05, port=None, env=None, straggler_s=60.0):
    """Run `argv` (a full command line: [python, script, args...]) as `world` ranks of one
    node.  Rank 0's stdout becomes this process's stdout, every other rank's stdout goes to
    stderr; stderr is inherited.  Returns the job's exit status: 0 if every rank exited 0,
    else the first non-zero status seen (a rank killed by a signal reports 128 + signal), or
    STRAGGLER_STATUS when ranks had to be terminated straggler_s after a rank exited 0."""
    if world < 1:
        raise ValueError("world must be >= 1")
    base = dict(os.environ if env is None else env)
    port = port or free_port()
    procs, pumps = [], []
    sys.stdout.flush()
    sys.stderr.flush()
    try:
        for r in range(world):
            p = subprocess.Popen(argv, env=rank_env(base, r, world, port), stdout=subprocess.PIPE,
                                 stdin=subprocess.DEVNULL)
            procs.append(p)
            t = threading.Thread(target=_pump, args=(p.stdout, 1 if r == 0 else 2), daemon=True)
            t.start()
            pumps.append(t)
        status = 0
        failed_at = None
        first_ok = None  # (time, rank) of the first rank that exited 0
        alive = set(range(world))
        while alive:
            for r in sorted(alive):
                rc = procs[r].poll()
                if rc is None:
                    continue
                alive.discard(r)
                if rc != 0 and status == 0:
                    status = 128 - rc if rc < 0 else rc
                    failed_at = time.monotonic()
                    print(f"[launch] rank {r} exited with status {rc}; waiting {grace_s:g} s for the others",
                          file=sys.stderr, flush=True)
                elif rc == 0 and first_ok is None:
                    first_ok = (time.monotonic(), r)
            now = time.monotonic()
            stuck = alive and failed_at is None and first_ok is not None and now - first_ok[0] > straggler_s
            if stuck:
                print(f"[launch] rank(s) {sorted(alive)} still running {straggler_s:g} s after rank {first_ok[1]} "
                      f"exited 0 (a collective nobody else joins?)", file=sys.stderr, flush=True)
                status = STRAGGLER_STATUS
            if alive and (stuck or (failed_at is not None and now - failed_at > grace_s)):
                for r in sorted(alive):
                    print(f"[launch] terminating rank {r} (pid {procs[r].pid})", file=sys.stderr, flush=True)
                    _stop(procs[r])
                alive.clear()
            if alive:
                time.sleep(poll_s)
        return status
    except BaseException:
        for p in procs:
            if p.poll() is None:
                _stop(p)
        raise
    finally:
        for t in pumps:
            t.join(timeout=5.0)


def _stop(p, wait_s=10.0):
    """SIGTERM, then SIGKILL, to this exact child."""
    try:
        p.send_signal(signal.SIGTERM)
        p.wait(timeout=wait_s)
    except subprocess.TimeoutExpired:
        p.kill()
        p.wait()
    except ProcessLookupError:
        pass


def needs_launch(gpus, env=None):
    """True when `--gpus N` asks for N > 1 ranks and this process is not one of them
    (no WORLD_SIZE from torch.distributed.run or from spawn_ranks)."""
    env = os.environ if env is None else env
    return gpus > 1 and "WORLD_SIZE" not in env
