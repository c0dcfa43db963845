"""Start the ranks of a one-node data-parallel run from one command.

The reference starts every device's trainer from a single ``python main.py …``: one thread per
GPU (main.py:289-297). Here a rank is a process (one per GPU, torch.distributed over RCCL), so
``python bench.py --gpus N`` without an external launcher starts its N rank processes itself:
each child gets the environment torchrun would give it (RANK, LOCAL_RANK, WORLD_SIZE,
LOCAL_WORLD_SIZE, MASTER_ADDR = 127.0.0.1, MASTER_PORT) and re-runs the same script with the
same arguments. The parent never touches the GPU (no HIP call, no ``torch.cuda`` query): it only
spawns, waits and forwards exit codes. If any rank fails, the others are stopped (by their own
PIDs) and the parent exits non-zero.
"""
from __future__ import annotations

import os
import signal
import socket
import subprocess
import sys
import time
from typing import List, Optional, Sequence

LAUNCHED_ENV = "GNN_LAUNCHED_BY"


def free_port(addr: str = "127.0.0.1") -> int:
    """A TCP port nothing listens on right now (the rendezvous store binds it next)."""
    s = socket.socket()
    try:
        s.bind((addr, 0))
        return int(s.getsockname()[1])
    finally:
        s.close()


def needs_launch(nranks: int, environ=None) -> bool:
    """True when `nranks` > 1 ranks are asked for and no launcher (torchrun or this module) has
    set up the rank environment."""
    env = os.environ if environ is None else environ
    return nranks > 1 and "WORLD_SIZE" not in env and LAUNCHED_ENV not in env


def rank_env(rank: int, world: int, port: int, base=None) -> dict:
    env = dict(os.environ if base is None else base)
    env.update({"RANK": str(rank), "LOCAL_RANK": str(rank), "WORLD_SIZE": str(world),
                "LOCAL_WORLD_SIZE": str(world), "GROUP_RANK": "0", "MASTER_ADDR": "127.0.0.1",
                "MASTER_PORT": str(port), LAUNCHED_ENV: str(os.getpid())})
    # the multi-process GPU runs on this pool need dmabuf IPC (no legacy IPC mode)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return env


def _stop(procs: Sequence[subprocess.Popen], grace: float) -> None:
    for p in procs:
        if p.poll() is None:
            try:
                p.send_signal(signal.SIGTERM)
            except ProcessLookupError:
                pass
    end = time.monotonic() + grace
    for p in procs:
        while p.poll() is None and time.monotonic() < end:
            time.sleep(0.05)
        if p.poll() is None:
            try:
                p.kill()
            except ProcessLookupError:
                pass
            p.wait()


def launch(argv: List[str], nranks: int, port: Optional[int] = None, poll_s: float = 0.1,
           grace_s: float = 10.0, quiet_ranks: bool = True) -> int:
    """Run `argv` (a full command, e.g. [sys.executable, 'bench.py', ...]) as `nranks` rank
    processes on this node and wait for them. Rank 0 inherits stdout (its one JSON line is the
    run's output); the other ranks' stdout goes to stderr. Returns 0 if every rank exited 0,
    otherwise the first failing rank's exit code (a signal death maps to 128 + signal); the
    surviving ranks are stopped as soon as one fails, so a rank blocked in a collective with
    the dead one does not hang the run."""
    if nranks < 1:
        raise ValueError(f"nranks must be >= 1, got {nranks}")
    port = port or free_port()
    procs: List[subprocess.Popen] = []

    def on_signal(signum, frame):  # a launcher stopped from outside takes its ranks with it
        _stop(procs, grace_s)
        sys.exit(128 + signum)

    old_handlers = {sig: signal.signal(sig, on_signal) for sig in (signal.SIGTERM, signal.SIGHUP)}
    try:
        for r in range(nranks):
            out = None if r == 0 or not quiet_ranks else sys.stderr
            procs.append(subprocess.Popen(argv, env=rank_env(r, nranks, port), stdout=out))
        failed = None
        while True:
            codes = [p.poll() for p in procs]
            bad = [(r, c) for r, c in enumerate(codes) if c not in (None, 0)]
            if bad:
                failed = bad[0]
                break
            if all(c == 0 for c in codes):
                return 0
            time.sleep(poll_s)
        r, c = failed
        print(f"[launch] rank {r} exited with {c}; stopping the other ranks", file=sys.stderr, flush=True)
        _stop(procs, grace_s)
        return c if c > 0 else 128 + (-c)
    except BaseException:
        _stop(procs, grace_s)
        raise
    finally:
        for sig, h in old_handlers.items():
            signal.signal(sig, h)


def relaunch_self(nranks: int) -> int:
    """Re-run this Python program (same script, same arguments) as `nranks` rank processes."""
    return launch([sys.executable, "-u", os.path.abspath(sys.argv[0]), *sys.argv[1:]], nranks)
