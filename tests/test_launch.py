"""CPU: `python bench.py --gpus N` starts its own N rank processes (gnn_amd.launch).

The reference starts every device's trainer from one command (main.py:289-297); here each rank
is a process, so without an external launcher the bench re-runs itself as N ranks with the
environment torchrun would give them. Covered: the rank environment and the rendezvous (world 2
over gloo: an all_reduce across the launched ranks), rank 0's stdout as the run's output, exit
codes (all 0 -> 0; a failing rank -> its code, the blocked survivors stopped), and the decision
to launch (not under torchrun, not for N = 1, not in --cpu mode).
"""
import json
import os
import subprocess
import sys
import textwrap
import time

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

RANK_SCRIPT = textwrap.dedent("""
    import json, os, sys, time
    import torch, torch.distributed as dist
    dist.init_process_group("gloo")
    r, w = dist.get_rank(), dist.get_world_size()
    t = torch.tensor([float(r + 1)])
    dist.all_reduce(t)
    mode = sys.argv[1]
    if mode == "fail" and r == 1:
        sys.exit(7)
    if mode == "fail":
        dist.barrier()  # never completes: rank 1 is gone; the launcher must stop this rank
        time.sleep(600)
    if r == 0:
        print(json.dumps({"world": w, "sum": t.item(), "env_world": int(os.environ["WORLD_SIZE"]),
                          "local": int(os.environ["LOCAL_RANK"]), "addr": os.environ["MASTER_ADDR"]}))
    else:
        print("rank", r, "stdout goes to stderr")
    dist.destroy_process_group()
""")


def _driver(tmp_path, mode, n=2):
    script = tmp_path / "rank.py"
    script.write_text(RANK_SCRIPT)
    code = ("import sys; sys.path.insert(0, %r); from gnn_amd import launch; "
            "sys.exit(launch.launch([sys.executable, %r, %r], %d, grace_s=3.0))" % (REPO, str(script), mode, n))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "GNN_LAUNCHED_BY")}
    t0 = time.monotonic()
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=180, env=env)
    return r, time.monotonic() - t0


def test_launch_world2_ok(tmp_path):
    r, _ = _driver(tmp_path, "ok")
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.strip() and not l.startswith("[Gloo]")]
    assert len(lines) == 1, r.stdout  # rank 0's line only: the other rank's stdout went to stderr
    out = json.loads(lines[0])
    assert out == {"world": 2, "sum": 3.0, "env_world": 2, "local": 0, "addr": "127.0.0.1"}
    assert "stdout goes to stderr" in r.stderr


STALL_SCRIPT = textwrap.dedent("""
    import os, sys, time
    sys.path.insert(0, os.environ["GNN_TEST_REPO"])
    import torch, torch.distributed as dist
    from gnn_amd.train import init_distributed, new_gloo_group
    rank, world, _ = init_distributed("gloo")
    side = new_gloo_group() if sys.argv[1] == "side" else None
    t = torch.ones(4)
    dist.all_reduce(t, group=side)  # both ranks: the groups work
    if rank == 1:
        time.sleep(600)  # skips the next collective, alive (a stalled rank, not a dead one)
    dist.all_reduce(t, group=side)  # rank 0 waits for rank 1: must fail after the timeout
    print("unreachable", flush=True)
""")


@pytest.mark.parametrize("group", ["main", "side"])
def test_stalled_collective_fails_the_run_within_the_timeout(tmp_path, group):
    """A rank that never reaches a collective must end the run non-zero within the collective
    timeout (GNN_DIST_TIMEOUT_S) plus the launcher's grace, naming the rank and the call — on the
    default group and on a gloo side group alike (the reference's Barrier waits forever,
    main.py:158,214; torch's defaults are 10 / 30 min)."""
    script = tmp_path / "stall.py"
    script.write_text(STALL_SCRIPT)
    code = ("import sys; sys.path.insert(0, %r); from gnn_amd import launch; "
            "sys.exit(launch.launch([sys.executable, %r, %r], 2, grace_s=3.0))" % (REPO, str(script), group))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "GNN_LAUNCHED_BY")}
    env.update(GNN_DIST_TIMEOUT_S="4", GNN_TEST_REPO=REPO)
    t0 = time.monotonic()
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=170, env=env)
    dt = time.monotonic() - t0
    assert r.returncode not in (0, None), r.stderr[-3000:]
    assert "unreachable" not in r.stdout
    assert "rank 0 exited with" in r.stderr, r.stderr[-3000:]
    assert "all_reduce" in r.stderr  # the traceback names the call that timed out
    assert dt < 4 + 3 + 60, dt  # timeout + grace + two interpreters' start-up


def test_collective_timeout_env(monkeypatch):
    from gnn_amd import train

    monkeypatch.delenv("GNN_DIST_TIMEOUT_S", raising=False)
    assert train.collective_timeout().total_seconds() == train.DEFAULT_TIMEOUT_S <= 180
    monkeypatch.setenv("GNN_DIST_TIMEOUT_S", "7.5")
    assert train.collective_timeout().total_seconds() == 7.5
    monkeypatch.setenv("GNN_DIST_TIMEOUT_S", "0")
    with pytest.raises(ValueError):
        train.collective_timeout()


def test_launch_failing_rank_stops_the_others(tmp_path):
    r, dt = _driver(tmp_path, "fail")
    assert r.returncode == 7, (r.returncode, r.stderr[-2000:])
    assert "rank 1 exited with 7" in r.stderr
    assert dt < 120  # rank 0 (blocked in a barrier) was stopped, not waited for


def test_needs_launch():
    from gnn_amd import launch

    assert launch.needs_launch(2, {})
    assert not launch.needs_launch(1, {})
    assert not launch.needs_launch(4, {"WORLD_SIZE": "4"})  # torchrun already started the ranks
    assert not launch.needs_launch(2, {launch.LAUNCHED_ENV: "123"})  # a launched child never re-launches
    env = launch.rank_env(1, 4, 29999, base={})
    assert (env["RANK"], env["LOCAL_RANK"], env["WORLD_SIZE"], env["MASTER_ADDR"], env["MASTER_PORT"]) == \
        ("1", "1", "4", "127.0.0.1", "29999")
    assert env["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"


def test_bench_relaunches_itself(monkeypatch):
    """bench.main() with --gpus 2 and no launcher environment hands over to the launcher before
    it builds the graph or touches the GPU."""
    sys.path.insert(0, REPO)
    import bench
    from gnn_amd import launch

    calls = []
    monkeypatch.setattr(launch, "relaunch_self", lambda n: calls.append(n) or 0)
    monkeypatch.setattr(bench.graphs, "make_dataset", lambda *a, **k: pytest.fail("built the graph first"))
    for k in ("WORLD_SIZE", launch.LAUNCHED_ENV):
        monkeypatch.delenv(k, raising=False)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "2", "--steps", "3"])
    with pytest.raises(SystemExit) as e:
        bench.main()
    assert e.value.code == 0 and calls == [2]


def test_launcher_stopped_from_outside_stops_its_ranks(tmp_path):
    """SIGTERM to the launcher (a driver's time limit) ends the ranks too, not just the parent."""
    import signal

    script = tmp_path / "rank.py"
    script.write_text("import os, sys, time\nopen(sys.argv[1] + '.' + os.environ['RANK'], 'w').write(str(os.getpid()))\n"
                      "time.sleep(600)\n")
    code = ("import sys; sys.path.insert(0, %r); from gnn_amd import launch; "
            "sys.exit(launch.launch([sys.executable, %r, %r], 2, grace_s=3.0))" % (REPO, str(script), str(tmp_path / "pid")))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "GNN_LAUNCHED_BY")}
    p = subprocess.Popen([sys.executable, "-c", code], env=env)
    pids = []
    for _ in range(200):
        if all(os.path.exists(tmp_path / f"pid.{r}") for r in range(2)):
            try:
                pids = [int((tmp_path / f"pid.{r}").read_text()) for r in range(2)]
                break
            except ValueError:
                pass
        time.sleep(0.1)
    assert len(pids) == 2
    p.send_signal(signal.SIGTERM)
    assert p.wait(timeout=60) == 128 + signal.SIGTERM
    for pid in pids:
        for _ in range(100):
            try:
                os.kill(pid, 0)
            except ProcessLookupError:
                break
            time.sleep(0.1)
        else:
            raise AssertionError(f"rank process {pid} survived its launcher")
