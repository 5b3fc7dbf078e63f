"""CPU: bench.py's `--gpus N` is authoritative.  `python bench.py --gpus N`
(the driver's BENCH command shape) starts N ranks itself, as a
torch.distributed.run child, and relays rank 0's one line; a launcher whose
world size disagrees with --gpus is refused before torch is imported, so no
line can claim a GPU count it did not run on (config 4's
8-GPU split; chunk.c:20-21 keeps chunks independent).  The GPU side of the
same path is tests/test_gpu_dist.py."""
import importlib.util
import json
import os
import subprocess
import sys

import pytest

from conftest import REPO

BENCH = os.path.join(REPO, "bench.py")


def _bench():
    spec = importlib.util.spec_from_file_location("bench_launch_mod", BENCH)
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def test_rank_plan_table():
    b = _bench()
    assert b.rank_plan(1, {}) == ("single", None)
    assert b.rank_plan(8, {}) == ("spawn", None)
    assert b.rank_plan(8, {"WORLD_SIZE": ""}) == ("spawn", None)
    assert b.rank_plan(2, {"WORLD_SIZE": "2"}) == ("ranks", None)
    assert b.rank_plan(1, {"WORLD_SIZE": "1"}) == ("ranks", None)
    for gpus, env in ((4, {"WORLD_SIZE": "2"}), (2, {"WORLD_SIZE": "4"}), (1, {"WORLD_SIZE": "8"}),
                      (8, {"WORLD_SIZE": "1"})):
        plan, err = b.rank_plan(gpus, env)
        assert plan is None and f"WORLD_SIZE={env['WORLD_SIZE']}" in err and f"--gpus {gpus}" in err
    assert b.rank_plan(0, {})[0] is None and b.rank_plan(-3, {})[0] is None
    assert "not an integer" in b.rank_plan(2, {"WORLD_SIZE": "two"})[1]


def test_world_size_mismatch_exits_before_torch_or_gpu():
    """WORLD_SIZE=2 ... --gpus 4: non-zero exit with a clear message, and the
    process never imported torch (so it cannot have initialised a GPU)."""
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, BENCH, "--gpus", "4", "--steps", "1"], env=env, capture_output=True,
                       text=True, timeout=120)
    assert r.returncode == 2 and not r.stdout.strip()
    assert "WORLD_SIZE=2" in r.stderr and "--gpus 4" in r.stderr
    probe = ("import runpy, sys\n"
             "sys.argv = ['bench.py', '--gpus', '4']\n"
             "try:\n"
             "    runpy.run_path(sys.argv_path, run_name='__main__')\n"
             "except SystemExit as e:\n"
             "    print('exit', e.code, 'torch' in sys.modules)\n").replace("sys.argv_path", repr(BENCH))
    r = subprocess.run([sys.executable, "-c", probe], env=env, capture_output=True, text=True, timeout=120)
    assert r.stdout.split() == ["exit", "2", "False"], r.stdout + r.stderr


def test_rank_launch_command_is_the_drivers():
    b = _bench()
    cmd = b.rank_launch_cmd(8, ["--gpus", "8", "--steps", "5"], 29517)
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=8" in cmd and "--nnodes=1" in cmd
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1" and cmd[cmd.index("--master-port") + 1] == "29517"
    assert cmd[-4:] == [BENCH, "--gpus", "8", "--steps", "5"][-4:] and os.path.abspath(cmd[-5]) == BENCH


def _stub(body):
    return [sys.executable, "-c", "import sys\n" + body]


def test_relay_prints_exactly_the_rank0_line(capfd):
    b = _bench()
    rc = b.relay(_stub("print('rank progress', flush=True)\n"
                       "print('{\"metric\": \"m\", \"value\": 1.5}', flush=True)\n"
                       "print('rank 1 bye', file=sys.stderr)\n"))
    out, err = capfd.readouterr()
    assert rc == 0
    assert out.splitlines() == ['{"metric": "m", "value": 1.5}'] and json.loads(out)["value"] == 1.5
    assert "rank progress" in err and "rank 1 bye" in err


def test_relay_keeps_the_childs_exit_status(capfd):
    b = _bench()
    assert b.relay(_stub("print('{\"value\": 1}'); sys.exit(3)")) == 3  # a line, but the launch failed
    out, _ = capfd.readouterr()
    assert out.strip() == '{"value": 1}'
    assert b.relay(_stub("sys.exit(5)")) == 5
    # exit 0 without exactly one line is a failure, never a silent success
    assert b.relay(_stub("print('{\"a\": 1}'); print('{\"b\": 2}')")) == 1
    out, err = capfd.readouterr()
    assert not out.strip() and "2 result lines" in err
    assert b.relay(_stub("pass")) == 1


def test_relay_reports_a_signal_death_as_128_plus_the_signal(capfd):
    """A child killed by signal S has returncode -S; sys.exit(-S) would exit
    256 - S, which reads as an ordinary error.  relay maps it to 128 + S."""
    import signal
    b = _bench()
    assert b.exit_status(-signal.SIGTERM) == 143 and b.exit_status(-signal.SIGKILL) == 137
    assert b.exit_status(0) == 0 and b.exit_status(3) == 3
    assert b.relay(_stub("import os, signal; os.kill(os.getpid(), signal.SIGKILL)")) == 137


def test_gpus_n_starts_n_ranks_through_torchrun():
    """No launcher, --gpus 2: bench.py starts torch.distributed.run with two
    ranks that run bench.py with WORLD_SIZE=2 == --gpus (plan "ranks", no
    mismatch).  Without a GPU here each rank then fails at its first device
    call, and that failure is the parent's exit status: no line, non-zero."""
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env["HIP_VISIBLE_DEVICES"] = ""
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--steps", "1", "--warmup", "0", "--chunks", "8"],
                       env=env, capture_output=True, text=True, timeout=300)
    assert "starting 2 ranks" in r.stderr and "--nproc-per-node=2" in r.stderr
    assert "must agree" not in r.stderr  # each rank saw WORLD_SIZE=2 and --gpus 2
    if r.returncode == 0:
        pytest.skip("a GPU is visible here; the GPU test runs this path")
    assert not [l for l in r.stdout.splitlines() if l.startswith("{")]


def test_relay_forwards_sigterm_and_the_ranks_die_with_it(tmp_path):
    """SIGTERM to bench.py's launcher reaches the rank launch (the driver's
    time limit, or a kill of the process it started), and the child exits
    with it instead of running on orphaned on the GPUs."""
    import signal
    import time
    pidfile = tmp_path / "child.pid"
    child = ("import os, sys, time\n"
             f"open({str(pidfile)!r}, 'w').write(str(os.getpid()))\n"
             "print('rank started', flush=True)\n"
             "time.sleep(120)\n")
    runner = ("import importlib.util, sys\n"
              f"spec = importlib.util.spec_from_file_location('b', {BENCH!r})\n"
              "b = importlib.util.module_from_spec(spec); spec.loader.exec_module(b)\n"
              f"sys.exit(b.relay([sys.executable, '-c', {child!r}]))\n")
    p = subprocess.Popen([sys.executable, "-c", runner], stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
    t0 = time.time()
    while not pidfile.exists() and time.time() - t0 < 60:
        time.sleep(0.05)
    assert pidfile.exists(), p.stderr.read() if p.poll() is not None else "child never started"
    cpid = int(pidfile.read_text())
    p.send_signal(signal.SIGTERM)
    rc = p.wait(timeout=60)
    assert rc == 128 + signal.SIGTERM  # the child's SIGTERM death, as a shell reports it
    with pytest.raises(ProcessLookupError):
        for _ in range(100):
            os.kill(cpid, 0)
            time.sleep(0.05)


def test_ensure_built_adds_the_experiments_library_only_for_variants(monkeypatch):
    """A non-default --ring/--lines/--nt loads build_variants/experiments:
    ensure_built must build it on a checkout that lacks it, and
    must not build it for the default kernel."""
    b = _bench()
    calls = []
    real_exists = os.path.exists
    monkeypatch.setattr(b.subprocess, "run", lambda cmd, check: calls.append(cmd))
    monkeypatch.setattr(b.os.path, "exists", lambda p: p != b.EXPERIMENTS_LIB and real_exists(p))
    b.ensure_built()
    assert calls == []
    b.ensure_built(experiments=True)
    assert len(calls) == 1 and calls[0][-1] == "experiments" and "lib" in calls[0]


@pytest.mark.parametrize("bad", [["--steps", "0"], ["--warmup", "-1"], ["--chunks", "0"], ["--gpus", "0"]])
def test_degenerate_arguments_exit_before_torch(bad):
    """A line needs at least one timed step over at least one chunk on at
    least one GPU: anything else exits 2 before torch is imported."""
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, "-X", "importtime", BENCH, *bad], env=env, capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 2 and not r.stdout.strip()
    assert "bench.py:" in r.stderr
    import re
    assert not re.search(r"\|\s+torch\b", r.stderr)  # -X importtime lists every import: torch never was
    assert re.search(r"\|\s+argparse\b", r.stderr)   # (and it does list them)
