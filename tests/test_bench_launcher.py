"""bench.py's own N-rank launcher (VERDICT r3 missing #1): `python bench.py --gpus N` with no
torchrun starts N worker processes itself, one per GPU, each with RANK / LOCAL_RANK / WORLD_SIZE /
MASTER_*; under a launcher --gpus must equal WORLD_SIZE. CPU only: the plan and the process
handling, with stand-in worker commands (the GPU run is bench.py itself on the box)."""
import os
import subprocess
import sys
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def test_plan_single_without_launcher():
    assert bench.launch_plan(1, {}) == ("single", None)


def test_plan_spawns_n_ranks_with_their_environment():
    kind, envs = bench.launch_plan(4, {"PATH": "/bin", "HSA_ENABLE_IPC_MODE_LEGACY": "0"})
    assert kind == "spawn" and len(envs) == 4
    ports = {e["MASTER_PORT"] for e in envs}
    assert len(ports) == 1 and int(ports.pop()) > 0
    for r, e in enumerate(envs):
        assert (e["RANK"], e["LOCAL_RANK"], e["WORLD_SIZE"]) == (str(r), str(r), "4")
        assert e["MASTER_ADDR"] == "127.0.0.1"
        assert e["PATH"] == "/bin" and e["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"  # inherited


def test_plan_keeps_a_given_master_port():
    _, envs = bench.launch_plan(2, {"MASTER_PORT": "29555"})
    assert [e["MASTER_PORT"] for e in envs] == ["29555", "29555"]


def test_plan_under_a_launcher():
    assert bench.launch_plan(8, {"WORLD_SIZE": "8", "RANK": "3"}) == ("rank", None)
    assert bench.launch_plan(1, {"WORLD_SIZE": "1"}) == ("single", None)
    with pytest.raises(ValueError):
        bench.launch_plan(8, {"WORLD_SIZE": "4"})
    with pytest.raises(ValueError):
        bench.launch_plan(0, {})


def test_bench_rejects_mismatched_world_size():
    env = dict(os.environ, WORLD_SIZE="2", RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4"], env=env,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 2 and "WORLD_SIZE=2" in r.stderr


def test_spawn_ranks_runs_every_rank(tmp_path):
    _, envs = bench.launch_plan(3, dict(os.environ))
    code = ("import os, pathlib; pathlib.Path(os.environ['OUT'], os.environ['RANK']).write_text("
            "os.environ['WORLD_SIZE'] + ' ' + os.environ['LOCAL_RANK'])")
    for e in envs:
        e["OUT"] = str(tmp_path)
    assert bench.spawn_ranks([sys.executable, "-c", code], envs, poll_s=0.05) == 0
    assert sorted(os.listdir(tmp_path)) == ["0", "1", "2"]
    assert (tmp_path / "2").read_text() == "3 2"


def test_spawn_ranks_fails_fast_and_stops_the_others():
    _, envs = bench.launch_plan(2, dict(os.environ))
    code = "import os, sys, time; sys.exit(3) if os.environ['RANK'] == '1' else time.sleep(60)"
    t0 = time.time()
    rc = bench.spawn_ranks([sys.executable, "-c", code], envs, poll_s=0.05)
    assert rc == 3
    assert time.time() - t0 < 30  # rank 0 was terminated, not waited for


def test_spawn_ranks_keeps_stdout_to_the_json_line(tmp_path):
    """Rank 0's stdout carries only its JSON line (runtime notices go to stderr); other ranks print to
    stderr."""
    _, envs = bench.launch_plan(2, dict(os.environ))
    code = ("import os; r = os.environ['RANK']; print('[Gloo] Rank', r, 'is connected'); "
            "print('{\"rank\": ' + r + '}') if r == '0' else None")
    script = tmp_path / "w.py"
    script.write_text(code)
    driver = ("import sys; sys.path.insert(0, %r); import bench, os; "
              "_, e = bench.launch_plan(2, dict(os.environ)); sys.exit(bench.spawn_ranks([sys.executable, %r], e, 0.05))"
              % (ROOT, str(script)))
    r = subprocess.run([sys.executable, "-c", driver], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0
    assert r.stdout.strip().splitlines() == ['{"rank": 0}']
    assert r.stderr.count("[Gloo]") == 2
