"""bench.py --gpus N starts its own N ranks when no launcher did.

The children run bench.py itself with SPFF_BENCH_STUB=1, which reports the rank layout
and returns before any device call, so this runs on the CPU container.
"""
import json
import os
import pathlib
import subprocess
import sys

ROOT = pathlib.Path(__file__).resolve().parents[1]


def _env(**kw):
    e = {k: v for k, v in os.environ.items()
         if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    e.update(kw)
    return e


def _run(args, env):
    return subprocess.run([sys.executable, str(ROOT / "bench.py"), *args], env=env,
                          capture_output=True, text=True, timeout=300)


def test_gpus_n_spawns_n_distinct_ranks():
    r = _run(["--gpus", "3", "--steps", "1"], _env(SPFF_BENCH_STUB="1"))
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [json.loads(ln) for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 3
    assert sorted(d["rank"] for d in lines) == [0, 1, 2]
    assert sorted(d["local_rank"] for d in lines) == [0, 1, 2]
    assert all(d["world_size"] == 3 and d["launched"] for d in lines)
    # one rendezvous for all ranks, on the loopback address
    assert len({tuple(d["master"]) for d in lines}) == 1
    assert lines[0]["master"][0] == "127.0.0.1"


def test_gpus_one_stays_in_process():
    r = _run(["--gpus", "1"], _env(SPFF_BENCH_STUB="1"))
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [json.loads(ln) for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1 and lines[0]["world_size"] == 1 and not lines[0]["launched"]


def test_launcher_mismatch_fails():
    env = _env(SPFF_BENCH_STUB="1", WORLD_SIZE="2", RANK="0", LOCAL_RANK="0",
               MASTER_ADDR="127.0.0.1", MASTER_PORT="29555")
    r = _run(["--gpus", "4"], env)
    assert r.returncode != 0
    assert "WORLD_SIZE=2" in r.stderr


def test_child_failure_propagates():
    # a child that fails makes the parent exit non-zero (here: rank 1 of 2 exits 3)
    sys.path.insert(0, str(ROOT))
    import bench
    code = ("import os, sys; sys.exit(3 if os.environ['RANK'] == '1' else 0)")
    rc = bench.launch_ranks(2, [], child_cmd=[sys.executable, "-c", code],
                            env=_env(SPFF_BENCH_KILL_AFTER="5"))
    assert rc == 3
