"""bench.py's own multi-rank launcher (`--gpus N` without torchrun) and its CPU-baseline leg, on the CPU:
the launcher path runs with the gloo backend over the TEST-ONLY host build of the engine (`--engine host`)."""

import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run_bench(*args, timeout=300):
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env.pop("RANK", None)
    out = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), *args], capture_output=True, text=True,
                         timeout=timeout, env=env, cwd=REPO)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout  # one JSON line, from rank 0 only
    return json.loads(lines[0])


def test_launcher_two_ranks_host_engine():
    sys.path.insert(0, os.path.join(REPO, "tests", "hostsim"))
    import driver

    driver.build()
    B, K, W = 8, 5, 2
    line = _run_bench("--engine", "host", "--gpus", "2", "--steps", str(K), "--warmup", str(W), "--envs", str(B),
                      "--preroll", "60", "--no-cpu-baseline")
    assert line["n_gpus"] == 2 and line["steps"] == K and line["warmup"] == W
    # lockstep with auto-reset: every env of both ranks takes exactly K timed decisions, summed over ranks
    assert line["decisions"] == 2 * B * K
    assert line["config"]["parallelism"] == "env-sharded x2"
    assert line["frozen_envs"] == 0 and line["roofline"] is None
    # the process group held both ranks, and what each rank measured adds up to the reported total
    assert line["ranks_seen"] == 2
    assert sorted(r["rank"] for r in line["per_rank"]) == [0, 1]
    assert sum(r["decisions"] for r in line["per_rank"]) == line["decisions"]
    assert all(r["decisions"] == B * K for r in line["per_rank"])
    assert max(r["elapsed_s"] for r in line["per_rank"]) <= line["ms_per_step"] * K / 1e3 + 1e-9


def test_launcher_one_rank_reports_ranks_seen():
    sys.path.insert(0, os.path.join(REPO, "tests", "hostsim"))
    import driver

    driver.build()
    line = _run_bench("--engine", "host", "--steps", "3", "--warmup", "1", "--envs", "4", "--preroll", "20",
                      "--no-cpu-baseline")
    assert line["n_gpus"] == 1 and line["ranks_seen"] == 1
    assert [r["rank"] for r in line["per_rank"]] == [0] and line["per_rank"][0]["decisions"] == line["decisions"]


@pytest.mark.parametrize("workload", ["tpch", "decima"])
def test_cpu_baseline_worker(workload):
    import bench

    dec, wall, _, _ = bench._cpu_worker((workload, 3, 1.0, 0.5, 0))
    assert dec > 0 and wall >= 1.0
    assert bench.usable_cpus() >= 1 and isinstance(bench.cpu_model(), str)
