"""bench.py --gpus N without an external launcher: the
script starts its own N rank processes (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set
before any device call), runs the strong split of ONE batch, gathers every step to rank 0
in the wire format, reassembles the last step and checks it against a world-1 run of a
sample of clusters; the parent relays rank 0's JSON line.  Here the ranks use gloo and the
C oracle as their "kernels" (tests/bench_oracle_backend.py); the launcher, partition,
gather, reassembly and output are bench.py's own code.  Reference loops split over the
ranks: binning.py:291, most_similar_representative.py:60."""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run_bench(*argv, timeout=300):
    env = dict(os.environ, SPX_BENCH_BACKEND="bench_oracle_backend:OracleBackend",
               PYTHONPATH=os.pathsep.join([os.path.join(REPO, "tests"), REPO]), OMP_NUM_THREADS="1")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT", "SPX_BENCH_SPAWNED"):
        env.pop(k, None)
    return subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), *argv], env=env, capture_output=True,
                          text=True, timeout=timeout)


@pytest.mark.parametrize("n", [2, 3])
def test_bench_gpus_n_spawns_ranks(n):
    r = _run_bench("--gpus", str(n), "--steps", "2", "--warmup", "1", "--clusters", "61", "--no-extras")
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout  # ONE JSON line, from rank 0
    d = json.loads(lines[0])
    assert d["n_gpus"] == n and d["scaling"] == "strong"
    cfg = d["config"]
    assert cfg["launcher"].startswith("bench.py --gpus N")
    assert cfg["clusters"] == 61 and sum(cfg["rank_clusters"]) == 61
    assert abs(sum(cfg["rank_cost_share"]) - 1.0) < 1e-3
    assert cfg["rank0_weight"] == 1.0 - 0.04 * (n - 1) and cfg["rank_cost_share"][0] < cfg["rank_cost_share"][1]
    a = cfg["assembled_last_step"]
    assert a["ok"] and a["reps_resolved"] and a["sample_equal_world1"] and a["clusters"] == 61
    assert a["consensus_peaks"] == a["planned_peaks"] == cfg["gathered_peaks_per_step"]
    assert cfg["gather_wire"].startswith("f32 bin sums")
    assert d["value"] > 0 and d["steps"] == 2 and d["warmup"] == 1


def test_bench_worker_failure_is_nonzero():
    """A rank that fails makes the launch fail (and the others are stopped), never a
    silent partial line: an unknown backend class fails every rank at start-up."""
    env_bad = dict(os.environ, SPX_BENCH_BACKEND="bench_oracle_backend:NoSuchBackend",
                   PYTHONPATH=os.pathsep.join([os.path.join(REPO, "tests"), REPO]))
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "SPX_BENCH_SPAWNED"):
        env_bad.pop(k, None)
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--steps", "1", "--warmup",
                        "0", "--clusters", "9", "--no-extras"], env=env_bad, capture_output=True, text=True,
                       timeout=300)
    assert r.returncode != 0
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
