"""Multi-rank sharding on CPU with gloo (world_size 2 and 3)."""
import os
import random
import subprocess
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_cocluster_matches_single_process(tmp_path, world):
    out = tmp_path / "ok.txt"
    port = random.randint(20000, 40000)
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    r = subprocess.run([sys.executable, os.path.join(HERE, "_dist_worker.py"), str(world), str(port), str(out)],
                       env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    assert out.read_text() == "ok"


def test_bench_launcher_starts_the_requested_ranks():
    """bench.py --gpus 2 (no WORLD_SIZE) starts 2 ranks via torch.distributed.run;
    --launcher-check wires them over gloo without touching a GPU."""
    import json
    root = os.path.dirname(HERE)
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--launcher-check"],
                       env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1]
    out = json.loads(line)
    assert out["n_gpus"] == 2
    assert sorted(x[0] for x in out["ranks_seen"]) == [0, 1]
    # the per-rank phase report of a real run, gathered over the same ranks
    pr = out["per_rank"]
    assert [x["rank"] for x in pr] == [0, 1]
    assert all(x["step_ms"] > 0 and set(x) >= {"boot_phase_ms", "allgather_ms", "slab_ms"} for x in pr)


@pytest.mark.parametrize("world", [2, 4])
def test_bench_launcher_check_end_to_end(world):
    """bench.py --launcher-check --gpus N end to end with N = 2 and 4 ranks:
    every rank reports, in rank order (what a --gpus 8 line's per_rank
    block is built from)."""
    import json
    root = os.path.dirname(HERE)
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", str(world), "--launcher-check"],
                       env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert out["n_gpus"] == world and [x["rank"] for x in out["per_rank"]] == list(range(world))
    assert sorted(x[1] for x in out["ranks_seen"]) == list(range(world))  # LOCAL_RANK = device per rank


def test_bench_refuses_more_gpus_than_visible():
    """bench.py --gpus N exits non-zero at once, with a message, when fewer
    than N devices are visible (here: none)."""
    root = os.path.dirname(HERE)
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["HIP_VISIBLE_DEVICES"] = ""
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "8", "--steps", "1"],
                       env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 2
    assert "requested but" in r.stderr
