"""CPU: the one-process-per-GPU launcher that `bench.py --gpus N` uses
(concurrentproject_amd.launch).  World-2 jobs run tests/launch_worker.py over gloo
with the oracle standing in for the kernels; bench.py itself must refuse to start
more ranks than there are GPUs."""
import json
import os
import subprocess
import sys
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
WORKER = os.path.join(ROOT, "tests", "launch_worker.py")


def test_rank_env_and_launcher_detection():
    from concurrentproject_amd.launch import launcher_env, rank_env
    assert not launcher_env({})
    assert launcher_env({"WORLD_SIZE": "1"}) and launcher_env({"TORCHELASTIC_RUN_ID": "x"})
    assert rank_env({}) == (1, 0, 0)
    assert rank_env({"WORLD_SIZE": "8", "RANK": "5", "LOCAL_RANK": "5"}) == (8, 5, 5)


def test_require_devices():
    from concurrentproject_amd.launch import LaunchError, require_devices
    assert require_devices(2, devices=8) == 8
    with pytest.raises(LaunchError, match="needs 2 visible GPUs"):
        require_devices(2, devices=1)


def test_launcher_batch_gloo_matches_c4_golden(tmp_path):
    """Two ranks, each scoring its contiguous block of the C4-order pairs (seeds 8192+k,
    N=8192); rank 0's gathered vector equals the committed C4 golden prefix."""
    from concurrentproject_amd.launch import spawn_ranks
    out = tmp_path / "batch.json"
    rc = spawn_ranks(2, [sys.executable, WORKER, "batch", str(out), "8192", "2"], timeout=600)
    assert rc == 0
    res = json.loads(out.read_text())
    assert res["world"] == 2 and res["rank_env"] == [2, 0, 0]
    gold = json.load(open(os.path.join(ROOT, "tests", "golden", "configs.json")))
    ref = gold.get("C4", gold["C3"])["scores"]
    assert res["scores"] == ref[:4]


@pytest.mark.parametrize("world,n,m", [(2, 1500, 700), (3, 1000, 450)])
def test_launcher_slab_gloo(tmp_path, world, n, m):
    """The column-slab path through the launcher: every rank ends with the pair's score."""
    import oracle
    from concurrentproject_amd.launch import spawn_ranks
    out = tmp_path / "slab.json"
    rc = spawn_ranks(world, [sys.executable, WORKER, "slab", str(out), str(n), str(m)], timeout=600)
    assert rc == 0
    res = json.loads(out.read_text())
    a, b = oracle.gen_pair(1048576, n)
    exp = oracle.score_linear(a, b[:m])
    assert res["score"] == exp and res["every_rank"] == [exp] * world
    assert len(set(res["bounds"])) == world + 1


def test_launcher_failure_stops_the_job(tmp_path):
    """A failing rank's status is the job's, and the ranks still waiting are terminated."""
    from concurrentproject_amd.launch import spawn_ranks
    t0 = time.monotonic()
    rc = spawn_ranks(2, [sys.executable, WORKER, "fail", str(tmp_path / "x"), "1"], timeout=100)
    assert rc == 3
    assert time.monotonic() - t0 < 60


def test_bench_refuses_more_gpus_than_visible():
    """`bench.py --gpus 2` on a host with fewer than 2 GPUs fails loudly before any rank starts."""
    import torch
    if torch.cuda.device_count() >= 2:
        pytest.skip("this host has >= 2 GPUs")
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1"],
                       capture_output=True, text=True, timeout=300,
                       env={k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "TORCHELASTIC_RUN_ID")})
    assert p.returncode == 2, (p.returncode, p.stderr[-2000:])
    assert "needs 2 visible GPUs" in p.stderr
    assert p.stdout.strip() == ""


def test_bench_gpus_must_match_launcher_world():
    """Under a launcher, --gpus must equal WORLD_SIZE."""
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1"],
                       capture_output=True, text=True, timeout=300, env=env)
    assert p.returncode != 0
    assert "launcher started 1 ranks" in p.stderr
