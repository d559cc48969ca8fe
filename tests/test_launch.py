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
    assert res["shard"] == [0, 2]


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
    rep = res["report"]   # bench.py's slab_ranks record, built by the same SlabRank.report
    assert rep["per_rank_columns"] == [res["bounds"][r + 1] - res["bounds"][r] for r in range(world)]
    assert rep["inflow_fine_grained"] == [None] * world and len(rep["per_rank_kernel_ms"]) == world


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
    assert "needs 2 visible GPUs" in p.stderr or "cannot count GPUs" in p.stderr
    assert p.stdout.strip() == ""


def test_bench_gpus_must_match_launcher_world():
    """Under a launcher, --gpus must equal WORLD_SIZE."""
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1"],
                       capture_output=True, text=True, timeout=300, env=env)
    assert p.returncode != 0
    assert "launcher started 1 ranks" in p.stderr


def _fake_topology(tmp_path, ngpu, ncpu=2, unreadable=()):
    """A KFD topology with ncpu CPU nodes and ngpu GPU nodes, and their render nodes."""
    topo, dri = tmp_path / "nodes", tmp_path / "dri"
    topo.mkdir()
    dri.mkdir()
    k = 0
    for _ in range(ncpu):
        (topo / str(k)).mkdir()
        (topo / str(k) / "properties").write_text("cpu_cores_count 64\nsimd_count 0\ndrm_render_minor 0\n")
        k += 1
    for g in range(ngpu):
        (topo / str(k)).mkdir()
        (topo / str(k) / "properties").write_text(
            "cpu_cores_count 0\nsimd_count 1024\ndrm_render_minor %d\nunique_id %d\n" % (128 + g, 1000 + g))
        if g not in unreadable:
            (dri / ("renderD%d" % (128 + g))).write_text("")
        k += 1
    return str(topo), str(dri)


def test_gpu_count_from_kfd_topology(tmp_path):
    """The parent of the ranks counts GPUs from the KFD topology (no HIP call), narrowed
    by the visibility variables; a render node it cannot open does not count."""
    from concurrentproject_amd.launch import LaunchError, gpu_count
    topo, dri = _fake_topology(tmp_path, 8, unreadable=(5,))
    assert gpu_count({}, topo, dri) == 7
    assert gpu_count({"HIP_VISIBLE_DEVICES": "0,1,2"}, topo, dri) == 3
    assert gpu_count({"CUDA_VISIBLE_DEVICES": "1"}, topo, dri) == 1
    assert gpu_count({"HIP_VISIBLE_DEVICES": "0,9,1"}, topo, dri) == 1     # stops at the first invalid index
    assert gpu_count({"HIP_VISIBLE_DEVICES": ""}, topo, dri) == 0
    assert gpu_count({"ROCR_VISIBLE_DEVICES": "2,3", "HIP_VISIBLE_DEVICES": "1"}, topo, dri) == 1
    assert gpu_count({"ROCR_VISIBLE_DEVICES": "GPU-%x" % 1003}, topo, dri) == 1
    # ROCr's own form: GPU- and 16 zero-padded hex digits (any case)
    assert gpu_count({"ROCR_VISIBLE_DEVICES": "GPU-%016x" % 1003}, topo, dri) == 1
    assert gpu_count({"ROCR_VISIBLE_DEVICES": "gpu-%016X,GPU-%016x" % (1003, 1004)}, topo, dri) == 2
    assert gpu_count({"ROCR_VISIBLE_DEVICES": "GPU-%016x,GPU-zz" % 1003}, topo, dri) == 1   # stops at a bad token
    with pytest.raises(LaunchError, match="cannot count GPUs"):
        gpu_count({}, str(tmp_path / "missing"), dri)


def test_bench_parent_never_initialises_hip(tmp_path, monkeypatch):
    """`bench.py --gpus 2`: the parent reaches spawn_ranks with HIP's device count made to
    raise (so it cannot have called it), and exits 2 when the topology shows too few GPUs."""
    import torch
    import bench
    import concurrentproject_amd.launch as launch

    def no_hip(*a, **k):
        raise AssertionError("the parent of the ranks called HIP")
    monkeypatch.setattr(torch._C, "_cuda_getDeviceCount", no_hip, raising=False)
    monkeypatch.setattr(torch.cuda, "device_count", no_hip)
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.delenv("TORCHELASTIC_RUN_ID", raising=False)
    monkeypatch.delenv("HIP_VISIBLE_DEVICES", raising=False)
    monkeypatch.delenv("CUDA_VISIBLE_DEVICES", raising=False)
    monkeypatch.delenv("ROCR_VISIBLE_DEVICES", raising=False)
    calls = []
    monkeypatch.setattr(launch, "spawn_ranks", lambda n, argv, **kw: calls.append((n, argv)) or 0)
    topo, dri = _fake_topology(tmp_path, 2)
    monkeypatch.setenv("SW_KFD_TOPOLOGY", topo)
    monkeypatch.setenv("SW_DRI_DIR", dri)

    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "2", "--steps", "1"])
    assert bench.start_ranks(bench.parse()) == 0
    assert calls and calls[0][0] == 2 and calls[0][1][1].endswith("bench.py")
    topo1, dri1 = _fake_topology(tmp_path / "one", 1) if (tmp_path / "one").mkdir() is None else (None, None)
    monkeypatch.setenv("SW_KFD_TOPOLOGY", topo1)
    monkeypatch.setenv("SW_DRI_DIR", dri1)
    assert bench.start_ranks(bench.parse()) == 2
    assert len(calls) == 1
