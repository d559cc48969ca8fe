"""sw_score_batch_multi (include/algoGPU.h): a batch sharded over the first ngpus GPUs
of the node, one host thread and stream per device, int32 scores gathered to device 0
over RCCL.

CPU: the shard plan equals dist.shard_bounds (the partition every other multi-GPU
path uses).  GPU: ngpus = 1 against the C3 golden (the reference-pinned scores);
more GPUs than visible fails with -1 and a message.  A GPU box here has one GPU, so
ngpus > 1 has not run on hardware."""
import pytest

import concurrentproject_amd as sw
from concurrentproject_amd.dist import shard_bounds


@pytest.mark.parametrize("npairs", [0, 1, 7, 1024, 8192, 8193])
@pytest.mark.parametrize("ngpus", [1, 2, 3, 8])
def test_shard_plan_matches_dist(npairs, ngpus):
    got = [sw.batch_shard(npairs, ngpus, r) for r in range(ngpus)]
    assert got == [shard_bounds(npairs, ngpus, r) for r in range(ngpus)]
    assert got[0][0] == 0 and got[-1][1] == npairs
    assert all(a[1] == b[0] for a, b in zip(got, got[1:]))


@pytest.mark.parametrize("npairs", [0, 1, 3, 7, 1024, 8191, 8192, 8193])
@pytest.mark.parametrize("ngpus", [1, 2, 3, 8])
def test_gather_plan(npairs, ngpus):
    """The RCCL gather of sw_score_batch_multi (the only exchange): device r sends exactly its
    shard's scores, which land at the shard's start in device 0's buffer, so the gathered vector
    is every score once, in pair order -- checked without a second GPU."""
    plan = sw.batch_gather_plan(npairs, ngpus)
    assert plan == [(hi - lo, lo) for lo, hi in (shard_bounds(npairs, ngpus, r) for r in range(ngpus))]
    covered = [0] * npairs
    for cnt, off in plan:
        assert cnt >= 0 and 0 <= off and off + cnt <= npairs
        for k in range(off, off + cnt):
            covered[k] += 1
    assert covered == [1] * npairs
    with pytest.raises(sw.SwError, match="invalid"):
        sw.batch_gather_plan(10, 0)


def test_shard_plan_rejects_bad_arguments():
    for args in ((10, 0, 0), (10, 2, 2), (-1, 2, 0), (10, 2, -1)):
        with pytest.raises(sw.SwError, match="invalid"):
            sw.batch_shard(*args)


@pytest.mark.gpu
def test_multi_one_gpu_c3_golden(engine, golden):
    c = golden("configs.json")["C3"]
    arena = engine.gen_batch(c["seed_base"], c["npairs"], c["N"])
    N = c["N"]
    pairs = [(arena[2 * N * k:2 * N * k + N], arena[2 * N * k + N:2 * N * (k + 1)]) for k in range(c["npairs"])]
    assert engine.score_batch(pairs, ngpus=1) == c["scores"]
    assert engine.last_stats()["cells"] == c["npairs"] * N * N
    # ragged and empty pairs keep their slots
    mixed = [pairs[0], (b"", b"ACGT"), (pairs[1][0][:1], pairs[1][1]), (b"ACGTACGT", b"ACG"), pairs[2]]
    assert engine.score_batch(mixed, ngpus=1) == engine.score_batch(mixed)


@pytest.mark.gpu
def test_multi_more_gpus_than_visible(engine):
    import torch
    n = torch.cuda.device_count()
    with pytest.raises(engine.SwError, match="visible"):
        engine.score_batch([(b"ACGT", b"ACGT")], ngpus=n + 1)
    with pytest.raises(engine.SwError, match="visible"):
        engine.score_batch([(b"ACGT", b"ACGT")], ngpus=n + 7)
