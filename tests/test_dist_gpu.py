"""GPU: the sharded batch path (dist.score_sharded -> score_batch_device -> RCCL
gather) with the real HIP kernels, at world size 1 over the "nccl" (RCCL)
backend: the C3 batch (1024 pairs, N = 8192) against the committed golden.  The
world > 1 decomposition is covered with gloo on the CPU (tests/test_dist.py);
8-GPU runs are the driver's scaling bench (bench.py --gpus N: the C4 batch)."""
import os
import socket

import pytest

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def test_score_sharded_nccl_world1_c3(engine, golden):
    import torch
    import torch.distributed as dist
    from concurrentproject_amd.dist import score_sharded, shard_bounds

    c = golden("configs.json")["C3"]
    N, P = c["N"], c["npairs"]
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ["MASTER_PORT"] = str(_free_port())
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        stream = torch.cuda.current_stream()

        def shard(lo, hi):
            # this rank's pairs generated on the host, resident in HBM, one launch
            arena = torch.from_numpy(engine.gen_batch(c["seed_base"] + lo, hi - lo, N)).cuda()
            scores = torch.full((hi - lo,), -1, dtype=torch.int32, device="cuda")
            k = range(hi - lo)
            engine.score_batch_device(arena.data_ptr(), [2 * N * i for i in k], [N] * (hi - lo),
                                      [2 * N * i + N for i in k], [N] * (hi - lo), scores.data_ptr(), flags=1,
                                      stream=stream.cuda_stream)
            engine.stream_status(stream.cuda_stream)
            return scores.cpu().tolist()

        assert shard_bounds(P, 1, 0) == (0, P)
        got = score_sharded(P, shard, device="cuda")
        assert got == c["scores"]
        assert engine.last_stats()["mode"] == 3     # the duo kernel ran
    finally:
        dist.destroy_process_group()
