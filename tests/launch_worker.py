"""One rank of a CPU job started by concurrentproject_amd.launch.spawn_ranks (test helper,
not collected by pytest).  The gloo backend stands in for RCCL and the CPU oracle for
the HIP kernels, so the rank logic of bench.py's multi-GPU workloads runs here:

    launch_worker.py batch OUT N PAIRS_PER_RANK   C4-order shards + score gather to rank 0
    launch_worker.py slab  OUT N M                one pair in column slabs, edges rank to rank
    launch_worker.py fail  OUT RANK_THAT_FAILS    that rank exits 3, the others wait

Rank 0 writes a JSON result to OUT.
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    mode, out = sys.argv[1], sys.argv[2]
    from concurrentproject_amd.launch import launcher_env, rank_env
    assert launcher_env(), "started without launcher variables"
    world, rank, local = rank_env()
    if mode == "fail":
        if rank == int(sys.argv[3]):
            sys.exit(3)
        time.sleep(120)          # spawn_ranks must terminate this rank
        return
    import numpy as np
    import torch
    import torch.distributed as dist
    dist.init_process_group("gloo")          # env:// from the launcher's variables
    try:
        import bench   # the rank logic bench.py runs at N GPUs, with the oracle as the scorer
        import oracle
        res = {"world": dist.get_world_size(), "rank_env": [world, rank, local]}
        if mode == "batch":
            n, per = int(sys.argv[3]), int(sys.argv[4])
            job = bench.BatchRank(torch, dist, world, rank, n, per, scorer="oracle")
            t_max, kern_ms = bench.time_launches(torch, job.launch, job.collective, 1, 0, job.stream, dist)
            res["scores"] = job.result()
            res["shard"] = [job.lo, job.hi]
        elif mode == "slab":
            n, m = int(sys.argv[3]), int(sys.argv[4])
            a, b = oracle.gen_pair(1048576, n)
            job = bench.SlabRank(torch, dist, n, m, a, b[:m], scorer="oracle")
            t_max, kern_ms = bench.time_launches(torch, job.launch, job.collective, 2, 0, job.stream, dist)
            score = torch.tensor([job.result()], dtype=torch.int32)
            allsc = [torch.zeros(1, dtype=torch.int32) for _ in range(world)]
            dist.all_gather(allsc, score)
            rep = job.report(kern_ms)
            res.update(score=int(score.item()), every_rank=[int(x.item()) for x in allsc], bounds=job.slabs.bounds,
                       report=rep)
            job.close()
        if rank == 0:
            with open(out, "w") as f:
                json.dump(res, f)
    finally:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
