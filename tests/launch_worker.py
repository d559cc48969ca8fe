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
        import oracle
        from concurrentproject_amd.dist import gather_scores, shard_bounds, slab_max
        res = {"world": dist.get_world_size(), "rank_env": [world, rank, local]}
        if mode == "batch":
            n, per = int(sys.argv[3]), int(sys.argv[4])
            lo, hi = shard_bounds(per * world, world, rank)
            local_scores = torch.tensor([oracle.score_linear(*oracle.gen_pair(8192 + k, n)) for k in range(lo, hi)],
                                        dtype=torch.int32)
            full = gather_scores(local_scores, per * world)
            res["scores"] = None if full is None else full.tolist()
        elif mode == "slab":
            import concurrentproject_amd as sw
            n, m = int(sys.argv[3]), int(sys.argv[4])
            a, b = oracle.gen_pair(1048576, n)
            b = b[:m]
            bounds = sw.slab_bounds(n, m, world, sw.SW_FLAG_DNA)
            lo, hi = bounds[rank], bounds[rank + 1]
            edge = None
            if rank > 0:
                eh = torch.empty(m, dtype=torch.int32)
                ee = torch.empty(m, dtype=torch.int32)
                dist.recv(eh, src=rank - 1)
                dist.recv(ee, src=rank - 1)
                edge = (eh.numpy(), ee.numpy())
            best, (oh, oe) = oracle.slab(a[lo:hi], b, edge=edge)
            if rank + 1 < world:
                dist.send(torch.from_numpy(np.ascontiguousarray(oh)), dst=rank + 1)
                dist.send(torch.from_numpy(np.ascontiguousarray(oe)), dst=rank + 1)
            score = slab_max(torch.tensor([best], dtype=torch.int32))
            allsc = [torch.zeros(1, dtype=torch.int32) for _ in range(world)]
            dist.all_gather(allsc, score)
            res.update(score=int(score.item()), every_rank=[int(x.item()) for x in allsc], bounds=bounds)
        if rank == 0:
            with open(out, "w") as f:
                json.dump(res, f)
    finally:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
