"""Probe: flow2 streamed kernel at several workgroups per CU, ring and linear edges;
kernel time of the second of two runs.

    python tools/probe_wgs.py N [rings] [wgs list] [timeout_s]"""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
import concurrentproject_amd as sw
torch.cuda.set_device(0)
sw.set_option("timeout", 5)
N = int(sys.argv[1]) if len(sys.argv) > 1 else 200000
a, b = sw.gen_pair(N, N)
arena = torch.from_numpy(np.concatenate([a, b])).cuda()
score = torch.zeros(1, dtype=torch.int32, device="cuda")
s = torch.cuda.current_stream().cuda_stream
RINGS = [int(x) for x in (sys.argv[2] if len(sys.argv) > 2 else "0,1").split(",")]
WGS = [int(x) for x in (sys.argv[3] if len(sys.argv) > 3 else "1,2,3,4").split(",")]
sw.set_option("timeout", int(sys.argv[4]) if len(sys.argv) > 4 else 5)
for ring in RINGS:
    for w in WGS:
        sw.set_option("ring", ring)
        sw.set_option("f2_wgs", w)
        sw.set_option("f2stream", 1)
        t = time.time()
        try:
            for _ in range(2):
                sw.score_batch_device(arena.data_ptr(), [0], [N], [N], [N], score.data_ptr(), flags=1, stream=s)
                sw.stream_status(s)
            st = sw.last_stats()
            print("N", N, "ring", ring, "wgs", w, "score", score.item(), "kernel_ms %.2f" % st["kernel_ms"],
                  "blocks", st["blocks"], "variant", st["variant"], "edge_MB %.1f" % (st["boundary_bytes"] / 1e6), flush=True)
        except Exception as e:
            print("ring", ring, "wgs", w, "ERROR", e, "s %.1f" % (time.time() - t), flush=True)
