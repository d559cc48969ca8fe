"""Single pairs over small alphabets other than {A,C,G,T} (the seven-letter path, sw_flow3.hip HEP)
against the byte path (option hep = 0) and the DNA path on the same shape.

Times kernel ms (sw_last_stats, the device entry point with the alphabet scanned on the device) of
one N x N pair per alphabet, hep = 1 and hep = 0, and checks both give the same score.  One JSON
line per alphabet and parameter set.

    python tools/bench_hep.py [--n N] [--reps R] [--params 1,-1,1,1;2,-3,5,2]
"""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=65536)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--params", default="1,-1,1,1;2,-3,5,2")
    a = ap.parse_args()
    import torch
    import concurrentproject_amd as sw
    N = a.n
    base_a, base_b = sw.gen_pair(65536 if N == 65536 else N, N)
    rng = np.random.default_rng(N)
    cases = {"acgt": (base_a, base_b)}
    x, y = base_a.copy(), base_b.copy()
    x[rng.random(N) < 0.01] = ord("N")
    y[rng.random(N) < 0.01] = ord("N")
    cases["acgt+1%N"] = (x, y)
    lower = np.frombuffer(b"acgt", np.uint8)
    cases["acgt lower"] = (lower[(base_a >> 1 ^ base_a >> 2) & 3], lower[(base_b >> 1 ^ base_b >> 2) & 3])
    seven = np.frombuffer(b"ACGTNRY", np.uint8)
    cases["7 letters"] = (seven[rng.integers(0, 7, N)], seven[rng.integers(0, 7, N)])
    scores = torch.zeros(1, dtype=torch.int32, device="cuda")
    for ptxt in a.params.split(";"):
        prm = [int(v) for v in ptxt.split(",")]
        sw.set_params(sw.Params(*prm))
        for name, (p, q) in cases.items():
            arena = torch.from_numpy(np.concatenate([p, q])).cuda()
            out = {"case": name, "n": N, "params": prm}
            got = {}
            for hep in ((1, 0) if name != "acgt" else (1,)):
                sw.set_option("hep", hep)
                ms = []
                for _ in range(a.reps + 1):
                    sw.score_batch_device(arena.data_ptr(), [0], [N], [N], [N], scores.data_ptr())
                    st = sw.last_stats()
                    ms.append(st["kernel_ms"])
                k = min(ms[1:])
                got[hep] = scores.item()
                out["hep%d" % hep] = {"kernel_ms": round(k, 4), "gcups": round(N * N / k / 1e6, 1), "dna": st["dna"],
                                      "mode": st["mode"], "W": st["W"], "C": st["C"], "variant": st["variant"]}
            sw.set_option("hep", 1)
            out["score"] = got[1]
            if 0 in got:
                out["scores_equal"] = got[0] == got[1]
                out["speedup"] = round(out["hep0"]["kernel_ms"] / out["hep1"]["kernel_ms"], 3)
            print(json.dumps(out), flush=True)
    sw.set_params(sw.Params())


if __name__ == "__main__":
    main()
