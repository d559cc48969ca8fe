# flow3 half-chunk links: which shapes mismatch the oracle, over repeated runs (GPU diagnostic)
import sys, os, numpy as np
sys.path.insert(0, os.getcwd())
import concurrentproject_amd as sw, oracle
ACGT = np.frombuffer(b"ACGT", np.uint8)
rng = np.random.default_rng(5)
def rel(n, m):
    a = ACGT[rng.integers(0, 4, n)]
    b = np.resize(a, m).copy(); mut = rng.random(m) < 0.1; b[mut] = ACGT[rng.integers(0, 4, int(mut.sum()))]
    return a, b
shapes = [(n, m) for n in (254, 300, 400, 500) for m in (40, 64, 100, 128, 200, 256, 400, 511, 512, 513, 700, 1000, 4000)]
pairs = [rel(n, m) for n, m in shapes]
sw.set_option("orient", 1); sw.set_option("mode", 5); sw.set_option("f2w", 2)
op = oracle.Params(1, -1, 1, 1)
exp = [oracle.score_linear(a, b, op) for a, b in pairs]
for C, hl in ((32, 1),):
    sw.set_option("C", C); sw.set_option("f3hl", hl)
    for rep in range(3):
        got = [sw.score(a, b) for a, b in pairs]
        print("C", C, "hl", hl, "rep", rep, [(s, e, g) for s, e, g in zip(shapes, exp, got) if e != g])
