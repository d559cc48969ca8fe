"""CPU: BASELINE config C1's path, the reference's own CPU harness TestFile.cpp
(main.cpp SmithWatermanScore vs LazySmith vs ParallelLazySmith_threads over
N = 1..5000, 10 random pairs each), compiled in place from the reference
sources exactly as its Makefile1 does (`make -C oracle ref` ->
oracle/_ref/test_runner1).  Mode 2 prints one `Success: 1` per length
(TestFile.cpp:110-120).  The binary needs the reference sources, so it exists
only where /root/reference does; skipped elsewhere."""
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "oracle", "_ref", "test_runner1")


@pytest.mark.skipif(not os.path.exists(BIN), reason="reference CPU harness not built (make -C oracle ref)")
def test_reference_cpu_harness_testfile():
    out = subprocess.run([BIN], input="2\n", capture_output=True, text=True, timeout=600, check=True).stdout
    lengths = [int(x) for x in re.findall(r"LENGTH: (\d+), NUMBER OF TESTS: 10", out)]
    assert lengths == [1, 50, 100, 500, 1000, 1500, 2000, 2500, 3000, 3500, 4000, 4500, 5000], out[-2000:]
    assert re.findall(r"Success: (\d)", out) == ["1"] * 13, out[-2000:]
