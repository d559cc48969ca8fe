"""GPU: the reference's own harness, unchanged, on the MI355X library.

oracle/_ref/test_runner2_mi355 is TestFileWithGPU.cpp + main.cpp + lazySmith*.cpp
compiled in place from the reference sources (`make -C oracle harness`) and
linked against concurrentproject_amd/libswmi355.so instead of the CUDA objects
(Makefile2:14-27).  For 10 random pairs of N=3000 it checks, per pair, that
SmithWatermanScore == LazySmith == ParallelLazySmith_threads ==
SequentialSmithWatermanScoreGPU == SmithWatermanLazyGPU ==
SmithWatermanScoreCUDA (TestFileWithGPU.cpp:104) and prints SUCCESS or ERROR.
Mode 1 (per-test) is used: mode 2's summary flag mis-parenthesises its check
(TestFileWithGPU.cpp:140).  The binary is built here (it needs the reference
sources) and travels to the GPU box with the snapshot; skipped if absent.
"""
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "oracle", "_ref", "test_runner2_mi355")

pytestmark = pytest.mark.gpu


@pytest.mark.skipif(not os.path.exists(BIN), reason="reference harness not built (make -C oracle harness)")
def test_reference_harness_all_success():
    out = subprocess.run([BIN], input="1\n", capture_output=True, text=True, timeout=600, check=True).stdout
    results = re.findall(r"TEST (\d+): score=(-?\d+)\n(SUCCESS|ERROR)", out)
    assert len(results) == 10, out[-2000:]
    assert all(r[2] == "SUCCESS" for r in results), out[-4000:]
    assert all(int(r[1]) > 0 for r in results)
