"""One process per GPU without an external launcher.

``bench.py --gpus N`` (and any other entry point) can be started two ways:

* by ``torch.distributed.run`` / torchrun, which sets RANK, LOCAL_RANK,
  WORLD_SIZE and MASTER_* before the script starts (``launcher_env()`` is then
  true and the script is one rank);
* standalone, with N > 1: the parent process -- which has not touched the GPU --
  checks that N devices are visible and starts N children of the same command,
  rank r on device r, with the same environment variables torchrun would set
  (MASTER_ADDR 127.0.0.1, a free port), waits for them and exits with the first
  failing child's status.  The parent never execs: the children are new
  processes, so nothing that initialised HIP is ever replaced.

The reference has no multi-GPU path; this is the entry
point of SURVEY.md 8(e) (pairs sharded over GPUs, RCCL only for the gather).
"""
from __future__ import annotations

import os
import socket
import subprocess
import sys
import time
from typing import Optional, Sequence

_LAUNCHER_KEYS = ("WORLD_SIZE", "TORCHELASTIC_RUN_ID")


class LaunchError(RuntimeError):
    """The requested ranks cannot be started (too few devices, bad arguments)."""


def launcher_env(environ=None) -> bool:
    """True when this process is one rank started by a launcher (torchrun or spawn_ranks)."""
    env = os.environ if environ is None else environ
    return any(k in env for k in _LAUNCHER_KEYS)


def rank_env(environ=None) -> tuple:
    """(world, rank, local_rank) from the launcher's variables (1, 0, 0 without one)."""
    env = os.environ if environ is None else environ
    return int(env.get("WORLD_SIZE", "1")), int(env.get("RANK", "0")), int(env.get("LOCAL_RANK", "0"))


def visible_devices() -> int:
    """GPUs this process could use.  torch.cuda.device_count() does not initialise
    HIP on this image, so the parent stays clean for spawning."""
    import torch
    return int(torch.cuda.device_count())


def require_devices(n: int, devices: Optional[int] = None) -> int:
    """Raise LaunchError unless at least n GPUs are visible; returns the count."""
    have = visible_devices() if devices is None else devices
    if have < n:
        raise LaunchError("--gpus %d needs %d visible GPUs, this host shows %d "
                          "(HIP_VISIBLE_DEVICES=%r)" % (n, n, have, os.environ.get("HIP_VISIBLE_DEVICES")))
    return have


def free_port(host: str = "127.0.0.1") -> int:
    s = socket.socket()
    try:
        s.bind((host, 0))
        return s.getsockname()[1]
    finally:
        s.close()


def spawn_ranks(nprocs: int, argv: Sequence[str], env: Optional[dict] = None, port: Optional[int] = None,
                timeout: Optional[float] = None, poll_s: float = 0.05) -> int:
    """Run ``argv`` as nprocs ranks of one job on this node and wait for all of them.

    Rank r gets RANK = LOCAL_RANK = r, WORLD_SIZE = LOCAL_WORLD_SIZE = nprocs,
    MASTER_ADDR = 127.0.0.1 and a common free MASTER_PORT (torchrun's variables).
    When one rank fails the others are terminated (by their own PIDs) and its
    exit status is returned; 0 when every rank succeeded.  A rank still running
    after ``timeout`` seconds fails the job with 124, as timeout(1) does."""
    if nprocs < 1:
        raise LaunchError("nprocs must be >= 1")
    base = dict(os.environ if env is None else env)
    for k in _LAUNCHER_KEYS:
        base.pop(k, None)
    port = port or free_port()
    procs = []
    for r in range(nprocs):
        e = dict(base)
        e.update(RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(nprocs), LOCAL_WORLD_SIZE=str(nprocs),
                 GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen(list(argv), env=e))
    t0 = time.monotonic()
    status = 0
    try:
        while True:
            codes = [p.poll() for p in procs]
            bad = [c for c in codes if c is not None and c != 0]
            if bad:
                status = bad[0]
                break
            if all(c == 0 for c in codes):
                break
            if timeout is not None and time.monotonic() - t0 > timeout:
                status = 124
                break
            time.sleep(poll_s)
    finally:
        for p in procs:
            if p.poll() is None:
                p.terminate()
        for p in procs:
            try:
                p.wait(timeout=30)
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()
    if status:
        print("spawn_ranks: a rank failed with status %d (%d ranks, %s)" % (status, nprocs, " ".join(argv[:2])),
              file=sys.stderr, flush=True)
    return status
