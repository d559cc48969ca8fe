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
    """GPUs this rank can use (HIP's count; a rank may initialise HIP).  The parent of
    spawned ranks counts with gpu_count() instead, which makes no HIP call at all."""
    import torch
    return int(torch.cuda.device_count())


KFD_TOPOLOGY = "/sys/class/kfd/kfd/topology/nodes"


def _props(path: str) -> dict:
    out = {}
    with open(path) as f:
        for line in f:
            parts = line.split()
            if len(parts) == 2:
                out[parts[0]] = parts[1]
    return out


def kfd_gpus(root: Optional[str] = None, dri: Optional[str] = None) -> list:
    """The GPU agents ROCr would enumerate, read from the KFD topology without any HIP or
    driver call: nodes with SIMDs (CPU nodes have none) whose render node
    /dev/dri/renderD<drm_render_minor> this process may open, in node order.  Each entry
    is the node's properties.  Raises LaunchError if the topology cannot be read."""
    root = root or os.environ.get("SW_KFD_TOPOLOGY", KFD_TOPOLOGY)
    dri = dri or os.environ.get("SW_DRI_DIR", "/dev/dri")
    try:
        nodes = sorted((int(d) for d in os.listdir(root) if d.isdigit()))
    except OSError as e:
        raise LaunchError("cannot count GPUs: KFD topology %s unreadable (%s)" % (root, e)) from None
    gpus = []
    for k in nodes:
        try:
            pr = _props(os.path.join(root, str(k), "properties"))
        except OSError:
            continue
        if int(pr.get("simd_count", "0")) <= 0:
            continue
        node = os.path.join(dri, "renderD%s" % pr.get("drm_render_minor", "-1"))
        if not os.access(node, os.R_OK | os.W_OK):
            continue
        gpus.append(pr)
    return gpus


def gpu_count(environ=None, root: Optional[str] = None, dri: Optional[str] = None) -> int:
    """Visible GPUs without initialising HIP: the KFD GPUs (kfd_gpus), narrowed by
    ROCR_VISIBLE_DEVICES (indices or GPU-<hex unique id>) and then by HIP_VISIBLE_DEVICES
    (or CUDA_VISIBLE_DEVICES): indices into that list, counted up to the first invalid one."""
    env = os.environ if environ is None else environ
    gpus = kfd_gpus(root, dri)
    rocr = env.get("ROCR_VISIBLE_DEVICES")
    if rocr is not None:
        # UUID tokens: ROCr prints GPU- and 16 zero-padded hex digits; compare the numbers
        ids = {int(g.get("unique_id", "0")): g for g in gpus}
        keep = []
        for tok in [t.strip() for t in rocr.split(",") if t.strip()]:
            if tok.isdigit() and int(tok) < len(gpus):
                keep.append(gpus[int(tok)])
                continue
            uid = None
            if tok[:4].upper() == "GPU-":
                try:
                    uid = int(tok[4:], 16)
                except ValueError:
                    uid = None
            if uid is not None and uid in ids:
                keep.append(ids[uid])
            else:
                break
        gpus = keep
    n = len(gpus)
    hip = env.get("HIP_VISIBLE_DEVICES", env.get("CUDA_VISIBLE_DEVICES"))
    if hip is not None:
        count = 0
        for tok in [t.strip() for t in hip.split(",") if t.strip()]:
            if not tok.isdigit() or int(tok) >= n:
                break
            count += 1
        n = count
    return n


def require_devices(n: int, devices: Optional[int] = None) -> int:
    """Raise LaunchError unless at least n GPUs are visible; returns the count.  The count
    is gpu_count()'s (KFD topology, no HIP call): this runs in the parent of the ranks."""
    have = gpu_count() if devices is None else devices
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
