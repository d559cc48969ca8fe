"""concurrentproject_amd -- MI355X (gfx950) Smith-Waterman score engine.

Python mirror of the reference's score interface (algoGPU.h:1-14 and the
harness calls of TestFileWithGPU.cpp:81-94) over the C-ABI of
``libswmi355.so`` (include/algoGPU.h).  Every call goes to the HIP kernels; there
is no CPU fallback: if the library is missing, importing the engine raises.

    import concurrentproject_amd as sw
    sw.SmithWatermanScoreCUDA(b"GATTACA", b"GCATGCU")      # -> 2
    sw.score_batch([(a0, b0), (a1, b1)])                     # -> [s0, s1]
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass
from typing import Iterable, Sequence

import numpy as np

__all__ = [
    "Params", "lib", "build", "SequentialSmithWatermanScoreGPU", "SmithWatermanLazyGPU",
    "SmithWatermanScoreCUDA", "SmithDiagonalGPU", "score", "score_batch", "score_batch_device",
    "set_params", "get_params", "set_option", "get_option", "last_stats", "gen_pair", "gen_batch",
    "SwError", "LIB_PATH", "SW_FLAG_DNA", "SW_FLAG_BYTES", "slab_bounds", "SlabBuffer", "slab_alloc",
    "ipc_open", "ipc_close", "score_slab_device", "Database",
]

HERE = os.path.dirname(os.path.abspath(__file__))
# SWMI355_LIB selects an instrumented build (tools/trace_flow.py); default: the in-tree library
LIB_PATH = os.environ.get("SWMI355_LIB") or os.path.join(HERE, "libswmi355.so")
SW_FLAG_DNA, SW_FLAG_BYTES = 1, 2


class SwError(RuntimeError):
    """A failed engine call (the C-ABI returned -1); the message is sw_last_error()."""


@dataclass(frozen=True)
class Params:
    """Scoring constants (main.cpp:20-23 defaults)."""
    match: int = 1
    mismatch: int = -1
    gap_init: int = 1
    gap_ext: int = 1


class _Stats(ctypes.Structure):
    _fields_ = [("kernel_ms", ctypes.c_float), ("total_ms", ctypes.c_float), ("cells", ctypes.c_longlong),
                ("W", ctypes.c_int), ("C", ctypes.c_int), ("dna", ctypes.c_int), ("blocks", ctypes.c_int),
                ("waves_per_cu", ctypes.c_int), ("items", ctypes.c_int), ("boundary_bytes", ctypes.c_longlong),
                ("mode", ctypes.c_int), ("variant", ctypes.c_int)]


_lib = None


def build(verbose: bool = False) -> str:
    """Compile libswmi355.so in-tree for gfx950 (hipcc; no GPU needed)."""
    import subprocess
    cmd = ["make", "-j4", "-C", os.path.join(HERE, "csrc")]
    if not verbose:
        cmd.insert(1, "-s")
    subprocess.run(cmd, check=True)
    return LIB_PATH


def source_stamp() -> str:
    """sha256 over the engine's sources and build flags (csrc/*.hip, *.h, *.cpp, Makefile and
    include/algoGPU.h): identifies the kernels a profile was taken with, across rebuilds."""
    import glob
    import hashlib
    h = hashlib.sha256()
    csrc = os.path.join(HERE, "csrc")
    files = sorted(glob.glob(os.path.join(csrc, "*.hip")) + glob.glob(os.path.join(csrc, "*.h")) +
                   glob.glob(os.path.join(csrc, "*.cpp")) + glob.glob(os.path.join(csrc, "*.inc")) +
                   [os.path.join(csrc, "Makefile"), os.path.join(HERE, "..", "include", "algoGPU.h")])
    for f in files:
        h.update(os.path.basename(f).encode())
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()


def lib() -> ctypes.CDLL:
    """The loaded engine.  Raises if libswmi355.so has not been built (no fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError("libswmi355.so not built: run concurrentproject_amd.build() "
                          "(hipcc --offload-arch=gfx950); there is no CPU fallback")
    L = ctypes.CDLL(LIB_PATH)
    u8p = ctypes.POINTER(ctypes.c_ubyte)
    i = ctypes.c_int
    for name in ("SequentialSmithWatermanScoreGPU", "SmithWatermanLazyGPU", "SmithWatermanScoreCUDA",
                 "SmithDiagonalGPU"):
        f = getattr(L, name)
        f.argtypes = [u8p, u8p, i, i]
        f.restype = i
    L.sw_set_params.argtypes = [i, i, i, i]
    L.sw_set_params.restype = i
    L.sw_get_params.argtypes = [ctypes.POINTER(i)] * 4
    L.sw_score_params.argtypes = [u8p, u8p, i, i, i, i, i, i]
    L.sw_score_params.restype = i
    L.sw_score_batch.argtypes = [ctypes.POINTER(u8p), ctypes.POINTER(i), ctypes.POINTER(u8p),
                                 ctypes.POINTER(i), i, ctypes.POINTER(i)]
    L.sw_score_batch.restype = i
    L.sw_score_batch_multi.argtypes = [ctypes.POINTER(u8p), ctypes.POINTER(i), ctypes.POINTER(u8p),
                                       ctypes.POINTER(i), i, ctypes.POINTER(i), i]
    L.sw_score_batch_multi.restype = i
    L.sw_batch_shard.argtypes = [i, i, i, ctypes.POINTER(i), ctypes.POINTER(i)]
    L.sw_batch_shard.restype = i
    if hasattr(L, "sw_batch_gather_plan"):   # (absent from pre-r05 builds that tools/ab.sh --libs may load)
        L.sw_batch_gather_plan.argtypes = [i, i, ctypes.POINTER(i), ctypes.POINTER(i)]
        L.sw_batch_gather_plan.restype = i
    L.sw_score_batch_device.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(i),
                                        ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(i), i, ctypes.c_void_p, i,
                                        ctypes.c_void_p]
    L.sw_score_batch_device.restype = i
    L.sw_stream_status.argtypes = [ctypes.c_void_p]
    L.sw_stream_status.restype = i
    L.sw_set_option.argtypes = [ctypes.c_char_p, ctypes.c_longlong]
    L.sw_set_option.restype = i
    L.sw_get_option.argtypes = [ctypes.c_char_p]
    L.sw_get_option.restype = ctypes.c_longlong
    L.sw_last_stats.argtypes = [ctypes.POINTER(_Stats)]
    L.sw_last_stats.restype = i
    L.sw_last_error.restype = ctypes.c_char_p
    L.sw_version.restype = i
    L.sw_gen_pair.argtypes = [ctypes.c_uint64, i, u8p, u8p]
    L.sw_gen_batch.argtypes = [ctypes.c_uint64, i, i, u8p]
    vp = ctypes.c_void_p
    L.sw_slab_bounds.argtypes = [ctypes.c_longlong, i, i, i, ctypes.POINTER(ctypes.c_longlong)]
    L.sw_slab_bounds.restype = i
    L.sw_score_slab_device.argtypes = [vp, ctypes.c_int64, i, ctypes.c_int64, i, vp, vp, ctypes.c_uint, vp, i, vp]
    L.sw_score_slab_device.restype = i
    L.sw_slab_alloc.argtypes = [i, ctypes.POINTER(vp), ctypes.c_char_p]
    L.sw_slab_alloc.restype = i
    L.sw_slab_free.argtypes = [vp]
    L.sw_slab_free.restype = i
    L.sw_ipc_open.argtypes = [ctypes.c_char_p, ctypes.POINTER(vp)]
    L.sw_ipc_open.restype = i
    L.sw_ipc_close.argtypes = [vp]
    L.sw_ipc_close.restype = i
    # FASTA databases (include/algoGPU.h)
    L.sw_db_open.argtypes = [ctypes.c_char_p]
    L.sw_db_open.restype = vp
    L.sw_db_from_fasta.argtypes = [ctypes.c_char_p, ctypes.c_longlong]
    L.sw_db_from_fasta.restype = vp
    L.sw_db_save.argtypes = [vp, ctypes.c_char_p]
    L.sw_db_save.restype = i
    L.sw_db_count.argtypes = [vp]
    L.sw_db_count.restype = i
    L.sw_db_residues.argtypes = [vp]
    L.sw_db_residues.restype = ctypes.c_longlong
    L.sw_db_record.argtypes = [vp, i, ctypes.POINTER(u8p), ctypes.POINTER(i), ctypes.POINTER(ctypes.c_char_p)]
    L.sw_db_record.restype = i
    L.sw_db_search.argtypes = [vp, u8p, i, ctypes.POINTER(i)]
    L.sw_db_search.restype = i
    L.sw_db_search_db.argtypes = [vp, vp, ctypes.POINTER(i)]
    L.sw_db_search_db.restype = i
    L.sw_db_close.argtypes = [vp]
    L.sw_db_close.restype = None
    _lib = L
    return L


def _u8(a) -> np.ndarray:
    if isinstance(a, str):
        a = a.encode("latin-1")
    if isinstance(a, (bytes, bytearray, memoryview)):
        return np.frombuffer(bytes(a), dtype=np.uint8)
    return np.ascontiguousarray(a, dtype=np.uint8)


def _ptr(arr: np.ndarray):
    return arr.ctypes.data_as(ctypes.POINTER(ctypes.c_ubyte))


def _check(rc: int) -> int:
    if rc < 0:
        raise SwError(lib().sw_last_error().decode(errors="replace"))
    return rc


def _pair_call(fname: str, seq1, seq2) -> int:
    a, b = _u8(seq1), _u8(seq2)
    return _check(getattr(lib(), fname)(_ptr(a), _ptr(b), len(a), len(b)))


# ---- the reference's algoGPU.h surface ----------------------------------------------------

def SequentialSmithWatermanScoreGPU(seq1, seq2) -> int:
    """algoGPU.h:5 (simpleGPU.cu:109): score of (seq1, seq2)."""
    return _pair_call("SequentialSmithWatermanScoreGPU", seq1, seq2)


def SmithWatermanLazyGPU(seq1, seq2) -> int:
    """algoGPU.h:7 (cudaLazy.cu:58)."""
    return _pair_call("SmithWatermanLazyGPU", seq1, seq2)


def SmithWatermanScoreCUDA(seq1, seq2) -> int:
    """algoGPU.h:9 (cudaSmithM.cu:128)."""
    return _pair_call("SmithWatermanScoreCUDA", seq1, seq2)


def SmithDiagonalGPU(seq1, seq2) -> int:
    """SmithDiagonalGPUrefactored.cu:174 (linear gap = G_INIT per residue)."""
    return _pair_call("SmithDiagonalGPU", seq1, seq2)


# ---- extensions ---------------------------------------------------------------------------

def score(seq1, seq2, params: Params | None = None) -> int:
    """Best local-alignment score; ``params`` overrides the process-wide constants for this call."""
    if params is None:
        return SmithWatermanScoreCUDA(seq1, seq2)
    a, b = _u8(seq1), _u8(seq2)
    return _check(lib().sw_score_params(_ptr(a), _ptr(b), len(a), len(b), params.match, params.mismatch,
                                        params.gap_init, params.gap_ext))


def score_batch(pairs: Iterable[Sequence], params: Params | None = None, ngpus: int = 0) -> list:
    """Scores of many independent pairs in one launch (sw_score_batch); with ngpus >= 1,
    sharded over the first ngpus GPUs with an RCCL gather of the scores
    (sw_score_batch_multi)."""
    arrs = [(_u8(a), _u8(b)) for a, b in pairs]
    n = len(arrs)
    if n == 0:
        return []
    u8p = ctypes.POINTER(ctypes.c_ubyte)
    A = (u8p * n)(*[_ptr(x) for x, _ in arrs])
    B = (u8p * n)(*[_ptr(y) for _, y in arrs])
    AL = (ctypes.c_int * n)(*[len(x) for x, _ in arrs])
    BL = (ctypes.c_int * n)(*[len(y) for _, y in arrs])
    out = (ctypes.c_int * n)()
    old = None
    if params is not None:
        old = get_params()
        set_params(params)
    try:
        if ngpus:
            _check(lib().sw_score_batch_multi(A, AL, B, BL, n, out, ngpus))
        else:
            _check(lib().sw_score_batch(A, AL, B, BL, n, out))
    finally:
        if old is not None:
            set_params(old)
    return list(out)


def batch_shard(npairs: int, ngpus: int, rank: int) -> tuple:
    """[lo, hi) of rank `rank`'s contiguous shard in sw_score_batch_multi (no GPU call)."""
    lo, hi = ctypes.c_int(), ctypes.c_int()
    _check(lib().sw_batch_shard(npairs, ngpus, rank, ctypes.byref(lo), ctypes.byref(hi)))
    return lo.value, hi.value


def batch_gather_plan(npairs: int, ngpus: int) -> list:
    """[(count, offset)] per device of sw_score_batch_multi's RCCL gather to device 0 (no GPU call)."""
    cnt, off = (ctypes.c_int * max(ngpus, 1))(), (ctypes.c_int * max(ngpus, 1))()
    _check(lib().sw_batch_gather_plan(npairs, ngpus, cnt, off))
    return [(cnt[r], off[r]) for r in range(ngpus)]


def score_batch_device(d_arena_ptr: int, a_off, alen, b_off, blen, d_scores_ptr: int, flags: int = 0,
                       stream: int | None = None) -> None:
    """Sequences already in device memory (arena pointer + byte offsets).  Asynchronous on ``stream``."""
    npairs = len(alen)
    ao = (ctypes.c_int64 * npairs)(*[int(x) for x in a_off])
    bo = (ctypes.c_int64 * npairs)(*[int(x) for x in b_off])
    al = (ctypes.c_int * npairs)(*[int(x) for x in alen])
    bl = (ctypes.c_int * npairs)(*[int(x) for x in blen])
    _check(lib().sw_score_batch_device(ctypes.c_void_p(d_arena_ptr), ao, al, bo, bl, npairs,
                                       ctypes.c_void_p(d_scores_ptr), flags,
                                       ctypes.c_void_p(stream) if stream else None))


def stream_status(stream: int | None = None) -> None:
    _check(lib().sw_stream_status(ctypes.c_void_p(stream) if stream else None))


# ---- one pair in column slabs across GPUs (dist.ColumnSlabs drives these) -----------------

SW_IPC_HANDLE_BYTES = 64


def slab_bounds(n: int, m: int, nslabs: int, flags: int) -> list:
    """Column bounds [b_0 = 0, ..., b_nslabs = n] of nslabs slabs; every slab but the
    last is a multiple of the planned kernel's column quantum (63 or 64*W)."""
    out = (ctypes.c_longlong * (nslabs + 1))()
    _check(lib().sw_slab_bounds(int(n), int(m), int(nslabs), int(flags), out))
    return [int(x) for x in out]


class SlabBuffer:
    """A slab's inflow edge: m zeroed 16-byte granules in device memory, and the
    IPC handle under which the rank that writes it maps it."""

    def __init__(self, m: int):
        p = ctypes.c_void_p()
        h = ctypes.create_string_buffer(SW_IPC_HANDLE_BYTES)
        kind = _check(lib().sw_slab_alloc(int(m), ctypes.byref(p), h))
        self.ptr = int(p.value)
        self.handle = h.raw
        self.fine_grained = kind == 1
        self.m = m

    def free(self) -> None:
        if self.ptr:
            _check(lib().sw_slab_free(ctypes.c_void_p(self.ptr)))
            self.ptr = 0


def slab_alloc(m: int) -> SlabBuffer:
    return SlabBuffer(m)


def ipc_open(handle: bytes) -> int:
    """Map another process's slab buffer (hipIpcOpenMemHandle); returns its device address here."""
    p = ctypes.c_void_p()
    _check(lib().sw_ipc_open(handle, ctypes.byref(p)))
    return int(p.value)


def ipc_close(ptr: int) -> None:
    if ptr:
        _check(lib().sw_ipc_close(ctypes.c_void_p(ptr)))


def score_slab_device(d_arena_ptr: int, col_off: int, n: int, row_off: int, m: int, d_inflow: int,
                      d_outflow: int, epoch: int, d_score_ptr: int, flags: int, stream: int | None = None) -> None:
    """One column slab (sw_score_slab_device): *d_score = max H over its cells."""
    _check(lib().sw_score_slab_device(ctypes.c_void_p(d_arena_ptr), int(col_off), int(n), int(row_off), int(m),
                                      ctypes.c_void_p(d_inflow) if d_inflow else None,
                                      ctypes.c_void_p(d_outflow) if d_outflow else None, int(epoch),
                                      ctypes.c_void_p(d_score_ptr), int(flags),
                                      ctypes.c_void_p(stream) if stream else None))


def set_params(p: Params) -> None:
    _check(lib().sw_set_params(p.match, p.mismatch, p.gap_init, p.gap_ext))


def get_params() -> Params:
    v = [ctypes.c_int() for _ in range(4)]
    lib().sw_get_params(*[ctypes.byref(x) for x in v])
    return Params(*[x.value for x in v])


def set_option(key: str, value: int) -> None:
    if lib().sw_set_option(key.encode(), int(value)) != 0:
        raise SwError("bad option %s=%r" % (key, value))


def get_option(key: str) -> int:
    return int(lib().sw_get_option(key.encode()))


def last_stats() -> dict:
    s = _Stats()
    lib().sw_last_stats(ctypes.byref(s))
    return {k: getattr(s, k) for k, _ in _Stats._fields_}


def gen_pair(seed: int, length: int) -> tuple:
    """cudaSmithM.cu:200-212 synthetic pair: mt19937_64(seed), a[i] then b[i] over 'ACGT'."""
    a = np.empty(length, dtype=np.uint8)
    b = np.empty(length, dtype=np.uint8)
    lib().sw_gen_pair(seed, length, _ptr(a), _ptr(b))
    return a, b


def gen_batch(seed_base: int, npairs: int, length: int) -> np.ndarray:
    """npairs pairs (pair k seeded seed_base+k) as one arena [a_0|b_0|a_1|b_1|...]."""
    arena = np.empty(2 * length * npairs, dtype=np.uint8)
    lib().sw_gen_batch(seed_base, npairs, length, _ptr(arena))
    return arena


from .db import Database  # noqa: E402  (FASTA databases, query x database search)
