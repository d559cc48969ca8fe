"""ctypes front-end for the CPU oracle (TEST INFRASTRUCTURE ONLY).

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may import this package.  The product path (``concurrentproject_amd``)
never imports it.

* ``libsworacle.so`` -- the C restatement in ``sw_oracle.c`` (main.cpp:40-90,
  lazySmith.cpp:15-42, std::mt19937_64 + uniform_int_distribution(0,3)).
* ``_ref/libswref*.so`` -- the reference's own main.cpp / lazySmith.cpp compiled
  in place from /root/reference (only present in the build container).
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from dataclasses import dataclass

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(HERE, "libsworacle.so")
_REF_DIR = os.path.join(HERE, "_ref")


class _Params(ctypes.Structure):
    _fields_ = [("match", ctypes.c_int), ("mismatch", ctypes.c_int),
                ("gap_init", ctypes.c_int), ("gap_ext", ctypes.c_int)]


@dataclass(frozen=True)
class Params:
    """Scoring constants; defaults are main.cpp:20-23."""
    match: int = 1
    mismatch: int = -1
    gap_init: int = 1
    gap_ext: int = 1

    def c(self) -> _Params:
        return _Params(self.match, self.mismatch, self.gap_init, self.gap_ext)


DEFAULT = Params()
# constants of the param-substituted reference builds (oracle/Makefile refvar)
REFVAR_PARAMS = (Params(2, -3, 5, 2), Params(1, -1, 3, 1))
_lib = None


def build() -> None:
    """Compile the C restatement (and, when /root/reference exists, oracle/_ref)."""
    subprocess.run(["make", "-s", "-C", HERE, "all"], check=True)
    if os.path.isdir("/root/reference"):
        subprocess.run(["make", "-s", "-C", HERE, "ref"], check=True)
        # param-substituted reference builds (G_INIT != G_EXT), for the long-pair pins
        for prm in REFVAR_PARAMS:
            subprocess.run(["make", "-s", "-C", HERE, "refvar", "MA=%d" % prm.match, "MI=%d" % prm.mismatch,
                            "GI=%d" % prm.gap_init, "GE=%d" % prm.gap_ext], check=True)
        # the reference harness linked against the MI355X library (needs it built)
        if os.path.exists(os.path.join(HERE, "..", "concurrentproject_amd", "libswmi355.so")):
            subprocess.run(["make", "-s", "-C", HERE, "harness"], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        u8p = ctypes.POINTER(ctypes.c_ubyte)
        pp = ctypes.POINTER(_Params)
        for name in ("swo_full", "swo_linear"):
            f = getattr(L, name)
            f.argtypes = [u8p, u8p, ctypes.c_int, ctypes.c_int, pp]
            f.restype = ctypes.c_int
        L.swo_linear_rows.argtypes = [u8p, u8p, ctypes.c_int, ctypes.c_int, pp, ctypes.c_int]
        L.swo_linear_rows.restype = ctypes.c_int
        L.swo_wavefront.argtypes = [u8p, u8p, ctypes.c_int, ctypes.c_int, pp, ctypes.c_int]
        L.swo_wavefront.restype = ctypes.c_int
        L.swo_batch.argtypes = [ctypes.POINTER(u8p), ctypes.POINTER(ctypes.c_int),
                                ctypes.POINTER(u8p), ctypes.POINTER(ctypes.c_int), ctypes.c_int,
                                pp, ctypes.POINTER(ctypes.c_int), ctypes.c_int, ctypes.c_int]
        L.swo_batch.restype = ctypes.c_int
        ip = ctypes.POINTER(ctypes.c_int)
        L.swo_slab.argtypes = [u8p, u8p, ctypes.c_int, ctypes.c_int, pp, ip, ip, ip, ip]
        L.swo_slab.restype = ctypes.c_int
        L.swo_gen_pair.argtypes = [ctypes.c_uint64, ctypes.c_int, u8p, u8p]
        L.swo_mt64_size.restype = ctypes.c_size_t
        L.swo_mt64_seed.argtypes = [ctypes.c_void_p, ctypes.c_uint64]
        L.swo_mt64_next.argtypes = [ctypes.c_void_p]
        L.swo_mt64_next.restype = ctypes.c_uint64
        L.swo_gen_pair_stream.argtypes = [ctypes.c_void_p, ctypes.c_int, u8p, u8p]
        L.swo_gen_seq_stream.argtypes = [ctypes.c_void_p, ctypes.c_int, u8p]
        _lib = L
    return _lib


def as_u8(a) -> np.ndarray:
    """str (latin-1 bytes), bytes or array-like -> contiguous uint8 array."""
    if isinstance(a, str):
        a = a.encode("latin-1")
    if isinstance(a, (bytes, bytearray, memoryview)):
        return np.frombuffer(bytes(a), dtype=np.uint8).copy()
    return np.ascontiguousarray(a, dtype=np.uint8)


def _u8(a) -> tuple:
    arr = as_u8(a)
    return arr, arr.ctypes.data_as(ctypes.POINTER(ctypes.c_ubyte))


def score_full(seq1, seq2, params: Params = DEFAULT) -> int:
    """main.cpp SmithWatermanScore restated (full matrix; O(n*m) memory)."""
    a, pa = _u8(seq1); b, pb = _u8(seq2)
    p = params.c()
    return lib().swo_full(pa, pb, len(a), len(b), ctypes.byref(p))


def score_linear(seq1, seq2, params: Params = DEFAULT, rows: int | None = None) -> int:
    """lazySmith.cpp LazySmith restated (linear space); ``rows`` limits to a row prefix."""
    a, pa = _u8(seq1); b, pb = _u8(seq2)
    p = params.c()
    r = len(b) if rows is None else rows
    return lib().swo_linear_rows(pa, pb, len(a), len(b), ctypes.byref(p), r)


def slab(cols, seq2, params: Params = DEFAULT, edge=None) -> tuple:
    """One column slab (swo_slab): ``cols`` are the slab's columns, ``edge`` the
    (H, E) int32 arrays of the column left of it (None: the matrix border).
    Returns (max H over the slab, (H, E) of its last column)."""
    a, pa = _u8(cols); b, pb = _u8(seq2)
    m = len(b)
    ip = ctypes.POINTER(ctypes.c_int)
    out_h = np.zeros(m, dtype=np.int32); out_e = np.zeros(m, dtype=np.int32)
    if edge is None:
        in_h = in_e = None
    else:
        eh, ee = (np.ascontiguousarray(x, dtype=np.int32) for x in edge)
        in_h, in_e = eh.ctypes.data_as(ip), ee.ctypes.data_as(ip)
    p = params.c()
    best = lib().swo_slab(pa, pb, len(a), m, ctypes.byref(p), in_h, in_e,
                          out_h.ctypes.data_as(ip), out_e.ctypes.data_as(ip))
    if best < 0:
        raise RuntimeError("swo_slab failed")
    return best, (out_h, out_e)


def score_slab(seq1, seq2, lo: int, hi: int, params: Params = DEFAULT) -> tuple:
    """Columns [lo, hi) of seq1 as a slab, with the true left edge (columns [0, lo)
    computed first).  Returns (max H over the slab, its last column's (H, E))."""
    a = as_u8(seq1)
    edge = None if lo == 0 else slab(a[:lo], seq2, params)[1]
    return slab(a[lo:hi], seq2, params, edge)


def score_wavefront(seq1, seq2, params: Params = DEFAULT, threads: int = 8) -> int:
    a, pa = _u8(seq1); b, pb = _u8(seq2)
    p = params.c()
    return lib().swo_wavefront(pa, pb, len(a), len(b), ctypes.byref(p), threads)


def score_batch(pairs, params: Params = DEFAULT, threads: int = 8, full: bool = False) -> list:
    """One pair per thread (CPU baseline for the batched configs)."""
    arrs = [(_u8(a)[0], _u8(b)[0]) for a, b in pairs]
    n = len(arrs)
    u8p = ctypes.POINTER(ctypes.c_ubyte)
    A = (u8p * n)(*[x.ctypes.data_as(u8p) for x, _ in arrs])
    B = (u8p * n)(*[y.ctypes.data_as(u8p) for _, y in arrs])
    AL = (ctypes.c_int * n)(*[len(x) for x, _ in arrs])
    BL = (ctypes.c_int * n)(*[len(y) for _, y in arrs])
    out = (ctypes.c_int * n)()
    p = params.c()
    rc = lib().swo_batch(A, AL, B, BL, n, ctypes.byref(p), out, threads, 1 if full else 0)
    if rc != 0:
        raise RuntimeError("swo_batch failed")
    return list(out)


def similar_pair(seed: int, n: int) -> tuple:
    """A pair with long alignments and long gaps (numpy PCG64, so any machine makes the same
    bytes): b is a copy of random DNA a with 8 % substitutions and an indel of 1..n/256 bases
    every ~n/64 positions, so G_INIT != G_EXT scores run through long E and F legs at any size
    (the generator's uniform pairs score tiny alignments with affine constants)."""
    rng = np.random.default_rng(seed)
    acgt = np.frombuffer(b"ACGT", np.uint8)
    a = acgt[rng.integers(0, 4, n)]
    b = a.copy()
    mut = rng.random(n) < 0.08
    b[mut] = acgt[rng.integers(0, 4, int(mut.sum()))]
    cuts = np.sort(rng.integers(0, n, 64))
    parts, prev = [], 0
    for c in cuts:
        parts.append(b[prev:c])
        ln = int(rng.integers(1, max(2, n // 256)))
        if rng.random() < 0.5:
            prev = min(n, c + ln)                            # deletion
        else:
            parts.append(acgt[rng.integers(0, 4, ln)])       # insertion
            prev = c
    parts.append(b[prev:])
    b = np.concatenate(parts)
    b = np.resize(b, n) if len(b) < n else b[:n]
    return np.ascontiguousarray(a), np.ascontiguousarray(b)


def gen_pair(seed: int, length: int) -> tuple:
    """cudaSmithM.cu:200-212 generator: mt19937_64(seed), a[i] then b[i]."""
    a = np.empty(length, dtype=np.uint8); b = np.empty(length, dtype=np.uint8)
    u8p = ctypes.POINTER(ctypes.c_ubyte)
    lib().swo_gen_pair(seed, length, a.ctypes.data_as(u8p), b.ctypes.data_as(u8p))
    return a, b


class Stream:
    """A persistent std::mt19937_64 for generators that draw several pairs from one engine."""

    def __init__(self, seed: int):
        self._buf = ctypes.create_string_buffer(lib().swo_mt64_size())
        lib().swo_mt64_seed(self._buf, seed)

    def next(self) -> int:
        return lib().swo_mt64_next(self._buf)

    def pair(self, length: int) -> tuple:
        a = np.empty(length, dtype=np.uint8); b = np.empty(length, dtype=np.uint8)
        u8p = ctypes.POINTER(ctypes.c_ubyte)
        lib().swo_gen_pair_stream(self._buf, length, a.ctypes.data_as(u8p), b.ctypes.data_as(u8p))
        return a, b

    def seq(self, length: int) -> np.ndarray:
        s = np.empty(length, dtype=np.uint8)
        lib().swo_gen_seq_stream(self._buf, length, s.ctypes.data_as(ctypes.POINTER(ctypes.c_ubyte)))
        return s


# ---- reference library (build container only) -------------------------------------------

def ref_lib(params: Params = DEFAULT):
    """The reference's own main.cpp/lazySmith.cpp (compiled from /root/reference), or None."""
    if params == DEFAULT:
        path = os.path.join(_REF_DIR, "libswref.so")
    else:
        path = os.path.join(_REF_DIR, "libswref_%d_%d_%d_%d.so" % (
            params.match, params.mismatch, params.gap_init, params.gap_ext))
    if not os.path.exists(path):
        return None
    L = ctypes.CDLL(path)
    u8p = ctypes.POINTER(ctypes.c_ubyte)
    for sym in ("_Z18SmithWatermanScorePhS_ii", "_Z9LazySmithPhS_ii"):
        f = getattr(L, sym)
        f.argtypes = [u8p, u8p, ctypes.c_int, ctypes.c_int]
        f.restype = ctypes.c_int
    return L


def ref_score(seq1, seq2, params: Params = DEFAULT, which: str = "full"):
    L = ref_lib(params)
    if L is None:
        return None
    a, pa = _u8(seq1); b, pb = _u8(seq2)
    sym = "_Z18SmithWatermanScorePhS_ii" if which == "full" else "_Z9LazySmithPhS_ii"
    return getattr(L, sym)(pa, pb, len(a), len(b))
