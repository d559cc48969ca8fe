"""FASTA databases and query x database search.

The reference drives database search only through the external CUDASW++4 tool
(timing.sh:3-8: ``makedb SwissProt.fasta benchdb/sp`` then
``align --query q.fa --db benchdb/sp``).  This is the same workflow over the
engine's C-ABI (include/algoGPU.h ``sw_db_*``): the parse, the database file
and the search all run in libswmi355.so; a search is one batch launch over
residues resident in HBM.  Scores are the reference's byte-equality affine
scores (main.cpp:28-66), so ``Database.search(q)[i]`` equals
``SmithWatermanScore(q, record i)``.

    db = Database.open("sp.fasta")          # or a file written by db.save()
    scores = db.search(b"MKTAYIAKQR...")    # one int per record, record order
    db.top(b"MKTAYIAKQR...", k=10)          # [(score, index, header), ...]
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

from . import SwError, _check, _ptr, _u8, lib


class Database:
    """A handle on an ``sw_db`` (records + their residues, host and HBM)."""

    def __init__(self, handle: int):
        if not handle:
            raise SwError(lib().sw_last_error().decode(errors="replace"))
        self._h = ctypes.c_void_p(handle)

    # ---- construction -------------------------------------------------------
    @classmethod
    def open(cls, path: str | os.PathLike) -> "Database":
        """A FASTA file or a database file written by :meth:`save`."""
        return cls(lib().sw_db_open(os.fsencode(path)))

    @classmethod
    def from_fasta(cls, text: bytes | str) -> "Database":
        if isinstance(text, str):
            text = text.encode("latin-1")
        return cls(lib().sw_db_from_fasta(text, len(text)))

    @classmethod
    def from_records(cls, records) -> "Database":
        """From (header, sequence) pairs; headers must not contain a line end."""
        parts = []
        for h, s in records:
            h = h.encode("latin-1") if isinstance(h, str) else bytes(h)
            parts.append(b">" + h + b"\n" + _u8(s).tobytes() + b"\n")
        return cls.from_fasta(b"".join(parts))

    def save(self, path: str | os.PathLike) -> None:
        """The binary database file (the ``makedb`` step)."""
        _check(lib().sw_db_save(self._h, os.fsencode(path)))

    def close(self) -> None:
        if self._h is not None and self._h.value:
            lib().sw_db_close(self._h)
        self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---- records --------------------------------------------------------------
    def __len__(self) -> int:
        return lib().sw_db_count(self._h)

    @property
    def residues(self) -> int:
        return lib().sw_db_residues(self._h)

    def record(self, i: int) -> tuple:
        """(header, residues as bytes) of record i."""
        seq = ctypes.POINTER(ctypes.c_ubyte)()
        n = ctypes.c_int()
        hdr = ctypes.c_char_p()
        _check(lib().sw_db_record(self._h, int(i), ctypes.byref(seq), ctypes.byref(n), ctypes.byref(hdr)))
        return hdr.value.decode("latin-1"), ctypes.string_at(seq, n.value) if n.value else b""

    def length(self, i: int) -> int:
        """Residues of record i (no copy: sw_db_record with seq = NULL)."""
        n = ctypes.c_int()
        _check(lib().sw_db_record(self._h, int(i), None, ctypes.byref(n), None))
        return n.value

    def header(self, i: int) -> str:
        """Header of record i (no residue copy)."""
        hdr = ctypes.c_char_p()
        _check(lib().sw_db_record(self._h, int(i), None, None, ctypes.byref(hdr)))
        return hdr.value.decode("latin-1")

    def lengths(self) -> np.ndarray:
        return np.array([self.length(i) for i in range(len(self))], dtype=np.int64)

    # ---- search ---------------------------------------------------------------
    def search(self, query) -> np.ndarray:
        """int32 score of ``query`` against every record, in record order."""
        q = _u8(query)
        out = np.zeros(len(self), dtype=np.int32)
        _check(lib().sw_db_search(self._h, _ptr(q), len(q), out.ctypes.data_as(ctypes.POINTER(ctypes.c_int))))
        return out

    def search_db(self, queries: "Database") -> np.ndarray:
        """[len(queries), len(self)] int32 scores of every query record against every record."""
        out = np.zeros((len(queries), len(self)), dtype=np.int32)
        _check(lib().sw_db_search_db(self._h, queries._h, out.ctypes.data_as(ctypes.POINTER(ctypes.c_int))))
        return out

    def top(self, query, k: int = 10) -> list:
        """The k best records: [(score, index, header)], score descending, index ascending on ties."""
        sc = self.search(query)
        idx = np.lexsort((np.arange(len(sc)), -sc.astype(np.int64)))[:k]
        return [(int(sc[i]), int(i), self.header(int(i))) for i in idx]
