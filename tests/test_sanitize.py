"""CPU: the host-side C/C++ under AddressSanitizer + UndefinedBehaviorSanitizer
(the reference builds with its sanitizers off,
.vscode/settings.json:53-55).

* the oracle restatement (oracle/sw_oracle.c, `make -C oracle asan`): every engine
  in it -- full matrices, linear space, the threaded wavefront, chained column
  slabs, the threaded batch -- on the KAT table, the raw-byte cases, the param sets
  and empty / one-sided pairs, each against the committed golden score;
* the database parsers and their C-ABI entry points (sw_db_host.cpp, the product's
  own host code, `make -C concurrentproject_amd/csrc asan`): well-formed FASTA and
  database files (with a save -> reopen round trip) and malformed ones (wrapped
  residue count, oversized header length, truncated file, offsets past the end).

Both binaries are built with -fno-sanitize-recover=all, so any finding aborts the
process; the tests also require an empty stderr."""
import json
import os
import struct
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ASAN = os.path.join(ROOT, "build", "asan")
ENV = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1:halt_on_error=1",
           UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")


def _build(target_dir):
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, target_dir), "asan"], check=True)


@pytest.fixture(scope="module")
def oracle_asan():
    _build("oracle")
    return os.path.join(ASAN, "oracle_asan")


@pytest.fixture(scope="module")
def db_asan():
    _build(os.path.join("concurrentproject_amd", "csrc"))
    return os.path.join(ASAN, "db_parse_asan")


def _hex(s):
    return s.hex() if s else "-"


def test_oracle_under_sanitizers(oracle_asan):
    gold = json.load(open(os.path.join(ROOT, "tests", "golden", "kat.json")))
    cases = []
    p0 = gold["params"]
    for c in gold["cases"]:
        cases.append((p0, c["seq1"].encode("latin-1"), c["seq2"].encode("latin-1"), c["score"]))
    for c in gold["byte_cases"]:
        cases.append((p0, bytes.fromhex(c["seq1_hex"]), bytes.fromhex(c["seq2_hex"]), c["score"]))
    for s in json.load(open(os.path.join(ROOT, "tests", "golden", "params.json")))["sets"]:
        for c in s["cases"]:
            cases.append((s["params"], c["seq1"].encode(), c["seq2"].encode(), c["score"]))
    cases += [(p0, b"", b"ACGT", 0), (p0, b"ACGT", b"", 0), (p0, b"", b"", 0), (p0, b"A", b"A", 1)]
    stdin = "".join("%d %d %d %d %s %s\n" % (*p, _hex(a), _hex(b)) for p, a, b, _ in cases)
    r = subprocess.run([oracle_asan], input=stdin, capture_output=True, text=True, timeout=600, env=ENV)
    assert r.returncode == 0, r.stderr[-4000:]
    assert r.stderr == "", r.stderr[-4000:]
    lines = r.stdout.split("\n")[:-1]
    assert len(lines) == len(cases)
    for (p, a, b, exp), line in zip(cases, lines):
        assert [int(x) for x in line.split()] == [exp] * 5, (p, a[:40], b[:40], line)


def _binary_db(records):
    """A database file in sw_db_save's layout (sw_db_host.cpp: magic, u64 count,
    u64 residues, u64 header bytes, {i64 off, i32 len, i32 header length}..., headers,
    residues), from (header, residues) tuples."""
    res = b"".join(r for _, r in records)
    hdr = b"".join(h for h, _ in records)
    out = b"SWMIDB01" + struct.pack("<QQQ", len(records), len(res), len(hdr))
    off = 0
    for h, r in records:
        out += struct.pack("<qii", off, len(r), len(h))
        off += len(r)
    return out + hdr + res


def test_db_parsers_under_sanitizers(db_asan, tmp_path):
    recs = [(b"rec one", b"ACGTACGTTT"), (b"", b""), (b"third", b"MKTAYIAKQR" * 30)]
    good = _binary_db(recs)
    hdr_end = 32 + 16 * len(recs)
    files = {
        # well-formed
        "plain.fa": (b">a\nACGT\nAC GT\n;comment\n>b\r\nTTTT\r\n\n>empty\n", "ok 3 12 "),
        "empty.fa": (b"", "ok 0 0 "),
        "blank.fa": (b"\n\n  \n", "ok 0 0 "),
        "noeol.fa": (b">x\nACG", "ok 1 3 "),
        "good.db": (good, "ok 3 310 "),
        # malformed FASTA
        "before.fa": (b"ACGT\n>a\nAC\n", "error FASTA: sequence data before"),
        # malformed database files
        "truncated.db": (good[:-5], "error database file"),
        "cut_table.db": (good[:40], "error database file"),
        "cut_counts.db": (good[:20], "error database file"),
        "magic_only.db": (b"SWMIDB01", "error database file"),
        "wrapped_nres.db": (good[:16] + struct.pack("<Q", (1 << 64) - 5) + good[24:], "error database file"),
        "huge_count.db": (good[:8] + struct.pack("<Q", 1 << 40) + good[16:], "error database file"),
        "count_past_table.db": (good[:8] + struct.pack("<Q", 1000) + good[16:], "error database file"),
        "oversized_hlen.db": (good[:32 + 12] + struct.pack("<i", 0x7FFFFFFF) + good[32 + 16:], "error database file"),
        "negative_hlen.db": (good[:32 + 12] + struct.pack("<i", -1) + good[32 + 16:], "error database file"),
        "negative_off.db": (good[:32] + struct.pack("<q", -1) + good[40:], "error database file"),
        "off_past_end.db": (good[:32] + struct.pack("<q", (1 << 62)) + good[40:], "error database file"),
        "len_past_end.db": (good[:40] + struct.pack("<i", 0x7FFFFFF0) + good[44:], "error database file"),
        "hbytes_wrong.db": (good[:24] + struct.pack("<Q", 3) + good[32:], "error database file"),
        "extra_bytes.db": (good + b"X", "error database file"),
    }
    assert hdr_end < len(good)
    paths = []
    for name, (data, _) in files.items():
        p = tmp_path / name
        p.write_bytes(data)
        paths.append(str(p))
    r = subprocess.run([db_asan] + paths, capture_output=True, text=True, timeout=300, env=ENV)
    assert r.returncode == 0, r.stderr[-4000:]
    assert r.stderr == "", r.stderr[-4000:]
    lines = r.stdout.split("\n")[:-1]
    assert len(lines) == len(files)
    for (name, (_, want)), line in zip(files.items(), lines):
        assert line.startswith(want), (name, line)
        assert "MISMATCH" not in line, (name, line)
