#!/usr/bin/env python3
"""Extract the gfx950 code objects embedded in libswmi355.so (its .hip_fatbin
section holds one clang offload bundle per compiled source) and disassemble them.

    python tools/codeobj.py [lib.so] [out_dir]     -> out_dir/co_<k>.elf + .s

Used by tests/test_abi.py to check the cache-policy bits of the hand-off
instructions without a GPU (the image's roc-obj tools need a Perl module it
lacks)."""
import os
import struct
import subprocess
import sys

MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"
OBJDUMP = "/opt/rocm/lib/llvm/bin/llvm-objdump"


def fatbin(path):
    """Bytes of the .hip_fatbin section (ELF64 little-endian)."""
    data = open(path, "rb").read()
    shoff, = struct.unpack_from("<Q", data, 0x28)
    shentsize, shnum, shstrndx = struct.unpack_from("<HHH", data, 0x3A)
    secs = [struct.unpack_from("<IIQQQQIIQQ", data, shoff + i * shentsize) for i in range(shnum)]
    stroff = secs[shstrndx][4]
    for s in secs:
        name = data[stroff + s[0]:data.index(b"\0", stroff + s[0])]
        if name == b".hip_fatbin":
            return data[s[4]:s[4] + s[5]]
    raise ValueError("no .hip_fatbin section in " + path)


def code_objects(path, arch="gfx950"):
    blob = fatbin(path)
    out = []
    pos = blob.find(MAGIC)
    while pos >= 0:
        n, = struct.unpack_from("<Q", blob, pos + len(MAGIC))
        p = pos + len(MAGIC) + 8
        for _ in range(n):
            off, size, tlen = struct.unpack_from("<QQQ", blob, p)
            triple = blob[p + 24:p + 24 + tlen].decode()
            p += 24 + tlen
            if triple.endswith(arch) and size:
                out.append(blob[pos + off:pos + off + size])
        pos = blob.find(MAGIC, pos + 1)
    return out


def disassemble(path, out_dir):
    os.makedirs(out_dir, exist_ok=True)
    texts = []
    for k, co in enumerate(code_objects(path)):
        elf = os.path.join(out_dir, "co_%d.elf" % k)
        with open(elf, "wb") as f:
            f.write(co)
        txt = subprocess.run([OBJDUMP, "-d", "--no-show-raw-insn", elf], capture_output=True, text=True,
                             check=True).stdout
        with open(elf[:-4] + ".s", "w") as f:
            f.write(txt)
        texts.append(txt)
    return texts


def functions(text):
    """{symbol: [instruction lines]} of an llvm-objdump -d listing.  Local labels of inline asm
    (L_loop_N, L_done_N, ... in the flow3 chunk loops) stay part of the enclosing function."""
    out, cur = {}, None
    for line in text.splitlines():
        if line.endswith(">:") and "<" in line:
            name = line[line.index("<") + 1:-2]
            if name.startswith("L_") and cur is not None:
                continue
            cur = name
            out[cur] = []
        elif cur is not None and line.startswith("\t"):
            out[cur].append(line.strip())
    return out


if __name__ == "__main__":
    lib = sys.argv[1] if len(sys.argv) > 1 else os.path.join(os.path.dirname(__file__), "..", "concurrentproject_amd",
                                                             "libswmi355.so")
    out = sys.argv[2] if len(sys.argv) > 2 else "build/codeobj"
    for t in disassemble(lib, out):
        print(len(t.splitlines()), "lines")
