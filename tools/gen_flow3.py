#!/usr/bin/env python3
"""Generates concurrentproject_amd/csrc/sw_flow3_loops.inc: the chunk loops of the
flow3 kernel (sw_flow3.hip) as hand-scheduled gfx950 assembly, one inline-asm
block per strip role (inflow kind x outflow kind).

    python tools/gen_flow3.py            # rewrite the .inc
    python tools/gen_flow3.py --check    # exit 1 if the committed .inc is stale

Why assembly: for one long pair every instruction of a wavefront step sits on the
critical path of a wave that runs alone on its SIMD (~1.9-2.1 ns per instruction,
DESIGN.md section 8).  The compiled flow2 chunk loop carried 29-78 SALU, 16 s_nop
(the compiler pads every read of an inline-asm result) and 10-35 extra VALU per
32 steps on top of the 304 step instructions.  Here the whole loop over a strip's
chunks is one asm block: the step is flow2's two-columns-per-lane linear-gap step
(sw_flow2.hip step_lin2, main.cpp:54-66 at G_INIT == G_EXT), and the per-chunk
hand-off work is ~20 instructions.

Register use inside the block is fixed (declared as clobbers):
  v64/v65 IO / L0 (they swap roles every step), v66 H_A, v67 max(H_A - G, 0),
  v68 H_B, v69 max(H_B - G, 0), v70/v71 tA/tB, v72/v73 score bytes of 4 rows,
  v74 running max, v[76:83] / v[84:91] row codes of the even / odd chunk,
  v92 inflow rows, v93 producer word, v94 code address, v95 inflow address,
  v96 outflow address, v97 producer word value, v98 consumer word value,
  v99 back-pressure read, v[100:101] granule, v105 granule offset (row * 8),
  v106 masked offset; s40 k0 (the chunk's first lane-0 row), s41 ring offset,
  s43 producer word seen, s44 consumer word seen, s45 failed, s46 slow-path count,
  s[48:49] clock.

Hand-off protocol (positions, words and slots: sw_flow3.hip header).
Hazards handled here (gfx950): a VALU write of a VGPR is >= 2 instructions before
a DPP read of it (the step order guarantees 4-10); no sub-dword (SDWA dst_sel)
writes; every LDS/SMEM result is waited for with an explicit lgkmcnt before use,
and the block drains lgkmcnt/vmcnt before it returns (the compiler does not see
the counters inside).
"""
import os
import sys

R = 512                 # ring rows (sw_flow3.hip F3_R)
BIG = 0x3FFFFFFF        # final producer word: every row available
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "concurrentproject_amd", "csrc", "sw_flow3_loops.inc")

ROLES_IN = ("none", "lds")
MID_AHEAD = int(os.environ.get("F3_MIDAHEAD", "1"))
LOOP_PAD = int(os.environ.get("F3_LOOP_PAD", "0"))
RING_ALIGN = int(os.environ.get("F3_RING_ALIGN", "0"))   # A/B: align the ring loops too
STAGED_PROMOTE = int(os.environ.get("F3_PROMOTE", "1"))   # A/B: staged alignment by VOP3 re-encoding (1) or s_nop only (0)
RING_NOPS = int(os.environ.get("F3_RING_NOPS", "0"))   # A/B: alignment nops in the ring loops (0: re-encodings only)
ROLES_OUT = ("none", "lds", "gran")


# step registers of the staged (C2) loops: H_A, max(H_A - G, 0), H_B, max(H_B - G, 0), tA, tB,
# the score bytes of columns A / B for 4 rows, the running max
STAGED = dict(H="v66", HGO="v67", HB="v68", HGOB="v69", TA="v70", TB="v71", PA="v72", PB="v73", M="v74")


def step(a, io, l0, b, r=STAGED):
    """One anti-diagonal step of the two-column linear-gap step (9 VALU, 128 cells)."""
    a(f"v_add_u32_sdwa {r['TA']}, sext({r['PA']}), {l0} dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_{b} "
      "src1_sel:DWORD")
    a(f"v_add_u32_sdwa {r['TB']}, sext({r['PB']}), {r['H']} dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_{b} "
      "src1_sel:DWORD")
    a(f"v_mov_b32_dpp {l0}, {io} wave_shl:1 row_mask:0xf bank_mask:0xf")
    a(f"v_add_u32_dpp {io}, {r['HB']}, %[ng] wave_shr:1 row_mask:0xf bank_mask:0xf")
    a(f"v_max3_i32 {r['H']}, {io}, {r['HGO']}, {r['TA']}")
    a(f"v_sub_u32_e64 {r['HGO']}, {r['H']}, %[G] clamp")
    a(f"v_max3_i32 {r['HB']}, {r['HGO']}, {r['HGOB']}, {r['TB']}")
    a(f"v_sub_u32_e64 {r['HGOB']}, {r['HB']}, %[G] clamp")
    a(f"v_max3_i32 {r['M']}, {r['M']}, {r['TA']}, {r['TB']}")



# ---- 8-byte alignment of the chunk loops ----------------------------------------------------
# A lone wave issues an 8-byte instruction (VOP3, DPP, SDWA, DS, buffer, VOP2 + literal) more
# slowly when it sits at an address = 4 mod 8: C2's flow3 kernel ran 2.76 ms with 82 % of its
# main loop's 8-B instructions there and 2.545 ms with 18 % (the same code shifted by one 4-B
# s_nop; profiles/r05_ab_align.md).  So every loop is laid out from its 64-B aligned label with
# all 8-B instructions on 8-B boundaries: before an 8-B instruction that would land at 4 mod 8,
# the nearest 4-B VOP1/VOP2 instruction since the previous 8-B one is re-encoded as VOP3 (_e64,
# 8 B, same operation), or, when that run holds none (SALU, waits), one s_nop 0 is inserted.
# Instruction sizes come from llvm-mc (gfx950), with each operand placeholder replaced by a
# register of its class.  Staged loops only: the ring loops (4 waves per SIMD, issue-bound)
# measured 1.5 % slower aligned (C5 166.6 -> 168.7 ms), the nops costing issue slots there.
LLVM_MC = "/opt/rocm/lib/llvm/bin/llvm-mc"
OPERAND_CLASS = {
    "rsrc": "s[0:3]", "rrs": "s[0:3]", "girs": "s[0:3]", "gors": "s[0:3]", "cross": "s[0:3]", "bpr": "s[0:3]",
    "m48": "s[0:1]", "lhi": "s[0:1]",
    "G": "s0", "GI": "s0", "GE": "s0", "k80": "s0", "end": "s0", "dlo": "s0", "dhi": "s0", "ek": "s0", "ek2": "s0",
    "m": "s0", "gimask8": "s0", "gomask8": "s0", "gimask16": "s0", "gomask16": "s0", "crv0": "s0", "bpbase": "s0",
    "fail": "s0", "slow": "s0", "ekp": "s0", "ek2p": "s0", "m16": "s[0:1]", "l63": "s[0:1]",
}
_SIZE_CACHE = {}
_PROMOTABLE = ("v_mov_b32", "v_add_u32", "v_sub_u32", "v_subrev_u32", "v_xor_b32", "v_max_i32", "v_max_u32",
               "v_min_i32", "v_lshrrev_b32", "v_lshlrev_b32", "v_and_b32", "v_or_b32", "v_cndmask_b32")


def _norm(line):
    import re
    return re.sub(r"%\[(\w+)\]", lambda m: OPERAND_CLASS.get(m.group(1), "v0"), line).replace("%=", "0")


def _is_code(line):
    t = line.strip()
    return t and not t.endswith(":") and not t.startswith(".")


def _sizes(lines):
    import re
    import subprocess
    todo = sorted({_norm(l) for l in lines if _is_code(l) and not l.startswith(("s_cbranch", "s_branch"))} -
                  set(_SIZE_CACHE))
    if todo:
        r = subprocess.run([LLVM_MC, "-arch=amdgcn", "-mcpu=gfx950", "-show-encoding"], input="\n".join(todo) + "\n",
                           capture_output=True, text=True, check=True)
        enc = [l for l in r.stdout.splitlines() if "encoding:" in l]
        assert len(enc) == len(todo), (len(enc), len(todo), r.stderr[:2000])
        for t, e in zip(todo, enc):
            _SIZE_CACHE[t] = len(re.search(r"encoding: \[(.*)\]", e).group(1).split(","))
    return [0 if not _is_code(l) else 4 if l.startswith(("s_cbranch", "s_branch")) else _SIZE_CACHE[_norm(l)]
            for l in lines]


def align8(lines, nops=True, promote=True):
    """The loop of an asm block (from its 64-B aligned L_loop label to the loop's back branch)
    with every 8-B instruction on an 8-B boundary (see above); nops = False: re-encodings only
    (an 8-B instruction after a run without a promotable one stays where it is); promote =
    False: s_nop padding only."""
    try:
        i0 = lines.index("L_loop_%=:")
        i1 = lines.index("s_cbranch_scc1 L_loop_%=")
    except ValueError:
        return lines
    body = lines[i0 + 1:i1]
    sz = _sizes(body)
    out, off, cand = [], 0, None        # cand: index in out of the last promotable 4-B VALU since an 8-B one
    for l, n in zip(body, sz):
        if n == 8 and off % 8 == 4:
            if cand is not None and promote:
                op, rest = out[cand].split(" ", 1)
                out[cand] = op + "_e64 " + rest
                off += 4
            elif nops:
                out.append("s_nop 0")
                off += 4
            cand = None
        out.append(l)
        off += n
        if n == 8:
            cand = None
        elif n == 4 and l.split(" ", 1)[0] in _PROMOTABLE:
            cand = len(out) - 1
    return lines[:i0 + 1] + out + lines[i1:]


def granule(a, rows):
    """Publish the `rows` newest outflow rows (lanes 64-rows..63 of the IO register v64,
    mask %[m48]) as 8-B granules {H-G, (H-G) ^ epoch ^ 0x5BD1E995} at row * 8 of the group
    edge, write-through (sw_flow3.hip header).  v105 = this lane's row * 8 (rows < 0 wrap
    to huge offsets: dropped by the buffer range check, as are rows past 2m)."""
    a("v_mov_b32 v100, v64")
    a("v_xor_b32 v101, %[ek], v64")
    a("v_cndmask_b32_e64 v106, -16, v105, %[m48]")
    a(f"v_add_u32 v105, {rows * 8:#x}, v105")    # (an independent VALU between the data writes and the store)
    a("buffer_store_dwordx2 v[100:101], v106, %[rsrc], 0 offen sc1")


def gen_role(IN, OUT_, spec=0, halfpub=True, C=32, hl=False):
    """The staged loop of one strip role at C-row chunks (C = 32 or 16).  hl: the LDS links
    hand off every half chunk (C = 32): the producer publishes its newest 16 rows at mid-chunk
    too, the consumer starts a chunk once its first 16 rows are in and takes the other 16 at
    mid-chunk (into lanes 0..15 of the I/O register, where the chunk-top rows 16..31 have
    rotated), so a link lags 63 + 16 steps at C = 32's per-chunk work.  At mid-chunk only lanes
    48..63 hold outflow (the chunk top replaced the whole IO register, so lanes 32..47 hold its
    inflow): the mid publish sends lanes 32..47 32 rows on (%[lmid]), onto write-ahead slots,
    never over rows the top already published.  Progress words count
    rows available - H (H = C/2 with hl, else C); the consumer's word counts rows consumed + R."""
    L = []
    a = L.append
    lds_in, lds_out, gran = IN == "lds", OUT_ == "lds", OUT_ == "gran"
    H = C // 2 if hl else C
    nd = C // 4                         # row-code dwords per chunk
    ncr = nd // 4                       # their 16-B LDS reads
    nw = 2 if lds_out else 0            # LDS writes of a chunk's publish (ring + mirror in one, the word)
    grows = C // 2 if halfpub else C    # rows per granule publish
    assert not hl or (C == 32 and spec == 4)
    # ---- entry (s_nop 4: the "s" operands may be fresh from v_readfirstlane, and buffer
    # instructions read them as descriptors: 5 wait states)
    a("s_nop 4")
    a("s_waitcnt vmcnt(0) lgkmcnt(0)")
    for r in ("v66", "v67", "v68", "v69", "v74"):
        a(f"v_mov_b32 {r}, 0")
    a("v_mov_b32 v64, %[ng]")
    a("v_mov_b32 v65, %[ng]")
    a("v_mov_b32 v94, %[code]")
    a("s_mov_b32 s40, 0")
    a(f"s_movk_i32 s41, {(64 - C) * 4:#x}")       # ((k0 + 64 - C) mod R) * 4 at k0 = 0
    a("s_mov_b32 s45, 0")
    a("s_mov_b32 s46, 0")
    a(f"s_movk_i32 s44, {R}")            # consumer word seen: 0 rows consumed (+ R)
    if lds_out:
        a(f"v_mov_b32 v97, {-64 - H}")   # producer word at chunk 0: k0 - 64 rows out, minus H
        a("v_add_u32 v96, s41, %[lout]")
    if lds_in:
        a(f"v_mov_b32 v98, {R + H}")     # consumer word after chunk 0's top: H rows consumed (+ R)
        a("v_add_u32 v95, s41, %[lin]")
        if hl:
            a("s_mov_b32 s50, 0xffff")   # lanes 0..15: the mid-chunk inflow rows
            a("s_mov_b32 s51, 0")
    if gran:
        a("v_mov_b32 v105, %[lrow]")
    for q in range(ncr):
        a(f"ds_read_b128 v[{76 + 4 * q}:{79 + 4 * q}], v94 offset:{16 * q}")
    if lds_in and spec:
        a("ds_read_b32 v93, %[pin]")
        a("ds_read_b32 v92, v95")
    a(".p2align 6")                # the chunk loop on a 64-B boundary (a lone wave's issue rate depends on it)
    for _ in range(LOOP_PAD):
        a("s_nop 0")
    a("L_loop_%=:")
    for p in (0, 1):
        cur = 76 if p == 0 else 84
        nxt = 84 if p == 0 else 76
        obase = C if p == 0 else 2 * C
        # ---- chunk top: publish the last chunk's outflow, take this chunk's inflow
        if lds_in and not spec:
            a("ds_read_b32 v93, %[pin]")
            a("ds_read_b32 v92, v95")
        if lds_out:
            if p == 0:   # back-pressure for this chunk's and the next chunk's publish
                if hl:   # (whose mid-chunk write-ahead lanes reach 16 rows further)
                    a(f"s_add_u32 s52, s40, {H}")
                    a("s_cmp_lt_i32 s44, s52")
                else:
                    a("s_cmp_lt_i32 s44, s40")
                a(f"s_cbranch_scc1 L_bp{p}_%=")
                a(f"L_bpr{p}_%=:")
            a(f"ds_write2st64_b32 v96, v64, v64 offset1:{R * 4 // 256}")   # the row and its mirror copy
            a("ds_write_b32 %[pout], v97")
        if gran:
            granule(a, grows)
        for q in range(ncr):
            a(f"ds_read_b128 v[{nxt + 4 * q}:{nxt + 4 * q + 3}], v94 offset:{obase + 16 * q}")
        if lds_in:
            after = 1 + nw + ncr         # LDS ops issued after the producer-word read
            a(f"s_waitcnt lgkmcnt({after})")
            a("v_readfirstlane_b32 s43, v93")
            a("s_cmp_lt_i32 s43, s40")
            a(f"s_cbranch_scc1 L_in{p}_%=")
            a(f"L_inr{p}_%=:")
            a(f"s_waitcnt lgkmcnt({after - 1})")
            a("v_mov_b32 v64, v92")
            a("ds_write_b32 %[qme], v98")
        else:
            a(f"s_waitcnt lgkmcnt({nw + ncr})")
            a("v_mov_b32 v64, %[ng]")
        # ---- C steps, C/4 groups of 4 rows (one v_perm_b32 per column per group)
        ng = C // 4
        spec_at = ng - spec // 4 if spec else None
        for u in range(ng):
            if spec and u == spec_at:
                book(a, p, lds_in, lds_out, C, H)
                a("ds_read_b32 v93, %[pin]")
                a("ds_read_b32 v92, v95")
            if hl and lds_in and u == ng // 2 - MID_AHEAD:
                # the second half's rows, read 4 steps ahead behind the producer's word
                a("ds_read_b32 v93, %[pin]")
                a(f"ds_read_b32 v102, v95 offset:{4 * H}")
            if hl and u == ng // 2:
                # ---- mid-chunk: the newest 16 outflow rows out, the chunk's other 16 rows in
                if lds_out:
                    a("v_add_u32 v103, %[lmid], v96")   # lanes 32..47 (the chunk top's inflow) 32 rows on
                    a(f"v_add_u32 v97, {H}, v97")
                    a(f"ds_write2st64_b32 v103, v64, v64 offset1:{R * 4 // 256}")
                    a("ds_write_b32 %[pout], v97")
                if lds_in:
                    a(f"s_waitcnt lgkmcnt({1 + (2 if lds_out else 0)})")
                    a("v_readfirstlane_b32 s43, v93")
                    if not (lds_out and p == 0):   # (the chunk top's back-pressure check set s52 = k0 + H)
                        a(f"s_add_u32 s52, s40, {H}")
                    a("s_cmp_lt_i32 s43, s52")
                    a(f"s_cbranch_scc1 L_mid{p}_%=")
                    a(f"L_midr{p}_%=:")
                    a(f"s_waitcnt lgkmcnt({2 if lds_out else 0})")
                    a("v_cndmask_b32_e64 v64, v64, v102, s[50:51]")
            # score bytes of 4 rows: selectors 4..7 pick pA (row symbols 0..3), 0..3 pick qA (0: no row,
            # 0x80; 1..3: row symbols 4..6 of a seven-letter alphabet, sw_flow3.hip HEP; DNA: 0x80808080)
            a(f"v_perm_b32 v72, %[pA], %[qA], v{cur + u}")
            a(f"v_perm_b32 v73, %[pB], %[qB], v{cur + u}")
            for b in range(4):
                io, l0 = ("v64", "v65") if b % 2 == 0 else ("v65", "v64")
                step(a, io, l0, b)
            if gran and halfpub and u == ng // 2 - 1:
                granule(a, grows)
        if not spec:
            book(a, p, lds_in, lds_out, C, H)
    a("s_cmp_lt_i32 s40, %[end]")
    a("s_cbranch_scc1 L_loop_%=")
    # ---- exit: the last chunk's outflow, then every row is out
    if lds_out:
        a("s_cmp_lt_i32 s44, s40")
        a("s_cbranch_scc1 L_bpx_%=")
        a("L_bpxr_%=:")
        a(f"ds_write2st64_b32 v96, v64, v64 offset1:{R * 4 // 256}")
        a(f"v_mov_b32 v97, {BIG:#x}")
        a("ds_write_b32 %[pout], v97")
    if gran:
        granule(a, grows)
    a("s_waitcnt vmcnt(0) lgkmcnt(0)")
    a("v_mov_b32 %[M], v74")
    a("s_mov_b32 %[fail], s45")
    a("s_mov_b32 %[slow], s46")
    a("s_branch L_done_%=")
    # ---- slow paths (a late producer word, or a full ring): bounded spins
    if lds_in:
        for p in (0, 1):
            slow_wait(a, f"L_in{p}_%=", f"L_inr{p}_%=", "v93", "%[pin]", "s43", reread="ds_read_b32 v92, v95")
            if hl:
                slow_wait(a, f"L_mid{p}_%=", f"L_midr{p}_%=", "v93", "%[pin]", "s43",
                          reread=f"ds_read_b32 v102, v95 offset:{4 * H}", target="s52")
    if lds_out:
        slow_wait(a, "L_bp0_%=", "L_bpr0_%=", "v99", "%[qnx]", "s44", target="s52" if hl else "s40")
        slow_wait(a, "L_bpx_%=", "L_bpxr_%=", "v99", "%[qnx]", "s44")
    a("L_done_%=:")
    return L


def book(a, p, lds_in, lds_out, C=32, H=None):
    """Advance k0, the ring offset and the words to the next chunk (H: rows a half-chunk
    publish already added to the producer word)."""
    H = C if H is None else H
    a(f"s_add_i32 s40, s40, {C}")
    a(f"s_add_u32 s41, s41, {4 * C:#x}")
    a(f"s_and_b32 s41, s41, {(R - 1) * 4:#x}")
    if lds_out:
        a("v_add_u32 v96, s41, %[lout]")
        a(f"v_add_u32 v97, {C if H == C else C - H}, v97")
    if lds_in:
        a("v_add_u32 v95, s41, %[lin]")
        a(f"v_add_u32 v98, {C}, v98")
    if p == 1:
        a(f"v_add_u32 v94, {2 * C}, v94")


def slow_wait(a, label, resume, vreg, addr, sreg, reread=None, target="s40"):
    """Re-read a progress word until it reaches `target` (k0, or k0 + 16 at a half-chunk
    link's mid-chunk), then resume; after the deadline (or once failed) give up: s45 = 1 and
    the kernel reports ERR_TIMEOUT."""
    a(f"{label}:")
    a("s_add_u32 s46, s46, 1")
    a("s_cmp_lg_u32 s45, 0")
    a(f"s_cbranch_scc1 {resume}")
    a(f"{label}_w:")
    a(f"ds_read_b32 {vreg}, {addr}")
    if reread:
        a(reread)
    a("s_waitcnt lgkmcnt(0)")
    a(f"v_readfirstlane_b32 {sreg}, {vreg}")
    a(f"s_cmp_ge_i32 {sreg}, {target}")
    a(f"s_cbranch_scc1 {resume}")
    slow_timeout(a, label)
    a(f"{label}_x:")
    a("s_mov_b32 s45, 1")
    a(f"s_branch {resume}")


CLOBBERS = ['"v%d"' % r for r in range(64, 107) if r not in (75, 104)] + \
    ['"s%d"' % r for r in range(40, 53) if r != 42 and r != 47] + ['"scc"', '"vcc"', '"memory"']


def emit(spec=0, halfpub=True):
    out = ["// GENERATED by tools/gen_flow3.py -- do not edit.  The flow3 chunk loops (sw_flow3.hip):",
           "// one inline-asm block per (chunk rows C, half-chunk LDS links HL, strip role), R = %d ring rows, SPEC = %d, HALFPUB = %d."
           % (R, spec, halfpub),
           "// Operands: see F3Loop in sw_flow3.hip; fixed registers: tools/gen_flow3.py.",
           "#pragma once", ""]
    for C, hl in ((32, 0), (16, 0), (32, 1)):
        for IN in ROLES_IN:
            for OUT_ in ROLES_OUT:
                body = align8(gen_role(IN, OUT_, spec, halfpub, C, bool(hl)), promote=STAGED_PROMOTE)
                out.append("template <> __device__ __forceinline__ F3Res f3_loop<%d, %d, F3_%s, F3_%s>(const F3Loop& x) {"
                           % (C, hl, IN.upper(), OUT_.upper()))
                out.append("    F3Res r;")
                out.append("    asm volatile(")
                for line in body:
                    out.append('        "%s\\n\\t"' % line)
                out.append('        : [M] "=v"(r.M), [fail] "=s"(r.fail), [slow] "=s"(r.slow)')
                out.append('        : [pA] "v"(x.pA), [pB] "v"(x.pB), [ng] "v"(x.ng), [G] "s"(x.G), [qA] "v"(x.qA),')
                out.append('          [qB] "v"(x.qB), [code] "v"(x.code), [lin] "v"(x.lin), [lout] "v"(x.lout), [pin] "v"(x.pin),')
                out.append('          [pout] "v"(x.pout), [qme] "v"(x.qme), [qnx] "v"(x.qnx), [end] "s"(x.end),')
                out.append('          [dlo] "s"(x.dlo), [dhi] "s"(x.dhi), [rsrc] "s"(x.rsrc), [ek] "s"(x.ek),')
                out.append('          [lrow] "v"(x.lrow), [m48] "s"(x.m48), [lmid] "v"(x.lmid)')
                out.append("        : " + ", ".join(CLOBBERS) + ");")
                out.append("    return r;")
                out.append("}")
                out.append("")
    return "\n".join(out)

# ============================================================================================
# Ring mode (C5: one pair N = 2^20, rows streamed, group edges through per-block rings):
# sw_flow3.hip sw_flow3r_kernel, sw_flow3r_loops.inc.  C = 64 or 32, no loader wave, up to 4
# workgroups per CU (the block's fixed registers stay below v108 so that 128 VGPRs suffice).
#   v40/v41 IO / L0, v42..v50 step (RING below), v[52:67] / v[68:83] row codes of the even /
#   odd chunk, v[84:85] granule inflow {H-G, key} (IN=GRAN) or LDS inflow row (v84), v86
#   producer word read, v87 code read address, v88 / v89 LDS inflow / outflow address,
#   v90 / v91 producer / consumer word values, v92 back-pressure read, v93 raw row byte,
#   v94 row code, v95 code write address, v[96:97] granule outflow, v98 its slot offset,
#   v99 its masked offset, v100 its position << 5, v101 granule inflow offset, v102 its
#   position << 5, v103 scratch, v104 consumer report, v105 code read offset, v106 raw row,
#   v107 granule outflow row;  s40 k0, s41 / s42 LDS out / in ring offset, s43 producer word,
#   s44 LDS consumer word, s45 failed, s46 slow-path count, s[48:49] clock, s[50:51] /
#   s[56:57] masks, s52 HBM consumer word, s53 code slot base, s54 / s55 scratch, s[58:59]
#   live lanes.
# Granules (ring edges): 8 B {H-G, (H-G) ^ epoch ^ 0x5BD1E995 ^ (position << 5)} at slot * 8;
# the position term rejects a slot still holding an earlier round's row (same epoch).
# ============================================================================================
RR = int(os.environ.get("F3_RR", "512"))   # LDS ring rows per in-workgroup link (sw_flow3.hip F3R_R)
RING = dict(H="v42", HGO="v43", HB="v44", HGOB="v45", TA="v46", TB="v47", PA="v48", PB="v49", M="v50")
# three columns per lane (ring mode, sw_flow3.hip flow3_ring<..., W3>): column C's H, max(H_C - G, 0),
# its t of even / odd steps and score bytes
RING3 = dict(RING, HC="v108", HGOC="v109", TC0="v110", TC1="v111", PC="v112")


# four and five columns per lane (ring mode, sw_flow3.hip flow3_ring<..., W45>: C5-sized pairs whose
# three-column strips outnumber the resident slots): column D's H, max(H_D - G, 0), t, score bytes;
# column E's H, max(H_E - G, 0), t of even / odd steps, score bytes.  The kernel's fixed registers stay
# below v122 (128 VGPRs: 4 waves per SIMD).
RING4 = dict(RING3, TC="v110", HD="v113", HGOD="v114", TD="v115", PD="v116")
RING5 = dict(RING4, HE="v117", HGOE="v118", TE0="v119", TE1="v120", PE="v121")
COLS = "ABCDE"


def colreg(r, c, what):
    """Register of column c (0..4) in a ring step map: what in H, HGO, P."""
    if c == 0:
        return {"H": r["H"], "HGO": r["HGO"], "P": r["PA"]}[what]
    return r[what + COLS[c]]


def step_w(a, io, l0, b, r, W):
    """One anti-diagonal step of the W-column linear-gap step (W = 4, 5; 64 W cells): step3 with
    more columns.  Every column's t first (column c's diagonal is column c-1's H of the last
    step), then the lane hand-off of the last column, then the column chain left to right
    (H_c = max3(left, up, t_c), HGO_c = max(H_c - G, 0)); the running max takes the t's in pairs
    (A,B), (C,D) every step and, at W = 5, column E's t of two steps on odd steps."""
    assert W in (4, 5)
    t = ["v46", "v47", "v110", "v115"] + ([r["TE1"] if b % 2 else r["TE0"]] if W == 5 else [])
    diag = [l0] + [colreg(r, c, "H") for c in range(W - 1)]
    for c in range(W):
        a(f"v_add_u32_sdwa {t[c]}, sext({colreg(r, c, 'P')}), {diag[c]} dst_sel:DWORD dst_unused:UNUSED_PAD "
          f"src0_sel:BYTE_{b} src1_sel:DWORD")
    a(f"v_mov_b32_dpp {l0}, {io} wave_shl:1 row_mask:0xf bank_mask:0xf")
    a(f"v_add_u32_dpp {io}, {colreg(r, W - 1, 'H')}, %[ng] wave_shr:1 row_mask:0xf bank_mask:0xf")
    left = io
    for c in range(W):
        a(f"v_max3_i32 {colreg(r, c, 'H')}, {left}, {colreg(r, c, 'HGO')}, {t[c]}")
        a(f"v_sub_u32_e64 {colreg(r, c, 'HGO')}, {colreg(r, c, 'H')}, %[G] clamp")
        left = colreg(r, c, "HGO")
    a(f"v_max3_i32 {r['M']}, {r['M']}, {t[0]}, {t[1]}")
    a(f"v_max3_i32 {r['M']}, {r['M']}, {t[2]}, {t[3]}")
    if W == 5 and b % 2:
        a(f"v_max3_i32 {r['M']}, {r['M']}, {r['TE0']}, {r['TE1']}")


def step3(a, io, l0, b, r):
    """One anti-diagonal step of the three-column linear-gap step (12.5 VALU, 192 cells): columns
    A, B, C = 3 lane, + 1, + 2; the left input of A is lane l-1's column C (the DPP-add), of B and
    C the clamped H - G of A and B in the same lane; the running max takes column C's t of two
    steps in one max3 (odd steps)."""
    tc = r["TC1"] if b % 2 else r["TC0"]
    a(f"v_add_u32_sdwa {r['TA']}, sext({r['PA']}), {l0} dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_{b} "
      "src1_sel:DWORD")
    a(f"v_add_u32_sdwa {r['TB']}, sext({r['PB']}), {r['H']} dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_{b} "
      "src1_sel:DWORD")
    a(f"v_add_u32_sdwa {tc}, sext({r['PC']}), {r['HB']} dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_{b} "
      "src1_sel:DWORD")
    a(f"v_mov_b32_dpp {l0}, {io} wave_shl:1 row_mask:0xf bank_mask:0xf")
    a(f"v_add_u32_dpp {io}, {r['HC']}, %[ng] wave_shr:1 row_mask:0xf bank_mask:0xf")
    a(f"v_max3_i32 {r['H']}, {io}, {r['HGO']}, {r['TA']}")
    a(f"v_sub_u32_e64 {r['HGO']}, {r['H']}, %[G] clamp")
    a(f"v_max3_i32 {r['HB']}, {r['HGO']}, {r['HGOB']}, {r['TB']}")
    a(f"v_sub_u32_e64 {r['HGOB']}, {r['HB']}, %[G] clamp")
    a(f"v_max3_i32 {r['HC']}, {r['HGOB']}, {r['HGOC']}, {tc}")
    a(f"v_sub_u32_e64 {r['HGOC']}, {r['HC']}, %[G] clamp")
    a(f"v_max3_i32 {r['M']}, {r['M']}, {r['TA']}, {r['TB']}")
    if b % 2:
        a(f"v_max3_i32 {r['M']}, {r['M']}, {r['TC0']}, {r['TC1']}")


def ring_granule(a, key="%[ek]", cp="sc1"):
    """Publish lanes 32..63 of IO (the 32 newest outflow rows, row v107) as 8-B granules
    at their ring slots, rows outside [0, m) dropped.  A slab's outflow to the next GPU
    (OUT = peer): key %[ekp], system scope (sc0 sc1)."""
    a("v_mov_b32 v96, v40")
    a(f"v_xor_b32 v97, {key}, v40")
    a("v_xor_b32 v97, v97, v100")
    a("v_cmp_gt_u32_e64 s[50:51], %[m], v107")          # 0 <= row < m (unsigned)
    a("s_and_b64 s[50:51], s[50:51], %[lhi]")
    a("v_cndmask_b32_e64 v99, -16, v98, s[50:51]")
    a("v_add_u32 v98, 0x100, v98")                      # 32 rows on
    a("v_and_b32 v98, %[gomask8], v98")
    a("v_add_u32 v100, 0x400, v100")
    a("v_add_u32 v107, 32, v107")
    a(f"buffer_store_dwordx2 v[96:97], v99, %[gors], 0 offen {cp}")


def ring_gin_check(a, C=64, key="%[ek]"):
    """s[58:59] = live lanes (lane < C, row k0 + lane < m); s[50:51] = live lanes whose granule fails."""
    a("s_sub_i32 s54, %[m], s40")
    if C < 64:
        a(f"s_min_i32 s54, s54, {C}")
    a("v_cmp_gt_i32_e64 s[58:59], s54, %[lane]")
    a("v_xor_b32 v103, v84, v85")
    a("v_xor_b32 v103, v103, v102")
    a(f"v_cmp_ne_u32_e64 s[56:57], {key}, v103")
    a("s_and_b64 s[50:51], s[58:59], s[56:57]")
    a("s_cmp_lg_u64 s[50:51], 0")


def gen_role_ring(IN, OUT_, C=64, hl=False, W=2, hep=False):
    """The ring-mode loop of one strip role at C-row chunks (64, or 32: half the hand-off
    lag).  The loop body is two chunks; the code ring is refilled 64 rows per body.
    hl (C = 64): half-chunk LDS links as in gen_role: the producer also publishes its newest
    32 rows (lanes 32..63) at mid-chunk, lanes 0..31 (the chunk top's inflow) onto the
    write-ahead slots 64 rows on (%[lmid] from the ring offset of chunk k0 + 64); the consumer
    starts a chunk on its first 32 rows and merges the other 32 into lanes 0..31 at mid-chunk.
    Words count rows available - 32; the back-pressure floor is k0 + 64 (the next mid-chunk's
    write-ahead).
    hep: a pair over up to seven byte values (sw_flow3.hip HEP): the streamed rows are already
    perm selectors (translated by the engine; 0 past the last row), so the refill writes them
    as they are, and the perms take each column's low word %[qA] / %[qB] / %[qC]."""
    L = []
    a = L.append
    lds_in, lds_out = IN == "lds", OUT_ == "lds"
    # granule inflow / outflow: ring edges (gran, device scope) or a column slab's edge to / from
    # another GPU (peer: system scope sc0 sc1, the slab key %[ekp]; linear edges, no back-pressure)
    gin, gout = IN in ("gran", "peer"), OUT_ in ("gran", "peer")
    kin, cin = ("%[ekp]", "sc0 sc1") if IN == "peer" else ("%[ek]", "sc1")
    kout, cout = ("%[ekp]", "sc0 sc1") if OUT_ == "peer" else ("%[ek]", "sc1")
    assert not hl or C == 64
    H = C // 2 if hl else C
    ncr = C // 16                                      # 16-B code reads per chunk
    # ---- entry (s_nop 4: descriptor operands may be fresh from v_readfirstlane)
    a("s_nop 4")
    a("s_waitcnt vmcnt(0) lgkmcnt(0)")
    assert W in (2, 3, 4, 5) and (W == 2 or (C == 64 and not hl))
    zero = ("v42", "v43", "v44", "v45", "v50") + (("v108", "v109") if W >= 3 else ()) + \
        (("v113", "v114") if W >= 4 else ()) + (("v117", "v118") if W == 5 else ())
    for r in zero:
        a(f"v_mov_b32 {r}, 0")
    a("v_mov_b32 v40, %[ng]")
    a("v_mov_b32 v41, %[ng]")
    a("v_mov_b32 v93, %[raw2]")                      # raw bytes of rows 128..191 (loaded by the caller)
    a("v_mov_b32 v105, %[cro]")
    a("v_mov_b32 v106, %[rrow]")
    a("s_mov_b32 s40, 0")
    # LDS outflow slot base: C = 64 lanes 0..63 hold rows k0 - 128 + lane at slots k0 + lane; C = 32
    # lanes 32..63 the new rows (slots k0 + lane, lane address (lane + 32) & 63 from base k0 + 32)
    a(f"s_movk_i32 s41, {(64 - C) * 4:#x}")
    a("s_movk_i32 s42, 0x200")                       # ((0 + 128) mod R) * 4
    a("s_movk_i32 s53, 0xc0")                        # slot base of rows 128..191's codes: ((0 + 3) & 3) * 64
    a("s_mov_b32 s45, 0")
    a("s_mov_b32 s46, 0")
    a(f"s_movk_i32 s44, {RR}")
    a("s_mov_b32 s52, 0")
    if lds_out:
        # producer word at chunk 0: rows available (< k0 - 63) - C, one row conservative
        a(f"v_mov_b32 v90, {(-64 - H) & 0xffffffff:#x}")
        a("v_add_u32 v89, s41, %[lout]")
    if lds_in:
        a(f"v_mov_b32 v91, {RR + H}")               # consumer word after chunk 0: H consumed (+ R)
        a("v_add_u32 v88, s42, %[lin]")
    if gout:
        a("v_mov_b32 v98, %[gooff]")
        a("v_mov_b32 v100, %[gopos]")
        a("v_mov_b32 v107, %[gorow]")
    if gin:
        a("v_mov_b32 v101, %[gioff]")
        a("v_mov_b32 v102, %[gipos]")
        a(f"buffer_load_dwordx2 v[84:85], v101, %[girs], 0 offen {cin}")
    for q in range(ncr):
        a(f"ds_read_b128 v[{52 + 4 * q}:{55 + 4 * q}], %[c0]" + (f" offset:{16 * q}" if q else ""))
    a("s_waitcnt vmcnt(0) lgkmcnt(0)")
    a(".p2align 6")                # the chunk loop on a 64-B boundary (a lone wave's issue rate depends on it)
    for _ in range(LOOP_PAD):
        a("s_nop 0")
    a("L_loop_%=:")
    for p in (0, 1):
        cur = 52 if p == 0 else 68
        nxt = 68 if p == 0 else 52
        refill = p == 0 or C == 64                    # 64 code rows per refill
        lds = []                                      # LDS ops of this chunk top, in issue order
        # 1. publish the last chunk's outflow (C = 32: lanes 32..63; lanes 0..31 write ahead,
        # into slots of the next chunk's rows or the ring's slack, never read before rewritten)
        if lds_out:
            if p == 0:
                if hl:
                    a("s_add_u32 s54, s40, 64")
                    a("s_cmp_lt_i32 s44, s54")
                else:
                    a("s_cmp_lt_i32 s44, s40")
                a(f"s_cbranch_scc1 L_bp{p}_%=")
                a(f"L_bpr{p}_%=:")
            a("ds_write_b32 v89, v40")
            a("ds_write_b32 %[pout], v90")
            lds += ["W1", "W2"]
        if gout:
            a("s_add_u32 s55, s40, %[bpbase]")
            a("s_sub_u32 s54, s52, s55")
            a("s_cmp_lt_i32 s54, 0")
            a(f"s_cbranch_scc1 L_bpg{p}_%=")
            a(f"L_bpgr{p}_%=:")
            ring_granule(a, kout, cout)
        # 2. this chunk's inflow words / rows (LDS)
        if lds_in:
            a("ds_read_b32 v86, %[pin]")
            a("ds_read_b32 v84, v88")
            lds += ["A", "B"]
        # 3. the raw bytes of the refill and the granules of chunk c (loaded one chunk ago); the
        # stores issued after those loads: the outflow granules (C = 64: mid-chunk and chunk top),
        # the consumed-rows report (after the last chunk's loads, at p = 1)
        stores_after = (2 if C == 64 else 1) * gout + (1 if gin and p == 0 else 0)
        a(f"s_waitcnt vmcnt({stores_after})")
        if gin:
            ring_gin_check(a, C, kin)
            a(f"s_cbranch_scc1 L_gin{p}_%=")
            a(f"L_ginr{p}_%=:")
            a("v_cndmask_b32_e64 v40, %[ng], v84, s[58:59]")
        elif not lds_in:
            a("v_mov_b32 v40, %[ng]")
        # 4. codes of 64 rows (128..191 ahead of the body's first row) into the wave's code
        # ring (slot base s53, mirror of slots [0, 64))
        if refill:
            if hep:
                a("v_mov_b32 v94, v93")
            else:
                a("v_lshrrev_b32 v94, 1, v93")
                a("v_lshrrev_b32 v103, 2, v93")
                a("v_xor_b32 v94, v94, v103")
                a("v_and_or_b32 v94, v94, 3, 4")
                a("v_cmp_ne_u32_e64 s[56:57], 0, v93")
                a("v_cndmask_b32_e64 v94, 0, v94, s[56:57]")
            a("v_add_u32 v95, s53, %[cwr]")
            a("ds_write_b8 v95, v94")
            a("s_cmp_eq_u32 s53, 0")
            a("s_cselect_b32 s54, 0, 64")                # the mirror (slots 256..319) or the sink (320..383)
            a("v_add_u32 v95, s54, %[cwm]")
            a("ds_write_b8 v95, v94")
            a("s_add_u32 s53, s53, 64")
            a("s_and_b32 s53, s53, 0xff")
            lds += ["C1", "C2"]
            # 5. raw bytes of the next refill
            a("v_add_u32 v106, 64, v106")
            a("buffer_load_ubyte v93, v106, %[rrs], 0 offen")
        if gin:   # granules of chunk c+1
            a(f"v_add_u32 v101, {C * 8:#x}, v101")
            a("v_and_b32 v101, %[gimask8], v101")
            a(f"v_add_u32 v102, {C << 5:#x}, v102")
            a(f"buffer_load_dwordx2 v[84:85], v101, %[girs], 0 offen {cin}")
            if p == 1:   # every other chunk: rows consumed (for the producer's back-pressure)
                a(f"s_add_u32 s54, s40, {C}")
                a("s_min_i32 s54, s54, %[m]")
                a("s_add_u32 s54, s54, %[crv0]")
                a("v_mov_b32 v104, s54")
                a("buffer_store_dword v104, %[croff], %[cross], 0 offen sc1")
        # 6. row codes of chunk c+1
        a("v_add_u32 v87, %[cbase], v105")
        for q in range(ncr):
            a(f"ds_read_b128 v[{nxt + 4 * q}:{nxt + 4 * q + 3}], v87 offset:{16 * q}" if q else
              f"ds_read_b128 v[{nxt}:{nxt + 3}], v87")
        a(f"v_add_u32 v105, {C}, v105")
        a("v_and_b32 v105, 0xff, v105")
        lds += ["N%d" % q for q in range(ncr)]
        # 7. LDS inflow: word check, rows into IO, consumed word
        if lds_in:
            after_a = len(lds) - 1 - lds.index("A")
            a(f"s_waitcnt lgkmcnt({after_a})")
            a("v_readfirstlane_b32 s43, v86")
            a("s_cmp_lt_i32 s43, s40")
            a(f"s_cbranch_scc1 L_in{p}_%=")
            a(f"L_inr{p}_%=:")
            a(f"s_waitcnt lgkmcnt({after_a - 1})")
            a("v_mov_b32 v40, v84")
            a("ds_write_b32 %[qme], v91")
        else:
            # this chunk's codes (read one chunk ago) must be in: every LDS op since is younger
            a(f"s_waitcnt lgkmcnt({len(lds)})")
        # 8. C steps, C/4 groups of 4 rows
        for u in range(C // 4):
            if hl and lds_in and u == C // 8 - 1:
                # the second half's rows, read 4 steps ahead behind the producer's word
                a("ds_read_b32 v86, %[pin]")
                a(f"ds_read_b32 v102, v88 offset:{4 * H}")
            if hl and u == C // 8:
                # ---- mid-chunk: the newest 32 outflow rows out, the chunk's other 32 rows in
                if lds_out:
                    a(f"s_add_u32 s55, s41, {4 * C:#x}")
                    a(f"s_and_b32 s55, s55, {(RR - 1) * 4:#x}")
                    a("v_add_u32 v96, s55, %[lmid]")
                    a(f"v_add_u32 v90, {H}, v90")
                    a("ds_write_b32 v96, v40")
                    a("ds_write_b32 %[pout], v90")
                if lds_in:
                    a(f"s_waitcnt lgkmcnt({1 + (2 if lds_out else 0)})")
                    a("v_readfirstlane_b32 s43, v86")
                    a(f"s_add_u32 s54, s40, {H}")
                    a("s_cmp_lt_i32 s43, s54")
                    a(f"s_cbranch_scc1 L_mid{p}_%=")
                    a(f"L_midr{p}_%=:")
                    a(f"s_waitcnt lgkmcnt({2 if lds_out else 0})")
                    a("v_cndmask_b32_e64 v40, v102, v40, %[lhi]")
            qa, qb, qc = ("%[qA]", "%[qB]", "%[qC]") if hep else ("%[k80]",) * 3
            a(f"v_perm_b32 v48, %[pA], {qa}, v{cur + u}")
            a(f"v_perm_b32 v49, %[pB], {qb}, v{cur + u}")
            if W >= 3:
                a(f"v_perm_b32 v112, %[pC], {qc}, v{cur + u}")
            if W >= 4:
                a(f"v_perm_b32 v116, %[pD], %[k80], v{cur + u}")
            if W == 5:
                a(f"v_perm_b32 v121, %[pE], %[k80], v{cur + u}")
            for b in range(4):
                io, l0 = ("v40", "v41") if b % 2 == 0 else ("v41", "v40")
                if W >= 4:
                    step_w(a, io, l0, b, RING5 if W == 5 else RING4, W)
                elif W == 3:
                    step3(a, io, l0, b, RING3)
                else:
                    step(a, io, l0, b, RING)
            if gout and C == 64 and u == 7:
                ring_granule(a, kout, cout)
        # 9. on to the next chunk
        a(f"s_add_i32 s40, s40, {C}")
        if lds_out:
            a(f"s_add_u32 s41, s41, {4 * C:#x}")
            a(f"s_and_b32 s41, s41, {(RR - 1) * 4:#x}")
            a("v_add_u32 v89, s41, %[lout]")
            a(f"v_add_u32 v90, {C - H if hl else C}, v90")
        if lds_in:
            a(f"s_add_u32 s42, s42, {4 * C:#x}")
            a(f"s_and_b32 s42, s42, {(RR - 1) * 4:#x}")
            a("v_add_u32 v88, s42, %[lin]")
            a(f"v_add_u32 v91, {C}, v91")
    a("s_cmp_lt_i32 s40, %[end]")
    a("s_cbranch_scc1 L_loop_%=")
    # ---- exit
    if lds_out:
        a("s_cmp_lt_i32 s44, s40")
        a("s_cbranch_scc1 L_bpx_%=")
        a("L_bpxr_%=:")
        a("ds_write_b32 v89, v40")
        a(f"v_mov_b32 v90, {BIG:#x}")
        a("ds_write_b32 %[pout], v90")
    if gout:
        a("s_add_u32 s55, s40, %[bpbase]")
        a("s_sub_u32 s54, s52, s55")
        a("s_cmp_lt_i32 s54, 0")
        a("s_cbranch_scc1 L_bpgx_%=")
        a("L_bpgxr_%=:")
        ring_granule(a, kout, cout)
    if gin:   # every row consumed
        a("s_add_u32 s54, %[m], %[crv0]")
        a("v_mov_b32 v104, s54")
        a("buffer_store_dword v104, %[croff], %[cross], 0 offen sc1")
    a("s_waitcnt vmcnt(0) lgkmcnt(0)")
    a("v_mov_b32 %[M], v50")
    a("s_mov_b32 %[fail], s45")
    a("s_mov_b32 %[slow], s46")
    a("s_branch L_done_%=")
    # ---- slow paths
    if lds_in:
        for p in (0, 1):
            slow_wait(a, f"L_in{p}_%=", f"L_inr{p}_%=", "v86", "%[pin]", "s43", reread="ds_read_b32 v84, v88")
            if hl:
                slow_wait(a, f"L_mid{p}_%=", f"L_midr{p}_%=", "v86", "%[pin]", "s43",
                          reread=f"ds_read_b32 v102, v88 offset:{4 * H}", target="s54")
    if lds_out:
        slow_wait(a, "L_bp0_%=", "L_bpr0_%=", "v92", "%[qnx]", "s44", target="s54" if hl else "s40")
        slow_wait(a, "L_bpx_%=", "L_bpxr_%=", "v92", "%[qnx]", "s44")
    if gout:
        for lab, res in (("L_bpg0_%=", "L_bpgr0_%="), ("L_bpg1_%=", "L_bpgr1_%="), ("L_bpgx_%=", "L_bpgxr_%=")):
            slow_bp_hbm(a, lab, res)
    if gin:
        for p in (0, 1):
            slow_gin(a, f"L_gin{p}_%=", f"L_ginr{p}_%=", C, kin, cin)
    a("L_done_%=:")
    return L


def slow_timeout(a, label):
    """The end of a slow-path poll: sleep and poll again ({label}_w); every 64th poll also reads
    the clock and gives up past the deadline ({label}_x).  s_memrealtime is an SMEM round trip,
    much slower than an LDS poll, so a late hand-off no longer pays one per poll (measured neutral
    on C2, C5 and the column slab, r05)."""
    a("s_add_u32 s46, s46, 1")
    a("s_and_b32 s48, s46, 63")
    a("s_cmp_lg_u32 s48, 0")
    a(f"s_cbranch_scc1 {label}_s")
    a("s_memrealtime s[48:49]")
    a("s_waitcnt lgkmcnt(0)")
    a("s_sub_u32 s48, s48, %[dlo]")
    a("s_subb_u32 s49, s49, %[dhi]")
    a("s_cmp_lt_i32 s49, 0")
    a("s_cbranch_scc0 %s_x" % label)
    a(f"{label}_s:")
    a("s_sleep 1")
    a(f"s_branch {label}_w")


def slow_bp_hbm(a, label, resume):
    """The consumer of a ring edge has not yet reported the rows this publish overwrites:
    re-read its word (HBM, sc1) until it covers them (serial-number compare)."""
    a(f"{label}:")
    a("s_add_u32 s46, s46, 1")
    a("s_cmp_lg_u32 s45, 0")
    a(f"s_cbranch_scc1 {resume}")
    a(f"{label}_w:")
    a("buffer_load_dword v92, off, %[bpr], 0 sc1")
    a("s_waitcnt vmcnt(0) lgkmcnt(0)")
    a("v_readfirstlane_b32 s52, v92")
    a("s_add_u32 s55, s40, %[bpbase]")
    a("s_sub_u32 s54, s52, s55")
    a("s_cmp_ge_i32 s54, 0")
    a(f"s_cbranch_scc1 {resume}")
    slow_timeout(a, label)
    a(f"{label}_x:")
    a("s_mov_b32 s45, 1")
    a(f"s_branch {resume}")


def slow_gin(a, label, resume, C=64, key="%[ek]", cp="sc1"):
    """The chunk's inflow granules are not all published yet: re-load and re-check."""
    a(f"{label}:")
    a("s_add_u32 s46, s46, 1")
    a("s_cmp_lg_u32 s45, 0")
    a(f"s_cbranch_scc1 {resume}")
    a(f"{label}_w:")
    a(f"buffer_load_dwordx2 v[84:85], v101, %[girs], 0 offen {cp}")
    a("s_waitcnt vmcnt(0) lgkmcnt(0)")
    ring_gin_check(a, C, key)
    a(f"s_cbranch_scc0 {resume}")
    slow_timeout(a, label)
    a(f"{label}_x:")
    a("s_mov_b32 s45, 1")
    a(f"s_branch {resume}")


ROLES_IN_RING = ("none", "lds", "gran")
# the extra roles of a column slab's kernel (C = 64): its first strip takes the previous GPU's
# edge (IN = peer), its last strip hands its edge to the next GPU (OUT = peer)
ROLES_SLAB = (("peer", "lds"), ("peer", "peer"), ("peer", "none"), ("gran", "peer"), ("lds", "peer"),
              ("none", "peer"))
CLOBBERS_RING = ['"v%d"' % r for r in range(40, 108) if r != 51] + \
    ['"s%d"' % r for r in range(40, 60) if r not in (47,)] + ['"scc"', '"vcc"', '"memory"']


def emit_ring():
    out = ["// GENERATED by tools/gen_flow3.py -- do not edit.  The flow3 ring-mode chunk loops",
           "// (sw_flow3.hip sw_flow3r_kernel): one inline-asm block per (chunk rows C, half-chunk LDS links HL, strip role), R = %d." % RR,
           "// Operands: see F3RLoop in sw_flow3.hip; fixed registers: tools/gen_flow3.py.",
           "#pragma once", ""]
    combos = [(C, hl, i, o) for C, hl in ((64, 0), (32, 0), (64, 1)) for i in ROLES_IN_RING for o in ROLES_OUT]
    combos += [(64, 0, i, o) for i, o in ROLES_SLAB]
    for C, hl, IN, OUT_ in combos:
        if True:
            body = align8(gen_role_ring(IN, OUT_, C, bool(hl)), nops=RING_NOPS) if RING_ALIGN else gen_role_ring(IN, OUT_, C, bool(hl))
            out.append("template <> __device__ __forceinline__ F3Res f3r_loop<%d, %d, F3_%s, F3_%s>(const F3RLoop& x) {"
                       % (C, hl, IN.upper(), OUT_.upper()))
            out.append("    F3Res r;")
            out.append("    asm volatile(")
            for line in body:
                out.append('        "%s\\n\\t"' % line)
            out.append('        : [M] "=v"(r.M), [fail] "=s"(r.fail), [slow] "=s"(r.slow)')
            out.append('        : [pA] "v"(x.pA), [pB] "v"(x.pB), [ng] "v"(x.ng), [G] "s"(x.G), [k80] "s"(x.k80),')
            out.append('          [m] "s"(x.m), [end] "s"(x.end), [dlo] "s"(x.dlo), [dhi] "s"(x.dhi), [lane] "v"(x.lane),')
            out.append('          [raw2] "v"(x.raw2), [cro] "v"(x.cro), [c0] "v"(x.c0), [cbase] "v"(x.cbase),')
            out.append('          [cwr] "v"(x.cwr), [cwm] "v"(x.cwm), [rrs] "s"(x.rrs), [rrow] "v"(x.rrow),')
            out.append('          [lin] "v"(x.lin), [lout] "v"(x.lout), [pin] "v"(x.pin), [pout] "v"(x.pout),')
            out.append('          [qme] "v"(x.qme), [qnx] "v"(x.qnx),')
            out.append('          [girs] "s"(x.girs), [gioff] "v"(x.gioff), [gipos] "v"(x.gipos), [gimask8] "s"(x.gimask8),')
            out.append('          [ek] "s"(x.ek), [cross] "s"(x.cross), [crv0] "s"(x.crv0), [croff] "v"(x.croff),')
            out.append('          [gors] "s"(x.gors), [gooff] "v"(x.gooff), [gopos] "v"(x.gopos), [gomask8] "s"(x.gomask8),')
            out.append('          [gorow] "v"(x.gorow), [lhi] "s"(x.lhi), [bpr] "s"(x.bpr), [bpbase] "s"(x.bpbase),')
            out.append('          [lmid] "v"(x.lmid), [ekp] "s"(x.ekp)')
            out.append("        : " + ", ".join(CLOBBERS_RING) + ");")
            out.append("    return r;")
            out.append("}")
            out.append("")
    return "\n".join(out)


OUT_RING = os.path.join(ROOT, "concurrentproject_amd", "csrc", "sw_flow3r_loops.inc")
OUT_RING3 = os.path.join(ROOT, "concurrentproject_amd", "csrc", "sw_flow3r3_loops.inc")
CLOBBERS_RING3 = CLOBBERS_RING + ['"v%d"' % r for r in range(108, 113)]


def emit_ring3():
    """Three columns per lane in ring mode (sw_flow3.hip flow3_ring<64, 0, false, SLAB, true>):
    C = 64, whole-chunk links, every ring role and the column-slab roles."""
    out = ["// GENERATED by tools/gen_flow3.py -- do not edit.  The flow3 ring-mode chunk loops at three",
           "// columns per lane (sw_flow3.hip sw_flow3r3_kernel): one inline-asm block per strip role, C = 64, R = %d." % RR,
           "// Operands: see F3RLoop in sw_flow3.hip; fixed registers: tools/gen_flow3.py (RING3).",
           "#pragma once", ""]
    # ALN = 1 (the column-slab kernel, one wave per SIMD): every 8-B instruction on an 8-B boundary,
    # padding with s_nop (slab 0 of 8: 32.5 -> 29.5 ms); ALN = 0 (C5, 4 waves per SIMD): as generated
    # (aligned there: 154.3 -> 161.1 ms with nops, 163.0 with VOP3 re-encodings)
    # HEP (aln 2 below): the ring roles of a pair over up to seven byte values (sw_flow3r3h_kernel)
    combos = [(i, o, 0) for i in ROLES_IN_RING for o in ROLES_OUT] + \
        [(i, o, 1) for i in ROLES_IN_RING for o in ROLES_OUT] + [(i, o, 1) for i, o in ROLES_SLAB] + \
        [(i, o, 2) for i in ROLES_IN_RING for o in ROLES_OUT]
    for IN, OUT_, aln in combos:
        hep = aln == 2
        body = gen_role_ring(IN, OUT_, 64, False, 3, hep)
        if aln == 1:
            body = align8(body, nops=True, promote=False)
        if hep:
            out.append("template <> __device__ __forceinline__ F3Res f3r3h_loop<F3_%s, F3_%s>(const F3RLoop& x) {"
                       % (IN.upper(), OUT_.upper()))
        else:
            out.append("template <> __device__ __forceinline__ F3Res f3r3_loop<F3_%s, F3_%s, %d>(const F3RLoop& x) {"
                       % (IN.upper(), OUT_.upper(), aln))
        out.append("    F3Res r;")
        out.append("    asm volatile(")
        for line in body:
            out.append('        "%s\\n\\t"' % line)
        out.append('        : [M] "=v"(r.M), [fail] "=s"(r.fail), [slow] "=s"(r.slow)')
        out.append('        : [pA] "v"(x.pA), [pB] "v"(x.pB), [pC] "v"(x.pC), [ng] "v"(x.ng), [G] "s"(x.G), ' +
                   ('[qA] "v"(x.qA), [qB] "v"(x.qB), [qC] "v"(x.qC),' if hep else '[k80] "s"(x.k80),'))
        out.append('          [m] "s"(x.m), [end] "s"(x.end), [dlo] "s"(x.dlo), [dhi] "s"(x.dhi), [lane] "v"(x.lane),')
        out.append('          [raw2] "v"(x.raw2), [cro] "v"(x.cro), [c0] "v"(x.c0), [cbase] "v"(x.cbase),')
        out.append('          [cwr] "v"(x.cwr), [cwm] "v"(x.cwm), [rrs] "s"(x.rrs), [rrow] "v"(x.rrow),')
        out.append('          [lin] "v"(x.lin), [lout] "v"(x.lout), [pin] "v"(x.pin), [pout] "v"(x.pout),')
        out.append('          [qme] "v"(x.qme), [qnx] "v"(x.qnx),')
        out.append('          [girs] "s"(x.girs), [gioff] "v"(x.gioff), [gipos] "v"(x.gipos), [gimask8] "s"(x.gimask8),')
        out.append('          [ek] "s"(x.ek), [cross] "s"(x.cross), [crv0] "s"(x.crv0), [croff] "v"(x.croff),')
        out.append('          [gors] "s"(x.gors), [gooff] "v"(x.gooff), [gopos] "v"(x.gopos), [gomask8] "s"(x.gomask8),')
        out.append('          [gorow] "v"(x.gorow), [lhi] "s"(x.lhi), [bpr] "s"(x.bpr), [bpbase] "s"(x.bpbase),')
        out.append('          [lmid] "v"(x.lmid), [ekp] "s"(x.ekp)')
        out.append("        : " + ", ".join(CLOBBERS_RING3) + ");")
        out.append("    return r;")
        out.append("}")
        out.append("")
    return "\n".join(out)

OUT_RING45 = os.path.join(ROOT, "concurrentproject_amd", "csrc", "sw_flow3r45_loops.inc")


def emit_ring45():
    """Four and five columns per lane in ring mode (sw_flow3.hip sw_flow3r45_kernel: a C5-sized
    pair cut into 252-column strips and, at its end, 315-column ones, so that every strip is
    resident in one round): C = 64, whole-chunk links, the nine ring roles, no slab roles."""
    out = ["// GENERATED by tools/gen_flow3.py -- do not edit.  The flow3 ring-mode chunk loops at four and",
           "// five columns per lane (sw_flow3.hip sw_flow3r45_kernel): one inline-asm block per (W, strip role),",
           "// C = 64, R = %d.  Operands: see F3RLoop in sw_flow3.hip; fixed registers: tools/gen_flow3.py (RING4/5)." % RR,
           "#pragma once", ""]
    for W in (4, 5):
        clob = CLOBBERS_RING3 + ['"v%d"' % r for r in range(113, 117 if W == 4 else 122)]
        for IN in ROLES_IN_RING:
            for OUT_ in ROLES_OUT:
                body = gen_role_ring(IN, OUT_, 64, False, W)
                out.append("template <> __device__ __forceinline__ F3Res f3r%d_loop<F3_%s, F3_%s>(const F3RLoop& x) {"
                           % (W, IN.upper(), OUT_.upper()))
                out.append("    F3Res r;")
                out.append("    asm volatile(")
                for line in body:
                    out.append('        "%s\\n\\t"' % line)
                out.append('        : [M] "=v"(r.M), [fail] "=s"(r.fail), [slow] "=s"(r.slow)')
                out.append('        : [pA] "v"(x.pA), [pB] "v"(x.pB), [pC] "v"(x.pC), [pD] "v"(x.pD),' +
                           (' [pE] "v"(x.pE),' if W == 5 else '') + ' [ng] "v"(x.ng), [G] "s"(x.G), [k80] "s"(x.k80),')
                out.append('          [m] "s"(x.m), [end] "s"(x.end), [dlo] "s"(x.dlo), [dhi] "s"(x.dhi), [lane] "v"(x.lane),')
                out.append('          [raw2] "v"(x.raw2), [cro] "v"(x.cro), [c0] "v"(x.c0), [cbase] "v"(x.cbase),')
                out.append('          [cwr] "v"(x.cwr), [cwm] "v"(x.cwm), [rrs] "s"(x.rrs), [rrow] "v"(x.rrow),')
                out.append('          [lin] "v"(x.lin), [lout] "v"(x.lout), [pin] "v"(x.pin), [pout] "v"(x.pout),')
                out.append('          [qme] "v"(x.qme), [qnx] "v"(x.qnx),')
                out.append('          [girs] "s"(x.girs), [gioff] "v"(x.gioff), [gipos] "v"(x.gipos), [gimask8] "s"(x.gimask8),')
                out.append('          [ek] "s"(x.ek), [cross] "s"(x.cross), [crv0] "s"(x.crv0), [croff] "v"(x.croff),')
                out.append('          [gors] "s"(x.gors), [gooff] "v"(x.gooff), [gopos] "v"(x.gopos), [gomask8] "s"(x.gomask8),')
                out.append('          [gorow] "v"(x.gorow), [lhi] "s"(x.lhi), [bpr] "s"(x.bpr), [bpbase] "s"(x.bpbase),')
                out.append('          [lmid] "v"(x.lmid), [ekp] "s"(x.ekp)')
                out.append("        : " + ", ".join(clob) + ");")
                out.append("    return r;")
                out.append("}")
                out.append("")
    return "\n".join(out)


# ============================================================================================
# The general affine (Gotoh) step, staged organisation (C2 with G_INIT != G_EXT):
# sw_flow3.hip sw_flow3a_kernel, sw_flow3a_loops.inc.  ONE column per lane (63 new columns
# per strip): a single long pair is latency-bound, and the critical path is (m + n / W) steps
# of (ops per step) instructions of a lone wave, 10.5 VALU at W = 1 against 18 at W = 2,
# so W = 1 is the shorter path for this step.  Two quantities flow
# lane to lane (H - G_INIT and E - G_EXT), each through a tied DPP-add and a rotating I/O
# register; LDS links carry both as one 8-B slot, workgroup edges as 16-B granules
# {H - GI, (H - GI) ^ ek, E - GE, (E - GE) ^ ek2} whose two halves each carry their own tag.
# Step (lane l, row i = k - l; main.cpp:54-66, clamped as DESIGN.md section 2):
#   t   = L0H + s(q, d) + G_INIT        SDWA byte of the 4-row profile perm; L0H = last hgL
#   L0H = wave_shl1(IOH), L0E = wave_shl1(IOE)    rotation; lane 63 keeps last (hgL, ehL)
#   hgL = IOH = H[l-1] - G_INIT, ehL = IOE = E[l-1] - G_EXT   tied DPP-adds (lane 0: inflow)
#   F   = max3(fh, hgO, 0)              fh = F(i-1) - G_EXT, hgO = H(i-1) - G_INIT
#   E   = max(ehL, hgL)                 (>= -G_INIT; H sees it through max3 with F >= 0)
#   H   = max3(t, E, F);  fh = F - G_EXT;  hgO = H - G_INIT;  M = max3(M, t, t') every 2 steps
# Registers: v64..v67 IO/L0 (even step: IOH v64, IOE v65, L0H v66, L0E v67; odd: swapped
# pairwise, so the chunk top always finds the I/O pair in v[64:65]), v68 H, v69 hgO, v70 F,
# v71 fh, v72 E, v73/v74 t of even/odd steps, v75 score bytes of 4 rows, v76 M,
# v[80:87] / v[88:95] row codes of the even / odd chunk, v[96:97] inflow row, v98 producer
# word read, v99 code address, v100 inflow address, v101 outflow address, v102 producer word
# value, v103 consumer word value, v104 back-pressure read, v105 mid-publish address,
# v[106:107] mid-chunk inflow row, v[108:111] granule, v112 granule offset (row * 16),
# v113 masked offset; SGPRs as gen_role.
# ============================================================================================
SZA = 8                  # bytes per LDS ring slot: (H - G_INIT, E - G_EXT)


def step_aff1(a, b, even):
    """One anti-diagonal step of the one-column affine step (10.5 VALU, 64 cells)."""
    ioh, ioe, l0h, l0e = ("v64", "v65", "v66", "v67") if even else ("v66", "v67", "v64", "v65")
    t = "v73" if even else "v74"
    a(f"v_add_u32_sdwa {t}, sext(v75), {l0h} dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_{b} src1_sel:DWORD")
    a(f"v_mov_b32_dpp {l0h}, {ioh} wave_shl:1 row_mask:0xf bank_mask:0xf")
    a(f"v_add_u32_dpp {ioh}, v68, %[ng] wave_shr:1 row_mask:0xf bank_mask:0xf")
    a(f"v_mov_b32_dpp {l0e}, {ioe} wave_shl:1 row_mask:0xf bank_mask:0xf")
    a(f"v_add_u32_dpp {ioe}, v72, %[nge] wave_shr:1 row_mask:0xf bank_mask:0xf")
    a("v_max3_i32 v70, v71, v69, 0")
    a(f"v_max_i32 v72, {ioe}, {ioh}")
    a(f"v_max3_i32 v68, {t}, v72, v70")
    a("v_subrev_u32 v71, %[GE], v70")
    a("v_subrev_u32 v69, %[GI], v68")
    if not even:
        a("v_max3_i32 v76, v76, v73, v74")


def granule_aff(a, rows):
    """Publish the `rows` newest outflow rows (lanes 64-rows..63 of the I/O pair v[64:65], mask
    %[m48]) as 16-B granules {H-GI, (H-GI) ^ ek, E-GE, (E-GE) ^ ek2} at row * 16, write-through."""
    a("v_mov_b32 v108, v64")
    a("v_xor_b32 v109, %[ek], v64")
    a("v_mov_b32 v110, v65")
    a("v_xor_b32 v111, %[ek2], v65")
    a("v_cndmask_b32_e64 v113, -16, v112, %[m48]")
    a(f"v_add_u32 v112, {rows * 16:#x}, v112")
    a("buffer_store_dwordx4 v[108:111], v113, %[rsrc], 0 offen sc1")


def book_aff(a, p, lds_in, lds_out, C, H):
    a(f"s_add_i32 s40, s40, {C}")
    a(f"s_add_u32 s41, s41, {SZA * C:#x}")
    a(f"s_and_b32 s41, s41, {(R - 1) * SZA:#x}")
    if lds_out:
        a("v_add_u32 v101, s41, %[lout]")
        a(f"v_add_u32 v102, {C if H == C else C - H}, v102")
    if lds_in:
        a("v_add_u32 v100, s41, %[lin]")
        a(f"v_add_u32 v103, {C}, v103")
    if p == 1:
        a(f"v_add_u32 v99, {2 * C}, v99")


def gen_role_aff(IN, OUT_, C=32, hl=True):
    """gen_role's staged loop (same chunks, words, half-chunk links, speculative inflow read
    4 steps ahead, granules every half chunk) around the one-column affine step."""
    L = []
    a = L.append
    lds_in, lds_out, gran = IN == "lds", OUT_ == "lds", OUT_ == "gran"
    H = C // 2 if hl else C
    ng = C // 4
    ncr = ng // 4                       # 16-B code reads per chunk
    nw = 2 if lds_out else 0
    assert C in (16, 32) and (not hl or C == 32)
    a("s_nop 4")
    a("s_waitcnt vmcnt(0) lgkmcnt(0)")
    for r in ("v68", "v70", "v72", "v76"):
        a(f"v_mov_b32 {r}, 0")
    a("v_mov_b32 v69, %[ng]")
    a("v_mov_b32 v71, %[nge]")
    a("v_mov_b32 v64, %[ng]")
    a("v_mov_b32 v66, %[ng]")
    a("v_mov_b32 v65, %[nge]")
    a("v_mov_b32 v67, %[nge]")
    a("v_mov_b32 v99, %[code]")
    a("s_mov_b32 s40, 0")
    a(f"s_movk_i32 s41, {(64 - C) * SZA:#x}")
    a("s_mov_b32 s45, 0")
    a("s_mov_b32 s46, 0")
    a(f"s_movk_i32 s44, {R}")
    if lds_out:
        a(f"v_mov_b32 v102, {-64 - H}")
        a("v_add_u32 v101, s41, %[lout]")
    if lds_in:
        a(f"v_mov_b32 v103, {R + H}")
        a("v_add_u32 v100, s41, %[lin]")
        if hl:
            a("s_mov_b32 s50, 0xffff")
            a("s_mov_b32 s51, 0")
    if gran:
        a("v_mov_b32 v112, %[lrow]")
    for q in range(ncr):
        a(f"ds_read_b128 v[{80 + 4 * q}:{83 + 4 * q}], v99 offset:{16 * q}")
    if lds_in:
        a("ds_read_b32 v98, %[pin]")
        a("ds_read_b64 v[96:97], v100")
    a(".p2align 6")                # the chunk loop on a 64-B boundary (a lone wave's issue rate depends on it)
    for _ in range(LOOP_PAD):
        a("s_nop 0")
    a("L_loop_%=:")
    for p in (0, 1):
        cur = 80 if p == 0 else 88
        nxt = 88 if p == 0 else 80
        obase = C if p == 0 else 2 * C
        if lds_out:
            if p == 0:
                if hl:
                    a(f"s_add_u32 s52, s40, {H}")
                    a("s_cmp_lt_i32 s44, s52")
                else:
                    a("s_cmp_lt_i32 s44, s40")
                a(f"s_cbranch_scc1 L_bp{p}_%=")
                a(f"L_bpr{p}_%=:")
            a(f"ds_write2st64_b64 v101, v[64:65], v[64:65] offset1:{R * SZA // 512}")
            a("ds_write_b32 %[pout], v102")
        if gran:
            granule_aff(a, C // 2)
        for q in range(ncr):
            a(f"ds_read_b128 v[{nxt + 4 * q}:{nxt + 4 * q + 3}], v99 offset:{obase + 16 * q}")
        if lds_in:
            after = 1 + nw + ncr
            a(f"s_waitcnt lgkmcnt({after})")
            a("v_readfirstlane_b32 s43, v98")
            a("s_cmp_lt_i32 s43, s40")
            a(f"s_cbranch_scc1 L_in{p}_%=")
            a(f"L_inr{p}_%=:")
            a(f"s_waitcnt lgkmcnt({after - 1})")
            a("v_mov_b32 v64, v96")
            a("v_mov_b32 v65, v97")
            a("ds_write_b32 %[qme], v103")
        else:
            a(f"s_waitcnt lgkmcnt({nw + ncr})")
            a("v_mov_b32 v64, %[ng]")
            a("v_mov_b32 v65, %[nge]")
        for u in range(ng):
            if u == ng - 1:
                book_aff(a, p, lds_in, lds_out, C, H)
                if lds_in:
                    a("ds_read_b32 v98, %[pin]")
                    a("ds_read_b64 v[96:97], v100")
            if hl and lds_in and u == ng // 2 - MID_AHEAD:
                a("ds_read_b32 v98, %[pin]")
                a(f"ds_read_b64 v[106:107], v100 offset:{SZA * H}")
            if hl and u == ng // 2:
                if lds_out:
                    a("v_add_u32 v105, %[lmid], v101")
                    a(f"v_add_u32 v102, {H}, v102")
                    a(f"ds_write2st64_b64 v105, v[64:65], v[64:65] offset1:{R * SZA // 512}")
                    a("ds_write_b32 %[pout], v102")
                if lds_in:
                    a(f"s_waitcnt lgkmcnt({1 + (2 if lds_out else 0)})")
                    a("v_readfirstlane_b32 s43, v98")
                    if not (lds_out and p == 0):
                        a(f"s_add_u32 s52, s40, {H}")
                    a("s_cmp_lt_i32 s43, s52")
                    a(f"s_cbranch_scc1 L_mid{p}_%=")
                    a(f"L_midr{p}_%=:")
                    a(f"s_waitcnt lgkmcnt({2 if lds_out else 0})")
                    a("v_cndmask_b32_e64 v64, v64, v106, s[50:51]")
                    a("v_cndmask_b32_e64 v65, v65, v107, s[50:51]")
            a(f"v_perm_b32 v75, %[pA], %[qA], v{cur + u}")
            for b in range(4):
                step_aff1(a, b, b % 2 == 0)
            if gran and u == ng // 2 - 1:
                granule_aff(a, C // 2)
    a("s_cmp_lt_i32 s40, %[end]")
    a("s_cbranch_scc1 L_loop_%=")
    if lds_out:
        a("s_cmp_lt_i32 s44, s40")
        a("s_cbranch_scc1 L_bpx_%=")
        a("L_bpxr_%=:")
        a(f"ds_write2st64_b64 v101, v[64:65], v[64:65] offset1:{R * SZA // 512}")
        a(f"v_mov_b32 v102, {BIG:#x}")
        a("ds_write_b32 %[pout], v102")
    if gran:
        granule_aff(a, C // 2)
    a("s_waitcnt vmcnt(0) lgkmcnt(0)")
    a("v_mov_b32 %[M], v76")
    a("s_mov_b32 %[fail], s45")
    a("s_mov_b32 %[slow], s46")
    a("s_branch L_done_%=")
    if lds_in:
        for p in (0, 1):
            slow_wait(a, f"L_in{p}_%=", f"L_inr{p}_%=", "v98", "%[pin]", "s43", reread="ds_read_b64 v[96:97], v100")
            if hl:
                slow_wait(a, f"L_mid{p}_%=", f"L_midr{p}_%=", "v98", "%[pin]", "s43",
                          reread=f"ds_read_b64 v[106:107], v100 offset:{SZA * H}", target="s52")
    if lds_out:
        slow_wait(a, "L_bp0_%=", "L_bpr0_%=", "v104", "%[qnx]", "s44", target="s52" if hl else "s40")
        slow_wait(a, "L_bpx_%=", "L_bpxr_%=", "v104", "%[qnx]", "s44")
    a("L_done_%=:")
    return L


CLOBBERS_AFF = ['"v%d"' % r for r in range(64, 114) if r not in (77, 78, 79)] + \
    ['"s%d"' % r for r in range(40, 53) if r != 42 and r != 47] + ['"scc"', '"vcc"', '"memory"']
OUT_AFF = os.path.join(ROOT, "concurrentproject_amd", "csrc", "sw_flow3a_loops.inc")


def emit_aff():
    out = ["// GENERATED by tools/gen_flow3.py -- do not edit.  The flow3 affine-step chunk loops",
           "// (sw_flow3.hip sw_flow3a_kernel): one inline-asm block per (chunk rows C, half-chunk LDS links HL,",
           "// strip role), R = %d ring rows of 8-B slots, inflow read 4 steps ahead, granules every half chunk." % R,
           "// Operands: see F3ALoop in sw_flow3.hip; fixed registers: tools/gen_flow3.py (gen_role_aff).",
           "#pragma once", ""]
    for C, hl in ((32, 1), (32, 0), (16, 0)):
        for IN in ROLES_IN:
            for OUT_ in ROLES_OUT:
                body = align8(gen_role_aff(IN, OUT_, C, bool(hl)), promote=STAGED_PROMOTE)
                out.append("template <> __device__ __forceinline__ F3Res f3a_loop<%d, %d, F3_%s, F3_%s>(const F3ALoop& x) {"
                           % (C, hl, IN.upper(), OUT_.upper()))
                out.append("    F3Res r;")
                out.append("    asm volatile(")
                for line in body:
                    out.append('        "%s\\n\\t"' % line)
                out.append('        : [M] "=v"(r.M), [fail] "=s"(r.fail), [slow] "=s"(r.slow)')
                out.append('        : [pA] "v"(x.pA), [ng] "v"(x.ng), [nge] "v"(x.nge), [GI] "s"(x.GI), [GE] "s"(x.GE),')
                out.append('          [qA] "v"(x.qA), [code] "v"(x.code), [lin] "v"(x.lin), [lout] "v"(x.lout),')
                out.append('          [pin] "v"(x.pin), [pout] "v"(x.pout), [qme] "v"(x.qme), [qnx] "v"(x.qnx),')
                out.append('          [end] "s"(x.end), [dlo] "s"(x.dlo), [dhi] "s"(x.dhi), [rsrc] "s"(x.rsrc),')
                out.append('          [ek] "s"(x.ek), [ek2] "s"(x.ek2), [lrow] "v"(x.lrow), [m48] "s"(x.m48),')
                out.append('          [lmid] "v"(x.lmid)')
                out.append("        : " + ", ".join(CLOBBERS_AFF) + ");")
                out.append("    return r;")
                out.append("}")
                out.append("")
    return "\n".join(out)


# ============================================================================================
# The general affine step in ring mode (C5 with G_INIT != G_EXT): sw_flow3.hip
# sw_flow3ra_kernel, sw_flow3ra_loops.inc.  Ring mode is throughput-bound (4 waves per SIMD),
# where what counts is issue cost per cell: TWO columns per lane, 18 VALU for 128 cells
# (13 slow-class) against 10.5 for 64 (8.5 slow) at one column.  gen_role_ring's organisation
# at C = 64 (no half-chunk links) with two flows: LDS slots of 8 B (H - GI, E - GE) and ring
# granules of 16 B {H-GI, (H-GI)^ek^(pos<<5), E-GE, (E-GE)^ek2^(pos<<5)}.
# Step (lane l: columns A, B; main.cpp:54-66 clamped as DESIGN.md section 2):
#   tA = L0H + s_A + G_INIT, tB = H_A(i-1) + s_B       (diagonals; profiles prof2 / prof3)
#   L0H/L0E = wave_shl1(IOH/IOE); IOH = H_B[l-1] - GI, IOE = E_B[l-1] - GE   (lane 0: inflow)
#   F_A = max3(fhA, hgOA, 0); E_A = max(IOE, IOH); H_A = max3(tA, E_A, F_A)
#   fhA = F_A - GE; hgOA = H_A - GI; E_B = max(E_A - GE, hgOA)
#   F_B = max3(fhB, hgOB, 0); H_B = max3(tB, E_B, F_B); fhB = F_B - GE; hgOB = H_B - GI
#   M = max3(M, tA, tB)
# Registers: v40..v43 IO/L0 (even step: IOH v40, IOE v41, L0H v42, L0E v43; odd swapped
# pairwise), v44 H_A, v45 hgOA, v46 fhA, v47 H_B, v48 hgOB, v49 fhB, v50 E_B, v51 tA,
# v52 tB, v53 F (temp), v54 E_A / E_A - GE (temp), v55 / v56 score bytes A / B, v57 M,
# v[58:73] / v[74:89] row codes of the even / odd chunk, v[90:93] granule inflow (or the LDS
# inflow row v[90:91]), v94 producer word read, v95 code read address, v96 / v97 LDS inflow /
# outflow address, v98 / v99 producer / consumer word values, v100 back-pressure read, v101 raw
# row byte, v102 row code, v103 code write address, v[104:107] granule outflow, v108 its slot
# offset, v109 its masked offset, v110 its position << 5, v111 granule inflow offset, v112 its
# position << 5, v113 scratch, v114 consumer report, v115 code read offset, v116 raw row,
# v117 granule outflow row; SGPRs as gen_role_ring.
# ============================================================================================


def step_aff2(a, b, even):
    """One anti-diagonal step of the two-column affine step (18 VALU, 128 cells)."""
    ioh, ioe, l0h, l0e = ("v40", "v41", "v42", "v43") if even else ("v42", "v43", "v40", "v41")
    a(f"v_add_u32_sdwa v51, sext(v55), {l0h} dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_{b} src1_sel:DWORD")
    a(f"v_add_u32_sdwa v52, sext(v56), v44 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_{b} src1_sel:DWORD")
    a(f"v_mov_b32_dpp {l0h}, {ioh} wave_shl:1 row_mask:0xf bank_mask:0xf")
    a(f"v_add_u32_dpp {ioh}, v47, %[ng] wave_shr:1 row_mask:0xf bank_mask:0xf")
    a(f"v_mov_b32_dpp {l0e}, {ioe} wave_shl:1 row_mask:0xf bank_mask:0xf")
    a(f"v_add_u32_dpp {ioe}, v50, %[nge] wave_shr:1 row_mask:0xf bank_mask:0xf")
    a("v_max3_i32 v53, v46, v45, 0")            # F_A
    a(f"v_max_i32 v54, {ioe}, {ioh}")           # E_A
    a("v_max3_i32 v44, v51, v54, v53")          # H_A
    a("v_subrev_u32 v46, %[GE], v53")           # fhA
    a("v_subrev_u32 v45, %[GI], v44")           # hgOA
    a("v_subrev_u32 v54, %[GE], v54")           # E_A - GE
    a("v_max_i32 v50, v54, v45")                # E_B
    a("v_max3_i32 v53, v49, v48, 0")            # F_B
    a("v_max3_i32 v47, v52, v50, v53")          # H_B
    a("v_subrev_u32 v49, %[GE], v53")           # fhB
    a("v_subrev_u32 v48, %[GI], v47")           # hgOB
    a("v_max3_i32 v57, v57, v51, v52")          # M


def step_aff3(a, b, even):
    """One anti-diagonal step of the three-column affine step (25.5 VALU, 192 cells): step_aff2
    with a column C (v118 H_C, v119 hgOC, v120 fhC, v121 E_C, the flowing E; v122 / v123 tC of
    even / odd steps, v124 score bytes C); E_B (v50) is a temporary here."""
    ioh, ioe, l0h, l0e = ("v40", "v41", "v42", "v43") if even else ("v42", "v43", "v40", "v41")
    tc = "v122" if even else "v123"
    a(f"v_add_u32_sdwa v51, sext(v55), {l0h} dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_{b} src1_sel:DWORD")
    a(f"v_add_u32_sdwa v52, sext(v56), v44 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_{b} src1_sel:DWORD")
    a(f"v_add_u32_sdwa {tc}, sext(v124), v47 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_{b} src1_sel:DWORD")
    a(f"v_mov_b32_dpp {l0h}, {ioh} wave_shl:1 row_mask:0xf bank_mask:0xf")
    a(f"v_add_u32_dpp {ioh}, v118, %[ng] wave_shr:1 row_mask:0xf bank_mask:0xf")
    a(f"v_mov_b32_dpp {l0e}, {ioe} wave_shl:1 row_mask:0xf bank_mask:0xf")
    a(f"v_add_u32_dpp {ioe}, v121, %[nge] wave_shr:1 row_mask:0xf bank_mask:0xf")
    a("v_max3_i32 v53, v46, v45, 0")            # F_A
    a(f"v_max_i32 v54, {ioe}, {ioh}")           # E_A
    a("v_max3_i32 v44, v51, v54, v53")          # H_A
    a("v_subrev_u32 v46, %[GE], v53")           # fhA
    a("v_subrev_u32 v45, %[GI], v44")           # hgOA
    a("v_subrev_u32 v54, %[GE], v54")           # E_A - GE
    a("v_max_i32 v50, v54, v45")                # E_B
    a("v_max3_i32 v53, v49, v48, 0")            # F_B
    a("v_max3_i32 v47, v52, v50, v53")          # H_B
    a("v_subrev_u32 v49, %[GE], v53")           # fhB
    a("v_subrev_u32 v48, %[GI], v47")           # hgOB
    a("v_subrev_u32 v50, %[GE], v50")           # E_B - GE
    a("v_max_i32 v121, v50, v48")               # E_C
    a("v_max3_i32 v53, v120, v119, 0")          # F_C
    a(f"v_max3_i32 v118, {tc}, v121, v53")      # H_C
    a("v_subrev_u32 v120, %[GE], v53")          # fhC
    a("v_subrev_u32 v119, %[GI], v118")         # hgOC
    a("v_max3_i32 v57, v57, v51, v52")          # M
    if not even:
        a("v_max3_i32 v57, v57, v122, v123")


def ring_granule_aff(a, key="%[ek]", key2="%[ek2]", cp="sc1"):
    """Publish lanes 32..63 of the I/O pair (the 32 newest outflow rows, row v117) as 16-B
    granules at their ring slots, rows outside [0, m) dropped (peer: slab keys, system scope)."""
    a("v_mov_b32 v104, v40")
    a(f"v_xor_b32 v105, {key}, v40")
    a("v_xor_b32 v105, v105, v110")
    a("v_mov_b32 v106, v41")
    a(f"v_xor_b32 v107, {key2}, v41")
    a("v_xor_b32 v107, v107, v110")
    a("v_cmp_gt_u32_e64 s[50:51], %[m], v117")
    a("s_and_b64 s[50:51], s[50:51], %[lhi]")
    a("v_cndmask_b32_e64 v109, -16, v108, s[50:51]")
    a("v_add_u32 v108, 0x200, v108")                    # 32 rows of 16 B on
    a("v_and_b32 v108, %[gomask16], v108")
    a("v_add_u32 v110, 0x400, v110")
    a("v_add_u32 v117, 32, v117")
    a(f"buffer_store_dwordx4 v[104:107], v109, %[gors], 0 offen {cp}")


def ring_gin_check_aff(a, key="%[ek]", key2="%[ek2]"):
    """s[58:59] = live lanes (row k0 + lane < m); s[50:51] = live lanes whose granule fails
    either half's check."""
    a("s_sub_i32 s54, %[m], s40")
    a("v_cmp_gt_i32_e64 s[58:59], s54, %[lane]")
    a("v_xor_b32 v113, v90, v91")
    a("v_xor_b32 v113, v113, v112")
    a(f"v_cmp_ne_u32_e64 s[56:57], {key}, v113")
    a("v_xor_b32 v113, v92, v93")
    a("v_xor_b32 v113, v113, v112")
    a(f"v_cmp_ne_u32_e64 vcc, {key2}, v113")
    a("s_or_b64 s[56:57], s[56:57], vcc")
    a("s_and_b64 s[50:51], s[58:59], s[56:57]")
    a("s_cmp_lg_u64 s[50:51], 0")


def gen_role_ring_aff(IN, OUT_, W=2, hep=False):
    """gen_role_ring (C = 64, whole-chunk links) around the two-column affine step (W = 3: the
    three-column one, step_aff3); hep as gen_role_ring."""
    C = 64
    L = []
    a = L.append
    lds_in, lds_out = IN == "lds", OUT_ == "lds"
    gin, gout = IN in ("gran", "peer"), OUT_ in ("gran", "peer")
    kin = ("%[ekp]", "%[ek2p]", "sc0 sc1") if IN == "peer" else ("%[ek]", "%[ek2]", "sc1")
    kout = ("%[ekp]", "%[ek2p]", "sc0 sc1") if OUT_ == "peer" else ("%[ek]", "%[ek2]", "sc1")
    ncr = C // 16
    a("s_nop 4")
    a("s_waitcnt vmcnt(0) lgkmcnt(0)")
    for r in ("v44", "v47", "v50", "v57") + (("v118", "v121") if W == 3 else ()):
        a(f"v_mov_b32 {r}, 0")
    for r in ("v45", "v48", "v40", "v42") + (("v119",) if W == 3 else ()):
        a(f"v_mov_b32 {r}, %[ng]")
    for r in ("v46", "v49", "v41", "v43") + (("v120",) if W == 3 else ()):
        a(f"v_mov_b32 {r}, %[nge]")
    a("v_mov_b32 v101, %[raw2]")
    a("v_mov_b32 v115, %[cro]")
    a("v_mov_b32 v116, %[rrow]")
    a("s_mov_b32 s40, 0")
    a("s_movk_i32 s41, 0")                             # (64 - C) * 8
    a(f"s_movk_i32 s42, {128 * SZA:#x}")               # ((0 + 128) mod R) * 8
    a("s_movk_i32 s53, 0xc0")
    a("s_mov_b32 s45, 0")
    a("s_mov_b32 s46, 0")
    a(f"s_movk_i32 s44, {RR}")
    a("s_mov_b32 s52, 0")
    if lds_out:
        a(f"v_mov_b32 v98, {(-64 - C) & 0xffffffff:#x}")
        a("v_add_u32 v97, s41, %[lout]")
    if lds_in:
        a(f"v_mov_b32 v99, {RR + C}")
        a("v_add_u32 v96, s42, %[lin]")
    if gout:
        a("v_mov_b32 v108, %[gooff]")
        a("v_mov_b32 v110, %[gopos]")
        a("v_mov_b32 v117, %[gorow]")
    if gin:
        a("v_mov_b32 v111, %[gioff]")
        a("v_mov_b32 v112, %[gipos]")
        a(f"buffer_load_dwordx4 v[90:93], v111, %[girs], 0 offen {kin[2]}")
    for q in range(ncr):
        a(f"ds_read_b128 v[{58 + 4 * q}:{61 + 4 * q}], %[c0]" + (f" offset:{16 * q}" if q else ""))
    a("s_waitcnt vmcnt(0) lgkmcnt(0)")
    a(".p2align 6")                # the chunk loop on a 64-B boundary (a lone wave's issue rate depends on it)
    for _ in range(LOOP_PAD):
        a("s_nop 0")
    a("L_loop_%=:")
    for p in (0, 1):
        cur = 58 if p == 0 else 74
        nxt = 74 if p == 0 else 58
        lds = []
        if lds_out:
            if p == 0:
                a("s_cmp_lt_i32 s44, s40")
                a(f"s_cbranch_scc1 L_bp{p}_%=")
                a(f"L_bpr{p}_%=:")
            a("ds_write_b64 v97, v[40:41]")
            a("ds_write_b32 %[pout], v98")
            lds += ["W1", "W2"]
        if gout:
            a("s_add_u32 s55, s40, %[bpbase]")
            a("s_sub_u32 s54, s52, s55")
            a("s_cmp_lt_i32 s54, 0")
            a(f"s_cbranch_scc1 L_bpg{p}_%=")
            a(f"L_bpgr{p}_%=:")
            ring_granule_aff(a, *kout)
        if lds_in:
            a("ds_read_b32 v94, %[pin]")
            a("ds_read_b64 v[90:91], v96")
            lds += ["A", "B"]
        stores_after = 2 * gout + (1 if gin and p == 0 else 0)
        a(f"s_waitcnt vmcnt({stores_after})")
        if gin:
            ring_gin_check_aff(a, kin[0], kin[1])
            a(f"s_cbranch_scc1 L_gin{p}_%=")
            a(f"L_ginr{p}_%=:")
            a("v_cndmask_b32_e64 v40, %[ng], v90, s[58:59]")
            a("v_cndmask_b32_e64 v41, %[nge], v92, s[58:59]")
        elif not lds_in:
            a("v_mov_b32 v40, %[ng]")
            a("v_mov_b32 v41, %[nge]")
        # codes of 64 rows (128..191 ahead of the body's first row) into the wave's code ring
        if hep:
            a("v_mov_b32 v102, v101")
        else:
            a("v_lshrrev_b32 v102, 1, v101")
            a("v_lshrrev_b32 v113, 2, v101")
            a("v_xor_b32 v102, v102, v113")
            a("v_and_or_b32 v102, v102, 3, 4")
            a("v_cmp_ne_u32_e64 s[56:57], 0, v101")
            a("v_cndmask_b32_e64 v102, 0, v102, s[56:57]")
        a("v_add_u32 v103, s53, %[cwr]")
        a("ds_write_b8 v103, v102")
        a("s_cmp_eq_u32 s53, 0")
        a("s_cselect_b32 s54, 0, 64")
        a("v_add_u32 v103, s54, %[cwm]")
        a("ds_write_b8 v103, v102")
        a("s_add_u32 s53, s53, 64")
        a("s_and_b32 s53, s53, 0xff")
        lds += ["C1", "C2"]
        a("v_add_u32 v116, 64, v116")
        a("buffer_load_ubyte v101, v116, %[rrs], 0 offen")
        if gin:
            a(f"v_add_u32 v111, {C * 16:#x}, v111")
            a("v_and_b32 v111, %[gimask16], v111")
            a(f"v_add_u32 v112, {C << 5:#x}, v112")
            a(f"buffer_load_dwordx4 v[90:93], v111, %[girs], 0 offen {kin[2]}")
            if p == 1:
                a(f"s_add_u32 s54, s40, {C}")
                a("s_min_i32 s54, s54, %[m]")
                a("s_add_u32 s54, s54, %[crv0]")
                a("v_mov_b32 v114, s54")
                a("buffer_store_dword v114, %[croff], %[cross], 0 offen sc1")
        a("v_add_u32 v95, %[cbase], v115")
        for q in range(ncr):
            a(f"ds_read_b128 v[{nxt + 4 * q}:{nxt + 4 * q + 3}], v95 offset:{16 * q}" if q else
              f"ds_read_b128 v[{nxt}:{nxt + 3}], v95")
        a(f"v_add_u32 v115, {C}, v115")
        a("v_and_b32 v115, 0xff, v115")
        lds += ["N%d" % q for q in range(ncr)]
        if lds_in:
            after_a = len(lds) - 1 - lds.index("A")
            a(f"s_waitcnt lgkmcnt({after_a})")
            a("v_readfirstlane_b32 s43, v94")
            a("s_cmp_lt_i32 s43, s40")
            a(f"s_cbranch_scc1 L_in{p}_%=")
            a(f"L_inr{p}_%=:")
            a(f"s_waitcnt lgkmcnt({after_a - 1})")
            a("v_mov_b32 v40, v90")
            a("v_mov_b32 v41, v91")
            a("ds_write_b32 %[qme], v99")
        else:
            a(f"s_waitcnt lgkmcnt({len(lds)})")
        for u in range(C // 4):
            qa, qb, qc = ("%[qA]", "%[qB]", "%[qC]") if hep else ("%[k80]",) * 3
            a(f"v_perm_b32 v55, %[pA], {qa}, v{cur + u}")
            a(f"v_perm_b32 v56, %[pB], {qb}, v{cur + u}")
            if W == 3:
                a(f"v_perm_b32 v124, %[pC], {qc}, v{cur + u}")
            for b in range(4):
                (step_aff3 if W == 3 else step_aff2)(a, b, b % 2 == 0)
            if gout and u == 7:
                ring_granule_aff(a, *kout)
        a(f"s_add_i32 s40, s40, {C}")
        if lds_out:
            a(f"s_add_u32 s41, s41, {SZA * C:#x}")
            a(f"s_and_b32 s41, s41, {(RR - 1) * SZA:#x}")
            a("v_add_u32 v97, s41, %[lout]")
            a(f"v_add_u32 v98, {C}, v98")
        if lds_in:
            a(f"s_add_u32 s42, s42, {SZA * C:#x}")
            a(f"s_and_b32 s42, s42, {(RR - 1) * SZA:#x}")
            a("v_add_u32 v96, s42, %[lin]")
            a(f"v_add_u32 v99, {C}, v99")
    a("s_cmp_lt_i32 s40, %[end]")
    a("s_cbranch_scc1 L_loop_%=")
    if lds_out:
        a("s_cmp_lt_i32 s44, s40")
        a("s_cbranch_scc1 L_bpx_%=")
        a("L_bpxr_%=:")
        a("ds_write_b64 v97, v[40:41]")
        a(f"v_mov_b32 v98, {BIG:#x}")
        a("ds_write_b32 %[pout], v98")
    if gout:
        a("s_add_u32 s55, s40, %[bpbase]")
        a("s_sub_u32 s54, s52, s55")
        a("s_cmp_lt_i32 s54, 0")
        a("s_cbranch_scc1 L_bpgx_%=")
        a("L_bpgxr_%=:")
        ring_granule_aff(a, *kout)
    if gin:
        a("s_add_u32 s54, %[m], %[crv0]")
        a("v_mov_b32 v114, s54")
        a("buffer_store_dword v114, %[croff], %[cross], 0 offen sc1")
    a("s_waitcnt vmcnt(0) lgkmcnt(0)")
    a("v_mov_b32 %[M], v57")
    a("s_mov_b32 %[fail], s45")
    a("s_mov_b32 %[slow], s46")
    a("s_branch L_done_%=")
    if lds_in:
        for p in (0, 1):
            slow_wait(a, f"L_in{p}_%=", f"L_inr{p}_%=", "v94", "%[pin]", "s43", reread="ds_read_b64 v[90:91], v96")
    if lds_out:
        slow_wait(a, "L_bp0_%=", "L_bpr0_%=", "v100", "%[qnx]", "s44")
        slow_wait(a, "L_bpx_%=", "L_bpxr_%=", "v100", "%[qnx]", "s44")
    if gout:
        for lab, res in (("L_bpg0_%=", "L_bpgr0_%="), ("L_bpg1_%=", "L_bpgr1_%="), ("L_bpgx_%=", "L_bpgxr_%=")):
            slow_bp_hbm_aff(a, lab, res)
    if gin:
        for p in (0, 1):
            slow_gin_aff(a, f"L_gin{p}_%=", f"L_ginr{p}_%=", *kin)
    a("L_done_%=:")
    return L


def slow_bp_hbm_aff(a, label, resume):
    a(f"{label}:")
    a("s_add_u32 s46, s46, 1")
    a("s_cmp_lg_u32 s45, 0")
    a(f"s_cbranch_scc1 {resume}")
    a(f"{label}_w:")
    a("buffer_load_dword v100, off, %[bpr], 0 sc1")
    a("s_waitcnt vmcnt(0) lgkmcnt(0)")
    a("v_readfirstlane_b32 s52, v100")
    a("s_add_u32 s55, s40, %[bpbase]")
    a("s_sub_u32 s54, s52, s55")
    a("s_cmp_ge_i32 s54, 0")
    a(f"s_cbranch_scc1 {resume}")
    slow_timeout(a, label)
    a(f"{label}_x:")
    a("s_mov_b32 s45, 1")
    a(f"s_branch {resume}")


def slow_gin_aff(a, label, resume, key="%[ek]", key2="%[ek2]", cp="sc1"):
    a(f"{label}:")
    a("s_add_u32 s46, s46, 1")
    a("s_cmp_lg_u32 s45, 0")
    a(f"s_cbranch_scc1 {resume}")
    a(f"{label}_w:")
    a(f"buffer_load_dwordx4 v[90:93], v111, %[girs], 0 offen {cp}")
    a("s_waitcnt vmcnt(0) lgkmcnt(0)")
    ring_gin_check_aff(a, key, key2)
    a(f"s_cbranch_scc0 {resume}")
    slow_timeout(a, label)
    a(f"{label}_x:")
    a("s_mov_b32 s45, 1")
    a(f"s_branch {resume}")


CLOBBERS_RING_AFF = ['"v%d"' % r for r in range(40, 118)] + \
    ['"s%d"' % r for r in range(40, 60) if r not in (47,)] + ['"scc"', '"vcc"', '"memory"']
OUT_RING_AFF = os.path.join(ROOT, "concurrentproject_amd", "csrc", "sw_flow3ra_loops.inc")


def emit_ring_aff():
    out = ["// GENERATED by tools/gen_flow3.py -- do not edit.  The flow3 ring-mode affine-step chunk loops",
           "// (sw_flow3.hip sw_flow3ra_kernel): one inline-asm block per strip role, C = 64, R = %d rows of 8-B slots;" % RR,
           "// f3ra3_loop: three columns per lane (step_aff3), ALN = 1 the s_nop-aligned ones of the column-slab kernel.",
           "// Operands: see F3RALoop in sw_flow3.hip; fixed registers: tools/gen_flow3.py (gen_role_ring_aff).",
           "#pragma once", ""]
    ring_roles = [(i, o) for i in ROLES_IN_RING for o in ROLES_OUT]
    # aln 2: the W3 ring roles of a pair over up to seven byte values (f3ra3h_loop, sw_flow3ra3h_kernel)
    combos = [(i, o, 2, 0) for i, o in ring_roles + list(ROLES_SLAB)] + \
        [(i, o, 3, 0) for i, o in ring_roles] + [(i, o, 3, 1) for i, o in ring_roles + list(ROLES_SLAB)] + \
        [(i, o, 3, 2) for i, o in ring_roles]
    for IN, OUT_, W, aln in combos:
        hep = aln == 2
        body = gen_role_ring_aff(IN, OUT_, W, hep)
        if W == 2 and RING_ALIGN:
            body = align8(body, nops=RING_NOPS)
        if aln == 1:
            body = align8(body, nops=True, promote=False)
        if W == 2:
            out.append("template <> __device__ __forceinline__ F3Res f3ra_loop<F3_%s, F3_%s>(const F3RALoop& x) {"
                       % (IN.upper(), OUT_.upper()))
        elif hep:
            out.append("template <> __device__ __forceinline__ F3Res f3ra3h_loop<F3_%s, F3_%s>(const F3RALoop& x) {"
                       % (IN.upper(), OUT_.upper()))
        else:
            out.append("template <> __device__ __forceinline__ F3Res f3ra3_loop<F3_%s, F3_%s, %d>(const F3RALoop& x) {"
                       % (IN.upper(), OUT_.upper(), aln))
        out.append("    F3Res r;")
        out.append("    asm volatile(")
        for line in body:
            out.append('        "%s\\n\\t"' % line)
        out.append('        : [M] "=v"(r.M), [fail] "=s"(r.fail), [slow] "=s"(r.slow)')
        out.append('        : [pA] "v"(x.pA), [pB] "v"(x.pB), [ng] "v"(x.ng), [nge] "v"(x.nge), [GI] "s"(x.GI),' if W == 2 else
                   '        : [pA] "v"(x.pA), [pB] "v"(x.pB), [pC] "v"(x.pC), [ng] "v"(x.ng), [nge] "v"(x.nge), [GI] "s"(x.GI),')
        out.append('          [GE] "s"(x.GE), ' + ('[qA] "v"(x.qA), [qB] "v"(x.qB), [qC] "v"(x.qC),' if hep else '[k80] "s"(x.k80),') +
                   ' [m] "s"(x.m), [end] "s"(x.end), [dlo] "s"(x.dlo),')
        out.append('          [dhi] "s"(x.dhi), [lane] "v"(x.lane), [raw2] "v"(x.raw2), [cro] "v"(x.cro), [c0] "v"(x.c0),')
        out.append('          [cbase] "v"(x.cbase), [cwr] "v"(x.cwr), [cwm] "v"(x.cwm), [rrs] "s"(x.rrs), [rrow] "v"(x.rrow),')
        out.append('          [lin] "v"(x.lin), [lout] "v"(x.lout), [pin] "v"(x.pin), [pout] "v"(x.pout),')
        out.append('          [qme] "v"(x.qme), [qnx] "v"(x.qnx),')
        out.append('          [girs] "s"(x.girs), [gioff] "v"(x.gioff), [gipos] "v"(x.gipos), [gimask16] "s"(x.gimask16),')
        out.append('          [ek] "s"(x.ek), [ek2] "s"(x.ek2), [cross] "s"(x.cross), [crv0] "s"(x.crv0), [croff] "v"(x.croff),')
        out.append('          [gors] "s"(x.gors), [gooff] "v"(x.gooff), [gopos] "v"(x.gopos), [gomask16] "s"(x.gomask16),')
        out.append('          [gorow] "v"(x.gorow), [lhi] "s"(x.lhi), [bpr] "s"(x.bpr), [bpbase] "s"(x.bpbase),')
        out.append('          [ekp] "s"(x.ekp), [ek2p] "s"(x.ek2p)')
        clob = CLOBBERS_RING_AFF + (['"v%d"' % r for r in range(118, 125)] if W == 3 else [])
        out.append("        : " + ", ".join(clob) + ");")
        out.append("    return r;")
        out.append("}")
        out.append("")
    return "\n".join(out)


# ============================================================================================
# Pool loops (staged organisation, sw_flow3.hip flow3_staged<..., POOL = true>, the default):
# the same strips, steps and chunks, WITHOUT the rotating I/O register.  The rotation exists to
# bring inflow row k to lane 0 at step k and to collect lane 63's outflow: one DPP move per
# flowing quantity per step (1 of the linear-gap step's 9.5 VALU, 2 of the affine step's
# 10.75).  Here every step k owns a register P(k) of a 32-step pool:
#   * inflow: 16-B broadcast LDS reads (one address for the whole wave) put row k into every
#     lane of P(k) before step k; the step's tied DPP-add (old = P(k)) writes H[l-1] - G into
#     lanes 1..63 and keeps the inflow in lane 0 -- no move.  No inflow (strip 0): bound_ctrl
#     zero-fills lane 0's source, so lane 0 gets 0 + (-G), the boundary value;
#   * diagonal: P(k - 1) is still intact at step k (it was the last step's hgL);
#   * outflow: after a half chunk lane 63 of P(c) .. P(c + 15) holds rows c - 63 .. c - 48; one
#     exec-masked (lane 63) run of 16-B LDS writes stores them into the consumer's ring.
# Per 16 steps this trades 16 (32 affine) DPP moves for 4 (8) reads, 4 (8) writes and 2 SALU.
# A 16-B group is G rows (4 linear-gap 4-B slots, 2 affine 8-B slots) and 4 aligned pool
# registers.  Input rows = steps and output rows = steps - 63 cannot both fall on the same
# 16-row halves of one wave, so wave w of a workgroup runs its halves shifted by SH = w steps
# (steps [16h + w, 16h + w + 16), pool index (k - w) mod 32): its output halves are then
# exactly wave w + 1's input halves, and every link's rows [32j + SH_consumer, + 32)
# ("window" j) occupy the ring slots [(32j + 128) mod R, + 32), contiguous (slot of row r:
# (r + 128 - SH_consumer) mod R).  The loader writes row r at slot (r + 128) mod R (wave 0
# runs SH = 0).  Words: prod = rows available (rows < prod are in the
# ring), cons = rows consumed + R; both move once per half chunk (16 rows), as the half-chunk
# links did.  The granule role (the group's last strip) writes its halves into its own ring
# and reads 16 rows back lane-parallel for the 8-B / 16-B granules.
# ============================================================================================
POOL_LOW = int(os.environ.get("F3P_LOW", "0"))   # A/B: linear-gap pool at v96..v127, control registers at v48..v63
POOL_BASE = 128
POOL_A = int(os.environ.get("F3P_A", "2"))     # steps a half's inflow reads are issued ahead of it
POOL_WD = int(os.environ.get("F3P_WD", "4"))   # steps the producer-word read runs ahead of the check
POOL_GS = int(os.environ.get("F3P_GS", "2"))   # steps between a granule read-back and its store
POOL_PAD = int(os.environ.get("F3P_PAD", "0"))   # A/B probe: 1 s_nop / 2 VALU before the step's DPP-add
POOL_NOW = int(os.environ.get("F3P_NOW", "0"))   # timing probe only (wrong results): no outflow data writes
POOL_NOR = int(os.environ.get("F3P_NOR", "0"))   # timing probe only (wrong results): no inflow data reads
POOL_SCRATCH = int(os.environ.get("F3P_SCRATCH", "1"))   # outflow writes by all lanes, 0..62 into scratch (no exec writes)
PC = dict(word="v100", caddr="v101", iaddr="v102", oaddr="v104", pval="v105", cval="v107", bp="v108",
          rbaddr="v109", goff="v110", gmask="v111", rb="v112", rb2="v113", go="v116")
PC_LOW = dict(word="v48", caddr="v49", iaddr="v50", oaddr="v51", pval="v52", cval="v53", bp="v54",
              rbaddr="v55", goff="v56", gmask="v57", rb="v58", rb2="v59", go="v60")


def _pool_base(aff):
    return 96 if (POOL_LOW and not aff) else POOL_BASE


def _pool_reg(k, PI, aff):
    idx = (k + PI) % 32
    return _pool_base(aff) + 2 * idx if aff else _pool_base(aff) + idx


def step_pool_lin(a, k, PI, bc):
    """One step of the two-column linear-gap step on pool register P(k): 8 VALU + the
    running max (the rotation is gone; sw_flow2.hip step_lin2, main.cpp:54-66)."""
    P = "v%d" % _pool_reg(k, PI, False)
    Pp = "v%d" % _pool_reg(k - 1, PI, False)
    b = k % 4
    a(f"v_add_u32_sdwa v70, sext(v72), {Pp} dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_{b} src1_sel:DWORD")
    a(f"v_add_u32_sdwa v71, sext(v73), v66 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_{b} src1_sel:DWORD")
    if POOL_PAD == 1:
        a("s_nop 0")
    elif POOL_PAD == 2:
        a("v_mov_b32 v119, v119")
    a(f"v_add_u32_dpp {P}, v68, %[ng] wave_shr:1 row_mask:0xf bank_mask:0xf" + (" bound_ctrl:1" if bc else ""))
    a(f"v_max3_i32 v66, {P}, v67, v70")
    a("v_sub_u32_e64 v67, v66, %[G] clamp")
    a("v_max3_i32 v68, v67, v69, v71")
    a("v_sub_u32_e64 v69, v68, %[G] clamp")
    a("v_max3_i32 v74, v74, v70, v71")


def step_pool_aff(a, k, PI, bc):
    """One step of the one-column affine step on pool registers (PH(k), PE(k)): 8 VALU + the
    running max every other step (step_aff1 without its two rotations)."""
    r = _pool_reg(k, PI, True)
    PH, PE = "v%d" % r, "v%d" % (r + 1)
    PHp = "v%d" % _pool_reg(k - 1, PI, True)
    t = "v73" if k % 2 == 0 else "v74"
    z = " bound_ctrl:1" if bc else ""
    a(f"v_add_u32_sdwa {t}, sext(v75), {PHp} dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_{k % 4} src1_sel:DWORD")
    a(f"v_add_u32_dpp {PH}, v68, %[ng] wave_shr:1 row_mask:0xf bank_mask:0xf" + z)
    a(f"v_add_u32_dpp {PE}, v72, %[nge] wave_shr:1 row_mask:0xf bank_mask:0xf" + z)
    a("v_max3_i32 v70, v71, v69, 0")
    a(f"v_max_i32 v72, {PE}, {PH}")
    a(f"v_max3_i32 v68, {t}, v72, v70")
    a("v_subrev_u32 v71, %[GE], v70")
    a("v_subrev_u32 v69, %[G], v68")
    if k % 2:
        a("v_max3_i32 v76, v76, v73, v74")


def resolve_lgkm(items):
    """items: ("i", text) | ("op", name, text) | ("wait", names).  Each wait becomes the
    s_waitcnt lgkmcnt(n) that holds until the newest issue of any of `names` (searched back
    cyclically: the body is a loop) has completed -- LDS ops complete in order."""
    n = len(items)
    out = []
    for i, it in enumerate(items):
        if it[0] == "i":
            out.append(it[1])
        elif it[0] == "op":
            out.append(it[2])
        else:
            cnt = 0
            for d in range(1, n + 1):
                j = (i - d) % n
                if items[j][0] == "op":
                    if items[j][1] in it[1]:
                        break
                    cnt += 1
            else:
                raise AssertionError("wait for %s: never issued" % (it[1],))
            w = "s_waitcnt lgkmcnt(%d)" % min(cnt, 15)
            if out and out[-1].startswith("s_waitcnt lgkmcnt("):   # merge adjacent waits
                prev = int(out[-1][len("s_waitcnt lgkmcnt("):-1])
                out[-1] = "s_waitcnt lgkmcnt(%d)" % min(prev, min(cnt, 15))
            else:
                out.append(w)
    return out


def gen_pool(IN, OUT_, SH, aff):
    """The staged chunk loop of one strip role on the register pool (see above): C = 32-row
    chunks, a body of two chunks (64 steps), 16-row links.  SH = the wave's index in its
    workgroup: its halves are the steps [16h + SH, 16h + SH + 16), whose outflow rows are
    exactly wave SH + 1's halves (rows = steps - 63); pool index of step k = (k - SH) mod 32."""
    G, SZ = (2, 8) if aff else (4, 4)
    gsz = 16 if aff else 8                # granule bytes per row
    PI = -SH
    PC = PC_LOW if (POOL_LOW and not aff) else globals()["PC"]
    lds_in, lds_out, gran = IN == "lds", OUT_ == "lds", OUT_ == "gran"
    A, WD, GS = POOL_A, POOL_WD, POOL_GS
    ngrp = 16 // G                        # 16-B groups per half
    ev = {p: [] for p in range(65)}       # items before step p (p = 64: after the last step)

    def base(pos):                        # s40 (k0) at body position pos, relative to the body's first row
        return 0 if pos < 32 else 32

    def place(e):
        """body position of an event at step e (relative to its half's body) and the row shift
        from that body to the one the event runs in"""
        if e < 0:
            return e + 64, 64
        if e > 64:
            return e - 64, -64
        return e, 0

    I = lambda t: ("i", t)

    def check(h, c, shift, pos, label):
        return [("wait", ("w%d" % h,)) if h is not None else I("s_waitcnt lgkmcnt(0)"),
                I(f"v_readfirstlane_b32 s43, {PC['word']}"),
                I(f"s_add_u32 s52, s40, {c + 16 + shift - base(pos)}"),
                I("s_cmp_lt_i32 s43, s52"),
                I(f"s_cbranch_scc1 L_in{label}_%="),
                I(f"L_inr{label}_%=:")]

    def reads(h, c, tag):
        out = []
        if h % 2 == 0:                    # a new window: ((32 j + 128) mod R) slots
            out.append(I(f"s_add_u32 s41, s41, {32 * SZ:#x}"))
            out.append(I(f"s_and_b32 s41, s41, {R * SZ - 1:#x}"))
            out.append(I(f"v_add_u32 {PC['iaddr']}, s41, %[lin]"))
        for i in range(ngrp):
            r = _pool_reg(c + G * i, PI, aff)
            if POOL_NOR and i > 0:
                continue
            out.append(("op", tag, f"ds_read_b128 v[{r}:{r + 3}], {PC['iaddr']} offset:{(h % 2) * 16 * SZ + 16 * i}"))
        return out

    slow_in = []
    # ---- consumer: half h covers steps [c, c + 16), c = 16 h + SH
    if lds_in:
        for h in range(4):
            c = 16 * h + SH
            pw, _ = place(c - A - WD)
            pc_, sh_c = place(c - A)
            pd, _ = place(c)
            ev[pw].append(("op", "w%d" % h, f"ds_read_b32 {PC['word']}, %[pin]"))
            its = check(h, c, sh_c, pc_, h) + reads(h, c, "d%d" % h)
            if h % 2 == 1:                # rows < c + 16 consumed: report once per window
                its.append(I(f"v_add_u32 {PC['cval']}, 32, {PC['cval']}"))
                its.append(("op", "q%d" % h, f"ds_write_b32 %[qme], {PC['cval']}"))
            ev[pc_].extend(its)
            ev[pd].append(("wait", ("d%d" % h,)))
            slow_in.append(str(h))
    # ---- producer: half h's outflow (rows c - 63 .. c - 48) once its last step is done
    if lds_out or gran:
        for h in range(4):
            c = 16 * h + SH
            pe, sh_e = place(c + 16)
            its = []
            if h % 2 == 0:
                if lds_out:               # the window's slots held rows < c - 31 - R
                    its += [I(f"s_add_u32 s52, s40, {c - 31 + sh_e - base(pe)}"),
                            I("s_cmp_lt_i32 s44, s52"),
                            I(f"s_cbranch_scc1 L_bp{h}_%="),
                            I(f"L_bpr{h}_%=:")]
                its += [I(f"s_add_u32 s42, s42, {32 * SZ:#x}"),
                        I(f"s_and_b32 s42, s42, {R * SZ - 1:#x}"),
                        I(f"v_add_u32 {PC['oaddr']}, s42, %[lout]")]
                if POOL_SCRATCH:          # lanes 0..62 write into their scratch slots
                    its.append(I(f"v_cndmask_b32_e64 {PC['oaddr']}, %[lsc], {PC['oaddr']}, %[l63]"))
                if gran:
                    its.append(I(f"v_add_u32 {PC['rbaddr']}, s42, %[lrb]"))
            if not POOL_SCRATCH:
                its.append(I("s_mov_b64 exec, %[l63]"))
            for i in range(ngrp):
                r = _pool_reg(c + G * i, PI, aff)
                if POOL_NOW and i > 0:
                    continue
                its.append(("op", "o%d" % h, f"ds_write_b128 {PC['oaddr']}, v[{r}:{r + 3}] offset:{(h % 2) * 16 * SZ + 16 * i}"))
            if not POOL_SCRATCH:
                its.append(I("s_mov_b64 exec, -1"))
            if lds_out:
                its.append(I(f"v_add_u32 {PC['pval']}, 16, {PC['pval']}"))
                its.append(("op", "p%d" % h, f"ds_write_b32 %[pout], {PC['pval']}"))
            if gran:                      # read the half back lane-parallel (lanes 0..15 = its rows)
                rb = f"v[{PC['rb'][1:]}:{PC['rb2'][1:]}]" if aff else PC['rb']
                its.append(("op", "r%d" % h, f"ds_read_b{64 if aff else 32} {rb}, {PC['rbaddr']} offset:{(h % 2) * 16 * SZ}"))
            ev[pe].extend(its)
            if gran:
                ps = min(pe + GS, 64)
                g = int(PC["go"][1:])
                st = [("wait", ("r%d" % h,))]
                if aff:
                    st += [I(f"v_mov_b32 v{g}, {PC['rb']}"),
                           I(f"v_xor_b32 v{g + 1}, %[ek], {PC['rb']}"),
                           I(f"v_mov_b32 v{g + 2}, {PC['rb2']}"),
                           I(f"v_xor_b32 v{g + 3}, %[ek2], {PC['rb2']}")]
                else:
                    st += [I(f"v_xor_b32 {PC['rb2']}, %[ek], {PC['rb']}")]
                st += [I(f"v_cndmask_b32_e64 {PC['gmask']}, -16, {PC['goff']}, %[m16]"),
                       I(f"v_add_u32 {PC['goff']}, {16 * gsz:#x}, {PC['goff']}")]
                if aff:
                    st.append(I(f"buffer_store_dwordx4 v[{g}:{g + 3}], {PC['gmask']}, %[rsrc], 0 offen sc1"))
                else:
                    st.append(I(f"buffer_store_dwordx2 v[{PC['rb'][1:]}:{PC['rb2'][1:]}], {PC['gmask']}, %[rsrc], 0 offen sc1"))
                ev[ps].extend(st)

    # ---- the body: chunk tops (codes of the next chunk), events, perms, steps
    body = []
    for k in range(64):
        if k == 32:
            body.append(I("s_add_i32 s40, s40, 32"))
        if k in (0, 32):
            body.append(("wait", ("c1",) if k == 0 else ("c0",)))
            nxt = (84 if not aff else 88) if k == 0 else (76 if not aff else 80)
            obase = 32 if k == 0 else 64
            for q in range(2):
                body.append(("op", "c0" if k == 0 else "c1",
                             f"ds_read_b128 v[{nxt + 4 * q}:{nxt + 4 * q + 3}], {PC['caddr']} offset:{obase + 16 * q}"))
        body.extend(ev[k])
        if k % 4 == 0:
            cur = (76 if k < 32 else 84) if not aff else (80 if k < 32 else 88)
            u = (k % 32) // 4
            if aff:
                body.append(I(f"v_perm_b32 v75, %[pA], %[k80], v{cur + u}"))
            else:
                body.append(I(f"v_perm_b32 v72, %[pA], %[k80], v{cur + u}"))
                body.append(I(f"v_perm_b32 v73, %[pB], %[k80], v{cur + u}"))
        lines = []
        (step_pool_aff if aff else step_pool_lin)(lines.append, k, PI, not lds_in)
        body.extend(I(t) for t in lines)
    body.extend(ev[64])
    body.append(I("s_add_i32 s40, s40, 32"))
    body.append(I(f"v_add_u32 {PC['caddr']}, 64, {PC['caddr']}"))
    loop = resolve_lgkm(body)

    L = []
    a = L.append
    a("s_nop 4")
    a("s_waitcnt vmcnt(0) lgkmcnt(0)")
    if aff:
        for r in ("v68", "v70", "v72", "v76"):
            a(f"v_mov_b32 {r}, 0")
        a("v_mov_b32 v69, %[ng]")
        a("v_mov_b32 v71, %[nge]")
        for i in range(32):
            a(f"v_mov_b32 v{POOL_BASE + 2 * i}, %[ng]")
            a(f"v_mov_b32 v{POOL_BASE + 2 * i + 1}, %[nge]")
    else:
        for r in ("v66", "v67", "v68", "v69", "v74"):
            a(f"v_mov_b32 {r}, 0")
        for i in range(32):
            a(f"v_mov_b32 v{_pool_base(False) + i}, %[ng]")
    a(f"v_mov_b32 {PC['caddr']}, %[code]")
    a("s_mov_b32 s40, 0")
    a(f"s_movk_i32 s41, {96 * SZ:#x}")     # window 0's slots (128) after its first update
    a(f"s_movk_i32 s42, {32 * SZ:#x}")     # the producer's windows: slots 64 after the first update
    a("s_mov_b32 s45, 0")
    a("s_mov_b32 s46, 0")
    a(f"s_movk_i32 s44, {R}")
    # (SH > 0: the body's first event writes the last body's half 3, here junk rows < -63)
    first = SH - 63 - (16 if SH > 0 else 0)
    if lds_out or gran:   # (the wrapped first write lands in window -3: slots of rows < -63)
        a(f"v_add_u32 {PC['oaddr']}, s42, %[lout]")
        if POOL_SCRATCH:
            a(f"v_cndmask_b32_e64 {PC['oaddr']}, %[lsc], {PC['oaddr']}, %[l63]")
    if gran:
        a(f"v_add_u32 {PC['rbaddr']}, s42, %[lrb]")
    if lds_out:   # rows available after the first publish: first + 16
        a(f"v_mov_b32 {PC['pval']}, {first & 0xffffffff:#x}")
    if lds_in:
        a(f"v_mov_b32 {PC['cval']}, {R + SH}")
        a(f"v_add_u32 {PC['iaddr']}, s41, %[lin]")   # (the last body's half 3 reads window -1)
    if gran:
        a(f"v_mov_b32 {PC['goff']}, %[lrow]")
    cur0 = 80 if aff else 76
    for q in range(2):
        a(f"ds_read_b128 v[{cur0 + 4 * q}:{cur0 + 4 * q + 3}], {PC['caddr']} offset:{16 * q}")
    if lds_in:   # the halves whose reads the body issues one body early: the last body's half 3, half 0
        for h in ([-1] if SH > 0 else []) + ([0] if SH - A < 0 else []):
            c = 16 * h + SH
            a(f"ds_read_b32 {PC['word']}, %[pin]")
            for it in check(None, c, 0, 0, "P%d" % (h + 1)) + reads(h % 4, c, "dP"):
                a(it[1] if it[0] == "i" else it[2])
            slow_in.append("P%d" % (h + 1))
    a("s_waitcnt lgkmcnt(0)")
    a(".p2align 6")
    a("L_loop_%=:")
    L.extend(loop)
    a("s_cmp_lt_i32 s40, %[end]")
    a("s_cbranch_scc1 L_loop_%=")
    if lds_out:
        a(f"v_mov_b32 {PC['pval']}, {BIG:#x}")
        a(f"ds_write_b32 %[pout], {PC['pval']}")
    a("s_waitcnt vmcnt(0) lgkmcnt(0)")
    a("v_mov_b32 %%[M], %s" % ("v76" if aff else "v74"))
    a("s_mov_b32 %[fail], s45")
    a("s_mov_b32 %[slow], s46")
    a("s_branch L_done_%=")
    for lab in slow_in:
        slow_wait(a, f"L_in{lab}_%=", f"L_inr{lab}_%=", PC["word"], "%[pin]", "s43", target="s52")
    if lds_out:
        for h in (0, 2):
            slow_wait(a, f"L_bp{h}_%=", f"L_bpr{h}_%=", PC["bp"], "%[qnx]", "s44", target="s52")
    a("L_done_%=:")
    return L


# the (IN, OUT) roles of each wave of a staged workgroup (shift SH = the wave): wave 0 takes the
# loader's ring or no inflow, waves 1..3 an LDS ring; waves 0..2 hand on through LDS, wave 3
# through granules; any wave may hold the pair's last strip (no outflow)
POOL_ROLES = [(0, "none", "lds"), (0, "none", "none"), (0, "lds", "lds"), (0, "lds", "none"),
              (1, "lds", "lds"), (1, "lds", "none"), (2, "lds", "lds"), (2, "lds", "none"),
              (3, "lds", "gran"), (3, "lds", "none")]
CLOBBERS_POOL = ['"v%d"' % r for r in range(64, 120)] + \
    ['"s%d"' % r for r in range(40, 53) if r != 47] + ['"scc"', '"vcc"', '"memory"']
OUT_POOL = os.path.join(ROOT, "concurrentproject_amd", "csrc", "sw_flow3p_loops.inc")


def emit_pool():
    out = ["// GENERATED by tools/gen_flow3.py -- do not edit.  The flow3 pool chunk loops (sw_flow3.hip",
           "// flow3_staged, POOL): inflow rows broadcast from LDS into a 32-step register pool, outflow by",
           "// lane 63 under an exec mask, no I/O rotation; C = 32, 16-row links, R = %d ring rows." % R,
           "// Operands: see F3PLoop in sw_flow3.hip; fixed registers: tools/gen_flow3.py (gen_pool).",
           "#pragma once", ""]
    for aff in (False, True):
        for w, IN, OUT_ in POOL_ROLES:
            body = align8(gen_pool(IN, OUT_, w, aff))
            if POOL_LOW and not aff:
                clob = ['"v%d"' % r for r in range(48, 128)] + CLOBBERS_POOL[56:]
            else:
                top = POOL_BASE + (64 if aff else 32)
                clob = CLOBBERS_POOL + ['"v%d"' % r for r in range(POOL_BASE, top)]
            out.append("template <> __device__ __forceinline__ F3Res f3p_loop<%d, F3_%s, F3_%s, %d>(const F3PLoop& x) {"
                       % (int(aff), IN.upper(), OUT_.upper(), w))
            out.append("    F3Res r;")
            out.append("    asm volatile(")
            for line in body:
                out.append('        "%s\\n\\t"' % line)
            out.append('        : [M] "=v"(r.M), [fail] "=s"(r.fail), [slow] "=s"(r.slow)')
            out.append('        : [pA] "v"(x.pA), [pB] "v"(x.pB), [ng] "v"(x.ng), [nge] "v"(x.nge), [G] "s"(x.G),')
            out.append('          [GE] "s"(x.GE), [k80] "s"(x.k80), [code] "v"(x.code), [lin] "v"(x.lin),')
            out.append('          [lout] "v"(x.lout), [lrb] "v"(x.lrb), [pin] "v"(x.pin), [pout] "v"(x.pout),')
            out.append('          [qme] "v"(x.qme), [qnx] "v"(x.qnx), [end] "s"(x.end), [dlo] "s"(x.dlo),')
            out.append('          [dhi] "s"(x.dhi), [rsrc] "s"(x.rsrc), [ek] "s"(x.ek), [ek2] "s"(x.ek2),')
            out.append('          [lrow] "v"(x.lrow), [m16] "s"(x.m16), [l63] "s"(x.l63), [lsc] "v"(x.lsc)')
            out.append("        : " + ", ".join(clob) + ");")
            out.append("    return r;")
            out.append("}")
            out.append("")
    return "\n".join(out)


def main():
    spec = int(os.environ.get("F3_SPEC", "4"))
    halfpub = os.environ.get("F3_HALFPUB", "1") != "0"
    text = emit(spec, halfpub)
    text_pool = emit_pool()
    text_ring3 = emit_ring3()
    text_ring45 = emit_ring45()
    text_ring = emit_ring()
    text_aff = emit_aff()
    text_ring_aff = emit_ring_aff()
    if "--check" in sys.argv:
        cur = open(OUT).read() if os.path.exists(OUT) else ""
        cur_r = open(OUT_RING).read() if os.path.exists(OUT_RING) else ""
        cur_a = open(OUT_AFF).read() if os.path.exists(OUT_AFF) else ""
        cur_ra = open(OUT_RING_AFF).read() if os.path.exists(OUT_RING_AFF) else ""
        cur_p = open(OUT_POOL).read() if os.path.exists(OUT_POOL) else ""
        cur_r3 = open(OUT_RING3).read() if os.path.exists(OUT_RING3) else ""
        cur_r45 = open(OUT_RING45).read() if os.path.exists(OUT_RING45) else ""
        sys.exit(0 if cur == text and cur_r == text_ring and cur_a == text_aff and cur_ra == text_ring_aff and
                 cur_p == text_pool and cur_r3 == text_ring3 and cur_r45 == text_ring45 else 1)
    with open(OUT_POOL, "w") as f:
        f.write(text_pool)
    with open(OUT_RING3, "w") as f:
        f.write(text_ring3)
    with open(OUT_RING45, "w") as f:
        f.write(text_ring45)
    with open(OUT_AFF, "w") as f:
        f.write(text_aff)
    with open(OUT_RING_AFF, "w") as f:
        f.write(text_ring_aff)
    path = OUT
    for i, arg in enumerate(sys.argv):
        if arg == "-o":
            path = sys.argv[i + 1]
    with open(path, "w") as f:
        f.write(text)
    with open(OUT_RING, "w") as f:
        f.write(text_ring)


if __name__ == "__main__":
    main()
