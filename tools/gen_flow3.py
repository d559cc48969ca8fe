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
ROLES_OUT = ("none", "lds", "gran")


def step(a, io, l0, b):
    """One anti-diagonal step of the two-column linear-gap step (9 VALU, 128 cells)."""
    a(f"v_add_u32_sdwa v70, sext(v72), {l0} dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_{b} src1_sel:DWORD")
    a(f"v_add_u32_sdwa v71, sext(v73), v66 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_{b} src1_sel:DWORD")
    a(f"v_mov_b32_dpp {l0}, {io} wave_shl:1 row_mask:0xf bank_mask:0xf")
    a(f"v_add_u32_dpp {io}, v68, %[ng] wave_shr:1 row_mask:0xf bank_mask:0xf")
    a(f"v_max3_i32 v66, {io}, v67, v70")
    a("v_sub_u32_e64 v67, v66, %[G] clamp")
    a("v_max3_i32 v68, v67, v69, v71")
    a("v_sub_u32_e64 v69, v68, %[G] clamp")
    a("v_max3_i32 v74, v74, v70, v71")


def granule(a):
    """Publish the 16 newest outflow rows (lanes 48..63 of the IO register v64) as
    8-B granules {H-G, (H-G) ^ epoch ^ 0x5BD1E995} at row * 8 of the group edge,
    write-through (sw_flow3.hip header).  v105 = this lane's row * 8 (rows < 0
    wrap to huge offsets: dropped by the buffer range check, as are rows past 2m)."""
    a("v_mov_b32 v100, v64")
    a("v_xor_b32 v101, %[ek], v64")
    a("v_cndmask_b32_e64 v106, -16, v105, %[m48]")
    a("v_add_u32 v105, 0x80, v105")     # (an independent VALU between the data writes and the store)
    a("buffer_store_dwordx2 v[100:101], v106, %[rsrc], 0 offen sc1")


def gen_role(IN, OUT_, spec=0, halfpub=True):
    L = []
    a = L.append
    lds_in, lds_out, gran = IN == "lds", OUT_ == "lds", OUT_ == "gran"
    nw = 3 if lds_out else 0            # LDS writes of a chunk's publish
    # ---- entry
    a("s_waitcnt vmcnt(0) lgkmcnt(0)")
    for r in ("v66", "v67", "v68", "v69", "v74"):
        a(f"v_mov_b32 {r}, 0")
    a("v_mov_b32 v64, %[ng]")
    a("v_mov_b32 v65, %[ng]")
    a("v_mov_b32 v94, %[code]")
    a("s_mov_b32 s40, 0")
    a("s_movk_i32 s41, 0x80")           # ((k0 + 32) mod R) * 4 at k0 = 0
    a("s_mov_b32 s45, 0")
    a("s_mov_b32 s46, 0")
    a(f"s_movk_i32 s44, {R}")            # consumer word seen: 0 rows consumed (+ R)
    if lds_out:
        a("v_mov_b32 v97, -96")          # producer word at chunk 0: k0 - 64 rows out, minus 32
        a("v_add_u32 v96, s41, %[lout]")
    if lds_in:
        a(f"v_mov_b32 v98, {R + 32}")    # consumer word after chunk 0: 32 rows consumed (+ R)
        a("v_add_u32 v95, s41, %[lin]")
    if gran:
        a("v_mov_b32 v105, %[lrow]")
    a("ds_read_b128 v[76:79], v94")
    a("ds_read_b128 v[80:83], v94 offset:16")
    if lds_in and spec:
        a("ds_read_b32 v93, %[pin]")
        a("ds_read_b32 v92, v95")
    a("L_loop_%=:")
    for p in (0, 1):
        cur = 76 if p == 0 else 84
        nxt = 84 if p == 0 else 76
        o0, o1 = (32, 48) if p == 0 else (64, 80)
        # ---- chunk top: publish the last chunk's outflow, take this chunk's inflow
        if lds_in and not spec:
            a("ds_read_b32 v93, %[pin]")
            a("ds_read_b32 v92, v95")
        if lds_out:
            if p == 0:   # back-pressure for this chunk's and the next chunk's publish
                a("s_cmp_lt_i32 s44, s40")
                a(f"s_cbranch_scc1 L_bp{p}_%=")
                a(f"L_bpr{p}_%=:")
            a("ds_write_b32 v96, v64")
            a(f"ds_write_b32 v96, v64 offset:{R * 4}")
            a("ds_write_b32 %[pout], v97")
        if gran:
            granule(a)
        a(f"ds_read_b128 v[{nxt}:{nxt + 3}], v94 offset:{o0}")
        a(f"ds_read_b128 v[{nxt + 4}:{nxt + 7}], v94 offset:{o1}")
        if lds_in:
            after = 1 + nw + 2           # LDS ops issued after the producer-word read
            a(f"s_waitcnt lgkmcnt({after})")
            a("v_readfirstlane_b32 s43, v93")
            a("s_cmp_lt_i32 s43, s40")
            a(f"s_cbranch_scc1 L_in{p}_%=")
            a(f"L_inr{p}_%=:")
            a(f"s_waitcnt lgkmcnt({after - 1})")
            a("v_mov_b32 v64, v92")
            a("ds_write_b32 %[qme], v98")
        else:
            a(f"s_waitcnt lgkmcnt({nw + 2})")
            a("v_mov_b32 v64, %[ng]")
        # ---- 32 steps, 8 groups of 4 rows (one v_perm_b32 per column per group)
        spec_at = 8 - spec // 4 if spec else None
        for u in range(8):
            if spec and u == spec_at:
                book(a, p, lds_in, lds_out)
                a("ds_read_b32 v93, %[pin]")
                a("ds_read_b32 v92, v95")
            a(f"v_perm_b32 v72, %[pA], %[k80], v{cur + u}")
            a(f"v_perm_b32 v73, %[pB], %[k80], v{cur + u}")
            for b in range(4):
                io, l0 = ("v64", "v65") if b % 2 == 0 else ("v65", "v64")
                step(a, io, l0, b)
            if gran and halfpub and u == 3:
                granule(a)
        if not spec:
            book(a, p, lds_in, lds_out)
    a("s_cmp_lt_i32 s40, %[end]")
    a("s_cbranch_scc1 L_loop_%=")
    # ---- exit: the last chunk's outflow, then every row is out
    if lds_out:
        a("s_cmp_lt_i32 s44, s40")
        a("s_cbranch_scc1 L_bpx_%=")
        a("L_bpxr_%=:")
        a("ds_write_b32 v96, v64")
        a(f"ds_write_b32 v96, v64 offset:{R * 4}")
        a(f"v_mov_b32 v97, {BIG:#x}")
        a("ds_write_b32 %[pout], v97")
    if gran:
        granule(a)
    a("s_waitcnt vmcnt(0) lgkmcnt(0)")
    a("v_mov_b32 %[M], v74")
    a("s_mov_b32 %[fail], s45")
    a("s_mov_b32 %[slow], s46")
    a("s_branch L_done_%=")
    # ---- slow paths (a late producer word, or a full ring): bounded spins
    if lds_in:
        for p in (0, 1):
            slow_wait(a, f"L_in{p}_%=", f"L_inr{p}_%=", "v93", "%[pin]", "s43", reread="ds_read_b32 v92, v95")
    if lds_out:
        slow_wait(a, "L_bp0_%=", "L_bpr0_%=", "v99", "%[qnx]", "s44")
        slow_wait(a, "L_bpx_%=", "L_bpxr_%=", "v99", "%[qnx]", "s44")
    a("L_done_%=:")
    return L


def book(a, p, lds_in, lds_out):
    """Advance k0, the ring offset and the words to the next chunk."""
    a("s_add_i32 s40, s40, 32")
    a("s_add_u32 s41, s41, 0x80")
    a(f"s_and_b32 s41, s41, {(R - 1) * 4:#x}")
    if lds_out:
        a("v_add_u32 v96, s41, %[lout]")
        a("v_add_u32 v97, 32, v97")
    if lds_in:
        a("v_add_u32 v95, s41, %[lin]")
        a("v_add_u32 v98, 32, v98")
    if p == 1:
        a("v_add_u32 v94, 64, v94")


def slow_wait(a, label, resume, vreg, addr, sreg, reread=None):
    """Re-read a progress word until it reaches s40 (k0), then resume; after the
    deadline (or once failed) give up: s45 = 1 and the kernel reports ERR_TIMEOUT."""
    a(f"{label}:")
    a("s_add_u32 s46, s46, 1")
    a("s_cmp_lg_u32 s45, 0")
    a(f"s_cbranch_scc1 {resume}")
    a(f"{label}_w:")
    a(f"ds_read_b32 {vreg}, {addr}")
    if reread:
        a(reread)
    a("s_memrealtime s[48:49]")
    a("s_waitcnt lgkmcnt(0)")
    a(f"v_readfirstlane_b32 {sreg}, {vreg}")
    a(f"s_cmp_ge_i32 {sreg}, s40")
    a(f"s_cbranch_scc1 {resume}")
    a("s_sub_u32 s48, s48, %[dlo]")
    a("s_subb_u32 s49, s49, %[dhi]")
    a("s_cmp_lt_i32 s49, 0")
    a("s_cbranch_scc0 %s_x" % label)
    a("s_sleep 1")
    a(f"s_branch {label}_w")
    a(f"{label}_x:")
    a("s_mov_b32 s45, 1")
    a(f"s_branch {resume}")


CLOBBERS = ['"v%d"' % r for r in range(64, 107) if r not in (75, 102, 103, 104)] + ['"s%d"' % r for r in range(40, 50) if r != 42 and r != 47] \
    + ['"scc"', '"vcc"', '"memory"']


def emit(spec=0, halfpub=True):
    out = ["// GENERATED by tools/gen_flow3.py -- do not edit.  The flow3 chunk loops (sw_flow3.hip):",
           "// one inline-asm block per strip role, R = %d ring rows, SPEC = %d, HALFPUB = %d." % (R, spec, halfpub),
           "// Operands: see F3Loop in sw_flow3.hip; fixed registers: tools/gen_flow3.py.",
           "#pragma once", ""]
    for IN in ROLES_IN:
        for OUT_ in ROLES_OUT:
            body = gen_role(IN, OUT_, spec, halfpub)
            out.append("template <> __device__ __forceinline__ F3Res f3_loop<F3_%s, F3_%s>(const F3Loop& x) {"
                       % (IN.upper(), OUT_.upper()))
            out.append("    F3Res r;")
            out.append("    asm volatile(")
            for line in body:
                out.append('        "%s\\n\\t"' % line)
            out.append('        : [M] "=v"(r.M), [fail] "=s"(r.fail), [slow] "=s"(r.slow)')
            out.append('        : [pA] "v"(x.pA), [pB] "v"(x.pB), [ng] "v"(x.ng), [G] "s"(x.G), [k80] "s"(x.k80),')
            out.append('          [code] "v"(x.code), [lin] "v"(x.lin), [lout] "v"(x.lout), [pin] "v"(x.pin),')
            out.append('          [pout] "v"(x.pout), [qme] "v"(x.qme), [qnx] "v"(x.qnx), [end] "s"(x.end),')
            out.append('          [dlo] "s"(x.dlo), [dhi] "s"(x.dhi), [rsrc] "s"(x.rsrc), [ek] "s"(x.ek),')
            out.append('          [lrow] "v"(x.lrow), [m48] "s"(x.m48)')
            out.append("        : " + ", ".join(CLOBBERS) + ");")
            out.append("    return r;")
            out.append("}")
            out.append("")
    return "\n".join(out)


def main():
    spec = int(os.environ.get("F3_SPEC", "4"))
    halfpub = os.environ.get("F3_HALFPUB", "1") != "0"
    text = emit(spec, halfpub)
    if "--check" in sys.argv:
        cur = open(OUT).read() if os.path.exists(OUT) else ""
        sys.exit(0 if cur == text else 1)
    path = OUT
    for i, arg in enumerate(sys.argv):
        if arg == "-o":
            path = sys.argv[i + 1]
    with open(path, "w") as f:
        f.write(text)


if __name__ == "__main__":
    main()
