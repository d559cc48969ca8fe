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
MID_AHEAD = int(os.environ.get("F3_MIDAHEAD", "1"))   # 4-step groups the mid-chunk inflow read runs ahead
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
            a(f"v_perm_b32 v72, %[pA], %[k80], v{cur + u}")
            a(f"v_perm_b32 v73, %[pB], %[k80], v{cur + u}")
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
    a("s_memrealtime s[48:49]")
    a("s_waitcnt lgkmcnt(0)")
    a(f"v_readfirstlane_b32 {sreg}, {vreg}")
    a(f"s_cmp_ge_i32 {sreg}, {target}")
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
                body = gen_role(IN, OUT_, spec, halfpub, C, bool(hl))
                out.append("template <> __device__ __forceinline__ F3Res f3_loop<%d, %d, F3_%s, F3_%s>(const F3Loop& x) {"
                           % (C, hl, IN.upper(), OUT_.upper()))
                out.append("    F3Res r;")
                out.append("    asm volatile(")
                for line in body:
                    out.append('        "%s\\n\\t"' % line)
                out.append('        : [M] "=v"(r.M), [fail] "=s"(r.fail), [slow] "=s"(r.slow)')
                out.append('        : [pA] "v"(x.pA), [pB] "v"(x.pB), [ng] "v"(x.ng), [G] "s"(x.G), [k80] "s"(x.k80),')
                out.append('          [code] "v"(x.code), [lin] "v"(x.lin), [lout] "v"(x.lout), [pin] "v"(x.pin),')
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
RR = 512                 # LDS ring rows per in-workgroup link (sw_flow3.hip F3R_R)
RING = dict(H="v42", HGO="v43", HB="v44", HGOB="v45", TA="v46", TB="v47", PA="v48", PB="v49", M="v50")


def ring_granule(a):
    """Publish lanes 32..63 of IO (the 32 newest outflow rows, row v107) as 8-B granules
    at their ring slots, rows outside [0, m) dropped."""
    a("v_mov_b32 v96, v40")
    a("v_xor_b32 v97, %[ek], v40")
    a("v_xor_b32 v97, v97, v100")
    a("v_cmp_gt_u32_e64 s[50:51], %[m], v107")          # 0 <= row < m (unsigned)
    a("s_and_b64 s[50:51], s[50:51], %[lhi]")
    a("v_cndmask_b32_e64 v99, -16, v98, s[50:51]")
    a("v_add_u32 v98, 0x100, v98")                      # 32 rows on
    a("v_and_b32 v98, %[gomask8], v98")
    a("v_add_u32 v100, 0x400, v100")
    a("v_add_u32 v107, 32, v107")
    a("buffer_store_dwordx2 v[96:97], v99, %[gors], 0 offen sc1")


def ring_gin_check(a, C=64):
    """s[58:59] = live lanes (lane < C, row k0 + lane < m); s[50:51] = live lanes whose granule fails."""
    a("s_sub_i32 s54, %[m], s40")
    if C < 64:
        a(f"s_min_i32 s54, s54, {C}")
    a("v_cmp_gt_i32_e64 s[58:59], s54, %[lane]")
    a("v_xor_b32 v103, v84, v85")
    a("v_xor_b32 v103, v103, v102")
    a("v_cmp_ne_u32_e64 s[56:57], %[ek], v103")
    a("s_and_b64 s[50:51], s[58:59], s[56:57]")
    a("s_cmp_lg_u64 s[50:51], 0")


def gen_role_ring(IN, OUT_, C=64, hl=False):
    """The ring-mode loop of one strip role at C-row chunks (64, or 32: half the hand-off
    lag).  The loop body is two chunks; the code ring is refilled 64 rows per body.
    hl (C = 64): half-chunk LDS links as in gen_role: the producer also publishes its newest
    32 rows (lanes 32..63) at mid-chunk, lanes 0..31 (the chunk top's inflow) onto the
    write-ahead slots 64 rows on (%[lmid] from the ring offset of chunk k0 + 64); the consumer
    starts a chunk on its first 32 rows and merges the other 32 into lanes 0..31 at mid-chunk.
    Words count rows available - 32; the back-pressure floor is k0 + 64 (the next mid-chunk's
    write-ahead)."""
    L = []
    a = L.append
    lds_in, lds_out = IN == "lds", OUT_ == "lds"
    gin, gout = IN == "gran", OUT_ == "gran"
    assert not hl or C == 64
    H = C // 2 if hl else C
    ncr = C // 16                                      # 16-B code reads per chunk
    # ---- entry (s_nop 4: descriptor operands may be fresh from v_readfirstlane)
    a("s_nop 4")
    a("s_waitcnt vmcnt(0) lgkmcnt(0)")
    for r in ("v42", "v43", "v44", "v45", "v50"):
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
        a("buffer_load_dwordx2 v[84:85], v101, %[girs], 0 offen sc1")
    for q in range(ncr):
        a(f"ds_read_b128 v[{52 + 4 * q}:{55 + 4 * q}], %[c0]" + (f" offset:{16 * q}" if q else ""))
    a("s_waitcnt vmcnt(0) lgkmcnt(0)")
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
            ring_granule(a)
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
            ring_gin_check(a, C)
            a(f"s_cbranch_scc1 L_gin{p}_%=")
            a(f"L_ginr{p}_%=:")
            a("v_cndmask_b32_e64 v40, %[ng], v84, s[58:59]")
        elif not lds_in:
            a("v_mov_b32 v40, %[ng]")
        # 4. codes of 64 rows (128..191 ahead of the body's first row) into the wave's code
        # ring (slot base s53, mirror of slots [0, 64))
        if refill:
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
            a("buffer_load_dwordx2 v[84:85], v101, %[girs], 0 offen sc1")
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
            a(f"v_perm_b32 v48, %[pA], %[k80], v{cur + u}")
            a(f"v_perm_b32 v49, %[pB], %[k80], v{cur + u}")
            for b in range(4):
                io, l0 = ("v40", "v41") if b % 2 == 0 else ("v41", "v40")
                step(a, io, l0, b, RING)
            if gout and C == 64 and u == 7:
                ring_granule(a)
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
        ring_granule(a)
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
            slow_gin(a, f"L_gin{p}_%=", f"L_ginr{p}_%=", C)
    a("L_done_%=:")
    return L


def slow_timeout(a, label):
    """s[48:49] = s_memrealtime (waited): on to {label}_w unless past the deadline, then fail."""
    a("s_sub_u32 s48, s48, %[dlo]")
    a("s_subb_u32 s49, s49, %[dhi]")
    a("s_cmp_lt_i32 s49, 0")
    a("s_cbranch_scc0 %s_x" % label)
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
    a("s_memrealtime s[48:49]")
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


def slow_gin(a, label, resume, C=64):
    """The chunk's inflow granules are not all published yet: re-load and re-check."""
    a(f"{label}:")
    a("s_add_u32 s46, s46, 1")
    a("s_cmp_lg_u32 s45, 0")
    a(f"s_cbranch_scc1 {resume}")
    a(f"{label}_w:")
    a("buffer_load_dwordx2 v[84:85], v101, %[girs], 0 offen sc1")
    a("s_memrealtime s[48:49]")
    a("s_waitcnt vmcnt(0) lgkmcnt(0)")
    ring_gin_check(a, C)
    a(f"s_cbranch_scc0 {resume}")
    slow_timeout(a, label)
    a(f"{label}_x:")
    a("s_mov_b32 s45, 1")
    a(f"s_branch {resume}")


ROLES_IN_RING = ("none", "lds", "gran")
CLOBBERS_RING = ['"v%d"' % r for r in range(40, 108) if r != 51] + \
    ['"s%d"' % r for r in range(40, 60) if r not in (47,)] + ['"scc"', '"vcc"', '"memory"']


def emit_ring():
    out = ["// GENERATED by tools/gen_flow3.py -- do not edit.  The flow3 ring-mode chunk loops",
           "// (sw_flow3.hip sw_flow3r_kernel): one inline-asm block per (chunk rows C, half-chunk LDS links HL, strip role), R = %d." % RR,
           "// Operands: see F3RLoop in sw_flow3.hip; fixed registers: tools/gen_flow3.py.",
           "#pragma once", ""]
    for C, hl in ((64, 0), (32, 0), (64, 1)):
        for IN, OUT_ in [(i, o) for i in ROLES_IN_RING for o in ROLES_OUT]:
            body = gen_role_ring(IN, OUT_, C, bool(hl))
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
            out.append('          [lmid] "v"(x.lmid)')
            out.append("        : " + ", ".join(CLOBBERS_RING) + ");")
            out.append("    return r;")
            out.append("}")
            out.append("")
    return "\n".join(out)


OUT_RING = os.path.join(ROOT, "concurrentproject_amd", "csrc", "sw_flow3r_loops.inc")


def main():
    spec = int(os.environ.get("F3_SPEC", "4"))
    halfpub = os.environ.get("F3_HALFPUB", "1") != "0"
    text = emit(spec, halfpub)
    text_ring = emit_ring()
    if "--check" in sys.argv:
        cur = open(OUT).read() if os.path.exists(OUT) else ""
        cur_r = open(OUT_RING).read() if os.path.exists(OUT_RING) else ""
        sys.exit(0 if cur == text and cur_r == text_ring else 1)
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
