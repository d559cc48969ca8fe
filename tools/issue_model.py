#!/usr/bin/env python3
"""VALU issue model of gfx950 from the committed microbenchmarks (tools only).

The guide's VALU peak (one wave64 instruction per SIMD every 2 cycles) holds only for
the simple VOP1/VOP2-class instructions.  tools/ubench_bank.hip measured, per SIMD and
wave64 instruction at 2-8 waves per SIMD (profiles/r03_ubench_issue_classes.jsonl):

  fast  ~0.95-1.1 ns  v_add_u32, v_sub_u32 (also VOP3 with clamp), v_mov_b32, v_add_f32,
                      v_fma_f32, v_max_u16, ...
  slow  ~1.75-1.9 ns  every 3-source VOP3 (v_max3_i32, v_perm_b32, v_add3_u32), every
                      VOP3P (v_pk_*), every DPP and SDWA form, v_max_i32
  v_max3_u16 ~3.4 ns

and one wave alone on its SIMD issues any of them every ~2.0-2.2 ns, plus ~1.7 ns per
s_nop or SALU instruction between them (profiles/r03_ubench_lone_wave.jsonl).

    python tools/issue_model.py <file.s> <kernel filter>    # census + model of a kernel

kernel_mix() classifies the instructions of a kernel's dominant loop (the smallest
backward-branch range holding >= 200 VALU: a chunk loop of the step) and issue_ns() prices one VALU
instruction of that mix at w waves per SIMD.  bench.py multiplies it by the
profiled SQ_INSTS_VALU to get the kernel's issue-time bound (roofline.issue)."""
import collections
import json
import os
import re
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TABLE = os.path.join(ROOT, "profiles", "r03_ubench_issue_classes.jsonl")

FAST_PROBES = ("v_add_u32 spread", "v_sub_u32_e64 spread", "v_sub_u32_e64 clamp", "v_mov_b32", "v_add_f32",
               "v_fma_f32", "v_max_u16")
SLOW_PROBES = ("v_max3_i32 spread", "v_perm_b32 spread", "v_pk_sub_u16 spread", "v_pk_add_u16 spread",
               "v_pk_maximum3_f16 spread", "v_add_u32_sdwa", "v_add_u32_dpp", "v_mov_b32_dpp", "v_add3_u32 spread",
               "v_max_i32")

_FAST_OPS = re.compile(r"^v_(add|sub|subrev)_(u32|i32|f32|co_u32)(_e32|_e64)?$|^v_mov_b(32|64)(_e32|_e64)?$|"
                       r"^v_(and|or|xor|not)_b32(_e32|_e64)?$|^v_(lshlrev|lshrrev|ashrrev)_b32(_e32|_e64)?$|"
                       r"^v_(max|min)_u16(_e32|_e64)?$|^v_fma_f32$|^v_mul_f32(_e32)?$|^v_cmp_\w+$|"
                       r"^v_readfirstlane_b32$|^v_readlane_b32$|^v_writelane_b32$")


def op_class(op):
    """'fast', 'slow' or 'slow3' (v_max3_u16) for a VALU mnemonic (unmeasured forms: 3-source
    VOP3, VOP3P, DPP and SDWA are slow, the rest fast)."""
    if op.startswith("v_max3_u16") or op.startswith("v_min3_u16"):
        return "slow3"
    if "_dpp" in op or "_sdwa" in op or op.startswith("v_pk_"):
        return "slow"
    if op.startswith(("v_max3", "v_min3", "v_med3", "v_perm", "v_add3", "v_alignbit", "v_lshl_add", "v_and_or",
                      "v_or3", "v_mad", "v_bfe", "v_bfi", "v_cndmask", "v_max_i32", "v_min_i32", "v_max_u32",
                      "v_min_u32", "v_maximum3", "v_minimum3")):
        return "slow"
    return "fast" if _FAST_OPS.match(op) else "slow"


def cost_table(path=TABLE):
    """{waves_per_simd: {'fast': ns, 'slow': ns, 'slow3': ns}} per SIMD per wave64 instruction."""
    rows = [json.loads(l) for l in open(path) if l.startswith("{")]
    out = {}
    for w in sorted({r["waves_per_simd"] for r in rows}):
        sel = [r for r in rows if r["waves_per_simd"] == w]
        fast = [r["ns_per_instr_per_simd"] for r in sel if r["probe"] in FAST_PROBES]
        slow = [r["ns_per_instr_per_simd"] for r in sel if r["probe"] in SLOW_PROBES]
        s3 = [r["ns_per_instr_per_simd"] for r in sel if r["probe"] == "v_max3_u16"]
        if fast and slow:
            out[w] = {"fast": statistics.median(fast), "slow": statistics.median(slow),
                      "slow3": statistics.median(s3) if s3 else 2 * statistics.median(slow)}
    return out


def issue_ns(mix, waves_per_simd, table=None):
    """Average ns per SIMD of one VALU instruction of `mix` ({class: fraction})."""
    table = table or cost_table()
    w = min(table, key=lambda k: (abs(k - waves_per_simd), k))
    return sum(frac * table[w][cls] for cls, frac in mix.items())


def _kernels(path):
    cur, body = None, []
    for line in open(path):
        m = re.match(r"^(_Z\S+):\s*(;.*)?$", line)
        if m:
            cur, body = m.group(1), []
            continue
        if cur is not None:
            if line.startswith(".Lfunc_end"):
                yield cur, body
                cur = None
            else:
                body.append(line.rstrip("\n"))


def kernel_mix(path, filt):
    """VALU class fractions of the chunk loop of the first kernel matching `filt`
    (a mangled-name fragment, see mangled_filter), plus the loop's instruction counts."""
    for name, body in _kernels(path):
        if filt not in name:
            continue
        # compiler blocks (.LBB...) and the labels of hand-written asm loops (flow3: L_loop_<n>)
        labels = {m.group(1): i for i, l in enumerate(body) for m in [re.match(r"^\s*(\.LBB\S+|L_\w+):", l)] if m}
        loops = []
        for i, l in enumerate(body):
            m = re.match(r"^\s+s_c?branch\w*\s+(\.LBB\S+|L_\w+)", l)
            if not m or m.group(1) not in labels or labels[m.group(1)] >= i:
                continue
            ops = [x.split()[0] for x in body[labels[m.group(1)]:i + 1] if re.match(r"^\s+[vsdgb][a-z_0-9]+", x)]
            loops.append((sum(1 for o in ops if o.startswith("v_")), ops))
        if not loops:
            return None
        # the smallest loop holding >= 200 VALU: a chunk loop of the step (the poll loops
        # inside it are small, the item loop around it holds every role's chunk loop)
        big = [x for x in loops if x[0] >= 200]
        ops = min(big, key=lambda x: x[0])[1] if big else max(loops, key=lambda x: x[0])[1]
        cls = collections.Counter(op_class(o) for o in ops if o.startswith("v_"))
        nv = sum(cls.values())
        return {"kernel": name, "valu": nv, "salu": sum(1 for o in ops if o.startswith("s_") and o != "s_nop"),
                "s_nop": ops.count("s_nop"), "mix": {k: v / nv for k, v in sorted(cls.items())}}
    return None


def mangled_filter(demangled):
    """'void swmi::(anonymous namespace)::sw_duo_kernel<8, 64, true, true>(swmi::KParams)'
    -> 'sw_duo_kernelILi8ELi64ELb1ELb1EE' (Itanium mangling of int / bool template args)."""
    m = re.search(r"::(\w+)<([^>]*)>", demangled)
    if not m:
        return re.search(r"::(\w+)\(", demangled).group(1)
    args = []
    for a in m.group(2).split(","):
        a = a.strip()
        args.append("Lb%dE" % (a == "true") if a in ("true", "false") else "Li%sE" % a)
    return m.group(1) + "I" + "".join(args) + "E"


def main():
    path, filt = sys.argv[1], sys.argv[2]
    km = kernel_mix(path, filt)
    print(json.dumps(km))
    t = cost_table()
    for w in sorted(t):
        print("waves/SIMD %d: %.3f ns per VALU instruction per SIMD (table %s)" % (w, issue_ns(km["mix"], w, t), t[w]))


if __name__ == "__main__":
    main()
