"""CPU tests of the VALU issue model bench.py prices its roofline.issue with
(tools/issue_model.py): the committed microbenchmark table parses into the two
instruction classes, the classifier puts the measured forms in the class they
were measured in, and a kernel's chunk-loop census comes out of a .s listing."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import issue_model  # noqa: E402


def test_cost_table_from_the_committed_measurements():
    t = issue_model.cost_table()
    assert set(t) >= {1, 2, 4, 8}
    for w in (2, 4, 8):
        # fast VOP2-class ~1 ns, slow 3-source / VOP3P / DPP / SDWA ~1.75-1.9 ns per SIMD
        assert 0.8 < t[w]["fast"] < 1.2 and 1.6 < t[w]["slow"] < 2.0, t[w]
        assert t[w]["slow3"] > t[w]["slow"]
    assert 1.9 < t[1]["fast"] < 2.3 and 1.9 < t[1]["slow"] < 2.3   # a lone wave: one issue every ~2 ns


def test_op_classes():
    fast = ("v_add_u32_e32", "v_sub_u32_e64", "v_mov_b32_e32", "v_add_f32_e32", "v_fma_f32", "v_max_u16_e32")
    slow = ("v_max3_i32", "v_perm_b32", "v_pk_sub_u16", "v_pk_maximum3_f16", "v_add_u32_sdwa", "v_add_u32_dpp",
            "v_mov_b32_dpp", "v_add3_u32", "v_max_i32_e32")
    assert all(issue_model.op_class(o) == "fast" for o in fast), [o for o in fast if issue_model.op_class(o) != "fast"]
    assert all(issue_model.op_class(o) == "slow" for o in slow), [o for o in slow if issue_model.op_class(o) != "slow"]
    assert issue_model.op_class("v_max3_u16") == "slow3"


def test_kernel_mix_and_price(tmp_path):
    body = ["\tv_max3_i32 v1, v2, v3, v4", "\tv_sub_u32_e64 v5, v1, s2 clamp", "\tv_add_u32_sdwa v6, v7, sext(v8)",
            "\tv_add_u32_dpp v9, v1, v2 wave_shr:1"] * 60
    s = ["_ZN4swmi12_GLOBAL__N_113sw_duo_kernelILi8ELi64ELb1ELb1EEEvNS_7KParamsE:", ".LBB0_1:"] + body + \
        ["\ts_cbranch_scc1 .LBB0_1", "\ts_endpgm", ".Lfunc_end0:"]
    p = tmp_path / "k.s"
    p.write_text("\n".join(s) + "\n")
    name = "void swmi::(anonymous namespace)::sw_duo_kernel<8, 64, true, true>(swmi::KParams)"
    km = issue_model.kernel_mix(str(p), issue_model.mangled_filter(name))
    assert km["valu"] == 240 and abs(km["mix"]["fast"] - 0.25) < 1e-9 and abs(km["mix"]["slow"] - 0.75) < 1e-9, km
    t = issue_model.cost_table()
    ns = issue_model.issue_ns(km["mix"], 2, t)
    assert abs(ns - (0.25 * t[2]["fast"] + 0.75 * t[2]["slow"])) < 1e-12
