#!/usr/bin/env python3
"""Schedule model of the ring-mode single-pair kernels (C5: one pair N = 2^20 cut into strips of
63*W new columns, four strips per workgroup, block j of a G-block grid running groups j, j+G, ...)
-- a planning tool for DESIGN.md section 8, not part of the product.

    python tools/sim_ring.py                 # the current plan and the alternatives

Model (time-stepped, dt per tick):
  * strip s needs its producer s-1 to lead by LAG steps (the 63-step lane skew plus the 64-row
    chunk hand-off); back-pressure: it may lead its consumer by at most RING + 63 steps;
  * a group starts when its block has finished the previous group (the group loop's barrier);
  * wave w of a block sits on SIMD w of the block's CU (blocks dealt round-robin over the CUs);
  * a SIMD's runnable waves share its issue slots: one wave alone issues a slow-class VALU every
    LONE ns, several together one every SLOW ns (FAST for the fast class: v_sub clamp, v_add,
    VOP2 moves) -- profiles/r03_ubench_issue_classes.jsonl, r06_ubench_fclass.jsonl;
  * a step of a W-column strip issues slow(W) + fast(W) instructions, plus OVH per step for the
    chunk's hand-off and code-ring work (calibrated on the measured C5 launch).
The chain update is exact within a tick: p_new[s] = min(cand[s], p_new[s-1] - LAG) is a running
minimum of cand[s] + LAG*s."""
import argparse
import numpy as np

LONE, SLOW, FAST = 2.05, 1.78, 1.03


def step_mix(W, affine=False):
    """(slow, fast) VALU per step of the W-column ring step (tools/gen_flow3.py step3 / step_aff3)."""
    if not affine:
        # per column: SDWA t, max3 H (slow), clamped sub (fast); per step: 2 DPP; M: max3 per two t;
        # one v_perm per column every 4 steps
        return W + 2 + W + W / 2 + W / 4, W
    # affine (step_aff3: 25.5 VALU per 3 columns): per column t, E/F maxima, H max3 (slow), three subs
    return 4 * W + 4 + W / 2 + W / 4 - 0.25 * W, 3 * W


def simulate(widths, cus=256, blocks_per_cu=4, lag=100, ring_in=512, ring_x=4096, m=1 << 20, ovh=1.0,
             dt=2000.0, affine=False, max_ms=600.0, timeline=False):
    """widths: columns per lane of every strip (in chain order).  Returns (ms, per-round stats);
    timeline: also each strip's first-step and end times (ns)."""
    S = len(widths)
    G = cus * blocks_per_cu
    groups = (S + 3) // 4
    s_idx = np.arange(S)
    grp = s_idx // 4
    blk = grp % G
    rnd = grp // G
    simd = (blk % cus) * 4 + (s_idx % 4)
    steps_total = m + 64
    slow = np.array([step_mix(w, affine)[0] for w in widths]) + ovh
    fast = np.array([step_mix(w, affine)[1] for w in widths])
    lone_ns = (slow + fast) * LONE          # ns per step alone on its SIMD
    shared_ns = slow * SLOW + fast * FAST   # ns of SIMD issue per step with company
    p = np.zeros(S)
    done_at = np.full(S, np.nan)
    # group start: round 0 at t = 0; round r once the block's group of round r-1 is done
    start = np.where(rnd == 0, 0.0, np.inf)
    # in-workgroup LDS rings, cross-block rings of ring_x rows, and the wrap ring (block G-1 -> block 0
    # of the next round) of m rows: no back-pressure
    ring_lim = np.where((s_idx % 4) == 3, np.where(grp % G == G - 1, m + 64, ring_x), ring_in) + 63
    t = 0.0
    first = np.full(S, np.nan)
    nsimd = cus * 4
    while np.isnan(done_at).any() and t < max_ms * 1e6:
        active = (start <= t) & np.isnan(done_at)
        # dependency limits from the last tick (runnable: not blocked)
        prev = np.concatenate([[np.inf], p[:-1]])
        nxt = np.concatenate([p[1:], [np.inf]])
        # a finished producer has published every row: its consumer may run to the end
        lim = np.where(prev >= steps_total, steps_total + lag, prev) - lag
        # runnable: not waiting for a producer that has not yet led by `lag` (a consumer bound at
        # exactly its producer's pace runs this tick at that pace)
        # (a consumer whose producer is running counts as runnable: the chain minimum below caps it
        # within the tick, so the wavefront's fill is not quantised to one strip per tick)
        runnable = active & (lim >= p - 1e-9) & (p <= nxt + ring_lim + 1e-9) & (prev > 0)
        runnable[0] = active[0] and p[0] <= nxt[0] + ring_lim[0] + 1e-9
        n_run = np.bincount(simd[runnable], minlength=nsimd)
        load = np.bincount(simd[runnable], weights=shared_ns[runnable], minlength=nsimd)
        # each runnable wave: its share of the SIMD (issue time of one step of every runnable wave)
        per_step = np.where(n_run[simd] <= 1, lone_ns, np.maximum(load[simd], lone_ns))
        adv = np.where(runnable, dt / per_step, 0.0)
        cand = np.minimum(p + adv, steps_total)
        cand = np.where(active, cand, p)
        # chain: p_new[s] <= p_new[s-1] - lag, exact as a running minimum of cand + lag*s; a finished
        # producer holds its consumers back no more: the minimum restarts after every finished strip
        # (segment offsets of -BIG per finished strip before s)
        fin_c = cand >= steps_total
        F = np.concatenate([[0], np.cumsum(fin_c)[:-1]]).astype(np.float64)
        BIG = 1e8
        y = np.minimum.accumulate(cand + lag * s_idx - BIG * F)
        p_new = np.minimum(cand, y - lag * s_idx + BIG * F)
        p_new = np.minimum(p_new, nxt + ring_lim)
        p_new = np.maximum(p_new, p)
        fin = (p_new >= steps_total) & np.isnan(done_at)
        done_at[fin] = t + dt
        first[(p_new > 0) & np.isnan(first)] = t
        p = p_new
        t += dt
        # groups whose block finished its previous group start now
        if fin.any():
            gdone = np.zeros(groups, bool)
            gd = np.isnan(done_at).reshape(-1) == False  # noqa: E712
            full = np.zeros(groups * 4, bool)
            full[:S] = gd
            full[S:] = True
            gdone = full.reshape(groups, 4).all(axis=1)
            nxt_g = np.arange(groups) + G
            ok = nxt_g < groups
            ready = np.zeros(groups, bool)
            ready[nxt_g[ok & gdone]] = True
            newly = ready[grp] & np.isinf(start)
            start[newly] = t
    st = {"strips": S, "groups": groups, "rounds": int(rnd.max()) + 1}
    if timeline:
        return t / 1e6, st, first, done_at
    return t / 1e6, st


def widths_mix(n4, n5):
    return [4] * n4 + [5] * n5


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lag", type=float, default=100)
    ap.add_argument("--ovh", type=float, default=1.0)
    ap.add_argument("--dt", type=float, default=5000.0)
    ap.add_argument("--affine", action="store_true")
    args = ap.parse_args()
    N = 1 << 20
    cases = [
        ("W3 (current), 4 blocks/CU", [3] * ((N - 3 + 188) // 189), 4),
        ("W2, 4 blocks/CU", [2] * ((N - 2 + 125) // 126), 4),
        ("W4, 4 blocks/CU", [4] * ((N - 4 + 251) // 252), 4),
        ("W5, 4 blocks/CU", [5] * ((N - 5 + 314) // 315), 4),
        ("W6, 4 blocks/CU", [6] * ((N - 6 + 377) // 378), 4),
        ("W4 x 3835 + W5 x 261 (4096 strips)", widths_mix(3835, 261), 4),
        ("W3, 6 blocks/CU (<= 80 VGPRs)", [3] * ((N - 3 + 188) // 189), 6),
    ]
    for name, w, bpc in cases:
        ms, st = simulate(w, blocks_per_cu=bpc, lag=args.lag, ovh=args.ovh, dt=args.dt, affine=args.affine)
        print("%-40s %7.1f ms  %s" % (name, ms, st), flush=True)


if __name__ == "__main__":
    main()
