#!/usr/bin/env python3
"""Model of sw_duo_lds_kernel's hand-off protocol (concurrentproject_amd/csrc/sw_kernels.hip):
the 4 waves of one workgroup walk the same rounds of a sequence of duos, each wave one strip
per round, at chunk granularity in a random interleaving.  Wave w -> w + 1 through a
DUO_R-slot ring with back-pressure, wave 3 -> wave 0 (next round) through the wrap buffer.
Progress words, floors and positions use the kernel's arithmetic.  Reports a deadlock (no
wave can move) or a slot read that does not hold the position the consumer expects.

    python tools/duo_lds_sim.py [trials]      (tests/test_duo_lds_protocol.py runs it on CPU)
"""
import random
import sys

W, C, R = 8, 64, 256
SW = 64 * W


def run(duos, seed=0, round_end_report=True):
    """duos: [(strips, m_pad)]; returns (ok, detail)."""
    rng = random.Random(seed)
    prod, cons = [0] * 4, [0] * 4
    ring = [[None] * R for _ in range(3)]
    wm = 64
    while wm < max(m for _, m in duos):
        wm *= 2
    wrap = [None] * wm
    bad = []

    def wave(w):
        base = prev = 0
        for strips, m in duos:
            nch = (m + SW - 1 + C - 1) // C
            span = nch * C + 128
            r = 0
            while 4 * r < strips:
                strip = 4 * r + w
                if strip < strips:
                    has_in, has_out = strip > 0, strip + 1 < strips
                    in_pb = base if w > 0 else prev
                    for c in range(nch):
                        k0 = c * C
                        if has_in:
                            need = in_pb + min(k0 + C, m)
                            while prod[(w + 3) & 3] < need:
                                yield ("wait_in", w, strip, k0)
                            for row in range(k0, min(k0 + C, m)):
                                got = ring[w - 1][(base + row) % R] if w > 0 else wrap[row % wm]
                                if got != in_pb + row:
                                    bad.append((w, strip, row, got, in_pb + row))
                            cons[w] = in_pb + k0 + C
                        if has_out:
                            if w < 3:
                                floor = base + k0 + C - SW + 1 - R
                                while cons[w + 1] < floor:
                                    yield ("wait_bp", w, strip, k0)
                            for lane in range(64):
                                row = k0 + lane - (SW - 1)
                                if 0 <= row < m:
                                    if w < 3:
                                        ring[w][(base + row) % R] = base + row
                                    else:
                                        wrap[row % wm] = base + row
                            prod[w] = base + min(max(0, k0 + C - SW + 1), m)
                        yield ("step", w, strip, k0)
                if round_end_report:
                    cons[w] = base + span
                prev, base, r = base, base + span, r + 1

    gens = [wave(w) for w in range(4)]
    done, state, stall = [False] * 4, [None] * 4, 0
    while not all(done):
        moved = False
        for w in rng.sample(range(4), 4):
            if done[w]:
                continue
            try:
                state[w] = next(gens[w])
                moved |= state[w][0] == "step"
            except StopIteration:
                done[w] = moved = True
        stall = 0 if moved else stall + 1
        if stall > 50:
            return False, ("deadlock", state)
    return (not bad), (("data", bad[:3]) if bad else None)


def random_duos(rng):
    return [(rng.randint(1, 9), rng.randint(1, 4200)) for _ in range(rng.randint(1, 6))]


def main():
    trials = int(sys.argv[1]) if len(sys.argv) > 1 else 500
    rng = random.Random(1)
    for t in range(trials):
        duos = random_duos(rng)
        ok, detail = run(duos, t)
        if not ok:
            print("FAIL", duos, detail)
            return 1
    print("ok: %d random duo sequences" % trials)
    return 0


if __name__ == "__main__":
    sys.exit(main())
