"""CPU checks of the duo kernels' byte encoding (sw_kernels.hip SENT_RAW, DESIGN.md section 2 "Duo on
raw bytes"): the penalty table over every byte pair and sentinel / dead half, and a u16 model of a
padded duo (dead columns past n, sentinel rows past m, the saturating arithmetic of StripDuo::step)
against the oracle, which shows that sentinel and dead cells never raise the maximum."""
import numpy as np
import pytest

SENT_ROW = 0x00FF      # a row word half below row 0 or past m
DEAD_COL = 0x007F      # a column word half past n


def pen(row_half, col_half, P):
    return min(row_half ^ col_half, P)


@pytest.mark.parametrize("P", [1, 2, 5, 9, 127])
def test_penalty_table(P):
    """Equal bytes 0, different bytes P, any sentinel or dead half P (never 0)."""
    b = np.arange(256)
    rows = (b << 8)[:, None]
    cols = (b << 8)[None, :]
    x = np.minimum(rows ^ cols, P)
    assert (np.diag(x) == 0).all()
    assert (x[~np.eye(256, dtype=bool)] == P).all()
    halves = list(b << 8)
    for h in halves:
        assert pen(SENT_ROW, h, P) == P
        assert pen(h, DEAD_COL, P) == P
    assert pen(SENT_ROW, DEAD_COL, P) == P


def duo_model(a, b, n_pad, m_pad, match, mismatch, gi, ge):
    """The duo step's arithmetic for one half (u16, saturating), over a padded n_pad x m_pad
    matrix: columns >= len(a) are dead, rows >= len(b) are sentinels (the RAW encoding), H = E
    = F = 0 on the border; returns the running max of t (StripDuo's M)."""
    P = match - mismatch
    col = [(int(c) << 8) for c in a] + [DEAD_COL] * (n_pad - len(a))
    row = [(int(r) << 8) for r in b] + [SENT_ROW] * (m_pad - len(b))
    sat = lambda v: max(v, 0)
    Aprev = [match] * (n_pad + 1)          # A = H + MATCH of the previous row (border H = 0)
    hgprev = [0] * (n_pad + 1)
    fh = [0] * (n_pad + 1)
    M = 0
    for i in range(m_pad):
        Acur = [match] + [0] * n_pad
        hgcur = [0] * (n_pad + 1)
        eh = 0
        for j in range(1, n_pad + 1):
            p = min(row[i] ^ col[j - 1], P)
            t = sat(Aprev[j - 1] - p)
            E = max(eh, hgcur[j - 1])
            F = max(fh[j], hgprev[j])
            H = max(t, E, F)
            assert H + match <= 65535
            M = max(M, t)
            Acur[j] = H + match
            hgcur[j] = sat(H - gi)
            eh = sat(E - ge)
            fh[j] = sat(F - ge)
        Aprev, hgprev = Acur, hgcur
    return M


@pytest.mark.parametrize("prm", [(1, -1, 1, 1), (2, -3, 5, 2), (3, -1, 4, 1)])
def test_padded_duo_model_equals_oracle(oracle_mod, prm):
    """Ragged pairs padded with dead columns and sentinel rows (as in a duo whose other pair is
    longer): the model's maximum equals the oracle's score of the unpadded pair."""
    rng = np.random.default_rng(31 + prm[0])
    alpha = np.frombuffer(b"ACDE\x00\x7f\xff\x80", np.uint8)
    op = oracle_mod.Params(*prm)
    for _ in range(12):
        n, m = int(rng.integers(1, 40)), int(rng.integers(1, 40))
        a = alpha[rng.integers(0, len(alpha), n)]
        b = np.resize(a, m).copy() if rng.random() < 0.5 else alpha[rng.integers(0, len(alpha), m)]
        n_pad, m_pad = n + int(rng.integers(0, 25)), m + int(rng.integers(0, 25))
        assert duo_model(a, b, n_pad, m_pad, *prm) == oracle_mod.score_linear(a, b, op), (n, m, n_pad, m_pad)
