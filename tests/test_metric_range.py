"""The path-metric range argument behind vd_kernel_tg.h's renormalisation (once per 32-stage block around
1.25 * 2^23), checked on CPU.

The kernel's metric word only stays exact while V = base + (metric - metric of position 0 at the last
renormalisation) * 2^S + field lies in [2^23, 2^24) (fp32 formats) or inside int32 (SOFT16).  Its bound
rests on three properties of the K=7 (0171, 0133) trellis with correlation branch metrics
(viterbiBM.cuh: BM[L] = +-s0 +- s1, larger is better; viterbiACS.cuh: max-select):
  1. the largest path metric never decreases from one stage to the next;
  2. it grows by at most the stage's largest branch metric;
  3. every metric lies within D = (K-1) * (BMmax - BMmin) of the largest.
A plain numpy add-compare-select over the reference's state/label map checks the three on saturated
noiseless codewords (the best path gains BMmax every stage), random full-range soft values and hard
decisions; the arithmetic of the per-format bound is checked against the binade for R = 32."""
import numpy as np
import pytest

K = 7
NS = 64


def _labels():
    """label L = (parity(R & 0171) << 1) | parity(R & 0133) of the branch O -> T with input bit b, R = (T << 1) | b
    (7 bits), O = ((T & 31) << 1) | b: the reference's trellis (viterbiBM.cuh bmIndCalc)."""
    par = lambda v: bin(v).count("1") & 1
    lab = np.zeros((NS, 2), dtype=np.int64)
    pred = np.zeros((NS, 2), dtype=np.int64)
    for T in range(NS):
        for b in range(2):
            R = ((T << 1) | b) & 127
            lab[T, b] = (par(R & 0o171) << 1) | par(R & 0o133)
            pred[T, b] = ((T & 31) << 1) | b
    return lab, pred


LAB, PRED = _labels()


def _encode(bits):
    reg = 0
    out = []
    for u in bits:
        reg = ((reg >> 1) | (int(u) << 6)) & 127
        out.append((bin(reg & 0o171).count("1") & 1, bin(reg & 0o133).count("1") & 1))
    return np.array(out, dtype=np.int64)


def _forward(s0, s1):
    """path metrics stage by stage (int64), with the per-stage branch metrics"""
    pm = np.zeros(NS, dtype=np.int64)
    hist = [pm.copy()]
    bms = []
    for a, b in zip(s0, s1):
        bm = np.array([-a - b, -a + b, a - b, a + b], dtype=np.int64)  # L = 0..3: (L>>1 ? +:-)s0 + (L&1 ? +:-)s1
        cand = pm[PRED] + bm[LAB]
        pm = cand.max(axis=1)
        hist.append(pm.copy())
        bms.append(bm)
    return np.array(hist), np.array(bms)


def _check_properties(s0, s1, bm_max, bm_min):
    hist, bms = _forward(s0, s1)
    mx = hist.max(axis=1)
    step = np.diff(mx)
    assert (step >= 0).all(), "largest metric decreased"
    assert (step <= bms.max(axis=1)).all(), "largest metric grew by more than the stage's best branch metric"
    spread = hist.max(axis=1) - hist.min(axis=1)
    assert spread.max() <= (K - 1) * (bm_max - bm_min)
    return step.max(), spread.max()


@pytest.mark.parametrize("seed", [1, 2])
def test_soft8_saturated_codeword(seed):
    # the CLI default SNR 15: soft values saturate at the codeword's signs (bit 0 -> +127, bit 1 -> -128)
    rng = np.random.default_rng(seed)
    c = _encode(rng.integers(0, 2, 3000))
    s = np.where(c == 0, 127, -128)
    grow, _ = _check_properties(s[:, 0], s[:, 1], 256, -256)
    assert grow >= 254  # the best path does gain (nearly) BMmax per stage: the worst case is exercised


@pytest.mark.parametrize("seed", [3, 4])
def test_soft8_full_range_random(seed):
    rng = np.random.default_rng(seed)
    s = rng.integers(-128, 128, (4000, 2))
    _check_properties(s[:, 0], s[:, 1], 256, -256)


@pytest.mark.parametrize("flip", [0.0, 0.05, 0.5])
def test_hard_decisions(flip):
    # HARD (viterbiBM.cuh): A = r0 + r1 - 1, B = r0 - r1 is the correlation form with s0 = r0 - 1/2,
    # s1 = r1 - 1/2; doubled here to stay in integers (BM in {-2, 0, 2})
    rng = np.random.default_rng(5)
    c = _encode(rng.integers(0, 2, 3000))
    r = c ^ (rng.random(c.shape) < flip)
    s = 2 * r - 1  # +-1: the correlation form of (r0 - 1/2, r1 - 1/2), scaled by 2
    _check_properties(s[:, 0], s[:, 1], 2, -2)


def test_bounds_fit_the_binade():
    """vd_kernel_tg.h 'Range' comment: with base 1.25 * 2^23 and R = 32 stages between renormalisations,
    [-(D + BMmax + 1), D + R * BMmax + BMmax + 2] units of 2^S fit in [2^23, 2^24) around the base."""
    base = 1.25 * 2 ** 23
    below, above = base - 2 ** 23, 2 ** 24 - base
    R = 32
    for name, bm_max, S in (("HARD", 1, 17), ("SOFT4", 16, 9), ("SOFT8", 256, 9), ("FP32", 16, 9)):
        D = (K - 1) * 2 * bm_max
        lo = (D + bm_max + 1) * 2 ** S
        hi = (D + R * bm_max + bm_max + 2) * 2 ** S
        assert lo <= below and hi < above, (name, lo, below, hi, above)
    # SOFT16 on int32 patterns, base 0, S = 9
    bm_max, S = 65536, 9
    D = (K - 1) * 2 * bm_max
    assert (D + R * bm_max + bm_max + 2) * 2 ** S < 2 ** 31 and (D + bm_max + 1) * 2 ** S < 2 ** 31
    # 40 stages would not fit SOFT8
    bm_max, S = 256, 9
    assert (6 * 512 + 40 * bm_max + bm_max + 2) * 2 ** S >= above


@pytest.mark.parametrize("name,bm_max,D,S,R,base", [
    ("HARD", 1, 12, 9, 96, 7680),     # 8-stage fields, one renormalisation per 96-stage group
    ("SOFT4", 16, 192, 5, 32, 8192),  # 4-stage fields (FP32 the same: BMmax 16)
    ("SOFT8", 256, 2816, 3, 8, 25600),  # 2-stage fields, D = 11 * 256 (vd_kernel_pk.h "SOFT8 range")
])
def test_packed_halves_fit(name, bm_max, D, S, R, base):
    """vd_kernel_pk.h PkFmt: the metric part of a candidate is a previous metric (within [-D, D + (R-1) BMmax]
    of position 0's at the last renormalisation: properties 1-3) plus a branch metric, so within
    [-(D + BMmax), D + R * BMmax] units of 2^S around the half's base; the history field (tags included)
    adds [0, 2^S).  The whole range lies inside an unsigned 16-bit half, so the 32-bit adds of the two halves
    never carry or borrow across them."""
    lo = base - (D + bm_max) * 2 ** S
    hi = base + (D + R * bm_max) * 2 ** S + 2 ** S - 1
    assert 0 <= lo and hi < 2 ** 16, (name, lo, hi)
    # one more group (HARD) / period (SOFT8) between renormalisations would not fit
    if name != "SOFT4":
        R2 = R + (96 if name == "HARD" else 8)
        assert base + (D + R2 * bm_max) * 2 ** S + 2 ** S - 1 >= 2 ** 16


def test_soft8_spread_bound():
    """D = 2816 for SOFT8: the largest spread seen over saturated codewords and random full-range inputs
    stays within 11 * 256 (vd_kernel_pk.h "SOFT8 range"; the generic (K-1)(BMmax-BMmin) would be 3072)."""
    rng = np.random.default_rng(5)
    worst = 0
    for _ in range(4):
        s = rng.integers(-128, 128, (2000, 2))
        hist, _ = _forward(s[:, 0], s[:, 1])
        worst = max(worst, int((hist.max(axis=1) - hist.min(axis=1)).max()))
        c = _encode(rng.integers(0, 2, 2000))
        hist, _ = _forward(np.where(c[:, 0] == 1, -128, 127), np.where(c[:, 1] == 1, -128, 127))
        worst = max(worst, int((hist.max(axis=1) - hist.min(axis=1)).max()))
    assert worst <= 11 * 256, worst
