"""Host model of vd_decode_pk's split single-batch launches (tools only, not a test of the product).

A chunk of W words (blocks of 32 stages) is cut into P parts at pk_cut(p, P, W) (vd_kernel_pk.h "Split"):
part 0 decodes from the chunk start, part p >= 1 from kPkWarm blocks before its cut, both from equal
metrics.  After each pass every part whose start vector (its renormalised metric vector at block
cut(p) - 1) differs from its left neighbour's end vector at that block is decoded again from block cut(p)
with that end vector.  The kernel caps the passes at 2 P and counts a wave that reaches the cap with a part
still differing (vd_split_cap_exits); this model checks that the cap can never bind:

  * the passes end within P (P - 1 re-decode passes): after re-decode pass k parts 0 .. k are exact;
  * every part's start and end vectors equal those of one decode of the whole chunk (so its words are);
  * an early-stopped re-decode (its vector equal, at a group end after the cut, to the run whose words
    stand there) leaves the end vector the full re-decode would have produced.

The trellis is the reference's (K = 7, polynomials 0171, 0133; viterbiACS.cuh); branch metrics are those of
SOFT8 input, A = s0 + s1, B = s0 - s1 (viterbiBM.cuh); vectors are renormalised to state 0's metric, so equal
vectors mean equal decisions from there on whatever the tie rule.  Inputs: uniformly random bytes (noise
only, the case where speculative starts fail most), noisy codewords, and an abstract chunk whose decode never
forgets its start vector (the worst case: exactly P passes).
Run: python tools/split_model.py
"""
import numpy as np

K_WARM = 6   # kPkWarm: warm-up blocks of a part p >= 1
GROUP = 3    # blocks per group (checkpoints and early stops are group ends)


def pk_cut(p, P, W, warm=K_WARM):
    """vd_kernel_pk.h pk_cut: kPkWarm + 3 round(p (W - kPkWarm) / (3 P)) for 0 < p < P"""
    if p == 0:
        return 0
    if p >= P:
        return W
    return warm + 3 * ((2 * p * (W - warm) + 3 * P) // (6 * P))


def _trellis():
    """predecessors of each state and the label index (0..3 = -A, -B, B, A) of each branch"""
    def par(v):
        return bin(v).count("1") & 1
    prev = np.zeros((64, 2), np.int64)
    lab = np.zeros((64, 2), np.int64)
    for T in range(64):
        for b in (0, 1):
            O = ((T & 31) << 1) | b          # the state before the input bit T >> 5 entered
            R = (T << 1) | b                  # 7-bit register: new bit at bit 6
            o0, o1 = par(R & 0o171), par(R & 0o133)
            prev[T, b] = O
            lab[T, b] = (o0 << 1) | o1
    return prev, lab


PREV, LAB = _trellis()


class Chunk:
    """stage branch metrics of one chunk of W words (32 W + 64 stages: the traceback reads two blocks past
    the last word); run() decodes blocks [b0, b1) from a start vector and returns the vector after each"""

    def __init__(self, W, rng, kind):
        n = 32 * (W + 2)
        if kind == "random":
            s = rng.integers(-128, 128, (n, 2))
        else:  # noisy codeword of random bits, quantised as SOFT8 at scale 40 (a few dB)
            bits = rng.integers(0, 2, n + 6)
            reg = np.zeros(n, np.int64)
            for t in range(n):
                reg[t] = sum(int(bits[t + 6 - i]) << (6 - i) for i in range(7))
            o0 = np.array([bin(int(r) & 0o171).count("1") & 1 for r in reg])
            o1 = np.array([bin(int(r) & 0o133).count("1") & 1 for r in reg])
            x = np.stack([1 - 2 * o0, 1 - 2 * o1], 1) + rng.normal(0, 0.9, (n, 2))
            s = np.clip(np.rint(x * 40), -128, 127).astype(np.int64)
        A, B = s[:, 0] + s[:, 1], s[:, 0] - s[:, 1]
        self.bm = np.stack([-A, -B, B, A], 1)  # per stage, per label
        self.W = W

    def run(self, v, b0, b1):
        """vectors (renormalised to state 0) at the end of blocks b0 .. b1 - 1, starting from vector v"""
        out = []
        pm = np.array(v, np.int64)
        for b in range(b0, b1):
            for t in range(32 * b, 32 * b + 32):
                c = pm[PREV] + self.bm[t][LAB]
                pm = c.max(axis=1)
            out.append(tuple(pm - pm[0]))
        return out


class NoConvergence:
    """the worst case for the pass loop: a chunk whose decode never forgets its start vector (each block's
    vector a hash of the previous one), so a part is exact only when started from its left neighbour's exact
    end vector -- the bound P must hold with equality"""

    def __init__(self, W):
        self.W = W

    def run(self, v, b0, b1):
        out = []
        h = v[0]  # the vector is its first entry (a restart from a kept vector continues the same decode)
        for b in range(b0, b1):
            h = hash((h, b))
            out.append((h,) + (0,) * 63)
        return out


def split_passes(ch, P, early_stop=True, warm=K_WARM):
    """The kernel's pass loop over P parts of one chunk; returns (passes, start vectors, end vectors).
    warm: warm-up blocks (the kernel's kPkWarm = 6; shorter warm-ups stress the bound: more parts fail)"""
    W = ch.W
    cut = [pk_cut(p, P, W, warm) for p in range(P + 1)]
    zero = (0,) * 64
    sv, ev = [None] * P, [None] * P
    runs = [None] * P  # the vectors of the run whose words currently stand, by chunk block
    for p in range(P):  # pass 0: part 0 from the chunk start, the others kPkWarm blocks early
        o = 0 if p == 0 else cut[p] - warm
        vec = ch.run(zero, o, cut[p + 1])
        runs[p] = {o + i: x for i, x in enumerate(vec)}
        runs[p][o - 1] = zero  # (warm-up 0: the start vector is the equal-metric one)
        if p:
            sv[p] = runs[p][cut[p] - 1]
        if p + 1 < P:
            ev[p] = runs[p][cut[p + 1] - 1]
    passes = 1
    while True:
        bad = [p for p in range(1, P) if sv[p] != ev[p - 1]]
        if not bad:
            return passes, sv, ev
        assert passes < 2 * P, "the kernel's pass cap would bind"
        passes += 1
        nev = list(ev)
        for p in bad:  # every differing part, from its cut, with its left neighbour's current end vector
            full = ch.run(ev[p - 1], cut[p], cut[p + 1])
            new = {cut[p] + i: x for i, x in enumerate(full)}
            if early_stop:
                # the first group end after the cut where the re-decode meets the standing run: from there on
                # the two are the same decode, so the standing run's end vector is the re-decode's
                meet = [b for b in range(cut[p] - 1 + GROUP, cut[p + 1], GROUP) if new[b] == runs[p].get(b)]
                if meet and p + 1 < P:
                    assert runs[p][cut[p + 1] - 1] == new[cut[p + 1] - 1]
            runs[p] = new
            sv[p] = ev[p - 1]
            if p + 1 < P:
                nev[p] = new[cut[p + 1] - 1]
        ev = nev


def check(W, P, kind, seed, warm=K_WARM):
    rng = np.random.default_rng(seed)
    ch = NoConvergence(W) if kind == "no-convergence" else Chunk(W, rng, kind)
    passes, sv, ev = split_passes(ch, P, warm=warm)
    whole = {i: x for i, x in enumerate(ch.run((0,) * 64, 0, W))}
    cut = [pk_cut(p, P, W, warm) for p in range(P + 1)]
    for p in range(1, P):
        assert sv[p] == whole[cut[p] - 1], (W, P, kind, seed, p)
    for p in range(P - 1):
        assert ev[p] == whole[cut[p + 1] - 1], (W, P, kind, seed, p)
    assert passes <= P, (W, P, kind, seed, passes)
    return passes


if __name__ == "__main__":
    for P, W in ((2, 64), (2, 157), (8, 157)):
        for kind in ("random", "codeword", "no-convergence"):
            for warm in (K_WARM, 0):
                ps = [check(W, P, kind, s, warm) for s in range(6)]
                print(f"P={P} W={W} {kind:8s} warm-up {warm}: passes {ps} (cap {2 * P}, bound {P})")
