"""Host model of vd_decode_pk's SOFT8 format (tools only, not a test of the product).

SOFT8 in an unsigned 16-bit half: V = BASE + metric * 8 + F, 2-stage history fields (S = 3), tags -+1, -+2
(tie rule of the core), renormalisation every 8 stages.  Read-out per field: x = V & 6 (the field's two
take-bits; F = 1 + 2 d is odd), then V = (V ^ x) + 3 (F back to 4; merged with the renormalisation every
fourth field).  Ring: per block, the 16 fields' d (2 bits each) of the survivor ending at each position, the
ring indexed by p' = rotl6(p, 1).  Traceback in position space: from p' = 0 (state 0) at a block end, each
field (t0, t0 + 1) back is p' ^= d << (t0 % 6); the decoded bits of the field are then bits t0 % 6, +1 of p'.

Checks, against a direct restatement of the reference ACS + traceback:
  * every value a stage forms stays in [0, 2^16) (the range bound of vd_kernel_pk.h) on saturated,
    all-extreme, codeword-like and random inputs, and the largest metric spread seen is <= D = 2816;
  * every traced word equals the reference's, for the M_B16 and M_B32 tie rules.
Run: python tools/pk2_model.py
"""
import sys
import numpy as np

S = 3
D = 11 * 256          # metric spread bound (vd_kernel_pk.h "SOFT8 range")
RN = 8                # stages between renormalisations
BASE = 3200 * 8       # a half's base: candidates within [-D - 256, D + RN * 256] units of position 0's metric
VB1 = BASE + 4


def rotr6(v, r):
    return ((v >> r) | (v << (6 - r))) & 63


def rotl6(v, r):
    return rotr6(v, (6 - r) % 6)


def par(v):
    return bin(v & 127).count("1") & 1


def own_label(p, k):
    T = rotr6(p, k)
    O = rotr6(p, (k + 5) % 6)
    R = (T << 1) | (O & 1)
    return (par(R & 0o171) << 1) | par(R & 0o133)


def bm_row(A, B):
    return [-A, -B, B, A]


def ref_acs(AB, core):
    PM = [0] * 64
    dec = []
    for t, (A, B) in enumerate(AB):
        bm = bm_row(A, B)
        nPM = [0] * 64
        d = [0] * 64
        for T in range(64):
            u = T >> 5
            c = []
            for b in (0, 1):
                O = ((T & 31) << 1) | b
                R = (T << 1) | b
                L = (par(R & 0o171) << 1) | par(R & 0o133)
                c.append(PM[O] + bm[L])
            if c[0] != c[1]:
                pick = 0 if c[0] > c[1] else 1
            elif core == "b32":
                pick = 1 if t % 6 == 0 else 1 - u
            else:
                pick = 1 - u
            nPM[T] = c[pick]
            d[T] = pick
        PM = nPM
        dec.append(d)
    return dec


def ref_traceback(dec, t_end, n):
    s = 0
    out = {}
    for t in range(t_end, t_end - n, -1):
        out[t] = dec[t][s]
        s = ((s & 31) << 1) | dec[t][s]
    return out


def cls(core, p, K):
    # +1: the own candidate wins ties (M_B32 phase 0, upper position half); else the exchanged one
    return 1 if (core == "b32" and K == 0 and (p & 32)) else 0


def model(AB, core):
    """returns ring[field][p'] (2 take-bits) and the largest spread / range seen"""
    V = [VB1] * 64  # indexed by position
    ring = []
    lo, hi, spread = 1 << 20, -1, 0
    for t, (A, B) in enumerate(AB):
        K = t % 6
        Q = (K + 5) % 6
        j = t % 2
        bm = bm_row(A, B)
        nV = [0] * 64
        for p in range(64):
            c = cls(core, p, K)
            e = bm[own_label(p, K)] * 8 + ((1 << j) if c else -(1 << j))
            t1 = V[p] + e
            t2 = V[p ^ (1 << Q)] - e
            lo, hi = min(lo, t1, t2), max(hi, t1, t2)
            nV[p] = max(t1, t2)
        V = nV
        m = [v >> 3 for v in V]
        spread = max(spread, max(m) - min(m))
        if j == 1:
            d = [0] * 64
            for p in range(64):
                F = V[p] & 7
                assert F & 1, "field of an odd value"
                d[p] = (F >> 1) & 3
                if core == "b32" and (t - 1) % 6 == 0 and (p & 32):
                    d[p] ^= 1  # the phase-0 bit of the upper half is own-won: the take-bit is its complement
            w = [0] * 64
            for p in range(64):
                w[rotl6(p, 1)] = d[p]
            ring.append(w)
            V = [(v ^ (v & 6)) + 3 for v in V]
            if t % RN == RN - 1:
                s = V[0] - VB1
                V = [v - s for v in V]
    return ring, lo, hi, spread


def trace_word(ring, k):
    """local word k: from state 0 at the end of block k + 2, emit block k + 1 (stages 32k+32 .. 32k+63)"""
    pp = 0
    bits = {}
    for f in range(16 * (k + 3) - 1, 16 * (k + 1) - 1, -1):
        t0 = 2 * f
        Kp = t0 % 6
        pp ^= ring[f][pp] << Kp
        bits[t0] = (pp >> Kp) & 1
        bits[t0 + 1] = (pp >> (Kp + 1)) & 1
    return bits


def trace_word_kernel(ring, k):
    """the kernel's form of trace_word (vd_kernel_pk.h pk2_traceback): the lane's LDS address A = 4 p', the
    per-lane shifts z[r] of the convergence block's fields, the emit block's pairs collected as 6-bit
    snapshots after fields 13, 10, 7, 4, 1 and rotated right by rho = 2u per group; returns the output word"""
    u = (k + 2) % 3
    z = [2 * ((u + r) % 3) + 2 for r in range(3)]
    A = 0
    nat = 0
    for blk, EM in ((k + 2, False), (k + 1, True)):
        for g in range(15, -1, -1):
            d = ring[16 * blk + g][A >> 2]
            zz = z[(g + 2) % 3] if EM else z[g % 3]
            A ^= d << zz
            if EM and g % 3 == 1:
                nat |= ((A >> 2) & 63) << (2 * g)
            if EM and g == 0:
                nat |= (A >> zz) & 3
    rho = 2 * u
    mlo = {0: 0xFFFFFFFC, 2: 0x3CF3CF3C, 4: 0x0C30C30C}[rho]
    grp = nat & ~3 & 0xFFFFFFFF
    a, b = grp >> rho, (grp << (6 - rho)) & 0xFFFFFFFF
    nat = (nat & 3) | (a & mlo) | (b & ~mlo & 0xFFFFFFFF)
    return int("{:032b}".format(nat)[::-1], 2)  # bitreverse: word bit i <-> stage 63 + 32k - i


def trace_word_skewed(ring, k, tbl):
    """trace_word_kernel on a skewed ring (round 6 study, not in the product: exact, 19 % fewer SOFT8 bank
    conflicts, 1.5 % slower; profiles/r06/ab_ring_skew/): slot s keeps position p' at dword p' ^ s; lane tbl's
    emit slot is tbl, its convergence slot tbl + 1.  A starts at 4 (tbl + 1), xt re-skews it between the
    blocks, cn takes the emit skew out of the snapshots (and out of field 0's pair)."""
    u = (k + 2) % 3
    z = [2 * ((u + r) % 3) + 2 for r in range(3)]
    xt = 4 * ((tbl + 1) ^ tbl)
    cn = (4 * tbl * 0x01041041) & 0xFFFFFFFF
    A = 4 * (tbl + 1)
    nat = 0
    for blk, EM, s in ((k + 2, False, tbl + 1), (k + 1, True, tbl)):
        stored = [ring[16 * blk + g] for g in range(16)]
        for g in range(15, -1, -1):
            row = [stored[g][q ^ s] for q in range(64)]  # the writer's dword p' ^ s holds position p'
            d = row[A >> 2]
            zz = z[(g + 2) % 3] if EM else z[g % 3]
            A ^= d << zz
            if EM and g % 3 == 1:
                nat |= ((A >> 2) & 63) << (2 * g)
            if EM and g == 0:
                nat |= ((A ^ (cn & 0xFC)) >> zz) & 3
        if not EM:
            A ^= xt
    nat ^= cn
    rho = 2 * u
    mlo = {0: 0xFFFFFFFC, 2: 0x3CF3CF3C, 4: 0x0C30C30C}[rho]
    grp = nat & ~3 & 0xFFFFFFFF
    a, b = grp >> rho, (grp << (6 - rho)) & 0xFFFFFFFF
    nat = (nat & 3) | (a & mlo) | (b & ~mlo & 0xFFFFFFFF)
    return int("{:032b}".format(nat)[::-1], 2)


def run(AB, core):
    dec = ref_acs(AB, core)
    ring, lo, hi, spread = model(AB, core)
    assert 0 <= lo and hi < 65536, (lo, hi)
    assert spread <= D, spread
    bad = 0
    nwords = len(AB) // 32 - 2
    for k in range(nwords):
        a = trace_word(ring, k)
        b = ref_traceback(dec, 32 * k + 95, 64)
        w = trace_word_kernel(ring, k)
        ws = trace_word_skewed(ring, k, k % 7)
        for t in range(32 * k + 32, 32 * k + 64):
            bad += a[t] != b[t]
            bad += ((w >> (63 + 32 * k - t)) & 1) != b[t]
            bad += ((ws >> (63 + 32 * k - t)) & 1) != b[t]
    return bad, lo, hi, spread


if __name__ == "__main__":
    rng = np.random.default_rng(1)
    n = 32 * 10
    worst = [1 << 20, -1, 0]
    total = 0
    for trial in range(8):
        for kind in ("random", "saturated", "extreme", "codeword", "sparse"):
            if kind == "random":
                s = rng.integers(-128, 128, (n, 2))
            elif kind == "saturated":
                s = np.where(rng.integers(0, 2, (n, 2)) == 1, 127, -128)
            elif kind == "extreme":
                s = np.full((n, 2), -128)
            elif kind == "codeword":
                bits = rng.integers(0, 2, n + 6)
                s = np.zeros((n, 2), dtype=np.int64)
                reg = 0
                for t in range(n):
                    reg = ((reg << 1) | int(bits[t])) & 127
                    r = int("{:07b}".format(reg)[::-1], 2)
                    o0, o1 = par(r & 0o171), par(r & 0o133)
                    s[t] = (127 if o0 else -128, 127 if o1 else -128)
            else:
                s = rng.integers(-128, 128, (n, 2)) * (rng.random((n, 2)) < 0.2)
            AB = [(int(a + b), int(a - b)) for a, b in s]
            for core in ("b16", "b32"):
                bad, lo, hi, sp = run(AB, core)
                total += bad
                worst = [min(worst[0], lo), max(worst[1], hi), max(worst[2], sp)]
                if bad:
                    print(kind, core, "mismatching bits:", bad)
    print("mismatching traceback bits:", total, " values in [%d, %d], largest spread %d (bound %d)" % (worst[0], worst[1], worst[2], D))
    sys.exit(1 if total else 0)
