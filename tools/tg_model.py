"""Host model of vd_decode_tg's add-compare-select (tools only, not a test of the product).

Replays the kernel's lane encoding, branch-metric table, tagged fp32 ACS (DPP and permlane-swap
stages), history read-out and word assembly on numpy float32 lanes, and compares the resulting
per-state decisions with a direct restatement of the reference ACS.  Use it to check
a change to the tagged scheme before spending GPU time on it.
"""
import sys
import numpy as np

f32 = np.float32


def rotr6(v, r):
    return ((v >> r) | (v << (6 - r))) & 63


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
    """reference decisions dec[t][T] (pick = LSB of chosen predecessor)"""
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
            elif core == "b16":
                pick = 1 - u
            else:
                pick = u
            nPM[T] = c[pick]
            d[T] = pick
        PM = nPM
        dec.append(d)
    return dec


def tg_pos(l):
    p2 = (l >> 2) & 1
    return (l & ~7) | (p2 << 2) | ((((l >> 1) & 1) ^ p2) << 1) | ((l & 1) ^ p2)


COL = [1, 2, 7, 8, 16, 32]


def cls(core, p, K):
    if core == "f16":
        return 1
    if core == "b16":
        return 0
    return 1 if (K == 0 and (p & 32)) else 0


def tg_model(AB, core, J):
    """kernel model; returns take[t][position]"""
    S = J + 1
    lanes = np.arange(64)
    pos = np.array([tg_pos(l) for l in lanes])
    VBASE = np.uint32(0x4B400000 + (1 << (S - 1)))
    V = np.full(64, VBASE, dtype=np.uint32).view(f32)
    takes = []
    nst = len(AB)
    acc = f32(0)
    hs = []
    for t in range(nst):
        A, B = AB[t]
        K = t % 6
        Q = (K + 5) % 6
        j = t % J
        tag = f32(2.0 ** j)

        def E(c, L):
            return f32(f32(bm_row(A, B)[L] * 2.0 ** S) + (tag if c else -tag))

        def idx_entry(p):  # own entry M(p) for position p
            return E(cls(core, p, K), own_label(p, K))

        if Q <= 3:
            m = np.array([idx_entry(pos[l]) for l in lanes], dtype=f32)
            t1 = (V + m).astype(f32)
            partner = np.array([l ^ COL[Q] for l in lanes])
            t2 = (V[partner] - m).astype(f32)
            V = np.maximum(t1, t2).astype(f32)
        else:
            bitn = Q
            X = np.zeros(64, dtype=f32)
            Y = np.zeros(64, dtype=f32)
            for l in lanes:
                p = pos[l]
                pp = p ^ (1 << Q)
                bit = (p >> Q) & 1
                eo, ex = idx_entry(p), idx_entry(pp)
                e1, e2 = (ex, eo) if bit else (eo, ex)
                sx = f32(-1) if bit else f32(1)
                X[l] = f32(e1 * sx + V[l])
                Y[l] = f32(e2 * (-sx) + V[l])
            d = 1 << bitn  # lane distance 16 or 32
            a2, b2 = X.copy(), Y.copy()
            for l in lanes:
                if (l & d) == 0:
                    a2[l] = X[l]
                    b2[l] = X[l + d]
                else:
                    a2[l] = Y[l - d]
                    b2[l] = Y[l]
            V = np.maximum(a2, b2).astype(f32)
        if j == J - 1:
            pat = V.view(np.uint32)
            bits = ((pat >> 1) & ((1 << J) - 1)).astype(np.int64)
            pat = (pat & np.uint32(~((1 << S) - 1) & 0xFFFFFFFF)) | np.uint32(1 << (S - 1))
            if t % 16 == 15:
                pat = (pat - (pat[0] - VBASE)).astype(np.uint32)
            V = pat.view(f32)
            if core == "f16":
                bits = (~bits) & ((1 << J) - 1)
            hs.append(bits)
        assert np.all((V.view(np.uint32) >> 23) == 0x96), "left [2^23, 2^24)"
    # per group: the J path bits of the survivor ending at each position (lane -> position index)
    words = []
    for bits in hs:
        w = np.zeros(64, dtype=np.int64)
        w[pos] = bits
        words.append(w)
    return words


def rotl6(v, r):
    return rotr6(v, (6 - r) % 6)


def group_traceback(words, J, core, t_end, n_groups):
    """kernel traceback: from state 0 at the end of stage t_end (a group end), back n_groups groups;
    returns picks (decoded bits) in stage order for the stages covered"""
    T = 0
    out_bits = {}
    g_end = (t_end + 1) // J - 1
    for g in range(g_end, g_end - n_groups, -1):
        t0 = g * J
        te = t0 + J - 1
        p = rotl6(T, te % 6)
        W = int(words[g][p])
        # J < 6 (vd_decode_pk's 4-stage fields): every stage of the field touches a different position bit,
        # so no suffix XOR; the state at the field start keeps 6 - J bits of T
        Y = W ^ (T << (J - 6)) if J >= 6 else W ^ (T >> (6 - J))
        o = Y
        sh = 6
        while sh < J:
            o ^= o >> sh
            sh *= 2
        if core == "b32":
            for jj in range(J):
                if (t0 + jj) % 6 == 0:
                    o = (o & ~(1 << jj)) | (W & (1 << jj))
        for jj in range(J):
            out_bits[t0 + jj] = (o >> jj) & 1
        T = o & 63 if J >= 6 else ((T << J) | o) & 63
    return out_bits


def ref_traceback(dec, t_end, n):
    s = 0
    out = {}
    for t in range(t_end, t_end - n, -1):
        out[t] = dec[t][s]
        s = ((s & 31) << 1) | dec[t][s]
    return out


def compare(AB, core, J):
    dec = ref_acs(AB, core)
    words = tg_model(AB, core, J)
    bad = 0
    n = len(AB)
    for t_end in range(J * 8 - 1, n, J):
        for ng in range(1, 8):
            a = group_traceback(words, J, core, t_end, ng)
            b = ref_traceback(dec, t_end, ng * J)
            for t in b:
                if a[t] != b[t]:
                    bad += 1
    return bad


if __name__ == "__main__":
    rng = np.random.default_rng(1)
    n = 192
    for ch, core, J, rngf in [("hard", "b32", 16, lambda: rng.integers(0, 2, 2)),
                              ("hard", "b16", 16, lambda: rng.integers(0, 2, 2)),
                              ("hard", "f16", 16, lambda: rng.integers(0, 2, 2)),
                              ("soft8", "b16", 8, lambda: rng.integers(-128, 128, 2)),
                              ("soft8", "b32", 8, lambda: rng.integers(-128, 128, 2)),
                              ("soft4", "b32", 4, lambda: rng.integers(-8, 8, 2)),
                              ("soft4", "b16", 4, lambda: rng.integers(-8, 8, 2)),
                              ("soft4", "f16", 4, lambda: rng.integers(-8, 8, 2))]:
        AB = []
        for _ in range(n):
            s = rngf()
            if ch == "hard":
                A, B = int(s[0] + s[1] - 1), int(s[0] - s[1])
            else:
                A, B = int(s[0] + s[1]), int(s[0] - s[1])
            AB.append((A, B))
        bad = compare(AB, core, J)
        print(ch, core, "mismatching traceback bits:", bad)
    sys.exit(0)
