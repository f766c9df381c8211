"""Bit identities behind the group traceback's per-lane constants (vd_kernel_tg.h traceback_word_tg,
tb_direct / tb_pack / tb_unpack), checked on the host for every state, phase and field length.

- position of state T at a field end of stage phase s (odd) is rotl6(T, s), read as bits
  [J-6 + (6-s), J + (6-s)) of TX = T * (2^(J-6) + 2^J), whose bits [J-6, J) are also T << (J-6);
- the offsets tb_direct computes for ph = 2((k+1) % 3) are those of s = ph+1, ph+3, ph+5 (mod 6);
- the M_B32 phase-0 masks 0x41041041 << ((12 - ph - 2d) % 6), d = 0, 1, 2, equal the d = 0 mask shifted
  right by 2d in the bits a field uses (J <= 16);
- tb_pack's 5-bit fields (the v_bfe_u32 offset operand uses bits 4:0 only) hold what tb_direct computes;
- a traceback batch starts at a multiple of 3 words whenever the batch length is (the hoisting condition).
"""
import pytest

P = 0x41041041


def rotl6(t, s):
    return ((t << s) | (t >> (6 - s))) & 63


def tb_direct(J, k):
    """Mirror of vd_kernel_tg.h tb_direct: (offsets, m50)."""
    ph = 2 * ((k + 1) % 3)
    off = [5 - ph + J - 6, (3 - ph if ph <= 2 else 9 - ph) + J - 6, (1 if ph == 0 else 7 - ph) + J - 6]
    return off, (P << ((12 - ph) % 6)) & 0xFFFFFFFF


def tb_pack(J, lane, fix5):
    off, _ = tb_direct(J, lane)
    ph = 2 * ((lane + 1) % 3)
    return off[0] | off[1] << 5 | off[2] << 10 | (((12 - ph) % 6) << 15 if fix5 else 0)


@pytest.mark.parametrize("J", [8, 16])
def test_tx_gives_position_and_xor_operand(J):
    mul = (1 << (J - 6)) | (1 << J)
    for k in range(3):
        off, _ = tb_direct(J, k)
        ph = 2 * ((k + 1) % 3)
        for c, o in enumerate(off):
            s = (ph + 2 * c + 1) % 6  # the three odd field-end phases
            for T in range(64):
                TX = T * mul
                assert (TX >> o) & 63 == rotl6(T, s)
                assert (TX & ((1 << J) - 1)) == (T << (J - 6))


def test_phase0_masks_shift_right_by_two():
    for ph in (0, 2, 4):
        m0 = (P << ((12 - ph) % 6)) & 0xFFFFFFFF
        for d in range(3):
            md = (P << ((12 - ph - 2 * d) % 6)) & 0xFFFFFFFF
            assert (m0 >> (2 * d)) & 0xFFFF == md & 0xFFFF


@pytest.mark.parametrize("J", [8, 16])
@pytest.mark.parametrize("fix5", [False, True])
def test_pack_unpack(J, fix5):
    for lane in range(64):
        w = tb_pack(J, lane, fix5)
        off, m50 = tb_direct(J, lane)
        assert [w & 31, (w >> 5) & 31, (w >> 10) & 31] == off
        if fix5:
            assert (P << ((w >> 15) & 31)) & 0xFFFFFFFF == m50


def test_traceback_batches_start_at_multiples_of_three():
    # kernel: first batch tbn = TBS - 3 (blockIdx.x & 3) words, later batches TBS words; with TBS = 12
    # every batch start kb is a multiple of 3, so word kb + lane has the lane's phase
    TBS = 12
    for blk in range(4):
        kb, tbn, starts = 0, TBS - 3 * (blk & 3), []
        for j in range(2, 400):
            if j - 1 - kb == tbn:
                starts.append(kb)
                kb, tbn = j - 1, TBS
        starts.append(kb)
        assert all(s % 3 == 0 for s in starts)
