"""CPU tests: pin the oracle (CPU restatement of the reference decode path) before trusting it.

The reference has no tests, fixtures or golden files.  Its parity is pinned by the
known-answer values of SURVEY.md §8(c), captured from a host emulation of the reference's own
kernel source before the environment refused further runs:
  * BEN at N=1,000,000, seeds (11, 22), for every input x metric column at SNR 0 and a sweep of
    SNRs for the headline columns (tests/golden/kat_ben.json);
  * SHA-256 of the packed HARD input and of the decoded output for seeds (5, 6), -n 400000 -s 1.3;
  * the harness generators (std::mt19937 bits, std::normal_distribution<float> noise) restated in C
    and checked against this container's libstdc++.
"""
import hashlib
import json
import os

import numpy as np
import pytest

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")

I = {"h": 0x0, "s4": 0x1, "s8": 0x2, "s16": 0x3, "f": 0x4}
M = {"b32": 0x00, "b16": 0x10, "f16": 0x20}


def load_kat():
    with open(os.path.join(GOLDEN, "kat_ben.json")) as f:
        return json.load(f)


def kat_cases():
    k = load_kat()
    out = []
    for row in k["ben"]:
        i, m = row["col"].split("/")
        out.append(pytest.param(row["snr"], I[i] | M[m] | k.get("extra_opts", {}).get(row["col"], 0), row["ben"],
                                id=f'{row["snr"]}-{row["col"]}'))
    return out


def test_generators_match_libstdcxx(vo):
    a = vo.gen_bits(123, 1 << 18)
    b = vo.gen_bits(123, 1 << 18, use_std=True)
    assert np.array_equal(a, b)
    x = vo.gen_normals(7, 0.7, 1 << 18)
    y = vo.gen_normals(7, 0.7, 1 << 18, use_std=True)
    assert np.array_equal(x.view(np.uint32), y.view(np.uint32))


def test_sha256_pins(vo):
    pins = load_kat()["sha256"]
    opt = vo.HARD | vo.M_B32
    bits, packed = vo.simulate(opt, 400_000, 1.3, 5, 6)
    assert hashlib.sha256(packed.tobytes()).hexdigest() == pins["input"]
    dec, ok = vo.decode(opt, packed)
    assert ok and dec.nbytes == 49_992
    assert hashlib.sha256(dec.tobytes()).hexdigest() == pins["output"]


@pytest.mark.parametrize("snr,opt,ben", kat_cases())
def test_known_answer_ben(vo, snr, opt, ben):
    bits, packed = vo.simulate(opt, 1_000_000, snr, 11, 22)
    dec, ok = vo.decode(opt, packed)
    assert ok, "metric left the reference's exact range"
    assert vo.ben(opt, bits, dec) == ben


def test_default_snr_error_free(vo):
    opt = vo.HARD | vo.M_B32
    bits, packed = vo.simulate(opt, 204_800, 15.0, 11, 22)
    dec, _ = vo.decode(opt, packed)
    assert vo.ben(opt, bits, dec) == 0


def test_dpx_equals_reg(vo):
    bits, packed = vo.simulate(vo.HARD | vo.M_B16, 300_000, 0.0, 11, 22)
    a, _ = vo.decode(vo.HARD | vo.M_B16 | vo.DPX, packed)
    b, _ = vo.decode(vo.HARD | vo.M_B16, packed)
    assert np.array_equal(a, b)


def test_o_b16_race_bracket(vo):
    # The reference's O_B16 path writes two words past the end of chunks with decLen%32==16
    # (SURVEY 8a row 13); which write wins is a race.  The emulated KAT (374610) lies between the
    # deterministic orderings: own-words-win 374618 and in-block-overrun-wins 374604.
    opt = vo.HARD | vo.M_B32 | vo.O_B16
    bits, packed = vo.simulate(opt, 1_000_000, 0.0, 11, 22)
    own, _ = vo.decode(opt, packed, b16_policy=0)
    blk, _ = vo.decode(opt, packed, b16_policy=2)
    b_own, b_blk = vo.ben(opt, bits, own), vo.ben(opt, bits, blk)
    assert (b_own, b_blk) == (374618, 374604)
    assert b_blk <= 374610 <= b_own


def test_fp16_metrics_stay_exact(vo):
    # fp16 is exact only while every metric is an integer of magnitude <= 2048; the oracle emulates
    # the reference normalisation schedule and reports any excursion (rc 1)
    for opt in (vo.HARD | vo.M_FP16, vo.SOFT4 | vo.M_FP16, vo.FP32 | vo.M_FP16):
        bits, packed = vo.simulate(opt, 500_000, -3.0, 1, 2)
        _, ok = vo.decode(opt, packed)
        assert ok


def test_options_valid_table(vo):
    # OptionsValid<options> (viterbi.h:22-41): 42 of the 60 combinations are enabled
    n = 0
    for i in range(5):
        for m in (0x00, 0x10, 0x20):
            for o in (0x000, 0x100):
                for c in (0x0000, 0x1000):
                    n += vo.options_valid(i | m | o | c)
    assert n == 42
    assert not vo.options_valid(vo.SOFT8 | vo.M_FP16)
    assert not vo.options_valid(vo.SOFT16 | vo.M_B16)
    assert not vo.options_valid(vo.HARD | vo.M_FP16 | vo.DPX)


def test_sizes(vo):
    # viterbi.cu:63-92 at the BASELINE sizes (SURVEY 8 preamble)
    assert vo.message_len(0, 64_000_000) == 31_999_936
    assert vo.output_size(0, 64_000_000) == 3_999_992
    assert vo.input_size(0, 64_000_000) == 8_000_000
    assert vo.input_size(vo.SOFT8, 64_000_000) == 64_000_000
    assert vo.input_size(vo.FP32, 64_000_000) == 256_000_000
    assert vo.message_len(0, 2_000_000) == 999_936


@pytest.mark.parametrize("ch", [0, 1, 2, 3, 4])
def test_packer_matches_harness_pipeline(vo, ch):
    """vo_pack (SoftDecisionPacker on given floats) equals the harness' own packing of the noiseless
    BPSK codeword (RandBitGen | ConvolutionalEncoder | AddNoise(+inf) | SoftDecisionPacker)."""
    n = 4096
    bits, packed = vo.simulate(ch, n, 0.0, 21, 22, noiseless=True)
    reg = 0
    vals = np.empty(2 * n, dtype=np.float32)
    for i, b in enumerate(bits):
        reg = ((reg >> 1) | (int(b) << 6)) & 127
        vals[2 * i] = 1.0 if bin(reg & 0o171).count("1") & 1 else -1.0
        vals[2 * i + 1] = 1.0 if bin(reg & 0o133).count("1") & 1 else -1.0
    assert np.array_equal(vo.pack(ch, vals, 40000.0).view(np.uint32), packed.view(np.uint32))


def test_short_buffers_raise(vo):
    """The wrapper refuses inputs shorter than the C side reads (round 4: a parity slice sized in packed words
    instead of bytes made decode_chunk read past the buffer and crash): a ValueError, not a read past the end."""
    opt = vo.SOFT8 | vo.M_B16
    n = 2 * 100_000
    bits, packed = vo.simulate(opt, n // 2, 1.0, 3, 4)
    ref, ok = vo.decode(opt, packed, input_num=n)
    assert ok and ref.size > 0
    short = packed[:packed.size // 4]  # the round-4 mistake: a quarter of the bytes
    with pytest.raises(ValueError, match="reads"):
        vo.decode(opt, short, input_num=n)
    with pytest.raises(ValueError, match="C-contiguous"):
        vo.decode(opt, np.repeat(packed, 2)[::2], input_num=n)
    with pytest.raises(ValueError):
        vo.decode(opt, list(packed), input_num=n)
    vals = np.zeros(n, dtype=np.float32)
    assert vo.pack(opt, vals, 40000.0, input_num=n).nbytes == vo.input_size(opt, n)
    with pytest.raises(ValueError, match="inputNum"):
        vo.pack(opt, vals[:n // 2], 40000.0, input_num=n)
