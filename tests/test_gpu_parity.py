"""GPU parity: the HIP decode path (through the C-ABI) vs the CPU oracle, bit-exact.

Every valid option combination of the reference (OptionsValid, viterbi.h:22-41) is decoded on the
MI355X and compared word-for-word with oracle/vd_oracle.c on the same seeded inputs: low SNR
(many ties and wrong survivors), mid SNR and the CLI default SNR 15.  Long chunks (more than one
traceback batch), empty chunks, ragged partitions and odd O_B16 word counts are covered, and the
known-answer BEN table of SURVEY 8(c) is re-checked end to end through the product.
"""
import hashlib

import numpy as np
import pytest

from vitdec import (DPX, FP32, HARD, M_B16, M_B32, M_FP16, O_B16, O_B32, REG, SOFT4, SOFT8, SOFT16)

INPUTS = [HARD, SOFT4, SOFT8, SOFT16, FP32]
METRICS = [M_B32, M_B16, M_FP16]


def valid_reg(vd, outs=(O_B32, O_B16)):
    return [i | m | o | REG for i in INPUTS for m in METRICS for o in outs if vd.options_valid(i | m | o | REG)]


def name(opt):
    i = {HARD: "h", SOFT4: "s4", SOFT8: "s8", SOFT16: "s16", FP32: "f"}[opt & 0xF]
    m = {M_B32: "b32", M_B16: "b16", M_FP16: "f16"}[opt & 0xF0]
    o = {O_B32: "o32", O_B16: "o16"}[opt & 0xF00]
    return f"{i}-{m}-{o}" + ("-dpx" if opt & DPX else "")


def _valid_list():
    import vitdec
    return [i | m | o | REG for i in INPUTS for m in METRICS for o in (O_B32, O_B16)
            if not ((i == SOFT8 and m == M_FP16) or (i == SOFT16 and m in (M_FP16, M_B16)))]


VALID = _valid_list()


def gpu_decode(vd, opt, packed, input_num=None):
    with vd.ViterbiCUDA(opt) as d:
        out, ms = d.run(packed, inputNum=input_num)
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("opt", VALID, ids=name)
@pytest.mark.parametrize("snr", [0.0, 1.2, 15.0])
def test_parity_1m(gpu, vo, opt, snr):
    bits, packed = vo.simulate(opt, 1_000_000, snr, 101, 202)
    ref, ok = vo.decode(opt, packed)
    assert ok, "oracle left the reference's exact metric range"
    out = gpu_decode(gpu, opt, packed)
    assert out.dtype == ref.dtype and out.shape == ref.shape
    bad = np.flatnonzero(out != ref)
    assert bad.size == 0, f"{bad.size} words differ, first at {bad[:5]}"


@pytest.mark.gpu
@pytest.mark.parametrize("opt", [HARD | M_B32, SOFT8 | M_B16, FP32 | M_FP16, SOFT16 | M_B32, SOFT4 | M_B16 | O_B16,
                                 HARD | M_FP16 | O_B16], ids=name)
def test_parity_long_chunks(gpu, vo, opt):
    # 4.2M bits: ~20 words per chunk -> two traceback batches per chunk
    bits, packed = vo.simulate(opt, 4_200_000, 1.1, 7, 8)
    ref, ok = vo.decode(opt, packed)
    assert ok
    out = gpu_decode(gpu, opt, packed)
    np.testing.assert_array_equal(out, ref)


@pytest.mark.gpu
@pytest.mark.parametrize("opt", VALID, ids=name)
def test_parity_full_range_inputs(gpu, vo, opt):
    # random channel words over each format's whole range (every soft value and sign combination, FP32
    # values from +-2^-10 to +-2^20 incl. exact integers and the clamp limits): the branch metrics span
    # [BMmin, BMmax], so the path-metric spread reaches the bound the tagged kernels are sized for
    # (vd_kernel_tg.h TgFmt; SOFT16's int32 patterns in particular)
    rng = np.random.default_rng(opt + 99)
    n = 2_000_000  # encoded values (1M bits)
    nbytes = gpu.lib().vd_input_size(opt, n)
    if (opt & 0xF) == FP32:
        mag = np.exp2(rng.uniform(-10, 20, n)).astype(np.float32)
        small = rng.random(n) < 0.2  # exact small integers, where the truncation to int decides
        mag[small] = rng.integers(0, 9, int(small.sum())).astype(np.float32)
        vals = np.where(rng.random(n) < 0.5, -mag, mag).astype(np.float32)
        vals[::97] = 7.0
        vals[1::97] = -8.0
        packed = vals
    else:
        packed = rng.integers(0, 2 ** 32, nbytes // 4, dtype=np.uint64).astype(np.uint32).view(np.int32)
    ref, ok = vo.decode(opt, packed, input_num=n)
    assert ok
    out = gpu_decode(gpu, opt, packed, input_num=n)
    bad = np.flatnonzero(out != ref)
    assert bad.size == 0, f"{bad.size} words differ, first at {bad[:5]}"


@pytest.mark.gpu
@pytest.mark.parametrize("n_bits", [160, 2_048, 3_008, 204_800, 206_400, 409_616, 1_000_016])
@pytest.mark.parametrize("opt", [HARD | M_B32, SOFT8 | M_B16 | O_B16, FP32 | M_FP16], ids=name)
def test_parity_ragged_and_empty_chunks(gpu, vo, opt, n_bits):
    # packNum < 6400 (most chunks empty), base/rem splits, odd O_B16 word counts
    bits, packed = vo.simulate(opt, n_bits, 0.6, 11, 12)
    ref, ok = vo.decode(opt, packed)
    out = gpu_decode(gpu, opt, packed)
    np.testing.assert_array_equal(out, ref)


@pytest.mark.gpu
def test_dpx_decodes_like_reg(gpu, vo):
    bits, packed = vo.simulate(HARD | M_B16, 300_000, 0.0, 5, 6)
    a = gpu_decode(gpu, HARD | M_B16 | DPX, packed)
    b = gpu_decode(gpu, HARD | M_B16 | REG, packed)
    np.testing.assert_array_equal(a, b)


# ---- known answers, through the product's own host harness + GPU decode ----
KAT_COLS = {"h/b32": HARD | M_B32, "h/b16": HARD | M_B16, "h/f16": HARD | M_FP16, "s8/b32": SOFT8 | M_B32,
            "s8/b16": SOFT8 | M_B16, "s4/b32": SOFT4 | M_B32, "s4/b16": SOFT4 | M_B16, "s4/f16": SOFT4 | M_FP16,
            "s16/b32": SOFT16 | M_B32, "f/b32": FP32 | M_B32, "f/b16": FP32 | M_B16, "f/f16": FP32 | M_FP16}
KAT = [(0.0, "h/b32", 374310), (0.0, "h/b16", 374582), (0.0, "h/f16", 375102), (0.0, "s8/b32", 373999),
       (0.0, "s8/b16", 373977), (0.0, "s4/b32", 375558), (0.0, "s4/b16", 375524), (0.0, "s4/f16", 375306),
       (0.0, "s16/b32", 229390), (0.0, "f/b32", 375556), (0.0, "f/b16", 375522), (0.0, "f/f16", 375292),
       (1.0, "h/b32", 5684), (1.0, "s8/b16", 5971), (1.0, "f/f16", 6201), (1.2, "h/b16", 929),
       (1.4, "h/f16", 102), (1.6, "s8/b16", 11), (2.0, "s16/b32", 0)]


@pytest.mark.gpu
@pytest.mark.parametrize("snr,col,ben", KAT, ids=[f"{s}-{c}" for s, c, _ in KAT])
def test_known_answer_ben(gpu, snr, col, ben):
    opt = KAT_COLS[col]
    bits, packed = gpu.simulate_host(opt, 1_000_000, snr, 11, 22)
    out = gpu_decode(gpu, opt, packed)
    assert gpu.count_errors(opt, bits, out) == ben


@pytest.mark.gpu
def test_sha256_pin(gpu):
    opt = HARD | M_B32
    bits, packed = gpu.simulate_host(opt, 400_000, 1.3, 5, 6)
    assert hashlib.sha256(packed.tobytes()).hexdigest() == \
        "07a65ee53e9bca21357374071441f8a531160357d1e82f9d915c80efea7eb7f8"
    out = gpu_decode(gpu, opt, packed)
    assert out.nbytes == 49_992
    assert hashlib.sha256(out.tobytes()).hexdigest() == \
        "c48c6382e8b94b2e09d829c4898f15ae6ddf814eadb23863fc069e6ef77d3bfb"


@pytest.mark.gpu
def test_o_b16_known_answer_within_race(gpu, vo):
    # reference O_B16 has a cross-chunk write race; the product is race-free
    # (every chunk writes only its own words) == oracle policy 0, 8 bits from the emulated KAT.
    opt = HARD | M_B32 | O_B16
    bits, packed = gpu.simulate_host(opt, 1_000_000, 0.0, 11, 22)
    out = gpu_decode(gpu, opt, packed)
    ref, _ = vo.decode(opt, packed, b16_policy=0)
    np.testing.assert_array_equal(out, ref)
    assert abs(gpu.count_errors(opt, bits, out) - 374610) <= 16


@pytest.mark.gpu
@pytest.mark.slow
@pytest.mark.parametrize("opt", [HARD | M_B32, SOFT8 | M_B16], ids=name)
def test_parity_full_32m(gpu, vo, opt):
    # BASELINE configs 2 and 3 at full size, every word checked against the oracle
    bits, packed = vo.simulate(opt, 32_000_000, 1.2, 1, 2)
    ref, ok = vo.decode(opt, packed, nthreads=16)
    assert ok
    out = gpu_decode(gpu, opt, packed)
    np.testing.assert_array_equal(out, ref)
    assert gpu.count_errors(opt, bits, out) == vo.ben(opt, bits, ref)


@pytest.mark.gpu
@pytest.mark.slow
def test_parity_full_32m_soft16(gpu, vo):
    # 32M bits of 16-bit soft input on the int32-pattern tagged kernel, every word against the oracle
    opt = SOFT16 | M_B32
    bits, packed = vo.simulate(opt, 32_000_000, 1.2, 5, 6)
    ref, ok = vo.decode(opt, packed, nthreads=16)
    assert ok
    out = gpu_decode(gpu, opt, packed)
    np.testing.assert_array_equal(out, ref)
    assert gpu.count_errors(opt, bits, out) == vo.ben(opt, bits, ref)


@pytest.mark.gpu
@pytest.mark.slow
def test_parity_full_32m_fp32_fp16(gpu, vo):
    # BASELINE configs[4]: 32M bits, FP32 soft input on the fp16 path-metric core, every word (tolerance 0)
    opt = FP32 | M_FP16
    bits, packed = vo.simulate(opt, 32_000_000, 1.2, 3, 4)
    ref, ok = vo.decode(opt, packed, nthreads=16)
    assert ok
    out = gpu_decode(gpu, opt, packed)
    np.testing.assert_array_equal(out, ref)


@pytest.mark.gpu
@pytest.mark.slow
def test_parity_256m_one_stream(gpu, vo):
    # BASELINE configs[3]'s 256M bits as ONE stream on one GPU (base = 1249 words per chunk):
    # long chunks, 40 traceback batches each; every word against the oracle, and the BEN equal
    opt = SOFT8 | M_B16
    bits, packed = vo.simulate(opt, 256_000_000, 1.3, 9, 10)
    ref, ok = vo.decode(opt, packed, nthreads=16)
    assert ok and ref.size == 255_999_936 // 32
    out = gpu_decode(gpu, opt, packed)
    np.testing.assert_array_equal(out, ref)
    assert gpu.count_errors(opt, bits, out) == vo.ben(opt, bits, ref)
