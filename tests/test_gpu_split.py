"""Segment launches (vd_kernel_tg.h "segment launches"): single 6400-chunk launches cut
into workgroup segments ("pieces": the last 256 chunks in 4 pieces each; "thirds": workgroups of 3 or 4
chunks in 4 segments that cross chunk boundaries).  A segment that starts inside a chunk starts
speculatively and is checked at its boundary after a workgroup barrier; one whose check fails
re-decodes from its left neighbour's end vector.  The decoded words must be identical to the unsplit launch (VD_NO_SPLIT=1) and
to the oracle, at SNRs where the speculation always converges and where it often does not (SNR 0: the
re-decode passes run, and the test requires that they did).  HARD, SOFT4, SOFT8 and FP32 single launches run
vd_decode_pk's split launch by default (mode "pk": one chunk per wave, its second part in the other int16
half with a speculative start, checked at the cut, re-decoded from the first part's vector when it
differs); "pieces" / "thirds" set VD_PK_SPLIT=0 to test vd_decode_tg's segment tables on them too."""
import os

import numpy as np
import pytest

from vitdec import FP32, HARD, M_B16, M_B32, M_FP16, O_B16, SOFT4, SOFT8, SOFT16
from test_gpu_parity import gpu_decode, name


PK_CH = (HARD, SOFT4, SOFT8, FP32)


def set_mode(mode):
    """environment of a decoder created next: 'pk' = the default (vd_decode_pk split for HARD/SOFT4/SOFT8/FP32),
    'pieces' / 'thirds' = vd_decode_tg segment tables for every format"""
    if mode in ("pieces", "thirds"):
        os.environ["VD_SPLIT"] = mode
        os.environ["VD_PK_SPLIT"] = "0"


def clear_mode():
    os.environ.pop("VD_SPLIT", None)
    os.environ.pop("VD_PK_SPLIT", None)


def decode_split_and_whole(gpu, opt, packed, n, mode=None):
    before = gpu.split_redecodes()
    set_mode(mode)
    try:
        out = gpu_decode(gpu, opt, packed)
    finally:
        clear_mode()
    redecodes = gpu.split_redecodes() - before
    os.environ["VD_NO_SPLIT"] = "1"
    try:
        whole = gpu_decode(gpu, opt, packed)
    finally:
        del os.environ["VD_NO_SPLIT"]
    return out, whole, redecodes


@pytest.mark.gpu
@pytest.mark.parametrize("opt", [HARD | M_B32, SOFT8 | M_B16, SOFT4 | M_B32, FP32 | M_FP16, SOFT16 | M_B32,
                                 HARD | M_B32 | O_B16, SOFT8 | M_B16 | O_B16, FP32 | M_FP16 | O_B16], ids=name)
@pytest.mark.parametrize("snr", [0.0, 1.0, 3.0])
@pytest.mark.parametrize("mode", ["pieces", "thirds", "pk"])
def test_split_equals_whole_16m(gpu, vo, opt, snr, mode):
    if mode == "pk" and (opt & 0xF) not in PK_CH:
        pytest.skip("no packed kernel for this input format")
    # 78 32-bit words per chunk: segment launch (>= 64); O_B16: 156-157 16-bit words per chunk (odd
    # counts: the last segment of a chunk writes its final half word only).  pieces: 256 chunks in 4
    # pieces; thirds: workgroups of 3 (4) chunks in 4 segments, segments crossing chunk boundaries
    n = 16_000_000
    bits, packed = gpu_sim(gpu, opt, n, snr)
    out, whole, redecodes = decode_split_and_whole(gpu, opt, packed, n, mode)
    bad = np.flatnonzero(out != whole)
    assert bad.size == 0, f"{bad.size} words differ (re-decoded pieces: {redecodes}), first {bad[:5]}"
    ref, ok = vo.decode(opt, packed, nthreads=16)
    assert ok
    bad = np.flatnonzero(out != ref)
    assert bad.size == 0, f"{bad.size} words differ from the oracle (re-decoded pieces: {redecodes}), first {bad[:5]}"
    if snr == 0.0:  # at 0 dB speculative starts often have not converged: the re-decode passes ran
        assert redecodes > 0


def gpu_sim(gpu, opt, n, snr):
    import torch
    nbytes = gpu.lib().vd_input_size(opt, 2 * n)
    bits = torch.zeros(n, dtype=torch.uint8, device="cuda")
    packed = torch.zeros((nbytes + 3) // 4 * 4, dtype=torch.uint8, device="cuda")
    gpu.simulate_device(opt, n, snr, 3, 4, bits.data_ptr(), packed.data_ptr())
    torch.cuda.synchronize()
    p = packed.cpu().numpy()[:nbytes]
    return bits.cpu().numpy(), p.view(np.float32 if (opt & 0xF) == FP32 else np.int32)


@pytest.mark.gpu
@pytest.mark.slow
@pytest.mark.parametrize("snr", [0.0, 1.2])
@pytest.mark.parametrize("opt", [HARD | M_B32, SOFT8 | M_B16], ids=name)
@pytest.mark.parametrize("mode", ["pieces", "thirds", "pk"])
def test_split_full_32m_matches_oracle(gpu, vo, opt, snr, mode):
    if mode == "pk" and (opt & 0xF) not in PK_CH:
        pytest.skip("no packed kernel for this input format")
    bits, packed = gpu_sim(gpu, opt, 32_000_000, snr)
    before = gpu.split_redecodes()
    set_mode(mode)
    try:
        out = gpu_decode(gpu, opt, packed)
    finally:
        clear_mode()
    redecodes = gpu.split_redecodes() - before
    ref, ok = vo.decode(opt, packed, nthreads=16)
    assert ok
    np.testing.assert_array_equal(out, ref)
    print(f"snr {snr}, {mode}: {redecodes} segments re-decoded")
    if snr == 0.0:
        assert redecodes > 0


@pytest.mark.gpu
def test_no_split_below_min_words(gpu):
    # 8M bits: 39 words per chunk, below kSplitMinWords: the launch is not split (nothing re-decoded)
    opt = SOFT8 | M_B16
    bits, packed = gpu_sim(gpu, opt, 8_000_000, 0.0)
    before = gpu.split_redecodes()
    out, whole, _ = decode_split_and_whole(gpu, opt, packed, 8_000_000)
    np.testing.assert_array_equal(out, whole)
    assert gpu.split_redecodes() == before
