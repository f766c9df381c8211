"""Batched HARD, SOFT4, SOFT8 and FP32 launches on vd_decode_pk (vd_kernel_pk.h): two chunks per wave, one in
each 16-bit half of the metric word (HARD: 8-stage history fields; SOFT4 / FP32: 4-stage fields; SOFT8:
2-stage fields, renormalised every 8 stages, position-space ring and traceback), 32- and 16-bit output words.  Every batch must equal the oracle word for word and the fp32 tagged kernel's output
(VD_NO_PK=1 at decoder creation selects it), for every metric core's tie rule, including chunk counts where
the two chunks of a wave differ in length (an odd number of long chunks), partitions with empty chunks, and
saturated inputs (SNR 15: the best path gains every stage, the largest range the int16 halves must hold)."""
import os

import numpy as np
import pytest
import torch

from vitdec import FP32, HARD, M_B16, M_B32, M_FP16, O_B16, SOFT4, SOFT8
from test_gpu_parity import name


def _batches(gpu, opt, nbits, snr, nb, seed):
    n = 2 * nbits
    nin = gpu.lib().vd_input_size(opt, n)
    stride = (nin + 255) // 256 * 256
    packed = torch.zeros(nb * stride, dtype=torch.uint8, device="cuda")
    bits = torch.empty(nbits, dtype=torch.uint8, device="cuda")
    for b in range(nb):
        gpu.simulate_device(opt, nbits, snr, seed + 2 * b, seed + 1 + 2 * b, bits.data_ptr(), packed.data_ptr() + b * stride)
    torch.cuda.synchronize()
    return packed, stride, nin


def _decode_batched(gpu, opt, packed, stride, n, nb, no_pk):
    nout = gpu.lib().vd_output_size(opt, n)
    ostride = (nout + 255) // 256 * 256
    out = torch.full((nb * ostride,), 0x5A, dtype=torch.uint8, device="cuda")
    old = os.environ.get("VD_NO_PK")
    os.environ["VD_NO_PK"] = "1" if no_pk else "0"
    try:
        with gpu.ViterbiCUDA(opt) as dec:
            dec.run_device_batch(packed.data_ptr(), stride, out.data_ptr(), ostride, n, nb)
            torch.cuda.synchronize()
    finally:
        if old is None:
            del os.environ["VD_NO_PK"]
        else:
            os.environ["VD_NO_PK"] = old
    for b in range(nb):  # nothing written between the batches' outputs
        assert bool((out[b * ostride + nout:(b + 1) * ostride] == 0x5A).all())
    return out, ostride, nout


PK_OPTS = ([ch | me for ch in (HARD, SOFT4, FP32) for me in (M_B32, M_B16, M_FP16)] + [SOFT8 | M_B32, SOFT8 | M_B16] +
           [HARD | M_B32 | O_B16, FP32 | M_FP16 | O_B16, SOFT8 | M_B16 | O_B16, SOFT8 | M_B32 | O_B16])


def test_packed_kernel_names():
    import vitdec
    for opt in PK_OPTS:
        assert vitdec.kernel_name(opt).startswith("vd_decode_pk<")


@pytest.mark.gpu
@pytest.mark.parametrize("opt", PK_OPTS, ids=name)
@pytest.mark.parametrize("nbits,snr", [(1_000_032, 0.5), (4_000_032, 1.2), (150_000, 0.0), (2_000_000, 15.0)])
def test_packed_batches_equal_oracle_and_fp32_kernel(gpu, vo, opt, nbits, snr):
    nb, n = 3, 2 * nbits
    pack = (nbits - 64) // 32
    packed, stride, nin = _batches(gpu, opt, nbits, snr, nb, 71)
    pk, ostride, nout = _decode_batched(gpu, opt, packed, stride, n, nb, no_pk=False)
    tg, _, _ = _decode_batched(gpu, opt, packed, stride, n, nb, no_pk=True)
    for b in range(nb):
        p = packed[b * stride:b * stride + nin].cpu().numpy().view(np.int32)
        ref, ok = vo.decode(opt, p, input_num=n, nthreads=16)
        got = pk[b * ostride:b * ostride + nout].cpu().numpy().view(ref.dtype)
        bad = np.flatnonzero(got != ref)
        assert bad.size == 0, f"batch {b}: {bad.size} of {ref.size} words differ (pack {pack}, rem {pack % 6400}), first {bad[:5]}"
        assert torch.equal(pk[b * ostride:b * ostride + nout], tg[b * ostride:b * ostride + nout])


def _single(gpu, opt, packed_t, nin, n, env):
    import vitdec  # noqa: F401
    nout = gpu.lib().vd_output_size(opt, n)
    out = torch.full((nout + 256,), 0x5A, dtype=torch.uint8, device="cuda")
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        with gpu.ViterbiCUDA(opt) as dec:
            dec.run_device(packed_t.data_ptr(), out.data_ptr(), n)
            torch.cuda.synchronize()
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    assert bool((out[nout:] == 0x5A).all())  # nothing written past the output
    return out[:nout]


@pytest.mark.gpu
@pytest.mark.parametrize("opt", [HARD | M_B32, HARD | M_B16, HARD | M_FP16, SOFT4 | M_B32, FP32 | M_FP16,
                                 HARD | M_B32 | O_B16, FP32 | M_FP16 | O_B16], ids=name)
@pytest.mark.parametrize("nbits,snr", [(13_107_264, 1.0), (20_000_000, 0.0), (9_000_000, 2.0), (32_000_000, 15.0)])
def test_packed_split_single_launch(gpu, vo, opt, nbits, snr):
    """Single-batch launches on vd_decode_pk's split kernel (one chunk per wave, cut at a multiple of 3 blocks,
    the second part started 6 blocks early and checked at the cut): equal to vd_decode_tg's segment launch
    (VD_PK_SPLIT=0), to the unsplit launch (VD_NO_SPLIT=1), to the split launch without tail workgroups
    (VD_PK_TAIL=0) and to the oracle.  With 6400 chunks on 1024 SIMDs the last 256 chunks go to tail
    workgroups (8 parts over 4 waves, checks across waves).  13.1M bits: 64 words per chunk (the smallest
    split); 9M bits: below it (not split)."""
    n = 2 * nbits
    packed, stride, nin = _batches(gpu, opt, nbits, snr, 1, 91)
    before = gpu.split_redecodes()
    pk = _single(gpu, opt, packed, nin, n, {})
    redec = gpu.split_redecodes() - before
    tg = _single(gpu, opt, packed, nin, n, {"VD_PK_SPLIT": "0"})
    whole = _single(gpu, opt, packed, nin, n, {"VD_NO_SPLIT": "1"})
    notail = _single(gpu, opt, packed, nin, n, {"VD_PK_TAIL": "0"})
    p = packed[:nin].cpu().numpy().view(np.int32)
    ref, ok = vo.decode(opt, p, input_num=n, nthreads=16)
    got = pk.cpu().numpy().view(ref.dtype)
    bad = np.flatnonzero(got != ref)
    assert bad.size == 0, f"{bad.size} of {ref.size} words differ (re-decoded: {redec}), first {bad[:5]}"
    assert torch.equal(pk, tg) and torch.equal(pk, whole) and torch.equal(pk, notail)


@pytest.mark.gpu
@pytest.mark.parametrize("opt", [HARD | M_B32, SOFT4 | M_B16, SOFT8 | M_B16, SOFT8 | M_B32, SOFT8 | M_B16 | O_B16], ids=name)
def test_packed_split_random_input_redecodes(gpu, vo, opt):
    """Uniformly random channel words: the second part's speculative start often does not converge (HARD:
    652 of 6400 chunks on the first run; SOFT8 about a fifth of the parts), so re-decodes run -- most of them
    stopping at a checkpoint one or two groups after the cut (vd_kernel_pk.h "Early stop"), the rest decoding
    the whole part -- and the words still equal the oracle's.  No wave reaches the re-decode pass cap with a
    part still differing (vd_split_cap_exits: the passes provably end within P, P = 2 per whole-chunk wave and
    8 per tail workgroup; tests/test_split_model.py checks that bound on the host model)."""
    nbits = 16_000_000
    n = 2 * nbits
    env = {}
    nin = gpu.lib().vd_input_size(opt, n)
    g = torch.Generator(device="cpu").manual_seed(5)
    packed = torch.randint(0, 256, (nin + 256,), dtype=torch.uint8, generator=g).to("cuda")
    before, caps = gpu.split_redecodes(), gpu.split_cap_exits()
    pk = _single(gpu, opt, packed, nin, n, env)
    redec = gpu.split_redecodes() - before
    assert gpu.split_cap_exits() == caps == 0
    p = packed[:nin].cpu().numpy().view(np.int32)
    ref, ok = vo.decode(opt, p, input_num=n, nthreads=16)
    got = pk.cpu().numpy().view(ref.dtype)
    bad = np.flatnonzero(got != ref)
    assert bad.size == 0, f"{bad.size} of {ref.size} words differ (re-decoded: {redec}), first {bad[:5]}"
    assert redec > 0, redec
    notail = _single(gpu, opt, packed, nin, n, dict(env, VD_PK_TAIL="0"))
    assert torch.equal(pk, notail)


@pytest.mark.gpu
@pytest.mark.parametrize("opt", [SOFT8 | M_B16, SOFT8 | M_B32, SOFT8 | M_B16 | O_B16], ids=name)
@pytest.mark.parametrize("nbits,snr", [(13_107_264, 1.0), (20_000_000, 0.0), (32_000_000, 15.0)])
def test_packed_split_soft8(gpu, vo, opt, nbits, snr):
    """SOFT8 single-batch launches split on vd_decode_pk: equal to the oracle, to vd_decode_tg's segment launch
    (VD_PK_SPLIT=0) and to the split launch without tail workgroups."""
    n = 2 * nbits
    packed, stride, nin = _batches(gpu, opt, nbits, snr, 1, 93)
    pk = _single(gpu, opt, packed, nin, n, {})
    tg = _single(gpu, opt, packed, nin, n, {"VD_PK_SPLIT": "0"})
    notail = _single(gpu, opt, packed, nin, n, {"VD_PK_TAIL": "0"})
    p = packed[:nin].cpu().numpy().view(np.int32)
    ref, ok = vo.decode(opt, p, input_num=n, nthreads=16)
    got = pk.cpu().numpy().view(ref.dtype)
    bad = np.flatnonzero(got != ref)
    assert bad.size == 0, f"{bad.size} of {ref.size} words differ, first {bad[:5]}"
    assert torch.equal(pk, tg) and torch.equal(pk, notail)


def _soft8_pattern(kind, nin, seed):
    """SOFT8 channel bytes that stress the int16 range of the 2-stage-field format: every byte -128 (BM +-256
    every stage), every byte 127, saturated random signs (-128 / 127), and uniformly random bytes"""
    g = torch.Generator(device="cpu").manual_seed(seed)
    if kind == "all_min":
        return torch.full((nin,), 0x80, dtype=torch.uint8)
    if kind == "all_max":
        return torch.full((nin,), 0x7F, dtype=torch.uint8)
    if kind == "saturated":
        return torch.where(torch.randint(0, 2, (nin,), generator=g) == 1, 0x7F, 0x80).to(torch.uint8)
    return torch.randint(0, 256, (nin,), dtype=torch.uint8, generator=g)


@pytest.mark.gpu
@pytest.mark.parametrize("opt", [SOFT8 | M_B16, SOFT8 | M_B32], ids=name)
@pytest.mark.parametrize("kind", ["all_min", "all_max", "saturated", "random"])
def test_packed_soft8_extreme_inputs(gpu, vo, opt, kind):
    """SOFT8 on vd_decode_pk: batched launches (3 batches) of synthetic channel bytes at the ends of the metric
    range (header of vd_kernel_pk.h: candidates within [-3072, 4864] units of position 0's metric, renormalised
    every 8 stages), equal to the oracle word for word; the single-batch launch of batch 0 too, both on the
    packed split kernel (the default for SOFT8 single batches) and on vd_decode_tg's segment launch
    (VD_PK_SPLIT=0)"""
    nbits = 13_107_264
    n = 2 * nbits
    nb = 3
    nin = gpu.lib().vd_input_size(opt, n)
    stride = (nin + 255) // 256 * 256
    host = torch.zeros(nb * stride, dtype=torch.uint8)
    for b in range(nb):
        host[b * stride:b * stride + nin] = _soft8_pattern(kind, nin, 11 + b)
    packed = host.to("cuda")
    pk, ostride, nout = _decode_batched(gpu, opt, packed, stride, n, nb, no_pk=False)
    single = _single(gpu, opt, packed[:stride], nin, n, {})
    single_tg = _single(gpu, opt, packed[:stride], nin, n, {"VD_PK_SPLIT": "0"})
    assert torch.equal(single, single_tg)
    for b in range(nb):
        p = host[b * stride:b * stride + nin].numpy().view(np.int32)
        ref, ok = vo.decode(opt, p, input_num=n, nthreads=16)
        got = pk[b * ostride:b * ostride + nout].cpu().numpy().view(ref.dtype)
        bad = np.flatnonzero(got != ref)
        assert bad.size == 0, f"batch {b}: {bad.size} of {ref.size} words differ, first {bad[:5]}"
        if b == 0:
            got1 = single.cpu().numpy().view(ref.dtype)
            bad = np.flatnonzero(got1 != ref)
            assert bad.size == 0, f"single launch: {bad.size} of {ref.size} words differ, first {bad[:5]}"
