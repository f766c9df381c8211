"""GPU parity of the float-input path: the reference's SoftDecisionPacker (src/viterbiDF.h:98-167) on
the device (vd_pack_device) and fused into the decode (vd_run_llr / vd_run_device_llr).

The checker is the oracle's restatement of the packer (oracle/vd_oracle.c vo_pack, x86 lrintf
semantics included: NaN and |v| >= 2^63 give LONG_MIN, SOFT4/SOFT8 narrow the long to int before
saturating) followed by the oracle decode of the packed words.  Bit-exact, every valid option.
"""
import numpy as np
import pytest

from vitdec import FP32, HARD, M_B16, M_B32, M_FP16, O_B16, O_B32, REG, SOFT4, SOFT8, SOFT16
from test_gpu_parity import VALID, name

CHANNELS = [HARD, SOFT4, SOFT8, SOFT16, FP32]


def channel_values(n, snr, seed):
    """BPSK +-1 of a random K=7 (0171, 0133) codeword plus AWGN (reference scaling sigma = 10^(-snr/5))."""
    rng = np.random.default_rng(seed)
    bits = rng.integers(0, 2, n // 2)
    reg = 0
    out = np.empty(n, dtype=np.float32)
    for i, b in enumerate(bits):
        reg = ((reg >> 1) | (int(b) << 6)) & 127
        out[2 * i] = 1.0 if bin(reg & 0o171).count("1") & 1 else -1.0
        out[2 * i + 1] = 1.0 if bin(reg & 0o133).count("1") & 1 else -1.0
    sigma = np.float32(10.0 ** (-snr / 5.0))
    return (out + rng.standard_normal(n).astype(np.float32) * sigma).astype(np.float32)


def channel_values_fast(n, snr, seed):
    """channel_values without the Python loop (numpy taps of the same encoder; other random draws)"""
    rng = np.random.default_rng(seed)
    b = np.concatenate([np.zeros(6, np.uint8), rng.integers(0, 2, n // 2).astype(np.uint8)])
    t = np.arange(6, b.size)
    o0 = b[t] ^ b[t - 1] ^ b[t - 2] ^ b[t - 3] ^ b[t - 6]  # 0171: register bits 6, 5, 4, 3, 0
    o1 = b[t] ^ b[t - 2] ^ b[t - 3] ^ b[t - 5] ^ b[t - 6]  # 0133: register bits 6, 4, 3, 1, 0
    out = np.empty(n, dtype=np.float32)
    out[0::2] = np.where(o0 == 1, 1.0, -1.0)
    out[1::2] = np.where(o1 == 1, 1.0, -1.0)
    sigma = np.float32(10.0 ** (-snr / 5.0))
    return (out + rng.standard_normal(n).astype(np.float32) * sigma).astype(np.float32)


def specials():
    """Ties, signed zeros, saturation, the x86 lrintf 'integer indefinite' cases, denormals."""
    v = [0.0, -0.0, 0.5, 1.5, 2.5, -0.5, -1.5, -2.5, 7.5, -8.5, 127.5, -128.5, 128.0, -129.0, 32767.5, -32768.5,
         40000.0, -40000.0, 2.0 ** 31, -(2.0 ** 31) - 512, 2.0 ** 32 + 5 * 256, 3.0e9, 9.3e18, -9.3e18, 1e30, -1e30,
         np.inf, -np.inf, np.nan, 1e-40, -1e-40, 0.49999997]
    return np.array(v, dtype=np.float32)


def gpu_pack(opt, values, scale):
    import torch
    import vitdec
    v = torch.from_numpy(values).cuda()
    nbytes = vitdec.lib().vd_input_size(opt, values.size)
    out = torch.zeros((nbytes + 3) // 4 * 4, dtype=torch.uint8, device="cuda")
    vitdec.pack_device(opt, v.data_ptr(), values.size, out.data_ptr(), scale=scale,
                       stream=torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    return out.cpu().numpy()[:nbytes]


@pytest.mark.gpu
@pytest.mark.parametrize("ch", CHANNELS)
@pytest.mark.parametrize("n", [4096, 4096 + 6, 2 * 333_333])
def test_pack_device_matches_packer(gpu, vo, ch, n):
    vals = channel_values(n, 1.0, 7 + n)
    got = gpu_pack(ch, vals, 40000.0)
    ref = vo.pack(ch, vals, 40000.0).view(np.uint8)[:got.size]
    assert np.array_equal(got, ref)


@pytest.mark.gpu
@pytest.mark.parametrize("ch", CHANNELS)
def test_pack_device_edge_values(gpu, vo, ch):
    vals = np.resize(specials(), 4 * 32 * 3)  # several words of every channel width
    for scale in (1.0, 40000.0):
        got = gpu_pack(ch, vals, scale)
        ref = vo.pack(ch, vals, scale).view(np.uint8)[:got.size]
        if ch == FP32:  # compare float bit patterns (NaN included)
            assert np.array_equal(got.view(np.uint32), ref.view(np.uint32))
        else:
            assert np.array_equal(got, ref), f"scale {scale}"


@pytest.mark.gpu
@pytest.mark.parametrize("opt", VALID, ids=name)
@pytest.mark.parametrize("snr", [0.0, 1.2])
def test_fused_llr_decode(gpu, vd, vo, opt, snr):
    vals = channel_values(2 * 200_000, snr, 11)
    packed = vo.pack(opt, vals, 40000.0)
    ref, ok = vo.decode(opt, packed, input_num=vals.size)
    assert ok
    with vd.ViterbiCUDA(opt) as d:
        out, _ = d.run_llr(vals, scale=40000.0)
        via_pack, _ = d.run(packed, inputNum=vals.size)
    assert np.array_equal(via_pack, ref)
    bad = np.flatnonzero(out != ref)
    assert bad.size == 0, f"{bad.size} words differ, first at {bad[:5]}"


@pytest.mark.gpu
@pytest.mark.parametrize("opt", [HARD | M_B32, SOFT4 | M_B16, SOFT8 | M_B16, SOFT16 | M_B32, FP32 | M_FP16],
                         ids=name)
def test_fused_llr_decode_with_edge_values(gpu, vd, vo, opt):
    vals = channel_values(2 * 50_000, 1.0, 5)
    rng = np.random.default_rng(3)
    idx = rng.choice(vals.size, 500, replace=False)
    vals[idx] = np.resize(specials(), idx.size)
    if (opt & 0xF) == FP32:  # the FP32 branch metric of NaN is not defined by the reference: keep finite
        vals[~np.isfinite(vals)] = 1e30
    packed = vo.pack(opt, vals, 40000.0)
    ref, ok = vo.decode(opt, packed, input_num=vals.size)
    with vd.ViterbiCUDA(opt) as d:
        out, _ = d.run_llr(vals, scale=40000.0)
    assert np.array_equal(out, ref)


@pytest.mark.gpu
def test_fused_llr_device_path_matches_host_path(gpu, vd):
    import torch
    opt = SOFT8 | M_B16
    vals = channel_values(2 * 100_000, 1.0, 9)
    with vd.ViterbiCUDA(opt) as d:
        host, _ = d.run_llr(vals)
        v = torch.from_numpy(vals).cuda()
        out = torch.zeros(d.getOutputSize(vals.size) // 4, dtype=torch.int32, device="cuda")
        d.run_device_llr(v.data_ptr(), out.data_ptr(), vals.size, stream=torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy().view(np.uint32), host)


@pytest.mark.gpu
@pytest.mark.parametrize("opt", [HARD | M_B32, SOFT8 | M_B16, SOFT16 | M_B32, FP32 | M_FP16, SOFT4 | M_B16 | O_B16],
                         ids=name)
def test_fused_llr_batch_equals_single(gpu, vd, vo, opt):
    """vd_run_device_llr_batch: 3 independent float batches in one launch, each equal to the oracle of its
    own packed words; the bytes between the batches' outputs stay untouched"""
    import torch
    n, nb = 2 * 150_000, 3
    vals = [channel_values(n, 0.5 + b, 21 + b) for b in range(nb)]
    refs = [vo.decode(opt, vo.pack(opt, v, 40000.0), input_num=n)[0] for v in vals]
    istride = (n * 4 + 255) // 256 * 256
    nout = vd.lib().vd_output_size(opt, n)
    ostride = (nout + 255) // 256 * 256 + 256
    inp = torch.zeros(nb * istride // 4, dtype=torch.float32, device="cuda")
    for b in range(nb):
        inp[b * istride // 4: b * istride // 4 + n] = torch.from_numpy(vals[b]).cuda()
    out = torch.full((nb * ostride,), 0xA5, dtype=torch.uint8, device="cuda")
    with vd.ViterbiCUDA(opt) as d:
        d.run_device_llr_batch(inp.data_ptr(), istride, out.data_ptr(), ostride, n, nb, 40000.0,
                               torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
    for b in range(nb):
        got = out[b * ostride: b * ostride + nout].cpu().numpy().view(refs[b].dtype)
        np.testing.assert_array_equal(got, refs[b])
        assert bool((out[b * ostride + nout: (b + 1) * ostride] == 0xA5).all())


@pytest.mark.gpu
@pytest.mark.parametrize("opt", [HARD | M_B32, SOFT4 | M_B16, FP32 | M_FP16, HARD | M_B16 | O_B16, SOFT8 | M_B16,
                                 SOFT8 | M_B32 | O_B16], ids=name)
def test_fused_llr_split_launch_on_packed_kernel(gpu, vd, vo, opt):
    """16M bits of float channel values in one fused launch: 78 words per chunk, so HARD / SOFT4 / SOFT8 / FP32
    run vd_decode_pk's split launch (tail workgroups included) with the packer fused into the table build
    (SOFT8 with M_B32's tie-tag complement and 16-bit output words too); equal to the oracle's pack + decode and
    to the unfused vd_decode_tg path (VD_NO_PK=1)"""
    import os
    vals = channel_values_fast(2 * 16_000_000, 1.0, 13)
    packed = vo.pack(opt, vals, 40000.0)
    ref, ok = vo.decode(opt, packed, input_num=vals.size, nthreads=16)
    assert ok
    with vd.ViterbiCUDA(opt) as d:
        out, _ = d.run_llr(vals, scale=40000.0)
    os.environ["VD_NO_PK"] = "1"
    try:
        with vd.ViterbiCUDA(opt) as d:
            tg, _ = d.run_llr(vals, scale=40000.0)
    finally:
        del os.environ["VD_NO_PK"]
    bad = np.flatnonzero(out != ref)
    assert bad.size == 0, f"{bad.size} words differ, first at {bad[:5]}"
    assert np.array_equal(tg, ref)


@pytest.mark.gpu
@pytest.mark.parametrize("opt", [SOFT8 | M_B16, SOFT8 | M_B32 | O_B16, HARD | M_B32], ids=name)
def test_fused_llr_split_random_floats_redecode(gpu, vd, vo, opt):
    """Float channel values that carry no codeword (standard normal noise, scaled so the quantiser spans its
    range): the split launch's speculative starts often do not converge, so the fused float-input kernel's
    re-decodes and early stops run (vd_split_redecodes grows), the words still equal the oracle's pack +
    decode, and no wave reaches the pass cap"""
    vals = (np.random.default_rng(17).standard_normal(2 * 16_000_000) * 2e-3).astype(np.float32)
    packed = vo.pack(opt, vals, 40000.0)
    ref, ok = vo.decode(opt, packed, input_num=vals.size, nthreads=16)
    before, caps = vd.split_redecodes(), vd.split_cap_exits()
    with vd.ViterbiCUDA(opt) as d:
        assert "split" in d.kernel_for(vals.size, 1, True)
        out, _ = d.run_llr(vals, scale=40000.0)
    redec = vd.split_redecodes() - before
    bad = np.flatnonzero(out != ref)
    assert bad.size == 0, f"{bad.size} words differ (re-decoded {redec}), first at {bad[:5]}"
    assert redec > 0, redec
    assert vd.split_cap_exits() == caps == 0
