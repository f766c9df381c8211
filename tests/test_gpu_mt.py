"""GPU parity of the reference-exact channel source (vd_channel_device / vd_simulate_device): the
harness chain RandBitGen | ConvolutionalEncoder(7, 0171, 0133) | AddNoise | SoftDecisionPacker
(src/viterbiDF.h:20-167, seeds as src/main.cpp:131-137) generated on the GPU must equal, bit for bit,
the oracle restatement (oracle/vd_oracle.c vo_channel, with the host glibc logf) and the product's host
harness (vd_simulate_host: libstdc++'s own std::mt19937 / normal_distribution<float>).  Through the GPU
decode it reproduces the reference's known-answer BEN values."""
import numpy as np
import pytest

from vitdec import FP32, HARD, M_B16, M_B32, M_FP16, SOFT4, SOFT8, SOFT16
from test_gpu_parity import KAT, KAT_COLS, gpu_decode


def gpu_channel(n, snr, bs, ns):
    import torch
    import vitdec
    bits = torch.zeros(max(n, 1), dtype=torch.uint8, device="cuda")
    vals = torch.zeros(max(2 * n, 4), dtype=torch.float32, device="cuda")
    vitdec.channel_device(n, snr, bs, ns, bits.data_ptr(), vals.data_ptr(),
                          stream=torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    return bits.cpu().numpy()[:n], vals.cpu().numpy()[:2 * n]


def gpu_simulate(opt, n, snr, bs, ns):
    import torch
    import vitdec
    nbytes = vitdec.lib().vd_input_size(opt, 2 * n)
    bits = torch.zeros(n, dtype=torch.uint8, device="cuda")
    packed = torch.zeros((nbytes + 3) // 4 * 4, dtype=torch.uint8, device="cuda")
    vitdec.simulate_device(opt, n, snr, bs, ns, bits.data_ptr(), packed.data_ptr(),
                           stream=torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    return bits.cpu().numpy(), packed.cpu().numpy()[:nbytes]


@pytest.mark.gpu
@pytest.mark.parametrize("n", [1, 16, 1008, 65536 + 16, 1_000_000])
@pytest.mark.parametrize("snr", [0.0, 1.2, 15.0])
def test_channel_matches_oracle(gpu, vo, n, snr):
    bits, vals = gpu_channel(n, snr, 11 + n, 22 + n)
    rb, rv = vo.channel(n, snr, 11 + n, 22 + n)
    np.testing.assert_array_equal(bits, rb)
    bad = np.flatnonzero(vals.view(np.uint32) != rv.view(np.uint32))
    assert bad.size == 0, f"{bad.size} values differ, first {bad[:5]}: {vals[bad[:5]]} vs {rv[bad[:5]]}"


@pytest.mark.gpu
def test_channel_noiseless(gpu, vo):
    # AddNoise's stddev = +inf branch (viterbiDF.h:79-85): snr = -inf gives pow(10, inf) = inf
    bits, vals = gpu_channel(5000, float("-inf"), 3, 4)
    rb, rv = vo.channel(5000, 0.0, 3, 4, noiseless=True)
    np.testing.assert_array_equal(bits, rb)
    np.testing.assert_array_equal(vals, rv)


@pytest.mark.gpu
@pytest.mark.parametrize("opt", [HARD | M_B32, SOFT4 | M_B16, SOFT8 | M_B16, SOFT16 | M_B32, FP32 | M_FP16])
@pytest.mark.parametrize("snr", [0.0, 1.2])
def test_simulate_matches_host_harness(gpu, opt, snr):
    n = 200_016
    bits, packed = gpu_simulate(opt, n, snr, 5, 6)
    hb, hp = gpu.simulate_host(opt, n, snr, 5, 6)  # libstdc++ generators, the reference's own
    np.testing.assert_array_equal(bits, hb)
    np.testing.assert_array_equal(packed, hp.view(np.uint8))


@pytest.mark.gpu
@pytest.mark.parametrize("snr,col,ben", KAT, ids=[f"{s}-{c}" for s, c, _ in KAT])
def test_known_answer_ben_from_gpu_source(gpu, snr, col, ben):
    opt = KAT_COLS[col]
    bits, packed = gpu_simulate(opt, 1_000_000, snr, 11, 22)
    dt = np.float32 if (opt & 0xF) == FP32 else np.int32
    out = gpu_decode(gpu, opt, packed.view(dt))
    assert gpu.count_errors(opt, bits, out) == ben


@pytest.mark.gpu
def test_full_size_soft8_matches_host_harness(gpu):
    n = 32_000_000
    bits, packed = gpu_simulate(SOFT8 | M_B16, n, 1.0, 1, 2)
    hb, hp = gpu.simulate_host(SOFT8 | M_B16, n, 1.0, 1, 2)
    assert np.array_equal(bits, hb)
    assert np.array_equal(packed, hp.view(np.uint8))
