"""vd_run_device_batch: several independent batches in one launch ("batched launches").
Each batch must decode exactly as a vd_run_device of that batch alone (the reference's 6400-chunk
partition per batch) and as the oracle; the input stride may be 0 (the same input for every batch);
bad arguments fail with VD_ERR_ARG before anything is launched."""
import numpy as np
import pytest
import torch

from vitdec import FP32, HARD, M_B16, M_B32, M_FP16, O_B16, SOFT4, SOFT8, SOFT16, VitdecError
from test_gpu_parity import name


def _inputs(gpu, opt, nbits, nb):
    """nb independent batches (seeds 51+2b, 52+2b) synthesised on the GPU into one contiguous tensor"""
    n = 2 * nbits
    nin = gpu.lib().vd_input_size(opt, n)
    stride = (nin + 255) // 256 * 256
    packed = torch.zeros(nb * stride, dtype=torch.uint8, device="cuda")
    bits = torch.empty(nbits, dtype=torch.uint8, device="cuda")
    for b in range(nb):
        gpu.simulate_device(opt, nbits, 1.0, 51 + 2 * b, 52 + 2 * b, bits.data_ptr(), packed.data_ptr() + b * stride)
    torch.cuda.synchronize()
    return packed, stride, nin


def _single(dec, packed_ptr, n, nout):
    out = torch.zeros(nout, dtype=torch.uint8, device="cuda")
    dec.run_device(packed_ptr, out.data_ptr(), n)
    torch.cuda.synchronize()
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("opt", [HARD | M_B32, SOFT8 | M_B16, FP32 | M_FP16, SOFT16 | M_B32, SOFT4 | M_B16 | O_B16,
                                 HARD | M_B32 | O_B16], ids=name)
@pytest.mark.parametrize("nbits", [16_000_000, 1_000_000, 150_000])
def test_batch_equals_single_runs(gpu, vo, opt, nbits):
    nb = 3
    n = 2 * nbits
    packed, stride, nin = _inputs(gpu, opt, nbits, nb)
    nout = gpu.lib().vd_output_size(opt, n)
    ostride = (nout + 255) // 256 * 256
    out = torch.full((nb * ostride,), 0xA5, dtype=torch.uint8, device="cuda")
    with gpu.ViterbiCUDA(opt) as dec:
        dec.run_device_batch(packed.data_ptr(), stride, out.data_ptr(), ostride, n, nb)
        torch.cuda.synchronize()
        for b in range(nb):
            single = _single(dec, packed.data_ptr() + b * stride, n, nout)
            got = out[b * ostride: b * ostride + nout]
            assert torch.equal(got, single), f"batch {b} differs from its single run"
            # bytes between the batches' outputs are untouched
            assert bool((out[b * ostride + nout: (b + 1) * ostride] == 0xA5).all())
    # the oracle on the last batch
    dt = np.float32 if (opt & 0xF) == FP32 else np.int32
    p = packed[(nb - 1) * stride: (nb - 1) * stride + nin].cpu().numpy().view(dt)
    ref, ok = vo.decode(opt, p, input_num=n, nthreads=16)
    assert ok
    got = out[(nb - 1) * ostride: (nb - 1) * ostride + nout].cpu().numpy().view(ref.dtype)
    np.testing.assert_array_equal(got, ref)


@pytest.mark.gpu
def test_batch_with_input_stride_zero(gpu):
    # API edge case: input stride 0, every batch decodes the same input into its own output (the bench
    # decodes distinct resident batches at a 256-byte-aligned stride instead)
    opt, nbits, nb = SOFT8 | M_B16, 32_000_000, 5
    n = 2 * nbits
    packed, stride, nin = _inputs(gpu, opt, nbits, 1)
    nout = gpu.lib().vd_output_size(opt, n)
    out = torch.zeros(nb * nout, dtype=torch.uint8, device="cuda")
    with gpu.ViterbiCUDA(opt) as dec:
        dec.run_device_batch(packed.data_ptr(), 0, out.data_ptr(), nout, n, nb)
        single = _single(dec, packed.data_ptr(), n, nout)
    for b in range(nb):
        assert torch.equal(out[b * nout:(b + 1) * nout], single)


@pytest.mark.gpu
def test_batch_argument_errors(gpu):
    opt, n = HARD | M_B32, 2_000_000
    nout = gpu.lib().vd_output_size(opt, n)
    buf = torch.zeros(4 * nout + 64, dtype=torch.uint8, device="cuda")
    p = buf.data_ptr()
    with gpu.ViterbiCUDA(opt) as dec:
        for args in [(p, 0, p, nout, n, 0),          # nbatch < 1
                     (p, 0, p, nout - 4, n, 2),      # overlapping outputs
                     (p, 2, p, nout, n, 2),          # stride not a multiple of 4
                     (p, 0, p, nout, 100, 2)]:       # inputNum too small
            with pytest.raises(VitdecError):
                dec.run_device_batch(*args)
        dec.run_device_batch(p, 0, p, 0, n, 1)  # nbatch 1: any output stride
        torch.cuda.synchronize()
