"""Split launches and device pointers under concurrent streams.

A split launch's piece-boundary vectors live in the workgroup's LDS (vd_kernel_tg.h "split chunks"), so
launches on any number of streams share no device scratch.  Here 100 asynchronous 16M-bit split launches
go to three streams, one of them held back behind an event until the other two have run ahead; every
output equals the oracle.  A launch on a stream of another device than the decoder's is refused."""
import numpy as np
import pytest
import torch

from vitdec import HARD, M_B16, M_B32, SOFT8, VitdecError
from test_gpu_split import gpu_sim


@pytest.mark.gpu
@pytest.mark.parametrize("opt", [HARD | M_B32, SOFT8 | M_B16], ids=["h-b32", "s8-b16"])
def test_split_launches_on_three_streams_one_held_back(gpu, vo, opt):
    n_bits, n_in, n_launch = 16_000_000, 4, 100
    n = 2 * n_bits
    nout = gpu.lib().vd_output_size(opt, n)
    inputs, refs = [], []
    for k in range(n_in):
        _, packed = gpu_sim(gpu, opt, n_bits, 0.0 + 0.5 * k)  # SNR 0: pieces re-decode, several passes
        ref, ok = vo.decode(opt, packed, nthreads=16)
        assert ok
        inputs.append(torch.from_numpy(packed.view(np.uint8).copy()).cuda())
        refs.append(ref)
    outs = [torch.zeros(nout, dtype=torch.uint8, device="cuda") for _ in range(n_launch)]
    streams = [torch.cuda.Stream() for _ in range(3)]
    gate_stream = torch.cuda.Stream()
    gate = torch.cuda.Event()
    torch.cuda.synchronize()
    before = gpu.split_redecodes()
    with gpu.ViterbiCUDA(opt) as dec:
        with torch.cuda.stream(gate_stream):
            torch.cuda._sleep(200_000_000)  # ~0.1 s: streams 0 and 2 run far ahead of stream 1
            gate.record(gate_stream)
        streams[1].wait_event(gate)
        for i in range(n_launch):
            s = streams[i % 3]
            dec.run_device(inputs[i % n_in].data_ptr(), outs[i].data_ptr(), n, s.cuda_stream)
        torch.cuda.synchronize()
    assert gpu.split_redecodes() > before  # the boundary checks failed somewhere and re-decodes ran
    for i in range(n_launch):
        got = outs[i].cpu().numpy().view(refs[0].dtype)
        bad = np.flatnonzero(got != refs[i % n_in])
        assert bad.size == 0, f"launch {i} (stream {i % 3}): {bad.size} words differ, first {bad[:5]}"


@pytest.mark.gpu
def test_null_stream_on_the_decoders_device(gpu, vo):
    # the null stream means the calling thread's current device, which must be the decoder's
    opt = HARD | M_B32
    bits, packed = vo.simulate(opt, 200_000, 1.0, 5, 6)
    ref, _ = vo.decode(opt, packed)
    inp = torch.from_numpy(packed.view(np.uint8).copy()).cuda()
    out = torch.zeros(ref.nbytes, dtype=torch.uint8, device="cuda")
    with gpu.ViterbiCUDA(opt, device=0) as dec:
        dec.run_device(inp.data_ptr(), out.data_ptr(), 400_000, 0)
        torch.cuda.synchronize()
    np.testing.assert_array_equal(out.cpu().numpy().view(ref.dtype), ref)


@pytest.mark.gpu
def test_stream_of_another_device_is_refused(gpu):
    if torch.cuda.device_count() < 2:
        pytest.skip("one GPU visible: no stream of another device to pass")
    with torch.cuda.device(1):
        s1 = torch.cuda.Stream()
    with gpu.ViterbiCUDA(HARD | M_B32, device=0) as dec:
        with pytest.raises(VitdecError, match="device"):
            dec.run_device(1 << 20, 1 << 20, 400_000, s1.cuda_stream)
