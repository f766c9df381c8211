"""tools only: zero-copy decode (kernel reads packed input from / writes decoded words to pinned host
memory over PCIe) vs the copy pipeline, HARD and SOFT8, 6 batches each."""
import os, sys, time, ctypes
import numpy as np
import torch
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gpu-accelerated-viterbi-decoder_amd"))
import vitdec
n = 64_000_000
nb = 6
for opt in (vitdec.HARD | vitdec.M_B32, vitdec.SOFT8 | vitdec.M_B16):
    nin = vitdec.lib().vd_input_size(opt, n) // 4
    nout = vitdec.lib().vd_output_size(opt, n) // 4
    pins = [vitdec.PinnedArray((nin,), np.int32) for _ in range(nb)]
    outs = [vitdec.PinnedArray((nout,), np.uint32) for _ in range(nb)]
    rng = np.random.default_rng(1)
    for p in pins:
        p.array[:] = rng.integers(-2**31, 2**31 - 1, nin, dtype=np.int64).astype(np.int32)
    dec = vitdec.ViterbiCUDA(opt, n)
    s = torch.cuda.current_stream()
    dec.run_device(pins[0].array.ctypes.data, outs[0].array.ctypes.data, n, s.cuda_stream)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for b in range(nb):
        dec.run_device(pins[b].array.ctypes.data, outs[b].array.ctypes.data, n, s.cuda_stream)
    torch.cuda.synchronize()
    zc = (time.perf_counter() - t0) * 1e3
    ref = [dec.run(p.array)[0] for p in pins]
    ok = all(np.array_equal(o.array, r) for o, r in zip(outs, ref))
    res, ms = dec.run_stream([p.array for p in pins], n)
    print(f"opt 0x{opt:x}: zero-copy {zc:.3f} ms ({zc/nb:.3f}/batch, match={ok}); copy pipeline {ms:.3f} ms ({ms/nb:.3f}/batch)")
    dec.close()
