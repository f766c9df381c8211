"""tools only: run the streaming host pipeline once for profiling (rocprofv3 --kernel-trace --memory-copy-trace)."""
import os, sys
import numpy as np
import torch  # noqa: F401  (same HIP runtime as bench.py)
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gpu-accelerated-viterbi-decoder_amd"))
import vitdec
opt = vitdec.HARD | vitdec.M_B32
n = 64_000_000
nb = int(sys.argv[1]) if len(sys.argv) > 1 else 6
pins = [vitdec.PinnedArray((vitdec.lib().vd_input_size(opt, n) // 4,), np.int32) for _ in range(nb)]
for p in pins:
    p.array[:] = np.random.default_rng(1).integers(-2**31, 2**31 - 1, p.array.size, dtype=np.int64).astype(np.int32)
dec = vitdec.ViterbiCUDA(opt, n)
dec.run_stream([pins[0].array], n)
outs, ms = dec.run_stream([p.array for p in pins], n)
print("wall ms", ms, "per batch", ms / nb)
