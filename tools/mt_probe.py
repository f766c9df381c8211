"""Timing probe (tools, not the product): GPU reference-exact channel source vs the host harness."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "gpu-accelerated-viterbi-decoder_amd"))
import vitdec  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 32_000_000
opt = vitdec.SOFT8 | vitdec.M_B16
s = torch.cuda.current_stream().cuda_stream
bits = torch.zeros(N, dtype=torch.uint8, device="cuda")
vals = torch.zeros(2 * N, dtype=torch.float32, device="cuda")
packed = torch.zeros(vitdec.lib().vd_input_size(opt, 2 * N), dtype=torch.uint8, device="cuda")
t = time.perf_counter()
vitdec.channel_device(N, 1.0, 1, 2, bits.data_ptr(), vals.data_ptr(), s)
print(f"first call (includes the jump polynomials, once per process): {time.perf_counter() - t:.3f} s", flush=True)
for name, fn in [("channel_device", lambda: vitdec.channel_device(N, 1.0, 1, 2, bits.data_ptr(), vals.data_ptr(), s)),
                 ("simulate_device", lambda: vitdec.simulate_device(opt, N, 1.0, 1, 2, bits.data_ptr(), packed.data_ptr(), s))]:
    ts = []
    for _ in range(6):
        torch.cuda.synchronize()
        t = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t)
    ts.sort()
    print(f"{name:16s} N={N}: median {ts[len(ts) // 2] * 1e3:.2f} ms  min {ts[0] * 1e3:.2f} ms "
          f"-> {N / ts[len(ts) // 2] / 1e9:.2f} Gbit/s", flush=True)
t = time.perf_counter()
hb, hp = vitdec.simulate_host(opt, N, 1.0, 1, 2)
th = time.perf_counter() - t
print(f"simulate_host    N={N}: {th * 1e3:.1f} ms (1 thread, libstdc++)  -> {N / th / 1e6:.2f} Mbit/s", flush=True)
print("host == device:", bool((packed.cpu().numpy() == hp.view("uint8")).all()), bool((bits.cpu().numpy() == hb).all()))
