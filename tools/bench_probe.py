"""Timing probe (tools, not the product): bench.py's step with torch-allocated inputs, zero-filled vs the
harness chain's data (vd_simulate_device), to find why bench.py's kernels run slower than tools/vd_capiab."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "gpu-accelerated-viterbi-decoder_amd"))
import torch  # noqa: E402
import vitdec  # noqa: E402

N = 32_000_000
K = 10
dev = 0
torch.cuda.set_device(dev)
stream = torch.cuda.current_stream()
sptr = stream.cuda_stream
W = [("hard_b32", 0x00), ("soft8_b16", 0x12)]


def make(fill, seed):
    bs = []
    for wi, (name, opt) in enumerate(W):
        n = 2 * N
        inp = torch.zeros(vitdec.lib().vd_input_size(opt, n), dtype=torch.uint8, device=dev)
        out = torch.empty(vitdec.lib().vd_output_size(opt, n), dtype=torch.uint8, device=dev)
        if fill == "harness":
            bits = torch.empty(N, dtype=torch.uint8, device=dev)
            vitdec.simulate_device(opt, N, float(sys.argv[1]) if len(sys.argv) > 1 else 2.0, 1 + 2 * wi + seed, 2 + 2 * wi + seed,
                                   bits.data_ptr(), inp.data_ptr(), sptr)
        elif fill == "random":
            inp.random_(0, 256)
        bs.append(dict(name=name, opt=opt, inp=inp, out=out, dec=vitdec.ViterbiCUDA(opt, 0, dev), n=n))
    torch.cuda.synchronize()
    return bs


def timed(bs):
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    res = []
    for rep in range(4):
        ev[0].record(stream)
        for i, b in enumerate(bs):
            for _ in range(K):
                b["dec"].run_device(b["inp"].data_ptr(), b["out"].data_ptr(), b["n"], sptr)
            ev[i + 1].record(stream)
        torch.cuda.synchronize()
        if rep:
            res.append((ev[0].elapsed_time(ev[1]) / K, ev[1].elapsed_time(ev[2]) / K))
    res.sort()
    return res[len(res) // 2]


sets = {f: make(f, 0) for f in ("zeros", "harness", "random")}
for rnd in range(2):
    for f, bs in sets.items():
        h, s = timed(bs)
        print(f"{f:8s} hard {h:.4f} ms  soft8 {s:.4f} ms", flush=True)
