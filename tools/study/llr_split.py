"""Fused float-input SOFT8 single-batch launch (vd_run_device_llr on the harness's codeword + AWGN at 2 dB, or
with argument "random" on random +-1 symbols plus 0.5 N(0,1) noise, not a codeword; scale 40000): vd_decode_tg segments (VD_PK_SPLIT=0) against the packed split kernel, timing and re-decode
counts, and the same packed words decoded without the fusion (tools only)."""
import os
import sys
import torch
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "gpu-accelerated-viterbi-decoder_amd"))
import vitdec

n = 64_000_000
opt = vitdec.SOFT8 | vitdec.M_B16
kind = sys.argv[1] if len(sys.argv) > 1 else "codeword"
if kind == "codeword":  # the harness's AddNoise output at 2 dB
    vals = torch.empty(n, dtype=torch.float32, device="cuda")
    src = torch.empty(n // 2, dtype=torch.uint8, device="cuda")
    vitdec.channel_device(n // 2, 2.0, 901, 902, src.data_ptr(), vals.data_ptr())
else:  # random +-1 symbols plus noise: not a codeword
    g = torch.Generator(device="cuda")
    g.manual_seed(5)
    vals = (torch.randint(0, 2, (n,), device="cuda", generator=g).float() * 2 - 1 + 0.5 * torch.randn(n, device="cuda", generator=g))
packed = torch.empty(vitdec.lib().vd_input_size(opt, n), dtype=torch.uint8, device="cuda")
vitdec.pack_device(opt, vals.data_ptr(), n, packed.data_ptr(), 40000.0)
outs = {}
for mode in ("0", "1"):
    os.environ["VD_PK_SPLIT"] = mode
    dec = vitdec.ViterbiCUDA(opt, n)
    out = torch.empty(vitdec.lib().vd_output_size(opt, n), dtype=torch.uint8, device="cuda")
    for name, fn in (("fused", lambda: dec.run_device_llr(vals.data_ptr(), out.data_ptr(), n, 40000.0)),
                     ("packed", lambda: dec.run_device(packed.data_ptr(), out.data_ptr(), n))):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        r0 = vitdec.split_redecodes(0)
        e = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        e[0].record()
        for _ in range(10):
            fn()
        e[1].record()
        torch.cuda.synchronize()
        outs[(mode, name)] = out.clone()
        print("VD_PK_SPLIT=" + mode, name, round(e[0].elapsed_time(e[1]) / 10, 4), "ms, re-decodes per launch",
              (vitdec.split_redecodes(0) - r0) / 10, dec.kernel_for(n, 1, name == "fused"), flush=True)
    dec.close()
print("equal:", all(torch.equal(outs[("0", "fused")], v) for v in outs.values()))
