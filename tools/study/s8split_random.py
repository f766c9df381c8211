"""SOFT8 single-batch launch on uniformly random channel bytes and on zeros: vd_decode_tg segments
(VD_PK_SPLIT=0) against the packed split kernel (default), timing + re-decode counts + word equality (tools only)."""
import os
import sys
import torch
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "gpu-accelerated-viterbi-decoder_amd"))
import vitdec

n = 64_000_000  # 32M message bits, SOFT8 values
res = {}
outs = {}
for kind in ("random", "zeros"):
    for mode in ("0", "1"):
        os.environ["VD_PK_SPLIT"] = mode
        opt = vitdec.SOFT8 | vitdec.M_B16
        dec = vitdec.ViterbiCUDA(opt, n)
        nin = vitdec.lib().vd_input_size(opt, n)
        nout = vitdec.lib().vd_output_size(opt, n)
        g = torch.Generator(device="cpu").manual_seed(3)
        inp = (torch.randint(0, 256, (nin,), dtype=torch.uint8, generator=g) if kind == "random"
               else torch.zeros(nin, dtype=torch.uint8)).to("cuda")
        out = torch.empty(nout, dtype=torch.uint8, device="cuda")
        for _ in range(2):
            dec.run_device(inp.data_ptr(), out.data_ptr(), n)
        torch.cuda.synchronize()
        r0 = vitdec.split_redecodes(0)
        e = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        e[0].record()
        for _ in range(10):
            dec.run_device(inp.data_ptr(), out.data_ptr(), n)
        e[1].record()
        torch.cuda.synchronize()
        ms = e[0].elapsed_time(e[1]) / 10
        outs[(kind, mode)] = out.clone()
        res[(kind, mode)] = (round(ms, 4), (vitdec.split_redecodes(0) - r0) / 10, dec.kernel_for(n))
        print(kind, "VD_PK_SPLIT=" + mode, res[(kind, mode)], flush=True)
    print(kind, "equal words:", bool(torch.equal(outs[(kind, "0")], outs[(kind, "1")])), flush=True)
