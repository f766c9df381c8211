"""Out-of-bounds stores of the shipped kernels, checked at run time (an LDS ring store one
slot below the wave's ring shipped for two rounds under green parity tests).

LDS: with the guard check on (vd_set_guard_check), every wave writes guard words before its branch-
metric table, between table and survivor ring and after the ring, and counts at kernel exit the guard
words it finds overwritten (vd_kernel_tg.h TgLds).  Global memory: every output buffer sits between
guard bytes that must come back untouched.  Every one of the 24 distinct kernels runs split (16M bits:
>= 64 words per chunk), batched and fused-LLR launches with both checks, and decodes oracle-exact.

The check is shown to catch the round-2 bug: tools/scc_scratch.sh builds a scratch copy of the library
whose renormalisation asm again omits its "scc" clobber (the compiler then branches on the subtraction's
borrow, tests/test_asm_lint.py); run through the same check, that library reports overwritten guards."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

from vitdec import FP32, HARD, M_B16, M_B32, M_FP16, O_B16, SOFT4, SOFT8, SOFT16
from test_gpu_parity import VALID, name
from test_gpu_split import gpu_sim

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SCRATCH_LIB = os.path.join(ROOT, "tools", "build", "scc_scratch", "lib", "libvitdec.so")
GUARD = 4096  # guard bytes before and after every output buffer
PAT = 0x5C


def guarded(nbytes):
    """(buffer, view of the nbytes between the guards)"""
    buf = torch.full((GUARD + nbytes + GUARD,), PAT, dtype=torch.uint8, device="cuda")
    return buf, buf[GUARD:GUARD + nbytes]


def guards_intact(buf):
    return bool((buf[:GUARD] == PAT).all()) and bool((buf[-GUARD:] == PAT).all())


def _decode_checked(gpu, opt, packed_np, n):
    """split / whole launch of one batch from device memory with both checks; returns the words"""
    nout = gpu.lib().vd_output_size(opt, n)
    inp = torch.from_numpy(packed_np.view(np.uint8).copy()).cuda()
    buf, out = guarded(nout)
    with gpu.ViterbiCUDA(opt) as dec:
        dec.set_guard_check(True)
        dec.run_device(inp.data_ptr(), out.data_ptr(), n, torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        bad = dec.guard_violations()
    assert bad == 0, f"{bad} LDS guard words overwritten"
    assert guards_intact(buf), "bytes around the output buffer were written"
    return out.cpu().numpy().view(np.uint16 if opt & O_B16 else np.uint32)


@pytest.mark.gpu
@pytest.mark.parametrize("opt", VALID, ids=name)
def test_guards_split_launch_every_kernel(gpu, vo, opt):
    n_bits = 16_000_000  # split launch (78 words per chunk); SNR 0.5: some pieces re-decode
    bits, packed = gpu_sim(gpu, opt, n_bits, 0.5)
    out = _decode_checked(gpu, opt, packed, 2 * n_bits)
    ref, ok = vo.decode(opt, packed, nthreads=16)
    assert ok
    bad = np.flatnonzero(out != ref)
    assert bad.size == 0, f"{bad.size} words differ, first at {bad[:5]}"


@pytest.mark.gpu
@pytest.mark.parametrize("opt", VALID, ids=name)
def test_guards_ragged_and_batched(gpu, vo, opt):
    # 206,400 bits: ragged partition (most chunks 1 word); 3 batches in one launch, outputs packed
    # between guard gaps
    n_bits, nb = 206_400, 3
    n = 2 * n_bits
    nin = gpu.lib().vd_input_size(opt, n)
    istride = (nin + 255) // 256 * 256
    nout = gpu.lib().vd_output_size(opt, n)
    ostride = (nout + 255) // 256 * 256 + 256
    refs, inps = [], torch.zeros(nb * istride, dtype=torch.uint8, device="cuda")
    for b in range(nb):
        _, packed = vo.simulate(opt, n_bits, 0.4 + b, 31 + b, 41 + b)
        refs.append(vo.decode(opt, packed)[0])
        inps[b * istride: b * istride + nin] = torch.from_numpy(packed.view(np.uint8)[:nin].copy()).cuda()
    buf, outs = guarded(nb * ostride)
    with gpu.ViterbiCUDA(opt) as dec:
        dec.set_guard_check(True)
        dec.run_device_batch(inps.data_ptr(), istride, outs.data_ptr(), ostride, n, nb,
                             torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        assert dec.guard_violations() == 0
    assert guards_intact(buf)
    for b in range(nb):
        got = outs[b * ostride: b * ostride + nout].cpu().numpy().view(refs[b].dtype)
        np.testing.assert_array_equal(got, refs[b])
        assert bool((outs[b * ostride + nout: (b + 1) * ostride] == PAT).all()), "gap between batches written"


@pytest.mark.gpu
@pytest.mark.parametrize("opt", [HARD | M_B32, SOFT4 | M_B16, SOFT8 | M_B16, SOFT16 | M_B32, FP32 | M_FP16,
                                 SOFT8 | M_B32 | O_B16], ids=name)
def test_guards_fused_llr(gpu, vo, opt):
    from test_gpu_llr import channel_values
    n = 2 * 300_000
    vals = channel_values(n, 1.0, 17)
    packed = vo.pack(opt, vals, 40000.0)
    ref, _ = vo.decode(opt, packed, input_num=n)
    v = torch.from_numpy(vals).cuda()
    buf, out = guarded(gpu.lib().vd_output_size(opt, n))
    with gpu.ViterbiCUDA(opt) as dec:
        dec.set_guard_check(True)
        dec.run_device_llr(v.data_ptr(), out.data_ptr(), n, 40000.0, torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        assert dec.guard_violations() == 0
    assert guards_intact(buf)
    np.testing.assert_array_equal(out.cpu().numpy().view(ref.dtype), ref)


_SCRATCH = r"""
import json, os, sys
import numpy as np
import torch
sys.path.insert(0, os.path.join(os.environ["VD_ROOT"], "gpu-accelerated-viterbi-decoder_amd"))
sys.path.insert(0, os.path.join(os.environ["VD_ROOT"], "oracle"))
import vitdec, vd_oracle
assert vitdec.LIB_PATH == os.environ["VITDEC_LIB"]
res = {}
for opt in (vitdec.FP32 | vitdec.M_FP16, vitdec.HARD | vitdec.M_B32, vitdec.SOFT8 | vitdec.M_B16):
    bits, packed = vd_oracle.simulate(opt, 1_000_000, 1.0, 3, 4)
    ref, _ = vd_oracle.decode(opt, packed)
    inp = torch.from_numpy(packed.view(np.uint8).copy()).cuda()
    n = 2_000_000
    out = torch.zeros(vitdec.lib().vd_output_size(opt, n), dtype=torch.uint8, device="cuda")
    with vitdec.ViterbiCUDA(opt) as d:
        d.set_guard_check(True)
        d.run_device(inp.data_ptr(), out.data_ptr(), n, torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        res[hex(opt)] = {"guard_violations": d.guard_violations(),
                         "words_differ": int((out.cpu().numpy().view(ref.dtype) != ref).sum())}
print(json.dumps(res))
"""


def scratch_state():
    """(usable, why): the scratch library exists and its BUILD_RECORD (tools/scc_scratch.sh) matches this tree's
    product sources -- a stale build is never loaded"""
    import vitdec
    rec = os.path.join(os.path.dirname(SCRATCH_LIB), "BUILD_RECORD")
    if not os.path.exists(SCRATCH_LIB) or not os.path.exists(rec):
        return False, f"{SCRATCH_LIB} not built (tools/scc_scratch.sh; __graft_entry__.build() runs it)"
    stale = vitdec.build_mismatch(open(rec).read().strip())
    if stale:
        return False, f"{SCRATCH_LIB} is stale ({stale}): rebuild it with tools/scc_scratch.sh"
    return True, ""


@pytest.mark.gpu
def test_guard_check_catches_the_round2_scc_clobber(gpu):
    """The scratch library (renormalisation asm without "scc" clobber) through the guard check: the check
    reports overwritten LDS guards, i.e. test_guards_* would fail on that build.  The scratch copy is made
    from this tree's sources (its build record must match them, or the test skips without loading it), and
    its decodes run on vd_decode_tg (VD_NO_PK=1), the kernel whose asm the copy breaks."""
    ok, why = scratch_state()
    if not ok:
        pytest.skip(why)
    ev = os.path.join(os.path.dirname(SCRATCH_LIB), "SCC_EVIDENCE")
    if not os.path.exists(ev):
        pytest.skip(f"{ev} missing: rebuild the scratch library with tools/scc_scratch.sh")
    if int(open(ev).read().strip() or 0) == 0:
        pytest.skip("this compiler keeps no SCC reader after the scratch copy's renormalisation "
                    "(tests/test_asm_lint.py scan of its ISA): the round-2 bug cannot show at run time")
    env = dict(os.environ, VD_ROOT=ROOT, VITDEC_LIB=SCRATCH_LIB, VD_NO_PK="1")
    r = subprocess.run([sys.executable, "-c", _SCRATCH], capture_output=True, text=True, timeout=180, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    res = json.loads(r.stdout.strip().splitlines()[-1])
    print(res)
    # the scratch ISA branches on the subtraction's borrow (SCC_EVIDENCE > 0, the scan of tests/test_asm_lint.py
    # at build time); the guard check must then see the consequence (rounds 4-5: it did).  No violation is a
    # failure.
    assert any(v["guard_violations"] > 0 for v in res.values()), f"the guard check caught nothing: {res}"
