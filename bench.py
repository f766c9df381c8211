#!/usr/bin/env python3
"""Benchmark: decoded Gb/s at K=7 R=1/2, 32M bits, hard + soft8 (BASELINE.json metric).

One step = one pass of the decode hot path over one batch of each headline workload, inputs
already resident in HBM:
  * HARD  input, M_B32 option       (BASELINE configs[1]: 32M bits, `-i h -m b32`)
  * SOFT8 input, M_B16 option       (BASELINE configs[2]: 32M bits, `-i s8 -m b16`)
Both on vd_decode_pk: exact-integer tagged metrics in the int16 halves of one word, two chunks per wave
(32-bit add, DPP subtract, v_pk_max_u16); HARD with 8-stage history fields, SOFT8 with 2-stage fields and a
renormalisation every 8 stages (vd_kernel_pk.h); both reproduce each option's tie rule word for word
(DESIGN.md 4).
value = decoded bits of both batches (2 x getMessageLen(64e6) = 63,999,872) / step time, summed
over ranks.  Multi-GPU (BASELINE configs[3]): one process per GPU, each rank decodes its own
independent batches (weak scaling, no data-path collective; an RCCL all_gather of per-rank
checksums runs once after the timed region).

Usage: python bench.py [--gpus N] [--steps K] [--warmup W]
   or: python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "gpu-accelerated-viterbi-decoder_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import vitdec  # noqa: E402

N_BITS = 32_000_000
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md)
SNR_DB = 2.0
WARM_S = 0.5      # minimum warm-up (seconds of steps) before the timed region
POOL = 128        # at most this many resident batches per workload (128 SOFT8 batches: 8.2 GB of input)
PMC_ROUND = "r06"  # profiles/<round>/: pmc_summary.json, ablate_batched.log, valu_model.json

WORKLOADS = [
    ("hard_b32", vitdec.HARD | vitdec.M_B32 | vitdec.O_B32),
    ("soft8_b16", vitdec.SOFT8 | vitdec.M_B16 | vitdec.O_B32),
]
# --workloads (profiling runs only, e.g. PMC passes over the other kernels; the default is the metric's
# two): name -> (options, float channel values fused into the decode)
ALL_WORKLOADS = {"hard_b32": (WORKLOADS[0][1], False), "soft8_b16": (WORKLOADS[1][1], False),
                 "fp32_f16": (vitdec.FP32 | vitdec.M_FP16 | vitdec.O_B32, False),
                 "soft4_b16": (vitdec.SOFT4 | vitdec.M_B16 | vitdec.O_B32, False),
                 "soft16_b32": (vitdec.SOFT16 | vitdec.M_B32 | vitdec.O_B32, False),
                 "hard_b32_ob16": (vitdec.HARD | vitdec.M_B32 | vitdec.O_B16, False),
                 "soft8_b16_llr": (vitdec.SOFT8 | vitdec.M_B16 | vitdec.O_B32, True)}
DEFAULT_WORKLOADS = ",".join(n for n, _ in WORKLOADS)


def algorithmic_bytes(opt, input_num):
    """HBM bytes a decode must move: packed channel input + packed decoded output."""
    return vitdec.lib().vd_input_size(opt, input_num) + vitdec.lib().vd_output_size(opt, input_num)


def cpu_baseline(batches):
    """Scalar host Viterbi (the oracle's CPU restatement, 1 thread) on the bench's own inputs.

    The sample is the full workload of one step: the same two 32M-bit batches the GPU decoded
    (copied from HBM), same 6400-chunk partition.  Its output is also compared word-for-word with
    the GPU output, so the bench line carries a full-size parity check."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import vd_oracle as vo
    dt = 0.0
    bits = 0
    match = True
    for b in batches:
        packed = b["inp"].cpu().numpy().view(np.float32 if (b["opt"] & 0xF) == vitdec.FP32 else np.int32)
        t0 = time.perf_counter()
        out, _ = vo.decode(b["opt"], packed, input_num=b["input_num"], nthreads=1)
        dt += time.perf_counter() - t0
        bits += b["msg"]
        gpu = b["out"].cpu().numpy().view(out.dtype)
        match = match and bool(np.array_equal(out, gpu))
    names = " + ".join(b["name"] for b in batches)
    # (ii) of SURVEY 8d: the same restatement over the independent chunks on every host thread this
    # process may use (the GPU box gives a job a 16-CPU share; os.cpu_count() shows the whole machine)
    nt = max(1, min(16, len(os.sched_getaffinity(0))))
    dt_mt = 0.0
    for b in batches:
        packed = b["inp"].cpu().numpy().view(np.float32 if (b["opt"] & 0xF) == vitdec.FP32 else np.int32)
        t0 = time.perf_counter()
        out, _ = vo.decode(b["opt"], packed, input_num=b["input_num"], nthreads=nt)
        dt_mt += time.perf_counter() - t0
        gpu = b["out"].cpu().numpy().view(out.dtype)
        match = match and bool(np.array_equal(out, gpu))
    all_cores = {"value": round(bits / dt_mt / 1e9, 6), "unit": "Gb/s", "cores": nt,
                 "sample": f"the same step on {nt} host threads (chunks split across threads) in {dt_mt:.2f} s"}
    return {"value": round(bits / dt / 1e9, 6), "unit": "Gb/s", "cores": 1, "kind": "port",
            "what": "naive scalar restatement (oracle): the reference's decode semantics as a plain int64 "
                    "64-state loop per chunk, not an optimised CPU decoder", "cpu_model": cpu_model(),
            "sample": f"one full bench step ({names}, 2 x 32M-bit batches, 6400-chunk partition) decoded by "
                      f"oracle/vd_oracle.c on 1 host thread in {dt:.1f} s; output identical to the GPU's: {match}",
            "matches_gpu": match, "all_cores": all_cores}


def parity_block(checks):
    """Word-for-word check of GPU outputs against the oracle (oracle/vd_oracle.c, the checker) on the host
    threads of this job, after the timed region: per path, the words compared and the mismatches.  checks:
    (path, options, packed input or float channel values, GPU output bytes, inputNum, packer scale or None
    -- with a scale the oracle packs the floats itself, SoftDecisionPacker restated, before decoding)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import vd_oracle as vo
    nt = max(1, min(16, len(os.sched_getaffinity(0))))
    res = {}
    t0 = time.perf_counter()
    for path, opt, inp, gout, n, scale in checks:
        packed = vo.pack(opt, inp.view(np.float32), scale, input_num=n) if scale is not None else inp.view(vo.in_dtype(opt))
        ref, ok = vo.decode(opt, packed, input_num=n, nthreads=nt)
        got = gout.view(np.uint8)[:ref.nbytes].view(ref.dtype)
        mism = int(np.count_nonzero(ref != got)) if got.size == ref.size else -1
        res[path] = {"options": hex(opt), "words": int(ref.size), "mismatches": mism}
    bad = [k for k, v in res.items() if v["mismatches"] != 0]
    return {"what": "GPU output vs oracle/vd_oracle.c (the CPU restatement) word for word, after the timed region: "
                    "both headline workloads (batch 0, and the last batch of the launch, whose waves run the "
                    "fairness controller), the other formats/cores (BASELINE configs[4] FP32/f16, SOFT4, SOFT16, "
                    "16-bit output words), the single-batch segment launches, and the fused float-input decode "
                    "(oracle: SoftDecisionPacker restated, then decode)",
            "paths": res, "all_match": not bad, "mismatching_paths": bad,
            "host_threads": nt, "seconds": round(time.perf_counter() - t0, 2)}


def cpu_model():
    """Host CPU model name (report the CPU next to the core count)."""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    import platform
    return platform.processor() or "unknown"


def load_pmc():
    """Per-kernel PMC summary committed under profiles/ (tools/pmc_summary.py over rocprofv3 --pmc
    passes of this bench): HBM bytes per launch (FETCH_SIZE x2 gfx950 correction + WRITE_SIZE) and
    VALU instruction counts."""
    p = os.path.join(ROOT, "profiles", PMC_ROUND, "pmc_summary.json")
    if os.path.exists(p):
        with open(p) as f:
            return json.load(f)
    return {}


N_SIMD = 1024     # 256 CUs x 4 SIMDs
OPS_PER_BIT = 256  # 64 ACS per decoded bit x {2 add, 1 max, 1 decision}
VALU_PEAK_TOPS = N_SIMD * 32 * 2.4e9 / 1e12  # lane-ops/s: SIMD-32, wave64 op in 2 cycles, 2.4 GHz
# the packed kernels do two int16 lane-ops per 32-bit lane-op (v_add_u32 / v_sub_u32 / v_pk_max_u16 on two
# chunks' halves): SURVEY 8d's "x2 for packed int16" peak
VALU_PEAK_TOPS_PACKED = 2 * VALU_PEAK_TOPS
N_XCD = 8         # rocprofv3 sums GRBM_GUI_ACTIVE over the 8 XCDs (MI355X_MICROARCH.md, DVFS give-back)


def acs_only_ms(name):
    """Instruction-mix ceiling of a workload's kernel: (ACS-only ms, full ms) per batch of the same batched
    launch on one box (tools/vd_pkab: 'ACS only' = no table build/reads, read-out, loads or traceback; 20
    batches per launch), from the committed ablation log of this round; None if absent.  Boxes differ by up
    to 15 %, so only the ratio of the two is carried over to the live kernel."""
    col = {"hard_b32": 0, "soft8_b16": 1, "fp32_f16": 2}.get(name)
    p = os.path.join(ROOT, "profiles", PMC_ROUND, "ablate_batched.log")
    if col is None or not os.path.exists(p):
        return None
    acs = full = None
    with open(p) as f:
        for line in f:
            cells = line.split(")")[-1].split() if line.startswith("ACS only") else line.split()[1:]
            if line.startswith("ACS only") and acs is None:
                acs = float(cells[col]) if len(cells) > col else None
            elif line.startswith("full ") and full is None:
                full = float(cells[col]) if len(cells) > col else None
    return (acs, full) if acs and full else None


def valu_model():
    """Per-opcode VALU cycle model (tools/isa_mix.py): each kernel's steady-state VALU mix per chunk-stage from
    its ISA, priced with this round's vd_ubench12 issue costs"""
    p = os.path.join(ROOT, "profiles", PMC_ROUND, "valu_model.json")
    if os.path.exists(p):
        with open(p) as f:
            return json.load(f)
    return {}


def valu_view(pmc, kernel_ms, stages, name, msg_bits):
    """The bound that binds: VALU issue.  From the committed PMC summary of this kernel
    (counters per dispatch, summed over the chip; the GRBM pass also ran --kernel-trace, so its kernel
    time and clock come from the same dispatches):
      cycles       = GRBM_GUI_ACTIVE / 8 XCDs                        (engine cycles of one dispatch)
      clock        = cycles / that run's kernel time
      issue_pct    = 100 * SQ_INSTS_VALU * 2 / (1024 * cycles)
                     (SIMD-32 model: a wave64 VALU instruction occupies its SIMD for 2 cycles at the
                     least; max/DPP/permlane/bit-field forms take 4 -- profiles/r02/ubench12.log)
      issue_pct_live = the same with the live kernel time at the PMC run's clock
      cycle_model_pct = 100 * (VALU cycles the kernel's instruction mix needs per SIMD) / cycles, where the
                     mix per chunk-stage comes from the kernel's ISA and each opcode's issue cost from this
                     round's vd_ubench12 (profiles/<round>/valu_model.json, tools/isa_mix.py); _live: at the
                     live kernel time
      mix ceiling  = the same launch with only the ACS recursion (tools/vd_ablate)."""
    c = pmc.get("counters_mean_per_dispatch", {})
    if not c or "SQ_INSTS_VALU" not in c:
        return None
    insts = c["SQ_INSTS_VALU"]
    # per chunk-stage (one chunk's 64 states for one stage): a wave-stage of vd_decode_tg; vd_decode_pk (batched
    # HARD) decodes two chunks per wave, so its wave-stages are half its chunk-stages
    v = {"insts_per_launch": round(insts), "insts_per_chunk_stage": round(insts / stages, 3),
         "chunk_stages_per_launch": stages}
    if "SQ_INSTS_LDS" in c:
        v["lds_insts_per_chunk_stage"] = round(c["SQ_INSTS_LDS"] / stages, 3)
    if "GRBM_GUI_ACTIVE" in c:
        cyc = c["GRBM_GUI_ACTIVE"] / N_XCD
        v["issue_pct"] = round(100.0 * insts * 2 / (N_SIMD * cyc), 1)
        v["cycles_per_inst_per_simd"] = round(N_SIMD * cyc / insts, 3)
        ghz = pmc.get("pmc_run_clock_ghz")
        if ghz:
            v["pmc_run_clock_ghz"] = round(ghz, 3)
            v["pmc_run_kernel_ms"] = round(pmc["pmc_run_kernel_ns_median"] * 1e-6, 4)
            v["issue_pct_live"] = round(100.0 * insts * 2 / (N_SIMD * kernel_ms * 1e-3 * ghz * 1e9), 1)
        model = valu_model().get("kernels", {}).get(name)
        if model and ghz:
            # VALU cycles the kernel's instruction mix needs per SIMD (tools/isa_mix.py: ISA mix x ubench costs)
            # against the SIMD cycles the live kernel time gives at the PMC run's clock
            need = model["valu_cycles_per_chunk_stage"] * stages / N_SIMD
            v["cycle_model"] = {"valu_cycles_per_chunk_stage": model["valu_cycles_per_chunk_stage"],
                                "valu_insts_per_chunk_stage_isa": model["valu_per_chunk_stage"],
                                "source": f"profiles/{PMC_ROUND}/valu_model.json (tools/isa_mix.py)"}
            v["cycle_model_pct_live"] = round(100.0 * need / (kernel_ms * 1e-3 * ghz * 1e9), 1)
            v["cycle_model_pct"] = round(100.0 * need / cyc, 1)
    ab = acs_only_ms(name)
    if ab:
        # the ablation box's ACS-only / full ratio applied to the live kernel time
        frac = ab[0] / ab[1]
        v["mix_ceiling"] = {"acs_only_ms": round(frac * kernel_ms, 4),
                            "gbps": round(msg_bits / (frac * kernel_ms * 1e-3) / 1e9, 2), "frac": round(frac, 3),
                            "ablation_ms": {"acs_only": ab[0], "full": ab[1]},
                            "source": f"profiles/{PMC_ROUND}/ablate_batched.log (tools/vd_pkab: codeword input, 20 batches per launch)"}
    v["source"] = f"profiles/{PMC_ROUND}/pmc_summary.json"
    return v


def stages_per_launch(opt, input_num):
    """wave-stages one decode launch runs: every chunk decodes its words plus a 64-stage window."""
    bpp = 16 if (opt & 0xF00) == vitdec.O_B16 else 32
    pack = vitdec.lib().vd_message_len(opt, input_num) // bpp
    n = vitdec.lib().vd_num_chunks()
    base, rem = divmod(pack, n)
    total = 0
    for words, cnt in ((base + 1, rem), (base, n - rem)):
        if words:
            total += cnt * (64 + (words * bpp + 31) // 32 * 32)
    return total


def rank_seed(rank, workload_index, step=0, world=1):
    """(bitSeed, noiseSeed) of the batch a rank decodes at a step: independent batches per rank and step
    (weak scaling), batch i = 2 (rank + world step) + workload seeded (1 + 2i, 2 + 2i) as SURVEY 8d's
    multi-GPU config (step 0: batch i = 2 rank + workload)."""
    i = 2 * (rank + world * step) + workload_index
    return (1 + 2 * i, 2 + 2 * i)


def resident_batches(opt, nbatch, seeds, dev, sptr):
    """nbatch independent 32M-bit batches of one format resident in HBM, each from its own seeds (the
    reference harness chain, vd_simulate_device): inputs at a 256-byte stride, source bits kept for the
    BER check."""
    input_num = 2 * N_BITS
    nin = vitdec.lib().vd_input_size(opt, input_num)
    istride = (nin + 255) // 256 * 256
    inps = torch.empty(nbatch * istride, dtype=torch.uint8, device=dev)
    bits = torch.empty(nbatch, N_BITS, dtype=torch.uint8, device=dev)
    for k in range(nbatch):
        bs, ns = seeds(k)
        vitdec.simulate_device(opt, N_BITS, SNR_DB, bs, ns, bits[k].data_ptr(), inps[k * istride:].data_ptr(), sptr)
    return inps, istride, bits


def resident_llr_batches(nbatch, seeds, dev, sptr):
    """nbatch independent 32M-bit batches of float channel values (the reference's AddNoise output,
    vd_channel_device: 64M floats each) resident in HBM, for the fused-quantisation decode"""
    n = 2 * N_BITS
    istride = (n * 4 + 255) // 256 * 256
    vals = torch.empty(nbatch * istride // 4, dtype=torch.float32, device=dev)
    bits = torch.empty(nbatch, N_BITS, dtype=torch.uint8, device=dev)
    for k in range(nbatch):
        bs, ns = seeds(k)
        vitdec.channel_device(N_BITS, SNR_DB, bs, ns, bits[k].data_ptr(), vals.data_ptr() + k * istride, sptr)
    return vals.view(torch.uint8), istride, bits


def batch_ber(opt, bits, outs, ostride, nout, k, msg):
    """decoded-bit error rate of batch k of a launch against its source bits"""
    dt = np.uint16 if (opt & 0xF00) == vitdec.O_B16 else np.uint32
    out_h = outs[k * ostride: k * ostride + nout].cpu().numpy().view(dt)
    return vitdec.count_errors(opt, bits[k].cpu().numpy(), out_h) / msg, out_h


def aggregate_gbps(bits_per_step, world, steps, elapsed_s):
    """Whole-job throughput: every rank decodes bits_per_step per step; elapsed is the max over ranks."""
    return bits_per_step * world * steps / elapsed_s / 1e9


def free_port():
    """A free TCP port on the loopback interface (rendezvous of the process group)."""
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


# Rehearsal of the N > 1 path on a 1-GPU box (tests/test_gpu_dist.py): every rank decodes on cuda:0 and the
# collectives run over gloo on host tensors.  Its numbers are not a measurement (the ranks share one GPU);
# the line says so in config.parallelism and config.rehearsal.
REHEARSE = os.environ.get("VD_BENCH_REHEARSE_SHARED_GPU") == "1"


def init_ranks(world, local):
    """The process group every run uses, N = 1 included, so the N = 1 point runs the same collectives as
    N > 1 (barrier, max over ranks, checksum gather, final gather): RCCL (backend "nccl") bound to this
    rank's GPU.  A plain `python bench.py` at N = 1 has no launcher environment; it becomes rank 0 of a
    1-rank group with its own rendezvous on 127.0.0.1."""
    if "MASTER_ADDR" not in os.environ or "WORLD_SIZE" not in os.environ:
        assert world == 1
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(free_port()), RANK="0", WORLD_SIZE="1",
                          LOCAL_RANK="0")
    if REHEARSE:
        torch.cuda.set_device(0)
        torch.distributed.init_process_group("gloo")
        return
    torch.cuda.set_device(local)
    torch.distributed.init_process_group("nccl", device_id=torch.device("cuda", local))


def max_over_ranks(elapsed, dev):
    t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
    return float(t.item())


def gather_checksums(sums, dev, world):
    """Per-rank XOR checksums of the decoded words (after timing), all_gather of a few int64s."""
    cs = torch.tensor(sums, dtype=torch.int64, device=dev)
    gathered = [torch.empty_like(cs) for _ in range(world)]
    torch.distributed.all_gather(gathered, cs)
    return [[int(v) for v in g.cpu()] for g in gathered]


def gather_outputs(outs, dev, world, rank):
    """The north_star's final gather: every rank's decoded words (uint8 tensors, equal sizes) collected
    on rank 0 over RCCL (torch.distributed.gather to dst 0: rank 0 receives world x the words, the other
    ranks only send theirs; gloo on CPU in tests/test_dist.py).  Outside the timed region.  Returns (ms,
    per-rank XOR checksums of what rank 0 received, None) on rank 0, (ms, None, None) elsewhere, or (None,
    None, error) on every rank when a rank could not build its buffers: the ranks agree on that
    (all_reduce of an ok flag) before anyone enters the collective, so no rank is left waiting in it."""
    err = None
    try:
        flat = torch.cat([o.view(-1) for o in outs])
        bufs = [torch.empty_like(flat) for _ in range(world)] if rank == 0 else None
    except Exception as e:  # e.g. torch.OutOfMemoryError on this rank only
        err = str(e)[:200]
    ok = torch.tensor([0 if err else 1], dtype=torch.int32, device=dev)
    torch.distributed.all_reduce(ok, op=torch.distributed.ReduceOp.MIN)
    if int(ok.item()) == 0:
        return None, None, err or "a peer rank could not build its gather buffers"
    torch.distributed.barrier()
    if flat.is_cuda:
        torch.cuda.synchronize()
    t = time.perf_counter()
    torch.distributed.gather(flat, gather_list=bufs, dst=0)
    if flat.is_cuda:
        torch.cuda.synchronize()
    ms = (time.perf_counter() - t) * 1e3
    if rank != 0:
        return ms, None, None
    sums = []
    for b in bufs:
        parts, off = [], 0
        for o in outs:
            n = o.numel()
            parts.append(int(np.bitwise_xor.reduce(b[off:off + n].cpu().numpy().view(np.uint32))))
            off += n
        sums.append(parts)
    return ms, sums, None


OTHER_CONFIGS = [
    ("fp32_f16", vitdec.FP32 | vitdec.M_FP16 | vitdec.O_B32),   # BASELINE configs[4]
    ("soft4_b16", vitdec.SOFT4 | vitdec.M_B16 | vitdec.O_B32),
    ("soft16_b32", vitdec.SOFT16 | vitdec.M_B32 | vitdec.O_B32),
    ("hard_b32_ob16", vitdec.HARD | vitdec.M_B32 | vitdec.O_B16),
]


def settle(fn, seconds=0.3):
    """Run fn back to back for `seconds` so a side measurement starts at the sustained GPU clock (the
    measurements before it leave the GPU idle; profiles/r02/clock_ramp.log)."""
    t0 = time.perf_counter()
    n = 0
    while time.perf_counter() - t0 < seconds:
        fn()
        n += 1
        if n % 8 == 0:
            torch.cuda.synchronize()
    torch.cuda.synchronize()


def other_configs_side_measurement(dev, sptr, stream, reps=20, keep=None):
    """Kernel-only Gb/s of the other input formats / cores at 32M bits (BASELINE configs[4] = FP32 input
    on the fp16 core, plus SOFT4, SOFT16 and 16-bit output words), inputs synthesised by the GPU channel
    source at the bench SNR.  Outside the timed region; never `value`.  keep: a list that receives host
    copies (input, output) of batch 0 and of the launch's last batch for the parity block."""
    res = {}
    for i, (name, opt) in enumerate(OTHER_CONFIGS):
        n = 2 * N_BITS
        inps, istride, bits = resident_batches(opt, reps, lambda k: (101 + 2 * i + 1000 * k, 102 + 2 * i + 1000 * k),
                                               dev, sptr)
        nout = vitdec.lib().vd_output_size(opt, n)
        ostride = (nout + 255) // 256 * 256
        outs = torch.empty(reps * ostride, dtype=torch.uint8, device=dev)
        dec = vitdec.ViterbiCUDA(opt, 0, dev)
        # as the timed region: `reps` independent batches in one launch (vd_run_device_batch), per batch =
        # time / reps
        run = lambda: dec.run_device_batch(inps.data_ptr(), istride, outs.data_ptr(), ostride, n, reps, sptr)
        settle(run)
        e = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        e[0].record(stream)
        run()
        e[1].record(stream)
        torch.cuda.synchronize()
        ms = e[0].elapsed_time(e[1]) / reps
        msg = vitdec.lib().vd_message_len(opt, n)
        ber = max(batch_ber(opt, bits, outs, ostride, nout, k, msg)[0] for k in (0, reps - 1))
        res[name] = {"kernel": dec.kernel_for(n, reps), "kernel_ms": round(ms, 4),
                     "gbps": round(msg / (ms * 1e-3) / 1e9, 2), "ber": ber, "batches_per_launch": reps}
        if keep is not None:  # host copies for the parity block: batch 0 and the last batch of the launch
            nin = vitdec.lib().vd_input_size(opt, n)
            for k in (0, reps - 1):
                keep.append((f"other_configs.{name}[batch {k}]", opt, inps[k * istride:k * istride + nin].cpu().numpy(),
                             outs[k * ostride:k * ostride + nout].cpu().numpy(), n, None))
        dec.close()
        del inps, bits, outs
    return res


def single_launch_side_measurement(batches, stream, sptr, reps=20, keep=None):
    """The reference run()'s unit of work on device buffers: one vd_run_device launch per 32M-bit batch
    (segment launch, 6400-chunk partition), `reps` of the bench's resident batches back to back, per batch
    = time / reps, into buffers of their own.  Outside the timed region; never `value` (the timed region
    batches its launches).  keep: receives batch 0's segment-launch output for the parity block."""
    res = {}
    for b in batches:
        K = b["outs"].numel() // b["ostride"]
        n = min(reps, K)
        souts = torch.empty(n * b["ostride"], dtype=torch.uint8, device=b["outs"].device)
        run = lambda: [b["dec"].run_device(b["inps"].data_ptr() + k * b["istride"],
                                           souts.data_ptr() + k * b["ostride"], b["input_num"], sptr)
                       for k in range(n)]
        settle(run)
        e = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        rd0 = vitdec.split_redecodes(b["inps"].device.index or 0)
        e[0].record(stream)
        run()
        e[1].record(stream)
        torch.cuda.synchronize()
        redec = vitdec.split_redecodes(b["inps"].device.index or 0) - rd0
        ms = e[0].elapsed_time(e[1]) / n
        nout = b["nout"]
        # every segment-launch output equals the batched launch's output of the same batch (word for word,
        # on the GPU); batch 0 also goes to the oracle in the parity block
        same = [bool(torch.equal(souts[k * b["ostride"]:k * b["ostride"] + nout], b["outs"][k * b["ostride"]:k * b["ostride"] + nout]))
                for k in range(n)]
        res[b["name"]] = {"kernel": b["dec"].kernel_for(b["input_num"], 1, b["llr"]), "kernel_ms": round(ms, 4),
                          "gbps": round(b["msg"] / (ms * 1e-3) / 1e9, 2), "launches": n,
                          "split_redecodes_per_launch": round(redec / n, 2),
                          "equals_batched_launch": f"{sum(same)} of {n} batches"}
        if keep is not None:
            keep.append((f"single_launch.{b['name']}[batch 0]", b["opt"], b["inp"].cpu().numpy(),
                         souts[:nout].cpu().numpy(), b["input_num"], None))
        del souts
    return res


def llr_side_measurement(dev, sptr, stream, reps=20, keep=None):
    """Float channel values in HBM (the reference's AddNoise output before SoftDecisionPacker: the harness
    chain's codeword + AWGN at SNR_DB, vd_channel_device): the GPU packer alone, packer + decode, and the fused
    decode (quantisation in the table build), SOFT8/int16.  Outside the timed region; not part of `value`.
    (Until round 5 the values were random +-1 symbols plus noise, not a codeword: noise to the decoder, on
    which speculative split starts rarely converge.)"""
    opt = vitdec.SOFT8 | vitdec.M_B16 | vitdec.O_B32
    n = 2 * N_BITS
    vals = torch.empty(n, dtype=torch.float32, device=dev)
    src = torch.empty(N_BITS, dtype=torch.uint8, device=dev)
    vitdec.channel_device(N_BITS, SNR_DB, 901, 902, src.data_ptr(), vals.data_ptr(), sptr)
    packed = torch.empty(vitdec.lib().vd_input_size(opt, n), dtype=torch.uint8, device=dev)
    out_fused = torch.empty(vitdec.lib().vd_output_size(opt, n), dtype=torch.uint8, device=dev)
    out_two = torch.empty_like(out_fused)
    dec = vitdec.ViterbiCUDA(opt, 0, dev)

    def timed(fn):
        settle(fn)
        e = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        e[0].record(stream)
        for _ in range(reps):
            fn()
        e[1].record(stream)
        torch.cuda.synchronize()
        return e[0].elapsed_time(e[1]) / reps

    pack = lambda: vitdec.pack_device(opt, vals.data_ptr(), n, packed.data_ptr(), 40000.0, sptr)
    two = lambda: (pack(), dec.run_device(packed.data_ptr(), out_two.data_ptr(), n, sptr))
    fused = lambda: dec.run_device_llr(vals.data_ptr(), out_fused.data_ptr(), n, 40000.0, sptr)
    t_pack, t_two, t_fused = timed(pack), timed(two), timed(fused)
    same = bool(torch.equal(out_fused, out_two))
    msg = vitdec.lib().vd_message_len(opt, n)
    # as the timed region and other_configs: `reps` distinct float batches in one launch
    # (vd_run_device_llr_batch); batch 0 is `vals`, the others fresh draws
    istride = n * 4
    many = torch.empty(reps * n, dtype=torch.float32, device=dev)
    many[:n] = vals
    for k in range(1, reps):
        vitdec.channel_device(N_BITS, SNR_DB, 901 + 2 * k, 902 + 2 * k, src.data_ptr(), many[k * n:].data_ptr(), sptr)
    del src
    nout = out_fused.numel()
    ostride = (nout + 255) // 256 * 256
    outs = torch.empty(reps * ostride, dtype=torch.uint8, device=dev)
    batched = lambda: dec.run_device_llr_batch(many.data_ptr(), istride, outs.data_ptr(), ostride, n, reps, 40000.0,
                                               sptr)
    settle(batched)
    e = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    e[0].record(stream)
    batched()
    e[1].record(stream)
    torch.cuda.synchronize()
    t_batched = e[0].elapsed_time(e[1]) / reps
    same_b = bool(torch.equal(outs[:nout], out_fused))
    if keep is not None:  # the oracle packs the same floats (SoftDecisionPacker restated) and decodes them
        keep.append(("llr_input.fused_single", opt, vals.cpu().numpy(), out_fused.cpu().numpy(), n, 40000.0))
        keep.append((f"llr_input.fused_batched[batch {reps - 1}]", opt, many[(reps - 1) * n:reps * n].cpu().numpy(),
                     outs[(reps - 1) * ostride:(reps - 1) * ostride + nout].cpu().numpy(), n, 40000.0))
    dec.close()
    del many, outs
    return {"workload": "64M float32 channel values (the harness's codeword + AWGN at %.1f dB, 32M-bit SOFT8 batch, "
                        "scale 40000) resident in HBM" % SNR_DB,
            "pack_ms": round(t_pack, 4), "pack_GBps": round(n * 4 / (t_pack * 1e-3) / 1e9, 1),
            "pack_then_decode_ms": round(t_two, 4), "fused_decode_ms": round(t_fused, 4),
            "fused_gbps": round(msg / (t_fused * 1e-3) / 1e9, 2), "fused_equals_pack_then_decode": same,
            "fused_batched": {"batches_per_launch": reps, "ms_per_batch": round(t_batched, 4),
                              "gbps": round(msg / (t_batched * 1e-3) / 1e9, 2), "batch0_equals_single": same_b}}


def channel_side_measurement(dev, sptr, reps=5, sample_bits=1_000_000):
    """The reference harness's channel source (RandBitGen | encoder | AddNoise | packer, SOFT8) for one
    32M-bit batch on the GPU (vd_simulate_device), against the host harness (libstdc++ generators, one
    thread) on a 1M-bit sample with the same seeds, checked equal.  Outside the timed region."""
    opt = vitdec.SOFT8 | vitdec.M_B16
    bits = torch.empty(N_BITS, dtype=torch.uint8, device=dev)
    packed = torch.empty(vitdec.lib().vd_input_size(opt, 2 * N_BITS), dtype=torch.uint8, device=dev)
    run = lambda n: vitdec.simulate_device(opt, n, SNR_DB, 7, 8, bits.data_ptr(), packed.data_ptr(), sptr)
    run(N_BITS)
    ts = []
    for _ in range(reps):
        torch.cuda.synchronize()
        t = time.perf_counter()
        run(N_BITS)
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t)
    t_dev = sorted(ts)[len(ts) // 2]
    t = time.perf_counter()
    hb, hp = vitdec.simulate_host(opt, sample_bits, SNR_DB, 7, 8)
    t_host = time.perf_counter() - t
    run(sample_bits)
    torch.cuda.synchronize()
    nb = hp.nbytes
    same = bool(np.array_equal(packed[:nb].cpu().numpy(), hp.view(np.uint8)) and
                np.array_equal(bits[:sample_bits].cpu().numpy(), hb))
    return {"workload": "32M-bit SOFT8 batch from seeds (7, 8)", "device_ms": round(t_dev * 1e3, 3),
            "device_gbit_per_s": round(N_BITS / t_dev / 1e9, 2),
            "host_harness": {"sample_bits": sample_bits, "ms": round(t_host * 1e3, 1),
                             "mbit_per_s": round(sample_bits / t_host / 1e6, 2), "threads": 1},
            "device_equals_host_on_sample": same}


def pcie_side_measurement(batches, dev, nb=6):
    """PCIe-inclusive rate (the reference run()'s scope: host buffers in, host buffers out): nb
    independent batches per workload (the bench's resident inputs) in pinned host memory through vd_run_stream, which decodes them
    zero-copy (the kernels read the packed words and write the decoded words over PCIe).  Outside the
    timed region; never `value`."""
    res = {"batches": nb, "host_buffers": "pinned (vd_host_alloc), zero-copy decode"}
    for b in batches:
        # the bench's own resident batches (distinct inputs; batch k % K)
        nin, K = b["inp"].numel(), b["outs"].numel() // b["ostride"]
        pdt = np.float32 if (b["opt"] & 0xF) == vitdec.FP32 else np.int32
        packed = b["inp"].cpu().numpy().view(pdt)
        pins = [vitdec.PinnedArray(packed.shape, packed.dtype) for _ in range(nb)]
        for k, p in enumerate(pins):
            o = (k % K) * b["istride"]
            p.array[:] = b["inps"][o:o + nin].cpu().numpy().view(pdt)
        dt = np.uint16 if (b["opt"] & 0xF00) == vitdec.O_B16 else np.uint32
        nout = vitdec.lib().vd_output_size(b["opt"], b["input_num"]) // np.dtype(dt).itemsize
        pouts = [vitdec.PinnedArray((nout,), dt) for _ in range(nb)]
        dec = vitdec.ViterbiCUDA(b["opt"], b["input_num"], dev)
        dec.run_stream([pins[0].array], b["input_num"], [pouts[0].array])  # warm-up
        outs, ms = dec.run_stream([p.array for p in pins], b["input_num"], [o.array for o in pouts])
        dec.close()
        res[b["name"]] = {"wall_ms": round(ms, 3), "gbps": round(nb * b["msg"] / (ms * 1e-3) / 1e9, 2),
                          "h2d_bytes_per_batch": packed.nbytes}
    return res


def launch_ranks(nproc, argv):
    """`bench.py --gpus N` (N > 1) without a torch.distributed launcher: start N ranks with
    torch.distributed.run as a CHILD process (this process has not touched the GPU and never will), pass
    its output through, and return its exit code.  Each rank re-enters main() with WORLD_SIZE set."""
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()), os.path.abspath(__file__), *argv]
    return subprocess.call(cmd)


def ranks_check(world, rank):
    """--ranks-check (tests): the rank layout `--gpus N` produces, over gloo, no GPU touched."""
    torch.distributed.init_process_group("gloo")
    got = [None] * world
    torch.distributed.all_gather_object(got, {"rank": rank, "local_rank": int(os.environ.get("LOCAL_RANK", "0"))})
    if rank == 0:
        print(json.dumps({"n_gpus": world, "ranks": got}), flush=True)
    torch.distributed.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--warm-s", type=float, default=WARM_S,
                    help="minimum warm-up in seconds of steps (GPU clock ramp; 0 for counter-collection runs)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-llr", action="store_true", help="skip the float-input (packer fused) side measurement")
    ap.add_argument("--no-pcie", action="store_true", help="skip the host-to-host pipelined side measurement")
    ap.add_argument("--no-channel", action="store_true", help="skip the channel-source side measurement")
    ap.add_argument("--no-other", action="store_true", help="skip the other-formats side measurement")
    ap.add_argument("--no-parity", action="store_true", help="skip the oracle parity block (profiling runs)")
    ap.add_argument("--workloads", default=DEFAULT_WORKLOADS,
                    help="profiling runs only: comma-separated workloads to time (" + ",".join(ALL_WORKLOADS) + ")")
    ap.add_argument("--ranks-check", action="store_true", help=argparse.SUPPRESS)  # tests: rank layout only
    args = ap.parse_args()

    if args.gpus < 1:
        sys.exit(f"bench.py: --gpus must be >= 1 (got {args.gpus})")
    if "WORLD_SIZE" not in os.environ:
        if args.gpus > 1:  # one process per GPU: start the ranks as children, before any GPU call here
            sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
        world = 1
    else:
        world = int(os.environ["WORLD_SIZE"])
        if world != args.gpus:
            sys.exit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}; launch one rank per GPU "
                     f"(torch.distributed.run --nproc-per-node {args.gpus}) or drop the launcher")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.ranks_check:
        return ranks_check(world, rank)
    if torch.cuda.device_count() < world and not REHEARSE:
        sys.exit(f"bench.py: {world} ranks but only {torch.cuda.device_count()} visible GPU(s)")
    init_ranks(world, local)
    dev = torch.cuda.current_device()
    cdev = "cpu" if REHEARSE else dev  # where the collectives' tensors live
    stream = torch.cuda.current_stream()
    sptr = stream.cuda_stream

    # resident inputs: each rank synthesises its own independent batches per workload in HBM (one per
    # step, each from its own seeds; at most POOL of them, step k decoding batch k % POOL), with the
    # reference harness's own chain (std::mt19937 bits and noise, BPSK+AWGN, quantiser at 40000)
    # generated bit-exactly on the GPU (vd_simulate_device)
    K = args.steps
    P = min(K, POOL)
    sizes = [P] * (K // P) + ([K % P] if K % P else [])  # batches per launch
    batches = []
    names = args.workloads.split(",")
    if any(n not in ALL_WORKLOADS for n in names):
        sys.exit(f"bench.py: unknown workload in {args.workloads} (known: {', '.join(ALL_WORKLOADS)})")
    metric_run = args.workloads == DEFAULT_WORKLOADS
    for wi, name in enumerate(names):
        opt, llr = ALL_WORKLOADS[name]
        input_num = 2 * N_BITS
        nout = vitdec.lib().vd_output_size(opt, input_num)
        seeds = lambda k: rank_seed(rank, wi, k, world)
        if llr:
            inps, istride, bits = resident_llr_batches(P, seeds, dev, sptr)
        else:
            inps, istride, bits = resident_batches(opt, P, seeds, dev, sptr)
        ostride = (nout + 255) // 256 * 256
        outs = torch.empty(P * ostride, dtype=torch.uint8, device=dev)  # one output per resident batch
        dec = vitdec.ViterbiCUDA(opt, 0, dev)
        nin = vitdec.lib().vd_input_size(opt, input_num)
        # inp / out: batch 0 (the step the CPU baseline and the PCIe side measurement repeat)
        batches.append(dict(name=name, opt=opt, llr=llr, input_num=input_num, inps=inps, istride=istride, outs=outs,
                            ostride=ostride, nout=nout, bits=bits, dec=dec, inp=inps[:nin], out=outs[:nout],
                            msg=vitdec.lib().vd_message_len(opt, input_num)))
    torch.cuda.synchronize()

    nw = len(batches)
    # The K steps are K independent batches per workload.  Each workload's batches go out as ONE launch
    # (vd_run_device_batch: batch k decodes its own resident input into its own output, every batch
    # exactly as a single vd_run_device would; K > POOL: launches of POOL batches), so the next batch's
    # chunks fill the launch tail that the slowest XCD sets (0.1776 -> 0.1673 ms per HARD
    # batch in tools/vd_benchab).  One HIP event between the workloads' launches times each kernel; per
    # batch = launch time / K.
    evs = [torch.cuda.Event(enable_timing=True) for _ in range(nw + 1)]

    def run(b):
        for nbatch in sizes:
            if b["llr"]:
                b["dec"].run_device_llr_batch(b["inps"].data_ptr(), b["istride"], b["outs"].data_ptr(), b["ostride"],
                                              b["input_num"], nbatch, 40000.0, sptr)
            else:
                b["dec"].run_device_batch(b["inps"].data_ptr(), b["istride"], b["outs"].data_ptr(), b["ostride"],
                                          b["input_num"], nbatch, sptr)

    # Warm-up: the W steps asked for, and at least WARM_S seconds of steps.  From idle the GPU takes
    # tens of milliseconds to reach its sustained clock; a timed region right behind a short warm-up read
    # ~17 % slow kernels (0.221 vs 0.186 ms HARD, profiles/r02/clock_ramp.log).  So nothing may leave the
    # GPU idle between the warm-up and the timed region: the first collective of a process (RCCL sets up
    # its kernels there, ~20 ms) and the wait for ranks that finished input synthesis later run BEFORE
    # the warm-up (one barrier), every rank then runs the same number of warm-up iterations (the max over
    # ranks of what each needs), and the barrier in front of the timed region finds the ranks aligned.
    # (With the set-up in that barrier the first timed launches ran on a cooled-down GPU: HARD 0.199 ms
    # instead of 0.159 ms per batch, profiles/r03/README.md.)
    torch.distributed.barrier()
    torch.cuda.synchronize()

    def warm_iteration():
        for b in batches:
            run(b)
        torch.cuda.synchronize()

    tw = time.perf_counter()
    warm_iteration()
    t_it = time.perf_counter() - tw
    n_more = max(-(-args.warmup // K), int(np.ceil(args.warm_s / max(t_it, 1e-6)))) - 1
    n_more = int(max_over_ranks(float(n_more), cdev))
    for _ in range(n_more):
        warm_iteration()
    nwarm = K * (1 + n_more)
    torch.distributed.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    evs[0].record(stream)
    for i, b in enumerate(batches):
        run(b)
        evs[i + 1].record(stream)
    torch.cuda.synchronize()
    torch.distributed.barrier()
    elapsed = time.perf_counter() - t0

    # per-launch durations from the HIP events on the launch stream; per batch = / K
    launch_ms = [evs[i].elapsed_time(evs[i + 1]) for i in range(nw)]
    kms = [t / K for t in launch_ms]
    # correctness side-channel (outside the timed region): the decoded-bit error rate of every batch
    # against its own source bits (max over the resident batches), and per-rank checksums of the decoded
    # words: per workload the xor over every resident batch's words, then the xor of batch 0's words (the
    # batch the final gather collects, which checks what rank 0 received against them)
    bers = []
    sums, sums0 = [], []
    for b in batches:
        ber_k, ck = [], 0
        for k in range(P):
            e, out_h = batch_ber(b["opt"], b["bits"], b["outs"], b["ostride"], b["nout"], k, b["msg"])
            ber_k.append(e)
            x = int(np.bitwise_xor.reduce(out_h.view(np.uint32)))
            ck ^= x
            if k == 0:
                sums0.append(x)
        bers.append(max(ber_k))
        sums.append(ck)
    # side measurements, the kernel-only ones first (the PCIe one leaves the GPU waiting on host copies)
    side = rank == 0 and metric_run
    # the other formats and the fused float input run in launches of as many batches as the timed region's
    # (at least 20): a shorter launch carries more of the once-per-launch ramp and tail per batch
    side_reps = max(20, P)
    # parity block (rank 0, every N): host copies of the outputs to check against the oracle at the end
    checks = [] if (rank == 0 and not args.no_parity) else None
    if checks is not None:
        for b in batches:
            for k in sorted({0, P - 1}):
                nin = 4 * b["input_num"] if b["llr"] else b["inp"].numel()  # float channel values / packed words
                checks.append((f"{b['name']}[batch {k}]", b["opt"],
                               b["inps"][k * b["istride"]:k * b["istride"] + nin].cpu().numpy(),
                               b["outs"][k * b["ostride"]:k * b["ostride"] + b["nout"]].cpu().numpy(), b["input_num"],
                               40000.0 if b["llr"] else None))
    other = None if (args.no_other or not side) else other_configs_side_measurement(dev, sptr, stream, side_reps, checks)
    single = None if (args.no_other or not side) else single_launch_side_measurement(batches, stream, sptr, keep=checks)
    llr = None if (args.no_llr or not side) else llr_side_measurement(dev, sptr, stream, side_reps, checks)
    chan = None if (args.no_channel or not side) else channel_side_measurement(dev, sptr)
    pcie = None if (args.no_pcie or not side) else pcie_side_measurement(batches, dev)
    # the same collectives at every N (N = 1: a 1-rank RCCL group)
    elapsed = max_over_ranks(elapsed, cdev)
    gathered = gather_checksums(sums + sums0, cdev, world)
    gms, gsums, err = gather_outputs([b["out"].cpu() if REHEARSE else b["out"] for b in batches], cdev, world, rank)
    final_gather = None
    if rank == 0:
        if err is not None:  # a side measurement: report it, keep the bench line
            final_gather = {"error": err}
        else:
            nbytes = sum(b["out"].numel() for b in batches)
            final_gather = {"what": "every rank's decoded words (batch 0 of each workload) gathered on rank 0 "
                                    "over RCCL (torch.distributed.gather, dst 0)",
                            "bytes_per_rank": nbytes, "world": world, "ms": round(gms, 3),
                            "GBps_into_rank0": round(nbytes * (world - 1) / (gms * 1e-3) / 1e9, 2),
                            "checksums_match": gsums == [g[nw:] for g in gathered]}

    if rank == 0:
        bits_per_step = sum(b["msg"] for b in batches)
        ms_per_step = elapsed / args.steps * 1e3
        value = aggregate_gbps(bits_per_step, world, args.steps, elapsed)
        # roofline of the SOFT8 kernel (HBM, algorithmic bytes = packed input + packed output): the two
        # kernels take about half the step each; SOFT8 moves 5.7x the bytes, so it is the one whose HBM
        # fraction means something.  per_kernel holds both.
        pmcs = load_pmc()

        def kernel_roofline(i):
            b = batches[i]
            alg = algorithmic_bytes(b["opt"], b["input_num"]) if not b["llr"] else \
                4 * b["input_num"] + vitdec.lib().vd_output_size(b["opt"], b["input_num"])
            ach = alg / (kms[i] * 1e-3) / 1e9
            pmc = pmcs.get(b["name"], {})
            stages = stages_per_launch(b["opt"], b["input_num"])
            return {"kernel": b["name"] + ": " + b["dec"].kernel_for(b["input_num"], sizes[0], b["llr"]), "ms": round(kms[i], 4),
                    "launch_ms": round(launch_ms[i], 4), "batches_per_launch": P, "launches": len(sizes),
                    "achieved": round(ach, 2), "frac": round(ach / HBM_PEAK_GBS, 5),
                    "algorithmic_bytes_per_batch": alg, "algorithmic_bytes_per_step_launches": alg * K,
                    "traffic": pmc.get("traffic_bytes"),
                    "valu": valu_view(pmc, kms[i], stages, b["name"], b["msg"])}

        rl = [kernel_roofline(i) for i in range(nw)]
        di = next((i for i, b in enumerate(batches) if b["name"] == "soft8_b16"), int(np.argmax(kms)))
        result = {
            "metric": "decoded Gb/s at K=7 R=1/2, 32M bits, hard+soft8",
            "value": round(value, 3),
            "unit": "Gb/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "exact integers in int16 halves (u16x2) for HARD and SOFT8 (int32 / int16 tie semantics)",
            "data": f"synthetic: the reference harness chain generated on the GPU bit-exactly (std::mt19937 "
                    f"bits, K=7 (0171,0133) encoder, BPSK + normal_distribution<float> AWGN at {SNR_DB} dB, "
                    f"quantiser scale 40000), seeds (1+2i, 2+2i) for batch i = 2 rank + workload",
            "config": {
                "workload": "per GPU per step: one 32M-bit HARD batch with the M_B32 option (int32 tie rule) + "
                            "one 32M-bit SOFT8 batch with the M_B16 option (int16 tie rule), BASELINE configs[1]+[2], "
                            "both on vd_decode_pk (exact-integer tagged metrics in the int16 halves of one word, "
                            "two chunks per wave: v_add_u32, v_sub_u32_dpp, v_pk_max_u16; HARD 8-stage history "
                            "fields, SOFT8 2-stage fields renormalised every 8 stages: DESIGN.md 4); each batch "
                            "uses the reference's 6400-chunk partition",
                "n_bits_per_batch": N_BITS,
                "decoded_bits_per_batch": batches[0]["msg"],
                "parallelism": (f"rehearsal: {world} ranks sharing cuda:0, collectives over gloo" if REHEARSE else
                                f"batch-shard x{world}" if world > 1 else "single GPU (1-rank RCCL group)"),
                "launch": {"entry": "vd_run_device_batch", "batches_per_launch": P, "launches": len(sizes),
                           "what": "each workload's K steps as one launch of K independent batches (K "
                                   "resident inputs from distinct seeds, every batch's BER checked against its "
                                   "source bits; K > 128: launches of 128 resident batches, step k decoding "
                                   "batch k % 128); kernel_ms is per batch = launch time / K",
                           "launch_ms": {b["name"]: round(t, 4) for b, t in zip(batches, launch_ms)},
                           "input_bytes_resident": {b["name"]: b["inps"].numel() for b in batches}},
                "kernel_ms": {b["name"]: round(k, 4) for b, k in zip(batches, kms)},
                "step_minus_kernels_us": round((ms_per_step - sum(kms)) * 1e3, 2),
                "warmup_steps_run": nwarm,
                "kernel_gbps": {b["name"]: round(b["msg"] / (k * 1e-3) / 1e9, 2) for b, k in zip(batches, kms)},
                "ber": {b["name"]: bers[i] for i, b in enumerate(batches)},
                "ber_is": "max over the K batches of a launch",
                "kernels": {b["name"]: b["dec"].kernel_for(b["input_num"], sizes[0], b["llr"]) for b in batches},
            },
            "roofline": {
                "bound": "valu",
                "bound_note": "VALU issue binds (add-compare-select, no MFMA); achieved/peak/frac are the HBM "
                              "view north_star asks for, valu holds the binding view",
                "kernel": rl[di]["kernel"],
                "achieved": rl[di]["achieved"],
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": rl[di]["frac"],
                "traffic": rl[di]["traffic"],
                "algorithmic_bytes_per_batch": rl[di]["algorithmic_bytes_per_batch"],
                "per": "one 32M-bit batch (launch time / batches per launch); traffic likewise per batch",
                "traffic_source": f"profiles/{PMC_ROUND}/pmc_summary.json (FETCH_SIZE x2 + WRITE_SIZE, per batch)",
                "valu": rl[di]["valu"],
                "int_op_roofline": {
                    "what": "SURVEY 8d: 256 int16 ops per decoded bit (64 ACS x {2 add, 1 max, 1 decision}) "
                            "against the packed int16 lane-op peak, 2 x 1024 SIMDs x 32 lanes x 2.4 GHz (SURVEY "
                            "8d: x2 for packed int16; a 2-cycle wave64 op on two chunks' halves). Not the binding "
                            "view: max / DPP forms take 4 cycles, so valu.mix_ceiling (the ACS-only ablation) is",
                    "ops_per_bit": OPS_PER_BIT,
                    "achieved_tops": round(OPS_PER_BIT * batches[di]["msg"] / (kms[di] * 1e-3) / 1e12, 2),
                    "peak_tops": round(VALU_PEAK_TOPS_PACKED, 2),
                    "frac": round(OPS_PER_BIT * batches[di]["msg"] / (kms[di] * 1e-3) / 1e12 / VALU_PEAK_TOPS_PACKED, 3),
                    "frac_vs_unpacked_peak": round(OPS_PER_BIT * batches[di]["msg"] / (kms[di] * 1e-3) / 1e12
                                                   / VALU_PEAK_TOPS, 3),
                },
                "per_kernel": {b["name"]: rl[i] for i, b in enumerate(batches)},
            },
            "checksums": [[hex(x) for x in g[:nw]] for g in gathered],
            "checksums_are": "per rank, per workload: xor of the decoded words over every resident batch",
        }
        if llr is not None:
            result["config"]["llr_input"] = llr
        if pcie is not None:
            result["config"]["pcie_inclusive"] = pcie
        if chan is not None:
            result["config"]["channel_source"] = chan
        if other is not None:
            result["config"]["other_configs"] = other
        if single is not None:
            result["config"]["single_launch"] = single
        if final_gather is not None:
            result["config"]["final_gather"] = final_gather
        if not metric_run:
            result["config"]["profiling_workloads"] = names
        if REHEARSE:
            result["config"]["rehearsal"] = "not a measurement: every rank decodes on the same GPU"
        if checks is not None:
            result["config"]["parity"] = parity_block(checks)
        if not args.no_cpu_baseline and metric_run and world == 1:  # rank 0 at N = 1 only (the bench contract)
            result["cpu_baseline"] = cpu_baseline(batches)
        print(json.dumps(result), flush=True)

    for b in batches:
        b["dec"].close()
    torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
