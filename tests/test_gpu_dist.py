"""bench.py's collectives on the GPU: a 1-rank RCCL (backend "nccl") group on cuda:0, in a fresh process.

The same functions the N > 1 bench runs -- max over ranks, the checksum all_gather and the
gather of decoded words to rank 0 -- on cuda tensors, so the first multi-GPU run is not their first run.
The world-size-2 form of the same logic runs over gloo in tests/test_dist.py."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

_SCRIPT = r"""
import json, os, sys
import numpy as np
import torch
sys.path.insert(0, os.environ["VD_ROOT"])
import bench
bench.init_ranks(1, 0)
dev = torch.cuda.current_device()
m = bench.max_over_ranks(1.25, dev)
g = bench.gather_checksums([0xDEAD0001, 0xBEEF0002, 7], dev, 1)
gen = torch.Generator(device="cuda")
gen.manual_seed(7)
outs = [torch.randint(0, 256, (16384,), dtype=torch.uint8, device=dev, generator=gen),
        torch.randint(0, 256, (4096,), dtype=torch.uint8, device=dev, generator=gen)]
ms, sums, err = bench.gather_outputs(outs, dev, 1, 0)
want = [int(np.bitwise_xor.reduce(o.cpu().numpy().view(np.uint32))) for o in outs]
torch.distributed.destroy_process_group()
print(json.dumps({"max": m, "sums": g, "gather": sums, "want": want, "err": err, "ms": ms,
                  "backend": "nccl"}))
"""


@pytest.mark.gpu
def test_rccl_one_rank_collectives_on_cuda_tensors():
    env = dict(os.environ, VD_ROOT=ROOT)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, "-c", _SCRIPT], capture_output=True, text=True, timeout=180, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    d = json.loads(r.stdout.strip().splitlines()[-1])
    assert d["err"] is None
    assert d["max"] == 1.25
    assert d["sums"] == [[0xDEAD0001, 0xBEEF0002, 7]]
    assert d["gather"] == [d["want"]] and d["want"][0] != 0


def _bench_json(cmd, env):
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-3000:]
    return json.loads(lines[0])


@pytest.mark.gpu
def test_batch_shard_rehearsal_equals_one_rank():
    """configs[3]'s batch sharding rehearsed on one GPU: 4 ranks (torch.distributed.run), each decoding its own
    batch on cuda:0 with the collectives over gloo (bench.py REHEARSE), against one rank decoding the same 4
    batches (seeds: batch i = 2 (rank + world step) + workload).  The per-rank checksums XOR to the one-rank
    run's, whose parity block checks batches 0 and 3 against the oracle, and the final gather reaches rank 0
    with every rank's words intact."""
    import bench
    flags = ["--warmup", "1", "--warm-s", "0", "--no-cpu-baseline", "--no-llr", "--no-pcie", "--no-channel",
             "--no-other"]
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT", "VD_BENCH_REHEARSE_SHARED_GPU"):
        env.pop(k, None)
    one = _bench_json([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "4", *flags], env)
    world = 4
    shard = _bench_json([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
                         "--master-addr", "127.0.0.1", "--master-port", str(bench.free_port()),
                         os.path.join(ROOT, "bench.py"), "--gpus", str(world), "--steps", "1", *flags],
                        dict(env, VD_BENCH_REHEARSE_SHARED_GPU="1"))
    assert shard["n_gpus"] == world and shard["config"]["rehearsal"]
    assert shard["config"]["parallelism"].startswith("rehearsal")
    assert all(v["mismatches"] == 0 for v in one["config"]["parity"]["paths"].values()), one["config"]["parity"]
    assert all(v["mismatches"] == 0 for v in shard["config"]["parity"]["paths"].values()), shard["config"]["parity"]
    cs = [[int(x, 16) for x in r] for r in shard["checksums"]]
    assert len(cs) == world
    want = [int(x, 16) for x in one["checksums"][0]]
    for w in range(len(want)):
        acc = 0
        for r in range(world):
            acc ^= cs[r][w]
        assert acc == want[w], (w, [hex(c[w]) for c in cs], hex(want[w]))
    fg = shard["config"]["final_gather"]
    assert fg["world"] == world and fg["checksums_match"] is True, fg
