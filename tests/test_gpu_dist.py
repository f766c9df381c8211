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
