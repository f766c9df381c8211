"""world_size-2 `gloo` tests (CPU) of bench.py's multi-GPU host logic.

The decode path shards by independent batches: each rank synthesises and decodes its own batches,
there is no collective on the data path, the step time is the max over ranks and the only
cross-rank traffic is one all_gather of per-rank checksums after the timed region.  The same
functions run under RCCL on the GPU box (bench.py under torch.distributed.run)."""
import os
import socket
import sys

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _outs(rank):
    return [torch.arange(16, dtype=torch.uint8) * 3 + 40 * rank, torch.arange(8, dtype=torch.uint8) + 7 * rank + 1]


def _xor_words(t):
    import numpy as np
    return int(np.bitwise_xor.reduce(t.numpy().view(np.uint32)))


def _worker(rank, world, port, q):
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bench
    elapsed = 1.0 + rank  # rank 1 is the slow one
    m = bench.max_over_ranks(elapsed, "cpu")
    sums = [0xDEAD0000 + rank, 0xBEEF0000 + rank]  # uint32 checksums, as bench computes them
    g = bench.gather_checksums(sums, "cpu", world)
    seeds = [bench.rank_seed(rank, wi) for wi in range(2)]
    # the final gather of decoded words (uint8 buffers, as the decode writes them) to rank 0
    outs = _outs(rank)
    _, gs, err = bench.gather_outputs(outs, "cpu", world, rank)
    assert err is None
    # one rank cannot build its buffers (torch.cat of nothing raises): both ranks skip the collective
    _, gs2, err2 = bench.gather_outputs(outs if rank == 0 else [], "cpu", world, rank)
    assert gs2 is None and err2
    q.put((rank, m, g, seeds, gs))
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_gloo_sharding():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, m, g, seeds, gs in res:
        assert m == 2.0  # max over ranks
        assert g == [[0xDEAD0000, 0xBEEF0000], [0xDEAD0001, 0xBEEF0001]]
        if rank == 0:  # rank 0 received every rank's words intact
            want = [[_xor_words(o) for o in _outs(r)] for r in range(world)]
            assert gs == want and want[0] != want[1]
        else:
            assert gs is None
    all_seeds = [s for _, _, _, seeds, _ in res for s in seeds]
    assert len(set(all_seeds)) == len(all_seeds)  # every rank decodes independent batches


def test_aggregate_is_whole_job():
    sys.path.insert(0, ROOT)
    import bench
    # 2 ranks x 2 batches x 31,999,936 bits in 1 step of 1 ms -> 256 Gb/s whole-job
    assert bench.aggregate_gbps(2 * 31_999_936, 2, 1, 1e-3) == pytest.approx(127.999744)
    assert bench.stages_per_launch(0x0, 64_000_000) == 1598 * 5088 + 4802 * 5056


def _bench(*args, env=None):
    import subprocess
    e = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        e.pop(k, None)
    e.update(env or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], capture_output=True, text=True,
                          timeout=180, env=e)


def test_gpus_flag_launches_one_rank_per_gpu():
    """`bench.py --gpus 2` (the driver's form) starts 2 ranks itself when no launcher set WORLD_SIZE
    (here over gloo with --ranks-check, which touches no GPU)."""
    import json
    r = _bench("--gpus", "2", "--ranks-check")
    assert r.returncode == 0, r.stderr[-2000:]
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["n_gpus"] == 2
    assert sorted(x["rank"] for x in line["ranks"]) == [0, 1]
    assert sorted(x["local_rank"] for x in line["ranks"]) == [0, 1]


def test_gpus_flag_must_match_launcher_world():
    r = _bench("--gpus", "4", "--ranks-check", env={"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0 and "--gpus 4 but WORLD_SIZE=2" in r.stderr
    r = _bench("--gpus", "0", "--ranks-check")
    assert r.returncode != 0
