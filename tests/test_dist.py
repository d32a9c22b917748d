"""Multi-GPU path on CPU: world_size-2 gloo ranks run bench.py's control-plane
helpers (barrier, MAX / SUM over ranks) and the byte-balanced shard partition
(independent shards, no data-path collective)."""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from tas_amd import pktgen, shard


def test_shard_ranges_uniform():
    for n, w in ((8 * (1 << 20), 8), (10, 3), (0, 2), (5, 8)):
        r = shard.shard_ranges(n, w)
        assert len(r) == w and r[0][0] == 0 and r[-1][1] == n
        assert all(a <= b for a, b in r) and all(r[i][1] == r[i + 1][0] for i in range(w - 1))
        sizes = [b - a for a, b in r]
        assert max(sizes) - min(sizes) <= 1


def test_shard_ranges_mixed_balanced_by_bytes():
    lens = pktgen.mixed_lengths(1 << 20, seed=3)
    for w in (1, 2, 4, 8):
        r = shard.shard_ranges(lens, w)
        assert r[0][0] == 0 and r[-1][1] == lens.size
        assert all(r[i][1] == r[i + 1][0] for i in range(w - 1))
        b = shard.shard_bytes(lens, r)
        assert sum(b) == int(lens.astype(np.int64).sum())
        # every shard within one max-size packet of the ideal share
        ideal = sum(b) / w
        assert max(abs(x - ideal) for x in b) <= 9000
    with pytest.raises(ValueError):
        shard.shard_ranges(10, 0)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bench
    try:
        bench.barrier(world)
        lens = pktgen.mixed_lengths(4096, seed=7)
        a, b = shard.shard_ranges(lens, world)[rank]
        my_bytes = float(lens[a:b].astype(np.int64).sum())
        tot = bench.sum_over_ranks(my_bytes, world)
        mx = bench.max_over_ranks(float(rank + 1) * 1.5, world)
        bench.barrier(world)
        q.put((rank, a, b, tot, mx))
    finally:
        dist.destroy_process_group()


def test_gloo_world2_aggregation():
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
    lens = pktgen.mixed_lengths(4096, seed=7)
    total = float(lens.astype(np.int64).sum())
    assert res[0][1] == 0 and res[0][2] == res[1][1] and res[1][2] == 4096
    for _, _, _, tot, mx in res:
        assert tot == total
        assert mx == 3.0


def test_bench_cli_defaults():
    import bench
    a = bench.parse([])
    assert a.gpus == 1 and a.workload == "tcp4" and a.steps > 0 and a.warmup >= 0
    a = bench.parse(["--gpus", "8", "--steps", "5", "--warmup", "1", "--workload", "shard8m"])
    assert (a.gpus, a.steps, a.warmup, a.workload) == (8, 5, 1, "shard8m")
