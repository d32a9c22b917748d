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


@pytest.mark.parametrize("world", [2, 8])
def test_gloo_world_aggregation(world):
    """bench.py's control plane at 2 ranks and at the driver's 8 (one process
    per GPU there): byte-balanced shards that tile the batch, the whole-job sum
    and the max over ranks."""
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
    assert res[0][1] == 0 and res[-1][2] == 4096
    assert all(res[r][2] == res[r + 1][1] for r in range(world - 1))
    for _, _, _, tot, mx in res:
        assert tot == total
        assert mx == world * 1.5


def test_bench_cli_defaults():
    import bench
    a = bench.parse([])
    assert a.gpus == 1 and a.workload == "tcp4" and a.steps > 0 and a.warmup >= 0
    a = bench.parse(["--gpus", "8", "--steps", "5", "--warmup", "1", "--workload", "shard8m"])
    assert (a.gpus, a.steps, a.warmup, a.workload) == (8, 5, 1, "shard8m")


def _bench(*args, timeout=180):
    import subprocess
    import sys
    from conftest import ROOT
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    return subprocess.run([sys.executable, str(ROOT / "bench.py"), *args], capture_output=True, text=True,
                          timeout=timeout, env=env, cwd=str(ROOT))


@pytest.mark.parametrize("n", [2, 8])
def test_bench_spawns_n_ranks_itself(n):
    """`bench.py --gpus N` with no launcher starts N rank processes of its own
    (here with the GPU-free control self-test: gloo barrier, MAX / SUM /
    gather over ranks); rank 0 prints the per-rank aggregate.  N = 8 is the
    driver's scaling run."""
    import json
    r = _bench("--gpus", str(n), "--control-selftest")
    assert r.returncode == 0, r.stderr[-2000:]
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["n_gpus"] == n and line["per_rank_value"] == [float(k + 1) for k in range(n)]
    assert line["sum"] == n * (n + 1) / 2 and line["max"] == float(n)
    assert line["ranks"] == [f"cpu{k}" for k in range(n)]


def test_bench_under_the_drivers_launcher_8_ranks():
    """The driver's own N > 1 command shape: torch.distributed.run with 8
    processes on one node, each rank reading RANK / WORLD_SIZE / MASTER_* from
    the environment (the GPU-free control self-test)."""
    import json
    import subprocess
    import sys
    from conftest import ROOT
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "8",
                        "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), str(ROOT / "bench.py"),
                        "--gpus", "8", "--control-selftest"], capture_output=True, text=True, timeout=300, env=env,
                       cwd=str(ROOT))
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [x for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1  # rank 0 alone prints
    line = json.loads(lines[0])
    assert line["n_gpus"] == 8 and line["per_rank_value"] == [float(k + 1) for k in range(8)]
    assert line["sum"] == 36.0 and line["max"] == 8.0


def test_bench_refuses_more_gpus_than_visible():
    """Fewer visible GPUs than --gpus is an error (no silent rehearsal)."""
    r = _bench("--gpus", "2", timeout=120)
    assert r.returncode == 2
    assert "needs 2 GPUs" in r.stderr and "--rehearse" in r.stderr


def test_bench_world_size_must_match_gpus():
    import subprocess
    import sys
    from conftest import ROOT
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "4", "--control-selftest"],
                       capture_output=True, text=True, timeout=120, env=env, cwd=str(ROOT))
    assert r.returncode != 0 and "WORLD_SIZE=2" in r.stderr


@pytest.mark.gpu
def test_bench_two_ranks_on_the_gpu_rehearsal():
    """The N > 1 bench path on the GPU box: `bench.py --gpus 2 --rehearse`
    starts two rank processes itself, each checksums its own 64K-frame batches
    on the GPU (here both share the one visible GPU, gloo control plane), and
    rank 0 prints the aggregate over both ranks (shards,
    no data-path collective)."""
    import json
    r = _bench("--gpus", "2", "--rehearse", "--steps", "5", "--warmup", "2", "--no-txseg", "--no-flow",
               "--no-contexts", "--no-flushmix", "--no-e2e", "--no-raw", "--no-cpu-baseline", "--no-pmc",
               timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][-1])
    assert line["n_gpus"] == 2 and len(line["per_rank_value"]) == 2 and line["ranks"]["rehearse"] is True
    assert line["kernel"] == "tcp4_tas14_kernel<hint>" and line["value"] > 0
    assert line["rx_verify"]["all_frames_verified"] is True
    # ranks sharing the GPU claim no pattern-ceiling or N x HBM fraction
    assert line["frac_of_n_hbm"] is None and line["roofline"]["pattern_ceiling"] is None


@pytest.mark.gpu
@pytest.mark.parametrize("workload", ["shard8m", "mixed"])
def test_bench_four_ranks_strong_scaling_rehearsal(workload):
    """The strong-scaling configs at N = 4 on the one-GPU box (`--rehearse`:
    four ranks share the GPU over gloo): the shards' packets and bytes add up
    to the config, contiguously; the mixed batch's shards are byte-balanced
    within one 9,000 B packet; `value` is all ranks' bytes over the slowest
    rank's time; and the rehearsal line claims no fraction above 1."""
    import json
    import bench
    ws = 4
    r = _bench("--gpus", str(ws), "--rehearse", "--workload", workload, "--steps", "5", "--warmup", "2",
               "--no-cpu-baseline", "--no-pmc", timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][-1])
    assert line["n_gpus"] == ws and line["ranks"]["rehearse"] is True and line["scaling"] == "strong"
    sh = line["shards"]
    if workload == "shard8m":
        total_n = bench.SHARD8M_N
        alg = [p * (bench.RAW_LEN + 2) for p in sh["packets"]]
        lens = None
    else:
        total_n = bench.MIXED_N
        lens = pktgen.mixed_lengths(total_n, seed=pktgen.SEED).astype(np.int64)
        ranges = shard.shard_ranges(lens, ws)
        alg = [int(lens[a:b].sum()) + 2 * (b - a) for a, b in ranges]
        ideal = lens.sum() / ws
        assert max(abs(int(lens[a:b].sum()) - ideal) for a, b in ranges) <= 9000
    assert sum(sh["packets"]) == total_n
    assert sh["first_packet"] == [int(v) for v in np.cumsum([0] + sh["packets"][:-1])]
    assert sh["bytes_per_step"] == alg
    # value: every rank's bytes over the slowest rank's K steps
    steps = line["steps"]
    exp = sum(alg) * steps / max(sh["seconds"]) / float(1 << 30)
    assert abs(line["value"] - exp) <= 0.01 * exp + 0.02

    def fracs(o):
        if isinstance(o, dict):
            for k, v in o.items():
                if "frac" in k and isinstance(v, (int, float)):
                    yield k, v
                yield from fracs(v)
        elif isinstance(o, list):
            for v in o:
                yield from fracs(v)
    assert line["frac_of_n_hbm"] is None
    assert all(v <= 1 for _, v in fracs(line)), list(fracs(line))

