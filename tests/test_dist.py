"""Multi-process (gloo, world_size 2, CPU) coverage of bench.py's multi-GPU logic: per-rank
shards, max-over-ranks timing and the counter merge (RCCL on GPU, gloo here).  Each rank's
per-GPU counters come from the oracle on that rank's shard (the checker stands in for the
GPU here), and the merged counters must equal the oracle's counters over the union."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _shard(rank):
    import pktgen
    rows, frames = pktgen.parity_set(seed=1000 + rank, n=300)
    return rows, frames


def _worker(rank, world, port, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "tests"), os.path.join(root, "dpdk-tcpipstack_amd")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world))
    import torch
    import torch.distributed as dist
    import bench
    import oracle
    import pktgen
    dist.init_process_group("gloo", rank=rank, world_size=world)
    rows, frames = _shard(rank)
    arena, off, lens = pktgen.pack_arena(frames)
    tcb, live = pktgen.table_arrays(rows)
    _, cnt = oracle.rx_batch(arena, off, lens, tcb, live)
    merged = bench.merge_counters(cnt, torch.device("cpu"))
    tmax = bench.max_over_ranks(float(rank + 1) * 0.5, torch.device("cpu"))
    tmin = bench.min_over_ranks(float(rank + 1) * 0.5, torch.device("cpu"))
    seeds = [bench.shard_seed(0x5EED0001, r) for r in range(world)]
    tsum = bench.sum_over_ranks(len(frames), torch.device("cpu"))
    bench.barrier(torch.device("cpu"))
    q.put((rank, merged.tolist(), tmax, tmin, seeds, tsum))
    dist.destroy_process_group()


def test_two_rank_counter_merge_and_timing():
    import oracle
    import pktgen
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    total = np.zeros(16, dtype=np.uint64)
    for r in range(world):
        rows, frames = _shard(r)
        arena, off, lens = pktgen.pack_arena(frames)
        tcb, live = pktgen.table_arrays(rows)
        total += oracle.rx_batch(arena, off, lens, tcb, live)[1]
    for rank, merged, tmax, tmin, seeds, tsum in out:
        assert merged == total.tolist()
        assert tsum == sum(len(_shard(r)[1]) for r in range(world))  # the value's numerator
        assert tmax == pytest.approx(1.0)  # max over ranks of (rank+1)/2
        assert tmin == pytest.approx(0.5)  # min over ranks (roofline kernel_us spread)
        assert len(set(seeds)) == world     # independent shard per rank


def test_cpu_replicas_split_the_sample():
    """bench.cpu_replicas: independent oracle processes over disjoint ranges of one sample."""
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "dpdk-tcpipstack_amd")]
    import bench
    import pktgen
    rows, frames = pktgen.parity_set(seed=7, n=200)
    arena, off, lens = pktgen.pack_arena(frames)
    tcb, live = pktgen.table_arrays(rows)
    r = bench.cpu_replicas(arena, off, lens, tcb, live, cores=2, seconds=0.5)
    assert r is not None and r["cores"] == 2 and r["mpps"] > 0 and r["gbs"] > 0
