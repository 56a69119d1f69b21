"""The N>1 bench path (orb_slam_amd/dist.py) on CPU: two gloo ranks, each
with its own shard; elapsed = max over ranks, work = sum (weak scaling)."""
import os
import socket

import numpy as np
import pytest
import torch.distributed as tdist
import torch.multiprocessing as mp

from orb_slam_amd import dist as odist, synth


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world), RANK=str(rank),
                      LOCAL_RANK=str(rank))
    tdist.init_process_group("gloo", rank=rank, world_size=world)
    w, r, lr = odist.env()
    frames = synth.sequence(64, 48, 2, seed=odist.shard_seed(2000, r))
    stats = [1.0 + r, 10.0 * (r + 1), float(frames.sum() % 997), 0.0]
    allst = odist.gather_stats(stats, tdist)
    rate, elapsed, work = odist.job_rate(allst)
    q.put((r, w, allst.tolist(), rate, elapsed, work))
    tdist.barrier()
    tdist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_multi_rank_gather_and_job_rate(world):
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    for r, w, allst, rate, elapsed, work in res:
        assert w == world
        a = np.array(allst)
        assert a.shape == (world, 4)
        # value = work of all ranks / the slowest rank's time (rank r: 1 + r s, 10 (r + 1) units)
        assert elapsed == float(world) and work == 5.0 * world * (world + 1) and rate == 5.0 * (world + 1)
        assert len(set(a[:, 2])) == world   # ranks own different sequences
    assert all(res[k][2] == res[0][2] for k in range(world))


def test_single_process_path():
    a = odist.gather_stats([2.0, 8.0])
    assert a.shape == (1, 2)
    assert odist.job_rate(a) == (4.0, 2.0, 8.0)
