"""Multi-process path of bench.py on CPU: world_size-2 gloo ranks shard the
object batch with no data-path collective, and the timing uses a barrier and
a max-reduce, as the MI355X run does over RCCL."""
import os
import socket

import pytest
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, total, q):
    import sys
    import time

    import torch
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    lo, hi = bench.shard_range(rank, world, total)
    dist.barrier()
    t0 = time.perf_counter()
    time.sleep(0.05 * (rank + 1))   # ranks finish at different times
    dist.barrier()
    elapsed = torch.tensor([time.perf_counter() - t0], dtype=torch.float64)
    dist.all_reduce(elapsed, op=dist.ReduceOp.MAX)
    cover = torch.zeros(total, dtype=torch.int32)
    cover[lo:hi] += 1
    dist.all_reduce(cover)   # test-only check that shards tile the batch
    q.put((rank, lo, hi, elapsed.item(), cover.tolist()))
    dist.destroy_process_group()


@pytest.mark.parametrize("world,total", [(2, 1024), (2, 7)])
def test_gloo_two_ranks_shard_and_time(world, total):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, total, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    spans = [(lo, hi) for _, lo, hi, _, _ in res]
    assert spans[0][0] == 0 and spans[-1][1] == total
    assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
    assert all(c == 1 for c in res[0][4])
    # max over ranks: everyone reports the slowest rank's time
    assert res[0][3] == res[1][3] and res[0][3] >= 0.1
