"""N > 1 path on the CPU: world sizes 2, 3 and 8 over gloo (127.0.0.1). Each rank verifies its
shard (here with the oracle, the CPU checker, since the container has no GPU; on the box
bench.py does the same with the kernels) and the verdict bitmaps are gathered; the result
must equal the single-process bitmap bit for bit. World 8 with n = 300 leaves ranks 5..7
with empty shards and rank 4 with a ragged one (the driver's 8-GPU split,
worker/src/worker.rs:158-169 being the reference's own per-worker split)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from narwhal_amd.shard import gather_bitmaps, shard_range


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _corpus(n):
    from oracle import oracle as O
    rng = np.random.Generator(np.random.PCG64(3))
    ks = O.keys(4)
    msgs = rng.integers(0, 256, size=(n, 32), dtype=np.uint8)
    pks = np.array([np.frombuffer(ks[i % 4][0], np.uint8) for i in range(n)])
    sigs = np.array([np.frombuffer(O.sign(ks[i % 4][1], msgs[i].tobytes()), np.uint8)
                     for i in range(n)])
    sigs[rng.choice(n, n // 7, replace=False), 40] ^= 1
    return msgs, pks, sigs


def _worker(rank, world, port, n, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oracle import oracle as O
    msgs, pks, sigs = _corpus(n)
    s, e = shard_range(n, rank, world)
    st = O.verify_strict_many(msgs[s:e], pks[s:e], sigs[s:e], nthreads=1)
    bits = np.zeros(((e - s + 63) // 64) * 64, dtype=np.uint8)
    bits[: e - s] = (st == 0)
    words = torch.from_numpy(np.packbits(bits, bitorder="little").view(np.int64).copy())
    full = gather_bitmaps(words, n, world)
    t = torch.tensor([float(rank + 1)])
    dist.all_reduce(t, op=dist.ReduceOp.MAX)      # bench's max-over-ranks timing
    if rank == 0:
        q.put((full.numpy().tobytes(), float(t.item())))
    dist.barrier()
    dist.destroy_process_group()


def test_shard_range_partitions():
    for n in (0, 1, 63, 64, 65, 1000, 12_500_000):
        for w in (1, 2, 3, 8):
            rs = [shard_range(n, r, w) for r in range(w)]
            assert rs[0][0] == 0 and rs[-1][1] == n
            for (a, b), (c, d) in zip(rs, rs[1:]):
                assert b == c and a <= b
            assert all(s % 64 == 0 or s == n for s, _ in rs)


@pytest.mark.timeout(300)
@pytest.mark.parametrize("world,n", [(2, 300), (3, 1000), (8, 300), (8, 1000)])
def test_gloo_bitmap_gather(world, n):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n, q)) for r in range(world)]
    for p in procs:
        p.start()
    full, tmax = q.get(timeout=240)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    sizes = [shard_range(n, r, world) for r in range(world)]
    if world == 8 and n == 300:
        assert [e - s for s, e in sizes] == [64, 64, 64, 64, 44, 0, 0, 0]
    from oracle import oracle as O
    msgs, pks, sigs = _corpus(n)
    st = O.verify_strict_many(msgs, pks, sigs, nthreads=1)
    ref = np.packbits((st == 0).astype(np.uint8), bitorder="little").tobytes()
    assert full == ref
    assert tmax == float(world)
