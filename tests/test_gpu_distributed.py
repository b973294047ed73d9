"""The N > 1 bench path on the HIP kernels: two ranks, one process each,
sharing the box's one GPU over a gloo group (the driver's 8-GPU runs use RCCL through the
same code). Each rank uploads its contiguous shard of one global corpus, verifies it with
nw_dev_verify_strict_many on its own stream, and the per-shard verdict bitmaps (device
tensors) are gathered with narwhal_amd.shard.gather_bitmaps — exactly bench.py's run_strict.
Rank 0 compares the gathered bitmap with the oracle bit for bit.

The ranks are started as fresh child processes (multiprocessing "spawn"), never by
replacing a process that has touched the GPU."""
import ctypes
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _corpus(n):
    """Seeded mixed corpus (honest + tampered + s-high-bits), built with the oracle."""
    from oracle import oracle as O
    rng = np.random.Generator(np.random.PCG64(11))
    ks = O.keys(8)
    msgs = rng.integers(0, 256, size=(n, 32), dtype=np.uint8)
    pks = np.array([np.frombuffer(ks[i % 8][0], np.uint8) for i in range(n)])
    sigs = np.array([np.frombuffer(O.sign(ks[i % 8][1], msgs[i].tobytes()), np.uint8)
                     for i in range(n)])
    sigs[rng.choice(n, n // 9, replace=False), 40] ^= 1
    sigs[rng.choice(n, n // 13, replace=False), 63] |= 0x40
    return msgs, pks, sigs


def _rank(rank, world, port, n, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world))
    try:
        from narwhal_amd import _lib
        from narwhal_amd.shard import gather_bitmaps, shard_range
        dist.init_process_group("gloo", rank=rank, world_size=world)
        torch.cuda.set_device(0)
        dev = torch.device("cuda", 0)
        L = _lib.lib()
        assert L.nw_init() > 0 and L.nw_set_device(0) == 0
        msgs, pks, sigs = _corpus(n)
        s, e = shard_range(n, rank, world)
        m = torch.from_numpy(msgs[s:e].copy()).to(dev)
        p = torch.from_numpy(pks[s:e].copy()).to(dev)
        g = torch.from_numpy(sigs[s:e].copy()).to(dev)
        st = torch.empty(e - s, dtype=torch.int32, device=dev)
        bm = torch.zeros((e - s + 63) // 64 * 8, dtype=torch.uint8, device=dev)
        stream = torch.cuda.Stream(device=dev)
        torch.cuda.synchronize()
        P = lambda t: ctypes.c_void_p(t.data_ptr())
        rc = L.nw_dev_verify_strict_many(P(m), 32, P(p), P(g), e - s, P(st), P(bm),
                                         ctypes.c_void_p(stream.cuda_stream))
        assert rc == 0, L.nw_last_error()
        stream.synchronize()
        full = gather_bitmaps(bm.view(torch.int64), n, world)
        assert full.device == dev
        if rank == 0:
            q.put(("ok", full.cpu().numpy().tobytes(), st.cpu().numpy().tolist()))
        dist.barrier()
        dist.destroy_process_group()
    except Exception as ex:                     # report, do not hang the parent
        q.put(("error", repr(ex), None))
        raise


@pytest.mark.timeout(240)
def test_two_ranks_shard_verify_gather_on_gpu():
    from oracle import oracle as O
    n = 1500                                    # not a multiple of 64: a ragged last shard
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank, args=(r, 2, port, n, q)) for r in range(2)]
    for p in procs:
        p.start()
    try:
        kind, full, st0 = q.get(timeout=200)
    finally:
        for p in procs:
            p.join(60)
            if p.is_alive():
                p.kill()
    assert kind == "ok", full
    assert all(p.exitcode == 0 for p in procs)
    msgs, pks, sigs = _corpus(n)
    st = O.verify_strict_many(msgs, pks, sigs, nthreads=1)
    assert st0 == st[: len(st0)].tolist()       # rank 0's statuses == oracle
    ref = np.packbits((st == 0).astype(np.uint8), bitorder="little").tobytes()
    assert full == ref


_RCCL_CHILD = r"""
import os, sys
sys.path.insert(0, os.environ["NW_ROOT"])
import torch, torch.distributed as dist
from narwhal_amd.shard import gather_bitmaps, _gather_words
os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=os.environ["NW_PORT"], RANK="0",
                  WORLD_SIZE="1")
torch.cuda.set_device(0)
dist.init_process_group("nccl", rank=0, world_size=1)
dev = torch.device("cuda", 0)
words = torch.arange(7, dtype=torch.int64, device=dev) * 0x0101010101010101
out = _gather_words(words, 7 * 64, 1)            # the all_gather itself, on the device
assert out.device == dev and out.dtype == torch.uint8
assert torch.equal(out.view(torch.int64), words), (out, words)
full = gather_bitmaps(words, 7 * 64 - 5, 1)
assert full.numel() == (7 * 64 - 5 + 7) // 8
dist.destroy_process_group()
print("rccl ok")
"""


@pytest.mark.timeout(180)
def test_rccl_all_gather_on_device():
    """The RCCL ("nccl" backend) branch of gather_bitmaps on the box's one GPU: a one-rank
    process group, the device-tensor all_gather the driver's 8-GPU run performs (gloo
    stages through host memory; RCCL gathers device memory directly)."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, NW_ROOT=root, NW_PORT=str(_free_port()))
    p = subprocess.run([sys.executable, "-c", _RCCL_CHILD], env=env, capture_output=True,
                       text=True, timeout=170)
    assert p.returncode == 0 and "rccl ok" in p.stdout, p.stderr[-3000:]
