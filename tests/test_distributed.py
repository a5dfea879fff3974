"""World-size-2 gloo rehearsal of the point-sharded path (msm_amd/dist.py) on CPU.

Each rank's shard MSM is computed by the oracle here (no GPU in this container) and shipped in
the same 32-word projective partial format libmsm's msm_compute_device_partial produces; the
gather / join code under test is the one bench.py runs over RCCL."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, n, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "webgpu-msm_amd")]
    import torch.distributed as dist
    from msm_amd.dist import shard_range, gather_partials, combine_on_root
    from oracle import oracle as O

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    lo, hi = shard_range(n, rank, world)
    ss = O.xorshift_scalars(n)[lo:hi]
    x, y = O.closed_form_msm(range(lo + 1, hi + 1), ss) if hi > lo else O.IDENTITY
    z = 3 + rank  # ship a non-normalised projective partial, as the GPU path does
    part = np.zeros(32, np.uint32)
    for j, v in enumerate((x * z % O.P, y * z % O.P, x * y % O.P * z % O.P, z)):
        part[8 * j: 8 * j + 8] = O.int_to_be_words(v)
    parts = gather_partials(part)
    res = combine_on_root(parts, rank)
    if rank == 0:
        q.put(res)
    dist.destroy_process_group()


@pytest.mark.parametrize("world,n", [(2, 1000), (2, 1), (3, 4096)])
def test_sharded_join_gloo(world, n):
    from oracle import oracle as O
    from msm_amd.dist import shard_range

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = q.get(timeout=180)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res == O.closed_form_msm(range(1, n + 1), O.xorshift_scalars(n))
    assert sum(b - a for a, b in (shard_range(n, r, world) for r in range(world))) == n


def _batch_worker(rank, world, port, n, k, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "webgpu-msm_amd")]
    import torch.distributed as dist
    from msm_amd.dist import shard_range, gather_partials, combine_batch_on_root
    from oracle import oracle as O

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    lo, hi = shard_range(n, rank, world)
    parts = np.zeros((k, 32), np.uint32)
    for b in range(k):  # K different MSMs: scalar seeds differ per MSM
        ss = O.xorshift_scalars(n, seed=1000 + b)[lo:hi]
        x, y = O.closed_form_msm(range(lo + 1, hi + 1), ss) if hi > lo else O.IDENTITY
        z = 2 + rank + b
        for j, v in enumerate((x * z % O.P, y * z % O.P, x * y % O.P * z % O.P, z)):
            parts[b, 8 * j: 8 * j + 8] = O.int_to_be_words(v)
    res = combine_batch_on_root(gather_partials(parts), rank)
    if rank == 0:
        q.put(res)
    dist.destroy_process_group()


@pytest.mark.parametrize("world,n,k", [(2, 500, 3), (3, 100, 2)])
def test_sharded_batch_join_gloo(world, n, k):
    # the pipelined multi-GPU bench path: K partials per rank, one all_gather, K joins on rank 0
    from oracle import oracle as O

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_batch_worker, args=(r, world, port, n, k, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = q.get(timeout=180)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res == [O.closed_form_msm(range(1, n + 1), O.xorshift_scalars(n, seed=1000 + b)) for b in range(k)]


def test_batched_join_matches_per_msm_join():
    """msm_combine_partials_many (one inversion for the batch) == msm_combine_partials per MSM,
    on projective partials with Z != 1 (host code only, no GPU)."""
    import msm_amd as M
    from oracle import oracle as O

    world, count = 5, 7
    rng = np.random.default_rng(5)
    parts = np.zeros((world, count, 32), np.uint32)
    for w in range(world):
        for k in range(count):
            x, y = O.scalar_mul(O.G, int(rng.integers(1, 2**60)))
            z = int(rng.integers(2, 2**62))
            vals = (x * z % O.P, y * z % O.P, x * y % O.P * z % O.P, z)  # (xz, yz, xyz, z)
            parts[w, k] = np.concatenate([O.int_to_be_words(v) for v in vals])
    got = M.combine_partials_many(parts)
    for k in range(count):
        assert got[k] == M.combine_partials(parts[:, k, :])
    exp0 = O.IDENTITY
    for w in range(world):
        z = O.be_words_to_int(parts[w, 0, 24:32])
        zi = O.inv(z)
        exp0 = O.aff_add(exp0, (O.be_words_to_int(parts[w, 0, 0:8]) * zi % O.P, O.be_words_to_int(parts[w, 0, 8:16]) * zi % O.P))
    assert got[0] == exp0
