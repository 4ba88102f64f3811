"""The N>1 path on CPU: two gloo ranks shard chains, gather to rank 0.

Each rank runs its block of chains through the CPU oracle with the global
chain ids (the engine's RNG contract), gathers with gather_to_root, and rank 0
checks the result is bit-identical to one process running all chains.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from mlx_mcmc_amd.distributed import gather_to_root, max_over_ranks, shard, sum_over_ranks


def test_shard_plan_covers_chains_in_order():
    for C in (1, 7, 256, 2048):
        for world in (1, 2, 3, 8):
            blocks = [shard(C, world, r) for r in range(world)]
            assert sum(c for _, c in blocks) == C
            assert [o for o, _ in blocks] == list(np.cumsum([0] + [c for _, c in blocks])[:-1])


def _chains(offset, count):
    from oracle import ns
    from oracle import samplers as S

    out = []
    for c in range(offset, offset + count):
        r = S.hmc(lambda p: ns.Normal(1.0, 2.0).log_prob(p["x"]), {"x": 0.0}, num_samples=30,
                  num_warmup=20, num_leapfrog_steps=5, seed=9, chain=c, record=False)
        out.append(r.samples)
    return torch.tensor(np.stack(out))


def _worker(rank, world, port, C, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        off, cnt = shard(C, world, rank)
        mine = _chains(off, cnt)
        allc = gather_to_root(mine)
        t = max_over_ranks(float(rank + 1))
        n = sum_over_ranks(float(cnt))   # per-rank counts (NUTS leaves in bench.py)
        if rank == 0:
            q.put((allc.numpy(), t, n))
    finally:
        dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_two_rank_shards_match_single_process():
    C, world = 5, 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, C, q)) for r in range(world)]
    for p in procs:
        p.start()
    got, tmax, nsum = q.get(timeout=300)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    ref = _chains(0, C).numpy()
    np.testing.assert_array_equal(got, ref)
    assert tmax == 2.0
    assert nsum == C
