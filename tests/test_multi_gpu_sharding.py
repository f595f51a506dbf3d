"""Multi-GPU path on CPU: the packet-index shards of hysteria_amd.shard cover the
batch exactly once, and W = 2 ranks under torch.distributed (gloo), each running
the oracle on its own shard, produce outputs whose concatenation is the
single-process output.  The GPU path uses the same shard functions (bench.py)."""
import os
import socket

import numpy as np
import pytest

from hysteria_amd.shard import byte_balanced_split, even_split, weak_shard
from oracle import salamander_ref as ref

PSK = b"average_password"


@pytest.mark.parametrize("n,world", [(0, 1), (1, 2), (7, 3), (1000, 8), (1 << 20, 8), (5, 8)])
def test_even_split_partitions(n, world):
    seen = 0
    for r in range(world):
        first, cnt = even_split(n, world, r)
        assert first == seen
        seen += cnt
        assert cnt in (n // world, n // world + 1)
    assert seen == n


def test_byte_balanced_split_partitions_and_balances():
    lens = ref.bimodal_lengths(3, 0, 100_000)
    for world in (1, 2, 3, 8):
        seen, shares = 0, []
        for r in range(world):
            first, cnt = byte_balanced_split(lens, world, r)
            assert first == seen
            seen += cnt
            shares.append(int(lens[first:first + cnt].sum()) + 8 * cnt)   # weight len + 8
        assert seen == lens.size
        assert max(shares) - min(shares) <= 2 * (1350 + 8)


def test_weak_shard():
    assert weak_shard(1 << 20, 3) == (3 << 20, 1 << 20)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank_main(rank, world, port, outdir):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    co = ref.COracle()
    n = 3000
    lens = ref.bimodal_lengths(3, 0, n)
    first, cnt = byte_balanced_split(lens, world, rank)
    my = lens[first:first + cnt]
    start = int(lens[:first].sum())                     # this shard's offset in the input stream
    in_off = np.zeros(cnt, np.uint64)
    in_off[1:] = np.cumsum(my[:-1], dtype=np.uint64)
    inp = co.fill_stream(1, start, int(my.sum()) + 16)
    salts = co.salts(2, first, cnt)
    cap = int(my.sum()) + 8 * cnt
    out, _, _, tot = co.batch(True, PSK, cnt, inp, in_off=in_off, in_len=my, salts=salts, out_cap=cap)
    assert tot == cap
    parts = [None] * world
    dist.all_gather_object(parts, out.tobytes())      # test-side check only, not the data path
    if rank == 0:
        with open(os.path.join(outdir, "joined.bin"), "wb") as f:
            f.write(b"".join(parts))
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_two_ranks_shards_concatenate_to_whole(tmp_path):
    import torch.multiprocessing as mp
    world = 2
    mp.spawn(_rank_main, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    co = ref.COracle()
    n = 3000
    lens = ref.bimodal_lengths(3, 0, n)
    in_off = np.zeros(n, np.uint64)
    in_off[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
    inp = co.fill_stream(1, 0, int(lens.sum()) + 16)
    whole, _, _, _ = co.batch(True, PSK, n, inp, in_off=in_off, in_len=lens, salts=co.salts(2, 0, n),
                              out_cap=int(lens.sum()) + 8 * n)
    assert (tmp_path / "joined.bin").read_bytes() == whole.tobytes()


@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_c_abi_shard_bounds_match_host_mirror(world):
    """hyobfs_shard_bounds (C ABI, host-only) and hysteria_amd.shard give the same ranges."""
    from hysteria_amd.shard import shard_bounds
    lens = ref.bimodal_lengths(3, 0, 20_000)
    b = shard_bounds(lens, lens.size, world)
    assert b == [byte_balanced_split(lens, world, r)[0] for r in range(world)] + [lens.size]
    for n in (0, 1, 7, 1 << 20):
        u = shard_bounds(None, n, world)
        assert u == [even_split(n, world, r)[0] for r in range(world)] + [n]
