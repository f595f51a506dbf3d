"""One rank of the multi-process sharding tests (test_multi_gpu_sharding.py and
test_gpu_parity.py): the configs[3] split by packet index, run through the
PRODUCT library on this rank's shard only, gathered over gloo for the check.

    RANK=r WORLD_SIZE=w MASTER_ADDR=127.0.0.1 MASTER_PORT=p python tests/shard_rank.py MODE N OUTDIR

MODE "emu": the CPU-emulated build of the product kernels (HYOBFS_LIB points at
tests/emu/libhyobfs_emu.so; buffers are host memory).  MODE "gpu": the HIP
library on cuda:(rank mod visible devices), device tensors.  Each rank obfuscates
its byte-balanced share of an N-datagram bimodal batch (hysteria_amd.shard, the
split bench.py uses) into a packed output; the gather is test-side only, the data
path has no collective.  Rank 0 writes the joined wire to OUTDIR/joined.bin.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

from oracle import salamander_ref as ref  # noqa: E402  (inputs only: seeded streams)


def main():
    mode, n, outdir = sys.argv[1], int(sys.argv[2]), sys.argv[3]
    import torch
    import torch.distributed as dist
    from hysteria_amd.salamander import SalamanderObfuscator
    from hysteria_amd.shard import byte_balanced_split

    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dist.init_process_group("gloo", rank=rank, world_size=world)
    lens = ref.bimodal_lengths(3, 0, n)
    first, cnt = byte_balanced_split(lens, world, rank)
    my = lens[first:first + cnt].astype(np.uint32)
    start = int(lens[:first].sum())                      # this shard's offset in the input stream
    in_off = np.zeros(cnt, np.uint64)
    if cnt:
        in_off[1:] = np.cumsum(my[:-1], dtype=np.uint64)
    inp = np.frombuffer(ref.stream_bytes(1, start, int(my.sum()) + 16), np.uint8).copy()
    salts = ref.splitmix64_array(2, first, cnt).astype(np.uint64)
    cap = int(my.sum()) + 8 * cnt
    out = np.zeros(cap + 16, np.uint8)
    o = SalamanderObfuscator(b"average_password", 0 if mode == "emu" else rank % torch.cuda.device_count())
    if mode == "emu":
        p = lambda a: a.ctypes.data  # noqa: E731
        o.obfuscate_batch(p(inp), cnt, in_off=p(in_off), in_len=p(my), salts=p(salts), out=p(out), out_cap=cap,
                          stream=0)
    else:
        dev = torch.device("cuda", rank % torch.cuda.device_count())
        t = lambda a, dt: torch.from_numpy(a.view(dt)).to(dev)  # noqa: E731
        d_out = torch.zeros(cap + 16, dtype=torch.uint8, device=dev)
        o.obfuscate_batch(t(inp, np.uint8), cnt, in_off=t(in_off, np.int64), in_len=t(my, np.int32),
                          salts=t(salts, np.int64), out=d_out, out_cap=cap)
        torch.cuda.synchronize(dev)
        out = d_out.cpu().numpy()
    o.close()
    parts = [None] * world
    dist.all_gather_object(parts, out[:cap].tobytes())   # test-side check only, not the data path
    if rank == 0:
        with open(os.path.join(outdir, "joined.bin"), "wb") as f:
            f.write(b"".join(parts))
    dist.barrier()
    dist.destroy_process_group()
    print(f"rank {rank} ok")


if __name__ == "__main__":
    main()
