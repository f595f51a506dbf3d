"""Multi-GPU path on CPU: the packet-index shards of hysteria_amd.shard cover the
batch exactly once, and W = 2 ranks under torch.distributed (gloo), each running
the oracle on its own shard, produce outputs whose concatenation is the
single-process output.  The same split through the PRODUCT: two rank processes
each run their shard through the CPU-emulated build of the HIP library
(tests/emu, the kernel sources compiled for the host), and on the GPU tier
through the HIP library itself (test_gpu_two_rank_processes_product_shards).
The GPU path uses the same shard functions (bench.py)."""
import glob
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "emu"))
from emu_build import ensure_emu_lib  # noqa: E402

from hysteria_amd.shard import byte_balanced_split, check_rank_devices, even_split, weak_shard
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


def test_check_rank_devices():
    """bench.py's rank binding check: distinct cards pass; two ranks on one card are a
    flagged rehearsal when the node has fewer cards than ranks, and an error when it
    has a card per rank (a misconfigured LOCAL_RANK / HIP_VISIBLE_DEVICES)."""
    ids = [f"0000:{0x11 + 16 * i:02x}:00.0" for i in range(8)]
    assert check_rank_devices(ids, 8) is False
    assert check_rank_devices(ids[:1], 1) is False
    assert check_rank_devices([ids[0], ids[0]], 1) is True       # --gpus 2 on a one-card box
    with pytest.raises(RuntimeError, match="share"):
        check_rank_devices([ids[0], ids[1], ids[0], ids[3]], 8)
    with pytest.raises(RuntimeError):
        check_rank_devices([ids[0], ids[0]], 2)


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


def _run_ranks(mode, n, outdir, world=2, extra_env=None, timeout=300):
    """Start `world` rank processes of tests/shard_rank.py; rank 0 leaves joined.bin."""
    port = _free_port()
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), LOCAL_RANK=str(r), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), **(extra_env or {}))
        procs.append(subprocess.Popen([sys.executable, os.path.join(os.path.dirname(__file__), "shard_rank.py"),
                                       mode, str(n), str(outdir)], env=env, stdout=subprocess.PIPE,
                                      stderr=subprocess.STDOUT, text=True))
    outs = []
    for p in procs:
        try:
            outs.append(p.communicate(timeout=timeout)[0])
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
    assert all(p.returncode == 0 for p in procs), [o[-2000:] for o in outs]


def _oracle_whole(n):
    co = ref.COracle()
    lens = ref.bimodal_lengths(3, 0, n)
    in_off = np.zeros(n, np.uint64)
    in_off[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
    inp = co.fill_stream(1, 0, int(lens.sum()) + 16)
    whole, _, _, _ = co.batch(True, PSK, n, inp, in_off=in_off, in_len=lens, salts=co.salts(2, 0, n),
                              out_cap=int(lens.sum()) + 8 * n)
    return whole.tobytes()


def test_gloo_two_ranks_emulated_product_shards(tmp_path):
    """Two rank processes, each obfuscating its byte-balanced shard of a bimodal batch
    with the product kernels (CPU-emulated build, ASan); joined = the oracle's whole batch."""
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    lib = os.path.join(root, "tests", "emu", "libhyobfs_emu.so")
    asan = sorted(glob.glob("/opt/rocm/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so"))
    if not asan or not os.path.exists("/opt/rocm/llvm/bin/clang++"):
        pytest.skip("clang/ASan runtime not available")
    ensure_emu_lib()
    n = 2000
    _run_ranks("emu", n, tmp_path, extra_env={"HYOBFS_LIB": lib, "LD_PRELOAD": asan[-1],
                                              "ASAN_OPTIONS": "detect_leaks=0", "HYEMU_CUS": "2"})
    assert (tmp_path / "joined.bin").read_bytes() == _oracle_whole(n)


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 3])
def test_gpu_rank_processes_product_shards(tmp_path, world):
    """bench.py's N-process layout on the GPU box: `world` rank processes (ranks map to
    GPUs modulo the visible devices), each runs its shard of a 200k-datagram bimodal
    batch through the HIP library; the gathered wire equals the oracle's whole batch."""
    n = 200_000
    _run_ranks("gpu", n, tmp_path, world=world, timeout=110)
    assert (tmp_path / "joined.bin").read_bytes() == _oracle_whole(n)


def test_n_gt_1_bench_line_is_self_contained():
    """The N > 1 bench line the driver's 8-GPU run prints, as a one-card --gpus 2
    rehearsal on the final sources recorded it (profiles/r06_final/): BASELINE's metric,
    weak scaling over configs[3]'s 8M-datagram shard per rank, the roofline with the PMC
    traffic of that shard (profiles/pmc_traffic.json, keyed by the build id), every rank's
    PCI bus id and call time, the shared-card flag, and no CPU baseline (rank 0 at N = 1
    only).  Every key the driver and the judge read is checked."""
    import json
    ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    line = json.loads(open(os.path.join(ROOT, "profiles", "r06_final", "bench_n2_one_gpu_rehearsal.json")).read())
    base = json.load(open(os.path.join(ROOT, "BASELINE.json")))
    assert line["metric"] == base["metric"] and line["unit"] == "GiB/s" and line["higher_is_better"] is True
    assert line["n_gpus"] == 2 and line["scaling"] == "weak" and line["value"] > 0 and line["ms_per_step"] > 0
    assert line["steps"] > 0 and line["warmup"] >= 0 and line["vs_baseline"] is None and line["dtype"] == "u8"
    cfg = line["config"]
    assert cfg["datagrams_per_gpu"] == 1 << 23 and cfg["global_datagrams"] == 2 << 23 and cfg["datagram_len"] == 1200
    roof = line["roofline"]
    assert roof["bound"] == "hbm" and roof["unit"] == "GB/s" and roof["peak"] == 8000.0
    assert roof["traffic"] and roof["traffic_over_algorithmic"] < 1.05   # the 8M shard's PMC entry
    assert roof["kernel_src_sha"] == roof["lib_build_id"]
    assert abs(roof["frac"] - roof["achieved"] / roof["peak"]) < 1e-3
    assert roof["algorithmic_bytes_per_launch"] == (1 << 23) * (2 * 1200 + 16)
    ranks = line["ranks"]
    assert [r["rank"] for r in ranks] == [0, 1]
    assert all(len(r["pci_bus_id"]) >= 12 and r["obf_call_ms"] > 0 for r in ranks)
    assert line["devices_shared"] is True   # the rehearsal ran both ranks on one card
    assert line["cpu_baseline"] is None and len(line["per_gpu_GiBs"]) == 2
    assert "deobfuscate" in line and line["deobfuscate"]["frac"] > 0
