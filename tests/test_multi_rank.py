"""CPU tests of the multi-GPU partition: world_size-2 gloo processes partition the group space exactly as
bench.py's ranks do, compute their share (here with the oracle, since no GPU is present), and the
combined result equals the single-rank result -- the property the N-GPU bench relies on (no group
lost or duplicated, no data-path collective).  The same property through the product (bench.py under
torch.distributed.run on the GPU) is tests/test_gpu_multirank.py."""
from __future__ import annotations

import hashlib
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from kcptube_amd.partition import combine_digests, group_range


def test_group_range_covers_exactly():
    for total in (0, 1, 7, 1 << 20, 8 << 20):
        for world in (1, 2, 3, 4, 8):
            spans = [group_range(total, world, r) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == total
            for (a, b), (c, d) in zip(spans, spans[1:]):
                assert b == c and a <= b
            sizes = [b - a for a, b in spans]
            assert max(sizes) - min(sizes) <= 1
    with pytest.raises(ValueError):
        group_range(10, 2, 2)


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, total, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oracle import Oracle
    o = Oracle()
    K, N, B, seed = 10, 13, 64, 0x5EED0003
    g0, g1 = group_range(total, world, rank)
    data = o.synth(seed, N, B, g0, g1 - g0, 0, K)
    par = o.encode_batch(K, N, data, B)
    masks = o.erasure_masks(seed, g1 - g0, N, N, 3, random_max=3, g0=g0)
    out, idx, st = o.decode_batch(K, N, data, par, masks, B)
    out[idx == 0xFF] = 0
    dig = hashlib.sha256(par.tobytes() + out.tobytes()).hexdigest()
    digs = [None] * world
    dist.all_gather_object(digs, dig)
    import torch
    t = torch.tensor([float(g1 - g0)])
    dist.all_reduce(t)
    if rank == 0:
        with open(os.path.join(out_dir, "res.txt"), "w") as f:
            f.write(combine_digests(digs) + " " + str(int(t.item())))
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_gloo_partition_matches_single_rank(tmp_path, oracle):
    total = 37
    port = _free_port()
    mp.spawn(_worker, args=(2, port, total, str(tmp_path)), nprocs=2, join=True)
    combined, n = open(tmp_path / "res.txt").read().split()
    assert int(n) == total
    # single-rank reference: same per-range digests computed in one process
    K, N, B, seed = 10, 13, 64, 0x5EED0003
    digs = []
    for r in range(2):
        g0, g1 = group_range(total, 2, r)
        data = oracle.synth(seed, N, B, g0, g1 - g0, 0, K)
        par = oracle.encode_batch(K, N, data, B)
        masks = oracle.erasure_masks(seed, g1 - g0, N, N, 3, random_max=3, g0=g0)
        out, idx, st = oracle.decode_batch(K, N, data, par, masks, B)
        out[idx == 0xFF] = 0
        digs.append(hashlib.sha256(par.tobytes() + out.tobytes()).hexdigest())
    assert combined == combine_digests(digs)
    # and the partition is a partition: the whole range in one go gives the same parity bytes
    data = oracle.synth(seed, N, B, 0, total, 0, K)
    par_all = oracle.encode_batch(K, N, data, B)
    g0, g1 = group_range(total, 2, 1)
    par_1 = oracle.encode_batch(K, N, oracle.synth(seed, N, B, g0, g1 - g0, 0, K), B)
    np.testing.assert_array_equal(par_all[g0:g1], par_1)


def test_bench_gpus_must_match_the_world(tmp_path):
    """`--gpus 3` inside a launcher-formed world of 1 is refused before any device work."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "3", "--no-cpu"], env=env,
                       capture_output=True, text=True, timeout=60)
    assert r.returncode == 2 and "world of 1" in r.stderr


def test_bench_spawns_one_process_per_rank(tmp_path):
    """bench.spawn_ranks (what `bench.py --gpus N` does without a launcher) starts N processes with the
    torch.distributed.run environment, one shared 127.0.0.1 rendezvous, and distinct ranks."""
    import sys
    import bench
    script = ("import os, sys; e = os.environ; "
              "open(os.path.join(sys.argv[1], e['RANK']), 'w').write("
              "' '.join(e[k] for k in ('RANK', 'LOCAL_RANK', 'WORLD_SIZE', 'MASTER_ADDR', 'MASTER_PORT')))")
    env_before = dict(os.environ)
    rc = bench.spawn_ranks([sys.executable, "-c", script, str(tmp_path)], 4, poll_s=0.05)
    assert rc == 0 and dict(os.environ) == env_before
    rows = [open(tmp_path / str(r)).read().split() for r in range(4)]
    assert [row[:3] for row in rows] == [[str(r), str(r), "4"] for r in range(4)]
    assert {row[3] for row in rows} == {"127.0.0.1"} and len({row[4] for row in rows}) == 1


def test_bench_spawn_fails_when_a_rank_fails():
    """One failing rank fails the job, and a peer left waiting (it would block in a barrier) is ended."""
    import sys
    import time
    import bench
    script = "import os, sys, time; r = int(os.environ['RANK']); time.sleep(60) if r == 0 else sys.exit(5)"
    t0 = time.time()
    rc = bench.spawn_ranks([sys.executable, "-c", script], 2, poll_s=0.05)
    assert rc == 5 and time.time() - t0 < 30


def test_bench_rank_groups_partition_the_global_space():
    """bench.py's own rank slicing (weak scaling: groups_per_gpu x world, split by group_range) tiles the
    global group space exactly, for every world size the driver runs."""
    import bench
    for per_gpu in (1, 4096, 1 << 20):
        for world in (1, 2, 4, 8):
            spans = [bench.rank_groups(per_gpu, world, r) for r in range(world)]
            assert all(t == per_gpu * world for _, _, t in spans)
            assert spans[0][0] == 0 and spans[-1][1] == per_gpu * world
            for (a, b, _), (c, d, _) in zip(spans, spans[1:]):
                assert b == c
            assert all(b - a == per_gpu for a, b, _ in spans)


def test_bench_refuses_oversubscription_without_rehearsal():
    """More ranks than visible GPUs is refused (exit 2) before the rendezvous, unless the run says it is a
    rehearsal; n_gpus then counts devices.  (CPU: no GPU is visible, so even one rank is refused.)"""
    import subprocess
    import sys
    import bench
    assert bench.check_devices(8, 8, False) is None
    assert bench.check_devices(2, 8, False) is None
    assert "only 1 visible GPU" in bench.check_devices(8, 1, False)
    assert bench.check_devices(8, 1, True) is None
    assert bench.check_devices(1, 0, True) == "no GPU visible"
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0", KFEC_BENCH_REHEARSAL="0")
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--no-cpu"], env=env,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 2 and "bench.py:" in r.stderr


def test_bench_device_check_counts_ranks_per_node():
    """bench.py compares LOCAL_WORLD_SIZE (ranks on this node), not the global world, with the node's GPUs:
    2 nodes x 4 GPUs (world 8, 4 local ranks) is allowed on a 4-GPU node, 8 local ranks are not."""
    import bench
    assert bench.check_devices(4, 4, False) is None
    assert "only 4 visible" in bench.check_devices(8, 4, False)


def test_per_rank_summary():
    """The multi-rank evidence: distinct devices over every rank, and value / (world x rank 0's own rate)."""
    import bench
    recs = [{"rank": r, "device": f"h{r // 4}:dev{r % 4}", "wall_ms_per_step": 10.0 + r, "groups": 100}
            for r in range(8)]
    payload = [1 << 30] * 8  # 1 GiB per rank per step
    value = 8 * (1 << 30) / 0.017 / 2**30  # what bench.py reports: all payload / the slowest rank's time
    s = bench.per_rank_summary(recs, value, payload)
    assert s["devices"] == 8 and s["slowest_rank"] == 7
    assert abs(s["rank0_equivalent_GiBps"] - 100.0) < 1e-6
    assert abs(s["scaling_efficiency"] - 10.0 / 17.0) < 1e-3
    one_dev = [dict(r, device="h0:dev0") for r in recs]  # a rehearsal: every rank on one GPU
    assert bench.per_rank_summary(one_dev, value, payload)["devices"] == 1
