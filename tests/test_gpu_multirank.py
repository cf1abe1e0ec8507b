"""SURVEY 8(e) through the product: bench.py's multi-rank path as the driver launches it
(torch.distributed.run, one process per rank, gloo barrier + max-reduce, group_range partition), with two
ranks sharing the box's one GPU.  The per-part digests of the recovered bytes, combined in part order,
must equal a single-rank run over the same global groups: no group lost, duplicated or changed."""
from __future__ import annotations

import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _last_json(stdout: str) -> dict:
    for line in reversed(stdout.strip().splitlines()):
        line = line.strip()
        if line.startswith("{"):
            return json.loads(line)
    raise AssertionError("no JSON line in:\n" + stdout[-2000:])


def _run(cmd, parts, rehearsal=True, timeout=240):
    # the box has one GPU: several ranks on it is a rehearsal, which bench.py refuses unless told so
    env = dict(os.environ, KFEC_BENCH_DIGEST=str(parts), HSA_ENABLE_IPC_MODE_LEGACY="0", PYTHONUNBUFFERED="1",
               KFEC_BENCH_REHEARSAL="1" if rehearsal else "0")
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, f"rc={r.returncode}\n{r.stdout[-3000:]}\n{r.stderr[-3000:]}"
    # the contract: rank 0 prints ONE JSON line and nothing else reaches stdout (gloo's rendezvous chatter, the
    # runtime's messages go to stderr) -- under torch.distributed.run too
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1 and lines[0].startswith("{"), r.stdout[-2000:]
    return _last_json(r.stdout)


@pytest.mark.parametrize("config", ["20:3", "10:3dec"])
def test_bench_two_ranks_match_single_rank(config):
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    per_gpu = 4096
    common = ["--config", config, "--no-cpu", "--steps", "2", "--warmup", "1"]
    two = _run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "bench.py", "--gpus", "2",
                "--groups", str(per_gpu)] + common, parts=2)
    one = _run([sys.executable, "bench.py", "--gpus", "1", "--groups", str(2 * per_gpu)] + common, parts=2)
    n_dev = torch.cuda.device_count()
    assert two["n_gpus"] == min(2, n_dev) and one["n_gpus"] == 1  # n_gpus counts devices, not ranks
    assert two["config"]["ranks"] == 2 and two["config"]["rehearsal"] == (n_dev < 2)
    assert two["verified_bit_exact"] and one["verified_bit_exact"]
    assert two["config"]["global_groups"] == one["config"]["global_groups"] == 2 * per_gpu
    assert two["recovered_shards_per_step"] == one["recovered_shards_per_step"] > 0
    assert two["combined_digest"] == one["combined_digest"]
    assert two["value"] > 0


def test_bench_gpus_flag_spawns_the_ranks_itself():
    """`python bench.py --gpus 2` (the driver's plain form, no launcher) forms a world of 2 ranks by itself
    and its result equals the single-rank run over the same global groups."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    common = ["--config", "20:3", "--no-cpu", "--steps", "2", "--warmup", "1"]
    two = _run([sys.executable, "bench.py", "--gpus", "2", "--groups", "4096"] + common, parts=2)
    one = _run([sys.executable, "bench.py", "--gpus", "1", "--groups", "8192"] + common, parts=2)
    assert two["config"]["ranks"] == 2 and two["verified_bit_exact"]
    assert two["n_gpus"] == min(2, torch.cuda.device_count())
    assert two["config"]["global_groups"] == 8192
    assert two["combined_digest"] == one["combined_digest"]


def test_bench_eight_ranks_match_single_rank():
    """Config 5's partition (BASELINE configs[4]: 8 ranks, independent group ranges, no collective) rehearsed on
    the box's GPU(s): `bench.py --gpus 8` with 2048 groups per rank must verify bit-exact and give the same
    combined digest (KFEC_BENCH_DIGEST=8, one SHA-256 per rank's range) as one rank over all 16384 groups."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    common = ["--config", "20:3", "--steps", "2", "--warmup", "1"]
    # the CPU leg runs at N > 1 too (rank 0, after every rank's GPU work): a small sample here
    eight = _run([sys.executable, "bench.py", "--gpus", "8", "--groups", "2048", "--cpu-seconds", "1",
                  "--cpu-groups", "1024"] + common, parts=8, timeout=300)
    one = _run([sys.executable, "bench.py", "--gpus", "1", "--groups", "16384", "--no-cpu"] + common, parts=8)
    assert eight["verified_bit_exact"] and one["verified_bit_exact"]
    assert eight["config"]["ranks"] == 8 and eight["n_gpus"] == min(8, torch.cuda.device_count())
    assert eight["config"]["global_groups"] == one["config"]["global_groups"] == 16384
    assert eight["recovered_shards_per_step"] == one["recovered_shards_per_step"] == 3 * 16384
    assert eight["combined_digest"] == one["combined_digest"]
    # per-rank evidence for the driver's SCALE runs: every rank's own event-timed kernels and device
    pr = eight["per_rank"]
    assert [r["rank"] for r in pr] == list(range(8))
    assert all(r["encode_ms"] > 0 and r["decode_ms"] > 0 and r["groups"] == 2048 for r in pr)
    assert eight["multi_rank"]["devices"] == eight["n_gpus"]
    assert 0 < eight["multi_rank"]["scaling_efficiency"] <= 1.5
    # every rank measured its own GPU's ceilings and reports its own fractions (north_star: per-GPU roofline)
    for r in pr:
        assert 0 < r["frac"] < 1.5 and r["read_ceiling"] > 0 and r["mix_ceiling"] > 0
        assert r["frac_of_ceiling"] > 0 and r["frac_of_mix_ceiling"] > 0
    # the reference CPU path in the same run, at N > 1 as at N = 1
    cb = eight["cpu_baseline"]
    assert cb and "error" not in cb, cb
    assert cb["value"] > 0 and cb["cores"] >= 1 and cb["kind"] in ("reference", "port")


def test_bench_refuses_more_ranks_than_gpus():
    """Without the rehearsal flag, more ranks than visible GPUs is an error (exit 2) before any device work."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    n = torch.cuda.device_count()
    env = dict(os.environ, KFEC_BENCH_REHEARSAL="0", HSA_ENABLE_IPC_MODE_LEGACY="0")
    r = subprocess.run([sys.executable, "bench.py", "--gpus", str(n + 1), "--groups", "64", "--no-cpu", "--steps", "1",
                        "--warmup", "0"], cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 2 and "visible GPU" in r.stderr
