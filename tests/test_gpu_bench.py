"""bench.py's single-GPU line as the driver reads it: one JSON line on stdout, the roofline with every
same-run ceiling -- the linear read, calib_mix at several occupancies, the product kernel's own arithmetic-free build
(tools/libkfec_arithfree.so) at several occupancies -- and the verification flag, for an encode+decode config and the
decode-only one.  Small batches: this checks the measurement path, not the numbers."""
from __future__ import annotations

import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("config", ["20:3", "10:3dec"])
def test_bench_line_carries_the_same_run_ceilings(config):
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    r = subprocess.run([sys.executable, "bench.py", "--config", config, "--groups", "16384", "--steps", "3", "--warmup", "1",
                        "--no-cpu"], cwd=ROOT, capture_output=True, text=True, timeout=240,
                       env=dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0"))
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["verified_bit_exact"] and d["n_gpus"] == 1 and d["value"] > 0
    roof = d["roofline"]
    assert roof["bound"] == "hbm" and 0 < roof["frac"] < 1.2 and roof["read_ceiling"] > 0
    # the arithmetic-free build of the product kernel ran, at its own occupancy and capped
    af = roof["arithfree_ms_by_occupancy"]
    assert roof["arithfree_ms"] and set(af) >= {"own", "4w", "3w", "2w"} and all(v > 0 for v in af.values())
    assert set(roof["mix_calib_GBps_by_occupancy"]) >= {"own", "4w", "3w", "2w"}
    # the mix ceiling is the fastest candidate, and says which one it was
    best_af = roof["algorithmic_bytes_per_launch"] / (min(af.values()) * 1e-3) / 1e9
    best = max(best_af, max(roof["mix_calib_GBps_by_occupancy"].values()))
    assert abs(roof["mix_ceiling"] - best) <= 0.002 * best
    assert roof["mix_ceiling_kind"] in ("arithfree", "calib_mix")
    assert roof["frac_of_mix_ceiling"] == pytest.approx(roof["achieved"] / roof["mix_ceiling"], rel=2e-3)


@pytest.mark.parametrize("K,N", [(20, 23), (8, 12), (40, 60), (200, 255)])
def test_arithfree_build_has_no_gf_arithmetic(K, N):
    """The ceiling build must not carry any of the product's GF arithmetic (a paired or burst MAC branch that forgot
    the XOR-only knob would make the 'ceiling' the product itself): its every parity row is the plain XOR of the
    group's data shards."""
    import ctypes
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    path = os.path.join(ROOT, "tools", "libkfec_arithfree.so")
    assert os.path.exists(path), "build it first: kcptube_amd.build.build_tools()"
    lib = ctypes.CDLL(path)
    vp, sz = ctypes.c_void_p, ctypes.c_size_t
    lib.kfec_create.argtypes = [sz, sz, ctypes.POINTER(vp)]
    lib.kfec_destroy.argtypes = [vp]
    lib.kfec_encode_batch.argtypes = [vp, sz, sz, sz, vp, vp, vp]
    ctx = vp()
    assert lib.kfec_create(K, N, ctypes.byref(ctx)) == 0
    try:
        G, B = 96, 1440
        gen = torch.Generator().manual_seed(K * 1000 + N)
        data = torch.randint(0, 256, (G, K, B), dtype=torch.uint8, generator=gen).cuda()
        parity = torch.zeros((G, N - K, B), dtype=torch.uint8, device="cuda")
        st = torch.cuda.current_stream()
        assert lib.kfec_encode_batch(ctx, G, B, B, data.data_ptr(), parity.data_ptr(), vp(st.cuda_stream)) == 0
        torch.cuda.synchronize()
        x = data[:, 0].clone()
        for j in range(1, K):
            x ^= data[:, j]
        assert torch.equal(parity, x.unsqueeze(1).expand(G, N - K, B))
    finally:
        lib.kfec_destroy(ctx)


def test_bench_line_200_55_is_priced_against_the_paired_mac_bound():
    """fec=200:55 is VALU-bound: the line's roofline is byte-MACs/s against the issue bound of the paired perm MAC
    the 8-row kernels use (6 v_perm_b32 + 3 v_bitop3_b32 per 8 byte-MACs), with the single-shard form's bound kept
    beside it; the arithmetic-free build of the encode, the HBM side's ceiling, must be far faster than the product."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    r = subprocess.run([sys.executable, "bench.py", "--config", "200:55", "--groups", "16384", "--steps", "2",
                        "--warmup", "1", "--no-cpu"], cwd=ROOT, capture_output=True, text=True, timeout=240,
                       env=dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0"))
    assert r.returncode == 0, r.stderr[-3000:]
    d = json.loads(r.stdout.strip().splitlines()[-1])
    roof = d["roofline"]
    assert d["verified_bit_exact"] and roof["bound"] == "valu" and roof["unit"] == "byte-MAC/s"
    assert roof["issue_bound_single"] < roof["peak"]  # the paired form issues fewer instructions per byte-MAC
    assert 0 < roof["frac"] < 1 and roof["frac"] < roof["frac_of_single_bound"]
    assert roof["arithfree_ms"] < 0.5 * d["encode_ms"]
