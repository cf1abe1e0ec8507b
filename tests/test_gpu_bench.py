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
