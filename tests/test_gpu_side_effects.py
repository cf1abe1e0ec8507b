"""What the resident per-call worker (kcptube_amd/csrc/kfec_worker.hip) does to the rest of the process.

* While one thread keeps calling kfec_encode, another thread's coder lifecycle (reset, create + destroy), an
  AEAD cipher and a batch queue created and destroyed, a raw hipMalloc/hipFree, hipHostMalloc/hipHostFree and a
  hipDeviceSynchronize must each return within a stated bound (BOUND_MS), while the calling thread keeps
  getting correct parity.  (HIP's frees and device syncs wait for every stream of the device, the worker's
  included; the worker's lease, KFEC_WORKER_LEASE_US, is what bounds them.)  tools/side_effects.cpp does the
  timing; round 4 measured ~370 ms for each of these before the lease (profiles/r04_side_effects.json).
* The 2 s "did not answer" fallback: with KFEC_WORKER_TEST_DEAF=1 the worker ignores every request; the first
  call must then come back from the launch path with the reference's bytes, the process must print one
  warning, serve no request through the worker, and exit promptly.
"""
from __future__ import annotations

import json
import os
import subprocess
import sys
import textwrap
import time

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BOUND_MS = 50.0
OPS = ["kfec_reset", "kfec_create_destroy", "kfec_aead_create_destroy", "kfec_txq_create_destroy",
       "hipMalloc_hipFree", "hipHostMalloc_hipHostFree", "hipDeviceSynchronize"]


@pytest.fixture(scope="module")
def gpu():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    exe = os.path.join(ROOT, "tools", "side_effects")
    if not os.path.exists(exe):
        pytest.skip("tools/side_effects not built (kcptube_amd.build.build_tools)")
    return exe


def test_device_wide_syncs_are_bounded_while_calls_continue(gpu):
    r = subprocess.run([gpu, "400"] + OPS, cwd=ROOT, capture_output=True, text=True, timeout=120,
                       env=dict(os.environ, KFEC_WORKER="1"))
    assert r.returncode == 0, r.stdout + r.stderr
    rows = [json.loads(line) for line in r.stdout.splitlines() if line.startswith("{")]
    assert [row["op"] for row in rows] == OPS
    for row in rows:
        assert row["a_ok"] and row["a_running_at_start"], row
        assert row["ms"] < BOUND_MS, row
        # the other thread was still calling when the operation returned: it did not wait for the calls to stop
        assert row["a_running_at_end"], row
        assert row["a_calls"] > 1000, row


@pytest.mark.parametrize("poll", ["1", "0"])
def test_worker_that_does_not_answer_falls_back_to_the_launch_path(oracle, poll):
    """Both poll modes: direct (every workgroup polls the host line) and relay (KFEC_WORKER_POLL=0: the followers
    poll workgroup 0's device-memory relay, whose quit value the deaf knob must not swallow, or they spin on and
    the process cannot exit)."""
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    script = textwrap.dedent("""
        import sys, time
        sys.path.insert(0, %r)
        import numpy as np
        from kcptube_amd import FecCode
        from kcptube_amd.fec import worker_requests
        from oracle import Oracle
        K, N, B = 20, 23, 1440
        rng = np.random.default_rng(7)
        data = rng.integers(0, 256, K * B, dtype=np.uint8).tobytes()
        c = FecCode(K, N)
        t0 = time.time()
        par = c.encode(data, len(data), B)
        t_first = time.time() - t0
        assert par == Oracle().encode(K, N, data, B)
        shares = {i: data[i * B:(i + 1) * B] for i in range(3, K)}
        shares.update({K + r: par[r] for r in range(3)})
        got = c.decode(shares, B)
        assert {i: bytes(v) for i, v in got.items()} == {i: data[i * B:(i + 1) * B] for i in range(3)}
        print("first_call_s %%.3f requests %%d" %% (t_first, worker_requests()))
        del c
    """ % ROOT)
    env = dict(os.environ, KFEC_WORKER_TEST_DEAF="1", KFEC_WORKER_POLL=poll)
    env.pop("KFEC_WORKER", None)  # default mode: fall back (KFEC_WORKER=1 would make it an error)
    t0 = time.time()
    r = subprocess.run([sys.executable, "-c", script], cwd=ROOT, capture_output=True, text=True, timeout=120,
                       env=env)
    elapsed = time.time() - t0
    assert r.returncode == 0, r.stdout + r.stderr
    assert "resident worker did not answer; using the launch path" in r.stderr
    assert r.stderr.count("did not answer") == 1
    first_s, requests = r.stdout.split()[1], int(r.stdout.split()[3])
    assert requests == 0
    assert 1.9 < float(first_s) < 5.0  # the 2 s wait, then the launch path
    assert elapsed < 60, elapsed  # process exit does not hang on the ignored worker


def test_worker_that_does_not_answer_is_an_error_when_required():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    script = textwrap.dedent("""
        import sys
        sys.path.insert(0, %r)
        from kcptube_amd import FecCode
        from kcptube_amd.fec import KfecError
        c = FecCode(4, 6)
        try:
            c.encode(bytes(4 * 64), 4 * 64, 64)
        except KfecError as e:
            print("error", e)
    """ % ROOT)
    env = dict(os.environ, KFEC_WORKER_TEST_DEAF="1", KFEC_WORKER="1")
    r = subprocess.run([sys.executable, "-c", script], cwd=ROOT, capture_output=True, text=True, timeout=120,
                       env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.startswith("error"), r.stdout + r.stderr
