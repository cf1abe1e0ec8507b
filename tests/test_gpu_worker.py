"""The resident per-call worker (kcptube_amd/csrc/kfec_worker.hip): kfec_encode / kfec_decode on one group
from host memory without a launch per call, against the oracle (fecpp.cpp:495-513, 518-587).

Covers the shapes at the worker's limits (R <= 16 parity / missing rows, (K + R) * pitch <= 36 KiB,
R * K <= 512) and just past them (the launch path takes those), inconsistent shares, block sizes
that are not multiples of 16, concurrent callers on more coders than slots, the idle exit and relaunch,
and that the worker and the launch path (KFEC_WORKER=0) give the same bytes.
"""
from __future__ import annotations

import hashlib
import os
import subprocess
import sys
import threading

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from kcptube_amd import load_library
    load_library()
    return torch.device("cuda:0")


def _roundtrip(c, oracle, K, N, B, rng, n_lost=None, corrupt=False):
    data = rng.integers(0, 256, K * B, dtype=np.uint8).tobytes()
    par = c.encode(data, len(data), B)
    assert par == oracle.encode(K, N, data, B), (K, N, B)
    shards = {i: data[i * B:(i + 1) * B] for i in range(K)}
    for r, p in enumerate(par):
        shards[K + r] = p
    R = N - K
    m = R if n_lost is None else n_lost
    lost = set(rng.choice(K, m, replace=False).tolist()) if m else set()
    sub = {s: shards[s] for s in range(N) if s not in lost}
    if corrupt:
        k = sorted(sub)[int(rng.integers(len(sub)))]
        sub[k] = bytes(x ^ 0xA5 for x in sub[k])
    got = c.decode(sub, B)
    assert got == oracle.decode(K, N, sub, B), (K, N, B, sorted(lost))
    if not corrupt:
        assert got == {i: shards[i] for i in sorted(lost)}


@pytest.mark.parametrize("K,N,B", [
    (1, 2, 1), (2, 3, 15), (20, 23, 1440), (10, 13, 1400), (20, 23, 1442), (5, 6, 17),
    (8, 24, 1440),     # R = 16, (K + R) * 1440 = 33.75 KiB: at the row limit
    (32, 48, 128),     # R * K = 512: at the table limit, 16 missing
    (8, 25, 1440),     # R = 17: past the row limit (launch path)
    (26, 29, 1440),    # (K + R) * pitch > 36 KiB (launch path)
    (33, 49, 16),      # R * K > 512 (launch path)
])
def test_worker_shapes_vs_oracle(dev, oracle, K, N, B):
    from kcptube_amd import FecCode
    from kcptube_amd.fec import worker_requests
    rng = np.random.default_rng(K * 1000 + N + B)
    c = FecCode(K, N)
    R = N - K
    n0 = worker_requests()
    losses = sorted({0, 1, min(R, K)}) + [min(R, K)]
    for i, m in enumerate(losses):
        _roundtrip(c, oracle, K, N, B, rng, n_lost=m, corrupt=i == len(losses) - 1)
    pitch = (B + 15) // 16 * 16
    W = int(os.environ.get("KFEC_WORKER_WGS", "8"))
    takes = R <= 16 and N * pitch <= 36 * 1024 and R * K <= 512 and K * (-(-(pitch // 16) // W)) * 16 <= 16 * 1024
    served = worker_requests() - n0
    if takes:  # every encode, and every decode that had a data shard to recover
        assert served == len(losses) + sum(1 for m in losses if m > 0), served
    else:
        assert served == 0, served


def test_worker_reset_reloads_tables(dev, oracle):
    """The worker caches the parity-row tables per matrix: a reset (new matrix, maybe at the same address)
    must not reuse them."""
    from kcptube_amd import FecCode
    rng = np.random.default_rng(3)
    c = FecCode(20, 23)
    for K, N in ((20, 23), (20, 24), (10, 13), (20, 23), (20, 22)):
        c.reset_martix(K, N)
        _roundtrip(c, oracle, K, N, 1440, rng)


def test_worker_concurrent_callers(dev, oracle):
    """More threads (each with its own coder) than worker slots: every result must be exact."""
    from kcptube_amd import FecCode
    errors = []

    def run(t):
        try:
            rng = np.random.default_rng(100 + t)
            K, N = [(20, 23), (10, 13), (8, 10), (30, 36)][t % 4]
            c = FecCode(K, N)
            for _ in range(40):
                _roundtrip(c, oracle, K, N, int(rng.integers(1, 1500)), rng, corrupt=bool(rng.random() < 0.2))
        except Exception as e:  # noqa: BLE001 - reported below
            errors.append(repr(e))

    ths = [threading.Thread(target=run, args=(t,)) for t in range(6)]
    for th in ths:
        th.start()
    for th in ths:
        th.join(timeout=120)
    assert not errors, errors[:3]


_DIGEST = r"""
import hashlib, sys, time
import numpy as np
sys.path.insert(0, {root!r})
from kcptube_amd import FecCode
h = hashlib.sha256()
rng = np.random.default_rng(42)
for trial in range(30):
    K = int(rng.integers(1, 30)); N = int(min(256, K + rng.integers(1, 8))); B = int(rng.integers(1, 1500))
    c = FecCode(K, N)
    data = rng.integers(0, 256, K * B, dtype=np.uint8).tobytes()
    par = c.encode(data, len(data), B)
    for p in par: h.update(p)
    shards = {{i: data[i * B:(i + 1) * B] for i in range(K)}}
    for r, p in enumerate(par): shards[K + r] = p
    keep = sorted(rng.choice(N, int(rng.integers(K, N + 1)), replace=False).tolist())
    for i, blk in sorted(c.decode({{s: shards[s] for s in keep}}, B).items()):
        h.update(bytes([i])); h.update(blk)
    if trial % 7 == 3: time.sleep(0.01)  # longer than the idle timeout below: the worker exits and relaunches
print(h.hexdigest())
"""


def test_worker_matches_launch_path_and_relaunches(dev):
    """Same bytes from the worker (with a 200 us idle timeout, so it exits and is relaunched many times), from
    the worker's other modes (requests in the pinned slot instead of device memory behind the BAR, full
    system-scope fences, every decode solve on the device) and from the launch path (KFEC_WORKER=0)."""
    code = _DIGEST.format(root=ROOT)
    outs = []
    other = {"KFEC_WORKER": "1", "KFEC_WORKER_BAR": "0", "KFEC_WORKER_FENCES": "0", "KFEC_WORKER_HOST_SOLVE": "0"}
    for env in ({"KFEC_WORKER": "1", "KFEC_WORKER_IDLE_US": "200"}, other, {"KFEC_WORKER": "0"}):
        e = dict(os.environ, **env)
        r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=180, env=e)
        assert r.returncode == 0, r.stderr[-2000:]
        outs.append(r.stdout.strip())
    assert outs[0] == outs[1] == outs[2] and len(outs[0]) == 64


def test_worker_stop_and_restart_with_coders(dev, oracle):
    """Destroying a device's last coder stops its workers (STOP doorbell, kernel joined); the next coder's first
    call relaunches them.  Repeated, with a ping in between (kfec_worker_ping)."""
    import gc
    from kcptube_amd import FecCode, load_library
    lib = load_library()
    rng = np.random.default_rng(9)
    for _ in range(3):
        gc.collect()  # (no other coder may be alive on the device for the stop to happen)
        c = FecCode(20, 23)
        assert lib.kfec_worker_ping(c._ctx) == 0
        _roundtrip(c, oracle, 20, 23, 1440, rng)
        del c
        gc.collect()


def test_worker_many_threads_random_shapes(dev, oracle):
    """8 threads, 2 slots, shapes inside and outside the worker's limits, decodes with inconsistent shares:
    every result equals the oracle's."""
    from kcptube_amd import FecCode
    errors = []

    def run(t):
        try:
            rng = np.random.default_rng(1000 + t)
            for _ in range(25):
                K = int(rng.integers(1, 40))
                N = int(min(256, K + rng.integers(1, 20)))
                B = int(rng.integers(1, 1600))
                c = FecCode(K, N)
                _roundtrip(c, oracle, K, N, B, rng, n_lost=int(rng.integers(0, min(N - K, K) + 1)),
                           corrupt=bool(rng.random() < 0.3))
        except Exception as e:  # noqa: BLE001 - reported below
            errors.append(repr(e)[:500])

    ths = [threading.Thread(target=run, args=(t,)) for t in range(8)]
    for th in ths:
        th.start()
    for th in ths:
        th.join(timeout=180)
    assert not errors, errors[:3]


def test_back_to_back_calls_across_leases(dev, oracle):
    """Continuous calls for ~25 worker leases (KFEC_WORKER_LEASE_US, 2 ms): workgroup 0 leaves at a lease only
    after a poll found no request pending, so no call waits for a relaunch plus a recompute of a request the
    other workgroups had already served; the tail stays bounded and every call is served by the worker."""
    import time
    from kcptube_amd import FecCode
    from kcptube_amd.fec import worker_requests
    K, N, B = 20, 23, 1440
    rng = np.random.default_rng(11)
    data = rng.integers(0, 256, K * B, dtype=np.uint8).tobytes()
    c = FecCode(K, N)
    exp = oracle.encode(K, N, data, B)
    assert c.encode(data, len(data), B) == exp
    r0 = worker_requests()
    times = []
    t_end = time.perf_counter() + 0.05
    while time.perf_counter() < t_end or len(times) < 500:
        t = time.perf_counter()
        p = c.encode(data, len(data), B)
        times.append(time.perf_counter() - t)
        if len(times) % 97 == 0:
            assert p == exp
    times.sort()
    assert worker_requests() - r0 == len(times)
    assert times[len(times) * 99 // 100] < 1e-3, times[-10:]
    assert times[-1] < 20e-3, times[-10:]
