"""GPU parity tests: the HIP coder (through the C ABI) against the oracle and the reference's golden data.

Bar: bit-exact.  Sizes the oracle finishes in seconds are compared byte for byte; the full-size configs
of BASELINE.json are checked through size-independent properties (encode -> erase -> decode round trip
recovers every erased shard; digests of digests).  Absent shard slots are filled with garbage before
every decode, so a kernel that read an erased slot would fail.
"""
from __future__ import annotations

import hashlib
import os
import subprocess

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from kcptube_amd import load_library
    load_library()  # must load: no fallback exists
    return torch.device("cuda:0")


def _np(t):
    return t.cpu().numpy()


def _masks_u64(t):
    return _np(t).view(np.uint64)


def _present_sets(masks: np.ndarray, N: int):
    out = []
    for g in range(masks.shape[0]):
        out.append([s for s in range(N) if int(masks[g, s >> 6]) >> (s & 63) & 1])
    return out


# ---------------------------------------------------------------------------------------------------
# golden fixtures (generated from the compiled reference coder)
# ---------------------------------------------------------------------------------------------------
def test_enc_matrix_golden(dev, golden):
    from kcptube_amd import FecCode
    _, arrs = golden
    for key in arrs.files:
        if not key.startswith("enc_"):
            continue
        _, K, N = key.split("_")
        c = FecCode(int(K), int(N))
        np.testing.assert_array_equal(c.enc_matrix(), arrs[key], err_msg=key)


def test_tiny_encode_decode_golden(dev, golden):
    from kcptube_amd import FecCode
    meta, arrs = golden
    for case in meta["tiny_cases"]:
        K, N, B, key = case["K"], case["N"], case["B"], case["key"]
        c = FecCode(K, N)
        data = arrs[key + "_in"].tobytes()
        par = c.encode(data, len(data), B)
        assert b"".join(par) == arrs[key + "_par"].tobytes(), key
        shards = {i: data[i * B:(i + 1) * B] for i in range(K)}
        for r, p in enumerate(par):
            shards[K + r] = p
        for pi in range(case["n_patterns"]):
            present = arrs[f"{key}_d{pi}_present"].tolist()
            out = c.decode({s: shards[s] for s in present}, B)
            ids = arrs[f"{key}_d{pi}_ids"].tolist()
            assert sorted(out) == ids, (key, pi)
            assert b"".join(out[i] for i in ids) == arrs[f"{key}_d{pi}_out"].tobytes(), (key, pi)


def test_selection_rule_golden(dev, golden):
    """with > K shares the missing row uses the highest-id share; corrupting an unused share
    changes nothing, corrupting the used one changes the output exactly as in the reference."""
    from kcptube_amd import FecCode
    meta, arrs = golden
    K, N, B = 20, 23, 64
    c = FecCode(K, N)
    data = arrs["sel_in"].tobytes()
    par = c.encode(data, len(data), B)
    shards = {i: data[i * B:(i + 1) * B] for i in range(K)}
    for r, p in enumerate(par):
        shards[K + r] = p
    for case in meta["selection_cases"]:
        corrupt = case["corrupt"]
        sub = {s: shards[s] for s in range(1, N)}
        if corrupt is not None:
            sub[corrupt] = bytes(x ^ 0xA5 for x in sub[corrupt])
        out = c.decode(sub, B)
        assert out[0] == arrs[f"sel_{corrupt}_out"].tobytes()
        assert (out[0] == shards[0]) == case["recovers_original"]


def test_error_conventions_golden(dev, golden):
    from kcptube_amd import FecCode
    meta, _ = golden
    errs = meta["errors"]
    for e in errs["ctor_invalid"]:
        if e["throws"]:
            with pytest.raises(ValueError):
                FecCode(e["K"], e["N"])
            c = FecCode()
            with pytest.raises(ValueError):
                c.reset_martix(e["K"], e["N"])
        else:
            c = FecCode(e["K"], e["N"])
            assert (c.get_K(), c.get_N()) == (e["K"], e["N"])
    buf = bytes(range(256))
    for e in errs["encode_empty"]:
        c = FecCode(e["K"], e["N"])
        out = c.encode(buf, e["data_length"], e["B"])
        assert (len(out) == 0) == e["empty"]
        assert hashlib.sha256(b"".join(out)).hexdigest() == e["par_sha"]
    for e in errs["decode_empty"]:
        K, N, B = e["K"], e["N"], 8
        c = FecCode(K, N)
        shards = {i: bytes([i + 1]) * B for i in range(K)}
        for p, blk in enumerate(c.encode(b"".join(shards[i] for i in range(K)), K * B, B)):
            shards[K + p] = blk
        sub = {s: shards.get(s, b"\x00" * B) for s in e["present"]}
        out = c.decode(sub, B)
        assert sorted(out) == e["ids"]
        assert hashlib.sha256(b"".join(out[i] for i in sorted(out))).hexdigest() == e["out_sha"]


@pytest.mark.parametrize("cfg_index", [0, 1, 2, 3])
def test_config_digests_golden(dev, golden, cfg_index):
    """SURVEY 8(d) configs at fixture size, fully on the device: synthetic input, parity, erasure masks and
    recovered shards must reproduce the reference's SHA-256 digests."""
    from kcptube_amd import FecCode
    meta, _ = golden
    d = meta["digests"][cfg_index]
    K, N, B, G, seed = d["K"], d["N"], d["B"], d["G"], d["seed"]
    R = N - K
    c = FecCode(K, N)
    data = torch.empty((G, K, B), dtype=torch.uint8, device=dev)
    par = torch.empty((G, R, B), dtype=torch.uint8, device=dev)
    c.synth(data, seed)
    c.encode_batch(data, par)
    masks = torch.empty((G, 4), dtype=torch.int64, device=dev)
    c.erasure_masks(masks, seed, d["pool"], d["erase_max"], d["random_count"])
    torch.cuda.synchronize()
    assert hashlib.sha256(_np(data).tobytes()).hexdigest() == d["data_sha"]
    assert hashlib.sha256(_np(par).tobytes()).hexdigest() == d["parity_sha"]
    out = torch.zeros((G, R, B), dtype=torch.uint8, device=dev)
    idx = torch.empty((G, R), dtype=torch.uint8, device=dev)
    st = torch.empty((G,), dtype=torch.uint8, device=dev)
    ws = c.decode_workspace(G)
    _scribble_absent(data, par, masks, K)
    c.decode_batch(data, par, masks, out, idx, st, ws)
    torch.cuda.synchronize()
    assert hashlib.sha256(_np(masks).tobytes()).hexdigest() == d["mask_sha"]
    out_np = _np(out)
    idx_np = _np(idx)
    # the reference returns only recovered shards; unused slots of ours are compared as zero-filled
    out_np[idx_np == 0xFF] = 0
    assert hashlib.sha256(out_np.tobytes()).hexdigest() == d["recovered_sha"]
    assert hashlib.sha256(idx_np.tobytes()).hexdigest() == d["recovered_idx_sha"]
    assert int((idx_np != 0xFF).sum()) == d["recovered_total"]
    assert int(_np(st).max()) == 0


def _scribble_absent(data, par, masks, K):
    """Overwrite every absent shard slot with 0xA5 garbage (they must never be read)."""
    m = _masks_u64(masks)
    G, R = par.shape[0], par.shape[1]
    N = K + R
    bits = np.zeros((G, N), bool)
    for s in range(N):
        bits[:, s] = (m[:, s >> 6] >> np.uint64(s & 63)) & np.uint64(1)
    absent_d = torch.from_numpy(~bits[:, :K]).to(data.device)
    absent_p = torch.from_numpy(~bits[:, K:]).to(data.device)
    data[absent_d] = 0xA5
    if R:
        par[absent_p] = 0x5A


# ---------------------------------------------------------------------------------------------------
# batched device path against the oracle, across layouts and kernel variants
# ---------------------------------------------------------------------------------------------------
CASES = [
    # K, N, B, pitch, G, erase (None = random 0..R over all N), note
    (20, 23, 1440, 1440, 37, 3, "headline shape, V=32, no tail granule"),
    (10, 13, 1400, 1400, 41, None, "B=1400 -> V=32 with a 6-dword tail granule, random erasures"),
    (10, 13, 1402, 1404, 19, 3, "pitch % 16 = 12 -> V=32, 1-dword tail, 2 overhang bytes"),
    (20, 23, 1407, 1407, 9, 3, "odd pitch -> bytewise kernel"),
    (20, 23, 1406, 1408, 9, 2, "pitch > B, tail granule with overhang"),
    (7, 9, 100, 100, 300, None, "many groups per workgroup"),
    (1, 2, 16, 16, 513, 1, "K=1"),
    (3, 5, 1, 1, 1000, None, "B=1, one column"),
    (16, 24, 256, 256, 33, 8, "R=8 -> MT=8, prep_small<8>"),
    (30, 42, 96, 96, 17, 12, "R=12 -> 2 row tiles, prep_wave"),
    (200, 255, 64, 64, 4, 55, "max D+R, 55 lost"),
    (5, 5, 32, 32, 10, 0, "R=0"),
    (128, 256, 48, 48, 3, 100, "R=128, m up to 100"),
    (255, 256, 40, 40, 6, 1, "K=255"),
    (5, 8, 9000, 9000, 7, 3, "B > 8 KiB, 2-dword tail"),
    (3, 5, 8193, 8208, 5, None, "B > 8 KiB, pitch > B, 1-dword tail with overhang"),
    (4, 7, 2047, 2047, 5, 3, "odd B, bytewise"),
    (6, 9, 2048, 2048, 5, 3, "B = 2048"),
    (6, 9, 2049, 2064, 5, 3, "B = 2049, pitch > B"),
    (3, 10, 100, 100, 50, None, "K < R: syndrome form RT=8 with prep MAXM=3"),
    (5, 11, 1440, 1440, 40, None, "R=6 -> syndrome RT=6 (K < R), random erasures"),
    (100, 104, 64, 64, 20, 4, "K > 64 with R <= 8: second present word"),
    (250, 255, 16, 16, 10, 5, "K > 192 with R <= 8: fourth present word"),
    (20, 23, 1440, 1440, 64, 0, "zero loss: nothing recovered, nothing read"),
    (40, 60, 1440, 1440, 64, 20, "R=20, V=32: T-table decode entries, ~7 groups per workgroup, one chunk"),
    (30, 42, 97, 97, 21, 12, "R=12, odd pitch: bytewise T-table decode, entries in several chunks"),
    (60, 80, 1440, 1440, 33, None, "R=20, random 0..21 erasures over all 80: mixed m, some groups empty"),
    (2, 5, 1440, 1440, 40, 2, "K < PD with MT=3: the encode's burst loop runs its tail only"),
    (7, 11, 1440, 1440, 30, 4, "MT=4, K=7: one burst trip and a 3-shard tail"),
    (9, 12, 1024, 1024, 50, None, "MT=3, K=9: two burst trips and a 1-shard tail, random erasures"),
    (10, 13, 1400, 1400, 3001, None, "516 chunks: XCD span order (KFEC_XCD_ORDER) with a padded last run, random"),
    (8, 12, 256, 256, 16411, 4, "513 chunks: XCD span order, one chunk past the threshold, MT=4"),
    (12, 24, 256, 256, 16400, 12, "R=12, 2 row tiles over 513 chunks: tile XCD spans (KFEC_XCD_TILE_SPAN), padded"),
    (30, 50, 512, 512, 8200, None, "R=20, 2 encode row tiles of 10 over 513 chunks, random erasures: tile spans, T-table decode"),
    (25, 50, 1440, 1440, 40, 25, "R=25 -> three 10-row encode tiles, the last computing 5 rows"),
    (9, 18, 1440, 1440, 30, 9, "R=9 -> one 10-row encode tile with a slack row"),
    (20, 25, 1440, 1440, 40, 5, "R=5 -> one 5-row encode tile, paired MAC"),
    (16, 23, 1440, 1440, 30, None, "R=7 -> one 7-row encode tile (odd K pairs + tail), random erasures"),
    (20, 25, 1440, 1440, 41, None, "R=5 -> syndrome decode RT=5, random erasures"),
    (20, 26, 1440, 1440, 20000, None, "R=6 -> syndrome RT=6 over 513+ chunks, random erasures (dense and listed shapes)"),
]


@pytest.mark.parametrize("K,N,B,pitch,G,erase,note", CASES)
def test_batch_vs_oracle(dev, oracle, K, N, B, pitch, G, erase, note):
    from kcptube_amd import FecCode
    rng = np.random.default_rng(K * 1000 + N * 7 + B)
    R = N - K
    c = FecCode(K, N)
    data_np = rng.integers(0, 256, (G, K, pitch), dtype=np.uint8)
    data = torch.from_numpy(data_np).to(dev)
    par = torch.full((G, R, pitch), 0x77, dtype=torch.uint8, device=dev)
    c.encode_batch(data, par, B=B)
    torch.cuda.synchronize()
    exp_par = oracle.encode_batch(K, N, data_np, B)
    np.testing.assert_array_equal(_np(par)[:, :, :B], exp_par[:, :, :B], err_msg=note)
    # writes stay inside [0, ceil(B/4)*4) of each slot (kfec.h), [0, B) for a pitch that is not dword aligned
    hi = B if pitch % 4 else min(pitch, (B + 3) // 4 * 4)
    assert (_np(par)[:, :, hi:] == 0x77).all(), note

    masks_np = np.zeros((G, 4), np.uint64)
    for g in range(G):
        bits = set(range(N))
        if erase is None:
            e = int(rng.integers(0, R + 2))  # sometimes more than R -> too few shares
            lost = rng.choice(N, min(e, N), replace=False)
        elif erase == 0:
            lost = []
        else:
            # mostly data losses; every 5th group loses parity too; every 7th loses one too many
            pool = K if g % 5 else N
            e = min(erase + (1 if g % 7 == 3 else 0), pool)
            lost = rng.choice(pool, e, replace=False)
        for s in lost:
            bits.discard(int(s))
        for s in bits:
            masks_np[g, s >> 6] |= np.uint64(1) << np.uint64(s & 63)
    masks = torch.from_numpy(masks_np.view(np.int64)).to(dev)
    exp_out, exp_idx, exp_st = oracle.decode_batch(K, N, data_np, exp_par, masks_np, B)
    _scribble_absent(data, par, masks, K)
    out = torch.zeros((G, max(R, 1), pitch), dtype=torch.uint8, device=dev)
    idx = torch.empty((G, max(R, 1)), dtype=torch.uint8, device=dev)
    st = torch.empty((G,), dtype=torch.uint8, device=dev)
    c.decode_batch(data, par, masks, out, idx, st, c.decode_workspace(G), B=B)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(_np(st), exp_st, err_msg=note)
    if R:
        np.testing.assert_array_equal(_np(idx)[:, :R], exp_idx, err_msg=note)
        got = _np(out)[:, :R, :B].copy()
        got[exp_idx == 0xFF] = 0
        want = exp_out[:, :, :B].copy()
        want[exp_idx == 0xFF] = 0
        np.testing.assert_array_equal(got, want, err_msg=note)
        assert (_np(out)[:, :, hi:] == 0).all(), note


@pytest.mark.parametrize("K,N,B,G", [(20, 23, 1440, 700), (10, 13, 1400, 500), (5, 11, 3000, 90), (3, 5, 40, 3000),
                                     (16, 24, 1440, 600), (20, 25, 1440, 600)])
def test_sparse_losses_take_the_listed_shape(dev, oracle, K, N, B, G):
    """Few groups lost data (a live link): the decode runs over the device-built list of those groups only
    (syn_list_kernel); every other group must come back 'nothing recovered' and untouched output slots."""
    from kcptube_amd import FecCode
    rng = np.random.default_rng(G + K)
    R = N - K
    c = FecCode(K, N)
    data_np = rng.integers(0, 256, (G, K, B), dtype=np.uint8)
    data = torch.from_numpy(data_np).to(dev)
    par = torch.empty((G, R, B), dtype=torch.uint8, device=dev)
    c.encode_batch(data, par)
    torch.cuda.synchronize()
    exp_par = _np(par)
    masks_np = np.zeros((G, 4), np.uint64)
    for g in range(G):
        lost = set(rng.choice(N, int(rng.integers(1, R + 1)), replace=False).tolist()) if g % 11 == 3 else set()
        for s_ in range(N):
            if s_ not in lost:
                masks_np[g, s_ >> 6] |= np.uint64(1) << np.uint64(s_ & 63)
    masks = torch.from_numpy(masks_np.view(np.int64)).to(dev)
    exp_out, exp_idx, exp_st = oracle.decode_batch(K, N, data_np, exp_par, masks_np, B)
    _scribble_absent(data, par, masks, K)
    out = torch.full((G, R, B), 0x3C, dtype=torch.uint8, device=dev)
    idx = torch.empty((G, R), dtype=torch.uint8, device=dev)
    st = torch.empty((G,), dtype=torch.uint8, device=dev)
    c.decode_batch(data, par, masks, out, idx, st, c.decode_workspace(G))
    torch.cuda.synchronize()
    np.testing.assert_array_equal(_np(st), exp_st)
    np.testing.assert_array_equal(_np(idx), exp_idx)
    got = _np(out)
    used = exp_idx != 0xFF
    np.testing.assert_array_equal(got[used], exp_out[used])
    assert (got[~used] == 0x3C).all()  # slots of groups / rows with nothing recovered are never written


def test_single_group_api_vs_oracle(dev, oracle):
    """fec_code-style host API (kfec_encode / kfec_decode) on random shapes, including inconsistent
    (corrupted) shares, against the oracle."""
    from kcptube_amd import FecCode
    rng = np.random.default_rng(7)
    for trial in range(60):
        K = int(rng.integers(1, 40))
        N = int(min(256, K + rng.integers(0, 10)))
        B = int(rng.integers(1, 200))
        c = FecCode(K, N)
        data = rng.integers(0, 256, K * B, dtype=np.uint8).tobytes()
        par = c.encode(data, len(data), B)
        assert par == oracle.encode(K, N, data, B)
        shards = {i: data[i * B:(i + 1) * B] for i in range(K)}
        for r, p in enumerate(par):
            shards[K + r] = p
        keep = sorted(rng.choice(N, int(rng.integers(max(K - 1, 0), N + 1)), replace=False).tolist())
        sub = {s: shards[s] for s in keep}
        if keep and rng.random() < 0.4:
            k = keep[int(rng.integers(len(keep)))]
            sub[k] = bytes(x ^ 0x3C for x in sub[k])
        assert c.decode(sub, B) == oracle.decode(K, N, sub, B), (K, N, B, keep)


def test_single_group_share_size_zero(dev, oracle):
    """decode(shares, 0) returns one empty block per missing data row, as the reference (fecpp.cpp:572-583);
    the oracle is pinned against the compiled reference for this case (tests/test_oracle.py)."""
    from kcptube_amd import FecCode
    rng = np.random.default_rng(11)
    for _ in range(40):
        K = int(rng.integers(1, 30))
        N = int(min(256, K + rng.integers(0, 8)))
        c = FecCode(K, N)
        keep = sorted(rng.choice(N + 2, int(rng.integers(max(K - 1, 0), N + 1)), replace=False).tolist())
        sub = {s: b"" for s in keep}
        assert c.decode(sub, 0) == oracle.decode(K, N, sub, 0), (K, N, keep)


def test_synth_and_masks_match_oracle(dev, oracle):
    from kcptube_amd import FecCode
    K, N, B = 10, 13, 1400
    c = FecCode(K, N)
    out = torch.empty((5, 3, 1400), dtype=torch.uint8, device=dev)
    c.synth(out, 0x1234, g0=17, s0=10)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(_np(out), oracle.synth(0x1234, N, B, 17, 5, 10, 3))
    masks = torch.empty((64, 4), dtype=torch.int64, device=dev)
    c.erasure_masks(masks, 99, 13, 3, True, g0=1000)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(_masks_u64(masks), oracle.erasure_masks(99, 64, N, 13, 3, random_max=3, g0=1000))
    c.erasure_masks(masks, 99, 13, 50000, 2, g0=77)  # i.i.d. 5% loss per shard
    torch.cuda.synchronize()
    np.testing.assert_array_equal(_masks_u64(masks), oracle.erasure_masks_iid(99, 64, N, 50000, g0=77))


# ---------------------------------------------------------------------------------------------------
# full-size configs of BASELINE.json: size-independent round-trip property
# ---------------------------------------------------------------------------------------------------
@pytest.mark.parametrize("K,N,B,G,pool,emax,rnd", [
    (20, 23, 1440, 1 << 20, 20, 3, 0),   # config 2 (1M groups)
    (10, 13, 1400, 1 << 20, 13, 3, 1),    # config 3 (random 1-3 of all 13)
    (200, 255, 1440, 1 << 14, 200, 55, 0),  # config 4 shape (16k of the 256k groups)
    (20, 23, 1440, 1 << 20, 23, 10000, 2),  # a live link: i.i.d. 1% loss of every shard
])
def test_full_size_roundtrip(dev, K, N, B, G, pool, emax, rnd):
    from kcptube_amd import FecCode
    R = N - K
    c = FecCode(K, N)
    data = torch.empty((G, K, B), dtype=torch.uint8, device=dev)
    par = torch.empty((G, R, B), dtype=torch.uint8, device=dev)
    c.synth(data, 0xF00D + K)
    c.encode_batch(data, par)
    masks = torch.empty((G, 4), dtype=torch.int64, device=dev)
    c.erasure_masks(masks, 0xBEEF, pool, emax, rnd)
    out = torch.empty((G, R, B), dtype=torch.uint8, device=dev)
    idx = torch.empty((G, R), dtype=torch.uint8, device=dev)
    st = torch.empty((G,), dtype=torch.uint8, device=dev)
    c.decode_batch(data, par, masks, out, idx, st, c.decode_workspace(G))
    mism = torch.zeros(1, dtype=torch.int64, device=dev)
    c.verify_recovered(data, out, idx, mism)
    torch.cuda.synchronize()
    assert int(mism.item()) == 0
    if rnd == 2:  # a group that lost more than R shards is "too few shares" (status 1), exactly those
        pres = _masks_u64(masks)
        cnt = np.bitwise_count(pres).sum(axis=1)
        np.testing.assert_array_equal(_np(st), (cnt < K).astype(np.uint8))
    else:
        assert int(st.max().item()) == 0
    n_rec = int((idx != 0xFF).sum().item())
    if rnd == 0:
        assert n_rec == G * min(emax, R)
    elif rnd == 1:
        assert 0 < n_rec <= G * 3
    else:  # ~18% of the groups lose a data shard at 1% per shard
        assert 0.1 * G < n_rec < 0.3 * G


def test_compat_header_program(dev):
    """include/fecpp_compat.hpp compiled into a C++ program (the drop-in as kcptube would use it)."""
    from kcptube_amd.build import COMPAT_TEST
    if not os.path.exists(COMPAT_TEST):
        pytest.fail("compat_test not built (run __graft_entry__.build())")
    r = subprocess.run([COMPAT_TEST], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert "COMPAT OK" in r.stdout

