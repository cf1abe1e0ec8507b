"""CPU tests: the oracle (our C restatement of fecpp::fec_code) is pinned against the reference.

Pins, in order of strength:
  1. tests/golden/ fixtures generated from the reference coder compiled from /root/reference sources
     (tests/golden/make_golden.py) -- always available, also on the GPU box;
  2. the compiled reference itself (oracle/_ref/libfecpp_ref.so) when present -- randomized differential.
"""
from __future__ import annotations

import hashlib

import numpy as np
import pytest


def sha(b: bytes) -> str:
    return hashlib.sha256(b).hexdigest()


# ---------------------------------------------------------------------------------------------------
# GF(2^8) known answers: tables equal shift-xor multiplication mod 0x11D, alpha = 2
# ---------------------------------------------------------------------------------------------------
def _slow_mul(a: int, b: int) -> int:
    r = 0
    while b:
        if b & 1:
            r ^= a
        a <<= 1
        if a & 0x100:
            a ^= 0x11D
        b >>= 1
    return r


def test_gf_tables_known_answers(oracle):
    exp, log, inv, mul = oracle.gf_tables()
    assert exp[0] == 1 and exp[1] == 2 and exp[8] == 0x1D and exp[255] == 1
    assert log[0] == 0xFF
    for a in range(256):
        for b in range(0, 256, 7):
            assert mul[a, b] == _slow_mul(a, b)
    for a in range(1, 256):
        assert _slow_mul(a, int(inv[a])) == 1
        assert exp[log[a]] == a


# ---------------------------------------------------------------------------------------------------
# golden fixtures
# ---------------------------------------------------------------------------------------------------
def test_enc_matrix_vs_golden(oracle, golden):
    _, arrs = golden
    n = 0
    for key in arrs.files:
        if key.startswith("enc_"):
            _, K, N = key.split("_")
            np.testing.assert_array_equal(oracle.enc_matrix(int(K), int(N)), arrs[key], err_msg=key)
            n += 1
    assert n >= 10


def test_known_parity_row_20_23(oracle):
    """parity row 0 of the 20:23 code."""
    row = oracle.enc_matrix(20, 23)[20].tobytes().hex()
    assert row == "b7ae0b720bcd293f84a0e57303dfd9bad5d02099"


def test_tiny_cases_vs_golden(oracle, golden):
    meta, arrs = golden
    for case in meta["tiny_cases"]:
        K, N, B, key = case["K"], case["N"], case["B"], case["key"]
        data = arrs[key + "_in"].tobytes()
        par = oracle.encode(K, N, data, B)
        assert b"".join(par) == arrs[key + "_par"].tobytes(), key
        shards = {i: data[i * B:(i + 1) * B] for i in range(K)}
        for r, p in enumerate(par):
            shards[K + r] = p
        for pi in range(case["n_patterns"]):
            present = arrs[f"{key}_d{pi}_present"].tolist()
            out = oracle.decode(K, N, {s: shards[s] for s in present}, B)
            ids = arrs[f"{key}_d{pi}_ids"].tolist()
            assert sorted(out) == ids
            assert b"".join(out[i] for i in ids) == arrs[f"{key}_d{pi}_out"].tobytes()


def test_selection_rule_vs_golden(oracle, golden):
    meta, arrs = golden
    K, N, B = 20, 23, 64
    data = arrs["sel_in"].tobytes()
    par = oracle.encode(K, N, data, B)
    shards = {i: data[i * B:(i + 1) * B] for i in range(K)}
    for r, p in enumerate(par):
        shards[K + r] = p
    for case in meta["selection_cases"]:
        corrupt = case["corrupt"]
        sub = {s: shards[s] for s in range(1, N)}
        if corrupt is not None:
            sub[corrupt] = bytes(x ^ 0xA5 for x in sub[corrupt])
        out = oracle.decode(K, N, sub, B)
        assert out[0] == arrs[f"sel_{corrupt}_out"].tobytes()
        assert (out[0] == shards[0]) == case["recovers_original"]
    # the rule itself: missing rows take the highest unused ids, descending
    assert oracle.select(20, 23, list(range(1, 23)))[0] == 22
    assert oracle.select(4, 8, [1, 3, 5, 6, 7])[:3] == [7, 1, 6]


def test_error_conventions_vs_golden(oracle, golden):
    meta, _ = golden
    errs = meta["errors"]
    for e in errs["ctor_invalid"]:
        if e["throws"]:
            with pytest.raises(ValueError):
                oracle.enc_matrix(e["K"], e["N"])
        else:
            oracle.enc_matrix(e["K"], e["N"])
    buf = bytes(range(256))
    for e in errs["encode_empty"]:
        out = oracle.encode(e["K"], e["N"], buf, e["B"], data_length=e["data_length"])
        assert (len(out) == 0) == e["empty"]
        assert sha(b"".join(out)) == e["par_sha"]
    for e in errs["decode_empty"]:
        K, N, B = e["K"], e["N"], 8
        shards = {i: bytes([i + 1]) * B for i in range(K)}
        for p, blk in enumerate(oracle.encode(K, N, b"".join(shards[i] for i in range(K)), B)):
            shards[K + p] = blk
        sub = {s: shards.get(s, b"\x00" * B) for s in e["present"]}
        out = oracle.decode(K, N, sub, B)
        assert sorted(out) == e["ids"]
        assert sha(b"".join(out[i] for i in sorted(out))) == e["out_sha"]


def test_splitmix_and_synth_definition(oracle, golden):
    meta, _ = golden
    M = (1 << 64) - 1

    def smix(x):  # pure-Python statement of the generator
        x = (x + 0x9E3779B97F4A7C15) & M
        x = ((x ^ (x >> 30)) * 0xBF58476D1CE4E5B9) & M
        x = ((x ^ (x >> 27)) * 0x94D049BB133111EB) & M
        return x ^ (x >> 31)

    for k, v in meta["splitmix64"].items():
        assert smix(int(k)) == v
    # byte b of slot s of group g = byte (b % 8) of smix(seed ^ ((g*N+s)*W + b//8))
    seed, N, B = 77, 13, 21
    out = oracle.synth(seed, N, B, 3, 2, 1, 2)
    W = (B + 7) // 8
    for gi, g in enumerate([3, 4]):
        for si, s in enumerate([1, 2]):
            for b in range(B):
                v = smix(seed ^ ((g * N + s) * W + b // 8))
                assert out[gi, si, b] == (v >> (8 * (b % 8))) & 0xFF


@pytest.mark.parametrize("cfg_index", [0, 1, 3])
def test_config_digests_vs_golden(oracle, golden, cfg_index):
    """The oracle's batched encode/decode reproduces the reference's digests of the SURVEY 8(d) configs."""
    meta, _ = golden
    d = meta["digests"][cfg_index]
    K, N, B, G, seed = d["K"], d["N"], d["B"], d["G"], d["seed"]
    data = oracle.synth(seed, N, B, 0, G, 0, K)
    assert sha(data.tobytes()) == d["data_sha"]
    par = oracle.encode_batch(K, N, data, B)
    assert sha(par.tobytes()) == d["parity_sha"]
    masks = oracle.erasure_masks(seed, G, N, d["pool"], d["erase_max"],
                                 random_max=d["erase_max"] if d["random_count"] else None)
    assert sha(masks.tobytes()) == d["mask_sha"]
    out, idx, st = oracle.decode_batch(K, N, data, par, masks, B)
    out[idx == 0xFF] = 0
    assert sha(out.tobytes()) == d["recovered_sha"]
    assert sha(idx.tobytes()) == d["recovered_idx_sha"]
    assert int(st.max()) == 0


# ---------------------------------------------------------------------------------------------------
# differential against the compiled reference (when oracle/_ref is built)
# ---------------------------------------------------------------------------------------------------
def test_oracle_vs_reference_randomized(oracle):
    from oracle import RefCoder
    if not RefCoder.available():
        pytest.skip("oracle/_ref not built (reference sources absent)")
    ref = RefCoder()
    rng = np.random.default_rng(2024)
    for _ in range(200):
        K = int(rng.integers(1, 48))
        N = int(min(256, K + rng.integers(0, 12)))
        B = int(rng.integers(1, 100))
        data = rng.integers(0, 256, K * B, dtype=np.uint8).tobytes()
        pa, pb = oracle.encode(K, N, data, B), ref.encode(K, N, data, B)
        assert pa == pb
        shards = {i: data[i * B:(i + 1) * B] for i in range(K)}
        for r, p in enumerate(pa):
            shards[K + r] = p
        keep = sorted(rng.choice(N, int(rng.integers(max(K - 1, 0), N + 1)), replace=False).tolist())
        sub = {s: shards[s] for s in keep}
        if keep and rng.random() < 0.3:
            k = keep[int(rng.integers(len(keep)))]
            sub[k] = bytes(x ^ 0x5A for x in sub[k])
        assert oracle.decode(K, N, sub, B) == ref.decode(K, N, sub, B)


def test_oracle_vs_reference_matrices_all_small(oracle):
    from oracle import RefCoder
    if not RefCoder.available():
        pytest.skip("oracle/_ref not built")
    ref = RefCoder()
    for K in range(1, 33):
        for N in (K, K + 1, K + 3, min(256, K + 40)):
            np.testing.assert_array_equal(oracle.enc_matrix(K, N), ref.enc_matrix(K, N))


def test_oracle_vs_reference_share_size_zero(oracle):
    """decode(shares, 0): the reference still maps every missing data row to an empty block
    (fecpp.cpp:572-583); {} for too few shares or a chosen id >= N."""
    from oracle import RefCoder
    if not RefCoder.available():
        pytest.skip("oracle/_ref not built")
    ref = RefCoder()
    rng = np.random.default_rng(5)
    for _ in range(60):
        K = int(rng.integers(1, 30))
        N = int(min(256, K + rng.integers(0, 8)))
        keep = sorted(rng.choice(N + 2, int(rng.integers(max(K - 1, 0), N + 1)), replace=False).tolist())
        sub = {s: b"" for s in keep}
        want = ref.decode(K, N, sub, 0)
        assert oracle.decode(K, N, sub, 0) == want, (K, N, keep)
        assert all(v == b"" for v in want.values())
