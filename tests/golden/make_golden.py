#!/usr/bin/env python3
"""Generate tests/golden/ fixtures from the REFERENCE coder (oracle/_ref/libfecpp_ref.so, compiled
from /root/reference/src/3rd_party/fecpp*.cpp by oracle/Makefile).  Run in the build container:

    make -C oracle && python tests/golden/make_golden.py

Outputs (committed; data only -- inputs and the reference's outputs):
  golden.npz   -- enc matrices, tiny encode/decode cases (inputs + outputs), selection-rule cases
  golden.json  -- SHA-256 digests of the SURVEY 8(d) configs at fixture size, error-convention cases

The reference has no tests of its own, so these fixtures are the pins.
Synthetic inputs use the counter-based definition of SURVEY 8(d) (oracle.Oracle.synth); the digest of
every synthesized input is stored as well, so a change in the generator is caught on its own.
"""
from __future__ import annotations

import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from oracle import Oracle, RefCoder  # noqa: E402

MATRIX_CONFIGS = [(1, 1), (1, 2), (3, 5), (10, 13), (20, 23), (200, 255), (1, 255), (128, 256),
                  (255, 256), (256, 256), (17, 40), (64, 96)]
TINY_KN = [(1, 2), (3, 5), (10, 13), (20, 23), (200, 255)]
TINY_B = [1, 15, 16, 17, 64]
SEED_TINY = 0x601D0000


def sha(b: bytes) -> str:
    return hashlib.sha256(b).hexdigest()


def main() -> None:
    ref = RefCoder()
    orc = Oracle()
    arrays: dict[str, np.ndarray] = {}
    meta: dict = {"generator": "tests/golden/make_golden.py", "reference": "fecpp (kcptube 20260131)"}

    # 1. encoding matrices (recovered from the reference by encoding unit vectors, B = 1)
    for K, N in MATRIX_CONFIGS:
        arrays[f"enc_{K}_{N}"] = ref.enc_matrix(K, N)

    # 2. tiny encode + decode cases
    cases = []
    rng = np.random.default_rng(12345)
    for K, N in TINY_KN:
        R = N - K
        for B in TINY_B:
            key = f"t_{K}_{N}_{B}"
            data = orc.synth(SEED_TINY + K * 1000 + B, N, B, 0, 1, 0, K).reshape(-1)
            par = ref.encode(K, N, data.tobytes(), B)
            arrays[key + "_in"] = data
            arrays[key + "_par"] = np.frombuffer(b"".join(par), np.uint8)
            shards = {i: data[i * B:(i + 1) * B].tobytes() for i in range(K)}
            for r, p in enumerate(par):
                shards[K + r] = p
            patterns = []
            # all R lost among data (max loss), parity-only loss, mixed, nothing lost, too few
            ndat = min(R, K)
            patterns.append(sorted(rng.choice(K, ndat, replace=False).tolist()))
            patterns.append(list(range(K, N))[: max(R - 1, 0)])
            if R >= 2 and K >= 1:
                patterns.append(sorted([int(rng.integers(K)), int(K + rng.integers(R))]))
            patterns.append([])
            patterns.append(sorted(rng.choice(N, min(R + 1, N), replace=False).tolist()))
            for pi, erased in enumerate(patterns):
                present = [s for s in range(N) if s not in set(erased)]
                out = ref.decode(K, N, {s: shards[s] for s in present}, B)
                ids = sorted(out)
                arrays[f"{key}_d{pi}_present"] = np.array(present, np.int32)
                arrays[f"{key}_d{pi}_ids"] = np.array(ids, np.int32)
                arrays[f"{key}_d{pi}_out"] = np.frombuffer(b"".join(out[i] for i in ids), np.uint8)
            cases.append({"K": K, "N": N, "B": B, "key": key, "n_patterns": len(patterns)})
    meta["tiny_cases"] = cases

    # 3. selection rule: 20:23, data 0 missing, shards 1..22 present (> K shares)
    K, N, B = 20, 23, 64
    data = orc.synth(0x5E1EC7, N, B, 0, 1, 0, K).reshape(-1)
    par = ref.encode(K, N, data.tobytes(), B)
    shards = {i: data[i * B:(i + 1) * B].tobytes() for i in range(K)}
    for r, p in enumerate(par):
        shards[K + r] = p
    sel_cases = []
    for corrupt in [None, 20, 21, 22]:
        sub = {s: shards[s] for s in range(1, N)}
        if corrupt is not None:
            sub[corrupt] = bytes(x ^ 0xA5 for x in sub[corrupt])
        out = ref.decode(K, N, sub, B)
        ok = out.get(0) == shards[0]
        arrays[f"sel_{corrupt}_out"] = np.frombuffer(out[0], np.uint8)
        sel_cases.append({"corrupt": corrupt, "recovers_original": bool(ok)})
    arrays["sel_in"] = data
    meta["selection_cases"] = sel_cases

    # 4. error conventions
    errs = {"ctor_invalid": [], "encode_empty": [], "decode_empty": []}
    for K, N in [(0, 0), (0, 5), (5, 0), (6, 5), (257, 257), (1, 257), (256, 256), (1, 1), (255, 256)]:
        errs["ctor_invalid"].append({"K": K, "N": N, "throws": ref.lib.ref_check_kn(K, N) != 0,
                                     "reset_throws": ref.lib.ref_check_reset(K, N) == -1})
    K, N, B = 4, 6, 8
    buf = bytes(range(256))
    for dl in [4 * 8, 4 * 8 + 7, 3 * 8, 5 * 8, 8 * 8, 12 * 8]:
        out = ref.encode(K, N, buf, B, data_length=dl)
        errs["encode_empty"].append({"K": K, "N": N, "B": B, "data_length": dl, "empty": len(out) == 0,
                                     "par_sha": sha(b"".join(out))})
    shards = {i: bytes([i + 1]) * B for i in range(K)}
    for p, blk in enumerate(ref.encode(K, N, b"".join(shards[i] for i in range(K)), B)):
        shards[K + p] = blk
    for present in [[0, 1, 2], [1, 2, 3, 4], [0, 1, 2, 3], [0, 2, 4, 5], [1, 2, 3, 9], [0, 1, 2, 3, 9]]:
        sub = {s: (shards[s] if s in shards else b"\x00" * B) for s in present}
        out = ref.decode(K, N, sub, B)
        errs["decode_empty"].append({"K": K, "N": N, "present": present, "ids": sorted(out),
                                     "out_sha": sha(b"".join(out[i] for i in sorted(out)))})
    meta["errors"] = errs

    # 5. SURVEY 8(d) configs at fixture size: digests of inputs, parity and recovered shards
    digests = []
    for cfg_id, (K, N, B, G, pool, emax, rnd) in enumerate([
        (20, 23, 1440, 4096, 20, 3, False),    # config 1 (golden 4k-group round trip)
        (10, 13, 1400, 2048, 13, 3, True),     # config 3 shape: random 1-3 of all 13
        (200, 255, 1440, 8, 200, 55, False),   # config 4 shape: 55 data lost
        (20, 23, 1440, 64, 20, 3, False),      # small GPU-side check
    ]):
        seed = 0x5EED0001 + cfg_id
        data = orc.synth(seed, N, B, 0, G, 0, K)
        par = np.zeros((G, N - K, B), np.uint8)
        rec = np.zeros((G, N - K, B), np.uint8)
        rec_idx = np.full((G, N - K), 0xFF, np.uint8)
        masks = orc.erasure_masks(seed, G, N, pool, emax, random_max=emax if rnd else None)
        for g in range(G):
            p = ref.encode(K, N, data[g].tobytes(), B)
            for r in range(N - K):
                par[g, r] = np.frombuffer(p[r], np.uint8)
            present = [s for s in range(N) if int(masks[g, s >> 6]) >> (s & 63) & 1]
            sub = {s: (data[g, s].tobytes() if s < K else p[s - K]) for s in present}
            out = ref.decode(K, N, sub, B)
            for t, i in enumerate(sorted(out)):
                rec[g, t] = np.frombuffer(out[i], np.uint8)
                rec_idx[g, t] = i
        digests.append({"cfg": cfg_id, "K": K, "N": N, "B": B, "G": G, "seed": seed, "pool": pool,
                        "erase_max": emax, "random_count": rnd,
                        "data_sha": sha(data.tobytes()), "parity_sha": sha(par.tobytes()),
                        "recovered_sha": sha(rec.tobytes()), "recovered_idx_sha": sha(rec_idx.tobytes()),
                        "mask_sha": sha(masks.tobytes()),
                        "recovered_total": int((rec_idx != 0xFF).sum())})
        print("digest cfg", cfg_id, digests[-1]["parity_sha"][:16], flush=True)
    meta["digests"] = digests
    # splitmix64 known answers (pure definition check)
    meta["splitmix64"] = {str(x): int(orc.lib.orc_splitmix64(x)) for x in [0, 1, 0x5EED0001, 2**63]}

    np.savez_compressed(os.path.join(HERE, "golden.npz"), **arrays)
    with open(os.path.join(HERE, "golden.json"), "w") as f:
        json.dump(meta, f, indent=1)
    print("wrote", len(arrays), "arrays")


if __name__ == "__main__":
    main()
