"""TEST INFRASTRUCTURE ONLY -- CPU parity checkers for the kfec HIP coder.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import this
package.  It is the checker, never the thing measured or shipped: the product path
(``kcptube_amd`` / ``libkfec.so``) never imports it and fails loudly without its HIP library.

Two checkers, both over ctypes:

* ``Oracle``  -- ``oracle/liboracle.so``, our plain-C restatement of ``fecpp::fec_code``
  (``/root/reference/src/3rd_party/fecpp.cpp``; per-function citations in ``rs_oracle.c``).
* ``RefCoder`` -- ``oracle/_ref/libfecpp_ref.so``, the reference coder itself, compiled from the
  reference's sources by ``oracle/Makefile`` (present wherever it was built; it travels to the GPU box
  with the snapshot).  ``RefCoder.available()`` says whether it is there.

Parity of ``Oracle`` is pinned against ``tests/golden/`` (fixtures generated from the compiled
reference by ``tests/golden/make_golden.py``) and against ``RefCoder`` where present.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
ORACLE_SO = os.path.join(_HERE, "liboracle.so")
REF_SO = os.path.join(_HERE, "_ref", "libfecpp_ref.so")

_u8p = C.POINTER(C.c_uint8)
_szp = C.POINTER(C.c_size_t)
_u64p = C.POINTER(C.c_uint64)

OK, EMPTY, EINVAL = 0, 1, -1


def build(force: bool = False) -> None:
    """Compile liboracle.so (and _ref/libfecpp_ref.so when the reference sources exist)."""
    if force or not os.path.exists(ORACLE_SO) or (
        os.path.getmtime(ORACLE_SO) < os.path.getmtime(os.path.join(_HERE, "rs_oracle.c"))
    ):
        subprocess.check_call(["make", "-s", "-C", _HERE, os.path.join(_HERE, "liboracle.so")])
    if os.path.isdir("/root/reference/src/3rd_party") and (
            force or not os.path.exists(REF_SO)
            or os.path.getmtime(REF_SO) < os.path.getmtime(os.path.join(_HERE, "ref_shim.cpp"))):
        subprocess.check_call(["make", "-s", "-C", _HERE, "ref"])


def _ptr(a: np.ndarray, t=_u8p):
    return a.ctypes.data_as(t)


class Oracle:
    """Our C restatement of fecpp::fec_code (liboracle.so)."""

    _lib = None

    def __init__(self):
        if Oracle._lib is None:
            if not os.path.exists(ORACLE_SO):
                build()
            lib = C.CDLL(ORACLE_SO)
            lib.orc_enc_matrix.argtypes = [C.c_size_t, C.c_size_t, _u8p]
            lib.orc_encode.argtypes = [C.c_size_t, C.c_size_t, _u8p, C.c_size_t, C.c_size_t, _u8p]
            lib.orc_decode.argtypes = [C.c_size_t, C.c_size_t, _szp, C.POINTER(_u8p), C.c_size_t,
                                       C.c_size_t, _szp, _u8p, _szp]
            lib.orc_select.argtypes = [C.c_size_t, C.c_size_t, _szp, C.c_size_t, _szp, _szp]
            lib.orc_gf_tables.argtypes = [_u8p, _u8p, _u8p, _u8p]
            lib.orc_splitmix64.argtypes = [C.c_uint64]
            lib.orc_splitmix64.restype = C.c_uint64
            lib.orc_synth.argtypes = [C.c_uint64, C.c_size_t, C.c_size_t, C.c_size_t, C.c_size_t,
                                      C.c_size_t, C.c_size_t, _u8p, C.c_size_t]
            lib.orc_erasure_mask.argtypes = [C.c_uint64, C.c_size_t, C.c_size_t, C.c_size_t,
                                             C.c_size_t, _u64p]
            lib.orc_erasure_mask_iid.argtypes = [C.c_uint64, C.c_size_t, C.c_size_t, C.c_size_t, _u64p]
            lib.orc_erasure_count.argtypes = [C.c_uint64, C.c_size_t, C.c_size_t]
            lib.orc_erasure_count.restype = C.c_size_t
            lib.orc_encode_batch.argtypes = [C.c_size_t] * 5 + [_u8p, _u8p]
            lib.orc_decode_batch.argtypes = [C.c_size_t] * 5 + [_u8p, _u8p, _u64p, _u8p, _u8p, _u8p]
            lib.orc_bench_roundtrip.argtypes = [C.c_size_t] * 7 + [C.c_uint64, C.POINTER(C.c_double)]
            lib.orc_bench_roundtrip.restype = C.c_double
            Oracle._lib = lib
        self.lib = Oracle._lib

    # ---- GF and matrix -------------------------------------------------------------------
    def gf_tables(self):
        exp = np.zeros(510, np.uint8); log = np.zeros(256, np.uint8)
        inv = np.zeros(256, np.uint8); mul = np.zeros((256, 256), np.uint8)
        self.lib.orc_gf_tables(_ptr(exp), _ptr(log), _ptr(inv), _ptr(mul))
        return exp, log, inv, mul

    def enc_matrix(self, K: int, N: int) -> np.ndarray:
        out = np.zeros((N, K), np.uint8)
        rc = self.lib.orc_enc_matrix(K, N, _ptr(out))
        if rc != OK:
            raise ValueError("fec_code: violated 1 <= K <= N <= 256")
        return out

    # ---- single group, fec_code semantics ---------------------------------------------------
    def encode(self, K: int, N: int, data: bytes | np.ndarray, block_size: int, data_length=None):
        buf = np.frombuffer(bytes(data), np.uint8).copy() if not isinstance(data, np.ndarray) else data
        dl = len(buf) if data_length is None else data_length
        out = np.zeros(max(N - K, 0) * max(block_size, 1), np.uint8)
        rc = self.lib.orc_encode(K, N, _ptr(buf), dl, block_size, _ptr(out))
        if rc == EINVAL:
            raise ValueError("fec_code: violated 1 <= K <= N <= 256")
        if rc == EMPTY:
            return []
        return [out[r * block_size:(r + 1) * block_size].tobytes() for r in range(N - K)]

    def select(self, K: int, N: int, ids):
        ids = sorted(ids)
        a = (C.c_size_t * max(len(ids), 1))(*ids)
        sel = (C.c_size_t * K)(); pos = (C.c_size_t * K)()
        rc = self.lib.orc_select(K, N, a, len(ids), sel, pos)
        return (list(sel) if rc == OK else None)

    def decode(self, K: int, N: int, shares: dict, share_size: int) -> dict:
        ids = sorted(shares)
        bufs = [np.frombuffer(bytes(shares[i]), np.uint8).copy() for i in ids]
        n = len(ids)
        ida = (C.c_size_t * max(n, 1))(*ids)
        pa = (_u8p * max(n, 1))(*[_ptr(b) for b in bufs])
        out = np.zeros(K * max(share_size, 1), np.uint8)
        oids = (C.c_size_t * K)()
        nout = C.c_size_t(0)
        rc = self.lib.orc_decode(K, N, ida, pa, n, share_size, oids, _ptr(out), C.byref(nout))
        if rc == EINVAL:
            raise ValueError("singular matrix")
        return {int(oids[t]): out[t * share_size:(t + 1) * share_size].tobytes() for t in range(nout.value)}

    # ---- synthetic inputs -------------------------------------------------------
    def synth(self, seed: int, N: int, B: int, g0: int, ng: int, s0: int, ns: int, pitch=None):
        pitch = B if pitch is None else pitch
        out = np.zeros((ng, ns, pitch), np.uint8)
        self.lib.orc_synth(seed, N, B, g0, ng, s0, ns, _ptr(out), pitch)
        return out

    def erasure_masks(self, seed: int, G: int, N: int, pool: int, cnt: int | None,
                      random_max: int | None = None, g0: int = 0) -> np.ndarray:
        masks = np.zeros((G, 4), np.uint64)
        for g in range(G):
            c = cnt if random_max is None else self.lib.orc_erasure_count(seed, g0 + g, random_max)
            self.lib.orc_erasure_mask(seed, g0 + g, N, pool, c, _ptr(masks[g], _u64p))
        return masks

    def erasure_masks_iid(self, seed: int, G: int, N: int, ppm: int, g0: int = 0) -> np.ndarray:
        """i.i.d. loss of every shard with probability ppm / 1e6 (kfec_erasure_masks random_count = 2)."""
        masks = np.zeros((G, 4), np.uint64)
        for g in range(G):
            self.lib.orc_erasure_mask_iid(seed, g0 + g, N, ppm, _ptr(masks[g], _u64p))
        return masks

    # ---- batched helpers -------------------------------------------------------------------
    def encode_batch(self, K: int, N: int, data: np.ndarray, B: int) -> np.ndarray:
        G, k, pitch = data.shape
        assert k == K
        par = np.zeros((G, N - K, pitch), np.uint8)
        self.lib.orc_encode_batch(K, N, G, B, pitch, _ptr(np.ascontiguousarray(data)), _ptr(par))
        return par

    def decode_batch(self, K: int, N: int, data: np.ndarray, parity: np.ndarray, present: np.ndarray,
                     B: int):
        G, _, pitch = data.shape
        R = N - K
        out = np.zeros((G, R, pitch), np.uint8)
        idx = np.full((G, R), 0xFF, np.uint8)
        st = np.zeros(G, np.uint8)
        self.lib.orc_decode_batch(K, N, G, B, pitch, _ptr(np.ascontiguousarray(data)),
                                  _ptr(np.ascontiguousarray(parity)),
                                  _ptr(np.ascontiguousarray(present), _u64p), _ptr(out), _ptr(idx),
                                  _ptr(st))
        return out, idx, st

    def bench_roundtrip(self, K, N, B, G, erase, threads, passes, seed):
        secs = C.c_double(0)
        bps = self.lib.orc_bench_roundtrip(K, N, B, G, erase, threads, passes, seed, C.byref(secs))
        return bps, secs.value


class RefCoder:
    """The reference fecpp coder compiled from /root/reference sources (oracle/_ref)."""

    _lib = None

    @staticmethod
    def available() -> bool:
        return os.path.exists(REF_SO)

    def __init__(self):
        if RefCoder._lib is None:
            if not self.available():
                raise FileNotFoundError(REF_SO)
            lib = C.CDLL(REF_SO)
            lib.ref_check_kn.argtypes = [C.c_size_t, C.c_size_t]
            lib.ref_check_reset.argtypes = [C.c_size_t, C.c_size_t]
            lib.ref_encode.argtypes = [C.c_size_t, C.c_size_t, _u8p, C.c_size_t, C.c_size_t, _u8p]
            lib.ref_encode.restype = C.c_long
            lib.ref_enc_matrix.argtypes = [C.c_size_t, C.c_size_t, _u8p]
            lib.ref_decode.argtypes = [C.c_size_t, C.c_size_t, _szp, C.POINTER(_u8p), C.c_size_t,
                                       C.c_size_t, _szp, _u8p]
            lib.ref_decode.restype = C.c_long
            lib.ref_bench_roundtrip.argtypes = [C.c_size_t] * 6 + [C.c_int, C.c_size_t, C.c_size_t,
                                                                  C.c_uint64, C.POINTER(C.c_double),
                                                                  _szp, C.c_int]
            lib.ref_bench_roundtrip.restype = C.c_double
            RefCoder._lib = lib
        self.lib = RefCoder._lib

    def enc_matrix(self, K, N):
        out = np.zeros((N, K), np.uint8)
        self.lib.ref_enc_matrix(K, N, _ptr(out))
        return out

    def encode(self, K, N, data, block_size, data_length=None):
        buf = np.frombuffer(bytes(data), np.uint8).copy()
        dl = len(buf) if data_length is None else data_length
        out = np.zeros(max(N - K, 1) * max(block_size, 1), np.uint8)
        n = self.lib.ref_encode(K, N, _ptr(buf), dl, block_size, _ptr(out))
        if n < 0:
            return []
        return [out[r * block_size:(r + 1) * block_size].tobytes() for r in range(n)]

    def decode(self, K, N, shares: dict, share_size: int) -> dict:
        ids = sorted(shares)
        bufs = [np.frombuffer(bytes(shares[i]), np.uint8).copy() for i in ids]
        n = len(ids)
        ida = (C.c_size_t * max(n, 1))(*ids)
        pa = (_u8p * max(n, 1))(*[_ptr(b) for b in bufs])
        out = np.zeros(K * max(share_size, 1), np.uint8)
        oids = (C.c_size_t * K)()
        m = self.lib.ref_decode(K, N, ida, pa, n, share_size, oids, _ptr(out))
        if m == -2:
            raise ValueError("singular matrix")
        return {int(oids[t]): out[t * share_size:(t + 1) * share_size].tobytes() for t in range(m)}

    def bench_roundtrip(self, K, N, B, G, pool, erase_max, random_count, threads, passes, seed,
                        decode_only=False):
        """payload bytes/s of (encode +) decode over G groups, the reference coder on `threads` cores"""
        secs = C.c_double(0)
        rec = C.c_size_t(0)
        bps = self.lib.ref_bench_roundtrip(K, N, B, G, pool, erase_max, int(random_count), threads,
                                           passes, seed, C.byref(secs), C.byref(rec), int(decode_only))
        return bps, secs.value, rec.value
