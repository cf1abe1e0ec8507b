"""Python host mirror of kcptube's AEAD packet modes on libkfec.so (include/kfec_aead.h).

=====================================================================  ==========================================
reference (file:line)                                                  here
=====================================================================  ==========================================
encrypt_decrypt<chacha20 / xchacha20>(password) (src/shares/aead.hpp    ``AeadCipher(mode, password)``
402-562): SHA-3(256) key, Botan ChaCha20Poly1305
encrypt_data(password, mode, data, length)                             ``AeadCipher.seal`` (batched, device)
(src/shares/data_operations.cpp:171-234)
decrypt_data(password, mode, data, length)                             ``AeadCipher.open_``
(src/shares/data_operations.cpp:373-435)
=====================================================================  ==========================================

The reference draws iv_raw inside change_iv() (uniform 16-bit, aead.hpp:464-475); the batched seal takes the
caller's draws as a uint16 tensor so that a test can replay them.  All work runs as gfx950 kernels on
device-resident ``torch`` tensors; there is no CPU path.
"""
from __future__ import annotations

import ctypes as C

from .fec import _check, _dptr, _stream_handle, _vp, load_library

AES_GCM = 4    # encryption_mode::aes_gcm (share_defines.hpp:29)
AES_OCB = 5    # encryption_mode::aes_ocb
CHACHA20 = 6   # encryption_mode::chacha20
XCHACHA20 = 7  # encryption_mode::xchacha20
MODES = {"aes_gcm": AES_GCM, "aes_ocb": AES_OCB, "chacha20": CHACHA20, "xchacha20": XCHACHA20}
TAG = 16
OVERHEAD = 18


class AeadCipher:
    """One connection's cipher: key = SHA-3(256)(password), per-iv tables built on the current device."""

    def __init__(self, mode, password: bytes | str):
        self._lib = load_library()
        self.mode = MODES.get(mode, mode) if isinstance(mode, str) else int(mode)
        if isinstance(password, str):
            password = password.encode()
        if self.mode not in (AES_GCM, AES_OCB, CHACHA20, XCHACHA20):
            raise ValueError(f"unsupported AEAD mode {mode!r}")
        if not password:
            raise ValueError("empty password (the reference leaves its cipher objects unset)")
        self._h = _vp()
        _check(self._lib.kfec_aead_create(self.mode, password, len(password), C.byref(self._h)), "kfec_aead_create")

    def __del__(self):
        try:
            if self._h.value:
                self._lib.kfec_aead_destroy(self._h)
                self._h = _vp()
        except Exception:
            pass

    @property
    def key(self) -> bytes:
        buf = (C.c_uint8 * 32)()
        _check(self._lib.kfec_aead_key(self._h, buf), "kfec_aead_key")
        return bytes(buf)

    def seal(self, src, off, length, iv, dst, out_len, stream=None) -> None:
        """encrypt_data for P packets [off[p], off[p] + length[p]) of src (uint8), iv_raw iv[p] (int16/uint16
        tensor [P]): dst [P][pitch] receives ciphertext || tag || iv_raw, out_len int32 [P] (0: empty or too
        long for the pitch)."""
        P = off.numel()
        _check(self._lib.kfec_aead_seal_batch(self._h, P, _dptr(src), src.numel(), _dptr(off), _dptr(length),
                                              _dptr(iv), _dptr(dst), dst.shape[-1], _dptr(out_len),
                                              _stream_handle(stream)), "kfec_aead_seal_batch")

    def open_(self, src, off, length, dst, out_len, ok, stream=None) -> None:
        """decrypt_data: plaintext to dst [P][pitch] (zeros where the tag fails), out_len int32 [P],
        ok uint8 [P]."""
        P = off.numel()
        _check(self._lib.kfec_aead_open_batch(self._h, P, _dptr(src), src.numel(), _dptr(off), _dptr(length),
                                              _dptr(dst), dst.shape[-1], _dptr(out_len), _dptr(ok),
                                              _stream_handle(stream)), "kfec_aead_open_batch")
