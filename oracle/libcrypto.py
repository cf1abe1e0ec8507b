"""TEST INFRASTRUCTURE ONLY: ctypes bindings of the container's OpenSSL 3 libcrypto, the independent
implementation oracle/aead_oracle.py is pinned against (tests/test_aead_oracle.py) and that the GPU AEAD tests
use as a second checker at sizes the pure-Python oracle is too slow for.  Never imported by the product."""
from __future__ import annotations

import ctypes as C

try:
    _crypto = C.CDLL("libcrypto.so.3")
except OSError:  # pragma: no cover - the image ships it
    _crypto = None

AVAILABLE = _crypto is not None

EVP_CTRL_AEAD_SET_IVLEN = 0x9
EVP_CTRL_AEAD_GET_TAG = 0x10
EVP_CTRL_AEAD_SET_TAG = 0x11


def _evp():
    c = _crypto
    c.EVP_CIPHER_CTX_new.restype = C.c_void_p
    c.EVP_CIPHER_CTX_free.argtypes = [C.c_void_p]
    for n in ("EVP_aes_256_gcm", "EVP_aes_256_ocb", "EVP_chacha20", "EVP_chacha20_poly1305"):
        getattr(c, n).restype = C.c_void_p
    c.EVP_EncryptInit_ex.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_char_p, C.c_char_p]
    c.EVP_EncryptUpdate.argtypes = [C.c_void_p, C.c_void_p, C.POINTER(C.c_int), C.c_char_p, C.c_int]
    c.EVP_EncryptFinal_ex.argtypes = [C.c_void_p, C.c_void_p, C.POINTER(C.c_int)]
    c.EVP_CIPHER_CTX_ctrl.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_void_p]
    return c


def evp_seal(cipher: str, key: bytes, iv: bytes, ad: bytes, pt: bytes) -> bytes:
    c = _evp()
    ctx = c.EVP_CIPHER_CTX_new()
    try:
        assert c.EVP_EncryptInit_ex(ctx, getattr(c, cipher)(), None, None, None) == 1
        assert c.EVP_CIPHER_CTX_ctrl(ctx, EVP_CTRL_AEAD_SET_IVLEN, len(iv), None) == 1
        if cipher == "EVP_aes_256_ocb":
            assert c.EVP_CIPHER_CTX_ctrl(ctx, EVP_CTRL_AEAD_SET_TAG, 16, None) == 1
        assert c.EVP_EncryptInit_ex(ctx, None, None, key, iv) == 1
        n = C.c_int(0)
        if ad:
            assert c.EVP_EncryptUpdate(ctx, None, C.byref(n), ad, len(ad)) == 1
        out = C.create_string_buffer(len(pt) + 32)
        total = 0
        if pt:
            assert c.EVP_EncryptUpdate(ctx, out, C.byref(n), pt, len(pt)) == 1
            total = n.value
        assert c.EVP_EncryptFinal_ex(ctx, C.byref(out, total), C.byref(n)) == 1
        total += n.value
        tag = C.create_string_buffer(16)
        assert c.EVP_CIPHER_CTX_ctrl(ctx, EVP_CTRL_AEAD_GET_TAG, 16, tag) == 1
        return out.raw[:total] + tag.raw
    finally:
        c.EVP_CIPHER_CTX_free(ctx)


def evp_chacha20(key: bytes, iv16: bytes, data: bytes) -> bytes:
    c = _evp()
    ctx = c.EVP_CIPHER_CTX_new()
    try:
        assert c.EVP_EncryptInit_ex(ctx, c.EVP_chacha20(), None, key, iv16) == 1
        out = C.create_string_buffer(len(data) + 64)
        n = C.c_int(0)
        assert c.EVP_EncryptUpdate(ctx, out, C.byref(n), data, len(data)) == 1
        return out.raw[:n.value]
    finally:
        c.EVP_CIPHER_CTX_free(ctx)


def evp_poly1305(key: bytes, msg: bytes) -> bytes:
    c = _crypto
    c.EVP_MAC_fetch.restype = C.c_void_p
    c.EVP_MAC_fetch.argtypes = [C.c_void_p, C.c_char_p, C.c_char_p]
    c.EVP_MAC_CTX_new.restype = C.c_void_p
    c.EVP_MAC_CTX_new.argtypes = [C.c_void_p]
    c.EVP_MAC_init.argtypes = [C.c_void_p, C.c_char_p, C.c_size_t, C.c_void_p]
    c.EVP_MAC_update.argtypes = [C.c_void_p, C.c_char_p, C.c_size_t]
    c.EVP_MAC_final.argtypes = [C.c_void_p, C.c_char_p, C.POINTER(C.c_size_t), C.c_size_t]
    c.EVP_MAC_CTX_free.argtypes = [C.c_void_p]
    c.EVP_MAC_free.argtypes = [C.c_void_p]
    mac = c.EVP_MAC_fetch(None, b"POLY1305", None)
    ctx = c.EVP_MAC_CTX_new(mac)
    try:
        assert c.EVP_MAC_init(ctx, key, 32, None) == 1
        if msg:
            assert c.EVP_MAC_update(ctx, msg, len(msg)) == 1
        out = C.create_string_buffer(16)
        n = C.c_size_t(0)
        assert c.EVP_MAC_final(ctx, out, C.byref(n), 16) == 1
        return out.raw[:n.value]
    finally:
        c.EVP_MAC_CTX_free(ctx)
        c.EVP_MAC_free(mac)


