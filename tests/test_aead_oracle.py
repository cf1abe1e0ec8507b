"""CPU pins of oracle/aead_oracle.py (the restatement of kcptube's AEAD packet modes):
every primitive against the container's OpenSSL 3 libcrypto -- an independent implementation of the same
published standards (Botan, the reference's library, is absent) -- plus the draft-irtf-cfrg-xchacha HChaCha20
vector, and the kcptube composition's own layout rules."""
from __future__ import annotations

import hashlib
import random
import struct

import pytest

from oracle import aead_oracle as ao

from oracle.libcrypto import AVAILABLE, evp_chacha20, evp_poly1305, evp_seal

needs_crypto = pytest.mark.skipif(not AVAILABLE, reason="libcrypto.so.3 not loadable")


LENGTHS = [0, 1, 15, 16, 17, 31, 63, 64, 65, 100, 255, 1024, 1447]


def _rb(rng, n):
    return bytes(rng.getrandbits(8) for _ in range(n))


@needs_crypto
def test_chacha20_block_64bit_counter_vs_libcrypto():
    """kcptube's chacha20 mode: 8-byte nonce, 64-bit counter in words 12-13 (OpenSSL's 16-byte IV is words
    12-15 verbatim, so the same state)."""
    rng = random.Random(1)
    for ctr in (0, 1, 2, 0xFFFFFFFF, 0x100000001):
        key, n = _rb(rng, 32), _rb(rng, 8)
        iv16 = struct.pack("<II", ctr & 0xFFFFFFFF, ctr >> 32) + n
        assert ao.chacha20_block(key, ctr, n) == evp_chacha20(key, iv16, b"\x00" * 64)
    key, n12 = _rb(rng, 32), _rb(rng, 12)
    assert ao.chacha20_block(key, 7, n12) == evp_chacha20(key, struct.pack("<I", 7) + n12, b"\x00" * 64)


@needs_crypto
def test_poly1305_vs_libcrypto():
    rng = random.Random(2)
    for n in LENGTHS + [16 * 90, 16 * 90 + 3]:
        key, msg = _rb(rng, 32), _rb(rng, n)
        assert ao.poly1305(key, msg) == evp_poly1305(key, msg), n


@needs_crypto
def test_chacha20poly1305_ietf_vs_libcrypto():
    rng = random.Random(3)
    for n in LENGTHS:
        key, nonce, pt = _rb(rng, 32), _rb(rng, 12), _rb(rng, n)
        assert ao.chacha20poly1305_seal(key, nonce, ao.AD, pt) == evp_seal("EVP_chacha20_poly1305", key, nonce,
                                                                            ao.AD, pt), n


@needs_crypto
def test_chacha20poly1305_draft_from_pinned_primitives():
    """The 8-byte-nonce construction Botan uses for kcptube's chacha20 mode, rebuilt from libcrypto's raw
    ChaCha20 and Poly1305: poly key = block 0, data from block 1, MAC over AD || le64 || C || le64."""
    rng = random.Random(4)
    for n in LENGTHS:
        key, nonce, pt = _rb(rng, 32), _rb(rng, 8), _rb(rng, n)
        polykey = evp_chacha20(key, b"\x00" * 8 + nonce, b"\x00" * 32)
        ct = evp_chacha20(key, struct.pack("<II", 1, 0) + nonce, pt)
        tag = evp_poly1305(polykey, ao.AD + struct.pack("<Q", len(ao.AD)) + ct + struct.pack("<Q", len(ct)))
        assert ao.chacha20poly1305_seal(key, nonce, ao.AD, pt) == ct + tag, n


def test_hchacha20_draft_vector():
    """draft-irtf-cfrg-xchacha-03, 2.2.1."""
    key = bytes(range(32))
    nonce = bytes.fromhex("000000090000004a0000000031415927")
    sub = ao.hchacha20(key, nonce)
    assert sub.hex() == "82413b4227b27bfed30e42508a877d73a0f9e4d58a74a853c12ec41326d3ecdc"


@needs_crypto
def test_xchacha20poly1305_ietf_layer_vs_libcrypto():
    """XChaCha20-Poly1305 = RFC 8439 under the HChaCha20 subkey with nonce 0^4 || n[16:24]: the RFC 8439
    layer is pinned here, HChaCha20 by its draft vector (the composition itself: parity unpinned)."""
    rng = random.Random(5)
    for n in LENGTHS:
        key, nonce, pt = _rb(rng, 32), _rb(rng, 24), _rb(rng, n)
        sub = ao.hchacha20(key, nonce[:16])
        assert ao.chacha20poly1305_seal(key, nonce, ao.AD, pt) == evp_seal(
            "EVP_chacha20_poly1305", sub, b"\x00" * 4 + nonce[16:], ao.AD, pt), n


@needs_crypto
@pytest.mark.parametrize("n", [0, 1, 16, 17, 100, 1447])
def test_aes256_gcm_16byte_iv_vs_libcrypto(n):
    rng = random.Random(6 + n)
    key, iv, pt = _rb(rng, 32), _rb(rng, 16), _rb(rng, n)
    assert ao.gcm_seal(key, iv, ao.AD, pt) == evp_seal("EVP_aes_256_gcm", key, iv, ao.AD, pt)


@needs_crypto
@pytest.mark.parametrize("n", [0, 1, 15, 16, 17, 48, 100, 1447])
def test_aes256_ocb_12byte_nonce_vs_libcrypto(n):
    rng = random.Random(7 + n)
    key, nonce, pt = _rb(rng, 32), _rb(rng, 12), _rb(rng, n)
    ct_tag = ao.ocb_seal(key, nonce, ao.AD, pt)
    assert ct_tag == evp_seal("EVP_aes_256_ocb", key, nonce, ao.AD, pt)
    assert ao.ocb_open(key, nonce, ao.AD, ct_tag) == pt


def test_kcptube_composition_layout():
    """Key = SHA-3(256)(password); nonce = iv_raw repeated; packet = ct || tag || iv_raw (LE16);
    empty data is refused; a flipped bit anywhere fails to open; the wrong password fails to open."""
    rng = random.Random(8)
    pw = b"kcptube test password"
    assert ao.derive_key(pw) == hashlib.sha3_256(pw).digest()
    assert ao.nonce("aes_gcm", 0xA1B2) == bytes.fromhex("b2a1") * 8
    assert ao.nonce("aes_ocb", 0xA1B2) == bytes.fromhex("b2a1") * 6
    assert ao.nonce("chacha20", 0xA1B2) == bytes.fromhex("b2a1") * 4
    assert ao.nonce("xchacha20", 0xA1B2) == bytes.fromhex("b2a1") * 12
    for mode in ao.MODES:
        assert ao.aead_seal(mode, pw, b"", 1) is None
        for n in (1, 17, 300):
            pt = _rb(rng, n)
            iv = rng.getrandbits(16)
            pkt = ao.aead_seal(mode, pw, pt, iv)
            assert len(pkt) == n + 16 + 2 and pkt[-2:] == struct.pack("<H", iv)
            assert ao.aead_open(mode, pw, pkt) == (pt, True)
            bad = bytearray(pkt)
            bad[rng.randrange(len(pkt) - 2)] ^= 0x04
            assert ao.aead_open(mode, pw, bytes(bad)) == (b"", False)
            assert ao.aead_open(mode, b"other", pkt) == (b"", False)
        assert ao.aead_open(mode, pw, b"\x01\x02") == (b"", False)
