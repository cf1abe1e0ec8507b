"""GPU parity tests of kcptube's aes_gcm / aes_ocb / chacha20 / xchacha20 packet modes (include/kfec_aead.h) against
oracle/aead_oracle.py (pinned against OpenSSL's libcrypto in tests/test_aead_oracle.py).

Bar: bit-exact sealed packets (ciphertext || tag || iv_raw) for every length class the kernels treat
differently -- lengths around the 16-byte MAC block, the 64-byte ChaCha20 block and the 512-byte row
round, with the MAC header (23 or 16 bytes) and trailer crossing chunk boundaries, and for aes_gcm past the
2048 bytes of tabulated keystream -- at unaligned source offsets; opening restores the plaintext, and any flipped bit (ciphertext, tag or iv_raw) fails with zeroed
output.  A 20k-packet batch is checked against libcrypto's ChaCha20 / Poly1305 / ChaCha20-Poly1305 /
AES-256-GCM / AES-256-OCB (the pure-Python oracle is too slow for it), and a 1M-packet batch round-trips on the device.
"""
from __future__ import annotations

import hashlib
import random
import struct

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

from oracle import aead_oracle as ao  # noqa: E402
from oracle import libcrypto as lc  # noqa: E402

MODES = ("chacha20", "xchacha20", "aes_gcm", "aes_ocb")
PW = b"kcptube aead test password"
LENGTHS = ([1, 2, 3, 4, 5, 7, 8, 9, 15, 16, 17, 23, 24, 25, 31, 32, 33, 40, 41, 42, 47, 48, 49, 55, 56, 57, 63, 64,
            65, 100, 127, 128, 129, 191, 192, 193, 255, 256, 257, 447, 448, 449, 489, 490, 495, 496, 497, 511, 512,
            513, 1000, 1400, 1420, 1449, 2047, 2048, 2049, 4095, 4096, 4100, 6000])


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from kcptube_amd import load_library
    load_library()
    return torch.device("cuda:0")


def _cipher(mode):
    from kcptube_amd.aead import AeadCipher
    return AeadCipher(mode, PW)


def _arena(chunks, dev, seed=0):
    """Byte strings at odd offsets (0-3 byte gaps) in one device buffer."""
    rng = random.Random(seed)
    buf = bytearray()
    offs, lens = [], []
    for c in chunks:
        buf += bytes(rng.randint(0, 3))
        offs.append(len(buf))
        lens.append(len(c))
        buf += c
    buf += bytes((-len(buf)) % 4 + 4)
    a = torch.tensor(np.frombuffer(bytes(buf), np.uint8).copy(), device=dev)
    return (a, torch.tensor(offs, dtype=torch.int64, device=dev),
            torch.tensor(lens, dtype=torch.int32, device=dev))


def _iv_tensor(ivs, dev):
    return torch.tensor(np.asarray(ivs, np.uint16).view(np.int16), device=dev)


def _seal(c, pts, ivs, dev, pitch=None, seed=0):
    src, off, ln = _arena(pts, dev, seed)
    pitch = pitch or (max(len(p) for p in pts) + 18 + 3) // 4 * 4 + 4
    dst = torch.full((len(pts), pitch), 0xA5, dtype=torch.uint8, device=dev)
    out = torch.full((len(pts),), -1, dtype=torch.int32, device=dev)
    c.seal(src, off, ln, _iv_tensor(ivs, dev), dst, out)
    torch.cuda.synchronize()
    return dst.cpu().numpy(), out.cpu().numpy()


def _open(c, pkts, dev, pitch=None, seed=1):
    src, off, ln = _arena(pkts, dev, seed)
    pitch = pitch or max(4, (max(len(p) for p in pkts) + 3) // 4 * 4)
    dst = torch.full((len(pkts), pitch), 0xA5, dtype=torch.uint8, device=dev)
    out = torch.full((len(pkts),), -1, dtype=torch.int32, device=dev)
    ok = torch.full((len(pkts),), 7, dtype=torch.uint8, device=dev)
    c.open_(src, off, ln, dst, out, ok)
    torch.cuda.synchronize()
    return dst.cpu().numpy(), out.cpu().numpy(), ok.cpu().numpy()


@pytest.mark.parametrize("pw", [b"x", b"kcptube", bytes(range(135)), bytes(range(136)), bytes(range(137)) * 3])
def test_key_is_sha3_256_of_the_password(dev, pw):
    from kcptube_amd.aead import AeadCipher
    for mode in MODES:
        assert AeadCipher(mode, pw).key == hashlib.sha3_256(pw).digest()


def test_refuses_empty_password_and_other_modes(dev):
    from kcptube_amd.aead import AeadCipher
    with pytest.raises(ValueError):
        AeadCipher("chacha20", b"")
    with pytest.raises(ValueError):
        AeadCipher(3, PW)  # plain_xor: not an AEAD mode (kfec_seal_batch has it)


@pytest.mark.parametrize("mode", MODES)
def test_seal_bit_exact_vs_oracle(dev, mode):
    rng = random.Random(11)
    c = _cipher(mode)
    pts = [bytes(rng.getrandbits(8) for _ in range(n)) for n in LENGTHS]
    ivs = [rng.getrandbits(16) for _ in pts] + []
    ivs[0], ivs[1] = 0, 0xFFFF
    dst, out = _seal(c, pts, ivs, dev)
    pitch = dst.shape[1]
    for p, (pt, iv) in enumerate(zip(pts, ivs)):
        want = ao.aead_seal(mode, PW, pt, iv)
        assert out[p] == len(pt) + 18, (mode, len(pt))
        got = bytes(dst[p, :out[p]])
        assert got == want, (mode, len(pt))
        end = (len(want) + 3) // 4 * 4
        assert not dst[p, len(want):end].any(), "zero pad to a multiple of 4"
        assert (dst[p, end:pitch] == 0xA5).all(), "nothing written past the padded packet"


@pytest.mark.parametrize("mode", MODES)
def test_open_roundtrip_and_forgeries(dev, mode):
    rng = random.Random(12)
    c = _cipher(mode)
    pts = [bytes(rng.getrandbits(8) for _ in range(n)) for n in LENGTHS]
    ivs = [rng.getrandbits(16) for _ in pts]
    pkts = [ao.aead_seal(mode, PW, pt, iv) for pt, iv in zip(pts, ivs)]
    dst, out, ok = _open(c, pkts, dev)
    for p, pt in enumerate(pts):
        assert ok[p] == 1 and out[p] == len(pt), (mode, len(pt))
        assert bytes(dst[p, :len(pt)]) == pt
        end = (len(pt) + 3) // 4 * 4
        assert not dst[p, len(pt):end].any()
    # one flipped bit anywhere -- ciphertext, tag, iv_raw -- fails, and leaves zeros in dst
    bad, where = [], []
    for pkt in pkts:
        for pos in {0, len(pkt) - 19, len(pkt) - 18, len(pkt) - 3, len(pkt) - 2, len(pkt) - 1,
                    rng.randrange(len(pkt))}:
            if pos < 0:
                continue
            b = bytearray(pkt)
            b[pos] ^= 1 << rng.randrange(8)
            bad.append(bytes(b))
            where.append(pos)
    dst, out, ok = _open(c, bad, dev)
    assert not ok.any() and not out.any()
    for p, pkt in enumerate(bad):
        n = len(pkt) - 18
        assert not dst[p, :(n + 3) // 4 * 4].any(), where[p]
    # the wrong key fails too
    other = __import__("kcptube_amd.aead", fromlist=["AeadCipher"]).AeadCipher(mode, PW + b"!")
    _, out, ok = _open(other, pkts[:8], dev)
    assert not ok.any()


@pytest.mark.parametrize("mode", MODES)
def test_lengths_the_reference_refuses(dev, mode):
    """seal: empty data, or no room in the pitch -> 0; open: fewer than 18 bytes (incl. <= 2) -> failure,
    exactly 18 bytes (empty ciphertext, valid tag) -> ok with no plaintext."""
    c = _cipher(mode)
    dst, out = _seal(c, [b"", b"abc", bytes(40)], [1, 2, 3], dev, pitch=40)
    assert list(out) == [0, 21, 0]
    assert bytes(dst[1, :21]) == ao.aead_seal(mode, PW, b"abc", 2)
    key, nonce = ao.derive_key(PW), ao.nonce(mode, 9)
    body = (ao.gcm_seal(key, nonce, ao.AD, b"") if mode == "aes_gcm" else
            ao.ocb_seal(key, nonce, ao.AD, b"") if mode == "aes_ocb" else
            ao.chacha20poly1305_seal(key, nonce, ao.AD, b""))
    empty_ok = body + struct.pack("<H", 9)
    pkts = [bytes(n) for n in range(18)] + [empty_ok]
    _, out, ok = _open(c, pkts, dev)
    assert not ok[:18].any() and not out.any()
    assert ok[18] == 1
    # plaintext longer than the output pitch
    big = ao.aead_seal(mode, PW, bytes(100), 5)
    _, out, ok = _open(c, [big], dev, pitch=96)
    assert out[0] == 0 and ok[0] == 0


def _libcrypto_seal(mode, key, pt, iv):
    """The same packet from libcrypto primitives (a second, independent checker for large batches)."""
    n = ao.nonce(mode, iv)
    if mode == "aes_gcm":
        return lc.evp_seal("EVP_aes_256_gcm", key, n, ao.AD, pt) + struct.pack("<H", iv)
    if mode == "aes_ocb":
        return lc.evp_seal("EVP_aes_256_ocb", key, n, ao.AD, pt) + struct.pack("<H", iv)
    if mode == "chacha20":
        polykey = lc.evp_chacha20(key, bytes(8) + n, bytes(32))
        ct = lc.evp_chacha20(key, struct.pack("<II", 1, 0) + n, pt)
        tag = lc.evp_poly1305(polykey, ao.AD + struct.pack("<Q", len(ao.AD)) + ct + struct.pack("<Q", len(ct)))
        return ct + tag + struct.pack("<H", iv)
    sub = ao.hchacha20(key, n[:16])
    return lc.evp_seal("EVP_chacha20_poly1305", sub, bytes(4) + n[16:], ao.AD, pt) + struct.pack("<H", iv)


@pytest.mark.skipif(not lc.AVAILABLE, reason="libcrypto.so.3 not loadable")
@pytest.mark.parametrize("mode", MODES)
def test_batch_vs_libcrypto(dev, mode):
    P = 20000
    g = torch.Generator(device="cpu").manual_seed(21)
    lens = torch.randint(1, 1501, (P,), generator=g).tolist()
    ivs = torch.randint(0, 65536, (P,), generator=g).tolist()
    data = np.random.default_rng(22).integers(0, 256, sum(lens), dtype=np.uint8).tobytes()
    pts, o = [], 0
    for n in lens:
        pts.append(data[o:o + n])
        o += n
    c = _cipher(mode)
    dst, out = _seal(c, pts, ivs, dev, pitch=1520)
    key = hashlib.sha3_256(PW).digest()
    for p in range(P):
        assert bytes(dst[p, :out[p]]) == _libcrypto_seal(mode, key, pts[p], ivs[p]), p


@pytest.mark.parametrize("mode", MODES)
def test_million_packets_roundtrip_on_device(dev, mode):
    """1M packets of 1..1500 bytes sealed and opened on the device: every tag verifies, plaintext returns."""
    P, pitch = 1 << 20, 1520
    g = torch.Generator(device=dev).manual_seed(31)
    lens = torch.randint(1, 1501, (P,), device=dev, dtype=torch.int32, generator=g)
    src = torch.randint(0, 256, (P * pitch,), device=dev, dtype=torch.uint8, generator=g)
    off = torch.arange(P, device=dev, dtype=torch.int64) * pitch + (torch.arange(P, device=dev) % 3)
    ivs = torch.randint(-32768, 32768, (P,), device=dev, dtype=torch.int16, generator=g)
    c = _cipher(mode)
    sealed = torch.empty((P, pitch), dtype=torch.uint8, device=dev)
    slen = torch.empty(P, dtype=torch.int32, device=dev)
    c.seal(src, off, lens, ivs, sealed, slen)
    assert torch.equal(slen, lens + 18)
    soff = torch.arange(P, device=dev, dtype=torch.int64) * pitch
    plain = torch.empty((P, pitch), dtype=torch.uint8, device=dev)
    plen = torch.empty(P, dtype=torch.int32, device=dev)
    ok = torch.empty(P, dtype=torch.uint8, device=dev)
    c.open_(sealed.view(-1), soff, slen, plain, plen, ok)
    assert bool(ok.all()) and torch.equal(plen, lens)
    col = torch.arange(pitch, device=dev)
    idx = (off.view(-1, 1) + col.view(1, -1)).clamp_(max=P * pitch - 1)
    want = torch.where(col.view(1, -1) < lens.view(-1, 1), src[idx], torch.zeros((), dtype=torch.uint8, device=dev))
    lim = ((lens + 3) // 4 * 4).view(-1, 1)
    assert torch.equal(torch.where(col.view(1, -1) < lim, plain, want), want)
