"""CPU: the device hash code (bdls_amd/csrc/sha256.h, blake2b.h -- dword loads
with funnel shifts at any byte alignment) compiled for the host by the
test-only harness, against hashlib on every length across the block edges,
large messages, and all four pointer alignments."""
import ctypes
import hashlib
import os
import random
import struct

import pytest

from tests.conftest import ROOT

LIB = os.path.join(ROOT, "tests", "native", "build", "libhostsim.so")
LENS = list(range(0, 300)) + [511, 512, 513, 1023, 1024, 1025, 4096, 4097, 13_337]


@pytest.fixture(scope="module")
def L():
    if not os.path.exists(LIB):
        pytest.skip("hostsim not built")
    return ctypes.CDLL(LIB)


def placed(msg, align):
    """msg copied at byte offset `align` of a fresh buffer (end of allocation
    right after the message, so over-reads would be visible to ASan builds)."""
    buf = ctypes.create_string_buffer(b"\xee" * align + msg, align + len(msg))
    return buf, ctypes.cast(ctypes.addressof(buf) + align, ctypes.c_void_p)


@pytest.mark.parametrize("align", [0, 1, 2, 3])
def test_sha256(L, align):
    rng = random.Random(align)
    out = (ctypes.c_uint32 * 8)()
    for n in LENS:
        m = rng.randbytes(n)
        buf, p = placed(m, align)
        L.hs_sha256(p, n, out)
        got = b"".join(struct.pack(">I", out[i]) for i in range(8))
        assert got == hashlib.sha256(m).digest(), n


@pytest.mark.parametrize("align", [0, 1, 2, 3])
def test_sha256_split_compression(L, align):
    """k_digest_grp's split form (sha256_load_block -> sha256_sched_wk ->
    sha256_rounds_wk): one span, and two spans with the seam at 0, 1, a block
    edge, the end and a random byte."""
    rng = random.Random(100 + align)
    out = (ctypes.c_uint32 * 8)()
    L.hs_sha256_split.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p,
                                  ctypes.c_uint32, ctypes.c_void_p]
    for n in LENS:
        m = rng.randbytes(n)
        want = hashlib.sha256(m).digest()
        buf, p = placed(m, align)
        L.hs_sha256_split(p, n, p, 0, out)
        assert b"".join(struct.pack(">I", out[i]) for i in range(8)) == want, n
        for k in {0, min(n, 1), min(n, 64), n, rng.randint(0, n)}:
            b1, p1 = placed(m[:k], align)
            b2, p2 = placed(m[k:], 3 - align)
            L.hs_sha256_split(p1, k, p2, n - k, out)
            assert b"".join(struct.pack(">I", out[i]) for i in range(8)) == want, (n, k)


@pytest.mark.parametrize("align", [0, 1, 2, 3])
def test_bdls_blake2b(L, align):
    # vendor/github.com/BDLS-bft/bdls/message.go:97-138 SignedProto.Hash framing
    rng = random.Random(10 + align)
    out = ctypes.create_string_buffer(32)
    for n in LENS:
        m = rng.randbytes(n)
        x, y = rng.randbytes(32), rng.randbytes(32)
        ver = rng.randrange(2**32)
        buf, p = placed(m, align)
        xb, xp = placed(x + y, align)
        L.hs_bdls_hash(ctypes.c_uint32(ver), xp, ctypes.c_void_p(xp.value + 32), p,
                       ctypes.c_uint32(n), out)
        want = hashlib.blake2b(b"BDLS_CONSENSUS_SIGNATURE" + struct.pack("<I", ver) + x + y
                               + struct.pack("<I", n) + m, digest_size=32).digest()
        assert out.raw == want, n


@pytest.mark.parametrize("align", [0, 1, 2, 3])
def test_sha3_256(L, align):
    # bccsp/sw/new.go:72 sha3.New256 (SHA3 family, msp/identities.go:219-227);
    # lengths straddle the 136-byte rate: 135/136/137, 271/272/273, ...
    rng = random.Random(20 + align)
    out = ctypes.create_string_buffer(32)
    for n in LENS + [135, 136, 137, 271, 272, 273, 407, 408, 409]:
        m = rng.randbytes(n)
        buf, p = placed(m, align)
        L.hs_sha3_256(p, ctypes.c_uint32(n), out)
        assert out.raw == hashlib.sha3_256(m).digest(), n
