"""CPU: the C-ABI library loads and exports every symbol include/bdls_hip.h
declares; host-only entry points (DER parsing) match the oracle; without a GPU
the engine fails loudly instead of falling back to the CPU."""
import ctypes
import os
import re

import pytest

from bdls_amd import _lib
from bdls_amd.bccsp import parse_der_sig
from oracle import ecdsa_ref as O
from tests.conftest import ROOT

HEADER = os.path.join(ROOT, "include", "bdls_hip.h")


def declared_symbols():
    txt = open(HEADER).read()
    return sorted(set(re.findall(r"\b(bh_[a-z0-9_]+)\s*\(", txt)))


def test_header_symbols_exported():
    L = _lib.lib()
    syms = declared_symbols()
    assert len(syms) >= 10
    for s in syms:
        assert hasattr(L, s), s
    assert set(syms) == set(_lib.EXPORTS)


def test_version():
    assert b"gfx950" in _lib.lib().bh_version()


def test_parse_der_matches_oracle(golden):
    for r in golden:
        sig = bytes.fromhex(r["sig"])
        rc, rv, sv = parse_der_sig(sig)
        want, wr, ws = O.unmarshal_ecdsa_signature(sig)
        assert rc == want, r["tag"]
        if rc == O.R_OK:
            assert rv == (wr if wr < 2**256 else None), r["tag"]
            assert sv == (ws if ws < 2**256 else None), r["tag"]


def test_parse_der_fuzz():
    import random
    rng = random.Random(7)
    base = O.marshal_ecdsa_signature(2**255 + 12345, 2**200 + 7)
    for _ in range(4000):
        b = bytearray(base)
        for _ in range(rng.randrange(1, 4)):
            op = rng.randrange(3)
            if op == 0 and b:
                b[rng.randrange(len(b))] = rng.randrange(256)
            elif op == 1 and b:
                del b[rng.randrange(len(b))]
            else:
                b.insert(rng.randrange(len(b) + 1), rng.randrange(256))
        sig = bytes(b)
        rc, rv, sv = parse_der_sig(sig)
        want, wr, ws = O.unmarshal_ecdsa_signature(sig)
        assert rc == want, sig.hex()
        if rc == O.R_OK:
            assert rv == (wr if wr < 2**256 else None) and sv == (ws if ws < 2**256 else None)


def test_no_gpu_fails_loudly():
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is visible")
    rc = _lib.lib().bh_init(0, 0)
    assert rc != 0
    assert _lib.last_error()
    from bdls_amd.bccsp import HipCSP
    with pytest.raises(_lib.EngineError):
        HipCSP()
