"""CPU: the oracle itself, pinned to the reference's fixed data.

* every committed golden record re-derives from oracle/ecdsa_ref.py;
* the independent C oracle (OpenSSL libcrypto for the group equation) agrees;
* the reference's own fixed DER reject vectors (bccsp/sw/impl_test.go:924-961)
  and boundary cases (bccsp/utils/ecdsa_test.go:19-110) hold;
* the real CA-issued signatures in msp/testdata/mspid verify as ECDSA and are
  rejected by Fabric's low-S rule, their low-S twins accept.
"""
import hashlib
import json
import os

import pytest

from oracle import ecdsa_ref as O

C = O.P256


def test_golden_rederive(golden):
    for r in golden:
        valid, reason = O.csp_verify(C, int(r["qx"], 16), int(r["qy"], 16),
                                     bytes.fromhex(r["sig"]), bytes.fromhex(r["digest"]))
        assert (valid, reason) == (r["valid"], r["reason"]), r["tag"]
        if "msg" in r:
            assert hashlib.sha256(bytes.fromhex(r["msg"])).hexdigest() == r["digest"]


def test_golden_vs_openssl(golden):
    from oracle import orc
    for r in golden:
        rc = orc.csp_verify(bytes.fromhex(r["qx"] + r["qy"]), bytes.fromhex(r["sig"]),
                            bytes.fromhex(r["digest"]))
        assert rc == r["reason"], r["tag"]


@pytest.mark.parametrize("hexv", ["300702018f0202fff1", "300702018f02020001", "300702018f02810101",
                                  "300702018f0281018f", "300a02018f020500000000 8f"])
def test_reference_der_reject_vectors(hexv):
    # bccsp/sw/impl_test.go:924-961 TestECDSASignatureEncoding
    v = bytes.fromhex(hexv.replace(" ", ""))
    with pytest.raises(O.Asn1Error):
        O.asn1_unmarshal_ecdsa_sig(v)


def test_reference_unmarshal_cases():
    # bccsp/utils/ecdsa_test.go:19-62 TestUnmarshalECDSASignature
    for raw in (b"", b"\x00"):
        assert O.unmarshal_ecdsa_signature(raw)[0] == O.R_DER
    assert O.unmarshal_ecdsa_signature(O.marshal_ecdsa_signature(-1, 1))[0] == O.R_R_NONPOS
    assert O.unmarshal_ecdsa_signature(O.marshal_ecdsa_signature(0, 1))[0] == O.R_R_NONPOS
    assert O.unmarshal_ecdsa_signature(O.marshal_ecdsa_signature(1, 0))[0] == O.R_S_NONPOS
    assert O.unmarshal_ecdsa_signature(O.marshal_ecdsa_signature(1, -1))[0] == O.R_S_NONPOS
    assert O.unmarshal_ecdsa_signature(O.marshal_ecdsa_signature(1, 1)) == (O.R_OK, 1, 1)


def test_reference_low_s_boundary():
    # bccsp/utils/ecdsa_test.go:64-89 TestIsLowS: n/2 is low, n/2 + 1 is high
    half = O.half_order(C)
    assert half == 0x7fffffff800000007fffffffffffffffde737d56d38bcf4279dce5617e3192a8
    sig_half = O.marshal_ecdsa_signature(1, half)
    sig_high = O.marshal_ecdsa_signature(1, half + 1)
    q = O.pubkey(C, 12345)
    assert O.csp_verify(C, *q, sig_half, b"\x01" * 32)[1] != O.R_HIGH_S
    assert O.csp_verify(C, *q, sig_high, b"\x01" * 32)[1] == O.R_HIGH_S


def test_marshal_roundtrip():
    for v in (1, 127, 128, 255, 256, 2**255, 2**256 - 1, -1, -128, -129, 0):
        rb = O.marshal_ecdsa_signature(v, 5)
        r, s, rest = O.asn1_unmarshal_ecdsa_sig(rb)
        assert (r, s, rest) == (v, 5, b"")


def test_mspid_fixture():
    fx = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "mspid_fixture.json")))
    qx, qy = int(fx["ca_qx"], 16), int(fx["ca_qy"], 16)
    assert O.on_curve(C, qx, qy)
    for cert in fx["certs"]:
        tbs, sig = bytes.fromhex(cert["tbs"]), bytes.fromhex(cert["sig"])
        r, s, _ = O.asn1_unmarshal_ecdsa_sig(sig)
        dg = hashlib.sha256(tbs).digest()
        # real CA signature: ECDSA-valid (Go ecdsa.Verify true) ...
        assert O.go_ecdsa_verify(C, qx, qy, dg, r, s) == O.R_OK
        # ... but high-S, so Fabric's bccsp/sw rejects it with an error
        assert s > O.half_order(C)
        assert O.csp_verify(C, qx, qy, sig, dg) == (False, O.R_HIGH_S)
        assert O.csp_verify(C, qx, qy, O.marshal_ecdsa_signature(r, C.n - s), dg) == (True, O.R_OK)


def test_mspid_fixture_matches_reference_files():
    """When the reference is mounted (this container), the committed fixture must
    equal what gen_golden.py extracts from msp/testdata/mspid."""
    ca = "/root/reference/msp/testdata/mspid/cacerts/ca.example.com-cert.pem"
    if not os.path.exists(ca):
        pytest.skip("reference not mounted")
    import importlib.util
    spec = importlib.util.spec_from_file_location(
        "gen_golden", os.path.join(os.path.dirname(__file__), "golden", "gen_golden.py"))
    g = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(g)
    der = g.pem_body(ca)
    tbs, sig = g.cert_parts(der)
    fx = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "mspid_fixture.json")))
    assert fx["certs"][0]["tbs"] == tbs.hex() and fx["certs"][0]["sig"] == sig.hex()
    assert g.cert_pubkey(der) == (int(fx["ca_qx"], 16), int(fx["ca_qy"], 16))
