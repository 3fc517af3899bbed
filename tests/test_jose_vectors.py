"""Known-answer tests for the hand-written JOSE primitives (controlplane/auth/jwt.py), the production
path of the reference's JWKS branch (/root/reference/app/core/security.py:154-176).

No independent crypto library is importable in this image (no cryptography / python-jose / ecdsa),
so the independent evidence is published vectors:

* RFC 7515 Appendix A.3 -- the ES256 JWS example (public key, compact serialization);
* RFC 6979 Appendix A.2.5 -- deterministic ECDSA on P-256 with SHA-256 (messages "sample" and
  "test"): public key from the private key, and (r, s) from the published nonce k;
* RFC 7515 Appendix A.1 -- the HS256 JWS example (HMAC key, compact serialization);
* rejection of malformed inputs: off-curve / out-of-range public keys, r or s outside [1, n-1],
  truncated and DER-encoded signatures, alg confusion.
"""
import hashlib

import pytest

from finetune_controller_amd.controlplane.auth import jwt as jose

# ---- RFC 7515 A.3 (ES256) ----
A3_JWK = {"kty": "EC", "crv": "P-256",
          "x": "f83OJ3D2xF1Bg8vub9tLe1gHMzV76e8Tus9uPHvRVEU",
          "y": "x_FEzRu9m36HLN_tue659LNpXW6pCyStikYjKIWI5a0"}
A3_TOKEN = ("eyJhbGciOiJFUzI1NiJ9"
            ".eyJpc3MiOiJqb2UiLA0KICJleHAiOjEzMDA4MTkzODAsDQogImh0dHA6Ly9leGFtcGxlLmNvbS9pc19yb290Ijp0cnVlfQ"
            ".DtEhU3ljbEg8L38VWAfUAqOyKAM6-Xx-F4GawxaepmXFCgfTjDxw5djxLa8ISlSApmWQxfKTUJqPP3-Kg6NU1Q")

# ---- RFC 6979 A.2.5 (P-256, SHA-256) ----
R6979_X = 0xC9AFA9D845BA75166B5C215767B1D6934E50C3DB36E89B127B8A622B120F6721
R6979_U = (0x60FED4BA255A9D31C961EB74C6356D68C049B8923B61FA6CE669622E60F29FB6,
           0x7903FE1008B8BC99A41AE9E95628BC64F2F1B20C2D7E9F5177A3C294D4462299)
R6979_SIGS = {
    b"sample": (0xA6E3C57DD01ABE90086538398355DD4C3B17AA873382B0F24D6129493D8AAD60,
                0xEFD48B2AACB6A8FD1140DD9CD45E81D69D2C877B56AAF991C34D0EA84EAF3716,
                0xF7CB1C942D657C41D436C7A1B6E29F65F3E900DBB9AFF4064DC4AB2F843ACDA8),
    b"test": (0xD16B6AE827F17175E040871A1C7EC3500192C4C92677336EC2537ACAEE0008E0,
              0xF1ABB023518351CD71D881567B1EA663ED3EFCF6C5132B354F28D3B0B7D38367,
              0x019F4113742A2B14BD25926B49C649155F267E60D3814B4C0CC84250E46F0083),
}

# ---- RFC 7515 A.1 (HS256) ----
A1_KEY_B64 = "AyM1SysPpbyDfgZld3umj1qzKObwVMkoqQ-EstJQLr_T-1qS0gZH75aKtMN3Yj0iPS4hcgUuTwjAzZr1Z9CAow"
A1_TOKEN = ("eyJ0eXAiOiJKV1QiLA0KICJhbGciOiJIUzI1NiJ9"
            ".eyJpc3MiOiJqb2UiLA0KICJleHAiOjEzMDA4MTkzODAsDQogImh0dHA6Ly9leGFtcGxlLmNvbS9pc19yb290Ijp0cnVlfQ"
            ".dBjftJeZ4CVP-mB92K27uhbUJU1p1r_wW1gFWFOEjXk")


def _sig(r: int, s: int) -> bytes:
    return r.to_bytes(32, "big") + s.to_bytes(32, "big")


def test_rfc7515_a3_es256_example_verifies():
    claims = jose.decode_es256(A3_TOKEN, A3_JWK, verify_exp=False)
    assert claims == {"iss": "joe", "exp": 1300819380, "http://example.com/is_root": True}
    # expiry is enforced when asked (the example expired in 2011)
    with pytest.raises(jose.ExpiredSignatureError):
        jose.decode_es256(A3_TOKEN, A3_JWK)
    # any change of the signing input or the signature fails
    h, p, s = A3_TOKEN.split(".")
    tampered = jose.b64url_encode(jose.b64url_decode(p).replace(b"joe", b"eve"))
    with pytest.raises(jose.JWTError):
        jose.decode_es256(f"{h}.{tampered}.{s}", A3_JWK, verify_exp=False)
    raw = bytearray(jose.b64url_decode(s))
    raw[10] ^= 1
    with pytest.raises(jose.JWTError):
        jose.decode_es256(f"{h}.{p}.{jose.b64url_encode(bytes(raw))}", A3_JWK, verify_exp=False)


@pytest.mark.parametrize("msg", sorted(R6979_SIGS))
def test_rfc6979_p256_sha256_vectors(msg):
    k, r, s = R6979_SIGS[msg]
    # public key from the private key (scalar multiplication)
    assert jose._affine(jose._jmul(R6979_X, (jose._G[0], jose._G[1], 1))) == R6979_U
    # the published nonce reproduces the published (r, s)
    z = int.from_bytes(hashlib.sha256(msg).digest(), "big")
    kx = jose._affine(jose._jmul(k, (jose._G[0], jose._G[1], 1)))[0] % jose._N
    assert kx == r
    assert pow(k, -1, jose._N) * (z + r * R6979_X) % jose._N == s
    # and the verifier accepts exactly that signature
    assert jose.ecdsa_p256_verify(R6979_U, msg, _sig(r, s))
    assert not jose.ecdsa_p256_verify(R6979_U, msg + b"!", _sig(r, s))


def test_rfc7515_a1_hs256_example_verifies():
    key = jose.b64url_decode(A1_KEY_B64)
    claims = jose.decode_hs256(A1_TOKEN, key, verify_exp=False)
    assert claims["iss"] == "joe" and claims["exp"] == 1300819380


def test_malformed_keys_and_signatures_are_rejected():
    k, r, s = R6979_SIGS[b"sample"]
    n, p = jose._N, jose._P
    good = _sig(r, s)
    assert jose.ecdsa_p256_verify(R6979_U, b"sample", good)
    ux, uy = R6979_U
    # public key not on the curve, or with coordinates outside the field
    assert not jose.ecdsa_p256_verify((ux, (uy + 1) % p), b"sample", good)
    assert not jose.ecdsa_p256_verify((ux + p, uy), b"sample", good)
    assert not jose.ecdsa_p256_verify((0, 0), b"sample", good)
    # r, s outside [1, n-1]
    for rr, ss in ((0, s), (r, 0), (n, s), (r, n), (r + n, s), (r, s + n)):
        if rr.bit_length() <= 256 and ss.bit_length() <= 256:
            assert not jose.ecdsa_p256_verify(R6979_U, b"sample", _sig(rr, ss))
    # truncated / padded / DER-shaped signatures
    assert not jose.ecdsa_p256_verify(R6979_U, b"sample", good[:63])
    assert not jose.ecdsa_p256_verify(R6979_U, b"sample", good + b"\x00")
    der = b"\x30\x44\x02\x20" + r.to_bytes(32, "big") + b"\x02\x20" + s.to_bytes(32, "big")
    assert not jose.ecdsa_p256_verify(R6979_U, b"sample", der)
    # ECDSA malleability: (r, n - s) is mathematically valid; like the `cryptography` backend the
    # reference's python-jose uses, it is accepted (JWS does not mandate low-S)
    assert jose.ecdsa_p256_verify(R6979_U, b"sample", _sig(r, n - s))


def test_alg_confusion_is_rejected():
    # an HS256 token must never pass the ES256 path (and vice versa)
    with pytest.raises(jose.JWTError, match="alg"):
        jose.decode_es256(A1_TOKEN, A3_JWK, verify_exp=False)
    with pytest.raises(jose.JWTError):
        jose.decode_hs256(A3_TOKEN, b"secret", verify_exp=False)
    with pytest.raises(jose.JWTError):
        jose.decode_es256(A3_TOKEN, {"kty": "EC", "crv": "P-384", "x": A3_JWK["x"], "y": A3_JWK["y"]},
                          verify_exp=False)


def test_every_malformed_token_is_a_jwt_error():
    """Garbage in any segment, a non-object header / claims, a non-numeric exp or a broken JWK must all
    surface as JWTError (a 401 upstream), never as a decoding exception (a 500)."""
    h = jose.b64url_encode(b'{"alg":"HS256"}')
    c = jose.b64url_encode(b'{"sub":"x"}')
    bad_tokens = [f"{h}.{c}.a",  # signature: 1 char past a multiple of 4 -> undecodable
                  f"{jose.b64url_encode(b'[1]')}.{c}.AAAA", f"{h}.{jose.b64url_encode(b'3')}.AAAA",
                  f"{h}.{c}", "..", "x.y.z"]
    for t in bad_tokens:
        with pytest.raises(jose.JWTError):
            jose.decode_hs256(t, b"k")
    t = jose.encode_hs256({"sub": "x", "exp": "tomorrow"}, "k")
    with pytest.raises(jose.JWTError, match="exp"):
        jose.decode_hs256(t, "k")
    with pytest.raises(jose.JWTError):
        jose.decode_es256(A3_TOKEN, {"kty": "EC", "crv": "P-256", "x": A3_JWK["x"]}, verify_exp=False)
    with pytest.raises(jose.JWTError):
        jose.decode_es256(A3_TOKEN.rsplit(".", 1)[0] + ".a", A3_JWK, verify_exp=False)
