"""Minimal JOSE: HS256 sign/verify and ES256 (P-256 ECDSA) verification from a JWK.

The reference uses python-jose (``/root/reference/app/core/security.py:5``); this dependency-free
implementation covers what the OpenBridge flow needs: HS256 development tokens, unverified claim
decoding, and ES256 signature verification against the IdP's JWKS (``kty=EC, crv=P-256``).
"""
from __future__ import annotations

import base64
import hashlib
import hmac
import json
import time


class JWTError(Exception):
    pass


class ExpiredSignatureError(JWTError):
    pass


def b64url_decode(s: str) -> bytes:
    s = s + "=" * (-len(s) % 4)
    return base64.urlsafe_b64decode(s.encode())


def b64url_encode(b: bytes) -> str:
    return base64.urlsafe_b64encode(b).rstrip(b"=").decode()


def _json_default(o):
    import datetime as _dt

    if isinstance(o, _dt.datetime):
        return int(o.timestamp())
    raise TypeError(f"not JSON serialisable: {type(o)}")


def encode_hs256(claims: dict, secret: str, headers: dict | None = None) -> str:
    h = {"alg": "HS256", "typ": "JWT", **(headers or {})}
    seg = b64url_encode(json.dumps(h, separators=(",", ":")).encode()) + "." + \
        b64url_encode(json.dumps(claims, separators=(",", ":"), default=_json_default).encode())
    sig = hmac.new(secret.encode(), seg.encode(), hashlib.sha256).digest()
    return seg + "." + b64url_encode(sig)


def _split(token: str):
    parts = token.split(".")
    if len(parts) != 3:
        raise JWTError("Not enough segments")
    try:
        header = json.loads(b64url_decode(parts[0]))
        claims = json.loads(b64url_decode(parts[1]))
    except Exception as e:
        raise JWTError(f"Invalid token encoding: {e}") from e
    if not isinstance(header, dict) or not isinstance(claims, dict):
        raise JWTError("Invalid token encoding: header and claims must be JSON objects")
    return parts, header, claims


def _signature(parts) -> bytes:
    # every malformed-token path ends in JWTError (a 401 upstream), never in a stray decoding error
    try:
        return b64url_decode(parts[2])
    except Exception as e:
        raise JWTError(f"Invalid signature encoding: {e}") from e


def get_unverified_header(token: str) -> dict:
    return _split(token)[1]


def get_unverified_claims(token: str) -> dict:
    return _split(token)[2]


def _check_claims(claims: dict, audience: str | None, verify_exp: bool, leeway: float = 0.0):
    if verify_exp and "exp" in claims:
        try:
            exp = float(claims["exp"])
        except (TypeError, ValueError) as e:
            raise JWTError("Invalid exp claim") from e
        if time.time() > exp + leeway:
            raise ExpiredSignatureError("Signature has expired")
    if audience is not None:
        aud = claims.get("aud")
        auds = aud if isinstance(aud, list) else [aud]
        if audience not in auds:
            raise JWTError("Invalid audience")


def decode_hs256(token: str, secret: str | bytes, audience: str | None = None, verify_exp: bool = True) -> dict:
    parts, header, claims = _split(token)
    if header.get("alg") != "HS256":
        raise JWTError("The specified alg value is not allowed")
    key = secret if isinstance(secret, bytes) else secret.encode()
    want = hmac.new(key, f"{parts[0]}.{parts[1]}".encode(), hashlib.sha256).digest()
    if not hmac.compare_digest(want, _signature(parts)):
        raise JWTError("Signature verification failed")
    _check_claims(claims, audience, verify_exp)
    return claims


# ---------------------------------------------------------------- P-256 ECDSA
_P = 0xFFFFFFFF00000001000000000000000000000000FFFFFFFFFFFFFFFFFFFFFFFF
_A = _P - 3
_B = 0x5AC635D8AA3A93E7B3EBBD55769886BC651D06B0CC53B0F63BCE3C3E27D2604B
_N = 0xFFFFFFFF00000000FFFFFFFFFFFFFFFFBCE6FAADA7179E84F3B9CAC2FC632551
_G = (0x6B17D1F2E12C4247F8BCE6E563A440F277037D812DEB33A0F4A13945D898C296,
      0x4FE342E2FE1A7F9B8EE7EB4A7C0F9E162BCE33576B315ECECBB6406837BF51F5)


def _jadd(p, q):
    # Jacobian point addition (None = infinity)
    if p is None:
        return q
    if q is None:
        return p
    X1, Y1, Z1 = p
    X2, Y2, Z2 = q
    Z1Z1, Z2Z2 = Z1 * Z1 % _P, Z2 * Z2 % _P
    U1, U2 = X1 * Z2Z2 % _P, X2 * Z1Z1 % _P
    S1, S2 = Y1 * Z2 * Z2Z2 % _P, Y2 * Z1 * Z1Z1 % _P
    if U1 == U2:
        if S1 != S2:
            return None
        return _jdouble(p)
    H = (U2 - U1) % _P
    R = (S2 - S1) % _P
    H2 = H * H % _P
    H3 = H * H2 % _P
    U1H2 = U1 * H2 % _P
    X3 = (R * R - H3 - 2 * U1H2) % _P
    Y3 = (R * (U1H2 - X3) - S1 * H3) % _P
    Z3 = H * Z1 * Z2 % _P
    return (X3, Y3, Z3)


def _jdouble(p):
    if p is None:
        return None
    X, Y, Z = p
    if Y == 0:
        return None
    YY = Y * Y % _P
    S = 4 * X * YY % _P
    ZZ = Z * Z % _P
    M = (3 * X * X + _A * ZZ * ZZ) % _P
    X3 = (M * M - 2 * S) % _P
    Y3 = (M * (S - X3) - 8 * YY * YY) % _P
    Z3 = 2 * Y * Z % _P
    return (X3, Y3, Z3)


def _jmul(k, p):
    r = None
    q = p
    while k:
        if k & 1:
            r = _jadd(r, q)
        q = _jdouble(q)
        k >>= 1
    return r


def _affine(p):
    if p is None:
        return None
    X, Y, Z = p
    zi = pow(Z, -1, _P)
    zi2 = zi * zi % _P
    return (X * zi2 % _P, Y * zi2 * zi % _P)


def _on_curve(x, y) -> bool:
    return (y * y - (x * x * x + _A * x + _B)) % _P == 0


def ecdsa_p256_verify(pub: tuple[int, int], msg: bytes, sig: bytes) -> bool:
    if len(sig) != 64:
        return False
    r, s = int.from_bytes(sig[:32], "big"), int.from_bytes(sig[32:], "big")
    x, y = pub
    if not (1 <= r < _N and 1 <= s < _N) or not (0 <= x < _P and 0 <= y < _P) or not _on_curve(x, y):
        return False
    z = int.from_bytes(hashlib.sha256(msg).digest(), "big")
    w = pow(s, -1, _N)
    u1, u2 = z * w % _N, r * w % _N
    pt = _affine(_jadd(_jmul(u1, (_G[0], _G[1], 1)), _jmul(u2, (pub[0], pub[1], 1))))
    return pt is not None and pt[0] % _N == r


def jwk_to_p256(jwk: dict) -> tuple[int, int]:
    if jwk.get("kty") != "EC" or jwk.get("crv") != "P-256":
        raise JWTError("unsupported JWK (need EC P-256)")
    try:
        return int.from_bytes(b64url_decode(jwk["x"]), "big"), int.from_bytes(b64url_decode(jwk["y"]), "big")
    except Exception as e:
        raise JWTError(f"malformed EC JWK: {e}") from e


def decode_es256(token: str, jwk: dict, audience: str | None = None, verify_exp: bool = True) -> dict:
    parts, header, claims = _split(token)
    if header.get("alg") != "ES256":
        raise JWTError("The specified alg value is not allowed")
    if not ecdsa_p256_verify(jwk_to_p256(jwk), f"{parts[0]}.{parts[1]}".encode(), _signature(parts)):
        raise JWTError("Signature verification failed")
    _check_claims(claims, audience, verify_exp)
    return claims


# signing helper for tests / dev IdP (deterministic-k is not needed here; random k from secrets)
def sign_es256(claims: dict, d: int, kid: str | None = None) -> str:
    import secrets

    h = {"alg": "ES256", "typ": "JWT"}
    if kid:
        h["kid"] = kid
    seg = b64url_encode(json.dumps(h, separators=(",", ":")).encode()) + "." + \
        b64url_encode(json.dumps(claims, separators=(",", ":"), default=_json_default).encode())
    z = int.from_bytes(hashlib.sha256(seg.encode()).digest(), "big")
    while True:
        k = secrets.randbelow(_N - 1) + 1
        r = _affine(_jmul(k, (_G[0], _G[1], 1)))[0] % _N
        s = pow(k, -1, _N) * (z + r * d) % _N
        if r and s:
            break
    return seg + "." + b64url_encode(r.to_bytes(32, "big") + s.to_bytes(32, "big"))


def p256_public_jwk(d: int, kid: str) -> dict:
    x, y = _affine(_jmul(d, (_G[0], _G[1], 1)))
    return {"kty": "EC", "crv": "P-256", "kid": kid, "alg": "ES256", "use": "sig",
            "x": b64url_encode(x.to_bytes(32, "big")), "y": b64url_encode(y.to_bytes(32, "big"))}
