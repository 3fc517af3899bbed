"""Authentication (C3): OpenBridge token validation, dev tokens, and the ASGI auth middleware.

Behaviour follows ``/root/reference/app/core/security.py``:
* token from the ``bridge-user`` cookie (JSON with ``token``) or ``Authorization: Bearer``;
* validation: ES256 against the IdP JWKS (cached 300 s) + OAuth2 introspection for user metadata
  (cached 60 s per ``sub``), falling back to introspection alone; in ``ENVIRONMENT=local`` a failed
  validation falls back to the HS256 development token (mock introspection);
* on success ``request.state.jwt_data`` (active / user_id / group_id) and ``request.state.decoded_jwt``
  (sub / aud / scp=available models / exp) are set; errors answer ``{"detail", "status_code"}``.

Fixes: the validator is built lazily (no crash when the client secret is unset),
and the middleware is pure ASGI so it also authenticates the ``/api/v1/logs/{job_id}`` WebSocket
(cookie, bearer header or ``?token=``), which the reference leaves open.
"""
from __future__ import annotations

import datetime as _dt
import json
import logging
import time
from urllib.parse import parse_qs

import httpx
from pydantic import BaseModel

from . import jwt as jose

logger = logging.getLogger("ftc.auth")


class HTTPAuthError(Exception):
    def __init__(self, status_code: int, detail: str):
        super().__init__(detail)
        self.status_code, self.detail = status_code, detail


class CookieData(BaseModel):
    subject: str
    user_type: str
    config: dict | None = None
    resources: list[str]
    token: str


class UserJWT(BaseModel):
    user_id: str
    audience: str | list[str] | None = None
    available_models: list[str]
    expires: int | None = None


class JWTExtraInfo(BaseModel):
    active: bool
    user_id: str | None = None
    group_id: str | None = None


def decode_jwt(token: str) -> UserJWT:
    try:
        p = jose.get_unverified_claims(token)
    except jose.JWTError as e:
        raise HTTPAuthError(401, f"Invalid token: {e}") from e
    return UserJWT(user_id=str(p.get("sub")), audience=p.get("aud"), available_models=list(p.get("scp") or []),
                   expires=p.get("exp"))


class TokenValidator:
    def __init__(self, jwks_url: str | None, introspection_url: str | None, client_id: str | None,
                 client_secret: str | None, jwks_cache_time: int = 300, metadata_cache_time: int = 60,
                 http: httpx.AsyncClient | None = None):
        self.jwks_url, self.introspection_url = jwks_url, introspection_url
        self.client_id, self.client_secret = client_id, client_secret
        self.jwks_cache_time, self.metadata_cache_time = jwks_cache_time, metadata_cache_time
        self._jwks, self._jwks_ts = None, 0.0
        self._meta: dict[str, tuple[float, dict]] = {}
        self._http = http

    def _client(self):
        return self._http or httpx.AsyncClient(timeout=10.0)

    async def _fetch_jwks(self) -> dict:
        now = time.time()
        if self._jwks is None or now - self._jwks_ts > self.jwks_cache_time:
            c = self._client()
            try:
                r = await c.get(self.jwks_url)
                r.raise_for_status()
                self._jwks, self._jwks_ts = r.json(), now
            finally:
                if c is not self._http:
                    await c.aclose()
        return self._jwks

    async def _public_jwk(self, token: str) -> dict | None:
        if not self.jwks_url:
            return None
        try:
            kid = jose.get_unverified_header(token).get("kid")
            if not kid:
                return None
            for k in (await self._fetch_jwks()).get("keys", []):
                if k.get("kid") == kid:
                    return k
        except Exception:
            return None
        return None

    async def _introspect(self, token: str) -> dict:
        if not self.introspection_url:
            raise HTTPAuthError(401, "Invalid token")
        c = self._client()
        try:
            r = await c.post(self.introspection_url, data={"token": token},
                             auth=httpx.BasicAuth(self.client_id or "", self.client_secret or ""),
                             headers={"Content-Type": "application/x-www-form-urlencoded"})
            r.raise_for_status()
            return r.json()
        finally:
            if c is not self._http:
                await c.aclose()

    def _cached(self, sub: str) -> dict | None:
        v = self._meta.get(sub)
        if v and time.time() - v[0] <= self.metadata_cache_time:
            return v[1]
        self._meta.pop(sub, None)
        return None

    async def validate_token(self, token: str) -> dict:
        jwk = await self._public_jwk(token)
        if jwk is not None:
            try:
                payload = jose.decode_es256(token, jwk, audience=None, verify_exp=True)
                if "sub" in payload and (hit := self._cached(payload["sub"])) is not None:
                    return hit
            except jose.JWTError:
                pass  # fall through to introspection
        info = await self._introspect(token)
        if not info.get("active", False):
            raise HTTPAuthError(401, "Invalid token")
        if "sub" in info:
            now = time.time()
            if len(self._meta) >= 1024:  # users who never came back: drop their expired entries
                self._meta = {k: v for k, v in self._meta.items() if now - v[0] <= self.metadata_cache_time}
            self._meta[info["sub"]] = (now, info)
        return info


# ---------------------------------------------------------------- development tokens
def dev_generate_token(secret: str, algorithm: str, user: str, models: list[str], hours: float = 1.0) -> str:
    if not secret:
        raise HTTPAuthError(500, "JWT_SECRET_KEY not configured. Please set it in your environment variables.")
    if algorithm != "HS256":
        raise HTTPAuthError(500, f"unsupported JWT_ALGORITHM {algorithm}")
    now = _dt.datetime.now(_dt.timezone.utc)
    return jose.encode_hs256({"sub": user, "aud": "local", "scp": models, "exp": now + _dt.timedelta(hours=hours),
                              "iat": now}, secret)


def verify_token(secret: str, algorithm: str, token: str) -> dict:
    if not secret:
        raise HTTPAuthError(500, "JWT_SECRET_KEY not configured. Please set it in your environment variables.")
    try:
        return jose.decode_hs256(token, secret, audience="local")
    except jose.ExpiredSignatureError as e:
        raise HTTPAuthError(401, "Token has expired") from e
    except jose.JWTError as e:
        raise HTTPAuthError(401, "Could not validate token") from e


def dev_mock_token_introspection(secret: str, algorithm: str, token: str) -> dict:
    p = verify_token(secret, algorithm, token)
    return {"active": True, "client_id": "client-id", "sub": p.get("sub"), "group_id": "mock-group-id"}


# ---------------------------------------------------------------- ASGI middleware
def _token_from_scope(scope) -> str:
    headers = {k.decode().lower(): v.decode() for k, v in scope.get("headers", [])}
    cookies = {}
    for part in headers.get("cookie", "").split(";"):
        if "=" in part:
            k, v = part.strip().split("=", 1)
            cookies[k] = v
    if "bridge-user" in cookies:
        raw = cookies["bridge-user"]
        # a cookie the client controls: anything unreadable is a 401, not a server error
        try:
            if raw.startswith('"') and raw.endswith('"'):
                raw = raw[1:-1].encode().decode("unicode_escape")
            try:
                data = json.loads(raw)
            except ValueError:
                from urllib.parse import unquote

                data = json.loads(unquote(raw))
            if not isinstance(data, dict) or not data.get("token"):
                raise ValueError("no token")
            return CookieData(**data).token
        except (ValueError, TypeError) as e:  # (pydantic's ValidationError is a ValueError)
            raise HTTPAuthError(401, "Missing or invalid Authorization header") from e
    auth = headers.get("authorization", "")
    if auth.startswith("Bearer "):
        return auth.split(" ", 1)[1]
    if scope["type"] == "websocket":
        q = parse_qs(scope.get("query_string", b"").decode())
        if q.get("token"):
            return q["token"][0]
    raise HTTPAuthError(401, "Missing or invalid Authorization header")


class OpenBridgeAuthMiddleware:
    def __init__(self, app, settings, validator_factory):
        self.app = app
        self.settings = settings
        self._factory = validator_factory
        self._validator = None

    @property
    def validator(self) -> TokenValidator:
        if self._validator is None:
            self._validator = self._factory()
        return self._validator

    async def __call__(self, scope, receive, send):
        if scope["type"] not in ("http", "websocket") or not scope["path"].startswith(self.settings.API_V1_STR):
            return await self.app(scope, receive, send)
        try:
            token = _token_from_scope(scope)
            try:
                info = await self.validator.validate_token(token)
            except Exception:
                if self.settings.ENVIRONMENT == "local":
                    logger.warning("local environment: using mock generated tokens")
                    info = dev_mock_token_introspection(self.settings.JWT_SECRET_KEY, self.settings.JWT_ALGORITHM, token)
                else:
                    raise
            state = scope.setdefault("state", {})
            state["jwt_data"] = JWTExtraInfo(active=bool(info.get("active")), user_id=info.get("sub"),
                                             group_id=info.get("group_id"))
            try:
                state["decoded_jwt"] = decode_jwt(token)
            except HTTPAuthError:
                # opaque (non-JWT) access token validated by introspection: claims come from the IdP
                scp = info.get("scp") or [x for x in str(info.get("scope", "")).split() if x]
                state["decoded_jwt"] = UserJWT(user_id=str(info.get("sub") or info.get("username")),
                                               audience=info.get("aud"), available_models=list(scp),
                                               expires=info.get("exp"))
        except HTTPAuthError as e:
            return await self._deny(scope, receive, send, e.status_code, e.detail)
        except Exception as e:
            logger.error("error validating token: %s", e, exc_info=True)
            return await self._deny(scope, receive, send, 500, "Something went wrong")
        return await self.app(scope, receive, send)

    @staticmethod
    async def _deny(scope, receive, send, status, detail):
        if scope["type"] == "websocket":
            await send({"type": "websocket.close", "code": 1008, "reason": str(detail)[:120]})
            return
        body = json.dumps({"detail": detail, "status_code": status}).encode()
        await send({"type": "http.response.start", "status": status,
                    "headers": [(b"content-type", b"application/json"), (b"content-length", str(len(body)).encode())]})
        await send({"type": "http.response.body", "body": body})


def auth_enabled(settings) -> bool:
    """The reference's install matrix (``/root/reference/app/api/middleware.py:21-45``)."""
    configured = bool(settings.OPENBRIDGE_INTROSPECTION_URL and settings.OPENBRIDGE_CLIENT_ID
                      and settings.OPENBRIDGE_CLIENT_SECRET)
    if not configured:
        if settings.ENVIRONMENT != "local":
            logger.critical("OpenBridge middleware not configured. Your API routes are exposed!")
        else:
            logger.warning("OpenBridge middleware not configured. Missing introspection URL or API key")
        return False
    if settings.ENVIRONMENT in ("local", "staging") and settings.DEV_DISABLE_INTROSPECTION:
        logger.warning("OpenBridge introspection disabled for development")
        return False
    return True
