"""Per-client rate limiting (C2): ``@limiter.limit("10/minute")`` on route handlers, keyed by the remote
address, same limits as the reference's SlowAPI decorators (``/root/reference/app/main.py:171-1166``).

Sliding-window counters in process memory (per API worker, like SlowAPI's default storage).
"""
from __future__ import annotations

import functools
import threading
import time
from collections import defaultdict, deque

_UNITS = {"second": 1, "minute": 60, "hour": 3600, "day": 86400}


class RateLimitExceeded(Exception):
    status_code = 429

    def __init__(self, limit: str):
        super().__init__(f"Rate limit exceeded: {limit}")
        self.limit = limit


def parse_limit(spec: str) -> tuple[int, float]:
    n, _, unit = spec.partition("/")
    unit = unit.strip().rstrip("s")
    return int(n), float(_UNITS[unit])


def remote_address(request) -> str:
    return request.client.host if request.client else "127.0.0.1"


class Limiter:
    SWEEP_EVERY = 4096  # hits between sweeps of idle (route, client) windows

    def __init__(self, key_func=remote_address, enabled: bool = True):
        self.key_func = key_func
        self.enabled = enabled
        self._hits: dict[tuple, deque] = defaultdict(deque)
        self._window: dict[tuple, float] = {}
        self._since_sweep = 0
        self._lock = threading.Lock()

    def reset(self):
        with self._lock:
            self._hits.clear()
            self._window.clear()

    def _sweep(self, now: float) -> None:
        # drop the windows of clients that have not called within their window: without this every
        # address that ever called stays in memory for the life of the worker
        for k in [k for k, q in self._hits.items() if not q or now - q[-1] >= self._window.get(k, 0.0)]:
            del self._hits[k]
            self._window.pop(k, None)

    def hit(self, route: str, key: str, spec: str) -> None:
        if not self.enabled:
            return
        n, window = parse_limit(spec)
        now = time.monotonic()
        with self._lock:
            self._since_sweep += 1
            if self._since_sweep >= self.SWEEP_EVERY:
                self._since_sweep = 0
                self._sweep(now)
            q = self._hits[(route, key)]
            self._window[(route, key)] = window
            while q and now - q[0] >= window:
                q.popleft()
            if len(q) >= n:
                raise RateLimitExceeded(spec)
            q.append(now)

    def limit(self, spec: str):
        def deco(fn):
            @functools.wraps(fn)
            async def wrapper(*args, **kwargs):
                request = kwargs.get("request")
                if request is None:
                    request = next((a for a in args if hasattr(a, "client") and hasattr(a, "url")), None)
                if request is not None:
                    self.hit(fn.__name__, self.key_func(request), spec)
                return await fn(*args, **kwargs)

            return wrapper

        return deco
