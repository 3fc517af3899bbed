"""Per-client sliding-window limiter (controlplane/api/ratelimit.py)."""
import pytest

from finetune_controller_amd.controlplane.api import ratelimit as rl


def test_sliding_window_and_idle_clients_are_forgotten(monkeypatch):
    now = [1000.0]
    monkeypatch.setattr(rl.time, "monotonic", lambda: now[0])
    lim = rl.Limiter()
    lim.SWEEP_EVERY = 8
    for _ in range(2):
        lim.hit("promote", "10.0.0.1", "2/minute")
    with pytest.raises(rl.RateLimitExceeded):
        lim.hit("promote", "10.0.0.1", "2/minute")
    now[0] += 61  # the window slid past both hits
    lim.hit("promote", "10.0.0.1", "2/minute")
    # many one-off clients, then time passes: their windows are swept, the table does not grow forever
    for i in range(100):
        lim.hit("jobs", f"192.168.0.{i}", "50/minute")
    now[0] += 120
    for _ in range(8):
        lim.hit("jobs", "10.9.9.9", "50/minute")
    assert len(lim._hits) <= 2 and ("jobs", "10.9.9.9") in lim._hits
