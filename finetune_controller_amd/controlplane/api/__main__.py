"""``python -m finetune_controller_amd.controlplane.api`` (console script ``ftc-api``) -- the API server.

Same process layout as the reference image (``/root/reference/Dockerfile:28``: uvicorn, 4 workers,
per-message deflate off); the app is built per worker by ``app_from_env`` (no import-time side effects).
"""
import argparse
import sys


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="ftc-api")
    ap.add_argument("--host", default="0.0.0.0")
    ap.add_argument("--port", type=int, default=8000)
    ap.add_argument("--workers", type=int, default=4)
    ap.add_argument("--log-level", default="info")
    a = ap.parse_args(argv)
    import uvicorn

    uvicorn.run("finetune_controller_amd.controlplane.api.app:app_from_env", factory=True, host=a.host, port=a.port,
                workers=a.workers, ws_per_message_deflate=False, log_level=a.log_level)
    return 0


if __name__ == "__main__":
    sys.exit(main())
