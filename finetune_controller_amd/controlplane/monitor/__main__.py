"""``python -m finetune_controller_amd.controlplane.monitor`` -- the standalone job monitor service."""
import asyncio
import logging
import sys

from ..context import AppContext
from ..core.config import get_settings
from ..core.logging_config import setup_logging
from .reconciler import run_service


def main() -> int:
    setup_logging()
    try:
        asyncio.run(run_service(AppContext.from_settings(get_settings())))
    except KeyboardInterrupt:
        pass
    except Exception:
        logging.getLogger("ftc.monitor").exception("fatal error")
        return 1
    return 0


if __name__ == "__main__":
    sys.exit(main())
