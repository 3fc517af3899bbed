"""Logging setup (C19): root INFO, ``ftc`` / ``app`` loggers DEBUG, coloured console output.

Mirrors ``/root/reference/app/utils/logging_config.py:5-44`` (which uses colorlog); the colour
formatter here is built in so no extra dependency is needed.
"""
from __future__ import annotations

import logging
import logging.config
import sys

_COLORS = {"DEBUG": "\033[36m", "INFO": "\033[32m", "WARNING": "\033[33m", "ERROR": "\033[31m",
           "CRITICAL": "\033[31;47m"}


class ColorFormatter(logging.Formatter):
    def __init__(self, fmt=None, use_color: bool | None = None):
        super().__init__(fmt or "%(asctime)s - %(name)s - %(levelname)s - %(message)s")
        self.use_color = sys.stderr.isatty() if use_color is None else use_color

    def format(self, record):
        s = super().format(record)
        if self.use_color:
            c = _COLORS.get(record.levelname, "")
            return f"{c}{s}\033[0m" if c else s
        return s


LOGGING_CONFIG = {
    "version": 1,
    "disable_existing_loggers": False,
    "formatters": {"colored": {"()": ColorFormatter}},
    "handlers": {"console": {"class": "logging.StreamHandler", "formatter": "colored", "level": "DEBUG"}},
    "loggers": {
        "": {"handlers": ["console"], "level": "INFO", "propagate": True},
        "ftc": {"handlers": ["console"], "level": "DEBUG", "propagate": False},
    },
}

_done = False


def setup_logging(force: bool = False) -> None:
    global _done
    if _done and not force:
        return
    logging.config.dictConfig(LOGGING_CONFIG)
    _done = True
