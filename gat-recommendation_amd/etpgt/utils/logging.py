"""Logging — API of etpgt/utils/logging.py (reference, :8-56): ``get_logger(name,
level, log_file)`` with a console handler (rich when importable) and an optional file
handler; repeated calls do not stack handlers."""

from __future__ import annotations

import logging


def get_logger(name: str, level: int = logging.INFO, log_file: str | None = None) -> logging.Logger:
    logger = logging.getLogger(name)
    logger.setLevel(level)
    if logger.handlers:
        return logger
    try:
        from rich.logging import RichHandler

        console: logging.Handler = RichHandler(rich_tracebacks=True, markup=True, show_time=True, show_path=True)
        console.setFormatter(logging.Formatter("%(message)s", datefmt="[%Y-%m-%d %H:%M:%S]"))
    except ImportError:  # rich is optional here
        console = logging.StreamHandler()
        console.setFormatter(logging.Formatter("%(asctime)s %(levelname)s %(message)s", datefmt="%H:%M:%S"))
    console.setLevel(level)
    logger.addHandler(console)
    if log_file:
        fh = logging.FileHandler(log_file)
        fh.setLevel(level)
        fh.setFormatter(logging.Formatter("%(asctime)s - %(name)s - %(levelname)s - %(message)s",
                                          datefmt="%Y-%m-%d %H:%M:%S"))
        logger.addHandler(fh)
    return logger
