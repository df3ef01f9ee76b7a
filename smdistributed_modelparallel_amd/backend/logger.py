"""Logging.

Behaviour parity with `smp/backend/logger.py:14-122`:
* ``SMP_LOG_LEVEL`` selects the level (trace/debug/info/warning/error/fatal/off, default info);
  the native runtime reads the same variable.
* ``SMP_LOG_HIDE_TIME`` drops the timestamp.
* ``SMP_LOG_ALLOW_FILES`` / ``SMP_LOG_BLOCK_FILES`` are comma-separated file-name filters.
"""
import logging
import os
import sys

TRACE = 5
logging.addLevelName(TRACE, "TRACE")

_LEVELS = {
    "trace": TRACE,
    "debug": logging.DEBUG,
    "info": logging.INFO,
    "warning": logging.WARNING,
    "warn": logging.WARNING,
    "error": logging.ERROR,
    "fatal": logging.CRITICAL,
    "critical": logging.CRITICAL,
    "off": logging.CRITICAL + 10,
}

_PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def get_log_level():
    name = os.environ.get("SMP_LOG_LEVEL", "info").strip().lower()
    return _LEVELS.get(name, logging.INFO)


class _FileFilter(logging.Filter):
    def __init__(self):
        super().__init__()
        allow = os.environ.get("SMP_LOG_ALLOW_FILES", "")
        block = os.environ.get("SMP_LOG_BLOCK_FILES", "")
        self.allow = [a.strip() for a in allow.split(",") if a.strip()]
        self.block = [b.strip() for b in block.split(",") if b.strip()]

    def filter(self, record):
        fname = os.path.basename(record.pathname)
        if self.allow and not any(a in fname for a in self.allow):
            return False
        if any(b in fname for b in self.block):
            return False
        try:
            record.relpath = os.path.relpath(record.pathname, _PKG_ROOT)
        except ValueError:
            record.relpath = record.pathname
        return True


_logger = None


def get_logger():
    global _logger
    if _logger is not None:
        return _logger
    logger = logging.getLogger("smdistributed_modelparallel_amd")
    logger.setLevel(get_log_level())
    logger.propagate = False
    if not logger.handlers:
        handler = logging.StreamHandler(sys.stdout)
        if os.environ.get("SMP_LOG_HIDE_TIME", "0") not in ("0", "", "false", "False"):
            fmt = "[%(levelname)s|%(relpath)s:%(lineno)d] %(message)s"
        else:
            fmt = "[%(asctime)s.%(msecs)03d: %(levelname)s %(relpath)s:%(lineno)d] %(message)s"
        handler.setFormatter(logging.Formatter(fmt, datefmt="%Y-%m-%d %H:%M:%S"))
        handler.addFilter(_FileFilter())
        logger.addHandler(handler)

    def trace(msg, *args, **kwargs):
        if logger.isEnabledFor(TRACE):
            logger._log(TRACE, msg, args, **kwargs)

    logger.trace = trace
    _logger = logger
    return logger
