"""Structured logging in the style of the reference's logrus output.

The reference prints ``INFO[0000] message`` lines and raises the level to
Debug with ``-v`` (``cmd/move2kube/move2kube.go:41-46``).  ``fatal`` logs and
raises :class:`FatalError` (the CLI turns it into exit code 1) instead of
calling ``os.Exit`` so that the library is usable in-process and in tests.
"""

import logging
import sys
import time

_START = time.time()
_LEVEL_NAMES = {
    logging.DEBUG: "DEBU",
    logging.INFO: "INFO",
    logging.WARNING: "WARN",
    logging.ERROR: "ERRO",
    logging.CRITICAL: "FATA",
}


class FatalError(RuntimeError):
    """Raised where the reference calls ``log.Fatalf``."""


class _LogrusFormatter(logging.Formatter):
    def format(self, record):
        elapsed = int(record.created - _START)
        lvl = _LEVEL_NAMES.get(record.levelno, record.levelname[:4])
        return "%s[%04d] %s" % (lvl, elapsed, record.getMessage())


logger = logging.getLogger("move2kube")
if not logger.handlers:
    _h = logging.StreamHandler(sys.stderr)
    _h.setFormatter(_LogrusFormatter())
    logger.addHandler(_h)
    logger.setLevel(logging.INFO)
    logger.propagate = False


def set_verbose(verbose=True):
    logger.setLevel(logging.DEBUG if verbose else logging.INFO)


def set_quiet():
    logger.setLevel(logging.ERROR)


debug = logger.debug
info = logger.info
warning = logger.warning
warn = logger.warning
error = logger.error


def fatal(msg, *args):
    logger.critical(msg, *args)
    raise FatalError(msg % args if args else msg)
