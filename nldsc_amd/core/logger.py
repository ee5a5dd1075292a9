"""Logger `nldsc` (message texts as nldsc/core/logger.py; stderr only unless $NLDSC_LOG_FILE is set,
the reference always creates ./nldsc.log at import time)."""
import logging
import os
import sys

log = logging.getLogger("nldsc")
if not log.handlers:
    log.setLevel(logging.DEBUG)
    _h = logging.StreamHandler(sys.stderr)
    _h.setLevel(logging.INFO)
    _h.setFormatter(logging.Formatter(" > %(message)s"))
    log.addHandler(_h)
    if os.environ.get("NLDSC_LOG_FILE"):
        _f = logging.FileHandler(os.environ["NLDSC_LOG_FILE"])
        _f.setLevel(logging.INFO)
        _f.setFormatter(logging.Formatter("%(asctime)s  %(name)s  %(levelname)s: %(message)s"))
        log.addHandler(_f)
    log.propagate = False
