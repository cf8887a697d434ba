"""Console + file logging with the reference's formats (util.py:98-114).

The reference uses ``colorlog`` (not installed here); the stream handler reproduces its
format ``' %(asctime)s %(filename)s [line:%(lineno)d] %(levelname)s %(message)s'`` with
ANSI colour on TTYs. The rank-0 file logger writes ``<save_folder>/log-ing`` (file name
kept for compatibility). The reference's undefined ``root_path`` fallback
is replaced by the current directory.
"""
from __future__ import annotations

import logging
import os
import sys

STREAM_FMT = " %(asctime)s %(filename)s [line:%(lineno)d] %(levelname)s %(message)s"
FILE_FMT = "%(asctime)s %(filename)s [line:%(lineno)d] %(levelname)s %(message)s"
_COLORS = {"DEBUG": "\033[36m", "INFO": "\033[32m", "WARNING": "\033[33m", "ERROR": "\033[31m",
           "CRITICAL": "\033[1;31m"}


class _ColorFormatter(logging.Formatter):
    def format(self, record):
        s = super().format(record)
        c = _COLORS.get(record.levelname)
        if c and sys.stderr.isatty():
            s = s.replace(record.levelname, f"{c}{record.levelname}\033[0m", 1)
        return s


def set_stream_logger(log_level=logging.DEBUG):
    for h in logging.root.handlers:
        if getattr(h, "_sdx_stream", False):
            return h
    sh = logging.StreamHandler()
    sh.setLevel(log_level)
    sh.setFormatter(_ColorFormatter(STREAM_FMT))
    sh._sdx_stream = True
    logging.root.addHandler(sh)
    return sh


def set_file_logger(work_dir=None, log_level=logging.DEBUG):
    work_dir = work_dir or os.getcwd()
    os.makedirs(work_dir, exist_ok=True)
    fh = logging.FileHandler(os.path.join(work_dir, "log-ing"))
    fh.setLevel(log_level)
    fh.setFormatter(logging.Formatter(FILE_FMT))
    logging.root.addHandler(fh)
    return fh


def setup_logging(save_folder: str, rank: int):
    logging.root.setLevel(logging.INFO)
    set_stream_logger(logging.DEBUG)
    if rank == 0:
        set_file_logger(work_dir=save_folder, log_level=logging.DEBUG)
