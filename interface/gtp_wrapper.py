"""Compatibility module for ``interface/gtp_wrapper.py`` (reference): the GTP engine lives in
rocalphago_amd.gtp.engine."""
from rocalphago_amd.gtp.engine import (ExtendedGtpEngine, GTPGameConnector, PASS,  # noqa: F401
                                       _gnugo, parse_vertex, run_gtp)


def run_gnugo(sgf_file_name, command):
    out = _gnugo(sgf_file_name, command)
    return out or ""
