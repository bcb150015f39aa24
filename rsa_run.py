#!/usr/bin/env python3
"""Drop-in run entry point (see ruleset-analysis_amd/cli.py)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import rsa_pkg  # noqa: E402

rsa_pkg.load()
from ruleset_analysis_amd.cli import run_main  # noqa: E402

if __name__ == '__main__':
    sys.exit(run_main())
