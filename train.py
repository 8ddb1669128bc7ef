#!/usr/bin/env python
"""Training entry point (reference flags + strategy selection); see distributedtensorflow_amd/cli.py."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from distributedtensorflow_amd.cli import main  # noqa: E402

if __name__ == "__main__":
    sys.exit(main())
