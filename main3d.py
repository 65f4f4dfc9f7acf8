#!/usr/bin/env python3
"""Reference-compatible entry point: see triton_client_amd/cli/main3d.py."""
import sys

from triton_client_amd.cli.main3d import main

if __name__ == "__main__":
    sys.exit(main())
