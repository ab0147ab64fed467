#!/usr/bin/env python3
"""Name-compatible entry for the reference's scripts/tracker.py: supervises N
worker ranks and recovers a failed job from its last checkpoint.  See
xflow_amd/tracker.py.

    python scripts/tracker.py -n 4 --max-restarts 2 --ckpt ckpt/ -- train test 0 10
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from xflow_amd.tracker import main  # noqa: E402

if __name__ == "__main__":
    sys.exit(main())
