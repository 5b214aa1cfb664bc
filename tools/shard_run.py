#!/usr/bin/env python3
"""One bench.py shard line (rank 0's photo shard of a multi-GPU rig, timed alone), for profiling:
    [ENV=...] python3 tools/shard_run.py config3 8     (rocprofv3 ... -- python3 tools/shard_run.py ...)"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

print(json.dumps(bench.shard_line(sys.argv[1], int(sys.argv[2]))))
