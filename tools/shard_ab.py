#!/usr/bin/env python3
"""Rank 0's photo shard of a BASELINE multi-GPU rig timed alone on this GPU (bench.py's shard line),
under environment variants, interleaved:  python tools/shard_ab.py config3 8 ROUNDS "VAR=a" ...
("-" = the defaults)."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
name, world, rounds = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
variants = sys.argv[4:] or ["-"]
CODE = f"""
import sys, json
sys.path.insert(0, {ROOT!r})
import bench
print(json.dumps(bench.shard_line({name!r}, {world})))
"""
for r in range(rounds):
    for v in variants:
        env = dict(os.environ)
        if v != "-":
            for kv in v.split():
                k, val = kv.split("=", 1)
                env[k] = val
        out = subprocess.run([sys.executable, "-c", CODE], capture_output=True, text=True, env=env, timeout=300)
        line = [l for l in out.stdout.splitlines() if l.startswith("{")]
        if not line:
            print(out.stdout[-2000:], out.stderr[-2000:])
            sys.exit(1)
        import json
        d = json.loads(line[-1])
        print(f"{name} x{world} round {r} {v}: {d['ms_per_step'] * 1e3:.2f} us/step  kernel {d['kernel']} "
              f"{d['kernel_ms_per_launch'] * 1e3:.2f} us  views {d['views']}")
