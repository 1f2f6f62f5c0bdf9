#!/usr/bin/env python3
"""The north-star sweep measurement of bench.py alone (syc 32 1 p=2, reference and forced cuts)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

if __name__ == "__main__":
    import bench

    print(json.dumps(bench.north_star_sweep(int(sys.argv[1]) if len(sys.argv) > 1 else 20)), flush=True)
