"""Run bench.py's configs[4] / configs[2] legs alone (for rocprofv3 kernel stats and PMC
passes of their kernels without the configs[1] steps around them).

  python scripts/bench_legs.py configs4 [configs2]   -> one JSON line per leg on stdout
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    legs = sys.argv[1:] or ["configs4", "configs2"]
    for name in legs:
        fn = {"configs4": bench.configs4_leg, "configs2": bench.configs2_leg}[name]
        print(json.dumps({name: fn(dev)}), flush=True)


if __name__ == "__main__":
    main()
