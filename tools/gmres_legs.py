#!/usr/bin/env python3
"""The bench's GMRES legs alone (config 3 at 256^3, config 1 at 32^3, config 4's wave step at
128^3): one JSON line per leg, for same-box A/B of two library trees (run this file from each
tree).  python tools/gmres_legs.py [--steps 20] [--legs 3 1 4]"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--legs", type=int, nargs="+", default=[3, 1, 4])
    a = ap.parse_args()
    import torch
    torch.cuda.set_device(0)
    for leg in a.legs:
        if leg == 4:
            r = bench.wave_gmres_leg(128, max(1, a.steps // 2))
        else:
            r = bench.gmres_leg(256 if leg == 3 else 32, a.steps)
        r.pop("unfused", None)
        print(json.dumps({"leg": leg, "tree": os.path.dirname(os.path.dirname(os.path.abspath(__file__))), **r}),
              flush=True)


if __name__ == "__main__":
    main()
