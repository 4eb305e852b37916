"""Per-shard kernel time of an N-way split of the R=64 n=7 (or R=128 n=6)
sweep, each shard run alone on this GPU: equal rank shares vs the
cost-balanced split of bote_sweep_split.  The slowest shard bounds an N-GPU
strong-scaling step (bench.py --gpus N), so max/mean is its efficiency loss.

  python scripts/shard_balance.py [--workload r64n7] [--parts 8]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch  # noqa: F401  (one HIP runtime)

from fantoch_amd.bote import DEFAULT_OBJECTIVES, DEFAULT_RANKING, DevicePlanet, Sweep
from fantoch_amd.dist import shard_range
from fantoch_amd.planet import Planet


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="r64n7", choices=["r64n7", "r128n6"])
    ap.add_argument("--parts", type=int, default=8)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    R, n = (64, 7) if a.workload == "r64n7" else (128, 6)
    p = Planet.synthetic(R)
    srv = np.arange(R, dtype=np.uint32)
    sw = Sweep(DevicePlanet(p), srv, srv, n, DEFAULT_OBJECTIVES, K=100, ranking=DEFAULT_RANKING, digest=True)
    out = {"workload": a.workload, "parts": a.parts, "kernel": sw.kernel_path()}
    for name, bounds in (("equal_ranks", [shard_range(sw.total, a.parts, i)[0] for i in range(a.parts)] + [sw.total]),
                         ("cost_split", sw.split(0, sw.total, a.parts))):
        ms = []
        for i in range(a.parts):
            sw.launch(bounds[i], bounds[i + 1])
            sw.result()
            sw.timing_reset()
            for _ in range(a.reps):
                sw.launch(bounds[i], bounds[i + 1])
            sw.result()
            t, k = sw.timing()
            ms.append(t / k)
        out[name] = {"bounds": bounds, "kernel_ms": [round(x, 4) for x in ms],
                     "max_over_mean": round(max(ms) / (sum(ms) / len(ms)), 4)}
        print(name, out[name]["max_over_mean"], out[name]["kernel_ms"], flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
