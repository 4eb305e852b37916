"""A rank of the world started by fantoch_amd.launch.run_world in
tests/test_launch.py: joins the gloo world from its environment, runs the
sharded sweep (fantoch_amd/dist.py) over the oracle-backed stand-in of the
GCP n=5 sweep, takes the census, and writes its view to <outdir>/rank<r>.json."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)


def main(outdir):
    import numpy as np
    import torch.distributed as dist

    import oracle as O
    from fantoch_amd.bote import DEFAULT_OBJECTIVES
    from fantoch_amd.dist import sharded_sweep, world_census
    from fantoch_amd.planet import Planet
    from oracle_sweep import OracleSweep

    dist.init_process_group("gloo")
    try:
        p = Planet.new()
        srv = np.arange(p.R, dtype=np.uint32)
        sw = OracleSweep(O.OraclePlanet.of(p), srv, srv, 5, DEFAULT_OBJECTIVES, 16)
        res = sharded_sweep(sw, stream=None, device="cpu")
        census = world_census(device="cpu")
        rank = dist.get_rank()
        with open(os.path.join(outdir, f"rank{rank}.json"), "w") as fh:
            json.dump({"rank": rank, "world": dist.get_world_size(), "census": census, "valid": res.valid,
                       "digest": res.digest, "tops": res.tops}, fh)
    finally:
        dist.destroy_process_group()


if __name__ == "__main__":
    main(sys.argv[1])
