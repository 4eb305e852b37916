"""Run sweeps through the device-assert build (scripts/build_variant.sh debug
-DBOTE_DEBUG; soft asserts) on the group kernel's PERM (n <= 7)
and qtab (n >= 8) paths and compare with the committed oracle fixtures:
  BOTE_LIB_PATH=fantoch_amd/lib_debug/libbote_hip.so python scripts/debug_check.py
A failed device assert makes bote_sweep_result raise BOTE_E_DEVICE."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np

    from fantoch_amd import _lib
    from fantoch_amd.bote import DEFAULT_OBJECTIVES, DEFAULT_RANKING, DevicePlanet, Sweep
    from fantoch_amd.planet import Planet

    assert "lib_debug" in _lib.LIB_PATH, "run with BOTE_LIB_PATH pointing at the debug build"
    gold = os.path.join(ROOT, "tests", "golden")
    t = json.load(open(os.path.join(gold, "topk.json")))
    cases, K = t["cases"], t["K"]
    gcp = Planet.new()
    dp = DevicePlanet(gcp, 0)
    planets = {None: (gcp, dp)}
    runs = [("gcp_n7", None), ("gcp_n9", None), ("gcp_n11", None), ("syn_r64n7", 64), ("syn_r128n6", 128)]
    for name, R in runs:
        fx = cases[name]
        if R not in planets:
            p = Planet.synthetic(R)
            planets[R] = (p, DevicePlanet(p, 0))
        p, d = planets[R]
        srv = np.arange(p.R, dtype=np.uint32)
        sw = Sweep(d, srv, srv, fx["n"], DEFAULT_OBJECTIVES, K=K, ranking=DEFAULT_RANKING,
                   digest=True, kernel="group")
        sw.launch(fx["rank_begin"], fx["rank_end"])
        r = sw.result()  # raises on a device assert
        ok = (r.valid, r.digest) == (int(fx["valid"]), int(fx["digest"])) and \
            [[(int(k), int(rk)) for k, rk in lst] for lst in r.tops] == \
            [[(int(k), int(rk)) for k, rk in lst] for lst in fx["tops"]]
        print(f"{name}: group kernel under BOTE_DEBUG, {fx['rank_end'] - fx['rank_begin']} configs, "
              f"asserts clean, result {'equals' if ok else 'DIFFERS FROM'} the oracle fixture (K={K})", flush=True)
        if not ok:
            sys.exit(1)
    print("debug build OK")


if __name__ == "__main__":
    main()
