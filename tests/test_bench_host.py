"""Host-side pieces of bench.py (CPU): the work-per-config figures DESIGN.md
§5 quotes, the workload table, the CPU-share rule and a small run of the
CPU baseline (the oracle over a seeded uniform rank sample, with the
workload's key set and objectives)."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def test_work_per_config_figures():
    # SURVEY.md §8d W, and the documented replacement W' 
    assert bench.work_per_config(7, 64) == 2955
    assert bench.work_per_config_group(7, 64) == 968
    assert bench.work_per_config_group(6, 128) == 1780
    assert bench.work_per_config_keys(6, 128) == 2632


def test_workloads_name_the_baseline_configs():
    w = bench.workloads()
    assert (w["r64n7"]["R"], w["r64n7"]["n"], w["r64n7"]["keys"]) == (64, 7, 0)
    assert (w["r128n6"]["R"], w["r128n6"]["n"], w["r128n6"]["keys"]) == (128, 6, 1)
    assert w["r128n6_base"]["keys"] == 0
    assert w["gcp"]["R"] is None


def test_cpu_share_follows_omp_num_threads(monkeypatch):
    monkeypatch.setenv("OMP_NUM_THREADS", "1")
    assert bench.host_cpu_share() == 1
    monkeypatch.setenv("OMP_NUM_THREADS", "not-a-number")
    assert bench.host_cpu_share() >= 1


@pytest.mark.parametrize("keys", [0, 1])
def test_cpu_baseline_small_sample(monkeypatch, keys):
    from fantoch_amd.bote import CONFIG5_OBJECTIVES, DEFAULT_OBJECTIVES
    from fantoch_amd.planet import Planet

    monkeypatch.setenv("OMP_NUM_THREADS", "2")
    objs = CONFIG5_OBJECTIVES if keys else DEFAULT_OBJECTIVES
    cb = bench.cpu_baseline(Planet.synthetic(64), 5, keys=keys, objectives=objs, budget_s=0.05, nsample=600,
                            cap_s=0.05)
    assert cb["kind"] == "port" and cb["unit"] == "configs/s" and cb["cores"] == 2
    assert cb["value"] > 0 and cb["single_thread"]["value"] > 0
    assert f"{len(objs)} objectives" in cb["sample"]
    assert ("extended key set" in cb["sample"]) == bool(keys)
    assert "drawn uniformly" in cb["sample"]


def test_profile_figures_only_for_the_profiled_build():
    """the line's VALU issue utilisation and HBM traffic come from
    profiles/pmc.json / traffic.json; they are quoted only when those were
    measured on the library being benched (bench.lib_build)."""
    pmc = {"valu_insts_per_config": 869.0, "clock_ghz": 2.35, "build": "aaaa", "source": "x"}
    traffic = {"bytes": 7.5e7, "build": "aaaa"}
    valu, tb, stale = bench.profile_figures(pmc, traffic, "aaaa", 621216192, 14.45)
    assert valu["same_build"] and 0.4 < valu["util"] < 0.6
    assert tb == 7.5e7 and stale == []
    valu, tb, stale = bench.profile_figures(pmc, traffic, "bbbb", 621216192, 14.45)
    assert valu["util"] is None and not valu["same_build"]
    assert tb is None and len(stale) == 2
    # a figure without a build (before round 5) is never quoted
    valu, tb, stale = bench.profile_figures(dict(pmc, build=None), None, "bbbb", 1, 1.0)
    assert valu["util"] is None and tb is None and len(stale) == 1


def test_lib_build_is_the_loaded_library():
    from fantoch_amd import _lib

    if not os.path.exists(_lib.LIB_PATH):
        pytest.skip("library not built")
    b = bench.lib_build()
    assert len(b) == 16 and int(b, 16) >= 0
