"""bench.py's N-rank entry on CPU (no GPU here): the launcher
(fantoch_amd/launch.py) forms an N-rank world whose ranks all run and agree
with the oracle fixture, and bench.py refuses a world that does not match
--gpus or more GPUs than are visible, before touching the GPU.
Reference: the parallelism replaced is search.rs:209-231 (rayon over client
sets)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(args, env_extra, drop=("WORLD_SIZE", "RANK", "LOCAL_RANK")):
    env = {k: v for k, v in os.environ.items() if k not in drop}
    env.update(env_extra)
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, capture_output=True, text=True,
                          env=env, timeout=300, cwd=ROOT)


@pytest.mark.parametrize("world", [2, 3])
def test_launcher_forms_world_and_every_rank_matches_fixture(tmp_path, world):
    sys.path.insert(0, ROOT)
    from fantoch_amd.launch import run_world

    rc = run_world(world, [os.path.join(ROOT, "tests", "dist_worker.py"), str(tmp_path)], timeout=240)
    assert rc == 0
    fx = json.load(open(os.path.join(ROOT, "tests", "golden", "topk.json")))["cases"]["gcp_n5"]
    for r in range(world):
        got = json.load(open(tmp_path / f"rank{r}.json"))
        assert got["rank"] == r and got["world"] == world
        assert got["census"]["ranks"] == list(range(world)) and got["census"]["backend"] == "gloo"
        assert (got["valid"], got["digest"]) == (int(fx["valid"]), int(fx["digest"]))
        for o, lst in enumerate(got["tops"]):
            assert [tuple(x) for x in lst] == [(int(k), int(rk)) for k, rk in fx["tops"][o][:len(lst)]]


def test_launcher_propagates_a_failing_rank(tmp_path):
    sys.path.insert(0, ROOT)
    from fantoch_amd.launch import run_world

    script = tmp_path / "fail_rank1.py"
    script.write_text("import os, sys, time\n"
                      "if os.environ['RANK'] == '1': sys.exit(3)\n"
                      "time.sleep(60)\n")
    assert run_world(2, [str(script)], timeout=50) == 3  # rank 0 is terminated, not waited for


def test_bench_refuses_more_gpus_than_visible():
    import torch

    n = torch.cuda.device_count()
    r = _bench(["--gpus", str(n + 1), "--steps", "1", "--warmup", "0", "--no-cpu-baseline"], {})
    assert r.returncode != 0
    assert "GPU(s) visible" in r.stderr, r.stderr
    assert r.stdout.strip() == ""  # no bench line


def test_bench_refuses_world_not_equal_to_gpus():
    r = _bench(["--gpus", "1", "--steps", "1", "--warmup", "0", "--no-cpu-baseline"],
               {"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0
    assert "!= --gpus 1" in r.stderr, r.stderr
    r = _bench(["--gpus", "4", "--steps", "1", "--warmup", "0", "--no-cpu-baseline"],
               {"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0 and "!= --gpus 4" in r.stderr, r.stderr


def test_launcher_retries_a_taken_rendezvous_port(tmp_path):
    """A world whose rank exits PORT_IN_USE (its rendezvous port was taken) is
    started again on a new port; other failures are not retried."""
    sys.path.insert(0, ROOT)
    from fantoch_amd.launch import PORT_IN_USE, run_world

    marker = tmp_path / "tried"
    script = tmp_path / "port_once.py"
    script.write_text("import os, pathlib, sys\n"
                      f"tried = list(pathlib.Path({str(tmp_path)!r}).glob('tried*'))\n"
                      f"pathlib.Path({str(marker)!r} + str(len(tried))).write_text(os.environ['MASTER_PORT'])\n"
                      f"sys.exit({PORT_IN_USE} if len(tried) == 0 and os.environ['RANK'] == '0' else 0)\n")
    assert run_world(1, [str(script)], timeout=60) == 0
    assert len(list(tmp_path.glob("tried*"))) == 2  # two attempts, on two ports
    assert run_world(1, [str(script)], timeout=60, port=12345) == 0  # (fixed port: marker exists, exits 0)
