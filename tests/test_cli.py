"""`python -m fantoch_amd` (fantoch_amd/cli.py): the reference's bote binary
(fantoch_bote/src/main.rs:4-85).  CPU: the distance table's format
(planet/mod.rs:144-177; the reference's own test, mod.rs:281-300, asserts only
that the 13-region table is produced), Rust's f64 Display, the flags.  GPU:
the whole command against the reference's asserted search values
(search.rs:671-751, tests/golden/reference_goldens.json)."""
import io
import json
import os
import subprocess
import sys

import pytest

from fantoch_amd import cli
from fantoch_amd.planet import Planet, Region

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = json.load(open(os.path.join(ROOT, "tests", "golden", "reference_goldens.json")))


def test_distance_table_format_13_regions():
    p = Planet.new()
    txt = cli.distance_table(p, cli.REGIONS13)
    lines = txt.split("\n")
    assert txt.endswith("\n") and lines[-1] == ""
    # header: `| |` then ` {:?} |` per region (Region's Debug is the bare name, region.rs:21-25)
    assert lines[0] == "| |" + "".join(f" {r} |" for r in cli.REGIONS13)
    assert lines[1] == "|:---:|" + ":---:|" * 13
    assert len(lines) == 2 + 13 + 1
    for a, line in zip(cli.REGIONS13, lines[2:15]):
        want = f"| __{a}__ |" + "".join(f" {p.ping_latency(Region(a), Region(b))} |" for b in cli.REGIONS13)
        assert line == want
    # self latency is 0 on the diagonal (planet/mod.rs:110 via dat.rs: self = 0)
    assert lines[2].split("|")[2].strip() == "0"


def test_distance_table_two_regions_literal():
    p = Planet.new()
    a, b = "europe-west2", "us-east1"
    ab, ba = p.ping_latency(a, b), p.ping_latency(b, a)
    assert cli.distance_table(p, [a, b]) == (f"| | {a} | {b} |\n|:---:|:---:|:---:|\n"
                                             f"| __{a}__ | 0 | {ab} |\n| __{b}__ | {ba} | 0 |\n")


def test_distance_table_unknown_region_raises():
    with pytest.raises(KeyError):
        cli.distance_table(Planet.new(), ["europe-west2", "mars-north1"])


@pytest.mark.parametrize("x,s", [(10360.3125, "10360.3125"), (10360.0, "10360"), (-0.0, "-0"), (0.1, "0.1"),
                                 (1e20, "100000000000000000000"), (1.5e-7, "0.00000015"),
                                 (float("nan"), "NaN"), (float("inf"), "inf"), (2.0 / 3.0, "0.6666666666666666")])
def test_rust_f64_display(x, s):
    assert cli.rust_f64(x) == s


def test_flags_parse():
    ap = cli.build_parser()
    a = ap.parse_args([])
    assert (a.cmd, a.input, a.min_n, a.max_n, a.ranking, a.ft_metric, a.chains, a.save_search) == \
        (None, "R13C13", 3, 13, "110,35,0,15", "F1F2", 1, True)
    a = ap.parse_args(["sweep", "--synthetic", "64", "--n", "7", "--gpus", "8", "--objectives", "config5",
                       "--keys", "tempo-all-leaders"])
    assert (a.synthetic, a.n, a.gpus, a.K) == (64, 7, 8, 100)
    from fantoch_amd import _lib
    from fantoch_amd.bote import CONFIG5_OBJECTIVES, DEFAULT_OBJECTIVES
    assert cli._objectives("config5") == list(CONFIG5_OBJECTIVES)
    assert cli._objectives("score,mean:af1,mean:ff1,cov:af1,mean:e") == list(DEFAULT_OBJECTIVES)
    assert cli._objectives("mean:ttf1") == [(_lib.OBJ_MEAN, _lib.SLOT_TT1)]


def test_distance_table_subcommand_runs_without_a_gpu():
    r = subprocess.run([sys.executable, "-m", "fantoch_amd", "distance-table", "--regions", "europe-west2,us-east1"],
                       capture_output=True, text=True, cwd=ROOT, timeout=300)
    assert r.returncode == 0, r.stderr
    assert r.stdout.startswith("| | europe-west2 | us-east1 |\n")


@pytest.mark.gpu
def test_main_reproduces_the_reference_binary(tmp_path):
    """main.rs end to end on the GPU: the distance table, then the best R13C13
    chain's score (search.rs:725: 10360.3 rounded) and stats_fmt lines, the
    n = 5 line equal to the reference's asserted string, and the chain's
    region order (search.rs:735-750)."""
    out = io.StringIO()
    cwd = os.getcwd()
    os.chdir(tmp_path)  # (main.rs saves 3_13_R13C13.data in the working directory)
    try:
        assert cli.main(["--show-order"], out=out) == 0
        assert os.path.exists("3_13_R13C13.data")
    finally:
        os.chdir(cwd)
    lines = out.getvalue().split("\n")
    assert lines[0].startswith("| | asia-southeast1 |")
    i = next(k for k, l in enumerate(lines) if l.startswith("score: "))
    assert i == 2 + 13 + 1  # table rows, then println!'s blank line
    g = GOLD["search"]
    assert f"{float(lines[i][len('score: '):]):.1f}" == g["score"]
    stats = lines[i + 1:i + 7]
    assert len(stats) == 6
    assert stats[1] == g["stats_fmt_n5"]
    assert lines[i + 7] == "sorted_config: [" + ", ".join(g["sorted_config"]) + "]"


@pytest.mark.gpu
def test_main_without_a_chain_fails_like_the_reference(tmp_path, capsys):
    """main.rs:66-69 `.next().unwrap()` panics when no evolving chain exists:
    ranking parameters no config meets give a non-zero exit and an error on
    stderr, not an empty success."""
    out = io.StringIO()
    rc = cli.main(["--no-save-search", "--no-distance-table", "--ranking", "100000,100000,0,15"], out=out)
    assert rc == 101
    assert out.getvalue() == ""
    assert "no evolving config chain" in capsys.readouterr().err
