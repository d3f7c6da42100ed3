"""CPU: the committed bench evidence of the latest round (profiles/rNN_bench/*.json)
is internally consistent: every roofline fraction is a
fraction (<= 1), counters are attached only from the benched build (rl_build_id
equal), the PMC summary they cite exists and holds that build's kernel time, and
the kernel's sampled average duration is not above the step it is part of
(a 1-in-8 event sample once overstated a 100-ms kernel)."""
import glob
import json
import os

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# the latest round's bench lines: profiles/rNN_bench/ (rounds 1-5) or profiles/rNN/bench/ (6 on)
ROUND = max(glob.glob(os.path.join(ROOT, "profiles", "r[0-9][0-9]_bench")) +
            glob.glob(os.path.join(ROOT, "profiles", "r[0-9][0-9]", "bench")),
            key=lambda d: int(os.path.relpath(d, os.path.join(ROOT, "profiles"))[1:3]))
ROUND_NO = int(os.path.relpath(ROUND, os.path.join(ROOT, "profiles"))[1:3])
LINES = sorted(glob.glob(os.path.join(ROUND, "*.json")))


def bench_line(path):
    """the bench's JSON line (a multi-rank run's file may also hold the launcher's chatter)"""
    return json.loads([l for l in open(path).read().splitlines() if l.startswith("{")][-1])


@pytest.mark.parametrize("path", LINES, ids=[os.path.basename(p) for p in LINES])
def test_bench_line_roofline_is_consistent(path):
    d = bench_line(path)
    r = d["roofline"]
    assert 0.0 < r["frac"] <= 1.0, r["frac"]
    assert r["bound"] in ("latency", "valu", "hbm")
    # one step = the train launch + the merge: its kernel cannot take longer (bench
    # lines from round 5 on time the private rows' every launch)
    if ROUND_NO >= 5:
        assert 0.0 < r["kernel_avg_ms"] <= d["ms_per_step"], (r["kernel_avg_ms"], d["ms_per_step"])
    assert r["hbm"]["fused_frac"] <= 1.0
    if r["hbm"]["traffic_frac"] is not None:
        assert r["hbm"]["traffic_frac"] <= 1.0
    if r["counters"] is not None:
        assert r["counters_build"].split()[0] == d["build_id"].split()[0]
        summary = os.path.join(ROOT, r["counters"].split(":")[0])
        assert os.path.exists(summary), summary
        sm = json.load(open(summary))
        if r.get("ceiling", "valu" if r["bound"] in ("latency", "valu") else "hbm") == "valu":
            assert r["frac"] == sm["valu_pipe_frac"]
        else:
            assert r["frac"] == r["hbm"]["traffic_frac"]
            assert r["traffic"] == sm["hbm_bytes_per_launch"]["total"]
    else:
        assert r["bound"] == "hbm"


def test_latest_round_is_checked():
    assert ROUND_NO >= 6 and len(LINES) >= 12, (ROUND, len(LINES))


def test_headline_line_is_the_default_workload():
    d = bench_line(os.path.join(ROUND, "bench_cfg2.json"))
    assert d["config"]["survey_cfg"] == 2 and d["config"]["lanes_per_gpu"] == 1 << 20
    assert d["cpu_baseline"]["kind"] == "port" and d["cpu_baseline"]["cores"] == 1
