"""CPU: the oracle's C restatements under AddressSanitizer + UndefinedBehaviorSanitizer
(SURVEY §5 "race detection / sanitizers").  Every fixture under tests/golden is
produced by oracle/rlref.c, and the CPU baseline by oracle/ref_faithful.c: both
manage their buffers by hand, so both run here with -fsanitize=address,undefined
-fno-sanitize-recover=all (oracle/Makefile `san`), where the first error aborts.
"""
import json
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "oracle", "_build")


@pytest.fixture(scope="module")
def san_build():
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "san"], check=True)
    return OUT


def _run(cmd):
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0",
               UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run(cmd, capture_output=True, text=True, env=env, timeout=600)
    assert r.returncode == 0, f"{cmd}: rc {r.returncode}\n{r.stderr[-4000:]}"
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr, r.stderr[-4000:]
    return r.stdout


def test_oracle_families_clean_under_asan_ubsan(san_build):
    """rlref.c: faithful loop, batched schedule (private / shared, fixed point and f64,
    split merge, reset-and-step, Dyna, NeuralPolicy) on every env; the quick sweep
    (one algorithm per env plus UCB + expected SARSA; `rlref_san` without `quick` runs
    all 180 families)"""
    out = _run([os.path.join(san_build, "rlref_san"), "quick"])
    assert out.startswith("san ok"), out


@pytest.mark.parametrize("env,map8,slip,agent,pol,sel,algo", [
    (0, 1, 1, 0, 0, 0, 1), (1, 0, 0, 1, 0, 0, 0), (2, 0, 0, 0, 0, 1, 2), (3, 0, 0, 0, 1, 0, 1),
    (3, 0, 0, 1, 0, 1, 0), (0, 0, 0, 1, 1, 1, 2)])
def test_ref_faithful_clean_under_asan_ubsan(san_build, env, map8, slip, agent, pol, sel, algo):
    """ref_faithful.c (hash-map tables, trace map, Vec histories; the oracle's RNG)"""
    out = _run([os.path.join(san_build, "ref_faithful_san"), str(env), str(map8), str(slip), str(agent),
                str(pol), str(sel), str(algo), "300", "30", "1", "1"])
    assert json.loads(out)["steps"] > 0
