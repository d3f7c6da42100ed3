"""GPU parity over the whole benchmarked window.

bench.py's cfg 2 / 2-slippery / 3 / 4 / 5 / 8 presets (2^20 / 2^20 / 2^20 / 2^17 /
2^19 lanes per GPU, groups of 512 / 512 / 512 / 256 / 512, K = 64), and cfg 4 at
BASELINE's whole 2^19 lanes on one GPU (`bench.py --config 4 --lanes 524288`), run for the
65 launches one default bench run makes (1 warm-up + 64 timed) and are compared
with `tests/golden/longrun.json`, made by the oracle's batched schedule in the
representation each configuration gets: the proven 2^-40 fixed point for the
headline cfg 2 (k_train_shared_o8, two generations of 1,024 resident groups per
launch), f64 for the rest (no range proof:
double_tabular_policy.rs:50-57 grows without bound, elegibility_traces_agent.rs:86-96
and UCB + expected SARSA reach NaN).  The bar is bit-exact raw words (fixed-point
integers, or f64 bits with NaN canonical), which implies equal NaN / +-inf masks
and finite L-inf = 0 < 1e-5.
"""
import base64
import hashlib
import json
import os
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
STAT_KEYS = {0: "train_steps", 1: "eval_steps", 2: "train_episodes", 3: "eval_episodes", 4: "reward_sum_q16",
             7: "trace_states", 8: "q_clamp_hits", 9: "delta_saturations"}


def _sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


@pytest.mark.parametrize("name", ["cfg2", "cfg2_slippery", "cfg3", "cfg4", "cfg5", "cfg4_2p19", "cfg8"])
def test_bench_window_matches_oracle(rl, name):
    sys.path.insert(0, HERE)
    from golden.make_fullsize import bench_params
    from golden.make_longrun import CASES
    g = json.load(open(os.path.join(HERE, "golden", "longrun.json")))[name]
    kw = bench_params(*CASES[name])
    assert kw == g["params"], "bench.py presets moved: regenerate tests/golden/longrun.json"
    dev = rl.Agent(rl.default_params(**{k: v for k, v in kw.items() if k != "reset_step"}))
    dev.set_reset_step(bool(kw["reset_step"]))
    assert dev.q_repr() == g["q_repr"] == ("fixed40" if name in ("cfg2", "cfg8") else "f64")   # slippery: f64 (r06)
    dev.run(g["launches"])
    assert dev.q_repr() == g["q_repr"]
    want = np.frombuffer(base64.b64decode(g["q_raw_i64_b64"]), "<i8")
    got = dev.q_raw().reshape(-1)
    q = dev.q().reshape(-1)
    assert int(np.isnan(q).sum()) == g["n_nan"] and int(np.isinf(q).sum()) == g["n_inf"]
    fin = np.isfinite(q)
    assert (float(np.abs(q[fin]).max()) if fin.any() else 0.0) == g["max_abs_finite"]
    bad = np.flatnonzero(got != want)
    wq = want.view("<f8") if g["q_repr"] == "f64" else want * 2.0 ** -40
    linf = float(np.abs(q[fin] - wq[fin]).max()) if fin.any() else 0.0
    assert bad.size == 0, f"{bad.size} Q entries differ (finite L-inf {linf}), first {bad[0]}: " \
                          f"dev {got[bad[0]]:#x} ref {want[bad[0]]:#x}"
    st, ref = dev.stats(), np.array(g["stats_u64"], np.uint64).view(np.int64)
    for i, k in STAT_KEYS.items():
        assert st[k] == int(ref[i]), (k, st[k], int(ref[i]))
    assert st["q_clamp_hits"] == 0 and st["delta_saturations"] == 0
    assert _sha(dev.epsilon().astype("<f8")) == g["eps_sha256"]
    if "ucb_t" in g:
        n, t = dev.ucb()
        assert t == g["ucb_t"]
        assert np.array_equal(np.asarray(n).reshape(-1), np.frombuffer(base64.b64decode(g["ucb_n_u64_b64"]), "<u8"))
    dev.close()
