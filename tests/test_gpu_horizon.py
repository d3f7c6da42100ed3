"""GPU parity over one full training horizon.

One learner group per SURVEY §8(d) configuration at bench.py's group size and
K = 64 runs the reference CLI's schedule — Agent::train(env, 1e5, 1e4) per lane
(src/agent.rs:66-118, src/bin/frozen_lake.rs:35-84), ε decaying over 1e5
episodes to its stall residue (uniform_epsilon_greed.rs:42-49) — and is compared
bit for bit with `tests/golden/horizon.json` (tests/golden/make_horizon.py).
cfg 3's Taxi lanes run ~1e7 steps each (the NaN regime truncates every episode
at 100 steps), so this file takes about a minute on one MI355X.
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
             7: "trace_states"}


def _sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


@pytest.mark.parametrize("name", ["cfg2", "cfg5", "cfg4", "cfg3"])
def test_full_horizon_matches_oracle(rl, name):
    sys.path.insert(0, os.path.join(HERE, "golden"))
    from make_horizon import horizon_params
    doc = json.load(open(os.path.join(HERE, "golden", "horizon.json")))
    g = doc[name]
    kw = horizon_params(g["survey_cfg"])
    assert kw == g["params"], "bench.py presets moved: regenerate tests/golden/horizon.json"
    dev = rl.Agent(rl.default_params(**{k: v for k, v in kw.items() if k != "reset_step"}))
    dev.set_reset_step(bool(kw["reset_step"]))
    assert dev.q_repr() == g["q_repr"]
    dev.train(doc["n_episodes"], doc["eval_at"])
    want = np.frombuffer(base64.b64decode(g["q_raw_i64_b64"]), "<i8")
    got = dev.q_raw().reshape(-1)
    q = dev.q().reshape(-1)
    assert int(np.isnan(q).sum()) == g["n_nan"] and int(np.isinf(q).sum()) == g["n_inf"]
    bad = np.flatnonzero(got != want)
    assert bad.size == 0, f"{bad.size} Q entries differ, first {bad[0]}: dev {got[bad[0]]:#x} ref {want[bad[0]]:#x}"
    st, ref = dev.stats(), np.array(g["stats_u64"], np.uint64).view(np.int64)
    for i, k in STAT_KEYS.items():
        assert st[k] == int(ref[i]), (k, st[k], int(ref[i]))
    eps = dev.epsilon().astype("<f8")
    assert _sha(eps) == g["eps_sha256"]
    assert sorted({float(x) for x in eps}) == g["eps_values"]
    if "ucb_t" in g:
        n, t = dev.ucb()
        assert t == g["ucb_t"]
        assert np.array_equal(np.asarray(n).reshape(-1), np.frombuffer(base64.b64decode(g["ucb_n_u64_b64"]), "<u8"))
    dev.close()
