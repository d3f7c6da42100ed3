"""GPU parity at the benchmarked sizes (VERDICT r01 "next" 2).

bench.py's own presets (SURVEY §8(d) cfg 2-5 + slippery cfg 2: 2^20 / 2^17 /
2^19 lanes per GPU, groups of 512 / 256, K = 64, the CLI's default ε schedule)
run for two launches on the device and are compared bit for bit with the
committed oracle fixtures `tests/golden/fullsize.json` (no oracle in this
process).  The parameters are rebuilt from bench.PRESETS, so these are the
kernel instantiations (k_train_shared_o8 for cfg 2 / 5, k_train_shared for
cfg 3 / 4) and launch geometries the bench times.
Reference loop: /root/reference/src/agent.rs:86-106.
"""
import base64
import hashlib
import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
STAT_KEYS = {0: "train_steps", 1: "eval_steps", 2: "train_episodes", 3: "eval_episodes",
             4: "reward_sum_q16", 7: "trace_states", 8: "q_clamp_hits", 9: "delta_saturations"}


def _fixtures():
    return json.load(open(os.path.join(HERE, "golden", "fullsize.json")))


def _sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


@pytest.mark.parametrize("name", ["cfg2", "cfg2_slippery", "cfg3", "cfg4", "cfg5", "cfg4_2p19", "cfg8"])
def test_bench_config_matches_fullsize_fixture(rl, name):
    import sys
    sys.path.insert(0, os.path.dirname(HERE))
    from golden.make_fullsize import bench_params, CASES
    g = _fixtures()[name]
    cfg, extra = CASES[name]
    kw = bench_params(cfg, extra)
    assert kw == g["params"], "bench.py presets moved: regenerate tests/golden/fullsize.json"
    dev = rl.Agent(rl.default_params(**{k: v for k, v in kw.items() if k != "reset_step"}))
    dev.set_reset_step(bool(kw["reset_step"]))
    dev.run(g["launches"])
    want = np.frombuffer(base64.b64decode(g["q_raw_i64_b64"]), "<i8")
    got = dev.q_raw().reshape(-1)
    bad = np.flatnonzero(got != want)
    assert bad.size == 0, f"{bad.size} Q entries differ, first {bad[0]}: dev {got[bad[0]]} ref {want[bad[0]]}"
    assert _sha(dev.q().astype("<f8")) == g["q_f64_sha256"]
    st, ref = dev.stats(), np.array(g["stats_u64"], np.uint64).view(np.int64)
    for i, k in STAT_KEYS.items():
        assert st[k] == int(ref[i]), (k, st[k], int(ref[i]))
    assert _sha(dev.epsilon().astype("<f8")) == g["eps_sha256"]
    if "ucb_t" in g:
        n, t = dev.ucb()
        assert t == g["ucb_t"]
        assert np.array_equal(np.asarray(n).reshape(-1),
                              np.frombuffer(base64.b64decode(g["ucb_n_u64_b64"]), "<u8"))
    dev.close()
