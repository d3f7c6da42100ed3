"""CPU: two restatements of the reference training loop, written separately
from the reference source, agree bit for bit (VERDICT r01 "next" 9).

* oracle/rlref.c `rlo_faithful` (dense-array Q) — the oracle every GPU test
  leans on;
* oracle/ref_faithful.c (built -DRF_XOSHIRO) — the CPU-baseline loop with the
  reference's own data structures (FxHashMap Q, Vec histories, per-call Vec
  allocations), here on the oracle's RNG stream;
* tests/golden/faithful_py.py — a plain-Python restatement (cfg 1 sizes).

All run src/agent.rs:66-141 and must end with the same Q bits, rewards and TD
errors: the C pair on every SURVEY §8(d) configuration family (FrozenLake,
CliffWalking traces, Taxi UCB + expected SARSA, Blackjack double Q with the
fxhash observation ids, ...), the Python one on FrozenLake.
"""
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
XO = os.path.join(ROOT, "oracle", "_build", "ref_faithful_xo")

CASES = [  # (map8x8, slippery, selector, algo, n_episodes, eval_at)
    (0, 0, "eps_greedy", "qlearning", 2000, 200),     # cfg 1 (reduced n)
    (1, 0, "eps_greedy", "qlearning", 1000, 100),     # cfg 2's env, one lane
    (1, 1, "eps_greedy", "sarsa", 600, 60),
    (0, 1, "eps_greedy", "expected_sarsa", 800, 80),
    (0, 0, "ucb", "qlearning", 300, 30),
    (1, 0, "ucb", "sarsa", 200, 20),
]
ENVS = {"frozen_lake": 0, "cliff_walking": 1, "taxi": 2, "blackjack": 3}
SEL = {"eps_greedy": 0, "ucb": 1}
ALGO = {"sarsa": 0, "qlearning": 1, "expected_sarsa": 2}
# the other §8(d) families: (env, agent, policy, selector, algo, n_episodes, eval_at)
OTHER = [
    ("cliff_walking", "traces", "tabular", "eps_greedy", "sarsa", 300, 30),          # cfg 4
    ("taxi", "one_step", "tabular", "ucb", "expected_sarsa", 200, 20),              # cfg 3
    ("blackjack", "one_step", "double", "eps_greedy", "qlearning", 3000, 300),      # cfg 5
    ("blackjack", "traces", "double", "ucb", "sarsa", 1000, 100),
    ("taxi", "traces", "double", "eps_greedy", "expected_sarsa", 150, 15),
    ("cliff_walking", "one_step", "double", "ucb", "qlearning", 300, 30),
]


def _run_xo(env, m8, slip, agent, policy, sel, algo, n, eval_at):
    if not os.path.exists(XO):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle")], check=True)
    out = subprocess.run([XO, str(ENVS[env]), str(m8), str(slip), str(int(agent == "traces")),
                          str(int(policy == "double")), str(SEL[sel]), str(ALGO[algo]), str(n), str(eval_at), "1",
                          "1", "1"], check=True, capture_output=True, text=True).stdout.split("\n")
    q = np.array([int(x, 16) for x in out if len(x) == 16], np.uint64).view(np.float64)
    tail = next(x for x in out if x.startswith("episodes")).split()
    return q, dict(episodes=int(tail[1]), errors=int(tail[3]), reward_sum=float(tail[5]),
                   error_sum=float(tail[7]), eps=float(tail[9]))


def _ref_faithful(m8, slip, sel, algo, n, eval_at):
    return _run_xo("frozen_lake", m8, slip, "one_step", "tabular", sel, algo, n, eval_at)


def _same(a, b):
    a, b = np.asarray(a, np.float64).reshape(-1), np.asarray(b, np.float64).reshape(-1)
    return a.shape == b.shape and bool(((a.view(np.uint64) == b.view(np.uint64)) | (np.isnan(a) & np.isnan(b))).all())


@pytest.mark.parametrize("case", OTHER, ids=lambda c: "-".join(map(str, c)))
def test_ref_faithful_other_envs_equal_oracle_faithful(oracle, case):
    """CliffWalking traces (FxHashMap trace swept whole), Taxi, Blackjack with the
    fxhash observation ids and the double policy's two maps: ref_faithful (the
    CPU baseline's code, on the oracle's RNG) == rlo_faithful bit for bit."""
    env, agent, policy, sel, algo, n, eval_at = case
    q, info = _run_xo(env, 0, 0, agent, policy, sel, algo, n, eval_at)
    p = oracle.default_params(env=env, agent=agent, policy=policy, selector=sel, algo=algo, n_episodes_for_decay=n)
    f = oracle.Faithful(p)
    f.train(n, eval_at)
    assert _same(q, f.q())
    rh, el, te = f.histories()
    assert info["episodes"] == len(el) == n and info["errors"] == len(te)
    es = 0.0
    for x in te:
        es += float(x)
    assert info["error_sum"] == es or (np.isnan(info["error_sum"]) and np.isnan(es))


@pytest.mark.parametrize("case", CASES, ids=lambda c: "-".join(map(str, c)))
def test_ref_faithful_equals_oracle_faithful(oracle, case):
    m8, slip, sel, algo, n, eval_at = case
    q, info = _ref_faithful(*case)
    p = oracle.default_params(env="frozen_lake", map8x8=m8, slippery=slip, selector=sel, algo=algo,
                              n_episodes_for_decay=n)
    f = oracle.Faithful(p)
    f.train(n, eval_at)
    want = f.q().reshape(-1)
    assert np.array_equal(q.view(np.uint64), want.view(np.uint64))
    rh, el, te = f.histories()
    assert info["episodes"] == len(el) == n and info["errors"] == len(te)
    rs = 0.0
    for x in rh:
        rs += float(x)
    es = 0.0
    for x in te:
        es += float(x)
    assert info["reward_sum"] == rs and info["error_sum"] == es


@pytest.mark.parametrize("case", [c for c in CASES if c[4] <= 1000], ids=lambda c: "-".join(map(str, c)))
def test_python_restatement_equals_oracle_faithful(oracle, case):
    from golden import faithful_py
    m8, slip, sel, algo, n, eval_at = case
    q, rh, el, te = faithful_py.run(bool(m8), bool(slip), sel, algo, n, eval_at)
    p = oracle.default_params(env="frozen_lake", map8x8=m8, slippery=slip, selector=sel, algo=algo,
                              n_episodes_for_decay=n)
    f = oracle.Faithful(p)
    f.train(n, eval_at)
    assert np.array_equal(np.array(q, np.float64).reshape(-1).view(np.uint64), f.q().reshape(-1).view(np.uint64))
    orh, oel, ote = f.histories()
    assert np.array_equal(np.array(rh, np.float64).view(np.uint64), orh.view(np.uint64))
    assert np.array_equal(np.array(el, np.uint64), oel)
    assert np.array_equal(np.array(te, np.float64).view(np.uint64), ote.view(np.uint64))


def test_python_restatement_reproduces_cfg1_fixture():
    """tests/golden/trajectories.json["cfg1"] (made by the C oracle) regenerated
    by the Python restatement: Q bits, reward / length histories, TD-error stream."""
    import base64
    import hashlib
    import json
    from golden import faithful_py
    g = json.load(open(os.path.join(ROOT, "tests", "golden", "trajectories.json")))["cfg1"]
    n, eval_at = g["params"]["n_episodes"], g["params"]["eval_at"]
    q, rh, el, te = faithful_py.run(False, False, "eps_greedy", "qlearning", n, eval_at)
    assert np.array(q, "<f8").reshape(-1).tobytes() == base64.b64decode(g["q_f64_b64"])
    assert np.array(rh, "<f8").tobytes() == base64.b64decode(g["reward_history_f64_b64"])
    assert np.array(el, "<u8").tobytes() == base64.b64decode(g["episode_length_u64_b64"])
    assert len(te) == g["n_training_error"]
    assert hashlib.sha256(np.array(te, "<f8").tobytes()).hexdigest() == g["training_error_sha256"]
