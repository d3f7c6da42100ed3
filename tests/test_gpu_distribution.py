"""GPU: the device's draw streams against the reference's own RNG, in distribution.

Every other parity test compares the device with the oracle on ONE stream
definition (per-lane xoshiro128+, DESIGN §2 "draws" / "cards"), bit for bit.
That stream replaces the reference's `rand::thread_rng()` (ChaCha12) and, at a
few draw sites, reshapes how words become draws (the ε test's high word first,
one u32 per power-of-two action draw, Blackjack's 16-bit card halves), each
argued to leave the distribution of every draw exactly unchanged.  This file
tests that argument end to end: `oracle/ref_faithful.c` in its ChaCha12 build
(rand 0.8.5's `StdRng` block cipher and `Uniform` mappings at the reference's
draw sites — the CPU baseline's build) runs `Agent::train` (src/agent.rs:66-118)
on independent streams, the device runs the same training on 4,096 private
lanes, and the per-run totals — training reward (the bins' reward_history sum)
and training steps (episode_length sum) — must be indistinguishable:
two-sample Kolmogorov-Smirnov and Welch tests, p >= 1e-3 each.  The final ε,
deterministic, must agree bit for bit.  A negative control (the device with
the ε schedule shortened from 0.5 n to 0.45 n episodes) must be rejected, so
the test has the power to see a change of that size.

Seeds are fixed on both sides, so the verdict is deterministic.
"""
import os
import subprocess

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
RF = os.path.join(ROOT, "oracle", "_build", "ref_faithful")
ENVS = {"frozen_lake": 0, "cliff_walking": 1, "taxi": 2, "blackjack": 3}
SEL = {"eps_greedy": 0, "ucb": 1}
ALGO = {"sarsa": 0, "qlearning": 1, "expected_sarsa": 2}
RUNS = 4096
THREADS = 16
P_MIN = 1e-3

# (env, map8x8, slippery, agent, policy, selector, algo, n_episodes): SURVEY §8(d) cfg 1-5
CASES = [
    ("frozen_lake", 0, 0, "one_step", "tabular", "eps_greedy", "qlearning", 2000),      # cfg 1
    ("frozen_lake", 1, 0, "one_step", "tabular", "eps_greedy", "qlearning", 2000),      # cfg 2's env
    ("frozen_lake", 1, 1, "one_step", "tabular", "eps_greedy", "qlearning", 1000),      # slippery
    ("taxi", 0, 0, "one_step", "tabular", "ucb", "expected_sarsa", 300),                # cfg 3
    ("cliff_walking", 0, 0, "traces", "tabular", "eps_greedy", "sarsa", 300),           # cfg 4
    ("blackjack", 0, 0, "one_step", "double", "eps_greedy", "qlearning", 3000),         # cfg 5
]


def _ref_runs(case):
    env, m8, slip, agent, policy, sel, algo, n = case
    if not os.path.exists(RF):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle")], check=True)
    out = subprocess.run([RF, str(ENVS[env]), str(m8), str(slip), str(int(agent == "traces")),
                          str(int(policy == "double")), str(SEL[sel]), str(ALGO[algo]), str(n), "0",
                          str(RUNS // THREADS), str(THREADS), "2"],
                         check=True, capture_output=True, text=True, timeout=300).stdout.split("\n")
    rows = [x.split() for x in out if x.startswith("episodes")]
    assert len(rows) == RUNS
    assert {int(r[1]) for r in rows} == {n}
    return dict(reward=np.array([float(r[5]) for r in rows]), steps=np.array([float(r[3]) for r in rows]),
                eps={float(r[9]) for r in rows})


def _dev_runs(rl, case, **over):
    env, m8, slip, agent, policy, sel, algo, n = case
    p = rl.default_params(env=env, map8x8=m8, slippery=slip, agent=agent, policy=policy, selector=sel, algo=algo,
                          n_lanes=RUNS, group_size=1, n_episodes_for_decay=n, seed=0xD15757, **over)
    dev = rl.Agent(p)
    try:
        dev.set_episode_log(n + 1)
        dev.train(n, 0)
        eps, lost = dev.episodes()
        assert lost == 0
        tr = eps[eps["mode"] == 0]
        lanes = tr["lane"].astype(np.int64)
        assert (np.bincount(lanes, minlength=RUNS) == n).all()
        return dict(reward=np.bincount(lanes, weights=tr["reward"], minlength=RUNS),
                    steps=np.bincount(lanes, weights=tr["length"].astype(np.float64), minlength=RUNS),
                    eps=dev.epsilon())
    finally:
        dev.close()


def _pvalues(a, b):
    from scipy.stats import ks_2samp, ttest_ind
    ks = ks_2samp(a, b).pvalue
    if np.all(a == a[0]) and np.all(b == b[0]):
        return ks, 1.0 if a[0] == b[0] else 0.0
    return ks, ttest_ind(a, b, equal_var=False).pvalue


@pytest.mark.parametrize("case", CASES, ids=lambda c: "-".join(map(str, (c[0], c[3], c[4], c[5], c[6]))))
def test_device_streams_match_chacha12_reference_in_distribution(rl, case):
    ref = _ref_runs(case)
    dev = _dev_runs(rl, case)
    # ε after n episodes is deterministic (uniform_epsilon_greed.rs:42-49): same bits
    assert len(ref["eps"]) == 1
    assert np.all(dev["eps"] == next(iter(ref["eps"])))
    for stat in ("reward", "steps"):
        ks, welch = _pvalues(dev[stat], ref[stat])
        msg = (f"{stat}: device mean {dev[stat].mean():.6g} sd {dev[stat].std():.4g}, "
               f"reference mean {ref[stat].mean():.6g} sd {ref[stat].std():.4g}; KS p {ks:.3g}, Welch p {welch:.3g}")
        print(msg)
        assert ks >= P_MIN and welch >= P_MIN, msg


def test_distribution_test_rejects_a_shorter_eps_schedule(rl):
    """negative control: the device with ε decaying over 0.45 n instead of 0.5 n
    episodes (frozen_lake.rs:84's exploration time) is told apart"""
    case = CASES[0]
    ref = _ref_runs(case)
    dev = _dev_runs(rl, case, exploration_time=0.45)
    ks_r, welch_r = _pvalues(dev["reward"], ref["reward"])
    ks_s, welch_s = _pvalues(dev["steps"], ref["steps"])
    print(f"negative control: reward KS {ks_r:.3g} Welch {welch_r:.3g}; steps KS {ks_s:.3g} Welch {welch_s:.3g}")
    assert min(ks_r, welch_r, ks_s, welch_s) < 1e-6
