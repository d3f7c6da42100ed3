"""GPU parity for the f64 representation of shared Q (rl.h rl_q_repr).

Every table outside the fixed point's proven range is f64 with the reference's
whole range (the double policy of cfg 5 grows without bound,
double_tabular_policy.rs:50-57; UCB + expected SARSA reaches NaN).
A step's contributions to an entry are summed exactly on the grid of the
largest (oracle/rlref.c fq_step_combine); the merge averages the changed
groups' values on the same kind of grid.  The device must equal the oracle bit
for bit (raw words = f64 bits, NaN canonical), including:
  - the representation each configuration gets and every switch between them;
  - one lane in shared f64 mode == the reference loop (rlo_faithful) exactly;
  - non-finite TD errors under eligibility traces (never-taken actions of a
    visited state get lr * (td * 0) = NaN, elegibility_traces_agent.rs:86-96);
  - UCB with c = +inf (the +inf early exit of the selection);
  - train(0) between runs is a no-op.
"""
import numpy as np
import pytest

from test_gpu_parity import _assert_q_equal, _assert_records_equal, _assert_stats_equal

pytestmark = pytest.mark.gpu

REPR_CASES = [
    (dict(env="frozen_lake", map8x8=1, algo="qlearning"), "fixed40"),
    (dict(env="taxi", algo="expected_sarsa"), "fixed40"),
    (dict(env="cliff_walking", selector="ucb", algo="sarsa"), "fixed40"),
    (dict(env="blackjack", algo="sarsa"), "fixed40"),
    (dict(env="blackjack", policy="double", algo="qlearning"), "f64"),
    (dict(env="cliff_walking", agent="traces", algo="sarsa"), "f64"),
    (dict(env="taxi", selector="ucb", algo="expected_sarsa"), "f64"),
    (dict(env="frozen_lake", algo="qlearning", gamma=1.0), "f64"),
    (dict(env="frozen_lake", map8x8=1, slippery=1, algo="qlearning"), "f64"),   # round 6: fix_faithful
]


@pytest.mark.parametrize("kw,want", REPR_CASES, ids=lambda v: str(v))
def test_representation_matches_oracle(rl, oracle, kw, want):
    p = rl.default_params(n_lanes=256, group_size=64, sync_every=8, **kw)
    dev, ref = rl.Agent(p), oracle.Batch(p)
    assert dev.q_repr() == ref.q_repr() == want


F64_CASES = [
    dict(env="frozen_lake", map8x8=1, algo="qlearning", group_size=256),           # o8 sweep form, forced f64
    dict(env="cliff_walking", algo="sarsa", group_size=64),
    dict(env="taxi", algo="expected_sarsa", group_size=100),                      # owner form
    dict(env="blackjack", algo="qlearning", group_size=512),                      # o8 f64 (compact rows)
    dict(env="blackjack", policy="double", algo="expected_sarsa", group_size=300, q_default=0.25),
    dict(env="taxi", selector="ucb", algo="qlearning", group_size=128),
    dict(env="frozen_lake", map8x8=1, agent="traces", policy="double", algo="sarsa", group_size=64),
]


@pytest.mark.parametrize("case", F64_CASES, ids=lambda c: "-".join(f"{v}" for v in c.values()))
def test_forced_f64_matches_oracle(rl, oracle, case):
    """set_q_mode('f64') on any configuration: records, Q bits, stats exact,
    in run mode and with the eval interleave."""
    p = rl.default_params(n_lanes=900, sync_every=16, n_episodes_for_decay=40, **case)
    dev, ref = rl.Agent(p), oracle.Batch(p)
    dev.set_q_mode("f64")
    ref.set_q_mode("f64")
    assert dev.q_repr() == ref.q_repr() == "f64"
    dev.set_recording(True)
    ref.set_record(True)
    dev.run(5)
    ref.run(5)
    _assert_records_equal(dev.records(), ref.records())
    assert np.array_equal(dev.q_raw(), ref.q_raw())
    dev.train(8, 4)
    ref.train_episodes(8, 4)
    _assert_records_equal(dev.records(), ref.records())
    assert np.array_equal(dev.q_raw(), ref.q_raw())
    _assert_stats_equal(dev, ref)


def test_representation_switches_match_oracle(rl, oracle):
    """fixed point -> (selector / algorithm change without a proof) f64 -> forced
    modes both ways, with training in between: exact at every stage."""
    p = rl.default_params(env="cliff_walking", algo="qlearning", n_lanes=700, group_size=128, sync_every=16,
                          n_episodes_for_decay=40)
    dev, ref = rl.Agent(p), oracle.Batch(p)
    assert dev.q_repr() == "fixed40"
    dev.run(4); ref.run(4)
    assert np.array_equal(dev.q_raw(), ref.q_raw())
    dev.set_q_mode("f64"); ref.set_q_mode("f64")
    dev.run(3); ref.run(3)
    assert dev.q_repr() == ref.q_repr() == "f64" and np.array_equal(dev.q_raw(), ref.q_raw())
    dev.set_q_mode("auto"); ref.set_q_mode("auto")
    assert dev.q_repr() == ref.q_repr()
    dev.run(2); ref.run(2)
    assert np.array_equal(dev.q_raw(), ref.q_raw())
    dev.set_action_selector("ucb"); ref.set_selector("ucb")
    dev.set_future_q_value_func("expected_sarsa"); ref.set_algo("expected_sarsa")
    assert dev.q_repr() == ref.q_repr() == "f64"
    dev.run(3); ref.run(3)
    assert np.array_equal(dev.q_raw(), ref.q_raw())
    dev.reset(); ref.reset()                       # back to q_default: provable again? (UCB + ES: no)
    assert dev.q_repr() == ref.q_repr()
    _assert_stats_equal(dev, ref)


@pytest.mark.parametrize("kw", [dict(env="blackjack", policy="double", algo="qlearning"),
                                dict(env="taxi", selector="ucb", algo="expected_sarsa"),
                                dict(env="cliff_walking", policy="double", selector="ucb", algo="sarsa")],
                         ids=["bj-double", "taxi-ucb-es", "cw-double-ucb"])
def test_one_lane_f64_is_the_reference_loop(rl, oracle, kw):
    """A single lane in a learner group (shared mode, f64): one contribution per
    entry per step is added exactly, and the merge of one group is its value —
    the device reproduces the faithful reference loop bit for bit."""
    n = 1500
    p = rl.default_params(n_episodes_for_decay=n, n_lanes=1, group_size=2, sync_every=37, **kw)
    dev = rl.Agent(p)
    dev.set_q_mode("f64")
    dev.train(n, n // 4)
    f = oracle.Faithful(p)
    f.train(n, n // 4)
    _assert_q_equal(dev.q(), f.q())


@pytest.mark.parametrize("case", [dict(env="cliff_walking", agent="traces", algo="sarsa", group_size=64),
                                  dict(env="taxi", agent="traces", algo="qlearning", group_size=128),
                                  dict(env="blackjack", agent="traces", policy="double", algo="sarsa",
                                       group_size=256)],
                         ids=["cw-pairs-bitmap", "taxi-pairs-list", "bj-pairs"])
def test_traces_nonfinite_td_matches_oracle(rl, oracle, case):
    """lr 1e300 drives Q to +-inf within a few steps; the traces sweep then forms
    lr * (td * E) with a non-finite td — NaN for E = 0, including the never-taken
    actions of visited states that the pair lists do not hold."""
    p = rl.default_params(n_lanes=800, sync_every=8, lr=1e300, n_episodes_for_decay=40, **case)
    dev, ref = rl.Agent(p), oracle.Batch(p)
    dev.run(6)
    ref.run(6)
    assert np.array_equal(dev.q_raw(), ref.q_raw())
    q = dev.q()
    assert (~np.isfinite(q)).any(), "no non-finite entry reached"
    _assert_stats_equal(dev, ref)


def test_ucb_c_inf_matches_oracle(rl, oracle):
    """UCB with c = +inf: unvisited and visited bonuses are both +inf, the first
    maximum wins (utils.rs:1-11) — the selection's +inf shortcut must not fire."""
    p = rl.default_params(env="taxi", selector="ucb", algo="sarsa", ucb_c=float("inf"), n_lanes=300,
                          group_size=64, sync_every=16)
    dev, ref = rl.Agent(p), oracle.Batch(p)
    dev.set_recording(True)
    ref.set_record(True)
    dev.run(3)
    ref.run(3)
    _assert_records_equal(dev.records(), ref.records())
    assert np.array_equal(dev.q_raw(), ref.q_raw())


@pytest.mark.parametrize("G", [1, 64], ids=["private", "shared"])
def test_train_zero_between_runs_is_a_noop(rl, oracle, G):
    """Agent::train(env, 0, ..) runs nothing (src/agent.rs:80): lanes left
    mid-episode by run() continue with their traces."""
    p = rl.default_params(env="cliff_walking", agent="traces", algo="sarsa", n_lanes=200, group_size=G,
                          sync_every=16, n_episodes_for_decay=40)
    dev, ref = rl.Agent(p), oracle.Batch(p)
    dev.run(2); ref.run(2)
    dev.train(0, 0); ref.train_episodes(0, 0)
    dev.run(2); ref.run(2)
    if G == 1:
        _assert_q_equal(dev.q(), ref.q())
    else:
        assert np.array_equal(dev.q_raw(), ref.q_raw())
    _assert_stats_equal(dev, ref)


@pytest.mark.parametrize("case", ["q_mode", "selector"])
def test_delta_cap_survives_representation_switch(rl, oracle, case):
    """a caller-owned merge buffer sized by rl_agent_delta_cap_words
    before a switch still fits after it — FrozenLake's table moving from the fixed
    point to f64 (set_q_mode), and Blackjack's selector moving from eps-greedy
    (484 compact LDS rows per table) to UCB (all S rows) — and the
    external-collective merge then equals rl_agent_run"""
    import ctypes as C
    # device memory from the HIP runtime librlamd itself is linked to (a torch of
    # another ROCm in the same process would bring a second runtime)
    hip = C.CDLL("libamdhip64.so")
    if case == "q_mode":
        p = rl.default_params(env="frozen_lake", map8x8=1, algo="qlearning", n_lanes=2048, group_size=256,
                              sync_every=8)
    else:
        p = rl.default_params(env="blackjack", algo="qlearning", n_lanes=2048, group_size=256, sync_every=8)
    dev, ref = rl.Agent(p), oracle.Batch(p)
    cap = dev.delta_cap_words()
    assert cap >= dev.delta_words()
    buf = C.c_void_p()
    assert hip.hipMalloc(C.byref(buf), C.c_size_t(cap * 8)) == 0
    try:
        assert hip.hipMemset(buf, 0, C.c_size_t(cap * 8)) == 0
        dev.set_delta_buffer(buf.value, cap)
        dev.set_merge_groups(8)
        if case == "q_mode":
            assert dev.q_repr() == "fixed40"
            dev.set_q_mode("f64")
            ref.set_q_mode("f64")
            assert dev.q_repr() == "f64"
        else:   # f64 over the compact rows, then UCB's dense ones
            dev.set_q_mode("f64")
            ref.set_q_mode("f64")
            before = dev.delta_words()
            dev.set_action_selector("ucb")
            ref.set_selector("ucb")
            assert dev.delta_words() > before
        assert cap >= dev.delta_words()
        for _ in range(3):
            dev.launch_train()        # one rank: the collectives are the identity
            dev.launch_fold()
            dev.launch_apply()
        dev.synchronize()
        ref.run(3)
        assert np.array_equal(dev.q_raw(), ref.q_raw())
    finally:
        dev.close()
        hip.hipFree(buf)
