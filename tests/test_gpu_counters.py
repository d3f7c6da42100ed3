"""GPU parity for the counters and arming rules.

- UCB visit counters are u64 (the reference keeps u128,
  src/action_selection/upper_confidence_bound.rs:11-12): seeded just below
  2^32, they must cross it without wrapping, bit-exact vs the oracle.
- Tables outside the fixed point's proven range are f64 (rl.h rl_q_repr): the
  hyper-parameters that used to clamp run unclamped, bit-exact vs the oracle.
- train() / evaluate() leave every lane in TRAIN at an episode start with an
  empty trace set (elegibility_traces_agent.rs:98-100), so run() keeps training.
"""
import numpy as np
import pytest

from test_gpu_parity import _assert_q_equal, _assert_records_equal, _assert_stats_equal

pytestmark = pytest.mark.gpu

NEAR = (1 << 32) - 40


def _seed_ucb(dev, ref, S, A, L=None, spread=32):
    rng = np.random.default_rng(7)
    shape = (S, A) if L is None else (L, S, A)
    n = (NEAR + rng.integers(0, spread, shape)).astype(np.uint64)
    t = np.uint64(1 << 40) if L is None else np.full(L, 1 << 40, np.uint64)
    dev.set_ucb(n, t)
    ref.set_ucb(n, t)
    return n


@pytest.mark.parametrize("case", [dict(env="taxi", algo="expected_sarsa", group_size=64),
                                  dict(env="taxi", algo="qlearning", group_size=128),
                                  dict(env="cliff_walking", agent="traces", algo="sarsa", group_size=64)],
                         ids=["taxi-es", "taxi-q", "cw-traces"])
def test_shared_ucb_counters_cross_2p32(rl, oracle, case):
    p = rl.default_params(selector="ucb", n_lanes=600, sync_every=16, **case)
    dev, ref = rl.Agent(p), oracle.Batch(p)
    dev.set_recording(True)
    ref.set_record(True)
    _seed_ucb(dev, ref, dev.S, dev.A)
    dev.run(4)
    ref.run(4)
    dn, dt = dev.ucb()
    rn, rt = ref.ucb()
    assert dn.dtype == np.uint64 and dt == rt
    assert np.array_equal(dn, rn)
    assert (dn > (1 << 32)).any(), "no counter crossed 2^32"
    _assert_records_equal(dev.records(), ref.records())
    assert np.array_equal(dev.q_raw(), ref.q_raw())


def test_private_ucb_counters_cross_2p32(rl, oracle):
    p = rl.default_params(env="taxi", selector="ucb", algo="expected_sarsa", n_lanes=40, group_size=1,
                          sync_every=32)
    dev, ref = rl.Agent(p), oracle.Batch(p)
    # one agent per lane touches few of its 3000 entries: seed them at 2^32 - 2 ..
    # 2^32 + 1 so the lanes' increments cross the u32 boundary
    n0 = _seed_ucb(dev, ref, dev.S, dev.A, L=40, spread=4) + np.uint64(38)
    dev.set_ucb(n0, np.full(40, 1 << 40, np.uint64))
    ref.set_ucb(n0, np.full(40, 1 << 40, np.uint64))
    dev.run(3)
    ref.run(3)
    dn, dt = dev.ucb()
    rn, rt = ref.ucb()
    assert np.array_equal(dn, rn) and np.array_equal(dt, rt)
    assert ((n0 < (1 << 32)) & (dn >= (1 << 32))).any()
    _assert_q_equal(dev.q(), ref.q())


def test_set_ucb_rejects_t_zero(rl):
    p = rl.default_params(env="taxi", selector="ucb", n_lanes=64, group_size=64)
    a = rl.Agent(p)
    with pytest.raises(rl.RLError):
        a.set_ucb(np.zeros((a.S, a.A), np.uint64), 0)


@pytest.mark.parametrize("case", [dict(env="cliff_walking", algo="qlearning", group_size=64),
                                  dict(env="cliff_walking", agent="traces", algo="sarsa", group_size=64),
                                  dict(env="taxi", selector="ucb", algo="qlearning", group_size=100)],
                         ids=["cw-q", "cw-traces", "taxi-ucb"])
def test_out_of_range_tables_are_f64(rl, oracle, case):
    """gamma 1, q_default -2047.5, lr 30: no range proof, so the table is f64 —
    values leave [-2048, 2048] unclamped, bit-exact vs the oracle (ABI v3 clamped
    and counted these; v4 has no clamp, the counters stay 0)."""
    p = rl.default_params(n_lanes=500, sync_every=16, gamma=1.0, lr=30.0, q_default=-2047.5, **case)
    dev, ref = rl.Agent(p), oracle.Batch(p)
    assert dev.q_repr() == ref.q_repr() == "f64"
    dev.run(4)
    ref.run(4)
    assert np.array_equal(dev.q_raw(), ref.q_raw())
    q = dev.q()
    assert (q[np.isfinite(q)] < -2048.0).any()
    st = dev.stats()
    assert st["q_clamp_hits"] == 0 and st["delta_saturations"] == 0
    _assert_stats_equal(dev, ref)


def test_default_configs_representation(rl):
    """At the reference CLI's hyper-parameters: FrozenLake Q-learning is proven
    (fixed point), traces and the double policy are f64; no counter moves."""
    for kw, want in ((dict(env="frozen_lake", map8x8=1), "fixed40"),
                     (dict(env="cliff_walking", agent="traces", algo="sarsa"), "f64"),
                     (dict(env="blackjack", policy="double"), "f64")):
        a = rl.Agent(rl.default_params(n_lanes=4096, group_size=256, **kw))
        assert a.q_repr() == want, kw
        a.run(4)
        st = a.stats()
        assert st["q_clamp_hits"] == 0 and st["delta_saturations"] == 0, (kw, st)


def test_run_evaluate_run_traces(rl, oracle):
    """run() leaves lanes mid-episode; evaluate() starts every lane at an empty
    trace set and train mode resumes after it: records, Q and stats bit-exact."""
    p = rl.default_params(env="cliff_walking", agent="traces", algo="sarsa", n_lanes=300, group_size=64,
                          sync_every=16, n_episodes_for_decay=40)
    dev, ref = rl.Agent(p), oracle.Batch(p)
    dev.set_recording(True)
    ref.set_record(True)
    dev.run(3)
    ref.run(3)
    dev.evaluate(2)
    ref.evaluate(2)
    dev.run(3)
    ref.run(3)
    _assert_records_equal(dev.records(), ref.records())
    assert np.array_equal(dev.q_raw(), ref.q_raw())
    _assert_stats_equal(dev, ref)


@pytest.mark.parametrize("G", [1, 64], ids=["private", "shared"])
def test_train_then_run_keeps_training(rl, oracle, G):
    p = rl.default_params(env="frozen_lake", n_lanes=128, group_size=G, sync_every=16,
                          n_episodes_for_decay=40)
    dev, ref = rl.Agent(p), oracle.Batch(p)
    dev.train(5, 0)
    ref.train_episodes(5, 0)
    s0 = dev.stats()["train_steps"]
    dev.run(2)
    ref.run(2)
    assert dev.stats()["train_steps"] > s0
    _assert_stats_equal(dev, ref)
    core, _ = dev.lane_state()
    assert ((core[:, 1] >> 12) & 3 == 0).all()     # every lane in TRAIN mode
    if G == 1:
        _assert_q_equal(dev.q(), ref.q())
    else:
        assert np.array_equal(dev.q_raw(), ref.q_raw())


@pytest.mark.parametrize("reset_step", [False, True], ids=["one-action", "reset-and-step"])
def test_double_policy_follows_f64_range(rl, oracle, reset_step):
    """The double policy writes one table with the TD error of the other
    (double_tabular_policy.rs:31-67), so A - B grows by (1 + lr) per update pair:
    the values leave the old fixed-point range (|Q| <= 2048) within the run and the
    f64 tables follow them, bit-exact vs the oracle, with no clamp."""
    p = rl.default_params(env="blackjack", policy="double", algo="qlearning", n_lanes=4096, group_size=512,
                          sync_every=64)
    dev, ref = rl.Agent(p), oracle.Batch(p)
    dev.set_reset_step(reset_step)
    ref.set_reset_step(reset_step)
    dev.run(40)
    ref.run(40)
    assert np.array_equal(dev.q_raw(), ref.q_raw())
    q = dev.q()
    assert dev.q_repr() == "f64" and np.nanmax(np.abs(q)) > 2048.0, np.nanmax(np.abs(q))
    st = dev.stats()
    assert st["q_clamp_hits"] == 0
    _assert_stats_equal(dev, ref)
