"""CPU: the oracle's NeuralPolicy / Network restatement and FrozenLakeEditedEnv.

* exp / expm1 / tanh (fdlibm sequences shared with the device) within 1-2 ulp of libm
* activation pairs (src/network/activation.rs) against a numpy restatement
* one Network::fit step equals the independent plain-Python restatement
  (tests/golden/tables.json kat.net_fit_leaky_relu6) bit for bit
* DenseLayer::new / reset initialisation ranges and determinism
* private batch (GPU semantics) == faithful single agent, lane by lane
* FrozenLakeEdited: reward 10 on G, -1 otherwise, truncation keeps the position
"""
import json
import os

import numpy as np
import pytest

GOLD = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "tables.json")))
KAT = GOLD["kat"]


def ulps(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return np.abs(a - b) / np.spacing(np.maximum(np.abs(b), np.finfo(np.float64).tiny))


def test_exp_expm1_tanh_vs_libm(oracle):
    rng = np.random.default_rng(7)
    L = oracle.lib()
    x = np.concatenate([rng.normal(0, 3, 4000), rng.uniform(-740, 705, 4000), rng.normal(0, 1e-4, 500),
                        [0.0, -0.0, 1e-300, 0.5, -0.5, 0.35, 1.04, -1.04, 22.5, -22.5]])
    e = np.array([L.rlo_exp(float(v)) for v in x])
    assert ulps(e, np.exp(x)).max() <= 1.0
    xm = x[np.abs(x) < 700]
    m = np.array([L.rlo_expm1(float(v)) for v in xm])
    assert ulps(m, np.expm1(xm)).max() <= 1.0
    t = np.array([L.rlo_tanh(float(v)) for v in xm])
    assert ulps(t, np.tanh(xm)).max() <= 2.0
    assert L.rlo_exp(float("inf")) == float("inf") and L.rlo_exp(float("-inf")) == 0.0
    assert np.isnan(L.rlo_exp(float("nan"))) and L.rlo_tanh(float("inf")) == 1.0


def act_np(name, v):
    """numpy restatement of activation.rs (libm exp/tanh: compared within a few ulp)"""
    sg = 1.0 / (1.0 + np.exp(-v))
    f = {"linear": v, "tanh": np.tanh(v), "relu": np.maximum(v, 0.0), "leaky_relu": np.maximum(v, 0.1 * v),
         "relu6": np.minimum(np.maximum(v, 0.0), 6.0), "leaky_relu6": np.minimum(np.maximum(v, 0.1 * v), 6.0),
         "sigmoid": sg, "swish": v * sg,
         "hard_swish": (v * np.minimum(np.maximum(v + 3.0, 0.0), 6.0)) / 6.0}[name]
    e = np.exp(v)
    fp = {"linear": np.ones_like(v), "tanh": 1.0 - np.tanh(v) ** 2, "relu": (v > 0).astype(float),
          "leaky_relu": np.where(v > 0, 1.0, 0.01), "relu6": ((v > 0) & (v < 6)).astype(float),
          "leaky_relu6": np.where((v > 0) & (v < 6), 1.0, 0.01), "sigmoid": sg * (1.0 - sg),
          "swish": (e * (v + e + 1.0)) / ((e + 1.0) * (e + 1.0)),
          "hard_swish": np.where(v > -3.0, (2.0 * v + 3.0) / 6.0, 0.0)}[name]
    return f, fp


@pytest.mark.parametrize("name", ["linear", "tanh", "relu", "leaky_relu", "relu6", "leaky_relu6", "sigmoid",
                                  "swish", "hard_swish"])
def test_activation_pairs(oracle, name):
    x = np.concatenate([np.linspace(-8, 8, 321), [0.0, 6.0, -3.0, 3.0]])
    f, fp = oracle.act(name, x)
    rf, rfp = act_np(name, x)
    assert np.allclose(f, rf, rtol=1e-14, atol=1e-300)
    assert np.allclose(fp, rfp, rtol=1e-13, atol=1e-15)


def test_network_fit_matches_independent_restatement(oracle):
    k = KAT["net_fit_leaky_relu6"]
    p = oracle.default_params(env="frozen_lake", policy="neural", net_hidden=k["hidden"])
    y = oracle.net_forward(p, k["w"], k["x"])
    assert np.array_equal(y, np.array(k["y"]))
    w2 = oracle.net_fit(p, k["w"], k["x"], k["target"], k["lr"])
    assert np.array_equal(w2, np.array(k["w_after"]))


def test_network_init_ranges(oracle):
    p = oracle.default_params(env="frozen_lake", policy="neural", net_hidden=32)
    n_in, n_par = oracle.net_dims(p)
    assert (n_in, n_par) == (1, 32 + 32 + 128 + 4)
    w0 = oracle.net_init(p, lane=3, gen=0)
    assert np.array_equal(w0, oracle.net_init(p, lane=3, gen=0))
    assert not np.array_equal(w0, oracle.net_init(p, lane=4, gen=0))
    l1, l2 = np.sqrt(6.0 / 33.0), np.sqrt(6.0 / 36.0)
    assert np.all(np.abs(w0[:32]) <= l1) and np.all(np.abs(w0[64:192]) <= l2)
    assert np.all(w0[32:64] == 0.0) and np.all(w0[192:] == 0.0)           # DenseLayer::new: bias 0
    w1 = oracle.net_init(p, lane=3, gen=1)
    assert np.all(w1[32:64] == 0.1) and np.all(w1[192:] == 0.1)           # DenseLayer::reset: bias 0.1
    assert not np.array_equal(w0[:32], w1[:32])


NEURAL_CASES = [
    dict(env="frozen_lake", agent="one_step", selector="eps_greedy", algo="qlearning", net_act1="leaky_relu6",
         decay_kind=1, eps_decay=0.5),
    dict(env="frozen_lake_edited", net_input="fl_obs", agent="one_step", selector="eps_greedy", algo="sarsa",
         net_act1="tanh", net_act2="linear"),
    dict(env="cliff_walking", agent="traces", selector="eps_greedy", algo="qlearning", net_act1="relu"),
    dict(env="taxi", agent="one_step", selector="ucb", algo="expected_sarsa", net_act1="sigmoid"),
    dict(env="blackjack", agent="one_step", selector="eps_greedy", algo="expected_sarsa", net_act1="swish",
         net_act2="softmax"),
]


@pytest.mark.parametrize("kw", NEURAL_CASES, ids=[c["env"] for c in NEURAL_CASES])
def test_neural_private_batch_equals_faithful(oracle, kw):
    p = oracle.default_params(policy="neural", n_lanes=3, group_size=1, sync_every=16, n_episodes_for_decay=20,
                              net_hidden=8, max_steps=30, **kw)
    b = oracle.Batch(p)
    b.train_episodes(12, 4)
    for lane in (0, 2):
        q = dict(p, lane_offset=lane)
        f = oracle.Faithful(q)
        f.train(12, 4)
        assert np.array_equal(f.weights().view(np.uint64), b.weights()[lane].view(np.uint64)), lane
        assert np.array_equal(f.q()[0].view(np.uint64), b.q()[lane, 0].view(np.uint64)), lane
    # Agent::reset -> Network::reset (new weights, bias 0.1) in both
    b.reset()
    f.reset()
    assert np.array_equal(f.weights(), b.weights()[2])


def test_frozen_lake_edited_rewards_and_truncation(oracle):
    p = oracle.default_params(env="frozen_lake_edited", max_steps=3)
    # 4x4: DOWN from 0 -> 4 (ground, -1), RIGHT x2 at row 1 -> 5 is a hole (-1, terminated)
    s0, s2, r, term, n = oracle.env_walk(p, [1, 2])
    assert s0 == 0 and list(s2) == [4, 5] and list(r) == [-1.0, -1.0] and list(term) == [False, True]
    # bump into the wall 3 times, then truncation keeps the position with -1.0
    s0, s2, r, term, n = oracle.env_walk(p, [0, 0, 0, 0])
    assert list(s2) == [0, 0, 0, 0] and list(r) == [-1.0] * 4 and list(term) == [False, False, False, True]
    # the goal pays 10 (path of the 4x4 KAT)
    k = KAT["fl4x4_path"]
    s0, s2, r, term, n = oracle.env_walk(oracle.default_params(env="frozen_lake_edited"), k["actions"])
    assert list(s2) == k["states"] and r[-1] == 10.0 and term[-1]
