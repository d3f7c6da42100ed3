"""CPU: bench.py's workload presets parse to the configurations they name
(SURVEY §8(d) cfg 2-5 and the §8(f) private rows 6-7), and the workload keys
under which profiles/counters.json files their counters are distinct."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _parse(monkeypatch, *argv):
    import bench
    monkeypatch.setattr(sys, "argv", ["bench.py", *argv])
    return bench.parse()


@pytest.mark.parametrize("cfg,env,policy,lanes,group", [
    (2, "frozen_lake", "tabular", 1 << 20, 512),
    (3, "taxi", "tabular", 1 << 20, 512),
    (4, "cliff_walking", "tabular", 1 << 17, 256),
    (5, "blackjack", "double", 1 << 19, 512),
    (6, "frozen_lake", "neural", 1 << 20, 1),
    (7, "cliff_walking", "tabular", 1 << 20, 1),
    (8, "taxi", "tabular", 1 << 20, 512),
])
def test_presets(monkeypatch, cfg, env, policy, lanes, group):
    a = _parse(monkeypatch, "--config", str(cfg))
    assert (a.env, a.policy, a.lanes, a.group) == (env, policy, lanes, group)
    if cfg == 6:   # src/bin/frozen_lake_neural.rs: the 4x4 map, eps <- eps * 0.5, DenseLayer(1, 32)
        assert a.map8x8 == 0 and a.extra["decay_kind"] == 1 and a.extra["eps_decay"] == 0.5
        assert a.extra["net_hidden"] == 32 and a.extra["net_act1"] == "leaky_relu6"
    if cfg == 7:   # src/bin/cliffwalking_model.rs: InternalModelAgent with 10 planning steps
        assert a.extra["planning"] == 10 and a.agent == "one_step" and a.algo == "qlearning"
    if cfg == 2:
        assert a.map8x8 == 1 and a.extra == {}
    if cfg == 8:   # cfg 3's Taxi + UCB, Q-learning target: the finite regime
        assert (a.selector, a.algo) == ("ucb", "qlearning")


def test_workload_keys_distinct(monkeypatch):
    import bench
    keys = set()
    for argv in (["--config", "2"], ["--config", "2", "--slippery", "1"], ["--config", "2", "--q-mode", "f64"],
                 ["--config", "3"], ["--config", "4"], ["--config", "4", "--lanes", str(1 << 19)],
                 ["--config", "5"], ["--config", "6"], ["--config", "7"], ["--config", "8"]):
        keys.add(bench.workload_key(_parse(monkeypatch, *argv)))
    assert len(keys) == 10
