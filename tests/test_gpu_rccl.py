"""The native merge collective (rl.h rl_comm_* / rl_agent_set_comm / rl_agent_sync):
an RCCL int64 all-reduce of the merge delta inside librlamd, no PyTorch.

Only one GPU is visible here, so the communicator has one rank (RCCL refuses two
ranks on one device); the all-reduce still runs for real on the agent's stream.
The N-rank decomposition (delta summed over ranks, then applied) is covered by
the gloo tests (tests/test_dist_gpu.py, tests/test_oracle_semantics.py), and
the driver's 8-GPU bench runs this path over xGMI."""
import numpy as np
import pytest

from test_gpu_parity import _assert_stats_equal

pytestmark = pytest.mark.gpu

CASES = [dict(env="frozen_lake", map8x8=1, algo="qlearning", group_size=128),
         dict(env="taxi", selector="ucb", algo="expected_sarsa", group_size=128),
         dict(env="cliff_walking", agent="traces", algo="sarsa", group_size=64),
         dict(env="blackjack", policy="double", algo="qlearning", group_size=256)]


@pytest.fixture(scope="module")
def comm(rl):
    c = rl.Comm(0, 1, rl.comm_unique_id(), 0)
    yield c
    c.close()


@pytest.mark.parametrize("case", CASES, ids=["fl", "taxi-ucb-es", "cw-traces", "bj-double"])
def test_rccl_merge_equals_local_merge(rl, oracle, comm, case):
    p = rl.default_params(n_lanes=3000, sync_every=16, n_episodes_for_decay=40, **case)
    plain, viacomm, manual = rl.Agent(p), rl.Agent(p), rl.Agent(p)
    viacomm.set_comm(comm)
    manual.set_comm(comm)
    plain.run(5)
    viacomm.run(5)
    for _ in range(5):
        manual.launch_train()
        manual.sync()
    ref = oracle.Batch(p)
    ref.run(5)
    for a in (plain, viacomm, manual):
        assert np.array_equal(a.q_raw(), ref.q_raw())
        _assert_stats_equal(a, ref)
    if case.get("selector") == "ucb":
        assert np.array_equal(viacomm.ucb()[0], ref.ucb()[0]) and viacomm.ucb()[1] == ref.ucb()[1]


def test_rccl_train_evaluate_agree_on_termination(rl, oracle, comm):
    p = rl.default_params(env="frozen_lake", n_lanes=700, group_size=64, sync_every=16,
                          n_episodes_for_decay=40)
    dev = rl.Agent(p)
    dev.set_comm(comm)
    dev.train(12, 4)
    dev.evaluate(3)
    ref = oracle.Batch(p)
    ref.train_episodes(12, 4)
    ref.evaluate(3)
    assert np.array_equal(dev.q_raw(), ref.q_raw())
    _assert_stats_equal(dev, ref)


def test_comm_rejects_private_mode(rl, comm):
    a = rl.Agent(rl.default_params(env="frozen_lake", n_lanes=8, group_size=1))
    with pytest.raises(rl.RLError):
        a.set_comm(comm)


@pytest.mark.parametrize("case", CASES, ids=["fl", "taxi-ucb-es", "cw-traces", "bj-double"])
def test_comm_peer_setup_world1(rl, oracle, case, monkeypatch):
    """rl_agent_set_comm's peer-read setup as the driver's N-GPU runs take it —
    the exchange handles all-gathered over RCCL (in place), the agreement, the
    self-test merge of known sums and maxima — run at world 1 (RLAMD_PEER_WORLD1:
    the box has one GPU), and every later merge of run() and train() through the
    peer kernels: bit-exact against the oracle"""
    monkeypatch.setenv("RLAMD_PEER_WORLD1", "1")
    c = rl.Comm(0, 1, rl.comm_unique_id(), 0)
    try:
        p = rl.default_params(n_lanes=3000, sync_every=16, n_episodes_for_decay=40, **case)
        a = rl.Agent(p)
        a.set_comm(c)
        assert a.merge_path() == "peer"
        a.run(5)
        a.train(4, 2)
        a.synchronize()
        ref = oracle.Batch(p)
        ref.run(5)
        ref.train_episodes(4, 2)
        assert np.array_equal(a.q_raw(), ref.q_raw())
        _assert_stats_equal(a, ref)
        a.set_comm(None)
        assert a.merge_path() == "local"
        a.close()
    finally:
        c.close()
