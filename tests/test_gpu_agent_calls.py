"""The per-call Agent surface: trait Agent's get_action / update
(/root/reference/src/agent.rs:52-62) through the C ABI (rl_agent_get_action,
rl_agent_update, rl_agent_env), driven by the reference's OWN loops written out
line by line below — Agent::train / Agent::evaluate (src/agent.rs:66-141) and the
Blackjack win-rate loop (src/bin/blackjack.rs:183-200) — over one lane's Env view
and agent.  The oracle is rlo_faithful (oracle/rlref.c), the single-env
restatement of those same loops: the TD stream, the histories, Q and epsilon must
be bit-identical.
"""
import ctypes as C

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def reference_evaluate(agent, env, n_episodes):
    """Agent::evaluate (src/agent.rs:120-141)"""
    reward_history, episode_length = [], []
    for _ in range(n_episodes):
        action_counter = 0
        epi_reward = 0.0
        curr_action = agent.get_action(int(env.reset()[0]))
        while True:
            action_counter += 1
            obs, reward, terminated = env.step([curr_action])
            next_action = agent.get_action(int(obs[0]))
            curr_action = next_action
            epi_reward += float(reward[0])
            if terminated[0]:
                reward_history.append(epi_reward)
                break
        episode_length.append(action_counter)
    return reward_history, episode_length


def reference_train(agent, env, n_episodes, eval_at, eval_episodes=100):
    """Agent::train (src/agent.rs:66-118): returns (reward_history, episode_length,
    training_error); the eval interleave calls evaluate(env, 100) (:107-108)"""
    reward_history, episode_length, training_error = [], [], []
    for episode in range(n_episodes):
        action_counter = 0
        epi_reward = 0.0
        curr_obs = int(env.reset()[0])
        curr_action = agent.get_action(curr_obs)
        while True:
            action_counter += 1
            obs, reward, terminated = env.step([curr_action])
            next_obs, reward, terminated = int(obs[0]), float(reward[0]), bool(terminated[0])
            next_action = agent.get_action(next_obs)
            td = agent.update(curr_obs, curr_action, reward, terminated, next_obs, next_action)
            training_error.append(td)
            curr_obs, curr_action = next_obs, next_action
            epi_reward += reward
            if terminated:
                reward_history.append(epi_reward)
                break
        if episode % eval_at == 0:
            reference_evaluate(agent, env, eval_episodes)
        episode_length.append(action_counter)
    return reward_history, episode_length, training_error


def win_rate_loop(agent, env, loop_len):
    """src/bin/blackjack.rs:179-200 (LOOP_LEN episodes of get_action + step)"""
    wins = losses = draws = steps = 0
    for _ in range(loop_len):
        curr_action = agent.get_action(int(env.reset()[0]))
        while True:
            obs, reward, terminated = env.step([curr_action])
            steps += 1
            curr_action = agent.get_action(int(obs[0]))
            if terminated[0]:
                r = float(reward[0])
                wins += r == 1.0
                losses += r == -1.0
                draws += r not in (1.0, -1.0)
                break
    return wins, losses, draws, steps


def _bits_equal(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    assert a.shape == b.shape, (a.shape, b.shape)
    same = (a.view(np.uint64) == b.view(np.uint64)) | (np.isnan(a) & np.isnan(b))
    assert same.all(), f"first difference at {np.argmin(same)}: {a[~same][:3]} vs {b[~same][:3]}"


CASES = [
    (dict(env="frozen_lake", algo="qlearning"), 60),
    (dict(env="frozen_lake", map8x8=1, slippery=1, algo="expected_sarsa"), 12),
    (dict(env="cliff_walking", agent="traces", algo="sarsa"), 12),
    (dict(env="taxi", selector="ucb", algo="expected_sarsa"), 6),
    (dict(env="taxi", policy="double", algo="sarsa", max_steps=40), 6),
    (dict(env="blackjack", policy="double", algo="qlearning"), 150),
    (dict(env="blackjack", agent="traces", selector="ucb", algo="sarsa"), 150),
    (dict(env="frozen_lake_edited", map8x8=1, algo="qlearning"), 12),
    (dict(env="frozen_lake", policy="neural", algo="qlearning", net_hidden=8), 12),
]


@pytest.mark.parametrize("case,n_ep", CASES, ids=lambda c: "-".join(f"{v}" for v in c.values())
                         if isinstance(c, dict) else str(c))
def test_reference_train_loop_over_agent_calls(rl, oracle, case, n_ep):
    """The reference's train loop over GpuEnv + GpuAgent (one lane) == rlo_faithful"""
    lane = 3
    p = rl.default_params(n_lanes=8, group_size=1, n_episodes_for_decay=n_ep, eval_episodes=20, **case)
    agent = rl.Agent(p)
    env = agent.env()
    # lane 3 of an 8-lane agent: its stream is (seed, lane_offset + 3)
    env_lane = _LaneEnv(env, lane)
    ag_lane = _LaneAgent(agent, lane)
    rh, el, te = reference_train(ag_lane, env_lane, n_ep, max(n_ep // 3, 1), eval_episodes=20)
    f = oracle.Faithful(dict(p, lane_offset=lane))
    f.train(n_ep, max(n_ep // 3, 1))
    frh, fel, fte = f.histories()
    _bits_equal(te, fte)
    _bits_equal(rh, frh)
    assert np.array_equal(np.asarray(el, np.uint64), fel)
    _bits_equal(agent.q()[lane].reshape(-1), f.q().reshape(-1))
    if case.get("selector", "eps_greedy") == "eps_greedy":
        assert agent.epsilon()[lane] == f.epsilon()
    # the other lanes were never touched: still the fresh agent
    fresh = rl.Agent(p)
    others = [i for i in range(8) if i != lane]
    _bits_equal(agent.q()[others].reshape(-1), fresh.q()[others].reshape(-1))


class _LaneEnv:
    """one lane's env of an Env view (rl_env_reset_lane / rl_env_step_lane), shaped
    as the reference's single env: reset() -> [obs], step([a]) -> ([obs], [r], [term])"""

    def __init__(self, env, lane):
        self.env, self.lane = env, lane

    def reset(self):
        return [self.env.reset_lane(self.lane)]

    def step(self, a):
        o, r, t = self.env.step_lane(self.lane, a[0])
        return [o], [r], [t]


class _LaneAgent:
    """one lane's agent: trait Agent's get_action / update"""

    def __init__(self, agent, lane):
        self.agent, self.lane = agent, lane

    def get_action(self, obs):
        return self.agent.get_action(obs, lane=self.lane)

    def update(self, *args):
        return self.agent.update(*args, lane=self.lane)


def test_blackjack_win_rate_loop(rl, oracle):
    """src/bin/blackjack.rs:183-200 after a training call: the same episodes, steps and
    draws as the oracle's evaluate (the loop IS Agent::evaluate's body), checked
    through the TD stream of a second train that follows it"""
    p = rl.default_params(env="blackjack", policy="double", n_lanes=1, group_size=1, lane_offset=11,
                          n_episodes_for_decay=200, eval_episodes=10)
    agent = rl.Agent(p)
    env = _LaneEnv(agent.env(), 0)
    ag = _LaneAgent(agent, 0)
    reference_train(ag, env, 200, 50, eval_episodes=10)
    w, l, d, steps = win_rate_loop(ag, env, 500)
    assert w + l + d == 500
    f = oracle.Faithful(dict(p, lane_offset=11))
    f.train(200, 50)
    assert f.evaluate(500) == steps
    _, _, te = reference_train(ag, env, 50, 25, eval_episodes=10)
    f.train(50, 25)
    _bits_equal(te, f.histories()[2])
    _bits_equal(agent.q()[0].reshape(-1), f.q().reshape(-1))


def test_batched_calls_equal_per_lane_calls(rl):
    """rl_agent_get_actions / rl_agent_updates (every lane at once) == the per-lane calls"""
    p = rl.default_params(env="taxi", selector="ucb", algo="expected_sarsa", n_lanes=64, group_size=1)
    a1, a2 = rl.Agent(p), rl.Agent(p)
    e1, e2 = a1.env(), a2.env()
    obs = e1.reset()
    assert np.array_equal(obs, e2.reset())
    act = a1.get_actions(obs)
    assert np.array_equal(act, [a2.get_action(int(o), lane=i) for i, o in enumerate(obs)])
    s2, r, t = e1.step(act)
    s2b, rb, tb = e2.step(act)
    assert np.array_equal(s2, s2b) and np.array_equal(r, rb) and np.array_equal(t, tb)
    nxt = a1.get_actions(s2)
    assert np.array_equal(nxt, [a2.get_action(int(o), lane=i) for i, o in enumerate(s2)])
    td1 = a1.updates(obs, act, r, t, s2, nxt)
    td2 = [a2.update(int(obs[i]), int(act[i]), float(r[i]), bool(t[i]), int(s2[i]), int(nxt[i]), lane=i)
           for i in range(64)]
    _bits_equal(td1, td2)
    _bits_equal(a1.q().reshape(-1), a2.q().reshape(-1))
    n1, t1 = a1.ucb()
    n2, t2 = a2.ucb()
    assert np.array_equal(n1, n2) and np.array_equal(t1, t2)


def test_agent_call_errors(rl):
    """shared mode has no per-call agent (RL_E_STATE); foreign observations and
    actions are RL_E_ARG; a lane's env refuses a step after termination (EnvNotReady)"""
    shared = rl.Agent(rl.default_params(env="frozen_lake", n_lanes=128, group_size=64))
    with pytest.raises(rl.RLError) as ex:
        shared.get_action(0)
    assert ex.value.code == 5
    agent = rl.Agent(rl.default_params(env="blackjack", n_lanes=2, group_size=1))
    with pytest.raises(rl.RLError) as ex:
        agent.get_action(12345)            # not an fxhash id of any Blackjack observation
    assert ex.value.code == 2
    obs = rl.lib().rl_obs_to_reference(3, (20 * 32 + 5) * 2)
    with pytest.raises(rl.RLError) as ex:
        agent.update(obs, 2, 0.0, False, obs, 0)     # action out of range (COUNT = 2)
    assert ex.value.code == 2
    with pytest.raises(rl.RLError) as ex:
        agent.get_action(obs, lane=2)
    assert ex.value.code == 2
    env = agent.env()
    with pytest.raises(rl.RLError) as ex:
        env.step_lane(0, 0)                # not reset yet
    assert ex.value.code == 1
    env.reset_lane(0)
    while not env.step_lane(0, 1)[2]:      # stick ends a Blackjack episode
        pass
    with pytest.raises(rl.RLError) as ex:
        env.step_lane(0, 0)
    assert ex.value.code == 1
    # a view whose agent is gone refuses every call (RL_E_STATE) instead of touching freed memory
    gone = rl.Agent(rl.default_params(n_lanes=1))
    h = C.c_void_p()
    rl.check(rl.lib().rl_agent_env(gone.h, C.byref(h)))
    with pytest.raises(rl.RLError) as ex:    # one view per agent
        rl.check(rl.lib().rl_agent_env(gone.h, C.byref(C.c_void_p())))
    assert ex.value.code == 5
    gone.close()
    o = C.c_uint64()
    assert rl.lib().rl_env_reset_lane(h, 0, C.byref(o)) == 5
    rl.lib().rl_env_destroy(h)


def test_batched_call_lengths_and_view_readiness(rl):
    """a batched call never reads past the caller's arrays (ValueError
    in Python, RL_E_ARG from the C ABI when n_lanes differs from the agent's), and
    a launch over the lanes clears the Env view's readiness (src/env.rs:17,24:
    the lane may have terminated since the view reset it)"""
    agent = rl.Agent(rl.default_params(env="frozen_lake", n_lanes=8, group_size=1))
    with pytest.raises(ValueError):
        agent.get_actions(np.zeros(4, np.uint64))
    with pytest.raises(ValueError):
        z = np.zeros(8, np.uint64)
        agent.updates(z, z[:7].astype(np.uint32), np.zeros(8), np.zeros(8, np.uint8), z, z.astype(np.uint32))
    obs = np.zeros(4, np.uint64)
    out = np.zeros(8, np.uint32)
    assert rl.lib().rl_agent_get_actions(agent.h, obs.ctypes.data, out.ctypes.data, 4) == 2
    assert rl.lib().rl_agent_get_actions(agent.h, np.zeros(8, np.uint64).ctypes.data, out.ctypes.data, 8) == 0
    env = agent.env()
    env.reset_lane(0)
    env.step_lane(0, 1)                     # ready after the reset
    agent.train(2, 0)                       # moves the lanes the view shares
    with pytest.raises(rl.RLError) as ex:
        env.step_lane(0, 1)
    assert ex.value.code == 1               # EnvNotReady until the view resets the lane
    env.reset_lane(0)
    env.step_lane(0, 1)
    # after run() a lane still mid-episode keeps stepping (Env::step of
    # an env that has not terminated), one that terminated needs a reset: the view
    # follows each lane record's LF_READY bit instead of refusing every lane
    LF_READY = 1 << 9
    for _ in range(6):
        agent.run(1)
        core, _aux = agent.lane_state()
        ready = (core[:, 1] & LF_READY) != 0
        for lane in range(8):
            if ready[lane]:
                env.step_lane(lane, 1)
            else:
                with pytest.raises(rl.RLError) as ex:
                    env.step_lane(lane, 1)
                assert ex.value.code == 1
        if ready.any() and not ready.all():
            break
    assert ready.any() and not ready.all(), core[:, 1]


def fused_train(agent, n_episodes, eval_at):
    """INTEGRATION.md §1.1's `impl Agent for GpuAgent` override of train
    (src/agent.rs:66-118) on a one-lane handle: ONE rl_agent_train (the fused
    private kernel) with the episode log and step records on, and the reference's
    history tuple read back from them"""
    agent.set_episode_log(2 * n_episodes + 8 * eval_at + 1024)
    agent.set_recording(True)
    agent.records()                           # drop older records
    agent.train(n_episodes, eval_at)
    eps, lost = agent.episodes()
    assert lost == 0
    recs = agent.records()[:, 0]
    agent.set_recording(False)
    train = eps[eps["mode"] == 0]
    td = recs["td"][((recs["kind"] == 2) | (recs["kind"] == 3)) & (recs["mode"] == 0)]
    return list(train["reward"]), list(train["length"]), list(td)


def fused_evaluate(agent, n_episodes):
    """the override of evaluate (src/agent.rs:120-141): one rl_agent_evaluate"""
    agent.set_episode_log(n_episodes + 1024)
    agent.evaluate(n_episodes)
    eps, lost = agent.episodes()
    assert lost == 0
    return list(eps["reward"]), list(eps["length"])


@pytest.mark.parametrize("case,n", [CASES[0], CASES[2], CASES[3], CASES[5]],
                         ids=["fl-q", "cw-traces", "taxi-ucb-es", "bj-double"])
def test_trait_override_equals_default_body(rl, case, n):
    """the override of train / evaluate (one fused launch
    sequence) returns exactly what the trait's default bodies return when they run
    over the per-call get_action / update: histories, TD stream, Q, epsilon"""
    p = rl.default_params(n_lanes=1, group_size=1, n_episodes_for_decay=n, **case)
    a1, a2 = rl.Agent(p), rl.Agent(p)
    env = a1.env()
    eval_at = max(n // 3, 1)
    r1, l1, te1 = reference_train(a1, env, n, eval_at)
    r2, l2, te2 = fused_train(a2, n, eval_at)
    _bits_equal(r1, r2)
    assert l1 == [int(x) for x in l2]
    _bits_equal(te1, te2)
    er1, el1 = reference_evaluate(a1, env, 20)
    er2, el2 = fused_evaluate(a2, 20)
    _bits_equal(er1, er2)
    assert el1 == [int(x) for x in el2]
    _bits_equal(a1.q().reshape(-1), a2.q().reshape(-1))
    _bits_equal(a1.epsilon(), a2.epsilon())
