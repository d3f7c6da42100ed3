"""Per-call Agent surface timing: how fast the trait's
required methods run through the C ABI, one kernel launch and one host round
trip each (rl_agent_get_action / rl_agent_update / rl_env_step_lane), beside the
batched forms and the fused override of train.

    python scripts/time_calls.py > gpurun_out/time_calls.json

FrozenLake 4x4 one-step Q-learning eps-greedy (the frozen_lake bin's agent), one
private lane; every figure is wall time on the host around the calls.
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rl-rust_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import rlamd as rl  # noqa: E402
from test_gpu_agent_calls import fused_train, reference_train  # noqa: E402


def rate(fn, n):
    fn()                                         # warm
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    return n / (time.perf_counter() - t0)


def main():
    out = {"workload": "FrozenLake 4x4 one-step Q-learning eps-greedy, private lanes (group_size 1)",
           "build_id": rl.build_id()}
    p = rl.default_params(n_lanes=1, group_size=1, n_episodes_for_decay=200)
    a = rl.Agent(p)
    env = a.env()
    env.reset_lane(0)
    out["get_action_calls_per_s"] = rate(lambda: a.get_action(0), 2000)
    out["update_calls_per_s"] = rate(lambda: a.update(0, 1, 0.0, False, 4, 2), 2000)
    out["env_step_lane_calls_per_s"] = rate(lambda: (env.reset_lane(0), env.step_lane(0, 1)), 1000) * 2
    # the trait's default train body over the per-call methods (reset, then per
    # step: env.step + get_action + update)
    a2 = rl.Agent(p)
    e2 = a2.env()
    t0 = time.perf_counter()
    _, lengths, _ = reference_train(a2, e2, 60, 1000)   # eval_at > n: the episode-0 evaluate only
    dt = time.perf_counter() - t0
    out["default_train_body_per_call"] = {"episodes": 60, "train_steps": int(sum(lengths)), "seconds": dt,
                                          "note": "includes the episode-0 evaluate(env, 100)"}
    # the override: one fused train (rl_agent_train) on the same one-lane handle
    a3 = rl.Agent(p)
    t0 = time.perf_counter()
    _, l3, _ = fused_train(a3, 60, 1000)
    dt3 = time.perf_counter() - t0
    out["override_train_fused"] = {"episodes": 60, "train_steps": int(sum(l3)), "seconds": dt3,
                                   "note": "episode log + step records on (the history tuple)"}
    out["override_speedup"] = dt / dt3
    # batched calls: every lane of a 65,536-lane handle at once
    L = 1 << 16
    pb = rl.default_params(n_lanes=L, group_size=1)
    b = rl.Agent(pb)
    obs = np.zeros(L, np.uint64)
    out["batched_get_actions_lane_calls_per_s"] = rate(lambda: b.get_actions(obs), 50) * L
    s, act = np.zeros(L, np.uint64), np.ones(L, np.uint32)
    r, t = np.zeros(L), np.zeros(L, np.uint8)
    s2, a2v = np.full(L, 4, np.uint64), np.full(L, 2, np.uint32)
    out["batched_updates_lane_calls_per_s"] = rate(lambda: b.updates(s, act, r, t, s2, a2v), 50) * L
    print(json.dumps(out))


if __name__ == "__main__":
    main()
