"""Merge latency budget: per SURVEY §8(d) workload at
bench.py's geometry, time on the agent's stream with HIP events
  - one train launch (launch_train: K steps + the merge's first phase),
  - the merge after it (rl_agent_sync: [MAX all-reduce] -> fold -> SUM
    all-reduce -> apply) with a world-1 RCCL communicator attached,
  - the same merge without a communicator (fold / apply kernels only),
the same through the peer-read path at world 1 (RLAMD_PEER_WORLD1), and the host
time of the train()/evaluate() loop per launch.  The difference
of the two merge timings is RCCL's fixed cost at world 1; DESIGN.md §6 projects
8 ranks from it.

    python scripts/time_merge.py [cfg ...]      (GPU; prints one JSON line per cfg)
"""
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "rl-rust_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

import rlamd as rl  # noqa: E402
from golden.make_fullsize import bench_params  # noqa: E402

N = 200


def timed(stream, fn, n=N):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    e0.record(stream)
    for _ in range(n):
        fn()
    e1.record(stream)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n, (t1 - t0) * 1e3 / n


def one(cfg, lanes=None):
    kw = bench_params(cfg, {"n_lanes": lanes} if lanes else {})
    a = rl.Agent(rl.default_params(**{k: v for k, v in kw.items() if k != "reset_step"}))
    a.set_reset_step(bool(kw["reset_step"]))
    s = torch.cuda.Stream()
    a.set_stream(s.cuda_stream)
    a.run(2)
    out = {"cfg": cfg, "q_repr": a.q_repr(), "lanes": kw["n_lanes"],
           # bytes all-reduced per merge: MAX words (f64 only) and SUM words
           "max_bytes": 8 * a.delta_max_words() if a.q_repr() == "f64" else 0,
           "sum_bytes": 8 * (a.delta_words() - a.delta_max_words())}
    out["train_launch_ms"], _ = timed(s, a.launch_train, 32)
    a.sync()
    out["merge_local_ms"], out["merge_local_host_ms"] = timed(s, a.sync)
    comm = rl.Comm(0, 1, rl.comm_unique_id(), 0)
    a.set_comm(comm)
    out["merge_rccl_w1_ms"], out["merge_rccl_w1_host_ms"] = timed(s, a.sync)
    out["run_launch_rccl_w1_ms"], _ = timed(s, lambda: a.run(1), 32)
    # the peer-read path at world 1 (RLAMD_PEER_WORLD1: set_comm's setup, then every
    # merge through the peer kernels; run(1) takes the fixed point's fused pair)
    os.environ["RLAMD_PEER_WORLD1"] = "1"
    a.set_comm(comm)
    assert a.merge_path() == "peer"
    out["merge_peer_w1_ms"], _ = timed(s, a.sync)
    out["run_launch_peer_w1_ms"], _ = timed(s, lambda: a.run(1), 32)
    del os.environ["RLAMD_PEER_WORLD1"]
    a.set_comm(comm)
    for tag, comm_on in (("rccl_w1", True), ("local", False)):
        a.set_comm(comm if comm_on else None)
        l0 = a.stats()["launches"]
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        st = a.train(3, 0)          # three episodes per lane: the exit test every launch
        ms = (time.perf_counter() - t0) * 1e3
        n = int(st["launches"] - l0)
        out[f"train3_{tag}"] = {"launches": n, "host_ms_per_launch": ms / max(n, 1)}
    a.set_comm(None)
    comm.close()
    a.close()
    return out


if __name__ == "__main__":
    # cfg or cfg:lanes (2:131072 = the north star's 2^20 lanes over 8 GPUs, one rank's shard)
    cfgs = sys.argv[1:] or ["2", "3", "4", "5", "2:131072"]
    for c in cfgs:
        cf, _, ln = c.partition(":")
        print(json.dumps(one(int(cf), int(ln) if ln else None)), flush=True)
