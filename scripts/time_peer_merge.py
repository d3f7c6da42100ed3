"""Latency of the one-shot peer-read merge (rl.h ABI 7) at
world 2 (PEER_RANKS=4: four): the ranks sharing the box's one GPU (RCCL refuses two ranks on one device, so the
handles travel over gloo), each with bench.py's agent for a workload's per-rank
shard, time on the agent's stream with HIP events
  - the merge alone (rl_agent_sync: [MAX peer reduce] -> fold -> SUM peer reduce
    -> apply), the ranks entering it together (a barrier before each batch),
  - one whole launch + merge (rl_agent_run(1)),
beside the same agent's merge with no peers (fold / apply only).  Both ranks issue
their merges back to back, so a peer-read merge's time includes waiting for the
other rank's flag; scripts/time_merge.py gives RCCL's world-1 figure.

    [PEER_RANKS=4] python scripts/time_peer_merge.py [cfg[:lanes_per_rank] ...]   (GPU; rank 0 prints one JSON line per case)
"""
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
N = 200


def spawn(argv, n):
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    procs = [subprocess.Popen([sys.executable, os.path.abspath(__file__)] + argv,
                              env=dict(os.environ, RANK=str(r), WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1",
                                       MASTER_PORT=str(port)), cwd=ROOT) for r in range(n)]
    rc = 0
    for p in procs:
        try:
            rc = rc or p.wait(timeout=600)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            return 124
    return rc


def rank_main(argv):
    import torch
    import torch.distributed as dist
    sys.path.insert(0, os.path.join(ROOT, "rl-rust_amd"))
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import rlamd as rl
    from golden.make_fullsize import bench_params
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    torch.cuda.set_device(0)
    dist.init_process_group("gloo")

    def timed(stream, fn, n=N):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        dist.barrier()
        e0.record(stream)
        for _ in range(n):
            fn()
        e1.record(stream)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / n

    cases = argv or ["2:131072", "2:524288", "4:131072", "5:262144", "3:524288"]
    # the first case once more ahead, not printed: the ranks' start-up (other
    # processes still loading, first launches) inflated the first case's timings
    for i, c in enumerate([cases[0]] + cases):
        cf, _, ln = c.partition(":")
        kw = bench_params(int(cf), {"n_lanes": int(ln)} if ln else {})
        L = kw["n_lanes"]
        kw["lane_offset"] = rank * L
        a = rl.Agent(rl.default_params(**{k: v for k, v in kw.items() if k != "reset_step"}))
        a.set_reset_step(bool(kw["reset_step"]))
        s = torch.cuda.Stream()
        a.set_stream(s.cuda_stream)
        out = {"cfg": int(cf), "lanes_per_rank": L, "ranks": world, "q_repr": a.q_repr(),
               "max_bytes": 8 * a.delta_max_words() if a.q_repr() == "f64" else 0,
               "sum_bytes": 8 * (a.delta_words() - a.delta_max_words())}
        a.run(2)
        out["merge_local_ms"] = timed(s, a.sync)
        hs = [None] * world
        dist.all_gather_object(hs, a.peer_handle())
        a.peer_attach(rank, world, hs)
        a.set_merge_groups(world * ((L + kw["group_size"] - 1) // kw["group_size"]))
        assert a.merge_path() == "peer"
        timed(s, a.sync, 20)     # warm: both ranks' first merges (code objects, IPC mappings)
        out["merge_peer_ms"] = timed(s, a.sync)
        out["run_launch_peer_ms"] = timed(s, lambda: a.run(1), 32)
        a.synchronize()      # raises if a peer wait timed out
        a.close()
        if rank == 0 and i > 0:
            print(json.dumps(out), flush=True)
        dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    if "RANK" in os.environ:
        rank_main(sys.argv[1:])
    else:
        sys.exit(spawn(sys.argv[1:], int(os.environ.get("PEER_RANKS", "2"))))
