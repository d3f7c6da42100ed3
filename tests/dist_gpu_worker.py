"""One rank of the N>1 merge rehearsal (run by tests/test_dist_gpu.py under
torch.distributed.run; gloo, every rank on the box's one GPU).

Each rank owns the contiguous global lanes [rank*L, (rank+1)*L) and runs the
bench.py step: rl_agent_launch_train -> all_reduce(MAX of the leading merge
words) -> rl_agent_launch_fold -> all_reduce(SUM of the rest) ->
rl_agent_launch_apply.  Rank 0 then runs ONE agent holding all world*L lanes
for the same number of launches (rl_agent_run: the in-process merge) and
writes whether raw Q, UCB counters and t are bit-identical, plus the step
counts, to the JSON file named by argv[1].
"""
import json
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rl-rust_amd"))
import rlamd  # noqa: E402


def main():
    out_path, case = sys.argv[1], json.loads(sys.argv[2])
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    torch.cuda.set_device(0)
    dist.init_process_group("gloo")
    n_launch = case.pop("n_launch")
    L = case.pop("lanes_per_rank")
    merge = case.pop("merge", "torch")
    train_eps = case.pop("train_episodes", 0)
    p = rlamd.default_params(n_lanes=L, lane_offset=rank * L, **case)
    a = rlamd.Agent(p)
    groups = (L + case["group_size"] - 1) // case["group_size"]
    path = None
    if merge == "peer":
        # rl.h ABI 7: the exchange regions' IPC handles all-gathered (here over gloo),
        # then every merge of run() / train() reads the peers' words in the library
        hs = [None] * world
        dist.all_gather_object(hs, a.peer_handle())
        a.peer_attach(rank, world, hs)
        a.set_merge_groups(world * groups)
        path = a.merge_path()
        repr_rank = a.q_repr()
        dist.barrier()
        for _ in range(n_launch):
            a.run(1)
        if train_eps:
            a.train(train_eps, 0)       # the control word summed over the peers too
        a.synchronize()
    else:
        delta = torch.zeros(a.delta_words(), dtype=torch.int64, device="cuda:0")
        mw = a.delta_max_words()
        a.set_delta_buffer(delta.data_ptr(), delta.numel())
        a.set_merge_groups(world * groups)          # the f64 merge grid counts every rank's groups
        repr_rank = a.q_repr()
        # torch's HIP runtime (its wheel's own) and librlamd's do not order each other's
        # streams: each hand-over synchronizes the side that wrote the buffer
        for _ in range(n_launch):
            a.launch_train()
            a.synchronize()
            dist.all_reduce(delta[:mw], op=dist.ReduceOp.MAX)
            torch.cuda.synchronize()
            a.launch_fold()
            a.synchronize()
            dist.all_reduce(delta[mw:])
            torch.cuda.synchronize()
            a.launch_apply()
        a.synchronize()
    q, qf = a.q_raw(), a.q()
    st = a.stats()["train_steps"]
    ucb = a.ucb() if case.get("selector") == "ucb" else None
    steps = torch.tensor([st], dtype=torch.int64)
    dist.all_reduce(steps)
    a.close()
    if rank == 0:
        one = rlamd.Agent(rlamd.default_params(n_lanes=world * L, lane_offset=0, **case))
        one.run(n_launch)
        if train_eps:
            one.train(train_eps, 0)
        one.synchronize()
        qf1 = one.q()
        res = {"q_equal": bool(np.array_equal(q, one.q_raw())),
               # f64 image incl. the sticky NaN/inf flags of UCB + expected SARSA
               "qf_equal": bool(np.array_equal(np.isnan(qf), np.isnan(qf1)) and
                                np.array_equal(np.nan_to_num(qf).view(np.uint64),
                                               np.nan_to_num(qf1).view(np.uint64))),
               "q_nonfinite": int(np.count_nonzero(~np.isfinite(qf))),
               "q_nonzero": int(np.count_nonzero(q)),
               "q_repr": [repr_rank, one.q_repr()],
               "steps_ranks": int(steps.item()), "steps_one": int(one.stats()["train_steps"]),
               "merge_path": path}
        if ucb is not None:
            u1 = one.ucb()
            res["ucb_equal"] = bool(np.array_equal(ucb[0], u1[0]) and ucb[1] == u1[1])
        one.close()
        json.dump(res, open(out_path, "w"))
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
