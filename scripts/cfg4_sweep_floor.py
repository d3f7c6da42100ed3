"""cfg 4's pair-pool sweep in isolation, on the GPU box:
  1. bench.py's cfg 4 agent (CliffWalking traces SARSA, 2^17 lanes, G 256,
     reset-and-step) runs WARM launches, then RECORD launches with step records
     on; each record gives what the training kernel holds for the lane after its
     env step: the pair (s, a) it updates, whether it trains, whether its episode
     ends (rl.h rl_step_record) -> one u16 per (launch, step, lane) in $TMPDIR;
  2. the same agent's launch time without records (HIP events on its stream);
  3. rl-rust_amd/exp/pool_sweep (scripts/pool_sweep.hip) replays those inputs
     through the pool sweep alone at the same grid, once with the item loop and
     once without, launch after launch (pools carried over in HBM); then the
     same inputs tiled over 2x and 4x the lanes (more groups per CU).
Rank-0 style: one JSON line per measurement on stdout.

    python scripts/cfg4_sweep_floor.py [warm] [record]      (GPU)
    SWEEP_INPUT=path python scripts/cfg4_sweep_floor.py ...  (only write the inputs)
"""
import json
import os
import subprocess
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rl-rust_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    warm = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    rec = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    import torch
    import rlamd as rl
    from golden.make_fullsize import bench_params
    kw = bench_params(4, {})
    L = kw["n_lanes"]
    K = kw["sync_every"]

    def agent():
        a = rl.Agent(rl.default_params(**{k: v for k, v in kw.items() if k != "reset_step"}))
        a.set_reset_step(bool(kw["reset_step"]))
        return a

    # 2. the real kernel's launch time at the same point of training
    a = agent()
    s = torch.cuda.Stream()
    a.set_stream(s.cuda_stream)
    a.run(warm)
    a.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    a.run(rec)
    e1.record(s)
    torch.cuda.synchronize()
    print(json.dumps({"what": "agent_launch", "lanes": L, "steps_per_launch": K, "launches": rec,
                      "ms_per_launch": e0.elapsed_time(e1) / rec}), flush=True)
    a.close()

    # 1. the inputs, recorded from a fresh agent (same seeds: the same run)
    a = agent()
    a.run(warm)
    a.set_recording(True)
    xs, items = [], []
    for _ in range(rec):
        a.run(1)
        r = a.records()
        assert r.shape == (K, L), r.shape
        step = (r["kind"] == 2) | (r["kind"] == 3)
        x = (r["s"].astype(np.uint32) * 4 + r["a"]).astype(np.uint16)
        x |= np.where(step, 1 << 8, 0).astype(np.uint16)
        x |= np.where(step & (r["term"] != 0), 1 << 9, 0).astype(np.uint16)
        xs.append(x)
    n_items = a.trace_items()
    a.close()
    steps = np.stack(xs)
    trains = int(((steps >> 8) & 1).sum())
    print(json.dumps({"what": "inputs", "train_steps": trains,
                      "episode_ends": int(((steps >> 9) & 1).sum()),
                      "agent_trace_items_end": int(n_items),
                      "items_per_lane_end": n_items / L}), flush=True)
    keep = os.environ.get("SWEEP_INPUT")   # write the inputs there and stop (rocprofv3 passes on the replay)
    if keep:
        steps.tofile(keep)
        return
    fd, path = tempfile.mkstemp(suffix=".u16")
    os.close(fd)
    try:
        steps.tofile(path)
        del steps, xs
        exe = os.path.join(ROOT, "rl-rust_amd", "exp", "pool_sweep")
        # warm + rec launches of inputs only cover rec launches: the replay starts
        # from empty pools, so its first launch is a fill-up and the later ones
        # are the steady state the agent runs in
        rc = 0
        for tile in (1, 2, 4):       # 2^17 lanes (cfg 4's grid), then the same lanes twice / 4x
            rc = rc or subprocess.run([exe, path, str(L), str(K), str(rec), str(tile)], timeout=300).returncode
    finally:
        os.unlink(path)
    sys.exit(rc)


if __name__ == "__main__":
    main()
