"""Known answers for multi-GPU bench runs: the oracle's
one-process result for the GLOBAL lane sets bench.py runs at N GPUs.

Lanes are partitioned contiguously by global id (rank r owns [r*L, (r+1)*L)),
every learner group lies inside one rank, and the merges are exact integer sums
(DESIGN.md §6), so an N-rank run of a global lane set ends with exactly the raw Q
words of one process running that whole set.  For each case: the SHA-256 of the
merged raw Q words (int64 little-endian, [P][S][A]: fixed-point raws or f64 bits)
and the training env-steps over all lanes after `launches` launches of K = 64.

bench.py prints the same digest (`q_check`) and compares it with the case whose
key matches its run; tests/test_gpu_global_q.py runs every case on one GPU.

Cases (the driver's command shape is --steps 20 --warmup 5: 25 launches):
  cfg2_L{1,2,4,8}M_25   bench.py --config 2 --gpus N (2^20 lanes per GPU, weak), N = 1, 2, 4, 8;
                        --lanes-total 1048576 at any N is cfg2_L1M_25 (strong)
  cfg2_L1M_65           the default bench run (1 + 64 launches) at 2^20 lanes in total
  cfg5_L4M_25           bench.py --config 5 --gpus 8 (2^19 per GPU = BASELINE's 2^22 in total)
  cfg4_L512K_25         bench.py --config 4 --gpus 4 (BASELINE's 2^19 envs over 4 GPUs: 2^17 per rank,
                        the N > 1 default) and bench.py --config 4 --lanes 524288 on one GPU

    python tests/golden/make_global_q.py        (the 2^23-lane case is the long one: about 15 min)
"""
import hashlib
import json
import os
import sys
from concurrent.futures import ProcessPoolExecutor

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, HERE)

M = 1 << 20
CASES = {
    "cfg2_L1M_25": (2, M, 25), "cfg2_L2M_25": (2, 2 * M, 25), "cfg2_L4M_25": (2, 4 * M, 25),
    "cfg2_L8M_25": (2, 8 * M, 25), "cfg2_L1M_65": (2, M, 65), "cfg5_L4M_25": (5, 4 * M, 25),
    "cfg4_L512K_25": (4, M // 2, 25),
}


def key_of(cfg, lanes, launches):
    from make_fullsize import bench_params
    kw = bench_params(cfg, {"n_lanes": lanes})
    return kw, {"env": kw["env"], "agent": kw["agent"], "policy": kw["policy"], "selector": kw["selector"],
                "algo": kw["algo"], "map8x8": kw.get("map8x8", 1), "slippery": kw.get("slippery", 0),
                "reset_step": int(kw["reset_step"]), "q_mode": "auto", "global_lanes": lanes,
                "group": kw["group_size"], "sync": kw["sync_every"], "launches": launches}


def run(name):
    import oracle_ffi as O
    cfg, lanes, launches = CASES[name]
    kw, key = key_of(cfg, lanes, launches)
    b = O.Batch(O.default_params(**{k: v for k, v in kw.items() if k != "reset_step"}))
    b.set_reset_step(bool(kw["reset_step"]))
    b.run(launches)
    raw = b.q_raw().astype("<i8")
    return name, {"key": key, "q_repr": b.q_repr(), "q_sha256": hashlib.sha256(raw.tobytes()).hexdigest(),
                  "train_steps": int(b.stats()[0])}


def main():
    import oracle_ffi
    oracle_ffi.build()
    names = sys.argv[1:] or list(CASES)
    path = os.path.join(HERE, "global_q.json")
    out = json.load(open(path)) if os.path.exists(path) else {}
    out["source"] = ("oracle/rlref.c batched schedule, one process over the whole global lane set "
                     "(tests/golden/make_global_q.py)")
    cases = out.setdefault("cases", {})
    with ProcessPoolExecutor(max_workers=min(len(names), 6)) as ex:
        for name, c in ex.map(run, names):
            cases[name] = c
            print(name, c["q_sha256"][:16], c["train_steps"], flush=True)
    out["cases"] = {k: cases[k] for k in sorted(cases)}
    json.dump(out, open(path, "w"), indent=1)
    open(path, "a").write("\n")


if __name__ == "__main__":
    main()
