"""File one workload's rocprofv3 evidence (scripts/profile.sh output dir) under
profiles/: <round>_<key>_kernel_stats.csv, <round>_<key>_summary.json, and the
entry bench.py reads back for `roofline.traffic` / `issue_frac`
(profiles/counters.json, keyed by workload: cfg2, cfg2_slippery, cfg3, ...).

    python scripts/collect_counters.py gpurun_out/prof_r04_cfg3 r04 --config 3 [--slippery 1] [--q-mode f64]

The entry records the profiled library's rl_build_id (from the bench JSON line in
<profdir>/trace.log); bench.py attaches it only to runs of that same library.
"""
import argparse
import json
import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, HERE)
sys.path.insert(0, ROOT)
from summarize_profile import summarize  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("profdir")
    ap.add_argument("round")
    ap.add_argument("--config", type=int, required=True)
    ap.add_argument("--slippery", type=int, default=0)
    ap.add_argument("--kernel", default=None, help="default: k_train_private for group 1 presets, else k_train_shared")
    ap.add_argument("--q-mode", default="auto")
    ap.add_argument("--lanes", type=int, default=None)
    a = ap.parse_args()
    import bench
    pr = bench.PRESETS[a.config]
    lanes = a.lanes or pr["lanes"]
    key = bench.workload_key(argparse.Namespace(config=a.config, slippery=a.slippery, q_mode=a.q_mode,
                                                lanes=lanes))
    # the library the profiled bench ran: its JSON line's build_id (rl_build_id)
    build_id = None
    for line in open(os.path.join(a.profdir, "trace.log")):
        if line.startswith("{"):
            build_id = json.loads(line).get("build_id")
    if not build_id:
        sys.exit(f"no bench line with a build_id in {a.profdir}/trace.log")
    s = summarize(a.profdir, a.kernel or ("k_train_private" if pr["group"] == 1 else "k_train_shared"))
    prof = os.path.join(ROOT, "profiles")
    stem = f"{a.round}_{key}"
    shutil.copy(os.path.join(a.profdir, "trace", "run_kernel_stats.csv"),
                os.path.join(prof, stem + "_kernel_stats.csv"))
    head = os.environ.get("RLAMD_HEAD")   # set by the GPU-box scripts (no .git there)
    if not head:
        try:
            head = subprocess.run(["git", "-C", ROOT, "rev-parse", "--short", "HEAD"], capture_output=True,
                                  text=True).stdout.strip()
        except OSError:
            head = "?"
    s["dir"] = f"{a.profdir} (copied; build at HEAD {head or '?'})"
    json.dump(s, open(os.path.join(prof, stem + "_summary.json"), "w"), indent=1)
    path = os.path.join(prof, "counters.json")
    tab = json.load(open(path)) if os.path.exists(path) else {}
    hb = s.get("hbm_bytes_per_launch", {})
    tab[key] = {"env": pr["env"], "algo": pr["algo"], "lanes": lanes, "group": pr["group"],
                "sync": 64, "slippery": a.slippery, "reset_step": pr.get("reset_step", 0), "q_mode": a.q_mode,
                "build_id": build_id,
                "hbm_bytes_per_launch": hb.get("total"),
                "valu_busy_frac": s.get("valu_busy_frac"),
                "valu_pipe_frac": s.get("valu_pipe_frac"),
                "valu_busy_rocm": s.get("valu_busy_rocm"),
                "lds_active_frac": s.get("lds_active_frac"),
                "lds_bank_conflict_frac": (s["pmc_mean_per_launch"].get("SQ_LDS_BANK_CONFLICT", 0.0) /
                                           s["pmc_mean_per_launch"]["SQ_LDS_IDX_ACTIVE"])
                if "SQ_LDS_IDX_ACTIVE" in s["pmc_mean_per_launch"] else None,
                "wave_cycle_split": s.get("wave_cycle_split"),
                "kernel_avg_ns": s.get("kernel_avg_ns"),
                "source": f"profiles/{stem}_summary.json: rocprofv3 separate --pmc passes (FETCH_SIZE x2 "
                          f"gfx950 correction + WRITE_SIZE; VALU pipe occupancy = (2 x SQ_INSTS_VALU + 2 x (FP64 "
                          f"add/mul/fma + INT64) + 6 x TRANS_F64) cycles / (GRBM_GUI_ACTIVE/8 x 1024 SIMDs)), mean "
                          f"per launch of the dominant kernel, library {build_id}"}
    json.dump(tab, open(path, "w"), indent=1, sort_keys=True)
    print(json.dumps(tab[key], indent=1))


if __name__ == "__main__":
    main()
