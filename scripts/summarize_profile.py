"""Summarize a rocprofv3 profile directory (scripts/profile.sh output) for the
dominant kernel: trace stats, per-launch PMC means, derived HBM bytes and
VALU utilisation.  Writes <dir>/summary.json and prints it."""
import collections
import csv
import glob
import json
import os
import sys



def summarize(d, kern="k_train_shared"):
    out = {"dir": d, "kernel_match": kern}
    stats = list(csv.DictReader(open(os.path.join(d, "trace", "run_kernel_stats.csv"))))
    out["kernel_stats"] = [{k: r[k] for k in ("Name", "Calls", "AverageNs", "Percentage")} for r in stats]
    pmc = collections.defaultdict(list)
    for f in glob.glob(os.path.join(d, "pmc_*", "run_counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            if kern in r["Kernel_Name"]:
                pmc[r["Counter_Name"]].append(float(r["Counter_Value"]))
    m = {k: sum(v) / len(v) for k, v in pmc.items()}
    out["pmc_mean_per_launch"] = m
    dom = next(r for r in stats if kern in r["Name"])
    t_ns = float(dom["AverageNs"])
    if "FETCH_SIZE" in m and "WRITE_SIZE" in m:
        # gfx950: FETCH_SIZE reads half the bytes of wide coalesced streaming reads
        # (MI355X_MICROARCH.md §HBM) -> x2; units are KiB.
        rd = 2 * m["FETCH_SIZE"] * 1024
        wr = m["WRITE_SIZE"] * 1024
        out["hbm_bytes_per_launch"] = {"read_corrected": rd, "write": wr, "total": rd + wr,
                                       "GBps": (rd + wr) / t_ns}
    if "SQ_INSTS_VALU" in m and "SQ_WAVES" in m:
        out["valu_instr_per_wave"] = m["SQ_INSTS_VALU"] / m["SQ_WAVES"]
        out["salu_instr_per_wave"] = m.get("SQ_INSTS_SALU", 0) / m["SQ_WAVES"]
        out["lds_instr_per_wave"] = m.get("SQ_INSTS_LDS", 0) / m["SQ_WAVES"]
    if "GRBM_GUI_ACTIVE" in m:
        cyc = m["GRBM_GUI_ACTIVE"] / 8            # summed over 8 XCDs
        out["clock_GHz"] = cyc / t_ns
        if "SQ_INSTS_VALU" in m:
            # 256 CUs x 4 SIMDs; a wave64 VALU op occupies a SIMD32 for 2 cycles
            out["valu_busy_frac"] = m["SQ_INSTS_VALU"] * 2 / (cyc * 256 * 4)
        if "SQ_INSTS_VALU" in m and "SQ_INSTS_VALU_INT64" in m:
            # VALU pipe occupancy: a wave64 op holds a SIMD32 for 2 cycles
            # (MI355X_MICROARCH.md), FP64 add/mul/fma and 64-bit integer ops run at half
            # rate (4), FP64 transcendentals at a quarter of that (8)
            f64 = m["SQ_INSTS_VALU_ADD_F64"] + m["SQ_INSTS_VALU_MUL_F64"] + m["SQ_INSTS_VALU_FMA_F64"]
            tr = m.get("SQ_INSTS_VALU_TRANS_F64", 0.0)
            cyc_valu = 2 * m["SQ_INSTS_VALU"] + 2 * (f64 + m["SQ_INSTS_VALU_INT64"]) + 6 * tr
            out["valu_pipe_frac"] = cyc_valu / (cyc * 256 * 4)
            out["valu_mix_per_wave_step_div_K"] = {"f64": f64 / m.get("SQ_WAVES", 1), "int64": m["SQ_INSTS_VALU_INT64"] / m.get("SQ_WAVES", 1),
                                                   "trans_f64": tr / m.get("SQ_WAVES", 1)}
        if "SQ_ACTIVE_INST_VALU" in m:
            # ROCm's VALUBusy (SQ_ACTIVE_INST_VALU quad-cycles per SIMD): 4 cycles per
            # wave-instruction, i.e. an upper bound for the pipe occupancy above
            out["valu_busy_rocm"] = m["SQ_ACTIVE_INST_VALU"] * 4 / (cyc * 256 * 4)
        if "SQ_LDS_IDX_ACTIVE" in m:
            out["lds_active_frac"] = m["SQ_LDS_IDX_ACTIVE"] / 256 / cyc
        if "SQ_LDS_BANK_CONFLICT" in m:
            out["lds_bank_conflict_cycles_per_cu"] = m["SQ_LDS_BANK_CONFLICT"] / 256
    if "SQ_WAVE_CYCLES" in m:
        w = m["SQ_WAVE_CYCLES"]
        out["wave_cycle_split"] = {k: m[k] / w for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY",
                                                          "SQ_WAIT_INST_LDS", "SQ_ACTIVE_INST_VALU",
                                                          "SQ_ACTIVE_INST_LDS", "SQ_ACTIVE_INST_SCA") if k in m}
    out["kernel_avg_ns"] = t_ns
    return out


if __name__ == "__main__":
    d = sys.argv[1]
    out = summarize(d, sys.argv[2] if len(sys.argv) > 2 else "k_train_shared")
    json.dump(out, open(os.path.join(d, "summary.json"), "w"), indent=1)
    print(json.dumps(out, indent=1))
