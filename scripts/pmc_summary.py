"""Summarise rocprofv3 --pmc counter CSVs: per kernel (name prefix), counters averaged over
dispatches, plus derived ratios (per wave: VALU / SALU / LDS / MFMA instructions, VALU:MFMA,
LDS bank-conflict share of LDS-active cycles, wait share of wave cycles).

    python scripts/pmc_summary.py gpurun_out/pmc1/run_counter_collection.csv [more.csv ...]
"""
import csv
import sys
from collections import defaultdict

KEEP = ("conv_stack", "conv_gl", "wgrad_gl", "dense_lds", "dual_halo", "wgrad_halo", "reduce_optim", "dense_", "head_kernel", "prologue",
        "conv_halo", "wgrad_tile", "conv_tile", "optim_kernel", "slab_reduce", "xgmi", "dense_wgrad", "dense_dx")


def main(paths):
    acc = defaultdict(lambda: defaultdict(list))
    for p in paths:
        with open(p) as f:
            for row in csv.DictReader(f):
                name = row["Kernel_Name"]
                if not any(k in name for k in KEEP):
                    continue
                short = name.split("(")[0][:48]
                acc[short][row["Counter_Name"]].append(float(row["Counter_Value"]))
                acc[short]["_vgpr"] = [float(row["VGPR_Count"])]
                acc[short]["_lds"] = [float(row["LDS_Block_Size"])]
    for k in sorted(acc):
        c = {n: sum(v) / len(v) for n, v in acc[k].items()}
        waves = c.get("SQ_WAVES", 0) or 1
        parts = ["%s=%.0f" % (n, v) for n, v in sorted(c.items()) if not n.startswith("_")]
        print("%s  [vgpr %d, lds %d]" % (k, c.get("_vgpr", 0), c.get("_lds", 0)))
        print("    " + " ".join(parts))
        d = []
        if "SQ_INSTS_VALU" in c:
            d.append("VALU/wave %.0f" % (c["SQ_INSTS_VALU"] / waves))
        if "SQ_INSTS_MFMA" in c and c["SQ_INSTS_MFMA"]:
            d.append("MFMA/wave %.0f" % (c["SQ_INSTS_MFMA"] / waves))
            if "SQ_INSTS_VALU" in c:
                d.append("VALU:MFMA %.1f" % (c["SQ_INSTS_VALU"] / c["SQ_INSTS_MFMA"]))
        if "SQ_INSTS_LDS" in c:
            d.append("LDS/wave %.0f" % (c["SQ_INSTS_LDS"] / waves))
        if "SQ_LDS_BANK_CONFLICT" in c and c.get("SQ_LDS_IDX_ACTIVE"):
            d.append("bank-conflict %.0f%% of LDS-active" % (100 * c["SQ_LDS_BANK_CONFLICT"] / c["SQ_LDS_IDX_ACTIVE"]))
        if "SQ_WAIT_ANY" in c and c.get("SQ_WAVE_CYCLES"):
            d.append("wait %.0f%% of wave cycles" % (100 * c["SQ_WAIT_ANY"] / c["SQ_WAVE_CYCLES"]))
        if "SQ_INSTS_SALU" in c and "SQ_WAVES" in c:
            d.append("SALU/wave %.0f" % (c["SQ_INSTS_SALU"] / waves))
        if "FETCH_SIZE" in c:
            d.append("HBM fetch %.1f KB, write %.1f KB" % (c["FETCH_SIZE"], c.get("WRITE_SIZE", 0)))
        if d:
            print("    -> " + ", ".join(d))


if __name__ == "__main__":
    main(sys.argv[1:])
