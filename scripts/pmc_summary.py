"""Summarise rocprofv3 --pmc passes per kernel: mean counter values per dispatch and the derived
figures that decide what limits a kernel (MI355X_MICROARCH.md: SQ_* cycle counters are quad-cycles
summed over waves, SQ_VALU_MFMA_BUSY_CYCLES counts cycles summed over SIMDs, GRBM_GUI_ACTIVE is summed
over the 8 XCDs; FETCH_SIZE is doubled for gfx950's wide streaming reads).

    python scripts/pmc_summary.py gpurun_out/r03_attn_pmc [--match attn_] > profiles/r03_attn_pmc.json
"""
import argparse
import csv
import glob
import json
import os
import re
from collections import defaultdict

SIMDS = 256 * 4


def short(name):
    m = re.search(r"(\w+_kernel)", name)
    base = m.group(1) if m else name[:60]
    t = re.search(r"_kernel<([^>]*)>", name)
    return base + (f"<{t.group(1)}>" if t else "")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--match", default="")
    a = ap.parse_args()
    vals = defaultdict(lambda: defaultdict(list))
    dur = defaultdict(list)
    for path in sorted(glob.glob(os.path.join(a.dir, "pmc*", "*counter_collection.csv"))):
        with open(path) as f:
            for row in csv.DictReader(f):
                if a.match not in row["Kernel_Name"]:
                    continue
                k = short(row["Kernel_Name"])
                vals[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
                if row["Counter_Name"] in ("GRBM_GUI_ACTIVE", "SQ_WAVES"):
                    dur[k].append((int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) * 1e-3)
    out = {}
    for k, cs in vals.items():
        m = {c: sum(v) / len(v) for c, v in cs.items()}
        d = {"counters": {c: round(v, 1) for c, v in sorted(m.items())}}
        if dur[k]:
            d["us_profiled"] = round(sum(dur[k]) / len(dur[k]), 1)
        gui = m.get("GRBM_GUI_ACTIVE")
        if gui:
            cyc = gui / 8                                     # kernel cycles (one XCD's clock)
            d["kernel_cycles"] = round(cyc)
            if "us_profiled" in d:
                d["clock_ghz"] = round(cyc / d["us_profiled"] / 1e3, 3)
            if "SQ_VALU_MFMA_BUSY_CYCLES" in m:
                d["mfma_busy_frac"] = round(m["SQ_VALU_MFMA_BUSY_CYCLES"] / (cyc * SIMDS), 4)
        wc = m.get("SQ_WAVE_CYCLES")
        if wc:
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU",
                      "SQ_ACTIVE_INST_LDS", "SQ_ACTIVE_INST_SCA", "SQ_ACTIVE_INST_VMEM", "SQ_ACTIVE_INST_MISC"):
                if c in m:
                    d[c.lower().replace("sq_", "") + "_frac_of_wave_cycles"] = round(m[c] / wc, 4)
        if "SQ_INSTS_MFMA" in m:
            n = m["SQ_INSTS_MFMA"]
            for c in ("SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_SALU", "SQ_INSTS_VMEM", "SQ_INSTS_SMEM"):
                if c in m:
                    d[c.lower().replace("sq_insts_", "") + "_per_mfma"] = round(m[c] / n, 3)
        if "SQ_LDS_BANK_CONFLICT" in m and m.get("SQ_LDS_IDX_ACTIVE"):
            d["lds_bank_conflict_frac"] = round(m["SQ_LDS_BANK_CONFLICT"] / m["SQ_LDS_IDX_ACTIVE"], 4)
        if "FETCH_SIZE" in m:
            d["hbm_read_bytes"] = round(m["FETCH_SIZE"] * 1024 * 2)      # KiB, x2 gfx950 correction
        if "WRITE_SIZE" in m:
            d["hbm_write_bytes"] = round(m["WRITE_SIZE"] * 1024)
        out[k] = d
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
