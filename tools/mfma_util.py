"""Per-kernel MFMA utilisation and wave-state shares from a rocprofv3 --pmc run that also carries
--kernel-trace (tools/pmc.sh): joins counter_collection.csv with kernel_trace.csv by dispatch.

    python tools/mfma_util.py gpurun_out/pmc_<tag>/mfma [--clock-ghz 2.4] [--json out.json]

util = SQ_VALU_MFMA_BUSY_CYCLES / (kernel duration x clock x 1024 SIMDs).  The MFMA-busy counter
counts cycles (32 per v_mfma_f32_32x32x16_bf16: MI355X_MICROARCH.md constants), summed over the
chip per dispatch; the denominator is the dispatch's own kernel-trace duration (not GRBM_GUI_ACTIVE)
at the peak clock the dense-MFMA peaks assume (2.4 GHz), so util is directly comparable with a
FLOP-based fraction of those peaks.  SQ_* wave-state counters (quad-cycles) are reported as shares
of SQ_WAVE_CYCLES when present."""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict

SIMDS = 256 * 4


def short_name(name: str) -> str:
    s = name.split("(")[0].replace("void ", "").replace("aa::", "").strip()
    return re.sub(r"<.*>", "", s)


def main():
    root = sys.argv[1]
    clock = float(sys.argv[sys.argv.index("--clock-ghz") + 1]) if "--clock-ghz" in sys.argv else 2.4
    dur = {}
    for f in glob.glob(os.path.join(root, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            dur[r["Dispatch_Id"]] = (short_name(r["Kernel_Name"]), int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    per = defaultdict(lambda: defaultdict(float))
    for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            per[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
    agg = defaultdict(lambda: defaultdict(list))
    for d, ctr in per.items():
        if d not in dur:
            continue
        name, ns = dur[d]
        agg[name]["ns"].append(ns)
        for c, v in ctr.items():
            agg[name][c].append(v)
    out = {}
    for name, d in sorted(agg.items()):
        n = len(d["ns"])
        ns = sum(d["ns"]) / n
        row = {"dispatches": n, "avg_us": ns / 1e3}
        mean = {c: sum(v) / len(v) for c, v in d.items() if c != "ns"}
        if "SQ_VALU_MFMA_BUSY_CYCLES" in mean:
            row["mfma_busy_cycles"] = mean["SQ_VALU_MFMA_BUSY_CYCLES"]
            row["mfma_util"] = mean["SQ_VALU_MFMA_BUSY_CYCLES"] / (ns * clock * SIMDS)
        wc = mean.get("SQ_WAVE_CYCLES")
        for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS"):
            if wc and c in mean:
                row[c.lower() + "_share"] = mean[c] / wc
        for c, v in mean.items():
            row.setdefault(c, v)
        out[name] = row
        print(f"{name:22s} n={n:4d} avg {ns / 1e3:8.2f} us  " +
              "  ".join(f"{k}={v:.3g}" for k, v in row.items() if k.endswith(("util", "_share"))))
    if "--json" in sys.argv:
        json.dump(out, open(sys.argv[sys.argv.index("--json") + 1], "w"), indent=1)


if __name__ == "__main__":
    main()
