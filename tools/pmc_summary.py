"""Aggregate rocprofv3 --pmc counter CSVs per kernel (mean per dispatch).
usage: python tools/pmc_summary.py gpurun_out/pmc_<tag> [--json out.json]"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def main():
    root = sys.argv[1]
    acc = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            name = r.get("Kernel_Name", "")
            short = name.split("(")[0].replace("aa::", "")
            acc[short][r["Counter_Name"]].append(float(r["Counter_Value"]))
    out = {}
    for k, d in sorted(acc.items()):
        out[k] = {c: sum(v) / len(v) for c, v in d.items()}
        print(k, {c: f"{v:.4g}" for c, v in out[k].items()})
    if "--json" in sys.argv:
        json.dump(out, open(sys.argv[sys.argv.index("--json") + 1], "w"), indent=1)


if __name__ == "__main__":
    main()
