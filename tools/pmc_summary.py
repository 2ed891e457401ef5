"""Aggregate rocprofv3 --pmc counter CSVs per kernel (mean per dispatch), and optionally write the
per-launch HBM traffic that bench.py reports as ``roofline.traffic``.

    python tools/pmc_summary.py gpurun_out/pmc_<tag> [--json counters.json] [--traffic profiles/traffic.json]

HBM bytes per launch follow MI355X_MICROARCH.md (HBM / rocprofv3): FETCH_SIZE and WRITE_SIZE are in
KiB, collected in separate passes; on gfx950 FETCH_SIZE reports half the bytes of a wide coalesced
streaming read, so hbm = (2 * FETCH_SIZE + WRITE_SIZE) * 1024.  Infinity-Cache hits are counted by
these fabric-side counters, so the figure is "bytes that left L2", an upper bound on HBM bytes.
"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict


def short_name(name: str) -> str:
    s = name.split("(")[0].replace("void ", "").replace("aa::", "").strip()
    return re.sub(r"<.*>", "", s)


def main():
    root = sys.argv[1]
    acc = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            acc[short_name(r.get("Kernel_Name", ""))][r["Counter_Name"]].append(float(r["Counter_Value"]))
    out = {}
    for k, d in sorted(acc.items()):
        out[k] = {c: sum(v) / len(v) for c, v in d.items()}
        print(k, {c: f"{v:.4g}" for c, v in out[k].items()})
    if "--json" in sys.argv:
        json.dump(out, open(sys.argv[sys.argv.index("--json") + 1], "w"), indent=1)
    if "--traffic" in sys.argv:
        traffic = {}
        for k, d in out.items():
            if "FETCH_SIZE" in d and "WRITE_SIZE" in d:
                traffic[k] = {"fetch_kib": d["FETCH_SIZE"], "write_kib": d["WRITE_SIZE"],
                              "hbm_bytes_per_launch": (2 * d["FETCH_SIZE"] + d["WRITE_SIZE"]) * 1024}
        traffic["_note"] = ("(2*FETCH_SIZE + WRITE_SIZE)*1024 per dispatch, mean over dispatches, separate --pmc "
                            "passes (MI355X_MICROARCH.md HBM section); k_gemm_bias mixes its two launch shapes")
        json.dump(traffic, open(sys.argv[sys.argv.index("--traffic") + 1], "w"), indent=1)


if __name__ == "__main__":
    main()
