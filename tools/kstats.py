#!/usr/bin/env python3
"""Per-kernel duration statistics from a rocprofv3 kernel trace (``--kernel-trace --output-format csv``,
the ``*_kernel_trace.csv`` file): launches, median / mean / min / max in microseconds, per kernel and
grid size (the fused ``k_lstm<.., RS>`` launch of steps 1..T-1 has 256 more workgroups than step 0's,
so the two forms come out as separate rows).

    python tools/kstats.py gpurun_out/prof/run_kernel_trace.csv profiles/r05_kernel_durations.csv

The bench line's ``roofline.median_launch_ms`` (dispatch timestamps of the same region) is checked
against this file's median row for the dominant kernel.
"""
import csv
import statistics
import sys


def col(header, *names):
    low = [h.lower() for h in header]
    for n in names:
        if n.lower() in low:
            return low.index(n.lower())
    raise KeyError(f"none of {names} in {header}")


def main(src, out):
    with open(src, newline="") as f:
        r = csv.reader(f)
        header = next(r)
        iname = col(header, "Kernel_Name", "KernelName", "Name")
        ibeg = col(header, "Start_Timestamp", "BeginNs", "Start")
        iend = col(header, "End_Timestamp", "EndNs", "End")
        try:
            igrid = col(header, "Grid_Size_X", "Grid_Size", "grd")
            iwg = col(header, "Workgroup_Size_X", "Workgroup_Size", "wgr")
        except KeyError:
            igrid = iwg = None
        groups = {}
        for row in r:
            name = row[iname]
            short = name.split("(")[0].replace("void ", "").strip()
            wgs = None
            if igrid is not None:
                try:
                    wgs = int(row[igrid]) // max(1, int(row[iwg]))
                except ValueError:
                    wgs = None
            groups.setdefault((short, wgs), []).append((int(row[iend]) - int(row[ibeg])) / 1e3)
    rows = []
    for (name, wgs), ds in groups.items():
        rows.append([name, wgs, len(ds), statistics.median(ds), statistics.fmean(ds), min(ds), max(ds), sum(ds)])
    rows.sort(key=lambda x: -x[-1])
    with open(out, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Kernel", "Workgroups", "Launches", "MedianUs", "MeanUs", "MinUs", "MaxUs", "TotalUs"])
        for x in rows:
            w.writerow(x[:3] + [f"{v:.3f}" for v in x[3:]])
    for x in rows[:12]:
        print(f"{x[0][:60]:60s} wg={x[1]} n={x[2]} med={x[3]:.2f} mean={x[4]:.2f} us")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
