"""Per-kernel summary of a rocprofv3 database (rocpd format, `run_results.db`) (tools only; round 6).

    python tools/prof_db.py gpurun_out/u/prof/run_results.db [--per N] [--seq NAME] [--like PATTERN]

Groups dispatches by (kernel, grid), prints launches / median / total microseconds (per --per
units, e.g. training steps), and with --seq the ordered dispatches of one unit whose names contain
NAME (grid, stream, duration) -- to attribute each GEMM launch of a step."""
import argparse
import sqlite3
import statistics


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--per", type=int, default=1, help="divide totals by this many units (steps)")
    ap.add_argument("--like", default="", help="only kernels whose name contains this")
    ap.add_argument("--seq", default="", help="print the dispatch sequence of the last unit, marked by this kernel")
    ap.add_argument("--top", type=int, default=30)
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = c.execute("select name, grid_x, grid_y, grid_z, workgroup_x, duration, start, stream_id, queue_id "
                     "from kernels order by start").fetchall()
    agg = {}
    for name, gx, gy, gz, wx, dur, st, sid, qid in rows:
        if a.like and a.like not in name:
            continue
        key = (name[:70], gx * gy * gz // max(wx, 1))
        agg.setdefault(key, []).append(dur / 1e3)
    tot = sum(sum(v) for v in agg.values())
    print(f"{len(rows)} dispatches, {tot / a.per:.1f} us per unit")
    for (n, wg), v in sorted(agg.items(), key=lambda kv: -sum(kv[1]))[:a.top]:
        print(f"{sum(v) / a.per:9.1f} us/unit {len(v) / a.per:6.2f} x  median {statistics.median(v):8.2f}  wg {wg:6d}  {n}")
    if a.seq:
        marks = [i for i, r in enumerate(rows) if a.seq in r[0]]
        if len(marks) >= 2:
            lo, hi = marks[-2] + 1, marks[-1] + 1
            t0 = rows[lo][6]
            for name, gx, gy, gz, wx, dur, st, sid, qid in rows[lo:hi]:
                print(f"  +{(st - t0) / 1e3:8.1f} us  q{qid} {dur / 1e3:7.2f} us  wg {gx * gy * gz // max(wx, 1):6d}  {name[:60]}")


if __name__ == "__main__":
    main()
