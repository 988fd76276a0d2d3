"""Summarise rocprofv3 --pmc sqlite outputs: per kernel (name filter) mean counter values per dispatch.

python tools/pmc_summary.py gpurun_out/pmc/<run dir> [more dirs] [--filter conv]
"""
import glob
import sqlite3
import sys
from collections import defaultdict


def load(d, filt):
    out = defaultdict(lambda: defaultdict(list))
    for db in glob.glob(f"{d}/**/*.db", recursive=True):
        c = sqlite3.connect(db)
        q = "select kernel_name, dispatch_id, counter_name, sum(value), max(duration) from counters_collection group by dispatch_id, counter_name"
        for k, disp, cn, v, dur in c.execute(q):
            if filt and filt not in k:
                continue
            out[k][cn].append(v)
            out[k]["_dur_ns"].append(dur)
    return out


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    filt = ""
    if "--filter" in sys.argv:
        filt = sys.argv[sys.argv.index("--filter") + 1]
        args = [a for a in args if a != filt]
    for d in args:
        res = load(d, filt)
        for k, cs in res.items():
            print(f"== {d}: {k[:110]}")
            for cn in sorted(cs):
                vals = cs[cn]
                vals = vals[len(vals) // 3:] or vals  # drop warm-up dispatches
                print(f"   {cn:28s} {sum(vals) / len(vals):16.1f}")


if __name__ == "__main__":
    main()
