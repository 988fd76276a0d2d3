"""Per-step kernel breakdown from a rocprofv3 ``kernel_trace.csv``.

Steps are delimited by a marker kernel (default: the fused loss forward
``seg_ce_fwd_kernel``, launched ``--per-step`` times per training step).  The
first ``--skip`` steps (warm-up / MIOpen find) are dropped, so the summary
reflects steady-state steps only.

  python tools/summarize_trace.py run_kernel_trace.csv --skip 3 --per-step 2
"""
from __future__ import annotations

import argparse
import csv
import re
import sys

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from summarize_kernel_stats import family  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--marker", default="seg_ce_fwd")
    ap.add_argument("--per-step", type=int, default=2)
    ap.add_argument("--skip", type=int, default=3)
    ap.add_argument("--top", type=int, default=45)
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    marks = [i for i, r in enumerate(rows) if a.marker in r["Kernel_Name"]]
    first_fwd = marks[a.skip * a.per_step] if len(marks) > a.skip * a.per_step else 0
    # a step starts after the previous step's last kernel; approximate the window
    # start as the first kernel after the (skip)-th step's final marker's step end:
    # use the kernel following the last marker of the skipped steps + its backward.
    start_idx = 0
    if a.skip > 0 and len(marks) >= a.skip * a.per_step:
        prev_last = marks[a.skip * a.per_step - 1]
        # the skipped step still runs its backward/optimizer after its marker; the
        # next step's first forward kernel is the earliest conv after that batch of
        # optimizer kernels -- approximate with midpoint between markers
        start_idx = (prev_last + first_fwd) // 2 if first_fwd else prev_last
    window = rows[start_idx:]
    nsteps = max(1, (len(marks) - a.skip * a.per_step) // a.per_step)
    t0 = int(window[0]["Start_Timestamp"])
    t1 = int(window[-1]["End_Timestamp"])
    busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in window)
    print(f"steps analysed: {nsteps}  wall {((t1 - t0) / 1e6) / nsteps:.3f} ms/step  "
          f"kernel-busy {busy / 1e6 / nsteps:.3f} ms/step  launches/step {len(window) / nsteps:.0f}")
    agg = {}
    fam = {}
    for r in window:
        d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        n = r["Kernel_Name"]
        k = agg.setdefault(n, [0, 0])
        k[0] += d
        k[1] += 1
        f = family(n)
        fam[f] = fam.get(f, 0) + d
    print("\n== by family (ms/step) ==")
    for f, t in sorted(fam.items(), key=lambda x: -x[1]):
        print(f"{t / 1e6 / nsteps:9.3f}  {100 * t / busy:5.1f}%  {f}")
    print(f"\n== top {a.top} kernels (ms/step, calls/step) ==")
    for n, (t, c) in sorted(agg.items(), key=lambda x: -x[1][0])[:a.top]:
        short = re.sub(r"\s+", " ", n)[:140]
        print(f"{t / 1e6 / nsteps:8.3f} {100 * t / busy:5.1f}% {c / nsteps:6.1f}  {short}")


if __name__ == "__main__":
    main()
