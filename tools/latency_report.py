"""Batch-1 inference latency breakdown from a rocprofv3 kernel trace of tools/profile_infer.py.

The HIP-graph engine replays the same kernel sequence every forward, so the kernels per forward (K)
are the period of the trace's kernel-name sequence; the last ``--iters`` x K kernels are the timed
replays.  Reports per forward: kernel count, summed kernel time, the wall span of one replay
(first kernel start to last kernel end) and the gaps between kernels, the kernel-duration histogram
and the top kernels -- which says whether a small model is bound by kernel work, by per-kernel
floors (many few-microsecond kernels on tiny maps), or by the gaps between launches.

  python tools/latency_report.py run_kernel_trace.csv --iters 200 [--wall-ms 1.23]
"""
import argparse
import collections
import csv


def period(names, max_p=20000):
    """Kernels per replay: the smallest p whose last three windows hold the same kernels.  Compared
    as multisets: with concurrent streams (ops/streams.py) the start-time order of kernels on two
    queues differs from replay to replay."""
    n = len(names)
    for p in range(1, min(max_p, n // 3) + 1):
        if names[n - p:] == names[n - 2 * p:n - p] == names[n - 3 * p:n - 2 * p]:
            return p
    for p in range(1, min(max_p, n // 3) + 1):
        a = collections.Counter(names[n - p:])
        if a == collections.Counter(names[n - 2 * p:n - p]) == collections.Counter(names[n - 3 * p:n - 2 * p]):
            return p
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--wall-ms", type=float, default=None, help="host-timed ms per image (profile_infer)")
    ap.add_argument("--top", type=int, default=15)
    a = ap.parse_args()
    rows = sorted(csv.DictReader(open(a.trace)), key=lambda r: int(r["Start_Timestamp"]))
    names = [r["Kernel_Name"] for r in rows]
    k = period(names)
    if k is None:
        raise SystemExit("no periodic replay found")
    n = min(a.iters, len(rows) // k - 1)
    sel = rows[len(rows) - n * k:]
    dur = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in sel]  # us
    busy = sum(dur) / n
    spans, gaps = [], []
    for i in range(n):
        blk = sel[i * k:(i + 1) * k]
        spans.append((int(blk[-1]["End_Timestamp"]) - int(blk[0]["Start_Timestamp"])) / 1e3)
        for x, y in zip(blk, blk[1:]):
            gaps.append(max(0, int(y["Start_Timestamp"]) - int(x["End_Timestamp"])) / 1e3)
    span = sorted(spans)[len(spans) // 2]
    gap = sum(gaps) / n
    print(f"kernels per forward {k}, forwards analysed {n}")
    print(f"per forward: kernel time {busy:.1f} us, replay span (median) {span:.1f} us, inter-kernel gaps {gap:.1f} us"
          f" ({gap / max(k - 1, 1):.2f} us per gap)")
    if a.wall_ms:
        print(f"host wall {a.wall_ms * 1e3:.1f} us per image: {a.wall_ms * 1e3 - span:.1f} us outside the replay span")
    bins = [2, 5, 10, 25, 50, 100, 1e9]
    hist = collections.Counter(next(b for b in bins if d <= b) for d in dur)
    acc = collections.Counter()
    for d, b in ((d, next(b for b in bins if d <= b)) for d in dur):
        acc[b] += d
    print("kernel duration histogram (per forward): " + ", ".join(
        f"<={b:g}us: {hist[b] / n:.0f} kernels {acc[b] / n:.0f} us" for b in bins if hist[b]))
    tot = collections.defaultdict(lambda: [0, 0.0])
    for r, d in zip(sel, dur):
        t = tot[r["Kernel_Name"][:110]]
        t[0] += 1
        t[1] += d
    print("top kernels (us per forward, calls per forward):")
    for name, (c, d) in sorted(tot.items(), key=lambda kv: -kv[1][1])[:a.top]:
        print(f"  {d / n:8.1f} {c / n:5.1f}  {name}")


if __name__ == "__main__":
    main()
