"""Summarise a rocprofv3 ``kernel_stats.csv``: top kernels by total time, grouped families."""
import csv
import re
import sys


def family(name: str) -> str:
    n = name.lower()
    rules = [("rtseg", r"interp|seg_ce|radix|sum_gt|seg_finalize|cast_out|act_mask|rtseg|kd_kl|confmat|bn_"),
             ("conv(miopen/ck)", r"conv|igemm|winograd|xdlops|implicit|miopensp|naive_conv|ck::|gridwise"),
             ("gemm(hipblaslt/rocblas)", r"gemm|cijk|hipblaslt|rocblas"),
             ("batchnorm", r"batch_?norm|bn_fwd|bn_bwd|miopenbatch|welford"),
             ("elementwise", r"elementwise|vectorized|unrolled|reduce|copy|fill|foreach|multi_tensor"),
             ("pool", r"pool|avg"), ("upsample(torch)", r"upsample|interp")]
    for fam, pat in rules:
        if re.search(pat, n):
            return fam
    return "other"


def main(path):
    rows = list(csv.DictReader(open(path)))
    tot_key = next(k for k in rows[0] if k.lower().startswith("totaldurationns") or k == "TotalDurationNs")
    cnt_key = next(k for k in rows[0] if k.lower() == "calls")
    name_key = next(k for k in rows[0] if k.lower() == "name")
    total = sum(float(r[tot_key]) for r in rows)
    fams = {}
    for r in rows:
        f = family(r[name_key])
        fams[f] = fams.get(f, 0.0) + float(r[tot_key])
    print(f"total kernel time: {total / 1e6:.2f} ms over {sum(int(r[cnt_key]) for r in rows)} launches")
    print("\n== by family ==")
    for f, t in sorted(fams.items(), key=lambda x: -x[1]):
        print(f"{t / 1e6:10.3f} ms  {100 * t / total:5.1f}%  {f}")
    print("\n== top 40 kernels ==")
    rows.sort(key=lambda r: -float(r[tot_key]))
    for r in rows[:40]:
        t = float(r[tot_key])
        print(f"{t / 1e6:9.3f} ms {100 * t / total:5.1f}% {int(r[cnt_key]):6d}x  {r[name_key][:150]}")


if __name__ == "__main__":
    main(sys.argv[1])
