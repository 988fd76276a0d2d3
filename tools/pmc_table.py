#!/usr/bin/env python3
"""Table of the conv kernels' PMC from tools/pmc_summary.py output (tools/gpu_pmc.sh summary.txt):
MFMA busy = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x duration x 2.4 GHz) from pass 1, the
instruction mix from pass 2 (pass-1 duration: the counters inflate it a little).

  python tools/pmc_table.py gpurun_out/r5_pmc/summary.txt
"""
import re
import sys
from collections import defaultdict


def main():
    rows = defaultdict(dict)
    probe = kern = None
    for line in open(sys.argv[1]):
        m = re.match(r"== .*/([^/]+)_p(\d): (.*)$", line.rstrip())
        if m:
            probe, kern = m.group(1), m.group(3)
            continue
        m = re.match(r"\s+(\S+)\s+([-0-9.eE+]+)$", line)
        if m and probe and "rtseg" in kern:
            rows[(probe, kern.replace("(anonymous namespace)::", "")[:70])][m.group(1)] = float(m.group(2))
    print(f"{'probe':28s} {'kernel':44s} {'dur_us':>7s} {'mfma%':>6s} {'VALU/MFMA':>9s} {'SALU/MFMA':>9s} "
          f"{'wait_inst%':>10s} {'lds_conf':>8s}")
    for (probe, kern), c in sorted(rows.items()):
        dur = c.get("_dur_ns", 0.0)
        mfma = c.get("SQ_INSTS_MFMA") or float("nan")
        busy = c.get("SQ_VALU_MFMA_BUSY_CYCLES")
        if busy is None or not dur:
            continue
        short = kern.split("(")[0].replace("void ", "").replace("rtseg::", "")
        print(f"{probe:28s} {short:44s} {dur / 1e3:7.1f} {100 * busy / (1024 * dur * 2.4):6.1f} "
              f"{c.get('SQ_INSTS_VALU', float('nan')) / mfma:9.2f} {c.get('SQ_INSTS_SALU', float('nan')) / mfma:9.2f} "
              f"{100 * c.get('SQ_WAIT_INST_ANY', 0) / max(c.get('SQ_WAVE_CYCLES', 1), 1):10.1f} "
              f"{c.get('SQ_LDS_BANK_CONFLICT', float('nan')):8.0f}")


if __name__ == "__main__":
    main()
