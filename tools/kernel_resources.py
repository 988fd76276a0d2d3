"""Per-kernel register / spill / LDS report of a HIP source (hipcc -Rpass-analysis).
usage: python tools/kernel_resources.py csrc/kernels/conv_igemm.hip [name-filter]"""
import os
import re
import subprocess
import sys


def main():
    src = sys.argv[1]
    filt = sys.argv[2] if len(sys.argv) > 2 else ""
    inc = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(src))), "include")
    out = subprocess.run(["hipcc", "--offload-arch=gfx950", "-O3", "-std=c++20", "-I" + inc, "-c", src, "-o",
                          "/tmp/_kr.o", "-Rpass-analysis=kernel-resource-usage"], capture_output=True, text=True)
    if out.returncode:
        sys.exit(out.stderr[-3000:])
    cur, rows = None, []
    for line in out.stderr.splitlines():
        m = re.search(r"remark: (Function Name|\s+[\w /\[\]]+): (.*?) \[-Rpass", line)
        if not m:
            continue
        k, v = m.group(1).strip(), m.group(2).strip()
        if k == "Function Name":
            cur = {"name": v}
            rows.append(cur)
        elif cur is not None:
            cur[k] = v
    for r in rows:
        if filt in r["name"]:
            print(f"{r.get('VGPRs', '?'):>4} v {r.get('AGPRs', '?'):>3} a  spill s{r.get('SGPRs Spill', '?'):>3} "
                  f"v{r.get('VGPRs Spill', '?'):>3} scratch {r.get('ScratchSize [bytes/lane]', '?'):>4}  occ {r.get('Occupancy [waves/SIMD]', '?')}  "
                  f"lds {r.get('LDS Size [bytes/block]', '?'):>6}  {r['name'][:110]}")


if __name__ == "__main__":
    main()
