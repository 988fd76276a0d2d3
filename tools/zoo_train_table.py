"""Render tools/zoo_train.py JSON lines as a markdown table (README / profiles).

  python tools/zoo_train_table.py bf16_*.jsonl [--fp32 fp32_*.jsonl ...]

One row per model: bf16 images/s, ms/step, peak memory, and the fp32 images/s when an fp32 sweep
is given (records without a ``dtype`` field are fp32: round 2's sweep predates the field)."""
import json
import sys


def load(paths, default_dtype):
    out = {}
    for p in paths:
        for line in open(p):
            if line.strip().startswith("{"):
                r = json.loads(line)
                out[(r["model"], r.get("dtype", default_dtype))] = r
    return out


def main(argv):
    bf, fp, cur = [], [], None
    for a in argv:
        if a == "--fp32":
            cur = fp
        else:
            (cur if cur is not None else bf).append(a)
    recs = load(bf, "bf16")
    recs.update(load(fp, "fp32"))
    models = sorted({m for m, _ in recs})
    print("| model | bf16 images/s | bf16 ms/step | peak GB | fp32 images/s | aux |")
    print("|---|---|---|---|---|---|")
    for m in models:
        b, f = recs.get((m, "bf16")), recs.get((m, "fp32"))
        cells = []
        if b is None:
            cells += ["", "", ""]
        elif "error" in b:
            cells += [f"error: {b['error'][:60]}", "", ""]
        else:
            cells += [f"{b['images_per_s']:.1f}", f"{b['ms_per_step']:.1f}", f"{b['peak_mem_gb']:.1f}"]
        cells.append("" if f is None or "error" in f else f"{f['images_per_s']:.1f}")
        aux = (b or f or {}).get("aux")
        print(f"| {m} | " + " | ".join(cells) + f" | {'yes' if aux else ''} |")


if __name__ == "__main__":
    main(sys.argv[1:])
