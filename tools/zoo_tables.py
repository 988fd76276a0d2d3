"""Markdown tables of a zoo sweep (tools/gpu_zoo_sweep.sh): training throughput and inference FPS.

  python tools/zoo_tables.py --train 'gpurun_out/zoo/train_*.jsonl' --fps 'gpurun_out/zoo/fps_*.jsonl'

The LAST record of a model wins (a chunk re-run after a fix supersedes the earlier one); records
with an ``error`` are listed as such.  Training rows: eager and, where measured, ``--graph-step``.
"""
import argparse
import glob
import json


def _records(pattern):
    out = []
    for p in sorted(glob.glob(pattern), key=lambda q: (len(q), q)):
        for line in open(p):
            line = line.strip()
            if line.startswith("{"):
                out.append(json.loads(line))
    return out


def train_table(recs):
    eager, graph = {}, {}
    for r in recs:
        (graph if r.get("graph_step") else eager)[r["model"]] = r
    rows = ["| model | bf16 images/s | ms/step | peak GB | graph-step images/s | aux |", "|---|---|---|---|---|---|"]
    for m in sorted(set(eager) | set(graph)):
        e, g = eager.get(m, {}), graph.get(m, {})
        if "error" in e:
            rows.append(f"| {m} | error: {e['error'][:60]} | | | | |")
            continue
        gs = f"{g['images_per_s']:.1f}" if g and "images_per_s" in g else ""
        rows.append(f"| {m} | {e.get('images_per_s', '')} | {e.get('ms_per_step', '')} | {e.get('peak_mem_gb', '')} "
                    f"| {gs} | {'yes' if e.get('aux') else ''} |")
    return "\n".join(rows)


def fps_table(recs):
    last = {}
    for r in recs:
        last[r["model"]] = r
    rows = ["| Model | RTX 2080 FPS (ref README) | MI355X fp32 FPS | x | MI355X bf16 FPS | x |",
            "|---|---|---|---|---|---|"]
    for m in sorted(last, key=str.lower):
        r = last[m]
        if "error" in r:
            rows.append(f"| {m} | {r['ref_fps_rtx2080']} | error | | | |")
            continue
        rows.append(f"| {m} | {r['ref_fps_rtx2080']} | {r['fps_fp32']:.0f} | {r['x_fp32']:.2f} "
                    f"| {r['fps_bf16']:.0f} | {r['x_bf16']:.2f} |")
    return "\n".join(rows)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--train", default="gpurun_out/zoo/train_*.jsonl")
    ap.add_argument("--fps", default="gpurun_out/zoo/fps_*.jsonl")
    a = ap.parse_args()
    tr, fp = _records(a.train), _records(a.fps)
    if tr:
        print(f"## Training ({len({r['model'] for r in tr})} models)\n")
        print(train_table(tr) + "\n")
    if fp:
        print(f"## Inference FPS ({len({r['model'] for r in fp})} rows)\n")
        print(fps_table(fp))


if __name__ == "__main__":
    main()
