"""Render tools/zoo_train.py JSON lines as a markdown table (README / profiles)."""
import json
import sys


def main(path):
    rows = [json.loads(line) for line in open(path) if line.strip().startswith("{")]
    print("| model | images/s | ms/step | peak GB | aux |")
    print("|---|---|---|---|---|")
    for r in rows:
        if "error" in r:
            print(f"| {r['model']} | error: {r['error'][:60]} | | | |")
        else:
            print(f"| {r['model']} | {r['images_per_s']:.1f} | {r['ms_per_step']:.1f} | {r['peak_mem_gb']:.1f} | "
                  f"{'yes' if r.get('aux') else ''} |")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/zoo_train.jsonl")
