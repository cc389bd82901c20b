"""Per-kernel launch statistics from a rocprofv3 --kernel-trace CSV (run_kernel_trace.csv), split by grid size,
so that a bench line's HIP-event average for its dominant kernel can be checked against the trace's launches
of the same shape (the timed region's launches all carry the full batch).
Usage: python tools/trace_summary.py TRACE.csv OUT.json [KERNEL_PREFIX ...]"""
import collections
import csv
import json
import sys


def main():
    path, out, prefixes = sys.argv[1], sys.argv[2], sys.argv[3:]
    rows = csv.DictReader(open(path))
    cols = rows.fieldnames
    gx = next((c for c in cols if c.lower().startswith("grid_size")), None)
    stat = collections.defaultdict(lambda: [0, 0.0])
    for r in rows:
        name = r["Kernel_Name"]
        if prefixes and not any(name.startswith(p) or name.split("(")[0].endswith(p) or p in name for p in prefixes):
            continue
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
        key = (name.split("(")[0], r.get(gx, "") if gx else "")
        stat[key][0] += 1
        stat[key][1] += d
    res = [dict(kernel=k[0], grid=k[1], launches=v[0], avg_ms=v[1] / v[0], total_ms=v[1])
           for k, v in sorted(stat.items(), key=lambda kv: -kv[1][1])]
    json.dump(dict(source=path, grid_column=gx, kernels=res), open(out, "w"), indent=1)
    for e in res[:20]:
        print(f"{e['kernel'][:70]:70s} grid {e['grid']:>9s} {e['launches']:6d} x {e['avg_ms']:.4f} ms")


if __name__ == "__main__":
    main()
