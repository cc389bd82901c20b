"""Per-iteration timeline of a lock-step solve from a rocprofv3 --kernel-trace CSV: for the LAST
solve of the trace (the timed step), each batch iteration's kernels (durations) and the gaps
between them.  Usage: python tools/trace_iter.py run_kernel_trace.csv [marker_kernel]"""
import collections
import csv
import sys


def short(name):
    n = name.split("(")[0].replace("void ", "")
    return n.split("<")[0].replace("tmpc::", "")


def main():
    path = sys.argv[1]
    marker = sys.argv[2] if len(sys.argv) > 2 else "k_ls_decide"
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    ks = [(short(r["Kernel_Name"]), int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows]
    # split into solves at k_init_state
    starts = [i for i, k in enumerate(ks) if k[0] == "k_init_state"]
    if not starts:
        starts = [0]
    seg = ks[starts[-1]:]
    # iterations: from one marker to the next
    marks = [i for i, k in enumerate(seg) if k[0] == marker]
    tot = collections.defaultdict(float)
    n = collections.defaultdict(int)
    wall0 = seg[0][1]
    busy = 0
    for name, s, e in seg:
        tot[name] += (e - s) / 1e3
        n[name] += 1
        busy += e - s
    wall = (seg[-1][2] - wall0) / 1e3
    print(f"last solve: {len(seg)} dispatches, wall {wall:.1f} us, kernel busy {busy / 1e3:.1f} us "
          f"({100 * busy / 1e3 / wall:.0f} %), {len(marks)} '{marker}' launches")
    for name in sorted(tot, key=lambda k: -tot[k]):
        print(f"  {name:28s} {n[name]:6d} {tot[name]:12.1f} us  avg {tot[name] / n[name]:9.1f} us")
    # tail profile: iterations bucketed
    if len(marks) > 2:
        per = []
        prev = 0
        for m in marks:
            it = seg[prev:m + 1]
            d = collections.defaultdict(float)
            for name, s, e in it:
                d[name] += (e - s) / 1e3
            span = (it[-1][2] - it[0][1]) / 1e3
            per.append((span, d))
            prev = m + 1
        print("iteration spans (us): first 8", [round(p[0]) for p in per[:8]], " last 8", [round(p[0]) for p in per[-8:]])
        tail = per[len(per) // 2:]
        agg = collections.defaultdict(float)
        for span, d in tail:
            for k, v in d.items():
                agg[k] += v
        tspan = sum(p[0] for p in tail)
        print(f"second half of the iterations: {len(tail)} iterations, {tspan:.0f} us span, per iteration "
              f"{tspan / len(tail):.1f} us:")
        for k in sorted(agg, key=lambda k: -agg[k]):
            print(f"    {k:28s} {agg[k] / len(tail):9.1f} us per iteration")


if __name__ == "__main__":
    main()
