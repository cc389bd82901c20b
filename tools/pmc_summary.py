"""Summarise rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes into HBM bytes per
launch for each kernel (written to profiles/).

gfx950 correction (MI355X_MICROARCH.md, HBM section): FETCH_SIZE counts
TCC_EA0_RDREQ x 64 B and reports exactly half the bytes of a wide coalesced
streaming read, so it is doubled; WRITE_SIZE is taken as is.  Both are in KiB.
Usage: python tools/pmc_summary.py FETCH_DIR WRITE_DIR OUT.json [SOURCE]
OUT.json for bench.py: profiles/pmc/<workload key>.json (bench.py workload_key); SOURCE names the run.
"""
import collections
import csv
import json
import os
import sys


def per_kernel(path, counter):
    tot = collections.defaultdict(float)
    disp = collections.defaultdict(set)
    for r in csv.DictReader(open(os.path.join(path, "run_counter_collection.csv"))):
        if r["Counter_Name"] != counter:
            continue
        k = r["Kernel_Name"].split("(")[0]
        tot[k] += float(r["Counter_Value"])
        disp[k].add(r["Dispatch_Id"])
    return {k: (tot[k] / len(disp[k]), len(disp[k])) for k in tot}


def main():
    fdir, wdir, out = sys.argv[1:4]
    source = sys.argv[4] if len(sys.argv) > 4 else f"{fdir}, {wdir}"
    f = per_kernel(fdir, "FETCH_SIZE")
    w = per_kernel(wdir, "WRITE_SIZE")
    res = {}
    for k in sorted(set(f) | set(w)):
        fk, nf = f.get(k, (0.0, 0))
        wk, nw = w.get(k, (0.0, 0))
        res[k] = {"dispatches": max(nf, nw), "fetch_size_kib_raw": fk, "write_size_kib": wk,
                  "hbm_bytes_per_launch": 2.0 * fk * 1024 + wk * 1024}
    json.dump({"correction": "bytes = 2 x FETCH_SIZE + WRITE_SIZE (KiB -> B); gfx950 FETCH_SIZE halving",
               "source": source, "kernels": res}, open(out, "w"), indent=1)
    for k, v in res.items():
        print(f"{k[:50]:50s} {v['dispatches']:4d} {v['hbm_bytes_per_launch'] / 1e6:10.2f} MB/launch")


if __name__ == "__main__":
    main()
