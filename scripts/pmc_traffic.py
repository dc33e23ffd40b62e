"""Per-launch HBM traffic of the wgrad kernels from rocprofv3 --pmc passes (separate passes for
FETCH_SIZE and WRITE_SIZE: they do not fit one pass on gfx950).

Correction (MI355X_MICROARCH.md §HBM): FETCH_SIZE reports 1/2 of the bytes of a wide coalesced
streaming read (16 B/lane) on gfx950 -> x2; WRITE_SIZE is exact for 16-B streaming stores. Both are
in KiB. Usage:
    python scripts/pmc_traffic.py FETCH_counter_collection.csv WRITE_counter_collection.csv out.json
"""
import collections
import csv
import json
import sys


def per_dispatch(path, counter):
    vals = collections.defaultdict(float)
    names = {}
    for r in csv.DictReader(open(path)):
        if r.get("Counter_Name") != counter:
            continue
        d = int(r["Dispatch_Id"])
        vals[d] += float(r["Counter_Value"])
        names[d] = r["Kernel_Name"]
    return vals, names


def main(fetch_csv, write_csv, out_json):
    f, fn = per_dispatch(fetch_csv, "FETCH_SIZE")
    w, wn = per_dispatch(write_csv, "WRITE_SIZE")
    # one smt_tile_wgrad call = one main kernel (wgrad_dma / wgrad_quarter) + a wgrad_reduce when split
    main_k = lambda n: ("wgrad_dma" in n or "wgrad_quarter" in n or "wgrad_partial" in n or "wgrad_mx_kernel" in n
                        or "wgrad_mx_quarter" in n)
    every = lambda names: [d for d, n in names.items() if "wgrad_" in n]
    calls = lambda names: max(1, sum(1 for n in names.values() if main_k(n)))
    fetch_kib = sum(f[d] for d in every(fn)) / calls(fn)
    write_kib = sum(w[d] for d in every(wn)) / calls(wn)
    res = {"kernel": "smt_tile_wgrad (wgrad_dma_kernel | wgrad_quarter_kernel, + wgrad_reduce_kernel when split)",
           "launches_fetch_pass": calls(fn), "launches_write_pass": calls(wn),
           "fetch_kib_per_call_raw": fetch_kib, "write_kib_per_call": write_kib,
           "hbm_bytes_per_call": (2.0 * fetch_kib + write_kib) * 1024.0,
           "correction": "FETCH_SIZE x2 (gfx950 half-count on 16-B streaming reads), WRITE_SIZE x1; KiB -> B"}
    json.dump(res, open(out_json, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main(*sys.argv[1:4])
