"""Turn rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE) of a bench run into per-launch HBM bytes.

    python scripts/collect_traffic.py <fetch_dir> <write_dir> [--kernel "graph_row_kernel<true, 1, 2, 4>"]
                                      [--out profiles/traffic_system_step.json]

Corrections (MI355X_MICROARCH.md §HBM, cdna_hip_programming.md §7): on gfx950 FETCH_SIZE
counts half the bytes of a coalesced streaming read (TCC_EA0_RDREQ x 64 B for 128-B
requests), so reads are doubled; WRITE_SIZE is taken as is.  Both are KiB per dispatch.
"""
import argparse
import csv
import glob
import json
import os


def per_dispatch(d, counter, kernel):
    vals = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter or kernel not in r["Kernel_Name"]:
                continue
            vals[r["Dispatch_Id"]] = vals.get(r["Dispatch_Id"], 0.0) + float(r["Counter_Value"])
    return list(vals.values())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_dir")
    ap.add_argument("write_dir")
    ap.add_argument("--kernel", default="graph_row_kernel<true, 1, 2, 4>")
    ap.add_argument("--out", default="profiles/traffic_system_step.json")
    ap.add_argument("--batch", type=int, default=None, help="workload batch recorded in the summary")
    ap.add_argument("--size", type=int, default=None, help="workload image side recorded in the summary")
    args = ap.parse_args()
    fetch = per_dispatch(args.fetch_dir, "FETCH_SIZE", args.kernel)
    write = per_dispatch(args.write_dir, "WRITE_SIZE", args.kernel)
    if not fetch or not write:
        raise SystemExit("no matching dispatches")
    rd = 2.0 * 1024.0 * sum(fetch) / len(fetch)
    wr = 1024.0 * sum(write) / len(write)
    res = {"kernel": args.kernel, "dispatches": len(fetch),
           "fetch_size_kib_mean": sum(fetch) / len(fetch), "write_size_kib_mean": sum(write) / len(write),
           "read_bytes_per_launch": rd, "write_bytes_per_launch": wr, "hbm_bytes_per_launch": rd + wr,
           "correction": "reads = 2 x FETCH_SIZE (gfx950 half-count of 128-B requests); writes = WRITE_SIZE"}
    if args.batch is not None:
        res["workload"] = {"batch": args.batch, "size": args.size}
    os.makedirs(os.path.dirname(args.out) or ".", exist_ok=True)
    with open(args.out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
