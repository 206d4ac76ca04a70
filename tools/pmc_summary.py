"""Summarise rocprofv3 PMC passes into per-launch HBM traffic of each kernel.

    python tools/pmc_summary.py FETCH_CSV WRITE_CSV OUT_JSON [label]

FETCH_SIZE / WRITE_SIZE are in KiB.  On gfx950 FETCH_SIZE reads exactly half
of the bytes of a wide coalesced streaming read (MI355X_MICROARCH.md §HBM), so
it is doubled; WRITE_SIZE is exact for 16-B stores.  Each counter came from its
own pass (a FETCH_SIZE and a WRITE_SIZE pass do not fit one TCC budget).
"""
import collections
import csv
import json
import sys


def per_kernel(path, counter):
    """Mean counter value per launch over the WORK launches of each kernel: launches
    under 1 % of the kernel's largest count are early exits (the lagged convergence
    poll queues one pass past the stop; it returns at once) and are
    left out of the mean, as the bench's HIP-event timing leaves them out."""
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == counter:
            acc[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    mean, n = {}, {}
    for k, v in acc.items():
        work = [x for x in v if x >= 0.01 * max(v)] or v
        mean[k], n[k] = sum(work) / len(work), len(work)
    return mean, n


def main():
    fetch_csv, write_csv, out = sys.argv[1:4]
    label = sys.argv[4] if len(sys.argv) > 4 else ""
    fetch, n_f = per_kernel(fetch_csv, "FETCH_SIZE")
    write, _ = per_kernel(write_csv, "WRITE_SIZE")
    rows = {}
    for k in sorted(set(fetch) | set(write)):
        rd = fetch.get(k, 0.0) * 1024 * 2      # gfx950: FETCH_SIZE = 1/2 of streamed bytes
        wr = write.get(k, 0.0) * 1024
        rows[k] = {"launches": n_f.get(k, 0), "FETCH_SIZE_KiB": fetch.get(k),
                   "WRITE_SIZE_KiB": write.get(k), "read_bytes_corrected": rd,
                   "write_bytes": wr, "hbm_bytes_per_launch": rd + wr}
    json.dump({"label": label, "correction": "read = FETCH_SIZE*1024*2 (gfx950), "
               "write = WRITE_SIZE*1024", "kernels": rows}, open(out, "w"), indent=1)
    for k, v in rows.items():
        print(f"{v['hbm_bytes_per_launch'] / 1e9:10.3f} GB/launch  {k[:90]}")


if __name__ == "__main__":
    main()
