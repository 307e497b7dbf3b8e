"""PMC HBM bytes of one pattern compression (bench.py --workload patterns): the FETCH_SIZE and
WRITE_SIZE passes (separate rocprofv3 --pmc runs) summed over every dispatch of the run and
divided by the number of compressions (k_pack dispatches); bytes = 2 * FETCH_SIZE * 1024 +
WRITE_SIZE * 1024 (MI355X_MICROARCH.md, gfx950).  Also per kernel: k_pack and the unpack.

usage: python scripts/r05/patterns_traffic.py <fetch dir> <write dir> <out json>
"""
import csv
import glob
import json
import os
import sys


def load(root, counter):
    per = {}  # (file, dispatch) -> (kernel, value)
    for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            if row["Counter_Name"] != counter:
                continue
            k = (f, row["Dispatch_Id"])
            name = row.get("Kernel_Name", "")
            v = per.get(k, (name, 0.0))[1] + float(row["Counter_Value"])
            per[k] = (name, v)
    return list(per.values())


def main():
    fetch, write = load(sys.argv[1], "FETCH_SIZE"), load(sys.argv[2], "WRITE_SIZE")
    calls = [sum(1 for n, _ in d if "k_pack" in n) for d in (fetch, write)]
    if not all(calls):
        sys.exit("no k_pack dispatches in the counter files")

    def per_call(d, n, key=None):
        return sum(v for name, v in d if key is None or key in name) / n

    out = {"workload": "bench.py --workload patterns (cfg4 alignment, 1000 taxa x 1M columns)",
           "compressions": calls,
           "fetch_size_kib_per_call": per_call(fetch, calls[0]),
           "write_size_kib_per_call": per_call(write, calls[1]),
           "rule": "bytes = 2*FETCH_SIZE*1024 + WRITE_SIZE*1024 (MI355X_MICROARCH.md HBM)"}
    out["hbm_bytes_per_call"] = (2 * out["fetch_size_kib_per_call"] +
                                 out["write_size_kib_per_call"]) * 1024
    for k in ("k_pack", "k_unpack"):
        out["hbm_bytes_" + k] = (2 * per_call(fetch, calls[0], k) +
                                 per_call(write, calls[1], k)) * 1024
    json.dump(out, open(sys.argv[3], "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
