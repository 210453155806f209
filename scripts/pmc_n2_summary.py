"""Per-launch HBM bytes of the main library kernel in scripts/pmc_n2.sh outputs (gpurun_out/pmc2/<mode>_<counter>/):
median over dispatches of the summed FETCH_SIZE (x2, 16-byte streaming reads, MI355X_MICROARCH.md HBM section) plus
WRITE_SIZE, in KiB x 1024, and the ratio to S = 256 MiB. usage: pmc_n2_summary.py TAG [TAG ...] (TAG = the mode, or
<mode>_n<N> for NRANKS=N runs)"""
import csv
import json
import statistics as st
import sys

S = 256 << 20


def summarize(mode, root="gpurun_out/pmc2"):
    vals = {}
    for c in ("FETCH_SIZE", "WRITE_SIZE"):
        per, names = {}, {}
        for row in csv.DictReader(open(f"{root}/{mode}_{c}/run_counter_collection.csv")):
            k = row["Kernel_Name"]
            if "ncclamd" not in k or "mapCheck" in k:
                continue
            d = int(row["Dispatch_Id"])
            per[d] = per.get(d, 0.0) + float(row["Counter_Value"])
            names[d] = k
        main = max(set(names.values()), key=lambda k: sum(1 for v in names.values() if v == k))
        xs = [v for d, v in per.items() if names[d] == main]
        vals[c] = (st.median(xs), len(xs), main.split("(")[0])
    total = vals["FETCH_SIZE"][0] * 1024 * 2 + vals["WRITE_SIZE"][0] * 1024
    return {"kernel": vals["FETCH_SIZE"][2], "dispatches": vals["FETCH_SIZE"][1],
            "fetch_size_kb_median": vals["FETCH_SIZE"][0], "write_size_kb_median": vals["WRITE_SIZE"][0],
            "bytes_per_launch": int(total), "over_S": round(total / S, 4)}


if __name__ == "__main__":
    print(json.dumps({m: summarize(m) for m in sys.argv[1:]}, indent=1))
