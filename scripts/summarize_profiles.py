"""Per-(kernel, grid) summary of rocprofv3 CSVs: kernel-trace durations and PMC FETCH_SIZE / WRITE_SIZE.

usage: summarize_profiles.py OUT.csv --trace run_kernel_trace.csv [--fetch run_counter_collection.csv]
                             [--write run_counter_collection.csv] [--match SUBSTRING] [--algbytes BYTES]
Grid = workgroups (grid size / workgroup size), i.e. the channel count of a collective launch. HBM bytes per
launch follow MI355X_MICROARCH.md §HBM: FETCH_SIZE (KiB) x 2 (gfx950 reports half of a wide streaming read)
x 1024 + WRITE_SIZE (KiB) x 1024. TCC counters are device-wide, so with several ranks on one GPU a pass
sees every rank's traffic during the profiled rank's dispatch."""
import argparse
import collections
import csv
import statistics


def rows(path):
    with open(path, newline="") as f:
        return list(csv.DictReader(f))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("out")
    ap.add_argument("--trace", required=True)
    ap.add_argument("--fetch")
    ap.add_argument("--write")
    ap.add_argument("--match", default="ncclamd")
    ap.add_argument("--algbytes", type=float, default=0.0, help="algorithmic bytes per launch (for the ratio)")
    a = ap.parse_args()
    dur = collections.defaultdict(list)
    for r in rows(a.trace):
        if a.match not in r["Kernel_Name"]:
            continue
        grid = int(r["Grid_Size_X"]) // int(r["Workgroup_Size_X"])
        dur[(r["Kernel_Name"], grid)].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    pmc = {}
    for name, path in (("FETCH_SIZE", a.fetch), ("WRITE_SIZE", a.write)):
        if not path:
            continue
        acc = collections.defaultdict(list)
        for r in rows(path):
            if a.match not in r["Kernel_Name"] or r["Counter_Name"] != name:
                continue
            grid = int(r["Grid_Size"]) // int(r["Workgroup_Size"])
            acc[(r["Kernel_Name"], grid)].append(float(r["Counter_Value"]))
        pmc[name] = {k: statistics.median(v) for k, v in acc.items()}
    with open(a.out, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["kernel", "workgroups", "launches", "avg_us", "median_us", "min_us", "max_us",
                    "fetch_kib_median", "write_kib_median", "hbm_bytes_per_launch", "hbm_over_algorithmic"])
        for (k, g), v in sorted(dur.items(), key=lambda kv: (kv[0][0], -kv[0][1])):
            fe = pmc.get("FETCH_SIZE", {}).get((k, g))
            wr = pmc.get("WRITE_SIZE", {}).get((k, g))
            hbm = (fe * 2 + wr) * 1024 if fe is not None and wr is not None else None
            w.writerow([k, g, len(v), round(statistics.mean(v), 2), round(statistics.median(v), 2), round(min(v), 2),
                        round(max(v), 2), fe, wr, int(hbm) if hbm else "",
                        round(hbm / a.algbytes, 4) if hbm and a.algbytes else ""])
    print(open(a.out).read())


if __name__ == "__main__":
    main()
