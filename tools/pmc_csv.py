"""Sum rocprofv3 --pmc counters of one kernel instance over the dispatches of counter_collection CSVs.

Usage: python tools/pmc_csv.py 'render_kernel<256, 7, 2>' file.csv [file.csv ...]
Prints {counter: sum, ..., "dispatches": n, "kernel_ns": summed dispatch durations}."""
import csv
import json
import sys


def main():
    pat, files = sys.argv[1], sys.argv[2:]
    tot, disp, ns = {}, set(), 0
    for f in files:
        with open(f) as fh:
            for r in csv.DictReader(fh):
                if pat not in r["Kernel_Name"]:
                    continue
                tot[r["Counter_Name"]] = tot.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
                key = (f, r["Dispatch_Id"])
                if key not in disp:
                    disp.add(key)
                    ns += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    tot["dispatches"] = len(disp)
    tot["kernel_ns"] = ns
    print(json.dumps(tot, indent=1))


if __name__ == "__main__":
    main()
