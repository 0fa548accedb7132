"""Per-kernel sums of rocprofv3 --pmc counter CSVs: python tools/pmc_dump.py DIR [DIR ...] [--match S]"""
import collections
import csv
import glob
import sys

args = [a for a in sys.argv[1:] if not a.startswith("--")]
match = sys.argv[sys.argv.index("--match") + 1] if "--match" in sys.argv else ""
d = collections.defaultdict(lambda: collections.defaultdict(float))
for a in args:
    for f in glob.glob(a + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if match and match not in r["Kernel_Name"]:
                continue
            d[r["Kernel_Name"][:60] + "|" + r["Grid_Size"]][r["Counter_Name"]] += float(r["Counter_Value"])
for k, v in d.items():
    print(k)
    print("   ", " ".join(f"{a}={b:.3e}" for a, b in sorted(v.items())))
