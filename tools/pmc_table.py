"""Per-kernel mean of every counter in a rocprofv3 --pmc output directory (counter_collection.csv).

  python tools/pmc_table.py DIR [kernel-substring ...]
"""
import collections
import csv
import glob
import os
import sys


def main():
    d = sys.argv[1]
    want = sys.argv[2:]
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"].split("(")[0].replace("void ", "").strip()
            if want and not any(w in name for w in want):
                continue
            acc[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for name, cs in sorted(acc.items()):
        print(name)
        for c, v in sorted(cs.items()):
            print("   %-24s %16.0f  (n=%d)" % (c, sum(v) / len(v), len(v)))


if __name__ == "__main__":
    main()
