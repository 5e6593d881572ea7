"""Mean per dispatch of every counter per kernel, from rocprofv3 --pmc csv directories (round-6 helper)."""
import collections
import csv
import glob
import sys

agg = collections.defaultdict(lambda: collections.defaultdict(list))
for d in sys.argv[1:]:
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        per = collections.defaultdict(float)
        for r in csv.DictReader(open(f)):
            per[(r["Kernel_Name"][:48], r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
        for (k, _, c), v in per.items():
            agg[k][c].append(v)
for k, d in sorted(agg.items()):
    if "rocclr" in k:
        continue
    print(k, {c: round(sum(v) / len(v)) for c, v in sorted(d.items())})
