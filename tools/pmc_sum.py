"""Sum rocprofv3 --pmc counter_collection.csv rows per counter for kernels matching a name,
over the last N dispatches (one solve).  python tools/pmc_sum.py DIR NAME [N]"""
import csv
import glob
import sys
from collections import defaultdict

d, name = sys.argv[1], sys.argv[2]
n = int(sys.argv[3]) if len(sys.argv) > 3 else 41
files = glob.glob(d + "/**/*counter_collection.csv", recursive=True)
rows = []
for f in files:
    rows += [r for r in csv.DictReader(open(f)) if name in r.get("Kernel_Name", "")]
disp = sorted({int(r["Dispatch_Id"]) for r in rows})[-n:]
keep = set(disp)
acc = defaultdict(float)
for r in rows:
    if int(r["Dispatch_Id"]) in keep:
        acc[r["Counter_Name"]] += float(r["Counter_Value"])
for k in sorted(acc):
    print("%-28s %.4g" % (k, acc[k]))
