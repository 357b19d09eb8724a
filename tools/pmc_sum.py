"""Sum a rocprofv3 counter over the dispatches of one kernel (development aid).
    python tools/pmc_sum.py DIR KERNEL_SUBSTRING [solves]"""
import csv, sys, glob, os
d, k = sys.argv[1], sys.argv[2]
solves = int(sys.argv[3]) if len(sys.argv) > 3 else 1
f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)[0]
tot = {}
for r in csv.DictReader(open(f)):
    if k in r["Kernel_Name"]:
        tot[r["Counter_Name"]] = tot.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
for n, v in tot.items():
    print("%s per solve: %.4g" % (n, v / solves))
