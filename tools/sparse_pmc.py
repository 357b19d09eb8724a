"""Per-kernel table of a sparse-engine profile round (development aid).

    python tools/sparse_pmc.py gpurun_out/r04g sp1 [solves_in_kt]

Reads <dir>/<tag>_kt (kernel trace of `solves_in_kt` solves, default 3; the first is the
synced solve, the rest replays) and the one-solve PMC passes <tag>_fetch, _write, _tcc,
_sq; prints, per kernel and per solve: ms (replays), FETCH_SIZE GB (raw: random 64-B
accesses, no streaming correction), WRITE_SIZE GB, L2 hit rate, memory-side read and
write requests, waves, mean waves resident (SQ_WAVE_CYCLES / SQ_BUSY_CYCLES), LDS bank
conflict ratio."""
import csv
import glob
import sys
from collections import defaultdict


def short(name):
    n = name.replace("(anonymous namespace)::", "").replace("void ", "").replace("gm::", "")
    if "rocprim" in n:
        return "rocprim " + n.split("wrapped_")[1].split("_config")[0] if "wrapped_" in n else "rocprim"
    return n.split("(")[0].split("<")[0]


def counters(d):
    acc = defaultdict(lambda: defaultdict(float))
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            acc[short(r["Kernel_Name"])][r["Counter_Name"]] += float(r["Counter_Value"])
    return acc


def main():
    d, tag = sys.argv[1], sys.argv[2]
    ns = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    kt = defaultdict(list)
    for f in glob.glob("%s/%s_kt/**/*kernel_trace.csv" % (d, tag), recursive=True):
        for r in csv.DictReader(open(f)):
            kt[short(r["Kernel_Name"])].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]) - int(r["Start_Timestamp"])))
    c = defaultdict(dict)
    for p in ("fetch", "write", "tcc", "sq"):
        for k, v in counters("%s/%s_%s" % (d, tag, p)).items():
            c[k].update(v)
    # replays: the launches after the first solve; a kernel's per-solve share is its
    # total duration over the trace minus the first solve's, divided by (ns - 1)
    starts = sorted(s for v in kt.values() for s, _ in v)
    print("%-28s %8s %8s %8s %6s %8s %8s %9s %6s %6s" % ("kernel", "ms", "fetchGB", "writeGB", "L2hit", "EA_rdG",
                                                        "EA_wrG", "waves", "res", "ldsc"))
    tot = 0.0
    rows = []
    for k, v in kt.items():
        ms = sum(dur for _, dur in v) / 1e6
        rows.append((ms, k))
    for ms_all, k in sorted(rows, reverse=True):
        v = sorted(kt[k])
        n = len(v) // ns if len(v) % ns == 0 else None
        ms = sum(dur for _, dur in v[len(v) - (n or 0) * (ns - 1):]) / 1e6 / (ns - 1) if n else ms_all / ns
        if ms < 0.05:
            continue
        tot += ms
        x = c.get(k, {})
        hit = x.get("TCC_HIT_sum", 0)
        miss = x.get("TCC_MISS_sum", 0)
        res = x["SQ_WAVE_CYCLES"] / x["SQ_BUSY_CYCLES"] if x.get("SQ_BUSY_CYCLES") else 0
        ldsc = x["SQ_LDS_BANK_CONFLICT"] / x["SQ_LDS_IDX_ACTIVE"] if x.get("SQ_LDS_IDX_ACTIVE") else 0
        print("%-28s %8.2f %8.1f %8.1f %6.2f %8.2f %8.2f %9.3g %6.1f %6.3f" % (
            k[:28], ms, x.get("FETCH_SIZE", 0) * 1024 / 1e9, x.get("WRITE_SIZE", 0) * 1024 / 1e9,
            hit / (hit + miss) if hit + miss else 0, x.get("TCC_EA0_RDREQ_sum", 0) / 1e9,
            x.get("TCC_EA0_WRREQ_sum", 0) / 1e9, x.get("SQ_WAVES", 0), res, ldsc))
    print("sum of kernels per replayed solve: %.1f ms" % tot)


if __name__ == "__main__":
    main()
