#!/usr/bin/env python3
"""Per-replay kernel times and counters of a sparse-engine profile (development aid).

    python tools/sparse_replay_profile.py gpurun_out/r05g sp [--json profiles/traffic_toot6x4.json]
    python tools/sparse_replay_profile.py gpurun_out/r06p o8 --window front_insert_one_wkernel --skip 1 \
        --json profiles/traffic_othello8_15.json     # Othello 8x8: synced solves, each starting at its root insert

<dir>/<tag>_kt: rocprofv3 --kernel-trace of `tools/solve_timed.py toot 6 4 N` (1 synced solve,
then N - 1 replays).  A replay starts with slot_fill_many_kernel (the one-launch refill of every
tier table, csrc/sparse.hip replay_with), so the replays are the windows between those launches;
the digest kernel that follows the last solve is left out.  Per kernel: mean ms per replay, and
from the one-solve PMC passes <tag>_fetch / _write / _tcc (a synced solve: the same expand,
retro and sort launches) FETCH_SIZE and WRITE_SIZE bytes (raw: random 64-B accesses, no
streaming correction), memory-side read / write requests and the L2 hit rate.  Also each
replay's kernel sum and its window's span (first kernel start to last kernel end).
"""
import argparse
import csv
import glob
import json
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
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("tag")
    ap.add_argument("--json", default=None)
    ap.add_argument("--window", default="slot_fill_many_kernel", help="the kernel that starts each solve's window")
    ap.add_argument("--skip", type=int, default=0, help="windows to leave out first (warm-up solves)")
    a = ap.parse_args()
    rows = []
    for f in glob.glob("%s/%s_kt/**/*kernel_trace.csv" % (a.dir, a.tag), recursive=True):
        for r in csv.DictReader(open(f)):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])))
    rows.sort()
    starts = [s for s, _, k in rows if k == a.window]
    if not starts:
        raise SystemExit("no replay in the trace")
    wins = []
    for i, b in enumerate(starts):
        e = starts[i + 1] if i + 1 < len(starts) else float("inf")
        ks = [(s, t, k) for s, t, k in rows if b <= s < e and k != "res_digest_kernel"]
        wins.append(ks)
    wins = wins[a.skip:]
    per = defaultdict(float)
    sums, spans = [], []
    for ks in wins:
        for s, t, k in ks:
            per[k] += (t - s) / 1e6 / len(wins)
        sums.append(sum(t - s for s, t, _ in ks) / 1e6)
        spans.append((max(t for _, t, _ in ks) - min(s for s, _, _ in ks)) / 1e6)
    c = defaultdict(dict)
    for p in ("fetch", "write", "tcc"):
        for k, v in counters("%s/%s_%s" % (a.dir, a.tag, p)).items():
            c[k].update(v)
    out = {"replays": len(wins), "kernel_sum_ms_per_replay": sums, "span_ms_per_replay": spans, "kernels": {}}
    print("%-28s %8s %9s %9s %7s %9s %9s" % ("kernel", "ms", "fetchGB", "writeGB", "L2hit", "EA_rd_G", "EA_wr_G"))
    for k, ms in sorted(per.items(), key=lambda x: -x[1]):
        x = c.get(k, {})
        hit, miss = x.get("TCC_HIT_sum", 0.0), x.get("TCC_MISS_sum", 0.0)
        rec = {"ms": round(ms, 3), "fetch_bytes": x.get("FETCH_SIZE", 0.0) * 1024,
               "write_bytes": x.get("WRITE_SIZE", 0.0) * 1024,
               "l2_hit": round(hit / (hit + miss), 4) if hit + miss else None,
               "ea_read_req": x.get("TCC_EA0_RDREQ_sum", 0.0), "ea_write_req": x.get("TCC_EA0_WRREQ_sum", 0.0)}
        out["kernels"][k] = rec
        if ms >= 0.05:
            print("%-28s %8.2f %9.1f %9.1f %7.3f %9.3f %9.3f" % (k[:28], ms, rec["fetch_bytes"] / 1e9,
                                                             rec["write_bytes"] / 1e9, rec["l2_hit"] or 0,
                                                             rec["ea_read_req"] / 1e9, rec["ea_write_req"] / 1e9))
    print("per replay: kernel sum %s ms, window span %s ms" % ([round(x, 2) for x in sums],
                                                            [round(x, 2) for x in spans]))
    if a.json:
        json.dump(out, open(a.json, "w"), indent=1)


if __name__ == "__main__":
    main()
