#!/usr/bin/env python3
"""Per-rank GPU time of the split box solve (8-heap game, root 0xFFFFFFFF) on ONE GPU, and the
multi-GPU time the op-list schedule gives with it (csrc/dist_box.hip).

    python tools/box_split_time.py [--ranks 2 4 8] [--reps 5] [--batch 4] [--split 0] [--sym 1]

For each G: one full loopback solve (digest checked against the committed oracle digest),
then every rank's op list alone (GM_OPT_DIST_SOLO: its cross-rank waits dropped, the others'
messages of the full solve standing in) with GM_OPT_TIMING, median over reps of each op's GPU
ms.  The multi-GPU estimate replays the op lists as a DAG: a rank's compute stream runs its
ops in order with the measured durations (the tier kernel writes the halo messages itself), an
exchange stream per axis waits for the tier that completes a message, and a message costs
--lat-us plus bytes over --link-gbs (one xGMI link per rank pair) from then to the receiver's
receive (the loopback device copy it replaces is not counted).  Prints one JSON line per G.
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BOP_TIER_, BOP_UNPACK_ = 0, 2
sys.path.insert(0, REPO)
os.environ.setdefault("GPU_MAX_HW_QUEUES", "8")   # as bench.py: a hardware queue per stream


def dag(ops_by_rank, ms_by_rank, bytes_of, lat_us, link_gbs, waits=None):
    """Critical path (ms) of every rank's op list: streams in order, events, sends -> receives.
    waits (a list, one float per rank): the time each rank's compute stream sat idle waiting
    for a message."""
    BOP_TIER, BOP_PACK, BOP_UNPACK, BOP_SEND, BOP_RECV, BOP_RECORD, BOP_WAIT = range(7)
    G = len(ops_by_rank)
    ev = {}          # (rank, kind, axis, batch) -> time recorded
    sent = {}        # (axis, batch, lower) -> time the message has arrived at the receiver
    link = {}        # (lower, axis) -> time the link is free
    end = [0.0] * G
    pc = [0] * G
    free = [dict() for _ in range(G)]   # stream -> time free
    progress = True
    while progress:
        progress = False
        for r in range(G):
            ops, ms = ops_by_rank[r], ms_by_rank[r]
            while pc[r] < len(ops):
                kind, axis, e, on_x, arg, peer = [int(x) for x in ops[pc[r]]]
                st = ("X", axis) if on_x else "S"
                t0 = free[r].get(st, 0.0)
                if kind == BOP_WAIT:
                    k = (peer, e, axis, arg)
                    if k not in ev:
                        break
                    free[r][st] = max(t0, ev[k])
                elif kind == BOP_RECORD:
                    ev[(r, e, axis, arg)] = t0
                    if e == 1:   # BEV_PACKED on X[axis]: the message is complete and leaves
                        nb = bytes_of(r, axis, arg)
                        go = max(t0, link.get((r, axis), 0.0))    # one message at a time per link
                        link[(r, axis)] = go + nb / (link_gbs * 1e6)
                        sent[(axis, arg, r)] = link[(r, axis)] + lat_us / 1000.0
                elif kind == BOP_SEND and not on_x:
                    # direct (loopback) lists: the tier wrote the boxes; the signal leaves from S
                    t1 = t0 + ms[pc[r]]
                    free[r][st] = t1
                    nb = bytes_of(r, axis, arg)
                    go = max(t1, link.get((r, axis), 0.0))
                    link[(r, axis)] = go + nb / (link_gbs * 1e6)
                    sent[(axis, arg, r)] = link[(r, axis)] + lat_us / 1000.0
                elif kind == BOP_RECV:
                    k = (axis, arg, peer)
                    if k not in sent:
                        break
                    if waits is not None:
                        waits[r] += max(0.0, sent[k] - t0)
                    free[r][st] = max(t0, sent[k])
                else:
                    free[r][st] = t0 + ms[pc[r]]
                pc[r] += 1
                progress = True
            end[r] = max(free[r].values()) if free[r] else 0.0
    if any(pc[r] < len(ops_by_rank[r]) for r in range(G)):
        raise RuntimeError("schedule replay stuck")
    return end


def flow_main(a):
    """The split dataflow: every rank's chain is one launch, cross-rank waits are per box.  Per
    G: the loopback solve with all ranks in ONE launch (workgroup w runs rank w % G, so at G = 8
    each rank runs on one XCD: G ranks on 1/G of the chip each, with the real box-level waits
    between them) and each rank's solo launch on the whole chip with its received boxes
    marked stored (its own critical path).  Printed per G: the concurrent time over the one-GPU
    time (the stagger and wait overhead of the split, at equal total compute), the slowest
    solo span, and their product -- the multi-GPU estimate that applies the measured
    overhead to a rank running alone on its own GPU."""
    import numpy as np
    import torch
    from gamesmanmpi_amd import Context, _lib
    ref = json.load(open(os.path.join(REPO, "tests", "golden", "oracle_digests.json")))["subtract_8"]
    stream = torch.cuda.Stream()

    def timed(ctx, reps):
        t = []
        for _ in range(reps + 1):
            ctx.solve(0xFFFFFFFF)
            t.append(ctx.stats()["kernel_ms"])
        return float(np.median(t[1:]))
    one = Context(_lib.GAME_SUBTRACT, (8,), device=0)
    one.set_stream(stream.cuda_stream)
    one.set_option(_lib.OPT_TIMING, 1)
    base = timed(one, a.reps)
    one.close()
    print(json.dumps({"ranks": 1, "ms": round(base, 4)}), flush=True)
    for G in a.ranks:
        ctx = Context(_lib.GAME_SUBTRACT, (8,), device=0)
        ctx.set_stream(stream.cuda_stream)
        for k, v in ((_lib.OPT_VIRTUAL_RANKS, G), (_lib.OPT_BOX_FLOW, 1), (_lib.OPT_DIST_SYMMETRY, a.sym),
                     (_lib.OPT_TIMING, 1)):
            ctx.set_option(k, v)
        conc = timed(ctx, a.reps)
        ok = ctx.digest() == (ref["digest"], 1 << 32)
        spans = []
        for r in range(G):
            ctx.set_option(_lib.OPT_DIST_SOLO, r + 1)
            sp = []
            for _ in range(a.reps + 1):
                ctx.solve(0xFFFFFFFF)
                sp.append(ctx.rank_stats()[r]["kernel_ms"])
            spans.append(float(np.median(sp[1:])))
        ctx.set_option(_lib.OPT_DIST_SOLO, 0)
        over = conc / base
        est = max(spans) * over
        print(json.dumps({"ranks": G, "flow": True, "digest_ok": ok, "concurrent_loopback_ms": round(conc, 4),
                          "overhead_vs_one_gpu": round(over, 3), "solo_span_ms": [round(x, 4) for x in spans],
                          "estimate_ms": round(est, 4), "estimate_speedup": round(base / est, 3),
                          "ideal_speedup_from_solo": round(base / max(spans), 3)}), flush=True)
        ctx.close()
        torch.cuda.empty_cache()
    return 0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ranks", type=int, nargs="+", default=[2, 4, 8])
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--batch", type=int, default=2)
    ap.add_argument("--split", type=int, default=0)
    ap.add_argument("--sym", type=int, default=1)
    ap.add_argument("--lat-us", type=float, default=15.0)
    ap.add_argument("--link-gbs", type=float, default=64.0)
    ap.add_argument("--dump", default=None, help="directory for per-G JSON dumps of the op lists and op times")
    ap.add_argument("--no-graph", action="store_true",
                    help="GM_OPT_GRAPH 0: the split solves' launches eager instead of one captured graph")
    ap.add_argument("--flow", action="store_true",
                    help="the split dataflow (GM_OPT_BOX_FLOW 1): per-rank solo spans and the concurrent loopback")
    a = ap.parse_args()
    if a.flow:
        return flow_main(a)
    import numpy as np
    import torch
    from gamesmanmpi_amd import Context, _lib
    ref = json.load(open(os.path.join(REPO, "tests", "golden", "oracle_digests.json")))["subtract_8"]
    stream = torch.cuda.Stream()
    one = Context(_lib.GAME_SUBTRACT, (8,), device=0)
    one.set_stream(stream.cuda_stream)
    one.set_option(_lib.OPT_TIMING, 1)
    t1 = []
    for _ in range(a.reps + 1):
        one.solve(0xFFFFFFFF)
        t1.append(one.stats()["kernel_ms"])
    base = float(np.median(t1[1:]))
    one.close()
    print(json.dumps({"ranks": 1, "ms": round(base, 4)}), flush=True)
    for G in a.ranks:
        ctx = Context(_lib.GAME_SUBTRACT, (8,), device=0)
        ctx.set_stream(stream.cuda_stream)
        for k, v in ((_lib.OPT_VIRTUAL_RANKS, G), (_lib.OPT_DIST_BATCH, a.batch), (_lib.OPT_BOX_SPLIT, a.split),
                     (_lib.OPT_DIST_SYMMETRY, a.sym), (_lib.OPT_TIMING, 1), (_lib.OPT_GRAPH, 0 if a.no_graph else 1)):
            ctx.set_option(k, v)
        ctx.solve(0xFFFFFFFF)
        ok = ctx.digest() == (ref["digest"], 1 << 32)
        loop_ms = ctx.stats()["kernel_ms"]
        sent = ctx.stats()["exchanged_bytes"]
        ops, ms, spans = [], [], []
        kw = dict(batch=a.batch, split=a.split, symmetry=a.sym, loopback=1)
        for r in range(G):
            ops.append(_lib.box_plan(G, r, _lib.BOXPLAN_OPS, **kw).reshape(-1, 6))
            ctx.set_option(_lib.OPT_DIST_SOLO, r + 1)   # queued whole behind a hold: no host gaps
            reps, sp = [], []
            for _ in range(a.reps + 1):
                ctx.set_option(_lib.OPT_TIMING, 2)      # per op (an event pair around each)
                ctx.solve(0xFFFFFFFF)
                reps.append(ctx.rank_op_ms(r))
                ctx.set_option(_lib.OPT_TIMING, 1)      # the span without per-op events
                ctx.solve(0xFFFFFFFF)
                sp.append(ctx.rank_stats()[r]["kernel_ms"])
            ms.append(np.median(np.array(reps[1:]), axis=0))
            spans.append(float(np.median(sp[1:])))
        ctx.set_option(_lib.OPT_DIST_SOLO, 0)
        offs = {}

        def bytes_of(r, axis, j):
            if (r, axis) not in offs:
                off = _lib.box_plan(G, r, _lib.BOXPLAN_SEND_OFF, axis=axis, **kw).astype(np.int64)
                ent = _lib.box_plan(G, r, _lib.BOXPLAN_SEND, axis=axis, **kw).astype(np.int64)
                offs[(r, axis)] = (off, np.where((ent >> 20) != 0, 2048, 4096))
            off, by = offs[(r, axis)]
            return int(by[off[j]:off[j + 1]].sum())
        waits = [0.0] * G
        end = dag(ops, ms, bytes_of, a.lat_us, a.link_gbs, waits)
        end0 = dag(ops, ms, bytes_of, 0.0, 1e9)
        # the DAG with the tier (and unpack) launches scaled so they sum to the rank's solo span --
        # the gaps between launches and the signal / event costs spread over them -- and the
        # other ops at zero: their per-op event pairs (GM_OPT_TIMING 2) time mostly themselves
        scaled = []
        for m, o, sp in zip(ms, ops, spans):
            mc = np.where(np.isin(o[:, 0], [BOP_TIER_, BOP_UNPACK_]), m, 0.0)
            scaled.append(mc * (sp / max(1e-9, float(mc.sum()))))
        end_s = dag(ops, scaled, bytes_of, a.lat_us, a.link_gbs)
        names = ["tier", "pack", "unpack", "send", "recv", "record", "wait"]   # pack: fused into tier
        worst = int(np.argmax(spans))
        by_kind = {names[k]: round(float(ms[worst][ops[worst][:, 0] == k].sum()), 4) for k in range(5)}
        counts = {names[k]: int((ops[worst][:, 0] == k).sum()) for k in range(7)}
        line = {"ranks": G, "batch": a.batch, "split": a.split, "sym": a.sym, "graph": not a.no_graph, "digest_ok": ok,
                "slowest_rank": worst, "slowest_ms_by_op_kind": by_kind, "slowest_op_counts": counts,
                "solo_span_ms": [round(x, 4) for x in spans],
                "modelled_ms_scaled_to_spans": round(max(end_s), 4),
                "modelled_speedup_scaled": round(base / max(end_s), 3),
                "tier_ms_sum": [round(float(m[o[:, 0] == 0].sum()), 4) for m, o in zip(ms, ops)],
                "modelled_ms": round(max(end), 4), "modelled_speedup": round(base / max(end), 3),
                "modelled_end_ms_by_rank": [round(x, 4) for x in end],
                "modelled_message_wait_ms_by_rank": [round(x, 4) for x in waits],
                "modelled_ms_free_links": round(max(end0), 4),
                "link_model": {"lat_us": a.lat_us, "gbs": a.link_gbs},
                "loopback_all_ranks_one_gpu_ms": round(loop_ms, 4), "halo_bytes_per_solve": sent}
        print(json.dumps(line), flush=True)
        if a.dump:   # the op lists and per-op ms, for replaying schedule variants offline
            os.makedirs(a.dump, exist_ok=True)
            with open(os.path.join(a.dump, "split_ops_G%d_B%d_s%d.json" % (G, a.batch, a.split)), "w") as f:
                json.dump({"G": G, "batch": a.batch, "split": a.split, "base_ms": base, "spans": spans,
                           "ops": [o.tolist() for o in ops], "ms": [m.tolist() for m in ms],
                           "send_bytes": {"%d,%d,%d" % (r, ax, j): bytes_of(r, ax, j) for r in range(G)
                                          for ax in range(3) for j in range(len(_lib.box_plan(G, r,
                                          _lib.BOXPLAN_SEND_OFF, axis=ax, **kw)) - 1)}}, f)
        ctx.close()
        torch.cuda.empty_cache()
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
