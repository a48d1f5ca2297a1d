#!/usr/bin/env python3
"""Tie bench.py's roofline to rocprofv3: the dominant kernel's per-dispatch
durations from a `rocprofv3 --kernel-trace --stats` run of the same bench
command, split by bench phase, against the line's `roofline.launch_ms`.

usage: python tools/prof_check.py <kernel_trace.csv> <bench.json> <out.json>

The bench runs, in order: the host path (warmup + 1 single + K timed batches
over the compute lanes, so a kernel may share the GPU with another lane's),
since round 6 the staged host path host_path_e2e (max(1, warmup) + 1 + K
batches, when the line carries it), then the HBM-resident passes (warmup + K timed, rotating over the lanes), K more
resident passes serialised with HIP events on every stage (the per-kernel
timing), then the side configs (config 5's rank shard launches the one-lane
kernels with no key-comb records: short dispatches). bench.py takes launch_ms
from the HIP events of the serialised passes: dispatches
[H + E + W + K, H + E + W + 2K) of the kernel in launch order (H = W + 1 + K,
E = the e2e phase's count or 0). rocprof's --stats
average mixes every phase.
"""
import csv
import json
import sys


def main():
    trace, bench, dst = sys.argv[1:4]
    b = json.load(open(bench))
    k = b["roofline"]["kernel"]
    steps, warm = b["steps"], b["warmup"]
    rows = [r for r in csv.DictReader(open(trace))
            if f"::{k}<bh::F30_p256>" in r["Kernel_Name"] or
            r["Kernel_Name"].startswith(f"void (anonymous namespace)::{k}<bh::F30_p256>")]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in rows]
    host_n = warm + 1 + steps
    e2e_n = (max(1, warm) + 1 + steps) if b.get("host_path_e2e") else 0
    lo = host_n + e2e_n + warm + steps
    timed = d[lo:lo + steps]
    out = {
        "kernel": k, "dispatches": len(d),
        "all_dispatch_mean_ms": round(sum(d) / len(d), 4) if d else None,
        "host_path_mean_ms": round(sum(d[:host_n]) / max(1, len(d[:host_n])), 4),
        "host_path_e2e_mean_ms": (round(sum(d[host_n:host_n + e2e_n]) / e2e_n, 4)
                                  if e2e_n else None),
        "resident_lanes_mean_ms": round(sum(d[lo - steps:lo]) / steps, 4),
        "resident_timed_mean_ms": round(sum(timed) / steps, 4) if len(timed) == steps else None,
        "resident_timed_dispatches": [lo, lo + steps],
        "bench_launch_ms": b["roofline"]["launch_ms"],
        "bench_frac": b["roofline"]["frac"],
    }
    if out["resident_timed_mean_ms"]:
        out["agreement"] = round(out["resident_timed_mean_ms"] / out["bench_launch_ms"], 4)
        out["frac_from_rocprof"] = round(b["roofline"]["frac"] * out["bench_launch_ms"]
                                         / out["resident_timed_mean_ms"], 4)
    out["note"] = ("phases by dispatch order: host path = first warmup + 1 + steps dispatches "
                   "(lanes overlap: durations include other lanes' kernels), then the staged "
                   "host path's max(1, warmup) + 1 + steps (if on the line), then warmup + "
                   "steps resident passes over the lanes (the timed `value`), then `steps` "
                   "serialised resident passes (resident_timed_*); bench_launch_ms = HIP events "
                   "over those serialised passes")
    json.dump(out, open(dst, "w"), indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
