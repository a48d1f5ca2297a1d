"""Timeline of the latency configs' device work from a rocprofv3
--kernel-trace (+ --hip-trace) CSV: for the last N calls of a
`bench.py --config 3|4` run, each kernel's start offset from the call's first
kernel, its duration, and the idle gaps between kernels (launch overhead and
host work), so a warm call's 0.5 ms splits into kernel time and gaps.
usage: python tools/lat_trace.py <kernel_trace.csv> [calls=5] [call_gap_us=150]"""
import csv
import json
import re
import sys


def short(name):
    m = re.search(r"(k_\w+)", name)
    return m.group(1) if m else name.split("(")[0][-40:]


def main():
    path = sys.argv[1]
    ncalls = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    gap_us = float(sys.argv[3]) if len(sys.argv) > 3 else 150.0
    ks = []
    with open(path) as f:
        for r in csv.DictReader(f):
            ks.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]),
                       r.get("Queue_Id", r.get("Stream_Id", ""))))
    ks.sort()
    calls, cur = [], []
    for k in ks:  # a call = kernels separated by less than gap_us from the previous end
        if cur and k[0] - max(e for _, e, _, _ in cur) > gap_us * 1e3:
            calls.append(cur)
            cur = []
        cur.append(k)
    if cur:
        calls.append(cur)
    out = []
    for c in calls[-ncalls:]:
        t0 = c[0][0]
        end = max(e for _, e, _, _ in c)
        busy, last = 0, t0
        for s, e, _, _ in c:  # union of kernel intervals
            if e > last:
                busy += e - max(s, last)
                last = e
        out.append({"span_us": round((end - t0) / 1e3, 1), "kernel_busy_us": round(busy / 1e3, 1),
                    "kernels": [(n, round((s - t0) / 1e3, 1), round((e - s) / 1e3, 1), q)
                                for s, e, n, q in c]})
    print(json.dumps({"calls_found": len(calls), "last": out}, indent=1))


if __name__ == "__main__":
    main()
