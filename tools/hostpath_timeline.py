#!/usr/bin/env python3
"""Host-path timeline from a rocprofv3 --kernel-trace --memory-copy-trace run of
bench.py (config 2, plain defaults): where each timed batch's upload starts
and ends, where its pass ends, and the gaps between them.

  python3 tools/hostpath_timeline.py <trace dir> [--steps K] [--out summary.json]

A batch's upload is the copy engine's H2D copies ending with the largest one
(the message bytes); its pass ends with k_bitmap. The timed batches are the
K whose uploads precede the resident upload (the last large H2D on the
compute stream), counted back from it. Prints and writes one JSON object.
"""
import argparse
import csv
import glob
import json
import os


def rows(path):
    with open(path) as f:
        return list(csv.DictReader(f))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--out")
    a = ap.parse_args()
    mc = rows(glob.glob(os.path.join(a.dir, "*_memory_copy_trace.csv"))[0])
    kt = rows(glob.glob(os.path.join(a.dir, "*_kernel_trace.csv"))[0])
    t0 = min(int(r["Start_Timestamp"]) for r in mc)
    ms = lambda r, k: (int(r[k]) - t0) / 1e6
    h2d = sorted((ms(r, "Start_Timestamp"), ms(r, "End_Timestamp"), r["Stream_Id"])
                 for r in mc if "HOST_TO_DEVICE" in r["Direction"])
    big = [x for x in h2d if x[1] - x[0] > 2.0]  # the message array of a batch
    # the copy stream carries the batches; the last big copy on another stream
    # is the resident upload (bench.py), the one before the timed run the probe
    copy_stream = max(set(s for _, _, s in big), key=lambda s: sum(1 for x in big if x[2] == s))
    resident = [x for x in big if x[2] != copy_stream]
    cut = resident[-1][0] if resident else float("inf")
    ups = [x for x in big if x[2] == copy_stream and x[0] < cut][-a.steps:]
    # a batch's first copy: the earliest copy-stream H2D after the previous
    # batch's message copy ended
    all_big = [x for x in big if x[2] == copy_stream]
    starts = []
    for s, e, _ in ups:
        before = [x[1] for x in all_big if x[1] <= s]
        prev_end = max(before) if before else -1.0
        first = [x[0] for x in h2d if x[2] == copy_stream and prev_end <= x[0] <= s]
        starts.append(min(first) if first else s)
    ends = [e for _, e, _ in ups]
    passes = sorted(ms(r, "End_Timestamp") for r in kt if "k_bitmap" in r["Kernel_Name"])
    # with lanes the k-th pass to END need not be batch k: the sorted pass
    # ends of the timed run
    # (the host batches all complete before the resident upload)
    run_passes = [p for p in passes if p <= cut][-a.steps:]
    spacing = [b - a_ for a_, b in zip(starts, starts[1:])]
    out = {
        "batches": len(ups),
        "upload_start_ms": [round(x, 3) for x in starts],
        "upload_end_ms": [round(x, 3) for x in ends],
        "pass_end_ms": [round(x, 3) for x in run_passes],
        "timed_span_ms": round(run_passes[-1] - starts[0], 3) if run_passes else None,
        "upload_busy_ms": round(sum(e - s for s, e in zip(starts, ends)), 3),
        "first_upload_gap_ms": round(starts[1] - ends[0], 3) if len(starts) > 1 else None,
        "upload_spacing_mean_ms": round(sum(spacing) / len(spacing), 3) if spacing else None,
        "pass_spacing_mean_ms": round((run_passes[-1] - run_passes[0]) / (len(run_passes) - 1), 3)
        if len(run_passes) > 1 else None,
        "drain_ms": round(run_passes[-1] - ends[-1], 3) if run_passes else None,
    }
    print(json.dumps(out, indent=1))
    if a.out:
        with open(a.out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
