#!/usr/bin/env python3
"""Per-wave timeline of k_ktab_ladder at config 2 (an experiment build with
-DBH_WAVE_TIMES, tools/build_exp.sh wt:-DBH_WAVE_TIMES=1).

usage: BDLS_HIP_LIB=$PWD/exp/libbdlship_wt.so python tools/wave_times.py [out.json]

Runs one serialised HBM-resident pass (bh_verify_dev with timing) of the
config-2 batch, then reads every wave's role (0 table build, 1 ladder, 2 u1 G),
CU and start / end (wall clock, 100 MHz) and prints where the kernel's time
goes: when each role's waves run, how long a build wave takes, and how many
waves of each role are resident over the kernel's duration.
"""
import ctypes
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bdls_amd import _lib, workload  # noqa: E402

TICK_NS = 10.0  # wall_clock64: 100 MHz


def main():
    dst = sys.argv[1] if len(sys.argv) > 1 else None
    _lib.ensure_init()
    L = _lib.lib()
    raw = ctypes.CDLL(_lib.LIB_PATH)
    raw.bh_wave_times.argtypes = [ctypes.c_void_p, ctypes.c_int]
    w = workload.generate(1 << 20, 65536, 256, 16, seed=2)
    DA = _lib.DeviceArray
    d = [DA.from_numpy(0, x) for x in w.arrays()]
    words, reason = DA(0, ((w.n + 63) // 64) * 8), DA(0, w.n)
    b = _lib.BhBatch(*[x.ptr for x in d])
    buf = np.zeros(65536 * 4, np.uint64)
    out = {}
    for rep in range(3):
        assert raw.bh_wave_times(None, 1) == 0
        tm = _lib.BhTiming()
        _lib.check(L.bh_verify_dev(0, 0, ctypes.byref(b), w.n, _lib.BH_F_HASH_SHA256, words.ptr,
                                   reason.ptr, None, 1, ctypes.byref(tm)))
        assert raw.bh_wave_times(buf.ctypes.data, 0) == 0
        ok = bool((reason.to_numpy(np.uint8, w.n) == w.reason).all())
        t = buf.reshape(-1, 4)
        t = t[t[:, 1] > 0]
        t0 = t[:, 0].min()
        s = (t[:, 0] - t0) * TICK_NS / 1e6  # ms
        e = (t[:, 1] - t0) * TICK_NS / 1e6
        role = t[:, 2]
        span = float(e.max())
        r = {"parity": ok, "kernel_ms_events": round(tm.build_ladder_ms, 4), "span_ms": round(span, 4),
             "waves": int(len(t)), "cus": int(len(np.unique(t[:, 3])))}
        for k, name in ((0, "build"), (1, "ladder"), (2, "u1G")):
            m = role == k
            if not m.any():
                continue
            dur = e[m] - s[m]
            r[name] = {"waves": int(m.sum()), "start_ms": [round(float(np.percentile(s[m], q)), 4) for q in (0, 50, 100)],
                       "end_ms": [round(float(np.percentile(e[m], q)), 4) for q in (0, 50, 90, 99, 100)],
                       "dur_ms": [round(float(np.percentile(dur, q)), 4) for q in (0, 50, 90, 100)]}
        # resident waves per role over 20 bins of the span
        bins = np.linspace(0, span, 21)
        mid = (bins[:-1] + bins[1:]) / 2
        r["resident_per_bin"] = {name: [int(((role == k) & (s <= x) & (e > x)).sum()) for x in mid]
                                 for k, name in ((0, "build"), (2, "u1G"))}
        out[f"rep{rep}"] = r
        print(json.dumps(r))
    if dst:
        json.dump(out, open(dst, "w"), indent=1)


if __name__ == "__main__":
    main()
