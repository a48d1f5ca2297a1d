"""The single-Verify tail study: bench.py's
single_verify_measure (native csp_load at 1..256 callers, cold and
registered) under the current environment (e.g. BH_BLOCKING_SYNC=0/1), with
the cgroup throttling counters csp_load now reports. One JSON line."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

threads = tuple(int(x) for x in sys.argv[1:]) or (1, 8, 64, 256)
out = bench.single_verify_measure(None, threads)
keep = {k: {f: v.get(f) for f in ("p50_us", "p99_us", "p999_us", "max_us", "verifies_per_s",
                                   "cgroup_nr_throttled", "cgroup_throttled_us", "bad", "wall_ms",
                                   "cpu_user_ms", "cpu_sys_ms", "vol_csw", "invol_csw",
                                   "cpus_pinned")}
        for k, v in out.items() if isinstance(v, dict) and "p50_us" in v}
keep["env"] = {k: v for k, v in os.environ.items() if k.startswith("BH_")}
print(json.dumps(keep))
