#!/usr/bin/env python3
"""Per-kernel summary of rocprofv3 --pmc passes (tools/gpu_check.sh step pmc).

usage: python tools/pmc_summary.py <dir with pmc_*/ subdirs or csvs> <out.json> [--traffic
       --workload=config<N>:n<records per rank> --source=<profiles dir>
       --traffic-out=<path, default profiles/traffic.json>]

bench.py prints the counters only when --workload names its own workload
(config2:n1048576 for the default line) and the kernel build matches.

For each kernel (short name) and counter: mean value per dispatch. With
--traffic, also writes profiles/traffic.json: HBM bytes per launch from
FETCH_SIZE (KB, doubled: gfx950 reports half of 16-B/lane reads, see
/opt/skills/guides/MI355X_MICROARCH.md "HBM") + WRITE_SIZE (KB).
"""
from __future__ import annotations

import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict


def short(name: str) -> str:
    m = re.search(r"::(k_\w+)", name)
    base = m.group(1) if m else name.split("(")[0]
    t = re.search(r"<(.*)>\(", name)
    return f"{base}<{t.group(1)}>" if t else base


def load(root: str):
    acc = defaultdict(lambda: defaultdict(list))
    meta = {}
    for path in glob.glob(os.path.join(root, "**", "*counter_collection*.csv"), recursive=True) + \
            glob.glob(os.path.join(root, "**", "pmc_*.csv"), recursive=True):
        with open(path) as f:
            rd = csv.DictReader(f)
            if "Counter_Name" not in (rd.fieldnames or []):
                continue  # kernel-trace / agent-info csvs of the same -o prefix
            for row in rd:
                k = short(row["Kernel_Name"])
                acc[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
                meta[k] = {"grid": int(row["Grid_Size"]), "wg": int(row["Workgroup_Size"]),
                           "vgpr": int(row["VGPR_Count"]), "sgpr": int(row["SGPR_Count"]),
                           "scratch": int(row["Scratch_Size"]), "lds": int(row["LDS_Block_Size"])}
    out = {}
    for k, cs in acc.items():
        out[k] = {"meta": meta[k], "counters": {c: sum(v) / len(v) for c, v in cs.items()},
                  "dispatches": max(len(v) for v in cs.values())}
    return out


def main():
    root, dst = sys.argv[1], sys.argv[2]
    tag = next((a.split("=", 1)[1] for a in sys.argv if a.startswith("--workload=")), None)
    s = load(root)
    with open(dst, "w") as f:
        json.dump(s, f, indent=1, sort_keys=True)
    if "--traffic" in sys.argv:
        sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        from bdls_amd.provenance import build_info, kernel_src_sha
        src = next((a.split("=", 1)[1] for a in sys.argv if a.startswith("--source=")), root)
        bi = build_info()
        if bi.get("kernel_src_sha") not in (None, kernel_src_sha()):
            raise SystemExit("BUILD_INFO.json describes other kernel sources: rebuild first")
        tr = {"source": f"{src} (rocprofv3 --pmc: FETCH_SIZE / WRITE_SIZE / SQ_INSTS_VALU + "
                        f"GRBM_GUI_ACTIVE / SQ_ACTIVE_INST_VALU + GRBM_GUI_ACTIVE, separate "
                        f"passes)",
              "workload": tag,
              # the kernel build these counters describe (bench.py refuses them
              # for any other): hash of the kernel sources + the library's rev
              "kernel_src_sha": kernel_src_sha(),
              "git_rev": bi.get("git_rev"), "lib_sha256": bi.get("sha256"),
              "correction": "FETCH_SIZE doubled per MI355X_MICROARCH.md (gfx950 reports half "
                            "of 16-B/lane read bytes); WRITE_SIZE as reported",
              "kernels": {}}
        for k, v in s.items():
            c = v["counters"]
            if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
                tr["kernels"][k] = {"fetch_bytes": 2 * c["FETCH_SIZE"] * 1024,
                                    "write_bytes": c["WRITE_SIZE"] * 1024,
                                    "bytes_per_launch": (2 * c["FETCH_SIZE"] + c["WRITE_SIZE"]) * 1024}
            if "SQ_INSTS_VALU" in c and "GRBM_GUI_ACTIVE" in c:
                # counter-based VALU issue utilisation: wave-instructions x
                # cycles each / (per-XCD cycles x 256 CUs x 4 SIMDs);
                # GRBM_GUI_ACTIVE is summed over the 8 XCDs (MI355X_MICROARCH.md
                # "DVFS give-back"). Two issue-cost models: 2 cycles (SIMD-32,
                # wave64 over 2 cycles, MI355X_MICROARCH.md:54) and 4 cycles
                # (one wave alone, and the measured u32 add / v_mad_u64_u32
                # issue rate of profiles/ubench.json).
                cyc = c["GRBM_GUI_ACTIVE"] / 8.0
                e = tr["kernels"].setdefault(k, {})
                e["sq_insts_valu"] = c["SQ_INSTS_VALU"]
                e["grbm_gui_active"] = c["GRBM_GUI_ACTIVE"]
                e["valu_util_2cyc"] = c["SQ_INSTS_VALU"] * 2 / (cyc * 1024) if cyc else None
                e["valu_util_4cyc"] = c["SQ_INSTS_VALU"] * 4 / (cyc * 1024) if cyc else None
            if "SQ_ACTIVE_INST_VALU" in c:
                # rocprof's VALUBusy: SQ_ACTIVE_INST_VALU (quad-cycles, summed
                # over waves) x 4 / (SIMDs x GRBM_GUI_ACTIVE per XCD); the
                # GRBM_GUI_ACTIVE of the same pass when collected there
                e = tr["kernels"].setdefault(k, {})
                g = c.get("GRBM_GUI_ACTIVE")
                e["sq_active_inst_valu"] = c["SQ_ACTIVE_INST_VALU"]
                e["valu_busy"] = (c["SQ_ACTIVE_INST_VALU"] * 4 / (g / 8.0 * 1024)) if g else None
        path = next((a.split("=", 1)[1] for a in sys.argv if a.startswith("--traffic-out=")),
                    os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                 "profiles", "traffic.json"))
        with open(path, "w") as f:
            json.dump(tr, f, indent=1, sort_keys=True)
    for k, v in sorted(s.items()):
        print(k, v["meta"], {c: round(x, 1) for c, x in v["counters"].items()})


if __name__ == "__main__":
    main()
