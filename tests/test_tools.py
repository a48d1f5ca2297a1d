"""CPU: the measurement tools that tie bench.py's line to rocprofv3 output.

tools/prof_check.py splits the dominant kernel's dispatches by bench phase
(host path, overlapped resident passes, serialised timing passes) and compares
the serialised passes' mean with the line's launch_ms; tools/pmc_summary.py
turns --pmc counter CSVs into per-launch HBM bytes (FETCH_SIZE doubled per the
gfx950 correction, + WRITE_SIZE) and VALU issue utilisation, stamped with the
kernel-source hash bench.py checks. Both are fed synthetic rocprofv3-shaped
CSVs here."""
import csv
import json
import os
import subprocess
import sys

from tests.conftest import ROOT

KNAME = "void (anonymous namespace)::k_keycomb<bh::F30_p256>(bh::Work, bh::Plan)"


def _trace(path, durations_ms):
    with open(path, "w", newline="") as f:
        w = csv.DictWriter(f, ["Kernel_Name", "Start_Timestamp", "End_Timestamp"])
        w.writeheader()
        t = 1_000_000
        for d in durations_ms:
            w.writerow({"Kernel_Name": KNAME, "Start_Timestamp": t,
                        "End_Timestamp": t + int(d * 1e6)})
            t += int(d * 1e6) + 1000
        # another kernel in between is ignored
        w.writerow({"Kernel_Name": "void (anonymous namespace)::k_prep<bh::F30_p256>(x)",
                    "Start_Timestamp": t, "End_Timestamp": t + 5})


def test_prof_check_phases(tmp_path):
    steps, warm = 4, 2
    host = [9.0] * (warm + 1 + steps)        # host path: warmup + 1 single + K
    lanes = [7.0] * (warm + steps)           # overlapped resident passes
    timed = [3.5, 3.6, 3.7, 3.6]             # serialised timing passes
    trace = tmp_path / "trace.csv"
    _trace(trace, host + lanes + timed)
    bench = tmp_path / "bench.json"
    bench.write_text(json.dumps({"steps": steps, "warmup": warm,
                                 "roofline": {"kernel": "k_keycomb", "launch_ms": 3.6,
                                              "frac": 0.8}}))
    out = tmp_path / "out.json"
    subprocess.run([sys.executable, os.path.join(ROOT, "tools", "prof_check.py"), str(trace),
                    str(bench), str(out)], check=True, capture_output=True)
    r = json.loads(out.read_text())
    assert r["dispatches"] == len(host + lanes + timed)
    assert abs(r["resident_timed_mean_ms"] - 3.6) < 1e-3
    assert abs(r["host_path_mean_ms"] - 9.0) < 1e-3
    assert abs(r["resident_lanes_mean_ms"] - 7.0) < 1e-3
    assert r["resident_timed_dispatches"] == [2 * warm + 1 + 2 * steps, 2 * warm + 1 + 3 * steps]
    assert abs(r["agreement"] - 1.0) < 1e-3 and abs(r["frac_from_rocprof"] - 0.8) < 1e-3


def test_pmc_summary_traffic(tmp_path):
    d = tmp_path / "pmc_FETCH"
    d.mkdir()
    rows = []
    for disp, (fetch, write, valu, grbm) in enumerate([(1000.0, 100.0, 4.0e6, 8.0e6),
                                                        (1200.0, 100.0, 4.0e6, 8.0e6)]):
        for name, val in (("FETCH_SIZE", fetch), ("WRITE_SIZE", write),
                          ("SQ_INSTS_VALU", valu), ("GRBM_GUI_ACTIVE", grbm)):
            rows.append({"Dispatch_Id": disp, "Kernel_Name": KNAME, "Counter_Name": name,
                         "Counter_Value": val, "Grid_Size": 1048576, "Workgroup_Size": 256,
                         "VGPR_Count": 104, "SGPR_Count": 112, "Scratch_Size": 0,
                         "LDS_Block_Size": 79872})
    with open(d / "pmc_counter_collection.csv", "w", newline="") as f:
        w = csv.DictWriter(f, list(rows[0]))
        w.writeheader()
        w.writerows(rows)
    traffic = tmp_path / "traffic.json"
    subprocess.run([sys.executable, os.path.join(ROOT, "tools", "pmc_summary.py"), str(tmp_path),
                    str(tmp_path / "summary.json"), "--traffic", "--workload=config2:n1048576",
                    f"--traffic-out={traffic}"], check=True, capture_output=True, cwd=ROOT)
    tr = json.loads(traffic.read_text())
    k = tr["kernels"]["k_keycomb<bh::F30_p256>"]
    assert k["fetch_bytes"] == 2 * 1100.0 * 1024 and k["write_bytes"] == 100.0 * 1024
    assert k["bytes_per_launch"] == (2 * 1100.0 + 100.0) * 1024
    # 4e6 wave-instructions x 4 cycles / (8e6 / 8 XCDs x 1024 SIMDs)
    assert abs(k["valu_util_4cyc"] - 4.0e6 * 4 / (1.0e6 * 1024)) < 1e-12
    assert tr["workload"] == "config2:n1048576"
    sys.path.insert(0, ROOT)
    from bdls_amd.provenance import kernel_src_sha
    assert tr["kernel_src_sha"] == kernel_src_sha()


def test_bench_refuses_foreign_counters(tmp_path, monkeypatch):
    """bench.py prints traffic / VALU counters only when profiles/traffic.json
    was taken on its own workload AND on the kernel build the loaded library
    came from (BUILD_INFO.json's kernel_src_sha, checked by the library's
    sha256); otherwise it says why."""
    sys.path.insert(0, ROOT)
    import bench
    from bdls_amd import _lib
    from bdls_amd.provenance import lib_kernel_sha
    if not os.path.exists(_lib.LIB_PATH):
        import pytest
        pytest.skip("library not built")
    cur = lib_kernel_sha(_lib.LIB_PATH)
    (tmp_path / "profiles").mkdir()
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    src, kernels, why = bench.load_counters(2, 1048576)
    assert src is None and "no profiles/traffic.json" in why
    good = {"workload": "config2:n1048576", "kernel_src_sha": cur, "git_rev": "x",
            "source": "s", "kernels": {"k_keycomb<bh::F30_p256>": {"bytes_per_launch": 1.0}}}
    tf = tmp_path / "profiles" / "traffic.json"
    tf.write_text(json.dumps(dict(good, workload="config2:n65536")))
    assert "not config2:n1048576" in bench.load_counters(2, 1048576)[2]
    if cur is None:  # a library build() did not record: nothing is trusted
        tf.write_text(json.dumps(good))
        assert "no build record" in bench.load_counters(2, 1048576)[2]
        return
    tf.write_text(json.dumps(dict(good, kernel_src_sha="0" * 16)))
    assert bench.load_counters(2, 1048576)[2].startswith("stale")
    tf.write_text(json.dumps(good))
    src, kernels, why = bench.load_counters(2, 1048576)
    assert why is None and cur in src and kernels == good["kernels"]


def test_hostpath_timeline(tmp_path):
    """tools/hostpath_timeline.py on a synthetic trace: 3 warm + 4 timed
    batches on the copy stream (a 0.1 ms index copy + a 4 ms message copy
    each), a resident upload on another stream, one k_bitmap per pass; the
    first timed batch's upload is followed by a 2 ms gap."""
    ms = lambda x: int(x * 1e6)
    copies, kernels, t = [], [], 0.0
    for b in range(7):
        if b == 4:
            t += 2.0  # the gap behind timed batch 0
        copies.append(("2", t, t + 0.1))
        copies.append(("2", t + 0.1, t + 4.1))
        kernels.append(t + 9.0)  # its pass ends 4.9 ms after its upload
        t += 4.1
    copies.append(("1", t + 20, t + 24))  # resident upload
    with open(tmp_path / "x_memory_copy_trace.csv", "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Direction", "Stream_Id", "Start_Timestamp", "End_Timestamp"])
        for s, a, b in copies:
            w.writerow(["MEMORY_COPY_HOST_TO_DEVICE", s, ms(a), ms(b)])
    with open(tmp_path / "x_kernel_trace.csv", "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Kernel_Name", "Start_Timestamp", "End_Timestamp"])
        for e in kernels:
            w.writerow(["k_bitmap", ms(e - 0.01), ms(e)])
    out = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "hostpath_timeline.py"),
                          str(tmp_path), "--steps", "3"], capture_output=True, check=True)
    d = json.loads(out.stdout)
    assert d["batches"] == 3
    assert abs(d["upload_spacing_mean_ms"] - 4.1) < 1e-3
    assert abs(d["drain_ms"] - 4.9) < 1e-3
    assert abs(d["timed_span_ms"] - (2 * 4.1 + 9.0)) < 1e-3
