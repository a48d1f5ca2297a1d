"""Which kernel build a measurement describes.

`kernel_src_sha()` hashes the sources the HIP code object is compiled from
(bdls_amd/csrc/verify_kernels.hip, every header under bdls_amd/csrc/, and the
Makefile that holds the compile flags). build() records it in
bdls_amd/lib/BUILD_INFO.json, tools/pmc_summary.py stamps it into
profiles/traffic.json, and bench.py prints PMC counters only when the stamp
equals the hash of the sources beside the library it runs -- counters taken on
another kernel shape are reported as stale (null), never beside a timing of a
different kernel.
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
