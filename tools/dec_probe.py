"""Config 3's host half alone: bh_fabric_block_preverify(BH_FAB_F_DECODE_ONLY)
on the bench's block (decode, identities, batch build; no device work), 200
calls, p50 / min in ms. BH_DECODE_THREADS / BH_FAB_TIMING from the caller."""
import ctypes
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from bdls_amd import _lib  # noqa: E402
from bdls_amd.workload import fabric as F  # noqa: E402

L = _lib.lib()
fb = F.generate_fabric_block(seed=3)
buf = np.frombuffer(fb.block + b"\0", np.uint8)
ntx, nend = ctypes.c_size_t(), ctypes.c_size_t()
txs = (_lib.BhFabTx * fb.ntx)()
cap = sum(len(e) for e in fb.tx_endorse) + 64 * fb.ntx
end = np.zeros(cap, np.uint8)
ms = []
for _ in range(200):
    t = time.perf_counter()
    _lib.check(L.bh_fabric_block_preverify(buf.ctypes.data, len(fb.block), _lib.BH_FAB_F_DECODE_ONLY,
                                           txs, fb.ntx, ctypes.byref(ntx), end.ctypes.data, cap,
                                           ctypes.byref(nend)))
    ms.append((time.perf_counter() - t) * 1e3)
ms.sort()
print(f"threads {os.environ.get('BH_DECODE_THREADS')} p50 {ms[100]:.4f} ms min {ms[0]:.4f}")
