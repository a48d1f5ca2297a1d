"""Bisect device vs host-sim: dump every intermediate after each stage."""
import ctypes, json, os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from tests.conftest import pack, GOLDEN
from bdls_amd import _lib
import torch
recs = [json.loads(l) for l in open(GOLDEN)]
fr = [r for r in recs if "msg" in r]
arrs = pack(fr, True)
n = len(fr); ns = (n + 63) // 64 * 64
words = 3 * 6 * 8 * ns + (3 * ns + 3) // 4
hs = ctypes.CDLL(os.path.join(ROOT, "tests/native/build/libhostsim.so"))
vp = ctypes.c_void_p
hs.hs_verify_dump.argtypes = [vp] * 7 + [ctypes.c_uint32] * 3 + [vp, vp]
hdump = np.zeros(words, np.uint32); hreason = np.zeros(n, np.uint8)
hs.hs_verify_dump(*[a.ctypes.data for a in arrs], n, 1, 1, hreason.ctypes.data, hdump.ctypes.data)
L = _lib.lib(); _lib.ensure_init()
L.bhx_debug_verify.argtypes = [ctypes.c_int, ctypes.POINTER(_lib.BhBatch), ctypes.c_size_t, ctypes.c_uint32, vp, vp, vp]
dev = torch.device("cuda:0")
def up(x):
    x = x.view(np.int64) if x.dtype == np.uint64 else x.view(np.int32) if x.dtype == np.uint32 else x
    return torch.from_numpy(np.ascontiguousarray(x)).to(dev)
t = [up(a) for a in arrs]
b = _lib.BhBatch(*[x.data_ptr() for x in t])
bm = torch.zeros(ns // 64, dtype=torch.int64, device=dev); rs = torch.zeros(n, dtype=torch.uint8, device=dev)
for trial in range(3):
    ddump = np.zeros(words, np.uint32)
    _lib.check(L.bhx_debug_verify(0, ctypes.byref(b), n, 1, bm.data_ptr(), rs.data_ptr(), ddump.ctypes.data))
    names = ["e", "r", "sm", "qx", "qy", "rm"]
    for stage in range(3):
        for a in range(6):
            o = ((stage * 6 + a) * 8) * ns
            h = hdump[o:o + 8 * ns].reshape(8, ns)[:, :n]; d = ddump[o:o + 8 * ns].reshape(8, ns)[:, :n]
            diff = np.nonzero((h != d).any(axis=0))[0]
            if len(diff): print("trial", trial, "stage", stage, names[a], "differs at", diff[:12].tolist())
        hs_ = hdump.view(np.uint8)[3*6*8*ns*4 + stage*ns:][:n]; ds_ = ddump.view(np.uint8)[3*6*8*ns*4 + stage*ns:][:n]
        diff = np.nonzero(hs_ != ds_)[0]
        if len(diff): print("trial", trial, "stage", stage, "st differs at", diff[:12].tolist(), hs_[diff[:4]], ds_[diff[:4]])
    print("trial", trial, "reason diff", np.nonzero(rs.cpu().numpy() != hreason)[0][:12].tolist(), "host-vs-golden", int((hreason != np.array([r['reason'] for r in fr])).sum()))
