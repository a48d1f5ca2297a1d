import json, os, sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tests.conftest import pack, GOLDEN
from bdls_amd.bccsp import verify_packed, HipCSP
from bdls_amd import _lib
recs = [json.loads(l) for l in open(GOLDEN)]
fr = [r for r in recs if "msg" in r]
HipCSP()
order = sys.argv[1] if len(sys.argv) > 1 else "fused_first"
def run(rs, fused):
    v, g = verify_packed(*pack(rs, fused), flags=1 if fused else 0)
    return [(i, r["tag"], int(x), r["reason"]) for i, (r, x) in enumerate(zip(rs, g)) if x != r["reason"]]
if order == "digest_first":
    print("digest(all)", run(recs, False)[:8])
print("fused(all)", run(fr, True)[:8])
print("digest(fused recs)", run(fr, False)[:8])
print("fused(all) again", run(fr, True)[:8])
bad = run(fr, True)
if bad:
    i0 = bad[0][0]
    for lo, hi in [(i0 - 1, i0 + 5), (0, i0 + 5), (i0 - 1, len(fr))]:
        print("fused subset", lo, hi, run(fr[max(0, lo):hi], True))
    print("singles", [run([fr[i]], True) for i in range(i0 - 1, i0 + 5)])
    # alignment: message offsets of the failing records
    pub, sig, so, sl, msg, mo, ml = pack(fr, True)
    print("msg_off", [(int(mo[i]), int(ml[i]), int(mo[i]) % 4) for i in range(i0 - 2, i0 + 5)])
    print("sig_off", [(int(so[i]), int(sl[i])) for i in range(i0 - 2, i0 + 5)])
