"""Band timeline of the affine fill (diagnostic stamps build): one two-front local
affine score of the 65536^2 configs[2] pair -> gpurun_out/<out>.txt, then a summary.
Slots per band: steady-state start, steady-state end, band end (us from the first).
usage: _aff_timeline.py <out-prefix> [kind] [rows]"""
import os
import sys

import numpy as np

out = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/aff_timeline"
kind = sys.argv[2] if len(sys.argv) > 2 else "local"
rows = int(sys.argv[3]) if len(sys.argv) > 3 else 65536
os.environ["ANYSEQ_STAMPS"] = "1"
os.environ["ANYSEQ_LIB"] = os.path.abspath("anyseq_amd/libanyseq_stamps.so")
sys.path.insert(0, ".")
import anyseq_amd as A  # noqa: E402

q, s = A.main_random_pair(65536, 65536)
q = q[:rows]
path = out + ".txt"
os.environ["ANYSEQ_TIMELINE"] = ""
A.score(kind, q, s, gap_open=-2, gap_extend=-1)
if os.path.exists(path):
    os.remove(path)
os.environ["ANYSEQ_TIMELINE"] = path
v = A.score(kind, q, s, gap_open=-2, gap_extend=-1)
os.environ["ANYSEQ_TIMELINE"] = ""
print("score", v)

NW = 4
rows_ = [ln.split() for ln in open(path) if not ln.startswith("#")]
hdr = [ln for ln in open(path) if ln.startswith("#")]
a = np.array([[float(x) for x in r] for r in rows_])
print(hdr[-1].strip() if hdr else "")
for front, sel in (("fwd", a[:, 0] < 2048), ("rev", a[:, 0] >= 2048)):
    b = a[sel]
    b = b[np.argsort(b[:, 0])]
    band = (b[:, 0] % 2048).astype(int)
    st, se, en = b[:, 1], b[:, 2], b[:, 3]
    b0 = b[:, 4] if b.shape[1] > 4 else np.full(len(b), -1.0)
    if (b0 >= 0).sum() > 2:
        ok = b0 >= 0
        d0 = np.diff(b0[ok])
        print(f"  C++ block-0 start: lag median {np.median(d0):.3f} us; block0 -> steady start median "
              f"{np.median((st - b0)[ok]):.3f} us")
    if (b0 <= -2).sum() > 2:   # asm path: -2 - (blocks without a prefetched top row)
        miss = -2 - b0[b0 <= -2]
        print(f"  prefetch misses per band: median {np.median(miss):.0f}, mean {miss.mean():.1f}, "
              f"max {miss.max():.0f}, band0 {miss[0]:.0f}")
    d = np.diff(st)
    de = np.diff(se)
    glob = band[1:] % NW == 0
    dur = se - st
    print(f"{front}: {len(b)} bands; last steady start {st[-1]:.1f} us, last end {en.max():.1f} us")
    print(f"  steady duration: band0 {dur[0]:.1f}, median {np.median(dur):.1f}, last {dur[-1]:.1f} us")
    print(f"  start lag: LDS hop median {np.median(d[~glob]):.3f} us, HBM hop median {np.median(d[glob]):.3f} us")
    print(f"  end lag:   LDS hop median {np.median(de[~glob]):.3f} us, HBM hop median {np.median(de[glob]):.3f} us")
    for k in range(NW):
        m = band[1:] % NW == k
        print(f"   into slot {k}: start lag {np.median(d[m]):.3f}, end lag {np.median(de[m]):.3f}")
    q4 = len(d) // 4
    print("  start lag by chain quarter:", " ".join(f"{np.mean(d[i*q4:(i+1)*q4]):.3f}" for i in range(4)))
