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
os.environ["ANYSEQ_LIB"] = os.path.abspath(os.environ.get("ANYSEQ_TL_LIB", "anyseq_amd/libanyseq_stamps.so"))
sys.path.insert(0, ".")
import anyseq_amd as A  # noqa: E402

q, s = A.main_random_pair(65536, 65536)
q = q[:rows]
path = out + ".txt"
os.environ["ANYSEQ_TIMELINE"] = ""
A.score(kind, q, s, gap_open=-2, gap_extend=-1)
for f_ in (path, path + ".ev", path + ".clk"):
    if os.path.exists(f_):
        os.remove(f_)
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
        mk = band % NW == k
        print(f"   into slot {k}: start lag {np.median(d[m]):.3f}, end lag {np.median(de[m]):.3f}; "
              f"slot-{k} steady duration median {np.median(dur[mk]):.2f} us")
    q4 = len(d) // 4
    print("  start lag by chain quarter:", " ".join(f"{np.mean(d[i*q4:(i+1)*q4]):.3f}" for i in range(4)))

# clock per band (shader cycles / 100 MHz ticks over the band, from its start to its end)
if os.path.exists(path + ".clk"):
    ck = [ln.split() for ln in open(path + ".clk") if not ln.startswith("#")]
    if ck:
        c = np.array([[float(x) for x in r] for r in ck])
        for front, sel in (("fwd", c[:, 0] < 2048), ("rev", c[:, 0] >= 2048)):
            b = c[sel]
            b = b[np.argsort(b[:, 0])]
            ghz = b[:, 1] / (b[:, 2] * 10.0)
            q4 = max(1, len(ghz) // 4)
            print(f"  {front} clock per band (GHz): band0 {ghz[0]:.3f}, by chain quarter "
                  + " ".join(f"{np.median(ghz[i*q4:(i+1)*q4]):.3f}" for i in range(4))
                  + f"; cycles per band: band0 {b[0, 1]:.0f}, median {np.median(b[:, 1]):.0f}")

# hand-off events of block 1000 (producer: its block 1002) per band, 10 ns ticks
if os.path.exists(path + ".ev"):
    ev = {}
    for ln in open(path + ".ev"):
        if ln.startswith("#"):
            continue
        x = [int(t) for t in ln.split()]
        ev[x[0]] = x[1:]
    for front, off in (("fwd", 0), ("rev", 2048)):
        lat1, lat2, wa, lagb, blk = [], [], [], [], []
        kinds = []
        for k in range(2047):
            p, c = ev.get(off + k), ev.get(off + k + 1)
            if not p or not c or not all(p[:3]) or not all(c[3:7]):
                continue
            kinds.append((k + 1) % NW == 0)
            lat1.append((c[4] - p[1]) / 100.0)
            lat2.append((c[5] - p[2]) / 100.0)
            wa.append((c[4] - c[3]) / 100.0)
            lagb.append((c[3] - p[0]) / 100.0)
            blk.append((c[6] - c[3]) / 100.0)
        if not lat1:
            continue
        tr = [(v[8] - v[7]) / 100.0 for v in (ev.get(off + k) for k in range(2048)) if v and len(v) > 10 and v[7] and v[8]]
        ep = [(v[9] - v[8]) / 100.0 for v in (ev.get(off + k) for k in range(2048)) if v and len(v) > 10 and v[9] and v[8]]
        tl = [(v[10] - v[9]) / 100.0 for v in (ev.get(off + k) for k in range(2048)) if v and len(v) > 10 and v[10] and v[9]]
        io = [((v[11] - p[1]) / 100.0, (v[11] - v[12]) / 100.0, (v[4] - v[11]) / 100.0)
              for k in range(1, 2048) for v, p in [(ev.get(off + k), ev.get(off + k - 1))]
              if v and p and len(v) > 12 and v[11] and p[1] and v[4]]
        if io:
            a = np.array(io)
            print(f"  {front} HBM hop via the I/O wave: producer publish -> I/O sees it {np.median(a[:, 0]):.3f} us "
                  f"(that poll's round trip {np.median(a[:, 1]):.3f} us); I/O -> consumer sees it {np.median(a[:, 2]):.3f} us")
        if tr:
            print(f"  {front}: main loop end -> epilogue entry median {np.median(tr):.3f} us; epilogue "
                  f"{np.median(ep):.3f} us; epilogue end -> band end {np.median(tl):.3f} us")
        # the band end (round 5): producer publishes its last half (slot 14) -> consumer
        # sees it (slot 13) -> consumer's loop end (steady end, the timeline file)
        se_of = {}
        for r in rows_:
            se_of[int(float(r[0]))] = float(r[2])
        lh = []
        for k in range(1, 2048):
            v, p = ev.get(off + k), ev.get(off + k - 1)
            if v and p and len(v) > 14 and len(p) > 14 and v[13] and p[14] and v[13] > p[14]:
                lh.append(((v[13] - p[14]) / 100.0, k % NW == 0))
        if lh:
            a = np.array([x[0] for x in lh]); hb = np.array([x[1] for x in lh])
            print(f"  {front} band end: producer's last half published -> consumer sees it: LDS hop median "
                  f"{np.median(a[~hb]):.3f} us, HBM hop median {np.median(a[hb]):.3f} us (n {len(a)})")
            t13 = {k: ev[off + k][13] / 100.0 for k in range(2048) if ev.get(off + k) and len(ev[off + k]) > 14 and ev[off + k][13]}
        kinds = np.array(kinds)
        for name, sel in (("LDS", ~kinds), ("HBM", kinds)):
            if sel.sum() == 0:
                continue
            m = lambda a: np.median(np.array(a)[sel])
            print(f"  {front} {name} hops ({sel.sum()}): publish->seen first half {m(lat1):.3f} us, "
                  f"second half {m(lat2):.3f} us; consumer block-start wait {m(wa):.3f} us; "
                  f"consumer block 1000 start - producer block 1002 start {m(lagb):.3f} us; "
                  f"consumer block time {m(blk):.3f} us")
