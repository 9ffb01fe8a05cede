"""Summarise timeline files (band start / first publish / end in µs)."""
import sys
import numpy as np
NW = 4
for path in sys.argv[1:]:
    rows = [l.split() for l in open(path) if not l.startswith("#")]
    hdr = [l for l in open(path) if l.startswith("#")]
    a = np.array([[float(x) for x in r] for r in rows])
    print(f"== {path}: {hdr[0].strip() if hdr else ''}")
    for front, sel in (("fwd", a[:, 0] < 2048), ("rev", a[:, 0] >= 2048)):
        b = a[sel]
        if len(b) < 2:
            continue
        b = b[np.argsort(b[:, 0])]
        st, pub, en = b[:, 1], b[:, 2], b[:, 3]
        band = (b[:, 0] % 2048).astype(int)
        d = np.diff(st)
        glob = band[1:] % NW == 0
        ok = pub > 0
        pd = st[1:] - pub[:-1]
        ok2 = pub[:-1] > 0
        print(f" {front}: {len(b)} bands, last start {st[-1]:.1f}, last end {en.max():.1f}, "
              f"dur med {np.median(en-st):.1f} (band0 {en[0]-st[0]:.1f}) | lag lds {np.median(d[~glob]):.2f} "
              f"glob {np.median(d[glob]) if glob.any() else 0:.2f} | st->pub {np.median(pub[ok]-st[ok]):.2f} | "
              f"pub->next lds {np.median(pd[ok2 & ~glob]) if (ok2 & ~glob).any() else 0:.2f} "
              f"glob {np.median(pd[ok2 & glob]) if (ok2 & glob).any() else 0:.2f}")

# band duration by wave slot in its workgroup (which SIMD neighbours the I/O wave)
for path in sys.argv[1:]:
    rows = [l.split() for l in open(path) if not l.startswith("#")]
    a = np.array([[float(x) for x in r] for r in rows])
    band = (a[:, 0] % 2048).astype(int)
    dur = a[:, 3] - a[:, 1]
    ok = a[:, 3] > 0
    print(" duration by wave slot:", " ".join(f"w{k}={np.median(dur[ok & (band % NW == k)]):.1f}" for k in range(NW)))
    mid = ok & (band > 64) & (band < 448)
    print(" mid-chain bands, start-to-start lag by slot:",
          " ".join(f"w{k}={np.median(np.diff(np.sort(a[mid & (band % NW == k), 1]))):.2f}" for k in range(NW)))
