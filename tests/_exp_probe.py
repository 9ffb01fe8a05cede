"""Time the fill on a lone band and on 64k^2 for each diagnostic library build."""
import os, subprocess, sys
if len(sys.argv) > 1 and sys.argv[1] == "--child":
    sys.path.insert(0, '.')
    import anyseq_amd as A
    qq, ss = A.main_random_pair(65536, 65536)
    out = []
    for n, m in [(64, 65536), (512, 65536), (65536, 65536)]:
        best = 1e9
        for _ in range(3):
            A.score('global', qq[:n], ss[:m]); ms, _ = A.last_fill_timing(); best = min(best, ms)
        out.append(f"{n}x{m}: {best:.3f} ms ({n*m/best/1e6:.0f})")
    print(os.path.basename(os.environ.get("ANYSEQ_LIB", "libanyseq.so")), " | ".join(out), flush=True)
else:
    for lib in sys.argv[1:]:
        env = dict(os.environ, ANYSEQ_LIB=os.path.abspath(lib))
        subprocess.run([sys.executable, __file__, "--child"], env=env, timeout=120, check=True)
