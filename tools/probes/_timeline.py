"""Band timeline (s_memrealtime stamps) of one score fill per shape -> gpurun_out/timeline*.txt.
usage: _timeline.py [lib] [rows ...]"""
import os, sys
lib = sys.argv[1] if len(sys.argv) > 1 else "anyseq_amd/libanyseq_stamps.so"
rows = [int(x) for x in sys.argv[2:]] or [65536]
os.environ["ANYSEQ_STAMPS"] = "1"
os.environ["ANYSEQ_LIB"] = os.path.abspath(lib)
sys.path.insert(0, '.')
import anyseq_amd as A
qq, ss = A.main_random_pair(65536, 65536)
A.set_tuning(1, 4, 0)
for n in rows:
    path = f"gpurun_out/timeline_{os.path.basename(lib)[:-3]}_{n}.txt"
    os.environ["ANYSEQ_TIMELINE"] = ""
    A.score('global', qq[:n], ss)
    if os.path.exists(path): os.remove(path)
    os.environ["ANYSEQ_TIMELINE"] = path
    A.score('global', qq[:n], ss)
    os.environ["ANYSEQ_TIMELINE"] = ""
