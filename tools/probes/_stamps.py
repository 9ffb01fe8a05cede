import os, sys
os.environ["ANYSEQ_STAMPS"] = "1"
os.environ["ANYSEQ_LIB"] = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "anyseq_amd", "libanyseq_stamps.so")
sys.path.insert(0, '.')
import anyseq_amd as A
qq, ss = A.main_random_pair(65536, 65536)
cfgs = [tuple(int(x) for x in c.split(',')) for c in sys.argv[1:]] or [(1, 4)]
for R, NW in cfgs:
    A.set_tuning(R, NW, 0)
    for n, m in [(64, 65536), (256, 65536), (4096, 65536), (65536, 65536)]:
        A.score('global', qq[:n], ss[:m]); A.score('global', qq[:n], ss[:m])
