"""Repeat the in-process sharded affine score (16384^2, 2 and 4 shards) and count
failures (spin timeouts) -- flake-rate probe for the local shard transport.
usage: shard_flake.py <iterations> [kind]"""
import sys, time
sys.path.insert(0, '.')
import anyseq_amd as A
it = int(sys.argv[1]) if len(sys.argv) > 1 else 20
kind = sys.argv[2] if len(sys.argv) > 2 else 'semiglobal'
q, s = A.main_random_pair(16384, 16384)
ref = A.score(kind, q, s, gap_open=-2, gap_extend=-1)
bad = 0
t0 = time.time()
for i in range(it):
    for ns in (2, 4):
        try:
            v = A.shard_score_local(kind, q, s, ns, gap_open=-2, gap_extend=-1)
            if v != ref:
                bad += 1
                print('mismatch', i, ns, v, ref, flush=True)
        except Exception as e:
            bad += 1
            print('error', i, ns, e, flush=True)
print(f'{kind}: {bad} failures in {2 * it} runs, {time.time() - t0:.1f} s', flush=True)
