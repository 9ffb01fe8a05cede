# Shard transport probe (GPU box): python tests/_shard_probe.py
import os, random, sys
sys.path.insert(0, '.')
os.environ["ANYSEQ_SHARD_DEBUG"] = os.environ.get("DBG", "0")
os.environ["GPU_MAX_HW_QUEUES"] = os.environ.get("HWQ", "24")
print({k: v for k, v in os.environ.items() if k.startswith(("AMD_", "HIP_", "HSA_", "GPU_", "ROC"))}, flush=True)
import anyseq_amd as A
rng = random.Random(5)
rnd = lambda n: "".join(rng.choice("ACGT") for _ in range(n))
print("mode", os.environ.get("ANYSEQ_SHARD_WAITVALUE"), os.environ.get("ANYSEQ_SHARD_DIRECT"), os.environ["GPU_MAX_HW_QUEUES"], flush=True)
for ns in (2,):
    for n, m in [(130, 200), (700, 901)]:
        q, s = rnd(n), rnd(m)
        try:
            print(ns, n, m, A.shard_score_local("global", q, s, ns), A.score("global", q, s), flush=True)
        except Exception as e:
            print("ERR", ns, n, m, e, flush=True)
            break
