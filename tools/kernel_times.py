"""Per-kernel device times of one range-proof batch (single lane), for
quick A/B experiments: python tools/kernel_times.py [B] [reps]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "fabric-token-sdk_amd"))
import random  # noqa: E402

import fts_gpu  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
raw = open(os.path.join(ROOT, "tests/golden/zkatdlog_pp.json"), "rb").read()
pp = fts_gpu.PublicParams(raw, bit_length=64, device=0)
rng = random.Random(5)
R = 21888242871839275222246405745257275088548364400416034343698204186575808495617
vals = [rng.getrandbits(64) for _ in range(B)]
bfs = [rng.randrange(R).to_bytes(32, "big") for _ in range(B)]
proofs, coms = pp.prove_range_batch(vals, bfs, seed=9)
b = pp.stage_range_proofs(proofs, coms)
acc = {}
for r in range(reps + 1):
    st = b.verify()
    assert int((st != 0).sum()) == 0
    if r:
        for k, (ms, mads) in b.timings().items():
            acc[k] = acc.get(k, 0.0) + ms / reps
tag = os.environ.get("TAG", "")
print(tag, " ".join("%s=%.3f" % (k, v) for k, v in acc.items()), flush=True)
